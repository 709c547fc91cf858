#!/bin/bash
# L2 hit / miss of the C5 LSTM layer steps: the fused two-layer launch (A/B library ab_lstm2.so with
# tools/archive/r06x_lstm_two_layer_launch.patch, AEC_CRN_LSTM_FUSE=1) against the two launches (=0),
# 256 streams; one --pmc pass each (TCC_HIT_sum, TCC_MISS_sum), no tracing domains.
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06z_l2
rm -rf $O; mkdir -p $O
export TMPDIR=/tmp
for f in 1 0; do
  (cd /tmp && AEC_HIP_LIB=$R/ab_libs/ab_lstm2.so AEC_CRN_LSTM_FUSE=$f HOPS=100 timeout -s KILL 120 \
      rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d $O/f$f -o run -- \
      python3 $R/tools/c5_mode_prof.py > $O/f$f.log 2>&1) || { tail -20 $O/f$f.log; exit 1; }
  echo "pass f$f done"
done
python3 - $O <<'PY'
import csv, glob, sys, collections
for f in ('f1', 'f0'):
    acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for p in glob.glob(f'{sys.argv[1]}/{f}/**/*counter_collection.csv', recursive=True):
        for r in csv.DictReader(open(p)):
            k = r['Kernel_Name'].split('(')[0][:60]
            if 'lstm' not in k: continue
            acc[k][r['Counter_Name']] += float(r['Counter_Value']); n[(k, r['Counter_Name'])] += 1
    for k, d in acc.items():
        h, m = d.get('TCC_HIT_sum', 0), d.get('TCC_MISS_sum', 0)
        L = n[(k, 'TCC_HIT_sum')]
        print(f, k, 'launches', L, 'hit/launch', round(h / max(L, 1)), 'miss/launch', round(m / max(L, 1)),
              'hit rate', round(h / max(h + m, 1), 3))
PY
