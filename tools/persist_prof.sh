#!/bin/bash
# Persistent LSTM recurrence: per-kernel durations (rocprofv3 kernel stats) of the
# DCCRN bench for the CRN_PERSIST_MODE values in MODES (0 = the real kernel).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for m in ${MODES:-0}; do
  AEC_CRN_PERSIST=${PERSIST:-1} CRN_PERSIST_MODE=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pprof_$m -o run -- python3 bench.py --pipeline crn --steps 3 --warmup 1 --no-cpu --no-rtf --inflight 1 > gpurun_out/pprof_$m.json 2> gpurun_out/pprof_$m.err || exit 1
  f=$(ls gpurun_out/pprof_$m/*/run_kernel_stats.csv 2>/dev/null | head -1)
  [ -n "$f" ] || f=$(ls gpurun_out/pprof_$m/run_kernel_stats.csv)
  python3 - "$f" "$m" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r['TotalDurationNs']))
for r in rows[:8]:
    print(sys.argv[2], r['Name'][:60], r['Calls'], round(float(r['AverageNs']) / 1e3, 1), 'us')
PY
done
