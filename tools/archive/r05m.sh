#!/bin/bash
# round 5 batch m: the normaliser look-ahead (aec_prepare, bench --lookahead) -- tests, A/B with
# the two moments kernels; then batch l (packed inverse FFT / pre-scaled synthesis window)
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_nlms.py $R/tests/test_gpu_parity.py -m gpu -x -q --timeout 240 --timeout-method thread > $O/r05m_tests.log 2>&1 || { echo "gpu tests failed"; grep -E "FAIL|Error|assert" $O/r05m_tests.log | head -20; tail -5 $O/r05m_tests.log; exit 1; }
tail -1 $O/r05m_tests.log
for i in 1 2; do for la in 0 1; do for mc in 0 3; do
  AEC_MOM_CFG=$mc timeout -k 10 150 python $R/bench.py --no-cpu --no-c3 --no-rtf --no-sweep --no-train --steps 40 --lookahead $la > $O/r05m_la${la}_m${mc}_$i.log 2>&1 || { echo "bench la=$la failed"; tail -5 $O/r05m_la${la}_m${mc}_$i.log; exit 1; }
  echo "lookahead $la mom $mc #$i: $(tail -1 $O/r05m_la${la}_m${mc}_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["kernel_ms_per_step"])')"
done; done; done
bash $R/tools/r05l.sh
bash $R/tools/env_ab.sh AEC_NLMS_PRIO "0 10 20 120" 2 > $O/r05m_prio.log 2>&1 || { echo "prio ab failed"; tail $O/r05m_prio.log; exit 1; }
cat $O/r05m_prio.log
