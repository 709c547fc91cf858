set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_nlms.py tests/test_gpu_api.py tests/test_train.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06c_gputest.log 2>&1 || { tail -30 gpurun_out/r06c_gputest.log; exit 1; }
tail -2 gpurun_out/r06c_gputest.log
bash tools/r06c_mom_ab.sh 3
