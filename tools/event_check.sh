#!/bin/bash
# HIP-event kernel times (bench.py sequential pass) next to a rocprofv3 trace of the same command.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$(pwd)
timeout -k 10 200 python bench.py --steps 20 --warmup 3 --no-cpu --no-c3 --no-rtf > gpurun_out/ev_bench.json 2> gpurun_out/ev_bench.err || exit 1
python -c "import json; d=json.loads(open('gpurun_out/ev_bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['kernel_ms_per_step'])"
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ev_trace -o run -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu --no-c3 --no-rtf > $R/gpurun_out/ev_trace.log 2>&1 || exit 1
cd $R && head -4 gpurun_out/ev_trace/run_kernel_stats.csv | cut -c1-160
grep -h '^{' gpurun_out/ev_trace.log | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('under tracer', d['ms_per_step'], d['kernel_ms_per_step'])"
