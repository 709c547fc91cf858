#!/bin/bash
# rocprofv3 kernel stats of the training step at B = 16 (train_conf) and 256 (run via gpurun)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/train_prof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for B in 16 256; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/b$B -o run -- \
      python3 $R/tools/train_probe.py --batch $B --steps 10 > $OUT/b$B.json 2> $OUT/b$B.err
done
