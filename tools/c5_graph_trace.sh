#!/bin/bash
# C5 per-hop step, direct launches vs hipGraph replays: kernel + HIP runtime traces
# (no counters) of tools/c5_mode_prof.py in each mode.  bash tools/c5_graph_trace.sh <tag>
set -uo pipefail
TAG=${1:-c5g}
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
cd /tmp
for m in 0 1; do
  OUT=$R/gpurun_out/${TAG}_graph$m
  rm -rf "$OUT"; mkdir -p "$OUT"
  echo "graph=$m" > "$OUT/cfg.txt"
  C5_GRAPH=$m timeout -k 10 240 rocprofv3 --kernel-trace --hip-runtime-trace --stats --output-format csv \
      -d "$OUT/trace" -o run -- python3 "$R/tools/c5_mode_prof.py" > "$OUT/c5.log" 2>&1 || { tail -20 "$OUT/c5.log"; exit 1; }
  grep '^{' "$OUT/c5.log"
done
python3 $R/tools/c5_hop_table.py $R/gpurun_out/${TAG}_graph0 $R/gpurun_out/${TAG}_graph1 > $R/gpurun_out/${TAG}_hop_table.txt
cat $R/gpurun_out/${TAG}_hop_table.txt
