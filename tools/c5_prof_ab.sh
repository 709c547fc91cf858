#!/bin/bash
# rocprofv3 kernel traces of the C5 per-hop step under env settings: bash tools/c5_prof_ab.sh "VAR=a" ...
set -uo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp
i=0
for cfg in "base" "$@"; do
  i=$((i+1))
  OUT=$R/gpurun_out/c5pab_$i
  rm -rf "$OUT"; mkdir -p "$OUT"
  echo "$cfg" > "$OUT/cfg.txt"
  (cd /tmp && env $( [ "$cfg" != base ] && echo $cfg ) HOPS=100 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
      python3 "$R/tools/c5_prof.py" > "$OUT/c5.log" 2>&1) || { tail -5 "$OUT/c5.log"; exit 1; }
  echo "$cfg traced"
done
