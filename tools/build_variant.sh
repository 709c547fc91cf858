#!/bin/bash
# Build an A/B variant of libaec_hip.so (timing experiments, AEC_HIP_LIB):
#   tools/build_variant.sh <name> [<git rev>|tree] [-DFLAG=..]...
# rev: build the library from that commit's csrc/ (default: the working tree).
# Variants are built with -DAEC_AB_KNOBS: the timing-only / work-skipping knobs of
# csrc/aec_knobs.h are read from the environment (the product build ignores them).
# Output: ab_libs/<name>.so (outside the package; git-ignored, travels with gpurun).
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
NAME=$1; shift
REV=${1:-tree}; [ $# -gt 0 ] && shift
SRC=$R/acoustic-echo-cancellation_amd/csrc
W=$(mktemp -d)
if [ -d "$REV" ]; then
  SRC=$(cd "$REV" && pwd)
elif [ "$REV" != tree ]; then
  git -C "$R" archive "$REV" acoustic-echo-cancellation_amd/csrc include | tar -x -C "$W"
  SRC=$W/acoustic-echo-cancellation_amd/csrc
fi
OUT=$R/ab_libs
mkdir -p "$OUT" "$W/obj"
SRCS=$(cd "$R" && python3 -c "import __graft_entry__ as g; print(' '.join(g.SOURCES))")
for s in $SRCS; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -fno-slp-vectorize -DAEC_AB_KNOBS "$@" \
      -I"$SRC" -c "$SRC/$s" -o "$W/obj/${s%.hip}.o" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "$W"/obj/*.o -o "$OUT/$NAME.so"
rm -rf "$W"
echo "built $OUT/$NAME.so"
