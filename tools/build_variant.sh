#!/bin/bash
# Build an A/B variant of libaec_hip.so (timing experiments, AEC_HIP_LIB):
#   tools/build_variant.sh <name> [<git rev>|tree] [-DFLAG=..]...
# rev: build the library from that commit's csrc/ (default: the working tree).
# Output: acoustic-echo-cancellation_amd/aec_amd/ab/<name>.so
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
OUT=$R/acoustic-echo-cancellation_amd/aec_amd/ab
mkdir -p "$OUT" "$W/obj"
SRCS="aec_api.hip aec_kernels.hip aec_gru.hip aec_gru_synth.hip aec_stream.hip crn_api.hip crn_kernels.hip crn_persist.hip crn_persist3.hip crn_stream.hip aec_train.hip"
for s in $SRCS; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -fno-slp-vectorize "$@" \
      -I"$SRC" -c "$SRC/$s" -o "$W/obj/${s%.hip}.o" &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "$W"/obj/*.o -o "$OUT/$NAME.so"
rm -rf "$W"
echo "built $OUT/$NAME.so"
