#!/bin/bash
# Build libaec_hip.so from the csrc/ + include/ of a git revision into build_ab/<name>.so
# (A/B against the working tree with tools/lib_ab.sh / AEC_HIP_LIB).  Runs on the CPU.
#   tools/build_ref_lib.sh <rev> <name> [file=rev ...]
# Each optional file=rev argument takes that csrc/ file (basename) from another revision
# ("WORK" = the working tree), so one change of a set can be A/B'd alone.
set -euo pipefail
REV=$1; NAME=$2
R=$(cd "$(dirname "$0")/.." && pwd)
T=$(mktemp -d)
trap 'rm -rf "$T"' EXIT
mkdir -p "$T/x/csrc" "$T/include" "$R/build_ab"
for f in $(git -C "$R" ls-tree --name-only "$REV" acoustic-echo-cancellation_amd/csrc/); do
  git -C "$R" show "$REV:$f" > "$T/x/csrc/$(basename "$f")"
done
shift 2
for o in "$@"; do
  f=${o%%=*}; r=${o#*=}
  if [ "$r" = WORK ]; then cp "$R/acoustic-echo-cancellation_amd/csrc/$f" "$T/x/csrc/$f"
  else git -C "$R" show "$r:acoustic-echo-cancellation_amd/csrc/$f" > "$T/x/csrc/$f"; fi
done
for f in $(git -C "$R" ls-tree --name-only "$REV" include/); do
  git -C "$R" show "$REV:$f" > "$T/include/$(basename "$f")"
done
objs=()
for s in "$T"/x/csrc/*.hip; do
  o="$T/$(basename "$s" .hip).o"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -fno-slp-vectorize \
      -I"$T/include" -c "$s" -o "$o" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC "${objs[@]}" -o "$R/build_ab/$NAME.so"
echo "built build_ab/$NAME.so from $REV"
