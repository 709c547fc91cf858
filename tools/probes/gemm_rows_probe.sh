#!/bin/bash
# Build tools/probes/gemm_rows_probe (links the library's crn_kernels.o; run build() first).
set -e
R=$(cd "$(dirname "$0")/../.." && pwd)
C=$R/acoustic-echo-cancellation_amd/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I"$C" -c "$R/tools/probes/gemm_rows_probe.hip" \
    -o /tmp/gemm_rows_probe.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 /tmp/gemm_rows_probe.o "$C/../build/crn_kernels.o" \
    -o "$R/tools/probes/gemm_rows_probe"
