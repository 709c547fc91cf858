// gemm_rows_probe.hip — time crn::launch_gemm_rows on the DCCRN v2 LSTM
// input-projection shape (layer 0: A rows (frame, sequence) gathered from the
// encoder's last channels-last map, K = 4 bins x 256 channels, N = 8192,
// bf16 in / out) and print ms and TFLOP/s.  Variants are selected by the
// CRN_GEMM_* environment knobs read inside launch_gemm_rows.
// Build: tools/probes/gemm_rows_probe.sh
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#include "crn_gemm.h"
#include "crn_launch.h"

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e_ = (x);                                                   \
        if (e_ != hipSuccess) {                                                \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            return 1;                                                          \
        }                                                                      \
    } while (0)

int main(int argc, char** argv) {
    const int64_t F = argc > 1 ? atoll(argv[1]) : 160256;   // frames (256 streams x 626)
    const int iters = argc > 2 ? atoi(argv[2]) : 10;
    const int S = 2, D = 4, C = 256, H = 1024, N = 8192;
    const int64_t ld_in = 2 * C;
    const int64_t src_elems = F * D * ld_in;
    crn::bf16_t *src, *w, *out;
    float* bias;
    CK(hipMalloc(&src, src_elems * 2));
    CK(hipMalloc(&w, (size_t)N * H * 2));
    CK(hipMalloc(&out, (size_t)F * S * N * 2));
    CK(hipMalloc(&bias, N * 4));
    {
        std::vector<crn::bf16_t> hw((size_t)N * H);
        uint32_t s = 12345;
        for (auto& v : hw) {
            s = s * 1664525u + 1013904223u;
            v = (crn::bf16_t)(0x3c00 + ((s >> 16) & 0x3ff));   // small positive bf16
        }
        CK(hipMemcpy(w, hw.data(), hw.size() * 2, hipMemcpyHostToDevice));
        std::vector<crn::bf16_t> hs(1 << 20);
        for (auto& v : hs) {
            s = s * 1664525u + 1013904223u;
            v = (crn::bf16_t)(0x3c00 + ((s >> 16) & 0x3ff) - 0x200);
        }
        for (int64_t o = 0; o < src_elems; o += (int64_t)hs.size())
            CK(hipMemcpy(src + o, hs.data(), std::min<int64_t>(hs.size(), src_elems - o) * 2, hipMemcpyHostToDevice));
        CK(hipMemset(bias, 0, N * 4));
    }
    crn::RowSrc a{};
    a.src = src;
    a.M = F * S;
    a.K = H;
    a.rshift = 1;
    a.rs_hi = D * ld_in;
    a.rs_lo = H / D;
    a.kshift = 8;
    a.ks = ld_in;
    a.pmul = 0;
    a.padd = 0;
    a.plim = D;
    a.base_off = C;
    a.src_elems = src_elems;
    crn::RowEpi e{out, a.M, N, 0, (int64_t)N, 0, 0, bias, 0.f, 0};
    const int nst = H * 2 / crn::kStageBytes;
    hipStream_t st;
    CK(hipStreamCreate(&st));
    for (int i = 0; i < 2; ++i) CK((crn::launch_gemm_rows<crn::bf16_t, crn::bf16_t>(a, w, H, nst, e, N, st)));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0, st));
    for (int i = 0; i < iters; ++i) CK((crn::launch_gemm_rows<crn::bf16_t, crn::bf16_t>(a, w, H, nst, e, N, st)));
    CK(hipEventRecord(e1, st));
    CK(hipEventSynchronize(e1));
    float ms = 0.f;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= iters;
    // checksum of a few output rows (compare variants: identical K order => identical bits)
    std::vector<crn::bf16_t> ho((size_t)4 * N);
    CK(hipMemcpy(ho.data(), out + (size_t)(a.M / 2) * N, ho.size() * 2, hipMemcpyDeviceToHost));
    uint64_t cs = 1469598103934665603ull;
    for (auto v : ho) cs = (cs ^ v) * 1099511628211ull;
    printf("M %lld N %d K %d: %.3f ms  %.1f TFLOP/s  checksum %016llx\n", (long long)a.M, N, H, ms,
           2.0 * a.M * N * H / (ms * 1e-3) / 1e12, (unsigned long long)cs);
    return 0;
}
