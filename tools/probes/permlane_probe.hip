// Semantics probe for v_permlane16_swap_b32 + DPP row_newbcast on gfx950 (prints lane maps).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <type_traits>
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) { f(std::integral_constant<int, B>{}); static_for<B + 1, E>(f); }
}
__global__ void k(int* o) {
    const int lane = threadIdx.x;
    const int x = lane & 31;   // "h_j" in lane j and j + 32
    auto sw = __builtin_amdgcn_permlane16_swap((unsigned)x, (unsigned)x, false, false);
    o[lane] = sw[0];
    o[64 + lane] = sw[1];
    const int X = (lane >> 5) ? (int)sw[1] : (int)sw[0];
    static_for<0, 16>([&](auto ni) { constexpr int n = decltype(ni)::value;
        o[128 + 64 * n + lane] = __builtin_amdgcn_update_dpp(0, X, 0x150 + n, 0xf, 0xf, false); });
}
int main() {
    int* d; hipMalloc(&d, (128 + 16 * 64) * 4);
    k<<<1, 64>>>(d);
    int h[128 + 16 * 64];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("sw0:"); for (int i = 0; i < 64; ++i) printf(" %d", h[i]); printf("\n");
    printf("sw1:"); for (int i = 0; i < 64; ++i) printf(" %d", h[64 + i]); printf("\n");
    int bad = 0;
    for (int n = 0; n < 16; ++n) for (int l = 0; l < 64; ++l) if (h[128 + 64 * n + l] != n + 16 * (l >> 5)) ++bad;
    printf("bcast mismatches: %d\n", bad);
    return bad != 0;
}
