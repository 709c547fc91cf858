// aec_stft.h — shared STFT staging helpers (internal): hop staging through
// raw buffer loads, windowed frame load and the real-FFT unpack used by the
// analysis / synthesis kernels of the Little_net path (aec_kernels.hip) and
// by the DCCRN front / back kernels (crn_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "aec_fft.h"

namespace aec {

constexpr int kHopStride = 288;          // floats per staged hop (256 + 32: frames g, g+1 on disjoint banks)

// Windowed packed input of frame g: v[a] = (x[32a+2lb], x[32a+2lb+1]) * hann
__device__ __forceinline__ void load_frame(float2 (&v)[16], const float* samp, const float* hann, int g, int lb) {
    const float2* s2 = reinterpret_cast<const float2*>(samp);
    const float2* h2 = reinterpret_cast<const float2*>(hann);
#pragma unroll
    for (int a = 0; a < 16; ++a) {
        const float2 x = s2[(g + (a >> 3)) * (kHopStride / 2) + 16 * (a & 7) + lb];
        const float2 w = h2[16 * a + lb];
        v[a] = make_float2(x.x * w.x, x.y * w.y);
    }
}

// After a forward fft256 (v[kP(k2)] = Z[lb + 16 k2]) unpack the real spectrum.
// Lane lb returns X[k] and X[256-k] for k = lb + 16 m, m = 0..7 in xa[m] / xb[m];
// lane 0, m = 0 returns X[0] in xa[0] and X[256] in xb[0]; lane 0 also returns
// X[128] in x128.  The partner Z[256-k] lives in lane (16-lb)&15 at k2 = 15-m
// (lane 0: its own k2 = (16-m)&15) and is fetched with DPP (mirror16).
__device__ __forceinline__ void rfft_unpack(const float2 (&v)[16], int lb, const float2* tw512,
                                            float2 (&xa)[8], float2 (&xb)[8], float2& x128) {
    static_for<0, 8>([&](auto mi) {
        constexpr int m = decltype(mi)::value;
        const float2 A = v[kP(m)];
        const float2 mir = mirror16(v[kP(15 - m)]);
        const float2 Bz = csel(lb == 0, v[kP((16 - m) & 15)], mir);
        const int k = lb + 16 * m;
        if (k == 0) {
            xa[m] = make_float2(A.x + A.y, 0.f);
            xb[m] = make_float2(A.x - A.y, 0.f);
        } else {
            rfft_pair(A, Bz, tw512[k], xa[m], xb[m]);
        }
    });
    x128 = conjf2(v[kP(8)]);
}

constexpr int kWaveFrames = 4;
constexpr int kWaveHops = kWaveFrames + 1;
constexpr int kWaveFloats = kWaveFrames * kGroupFloats;     // >= kWaveHops * kHopStride
constexpr int kWavePf = kWaveHops;                          // float4 per lane per signal

// Wave-local staging: the 5 hops [t-1, t+4) of frames t .. t+3; lane owns
// float4 slot `lane` of every hop.  Raw buffer loads through a per-row
// descriptor (wave-uniform base, n*4 bytes): 32-bit offsets, and the
// hardware range check returns 0 outside the row (negative offsets wrap to
// out-of-range), so the reference's zero padding needs no branches;
// wave_commit re-applies the exact [0, n) mask.  Rows that are not 16-B
// aligned take dword loads (wave-uniform branch).
#ifndef AEC_LOAD_CPOL
#define AEC_LOAD_CPOL 2   // sample loads are nt (each hop is read once per transform); 0 = default policy (A/B)
#endif
__device__ __forceinline__ void wave_prefetch(float4 (&pf)[kWavePf], const float* __restrict__ row, int n,
                                              int t, int lane, bool aligned) {
    // the row / length are wave-uniform (one item per wave); make that provable so
    // hipcc keeps the descriptor in SGPRs (no waterfall loop per load)
    const uint64_t ra = reinterpret_cast<uint64_t>(row);
    const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)ra);
    const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(ra >> 32));
    const int nb = __builtin_amdgcn_readfirstlane(n * 4);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        reinterpret_cast<void*>(((uint64_t)hi << 32) | lo), (short)0, nb, 0x00020000);
    const int base = ((t - 1) * kHop + 4 * lane) * 4;
    if (__builtin_expect(aligned, 1)) {
#pragma unroll
        for (int u = 0; u < kWavePf; ++u) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, base + u * kHop * 4, 0, AEC_LOAD_CPOL);
            pf[u] = make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]),
                                __uint_as_float(v[3]));
        }
    } else {
#pragma unroll
        for (int u = 0; u < kWavePf; ++u) {
            const int o = base + u * kHop * 4;
            pf[u] = make_float4(__uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, o + 0, 0, AEC_LOAD_CPOL)),
                                __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, o + 4, 0, AEC_LOAD_CPOL)),
                                __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, o + 8, 0, AEC_LOAD_CPOL)),
                                __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, o + 12, 0, AEC_LOAD_CPOL)));
        }
    }
}
// Normalise (x - c) inside [0, n) only — the zero padding stays 0 — and stage.
__device__ __forceinline__ void wave_commit(float* wr, const float4 (&pf)[kWavePf], float c, int n,
                                            int t, int lane) {
    const int base = (t - 1) * kHop + 4 * lane;
#pragma unroll
    for (int u = 0; u < kWavePf; ++u) {
        const int i = base + u * kHop;
        float4 v = pf[u];
        v.x = (i + 0 >= 0 && i + 0 < n) ? v.x - c : 0.f;
        v.y = (i + 1 >= 0 && i + 1 < n) ? v.y - c : 0.f;
        v.z = (i + 2 >= 0 && i + 2 < n) ? v.z - c : 0.f;
        v.w = (i + 3 >= 0 && i + 3 < n) ? v.w - c : 0.f;
        *reinterpret_cast<float4*>(wr + u * kHopStride + 4 * lane) = v;
    }
}

}  // namespace aec
