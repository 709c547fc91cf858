// aec_nlms16.hip — K2n, 16-wave form: the per-stream analysis with the
// FD-NLMS canceller (SURVEY.md §8 a1-a6 + a13) with one role per wave
// quartet, one wave of each role per SIMD:
//
//   waves  0..3  NEAR: near transform (chunk c) -> near_erb -> feats[64..95]
//   waves  4..7  MIC : mic_erb = ERB(|E|) of chunk c-2 from the |E| rows the
//                      NL waves left in LDS -> feats[0..31]; mic transform
//                      (chunk c) -> spectrum row M in the wave's LDS scratch
//   waves  8..11 REF : ref transform (chunk c) -> ref_erb -> feats[32..63];
//                      spectrum row R in the wave's LDS scratch
//   waves 12..15 NL  : the 16 recursion steps of chunk c-1, bin per lane
//                      (lane 0 also bin 256), E rows -> the spectrum buffer,
//                      |E| at mags_to_scr's swizzled words -> LDS (chunk & 1)
//
// A tick is 16 frames (frame 4 (w % 4) + g of the chunk on 16-lane group g
// of transform wave w).  Tick end: barrier 1 (the M / R rows and |E| rows
// complete); the NL waves copy M, R of their bin for the 16 frames into
// registers; barrier 2 (rows consumed).
//
// Against the 12-wave nlms_analysis_kernel (aec_kernels.hip, 3 waves per
// SIMD: mic = near + mic transforms, ref = mic_erb + ref transform + ref ERB,
// nlms), every transform role here does one transform and at most one ERB
// pass per tick, and the mic_erb pass reads 37 KiB of |E| rows instead of a
// 72 KiB double-buffered copy of E, which leaves the LDS for the fourth wave
// per SIMD.  Every value is computed by the same device functions in the
// same order (the transform, NlmsBin, mag, the ERB projection, row_to_scr),
// so feats and E are bit-identical to the 12-wave
// kernel (tests/test_gpu_nlms.py).  TAPS <= 4 (the recursion state and the
// 16-frame row copies fit 128 VGPRs).
//
// Measured (MI355X, 256 x 10 s, taps 4): 0.358 ms against the 12-wave
// kernel's 0.335 ms, so it is off by default (AEC_NLMS16=1 selects it).  The
// fourth wave per SIMD did not buy latency hiding: removing the mic / ref
// transforms saves 0.147 ms here, the recursion 0.065, the mic_erb pass
// 0.026 (tools/n16_modes.sh).  A first form that read E back through the
// cache for mic_erb (instead of |E| rows the NL waves write to LDS) took
// 0.42 ms: the load latency landed at the top of each tick.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "aec_fft.h"
#include "aec_frame.h"
#include "aec_launch.h"
#include "aec_stft.h"
#include "aec_tables.h"

namespace aec {

namespace {
constexpr int kW16 = 16;
constexpr int kT16 = 64 * kW16;
constexpr int kSched16 = 32;              // ERB schedule entries per lane (host check)
constexpr int kMagRow = 288;              // floats per |E| row (257 swizzled words + pad)
constexpr int kRow16 = 256;               // float2 per spectrum row

struct Carve16 {
    int sched = 0, comb = 0, tw512 = 0, twT = 0, hann = 0, tf = 0, mag = 0, total = 0;
    constexpr Carve16() {
        int o_ = 0;
        auto take = [&](int n) { const int r = o_; o_ += (n + 3) & ~3; return r; };
        sched = take(kSched16 * 16 * 4);
        comb = take(64);
        tw512 = take(516);
        twT = take(512);
        hann = take(512);
        tf = take(12 * kWaveFloats);      // NEAR0-3, MIC0-3, REF0-3 scratch
        mag = take(2 * kFPB * kMagRow);   // |E| rows of a chunk, double-buffered (chunk & 1), NL -> MIC
        total = o_;
    }
};
constexpr Carve16 kC16{};
static_assert(kC16.total * 4 <= 160 * 1024, "LDS budget");

template <int OFF>
__device__ __forceinline__ float* lds16() {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    return smem + OFF;
}

__device__ __forceinline__ void barrier_lds16() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xC07F);       // lgkmcnt(0), vmcnt / expcnt untouched
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// An LDS float pointer at a byte offset the compiler cannot see through, so
// the constant part of every access below it folds into the 16-bit DS
// offset field: regions past 64 KiB otherwise need one VGPR per distinct
// address (hoisted out of the tick loop, they spill at 128 VGPRs).
__device__ __forceinline__ float* lds_at(uint32_t byte_off) {
    asm volatile("" : "+v"(byte_off));
    return lds16<0>() + (byte_off >> 2);
}

// mags_to_scr (aec_frame.h) with the same values at the same LDS words,
// addressed as base + immediate: the swizzle k ^ sw (sw = 16 s, s = g & 1)
// flips bit 4 of k, i.e. adds +-16 s by the parity of k / 16.  So four
// per-lane bases cover the 17 words (the XOR form costs one VGPR per word).
__device__ __forceinline__ void mags_to_scr16(float* scr, int lb, int sw, const float2 (&xa)[8], const float2 (&xb)[8],
                                              float2 x128) {
    const int d = lb == 0 ? sw : -sw;                 // bin 256 - k: lane 0 sits on the other parity
    float* pa0 = scr + lb + sw;                       // k = lb + 16 m, m even
    float* pa1 = scr + lb - sw;                       //                m odd
    float* pb0 = scr + 256 - lb + d;                  // 256 - k,        m even
    float* pb1 = scr + 256 - lb - d;                  //                 m odd
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        ((m & 1) ? pa1 : pa0)[16 * m] = mag(xa[m]);
        ((m & 1) ? pb1 : pb0)[-16 * m] = mag(xb[m]);   // lane 0, m = 0: bin 256 (xb[0] = X[256])
    }
    if (lb == 0) scr[128 + sw] = mag(x128);
}

// erb_project (aec_frame.h) with the partial sums at `part` instead of
// scr + 512: the same entries in the same order.
__device__ __forceinline__ void erb_project16(const float* scr, float* part, const float4* sSched, const int2* sComb,
                                              int L, int lb, int sw, float* fo) {
    float a0 = 0.f, a1 = 0.f, a2 = 0.f;
    for (int e = 0; e < L; e += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const float4 en = sSched[(e + u) * 16 + lb];
            const float mg = scr[__float_as_int(en.x) ^ sw];
            a0 = fmaf(en.y, mg, a0);
            a1 = fmaf(en.z, mg, a1);
            a2 = fmaf(en.w, mg, a2);
        }
    }
    part[3 * lb + 0] = a0;
    part[3 * lb + 1] = a1;
    part[3 * lb + 2] = a2;
    wave_fence();
    if (fo) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int band = lb + 16 * h;
            const int2 cb = sComb[band];
            fo[band] = part[cb.x] + (cb.y >= 0 ? part[cb.y] : 0.f);
        }
    }
    wave_fence();
}

struct Stream16 {
    int b, n, nch, nticks;
    int64_t T;
};

// ------------------------------------------------------- NL role ---------
template <int TAPS>
__device__ __forceinline__ void role_nl16(const NlmsArgs& p, const Stream16& s) {
    const int lane = threadIdx.x & 63, q = (threadIdx.x >> 6) - 12;
    const int k = lane + 64 * q;                              // bin k; k = 0 also bin 256
    // one base per row region (each < 64 KiB): MIC rows, REF rows
    const float2* mrow = reinterpret_cast<const float2*>(lds_at((kC16.tf + 4 * kWaveFloats) * 4 + 8 * k));
    const float2* rrow = reinterpret_cast<const float2*>(lds_at((kC16.tf + 8 * kWaveFloats) * 4 + 8 * k));
    float2* spec = p.spec + (int64_t)s.b * p.Tmax * kRow16;
    NlmsBin<TAPS> st;
    st.reset(k == 0);
    const float mu = p.mu, beta = p.beta, delta = p.delta;
    float2 dd[kFPB], rr[kFPB];
    for (int c = 0; c < s.nticks; ++c) {
        const int c1 = c - 1;
        if (c1 >= 0 && c1 < s.nch && !(p.mode & 1)) {
            const int64_t t0 = (int64_t)c1 * kFPB;
            const int nv = (int)min((int64_t)kFPB, s.T - t0);     // frames of the chunk inside the stream
            float2* ep = spec + t0 * kRow16 + k;
            // |E| rows for the MIC waves' mic_erb pass, at mags_to_scr's swizzled words
            // (frame i is read by group i % 4: sw = 16 (i & 1)); lane 0: bins 0 and 256
            float* mg0 = lds_at((kC16.mag + (c1 & 1) * kFPB * kMagRow + (k == 0 ? 0 : k)) * 4);
            float* mg1 = lds_at((kC16.mag + (c1 & 1) * kFPB * kMagRow + (k == 0 ? 16 : (k ^ 16))) * 4);
#pragma unroll
            for (int i = 0; i < kFPB; ++i) {
                const float2 e = st.step(dd[i], rr[i], mu, beta, delta);
                if (i < nv) *ep = e;
                ep += kRow16;
                float* mg = ((i & 1) ? mg1 : mg0) + i * kMagRow;
                mg[0] = mag(k == 0 ? make_float2(e.x, 0.f) : e);
                if (k == 0) mg[256] = mag(make_float2(e.y, 0.f));
            }
        }
        __syncthreads();                                      // E stored; rows of chunk c complete
        if (c < s.nch) {
#pragma unroll
            for (int i = 0; i < kFPB; ++i) {   // frame i: wave i / 4, group i % 4 of each role
                const int o = ((i >> 2) * kWaveFloats + (i & 3) * kGroupFloats) / 2;
                dd[i] = mrow[o];
                rr[i] = rrow[o];
            }
        }
        barrier_lds16();                                      // rows consumed
    }
}

// ------------------------------------------------- transform roles -------
// KIND 0 NEAR, 1 MIC, 2 REF (signal index: mic 0, ref 1, near 2)
template <int KIND>
__device__ __forceinline__ void role_tf16(const NlmsArgs& p, const Stream16& s) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int gg = lane >> 4, lb = lane & 15, sw = 16 * (gg & 1);
    const int m = wave & 3;
    float* wr = lds_at((kC16.tf + wave * kWaveFloats) * 4);
    float* scr = wr + gg * kGroupFloats;
    const float4* sSched = reinterpret_cast<const float4*>(lds16<kC16.sched>());
    const int2* sComb = reinterpret_cast<const int2*>(lds16<kC16.comb>());
    const float2* sTw512 = reinterpret_cast<const float2*>(lds16<kC16.tw512>());
    const float2* sTwT = reinterpret_cast<const float2*>(lds16<kC16.twT>());
    const float* sHann = lds16<kC16.hann>();
    const int L = p.sched_len;
    constexpr int sig = KIND == 0 ? 2 : (KIND == 1 ? 0 : 1);
    const bool on = KIND != 0 || p.nsig == 3;
    const float* row = on ? p.sig[sig] + (int64_t)s.b * p.ld : nullptr;
    const bool al = on && ((p.ld & 3) == 0) && ((reinterpret_cast<uintptr_t>(p.sig[sig]) & 15) == 0);
    const int n = KIND == 1 ? s.n : p.slen[4 * s.b + sig];
    const float cval = on ? p.cvals[s.b * 3 + sig] : 0.f;
    float* feats = p.feats + (int64_t)s.b * p.Tmax * 96;
    constexpr int foff = KIND == 0 ? 64 : (KIND == 1 ? 0 : 32);
    const bool tf = on && !(p.mode & (KIND == 0 ? 2 : 8));
    const bool erb = KIND != 0 || !(p.mode & 2);
    float4 pf[kWavePf];
    if (tf) wave_prefetch(pf, row, n, 4 * m, lane, al);
    for (int c = 0; c < s.nticks; ++c) {
        if (KIND == 1) {
            const int c2 = c - 2;                             // mic_erb of chunk c-2 (|E| rows from tick c-1)
            if (c2 >= 0 && c2 < s.nch && !(p.mode & 4)) {
                const int64_t t2 = (int64_t)c2 * kFPB + 4 * m + gg;
                const float* mrow = lds_at((kC16.mag + ((c2 & 1) * kFPB + 4 * m + gg) * kMagRow) * 4);
                erb_project16(mrow, scr + 512, sSched, sComb, L, lb, sw, t2 < s.T ? feats + t2 * 96 : nullptr);
            }
        }
        if (c < s.nch && tf) {
            const int wt = c * kFPB + 4 * m;
            const int64_t t = wt + gg;
            float2 xa[8], xb[8], x128;
            asm volatile("" ::: "memory");
            wave_commit(wr, pf, cval, n, wt, lane);
            if (c + 1 < s.nch) wave_prefetch(pf, row, n, wt + kFPB, lane, al);
            wave_fence();
            {
                float2 v[16];
                load_frame(v, wr, sHann, gg, lb);
                wave_fence();
                fft256<false>(v, lb, scr, sTwT);
                rfft_unpack(v, lb, sTw512, xa, xb, x128);
            }
            if (KIND != 1 && erb) {
                mags_to_scr16(scr, lb, sw, xa, xb, x128);
                wave_fence();
                erb_project(scr, sSched, sComb, L, lb, sw, t < s.T ? feats + t * 96 + foff : nullptr);
            }
            if (KIND != 0) row_to_scr(scr, lb, xa, xb, x128);   // M / R row of frame t, for the NL waves
        }
        __syncthreads();                                      // rows of chunk c complete
        barrier_lds16();                                      // rows consumed
    }
}

template <int TAPS>
__global__ __launch_bounds__(kT16, 1) void nlms16_kernel(NlmsArgs p) {
    const int tid = threadIdx.x, wave = tid >> 6;
    const int L = p.sched_len;
    Stream16 s;
    s.b = p.b0 + blockIdx.x;
    s.n = (int)p.lens[s.b];
    s.T = s.n / kHop + 1;
    s.nch = (int)((s.T + kFPB - 1) / kFPB);
    s.nticks = s.nch + 2;
    {
        const DevTables* tb = reinterpret_cast<const DevTables*>(p.tables);
        const float4* sch = reinterpret_cast<const float4*>(p.sched);
        float4* sSched = reinterpret_cast<float4*>(lds16<kC16.sched>());
        for (int i = tid; i < L * 16; i += kT16) sSched[i] = sch[i];
        if (tid < 32)
            reinterpret_cast<int2*>(lds16<kC16.comb>())[tid] = reinterpret_cast<const int2*>(p.sched + 4 * 16 * L)[tid];
        if (tid < 258) reinterpret_cast<float2*>(lds16<kC16.tw512>())[tid] = tb->tw512[tid];
        if (tid < 256) reinterpret_cast<float2*>(lds16<kC16.twT>())[tid] = tb->twT[tid];
        if (tid < 512) lds16<kC16.hann>()[tid] = tb->hann[tid];
    }
    __syncthreads();
#ifndef N16_ROLES
#define N16_ROLES 0xF          // build experiments only: bit r compiles role r (NEAR MIC REF NL)
#endif
    auto idle = [&]() { for (int c = 0; c < s.nticks; ++c) { __syncthreads(); barrier_lds16(); } };
    const int role = wave >> 2;
    {
        // AEC_NLMS_PRIO digits near|mic|ref|nl (timing experiments)
        const int pr = role == 3 ? p.prio % 10 : role == 2 ? (p.prio / 10) % 10 : role == 1 ? (p.prio / 100) % 10
                                                                                            : (p.prio / 1000) % 10;
        switch (pr) {
            case 1: __builtin_amdgcn_s_setprio(1); break;
            case 2: __builtin_amdgcn_s_setprio(2); break;
            case 3: __builtin_amdgcn_s_setprio(3); break;
            default: break;
        }
    }
    if (role == 3) { if constexpr (N16_ROLES & 8) role_nl16<TAPS>(p, s); else idle(); }
    else if (role == 0) { if constexpr (N16_ROLES & 1) role_tf16<0>(p, s); else idle(); }
    else if (role == 1) { if constexpr (N16_ROLES & 2) role_tf16<1>(p, s); else idle(); }
    else { if constexpr (N16_ROLES & 4) role_tf16<2>(p, s); else idle(); }
}

template <int TAPS>
static hipError_t launch_nlms16_t(const NlmsArgs& a, int nb, hipStream_t st) {
    static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(nlms16_kernel<TAPS>),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (attr != hipSuccess) return attr;
    hipLaunchKernelGGL(nlms16_kernel<TAPS>, dim3(nb), dim3(kT16), (size_t)kC16.total * 4, st, a);
    return hipGetLastError();
}
}  // namespace

bool nlms16_supported(int taps, int sched_len) { return taps >= 1 && taps <= 4 && sched_len <= kSched16; }

hipError_t launch_nlms16(const NlmsArgs& a, int nb, hipStream_t st) {
    if (nb <= 0) return hipSuccess;
    if (!nlms16_supported(a.taps, a.sched_len)) return hipErrorInvalidValue;
    switch (a.taps) {
        case 1: return launch_nlms16_t<1>(a, nb, st);
        case 2: return launch_nlms16_t<2>(a, nb, st);
        case 3: return launch_nlms16_t<3>(a, nb, st);
        default: return launch_nlms16_t<4>(a, nb, st);
    }
}

}  // namespace aec
