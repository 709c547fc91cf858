// aec_kernels.hip — gfx950 STFT-side kernels of the Stage-2 AEC hot path.
//
// Reference path: Little_net.forward (Stage2_lhm/scripts/network/ERB.py:252-334).
// Pipeline per batch of B streams (each stream has batch=1 semantics):
//
//   K1 moments_kernel   partial sums for x <- x - mean(x)/std(x) (ERB.py:254-256)
//   K2 analysis_kernel  frame + Hann + rFFT-512 (attention_ccrn.py:45-52) -> |X| (ERB.py:277-279)
//                       -> ERB band energies (ERB.py:282-284) for mic / ref / near
//   K3 gru_kernel       (aec_gru.hip) GRU + head + mask -> est_erb, loss
//   K4 synthesis_kernel gain = est_erb @ erb^T (ERB.py:306-310) * mic spectrum
//                       -> irFFT-512 + Hann + overlap-add / WOLA (attention_ccrn.py:82-101)
//                       -> + 1e-9 (ERB.py:316)
//
// HBM layout (row-major, float32 unless noted):
//   signals  [B][ld]              caller-owned
//   mom      [B][3][8] double2    per-chunk (sum x, sum x^2)
//   feats    [B][Tmax][96]        mic_erb | ref_erb | near_erb per frame
//   est      [B][Tmax][32]        est_erb per frame
//   out      [B][ld_out]          caller-owned, 256*(N_b/256) samples per row
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "aec_fft.h"
#include "aec_launch.h"
#include "aec_tables.h"

namespace aec {

// --------------------------------------------------------------------------
// K1: per-(stream, signal, chunk) float64 partial moments.  The normaliser
// scalar c = mean/std (unbiased) is finished by every consumer from the
// kMomChunks partials in a fixed order (deterministic, no atomics).
// --------------------------------------------------------------------------
__global__ __launch_bounds__(256) void moments_kernel(const float* __restrict__ mic,
                                                      const float* __restrict__ ref,
                                                      const float* __restrict__ near, int64_t ld,
                                                      const int64_t* __restrict__ lens,
                                                      double2* __restrict__ mom) {
    const int ch = blockIdx.x, s = blockIdx.y, b = blockIdx.z;
    const float* base = (s == 0 ? mic : (s == 1 ? ref : near));
    const float* x = base + (int64_t)b * ld;
    const int64_t n = lens[b];
    // chunk start = a multiple of 1024 samples (float4-aligned); a vector pass
    // reads 4096 samples (4 float4 per thread), the tail is scalar
    const int64_t per = ((n + kMomChunks - 1) / kMomChunks + 1023) & ~(int64_t)1023;
    const int64_t lo = ch * per, hi = min(n, lo + per);
    double s1 = 0.0, s2 = 0.0;
    const int tid = threadIdx.x;
    if (lo < hi) {
        if ((reinterpret_cast<uintptr_t>(x) & 15) == 0) {
            const int64_t hi4 = lo + ((hi - lo) & ~(int64_t)4095);   // full passes: 256 threads x 4 float4
            const float4* x4 = reinterpret_cast<const float4*>(x);
            for (int64_t i = lo / 4 + tid; i < hi4 / 4; i += 1024) {
                float4 v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) v[u] = x4[i + 256 * u];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const double a = v[u].x, bb = v[u].y, c = v[u].z, d = v[u].w;
                    s1 += (a + bb) + (c + d);
                    s2 += (a * a + bb * bb) + (c * c + d * d);
                }
            }
            for (int64_t i = hi4 + tid; i < hi; i += 256) {
                const double a = x[i];
                s1 += a;
                s2 += a * a;
            }
        } else {
            for (int64_t i = lo + tid; i < hi; i += 256) {
                const double a = x[i];
                s1 += a;
                s2 += a * a;
            }
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        s1 += __shfl_xor(s1, o);
        s2 += __shfl_xor(s2, o);
    }
    __shared__ double r1[4], r2[4];
    if ((tid & 63) == 0) {
        r1[tid >> 6] = s1;
        r2[tid >> 6] = s2;
    }
    __syncthreads();
    if (tid == 0)
        mom[((int64_t)b * 3 + s) * kMomChunks + ch] =
            make_double2((r1[0] + r1[1]) + (r1[2] + r1[3]), (r2[0] + r2[1]) + (r2[2] + r2[3]));
}

// c = mean(x)/std(x, unbiased) from the partials (ERB.py:254-256).
__device__ __forceinline__ float norm_scalar(const double2* __restrict__ mom, int b, int s, int64_t n) {
    const double2* m = mom + ((int64_t)b * 3 + s) * kMomChunks;
    double S1 = 0.0, S2 = 0.0;
#pragma unroll
    for (int i = 0; i < kMomChunks; ++i) {
        const double2 v = m[i];
        S1 += v.x;
        S2 += v.y;
    }
    const double dn = (double)n;
    const double mean = S1 / dn;
    double num = S2 - S1 * mean;
    if (num < 0.0) num = 0.0;                      // rounding on a constant signal
    const double sd = sqrt(num / (dn - 1.0));      // n == 1 -> 0/0 = nan, as torch.std
    return (float)(mean / sd);
}

// --------------------------------------------------------------------------
// shared helpers for K2 / K4
// --------------------------------------------------------------------------
constexpr int kHopsPB = kFPB + 1;        // sample hops staged per block
constexpr int kHopStride = 288;          // floats per staged hop (256 + 32: frames g, g+1 on disjoint banks)

// Stage hops [t0-1, t0+16) of one normalised signal row into LDS.  Samples
// outside [0, n) are the reference's zero padding (F.pad after the
// normaliser, attention_ccrn.py:48) and stay 0.
__device__ __forceinline__ void stage_hops(float* samp, const float* __restrict__ row, int64_t n,
                                           int64_t t0, float c, bool aligned) {
    const int64_t base = (t0 - 1) * kHop;
    for (int q = threadIdx.x; q < kHopsPB * (kHop / 4); q += blockDim.x) {
        const int64_t i = base + 4 * q;
        float4 v;
        if (aligned && i >= 0 && i + 3 < n) {
            v = *reinterpret_cast<const float4*>(row + i);
            v.x -= c; v.y -= c; v.z -= c; v.w -= c;
        } else {
            v.x = (i + 0 >= 0 && i + 0 < n) ? row[i + 0] - c : 0.f;
            v.y = (i + 1 >= 0 && i + 1 < n) ? row[i + 1] - c : 0.f;
            v.z = (i + 2 >= 0 && i + 2 < n) ? row[i + 2] - c : 0.f;
            v.w = (i + 3 >= 0 && i + 3 < n) ? row[i + 3] - c : 0.f;
        }
        *reinterpret_cast<float4*>(samp + (q >> 6) * kHopStride + (q & 63) * 4) = v;
    }
}

// Register-staged variant of stage_hops: prefetch_hops issues the global
// loads of the raw samples (0 outside [0, n)), commit_hops normalises and
// writes them to LDS.  Thread t owns float4 slots q = t + 256 u, u < kPf.
constexpr int kPf = (kHopsPB * (kHop / 4) + 255) / 256;     // 5
__device__ __forceinline__ void prefetch_hops(float4 (&pf)[kPf], const float* __restrict__ row, int64_t n,
                                              int64_t t0, bool aligned) {
    const int64_t base = (t0 - 1) * kHop;
#pragma unroll
    for (int u = 0; u < kPf; ++u) {
        const int q = threadIdx.x + 256 * u;
        const int64_t i = base + 4 * q;
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (q < kHopsPB * (kHop / 4)) {
            if (aligned && i >= 0 && i + 3 < n) {
                v = *reinterpret_cast<const float4*>(row + i);
            } else {
                if (i + 0 >= 0 && i + 0 < n) v.x = row[i + 0];
                if (i + 1 >= 0 && i + 1 < n) v.y = row[i + 1];
                if (i + 2 >= 0 && i + 2 < n) v.z = row[i + 2];
                if (i + 3 >= 0 && i + 3 < n) v.w = row[i + 3];
            }
        }
        pf[u] = v;
    }
}
// Normalise (x - c) inside [0, n) only — the zero padding stays 0 — and stage.
__device__ __forceinline__ void commit_hops(float* samp, const float4 (&pf)[kPf], float c, int64_t n, int64_t t0) {
    const int64_t base = (t0 - 1) * kHop;
#pragma unroll
    for (int u = 0; u < kPf; ++u) {
        const int q = threadIdx.x + 256 * u;
        if (q < kHopsPB * (kHop / 4)) {
            const int64_t i = base + 4 * q;
            float4 v = pf[u];
            v.x = (i + 0 >= 0 && i + 0 < n) ? v.x - c : 0.f;
            v.y = (i + 1 >= 0 && i + 1 < n) ? v.y - c : 0.f;
            v.z = (i + 2 >= 0 && i + 2 < n) ? v.z - c : 0.f;
            v.w = (i + 3 >= 0 && i + 3 < n) ? v.w - c : 0.f;
            *reinterpret_cast<float4*>(samp + (q >> 6) * kHopStride + (q & 63) * 4) = v;
        }
    }
}

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
// lane 0, m = 0 returns X[0] in xa[0] and X[256] in xb[0]; every lane returns
// X[128] in x128 (only lane 0 uses it).  sw = 16*(g&1) XOR-swizzles the LDS
// image so adjacent frames' b64 accesses fall on disjoint banks.
__device__ __forceinline__ void rfft_unpack(const float2 (&v)[16], int lb, int sw, float* scr, const float2* tw512,
                                            float2 (&xa)[8], float2 (&xb)[8], float2& x128) {
    float2* s2 = reinterpret_cast<float2*>(scr);
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2) s2[(lb + 16 * k2) ^ sw] = v[kP(k2)];
    wave_fence();
    float2 A[8], Bz[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        A[m] = s2[(lb + 16 * m) ^ sw];
        Bz[m] = s2[((256 - lb - 16 * m) & 255) ^ sw];
    }
    const float2 z128 = s2[128 ^ sw];
    wave_fence();
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        const int k = lb + 16 * m;
        if (k == 0) {
            xa[m] = make_float2(A[m].x + A[m].y, 0.f);
            xb[m] = make_float2(A[m].x - A[m].y, 0.f);
        } else {
            rfft_pair(A[m], Bz[m], tw512[k], xa[m], xb[m]);
        }
    }
    x128 = conjf2(z128);
}

// |X| = sqrt(re^2 + im^2 + 1e-9) (ERB.py:277-279).  The argument is >= 1e-9,
// never denormal, so the hardware v_sqrt_f32 (<= 1 ulp) needs no IEEE fix-up.
__device__ __forceinline__ float mag(float2 x) {
    return __builtin_amdgcn_sqrtf(fmaf(x.x, x.x, fmaf(x.y, x.y, 1e-9f)));
}

__device__ __forceinline__ void stage_common_tables(const DevTables* tb, float2* sTw256, float2* sTw512,
                                                    float* sHann) {
    const int tid = threadIdx.x;
    sTw256[tid] = tb->tw256[tid];
    sTw512[tid] = tb->tw512[tid];
    if (tid == 0) sTw512[256] = tb->tw512[256];
    sHann[tid] = tb->hann[tid];
    sHann[tid + 256] = tb->hann[tid + 256];
}

// --------------------------------------------------------------------------
// K2: analysis.  grid = (ceil(Tmax/16), B), block = 256 (16 frames x 16 lanes)
// ERB projection: every lane runs the same number (Lmax) of scheduled entries
// (bin, w0, w1, w2) -> three partial accumulators; bands wider than the
// schedule's split width are summed from two partials (ErbSched, aec_tables.h).
// --------------------------------------------------------------------------
__global__ __launch_bounds__(256) void analysis_kernel(AnalysisArgs p) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int b = blockIdx.y;
    const int64_t n = p.lens[b];
    const int64_t T = n / kHop + 1;
    const int64_t t0 = (int64_t)blockIdx.x * kFPB;
    if (t0 >= T) return;
    const int tid = threadIdx.x;
    const int L = p.sched_len;                                        // multiple of 4

    float2* sTw256 = reinterpret_cast<float2*>(smem);                 // 256 float2
    float2* sTw512 = sTw256 + 256;                                    // 258 float2
    float* sHann = reinterpret_cast<float*>(sTw512 + 258);            // 512
    float* sWork = sHann + 512;                                       // 16 * 576
    float4* sSched = reinterpret_cast<float4*>(sWork + kFPB * kGroupFloats);   // L * 16
    int2* sComb = reinterpret_cast<int2*>(sSched + L * 16);           // 32

    stage_common_tables(reinterpret_cast<const DevTables*>(p.tables), sTw256, sTw512, sHann);
    {
        const float4* sch = reinterpret_cast<const float4*>(p.sched);
        for (int i = tid; i < L * 16; i += 256) sSched[i] = sch[i];
        if (tid < 32) sComb[tid] = reinterpret_cast<const int2*>(p.sched + 4 * 16 * L)[tid];
    }
    const int g = tid >> 4, lb = tid & 15, sw = 16 * (g & 1);
    const int64_t t = t0 + g;
    float* scr = sWork + g * kGroupFloats;
    const bool aligned_ld = ((p.ld & 3) == 0);

    float cs[3];
    for (int s = 0; s < p.nsig; ++s) cs[s] = norm_scalar(p.mom, b, s, n);
    // register prefetch of one signal's 17 hops (5 float4 per thread): the
    // loads of signal s+1 are in flight while signal s is transformed
    float4 pf[kPf];
    prefetch_hops(pf, p.sig[0] + (int64_t)b * p.ld, n, t0, aligned_ld && ((reinterpret_cast<uintptr_t>(p.sig[0]) & 15) == 0));

    for (int s = 0; s < p.nsig; ++s) {
        __syncthreads();                           // previous use of sWork finished
        commit_hops(sWork, pf, cs[s], n, t0);
        if (s + 1 < p.nsig)
            prefetch_hops(pf, p.sig[s + 1] + (int64_t)b * p.ld, n, t0,
                          aligned_ld && ((reinterpret_cast<uintptr_t>(p.sig[s + 1]) & 15) == 0));
        __syncthreads();
        float2 v[16];
        load_frame(v, sWork, sHann, g, lb);
        __syncthreads();                           // all frames read before scratch reuse
        fft256<false>(v, lb, scr, sTw256);
        float2 xa[8], xb[8], x128;
        rfft_unpack(v, lb, sw, scr, sTw512, xa, xb, x128);
        // magnitudes (ERB.py:277-279) -> scr[k ^ sw], k = 0..256
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const int k = lb + 16 * m;
            scr[k ^ sw] = mag(xa[m]);
            scr[(k == 0 ? 256 : 256 - k) ^ sw] = mag(xb[m]);
        }
        if (lb == 0) scr[128 ^ sw] = mag(x128);
        wave_fence();
        // balanced ERB schedule: L entries per lane, 3 partial sums
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
        float* part = scr + 512;
        part[3 * lb + 0] = a0;
        part[3 * lb + 1] = a1;
        part[3 * lb + 2] = a2;
        wave_fence();
        if (t < T) {
            float* fo = p.feats + ((int64_t)b * p.Tmax + t) * 96 + 32 * s;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int band = lb + 16 * h;
                const int2 cb = sComb[band];
                fo[band] = part[cb.x] + (cb.y >= 0 ? part[cb.y] : 0.f);
            }
        }
        wave_fence();
    }
}

// --------------------------------------------------------------------------
// K4: synthesis.  grid = (ceil(nhop_max/15), B), block = 256.  A block
// re-derives the mic spectra of 16 consecutive frames, applies the ERB gains,
// inverse-transforms them and overlap-adds 15 output hops.
// --------------------------------------------------------------------------
__global__ __launch_bounds__(256) void synthesis_kernel(SynthArgs p) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int b = blockIdx.y;
    const int64_t n = p.lens[b];
    const int64_t T = n / kHop + 1;
    const int64_t nhop = T - 1;
    const int64_t h0 = (int64_t)blockIdx.x * kHopsOut;
    if (h0 >= nhop) return;
    const int tid = threadIdx.x;

    float2* sTw256 = reinterpret_cast<float2*>(smem);
    float2* sTw512 = sTw256 + 256;
    float* sHann = reinterpret_cast<float*>(sTw512 + 258);
    float* sCoff = sHann + 512;                                  // 256: 1/(window^2 OLA + 1e-8)
    float* sEst = sCoff + 256;                                   // 16 * 32
    float* sWork = sEst + kFPB * 32;                             // 16 * 576
    float4* sBin = reinterpret_cast<float4*>(sWork + kFPB * kGroupFloats);   // 257 (+3 pad)

    stage_common_tables(reinterpret_cast<const DevTables*>(p.tables), sTw256, sTw512, sHann);
    sCoff[tid] = reinterpret_cast<const DevTables*>(p.tables)->inv_coff[tid];
    {
        const float4* bt = reinterpret_cast<const float4*>(p.bintab);
        sBin[tid] = bt[tid];
        if (tid == 0) sBin[256] = bt[256];
        for (int i = tid; i < kFPB * 32; i += 256) {
            const int64_t t = h0 + (i >> 5);
            sEst[i] = (t < T) ? p.est[((int64_t)b * p.Tmax + t) * 32 + (i & 31)] : 0.f;
        }
    }
    const float* row = p.mic + (int64_t)b * p.ld;
    const bool aligned = ((p.ld & 3) == 0) && ((reinterpret_cast<uintptr_t>(p.mic) & 15) == 0);
    stage_hops(sWork, row, n, h0, norm_scalar(p.mom, b, 0, n), aligned);
    __syncthreads();
    const int g = tid >> 4, lb = tid & 15, sw = 16 * (g & 1);
    float* scr = sWork + g * kGroupFloats;
    float2 v[16];
    load_frame(v, sWork, sHann, g, lb);
    __syncthreads();
    fft256<false>(v, lb, scr, sTw256);
    float2 xa[8], xb[8], x128;
    rfft_unpack(v, lb, sw, scr, sTw512, xa, xb, x128);

    // ERB gain per bin: g[k] = sum_j est_erb[j] erb[k][j] over the <= 2 bands
    // covering bin k (ERB.py:306-307), applied to the mic spectrum (:309-310)
    const float* est = sEst + g * 32;
    auto gain = [&](int k) {
        const float4 e = sBin[k];
        return e.y * est[__float_as_int(e.x)] + e.w * est[__float_as_int(e.z)];
    };
    float2* s2 = reinterpret_cast<float2*>(scr);
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        const int k = lb + 16 * m;
        if (k == 0) {
            // DC / Nyquist: irfft ignores the imaginary parts
            const float s0 = gain(0) * xa[m].x, s256 = gain(256) * xb[m].x;
            s2[0 ^ sw] = make_float2(s0 + s256, s0 - s256);
        } else {
            float2 Zk, Zmk;
            irfft_pair(cscale(xa[m], gain(k)), cscale(xb[m], gain(256 - k)), sTw512[k], Zk, Zmk);
            s2[k ^ sw] = Zk;
            s2[(256 - k) ^ sw] = Zmk;
        }
    }
    if (lb == 0) {
        const float2 S = cscale(x128, gain(128));
        s2[128 ^ sw] = make_float2(2.f * S.x, -2.f * S.y);   // 2*conj(S[128])
    }
    wave_fence();
#pragma unroll
    for (int a = 0; a < 16; ++a) v[a] = s2[(16 * a + lb) ^ sw];
    wave_fence();
    fft256<true>(v, lb, scr, sTw256);
    // v[kP(m2)] = 512 * (x[2m] + i x[2m+1]), m = lb + 16 m2 ; window + 1/512
#pragma unroll
    for (int m2 = 0; m2 < 16; ++m2) {
        const int nn = 2 * (lb + 16 * m2);
        const float2 z = v[kP(m2)];
        s2[lb + 16 * m2] = make_float2(z.x * (sHann[nn] * (1.f / 512.f)), z.y * (sHann[nn + 1] * (1.f / 512.f)));
    }
    __syncthreads();
    // overlap-add + WOLA normalisation + trim (attention_ccrn.py:92-99) + 1e-9 (ERB.py:316)
    float* orow = p.out + (int64_t)b * p.ld_out;
    const int nh = (int)min((int64_t)kHopsOut, nhop - h0);
    const bool oal = ((p.ld_out & 3) == 0) && ((reinterpret_cast<uintptr_t>(p.out) & 15) == 0);
    if (oal) {
        for (int e = tid; e < nh * (kHop / 4); e += 256) {
            const int i = e >> 6, r = (e & 63) * 4;
            const float4 a = *reinterpret_cast<const float4*>(sWork + i * kGroupFloats + 256 + r);
            const float4 c = *reinterpret_cast<const float4*>(sWork + (i + 1) * kGroupFloats + r);
            const float4 cf = *reinterpret_cast<const float4*>(sCoff + r);
            float4 o;
            o.x = (a.x + c.x) * cf.x + 1e-9f;
            o.y = (a.y + c.y) * cf.y + 1e-9f;
            o.z = (a.z + c.z) * cf.z + 1e-9f;
            o.w = (a.w + c.w) * cf.w + 1e-9f;
            *reinterpret_cast<float4*>(orow + (h0 + i) * kHop + r) = o;
        }
    } else {
        for (int e = tid; e < nh * kHop; e += 256) {
            const int i = e >> 8, r = e & 255;
            const float a = sWork[i * kGroupFloats + 256 + r];
            const float c = sWork[(i + 1) * kGroupFloats + r];
            orow[(h0 + i) * kHop + r] = (a + c) * sCoff[r] + 1e-9f;
        }
    }
}

// --------------------------------------------------------------------------
// host-side launchers (called by aec_api.hip)
// --------------------------------------------------------------------------
hipError_t launch_moments(const float* mic, const float* ref, const float* near, int64_t ld,
                          const int64_t* lens, double2* mom, int B, int nsig, hipStream_t st) {
    hipLaunchKernelGGL(moments_kernel, dim3(kMomChunks, nsig, B), dim3(256), 0, st, mic, ref, near, ld, lens, mom);
    return hipGetLastError();
}

hipError_t launch_analysis(const AnalysisArgs& a, int B, hipStream_t st) {
    const dim3 grid((unsigned)((a.Tmax + kFPB - 1) / kFPB), B);
    hipLaunchKernelGGL(analysis_kernel, grid, dim3(256), analysis_smem_bytes(a.sched_len), st, a);
    return hipGetLastError();
}

hipError_t launch_synthesis(const SynthArgs& a, int B, hipStream_t st) {
    const int64_t nhop = a.Tmax - 1;
    if (nhop <= 0) return hipSuccess;
    const dim3 grid((unsigned)((nhop + kHopsOut - 1) / kHopsOut), B);
    hipLaunchKernelGGL(synthesis_kernel, grid, dim3(256), synthesis_smem_bytes(), st, a);
    return hipGetLastError();
}

}  // namespace aec
