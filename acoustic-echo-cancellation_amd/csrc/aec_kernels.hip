// aec_kernels.hip — gfx950 kernels for the Stage-2 AEC hot path.
//
// Reference path: Little_net.forward (Stage2_lhm/scripts/network/ERB.py:252-334).
// Pipeline per batch of B streams (each stream has batch=1 semantics):
//
//   K1 moments_kernel   x <- x - mean(x)/std(x) scalar per stream & signal (ERB.py:254-256)
//   K2 analysis_kernel  frame + Hann + rFFT-512 (attention_ccrn.py:45-52) -> |X| (ERB.py:277-279)
//                       -> ERB band energies (ERB.py:282-284) for mic / ref / near
//   K3 gru_kernel       x=[mic_erb,|mic_erb-ref_erb|] -> GRU(64->32) (ERB.py:287-293)
//                       -> relu(Linear) -> sigmoid(Linear) mask (ERB.py:295-301)
//                       -> est_erb = mask*mic_erb (ERB.py:304) and the loss (ERB.py:318-323)
//   K4 synthesis_kernel gain = est_erb @ erb^T (ERB.py:306-310) * mic spectrum
//                       -> irFFT-512 + Hann + overlap-add / WOLA (attention_ccrn.py:82-101)
//                       -> + 1e-9 (ERB.py:316)
//
// HBM layout (row-major, float32):
//   signals  [B][ld]            caller-owned
//   cvals    [B][3]             normaliser scalars (mic, ref, near)
//   feats    [B][Tmax][96]      mic_erb | ref_erb | near_erb per frame
//   est      [B][Tmax][32]      est_erb per frame
//   out      [B][ld_out]        caller-owned, 256*(N_b/256) samples per row
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "aec_fft.h"
#include "aec_tables.h"
#include "aec_launch.h"

namespace aec {

// --------------------------------------------------------------------------
// K1: per-(stream, signal) moments -> c = mean / std (unbiased), float64 sums
// --------------------------------------------------------------------------
__global__ __launch_bounds__(256) void moments_kernel(const float* __restrict__ mic,
                                                      const float* __restrict__ ref,
                                                      const float* __restrict__ near, int64_t ld,
                                                      const int64_t* __restrict__ lens,
                                                      float* __restrict__ cvals) {
    const int b = blockIdx.x, s = blockIdx.y;
    const float* base = (s == 0 ? mic : (s == 1 ? ref : near));
    const float* x = base + (int64_t)b * ld;
    const int64_t n = lens[b];
    double s1 = 0.0, s2 = 0.0;
    const int tid = threadIdx.x;
    if ((reinterpret_cast<uintptr_t>(x) & 15) == 0) {
        const int64_t n4 = n >> 2;
        const float4* x4 = reinterpret_cast<const float4*>(x);
        for (int64_t i = tid; i < n4; i += 256) {
            const float4 v = x4[i];
            const double a = v.x, bb = v.y, c = v.z, d = v.w;
            s1 += (a + bb) + (c + d);
            s2 += (a * a + bb * bb) + (c * c + d * d);
        }
        for (int64_t i = (n4 << 2) + tid; i < n; i += 256) {
            const double a = x[i];
            s1 += a;
            s2 += a * a;
        }
    } else {
        for (int64_t i = tid; i < n; i += 256) {
            const double a = x[i];
            s1 += a;
            s2 += a * a;
        }
    }
    // wave reduction (64 lanes) then across the 4 waves
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
    if (tid == 0) {
        const double S1 = (r1[0] + r1[1]) + (r1[2] + r1[3]);
        const double S2 = (r2[0] + r2[1]) + (r2[2] + r2[3]);
        const double dn = (double)n;
        const double mean = S1 / dn;
        double num = S2 - S1 * mean;
        if (num < 0.0) num = 0.0;                      // rounding on a constant signal
        const double sd = sqrt(num / (dn - 1.0));      // n == 1 -> 0/0 = nan, as torch.std
        cvals[b * 3 + s] = (float)(mean / sd);
    }
}

// --------------------------------------------------------------------------
// shared helpers for K2 / K4
// --------------------------------------------------------------------------
constexpr int kHopsPB = kFPB + 1;        // sample hops staged per block

// Stage hops [t0-1, t0+16) of one (normalised) signal row into LDS.  Samples
// outside [0, n) are the reference's zero padding (F.pad after the
// normaliser, attention_ccrn.py:48) and stay 0.
__device__ __forceinline__ void stage_hops(float* samp, const float* __restrict__ row, int64_t n,
                                           int64_t t0, float c, bool aligned) {
    float4* s4 = reinterpret_cast<float4*>(samp);
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
        s4[q] = v;
    }
}

// Windowed packed input of frame g: v[a] = (x[32a+2lb], x[32a+2lb+1]) * hann
__device__ __forceinline__ void load_frame(float2 (&v)[16], const float* samp, const float* hann, int g, int lb) {
    const float2* s2 = reinterpret_cast<const float2*>(samp) + 128 * g;
    const float2* h2 = reinterpret_cast<const float2*>(hann);
#pragma unroll
    for (int a = 0; a < 16; ++a) {
        const float2 x = s2[16 * a + lb];
        const float2 w = h2[16 * a + lb];
        v[a] = make_float2(x.x * w.x, x.y * w.y);
    }
}

// After a forward fft256 (v[kP(k2)] = Z[lb + 16 k2]) unpack the real spectrum.
// Lane lb returns X[k] and X[256-k] for k = lb + 16 m, m = 0..7 in xa[m] / xb[m];
// lane 0, m = 0 returns X[0] in xa[0] and X[256] in xb[0]; every lane returns
// X[128] in x128 (only lane 0 uses it).
__device__ __forceinline__ void rfft_unpack(const float2 (&v)[16], int lb, float* scr, const float2* tw512,
                                            float2 (&xa)[8], float2 (&xb)[8], float2& x128) {
    float2* s2 = reinterpret_cast<float2*>(scr);
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2) s2[lb + 16 * k2] = v[kP(k2)];
    wave_fence();
    float2 A[8], Bz[8];
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        A[m] = s2[lb + 16 * m];
        Bz[m] = s2[(256 - lb - 16 * m) & 255];
    }
    const float2 z128 = s2[128];
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

// --------------------------------------------------------------------------
// K2: analysis.  grid = (ceil(Tmax/16), B), block = 256 (16 frames x 16 lanes)
// --------------------------------------------------------------------------

__global__ __launch_bounds__(256) void analysis_kernel(AnalysisArgs p) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int b = blockIdx.y;
    const int64_t n = p.lens[b];
    const int64_t T = n / kHop + 1;
    const int64_t t0 = (int64_t)blockIdx.x * kFPB;
    if (t0 >= T) return;
    const int tid = threadIdx.x;

    // LDS carve (16-B aligned offsets)
    float2* sTw256 = reinterpret_cast<float2*>(smem);                 // 256 float2
    float2* sTw512 = sTw256 + 256;                                    // 258 float2 (257 used)
    float* sHann = reinterpret_cast<float*>(sTw512 + 258);            // 512
    float* sWork = sHann + 512;                                       // 16 * 576 floats
    int* sBandPtr = reinterpret_cast<int*>(sWork + kFPB * kGroupFloats);   // 36 ints (33 used)
    int* sBandBin = sBandPtr + 36;                                    // nnz
    float* sBandW = reinterpret_cast<float*>(sBandBin + ((p.nnz + 3) & ~3));

    {
        const DevTables* tb = reinterpret_cast<const DevTables*>(p.tables);
        for (int i = tid; i < 256; i += 256) sTw256[i] = tb->tw256[i];
        for (int i = tid; i < 257; i += 256) sTw512[i] = tb->tw512[i];
        for (int i = tid; i < 512; i += 256) sHann[i] = tb->hann[i];
        const ErbCSRView e = erb_view(p.erb_csr, p.nnz);
        for (int i = tid; i < 33; i += 256) sBandPtr[i] = e.band_ptr[i];
        for (int i = tid; i < p.nnz; i += 256) {
            sBandBin[i] = e.band_bin[i];
            sBandW[i] = e.band_w[i];
        }
    }
    const int g = tid >> 4, lb = tid & 15;
    const int64_t t = t0 + g;
    float* scr = sWork + g * kGroupFloats;
    const bool aligned_ld = ((p.ld & 3) == 0);

    for (int s = 0; s < p.nsig; ++s) {
        const float* row = p.sig[s] + (int64_t)b * p.ld;
        const bool aligned = aligned_ld && ((reinterpret_cast<uintptr_t>(p.sig[s]) & 15) == 0);
        __syncthreads();                           // previous use of sWork finished
        stage_hops(sWork, row, n, t0, p.cvals[b * 3 + s], aligned);
        __syncthreads();
        float2 v[16];
        load_frame(v, sWork, sHann, g, lb);
        __syncthreads();                           // all frames read before scratch reuse
        fft256<false>(v, lb, scr, sTw256);
        float2 xa[8], xb[8], x128;
        rfft_unpack(v, lb, scr, sTw512, xa, xb, x128);
        // magnitudes -> scr[0..256]
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const int k = lb + 16 * m;
            const float ma = sqrtf(xa[m].x * xa[m].x + xa[m].y * xa[m].y + 1e-9f);
            const float mb = sqrtf(xb[m].x * xb[m].x + xb[m].y * xb[m].y + 1e-9f);
            scr[k] = ma;
            scr[k == 0 ? 256 : 256 - k] = mb;
        }
        if (lb == 0) scr[128] = sqrtf(x128.x * x128.x + x128.y * x128.y + 1e-9f);
        wave_fence();
        if (t < T) {
            float* fo = p.feats + ((int64_t)b * p.Tmax + t) * 96 + 32 * s;
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int band = h == 0 ? lb : 31 - lb;
                float acc = 0.f;
                for (int i = sBandPtr[band]; i < sBandPtr[band + 1]; ++i) acc += sBandW[i] * scr[sBandBin[i]];
                fo[band] = acc;
            }
        }
    }
}

// --------------------------------------------------------------------------
// K3: GRU recurrence + head.  grid = B, block = 256:
//   wave 0      : the recurrence (h_t depends on h_{t-1}); one step per frame
//   waves 1..3  : helpers, software-pipelined one chunk (16 frames) ahead and
//                 behind the recurrence: x-load (c+2), gi = W_ih x + b (c+1),
//                 head / mask / est_erb / loss (c-1)
// --------------------------------------------------------------------------

__device__ __forceinline__ float sigmoidf_(float x) {
    return __builtin_amdgcn_rcpf(1.f + __expf(-x));
}
__device__ __forceinline__ float tanhf_(float x) {
    return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __expf(2.f * x));
}

typedef float f2v __attribute__((ext_vector_type(2)));


__global__ __launch_bounds__(256) void gru_kernel(GruArgs p) {
    __shared__ __attribute__((aligned(16))) float sX[2][kCH][64];
    __shared__ __attribute__((aligned(16))) float sGi[2][kCH][96];
    __shared__ __attribute__((aligned(16))) float sH[2][kCH][32];
    __shared__ __attribute__((aligned(16))) float sMic[4][kCH][32];
    __shared__ __attribute__((aligned(16))) float sO[6][32];
    __shared__ float sLoss[4];

    const int b = blockIdx.x;
    const int64_t n = p.lens[b];
    const int T = (int)(n / kHop + 1);
    const int nch = (T + kCH - 1) / kCH;
    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const float* W_ih = p.w;                  // [96][64]
    const float* W_hh = p.w + 96 * 64;        // [96][32]
    const float* b_ih = W_hh + 96 * 32;       // [96]
    const float* b_hh = b_ih + 96;            // [96]
    const float* W1 = b_hh + 96;              // [32][64]
    const float* b1 = W1 + 32 * 64;           // [32]
    const float* W2 = b1 + 32;                // [32][32]
    const float* b2 = W2 + 32 * 32;           // [32]
    const float* fb = p.feats + (int64_t)b * p.Tmax * 96;

    if (wave == 0) {
        // ---------------- recurrence wave ----------------
        const int j = lane & 31, half = lane >> 5;
        f2v w[32];
        {
            const float* rA = W_hh + (half ? (32 + j) : j) * 32;   // r_j (half 0) / z_j (half 1)
            const float* rN = W_hh + (64 + j) * 32;
#pragma unroll
            for (int k = 0; k < 32; ++k) w[k] = f2v{rA[k], rN[k]};
        }
        const float bhn = b_hh[64 + j];
        float hj = 0.f;
        for (int c = -2; c <= nch; ++c) {
            if (c >= 0 && c < nch) {
                const int f_end = min(kCH, T - c * kCH);
                const float* gi = &sGi[c & 1][0][0];
                for (int f = 0; f < f_end; ++f) {
                    f2v acc0 = {0.f, 0.f}, acc1 = {0.f, 0.f};
                    const int t = c * kCH + f;
                    if (t > 0) {
                        const float* hp = (f > 0) ? &sH[c & 1][f - 1][0] : &sH[(c - 1) & 1][kCH - 1][0];
                        const float4* hp4 = reinterpret_cast<const float4*>(hp);
#pragma unroll
                        for (int q = 0; q < 8; ++q) {
                            const float4 hv = hp4[q];
                            acc0 = __builtin_elementwise_fma(w[4 * q + 0], f2v{hv.x, hv.x}, acc0);
                            acc1 = __builtin_elementwise_fma(w[4 * q + 1], f2v{hv.y, hv.y}, acc1);
                            acc0 = __builtin_elementwise_fma(w[4 * q + 2], f2v{hv.z, hv.z}, acc0);
                            acc1 = __builtin_elementwise_fma(w[4 * q + 3], f2v{hv.w, hv.w}, acc1);
                        }
                    }
                    const f2v acc = acc0 + acc1;
                    const float sA = acc.x;            // r-dot (half 0) or z-dot (half 1)
                    const float sN = acc.y;            // n-dot (both halves)
                    // v_permlane32_swap: lanes 32..63 of vdst <-> lanes 0..31 of vsrc, so the
                    // other half's value is res[1] in lanes 0..31 and res[0] in lanes 32..63
                    const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(sA), __float_as_uint(sA), false, false);
                    const float other = __uint_as_float(half ? sw[0] : sw[1]);
                    const float rdot = half ? other : sA;
                    const float zdot = half ? sA : other;
                    const float r = sigmoidf_(gi[f * 96 + j] + rdot);
                    const float z = sigmoidf_(gi[f * 96 + 32 + j] + zdot);
                    const float nn = tanhf_(gi[f * 96 + 64 + j] + r * (sN + bhn));
                    hj = (1.f - z) * nn + z * hj;
                    if (half == 0) sH[c & 1][f][j] = hj;
                    wave_fence();
                }
            }
            __syncthreads();
        }
    } else {
        // ---------------- helper waves ----------------
        const int hl = tid - 64;                       // 0..191
        // gi role: row = hl % 96, frames f = fpar, fpar+2, ...
        const int grow = hl % 96, gpar = hl / 96;
        float wih[64];
#pragma unroll
        for (int k = 0; k < 64; ++k) wih[k] = W_ih[grow * 64 + k];
        const float gbias = b_ih[grow] + (grow < 64 ? b_hh[grow] : 0.f);
        // head role: j = hl & 31, frames f = fg, fg+6, fg+12
        const int hj_ = hl & 31, fg = hl >> 5;
        float w1[64], w2[32];
#pragma unroll
        for (int k = 0; k < 64; ++k) w1[k] = W1[hj_ * 64 + k];
#pragma unroll
        for (int k = 0; k < 32; ++k) w2[k] = W2[hj_ * 32 + k];
        const float b1j = b1[hj_], b2j = b2[hj_];
        float lacc = 0.f;

        for (int c = -2; c <= nch; ++c) {
            // (a) x-load for chunk c+2 -> sX[(c+2)&1], mic_erb -> sMic[(c+2)&3]
            {
                const int cc = c + 2;
                if (cc < nch) {
                    for (int e = hl; e < kCH * 32; e += 192) {
                        const int f = e >> 5, jj = e & 31;
                        const int t = cc * kCH + f;
                        float me = 0.f, re = 0.f;
                        if (t < T) {
                            me = fb[(int64_t)t * 96 + jj];
                            re = fb[(int64_t)t * 96 + 32 + jj];
                        }
                        sX[cc & 1][f][jj] = me;
                        sX[cc & 1][f][32 + jj] = fabsf(me - re);
                        sMic[cc & 3][f][jj] = me;
                    }
                }
            }
            // (b) gi for chunk c+1
            {
                const int cc = c + 1;
                if (cc >= 0 && cc < nch) {
                    for (int f = gpar; f < kCH; f += 2) {
                        const float4* x4 = reinterpret_cast<const float4*>(&sX[cc & 1][f][0]);
                        f2v a0 = {0.f, 0.f}, a1 = {0.f, 0.f};
#pragma unroll
                        for (int q = 0; q < 16; ++q) {
                            const float4 xv = x4[q];
                            a0 = __builtin_elementwise_fma(f2v{wih[4 * q], wih[4 * q + 1]}, f2v{xv.x, xv.y}, a0);
                            a1 = __builtin_elementwise_fma(f2v{wih[4 * q + 2], wih[4 * q + 3]}, f2v{xv.z, xv.w}, a1);
                        }
                        const f2v s2 = a0 + a1;
                        sGi[cc & 1][f][grow] = gbias + (s2.x + s2.y);
                    }
                }
            }
            // (c) head for chunk c-1
            {
                const int cc = c - 1;
                if (cc >= 0 && cc < nch) {
                    for (int f = fg; f < kCH; f += 6) {
                        const int t = cc * kCH + f;
                        if (t >= T) break;               // uniform within the 32-lane group
                        const float4* h4 = reinterpret_cast<const float4*>(&sH[cc & 1][f][0]);
                        const float4* m4 = reinterpret_cast<const float4*>(&sMic[cc & 3][f][0]);
                        f2v a0 = {0.f, 0.f}, a1 = {0.f, 0.f};
#pragma unroll
                        for (int q = 0; q < 8; ++q) {
                            const float4 hv = h4[q];
                            const float4 mv = m4[q];
                            a0 = __builtin_elementwise_fma(f2v{w1[4 * q], w1[4 * q + 1]}, f2v{hv.x, hv.y}, a0);
                            a1 = __builtin_elementwise_fma(f2v{w1[4 * q + 2], w1[4 * q + 3]}, f2v{hv.z, hv.w}, a1);
                            a0 = __builtin_elementwise_fma(f2v{w1[32 + 4 * q], w1[32 + 4 * q + 1]}, f2v{mv.x, mv.y}, a0);
                            a1 = __builtin_elementwise_fma(f2v{w1[32 + 4 * q + 2], w1[32 + 4 * q + 3]}, f2v{mv.z, mv.w}, a1);
                        }
                        const f2v s1 = a0 + a1;
                        const float o = fmaxf(b1j + (s1.x + s1.y), 0.f);
                        sO[fg][hj_] = o;
                        wave_fence();
                        const float4* o4 = reinterpret_cast<const float4*>(&sO[fg][0]);
                        f2v c0 = {0.f, 0.f}, c1 = {0.f, 0.f};
#pragma unroll
                        for (int q = 0; q < 8; ++q) {
                            const float4 ov = o4[q];
                            c0 = __builtin_elementwise_fma(f2v{w2[4 * q], w2[4 * q + 1]}, f2v{ov.x, ov.y}, c0);
                            c1 = __builtin_elementwise_fma(f2v{w2[4 * q + 2], w2[4 * q + 3]}, f2v{ov.z, ov.w}, c1);
                        }
                        wave_fence();
                        const f2v s2 = c0 + c1;
                        const float mask = sigmoidf_(b2j + (s2.x + s2.y));
                        const float me = sMic[cc & 3][f][hj_];
                        const float est = mask * me;
                        const int64_t o_idx = ((int64_t)b * p.Tmax + t) * 32 + hj_;
                        p.est[o_idx] = est;
                        if (p.dbg_h) p.dbg_h[o_idx] = sH[cc & 1][f][hj_];
                        if (p.dbg_mask) p.dbg_mask[o_idx] = mask;
                        if (p.has_near) {
                            const float ne = fb[(int64_t)t * 96 + 64 + hj_];
                            const float d = sqrtf(ne) - sqrtf(est);
                            lacc += d * d;
                        }
                    }
                }
            }
            __syncthreads();
        }
        if (p.loss) {
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) lacc += __shfl_xor(lacc, o);
            if (lane == 0) sLoss[wave] = lacc;
        }
    }
    if (p.loss) {
        __syncthreads();
        if (tid == 0) p.loss[b] = ((sLoss[1] + sLoss[2]) + sLoss[3]) / (float)(T * 32);
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
    float* sCoff = sHann + 512;                                  // 256
    float* sEst = sCoff + 256;                                   // 16 * 32
    float* sWork = sEst + kFPB * 32;                             // 16 * 576
    int* sBinPtr = reinterpret_cast<int*>(sWork + kFPB * kGroupFloats);   // 260 ints (258 used)
    int* sBinBand = sBinPtr + 260;
    float* sBinW = reinterpret_cast<float*>(sBinBand + ((p.nnz + 3) & ~3));

    {
        const DevTables* tb = reinterpret_cast<const DevTables*>(p.tables);
        for (int i = tid; i < 256; i += 256) { sTw256[i] = tb->tw256[i]; sCoff[i] = tb->coffp[i]; }
        for (int i = tid; i < 257; i += 256) sTw512[i] = tb->tw512[i];
        for (int i = tid; i < 512; i += 256) sHann[i] = tb->hann[i];
        const ErbCSRView e = erb_view(p.erb_csr, p.nnz);
        for (int i = tid; i < 258; i += 256) sBinPtr[i] = e.bin_ptr[i];
        for (int i = tid; i < p.nnz; i += 256) {
            sBinBand[i] = e.bin_band[i];
            sBinW[i] = e.bin_w[i];
        }
        for (int i = tid; i < kFPB * 32; i += 256) {
            const int64_t t = h0 + (i >> 5);
            sEst[i] = (t < T) ? p.est[((int64_t)b * p.Tmax + t) * 32 + (i & 31)] : 0.f;
        }
    }
    const float* row = p.mic + (int64_t)b * p.ld;
    const bool aligned = ((p.ld & 3) == 0) && ((reinterpret_cast<uintptr_t>(p.mic) & 15) == 0);
    stage_hops(sWork, row, n, h0, p.cvals[b * 3 + 0], aligned);
    __syncthreads();
    const int g = tid >> 4, lb = tid & 15;
    float* scr = sWork + g * kGroupFloats;
    float2 v[16];
    load_frame(v, sWork, sHann, g, lb);
    __syncthreads();
    fft256<false>(v, lb, scr, sTw256);
    float2 xa[8], xb[8], x128;
    rfft_unpack(v, lb, scr, sTw512, xa, xb, x128);

    // ERB gains per bin and the complex gain on the mic spectrum (ERB.py:304-310)
    const float* est = sEst + g * 32;
    auto gain = [&](int k) {
        float acc = 0.f;
        for (int i = sBinPtr[k]; i < sBinPtr[k + 1]; ++i) acc += sBinW[i] * est[sBinBand[i]];
        return acc;
    };
    float2* s2 = reinterpret_cast<float2*>(scr);
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        const int k = lb + 16 * m;
        if (k == 0) {
            // DC / Nyquist: irfft ignores the imaginary parts
            const float g0 = gain(0), g256 = gain(256);
            const float s0 = g0 * xa[m].x, s256 = g256 * xb[m].x;
            s2[0] = make_float2(s0 + s256, s0 - s256);
        } else {
            const float ga = gain(k), gb = gain(256 - k);
            float2 Zk, Zmk;
            irfft_pair(cscale(xa[m], ga), cscale(xb[m], gb), sTw512[k], Zk, Zmk);
            s2[k] = Zk;
            s2[256 - k] = Zmk;
        }
    }
    if (lb == 0) {
        const float2 S = cscale(x128, gain(128));
        s2[128] = make_float2(2.f * S.x, -2.f * S.y);   // 2*conj(S[128])
    }
    wave_fence();
#pragma unroll
    for (int a = 0; a < 16; ++a) v[a] = s2[16 * a + lb];
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
    for (int e = tid; e < nh * kHop; e += 256) {
        const int i = e >> 8, r = e & 255;
        const float a = sWork[i * kGroupFloats + 256 + r];
        const float c = sWork[(i + 1) * kGroupFloats + r];
        orow[(h0 + i) * kHop + r] = (a + c) / sCoff[r] + 1e-9f;
    }
}

// --------------------------------------------------------------------------
// host-side launchers (called by aec_api.hip)
// --------------------------------------------------------------------------
hipError_t launch_moments(const float* mic, const float* ref, const float* near, int64_t ld,
                          const int64_t* lens, float* cvals, int B, int nsig, hipStream_t st) {
    hipLaunchKernelGGL(moments_kernel, dim3(B, nsig), dim3(256), 0, st, mic, ref, near, ld, lens, cvals);
    return hipGetLastError();
}

hipError_t launch_analysis(const AnalysisArgs& a, int B, hipStream_t st) {
    const dim3 grid((unsigned)((a.Tmax + kFPB - 1) / kFPB), B);
    hipLaunchKernelGGL(analysis_kernel, grid, dim3(256), analysis_smem_bytes(a.nnz), st, a);
    return hipGetLastError();
}

hipError_t launch_gru(const GruArgs& a, int B, hipStream_t st) {
    hipLaunchKernelGGL(gru_kernel, dim3(B), dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_synthesis(const SynthArgs& a, int B, hipStream_t st) {
    const int64_t nhop = a.Tmax - 1;
    if (nhop <= 0) return hipSuccess;
    const dim3 grid((unsigned)((nhop + kHopsOut - 1) / kHopsOut), B);
    hipLaunchKernelGGL(synthesis_kernel, grid, dim3(256), synthesis_smem_bytes(a.nnz), st, a);
    return hipGetLastError();
}

}  // namespace aec
