// aec_frame.h — per-frame device pieces shared by the batch kernels
// (aec_kernels.hip, aec_gru.hip) and the fused streaming step
// (aec_stream.hip): magnitudes, the balanced ERB projection, the NLMS bin
// recursion, spectrum row packing, the synthesis frame (gains -> irFFT ->
// window) and the GRU gate nonlinearities.  One definition, so a streamed
// hop runs the same arithmetic as the batch path.
#pragma once
#include <hip/hip_runtime.h>

#include "aec_fft.h"

namespace aec {

// |X| = sqrt(re^2 + im^2 + 1e-9) (ERB.py:277-279).  The argument is >= 1e-9,
// never denormal, so the hardware v_sqrt_f32 (<= 1 ulp) needs no IEEE fix-up.
__device__ __forceinline__ float mag(float2 x) {
    return __builtin_amdgcn_sqrtf(fmaf(x.x, x.x, fmaf(x.y, x.y, 1e-9f)));
}

// Balanced ERB projection of one frame's magnitudes (scr[k ^ sw], k = 0..256)
// onto the 32 bands (ERB.py:282-284): L scheduled entries per lane, three
// partial sums, pieces of split bands combined through comb.  fo = the
// frame's 32-float feature row, or null (frame beyond the stream: compute
// nothing visible).  Leaves the wave fenced.
template <int PART = 512>
__device__ __forceinline__ void erb_project(float* scr, const float4* sSched, const int2* sComb, int L, int lb,
                                            int sw, float* fo) {
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
    float* part = scr + PART;                      // 48 partials after the magnitudes
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

// Two frames' ERB projections with the same lane schedule in one pass (rows sa, sb with the same
// swizzle sw): each schedule entry is read once for both gathers, so a wave projecting two frames
// per tick (K2n's ref waves: mic_erb of chunk c-2 and ref_erb of chunk c) halves its schedule reads
// and dependent LDS round trips.  Per frame the same entries and FMA order as erb_project (the same
// bits).  pa / pb: each frame's 48 partials; foa / fob: feature rows or null.
__device__ __forceinline__ void erb_project2(const float* sa, float* pa, float* foa, const float* sb, float* pb,
                                             float* fob, const float4* sSched, const int2* sComb, int L, int lb,
                                             int sw) {
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, b0 = 0.f, b1 = 0.f, b2 = 0.f;
    for (int e = 0; e < L; e += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const float4 en = sSched[(e + u) * 16 + lb];
            const int ix = __float_as_int(en.x) ^ sw;
            const float ma = sa[ix], mb = sb[ix];
            a0 = fmaf(en.y, ma, a0);
            a1 = fmaf(en.z, ma, a1);
            a2 = fmaf(en.w, ma, a2);
            b0 = fmaf(en.y, mb, b0);
            b1 = fmaf(en.z, mb, b1);
            b2 = fmaf(en.w, mb, b2);
        }
    }
    pa[3 * lb + 0] = a0;
    pa[3 * lb + 1] = a1;
    pa[3 * lb + 2] = a2;
    pb[3 * lb + 0] = b0;
    pb[3 * lb + 1] = b1;
    pb[3 * lb + 2] = b2;
    wave_fence();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const int band = lb + 16 * h;
        const int2 cb = sComb[band];
        if (foa) foa[band] = pa[cb.x] + (cb.y >= 0 ? pa[cb.y] : 0.f);
        if (fob) fob[band] = pb[cb.x] + (cb.y >= 0 ? pb[cb.y] : 0.f);
    }
    wave_fence();
}

// Packed-FP32 complex helpers for the recursion: a complex value is a
// float2 vector, so the products below map to v_pk_mul_f32 / v_pk_fma_f32
// (two lanes of arithmetic per instruction slot).
typedef float v2f __attribute__((ext_vector_type(2)));
__device__ __forceinline__ v2f vfma(v2f a, v2f b, v2f c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ v2f vsplat(float a) { return v2f{a, a}; }
__device__ __forceinline__ v2f vrot(v2f a) { return v2f{-a.y, a.x}; }       // i * a

// One lane's NLMS.  A lane runs either one complex bin or, on the lane that
// owns row slot 0, the two real bins 0 and 256 side by side (x, y halves).
// Both cases are the same scalar instruction stream over per-tap operands
// derived once when R[t] enters the history (hist()):
//   complex bin:  p1 = r.x, p2 = -r.y, p4 = r.x      dual real:  p1 = r.x, p2 = 0, p4 = r.y
//   y.x = sum_l w.x p1 + w.y p2        y.y = sum_l w.y p4 - w.x p2
//         (complex: W R;  dual: (w.x r.x, w.y r.y))
//   W.x += ge.x p1 - ge.y p2           W.y += ge.y p4 + ge.x p2
//         (complex: W += ge conj(R);  dual: per half)
//   q  = (p1^2 + p2^2, p4^2 + p2^2)    (|R|^2 in both halves / (r.x^2, r.y^2))
// with ge = e * mu / (P + delta) per half.  Plain f32 FMAs: on gfx950 a
// v_pk_fma_f32 costs at least two v_fma_f32 issue slots, so the packed form of
// this recursion (one complex value per VGPR pair, operand masks) issued ~100
// slot-equivalents per step against ~60 here, on a chain of dependent packed
// ops; the recursion's waves share their SIMDs with the transforms.
template <int TAPS>
struct NlmsBin {
    float2 w[TAPS];
    float p1[TAPS], p2[TAPS], p4[TAPS];   // operands of R[t], R[t-1], ...
    float qx[TAPS], qy[TAPS];             // per-half |R|^2 of the same entries
    float2 p;                             // smoothed power per half
    bool dual;
    __device__ __forceinline__ void reset(bool dual_) {
        dual = dual_;
#pragma unroll
        for (int l = 0; l < TAPS; ++l) {
            w[l] = make_float2(0.f, 0.f);
            p1[l] = p2[l] = p4[l] = qx[l] = qy[l] = 0.f;
        }
        p = make_float2(0.f, 0.f);
    }
    // history slot l <- the operands of far-end bin value r (step() uses the
    // same expressions for slot 0; the streaming steps restore their saved
    // history through this)
    __device__ __forceinline__ void hist(int l, float2 r) {
        p1[l] = r.x;
        p2[l] = dual ? 0.f : -r.y;
        p4[l] = dual ? r.y : r.x;
        const float s = p2[l] * p2[l];
        qx[l] = fmaf(p1[l], p1[l], s);
        qy[l] = fmaf(p4[l], p4[l], s);
    }
    // One frame: returns E = D - sum_l W[l] R[t-l] and adapts W.
    __device__ __forceinline__ float2 step(float2 d, float2 r, float mu, float beta, float delta) {
#pragma unroll
        for (int l = TAPS - 1; l >= 1; --l) {
            p1[l] = p1[l - 1];
            p2[l] = p2[l - 1];
            p4[l] = p4[l - 1];
            qx[l] = qx[l - 1];
            qy[l] = qy[l - 1];
        }
        hist(0, r);
        // y: two partial chains per half (taps [0, H) and [H, TAPS)), then one add
        constexpr int H = (TAPS + 1) / 2;
        float yx[2], yy[2], px[2], py[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int l0 = h ? H : 0, l1 = h ? TAPS : H;
            yx[h] = yy[h] = px[h] = py[h] = 0.f;
#pragma unroll
            for (int l = l0; l < l1; ++l) {
                yx[h] = fmaf(w[l].x, p1[l], fmaf(w[l].y, p2[l], yx[h]));
                yy[h] = fmaf(w[l].y, p4[l], fmaf(-w[l].x, p2[l], yy[h]));
                px[h] += qx[l];
                py[h] += qy[l];
            }
        }
        const float ex = d.x - (yx[0] + yx[1]);
        const float ey = d.y - (yy[0] + yy[1]);
        p.x = fmaf(beta, p.x, (1.f - beta) * (px[0] + px[1]));
        p.y = fmaf(beta, p.y, (1.f - beta) * (py[0] + py[1]));
        const float gx = ex * (__builtin_amdgcn_rcpf(p.x + delta) * mu);
        const float gy = ey * (__builtin_amdgcn_rcpf(p.y + delta) * mu);
#pragma unroll
        for (int l = 0; l < TAPS; ++l) {
            w[l].x = fmaf(gx, p1[l], fmaf(-gy, p2[l], w[l].x));
            w[l].y = fmaf(gy, p4[l], fmaf(gx, p2[l], w[l].y));
        }
        return make_float2(ex, ey);
    }
};

__device__ __forceinline__ void mags_to_scr(float* scr, int lb, int sw, const float2 (&xa)[8], const float2 (&xb)[8],
                                            float2 x128) {
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        const int kk = lb + 16 * m;
        scr[kk ^ sw] = mag(xa[m]);
        scr[(kk == 0 ? 256 : 256 - kk) ^ sw] = mag(xb[m]);
    }
    if (lb == 0) scr[128 ^ sw] = mag(x128);
}

__device__ __forceinline__ void row_to_scr(float* scr, int lb, const float2 (&xa)[8], const float2 (&xb)[8],
                                           float2 x128) {
    float2* row = reinterpret_cast<float2*>(scr);
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        const int kk = lb + 16 * m;
        if (kk == 0) {
            row[0] = make_float2(xa[0].x, xb[0].x);                   // (X[0], X[256]), both real
        } else {
            row[kk] = xa[m];
            row[256 - kk] = xb[m];
        }
    }
    if (lb == 0) row[128] = x128;
}

// A spectrum row (256 float2, slot 0 = (X[0], X[256])) back to the unpacked
// pairs rfft_unpack produces: xa[m] = X[k], xb[m] = X[256-k], k = lb + 16 m
// (lane 0, m = 0: X[0] / X[256] with zero imaginary parts), x128 = X[128].
// ok == false yields zeros (a frame past the stream end).
__device__ __forceinline__ void row_to_pairs(const float2* row, int lb, bool ok, float2 (&xa)[8], float2 (&xb)[8],
                                             float2& x128) {
    const float2 z = make_float2(0.f, 0.f);
#pragma unroll
    for (int m = 0; m < 8; ++m) {
        const int kk = lb + 16 * m;
        const float2 a = ok ? row[kk] : z;
        const float2 c = ok ? row[(256 - kk) & 255] : z;
        xa[m] = kk == 0 ? make_float2(a.x, 0.f) : a;
        xb[m] = kk == 0 ? make_float2(a.y, 0.f) : c;
    }
    x128 = ok ? row[128] : z;
}

__device__ __forceinline__ void synth_pack(const float2 (&xa)[8], const float2 (&xb)[8], float2 x128,
                                           const float* est, const float4* sBin, const float2* sTw512, int lb,
                                           float2 (&v)[16]) {
    auto gain = [&](int kk) {
        const float4 e = sBin[kk];
        return e.y * est[__float_as_int(e.x)] + e.w * est[__float_as_int(e.z)];
    };
    // inverse pack: lane lb forms 2Z'[k] and 2Z'[256-k] for k = lb + 16 m; the
    // inverse FFT wants v[a] = 2Z'[16a + lb]: a <= 7 is this lane's own Zk[a],
    // a >= 8 is Zmk[15-a] of lane (16-lb)&15 (DPP), lane 0 patched.
    float2 Zk[8], Zmk[8];
    static_for<0, 8>([&](auto mi) {
        constexpr int m = decltype(mi)::value;
        const int kk = lb + 16 * m;
        // kk == 0 (lane 0, m = 0): DC / Nyquist, irfft ignores their imaginary parts;
        // gain(256 - 0) indexes bin 256 = Nyquist, as required
        const float ga = gain(kk), gb = gain(256 - kk);
        float2 zk, zmk;
        irfft_pair(cscale(xa[m], ga), cscale(xb[m], gb), sTw512[kk], zk, zmk);
        const float s0 = ga * xa[m].x, s256 = gb * xb[m].x;
        Zk[m] = csel(kk == 0, make_float2(s0 + s256, s0 - s256), zk);
        Zmk[m] = csel(kk == 0, Zk[m], zmk);
    });
    float2 z128 = make_float2(0.f, 0.f);
    if (lb == 0) {
        const float2 S = cscale(x128, gain(128));
        z128 = make_float2(2.f * S.x, -2.f * S.y);   // 2*conj(S[128])
    }
#pragma unroll
    for (int a = 0; a < 8; ++a) v[a] = Zk[a];
    static_for<8, 16>([&](auto ai) {
        constexpr int a = decltype(ai)::value;
        const float2 mir = mirror16(Zmk[15 - a]);
        v[a] = csel(lb != 0, mir, a == 8 ? z128 : Zmk[(16 - a) & 7]);
    });
}

// irFFT-256 of the packed frame, window and 1/512 -> scr[0..511] (natural order).
// PRE: sHann holds hann / 512 (exact: a power-of-two scale of normal values), so the
// product is the same float with one multiply instead of two.
template <bool PRE = false>
__device__ __forceinline__ void synth_fft(float2 (&v)[16], const float2* sTwT, const float* sHann, float* scr, int lb) {
    fft256<true>(v, lb, scr, sTwT);
    // v[kP(m2)] = 512 * (x[2m] + i x[2m+1]), m = lb + 16 m2 ; window + 1/512
    float2* s2 = reinterpret_cast<float2*>(scr);
    const float2* h2 = reinterpret_cast<const float2*>(sHann);
#pragma unroll
    for (int m2 = 0; m2 < 16; ++m2) {
        const float2 z = v[kP(m2)];
        const float2 w = h2[lb + 16 * m2];
        if constexpr (PRE) s2[lb + 16 * m2] = make_float2(z.x * w.x, z.y * w.y);
        else s2[lb + 16 * m2] = make_float2(z.x * (w.x * (1.f / 512.f)), z.y * (w.y * (1.f / 512.f)));
    }
}

// irFFT-256 of the packed frame without the window: scr[0..511] = 512 x (time samples), natural
// order; the overlap-add applies hann / 512 (aec_gru_synth.hip, AEC_OLA_WIN)
__device__ __forceinline__ void synth_fft_raw(float2 (&v)[16], const float2* sTwT, float* scr, int lb) {
    fft256<true>(v, lb, scr, sTwT);
    float2* s2 = reinterpret_cast<float2*>(scr);
#pragma unroll
    for (int m2 = 0; m2 < 16; ++m2) s2[lb + 16 * m2] = v[kP(m2)];
}

// Synthesis of one frame by its 16-lane group: per-bin ERB gain
// g[k] = sum_j est_erb[j] erb[k][j] over the <= 2 bands covering bin k
// (ERB.py:306-307) applied to the spectrum (:309-310), inverse real pack,
// irFFT-256, Hann window and 1/512 (attention_ccrn.py:82-91).  Leaves the 512
// windowed time samples in scr[0..511] (natural order) for the overlap-add.
//   est : the frame's 32 est_erb values;  sBin: float4[257] transpose table
__device__ __forceinline__ void synth_frame(const float2 (&xa)[8], const float2 (&xb)[8], float2 x128,
                                            const float* est, const float4* sBin, const float2* sTw512,
                                            const float2* sTwT, const float* sHann, float* scr, int lb) {
    float2 v[16];
    synth_pack(xa, xb, x128, est, sBin, sTw512, lb, v);
    synth_fft(v, sTwT, sHann, scr, lb);
}

// c = mean(x)/std(x, unbiased) from the partials (ERB.py:254-256).
__device__ __forceinline__ float norm_scalar(const double2* __restrict__ mom, int b, int s, int64_t n) {
    constexpr int kMomChunks = 8;   // aec_launch.h
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

// GRU gate nonlinearities (nn.GRU, ERB.py:213): fast exp / reciprocal.
__device__ __forceinline__ float sigmoidf_(float x) {
    return __builtin_amdgcn_rcpf(1.f + __expf(-x));
}
__device__ __forceinline__ float tanhf_(float x) {
    return 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __expf(2.f * x));
}

// ---------------------------------------------------------------------------
// GRU cell pieces (nn.GRU(64, 32) gate order r, z, n; ERB.py:213, 293) and
// the head (linear1 / relu / linear2 / sigmoid, ERB.py:295-301), shared by
// gru_kernel, gru_synth_kernel and stream_step_kernel so the three run the
// same accumulation order (bit-identical results).
// ---------------------------------------------------------------------------
typedef float f2v __attribute__((ext_vector_type(2)));

// gi = W_ih[row] . x + bias (x: 64 floats in LDS, 16-B aligned)
__device__ __forceinline__ float gru_gi(const float (&wih)[64], const float* x, float gbias) {
    const float4* x4 = reinterpret_cast<const float4*>(x);
    f2v a0 = {0.f, 0.f}, a1 = {0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const float4 xv = x4[q];
        a0 = __builtin_elementwise_fma(f2v{wih[4 * q], wih[4 * q + 1]}, f2v{xv.x, xv.y}, a0);
        a1 = __builtin_elementwise_fma(f2v{wih[4 * q + 2], wih[4 * q + 3]}, f2v{xv.z, xv.w}, a1);
    }
    const f2v s2 = a0 + a1;
    return gbias + (s2.x + s2.y);
}

// One recurrence step on a wave: lane l owns unit j = l & 31 and the k-half
// kh = l >> 5 of rows r_j, z_j, n_j of W_hh (wrz[k] = (W_r[j][16kh+k],
// W_z[j][16kh+k]), wn[i] = W_n[j][16kh+2i .. +1]); hb = h_{t-1} (32 floats in
// LDS); the halves' partial dots meet through v_permlane32_swap.  Returns h_t[j]
// (identical in both halves).
__device__ __forceinline__ float gru_step(const f2v (&wrz)[16], const f2v (&wn)[8], const float* hb, int kh, float gr,
                                         float gz, float gn, float bhn, float hprev) {
    const float4* h4 = reinterpret_cast<const float4*>(hb + 16 * kh);
    const float4 q0 = h4[0], q1 = h4[1], q2 = h4[2], q3 = h4[3];
    const float hk[16] = {q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w,
                          q2.x, q2.y, q2.z, q2.w, q3.x, q3.y, q3.z, q3.w};
    f2v arz[4] = {f2v{0.f, 0.f}, f2v{0.f, 0.f}, f2v{0.f, 0.f}, f2v{0.f, 0.f}};
    f2v an[2] = {f2v{0.f, 0.f}, f2v{0.f, 0.f}};
#pragma unroll
    for (int k = 0; k < 16; ++k) arz[k & 3] = __builtin_elementwise_fma(wrz[k], f2v{hk[k], hk[k]}, arz[k & 3]);
#pragma unroll
    for (int i = 0; i < 8; ++i) an[i & 1] = __builtin_elementwise_fma(wn[i], f2v{hk[2 * i], hk[2 * i + 1]}, an[i & 1]);
    const f2v rz = (arz[0] + arz[1]) + (arz[2] + arz[3]);
    const f2v n2 = an[0] + an[1];
    const float pr = rz.x, pz = rz.y, pn = n2.x + n2.y;
    // v_permlane32_swap: lanes 32..63 of vdst <-> lanes 0..31 of vsrc, so the
    // other half's value is res[1] in lanes 0..31 and res[0] in lanes 32..63
    const auto sr = __builtin_amdgcn_permlane32_swap(__float_as_uint(pr), __float_as_uint(pr), false, false);
    const auto sz = __builtin_amdgcn_permlane32_swap(__float_as_uint(pz), __float_as_uint(pz), false, false);
    const auto sn = __builtin_amdgcn_permlane32_swap(__float_as_uint(pn), __float_as_uint(pn), false, false);
    const float rdot = pr + __uint_as_float(kh ? sr[0] : sr[1]);
    const float zdot = pz + __uint_as_float(kh ? sz[0] : sz[1]);
    const float ndot = pn + __uint_as_float(kh ? sn[0] : sn[1]);
    const float r = sigmoidf_(gr + rdot);
    const float z = sigmoidf_(gz + zdot);
    const float nn = tanhf_(gn + r * (ndot + bhn));
    return (1.f - z) * nn + z * hprev;
}

// Head of unit j for one frame, by a group of 32 lanes (lane j of the group):
// o = relu(W1[j] . [h, mic_erb] + b1) through the group's 32-float LDS row,
// mask = sigmoid(W2[j] . o + b2).  h, mic: 32 floats each in LDS (16-B aligned).
__device__ __forceinline__ float head_mask(const float (&w1)[64], const float (&w2)[32], float b1j, float b2j,
                                          const float* h, const float* mic, float* orow, int j) {
    const float4* h4 = reinterpret_cast<const float4*>(h);
    const float4* m4 = reinterpret_cast<const float4*>(mic);
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
    orow[j] = fmaxf(b1j + (s1.x + s1.y), 0.f);
    wave_fence();
    const float4* o4 = reinterpret_cast<const float4*>(orow);
    f2v c0 = {0.f, 0.f}, c1 = {0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const float4 ov = o4[q];
        c0 = __builtin_elementwise_fma(f2v{w2[4 * q], w2[4 * q + 1]}, f2v{ov.x, ov.y}, c0);
        c1 = __builtin_elementwise_fma(f2v{w2[4 * q + 2], w2[4 * q + 3]}, f2v{ov.z, ov.w}, c1);
    }
    wave_fence();                                   // the row is reused by the group's next frame
    const f2v s2 = c0 + c1;
    return sigmoidf_(b2j + (s2.x + s2.y));
}

}  // namespace aec
