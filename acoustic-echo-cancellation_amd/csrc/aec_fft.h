// aec_fft.h — gfx950 device building blocks for the 512-point STFT / iSTFT.
//
// The reference computes its STFT as conv1d with a 514x512 windowed-DFT basis
// and its iSTFT as conv_transpose1d with the pinv basis
// (Stage2_lhm/scripts/network/attention_ccrn.py:8-101).  Both are exactly a
// windowed rFFT-512 / irFFT-512, so here a real 512-point
// frame is packed into a 256-point complex sequence z[m] = x[2m] + i x[2m+1]
// and transformed with a radix-16 x 16 FFT held in registers:
//
//   one 16-lane group per frame, lane b holds z[16a + b], a = 0..15
//   DFT16 over a (registers) -> twiddle W256^(b k1) -> LDS transpose (row stride
//   18 complex: conflict-free b64 writes / b128 reads) -> DFT16 over b
//   -> lane k1 holds Z[k1 + 16 k2].
//
// A wave (64 lanes) therefore transforms 4 frames at once with one LDS round
// trip; no block barrier is needed inside a transform (all lanes of a group
// live in one wave and LDS ops of a wave execute in order).
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

namespace aec {

constexpr int kWin = 512;
constexpr int kHop = 256;
constexpr int kBins = 257;
constexpr int kBands = 32;
constexpr int kGroupFloats = 576;   // per-frame LDS scratch: 16 rows x 36 floats

// Compile-time loop: f(std::integral_constant<int, I>) for I in [B, E).  Used
// where a register-array index must stay static (a loop holding convergent
// DPP intrinsics is not always fully unrolled, which would demote the array
// to scratch memory).
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 conjf2(float2 a) { return make_float2(a.x, -a.y); }
// Per-component select (a float2 struct select can be lowered to a
// stack-indexed load).
__device__ __forceinline__ float2 csel(bool c, float2 a, float2 b) {
    return make_float2(c ? a.x : b.x, c ? a.y : b.y);
}
__device__ __forceinline__ float2 cscale(float2 a, float s) { return make_float2(a.x * s, a.y * s); }

// a * (c + i*s)
__device__ __forceinline__ float2 crot(float2 a, float c, float s) {
    return make_float2(a.x * c - a.y * s, a.x * s + a.y * c);
}

// 4-point DFT in place.  Forward uses W4 = -i, inverse W4 = +i (unnormalised).
template <bool INV>
__device__ __forceinline__ void dft4(float2& a0, float2& a1, float2& a2, float2& a3) {
    const float2 t0 = cadd(a0, a2), t1 = csub(a0, a2);
    const float2 t2 = cadd(a1, a3), t3 = csub(a1, a3);
    a0 = cadd(t0, t2);
    a2 = csub(t0, t2);
    if (!INV) {   // t1 - i t3 , t1 + i t3
        a1 = make_float2(t1.x + t3.y, t1.y - t3.x);
        a3 = make_float2(t1.x - t3.y, t1.y + t3.x);
    } else {
        a1 = make_float2(t1.x - t3.y, t1.y + t3.x);
        a3 = make_float2(t1.x + t3.y, t1.y - t3.x);
    }
}

// Position of output index k after dft16: C[k] lives in v[kP(k)].
__host__ __device__ constexpr int kP(int k) { return 4 * (k & 3) + (k >> 2); }

// 16-point DFT in registers (radix 4 x 4).  Input v[a] = c[a] (natural order);
// output C[k] = sum_a c[a] W16^(+-a k) at v[kP(k)].
template <bool INV>
__device__ __forceinline__ void dft16(float2 (&v)[16]) {
    constexpr float C1 = 0.92387953251128674f;   // cos(pi/8)
    constexpr float S1 = 0.38268343236508978f;   // sin(pi/8)
    constexpr float R2 = 0.70710678118654752f;
    constexpr float sg = INV ? 1.f : -1.f;       // W16^m = cos(2pi m/16) + i*sg*sin(2pi m/16)
#pragma unroll
    for (int a0 = 0; a0 < 4; ++a0) dft4<INV>(v[a0], v[a0 + 4], v[a0 + 8], v[a0 + 12]);
    // v[a0 + 4 k0] = D[a0][k0]; twiddle by W16^(a0 k0)
    v[1 + 4] = crot(v[1 + 4], C1, sg * S1);     // W^1
    v[1 + 8] = crot(v[1 + 8], R2, sg * R2);     // W^2
    v[1 + 12] = crot(v[1 + 12], S1, sg * C1);   // W^3
    v[2 + 4] = crot(v[2 + 4], R2, sg * R2);     // W^2
    v[2 + 8] = INV ? make_float2(-v[2 + 8].y, v[2 + 8].x)          // * (+i)
                   : make_float2(v[2 + 8].y, -v[2 + 8].x);         // * (-i)   W^4
    v[2 + 12] = crot(v[2 + 12], -R2, sg * R2);  // W^6
    v[3 + 4] = crot(v[3 + 4], S1, sg * C1);     // W^3
    v[3 + 8] = crot(v[3 + 8], -R2, sg * R2);    // W^6
    v[3 + 12] = crot(v[3 + 12], -C1, -sg * S1); // W^9 = cos(9pi/8) + i sg sin(9pi/8)
#pragma unroll
    for (int k0 = 0; k0 < 4; ++k0) dft4<INV>(v[4 * k0], v[4 * k0 + 1], v[4 * k0 + 2], v[4 * k0 + 3]);
}

__device__ __forceinline__ void wave_fence() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// 256-point complex FFT for one 16-lane group.
//   in : v[a] = z[16a + lb]
//   out: v[kP(k2)] = Z[lb + 16 k2]   (unnormalised, sign per INV)
// scr: this group's LDS scratch (>= 16*36 floats, 16-B aligned).
// twT: LDS table twT[k1*16 + lb] = W256^(lb k1) (lane-major: the 16 lanes of a
//      group read 16 consecutive entries, conflict-free; a gather
//      tw[(lb*k1) & 255] would be 2-4-way conflicted for k1 = 4, 8, 12).
template <bool INV>
__device__ __forceinline__ void fft256_scalar(float2 (&v)[16], int lb, float* scr, const float2* twT) {
    dft16<INV>(v);
    float2* s2 = reinterpret_cast<float2*>(scr);
    // all 15 twiddle reads first: interleaved with the transpose writes (which
    // may alias as far as the compiler knows) each read would wait for the
    // previous write, exposing the LDS latency 15 times.  (A packed-FP32
    // variant of these helpers was measured slower: 0.285 vs 0.245 ms for
    // the analysis kernel — more v_mov for operand pairs and a stack temp.)
    float2 w[15];
    static_for<0, 15>([&](auto ii) {
        constexpr int i = decltype(ii)::value;
        w[i] = twT[(i + 1) * 16 + lb];
    });
    s2[lb] = v[kP(0)];
    static_for<0, 15>([&](auto ii) {
        constexpr int i = decltype(ii)::value;
        float2 t = w[i];
        if (INV) t.y = -t.y;
        s2[(i + 1) * 18 + lb] = cmul(v[kP(i + 1)], t);
    });
    wave_fence();
    const float4* s4 = reinterpret_cast<const float4*>(scr) + lb * 9;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const float4 t = s4[q];
        v[2 * q] = make_float2(t.x, t.y);
        v[2 * q + 1] = make_float2(t.z, t.w);
    }
    wave_fence();
    dft16<INV>(v);
}

// ---------------------------------------------------------------------------
// Packed-FP32 FFT core (AEC_FFT_PK, default).  A complex value is one
// 64-bit VGPR pair, so every complex add / sub is ONE v_pk_add_f32 and every
// complex rotation is one v_pk_mul_f32 + one v_pk_fma_f32; the lane swaps and
// sign flips of the radix-4 butterfly (t1 -/+ i t3) and of the twiddle
// product ride on the VOP3P op_sel / neg modifiers instead of extra VALU.
// fft256: 381 -> 231 VALU per call (gfx950 ISA count); the NLMS analysis
// kernel 3531 -> 3045 static VALU, 1.5-2 % faster (the transforms share the
// SIMDs with LDS-latency-bound work, so the issue savings only partly show).
// The arithmetic is the scalar core's up to fma contraction (~1 ulp per stage).
// ---------------------------------------------------------------------------
typedef float pf2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ pf2 pswap(pf2 a) { return __builtin_shufflevector(a, a, 1, 0); }

// t1 - i t3 = (t1.x + t3.y, t1.y - t3.x)
__device__ __forceinline__ pf2 p_sub_i(pf2 t1, pf2 t3) {
    pf2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_hi:[0,1]" : "=v"(r) : "v"(t1), "v"(t3));
    return r;
}
// t1 + i t3 = (t1.x - t3.y, t1.y + t3.x)
__device__ __forceinline__ pf2 p_add_i(pf2 t1, pf2 t3) {
    pf2 r;
    asm("v_pk_add_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[1,0] neg_lo:[0,1]" : "=v"(r) : "v"(t1), "v"(t3));
    return r;
}
// x * t (CONJ: x * conj(t)) for a twiddle t loaded as a pair
template <bool CONJ>
__device__ __forceinline__ pf2 p_cmul(pf2 x, pf2 t) {
    pf2 m, r;
    asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[1,0]" : "=v"(m) : "v"(x), "v"(t));      // (x.x t.x, x.y t.x)
    if (!CONJ)   // (x.x t.x - x.y t.y, x.y t.x + x.x t.y)
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_lo:[0,1,0]"
            : "=v"(r) : "v"(x), "v"(t), "v"(m));
    else         // (x.x t.x + x.y t.y, x.y t.x - x.x t.y)
        asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_hi:[0,1,0]"
            : "=v"(r) : "v"(x), "v"(t), "v"(m));
    return r;
}
// a * (c + i s), c and s compile-time
__device__ __forceinline__ pf2 p_rot(pf2 a, float c, float sn) {
    return __builtin_elementwise_fma(pswap(a), pf2{-sn, sn}, a * pf2{c, c});
}

template <bool INV>
__device__ __forceinline__ void p_dft4(pf2& a0, pf2& a1, pf2& a2, pf2& a3) {
    const pf2 t0 = a0 + a2, t1 = a0 - a2, t2 = a1 + a3, t3 = a1 - a3;
    a0 = t0 + t2;
    a2 = t0 - t2;
    if (!INV) { a1 = p_sub_i(t1, t3); a3 = p_add_i(t1, t3); }
    else      { a1 = p_add_i(t1, t3); a3 = p_sub_i(t1, t3); }
}

template <bool INV>
__device__ __forceinline__ void p_dft16(pf2 (&v)[16]) {
    constexpr float C1 = 0.92387953251128674f;
    constexpr float S1 = 0.38268343236508978f;
    constexpr float R2 = 0.70710678118654752f;
    constexpr float sg = INV ? 1.f : -1.f;
#pragma unroll
    for (int a0 = 0; a0 < 4; ++a0) p_dft4<INV>(v[a0], v[a0 + 4], v[a0 + 8], v[a0 + 12]);
    v[1 + 4] = p_rot(v[1 + 4], C1, sg * S1);
    v[1 + 8] = p_rot(v[1 + 8], R2, sg * R2);
    v[1 + 12] = p_rot(v[1 + 12], S1, sg * C1);
    v[2 + 4] = p_rot(v[2 + 4], R2, sg * R2);
    v[2 + 8] = INV ? p_add_i(pf2{0.f, 0.f}, v[2 + 8]) : p_sub_i(pf2{0.f, 0.f}, v[2 + 8]);   // * (+-i)
    v[2 + 12] = p_rot(v[2 + 12], -R2, sg * R2);
    v[3 + 4] = p_rot(v[3 + 4], S1, sg * C1);
    v[3 + 8] = p_rot(v[3 + 8], -R2, sg * R2);
    v[3 + 12] = p_rot(v[3 + 12], -C1, -sg * S1);
#pragma unroll
    for (int k0 = 0; k0 < 4; ++k0) p_dft4<INV>(v[4 * k0], v[4 * k0 + 1], v[4 * k0 + 2], v[4 * k0 + 3]);
}

template <bool INV>
__device__ __forceinline__ void fft256_packed(float2 (&v)[16], int lb, float* scr, const float2* twT) {
    pf2 u[16];
#pragma unroll
    for (int a = 0; a < 16; ++a) u[a] = pf2{v[a].x, v[a].y};
    p_dft16<INV>(u);
    pf2* s2 = reinterpret_cast<pf2*>(scr);
    const pf2* tw = reinterpret_cast<const pf2*>(twT);
    pf2 w[15];
    static_for<0, 15>([&](auto ii) {
        constexpr int i = decltype(ii)::value;
        w[i] = tw[(i + 1) * 16 + lb];
    });
    s2[lb] = u[kP(0)];
    static_for<0, 15>([&](auto ii) {
        constexpr int i = decltype(ii)::value;
        s2[(i + 1) * 18 + lb] = p_cmul<INV>(u[kP(i + 1)], w[i]);
    });
    wave_fence();
    const pf2* sr = reinterpret_cast<const pf2*>(scr) + lb * 18;
#pragma unroll
    for (int q = 0; q < 16; ++q) u[q] = sr[q];
    wave_fence();
    p_dft16<INV>(u);
#pragma unroll
    for (int a = 0; a < 16; ++a) v[a] = make_float2(u[a].x, u[a].y);
}

#ifndef AEC_FFT_PK
#define AEC_FFT_PK 1
#endif
#ifndef AEC_FFT_PK_INV
#define AEC_FFT_PK_INV 1   // the inverse on the packed core too (0: scalar inverse, A/B builds)
#endif
template <bool INV>
__device__ __forceinline__ void fft256(float2 (&v)[16], int lb, float* scr, const float2* twT) {
    // both directions on the packed core: in round 2 the packed inverse made the fused GRU +
    // synthesis kernel 4 % slower (one recurrence wave per block shared the SIMDs with the
    // synthesis waves); with two streams per block and the overlap-add on the recurrence waves
    // it shortens the synthesis waves' tick share (9.2-9.7 k -> 8.9-9.4 k cycles) and the kernel
    // by 1-2 % (profiles/r05_notes.md, r05m / r05t).  Every synthesis path runs this same inverse
    // (the fused / separate / streaming kernels are tested bit-identical)
    if constexpr (AEC_FFT_PK && (!INV || AEC_FFT_PK_INV)) fft256_packed<INV>(v, lb, scr, twT);
    else fft256_scalar<INV>(v, lb, scr, twT);
}

// Cross-lane partner within each 16-lane row: out[lb] = x[(16 - lb) & 15]
// (row_mirror then row_ror:1, two DPP moves, no LDS).  Lane 0 receives its
// own value; callers patch lane 0.
__device__ __forceinline__ float mirror16(float x) {
    const int y = __builtin_amdgcn_mov_dpp(__float_as_int(x), 0x140, 0xF, 0xF, false);   // row_mirror
    return __int_as_float(__builtin_amdgcn_mov_dpp(y, 0x121, 0xF, 0xF, false));          // row_ror:1
}
__device__ __forceinline__ float2 mirror16(float2 x) { return make_float2(mirror16(x.x), mirror16(x.y)); }

// Forward real-FFT unpack for one pair (k, 256-k), 1 <= k <= 127:
//   A = Z[k], Bz = Z[256-k], w = W512^k  ->  X[k], X[256-k]
__device__ __forceinline__ void rfft_pair(float2 A, float2 Bz, float2 w, float2& Xk, float2& Xmk) {
    const float2 Bc = conjf2(Bz);
    const float2 Fe = cscale(cadd(A, Bc), 0.5f);
    const float2 D = cscale(csub(A, Bc), 0.5f);
    const float2 Fo = make_float2(D.y, -D.x);          // -i * D
    const float2 t = cmul(w, Fo);
    Xk = cadd(Fe, t);
    Xmk = conjf2(csub(Fe, t));
}

// Inverse real-FFT pack for one pair (k, 256-k): S[k], S[256-k] -> 2*Z'[k],
// 2*Z'[256-k] such that IDFT256(2 Z') = 512 * (x[2m] + i x[2m+1]).
__device__ __forceinline__ void irfft_pair(float2 Sk, float2 Smk, float2 w, float2& Zk, float2& Zmk) {
    const float2 Bc = conjf2(Smk);
    const float2 Fe = cadd(Sk, Bc);
    const float2 Fo = cmul(csub(Sk, Bc), conjf2(w));
    Zk = make_float2(Fe.x - Fo.y, Fe.y + Fo.x);                       // Fe + i Fo
    Zmk = make_float2(Fe.x + Fo.y, -Fe.y + Fo.x);                     // conj(Fe) + i conj(Fo)
}

}  // namespace aec
