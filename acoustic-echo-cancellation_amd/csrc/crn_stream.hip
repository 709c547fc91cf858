// crn_stream.hip — fused kernels of the DCCRN per-hop step (aec_crn_stream_step).
//
// At one frame per stream the step's launches are latency chains: a launch
// costs ~5 us even when its work is a few hundred thousand MACs.  The front of
// the hop (the frame [prev hop | cur hop] of mic and far -> rFFT-512 ->
// FD-NLMS step -> X0 -> the narrow encoder levels) therefore runs as ONE
// launch, one block per stream, with the intermediate maps in LDS:
//
//   ConvSTFT          dccrn.py:45-52    (aec_fft.h / aec_stft.h transforms)
//   FD-NLMS           aec::NlmsBin       (build-defined, aec_hip.h)
//   encoder 0 .. n-1  dccrn2.py:49-62 / dccrn.py:463-478: ComplexConv2d k=(5,1)
//                     s=(2,1) p=(2,0) + folded (Complex)BatchNorm + PReLU, as
//                     implicit GEMMs on v_mfma_f32_16x16x32_bf16
//
// The back of the hop (the last three decoder levels with their skips, the
// mask, the masked spectrum's irFFT-512 and the overlap-add) is a second
// launch of the same form (crn_stream_dec_kernel):
//
//   decoder cl = 3..1 dccrn2.py:83-111 / dccrn.py:480-509: ComplexConvTranspose2d
//                     on complex_cat(dec, enc skip) (both output parities per GEMM)
//   mask + ConviSTFT  dccrn2.py:185-215, dccrn.py:80-100
//
// Each level is the batch path's GEMM restated: the same packed weights, the
// same 32-k chunks accumulated in the same order from zero, the same epilogue
// (v >= 0 ? v : alpha v, then bf16), so its outputs equal the row-GEMM
// kernel's, and the transforms are the batch kernels' code
// (tests/test_gpu_crn.py::test_fused_stream_bit_exact).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "aec_fft.h"
#include "aec_frame.h"
#include "aec_stft.h"
#include "aec_tables.h"
#include "crn_gemm.h"
#include "crn_launch.h"

namespace crn {

#ifdef AEC_STREAM_PROF
// timing experiments only (tools/stream_prof.py): s_memtime at the phase boundaries of block 0 of
// the fused kernels (wave 0, lane 0): [kernel 0 = enc, 1 = dec][phase]
__device__ unsigned long long g_sprof[2][16];
#define SPROF(kern, ph)                                                                               \
    do {                                                                                              \
        if (blockIdx.x == 0 && threadIdx.x == 0) g_sprof[kern][ph] = __builtin_amdgcn_s_memtime();   \
    } while (0)
#else
#define SPROF(kern, ph) do {} while (0)
#endif


namespace {

constexpr int kMapElems = 2048;

// block barrier that drains LDS only: the global stores of the level outputs (read by a later
// launch) and the register loads of weight fragments stay in flight across it
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}    // bf16 elements of one level's output map (Fo x N = 8 tiles of 16 x 16)

// X0 bin k (1..256) as 8 bf16: (mic.re, far.re, mic.im, far.im, 0, 0, 0, 0) (dccrn.py:559-561)
__device__ __forceinline__ void x0_put(bf16_t* x0, int k, float2 m, float2 f) {
    u32x4 v;
    v[0] = (uint32_t)f2bf(m.x) | ((uint32_t)f2bf(f.x) << 16);
    v[1] = (uint32_t)f2bf(m.y) | ((uint32_t)f2bf(f.y) << 16);
    v[2] = 0u;
    v[3] = 0u;
    *reinterpret_cast<u32x4*>(x0 + (k - 1) * 8) = v;
}

}  // namespace

template <int TAPS>
__global__ __launch_bounds__(256) void crn_stream_enc_kernel(StreamEncArgs p) {
    __shared__ __attribute__((aligned(16))) float sTab[256 * 2 + 258 * 2 + 512];
    __shared__ __attribute__((aligned(16))) float sGrp[2][aec::kGroupFloats];
    __shared__ __attribute__((aligned(16))) float2 sRow[2][256];
    __shared__ __attribute__((aligned(16))) bf16_t sX0[256 * 8];
    __shared__ __attribute__((aligned(16))) bf16_t sMap[2][kMapElems];
    float2* sTwT = reinterpret_cast<float2*>(sTab);
    float2* sTw512 = sTwT + 256;
    float* sHann = reinterpret_cast<float*>(sTw512 + 258);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int b = blockIdx.x;
    SPROF(0, 0);

    // 1. every independent load first: the two hops of both signals (one float4 per thread;
    //    the current hop also saved to the ring), the tables, the NLMS state and the weight
    //    fragments of every level
    {
        const int s = tid >> 7, h = (tid >> 6) & 1, i = tid & 63;
        float4 v;
        if (h == 0) {
            v = reinterpret_cast<const float4*>((s ? p.prev_far : p.prev_mic) + (int64_t)b * 256)[i];
        } else {
            const float* cur = (s ? p.cur_far : p.cur_mic) + (int64_t)b * p.ld_cur;
            if ((p.ld_cur & 3) == 0 && ((reinterpret_cast<uintptr_t>(p.cur_mic) | reinterpret_cast<uintptr_t>(p.cur_far)) & 15) == 0)
                v = reinterpret_cast<const float4*>(cur)[i];
            else
                v = make_float4(cur[4 * i], cur[4 * i + 1], cur[4 * i + 2], cur[4 * i + 3]);
            float* save = s ? p.save_far : p.save_mic;
            if (save) reinterpret_cast<float4*>(save + (int64_t)b * 256)[i] = v;
        }
        reinterpret_cast<float4*>(sGrp[s] + h * aec::kHopStride)[i] = v;
    }
    const float2 t0 = p.tab->twT[tid], t1 = p.tab->tw512[tid];
    const float2 t2 = tid < 2 ? p.tab->tw512[256 + tid] : make_float2(0.f, 0.f);
    const float h0 = p.tab->hann[tid], h1 = p.tab->hann[tid + 256];
    aec::NlmsBin<(TAPS > 0 ? TAPS : 1)> nb;
    float2 rh[TAPS > 1 ? TAPS - 1 : 1];
    float2* nst = nullptr;
    if constexpr (TAPS > 0) {
        const int k = tid;
        nst = p.state + (int64_t)b * (2 * TAPS) * 256;
        nb.reset(k == 0);
#pragma unroll
        for (int l = 0; l < TAPS; ++l) {
            const float2 w = nst[l * 256 + k];
            nb.w[l] = aec::v2f{w.x, w.y};
        }
#pragma unroll
        for (int l = 0; l + 1 < TAPS; ++l) rh[l] = nst[(TAPS + l) * 256 + k];
        const float2 pp = nst[(2 * TAPS - 1) * 256 + k];
        nb.p = aec::v2f{pp.x, pp.y};
    }
    // weight fragments: level i, this wave's N tile nt = wave % NT, chunk c: row nt*16 + (lane & 15),
    // k = 32 c + 8 (lane >> 4) .. + 7 (the 16x16x32 B operand)
    u32x4 bw[3][kStreamEncChunks];
    float bias[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        if (i >= p.nlev) break;
        const StreamEncLevel& L = p.lev[i];
        const int NT = L.N >> 4;
        const int n = (wave % NT) * 16 + (lane & 15);
        bias[i] = L.bias[n];
        const bf16_t* wr = L.w + (int64_t)n * L.kpad + 8 * (lane >> 4);
#pragma unroll
        for (int c = 0; c < kStreamEncChunks; ++c)
            bw[i][c] = c < L.nchunk ? *reinterpret_cast<const u32x4*>(wr + 32 * c) : u32x4{0u, 0u, 0u, 0u};
    }
    // level 3 (16 output bins x 128 channels): this wave's N tiles wave and wave + 4
    u32x4 bw3[2][kStreamEncChunks3];
    float bias3[2] = {0.f, 0.f};
    if (p.nlev > 3) {
        const StreamEncLevel& L = p.lev[3];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int n = (wave + 4 * t) * 16 + (lane & 15);
            bias3[t] = L.bias[n];
            const bf16_t* wr = L.w + (int64_t)n * L.kpad + 8 * (lane >> 4);
            aec::static_for<0, kStreamEncChunks3>([&](auto ci) {
                constexpr int c = decltype(ci)::value;
                bw3[t][c] = c < L.nchunk ? *reinterpret_cast<const u32x4*>(wr + 32 * c) : u32x4{0u, 0u, 0u, 0u};
            });
        }
    }
    sTwT[tid] = t0;
    sTw512[tid] = t1;
    if (tid < 2) sTw512[256 + tid] = t2;
    sHann[tid] = h0;
    sHann[tid + 256] = h1;
    lds_barrier();
    SPROF(0, 1);

    // 2. the two transforms on waves 0 (mic) and 1 (far), lanes 0-15: the batch front's
    //    transform code (bit-identical frames) -> packed spectrum rows (slot 0 = (X[0], X[256]))
    if (wave < 2 && lane < 16) {
        const int lb = lane;
        float* reg = sGrp[wave];
        float2 v[16];
        float2 xa[8], xb[8], x128;
        aec::load_frame(v, reg, sHann, 0, lb);
        aec::wave_fence();
        aec::fft256<false>(v, lb, reg, sTwT);
        aec::rfft_unpack(v, lb, sTw512, xa, xb, x128);
        float2* row = sRow[wave];
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const int kk = lb + 16 * m;
            if (kk == 0) {
                row[0] = make_float2(xa[0].x, xb[0].x);
            } else {
                row[kk] = xa[m];
                row[256 - kk] = xb[m];
            }
        }
        if (lb == 0) row[128] = x128;
    }
    lds_barrier();
    SPROF(0, 2);

    // 3. bin slot k = tid: the NLMS step (crn_stream_nlms_kernel's arithmetic) and X0
    {
        const int k = tid;
        const float2 rm = sRow[0][k], rf = sRow[1][k];
        float2 e = rm;
        if constexpr (TAPS > 0) {
#pragma unroll
            for (int l = 0; l + 1 < TAPS; ++l) {
                const aec::v2f r{rh[l].x, rh[l].y};
                nb.a[l] = r * nb.ma;
                nb.bq[l] = aec::vfma(aec::v2f{r.y, r.x}, nb.mb, r * nb.mc);
                nb.qq[l] = aec::vfma(nb.a[l], nb.a[l], nb.bq[l] * nb.bq[l]);
            }
            e = nb.step(rm, rf, p.mu, p.beta, p.delta);
#pragma unroll
            for (int l = 0; l < TAPS; ++l) nst[l * 256 + k] = make_float2(nb.w[l].x, nb.w[l].y);
            if constexpr (TAPS > 1) {
                nst[TAPS * 256 + k] = rf;
#pragma unroll
                for (int l = 1; l + 1 < TAPS; ++l) nst[(TAPS + l) * 256 + k] = rh[l - 1];
            }
            nst[(2 * TAPS - 1) * 256 + k] = make_float2(nb.p.x, nb.p.y);
            p.espec[(int64_t)b * 256 + k] = e;
        }
        if (k > 0)
            x0_put(sX0, k, e, rf);
        else   // slot 0 holds (X[0], X[256]): the Nyquist bin 256; DC is not an encoder input
            x0_put(sX0, 256, make_float2(e.y, 0.f), make_float2(rf.y, 0.f));
    }
    lds_barrier();
    SPROF(0, 3);

    // 4. encoder levels: 8 output tiles of 16 bins x 16 channels per level, two per wave (N tile
    //    nt = wave % NT, M tiles m0 = wave / NT and m0 + 4 / NT); the implicit A rows read the
    //    input map in LDS (input bin 2 j - 2 + tap, zero outside [0, Fin))
    const bf16_t* in = sX0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        if (i >= p.nlev) break;
        const StreamEncLevel& L = p.lev[i];
        const int Fin = 256 >> i, Fo = Fin >> 1;
        const int NT = L.N >> 4;
        const int nt = wave % NT, m0 = wave / NT, m1 = m0 + 4 / NT;
        const int cs = L.cin_shift;
        f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int c = 0; c < kStreamEncChunks; ++c) {
            if (c >= L.nchunk) continue;
            const int k0 = 32 * c + 8 * (lane >> 4);
            const int tap = k0 >> cs, q0 = k0 & ((1 << cs) - 1);
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const int j = (t ? m1 : m0) * 16 + (lane & 15);
                const int ib = 2 * j - 2 + tap;
                u32x4 a = {0u, 0u, 0u, 0u};
                if (tap < 5 && ib >= 0 && ib < Fin) a = *reinterpret_cast<const u32x4*>(in + (ib << cs) + q0);
                mma_chunk(acc[t], a, bw[i][c], bf16_t{});
            }
        }
        bf16_t* map = sMap[i & 1];
        const bool keep = i + 1 < p.nlev;
        bf16_t* out = L.out + (int64_t)b * Fo * L.ldo + L.choff;
        const int n = nt * 16 + (lane & 15);
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = (t ? m1 : m0) * 16 + 4 * (lane >> 4) + r;
                float v = acc[t][r] + bias[i];
                v = v >= 0.f ? v : L.alpha * v;
                const bf16_t o = f2bf(v);
                if (keep) map[row * L.N + n] = o;
                out[(int64_t)row * L.ldo + n] = o;
            }
        lds_barrier();
        SPROF(0, 4 + i);
        in = map;
    }
    // 5. level 3: one M tile (the 16 output bins) x N tiles wave, wave + 4; the outputs staged in
    //    LDS, then stored as 16-B row chunks with their MX-fp8 shadow (the row GEMM epilogue's
    //    mx8_chunk: a 32-column group's 4 chunks in 4 adjacent lanes)
    if (p.nlev > 3) {
        const StreamEncLevel& L = p.lev[3];
        const int cs = L.cin_shift;
        f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
        aec::static_for<0, kStreamEncChunks3>([&](auto ci) {
            constexpr int c = decltype(ci)::value;
            if (c < L.nchunk) {
                const int k0 = 32 * c + 8 * (lane >> 4);
                const int tap = k0 >> cs, q0 = k0 & ((1 << cs) - 1);
                const int ib = 2 * (lane & 15) - 2 + tap;
                u32x4 a = {0u, 0u, 0u, 0u};
                if (tap < 5 && ib >= 0 && ib < 32) a = *reinterpret_cast<const u32x4*>(in + (ib << cs) + q0);
                mma_chunk(acc[0], a, bw3[0][c], bf16_t{});
                mma_chunk(acc[1], a, bw3[1][c], bf16_t{});
            }
        });
        bf16_t* stage = sMap[1];                      // level 1's map, consumed by level 2
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = 4 * (lane >> 4) + r, n = (wave + 4 * t) * 16 + (lane & 15);
                float v = acc[t][r] + bias3[t];
                v = v >= 0.f ? v : L.alpha * v;
                stage[row * 128 + n] = f2bf(v);
            }
        lds_barrier();
        const int row = tid >> 4, chn = tid & 15;
        const u32x4 v = *reinterpret_cast<const u32x4*>(stage + row * 128 + 8 * chn);
        const int64_t eo = ((int64_t)b * 16 + row) * L.ldo + L.choff + 8 * chn;
        *reinterpret_cast<u32x4*>(L.out + eo) = v;
        if (L.q8) mx8_chunk(v, true, L.q8, L.qs, eo, (chn & 3) == 0);
        SPROF(0, 7);
    }
}

hipError_t launch_stream_enc(const StreamEncArgs& a, int taps, hipStream_t st) {
    if (a.B <= 0) return hipSuccess;
    if (a.nlev < 1 || a.nlev > 4) return hipErrorInvalidValue;
    if (a.nlev > 3) {
        const StreamEncLevel& L = a.lev[3];
        if (L.N != 128 || L.cin_shift != 6 || a.lev[2].N != 64 || L.nchunk < 1 || L.nchunk > kStreamEncChunks3 ||
            L.kpad < 32 * L.nchunk || L.kpad % 8 || L.ldo % 8 || L.choff % 8 || !L.w || !L.bias || !L.out ||
            (L.q8 && (L.ldo % 32 || L.choff % 32 || !L.qs)))
            return hipErrorInvalidValue;
    }
    for (int i = 0; i < std::min(a.nlev, 3); ++i) {
        const StreamEncLevel& L = a.lev[i];
        const int Fo = 128 >> i;
        if (L.N % 16 || (Fo / 16) * (L.N / 16) != 8 || 4 % (L.N / 16) || L.nchunk < 1 ||
            L.nchunk > kStreamEncChunks || L.cin_shift < 3 || (i > 0 && (1 << L.cin_shift) != a.lev[i - 1].N) ||
            (i == 0 && L.cin_shift != 3) || L.kpad < 32 * L.nchunk || L.kpad % 8 || !L.w || !L.bias || !L.out)
            return hipErrorInvalidValue;
    }
    switch (taps) {
#define CRN_ENC_CASE(N)                                                                               \
    case N: hipLaunchKernelGGL((crn_stream_enc_kernel<N>), dim3((unsigned)a.B), dim3(256), 0, st, a); break;
        CRN_ENC_CASE(0) CRN_ENC_CASE(1) CRN_ENC_CASE(2) CRN_ENC_CASE(3) CRN_ENC_CASE(4)
        CRN_ENC_CASE(5) CRN_ENC_CASE(6) CRN_ENC_CASE(7) CRN_ENC_CASE(8)
#undef CRN_ENC_CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// --------------------------------------------------------------------------
// Fused back: decoder levels cl = 3, 2, 1 + mask + irFFT + overlap-add, one block per stream
// --------------------------------------------------------------------------
namespace {

// one decoder level: 8 output tiles of 16 input bins x 16 columns, two per wave (N tile nt =
// wave % NT, M tiles m0 = wave / NT, m0 + 4 / NT); A rows: input bins i - 1 + j (j = k / Cin),
// zero outside [0, Fin); the 32-k chunks accumulated in order from zero
template <int NC>
__device__ __forceinline__ void dec_tiles(f32x4 (&acc)[2], const bf16_t* in, int Fin, int cs, int nchunk,
                                          const u32x4 (&bw)[NC], int m0, int m1, int lane) {
    acc[0] = f32x4{0.f, 0.f, 0.f, 0.f};
    acc[1] = f32x4{0.f, 0.f, 0.f, 0.f};
    // compile-time chunk indices (a runtime-bounded loop would leave bw[] in scratch)
    aec::static_for<0, NC>([&](auto ci) {
        constexpr int c = decltype(ci)::value;
        if (c < nchunk) {
            const int k0 = 32 * c + 8 * (lane >> 4);
            const int j = k0 >> cs, q0 = k0 & ((1 << cs) - 1);
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const int i = (t ? m1 : m0) * 16 + (lane & 15);
                const int ib = i - 1 + j;
                u32x4 a = {0u, 0u, 0u, 0u};
                if (j < 3 && ib >= 0 && ib < Fin) a = *reinterpret_cast<const u32x4*>(in + (ib << cs) + q0);
                mma_chunk(acc[t], a, bw[c], bf16_t{});
            }
        }
    });
}

template <int NC>
__device__ __forceinline__ void load_bw(u32x4 (&bw)[NC], const StreamDecLevel& L, int n) {
    const bf16_t* wr = L.w + (int64_t)n * L.kpad + 8 * ((threadIdx.x & 63) >> 4);
    aec::static_for<0, NC>([&](auto ci) {
        constexpr int c = decltype(ci)::value;
        bw[c] = c < L.nchunk ? *reinterpret_cast<const u32x4*>(wr + 32 * c) : u32x4{0u, 0u, 0u, 0u};
    });
}

}  // namespace

template <int MODE>
__global__ __launch_bounds__(256) void crn_stream_dec_kernel(StreamDecArgs p) {
    constexpr int kMap = 4096;                    // bf16 elements of a level's input map (Fin x Cin)
    __shared__ __attribute__((aligned(16))) bf16_t sIn[3][kMap];
    __shared__ __attribute__((aligned(16))) float2 sMask[256];
    __shared__ __attribute__((aligned(16))) float2 sRow[256];
    __shared__ __attribute__((aligned(16))) float2 sS[260];
    __shared__ __attribute__((aligned(16))) float sTab[258 * 2 + 256 * 2 + 512 + 256];
    __shared__ __attribute__((aligned(16))) float sGrp[aec::kGroupFloats];
    float2* sTw512 = reinterpret_cast<float2*>(sTab);
    float2* sTwT = sTw512 + 258;
    float* sHann = reinterpret_cast<float*>(sTwT + 256);
    float* sCoff = sHann + 512;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int b = blockIdx.x;
    SPROF(1, 0);

    // 1. independent loads: level 0's whole input map, the encoder halves of the later maps, the
    //    spectrum source (E row or the mic frame), the OLA tail, tables, weight fragments, biases
    // (the map pieces are loaded into registers first, all in flight together, then stored:
    //  kDecPieces 16-B pieces per thread for level 0 (32 x 128 bf16) and one each for the two
    //  encoder halves (launch_stream_dec checks the shapes))
    constexpr int kDecPieces = 2;
    u32x4 mp[kDecPieces + 2];
    const StreamDecLevel& L0 = p.lev[0];
    const u32x4* src0 = reinterpret_cast<const u32x4*>(L0.src + (int64_t)b * (32 << L0.cin_shift));
#pragma unroll
    for (int i = 0; i < kDecPieces; ++i) mp[i] = src0[tid + 256 * i];
#pragma unroll
    for (int l = 1; l < 3; ++l) {                // encoder half: channels [C/2, C) of Fin rows, one piece per thread
        const StreamDecLevel& L = p.lev[l];
        const int Fin = 32 << l, C = 1 << L.cin_shift, half = C / 2, per = half / 8;
        const int r = tid / per, q = tid % per;
        mp[kDecPieces + l - 1] = *reinterpret_cast<const u32x4*>(L.src + ((int64_t)b * Fin + r) * C + half + 8 * q);
    }
    if (p.espec) {
        sRow[tid] = p.espec[(int64_t)b * 256 + tid];
    } else {
        const int h = tid >> 6, i = tid & 63;
        if (h < 2)
            reinterpret_cast<float4*>(sGrp + h * aec::kHopStride)[i] =
                reinterpret_cast<const float4*>((h ? p.cur_mic : p.prev_mic) + (int64_t)b * 256)[i];
    }
    const float tl = p.tail[(int64_t)b * 256 + tid];
    sTw512[tid] = p.tab->tw512[tid];
    if (tid < 2) sTw512[256 + tid] = p.tab->tw512[256 + tid];
    sTwT[tid] = p.tab->twT[tid];
    sHann[tid] = p.tab->hann[tid];
    sHann[tid + 256] = p.tab->hann[tid + 256];
    sCoff[tid] = p.tab->inv_coff[tid];
    u32x4 bw0[kStreamDecChunks0], bw1[kStreamDecChunks1], bw2[kStreamDecChunks2];
    int nt[3], m0[3], m1[3];
    float bias[3];
#pragma unroll
    for (int l = 0; l < 3; ++l) {
        const int NT = (p.lev[l].N + 15) >> 4;
        nt[l] = wave % NT;
        m0[l] = wave / NT;
        m1[l] = m0[l] + 4 / NT;
        const int n = nt[l] * 16 + (lane & 15);
        bias[l] = n < p.lev[l].N ? p.lev[l].bias[n] : 0.f;
    }
    load_bw(bw0, p.lev[0], nt[0] * 16 + (lane & 15));
    load_bw(bw1, p.lev[1], nt[1] * 16 + (lane & 15));
    load_bw(bw2, p.lev[2], nt[2] * 16 + (lane & 15));
#pragma unroll
    for (int i = 0; i < kDecPieces; ++i) reinterpret_cast<u32x4*>(sIn[0])[tid + 256 * i] = mp[i];
#pragma unroll
    for (int l = 1; l < 3; ++l) {
        const int C = 1 << p.lev[l].cin_shift, half = C / 2, per = half / 8;
        const int r = tid / per, q = tid % per;
        *reinterpret_cast<u32x4*>(sIn[l] + r * C + half + 8 * q) = mp[kDecPieces + l - 1];
    }
    lds_barrier();
    SPROF(1, 1);

    // 2. decoder levels cl = 3, 2: output bins 2 i + parity, channel n -> the next map's decoder half
#pragma unroll
    for (int l = 0; l < 2; ++l) {
        const StreamDecLevel& L = p.lev[l];
        const int Fin = 32 << l, Co = L.N >> 1, Cn = 1 << p.lev[l + 1].cin_shift;
        f32x4 acc[2];
        if (l == 0) dec_tiles(acc, sIn[0], Fin, L.cin_shift, L.nchunk, bw0, m0[0], m1[0], lane);
        else dec_tiles(acc, sIn[1], Fin, L.cin_shift, L.nchunk, bw1, m0[1], m1[1], lane);
        const int n = nt[l] * 16 + (lane & 15), par = n >= Co, ch = n - par * Co;
        bf16_t* next = sIn[l + 1];
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int i = (t ? m1[l] : m0[l]) * 16 + 4 * (lane >> 4) + r;
                float v = acc[t][r] + bias[l];
                v = v >= 0.f ? v : L.alpha * v;
                next[(2 * i + par) * Cn + ch] = f2bf(v);
            }
        lds_barrier();
        SPROF(1, 2 + l);
    }
    // 3. the mask level (cl = 1): columns (parity, re / im), f32, act none (v2) / tanh (v1)
    {
        const StreamDecLevel& L = p.lev[2];
        f32x4 acc[2];
        dec_tiles(acc, sIn[2], 128, L.cin_shift, L.nchunk, bw2, m0[2], m1[2], lane);
        const int n = lane & 15;
        if (n < 4) {
#pragma unroll
            for (int t = 0; t < 2; ++t)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int i = (t ? m1[2] : m0[2]) * 16 + 4 * (lane >> 4) + r;
                    float v = acc[t][r] + bias[2];
                    if (L.act == 2) v = tanhf(v);              // the batch epilogue's apply_act<2>
                    reinterpret_cast<float*>(sMask)[(2 * i + (n >> 1)) * 2 + (n & 1)] = v;
                }
        }
    }
    // the mic spectrum (no NLMS): the batch front's transform of [prev | cur]
    if (!p.espec && wave == 0 && lane < 16) {
        float2 v[16];
        float2 xa[8], xb[8], x128;
        aec::load_frame(v, sGrp, sHann, 0, lane);
        aec::wave_fence();
        aec::fft256<false>(v, lane, sGrp, sTwT);
        aec::rfft_unpack(v, lane, sTw512, xa, xb, x128);
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const int kk = lane + 16 * m;
            if (kk == 0) {
                sRow[0] = make_float2(xa[0].x, xb[0].x);
            } else {
                sRow[kk] = xa[m];
                sRow[256 - kk] = xb[m];
            }
        }
        if (lane == 0) sRow[128] = x128;
    }
    lds_barrier();
    SPROF(1, 4);
    // 4. the mask on every bin (thread k: bin k; thread 0 also the Nyquist bin; DC's mask is 0)
    {
        const int k = tid;
        const float2 x = sRow[k];
        if (k == 0) {
            sS[0] = apply_mask<MODE>(make_float2(x.x, 0.f), make_float2(0.f, 0.f));
            sS[256] = apply_mask<MODE>(make_float2(x.y, 0.f), sMask[255]);
        } else {
            sS[k] = apply_mask<MODE>(x, sMask[k - 1]);
        }
    }
    lds_barrier();
    SPROF(1, 5);
    // 5. inverse pack, irFFT-256, window, overlap-add (crn_stream_back_kernel's code), wave 0 lanes 0-15
    if (wave == 0 && lane < 16) {
        const int lb = lane;
        float2 xa[8], xb[8];
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const int kk = lb + 16 * m;
            xa[m] = sS[kk];
            xb[m] = sS[256 - kk];
        }
        const float2 x128 = sS[128];
        float2 Zk[8], Zmk[8], v[16];
        aec::static_for<0, 8>([&](auto mi) {
            constexpr int m = decltype(mi)::value;
            const int kk = lb + 16 * m;
            float2 zk, zmk;
            aec::irfft_pair(xa[m], xb[m], sTw512[kk], zk, zmk);
            const float s0 = xa[m].x, s256 = xb[m].x;
            Zk[m] = aec::csel(kk == 0, make_float2(s0 + s256, s0 - s256), zk);
            Zmk[m] = aec::csel(kk == 0, Zk[m], zmk);
        });
        float2 z128 = make_float2(0.f, 0.f);
        if (lb == 0) z128 = make_float2(2.f * x128.x, -2.f * x128.y);
#pragma unroll
        for (int a = 0; a < 8; ++a) v[a] = Zk[a];
        aec::static_for<8, 16>([&](auto ai) {
            constexpr int a = decltype(ai)::value;
            const float2 mir = aec::mirror16(Zmk[15 - a]);
            v[a] = aec::csel(lb != 0, mir, a == 8 ? z128 : Zmk[(16 - a) & 7]);
        });
        aec::wave_fence();
        aec::fft256<true>(v, lb, sGrp, sTwT);
        float2* s2 = reinterpret_cast<float2*>(sGrp);
        const float2* h2 = reinterpret_cast<const float2*>(sHann);
#pragma unroll
        for (int m2 = 0; m2 < 16; ++m2) {
            const float2 zz = v[aec::kP(m2)];
            const float2 w = h2[lb + 16 * m2];
            s2[lb + 16 * m2] = make_float2(zz.x * (w.x * (1.f / 512.f)), zz.y * (w.y * (1.f / 512.f)));
        }
    }
    lds_barrier();
    SPROF(1, 6);
    {
        const int r = tid;
        p.out[(int64_t)b * p.ld_out + r] = (tl + sGrp[r]) * sCoff[r];
        p.tail[(int64_t)b * 256 + r] = sGrp[256 + r];
    }
    SPROF(1, 7);
}

hipError_t launch_stream_dec(const StreamDecArgs& a, int mode, hipStream_t st) {
    if (a.B <= 0) return hipSuccess;
    const int caps[3] = {kStreamDecChunks0, kStreamDecChunks1, kStreamDecChunks2};
    for (int l = 0; l < 3; ++l) {
        const StreamDecLevel& L = a.lev[l];
        const int Fin = 32 << l, NT = (L.N + 15) / 16;
        if (!L.w || !L.bias || !L.src || L.nchunk < 1 || L.nchunk > caps[l] || L.kpad < 32 * L.nchunk ||
            (Fin / 16) * NT != 8 || 4 % NT || (Fin << L.cin_shift) > 4096 || L.cin_shift < 4 ||
            (l < 2 && (L.N % 32 || L.act != 1 || L.N != (1 << a.lev[l + 1].cin_shift))) ||   // Co = next map's half
            (l == 2 && (L.N != 4 || L.act == 1)))
            return hipErrorInvalidValue;
        const int C = 1 << L.cin_shift;
        if (l == 0 ? Fin * C != 2 * 256 * 8 : Fin * (C / 2) != 256 * 8) return hipErrorInvalidValue;   // the load's piece counts
    }
    switch (mode) {
        case 0: hipLaunchKernelGGL(crn_stream_dec_kernel<0>, dim3((unsigned)a.B), dim3(256), 0, st, a); break;
        case 1: hipLaunchKernelGGL(crn_stream_dec_kernel<1>, dim3((unsigned)a.B), dim3(256), 0, st, a); break;
        case 2: hipLaunchKernelGGL(crn_stream_dec_kernel<2>, dim3((unsigned)a.B), dim3(256), 0, st, a); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace crn

#ifdef AEC_STREAM_PROF
extern "C" int aec_debug_stream_prof(void* host, size_t bytes) {
    if (bytes < sizeof(crn::g_sprof)) return -1;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(crn::g_sprof), sizeof(crn::g_sprof)) == hipSuccess ? 0 : -2;
}
#endif
