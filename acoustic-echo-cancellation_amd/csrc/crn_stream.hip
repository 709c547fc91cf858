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
// The level maps in LDS keep one bin per row, padded by 16 B: a level's A fragment reads the 16
// lanes' bins two apart (encoder) or adjacent (decoder), which unpadded land on 4 to 16 copies of
// the same bank slots (32- to 256-B rows); padded, a 16-lane group spreads over 8 or 16 slots.
constexpr int kPadMapElems = 128 * (16 + 8);   // the largest padded encoder map: level 0's 128 x (16 + 8)

// block barrier that drains LDS only: the global stores of the level outputs (read by a later
// launch) and the register loads of weight fragments stay in flight across it
__device__ __forceinline__ void lds_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}    // bf16 elements of one level's output map (Fo x N = 8 tiles of 16 x 16)

// A 16-B piece of an implicit A row from an LDS map, zero when !ok.  The read always happens, at
// row 0 when !ok (every map has one), and the zero is selected afterwards: a guarded read compiled
// to a branch and an lgkmcnt(0) wait per MFMA, where branch-free reads of a chunk stay in flight
// together.
__device__ __forceinline__ u32x4 lds_frag(const bf16_t* map, int row, int rs, int q0, bool ok) {
    const u32x4 v = *reinterpret_cast<const u32x4*>(map + (ok ? row : 0) * rs + q0);
    return ok ? v : u32x4{0u, 0u, 0u, 0u};
}

// FR frames' two 16 x 16 output tiles (M tiles m0, m1) of one conv level over NC 32-k chunks:
// implicit A rows from the LDS maps (input bin ST * j + OFF + tap of output row j, TAPS taps,
// 2^CS channels per bin, RS elements per map row), B fragments in registers.  Compile-time chunk
// count and shapes: the reads of a chunk for every frame go out together and the chunk loop
// carries no branch (a runtime-bounded one compiled to a branch and an lgkmcnt(0) wait per chunk).
// Per accumulator the chunks run in order from zero: the row GEMM's sum.
// TR: transposed accumulators (the operands swapped: a lane holds 4 adjacent columns 4 (lane >> 4)
// .. + 3 of row lane & 15, so the epilogue writes 8 B at a time); the same products summed the same
// way per element.
template <int FR, int NC, int CS, int RS, int ST, int OFF, int TAPS, int FIN, int NCAP, bool TR = false>
__device__ __forceinline__ void conv_tiles(f32x4 (&acc)[FR][2], const bf16_t* const (&in)[FR], const u32x4 (&bw)[NCAP],
                                           int m0, int m1, int lane) {
#pragma unroll
    for (int fr = 0; fr < FR; ++fr) acc[fr][0] = acc[fr][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    aec::static_for<0, NC>([&](auto ci) {
        constexpr int c = decltype(ci)::value;
        const int k0 = 32 * c + 8 * (lane >> 4);
        const int tap = k0 >> CS, q0 = k0 & ((1 << CS) - 1);
        u32x4 a[FR][2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int ib = ST * ((t ? m1 : m0) * 16 + (lane & 15)) + OFF + tap;
            const bool ok = tap < TAPS && ib >= 0 && ib < FIN;
#pragma unroll
            for (int fr = 0; fr < FR; ++fr) a[fr][t] = lds_frag(in[fr], ib, RS, q0, ok);
        }
#pragma unroll
        for (int fr = 0; fr < FR; ++fr)
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                if constexpr (TR) mma_chunk(acc[fr][t], bw[c], a[fr][t], bf16_t{});
                else mma_chunk(acc[fr][t], a[fr][t], bw[c], bf16_t{});
            }
    });
}

// conv_tiles' form for one M tile (m0) and two N tiles (weights bwa, bwb): one A piece per frame
// and chunk feeds both (encoder level 3: 16 output bins)
template <int FR, int NC, int CS, int RS, int ST, int OFF, int TAPS, int FIN, int NCAP, bool TR = false>
__device__ __forceinline__ void conv_tiles_n2(f32x4 (&acc)[FR][2], const bf16_t* const (&in)[FR],
                                              const u32x4 (&bwa)[NCAP], const u32x4 (&bwb)[NCAP], int m0, int lane) {
#pragma unroll
    for (int fr = 0; fr < FR; ++fr) acc[fr][0] = acc[fr][1] = f32x4{0.f, 0.f, 0.f, 0.f};
    aec::static_for<0, NC>([&](auto ci) {
        constexpr int c = decltype(ci)::value;
        const int k0 = 32 * c + 8 * (lane >> 4);
        const int tap = k0 >> CS, q0 = k0 & ((1 << CS) - 1);
        const int ib = ST * (m0 * 16 + (lane & 15)) + OFF + tap;
        const bool ok = tap < TAPS && ib >= 0 && ib < FIN;
        u32x4 a[FR];
#pragma unroll
        for (int fr = 0; fr < FR; ++fr) a[fr] = lds_frag(in[fr], ib, RS, q0, ok);
#pragma unroll
        for (int fr = 0; fr < FR; ++fr) {
            if constexpr (TR) {
                mma_chunk(acc[fr][0], bwa[c], a[fr], bf16_t{});
                mma_chunk(acc[fr][1], bwb[c], a[fr], bf16_t{});
            } else {
                mma_chunk(acc[fr][0], a[fr], bwa[c], bf16_t{});
                mma_chunk(acc[fr][1], a[fr], bwb[c], bf16_t{});
            }
        }
    });
}

// the PReLU epilogue of 4 adjacent columns (v + bias, then v >= 0 ? v : alpha v) as 4 bf16 in 8 B
__device__ __forceinline__ uint2 prelu4_bf16(const f32x4& v, const float4& bias, float alpha) {
    const float b[4] = {bias.x, bias.y, bias.z, bias.w};
    uint32_t o[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        float x = v[r] + b[r];
        x = x >= 0.f ? x : alpha * x;
        o[r] = f2bf(x);
    }
    return make_uint2(o[0] | (o[1] << 16), o[2] | (o[3] << 16));
}

// A scaled-MFMA operand kept live past the instruction that reads it: the B fragment of a first
// stage (C = 0) is otherwise dead after the MFMA, and under register pressure the allocator gave
// its registers to the MFMA's own destination (vdst = a[56:59] with srcB = a[56:63]), which read
// back corrupted operands (NaN outputs); the scale registers were rewritten two cycles after the
// issue.  An empty asm that reads them after the MFMA forbids both reuses.
// CRN_NO_CODEGEN_GUARDS (tests/test_isa_guard.py only, never a product build): every workaround of
// this file compiled out, so the CPU-side code-object check can show that it catches their absence.
#ifndef CRN_NO_CODEGEN_GUARDS
__device__ __forceinline__ void keep_live(const i32x8& b) { asm volatile("" ::"v"(b)); }
__device__ __forceinline__ void keep_live(int x) { asm volatile("" ::"v"(x)); }
#else
__device__ __forceinline__ void keep_live(const i32x8&) {}
__device__ __forceinline__ void keep_live(int) {}
#endif
// After a run of scaled MFMAs: no instruction is scheduled into the run (sched_barrier) and ~48
// cycles pass before any later instruction may rewrite an operand or scale register.  With the
// epilogue's register reads ten cycles after the last MFMA, the level's outputs differed from the
// MX GEMM's in the last bits for a few columns; the scale operands are evidently still read after
// the issue, and the compiler's hazard recognizer does not pad for it.
__device__ __forceinline__ void mx_drain() {
#ifndef CRN_NO_CODEGEN_GUARDS
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 15" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#endif
}
static_assert(2 * kPadMapElems >= 16 * 256, "level 4 staging spans both maps");

// mx8_chunk's arithmetic (crn_gemm.h) returning the chunk's 8 e4m3 bytes and its group's E8M0 code
// instead of storing them (the fused front keeps level 3's shadow in LDS for level 4 as well)
__device__ __forceinline__ uint2 mx8_pack_chunk(const u32x4& v, int& code_out) {
    float x[8];
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        x[2 * i] = __uint_as_float(v[i] << 16);
        x[2 * i + 1] = __uint_as_float(v[i] & 0xFFFF0000u);
        amax = fmaxf(amax, fmaxf(fabsf(x[2 * i]), fabsf(x[2 * i + 1])));
    }
    amax = fmaxf(amax, __shfl_xor(amax, 1));
    amax = fmaxf(amax, __shfl_xor(amax, 2));
    const int ebits = (int)((__float_as_uint(amax) >> 23) & 0xFF);
    const int code = ebits > 8 ? ebits - 8 : 0;
    uint32_t pk[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        float y[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) y[j] = fminf(fmaxf(ldexpf(x[4 * i + j], 127 - code), -448.f), 448.f);
        int w = __builtin_amdgcn_cvt_pk_fp8_f32(y[0], y[1], 0, false);
        w = __builtin_amdgcn_cvt_pk_fp8_f32(y[2], y[3], w, true);
        pk[i] = (uint32_t)w;
    }
    code_out = code;
    return make_uint2(pk[0], pk[1]);
}

// net_conf's encoder levels 0-3 (conv_channels 4, 16, 32, 64, 128: N = 16 << i, K = 5 taps x
// 8 / 16 / 32 / 64 input channels): the shapes the batch kernels are compiled for
constexpr int kEncNC[4] = {2, 3, 5, 10};

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

// MX4: encoder level 4 folded in (its weight fragments hold ~180 VGPRs, so the kernel without it is
// a separate instantiation: at many streams per CU its occupancy, not the extra launch, decides;
// without the fold and with <= 4 taps it fits 2 waves per SIMD with no scratch)
template <int TAPS, bool MX4>
__global__ __launch_bounds__(256, MX4 || TAPS > 4 ? 1 : 2) void crn_stream_enc_kernel(StreamEncArgs p) {
    __shared__ __attribute__((aligned(16))) float sTab[256 * 2 + 258 * 2 + 512];
    __shared__ __attribute__((aligned(16))) float sGrp[2][aec::kGroupFloats];
    __shared__ __attribute__((aligned(16))) float2 sRow[2][256];
    __shared__ __attribute__((aligned(16))) bf16_t sX0[256 * 8];
    __shared__ __attribute__((aligned(16))) bf16_t sMap[2][kPadMapElems];
    __shared__ __attribute__((aligned(16))) uint8_t sQ3[16 * (128 + 16)];   // level 3's e4m3 shadow (level 4)
    __shared__ uint8_t sQ3s[16 * 4];
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
            nb.w[l] = w;
        }
#pragma unroll
        for (int l = 0; l + 1 < TAPS; ++l) rh[l] = nst[(TAPS + l) * 256 + k];
        const float2 pp = nst[(2 * TAPS - 1) * 256 + k];
        nb.p = pp;
    }
    // weight fragments: level i, this wave's N tile nt = wave % NT, chunk c: row nt*16 + (lane & 15),
    // k = 32 c + 8 (lane >> 4) .. + 7 (the 16x16x32 B operand)
    u32x4 bw[3][kStreamEncChunks];
    float4 bias[3];                               // the TR epilogue's 4 columns nt * 16 + 4 (lane >> 4) .. + 3
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        if (i >= p.nlev) break;
        const StreamEncLevel& L = p.lev[i];
        const int NT = L.N >> 4;
        const int n = (wave % NT) * 16 + (lane & 15);
        bias[i] = *reinterpret_cast<const float4*>(L.bias + (wave % NT) * 16 + 4 * (lane >> 4));
        const bf16_t* wr = L.w + (int64_t)n * L.kpad + 8 * (lane >> 4);
#pragma unroll
        for (int c = 0; c < kStreamEncChunks; ++c)
            bw[i][c] = c < L.nchunk ? *reinterpret_cast<const u32x4*>(wr + 32 * c) : u32x4{0u, 0u, 0u, 0u};
    }
    // level 3 (16 output bins x 128 channels): this wave's N tiles wave and wave + 4
    u32x4 bw3[2][kStreamEncChunks3];
    float4 bias3[2] = {make_float4(0.f, 0.f, 0.f, 0.f), make_float4(0.f, 0.f, 0.f, 0.f)};
    if (p.nlev > 3) {
        const StreamEncLevel& L = p.lev[3];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int n = (wave + 4 * t) * 16 + (lane & 15);
            bias3[t] = *reinterpret_cast<const float4*>(L.bias + (wave + 4 * t) * 16 + 4 * (lane >> 4));
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
            for (int l = 0; l + 1 < TAPS; ++l) nb.hist(l, rh[l]);
            e = nb.step(rm, rf, p.mu, p.beta, p.delta);
#pragma unroll
            for (int l = 0; l < TAPS; ++l) nst[l * 256 + k] = nb.w[l];
            if constexpr (TAPS > 1) {
                nst[TAPS * 256 + k] = rf;
#pragma unroll
                for (int l = 1; l + 1 < TAPS; ++l) nst[(TAPS + l) * 256 + k] = rh[l - 1];
            }
            nst[(2 * TAPS - 1) * 256 + k] = nb.p;
            p.espec[(int64_t)b * 256 + k] = e;
        }
        if (k > 0)
            x0_put(sX0, k, e, rf);
        else   // slot 0 holds (X[0], X[256]): the Nyquist bin 256; DC is not an encoder input
            x0_put(sX0, 256, make_float2(e.y, 0.f), make_float2(rf.y, 0.f));
    }
    lds_barrier();
    SPROF(0, 3);

    // level 4 (MX, optional): this wave's B fragments of N tiles wave + 4 t (t = 0..3), stage st =
    // tap st: bytes 128 st + 16 g and + 64 (the MX GEMM core's operand map), their scale bytes, and
    // the lane's bias per tile (the non-transposed accumulator: column (lane & 15) of the tile).
    // Requested here, after the transforms and the NLMS step (180 VGPRs fewer live through them),
    // so their L2 latency runs under levels 0-3.
    constexpr bool mx4 = MX4;                                    // launch_stream_enc: == (p.mx4.wq != nullptr)
    u32x4 mb4[4][kStreamEncMxStages][2];
    uint32_t msw4[4][kStreamEncMxStages];
    float mbias4[4];
    if (mx4) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int n = (wave + 4 * t) * 16 + (lane & 15);
            const uint8_t* wr = p.mx4.wq + (int64_t)n * 640 + 16 * (lane >> 4);
            const uint32_t* sr = reinterpret_cast<const uint32_t*>(p.mx4.wsc + (int64_t)n * 20);
#pragma unroll
            for (int st = 0; st < kStreamEncMxStages; ++st) {
                mb4[t][st][0] = *reinterpret_cast<const u32x4*>(wr + 128 * st);
                mb4[t][st][1] = *reinterpret_cast<const u32x4*>(wr + 128 * st + 64);
                msw4[t][st] = (sr[st] >> (8 * (lane >> 4))) & 0xFFu;   // this lane's scale byte
            }
            mbias4[t] = p.mx4.bias[n];
        }
    }
    // 4. encoder levels 0-2 (net_conf's shapes, checked by launch_stream_enc): 8 output tiles of 16
    //    bins x 16 channels per level, two per wave (N tile nt = wave % NT, M tiles m0 = wave / NT and
    //    m0 + 4 / NT); the implicit A rows read the input map in LDS (input bin 2 j - 2 + tap, zero
    //    outside [0, Fin))
    f32x4 acc[1][2];
    auto level_out = [&](auto Ic, int nt, int m0, int m1, bool keep) {
        constexpr int i = decltype(Ic)::value, N = 16 << i, Fo = 128 >> i;
        const StreamEncLevel& L = p.lev[i];
        bf16_t* map = sMap[i & 1];
        bf16_t* out = L.out + (int64_t)b * Fo * L.ldo + L.choff;
        const int n0 = nt * 16 + 4 * (lane >> 4);   // transposed accumulators: 4 adjacent columns
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int row = (t ? m1 : m0) * 16 + (lane & 15);
            const uint2 o = prelu4_bf16(acc[0][t], bias[i], L.alpha);
            if (keep) *reinterpret_cast<uint2*>(map + row * (N + 8) + n0) = o;
            *reinterpret_cast<uint2*>(out + (int64_t)row * L.ldo + n0) = o;
        }
        lds_barrier();
        SPROF(0, 4 + i);
    };
    {
        const bf16_t* in[1] = {sX0};
        conv_tiles<1, kEncNC[0], 3, 8, 2, -2, 5, 256, kStreamEncChunks, true>(acc, in, bw[0], wave, wave + 4, lane);
        level_out(std::integral_constant<int, 0>{}, 0, wave, wave + 4, true);
    }
    {
        const bf16_t* in[1] = {sMap[0]};
        conv_tiles<1, kEncNC[1], 4, 16 + 8, 2, -2, 5, 128, kStreamEncChunks, true>(acc, in, bw[1], wave / 2, wave / 2 + 2, lane);
        level_out(std::integral_constant<int, 1>{}, wave % 2, wave / 2, wave / 2 + 2, true);
    }
    {
        const bf16_t* in[1] = {sMap[1]};
        conv_tiles<1, kEncNC[2], 5, 32 + 8, 2, -2, 5, 64, kStreamEncChunks, true>(acc, in, bw[2], 0, 1, lane);
        level_out(std::integral_constant<int, 2>{}, wave, 0, 1, p.nlev > 3);
    }
    // 5. level 3: one M tile (the 16 output bins) x N tiles wave, wave + 4; the outputs staged in
    //    LDS, then stored as 16-B row chunks with their MX-fp8 shadow (the row GEMM epilogue's
    //    mx8_chunk: a 32-column group's 4 chunks in 4 adjacent lanes)
    if (p.nlev > 3) {
        const StreamEncLevel& L = p.lev[3];
        const bf16_t* in[1] = {sMap[0]};
        conv_tiles_n2<1, kEncNC[3], 6, 64 + 8, 2, -2, 5, 32, kStreamEncChunks3, true>(acc, in, bw3[0], bw3[1], 0, lane);
        bf16_t* stage = sMap[1];                      // level 1's map, consumed by level 2
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int row = lane & 15, n0 = (wave + 4 * t) * 16 + 4 * (lane >> 4);
            *reinterpret_cast<uint2*>(stage + row * 128 + n0) = prelu4_bf16(acc[0][t], bias3[t], L.alpha);
        }
        lds_barrier();
        const int row = tid >> 4, chn = tid & 15;
        const u32x4 v = *reinterpret_cast<const u32x4*>(stage + row * 128 + 8 * chn);
        const int64_t eo = ((int64_t)b * 16 + row) * L.ldo + L.choff + 8 * chn;
        *reinterpret_cast<u32x4*>(L.out + eo) = v;
        if (mx4) {
            // the shadow to HBM (decoder level 4 reads it) and into LDS for level 4: rows of 128 e4m3
            // (+16 B pad), 4 E8M0 per row
            int code;
            const uint2 pk = mx8_pack_chunk(v, code);
            *reinterpret_cast<uint2*>(L.q8 + eo) = pk;
            if ((chn & 3) == 0) L.qs[eo >> 5] = (uint8_t)code;
            *reinterpret_cast<uint2*>(sQ3 + row * (128 + 16) + 8 * chn) = pk;
            if ((chn & 3) == 0) sQ3s[row * 4 + (chn >> 2)] = (uint8_t)code;
        } else if (L.q8) {
            mx8_chunk(v, true, L.q8, L.qs, eo, (chn & 3) == 0);
        }
        SPROF(0, 7);
    }
    // 6. level 4 (MX-fp8, optional): 8 output bins j (rows 8..15 of the M tile unused) x N tiles
    //    wave + 4 t; input bin 2 j - 2 + tap, tap = stage; then + bias, PReLU, bf16, staged in LDS
    //    (level 2's map, consumed) and stored as 16-B row chunks with the output's MX-fp8 shadow
    if (mx4) {
        lds_barrier();
        const int g = lane >> 4, r = lane & 15;
        f32x4 acc4[4] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f},
                         f32x4{0.f, 0.f, 0.f, 0.f}};
        // every stage's A fragment and scale first, then the MFMAs, then every operand kept live to the
        // end of the level (see keep_live: no operand register is rewritten while an MFMA may read it)
        i32x8 af[kStreamEncMxStages];
        int sa[kStreamEncMxStages];
        aec::static_for<0, kStreamEncMxStages>([&](auto si) {
            constexpr int st = decltype(si)::value;
            const int ib = 2 * r - 2 + st;
            const bool ok = r < 8 && ib >= 0 && ib < 16;
            const uint8_t* rowp = sQ3 + (ok ? ib : 0) * (128 + 16);
            const u32x4 lo = *reinterpret_cast<const u32x4*>(rowp + 16 * g);
            const u32x4 hi = *reinterpret_cast<const u32x4*>(rowp + 64 + 16 * g);
            const u32x4 z = {0u, 0u, 0u, 0u};
            const u32x4 l2 = ok ? lo : z, h2 = ok ? hi : z;
            af[st] = i32x8{(int)l2[0], (int)l2[1], (int)l2[2], (int)l2[3], (int)h2[0], (int)h2[1], (int)h2[2], (int)h2[3]};
            sa[st] = ok ? (int)sQ3s[(ok ? ib : 0) * 4 + g] : 0;
        });
        auto bfrag = [&](int t, auto Sc) {
            constexpr int st = decltype(Sc)::value;
            return i32x8{(int)mb4[t][st][0][0], (int)mb4[t][st][0][1], (int)mb4[t][st][0][2], (int)mb4[t][st][0][3],
                         (int)mb4[t][st][1][0], (int)mb4[t][st][1][1], (int)mb4[t][st][1][2], (int)mb4[t][st][1][3]};
        };
        aec::static_for<0, kStreamEncMxStages>([&](auto si) {
            constexpr int st = decltype(si)::value;
#pragma unroll
            for (int t = 0; t < 4; ++t)
                acc4[t] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af[st], bfrag(t, si), acc4[t], 0, 0, 0, sa[st], 0,
                                                                           (int)msw4[t][st]);
        });
        mx_drain();
        aec::static_for<0, kStreamEncMxStages>([&](auto si) {
            constexpr int st = decltype(si)::value;
            keep_live(af[st]);
            keep_live(sa[st]);
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                keep_live(bfrag(t, si));
                keep_live((int)msw4[t][st]);
            }
        });
        // every lane writes its rows, the unused 8 .. 15 included: with a `g < 2` guard the compiler
        // sank the MFMAs (pure, used only there) into the lanes-0..31 region, where the operand moves
        // of lanes 32..63 (k bytes 32..63, 96..127 of every row) did not run
        bf16_t* st4 = &sMap[0][0];                                  // [16 rows][256 channels] (both maps)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            const int n = (wave + 4 * t) * 16 + r;
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                float v = acc4[t][rr] + mbias4[t];
                v = v >= 0.f ? v : p.mx4.alpha * v;
                st4[(4 * g + rr) * 256 + n] = f2bf(v);
            }
        }
        lds_barrier();
        const int row = tid >> 5, chn = tid & 31;
        const u32x4 v = *reinterpret_cast<const u32x4*>(st4 + row * 256 + 8 * chn);
        const int64_t eo = ((int64_t)b * 8 + row) * p.mx4.ldo + p.mx4.choff + 8 * chn;
        *reinterpret_cast<u32x4*>(p.mx4.out + eo) = v;
        if (p.mx4.q8) mx8_chunk(v, true, p.mx4.q8, p.mx4.qs, eo, (chn & 3) == 0);
    }
}

hipError_t launch_stream_enc(const StreamEncArgs& a, int taps, hipStream_t st) {
    if (a.B <= 0) return hipSuccess;
    if (a.nlev < 3 || a.nlev > 4) return hipErrorInvalidValue;
    if (a.mx4.wq && (a.nlev != 4 || !a.lev[3].q8 || !a.lev[3].qs || !a.mx4.wsc || !a.mx4.bias || !a.mx4.out ||
                     a.mx4.ldo % 8 || a.mx4.choff % 32 || (a.mx4.q8 && (!a.mx4.qs || a.mx4.ldo % 32))))
        return hipErrorInvalidValue;
    if (a.nlev > 3) {
        const StreamEncLevel& L = a.lev[3];
        if (L.N != 128 || L.cin_shift != 6 || a.lev[2].N != 64 || L.nchunk != kEncNC[3] ||
            L.kpad < 32 * L.nchunk || L.kpad % 8 || L.ldo % 8 || L.choff % 8 || !L.w || !L.bias || !L.out ||
            (L.q8 && (L.ldo % 32 || L.choff % 32 || !L.qs)))
            return hipErrorInvalidValue;
    }
    for (int i = 0; i < std::min(a.nlev, 3); ++i) {
        const StreamEncLevel& L = a.lev[i];
        const int Fo = 128 >> i;
        if (L.N != (16 << i) || (Fo / 16) * (L.N / 16) != 8 || L.nchunk != kEncNC[i] || L.cin_shift != 3 + i ||
            L.kpad < 32 * L.nchunk || L.kpad % 8 || !L.w || !L.bias || !L.out)
            return hipErrorInvalidValue;
    }
    switch (taps) {
#define CRN_ENC_CASE(N)                                                                               \
    case N:                                                                                           \
        if (a.mx4.wq)                                                                                 \
            hipLaunchKernelGGL((crn_stream_enc_kernel<N, true>), dim3((unsigned)a.B), dim3(256), 0, st, a); \
        else                                                                                          \
            hipLaunchKernelGGL((crn_stream_enc_kernel<N, false>), dim3((unsigned)a.B), dim3(256), 0, st, a); \
        break;
        CRN_ENC_CASE(0) CRN_ENC_CASE(1) CRN_ENC_CASE(2) CRN_ENC_CASE(3) CRN_ENC_CASE(4)
        CRN_ENC_CASE(5) CRN_ENC_CASE(6) CRN_ENC_CASE(7) CRN_ENC_CASE(8)
#undef CRN_ENC_CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// --------------------------------------------------------------------------
// Batch encoder front (the batch forward of C3 / C4 and its fp8 form): encoder levels 0-3 of
// every frame from X0 in HBM, the per-hop front's level arithmetic over FR frames per block at
// once, the maps in LDS.  A persistent frame loop keeps the weight fragments of all four levels
// in registers for the whole launch; X0 of the next FR frames is fetched into registers while
// the current ones run.  Each level's map leaves LDS as 16-B rows (the encoder half of
// cat[l + 1]); level 3 also writes its MX-fp8 shadow.  Same packed weights, the same 32-k
// chunks in the same order from zero and the same epilogue as the row GEMMs these four
// launches replace, so the maps are bit-identical (tests/test_gpu_crn.py::test_batch_enc_fused_bit_exact).
// The LDS maps are padded as the per-hop kernels' (kPadMapElems).
// --------------------------------------------------------------------------
template <int FR>
__global__ __launch_bounds__(256, 1) void crn_enc_batch_kernel(EncBatchArgs p) {
    __shared__ __attribute__((aligned(16))) bf16_t sX0[FR][256 * 8];
    __shared__ __attribute__((aligned(16))) bf16_t sMap[2][FR][kPadMapElems];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    // weight fragments (crn_stream_enc_kernel's map): levels 0-2, this wave's N tile wave % NT;
    // level 3, N tiles wave and wave + 4
    u32x4 bw0[kEncNC[0]], bw1[kEncNC[1]], bw2[kEncNC[2]], bw3a[kEncNC[3]], bw3b[kEncNC[3]];
    float4 bias[3];
    auto load_w = [&](auto& bw, const StreamEncLevel& L, int n) {
        const bf16_t* wr = L.w + (int64_t)n * L.kpad + 8 * (lane >> 4);
        aec::static_for<0, (int)(sizeof(bw) / sizeof(bw[0]))>([&](auto ci) {
            constexpr int c = decltype(ci)::value;
            bw[c] = *reinterpret_cast<const u32x4*>(wr + 32 * c);
        });
    };
    {
        const int n0 = (wave % 1) * 16 + (lane & 15), n1 = (wave % 2) * 16 + (lane & 15), n2 = (wave % 4) * 16 + (lane & 15);
        load_w(bw0, p.lev[0], n0);
        load_w(bw1, p.lev[1], n1);
        load_w(bw2, p.lev[2], n2);
        // TR epilogue: the lane's 4 columns nt * 16 + 4 (lane >> 4) .. + 3
        const int g4 = 4 * (lane >> 4);
        bias[0] = *reinterpret_cast<const float4*>(p.lev[0].bias + g4);
        bias[1] = *reinterpret_cast<const float4*>(p.lev[1].bias + (wave % 2) * 16 + g4);
        bias[2] = *reinterpret_cast<const float4*>(p.lev[2].bias + (wave % 4) * 16 + g4);
    }
    const int n3a = wave * 16 + (lane & 15), n3b = (wave + 4) * 16 + (lane & 15);
    load_w(bw3a, p.lev[3], n3a);
    load_w(bw3b, p.lev[3], n3b);
    const float4 bias3[2] = {*reinterpret_cast<const float4*>(p.lev[3].bias + wave * 16 + 4 * (lane >> 4)),
                             *reinterpret_cast<const float4*>(p.lev[3].bias + (wave + 4) * 16 + 4 * (lane >> 4))};
    const int64_t F = p.F, step = (int64_t)gridDim.x * FR;
    // X0 of frames fb .. fb + FR - 1: 4 KB each = one 16-B piece per thread
    u32x4 nx[FR];
    auto fetch = [&](int64_t fb) {
#pragma unroll
        for (int fr = 0; fr < FR; ++fr) {
            const int64_t f = fb + fr;
            nx[fr] = f < F ? reinterpret_cast<const u32x4*>(p.x0 + f * 2048)[tid] : u32x4{0u, 0u, 0u, 0u};
        }
    };
    // level i's epilogue: PReLU, bf16 into the padded map, then the map -> cat[i + 1]'s encoder half
    // (map row `row` = N contiguous channels)
    auto level_out = [&](auto Ic, const f32x4 (&acc)[FR][2], int nt, int m0, int m1, int64_t f0) {
        constexpr int i = decltype(Ic)::value, N = 16 << i;
        const StreamEncLevel& L = p.lev[i];
        const int n0 = nt * 16 + 4 * (lane >> 4);
#pragma unroll
        for (int fr = 0; fr < FR; ++fr)
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const int row = (t ? m1 : m0) * 16 + (lane & 15);
                *reinterpret_cast<uint2*>(sMap[i & 1][fr] + row * (N + 8) + n0) = prelu4_bf16(acc[fr][t], bias[i], L.alpha);
            }
        lds_barrier();
        constexpr int Fo = 128 >> i;
        const int e0 = 8 * tid, row = e0 / N, ch0 = e0 % N;
#pragma unroll
        for (int fr = 0; fr < FR; ++fr) {
            const int64_t f = f0 + fr;
            if (f < F)
                *reinterpret_cast<u32x4*>(L.out + (f * Fo + row) * L.ldo + L.choff + ch0) =
                    *reinterpret_cast<const u32x4*>(sMap[i & 1][fr] + row * (N + 8) + ch0);
        }
    };
    fetch((int64_t)blockIdx.x * FR);
    for (int64_t f0 = (int64_t)blockIdx.x * FR; f0 < F; f0 += step) {
#pragma unroll
        for (int fr = 0; fr < FR; ++fr) reinterpret_cast<u32x4*>(sX0[fr])[tid] = nx[fr];
        lds_barrier();
        fetch(f0 + step);
        f32x4 acc[FR][2];
        {   // level 0: 128 output bins x 16 channels (8 M tiles, 1 N tile) from X0 (16-B rows)
            const bf16_t* in[FR];
#pragma unroll
            for (int fr = 0; fr < FR; ++fr) in[fr] = sX0[fr];
            conv_tiles<FR, kEncNC[0], 3, 8, 2, -2, 5, 256, kEncNC[0], true>(acc, in, bw0, wave, wave + 4, lane);
            level_out(std::integral_constant<int, 0>{}, acc, 0, wave, wave + 4, f0);
        }
        {   // level 1: 64 x 32 (4 M tiles x 2 N tiles)
            const bf16_t* in[FR];
#pragma unroll
            for (int fr = 0; fr < FR; ++fr) in[fr] = sMap[0][fr];
            conv_tiles<FR, kEncNC[1], 4, 16 + 8, 2, -2, 5, 128, kEncNC[1], true>(acc, in, bw1, wave / 2, wave / 2 + 2, lane);
            level_out(std::integral_constant<int, 1>{}, acc, wave % 2, wave / 2, wave / 2 + 2, f0);
        }
        {   // level 2: 32 x 64 (2 M tiles x 4 N tiles)
            const bf16_t* in[FR];
#pragma unroll
            for (int fr = 0; fr < FR; ++fr) in[fr] = sMap[1][fr];
            conv_tiles<FR, kEncNC[2], 5, 32 + 8, 2, -2, 5, 64, kEncNC[2], true>(acc, in, bw2, 0, 1, lane);
            level_out(std::integral_constant<int, 2>{}, acc, wave, 0, 1, f0);
        }
        // level 3: the 16 output bins x N tiles wave, wave + 4, staged in level 1's map
        {
            const StreamEncLevel& L = p.lev[3];
            const bf16_t* in[FR];
#pragma unroll
            for (int fr = 0; fr < FR; ++fr) in[fr] = sMap[0][fr];
            conv_tiles_n2<FR, kEncNC[3], 6, 64 + 8, 2, -2, 5, 32, kEncNC[3], true>(acc, in, bw3a, bw3b, 0, lane);
#pragma unroll
            for (int fr = 0; fr < FR; ++fr)
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const int row = lane & 15, n0 = (wave + 4 * t) * 16 + 4 * (lane >> 4);
                    *reinterpret_cast<uint2*>(sMap[1][fr] + row * 128 + n0) = prelu4_bf16(acc[fr][t], bias3[t], L.alpha);
                }
            lds_barrier();
            const int row = tid >> 4, chn = tid & 15;
#pragma unroll
            for (int fr = 0; fr < FR; ++fr) {
                const int64_t f = f0 + fr;
                const bool ok = f < F;
                const u32x4 v = *reinterpret_cast<const u32x4*>(sMap[1][fr] + row * 128 + 8 * chn);
                const int64_t eo = ((ok ? f : 0) * 16 + row) * L.ldo + L.choff + 8 * chn;
                if (ok) *reinterpret_cast<u32x4*>(L.out + eo) = v;
                if (L.q8) mx8_chunk(v, ok, L.q8, L.qs, eo, (chn & 3) == 0);
            }
        }
    }
}

// the shapes crn_enc_batch_kernel takes (those of crn_stream_enc_kernel's four levels)
bool enc_batch_ok(const EncBatchArgs& a) {
    if (a.F <= 0 || !a.x0) return false;
    for (int i = 0; i < 4; ++i) {
        const StreamEncLevel& L = a.lev[i];
        if (!L.w || !L.bias || !L.out || L.kpad % 8 || L.ldo % 8 || L.choff % 8 || L.nchunk != kEncNC[i] ||
            L.kpad < 32 * L.nchunk || L.N != (16 << i) || L.cin_shift != 3 + i)
            return false;
        if (i < 3) {
            const int Fo = 128 >> i;
            if (L.N % 16 || (Fo / 16) * (L.N / 16) != 8 || 4 % (L.N / 16) || L.nchunk > kStreamEncChunks ||
                L.cin_shift < 3 || (i > 0 && (1 << L.cin_shift) != a.lev[i - 1].N) || (i == 0 && L.cin_shift != 3) ||
                L.q8)
                return false;
        } else if (L.N != 128 || L.cin_shift != 6 || a.lev[2].N != 64 || L.nchunk > kStreamEncChunks3 ||
                   (L.q8 && (L.ldo % 32 || L.choff % 32 || !L.qs))) {
            return false;
        }
    }
    return true;
}

// Grid of a persistent frame-loop kernel: CUs x resident 256-thread blocks, cached per device id
// (handles on different devices of one process each get their own device's figure).
template <typename K>
static int persistent_grid(K* kern) {
    constexpr int kMaxDev = 64;
    static int cache[kMaxDev] = {};
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (dev < 0 || dev >= kMaxDev) dev = 0;
    if (cache[dev] == 0) {
        int ncu = 0, per = 0;
        (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
        (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void*>(kern), 256, 0);
        cache[dev] = std::max(1, ncu) * std::max(1, per);
    }
    return cache[dev];
}

template <int FR>
static hipError_t launch_enc_batch_fr(const EncBatchArgs& a, hipStream_t st) {
    const int grid = persistent_grid(crn_enc_batch_kernel<FR>);
    const int64_t need = (a.F + FR - 1) / FR;
    hipLaunchKernelGGL(crn_enc_batch_kernel<FR>, dim3((unsigned)std::min<int64_t>(grid, need)), dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_enc_batch(const EncBatchArgs& a, hipStream_t st) {
    if (a.F <= 0) return hipSuccess;
    if (!enc_batch_ok(a)) return hipErrorInvalidValue;
    static const int fr = AEC_AB_KNOB("AEC_CRN_ENC_FR", 4);
    switch (fr) {
        case 2: return launch_enc_batch_fr<2>(a, st);
        case 8: return launch_enc_batch_fr<8>(a, st);
        default: return launch_enc_batch_fr<4>(a, st);
    }
}

// --------------------------------------------------------------------------
// Fused back: decoder levels cl = 3, 2, 1 + mask + irFFT + overlap-add, one block per stream
// --------------------------------------------------------------------------
namespace {

// A decoder level (conv_tiles with ST = 1, OFF = -1, 3 taps): 8 output tiles of 16 input bins x 16
// columns, two per wave (N tile nt = wave % NT, M tiles m0 = wave / NT, m0 + 4 / NT); A rows:
// input bins i - 1 + j (j = k / Cin), zero outside [0, Fin).  load_bw: a wave's B fragments.
template <int NC>
__device__ __forceinline__ void load_bw(u32x4 (&bw)[NC], const StreamDecLevel& L, int n) {
    const bf16_t* wr = L.w + (int64_t)n * L.kpad + 8 * ((threadIdx.x & 63) >> 4);
    aec::static_for<0, NC>([&](auto ci) {
        constexpr int c = decltype(ci)::value;
        bw[c] = c < L.nchunk ? *reinterpret_cast<const u32x4*>(wr + 32 * c) : u32x4{0u, 0u, 0u, 0u};
    });
}

}  // namespace

// MX: decoder level cl = 4 folded in (a separate instantiation, as crn_stream_enc_kernel's MX4)
template <int MODE, bool MX>
__global__ __launch_bounds__(256) void crn_stream_dec_kernel(StreamDecArgs p) {
    constexpr int kMap = 5120;                    // bf16 elements of a level's padded input map (Fin x (Cin + 8))
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
    constexpr bool mx = MX;                                     // launch_stream_dec: == (p.mx.wq != nullptr)
    const u32x4* src0 = reinterpret_cast<const u32x4*>(L0.src + (int64_t)b * (32 << L0.cin_shift));
    // cl = 4 (MX): cat[4]'s shadow row pieces (16 bins x 256 B, one per thread), its scales (16 x 8
    // B, threads < 32), this wave's B fragments of N tiles wave, wave + 4 (stage st: bytes 128 st +
    // 16 g and + 64; the MX GEMM core's operand map) and their scale words
    u32x4 xq = {0u, 0u, 0u, 0u};
    uint32_t xs = 0;
    u32x4 mb[2][kStreamMxStages][2];
    uint32_t msw[2][kStreamMxStages];
    if (mx) {
        // level 0's encoder half only (channels 64 .. 127 of 32 bins: one piece per thread)
        mp[0] = src0[(tid >> 3) * 16 + 8 + (tid & 7)];
        xq = reinterpret_cast<const u32x4*>(p.mx.q8 + (int64_t)b * 4096)[tid];
        if (tid < 32) xs = reinterpret_cast<const uint32_t*>(p.mx.qs + (int64_t)b * 128)[tid];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int n = (wave + 4 * t) * 16 + (lane & 15);
            const uint8_t* wr = p.mx.wq + (int64_t)n * 768 + 16 * (lane >> 4);
            const uint32_t* sr = reinterpret_cast<const uint32_t*>(p.mx.wsc + (int64_t)n * 24);
#pragma unroll
            for (int st = 0; st < kStreamMxStages; ++st) {
                mb[t][st][0] = *reinterpret_cast<const u32x4*>(wr + 128 * st);
                mb[t][st][1] = *reinterpret_cast<const u32x4*>(wr + 128 * st + 64);
                msw[t][st] = sr[st];
            }
        }
    } else {
#pragma unroll
        for (int i = 0; i < kDecPieces; ++i) mp[i] = src0[tid + 256 * i];
    }
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
    f32x4 bias[3];
#pragma unroll
    for (int l = 0; l < 3; ++l) {
        const int NT = (p.lev[l].N + 15) >> 4;
        nt[l] = wave % NT;
        m0[l] = wave / NT;
        m1[l] = m0[l] + 4 / NT;
        const int n = nt[l] * 16 + (lane & 15);
        // transposed accumulators: the lane's 4 columns nt * 16 + 4 (lane >> 4) .. + 3
        const int c4 = nt[l] * 16 + 4 * (lane >> 4);
#pragma unroll
        for (int q = 0; q < 4; ++q) bias[l][q] = c4 + q < p.lev[l].N ? p.lev[l].bias[c4 + q] : 0.f;
    }
    load_bw(bw0, p.lev[0], nt[0] * 16 + (lane & 15));
    load_bw(bw1, p.lev[1], nt[1] * 16 + (lane & 15));
    load_bw(bw2, p.lev[2], nt[2] * 16 + (lane & 15));
    __shared__ __attribute__((aligned(16))) uint8_t sX4[16 * (256 + 16)];   // cat[4]'s shadow, rows padded
    __shared__ uint32_t sX4s[32];
    if (mx) {
        *reinterpret_cast<u32x4*>(sIn[0] + (tid >> 3) * (128 + 8) + 64 + 8 * (tid & 7)) = mp[0];
        *reinterpret_cast<u32x4*>(sX4 + (tid >> 4) * (256 + 16) + 16 * (tid & 15)) = xq;
        if (tid < 32) sX4s[tid] = xs;
    } else {
        const int C = 1 << L0.cin_shift, per = C / 8;   // 16-B pieces per map row
#pragma unroll
        for (int i = 0; i < kDecPieces; ++i) {
            const int pc = tid + 256 * i, r = pc / per, q = pc % per;
            *reinterpret_cast<u32x4*>(sIn[0] + r * (C + 8) + 8 * q) = mp[i];
        }
    }
#pragma unroll
    for (int l = 1; l < 3; ++l) {
        const int C = 1 << p.lev[l].cin_shift, half = C / 2, per = half / 8;
        const int r = tid / per, q = tid % per;
        *reinterpret_cast<u32x4*>(sIn[l] + r * (C + 8) + half + 8 * q) = mp[kDecPieces + l - 1];
    }
    lds_barrier();
    SPROF(1, 1);

    // 1b. cl = 4 (MX): 16 input bins i (one M tile) x N tiles wave, wave + 4 (parity n >= 64,
    //     channel n % 64) -> level 0's decoder half; input bin i - 1 + tap, tap = stage / 2
    if (mx) {
        f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
        const int g = lane >> 4, r = lane & 15;
        auto run = [&](auto S0, auto S1, f32x4 (&part)[2]) {
            aec::static_for<decltype(S0)::value, decltype(S1)::value>([&](auto si) {
                constexpr int st = decltype(si)::value, tap = st >> 1, kb = (st & 1) * 128;
                const int ib = r - 1 + tap;
                const bool ok = ib >= 0 && ib < 16;
                const uint8_t* row = sX4 + (ok ? ib : 0) * (256 + 16) + kb;
                const u32x4 lo = *reinterpret_cast<const u32x4*>(row + 16 * g);
                const u32x4 hi = *reinterpret_cast<const u32x4*>(row + 64 + 16 * g);
                const u32x4 z = {0u, 0u, 0u, 0u};
                const u32x4 l2 = ok ? lo : z, h2 = ok ? hi : z;
                const i32x8 af = i32x8{(int)l2[0], (int)l2[1], (int)l2[2], (int)l2[3], (int)h2[0], (int)h2[1], (int)h2[2], (int)h2[3]};
                const int sa = ok ? (int)((sX4s[(ok ? ib : 0) * 2 + (st & 1)] >> (8 * g)) & 0xFFu) : 0;
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const i32x8 bf = i32x8{(int)mb[t][st][0][0], (int)mb[t][st][0][1], (int)mb[t][st][0][2], (int)mb[t][st][0][3],
                                           (int)mb[t][st][1][0], (int)mb[t][st][1][1], (int)mb[t][st][1][2], (int)mb[t][st][1][3]};
                    const int sb = (int)((msw[t][st] >> (8 * g)) & 0xFFu);
                    part[t] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af, bf, part[t], 0, 0, 0, sa, 0, sb);
                    keep_live(bf);
                    keep_live(sb);
                }
                keep_live(af);
                keep_live(sa);
            });
        };
        if (p.mx.ksplit == 2) {   // gemm_mx8_kernel's reducer: 0 + slice 0 + slice 1
            f32x4 p0[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
            f32x4 p1[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
            run(std::integral_constant<int, 0>{}, std::integral_constant<int, 3>{}, p0);
            run(std::integral_constant<int, 3>{}, std::integral_constant<int, 6>{}, p1);
            mx_drain();
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                acc[t] += p0[t];
                acc[t] += p1[t];
            }
        } else {
            run(std::integral_constant<int, 0>{}, std::integral_constant<int, 6>{}, acc);
            mx_drain();
        }
        // epilogue (rows_epilogue_lds's: + bias, PReLU, bf16): acc[t][rr] = row 4 g + rr, column n
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int n = (wave + 4 * t) * 16 + r, par = n >= 64, ch = n - 64 * par;
            const float bn = p.mx.bias[n];
#pragma unroll
            for (int rr = 0; rr < 4; ++rr) {
                const int i = 4 * g + rr;
                float v = acc[t][rr] + bn;
                v = v >= 0.f ? v : p.mx.alpha * v;
                sIn[0][(2 * i + par) * (128 + 8) + ch] = f2bf(v);
            }
        }
        lds_barrier();
    }

    // 2. decoder levels cl = 3, 2: output bins 2 i + parity, channel n -> the next map's decoder half
#pragma unroll
    for (int l = 0; l < 2; ++l) {
        const StreamDecLevel& L = p.lev[l];
        const int Co = L.N >> 1, Cn = 1 << p.lev[l + 1].cin_shift;
        f32x4 acc2[1][2];
        const bf16_t* in[1] = {sIn[l]};
        if (l == 0) conv_tiles<1, kStreamDecChunks0, 7, 128 + 8, 1, -1, 3, 32, kStreamDecChunks0, true>(acc2, in, bw0, m0[0], m1[0], lane);
        else conv_tiles<1, kStreamDecChunks1, 6, 64 + 8, 1, -1, 3, 64, kStreamDecChunks1, true>(acc2, in, bw1, m0[1], m1[1], lane);
        const f32x4 (&acc)[2] = acc2[0];
        const int c4 = nt[l] * 16 + 4 * (lane >> 4), par = c4 >= Co, ch = c4 - par * Co;
        bf16_t* next = sIn[l + 1];
        const float4 b4 = make_float4(bias[l][0], bias[l][1], bias[l][2], bias[l][3]);
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int i = (t ? m1[l] : m0[l]) * 16 + (lane & 15);
            *reinterpret_cast<uint2*>(next + (2 * i + par) * (Cn + 8) + ch) = prelu4_bf16(acc[t], b4, L.alpha);
        }
        lds_barrier();
        SPROF(1, 2 + l);
    }
    // 3. the mask level (cl = 1): columns (parity, re / im), f32, act none (v2) / tanh (v1)
    {
        const StreamDecLevel& L = p.lev[2];
        f32x4 acc2[1][2];
        const bf16_t* in[1] = {sIn[2]};
        conv_tiles<1, kStreamDecChunks2, 5, 32 + 8, 1, -1, 3, 128, kStreamDecChunks2, true>(acc2, in, bw2, m0[2], m1[2], lane);
        const f32x4 (&acc)[2] = acc2[0];
        // materialised in every lane before the lane-divergent store (else the compiler may sink the
        // MFMAs into it, where the other lanes' operand reads do not run; see the level-4 epilogue)
#ifndef CRN_NO_CODEGEN_GUARDS
        asm volatile("" ::"v"(acc[0]), "v"(acc[1]));
#endif
        // the 4 columns (parity, re / im) of input bin i sit in the lanes with lane >> 4 == 0
        if ((lane >> 4) == 0) {
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const int i = (t ? m1[2] : m0[2]) * 16 + (lane & 15);
                float v[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    v[q] = acc[t][q] + bias[2][q];
                    if (L.act == 2) v[q] = tanhf(v[q]);            // the batch epilogue's apply_act<2>
                }
                *reinterpret_cast<float4*>(reinterpret_cast<float*>(sMask) + 4 * i) = make_float4(v[0], v[1], v[2], v[3]);
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

// --------------------------------------------------------------------------
// Batch decoder levels cl = 3, 2 (the batch forward of C3 / C4): FR frames per block in a
// persistent frame loop, the per-hop back's level arithmetic (conv_tiles, both parities per
// GEMM, the PReLU epilogue) with the maps in padded LDS rows; cat[2]'s decoder half never
// leaves LDS, cat[1]'s leaves as 16-B rows for crn_back_kernel's mask level.  The inputs of
// the next FR frames (cat[3] whole, cat[2]'s encoder half) are fetched into registers while
// the current ones run.  Bit-identical to the two row GEMMs (test_batch_dec_fused_bit_exact).
// --------------------------------------------------------------------------
template <int FR>
__global__ __launch_bounds__(256, 1) void crn_dec_batch_kernel(DecBatchArgs p) {
    constexpr int kA = 32 * (128 + 8), kB = 64 * (64 + 8), kO = 128 * 16;
    __shared__ __attribute__((aligned(16))) bf16_t sA[FR][kA];
    __shared__ __attribute__((aligned(16))) bf16_t sB[FR][kB];
    __shared__ __attribute__((aligned(16))) bf16_t sO[FR][kO];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const StreamDecLevel& LA = p.lev[0];
    const StreamDecLevel& LB = p.lev[1];
    u32x4 bw0[kStreamDecChunks0], bw1[kStreamDecChunks1];
    const int nt0 = wave % 4, nt1 = wave % 2, mb0 = wave / 2;      // level A: 4 N tiles x M tiles 0, 1
    const int n0 = nt0 * 16 + (lane & 15), n1 = nt1 * 16 + (lane & 15);
    load_bw(bw0, LA, n0);
    load_bw(bw1, LB, n1);
    // TR epilogue: the lane's 4 columns nt * 16 + 4 (lane >> 4) .. + 3 (one parity: Co % 4 == 0)
    const int c0 = nt0 * 16 + 4 * (lane >> 4), c1 = nt1 * 16 + 4 * (lane >> 4);
    const float4 bias0 = *reinterpret_cast<const float4*>(LA.bias + c0);
    const float4 bias1 = *reinterpret_cast<const float4*>(LB.bias + c1);
    const int64_t F = p.F, step = (int64_t)gridDim.x * FR;
    // cat[3]: 512 16-B pieces per frame (2 per thread); cat[2]'s encoder half: 64 rows x 4 pieces
    u32x4 na[FR][2], nb[FR];
    auto fetch = [&](int64_t fb) {
#pragma unroll
        for (int fr = 0; fr < FR; ++fr) {
            const int64_t f = fb + fr;
            const bool ok = f < F;
            const u32x4* a3 = reinterpret_cast<const u32x4*>(LA.src + (ok ? f : 0) * 4096);
            na[fr][0] = ok ? a3[tid] : u32x4{0u, 0u, 0u, 0u};
            na[fr][1] = ok ? a3[tid + 256] : u32x4{0u, 0u, 0u, 0u};
            nb[fr] = ok ? *reinterpret_cast<const u32x4*>(LB.src + ((ok ? f : 0) * 64 + (tid >> 2)) * 64 + 32 + 8 * (tid & 3))
                        : u32x4{0u, 0u, 0u, 0u};
        }
    };
    fetch((int64_t)blockIdx.x * FR);
    for (int64_t f0 = (int64_t)blockIdx.x * FR; f0 < F; f0 += step) {
#pragma unroll
        for (int fr = 0; fr < FR; ++fr) {
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int pc = tid + 256 * h, r = pc >> 4, q = pc & 15;
                *reinterpret_cast<u32x4*>(sA[fr] + r * 136 + 8 * q) = na[fr][h];
            }
            *reinterpret_cast<u32x4*>(sB[fr] + (tid >> 2) * 72 + 32 + 8 * (tid & 3)) = nb[fr];
        }
        lds_barrier();
        fetch(f0 + step);
        // level cl = 3: M = 32 input bins (tiles 0, 1), N = 64 (parity x 32 channels) -> sB's decoder half
        {
            f32x4 acc[FR][2];
            const bf16_t* in[FR];
#pragma unroll
            for (int fr = 0; fr < FR; ++fr) in[fr] = sA[fr];
            conv_tiles<FR, kStreamDecChunks0, 7, 136, 1, -1, 3, 32, kStreamDecChunks0, true>(acc, in, bw0, 0, 1, lane);
            const int par = c0 >= 32, ch = c0 - 32 * par;
#pragma unroll
            for (int fr = 0; fr < FR; ++fr)
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const int i = t * 16 + (lane & 15);
                    *reinterpret_cast<uint2*>(sB[fr] + (2 * i + par) * 72 + ch) = prelu4_bf16(acc[fr][t], bias0, LA.alpha);
                }
        }
        lds_barrier();
        // level cl = 2: M = 64 input bins (tiles mb0, mb0 + 2), N = 32 (parity x 16 channels) -> sO
        {
            f32x4 acc[FR][2];
            const bf16_t* in[FR];
#pragma unroll
            for (int fr = 0; fr < FR; ++fr) in[fr] = sB[fr];
            conv_tiles<FR, kStreamDecChunks1, 6, 72, 1, -1, 3, 64, kStreamDecChunks1, true>(acc, in, bw1, mb0, mb0 + 2, lane);
            const int par = c1 >= 16, ch = c1 - 16 * par;
#pragma unroll
            for (int fr = 0; fr < FR; ++fr)
#pragma unroll
                for (int t = 0; t < 2; ++t) {
                    const int i = (mb0 + 2 * t) * 16 + (lane & 15);
                    *reinterpret_cast<uint2*>(sO[fr] + (2 * i + par) * 16 + ch) = prelu4_bf16(acc[fr][t], bias1, LB.alpha);
                }
        }
        lds_barrier();
        // cat[1]'s decoder half: 128 rows x 32 B (two 16-B pieces per row, one per thread)
#pragma unroll
        for (int fr = 0; fr < FR; ++fr) {
            const int64_t f = f0 + fr;
            if (f < F)
                *reinterpret_cast<u32x4*>(p.out + (f * 128 + (tid >> 1)) * p.ldo1 + 8 * (tid & 1)) =
                    *reinterpret_cast<const u32x4*>(sO[fr] + tid * 8);
        }
    }
}

bool dec_batch_ok(const DecBatchArgs& a) {
    if (a.F <= 0 || !a.out || a.ldo1 % 8 || a.ldo1 < 16) return false;
    const int caps[2] = {kStreamDecChunks0, kStreamDecChunks1};
    const int cs[2] = {7, 6}, N[2] = {64, 32};
    for (int l = 0; l < 2; ++l) {
        const StreamDecLevel& L = a.lev[l];
        if (!L.w || !L.bias || !L.src || L.nchunk != caps[l] || L.kpad < 32 * L.nchunk || L.kpad % 8 ||
            L.act != 1 || L.cin_shift != cs[l] || L.N != N[l])
            return false;
    }
    return true;
}

hipError_t launch_dec_batch(const DecBatchArgs& a, hipStream_t st) {
    if (a.F <= 0) return hipSuccess;
    if (!dec_batch_ok(a)) return hipErrorInvalidValue;
    constexpr int FR = 4;
    const int grid = persistent_grid(crn_dec_batch_kernel<FR>);
    const int64_t need = (a.F + FR - 1) / FR;
    hipLaunchKernelGGL(crn_dec_batch_kernel<FR>, dim3((unsigned)std::min<int64_t>(grid, need)), dim3(256), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_stream_dec(const StreamDecArgs& a, int mode, hipStream_t st) {
    if (a.B <= 0) return hipSuccess;
    const int caps[3] = {kStreamDecChunks0, kStreamDecChunks1, kStreamDecChunks2};
    for (int l = 0; l < 3; ++l) {
        const StreamDecLevel& L = a.lev[l];
        const int Fin = 32 << l, NT = (L.N + 15) / 16;
        if (!L.w || !L.bias || !L.src || L.nchunk != caps[l] || L.kpad < 32 * L.nchunk || L.cin_shift != 7 - l ||
            (Fin / 16) * NT != 8 || 4 % NT || (Fin << L.cin_shift) > 4096 ||
            (l < 2 && (L.N % 32 || L.act != 1 || L.N != (1 << a.lev[l + 1].cin_shift))) ||   // Co = next map's half
            (l == 2 && (L.N != 4 || L.act == 1)))
            return hipErrorInvalidValue;
        const int C = 1 << L.cin_shift;
        if (l == 0 ? Fin * C != 2 * 256 * 8 : Fin * (C / 2) != 256 * 8) return hipErrorInvalidValue;   // the load's piece counts
    }
    if (mode < 0 || mode > 2) return hipErrorInvalidValue;
    const bool mx = a.mx.wq != nullptr;
#define CRN_DEC_CASE(M)                                                                                     \
    if (mode == M) {                                                                                        \
        if (mx)                                                                                             \
            hipLaunchKernelGGL((crn_stream_dec_kernel<M, true>), dim3((unsigned)a.B), dim3(256), 0, st, a);  \
        else                                                                                                \
            hipLaunchKernelGGL((crn_stream_dec_kernel<M, false>), dim3((unsigned)a.B), dim3(256), 0, st, a); \
    }
    CRN_DEC_CASE(0) CRN_DEC_CASE(1) CRN_DEC_CASE(2)
#undef CRN_DEC_CASE
    return hipGetLastError();
}

}  // namespace crn

#ifdef AEC_STREAM_PROF
extern "C" int aec_debug_stream_prof(void* host, size_t bytes) {
    if (bytes < sizeof(crn::g_sprof)) return -1;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(crn::g_sprof), sizeof(crn::g_sprof)) == hipSuccess ? 0 : -2;
}
#endif
