// aec_pipe.hip — K6: the whole per-frame loop of one stream in one block (gfx950).
//
// Reference path: Little_net.forward (Stage2_lhm/scripts/network/ERB.py:252-334)
// with its ConvSTFT / ConviSTFT (scripts/network/attention_ccrn.py:45-101),
// plus the build-defined FD-NLMS between the STFT and the
// post-filter.
//
// Why one block per stream.  The per-stream GRU (ERB.py:293) is a chain of T
// dependent steps of ~680 cycles: ~0.2 ms for a 10 s stream whatever else the
// chip does.  Run as separate kernels (analysis for every stream, then GRU +
// synthesis for every stream) the analysis and the recurrence serialise and
// the error spectrum E makes a 2 KiB-per-frame round trip through HBM.  Here
// all roles of a stream share its CU and run as a pipeline over chunks of 8
// frames ("ticks"), so the transforms, the NLMS and the synthesis hide under
// the recurrence, and E only crosses a 4-chunk ring that stays in the XCD's L2.
//
// 16 waves (128 VGPRs each, 4 per SIMD; waves w, w+4, w+8, w+12 share a SIMD),
// roles by wave index; in tick c ("|" = the mid-tick barrier B1, every tick
// ends with B2):
//   w0       GRU   recurrence of chunk c-3 (kGruA steps | the rest)
//   w1       HD    head / mask / est_erb / loss of chunk c-4 (4 frames | 4 frames)
//   w2, w3   GI    gi = W_ih x + b of chunk c-2 | overlap-add + WOLA of chunk c-5 -> out
//   w4..w7   NL    NLMS recursion of chunk c-1 -> E rows (LDS + ring) | copy the
//                  M / R rows of chunk c into registers (bin k = lane + 64 (w-4);
//                  lane 0 also bin 256)
//   w8, w9   MIC   mic transform of chunk c -> M rows | mic_erb = ERB(|E|) of chunk c-1
//   w10,w11  REF   ref transform of chunk c -> ref_erb, R rows |
//   w12,w13  NEAR  near transform of chunk c -> near_erb (loss) |
//   w14,w15  SY    synthesis of chunk c-5 (gains, irFFT, window) | E rows of chunk c-4
//                  from the ring into LDS
// Every wave that transforms does one 4-frame pass per tick, all of them
// before B1, so the tick is one transform pass plus the mic_erb pass long.
// B1 orders the M / R rows (written before it) against the NL copy and the E
// rows against the mic_erb pass; B2 frees them for the next tick.  Hand-offs
// more than one tick apart go through LDS rings indexed by chunk.
//
// Per-frame arithmetic is the batch kernels' own (aec_frame.h / aec_stft.h /
// aec_fft.h: same FFT, ERB schedule, NlmsBin, gi / gru_step / head_mask,
// synth_frame, OLA expression), so the waveform and every intermediate are
// bit-identical to nlms_analysis_kernel + gru_synth_kernel (NLMS) and to
// analysis_kernel + gru_kernel + synthesis_kernel (bypass, taps = 0: E = M);
// only the loss is summed in another order (tests/test_gpu_nlms.py).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "aec_fft.h"
#include "aec_frame.h"
#include "aec_launch.h"
#include "aec_stft.h"
#include "aec_tables.h"

#ifndef PIPE_GRU_A
#define PIPE_GRU_A 6          // GRU steps before the mid-tick barrier (the rest after it)
#endif

namespace aec {

namespace {
constexpr int kPF = kPipeFrames;          // 8 frames per tick
constexpr int kWaves = 16;
constexpr int kThreads = 64 * kWaves;
constexpr int kERowP = 512 + 48;          // LDS error row: 256 float2 + ERB partials
constexpr int kEstSP = 33;
constexpr int kSchedMax = 32;             // ERB schedule entries per lane (erb_conf: 32)
constexpr int kGruA = PIPE_GRU_A;

enum : int { W_GRU = 0, W_HD = 1, W_GI0 = 2, W_NL0 = 4, W_MIC0 = 8, W_REF0 = 10, W_NEAR0 = 12, W_SY0 = 14 };

// LDS carve (floats).  Every offset is a compile-time constant: LDS addresses
// become instruction immediates and cost no SGPR / VGPR.
struct Carve {
    int sched = 0, comb = 0, tw512 = 0, twT = 0, hann = 0, coff = 0, bin = 0, tf = 0, sy = 0, e = 0, gi = 0,
        h = 0, hb = 0, micr = 0, refr = 0, nearr = 0, est = 0, o = 0, ec = 0, c = 0, w2t = 0, sye = 0, total = 0;
    constexpr Carve() {
        int o_ = 0;
        auto take = [&](int n) { const int r = o_; o_ += (n + 3) & ~3; return r; };
        sched = take(64 * kSchedMax);
        comb = take(64);
        tw512 = take(516);
        twT = take(512);
        hann = take(512);
        coff = take(256);
        bin = take(260 * 4);
        tf = take(6 * kWaveFloats);          // MIC0, MIC1, REF0, REF1, NEAR0, NEAR1
        sy = take(2 * kWaveFloats);
        e = take(kPF * kERowP);
        gi = take(2 * kPF * 96);
        h = take(2 * kPF * 32);
        hb = take(32);
        micr = take(4 * kPF * 32);           // mic_erb ring (chunk & 3)
        refr = take(4 * kPF * 32);           // ref_erb ring (chunk & 3)
        nearr = take(8 * kPF * 32);          // near_erb ring (chunk & 7)
        est = take(2 * kPF * kEstSP);
        o = take(2 * 32);
        ec = take(2 * 256);                  // OLA tail: second half of a chunk's last frame
        c = take(4);
        w2t = take(32 * 32);                 // linear2 weight transposed [k][j] (head wave)
        sye = take(kPF * 512);               // E rows of the chunk the SY waves synthesise next
        total = o_;
    }
};
constexpr Carve kC{};
static_assert(kC.total * 4 <= 160 * 1024, "LDS budget");

template <int OFF>
__device__ __forceinline__ float* lds() {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    return smem + OFF;
}

__device__ __forceinline__ void barrier_lds() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xC07F);       // lgkmcnt(0), vmcnt / expcnt untouched
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ void wait_vm0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// One transform pass: stage the prefetched hops of 4 frames at wt (x - c inside
// [0, n)), prefetch the next task, window + rFFT-512 -> xa / xb / x128.
__device__ __forceinline__ void transform4(float* wr, float* scr, float4 (&pf)[kWavePf], float cval, int n, int wt,
                                           int lane, int gg, int lb, const float* sHann, const float2* sTwT,
                                           const float2* sTw512, const float* next_row, int next_n, int next_wt,
                                           bool next_al, float2 (&xa)[8], float2 (&xb)[8], float2& x128) {
    asm volatile("" ::: "memory");
    wave_commit(wr, pf, cval, n, wt, lane);
    if (next_row) wave_prefetch(pf, next_row, next_n, next_wt, lane, next_al);
    wave_fence();
    float2 v[16];
    load_frame(v, wr, sHann, gg, lb);
    wave_fence();
    fft256<false>(v, lb, scr, sTwT);
    rfft_unpack(v, lb, sTw512, xa, xb, x128);
}

__device__ __forceinline__ bool row_aligned(const float* base, int64_t ld) {
    return ((ld & 3) == 0) && ((reinterpret_cast<uintptr_t>(base) & 15) == 0);
}

// gi = W_ih[row] . x + bias with x = [mic_erb, |mic_erb - ref_erb|] read from
// the two feature rows (ERB.py:287-290), W_ih[row] in registers: gru_gi's exact
// operation order (aec_frame.h), so the same bits.  Partly unrolled: the fully
// unrolled form hoists all 16 x vectors and spills at 128 VGPRs.
__device__ __forceinline__ float gi_row(const float (&wih)[64], const float* xm, const float* xr, float gbias) {
    const float4* m4 = reinterpret_cast<const float4*>(xm);
    const float4* r4 = reinterpret_cast<const float4*>(xr);
    f2v a0 = {0.f, 0.f}, a1 = {0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 8; ++q) {
        const float4 xv = m4[q];
        a0 = __builtin_elementwise_fma(f2v{wih[4 * q], wih[4 * q + 1]}, f2v{xv.x, xv.y}, a0);
        a1 = __builtin_elementwise_fma(f2v{wih[4 * q + 2], wih[4 * q + 3]}, f2v{xv.z, xv.w}, a1);
    }
#pragma unroll
    for (int q = 8; q < 16; ++q) {
        const float4 a = m4[q - 8], r = r4[q - 8];
        const float4 xv = make_float4(fabsf(a.x - r.x), fabsf(a.y - r.y), fabsf(a.z - r.z), fabsf(a.w - r.w));
        a0 = __builtin_elementwise_fma(f2v{wih[4 * q], wih[4 * q + 1]}, f2v{xv.x, xv.y}, a0);
        a1 = __builtin_elementwise_fma(f2v{wih[4 * q + 2], wih[4 * q + 3]}, f2v{xv.z, xv.w}, a1);
    }
    const f2v s2 = a0 + a1;
    return gbias + (s2.x + s2.y);
}

// head_mask (aec_frame.h) with linear2's weights read from LDS (w2t[k][j] =
// W2[j][k]) instead of registers: the same operations in the same order.
__device__ __forceinline__ float head_mask_w2lds(const float (&w1)[64], const float* w2t, float b1j, float b2j,
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
        const float w0 = w2t[(4 * q) * 32 + j], w1_ = w2t[(4 * q + 1) * 32 + j];
        const float w2_ = w2t[(4 * q + 2) * 32 + j], w3 = w2t[(4 * q + 3) * 32 + j];
        c0 = __builtin_elementwise_fma(f2v{w0, w1_}, f2v{ov.x, ov.y}, c0);
        c1 = __builtin_elementwise_fma(f2v{w2_, w3}, f2v{ov.z, ov.w}, c1);
    }
    wave_fence();                                   // the row is reused by the group's next frame
    const f2v s2 = c0 + c1;
    return sigmoidf_(b2j + (s2.x + s2.y));
}

struct PipeStream {
    int b, n, T, nhop, nch, nticks;
    bool have_near;
};

}  // namespace

size_t pipe_smem_bytes(int sched_len) { return sched_len <= kSchedMax ? (size_t)kC.total * 4 : SIZE_MAX; }

// ---------------------------------------------------------------- GRU -----
__device__ __forceinline__ void role_gru(const PipeArgs& p, const PipeStream& s) {
    const int lane = threadIdx.x & 63;
    float* sGi = lds<kC.gi>();
    float* sH = lds<kC.h>();
    float* sHb = lds<kC.hb>();
    __builtin_amdgcn_s_setprio(3);
    const float* W_hh = p.w + 96 * 64;
    const float* b_hh = W_hh + 96 * 32 + 96;
    const int j = lane & 31, kh = lane >> 5;
    f2v wrz[16], wn[8];
    {
        const float* rR = W_hh + j * 32 + 16 * kh;
        const float* rZ = W_hh + (32 + j) * 32 + 16 * kh;
        const float* rN = W_hh + (64 + j) * 32 + 16 * kh;
#pragma unroll
        for (int k = 0; k < 16; ++k) wrz[k] = f2v{rR[k], rZ[k]};
#pragma unroll
        for (int i = 0; i < 8; ++i) wn[i] = f2v{rN[2 * i], rN[2 * i + 1]};
    }
    const float bhn = b_hh[64 + j];
    float hj = 0.f;
    if (lane < 32) sHb[lane] = 0.f;
    for (int c = 0; c < s.nticks; ++c) {
        const int cg = c - 3;
        const bool act = cg >= 0 && cg < s.nch && !(p.mode & 1);
        const int f_end = act ? min(kPF, s.T - cg * kPF) : 0;
        const float* gi = sGi + (cg & 1) * kPF * 96;
        float* hrow = sH + (cg & 1) * kPF * 32;
        auto steps = [&](int f0, int f1) {
            if (f0 >= f1) return;
            float gr = gi[f0 * 96 + j], gz = gi[f0 * 96 + 32 + j], gn = gi[f0 * 96 + 64 + j];
            for (int f = f0; f < f1; ++f) {
                const int fn = f + 1 < f1 ? f + 1 : f;
                const float ngr = gi[fn * 96 + j], ngz = gi[fn * 96 + 32 + j], ngn = gi[fn * 96 + 64 + j];
                hj = gru_step(wrz, wn, sHb, kh, gr, gz, gn, bhn, hj);
                if (kh == 0) {
                    sHb[j] = hj;
                    hrow[f * 32 + j] = hj;
                }
                gr = ngr; gz = ngz; gn = ngn;
            }
        };
        steps(0, min(kGruA, f_end));
        barrier_lds();
        steps(kGruA, f_end);
        barrier_lds();
    }
}

// ------------------------------------------------ head / mask / est / loss ----
__device__ __forceinline__ void role_hd(const PipeArgs& p, const PipeStream& s) {
    const int lane = threadIdx.x & 63;
    const float* sH = lds<kC.h>();
    const float* sMicR = lds<kC.micr>();
    const float* sNearR = lds<kC.nearr>();
    float* sEst = lds<kC.est>();
    float* sO = lds<kC.o>();
    const float* W1 = p.w + 96 * 64 + 96 * 32 + 96 + 96;
    const float* b1 = W1 + 32 * 64;
    const float* W2 = b1 + 32;
    const float* b2 = W2 + 32 * 32;
    const int g = lane >> 5, j = lane & 31;
    float w1[64];
#pragma unroll
    for (int k = 0; k < 64; ++k) w1[k] = W1[j * 64 + k];
    const float* sW2T = lds<kC.w2t>();                        // W2[j][k] at [k][j]: conflict-free
    const float b1j = b1[j], b2j = b2[j];
    (void)W2;
    float lacc = 0.f;
    for (int c = 0; c < s.nticks; ++c) {
        const int ch = c - 4;
        const bool act = ch >= 0 && ch < s.nch && !(p.mode & 4);
        auto frames = [&](int f0) {
#pragma unroll 1
            for (int f = f0 + g; f < f0 + 4; f += 2) {
                const int t = ch * kPF + f;
                float est = 0.f;
                if (t < s.T) {                                    // uniform within the 32-lane group
                    const float* hrow = sH + ((ch & 1) * kPF + f) * 32;
                    const float* mrow = sMicR + ((ch & 3) * kPF + f) * 32;
                    const float mask = head_mask_w2lds(w1, sW2T, b1j, b2j, hrow, mrow, sO + g * 32, j);
                    est = mask * mrow[j];
                    if (s.have_near) {
                        const float d = sqrtf(sNearR[((ch & 7) * kPF + f) * 32 + j]) - sqrtf(est);
                        lacc += d * d;
                    }
                    if (p.est) {
                        const int64_t o_idx = ((int64_t)s.b * p.Tmax + t) * 32 + j;
                        p.est[o_idx] = est;
                        if (p.dbg_h) p.dbg_h[o_idx] = hrow[j];
                        if (p.dbg_mask) p.dbg_mask[o_idx] = mask;
                    }
                }
                sEst[((ch & 1) * kPF + f) * kEstSP + j] = est;    // frames past the end: gain 0
            }
        };
        if (act) frames(0);
        barrier_lds();
        if (act) frames(4);
        barrier_lds();
    }
    if (p.loss) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) lacc += __shfl_xor(lacc, o);
        if (lane == 0) p.loss[s.b] = lacc / (float)(s.T * 32);
    }
}

// ----------------------- input projection | overlap-add + WOLA ----------
__device__ __forceinline__ void role_gi(const PipeArgs& p, const PipeStream& s) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int w = wave - W_GI0;
    const float* sMicR = lds<kC.micr>();
    const float* sRefR = lds<kC.refr>();
    float* sGi = lds<kC.gi>();
    const float* sSY = lds<kC.sy>();
    const float* sCoff = lds<kC.coff>();
    float* sEC = lds<kC.ec>();
    // gi: row = 64 w + lane (wave 1: lanes 0..31), all 8 frames of the chunk
    const int grow = 64 * w + lane;
    const bool has_row = grow < 96;
    const int rr = has_row ? grow : 0;
    float wih[64];
#pragma unroll
    for (int k = 0; k < 64; ++k) wih[k] = p.w[rr * 64 + k];
    const float* b_ih = p.w + 96 * 64 + 96 * 32;
    const float* b_hh = b_ih + 96;
    const float gbias = b_ih[rr] + (rr < 64 ? b_hh[rr] : 0.f);
    float* orow = p.out + (int64_t)s.b * p.ld_out;
    const bool oal = row_aligned(p.out, p.ld_out);
    // output hop j (256 samples) = second half of one frame + first half of the next
    auto ola = [&](const float* a_half, const float* c_half, int64_t j) {
        if (j < 0 || j >= s.nhop) return;
        if (oal) {
            const int r = 4 * lane;
            const float4 a = *reinterpret_cast<const float4*>(a_half + r);
            const float4 cv = *reinterpret_cast<const float4*>(c_half + r);
            const float4 cf = *reinterpret_cast<const float4*>(sCoff + r);
            typedef float f4v __attribute__((ext_vector_type(4)));
            f4v o;
            o.x = (a.x + cv.x) * cf.x + 1e-9f;
            o.y = (a.y + cv.y) * cf.y + 1e-9f;
            o.z = (a.z + cv.z) * cf.z + 1e-9f;
            o.w = (a.w + cv.w) * cf.w + 1e-9f;
            __builtin_nontemporal_store(o, reinterpret_cast<f4v*>(orow + j * kHop + r));
        } else {
#pragma unroll
            for (int u = 0; u < 4; ++u) {
                const int r = lane + 64 * u;
                orow[j * kHop + r] = (a_half[r] + c_half[r]) * sCoff[r] + 1e-9f;
            }
        }
    };
    auto fr = [&](int f) { return sSY + (f >> 2) * kWaveFloats + (f & 3) * kGroupFloats; };
    for (int c = 0; c < s.nticks; ++c) {
        const int cs = c - 2;
        if (has_row && cs >= 0 && cs < s.nch && !(p.mode & 64)) {
#pragma unroll 1
            for (int f = 0; f < kPF; ++f) {
                const int row = (cs & 3) * kPF + f;
                sGi[((cs & 1) * kPF + f) * 96 + grow] = gi_row(wih, sMicR + row * 32, sRefR + row * 32, gbias);
            }
        }
        barrier_lds();
        const int co = c - 5;
        if (co >= 0 && co < s.nch && !(p.mode & 2)) {
            // hops j0 + f: wave 0 f = -1 (previous chunk's frame 7 + frame 0) .. 3, wave 1 f = 4 .. 6
            const int64_t j0 = (int64_t)co * kPF;
            const int f_lo = w == 0 ? -1 : 4, f_hi = w == 0 ? 4 : 7;
#pragma unroll 1
            for (int f = f_lo; f < f_hi; ++f)
                ola(f < 0 ? sEC + ((co - 1) & 1) * 256 : fr(f) + 256, fr(f + 1), j0 + f);
            if (w == 1)
                for (int r = lane; r < 256; r += 64) sEC[(co & 1) * 256 + r] = fr(7)[256 + r];
        }
        barrier_lds();
    }
}

// ---------------------------------------------------------- synthesis ----
__device__ __forceinline__ void role_sy(const PipeArgs& p, const PipeStream& s) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int gg = lane >> 4, lb = lane & 15;
    const int w = wave - W_SY0;
    const int fi = 4 * w + gg;                                // frame of the chunk this group synthesises
    float* scr = lds<kC.sy>() + w * kWaveFloats + gg * kGroupFloats;
    const float* sEst = lds<kC.est>();
    const float4* sBin = reinterpret_cast<const float4*>(lds<kC.bin>());
    const float2* sTw512 = reinterpret_cast<const float2*>(lds<kC.tw512>());
    const float2* sTwT = reinterpret_cast<const float2*>(lds<kC.twT>());
    const float* sHann = lds<kC.hann>();
    float* sSyE = lds<kC.sye>();
    const float2* ring = p.ring + (int64_t)s.b * kPipeRingRows * 256;
    for (int c = 0; c < s.nticks; ++c) {
        const int cs = c - 5;
        if (cs >= 0 && cs < s.nch && !(p.mode & 2)) {
            float2 xa[8], xb[8], x128;
            row_to_pairs(reinterpret_cast<const float2*>(sSyE + fi * 512), lb, true, xa, xb, x128);
            synth_frame(xa, xb, x128, sEst + ((cs & 1) * kPF + fi) * kEstSP, sBin, sTw512, sTwT, sHann, scr, lb);
        }
        barrier_lds();
        // E rows of chunk c-4 (this wave's 4 frames) -> sSyE, nt loads: written by the NL
        // waves of this CU three ticks ago, served by the XCD's L2 (L1 bypassed)
        const int cl = c - 4;
        if (cl >= 0 && cl < s.nch && !(p.mode & 2)) {
            typedef float f4t __attribute__((ext_vector_type(4)));
            const f4t* src = reinterpret_cast<const f4t*>(ring + ((cl & 3) * kPF + 4 * w) * 256);
            f4t* dst = reinterpret_cast<f4t*>(sSyE + 4 * w * 512);
            f4t v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = __builtin_nontemporal_load(src + lane + 64 * u);
#pragma unroll
            for (int u = 0; u < 8; ++u) dst[lane + 64 * u] = v[u];
        }
        wait_vm0();            // the ring slot read here is rewritten by the NL waves next tick
        barrier_lds();
    }
}

// --------------------------------------------------- NLMS recursion ------
template <int TAPS>
__device__ __forceinline__ void role_nl(const PipeArgs& p, const PipeStream& s) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int q = wave - W_NL0;
    const int k = lane + 64 * q;                               // bin k; lane 0 also bin 256
    float* sE = lds<kC.e>();
    const float* sTF = lds<kC.tf>();
    float2* ring = p.ring + (int64_t)s.b * kPipeRingRows * 256;
    NlmsBin<(TAPS > 0 ? TAPS : 1)> st;
    st.reset(k == 0);
    const float mu = p.mu, beta = p.beta, delta = p.delta;
    float2 dd[kPF], rr[kPF];
    for (int c = 0; c < s.nticks; ++c) {
        const int c1 = c - 1;
        if (c1 >= 0 && c1 < s.nch && !(p.mode & 8)) {
            float2* rs = ring + (c1 & 3) * kPF * 256;
#pragma unroll
            for (int i = 0; i < kPF; ++i) {
                float2 e;
                if constexpr (TAPS > 0) e = st.step(dd[i], rr[i], mu, beta, delta);
                else e = dd[i];                                // NLMS bypass: E = M (Little_net's own path)
                reinterpret_cast<float2*>(sE + i * kERowP)[k] = e;
                rs[i * 256 + k] = e;
            }
        }
        barrier_lds();
        if (c < s.nch && !(p.mode & 8)) {
#pragma unroll
            for (int i = 0; i < kPF; ++i) {
                const float* mb = sTF + (i >> 2) * kWaveFloats + (i & 3) * kGroupFloats;         // MIC waves
                const float* rb = sTF + (2 + (i >> 2)) * kWaveFloats + (i & 3) * kGroupFloats;   // REF waves
                dd[i] = reinterpret_cast<const float2*>(mb)[k];
                if constexpr (TAPS > 0) rr[i] = reinterpret_cast<const float2*>(rb)[k];
            }
        }
        wait_vm0();            // this tick's E stores are in L2 before the SY waves read them
        barrier_lds();
    }
}

// ------------------------------------------------------- transforms ------
// kind 0 (MIC): mic transform -> M rows | mic_erb = ERB(|E|) of chunk c-1
// kind 1 (REF): ref transform -> ref_erb, R rows |
// kind 2 (NEAR): near transform -> near_erb |
template <int KIND>
__device__ __forceinline__ void role_tf(const PipeArgs& p, const PipeStream& s) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int gg = lane >> 4, lb = lane & 15, sw = 16 * (gg & 1);
    const int m = wave - (KIND == 0 ? W_MIC0 : (KIND == 1 ? W_REF0 : W_NEAR0));
    float* wr = lds<kC.tf>() + (2 * KIND + m) * kWaveFloats;
    float* scr = wr + gg * kGroupFloats;
    const float4* sSched = reinterpret_cast<const float4*>(lds<kC.sched>());
    const int2* sComb = reinterpret_cast<const int2*>(lds<kC.comb>());
    const float2* sTw512 = reinterpret_cast<const float2*>(lds<kC.tw512>());
    const float2* sTwT = reinterpret_cast<const float2*>(lds<kC.twT>());
    const float* sHann = lds<kC.hann>();
    float* sE = lds<kC.e>();
    float* ring_erb = KIND == 0 ? lds<kC.micr>() : (KIND == 1 ? lds<kC.refr>() : lds<kC.nearr>());
    const int L = p.sched_len;
    const bool on = KIND != 2 || s.have_near;
    const float* row = on ? p.sig[KIND == 0 ? 0 : (KIND == 1 ? 1 : 2)] + (int64_t)s.b * p.ld : nullptr;
    const bool al = on && row_aligned(p.sig[KIND == 0 ? 0 : (KIND == 1 ? 1 : 2)], p.ld);
    const int n = KIND == 0 ? s.n : p.slen[4 * s.b + KIND];
    const float cval = lds<kC.c>()[KIND];
    float* feats = p.feats ? p.feats + (int64_t)s.b * p.Tmax * 96 : nullptr;
    const int foff = KIND == 0 ? 0 : (KIND == 1 ? 32 : 64);
    const bool tf = on && !(p.mode & (KIND == 0 ? 16 : (KIND == 1 ? 32 : 128)));
    float4 pf[kWavePf];
    if (on) wave_prefetch(pf, row, n, 4 * m, lane, al);
    for (int c = 0; c < s.nticks; ++c) {
        if (c < s.nch && tf) {
            const int wt = c * kPF + 4 * m;
            const int t = wt + gg;
            float2 xa[8], xb[8], x128;
            transform4(wr, scr, pf, cval, n, wt, lane, gg, lb, sHann, sTwT, sTw512, c + 1 < s.nch ? row : nullptr, n,
                       wt + kPF, al, xa, xb, x128);
            if (KIND != 0) {
                mags_to_scr(scr, lb, sw, xa, xb, x128);
                wave_fence();
                float* fo = ring_erb + (((KIND == 1 ? (c & 3) : (c & 7))) * kPF + 4 * m + gg) * 32;
                erb_project(scr, sSched, sComb, L, lb, sw, fo);
                if (feats && t < s.T) {
                    feats[(int64_t)t * 96 + foff + lb] = fo[lb];
                    feats[(int64_t)t * 96 + foff + lb + 16] = fo[lb + 16];
                }
            }
            if (KIND != 2) row_to_scr(scr, lb, xa, xb, x128);   // M / R row of frame t, for the NL waves
        }
        barrier_lds();
        const int c1 = c - 1;
        if (KIND == 0 && c1 >= 0 && c1 < s.nch && !(p.mode & 16)) {
            // mic_erb of chunk c-1 from its E rows (complete since B1)
            const int fi = 4 * m + gg;
            const int t = c1 * kPF + fi;
            float* er = sE + fi * kERowP;
            float2 xa[8], xb[8], x128;
            row_to_pairs(reinterpret_cast<const float2*>(er), lb, true, xa, xb, x128);
            wave_fence();
            mags_to_scr(er, lb, sw, xa, xb, x128);
            wave_fence();
            float* fo = ring_erb + ((c1 & 3) * kPF + fi) * 32;
            erb_project(er, sSched, sComb, L, lb, sw, fo);
            if (feats && t < s.T) {
                feats[(int64_t)t * 96 + lb] = fo[lb];
                feats[(int64_t)t * 96 + lb + 16] = fo[lb + 16];
            }
        }
        barrier_lds();
    }
}

template <int TAPS>
__global__ __launch_bounds__(kThreads, 1) void pipe_kernel(PipeArgs p) {
    const int tid = threadIdx.x, wave = tid >> 6;
    const int L = p.sched_len;
    PipeStream s;
    s.b = p.b0 + blockIdx.x;
    s.n = (int)p.lens[s.b];                             // mic: frames and output hops
    s.T = s.n / kHop + 1;
    s.nhop = s.n / kHop;
    s.nch = (s.T + kPF - 1) / kPF;
    s.nticks = s.nch + 5;
    s.have_near = p.nsig == 3;
    {
        const DevTables* tb = reinterpret_cast<const DevTables*>(p.tables);
        const float4* sch = reinterpret_cast<const float4*>(p.sched);
        float4* sSched = reinterpret_cast<float4*>(lds<kC.sched>());
        for (int i = tid; i < L * 16; i += kThreads) sSched[i] = sch[i];
        if (tid < 32)
            reinterpret_cast<int2*>(lds<kC.comb>())[tid] = reinterpret_cast<const int2*>(p.sched + 4 * 16 * L)[tid];
        if (tid < 257) reinterpret_cast<float4*>(lds<kC.bin>())[tid] = reinterpret_cast<const float4*>(p.bintab)[tid];
        if (tid < 258) reinterpret_cast<float2*>(lds<kC.tw512>())[tid] = tb->tw512[tid];
        if (tid < 256) {
            reinterpret_cast<float2*>(lds<kC.twT>())[tid] = tb->twT[tid];
            lds<kC.coff>()[tid] = tb->inv_coff[tid];
        }
        if (tid < 512) {
            lds<kC.hann>()[tid] = tb->hann[tid];
            lds<kC.ec>()[tid] = 0.f;
        }
        {
            const float* W2 = p.w + 96 * 64 + 96 * 32 + 96 + 96 + 32 * 64 + 32;
            for (int i = tid; i < 32 * 32; i += kThreads) lds<kC.w2t>()[(i & 31) * 32 + (i >> 5)] = W2[i];
        }
        if (tid < 3) lds<kC.c>()[tid] = tid < p.nsig ? norm_scalar(p.mom, s.b, tid, p.slen[4 * s.b + tid]) : 0.f;
    }
    __syncthreads();
#ifndef PIPE_ROLES
#define PIPE_ROLES 0xFF        // build experiments only: bit r compiles role r (GRU HD GI NL MIC REF NEAR SY)
#endif
    auto idle = [&]() { for (int c = 0; c < s.nticks; ++c) { barrier_lds(); barrier_lds(); } };
    if (wave == W_GRU) { if constexpr (PIPE_ROLES & 1) role_gru(p, s); else idle(); }
    else if (wave == W_HD) { if constexpr (PIPE_ROLES & 2) role_hd(p, s); else idle(); }
    else if (wave < W_NL0) { if constexpr (PIPE_ROLES & 4) role_gi(p, s); else idle(); }
    else if (wave < W_MIC0) { if constexpr (PIPE_ROLES & 8) role_nl<TAPS>(p, s); else idle(); }
    else if (wave < W_REF0) { if constexpr (PIPE_ROLES & 16) role_tf<0>(p, s); else idle(); }
    else if (wave < W_NEAR0) { if constexpr (PIPE_ROLES & 32) role_tf<1>(p, s); else idle(); }
    else if (wave < W_SY0) { if constexpr (PIPE_ROLES & 64) role_tf<2>(p, s); else idle(); }
    else { if constexpr (PIPE_ROLES & 128) role_sy(p, s); else idle(); }
}

template <int TAPS>
static hipError_t launch_pipe_t(const PipeArgs& a, int nb, hipStream_t st) {
    static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(pipe_kernel<TAPS>),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (attr != hipSuccess) return attr;
    hipLaunchKernelGGL(pipe_kernel<TAPS>, dim3(nb), dim3(kThreads), pipe_smem_bytes(a.sched_len), st, a);
    return hipGetLastError();
}

hipError_t launch_pipe(const PipeArgs& a, int nb, hipStream_t st) {
    if (nb <= 0) return hipSuccess;
    if (pipe_smem_bytes(a.sched_len) > 160 * 1024) return hipErrorInvalidValue;
    switch (a.taps) {
        case 0: return launch_pipe_t<0>(a, nb, st);
        case 1: return launch_pipe_t<1>(a, nb, st);
        case 2: return launch_pipe_t<2>(a, nb, st);
        case 3: return launch_pipe_t<3>(a, nb, st);
        case 4: return launch_pipe_t<4>(a, nb, st);
        case 5: return launch_pipe_t<5>(a, nb, st);
        case 6: return launch_pipe_t<6>(a, nb, st);
        case 7: return launch_pipe_t<7>(a, nb, st);
        case 8: return launch_pipe_t<8>(a, nb, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace aec
