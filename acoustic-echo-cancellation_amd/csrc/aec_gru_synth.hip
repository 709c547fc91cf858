// aec_gru_synth.hip — K3+K4 fused: the post-filter recurrence and the
// synthesis of the same stream in one block (gfx950).
//
// Reference: nn.GRU + linear1/relu + linear2/sigmoid + mask + loss
// (Stage2_lhm/scripts/network/ERB.py:213-217, 287-323), then the ERB gains,
// conv-iSTFT and WOLA (ERB.py:304-316, attention_ccrn.py:82-101).
//
// The GRU is one dependent step per frame (latency-bound: ~680 cycles a
// step on one wave), so gru_kernel leaves its CU mostly idle while the
// separate synthesis kernel then streams the error spectrum back in.  Here
// the synthesis waves of the stream run inside the GRU's own tick pipeline,
// two chunks behind the recurrence, and a block carries NS = 2 streams (one
// recurrence wave each, on different SIMDs; 8 frames of each per tick):
//
//   waves 0..NS-1  recurrence of stream s, chunk c          (gru_kernel's code)
//   3 gi waves     stage feats of chunk c+2, load chunk c+3, gi = W_ih x + b of chunk c+1
//   3 head waves   head / mask / est_erb / loss of chunk c-1 -> est (HBM + LDS ring);
//                  OLA + WOLA of chunk c-3 from the frame ring -> out
//   4 synth waves  synthesis (gains, irFFT, window) of chunk c-2 into the LDS
//                  frame ring (NS = 2: the window is applied in the overlap-add);
//                  E rows of chunk c-1 into registers
//
// one block barrier per tick of 16 frame slots.  The arithmetic of every
// output sample is the unfused path's (synth_frame, the same OLA expression),
// so the result is bit-identical to gru_kernel + synthesis_kernel
// (tests/test_gpu_nlms.py::test_fused_synthesis_bit_exact) for any NS.
#ifndef AEC_OUT_NT
#define AEC_OUT_NT 1   // waveform stores nt: written once, never re-read on the device (fused kernel -1 %)
#endif
#ifndef AEC_OLA_REC
#define AEC_OLA_REC 1   // NS = 2: overlap-add on the recurrence waves (0: on the head waves, A/B builds)
#endif
#ifndef AEC_OLA_WIN
// NS = 2: the synthesis window applied in the recurrence waves' overlap-add instead of the synthesis
// waves (bit-identical; gru_synth 0.360-0.366 against 0.387 ms, profiles/r05_notes.md r05z2)
#define AEC_OLA_WIN 1
#endif
#ifndef AEC_SYN_HANN_PRE
#define AEC_SYN_HANN_PRE 0   // synthesis window table pre-scaled by 1/512 (bit-identical; A/B)
#endif
// Recurrence loop form: h stored by both K halves (the same value) instead of lanes kh == 0 only,
// and full chunks as an unrolled TF-step sequence.  Bit-identical; batch 1 0.2635 -> 0.2585 ms,
// 64 streams 0.349 -> 0.342 ms, the C2 step unchanged (profiles/r06l_rec_ab.log).
#ifndef AEC_REC_ALLST
#define AEC_REC_ALLST 1
#endif
#ifndef AEC_REC_FULL
#define AEC_REC_FULL 1
#endif
#ifndef AEC_SPEC_LD_NT
#define AEC_SPEC_LD_NT 0   // E-spectrum row loads nt (A/B builds only)
#endif
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "aec_fft.h"
#include "aec_frame.h"
#include "aec_launch.h"
#include "aec_tables.h"

namespace aec {

namespace {
constexpr int kGiWaves = 3, kHeadWaves = 3, kSynWaves = 4;
constexpr int kHelperWaves = kGiWaves + kHeadWaves + kSynWaves;      // 10
constexpr int kGiLanes = 64 * kGiWaves;                               // 192
constexpr int kHeadLanes = 64 * kHeadWaves;                           // 192
constexpr int kHeadGrp = kHeadLanes / 32;                             // 6 groups of 32 lanes
constexpr int kEstS = 33;                                             // est ring row stride
constexpr int kMaxNS = 2;                                             // streams per block

// LDS carve (floats).  A tick holds kCH = 16 frame slots: NS streams x kCH / NS frames
// (slot q = stream q / TF, frame q % TF of the stream's chunk)
constexpr int oX = 0;                                   // [2][16][64]
constexpr int oGi = oX + 2 * kCH * 64;                  // [2][16][96]
constexpr int oH = oGi + 2 * kCH * 96;                  // [2][16][32]
constexpr int oMic = oH + 2 * kCH * 32;                 // [4][16][32]
constexpr int oNear = oMic + 4 * kCH * 32;              // [4][16][32]
constexpr int oO = oNear + 4 * kCH * 32;                // [6][32]
constexpr int oLoss = oO + kHeadGrp * 32;               // [kHeadWaves][NS]
constexpr int oHb = oLoss + 8;                          // [NS][32]
constexpr int oEst = oHb + 32 * kMaxNS;                 // [2][16][33] (+2 pad)
constexpr int oBin = (oEst + 2 * kCH * kEstS + 2 + 3) & ~3;   // float4[257] (+3)
constexpr int oTw512 = oBin + 260 * 4;                  // float2[258]
constexpr int oTwT = oTw512 + 258 * 2;                  // float2[256]
constexpr int oHann = oTwT + 256 * 2;                   // [512]
constexpr int oCoff = oHann + 512;                      // [256]
constexpr int oTail = oCoff + 256;                      // [2][NS][256]
constexpr int oOut = oTail + 2 * kMaxNS * 256;          // [2][4 waves][4 groups][576] frame ring
constexpr int kFusedFloats = oOut + 2 * kSynWaves * 4 * kGroupFloats;
static_assert(oOut % 4 == 0 && oBin % 4 == 0, "16-B alignment");
static_assert(kHeadWaves * kMaxNS <= 8, "loss slots");
}  // namespace

size_t gru_synth_smem_bytes() { return (size_t)kFusedFloats * 4; }

#ifdef AEC_TICK_PROF
// timing experiments only (tools/gru_tick_prof.py): s_memtime stamps of (consumer) blocks 0 and 64 per wave and
// tick: loop top, work done (before the tick barrier)
__device__ unsigned long long g_gtick[2][12][96][2];
#define GTICK(slot)                                                                                    \
    do {                                                                                               \
        if ((blk == 0 || blk == 64) && lane == 0 && c + 3 < 96)                                        \
            g_gtick[blk ? 1 : 0][wave][c + 3][slot] = __builtin_amdgcn_s_memtime();                     \
    } while (0)
#else
#define GTICK(slot) do {} while (0)
#endif

// The tick barrier: LDS traffic drained (lgkmcnt(0)), global loads and
// stores left in flight.  __syncthreads would also drain vmcnt, exposing the
// HBM latency of the loads issued for the NEXT tick (feats, E rows) once per
// tick; the compiler waits for those registers where they are used.  The
// empty asm keeps the compiler from moving memory accesses across it.
__device__ __forceinline__ void tick_barrier() {
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xC07F);        // gfx9: vmcnt 63, expcnt 7, lgkmcnt 0
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

// role of hardware wave k = nibble k (0: identity).  NS = 1: SIMD0 rec gi0 gi1 | gi2 head0 syn0 |
// head1 syn1 syn2 | head2 syn3 (role waves: 0 recurrence, 1-3 gi, 4-6 head, 7-10 synthesis)
template <int NS>
constexpr unsigned long long kRoleMap = NS == 1 ? 0x972A8416530ull : 0ull;

// Device-coherent (sc1) 4- and 8-byte accesses for the data the small-batch pipeline hands from a
// producer block to a consumer block of the same launch (other CUs, other XCDs): relaxed agent-scope
// atomics, which the compiler emits as sc1 loads / stores past the non-coherent caches.
__device__ __forceinline__ float ld_coherent(const float* a) {
    return __uint_as_float(__hip_atomic_load(reinterpret_cast<unsigned*>(const_cast<float*>(a)), __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ float2 ld_coherent2(const float2* a) {
    const unsigned long long v = __hip_atomic_load(reinterpret_cast<unsigned long long*>(const_cast<float2*>(a)),
                                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return make_float2(__uint_as_float((unsigned)v), __uint_as_float((unsigned)(v >> 32)));
}
__device__ __forceinline__ void st_coherent(float* a, float v) {
    __hip_atomic_store(reinterpret_cast<unsigned*>(a), __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_coherent2(float2* a, float2 v) {
    const unsigned long long u = (unsigned long long)__float_as_uint(v.x) | ((unsigned long long)__float_as_uint(v.y) << 32);
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(a), u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Producer block of the small-batch pipeline (gru_synth_kernel<1, true>, blocks 0 .. nb-1): stream
// b's FD-NLMS recursion and mic_erb, one 16-frame chunk per tick, ahead of the consumer block
// (nb + b) that runs the GRU and the synthesis of the same stream.  The arithmetic is the split
// path's own: nlms_recursion_kernel's NlmsBin steps (waves 0-3, one lane per bin slot, rows
// prefetched 8 frames ahead) into an LDS ring, then mic_erb_kernel's pass over those rows (waves
// 4-7, 4 frames each, one chunk behind), so E, the features and the waveform are bit-identical to
// the three-launch split path (tests/test_gpu_nlms.py::test_small_batch_pipeline_bit_exact).  The E
// rows and mic_erb leave through sc1 stores; every storing wave drains (vmcnt(0)) before the tick
// barrier, after which one lane publishes (epoch << 32) | chunks done.
template <int TAPS>
__device__ __forceinline__ void pipe_producer(const GruArgs& p, const PipeArgs& q, int b, float* smem) {
    constexpr int kERowF = 512 + 48;                   // magnitudes (swizzled) + 48 ERB partials
    constexpr int oPSched = 0;                         // float4[48][16]
    constexpr int oPComb = oPSched + 48 * 16 * 4;      // int2[32]
    constexpr int oPE = oPComb + 64;                   // float2[2][16][256] E ring
    constexpr int oPScr = oPE + 2 * kCH * 256 * 2;     // [16][kERowF]
    static_assert(oPScr + kCH * kERowF <= kFusedFloats, "producer LDS");
    float4* sSched = reinterpret_cast<float4*>(smem + oPSched);
    int2* sComb = reinterpret_cast<int2*>(smem + oPComb);
    float2* sE = reinterpret_cast<float2*>(smem + oPE);
    float* sScr = smem + oPScr;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int L = q.sched_len;
    for (int i = tid; i < L * 16; i += blockDim.x) sSched[i] = reinterpret_cast<const float4*>(q.sched)[i];
    if (tid < 32) sComb[tid] = reinterpret_cast<const int2*>(q.sched + 4 * 16 * L)[tid];
    __syncthreads();
    const int64_t T = p.lens[b] / kHop + 1;
    const int nch = (int)((T + kCH - 1) / kCH);
    const unsigned long long ep = q.epoch << 32;
    if (wave < 4) {
        const int k = tid;
        const float2* r0 = q.rows + (int64_t)b * p.Tmax * 512;
        NlmsBin<TAPS> st;
        st.reset(k == 0);
        float2 dd[8], rr[8];
        auto fetch = [&](int64_t t, int i) {               // rows past the end: any valid row (results unused)
            const int64_t tc = t < T ? t : T - 1;
            dd[i] = r0[tc * 512 + k];
            rr[i] = r0[tc * 512 + 256 + k];
        };
#pragma unroll
        for (int i = 0; i < 8; ++i) fetch(i, i);
        for (int c = 0; c <= nch; ++c) {
            if (c < nch) {
                float2* er = sE + (c & 1) * (kCH * 256) + k;
#pragma unroll
                for (int hh = 0; hh < 2; ++hh)
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        const float2 e = st.step(dd[i], rr[i], q.mu, q.beta, q.delta);
                        er[(8 * hh + i) * 256] = e;
                        fetch((int64_t)c * kCH + 8 * hh + i + 8, i);
                    }
            }
            tick_barrier();
            if (tid == 0 && c >= 1 && !q.stall)
                __hip_atomic_store(q.progress + b, ep | (unsigned long long)c, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
    } else if (wave < 8) {
        const int w4 = wave - 4;
        const int gg = lane >> 4, lb = lane & 15, sw = 16 * (gg & 1);
        const int fs = 4 * w4 + gg;                        // the group's frame slot of the chunk
        float* er = sScr + fs * kERowF;
        float2 xa[8], xb[8], x128;
        for (int c = 0; c <= nch; ++c) {
            if (c >= 1) {
                const int cp = c - 1;
                const float2* rowc = sE + (cp & 1) * (kCH * 256);
                const int64_t t = (int64_t)cp * kCH + fs;
                row_to_pairs(rowc + fs * 256, lb, true, xa, xb, x128);
                mags_to_scr(er, lb, sw, xa, xb, x128);
                wave_fence();
                erb_project(er, sSched, sComb, L, lb, sw, nullptr);
                if (t < T) {                               // erb_project's feature-row expression
                    const float* part = er + 512;
                    float* fo = q.feats + ((int64_t)b * p.Tmax + t) * 96;
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        const int band = lb + 16 * h;
                        const int2 cb = sComb[band];
                        st_coherent(fo + band, part[cb.x] + (cb.y >= 0 ? part[cb.y] : 0.f));
                    }
                }
#pragma unroll
                for (int j = 0; j < 16; ++j) {             // the wave's 4 E rows -> spec
                    const int idx = lane + 64 * j, fr = 4 * w4 + (idx >> 8), slot = idx & 255;
                    const int64_t tt = (int64_t)cp * kCH + fr;
                    if (tt < T) st_coherent2(q.spec + ((int64_t)b * p.Tmax + tt) * 256 + slot, rowc[fr * 256 + slot]);
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            tick_barrier();
        }
    } else {
        for (int c = 0; c <= nch; ++c) tick_barrier();
    }
}

// NS streams per block (one recurrence wave each, waves 0 .. NS-1), TF = 16 / NS frames of
// every stream per tick, so the helper roles see 16 frame slots per tick whatever NS is.
// With NS = 2 the block holds two independent recurrence chains on two SIMDs (the chain of
// one stream leaves its CU mostly idle) and half the blocks occupy half the CUs for about
// the same time: the CUs the other half frees run the next batch's analysis kernel.
// PIPE (NS = 1): blocks 0 .. nb-1 are the streams' producers (pipe_producer), block nb + i consumes
// stream i: its gi waves wait for a chunk's mic_erb and its synthesis waves for its E rows (polls
// of the producer's counter, sc1 loads of the rows).  Producers come first in the grid, so every
// consumer's producer was dispatched before it (no wait on a block that cannot start).
template <int NS, bool PIPE = false>
__global__ __launch_bounds__(64 * (NS + kHelperWaves), 1) void gru_synth_kernel(GruArgs p, SynthArgs y, int nb,
                                                                                 PipeArgs q) {
    static_assert(!PIPE || NS == 1, "the pipeline runs one stream per consumer block");
    constexpr int TF = kCH / NS;
    constexpr int kThreads = 64 * (NS + kHelperWaves);
    extern __shared__ __attribute__((aligned(16))) float smem[];
    float* sX = smem + oX;
    float* sGi = smem + oGi;
    float* sH = smem + oH;
    float* sMic = smem + oMic;
    float* sNear = smem + oNear;
    float* sO = smem + oO;
    float* sLoss = smem + oLoss;
    float* sHb = smem + oHb;
    float* sEst = smem + oEst;
    float4* sBin = reinterpret_cast<float4*>(smem + oBin);
    float2* sTw512 = reinterpret_cast<float2*>(smem + oTw512);
    float2* sTwT = reinterpret_cast<float2*>(smem + oTwT);
    float* sHann = smem + oHann;
    float* sCoff = smem + oCoff;
    float* sTail = smem + oTail;
    float* sOut = smem + oOut;
    if constexpr (PIPE) {
        if ((int)blockIdx.x < nb) {
            pipe_producer<kPipeTaps>(p, q, p.b0 + (int)blockIdx.x, smem);
            return;
        }
    }
    const int blk = PIPE ? (int)blockIdx.x - nb : (int)blockIdx.x;

    // the block's streams (an odd last block: stream 1 absent, its addresses those of stream 0)
    int bs[NS], Ts[NS], nchs[NS];
    int64_t nhops[NS];
    bool vs[NS];
    int nchmax = 0;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
        const int i = NS * blk + s;
        vs[s] = i < nb;
        bs[s] = p.b0 + (vs[s] ? i : NS * blk);
        const int64_t n = p.lens[bs[s]];
        Ts[s] = vs[s] ? (int)(n / kHop + 1) : 0;
        nhops[s] = vs[s] ? n / kHop : 0;                  // output hops (T - 1)
        nchs[s] = (Ts[s] + TF - 1) / TF;
        nchmax = max(nchmax, nchs[s]);
    }
    // Role placement: hardware wave i (SIMD i % 4) runs role wave (wmap >> 4 i) & 15; every index
    // below uses the role ids.  NS = 2 keeps the identity; NS = 1 (11 waves, SIMD 3 holds two) puts
    // the two lightest roles (gi waves) beside the recurrence wave, whose priority slows whatever
    // shares its SIMD: tick 11.0 k -> 9.6 k cycles, batch 1 0.257 -> 0.233 ms (r06o_wmap1_ab.log).
    // A/B builds: y.wmap (AEC_GRU_WMAP) overrides it.
#if AEC_AB_BUILD
    const unsigned long long wmap = y.wmap ? y.wmap : kRoleMap<NS>;
#else
    constexpr unsigned long long wmap = kRoleMap<NS>;
#endif
    const int lane = threadIdx.x & 63;
    const int wave = wmap ? (int)((wmap >> (4 * (threadIdx.x >> 6))) & 15) : (int)(threadIdx.x >> 6);
    const int tid = wave * 64 + lane;
    const float* W_ih = p.w;                  // [96][64]
    const float* W_hh = p.w + 96 * 64;        // [96][32]
    const float* b_ih = W_hh + 96 * 32;       // [96]
    const float* b_hh = b_ih + 96;            // [96]
    const float* W1 = b_hh + 96;              // [32][64]
    const float* b1 = W1 + 32 * 64;           // [32]
    const float* W2 = b1 + 32;                // [32][32]
    const float* b2 = W2 + 32 * 32;           // [32]
    // PIPE: wait until the producer has published chunks [0, need) of the block's stream (lane 0
    // polls; bounded: past q.spin_limit polls the wave sets the error word and stops waiting)
    bool stalled = false;
    auto wait_chunks = [&](int need) {
        if constexpr (PIPE) {
            if (stalled) return;
            const unsigned long long target = (q.epoch << 32) | (unsigned long long)need;
            int bad = 0;
            if (lane == 0) {
                int n = 0;
                while (__hip_atomic_load(q.progress + bs[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
                    __builtin_amdgcn_s_sleep(1);
                    if (++n > q.spin_limit) {
                        __hip_atomic_store(q.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                        bad = 1;
                        break;
                    }
                }
            }
            stalled = __builtin_amdgcn_readfirstlane(bad) != 0;
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");    // no load above the poll
        }
    };

    // synthesis tables (read after the first tick barrier)
    {
        const DevTables* tb = reinterpret_cast<const DevTables*>(y.tables);
        const float4* bt = reinterpret_cast<const float4*>(y.bintab);
        for (int i = tid; i < 257; i += kThreads) sBin[i] = bt[i];
        for (int i = tid; i < 258; i += kThreads) sTw512[i] = tb->tw512[i];
        for (int i = tid; i < 256; i += kThreads) {
            sTwT[i] = tb->twT[i];
            sCoff[i] = tb->inv_coff[i];
        }
        for (int i = tid; i < 2 * NS * 256; i += kThreads) sTail[i] = 0.f;
        for (int i = tid; i < 512; i += kThreads) sHann[i] = AEC_SYN_HANN_PRE ? tb->hann[i] * (1.f / 512.f) : tb->hann[i];
    }

    {
        // role priorities (AEC_FUSED_MODE bits 3-4 synthesis, 5-6 head, 7-8 gi; timing experiments;
        // bits 9 / 10 / 11 skip the recurrence / head / gi, tools/modes_r03.sh)
        const int hw = wave - NS;
        const int role_prio = hw < 0 ? 0 : (hw < kGiWaves ? (y.fmode >> 7) & 3
                              : (hw < kGiWaves + kHeadWaves ? (y.fmode >> 5) & 3 : (y.fmode >> 3) & 3));
        switch (role_prio) {
            case 1: __builtin_amdgcn_s_setprio(1); break;
            case 2: __builtin_amdgcn_s_setprio(2); break;
            case 3: __builtin_amdgcn_s_setprio(3); break;
            default: break;
        }
    }
    // NS = 2: the overlap-add of chunk c-3 runs on the recurrence waves (each its own stream, after
    // the tick's steps; the host takes NS = 1 for an output that is not 16-B aligned) instead of the
    // head waves: the same expressions.  Without the head's overlap-add code the kernel fits 160
    // VGPRs, so a 32-VGPR moments wave (the look-ahead pass of another batch) fits beside it.
    constexpr bool ola_rec = NS == 2 && AEC_OLA_REC;
    if (wave < NS) {
        // ---------------- recurrence wave of stream `wave` (gru_kernel wave 0) ----------------
        __builtin_amdgcn_s_setprio(3);
        const int s = wave;
        const int T = Ts[s], nch = nchs[s];
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
        float* hb = sHb + 32 * s;
        if (lane < 32) hb[lane] = 0.f;
        for (int c = -3; c <= nchmax + 2; ++c) {
            GTICK(0);
            if (c >= 0 && c < nch && !(y.fmode & 512)) {
                const int f_end = min(TF, T - c * TF);
                const float* gi = sGi + ((c & 1) * kCH + s * TF) * 96;
                float* hrow = sH + ((c & 1) * kCH + s * TF) * 32;
                float gr = gi[j], gz = gi[32 + j], gn = gi[64 + j];
                auto step = [&](int f, int fn) {
                    const float ngr = gi[fn * 96 + j], ngz = gi[fn * 96 + 32 + j], ngn = gi[fn * 96 + 64 + j];
                    hj = gru_step(wrz, wn, hb, kh, gr, gz, gn, bhn, hj);
                    // both K halves hold the same h_j (a + b == b + a): every lane stores, no exec-mask branch
                    if (AEC_REC_ALLST || kh == 0) {
                        hb[j] = hj;
                        hrow[f * 32 + j] = hj;
                    }
                    gr = ngr; gz = ngz; gn = ngn;
                };
                if (AEC_REC_FULL && f_end == TF) {
#pragma unroll
                    for (int f = 0; f < TF; ++f) step(f, f + 1 < TF ? f + 1 : f);
                } else {
                    for (int f = 0; f < f_end; ++f) step(f, f + 1 < f_end ? f + 1 : f);
                }
            }
            const int k = c - 3;
            if (ola_rec && k >= 0 && k < nch && !(y.fmode & 2)) {
                // lane: float4 column r = 4 lane of the chunk's TF hops; frame halves from the ring
                // (all loads first), hop j0 + i = frame i-1 (2nd half) + frame i (1st half)
                const float* ring = sOut + (k & 1) * (kSynWaves * 4 * kGroupFloats) + s * TF * kGroupFloats;
                const float* tail_in = sTail + ((k & 1) * NS + s) * 256;
                const int64_t j0 = (int64_t)k * TF - 1;
                const int nh = (int)min((int64_t)TF, nhops[s] - j0);
                const int r = 4 * lane;
                float4 fh[NS == 2 ? TF : 1], sh[NS == 2 ? TF : 1];
                const float4 tl = *reinterpret_cast<const float4*>(tail_in + r);
                const float4 cf = *reinterpret_cast<const float4*>(sCoff + r);
                // AEC_OLA_WIN: the ring holds the raw irFFT output; window x 1/512 here (hann / 512
                // is exact).  The products go through inline asm: HIP contracts across statements
                // (-ffp-contract=fast), and a product fused into the following add would round
                // differently from synth_fft's stored product
                float4 w1 = make_float4(1.f, 1.f, 1.f, 1.f), w2 = w1;
                if constexpr (AEC_OLA_WIN) {
                    const float4 h1 = *reinterpret_cast<const float4*>(sHann + r);
                    const float4 h2 = *reinterpret_cast<const float4*>(sHann + 256 + r);
                    w1 = make_float4(h1.x * (1.f / 512.f), h1.y * (1.f / 512.f), h1.z * (1.f / 512.f), h1.w * (1.f / 512.f));
                    w2 = make_float4(h2.x * (1.f / 512.f), h2.y * (1.f / 512.f), h2.z * (1.f / 512.f), h2.w * (1.f / 512.f));
                }
                auto mulr = [](float x, float y) {
                    float r;
                    asm("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y));
                    return r;
                };
#pragma unroll
                for (int i = 0; i < TF; ++i) {
                    fh[i] = *reinterpret_cast<const float4*>(ring + i * kGroupFloats + r);
                    sh[i] = *reinterpret_cast<const float4*>(ring + i * kGroupFloats + 256 + r);
                }
                float* orow = y.out + (int64_t)bs[s] * y.ld_out;
#pragma unroll
                for (int i = 0; i < TF; ++i) {
                    if (i >= nh || j0 + i < 0) continue;
                    float4 a = i == 0 ? tl : sh[i - 1], b = fh[i];
                    if constexpr (AEC_OLA_WIN) {
                        a = make_float4(mulr(a.x, w2.x), mulr(a.y, w2.y), mulr(a.z, w2.z), mulr(a.w, w2.w));
                        b = make_float4(mulr(b.x, w1.x), mulr(b.y, w1.y), mulr(b.z, w1.z), mulr(b.w, w1.w));
                    }
                    float4 o;
                    o.x = (a.x + b.x) * cf.x + 1e-9f;
                    o.y = (a.y + b.y) * cf.y + 1e-9f;
                    o.z = (a.z + b.z) * cf.z + 1e-9f;
                    o.w = (a.w + b.w) * cf.w + 1e-9f;
#if AEC_OUT_NT
                    typedef float f4v __attribute__((ext_vector_type(4)));
                    __builtin_nontemporal_store(f4v{o.x, o.y, o.z, o.w}, reinterpret_cast<f4v*>(orow + (j0 + i) * kHop + r));
#else
                    *reinterpret_cast<float4*>(orow + (j0 + i) * kHop + r) = o;
#endif
                }
                *reinterpret_cast<float4*>(sTail + (((k + 1) & 1) * NS + s) * 256 + r) = sh[TF - 1];
            }
            GTICK(1);
            tick_barrier();
        }
    } else if (wave < NS + kGiWaves) {
        // ---------------- feats staging + input projection ----------------
        const int hl = tid - 64 * NS;                         // 0..191
        const int grow = hl % 96, fq = hl / 96;               // slots fq, fq + 2, ...
        float wih[64];
#pragma unroll
        for (int k = 0; k < 64; ++k) wih[k] = W_ih[grow * 64 + k];
        const float gbias = b_ih[grow] + (grow < 64 ? b_hh[grow] : 0.f);
        constexpr int kStU = (kCH * 32 + kGiLanes - 1) / kGiLanes;    // 3 elements per lane
        float pm[kStU], pr[kStU], pn[kStU];
        auto load_chunk = [&](int cc) {
#pragma unroll
            for (int u = 0; u < kStU; ++u) {
                const int e = hl + u * kGiLanes;
                const int q = e >> 5, s = q / TF;
                const int t = cc * TF + q % TF;
                int Tq = 0, bq = bs[0];
#pragma unroll
                for (int z = 0; z < NS; ++z)
                    if (s == z) Tq = Ts[z], bq = bs[z];
                const bool ok = e < kCH * 32 && t < Tq;
                const float* f = p.feats + ((int64_t)bq * p.Tmax + t) * 96 + (e & 31);
                if constexpr (PIPE) pm[u] = ok ? ld_coherent(f) : 0.f;       // mic_erb from the producer
                else pm[u] = ok ? f[0] : 0.f;
                pr[u] = ok ? f[32] : 0.f;
                pn[u] = ok && p.has_near ? f[64] : 0.f;
            }
        };
#pragma unroll
        for (int u = 0; u < kStU; ++u) pm[u] = pr[u] = pn[u] = 0.f;
        for (int c = -3; c <= nchmax + 2; ++c) {
            GTICK(0);
            const int cs = c + 2;
            if (cs >= 0 && cs < nchmax) {
#pragma unroll
                for (int u = 0; u < kStU; ++u) {
                    const int e = hl + u * kGiLanes;
                    if (e < kCH * 32) {
                        const int q = e >> 5, jj = e & 31;
                        sX[((cs & 1) * kCH + q) * 64 + jj] = pm[u];
                        sX[((cs & 1) * kCH + q) * 64 + 32 + jj] = fabsf(pm[u] - pr[u]);
                        sMic[((cs & 3) * kCH + q) * 32 + jj] = pm[u];
                        sNear[((cs & 3) * kCH + q) * 32 + jj] = pn[u];
                    }
                }
            }
            if (c + 3 < nchmax) {
                wait_chunks(c + 4);
                load_chunk(c + 3);
            }
            const int cg = c + 1;
            if (cg >= 0 && cg < nchmax && !(y.fmode & 2048)) {
#pragma unroll 2
                for (int i = 0; i < kCH / 2; ++i) {
                    const int q = fq + 2 * i;
                    sGi[((cg & 1) * kCH + q) * 96 + grow] = gru_gi(wih, sX + ((cg & 1) * kCH + q) * 64, gbias);
                }
            }
            GTICK(1);
            tick_barrier();
        }
    } else if (wave < NS + kGiWaves + kHeadWaves) {
        // ---------------- head / mask / est_erb / loss ----------------
        const int hh = tid - 64 * (NS + kGiWaves);            // 0..191
        const int hj_ = hh & 31, fg = hh >> 5;                // slots fg, fg + 6, fg + 12
        float w1[64], w2[32];
#pragma unroll
        for (int k = 0; k < 64; ++k) w1[k] = W1[hj_ * 64 + k];
#pragma unroll
        for (int k = 0; k < 32; ++k) w2[k] = W2[hj_ * 32 + k];
        const float b1j = b1[hj_], b2j = b2[hj_];
        float lacc[NS];
#pragma unroll
        for (int s = 0; s < NS; ++s) lacc[s] = 0.f;
        const bool oal = ((y.ld_out & 3) == 0) && ((reinterpret_cast<uintptr_t>(y.out) & 15) == 0);
        for (int c = -3; c <= nchmax + 2; ++c) {
            GTICK(0);
            const int ch = c - 1;
            if (ch >= 0 && ch < nchmax && !(y.fmode & 1024)) {
                for (int q = fg; q < kCH; q += kHeadGrp) {
                    const int s = q / TF, t = ch * TF + q % TF;
                    int Tq = 0, bq = bs[0];
#pragma unroll
                    for (int z = 0; z < NS; ++z)
                        if (s == z) Tq = Ts[z], bq = bs[z];
                    float est = 0.f;
                    if (t < Tq) {                             // uniform within the 32-lane group
                        const float mask = head_mask(w1, w2, b1j, b2j, sH + ((ch & 1) * kCH + q) * 32,
                                                     sMic + ((ch & 3) * kCH + q) * 32, sO + fg * 32, hj_);
                        const float me = sMic[((ch & 3) * kCH + q) * 32 + hj_];
                        est = mask * me;
                        const int64_t o_idx = ((int64_t)bq * p.Tmax + t) * 32 + hj_;
                        p.est[o_idx] = est;
                        if (p.dbg_h) p.dbg_h[o_idx] = sH[((ch & 1) * kCH + q) * 32 + hj_];
                        if (p.dbg_mask) p.dbg_mask[o_idx] = mask;
                        if (p.has_near) {
                            const float d = sqrtf(sNear[((ch & 3) * kCH + q) * 32 + hj_]) - sqrtf(est);
#pragma unroll
                            for (int z = 0; z < NS; ++z)
                                if (s == z) lacc[z] += d * d;
                        }
                    }
                    sEst[((ch & 1) * kCH + q) * kEstS + hj_] = est;   // frames past the end: gain 0
                }
            }
            // OLA + WOLA of chunk k = c - 3 of every stream (its TF frames in ring k & 1, slots
            // s TF ..): hops TF k - 1 .. TF k + TF - 2; hop TF k - 1 uses the tail of frame TF k - 1
            const int k = c - 3;
            if (!ola_rec && k >= 0 && k < nchmax && !(y.fmode & 2)) {
#pragma unroll
                for (int s = 0; s < NS; ++s) {
                    if (k >= nchs[s]) continue;
                    const float* ring = sOut + (k & 1) * (kSynWaves * 4 * kGroupFloats) + s * TF * kGroupFloats;
                    const float* tail_in = sTail + ((k & 1) * NS + s) * 256;
                    const int64_t j0 = (int64_t)k * TF - 1;
                    const int nh = (int)min((int64_t)TF, nhops[s] - j0);    // hops j0 .. j0 + nh - 1 below nhop
                    float* orow = y.out + (int64_t)bs[s] * y.ld_out;
                    if (oal) {
                        for (int e = hh; e < TF * (kHop / 4); e += kHeadLanes) {
                            const int i = e >> 6, r = (e & 63) * 4;     // hop j0 + i = frame i-1 (2nd half) + frame i
                            if (i >= nh || j0 + i < 0) continue;
                            const float4 a = i == 0 ? *reinterpret_cast<const float4*>(tail_in + r)
                                                    : *reinterpret_cast<const float4*>(ring + (i - 1) * kGroupFloats + 256 + r);
                            const float4 cv = *reinterpret_cast<const float4*>(ring + i * kGroupFloats + r);
                            const float4 cf = *reinterpret_cast<const float4*>(sCoff + r);
                            float4 o;
                            o.x = (a.x + cv.x) * cf.x + 1e-9f;
                            o.y = (a.y + cv.y) * cf.y + 1e-9f;
                            o.z = (a.z + cv.z) * cf.z + 1e-9f;
                            o.w = (a.w + cv.w) * cf.w + 1e-9f;
#if AEC_OUT_NT
                            typedef float f4v __attribute__((ext_vector_type(4)));
                            __builtin_nontemporal_store(f4v{o.x, o.y, o.z, o.w},
                                                        reinterpret_cast<f4v*>(orow + (j0 + i) * kHop + r));
#else
                            *reinterpret_cast<float4*>(orow + (j0 + i) * kHop + r) = o;
#endif
                        }
                    } else {
                        for (int e = hh; e < TF * kHop; e += kHeadLanes) {
                            const int i = e >> 8, r = e & 255;
                            if (i >= nh || j0 + i < 0) continue;
                            const float a = i == 0 ? tail_in[r] : ring[(i - 1) * kGroupFloats + 256 + r];
                            const float cv = ring[i * kGroupFloats + r];
                            orow[(j0 + i) * kHop + r] = (a + cv) * sCoff[r] + 1e-9f;
                        }
                    }
                    for (int r = hh; r < 256; r += kHeadLanes)
                        sTail[(((k + 1) & 1) * NS + s) * 256 + r] = ring[(TF - 1) * kGroupFloats + 256 + r];
                }
            }
            GTICK(1);
            tick_barrier();
        }
        if (p.loss) {
#pragma unroll
            for (int s = 0; s < NS; ++s) {
                float l = lacc[s];
#pragma unroll
                for (int o = 32; o > 0; o >>= 1) l += __shfl_xor(l, o);
                if (lane == 0) sLoss[(wave - NS - kGiWaves) * NS + s] = l;
            }
        }
    } else {
        // ---------------- synthesis waves ----------------
        const int sw = wave - (NS + kGiWaves + kHeadWaves);   // 0..3
        const int gg = lane >> 4, lb = lane & 15;
        const int fl = 4 * sw + gg;                           // slot this group synthesises
        const int s = fl / TF, fs = fl % TF;
        int64_t nhop = 0;
        int bq = bs[0];
#pragma unroll
        for (int z = 0; z < NS; ++z)
            if (s == z) nhop = nhops[z], bq = bs[z];
        const int64_t sstride = y.spec_stride ? y.spec_stride : 256;
        const float2* spec = y.spec + (int64_t)bq * y.Tmax * sstride;
        float2 xa[8] = {}, xb[8] = {}, x128 = {};
        auto load_rows = [&](int cc) {
            // E rows of chunk cc.  A frame past the last one (t > nhop) feeds no
            // written hop (hop j reads frames j and j + 1 <= nhop), so it may
            // read any valid row: the index is clamped, the loads stay plain
            // global loads with no per-lane select.
            const int64_t t = min((int64_t)cc * TF + fs, nhop);
            const float2* row = spec + t * sstride;
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                const int kk = lb + 16 * m;
#if AEC_SPEC_LD_NT
                if constexpr (PIPE) {
                    const float2 a = ld_coherent2(row + kk), c2 = ld_coherent2(row + ((256 - kk) & 255));
                    xa[m] = kk == 0 ? make_float2(a.x, 0.f) : a;
                    xb[m] = kk == 0 ? make_float2(a.y, 0.f) : c2;
                    continue;
                }
                typedef float f2v __attribute__((ext_vector_type(2)));
                const f2v av = __builtin_nontemporal_load(reinterpret_cast<const f2v*>(row + kk));
                const f2v cv = __builtin_nontemporal_load(reinterpret_cast<const f2v*>(row + ((256 - kk) & 255)));
                const float2 a = make_float2(av.x, av.y), c2 = make_float2(cv.x, cv.y);
#else
                const float2 a = PIPE ? ld_coherent2(row + kk) : row[kk];
                const float2 c2 = PIPE ? ld_coherent2(row + ((256 - kk) & 255)) : row[(256 - kk) & 255];
#endif
                xa[m] = kk == 0 ? make_float2(a.x, 0.f) : a;
                xb[m] = kk == 0 ? make_float2(a.y, 0.f) : c2;
            }
            x128 = PIPE ? ld_coherent2(row + 128) : row[128];
        };
        for (int c = -3; c <= nchmax + 2; ++c) {
            GTICK(0);
            // (2) synthesis of chunk c - 2 into ring (c - 2) & 1 (rows loaded last tick); the
            // E rows of chunk c - 1 for the next tick are requested as soon as the inverse pack
            // has consumed this tick's rows, so their load runs under the inverse transform
            const int cs = c - 2;
            const bool next = c - 1 >= 0 && c - 1 < nchmax && !(y.fmode & 4);
            if (cs >= 0 && cs < nchmax && !(y.fmode & 1)) {
                float* scr = sOut + (cs & 1) * (kSynWaves * 4 * kGroupFloats) + fl * kGroupFloats;
                float2 v[16];
                synth_pack(xa, xb, x128, sEst + ((cs & 1) * kCH + fl) * kEstS, sBin, sTw512, lb, v);
                if (next) {
                    wait_chunks(c);
                    load_rows(c - 1);
                }
                if constexpr (ola_rec && AEC_OLA_WIN) synth_fft_raw(v, sTwT, scr, lb);
                else synth_fft<AEC_SYN_HANN_PRE>(v, sTwT, sHann, scr, lb);
            } else if (next) {
                wait_chunks(c);
                load_rows(c - 1);
            }
            GTICK(1);
            tick_barrier();
        }
    }
    if (p.loss) {
        __syncthreads();
        if (tid < NS) {
            float sum = 0.f;
            for (int w = 0; w < kHeadWaves; ++w) sum += sLoss[w * NS + tid];
            int Tq = 0, bq = 0;
            bool v = false;
#pragma unroll
            for (int z = 0; z < NS; ++z)
                if (tid == z) Tq = Ts[z], bq = bs[z], v = vs[z];
            if (v) p.loss[bq] = sum / (float)(Tq * 32);
        }
    }
}

#if AEC_AB_BUILD
// role placements for NS = 1 (role waves: 0 recurrence, 1-3 gi, 4-6 head, 7-10 synthesis; hardware
// wave i on SIMD i % 4, so SIMD 3 holds two waves), entry k = role of hardware wave k
static unsigned long long wmap_ns1(int wm) {
    static const unsigned long long kWmaps1[] = {
        0xA9876543210ull,       // 0 identity: SIMD0 rec head0 syn1 | gi0 head1 syn2 | gi1 head2 syn3 | gi2 syn0
        0x972A8416530ull,       // 1 (the product's kRoleMap<1>): rec gi0 gi1 | gi2 head0 syn0 | head1 syn1 syn2 | head2 syn3
        0x874A6519320ull,       // 2: rec gi0 head0 | gi1 head1 syn0 | gi2 head2 syn1 | syn2 syn3
        0x987A5416320ull,       // 3: rec gi0 syn0 | gi1 head0 syn1 | gi2 head1 syn2 | head2 syn3
        0xA8269715430ull,       // 4: rec gi0 gi1 | gi2 syn0 syn1 | head0 syn2 syn3 | head1 head2
    };
    return wm >= 0 && wm < (int)(sizeof(kWmaps1) / sizeof(kWmaps1[0])) ? kWmaps1[wm] : 0;
}
#endif

// Streams per block.  NS = 1 finishes a batch sooner (a stream's recurrence takes 16 frames per
// tick, against 8 with NS = 2: 0.26 against 0.39 ms for 256 streams alone); NS = 2 takes half the
// CUs for about as long, and with batches in flight those CUs run the next batch's analysis (the
// C2 step 1.3 % faster).  So NS = 1 while the batch fills at most half the CUs (the
// latency-bound calls: batch 1 0.454 -> 0.364 ms, 64 streams 0.588 -> 0.479 ms,
// profiles/r06h_b1.log), NS = 2 above.  AEC_GRU_NS = 1 / 2 forces one (a mode knob, read per
// launch; the two are bit-identical in the waveform and est_erb, the loss is summed in another
// order, <= 1e-6 relative).
hipError_t launch_gru_synth(const GruArgs& g, const SynthArgs& y, int B, hipStream_t st) {
    if (B <= 0) return hipSuccess;
    // NS = 2 writes the waveform with 16-B stores (overlap-add on the recurrence waves)
    const bool al16 = y.ld_out % 4 == 0 && (reinterpret_cast<uintptr_t>(y.out) & 15) == 0;
    const int force = AEC_MODE_KNOB("AEC_GRU_NS", 0);
    const bool one = force == 1 || (force != 2 && 2 * (int64_t)B <= (int64_t)std::max(y.num_cus, 2));
    const int ns = one || (AEC_OLA_REC && !al16) ? 1 : 2;
    SynthArgs ya = y;
    ya.wmap = 0;
#if AEC_AB_BUILD
    // role placements for NS = 2 (role waves: 0-1 recurrence, 2-4 gi, 5-7 head, 8-11 synthesis;
    // hardware wave i runs on SIMD i % 4), entry k = role of hardware wave k
    static const unsigned long long kWmaps[] = {
        0,                      // identity: SIMD0 rec0 gi2 syn0 | rec1 head0 syn1 | gi0 head1 syn2 | gi1 head2 syn3
        0x46327591BA80ull,      // 1: rec0 rec1 gi0 | syn0 syn1 gi1 | syn2 head0 head1 | syn3 head2 gi2
        0xBA9874326510ull,      // 2: rec0 gi0 syn0 | rec1 gi1 syn1 | head0 gi2 syn2 | head1 head2 syn3
        0x4765B321A980ull,      // 3: rec0 rec1 head0 | syn0 gi0 head1 | syn1 gi1 head2 | syn2 syn3 gi2
        0x76584321BA90ull,      // 4: rec0 rec1 syn0 | syn1 gi0 head0 | syn2 gi1 head1 | syn3 gi2 head2
    };
    const int wm = AEC_AB_KNOB("AEC_GRU_WMAP", 0);
    if (ns == 2 && wm > 0 && wm < (int)(sizeof(kWmaps) / sizeof(kWmaps[0]))) ya.wmap = kWmaps[wm];
    if (ns == 1) ya.wmap = wmap_ns1(AEC_AB_KNOB("AEC_GRU_WMAP", 1));
#endif
#define AEC_GRU_SYNTH(NS_)                                                                                     \
    do {                                                                                                       \
        static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(gru_synth_kernel<NS_>), \
                                                           hipFuncAttributeMaxDynamicSharedMemorySize,         \
                                                           (int)gru_synth_smem_bytes());                       \
        if (attr != hipSuccess) return attr;                                                                   \
        hipLaunchKernelGGL(gru_synth_kernel<NS_>, dim3((B + NS_ - 1) / NS_), dim3(64 * (NS_ + kHelperWaves)),   \
                           gru_synth_smem_bytes(), st, g, ya, B, PipeArgs{});                                  \
    } while (0)
    if (ns == 1)
        AEC_GRU_SYNTH(1);
    else
        AEC_GRU_SYNTH(2);
#undef AEC_GRU_SYNTH
    return hipGetLastError();
}

// The small-batch pipeline (B <= the split path's limit, 2 B blocks <= one per CU: the host checks):
// B producer blocks, then B consumer blocks (NS = 1).
hipError_t launch_gru_synth_pipe(const GruArgs& g, const SynthArgs& y, const PipeArgs& q, int B, hipStream_t st) {
    if (B <= 0) return hipSuccess;
    if (!q.rows || !q.spec || !q.feats || !q.sched || q.sched_len > 48 || !q.progress || !q.err || !y.spec ||
        q.spin_limit <= 0 || (y.spec_stride != 0 && y.spec_stride != 256))
        return hipErrorInvalidValue;
    static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(gru_synth_kernel<1, true>),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       (int)gru_synth_smem_bytes());
    if (attr != hipSuccess) return attr;
    SynthArgs ya = y;
    ya.wmap = 0;
#if AEC_AB_BUILD
    ya.wmap = wmap_ns1(AEC_AB_KNOB("AEC_GRU_WMAP", 1));
#endif
    hipLaunchKernelGGL((gru_synth_kernel<1, true>), dim3(2 * B), dim3(64 * (1 + kHelperWaves)), gru_synth_smem_bytes(),
                       st, g, ya, B, q);
    return hipGetLastError();
}

}  // namespace aec

#ifdef AEC_TICK_PROF
extern "C" int aec_debug_gru_tick_prof(void* host, size_t bytes) {
    if (bytes < sizeof(aec::g_gtick)) return -1;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(aec::g_gtick), sizeof(aec::g_gtick)) == hipSuccess ? 0 : -2;
}
#endif
