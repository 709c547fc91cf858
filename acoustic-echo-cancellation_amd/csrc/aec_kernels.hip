// aec_kernels.hip — gfx950 STFT-side kernels of the Stage-2 AEC hot path.
//
// Reference path: Little_net.forward (Stage2_lhm/scripts/network/ERB.py:252-334).
// Pipeline per batch of B streams (each stream has batch=1 semantics):
//
//   K1 moments_lds_kernel  partial sums for x <- x - mean(x)/std(x) (ERB.py:254-256)
//   K2 analysis_kernel  frame + Hann + rFFT-512 (attention_ccrn.py:45-52) -> |X| (ERB.py:277-279)
//                       -> ERB band energies (ERB.py:282-284) for mic / ref / near
//   K2n nlms_analysis_kernel  K2 with the FD-NLMS canceller (one block per stream);
//                       for few streams the split path: K2 + spectrum rows,
//                       nlms_recursion_kernel, mic_erb_kernel
//   K3 gru_kernel       (aec_gru.hip) GRU + head + mask -> est_erb, loss
//   K4 synthesis_kernel gain = est_erb @ erb^T (ERB.py:306-310) * mic spectrum
//                       -> irFFT-512 + Hann + overlap-add / WOLA (attention_ccrn.py:82-101)
//                       -> + 1e-9 (ERB.py:316)
//   (K3 + K4 fused on the NLMS path: aec_gru_synth.hip; the per-hop streaming
//    step: aec_stream.hip)
//
// HBM layout (row-major, float32 unless noted):
//   signals  [B][ld]              caller-owned
//   mom      [B][3][8] double2    per-chunk (sum x, sum x^2)
//   feats    [B][Tmax][96]        mic_erb | ref_erb | near_erb per frame
//   est      [B][Tmax][32]        est_erb per frame
//   spec     [B][Tmax][256] float2  NLMS error spectrum E (slot 0 = (E[0], E[256]))
//   rows     [B][Tmax][2][256] float2  split path only: mic / ref spectrum rows
//   out      [B][ld_out]          caller-owned, 256*(N_b/256) samples per row
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <cstdlib>

#ifndef AEC_SPEC_ST_NT
#define AEC_SPEC_ST_NT 0   // E-spectrum stores nt (A/B builds only)
#endif

#include "aec_fft.h"
#include "aec_frame.h"
#include "aec_launch.h"
#include "aec_stft.h"
#include "aec_tables.h"

namespace aec {
#ifdef AEC_TICK_PROF
constexpr int kNlmsWavesProf = 12;
#endif

// --------------------------------------------------------------------------
// K1: per-(stream, signal, chunk) float64 partial moments.  The normaliser
// scalar c = mean/std (unbiased) is finished by every consumer from the
// kMomChunks partials in a fixed order (deterministic, no atomics).
// --------------------------------------------------------------------------
// K1 through LDS-DMA: thread tid sums float4 lo/4 + tid + 256 m for m = 0, 1, ... (then a fixed
// wave + block reduction); the loads land in a per-wave LDS ring (buffer_load ... lds, 4 KB in flight
// per wave) instead of registers (round 5's register-loaded moments_kernel gave bit-identical
// partials; it was retired in round 6 with the other timing variants).  The point is its footprint: 30 VGPRs and 16 KiB of LDS per block, which fits beside a
// K2n block (153 -> 160 VGPRs x 3 waves per SIMD, 131 KiB of LDS) or a gru_synth block (160 x 3,
// 132 KiB) on the same CU, so with batches in flight the next batch's moments pass (aec_prepare)
// streams under the compute kernels instead of holding whole CUs (the register-loaded kernel
// needs 36 VGPRs, 4 more than such a CU has left).
#ifndef AEC_MOM_SLOTS
#define AEC_MOM_SLOTS 4
#endif
constexpr int kMomSlots = AEC_MOM_SLOTS;   // ring of 4 KiB rounds (4: 16 KiB, 30 VGPRs; 5: 20 KiB, 32 VGPRs)
__device__ __forceinline__ void mom_wait_vm(int n) {
    // s_waitcnt vmcnt(n) (n < 16), other counters left alone
    switch (n) {
        case 0: __builtin_amdgcn_s_waitcnt(0x0F70); break;
        case 1: __builtin_amdgcn_s_waitcnt(0x0F71); break;
        case 2: __builtin_amdgcn_s_waitcnt(0x0F72); break;
        case 3: __builtin_amdgcn_s_waitcnt(0x0F73); break;
        case 4: __builtin_amdgcn_s_waitcnt(0x0F74); break;
        default: __builtin_amdgcn_s_waitcnt(0x0F75); break;
    }
}
// the one-item form compiles to <= 32 VGPRs and <= 20 KiB of LDS: one block fits beside a K2n (160 VGPRs x 3
// waves per SIMD, 131 KiB) or a gru_synth block (160 x 3, 132 KiB)
__global__ __launch_bounds__(256) void moments_lds_kernel(const float* __restrict__ mic, const float* __restrict__ ref,
                                                          const float* __restrict__ near, int64_t ld,
                                                          const int32_t* __restrict__ slen, double2* __restrict__ mom,
                                                          int b0) {
    // one array per ring slot: a read of slot j waits only for the DMAs into slot j
    __shared__ __attribute__((aligned(16))) float4 sR0[256];
    __shared__ __attribute__((aligned(16))) float4 sR1[256];
    __shared__ __attribute__((aligned(16))) float4 sR2[256];
    __shared__ __attribute__((aligned(16))) float4 sR3[256];
    __shared__ __attribute__((aligned(16))) float4 sR4[256];
    __shared__ __attribute__((aligned(16))) float4 sR5[256];
    __shared__ double r1[4], r2[4];
    // one item per block: the 3-D grid (chunk, signal, stream)
    const int ch = (int)blockIdx.x, s = (int)blockIdx.y, b = b0 + (int)blockIdx.z;
    const float* base = (s == 0 ? mic : (s == 1 ? ref : near));
    const float* x = base + (int64_t)b * ld;
    const int64_t n = slen[4 * b + s];
    const int64_t per = ((n + kMomChunks - 1) / kMomChunks + 1023) & ~(int64_t)1023;
    const int64_t lo = ch * per, hi = min(n, lo + per);
    double s1 = 0.0, s2 = 0.0;
    const int tid = threadIdx.x, wave = tid >> 6;
    auto acc4 = [&](const float4 v) {
        const double a = v.x, bb = v.y, c = v.z, d = v.w;
        s1 += (a + bb) + (c + d);
        s2 += (a * a + bb * bb) + (c * c + d * d);
    };
    if (lo < hi) {
        int64_t i = lo + tid;
        if ((reinterpret_cast<uintptr_t>(x) & 15) == 0) {
            const int64_t end4 = hi / 4, b4 = lo / 4;
            const int M = (int)((end4 - b4 + 255) / 256);      // DMA rounds (the last may be partial)
            const uint64_t xa = reinterpret_cast<uint64_t>(x + 4 * b4);
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                reinterpret_cast<void*>(xa), (short)0, (int)((end4 - b4) * 16), 0x00020000);
            // slot J is a distinct __shared__ array, named at compile time (static_for), so the
            // compiler's wait before an LDS read covers only the DMAs into that slot
            auto slot = [&](auto Jc) -> float4* {
                constexpr int J = decltype(Jc)::value;
                if constexpr (J == 0) return sR0;
                else if constexpr (J == 1) return sR1;
                else if constexpr (J == 2) return sR2;
                else if constexpr (J == 3) return sR3;
                else if constexpr (J == 4) return sR4;
                else return sR5;
            };
            auto issue = [&](int m, float4* sl) {              // the wave's 64 float4 of round m -> slot
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rs, (__attribute__((address_space(3))) void*)(sl + 64 * wave), 16,
                    (uint32_t)((256 * m + tid) * 16), 0, 0, 2);  // nt: each sample is read once here
            };
            static_for<0, kMomSlots>([&](auto Jc) {
                constexpr int J = decltype(Jc)::value;
                if (J < M) issue(J, slot(Jc));
            });
            for (int m0 = 0; m0 < M; m0 += kMomSlots) {
                static_for<0, kMomSlots>([&](auto Jc) {
                    constexpr int J = decltype(Jc)::value;
                    const int m = m0 + J;
                    if (m < M) {
                        mom_wait_vm(min(kMomSlots - 1, M - 1 - m));     // round m landed
                        // the read in asm: the compiler's own DMA tracking would wait for every
                        // DMA in flight (vmcnt(0)) before any LDS read; the wait above is exact
                        const uint32_t la = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) const void*)(
                            slot(Jc) + tid);
                        float4 v;
                        asm volatile("ds_read_b128 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(la) : "memory");
                        if (b4 + tid + 256 * (int64_t)m < end4) acc4(v);
                        if (m + kMomSlots < M) issue(m + kMomSlots, slot(Jc));
                    }
                });
            }
            i = end4 * 4 + tid;
        }
        for (; i < hi; i += 256) {
            const double a = x[i];
            s1 += a;
            s2 += a * a;
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        s1 += __shfl_xor(s1, o);
        s2 += __shfl_xor(s2, o);
    }
    if ((tid & 63) == 0) {
        r1[tid >> 6] = s1;
        r2[tid >> 6] = s2;
    }
    __syncthreads();
    if (tid == 0) {
        double t1[4], t2[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) { t1[q] = r1[q]; t2[q] = r2[q]; }
#pragma unroll
        for (int st = 1; st < 4; st <<= 1)
#pragma unroll
            for (int q = 0; q + st < 4; q += 2 * st) { t1[q] += t1[q + st]; t2[q] += t2[q + st]; }
        mom[((int64_t)b * 3 + s) * kMomChunks + ch] = make_double2(t1[0], t2[0]);
    }
}

// c for every (stream, signal): cvals[b*3 + s]
__global__ __launch_bounds__(256) void norm_finalize_kernel(const double2* __restrict__ mom,
                                                            const int32_t* __restrict__ slen,
                                                            float* __restrict__ cvals, int b0, int b1, int nsig) {
    const int i = b0 * 3 + blockIdx.x * 256 + threadIdx.x;
    if (i >= b1 * 3) return;
    const int b = i / 3, s = i % 3;
    cvals[i] = s < nsig ? norm_scalar(mom, b, s, slen[4 * b + s]) : 0.f;
}

// --------------------------------------------------------------------------
// K2: analysis.  grid = (ceil(Tmax/16), B), block = 256.  Each wave owns 4
// consecutive frames (16 lanes per frame) and its own LDS region, stages its
// own 5 hops per signal and runs the whole per-frame chain with wave-level
// ordering only — the block barrier is used once, for the shared tables.
// ERB projection: every lane runs the same number (L) of scheduled entries
// (bin, w0, w1, w2) -> three partial accumulators; bands wider than the
// schedule's split width are summed from two partials (ErbTables, aec_tables.h).
// The schedule is ordered so the 32 lanes of each mag gather hit 32 banks.
// --------------------------------------------------------------------------

// SIGPAR (few streams, the whole list in one round of waves): one (item, signal) task per wave
// instead of an item's three signals in sequence, so a short call's latency is one transform, not
// three; the same per-signal arithmetic (the same bits).
template <bool SIGPAR>
__global__ __launch_bounds__(256, 3) void analysis_kernel(AnalysisArgs p) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tid = threadIdx.x;
    const int L = p.sched_len;                                        // multiple of 4

    float4* sSched = reinterpret_cast<float4*>(smem);                 // L * 16
    int2* sComb = reinterpret_cast<int2*>(sSched + L * 16);           // 32
    float2* sTw512 = reinterpret_cast<float2*>(sComb + 32);           // 258
    float2* sTwT = sTw512 + 258;                                      // 256
    float* sHann = reinterpret_cast<float*>(sTwT + 256);              // 512
    float* sWave = sHann + 512;                                       // 4 * kWaveFloats

    const DevTables* tb = reinterpret_cast<const DevTables*>(p.tables);
    {
        sTwT[tid] = tb->twT[tid];
        const float4* sch = reinterpret_cast<const float4*>(p.sched);
        for (int i = tid; i < L * 16; i += 256) sSched[i] = sch[i];
        if (tid < 32) sComb[tid] = reinterpret_cast<const int2*>(p.sched + 4 * 16 * L)[tid];
        sTw512[tid] = tb->tw512[tid];
        if (tid < 2) sTw512[256 + tid] = tb->tw512[256 + tid];
        sHann[tid] = tb->hann[tid];
        sHann[tid + 256] = tb->hann[tid + 256];
    }
    const int wave = tid >> 6, lane = tid & 63;
    const int gg = lane >> 4, lb = lane & 15, sw = 16 * (gg & 1);
    float* wr = sWave + wave * kWaveFloats;
    float* scr = wr + gg * kGroupFloats;
    // float4 fast path needs every row 16-B aligned (bit s of `al`)
    const bool aligned_ld = ((p.ld & 3) == 0);
    int al = 0;
    for (int s = 0; s < p.nsig; ++s)
        al |= (aligned_ld && ((reinterpret_cast<uintptr_t>(p.sig[s]) & 15) == 0)) << s;
    __syncthreads();                                                  // tables staged; no block barrier below

    // Persistent wave: items gw, gw + NW, ... of the host-built work list
    // (one item = 4 consecutive frames of one stream).  The samples of the
    // next (item, signal) task are prefetched into registers while the
    // current one is transformed; the next item's descriptor one item ahead.
    const int NW = gridDim.x * 4;
    int64_t k = (int64_t)blockIdx.x * 4 + wave;
    float4 pf[kWavePf];
    if constexpr (SIGPAR) {
        if (k >= p.nitems * p.nsig) return;
    } else {
        if (k >= p.nitems) return;
    }
    WorkItem it = p.items[SIGPAR ? k / p.nsig : k];
    const int s0 = SIGPAR ? (int)(k % p.nsig) : 0;
    // signal s's own length: its normaliser and zero padding (mic = it.n)
    wave_prefetch(pf, p.sig[s0] + (int64_t)it.b * p.ld, s0 == 0 ? (int)it.n : p.slen[4 * it.b + s0], it.wt, lane,
                  (al >> s0) & 1);
    for (;;) {
        const int64_t k2 = k + NW;
        const WorkItem it2 = k2 < p.nitems && !SIGPAR ? p.items[k2] : it;
        const int64_t T = it.n / kHop + 1;
        const int64_t t = it.wt + gg;                                 // this group's frame
        for (int s = s0; s < (SIGPAR ? s0 + 1 : p.nsig); ++s) {
            // keep the LDS table reads inside the loop (hoisting the loop-invariant
            // schedule / twiddle / window reads would pin ~100 VGPRs)
            asm volatile("" ::: "memory");
            const int ns = s == 0 ? (int)it.n : p.slen[4 * it.b + s];
            const float cv = p.cvals ? p.cvals[it.b * 3 + s] : norm_scalar(p.mom, it.b, s, p.slen[4 * it.b + s]);
            wave_commit(wr, pf, cv, ns, it.wt, lane);
            if (SIGPAR) {
            } else if (s + 1 < p.nsig) {
                wave_prefetch(pf, p.sig[s + 1] + (int64_t)it.b * p.ld, p.slen[4 * it.b + s + 1], it.wt, lane,
                              (al >> (s + 1)) & 1);
            } else if (k2 < p.nitems) {
                wave_prefetch(pf, p.sig[0] + (int64_t)it2.b * p.ld, (int)it2.n, it2.wt, lane, al & 1);
            }
            wave_fence();
            float2 v[16];
            load_frame(v, wr, sHann, gg, lb);
            wave_fence();                                             // samples read before scratch reuse
            fft256<false>(v, lb, scr, sTwT);
            float2 xa[8], xb[8], x128;
            rfft_unpack(v, lb, sTw512, xa, xb, x128);
            if (p.rows && s < 2 && t < T) {
                // packed row of mic / ref for the small-batch NLMS recursion (row_to_scr's layout)
                float2* row = p.rows + (((int64_t)it.b * p.Tmax + t) * 2 + s) * 256;
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
            // magnitudes (ERB.py:277-279) -> scr[k ^ sw], k = 0..256
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                const int kk = lb + 16 * m;
                scr[kk ^ sw] = mag(xa[m]);
                scr[(kk == 0 ? 256 : 256 - kk) ^ sw] = mag(xb[m]);
            }
            if (lb == 0) scr[128 ^ sw] = mag(x128);
            wave_fence();
            erb_project(scr, sSched, sComb, L, lb, sw,
                        t < T ? p.feats + ((int64_t)it.b * p.Tmax + t) * 96 + 32 * s : nullptr);
        }
        if (SIGPAR || k2 >= p.nitems) break;      // SIGPAR: the host gives every task its own wave
        k = k2;
        it = it2;
    }
}

// --------------------------------------------------------------------------
// K2n: analysis with the frequency-domain NLMS linear echo canceller
// (SURVEY.md §8 a13 — absent from the reference, which feeds the raw mic
// spectrum to the post-filter; parity is held by the tests against the
// float64 restatement of this recursion, tests/test_gpu_nlms.py).
//
// The NLMS is sequential over frames and independent over (stream, bin), so
// one block owns one stream and walks it in chunks of 16 frames ("ticks").
// The block has 12 waves in three roles, one of each per SIMD (wave w ->
// role w / 4; frames 4 (w % 4) .. +3 of a chunk):
//   mic  waves, tick c: near transform -> near_erb; mic transform ->
//        spectrum row M[f] (left in the group's LDS scratch);
//   ref  waves, tick c: mic_erb of chunk c-2 from the error rows E (read back
//        from the spectrum buffer); ref transform -> ref_erb -> row R[f];
//   nlms waves, tick c: the 16 recursion steps of chunk c-1 for bin k = lane
//        (+ bin 256 on lane 0), from registers, E rows -> spectrum buffer.
// So the latency-bound recursion runs beside the transforms of the next
// chunk.  Tick end: barrier; the nlms waves copy (M, R) of their bin for the
// 16 frames into registers; barrier (rows consumed).  Taps, power and
// far-end history stay in the nlms waves' registers for the whole stream.
// Row layout: 256 float2, slot 0 packs the real pair (X[0], X[256]).
// Per bin and frame:
//   E = D - sum_l W[l] R[t-l];  P = beta P + (1-beta) sum_l |R[t-l]|^2;
//   W[l] += mu E conj(R[t-l]) / (P + delta)
// HBM traffic beyond K2: the E spectrum, 2 KiB per frame, written once and
// read back once (L2-resident) for mic_erb.
// --------------------------------------------------------------------------
#ifdef AEC_TICK_PROF
// timing experiments only (tools/tick_prof.py): s_memtime stamps of blocks 0 and 128 per wave and
// tick: loop top, work done, after barrier 1, after barrier 2
__device__ unsigned long long g_tick[2][kNlmsWavesProf][48][4];
#define TICK_STAMP(slot)                                                                               \
    do {                                                                                               \
        if ((blockIdx.x == 0 || blockIdx.x == 128) && lane == 0 && c < 48)                             \
            g_tick[blockIdx.x ? 1 : 0][wave][c][slot] = __builtin_amdgcn_s_memtime();                  \
    } while (0)
#else
#define TICK_STAMP(slot) do {} while (0)
#endif
constexpr int kSpecRow = 256;          // float2 per spectrum row
constexpr int kNlmsWaves = 12;
constexpr int kERow = 512 + 48;        // floats per LDS error row (split path): 256 float2, then ERB partials
#ifndef AEC_NLMS_MAGROW
#define AEC_NLMS_MAGROW 1              // K2n: the nlms waves write |E| rows (0: E rows, mags on the ref waves)
#endif
// K2n LDS row per frame of a chunk: with AEC_NLMS_MAGROW the nlms waves store |E[k]| at k ^ sw (the
// swizzle of the group that projects the frame, sw = 16 (i & 1) for frame i), bins 0..256 -> 273
// floats, then erb_project's 48 partials at kMagPart; otherwise the E row (256 float2) as before
constexpr int kMagPart = 288;
constexpr int kNRow = AEC_NLMS_MAGROW ? kMagPart + 48 : kERow;

__device__ __forceinline__ void nlms_transform(float* wr, float* scr, float4 (&pf)[kWavePf], float cval, int n, int wt,
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

template <int TAPS>
__global__ __launch_bounds__(kNlmsWaves * 64, 1) void nlms_analysis_kernel(NlmsArgs p) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tid = threadIdx.x;
    const int L = p.sched_len;

    float4* sSched = reinterpret_cast<float4*>(smem);                 // L * 16
    int2* sComb = reinterpret_cast<int2*>(sSched + L * 16);           // 32
    float2* sTw512 = reinterpret_cast<float2*>(sComb + 32);           // 258
    float2* sTwT = sTw512 + 258;                                      // 256
    float* sHann = reinterpret_cast<float*>(sTwT + 256);              // 512
    float* sWave = sHann + 512;                                       // 8 * kWaveFloats (mic, ref waves)
    float* sE = sWave + 8 * kWaveFloats;                              // 2 x kFPB error rows (kNRow floats)

    const DevTables* tb = reinterpret_cast<const DevTables*>(p.tables);
    if (tid < 256) {
        sTwT[tid] = tb->twT[tid];
        sTw512[tid] = tb->tw512[tid];
        if (tid < 2) sTw512[256 + tid] = tb->tw512[256 + tid];
        sHann[tid] = tb->hann[tid];
        sHann[tid + 256] = tb->hann[tid + 256];
        if (tid < 32) sComb[tid] = reinterpret_cast<const int2*>(p.sched + 4 * 16 * L)[tid];
    }
    {
        const float4* sch = reinterpret_cast<const float4*>(p.sched);
        for (int i = tid; i < L * 16; i += kNlmsWaves * 64) sSched[i] = sch[i];
    }
    const int wave = tid >> 6, lane = tid & 63;
    const int role = wave >> 2, q = wave & 3;                        // 0 mic, 1 ref, 2 nlms
    {
        // VALU issue between the three waves of a SIMD goes by priority, then age
        const int pr = role == 0 ? p.prio / 100 : (role == 1 ? (p.prio / 10) % 10 : p.prio % 10);
        switch (pr) {
            case 1: __builtin_amdgcn_s_setprio(1); break;
            case 2: __builtin_amdgcn_s_setprio(2); break;
            case 3: __builtin_amdgcn_s_setprio(3); break;
            default: break;
        }
    }
    const int gg = lane >> 4, lb = lane & 15, sw = 16 * (gg & 1);
    float* wr = sWave + (role < 2 ? wave : 0) * kWaveFloats;
    float* scr = wr + gg * kGroupFloats;
    const int b = p.b0 + blockIdx.x;
    const int n = (int)p.lens[b];                                   // mic: frame count
    const int n_ref = p.slen[4 * b + 1], n_near = p.slen[4 * b + 2];
    const int64_t T = n / kHop + 1;
    const int nch = (int)((T + kFPB - 1) / kFPB);
    const bool have_near = p.nsig == 3;
    const int64_t ld = p.ld;
    const float* row_mic = p.sig[0] + (int64_t)b * ld;
    const float* row_ref = p.sig[1] + (int64_t)b * ld;
    const float* row_near = have_near ? p.sig[2] + (int64_t)b * ld : nullptr;
    const bool al_ld = (ld & 3) == 0;
    const bool al_mic = al_ld && ((reinterpret_cast<uintptr_t>(p.sig[0]) & 15) == 0);
    const bool al_ref = al_ld && ((reinterpret_cast<uintptr_t>(p.sig[1]) & 15) == 0);
    const bool al_near = have_near && al_ld && ((reinterpret_cast<uintptr_t>(p.sig[2]) & 15) == 0);
    float2* spec = p.spec + (int64_t)b * p.Tmax * kSpecRow;
    float* feats = p.feats + (int64_t)b * p.Tmax * 96;
    const float mu = p.mu, beta = p.beta, delta = p.delta;
    // mic_erb of chunk c2 from its error rows (complete since the barriers of
    // tick c2 + 1); this group's frame 4 q + gg.  Run by the ref waves
    // (erb_role 1, merged with the ref ERB), by the nlms waves after their
    // recursion (erb_role 2, A/B only), or, without a near signal, by the mic
    // waves (erb_role 0: their near transform is gone, so the pass leaves the
    // ref waves and the two transform roles carry one transform and one ERB
    // projection pass each)
    const int erb_role = p.erb_role == 2 ? 2 : (p.erb_role == 0 && !have_near ? 0 : 1);
    auto mic_erb_pass = [&](int c2) {
        const int64_t t2 = (int64_t)c2 * kFPB + 4 * q + gg;
        float* er = sE + (c2 & 1) * kFPB * kNRow + (4 * q + gg) * kNRow;
#if AEC_NLMS_MAGROW
        // |E| row already in place (the nlms waves' stores, complete since tick c2 + 1's barriers)
        erb_project<kMagPart>(er, sSched, sComb, L, lb, sw, t2 < T ? feats + t2 * 96 : nullptr);
        return;
#endif
        const float2* row = reinterpret_cast<const float2*>(er);
        float2 xa[8], xb[8], x128;
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const int kk = lb + 16 * m;
            xa[m] = row[kk];
            xb[m] = row[(256 - kk) & 255];
        }
        x128 = row[128];
        xa[0] = lb == 0 ? make_float2(xa[0].x, 0.f) : xa[0];
        xb[0] = lb == 0 ? make_float2(xb[0].y, 0.f) : xb[0];     // slot 0 = (E[0], E[256])
        wave_fence();
        mags_to_scr(er, lb, sw, xa, xb, x128);
        wave_fence();
        erb_project(er, sSched, sComb, L, lb, sw, t2 < T ? feats + t2 * 96 : nullptr);
    };
    __syncthreads();

    // The nlms waves and the transform waves run separate loops with the same
    // two barriers per tick, so the register allocator sees the recursion's
    // state and the transforms' working set in disjoint regions.
    if (role == 2) {
        const int k = lane + 64 * q;                                  // bin k; k = 0 also bin 256
        NlmsBin<TAPS> st;
        st.reset(k == 0);
        float2 dd[kFPB], rr[kFPB];
        for (int c = 0; c < nch + 2; ++c) {
            TICK_STAMP(0);
            const int c1 = c - 1;
            if (c1 >= 0 && c1 < nch && !(p.mode & 1)) {
                // recursion of chunk c-1 -> E rows (LDS buffer c-1 & 1, spectrum
                // buffer); frames past the stream end only perturb state nobody
                // reads again (the unrolled loop stays branch-free)
                const int64_t t0 = (int64_t)c1 * kFPB;
                float* eb = sE + (c1 & 1) * kFPB * kNRow;
#pragma unroll
                for (int i = 0; i < kFPB; ++i) {
                    const float2 e = st.step(dd[i], rr[i], mu, beta, delta);
#if AEC_NLMS_MAGROW
                    // |E| (mags_to_scr's expression: slot 0's real pair as (E, 0) each) at k ^ sw_i
                    // bin 256 (lane k = 0's second real bin): every lane computes and stores it, the
                    // others into the row's partials area (rewritten by the mic_erb pass before it is
                    // read; lanes of a 32-lane half on distinct banks), so the wave holding slot 0
                    // runs no divergent branch
                    const int swi = 16 * (i & 1);
                    eb[i * kNRow + (k ^ swi)] = mag(make_float2(e.x, k == 0 ? 0.f : e.y));
                    eb[i * kNRow + (k == 0 ? (256 ^ swi) : kMagPart + (k & 31))] = mag(make_float2(e.y, 0.f));
#else
                    reinterpret_cast<float2*>(eb + i * kERow)[k] = e;
#endif
                    if (t0 + i < T) {
#if AEC_SPEC_ST_NT
                        typedef float f2v __attribute__((ext_vector_type(2)));
                        f2v ev; ev.x = e.x; ev.y = e.y;
                        __builtin_nontemporal_store(ev, reinterpret_cast<f2v*>(spec + (t0 + i) * kSpecRow + k));
#else
                        spec[(t0 + i) * kSpecRow + k] = e;
#endif
                    }
                }
            }
            if (erb_role == 2 && c >= 2 && !(p.mode & 4)) mic_erb_pass(c - 2);
            TICK_STAMP(1);
            __syncthreads();                                          // rows of chunk c complete
            TICK_STAMP(2);
            if (c < nch) {
#pragma unroll
                for (int i = 0; i < kFPB; ++i) {
                    const float* base = sWave + (i >> 2) * kWaveFloats + (i & 3) * kGroupFloats;
                    dd[i] = reinterpret_cast<const float2*>(base)[k];
                    rr[i] = reinterpret_cast<const float2*>(base + 4 * kWaveFloats)[k];
                }
            }
            __syncthreads();                                          // rows consumed
            TICK_STAMP(3);
        }
        return;
    }

    // mic waves walk near(c), mic(c), near(c+1), ...; ref waves ref(c), ref(c+1), ...
    float4 pf[kWavePf];
    if (role == 0) {
        if (have_near) wave_prefetch(pf, row_near, n_near, 4 * q, lane, al_near);
        else wave_prefetch(pf, row_mic, n, 4 * q, lane, al_mic);
    } else {
        wave_prefetch(pf, row_ref, n_ref, 4 * q, lane, al_ref);
    }
    for (int c = 0; c < nch + 2; ++c) {
        TICK_STAMP(0);
        const int wt = c * kFPB + 4 * q;
        const int64_t t = wt + gg;
        float2 xa[8], xb[8], x128;
        if (role == 0) {
            if (c < nch && !(p.mode & 8)) {
                if (have_near) {
                    nlms_transform(wr, scr, pf, p.cvals[b * 3 + 2], n_near, wt, lane, gg, lb, sHann, sTwT, sTw512,
                                   row_mic, n, wt, al_mic, xa, xb, x128);
                    if (!(p.mode & 2)) {
                        mags_to_scr(scr, lb, sw, xa, xb, x128);
                        wave_fence();
                        erb_project(scr, sSched, sComb, L, lb, sw, t < T ? feats + t * 96 + 64 : nullptr);
                    }
                }
                const bool more = c + 1 < nch;
                nlms_transform(wr, scr, pf, p.cvals[b * 3 + 0], n, wt, lane, gg, lb, sHann, sTwT, sTw512,
                               more ? (have_near ? row_near : row_mic) : nullptr, have_near ? n_near : n, wt + kFPB,
                               have_near ? al_near : al_mic, xa, xb, x128);
                row_to_scr(scr, lb, xa, xb, x128);
            }
            if (erb_role == 0 && c >= 2 && !(p.mode & 4)) mic_erb_pass(c - 2);
        } else {
            const bool erb2 = erb_role == 1 && c >= 2 && !(p.mode & 4);     // mic_erb of chunk c-2 due
            if (c < nch && !(p.mode & 8)) {
                nlms_transform(wr, scr, pf, p.cvals[b * 3 + 1], n_ref, wt, lane, gg, lb, sHann, sTwT, sTw512,
                               c + 1 < nch ? row_ref : nullptr, n_ref, wt + kFPB, al_ref, xa, xb, x128);
                mags_to_scr(scr, lb, sw, xa, xb, x128);
                wave_fence();
                if (erb2 && AEC_NLMS_MAGROW && !(p.mode & 16)) {
                    // ref_erb of chunk c and mic_erb of chunk c-2 (|E| rows) in one pass over the schedule
                    const int64_t t2 = (int64_t)(c - 2) * kFPB + 4 * q + gg;
                    float* er = sE + (c & 1) * kFPB * kNRow + (4 * q + gg) * kNRow;   // (c - 2) & 1
                    erb_project2(er, er + kMagPart, t2 < T ? feats + t2 * 96 : nullptr, scr, scr + 512,
                                 t < T ? feats + t * 96 + 32 : nullptr, sSched, sComb, L, lb, sw);
                } else {
                    if (erb2) mic_erb_pass(c - 2);
                    erb_project(scr, sSched, sComb, L, lb, sw, t < T ? feats + t * 96 + 32 : nullptr);
                }
                row_to_scr(scr, lb, xa, xb, x128);
            } else if (erb2) {
                mic_erb_pass(c - 2);
            }
        }
        TICK_STAMP(1);
        __syncthreads();                                              // rows of chunk c complete
        TICK_STAMP(2);
        __syncthreads();                                              // rows consumed
        TICK_STAMP(3);
    }
}

// --------------------------------------------------------------------------
// K4: synthesis.  One block of 256 threads per item of a host-built list
// (stream b, first output hop h0).  The block re-derives the mic spectra of
// the 16 frames h0 .. h0+15 (each wave stages and transforms 4 of them),
// applies the ERB gains, inverse-transforms and, after a block barrier,
// overlap-adds the 15 output hops h0 .. h0+14.  (A persistent variant that
// prefetches the next item was measured slower: the prefetch registers live
// across both transforms and cost a wave per SIMD.)  est_erb rows are padded
// to 33 floats (two frames' gathers of the same band hit different banks).
// --------------------------------------------------------------------------
constexpr int kEstStride = 33;

template <bool kSpec>
__global__ __launch_bounds__(256) void synthesis_kernel(SynthArgs p) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tid = threadIdx.x;

    float4* sBin = reinterpret_cast<float4*>(smem);                   // 257 (+3 pad)
    float2* sTw512 = reinterpret_cast<float2*>(sBin + 260);           // 258
    float2* sTwT = sTw512 + 258;                                      // 256
    float* sHann = reinterpret_cast<float*>(sTwT + 256);              // 512
    float* sCoff = sHann + 512;                                       // 256: 1/(window^2 OLA + 1e-8)
    float* sEst = sCoff + 256;                                        // 16 * 33 (+4 pad)
    float* sWave = sEst + kFPB * kEstStride + 4;                      // 4 * kWaveFloats

    const DevTables* tb = reinterpret_cast<const DevTables*>(p.tables);
    {
        const float4* bt = reinterpret_cast<const float4*>(p.bintab);
        sBin[tid] = bt[tid];
        if (tid == 0) sBin[256] = bt[256];
        sTwT[tid] = tb->twT[tid];
        sTw512[tid] = tb->tw512[tid];
        if (tid < 2) sTw512[256 + tid] = tb->tw512[256 + tid];
        sHann[tid] = tb->hann[tid];
        sHann[tid + 256] = tb->hann[tid + 256];
        sCoff[tid] = tb->inv_coff[tid];
    }
    const int wave = tid >> 6, lane = tid & 63;
    const int gg = lane >> 4, lb = lane & 15;
    const int g = tid >> 4;                                           // frame h0 + g
    float* wr = sWave + wave * kWaveFloats;
    float* scr = wr + gg * kGroupFloats;
    const bool aligned = ((p.ld & 3) == 0) && ((reinterpret_cast<uintptr_t>(p.mic) & 15) == 0);
    const bool oal = ((p.ld_out & 3) == 0) && ((reinterpret_cast<uintptr_t>(p.out) & 15) == 0);

    const WorkItem it = p.items[blockIdx.x];
    {
        const int b = it.b;
        const int64_t n = it.n;
        const int64_t T = n / kHop + 1;
        const int64_t h0 = it.wt;
        float4 pf[kWavePf];
        if (!kSpec)
            wave_prefetch(pf, p.mic + (int64_t)b * p.ld, (int)n, (int)(h0 + kWaveFrames * wave), lane, aligned);
        for (int i = tid; i < kFPB * 32; i += 256) {
            const int64_t t = h0 + (i >> 5);
            sEst[(i >> 5) * kEstStride + (i & 31)] = (t < T) ? p.est[((int64_t)b * p.Tmax + t) * 32 + (i & 31)] : 0.f;
        }
        if (!kSpec) wave_commit(wr, pf, p.cvals[b * 3 + 0], (int)n, (int)(h0 + kWaveFrames * wave), lane);
    }
    __syncthreads();                                                  // tables + est staged
    {
        const int b = it.b;
        const int64_t nhop = it.n / kHop;                             // T - 1
        const int64_t h0 = it.wt;
        float2 v[16];
        float2 xa[8], xb[8], x128;
        if (kSpec) {
            // NLMS error spectrum of frame h0 + g (slot 0 = (E[0], E[256]))
            const int64_t t = h0 + g;
            const bool ok = t <= nhop;
            const float2* row = p.spec + ((int64_t)b * p.Tmax + (ok ? t : 0)) * 256;
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
        } else {
            load_frame(v, wr, sHann, gg, lb);
            wave_fence();
            fft256<false>(v, lb, scr, sTwT);
            rfft_unpack(v, lb, sTw512, xa, xb, x128);
        }

        synth_frame(xa, xb, x128, sEst + g * kEstStride, sBin, sTw512, sTwT, sHann, scr, lb);
        __syncthreads();
        // overlap-add + WOLA normalisation + trim (attention_ccrn.py:92-99) + 1e-9 (ERB.py:316)
        float* orow = p.out + (int64_t)b * p.ld_out;
        const int nh = (int)min((int64_t)kHopsOut, nhop - h0);
        if (oal) {
            for (int e = tid; e < nh * (kHop / 4); e += 256) {
                const int i = e >> 6, r = (e & 63) * 4;
                const float4 a = *reinterpret_cast<const float4*>(sWave + i * kGroupFloats + 256 + r);
                const float4 c = *reinterpret_cast<const float4*>(sWave + (i + 1) * kGroupFloats + r);
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
                const float a = sWave[i * kGroupFloats + 256 + r];
                const float c = sWave[(i + 1) * kGroupFloats + r];
                orow[(h0 + i) * kHop + r] = (a + c) * sCoff[r] + 1e-9f;
            }
        }
    }
}

// --------------------------------------------------------------------------
// Small-batch NLMS path.  K2n runs one block per stream; with few streams the
// chip idles and a 10 s stream takes ~0.26 ms (40 ticks).  Here the
// transforms run frame-parallel in K2 (which also writes the packed mic / ref
// rows), the recursion is one block per stream over all frames (bin per
// lane, rows prefetched kRecP frames ahead), and mic_erb = ERB(|E|) runs
// frame-parallel again.  The per-frame arithmetic is K2n's own (NlmsBin,
// the same row layout and ERB pass), so the output is bit-identical.
// --------------------------------------------------------------------------
constexpr int kRecP = 8;

template <int TAPS>
__global__ __launch_bounds__(256) void nlms_recursion_kernel(const float2* __restrict__ rows, float2* __restrict__ spec,
                                                             const int64_t* __restrict__ lens, int64_t Tmax, float mu,
                                                             float beta, float delta, int b0, float2* dummy_rows) {
    const int b = b0 + blockIdx.x;
    const int64_t T = lens[b] / kHop + 1;
    const int k = threadIdx.x;
    const float2* r0 = rows + (int64_t)b * Tmax * 512;
    float2* e0 = spec + (int64_t)b * Tmax * kSpecRow;
    NlmsBin<TAPS> st;
    st.reset(k == 0);
    float2 dd[kRecP], rr[kRecP];
    auto fetch = [&](int64_t t, int i) {                  // rows past the end: any valid row (results unused)
        const int64_t tc = t < T ? t : T - 1;
        dd[i] = r0[tc * 512 + k];
        rr[i] = r0[tc * 512 + 256 + k];
    };
    // frames past the end store to this stream's dummy row (after the [B][Tmax][2][256]
    // rows): every store is unconditional, so the compiler's vmcnt bookkeeping
    // stays exact across the loop and the prefetched rows are not waited for early
    float2* dummy = dummy_rows + (int64_t)b * 256 + k;
#pragma unroll
    for (int i = 0; i < kRecP; ++i) fetch(i, i);
    for (int64_t t0 = 0; t0 < T; t0 += kRecP) {
#pragma unroll
        for (int i = 0; i < kRecP; ++i) {
            const float2 e = st.step(dd[i], rr[i], mu, beta, delta);
            *(t0 + i < T ? e0 + (t0 + i) * kSpecRow + k : dummy) = e;
            fetch(t0 + i + kRecP, i);
        }
    }
}

// mic_erb of every frame from its E row (K2n's mic_erb pass, frame-parallel):
// one 4-frame work item per wave, 4 waves per block
__global__ __launch_bounds__(256) void mic_erb_kernel(const float2* __restrict__ spec, float* __restrict__ feats,
                                                      const int64_t* __restrict__ lens, int64_t Tmax,
                                                      const float* __restrict__ sched, int L,
                                                      const WorkItem* __restrict__ items, int64_t nitems) {
    __shared__ __attribute__((aligned(16))) float4 sSched[48 * 16];
    __shared__ int2 sComb[32];
    __shared__ __attribute__((aligned(16))) float sScr[16][kERow];
    const int tid = threadIdx.x;
    for (int i = tid; i < L * 16; i += 256) sSched[i] = reinterpret_cast<const float4*>(sched)[i];
    if (tid < 32) sComb[tid] = reinterpret_cast<const int2*>(sched + 4 * 16 * L)[tid];
    __syncthreads();
    const int wave = tid >> 6, lane = tid & 63;
    const int gg = lane >> 4, lb = lane & 15, sw = 16 * (gg & 1);
    const int64_t item = (int64_t)blockIdx.x * 4 + wave;
    if (item >= nitems) return;
    const WorkItem it = items[item];
    const int64_t T = it.n / kHop + 1;
    const int64_t t = it.wt + gg;
    float* er = sScr[4 * wave + gg];
    float2 xa[8], xb[8], x128;
    row_to_pairs(spec + ((int64_t)it.b * Tmax + (t < T ? t : 0)) * kSpecRow, lb, true, xa, xb, x128);
    mags_to_scr(er, lb, sw, xa, xb, x128);
    wave_fence();
    erb_project(er, sSched, sComb, L, lb, sw, t < T ? feats + ((int64_t)it.b * Tmax + t) * 96 : nullptr);
}

hipError_t launch_nlms_recursion(const float2* rows, float2* spec, const int64_t* lens, int64_t Tmax, int taps,
                                 float mu, float beta, float delta, int b0, int nb, float2* dummy_rows, hipStream_t st) {
    if (nb <= 0) return hipSuccess;
    switch (taps) {
#define AEC_REC_CASE(T)                                                                                       \
        case T: hipLaunchKernelGGL(nlms_recursion_kernel<T>, dim3(nb), dim3(256), 0, st, rows, spec, lens, Tmax, mu, \
                                   beta, delta, b0, dummy_rows); break;
        AEC_REC_CASE(1) AEC_REC_CASE(2) AEC_REC_CASE(3) AEC_REC_CASE(4)
        AEC_REC_CASE(5) AEC_REC_CASE(6) AEC_REC_CASE(7) AEC_REC_CASE(8)
#undef AEC_REC_CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

hipError_t launch_mic_erb(const float2* spec, float* feats, const int64_t* lens, int64_t Tmax, const float* sched,
                          int sched_len, const WorkItem* items, int64_t nitems, hipStream_t st) {
    if (nitems <= 0) return hipSuccess;
    if (sched_len > 48) return hipErrorInvalidValue;
    hipLaunchKernelGGL(mic_erb_kernel, dim3((unsigned)((nitems + 3) / 4)), dim3(256), 0, st, spec, feats, lens, Tmax,
                       sched, sched_len, items, nitems);
    return hipGetLastError();
}

// --------------------------------------------------------------------------
// host-side launchers (called by aec_api.hip)
// --------------------------------------------------------------------------
hipError_t launch_moments(const float* mic, const float* ref, const float* near, int64_t ld,
                          const int32_t* slen, double2* mom, int b0, int nb, int nsig, hipStream_t st) {
    if (nb <= 0) return hipSuccess;
    // moments_lds_kernel, one 256-thread block per (chunk, signal, stream), 4 KiB rounds through a
    // 4-round LDS ring: 30 VGPRs and 16 KiB, so a block fits beside a K2n or gru_synth block and the
    // look-ahead pass (aec_prepare) of the next batch streams under the compute kernels of the
    // batches in flight (C2 0.581-0.592 against 0.597-0.600 ms, profiles/r05r_persist8_lookahead_ab.log).
    // Standalone 0.080 ms for 256 x 10 s x 3 signals.
    // (Round 6: a canonical one-wave-per-chunk form with f32 pre-summed float4s measured 0.4 % slower
    // in the step, profiles/r06c_moments_canonical_ab.log, tools/archive/r06c_canonical_moments.patch.)
    hipLaunchKernelGGL(moments_lds_kernel, dim3(kMomChunks, nsig, nb), dim3(256), 0, st, mic, ref, near, ld, slen, mom,
                       b0);
    return hipGetLastError();
}

hipError_t launch_norm_finalize(const double2* mom, const int32_t* slen, float* cvals, int b0, int b1, int nsig,
                                hipStream_t st) {
    if (b1 <= b0) return hipSuccess;
    hipLaunchKernelGGL(norm_finalize_kernel, dim3(((b1 - b0) * 3 + 255) / 256), dim3(256), 0, st, mom, slen, cvals,
                       b0, b1, nsig);
    return hipGetLastError();
}

hipError_t launch_analysis(const AnalysisArgs& a, hipStream_t st) {
    if (a.nitems <= 0) return hipSuccess;
    // persistent: at most kAnalysisBlocksPerCU blocks per CU, 4 waves (items) each
    const int64_t cap = (int64_t)a.num_cus * kAnalysisBlocksPerCU;
    // few streams: one (item, signal) task per wave when the whole list fits one round of waves
    const int64_t tasks = a.nitems * a.nsig;
    if ((tasks + 3) / 4 <= cap) {
        hipLaunchKernelGGL(analysis_kernel<true>, dim3((unsigned)((tasks + 3) / 4)), dim3(256),
                           analysis_smem_bytes(a.sched_len), st, a);
        return hipGetLastError();
    }
    const int64_t want = (a.nitems + 3) / 4;
    const unsigned grid = (unsigned)(want < cap ? want : cap);
    hipLaunchKernelGGL(analysis_kernel<false>, dim3(grid), dim3(256), analysis_smem_bytes(a.sched_len), st, a);
    return hipGetLastError();
}

hipError_t launch_synthesis(const SynthArgs& a, hipStream_t st) {
    if (a.nitems <= 0) return hipSuccess;
    if (a.spec)
        hipLaunchKernelGGL(synthesis_kernel<true>, dim3((unsigned)a.nitems), dim3(256), synthesis_smem_bytes(), st, a);
    else
        hipLaunchKernelGGL(synthesis_kernel<false>, dim3((unsigned)a.nitems), dim3(256), synthesis_smem_bytes(), st, a);
    return hipGetLastError();
}

template <int TAPS>
static hipError_t launch_nlms_t(const NlmsArgs& a, int nb, hipStream_t st) {
    // > 64 KiB of LDS: opt in once per instantiation
    static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(nlms_analysis_kernel<TAPS>),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (attr != hipSuccess) return attr;
    hipLaunchKernelGGL(nlms_analysis_kernel<TAPS>, dim3(nb), dim3(kNlmsWaves * 64), nlms_smem_bytes(a.sched_len, TAPS),
                       st, a);
    return hipGetLastError();
}

hipError_t launch_nlms_analysis(const NlmsArgs& a, int nb, hipStream_t st) {
    if (nb <= 0) return hipSuccess;
    switch (a.taps) {
        case 1: return launch_nlms_t<1>(a, nb, st);
        case 2: return launch_nlms_t<2>(a, nb, st);
        case 3: return launch_nlms_t<3>(a, nb, st);
        case 4: return launch_nlms_t<4>(a, nb, st);
        case 5: return launch_nlms_t<5>(a, nb, st);
        case 6: return launch_nlms_t<6>(a, nb, st);
        case 7: return launch_nlms_t<7>(a, nb, st);
        case 8: return launch_nlms_t<8>(a, nb, st);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace aec

#ifdef AEC_TICK_PROF
extern "C" int aec_debug_tick_prof(void* host, size_t bytes) {
    if (bytes < sizeof(aec::g_tick)) return -1;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(aec::g_tick), sizeof(aec::g_tick)) == hipSuccess ? 0 : -2;
}
#endif
