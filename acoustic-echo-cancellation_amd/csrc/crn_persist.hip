// crn_persist.hip — persistent LSTM recurrence of the DCCRN (gfx950).
//
// Reference: NavieComplexLSTM (dccrn.py:423-450) inside DCCRN v2
// (dccrn2.py:67-80, 147-157): per layer, 2 LSTM cells (real_lstm,
// imag_lstm) x 2 input sequences (x_r, x_i) with h, c of width H, run over T
// frames.  The input projection Gx = x W_ih^T + b is hoisted for all frames
// (one GEMM per layer, crn_kernels.hip); what remains per frame is
//     gates = Gx[t] + h_{t-1} W_hh^T ;  c, h = cell(gates, c)     (i, f, g, o)
// which lstm_step_kernel runs as one launch per frame (1,252 launches per
// 256 x 10 s batch at ~15.7 us: ~2.5 us launch, ~10 us re-streaming 512 KiB of
// h and W_hh per CU from L2 / MALL).
//
// Here one launch runs all T frames of a layer:
//   * 256 blocks, one per CU; block = (team, slice); team = (cell, group of
//     64 streams = 128 rows (stream, sequence)); slice = 32 units (128 gate
//     columns) of that cell.  A team is 32 blocks: blockIdx % nteams is the
//     team, so with the hardware's round-robin dealing a team shares one XCD.
//   * W_hh of the block's 128 gate rows (256 KiB bf16) stays in registers for
//     the whole layer: 4 waves, wave (ug, kh) holds 16 units x 4 gates x one
//     K half (4 x 16 MFMA B fragments = all 256 AGPRs; the accumulators are
//     VGPRs), so the only per-frame operand traffic is h_{t-1} of the team.
//   * The team's 128 rows split into halves H0 (streams 0..31 of the group)
//     and H1 (32..63), each with its own arrival counter.  Phase (hm, t) runs
//     the gates GEMM of half hm for frame t (8 K chunks of 64, moved global ->
//     LDS by buffer-load-to-LDS DMA, sc1, 3 chunks in flight) and, between its
//     MFMAs, the cell update of the other half (the frame it finished last):
//     partner partial sums, Gx, c, the seven transcendentals per cell and the
//     h write.  That half's h leaves after chunk 3 and its hand-off to the team
//     runs under chunks 4..7, so the next phase of that half normally finds
//     its counter already reached.  Phases: (H0, t) finishes (H1, t-1);
//     (H1, t) finishes (H0, t).  The instruction order inside a phase is fixed
//     by scheduling barriers: MFMA, cell-update stage, MFMA.
//   * Per wave (ug, kh): the 4 row tiles of a half are accumulator slots
//     s = 0..3, row tile s ^ 2kh (slots 0, 1 are the tiles this wave finishes,
//     2, 3 go to the partner wave of the other K half through LDS).  c stays in
//     LDS; Gx of a wave's rows is loaded into registers a phase ahead.
//   * h_t leaves as sc1 (write-through) 16-B stores into y of frame t (the
//     layer output, written once per launch); after every wave's store has
//     completed, one agent-scope atomic add per block on the half's counter.
//     A block starts phase (hm, t) after the counter reaches 32 t and reads
//     h_{t-1} from y of frame t-1 with sc1 DMA: no cache can hold an older copy
//     of a y line (it is read only after its last write in this launch).  A
//     two-slot exchange ring read back by the same CUs every other frame
//     returned stale h from frame 3 on.
//   * Every spin is bounded: a wave whose team stalls past the bound sets the
//     error word and stops waiting; its team-mates time out the same way, so
//     the grid always drains.  The host reads the error word before the call
//     that launched the grid returns (crn_api.hip, run_persist / persist_check),
//     serialises persistent launches per device (a second one co-resident with
//     the first could starve it of CUs) and sizes the grid to at most one block
//     per CU.
//
// Numerics: bf16 h / W, f32 accumulation and cell state, the step kernel's
// cell arithmetic; the K halves are summed separately (not bit-identical to
// lstm_step_kernel; batch composition stays bit-exact since every row runs
// the same code).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "crn_gemm.h"
#include "crn_launch.h"

#ifndef CRN_PERSIST_AUX
#define CRN_PERSIST_AUX 16   // cache policy of the h hand-off DMA: sc1
#endif

namespace crn {

namespace {
constexpr int kPH = 1024;                 // H (net_conf: hidden_dim * conv_channels[-1] / 2)
constexpr int kPC = 2, kPS = 2;           // cells, sequences (NavieComplexLSTM)
constexpr int kPU = 32;                   // units per block
constexpr int kPRows = 128;               // rows (stream, sequence) per team
constexpr int kPThreads = 256;
}  // namespace

namespace {
constexpr int kQH = 64;                                 // rows per half
constexpr int kQChunk = 2 * kQH * 128;                  // one K chunk of a half: [2 kh][64 rows][128 B]
// LDS: separate static arrays, so that the compiler's wait for LDS written by DMA
// (it cannot see which DMA wrote which bytes) applies to the A buffers only
constexpr int kQX = 2 * 2 * 2 * 4 * 64;                 // float4 [ug][dest kh][own slot][q][lane]
constexpr int kQC = kPRows * 33;                        // f32 [128 rows][33] cell state
constexpr int kQHS = 4 * 32 * 16;                       // bf16 [wave][32 rows][16 units] h staging
static_assert(4 * kQChunk + 16 * kQX + 4 * kQC + 2 * kQHS <= 160 * 1024, "LDS budget");
constexpr float kL2e = 1.4426950408889634f;

__device__ __forceinline__ float med3(float x, float lo, float hi) { return __builtin_amdgcn_fmed3f(x, lo, hi); }
__device__ __forceinline__ void sched_fence() { __builtin_amdgcn_sched_barrier(0); }
template <class F, int... I>
__device__ __forceinline__ void static_for_seq(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {   // f(integral_constant<int, 0>) ... f(<N - 1>)
    static_for_seq(f, std::make_integer_sequence<int, N>{});
}
}  // namespace

__global__ __launch_bounds__(kPThreads, 1) void lstm_persist2_kernel(PersistArgs p) {
    // one array per A buffer: the DMA into buffer (j + 3) % 4 must not look like a write to
    // the buffer read at chunk j (the compiler would wait for it)
    __shared__ __attribute__((aligned(16))) char sQA0[kQChunk];
    __shared__ __attribute__((aligned(16))) char sQA1[kQChunk];
    __shared__ __attribute__((aligned(16))) char sQA2[kQChunk];
    __shared__ __attribute__((aligned(16))) char sQA3[kQChunk];
    auto abuf = [&](auto Jc) -> char* {
        constexpr int b = decltype(Jc)::value & 3;
        if constexpr (b == 0) return sQA0;
        else if constexpr (b == 1) return sQA1;
        else if constexpr (b == 2) return sQA2;
        else return sQA3;
    };
    __shared__ float4 sQX[kQX];
    __shared__ float sQC[kQC];
    __shared__ __attribute__((aligned(16))) bf16_t sQH[kQHS];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int ug = wave & 1, kh = wave >> 1;
    const int nteams = 2 * p.G;
    const int team = blockIdx.x % nteams, slice = blockIdx.x / nteams;
    const int cell = team & 1, group = team >> 1;
    const int u0 = slice * kPU;
    const int fr = lane & 15, fq = lane >> 4;
    int* err = p.sync + kPersistErr;
    bool stalled = false;                                   // wave-uniform: a poll timed out (error word set)

    u32x4 wreg[4][16];
    {
        const bf16_t* wb = p.whh + ((size_t)cell * 4 * kPH + (size_t)((2 * slice + ug) * 4) * 16 + fr) * kPH +
                           512 * kh + 8 * fq;
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int ks = 0; ks < 16; ++ks)
                wreg[q][ks] = *reinterpret_cast<const u32x4*>(wb + (size_t)q * 16 * kPH + 32 * ks);
    }
    float* sC = sQC;
    const int jl = 16 * ug + fr;
    // the lane's cells: half hf, own slot k (row tile 2 kh + k of the half), rows 4 fq + i of the tile
#pragma unroll
    for (int hf = 0; hf < 2; ++hf)
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int i = 0; i < 4; ++i) sC[(64 * hf + 32 * kh + 16 * k + 4 * fq + i) * 33 + jl] = 0.f;

    const uint64_t yframe = (uint64_t)p.B * kPC * kPS * kPH;
    const uint32_t yrow0 = (uint32_t)((size_t)(p.b0 + group * 64) * kPC * kPS * kPH * 2 + (size_t)cell * kPS * kPH * 2);
    const int nvs = min(64, p.nb - group * 64);             // valid streams of the team
    const uint64_t gxframe = (uint64_t)p.B * kPS * kPC * 4 * kPH;
    // Gx row r of the team is 16 KiB after row 0; the wave's 16 units are 128 B at 128 ug
    const uint32_t gu = __builtin_amdgcn_readfirstlane(
        (uint32_t)(((size_t)2 * (p.b0 + group * 64) * kPC * 4 * kPH + (size_t)cell * 4 * kPH + (size_t)u0 * 4) * 2 +
                   128 * ug));

    // ---- Gx of the lane's 8 cells of half HF, frame t, into registers (8 buffer loads per wave;
    //      out-of-range rows read 0 without a branch, so every wave issues the same count)
    uint2 gxr[2][2][4];                                     // [half][own slot][row i]
    auto load_gx = [&](auto HFc, int t, bool valid) {
        constexpr int HF = decltype(HFc)::value;
        const __amdgpu_buffer_rsrc_t rg = make_rsrc(p.gx + (size_t)(valid ? t : 0) * gxframe, gxframe * 2);
        const uint32_t so = __builtin_amdgcn_readfirstlane(gu + (uint32_t)(64 * HF + 32 * kh) * 16384u);
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int x = 16 * k + 4 * fq + i;           // row of the wave's 32
                const int st = 32 * HF + 16 * kh + (x >> 1);
                const uint32_t vo = (valid && st < nvs) ? (uint32_t)(x * 16384 + fr * 8) : kOOB;
                const auto v = __builtin_amdgcn_raw_buffer_load_b64(rg, vo, so, 0);
                gxr[HF][k][i] = make_uint2(v[0], v[1]);
            }
    };
    // A chunk j of half hm from y frame (ry): rows 32 ug .. 32 ug + 31 of the half, K half kh
    uint32_t vlA[2];
#pragma unroll
    for (int par = 0; par < 2; ++par) {
        const int q = (lane & 7) ^ (((lane >> 4) + 4 * par) & 7);
        vlA[par] = (uint32_t)((16 * ug + (lane >> 4)) * 8192 + ((lane >> 3) & 1) * 2048 + 16 * q);
    }
    auto issue_a = [&](int hm, auto Jc, const __amdgpu_buffer_rsrc_t& ry) {
        constexpr int j = decltype(Jc)::value;
        char* buf = abuf(Jc) + kh * (kQH * 128) + 32 * ug * 128;
        const uint32_t so = __builtin_amdgcn_readfirstlane(yrow0 + (uint32_t)(32 * hm) * 8192u +
                                                           (uint32_t)(512 * kh + 64 * j) * 2);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int st = 32 * hm + 16 * ug + 4 * i + (lane >> 4);
            const uint32_t vo = st < nvs ? vlA[i & 1] : kOOB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(ry, (__attribute__((address_space(3))) void*)(buf + 8 * i * 128),
                                                     16, vo, (int)(so + (uint32_t)i * 32768u), 0, CRN_PERSIST_AUX);
        }
    };
    // counter of the next phase's half read ahead (chunk 7 of the current phase): when the team is
    // already there, the next poll skips its device-scope round trip.  A vector load through an
    // offset the compiler cannot see as zero, so it is neither scalarised nor waited for at once.
    int pre_v = 0, pre_hm = -1;
    auto read_ahead = [&](int hm) {
        int z;
        asm volatile("v_mov_b32 %0, 0" : "=v"(z));
        pre_v = __hip_atomic_load(p.sync + (team * 2 + hm) * 16 + z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        pre_hm = hm;
    };
    auto poll = [&](int hm, int target) {
        if (stalled) return;
        target += p.stall;
        if (pre_hm == hm) {
            pre_hm = -1;
            if (__builtin_amdgcn_readfirstlane(pre_v) >= target) return;
        }
        int bad = 0;
        if (lane == 0) {
            int* cnt = p.sync + (team * 2 + hm) * 16;
            int n = 0;
            while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
                __builtin_amdgcn_s_sleep(1);
                if (++n > p.spin_limit) {
                    __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    bad = 1;
                    break;
                }
            }
        }
        stalled = __builtin_amdgcn_readfirstlane(bad) != 0;
    };
    // one arrival per block per half and frame (32 atomics per counter and frame, not 128): called
    // behind a workgroup barrier that follows every wave's wait completing its h store
    auto arrive = [&](int hf) {
        if (wave == 0 && lane == 0)
            __hip_atomic_fetch_add(p.sync + (team * 2 + hf) * 16, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };

    f32x4 acc[2][4][4];                                     // [half][slot][gate]
    // finish state (one tile's loads in flight, one cell's temporaries)
    float4 xv[2][4];
    float cv[2][4];
    float zi, zf, zg, zo, ef, ei, eg, eo, cn, ec;
    const float4* xs = sQX;
    float4* xw = sQX;
    bf16_t* hs = sQH + wave * 512;

    // one stage of the cell update of half HF (compile-time stage index ST, 0 .. 52)
    auto stage = [&](auto HFc, auto STc) {
        constexpr int HF = decltype(HFc)::value, ST = decltype(STc)::value;
        constexpr int kLoad1 = 21;                          // tile 1's loads go out during tile 0's last cell
        auto loads = [&](auto Kc) {
            constexpr int K = decltype(Kc)::value;
#pragma unroll
            for (int q = 0; q < 4; ++q) xv[K][q] = xs[(((ug * 2 + kh) * 2 + K) * 4 + q) * 64 + lane];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                cv[K][i] = sC[(64 * HF + 32 * kh + 16 * K + 4 * fq + i) * 33 + jl];
            }
        };
        auto xadd = [&](auto Kc) {
            constexpr int K = decltype(Kc)::value;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                f32x4& a = acc[HF][K][q];
                a = f32x4{a[0] + xv[K][q].x, a[1] + xv[K][q].y, a[2] + xv[K][q].z, a[3] + xv[K][q].w};
            }
        };
        // cell (K, I), sub-stage SS (0..5): i, f, g, o = sig(zi), sig(zf), tanh(zg), sig(zo);
        // c' = f c + i g = [c (1+ei)(1+eg) + (1-eg)(1+ef)] / [(1+ef)(1+ei)(1+eg)] with ex = e^-zx
        // (eg = e^-2zg); clamps keep the products finite (|zi|, |zf| <= 20, |zg|, |c'| <= 10: below
        // f32 resolution of sigmoid / tanh there); h = o tanh(c') = (1-ec) / [(1+eo)(1+ec)]
        auto cellst = [&](auto Kc, auto Ic, auto SSc) {
            constexpr int K = decltype(Kc)::value, I = decltype(Ic)::value, SS = decltype(SSc)::value;
            if constexpr (SS == 0) {
                const uint2 g = gxr[HF][K][I];
                zi = med3(acc[HF][K][0][I] + __uint_as_float(g.x << 16), -20.f, 20.f);
                zf = med3(acc[HF][K][1][I] + __uint_as_float(g.x & 0xFFFF0000u), -20.f, 20.f);
                zg = med3(acc[HF][K][2][I] + __uint_as_float(g.y << 16), -10.f, 10.f);
                zo = acc[HF][K][3][I] + __uint_as_float(g.y & 0xFFFF0000u);
            } else if constexpr (SS == 1) {
                ef = __builtin_amdgcn_exp2f(zf * -kL2e);
                ei = __builtin_amdgcn_exp2f(zi * -kL2e);
            } else if constexpr (SS == 2) {
                eg = __builtin_amdgcn_exp2f(zg * (-2.f * kL2e));
                eo = __builtin_amdgcn_exp2f(zo * -kL2e);
            } else if constexpr (SS == 3) {
                const float a = 1.f + ef, bd = (1.f + ei) * (1.f + eg);
                cn = (cv[K][I] * bd + (1.f - eg) * a) * __builtin_amdgcn_rcpf(a * bd);
                sC[(64 * HF + 32 * kh + 16 * K + 4 * fq + I) * 33 + jl] = cn;
            } else if constexpr (SS == 4) {
                ec = __builtin_amdgcn_exp2f(med3(cn, -10.f, 10.f) * (-2.f * kL2e));
            } else {
                const float h = (1.f - ec) * __builtin_amdgcn_rcpf((1.f + eo) * (1.f + ec));
                hs[(16 * K + 4 * fq + I) * 16 + fr] = f2bf(h);
            }
        };
        // plan: 0 loads(0) | 2 xadd(0) | 3..26 cells (0, 0..3) | 21 loads(1) | 27 xadd(1) | 28..51 cells (1, 0..3)
        if constexpr (ST == 0) loads(std::integral_constant<int, 0>{});
        if constexpr (ST == kLoad1) loads(std::integral_constant<int, 1>{});
        if constexpr (ST == 2) xadd(std::integral_constant<int, 0>{});
        if constexpr (ST == 27) xadd(std::integral_constant<int, 1>{});
        if constexpr (ST >= 3 && ST < 27)
            cellst(std::integral_constant<int, 0>{}, std::integral_constant<int, (ST - 3) / 6>{},
                   std::integral_constant<int, (ST - 3) % 6>{});
        if constexpr (ST >= 28 && ST < 52)
            cellst(std::integral_constant<int, 1>{}, std::integral_constant<int, (ST - 28) / 6>{},
                   std::integral_constant<int, (ST - 28) % 6>{});
    };
    constexpr int kStages = 52;
    // h of half hf, frame t: the wave's 32 rows x 16 units, one 16-B sc1 store per lane
    auto publish = [&](int hf, int t) {
        const int x = lane >> 1, hh = lane & 1;
        const u32x4 v = *reinterpret_cast<const u32x4*>(reinterpret_cast<const char*>(hs) + x * 32 + hh * 16);
        const int st = 32 * hf + 16 * kh + (x >> 1);
        const __amdgpu_buffer_rsrc_t ry = make_rsrc(p.y + (size_t)t * yframe, yframe * 2);
        const uint32_t off = st < nvs ? yrow0 + (uint32_t)(st * 8192 + (x & 1) * 2048 + (u0 + 16 * ug + 8 * hh) * 2)
                                      : kOOB;
        __builtin_amdgcn_raw_buffer_store_b128(v, ry, off, 0, 16);
    };
    auto write_x = [&](auto HMc) {                          // sent slots 2, 3 -> the partner wave
        constexpr int HM = decltype(HMc)::value;
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const f32x4 v = acc[HM][2 + k][q];
                xw[(((ug * 2 + (1 - kh)) * 2 + k) * 4 + q) * 64 + lane] = make_float4(v[0], v[1], v[2], v[3]);
            }
    };
    // phase without gates GEMM (frame 0 of a half: h_{-1} = 0; or the last finish)
    auto phase_plain = [&](auto HMc, bool zero_hm, int tf, int T) {
        constexpr int HM = decltype(HMc)::value, HF = 1 - HM;
        __syncthreads();                                     // partner partial sums of HF visible
        if (tf >= 0) {
            static_for<kStages>([&](auto S) { stage(std::integral_constant<int, HF>{}, S); });
            publish(HF, tf);
            wait_vm<0>();
            __syncthreads();                                 // every wave's store done; reads of X done before it is rewritten
            arrive(HF);
            load_gx(std::integral_constant<int, HF>{}, tf + 1, tf + 1 < T);
        }
        if (zero_hm) {
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int q = 0; q < 4; ++q) acc[HM][s][q] = f32x4{0.f, 0.f, 0.f, 0.f};
            write_x(HMc);
        }
    };
    // phase with the gates GEMM of half HM for frame tm (>= 1) and the cell update of (HF, tf)
    auto phase_mfma = [&](auto HMc, int tm, int tf, int T) {
        constexpr int HM = decltype(HMc)::value, HF = 1 - HM;
        poll(HM, 32 * tm);                                   // h of (HM, tm - 1) from the whole team
        const __amdgpu_buffer_rsrc_t ry = make_rsrc(p.y + (size_t)(tm - 1) * yframe, yframe * 2);
        issue_a(HM, std::integral_constant<int, 0>{}, ry);
        issue_a(HM, std::integral_constant<int, 1>{}, ry);
        issue_a(HM, std::integral_constant<int, 2>{}, ry);
        const int rsw = ((fr >> 1) & 7);                     // swizzle key of every A row the lane reads
        static_for<8>([&](auto Jc) {
                constexpr int j = decltype(Jc)::value;
                // issue order (vmcnt is in order): C0 C1 C2 | C3 | C4 | C5 | C6 S | C7 G: 4 DMAs per chunk,
                // the h store S, 8 Gx loads G.  j = 5 also completes S.  Wave 0 adds the arrival atomic
                // after the j = 5 barrier: counted as absent, which only makes its later waits stricter.
                constexpr int kWait[8] = {8, 8, 8, 8, 9, 12, 13, 8};
                wait_vm<kWait[j]>();
                __builtin_amdgcn_s_barrier();
                if constexpr (j == 5) arrive(HF);
                if constexpr (j == 7)
                    if (p.read_ahead && (HM == 0 || tm + 1 < T)) read_ahead(HF);   // the next phase polls half HF
                if constexpr (j + 3 < 8) issue_a(HM, std::integral_constant<int, j + 3>{}, ry);
                if constexpr (j == 4) load_gx(std::integral_constant<int, HF>{}, tf + 1, tf + 1 < T);
                const char* base = abuf(Jc) + kh * (kQH * 128);
                auto read_af = [&](int n) {                  // group n: ks2 = n / 4, slot n % 4 (row tile slot ^ 2 kh)
                    const int rl = 16 * ((n & 3) ^ (2 * kh)) + fr;
                    return *reinterpret_cast<const u32x4*>(base + rl * 128 + ((((n >> 2) * 4 + fq) ^ rsw) * 16));
                };
                u32x4 afr[3];
                afr[0] = read_af(0);
                afr[1] = read_af(1);
                static_for<8>([&](auto Nc) {
                        constexpr int n = decltype(Nc)::value, ks2 = n >> 2, s = n & 3;
                        if constexpr (n + 2 < 8) afr[(n + 2) % 3] = read_af(n + 2);
                        const u32x4 af = afr[n % 3];
                        static_for<4>([&](auto Qc) {
                                constexpr int q = decltype(Qc)::value;
                                if constexpr (j == 0 && ks2 == 0)
                                    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0"
                                                 : "=&v"(acc[HM][s][q]) : "v"(af), "a"(wreg[q][2 * j + ks2]));
                                else
                                    asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                                                 : "+v"(acc[HM][s][q]) : "v"(af), "a"(wreg[q][2 * j + ks2]));
                                sched_fence();
                                if constexpr (q & 1) {
                                    constexpr int st = 2 * (8 * j + n) + (q >> 1);
                                    if constexpr (st < kStages)
                                        stage(std::integral_constant<int, HF>{}, std::integral_constant<int, st>{});
                                    sched_fence();
                                }
                        });
                });
                if constexpr (j == 3) publish(HF, tf);
        });
        // inline-asm MFMA results: wait states before the DS writes read them
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
        write_x(HMc);
    };

    const int T = p.T;
    load_gx(std::integral_constant<int, 0>{}, 0, true);
    load_gx(std::integral_constant<int, 1>{}, 0, true);
    phase_plain(std::integral_constant<int, 0>{}, true, -1, T);     // (H0, 0): h_{-1} = 0
    phase_plain(std::integral_constant<int, 1>{}, true, 0, T);      // (H1, 0), finish (H0, 0)
    for (int t = 1; t < T; ++t) {
        phase_mfma(std::integral_constant<int, 0>{}, t, t - 1, T);  // (H0, t), finish (H1, t - 1)
        phase_mfma(std::integral_constant<int, 1>{}, t, t, T);      // (H1, t), finish (H0, t)
    }
    phase_plain(std::integral_constant<int, 0>{}, false, T - 1, T); // finish (H1, T - 1)
    wait_vm<0>();
}

bool persist_supported(int H, int cells, int seqs, int num_cus) {
    return H == kPH && cells == kPC && seqs == kPS && num_cus >= 64;
}

hipError_t launch_lstm_persist(const PersistArgs& a, hipStream_t st) {
    if (a.nb <= 0 || a.T <= 0) return hipSuccess;
    if (a.G < 1 || a.G > 4 || 2 * a.nb > 128 * a.G) return hipErrorInvalidValue;
    const void* fn = reinterpret_cast<const void*>(lstm_persist2_kernel);
    // Co-residency: one block per CU (LDS and registers), grid <= CUs (the caller chunks the
    // streams by the CU count).  A plain launch: hipLaunchCooperativeKernel gives the same
    // guarantee but its queue crashed rocprofv3 at process exit.
    static const int per_cu = [fn] {
        int n = 0;
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, kPThreads, 0) == hipSuccess ? n : 0;
    }();
    if (per_cu < 1) return hipErrorCooperativeLaunchTooLarge;
    PersistArgs args = a;
    void* kargs[] = {&args};
    return hipLaunchKernel(fn, dim3(64 * a.G), dim3(kPThreads), kargs, 0, st);
}

}  // namespace crn
