// ARCHIVED (round 6): not built into libaec_hip.so. The 8-wave persistent LSTM recurrence was
// bit-identical to crn_persist.hip and measured 15 % slower; kept for the record.
// crn_persist3.hip — persistent LSTM recurrence of the DCCRN, 8 waves per
// block (gfx950).  The geometry, hand-off protocol and numerics are
// lstm_persist2_kernel's (crn_persist.hip; reference NavieComplexLSTM,
// dccrn.py:423-450 inside DCCRN v2, dccrn2.py:67-80): one launch runs all T
// frames of a layer, 256 blocks = (team, slice), a team = (cell, 64 streams =
// 128 rows) of 32 blocks, a block = 32 units x 4 gates of W_hh, the team's
// rows in two halves whose phases alternate.  What changes is the split of a
// block's work over its waves:
//   * 8 waves, two per SIMD: wave (uq, kh) holds 8 units x 4 gates x one K
//     half of W_hh (2 column tiles x 16 K steps = 128 AGPRs), so two waves fit
//     a SIMD and one wave's cell update and DMA issues run while the other
//     wave's MFMAs execute (v2: one wave per SIMD, whose MFMA gaps could not
//     hold the cell-update stages and DMA issues).
//   * A column tile is 8 units x 2 gates: lane fr holds gate 2t + (fr >> 3) of
//     unit fr & 7, so the four gates of a cell sit in lanes fr and fr ^ 8; one
//     DPP row_ror:8 exchange per tile brings them together, each lane finishing
//     two of the tile's four rows.
//   * The partial sums of the two K halves meet through LDS as in v2 (the
//     partner wave (uq, 1 - kh) shares the SIMD).
// The K halves are summed separately as in v2 and the cell arithmetic is v2's,
// in the same order: results equal v2's bit for bit
// (tests/test_gpu_crn.py::test_persistent_recurrence_8_waves_bit_exact).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

#include "crn_gemm.h"
#include "crn_launch.h"

#ifndef CRN_PERSIST_AUX
#define CRN_PERSIST_AUX 16   // cache policy of the h hand-off DMA: sc1
#endif

namespace crn {

namespace {
constexpr int kP3H = 1024;                               // H
constexpr int kPC = 2, kPS = 2;                          // cells, sequences (NavieComplexLSTM)
constexpr int kP3U = 32;                                 // units per block
constexpr int kP3Rows = 128;                             // rows (stream, sequence) per team
constexpr int kP3Threads = 512;
constexpr int kP3QH = 64;                                // rows per half
constexpr int kP3Chunk = 2 * kP3QH * 128;                // one K chunk of a half: [2 kh][64 rows][128 B]
constexpr int kP3X = 4 * 2 * 2 * 2 * 64;                 // float4 [uq][dest kh][own slot][tile][lane]
constexpr int kP3C = kP3Rows * 33;                       // f32 [128 rows][33] cell state
constexpr int kP3HS = 8 * 32 * 8;                        // bf16 [wave][32 rows][8 units] h staging
static_assert(4 * kP3Chunk + 2 * 16 * kP3X + 4 * kP3C + 2 * kP3HS <= 160 * 1024, "LDS budget");
constexpr float kL2e3 = 1.4426950408889634f;

__device__ __forceinline__ float med3_3(float x, float lo, float hi) { return __builtin_amdgcn_fmed3f(x, lo, hi); }
__device__ __forceinline__ void sched_fence3() { __builtin_amdgcn_sched_barrier(0); }
template <class F, int... I>
__device__ __forceinline__ void sfor_seq3(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void sfor3(F&& f) {   // f(integral_constant<int, 0>) ... f(<N - 1>)
    sfor_seq3(f, std::make_integer_sequence<int, N>{});
}
// x of lane l ^ 8 within each 16-lane row (DPP row_ror:8)
__device__ __forceinline__ float xor8(float x) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x128, 0xF, 0xF, false));
}
}  // namespace

__global__ __launch_bounds__(kP3Threads, 1) void lstm_persist3_kernel(PersistArgs p) {
    // one array per A buffer (the DMA into buffer (j + 3) % 4 must not look like a write to the
    // buffer read at chunk j)
    __shared__ __attribute__((aligned(16))) char sA0[kP3Chunk];
    __shared__ __attribute__((aligned(16))) char sA1[kP3Chunk];
    __shared__ __attribute__((aligned(16))) char sA2[kP3Chunk];
    __shared__ __attribute__((aligned(16))) char sA3[kP3Chunk];
    auto abuf = [&](auto Jc) -> char* {
        constexpr int b = decltype(Jc)::value & 3;
        if constexpr (b == 0) return sA0;
        else if constexpr (b == 1) return sA1;
        else if constexpr (b == 2) return sA2;
        else return sA3;
    };
    __shared__ float4 sX[kP3X];     // partial sums sent to the partner wave (slots 2, 3)
    __shared__ float4 sXo[kP3X];    // the wave's own slots 0, 1 (their registers are free during the next phase)
    __shared__ float sC[kP3C];
    __shared__ __attribute__((aligned(16))) bf16_t sHS[kP3HS];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int uq = wave & 3, kh = wave >> 2;                 // waves w and w + 4 share a SIMD
    const int nteams = 2 * p.G;
    const int team = blockIdx.x % nteams, slice = blockIdx.x / nteams;
    const int cell = team & 1, group = team >> 1;
    const int u0 = slice * kP3U;
    const int fr = lane & 15, fq = lane >> 4;
    const bool lo = fr < 8;                                  // rows 0, 1 of each own tile group (else 2, 3)
    const int u = fr & 7, jl = 8 * uq + u;                   // the lane's unit (of the block's 32)
    const int i0 = lo ? 0 : 2;
    int* err = p.sync + kPersistErr;
    bool stalled = false;

    // W_hh of the wave: tile t, column fr = gate 2t + (fr >> 3) of unit jl, K half kh
    u32x4 wreg[2][16];
    {
        const int ub = 2 * slice + (uq >> 1);                // packed 16-unit block
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            const int row = ub * 64 + (2 * t + (fr >> 3)) * 16 + (uq & 1) * 8 + u;
            const bf16_t* wb = p.whh + ((size_t)cell * 4 * kP3H + row) * kP3H + 512 * kh + 8 * fq;
#pragma unroll
            for (int ks = 0; ks < 16; ++ks) wreg[t][ks] = *reinterpret_cast<const u32x4*>(wb + 32 * ks);
        }
    }
#pragma unroll
    for (int hf = 0; hf < 2; ++hf)
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int ii = 0; ii < 2; ++ii) sC[(64 * hf + 32 * kh + 16 * k + 4 * fq + i0 + ii) * 33 + jl] = 0.f;

    const uint64_t yframe = (uint64_t)p.B * kPC * kPS * kP3H;
    const uint32_t yrow0 = (uint32_t)((size_t)(p.b0 + group * 64) * kPC * kPS * kP3H * 2 + (size_t)cell * kPS * kP3H * 2);
    const int nvs = min(64, p.nb - group * 64);             // valid streams of the team
    const uint64_t gxframe = (uint64_t)p.B * kPS * kPC * 4 * kP3H;
    // Gx row r of the team is 16 KiB after row 0; the wave's 8 units are 64 B at 64 uq
    const uint32_t gu = __builtin_amdgcn_readfirstlane(
        (uint32_t)(((size_t)2 * (p.b0 + group * 64) * kPC * 4 * kP3H + (size_t)cell * 4 * kP3H + (size_t)u0 * 4) * 2 +
                   64 * uq));

    // Gx of the lane's 4 cells of half HF, frame t (4 buffer loads per wave; out-of-range rows read
    // 0).  One buffer: the half finished next is loaded once the current finish has read it (v2
    // keeps both halves in registers; here they would not fit beside 128 AGPRs of W_hh)
    uint2 gxr[2][2];                                         // [own slot][row ii]
    auto load_gx = [&](auto HFc, int t, bool valid) {
        constexpr int HF = decltype(HFc)::value;
        const __amdgpu_buffer_rsrc_t rg = make_rsrc(p.gx + (size_t)(valid ? t : 0) * gxframe, gxframe * 2);
        const uint32_t so = __builtin_amdgcn_readfirstlane(gu + (uint32_t)(64 * HF + 32 * kh) * 16384u);
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int ii = 0; ii < 2; ++ii) {
                const int x = 16 * k + 4 * fq + i0 + ii;     // row of the wave's 32
                const int st = 32 * HF + 16 * kh + (x >> 1);
                const uint32_t vo = (valid && st < nvs) ? (uint32_t)(x * 16384 + u * 8) : kOOB;
                const auto v = __builtin_amdgcn_raw_buffer_load_b64(rg, vo, so, 0);
                gxr[k][ii] = make_uint2(v[0], v[1]);
            }
    };
    // A chunk j of half hm from y frame (ry): rows 16 uq .. 16 uq + 15 of the half, K half kh
    uint32_t vlA[2];
#pragma unroll
    for (int par = 0; par < 2; ++par) {
        const int q = (lane & 7) ^ (((lane >> 4) + 4 * par) & 7);
        vlA[par] = (uint32_t)((8 * uq + (lane >> 4)) * 8192 + ((lane >> 3) & 1) * 2048 + 16 * q);
    }
    auto issue_a = [&](int hm, auto Jc, const __amdgpu_buffer_rsrc_t& ry) {
        constexpr int j = decltype(Jc)::value;
        char* buf = abuf(Jc) + kh * (kP3QH * 128) + 16 * uq * 128;
        const uint32_t so = __builtin_amdgcn_readfirstlane(yrow0 + (uint32_t)(32 * hm) * 8192u +
                                                           (uint32_t)(512 * kh + 64 * j) * 2);
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int st = 32 * hm + 8 * uq + 4 * i + (lane >> 4);
            const uint32_t vo = st < nvs ? vlA[i] : kOOB;
            __builtin_amdgcn_raw_ptr_buffer_load_lds(ry, (__attribute__((address_space(3))) void*)(buf + 8 * i * 128),
                                                     16, vo, (int)(so + (uint32_t)i * 32768u), 0, CRN_PERSIST_AUX);
        }
    };
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
    auto arrive = [&](int hf) {
        if (wave == 0 && lane == 0)
            __hip_atomic_fetch_add(p.sync + (team * 2 + hf) * 16, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    };

    f32x4 acc[2][4][2];                                     // [half][slot][tile] (acc[HF] dead once in LDS)
    float4 xv[2];                                           // partner partial sums of one own slot
    f32x4 fin[2];                                           // own partial sums, then + xv (gate pre-activations)
    float cv[2][2];                                         // c of the lane's cells [own slot][row ii]
    float zi, zf, zg, zo, ef, ei, eg, eo, cn, ec;
    const float4* xs = sX;
    float4* xw = sX;
    bf16_t* hs = sHS + wave * 256;

    // one stage of the cell update of half HF (compile-time stage index ST, 0 .. kStages - 1)
    auto stage = [&](auto HFc, auto STc) {
        constexpr int HF = decltype(HFc)::value, ST = decltype(STc)::value;
        auto loads = [&](auto Kc) {
            constexpr int K = decltype(Kc)::value;
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const float4 o = sXo[(((uq * 2 + kh) * 2 + K) * 2 + t) * 64 + lane];
                fin[t] = f32x4{o.x, o.y, o.z, o.w};
                xv[t] = xs[(((uq * 2 + kh) * 2 + K) * 2 + t) * 64 + lane];
            }
#pragma unroll
            for (int ii = 0; ii < 2; ++ii) cv[K][ii] = sC[(64 * HF + 32 * kh + 16 * K + 4 * fq + i0 + ii) * 33 + jl];
        };
        auto xadd = [&](auto Kc) {
            constexpr int K = decltype(Kc)::value;
#pragma unroll
            for (int t = 0; t < 2; ++t)
                fin[t] = f32x4{fin[t][0] + xv[t].x, fin[t][1] + xv[t].y, fin[t][2] + xv[t].z, fin[t][3] + xv[t].w};
        };
        // cell (K, row i0 + II), sub-stage SS: v2's expressions (crn_persist.hip)
        auto cellst = [&](auto Kc, auto Ic, auto SSc) {
            constexpr int K = decltype(Kc)::value, II = decltype(Ic)::value, SS = decltype(SSc)::value;
            if constexpr (SS == 0) {
                // gates of (row, unit): own tile values at row i0 + II, the partner lane's (fr ^ 8)
                // for the same row; the partner sends the rows this lane finishes
                const float a0l = fin[0][II], a0h = fin[0][2 + II];
                const float a1l = fin[1][II], a1h = fin[1][2 + II];
                const float r0 = xor8(lo ? a0h : a0l), r1 = xor8(lo ? a1h : a1l);
                const float o0 = lo ? a0l : a0h, o1 = lo ? a1l : a1h;
                const uint2 g = gxr[K][II];
                zi = med3_3((lo ? o0 : r0) + __uint_as_float(g.x << 16), -20.f, 20.f);
                zf = med3_3((lo ? r0 : o0) + __uint_as_float(g.x & 0xFFFF0000u), -20.f, 20.f);
                zg = med3_3((lo ? o1 : r1) + __uint_as_float(g.y << 16), -10.f, 10.f);
                zo = (lo ? r1 : o1) + __uint_as_float(g.y & 0xFFFF0000u);
            } else if constexpr (SS == 1) {
                ef = __builtin_amdgcn_exp2f(zf * -kL2e3);
                ei = __builtin_amdgcn_exp2f(zi * -kL2e3);
            } else if constexpr (SS == 2) {
                eg = __builtin_amdgcn_exp2f(zg * (-2.f * kL2e3));
                eo = __builtin_amdgcn_exp2f(zo * -kL2e3);
            } else if constexpr (SS == 3) {
                const float a = 1.f + ef, bd = (1.f + ei) * (1.f + eg);
                cn = (cv[K][II] * bd + (1.f - eg) * a) * __builtin_amdgcn_rcpf(a * bd);
                sC[(64 * HF + 32 * kh + 16 * K + 4 * fq + i0 + II) * 33 + jl] = cn;
            } else if constexpr (SS == 4) {
                ec = __builtin_amdgcn_exp2f(med3_3(cn, -10.f, 10.f) * (-2.f * kL2e3));
            } else {
                const float h = (1.f - ec) * __builtin_amdgcn_rcpf((1.f + eo) * (1.f + ec));
                hs[(16 * K + 4 * fq + i0 + II) * 8 + u] = f2bf(h);
            }
        };
        // plan: 0 loads(0) | 2 xadd(0) | 3..14 cells (0, 0..1) | 12 loads(1) | 15 xadd(1) | 16..27 cells (1, 0..1)
        // (fin of slot 0 is last read at stage 9, the second cell's sub-stage 0)
        if constexpr (ST == 0) loads(std::integral_constant<int, 0>{});
        if constexpr (ST == 12) loads(std::integral_constant<int, 1>{});
        if constexpr (ST == 2) xadd(std::integral_constant<int, 0>{});
        if constexpr (ST == 15) xadd(std::integral_constant<int, 1>{});
        if constexpr (ST >= 3 && ST < 15)
            cellst(std::integral_constant<int, 0>{}, std::integral_constant<int, (ST - 3) / 6>{},
                   std::integral_constant<int, (ST - 3) % 6>{});
        if constexpr (ST >= 16 && ST < 28)
            cellst(std::integral_constant<int, 1>{}, std::integral_constant<int, (ST - 16) / 6>{},
                   std::integral_constant<int, (ST - 16) % 6>{});
    };
    constexpr int kStages = 28;
    // h of half hf, frame t: the wave's 32 rows x 8 units, one 8-B sc1 store per lane
    auto publish = [&](int hf, int t) {
        const int x = lane >> 1, part = lane & 1;
        const uint2 v = *reinterpret_cast<const uint2*>(reinterpret_cast<const char*>(hs) + x * 16 + part * 8);
        const int st = 32 * hf + 16 * kh + (x >> 1);
        const __amdgpu_buffer_rsrc_t ry = make_rsrc(p.y + (size_t)t * yframe, yframe * 2);
        const uint32_t off = st < nvs ? yrow0 + (uint32_t)(st * 8192 + (x & 1) * 2048 + (u0 + 8 * uq + 4 * part) * 2)
                                      : kOOB;
        typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{v.x, v.y}, ry, off, 0, 16);
    };
    auto write_x = [&](auto HMc) {                          // slots 2, 3 -> the partner wave; 0, 1 -> own
        constexpr int HM = decltype(HMc)::value;
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const f32x4 v = acc[HM][2 + k][t], w = acc[HM][k][t];
                xw[(((uq * 2 + (1 - kh)) * 2 + k) * 2 + t) * 64 + lane] = make_float4(v[0], v[1], v[2], v[3]);
                sXo[(((uq * 2 + kh) * 2 + k) * 2 + t) * 64 + lane] = make_float4(w[0], w[1], w[2], w[3]);
            }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // before the barrier that hands them over
    };
    auto phase_plain = [&](auto HMc, bool zero_hm, int tf, int T) {
        constexpr int HM = decltype(HMc)::value, HF = 1 - HM;
        __syncthreads();                                     // partner partial sums of HF visible
        if (tf >= 0) {
            sfor3<kStages>([&](auto S) { stage(std::integral_constant<int, HF>{}, S); });
            publish(HF, tf);
            wait_vm<0>();
            __syncthreads();                                 // every wave's store done; reads of X done
            arrive(HF);
            if (zero_hm) load_gx(HMc, tf, true);             // the next phase finishes (HM, tf)
        }
        if (zero_hm) {
#pragma unroll
            for (int s = 0; s < 4; ++s)
#pragma unroll
                for (int t = 0; t < 2; ++t) acc[HM][s][t] = f32x4{0.f, 0.f, 0.f, 0.f};
            write_x(HMc);
        }
    };
    auto phase_mfma = [&](auto HMc, int tm, int tf, int T) {
        constexpr int HM = decltype(HMc)::value, HF = 1 - HM;
        poll(HM, 32 * tm);                                   // h of (HM, tm - 1) from the whole team
        const __amdgpu_buffer_rsrc_t ry = make_rsrc(p.y + (size_t)(tm - 1) * yframe, yframe * 2);
        issue_a(HM, std::integral_constant<int, 0>{}, ry);
        issue_a(HM, std::integral_constant<int, 1>{}, ry);
        issue_a(HM, std::integral_constant<int, 2>{}, ry);
        const int rsw = ((fr >> 1) & 7);
        sfor3<8>([&](auto Jc) {
            constexpr int j = decltype(Jc)::value;
            // issue order (vmcnt is in order): C0 C1 C2 | C3 | C4 | C5 | C6 S | C7 G: 2 DMAs per
            // chunk, the h store S, 4 Gx loads G; j = 5 also completes S
            constexpr int kWait[8] = {4, 4, 4, 4, 5, 6, 7, 4};
            wait_vm<kWait[j]>();
            __builtin_amdgcn_s_barrier();
            if constexpr (j == 5) arrive(HF);
            if constexpr (j == 7)
                if (p.read_ahead && (HM == 0 || tm + 1 < T)) read_ahead(HF);
            if constexpr (j + 3 < 8) issue_a(HM, std::integral_constant<int, j + 3>{}, ry);
            if constexpr (j == 4) load_gx(HMc, tm, true);    // the next phase finishes (HM, tm)
            const char* base = abuf(Jc) + kh * (kP3QH * 128);
            auto read_af = [&](int n) {                      // group n: ks2 = n / 4, slot n % 4
                const int rl = 16 * ((n & 3) ^ (2 * kh)) + fr;
                return *reinterpret_cast<const u32x4*>(base + rl * 128 + ((((n >> 2) * 4 + fq) ^ rsw) * 16));
            };
            u32x4 afr[3];
            afr[0] = read_af(0);
            afr[1] = read_af(1);
            sfor3<8>([&](auto Nc) {
                constexpr int n = decltype(Nc)::value, ks2 = n >> 2, s = n & 3;
                if constexpr (n + 2 < 8) afr[(n + 2) % 3] = read_af(n + 2);
                const u32x4 af = afr[n % 3];
                sfor3<2>([&](auto Tc) {
                    constexpr int t = decltype(Tc)::value;
                    if constexpr (j == 0 && ks2 == 0)
                        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0"
                                     : "=&v"(acc[HM][s][t]) : "v"(af), "a"(wreg[t][2 * j + ks2]));
                    else
                        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                                     : "+v"(acc[HM][s][t]) : "v"(af), "a"(wreg[t][2 * j + ks2]));
                    sched_fence3();
                });
                constexpr int st = 8 * j + n;
                if constexpr (st < kStages) stage(std::integral_constant<int, HF>{}, std::integral_constant<int, st>{});
                sched_fence3();
            });
            if constexpr (j == 3) publish(HF, tf);
        });
        // inline-asm MFMA results: wait states before the DS writes read them
        asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
        write_x(HMc);
    };

    const int T = p.T;
    load_gx(std::integral_constant<int, 0>{}, 0, true);              // finished by (H1, 0)'s phase
    phase_plain(std::integral_constant<int, 0>{}, true, -1, T);     // (H0, 0): h_{-1} = 0
    phase_plain(std::integral_constant<int, 1>{}, true, 0, T);      // (H1, 0), finish (H0, 0)
    for (int t = 1; t < T; ++t) {
        phase_mfma(std::integral_constant<int, 0>{}, t, t - 1, T);  // (H0, t), finish (H1, t - 1)
        phase_mfma(std::integral_constant<int, 1>{}, t, t, T);      // (H1, t), finish (H0, t)
    }
    phase_plain(std::integral_constant<int, 0>{}, false, T - 1, T); // finish (H1, T - 1)
    wait_vm<0>();
}

hipError_t launch_lstm_persist3(const PersistArgs& a, hipStream_t st) {
    if (a.nb <= 0 || a.T <= 0) return hipSuccess;
    if (a.G < 1 || a.G > 4 || 2 * a.nb > 128 * a.G) return hipErrorInvalidValue;
    const void* fn = reinterpret_cast<const void*>(lstm_persist3_kernel);
    static const int per_cu = [fn] {
        int n = 0;
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, kP3Threads, 0) == hipSuccess ? n : 0;
    }();
    if (per_cu < 1) return hipErrorCooperativeLaunchTooLarge;
    PersistArgs args = a;
    void* kargs[] = {&args};
    return hipLaunchKernel(fn, dim3(64 * a.G), dim3(kP3Threads), kargs, 0, st);
}

}  // namespace crn
