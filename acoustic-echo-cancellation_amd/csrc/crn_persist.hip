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
//     columns) of that cell.  A team is 32 blocks: blockIdx % 8 is the team,
//     so with the hardware's round-robin dealing a team shares one XCD.
//   * W_hh of the block's 128 gate rows (256 KiB bf16) stays in registers for
//     the whole layer: 4 waves, wave (ug, kh) holds 16 units x 4 gates x one
//     K half (4 x 16 MFMA B fragments = all 256 AGPRs; the accumulators are
//     VGPRs), so the only per-frame operand traffic is h_{t-1} of the team
//     (256 KiB per block).
//   * c stays in LDS.  Gx of the frame arrives by DMA into a consumed A
//     buffer during the last K chunks.
//   * h_t leaves through LDS as sc1 (write-through) 16-B stores into y of
//     frame t (the layer output, written once per launch), then one
//     agent-scope atomic add per block on the team's arrival counter.  A block
//     starts frame t after its team's counter reaches 32 t (sc1 poll, bounded,
//     then a workgroup barrier before any load of h) and reads h_{t-1} from y
//     of frame t-1 with sc1 DMA: no cache can hold an older copy of a y line
//     (it is read only after its last write in this launch).  A two-slot
//     exchange ring read back by the same CUs every other frame returned
//     stale h from frame 3 on.
//   * Per frame a wave multiplies its K half: 8 K-chunks of 64 (two producer
//     slices), moved global -> LDS by buffer-load-to-LDS DMA (sc1) by the two
//     waves of that half, 4 buffers (3 chunks in flight; the VGPRs hold W);
//     the K halves' partial sums meet through LDS (each wave finishes half of
//     the rows: own + partner, the same sum either way).
//   * Every spin is bounded: a block whose team stalls past the bound sets the
//     error word and leaves; its team-mates time out the same way, so the grid
//     always drains.  The host serialises persistent launches per device
//     (a second one co-resident with the first could starve it of CUs) and
//     sizes the grid to at most one block per CU.
//
// Numerics: bf16 h / W, f32 accumulation and cell state, the step kernel's
// cell arithmetic; the K halves are summed separately (not bit-identical to
// lstm_step_kernel; batch composition stays bit-exact since every row runs
// the same code).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

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
constexpr int kPSlices = kPH / kPU;       // 32 blocks per team
constexpr int kPThreads = 256;
constexpr int kNBuf = 4;                  // A chunk buffers (3 chunks in flight)
constexpr int kABuf = kPRows * 128;       // one K half of one chunk: 128 rows x 128 B (swizzled 16-B slots)
constexpr int oA = 0;                              // [kNBuf][2 kh][128][128 B]
constexpr int oH = oA + kNBuf * 2 * kABuf;         // [128][32] bf16 (h_t of the block)
constexpr int oC = oH + kPRows * kPU * 2;          // [128][33] f32 cell state of the block
constexpr int oFlag = oC + kPRows * 33 * 4;        // abort flag
constexpr int kPLds = oFlag + 16;
static_assert(2 * 2 * kABuf >= 4 * 16 * 1024 && 2 * kABuf >= kPRows * 256, "exchange / Gx reuse the A buffers");
static_assert(kPLds <= 160 * 1024, "LDS budget");

__device__ __forceinline__ float psig(float x) { return __builtin_amdgcn_rcpf(1.f + __expf(-x)); }
__device__ __forceinline__ float ptanh(float x) { return 2.f * psig(2.f * x) - 1.f; }
__device__ __forceinline__ void vm_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
}  // namespace

__global__ __launch_bounds__(kPThreads, 1) void lstm_persist_kernel(PersistArgs p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // uniform: LDS-DMA targets go to M0
    const int ug = wave & 1, kh = wave >> 1;
    const int nteams = 2 * p.G;
    const int team = blockIdx.x % nteams, slice = blockIdx.x / nteams;
    const int cell = team & 1, group = team >> 1;
    const int u0 = slice * kPU;
    const int fr = lane & 15, fq = lane >> 4;
    int* cnt = p.sync + team * 16;                          // one 64-B line per team counter (<= 8 teams)
    int* err = p.sync + 8 * 16;
    int* sFlag = reinterpret_cast<int*>(smem + oFlag);
    if (tid == 0) *sFlag = 0;

    // ---- W_hh fragments of this wave: rows ((2 slice + ug) * 4 + q) * 16 + fr of the cell, K half kh
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
    // rows finished by this wave: row tiles 4 kh .. 4 kh + 3; lane: rows 16 rt + 4 fq + i, unit u0 + 16 ug + fr
    // (c of those rows in LDS: each lane reads / writes only its own words)
    float* sC = reinterpret_cast<float*>(smem + oC);
    const int jl = 16 * ug + fr;
#pragma unroll
    for (int rl = 0; rl < 4; ++rl)
#pragma unroll
        for (int i = 0; i < 4; ++i) sC[(16 * (4 * kh + rl) + 4 * fq + i) * 33 + jl] = 0.f;

    // y frame f: [B][CELLS][S][H] bf16, 8 KiB per stream; the team's rows start at stream b0 + 64 group
    const uint64_t yframe = (uint64_t)p.B * kPC * kPS * kPH;   // elements per frame
    const uint32_t yrow0 = (uint32_t)((size_t)(p.b0 + group * 64) * kPC * kPS * kPH * 2 + (size_t)cell * kPS * kPH * 2);
    const int nrows = min(kPRows, 2 * (p.nb - group * 64));   // valid rows of the team (<= 0: none)

    for (int t = 0; t < p.T; ++t) {
        // ---- Gx of frame t (128 rows x 256 B: 4 gates of the block's 32 units) by DMA into
        //      A buffer 0 once chunk 4 has been consumed (8 instructions per wave of 4 rows)
        const __amdgpu_buffer_rsrc_t rgx = make_rsrc(p.gx + (size_t)t * p.B * kPS * kPC * 4 * kPH,
                                                     (uint64_t)p.B * kPS * kPC * 4 * kPH * 2);
        // row r of the team = Gx row (2 (b0 + 64 group) + r) of the frame: 16 KiB apart
        const uint32_t gu = __builtin_amdgcn_readfirstlane(
            (uint32_t)(((size_t)2 * (p.b0 + group * 64) * kPC * 4 * kPH + (size_t)cell * 4 * kPH + (size_t)u0 * 4) * 2));
        auto issue_gx = [&]() {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int row = 4 * (8 * wave + i) + (lane >> 4);
                const uint32_t vo = (row < nrows && !(p.mode & 16)) ? (uint32_t)((lane >> 4) * 16384 + (lane & 15) * 16) : kOOB;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rgx, (__attribute__((address_space(3))) void*)(smem + oA + (8 * wave + i) * 1024), 16, vo,
                    (int)(gu + (uint32_t)(4 * (8 * wave + i)) * 16384u), 0, 0);
            }
        };
        // ---- wait for the team's h_{t-1} (32 arrivals per frame)
        if (t > 0 && !(p.mode & 4)) {
            if (tid == 0) {
                const int target = kPSlices * t;
                int n = 0;
                while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
                    __builtin_amdgcn_s_sleep(1);
                    if (++n > p.spin_limit) {
                        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                        *sFlag = 1;
                        break;
                    }
                }
            }
            __syncthreads();
            if (*sFlag) return;
        }
        // ---- gates = h_{t-1} W_hh^T over this wave's K half
        f32x4 acc[8][4];
#pragma unroll
        for (int rt = 0; rt < 8; ++rt)
#pragma unroll
            for (int q = 0; q < 4; ++q) acc[rt][q] = f32x4{0.f, 0.f, 0.f, 0.f};
        if (t > 0 && !(p.mode & 2)) {
            // h_{t-1} is y of frame t-1 (written once in this launch, read only after the
            // team's counter: no cache can hold an older copy of it).  Chunk j of half kh =
            // units 512 kh + 64 j .. +63 (128 B per row); this wave DMAs rows 64 ug .. 64 ug + 63
            // (8 instructions of 8 rows, sc1) into buffer j % kNBuf, 16-B slot s of row r
            // holding logical chunk s ^ ((r >> 1) & 7).  Row r = (stream r / 2, sequence r % 2):
            //   offset = yrow0 + (r >> 1) 8 KiB + (r & 1) 2 KiB + (512 kh + 64 j) 2 + 16 q
            const __amdgpu_buffer_rsrc_t ry = make_rsrc(p.y + (size_t)(t - 1) * yframe, yframe * 2);
            uint32_t vl[2];
#pragma unroll
            for (int par = 0; par < 2; ++par) {
                const int q = (lane & 7) ^ (((lane >> 4) + 4 * par) & 7);   // swz_slot<128>(64 ug + 8 i + lane / 8, .)
                vl[par] = (uint32_t)((32 * ug + (lane >> 4)) * 8192 + ((lane >> 3) & 1) * 2048 + 16 * q);
            }
            const int nvs = min(64, p.nb - group * 64);          // valid streams of the team
            auto issue = [&](int j) {
                char* buf = smem + oA + ((j % kNBuf) * 2 + kh) * kABuf + 64 * ug * 128;
                const uint32_t so = __builtin_amdgcn_readfirstlane(yrow0 + (uint32_t)(512 * kh + 64 * j) * 2);
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const int st = 32 * ug + 4 * i + (lane >> 4);  // stream of this lane's row
                    const uint32_t vo = (st < nvs && !(p.mode & 1)) ? vl[i & 1] : kOOB;
                    __builtin_amdgcn_raw_ptr_buffer_load_lds(
                        ry, (__attribute__((address_space(3))) void*)(buf + 8 * i * 128), 16, vo,
                        (int)(so + (uint32_t)i * 32768u), 0, CRN_PERSIST_AUX);
                }
            };
            static_assert(kNBuf == 4, "the vmcnt schedule below assumes 4 buffers");
#pragma unroll
            for (int j = 0; j < kNBuf - 1; ++j) issue(j);
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                // outstanding after chunk j: chunks j+1, j+2 (j <= 5), chunk 7 + Gx (j = 6), Gx (j = 7)
                if (j < 7) wait_vm<16>();
                else wait_vm<8>();
                __builtin_amdgcn_s_barrier();                  // chunk j landed (every wave's part)
                if (j + kNBuf - 1 < 8) issue(j + kNBuf - 1);   // into the buffer read at iteration j - 1
                if (j == 5) issue_gx();                        // buffer 0 (chunk 4) is free
                const char* base = smem + oA + ((j % kNBuf) * 2 + kh) * kABuf;
                // A fragment of step n = (ks2, rt) = (n / 8, n % 8); the MFMA asm is volatile, so the
                // compiler keeps every LDS read where it is written: read two steps ahead (a ring of
                // 3 fragments) so the read latency hides behind the previous steps' MFMAs
                auto read_af = [&](int n) {
                    const int r = 16 * (n & 7) + fr;
                    return *reinterpret_cast<const u32x4*>(base + r * 128 + swz_slot<128>(r, (n >> 3) * 4 + fq) * 16);
                };
                u32x4 afr[3];
                afr[0] = read_af(0);
                afr[1] = read_af(1);
#pragma unroll
                for (int n = 0; n < 16; ++n) {
                    const int ks2 = n >> 3, rt = n & 7;
                    if (n + 2 < 16) afr[(n + 2) % 3] = read_af(n + 2);
                    const u32x4 af = afr[n % 3];
                    // MFMA as inline asm so W_hh stays in AGPRs (operand "a"): with the builtin
                    // the allocator keeps W in arch VGPRs and spills it (256 W + 128 acc)
#ifndef CRN_PERSIST_ASM
#define CRN_PERSIST_ASM 1
#endif
#if !CRN_PERSIST_ASM
#pragma unroll
                    for (int q = 0; q < 4; ++q) mma_chunk(acc[rt][q], af, wreg[q][2 * j + ks2], bf16_t{});
#else
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        if (j == 0 && ks2 == 0)
                            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, 0"
                                         : "=v"(acc[rt][q]) : "v"(af), "a"(wreg[q][2 * j + ks2]));
                        else
                            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0"
                                         : "+v"(acc[rt][q]) : "v"(af), "a"(wreg[q][2 * j + ks2]));
                    }
#endif
                }
            }
            // the accumulators were written by inline-asm MFMAs, which the compiler's hazard
            // tracking does not see: wait states before any VALU / DS read of them
            asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory");
            wait_vm<0>();
            __syncthreads();                                   // Gx landed; A buffers 2, 3 free
        } else {
            issue_gx();
            wait_vm<0>();
            __syncthreads();
        }
        // ---- K halves meet, then the cell update.  The wave's K half picks which row tiles it
        //      sends / finishes; KH is a template constant so acc stays in registers (a runtime
        //      row-tile index would put the accumulators in scratch memory).
        bf16_t* sH = reinterpret_cast<bf16_t*>(smem + oH);
        auto finish = [&](auto khc) {
            constexpr int KH = decltype(khc)::value, OKH = 1 - KH;
            float4* xs = reinterpret_cast<float4*>(smem + oA + 2 * 2 * kABuf);   // [ug][dest kh][rt][q][lane]
#pragma unroll
            for (int rl = 0; rl < 4; ++rl)
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const f32x4 v = acc[4 * OKH + rl][q];
                    xs[(((ug * 2 + OKH) * 4 + rl) * 4 + q) * 64 + lane] = make_float4(v[0], v[1], v[2], v[3]);
                }
            __syncthreads();
            // one row tile at a time: partner's partial sums, then its 4 x 4 cell updates
#pragma unroll
            for (int rl = 0; rl < 4; ++rl) {
                asm volatile("" ::: "memory");                 // keep the tiles' LDS traffic apart
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const float4 v = xs[(((ug * 2 + KH) * 4 + rl) * 4 + q) * 64 + lane];
                    f32x4& a = acc[4 * KH + rl][q];
                    a = f32x4{a[0] + v.x, a[1] + v.y, a[2] + v.z, a[3] + v.w};
                }
                // cell update (gate order i, f, g, o) for rows 16 rt + 4 fq + i, unit jl
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int rt = 4 * KH + rl;
                    const int r = 16 * rt + 4 * fq + i;
                    const uint2 gv = *reinterpret_cast<const uint2*>(smem + oA + r * 256 + jl * 8);   // Gx row r
                    const float g0 = __uint_as_float(gv.x << 16), g1 = __uint_as_float(gv.x & 0xFFFF0000u);
                    const float g2 = __uint_as_float(gv.y << 16), g3 = __uint_as_float(gv.y & 0xFFFF0000u);
                    float* cp = sC + r * 33 + jl;
                    const f32x4& a0 = acc[4 * KH + rl][0];
                    const f32x4& a1 = acc[4 * KH + rl][1];
                    const f32x4& a2 = acc[4 * KH + rl][2];
                    const f32x4& a3 = acc[4 * KH + rl][3];
                    const float c = psig(a1[i] + g1) * *cp + psig(a0[i] + g0) * ptanh(a2[i] + g2);
                    *cp = c;
                    const float h = psig(a3[i] + g3) * ptanh(c);
                    sH[r * kPU + jl] = f2bf(h);
                }
            }
        };
        if (!(p.mode & 32)) {
            if (kh == 0) finish(std::integral_constant<int, 0>{});
            else finish(std::integral_constant<int, 1>{});
        }
        __syncthreads();
        // ---- publish h_t: y of frame t, sc1 (write-through) 16-B stores, 64 B per row
        {
            const __amdgpu_buffer_rsrc_t ry = make_rsrc(p.y + (size_t)t * yframe, yframe * 2);
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int piece = tid + kPThreads * i;        // 512 pieces: row r, 16-B quarter
                const int r = piece >> 2, qq = piece & 3;
                if (r < nrows && !(p.mode & 8)) {
                    const u32x4 v = *reinterpret_cast<const u32x4*>(smem + oH + r * kPU * 2 + qq * 16);
                    const uint32_t off = yrow0 + (uint32_t)((r >> 1) * 8192 + (r & 1) * 2048 + u0 * 2 + qq * 16);
                    __builtin_amdgcn_raw_buffer_store_b128(v, ry, off, 0, 16);   // sc1
                }
            }
            vm_drain();                                        // every storing wave: stores complete
            __syncthreads();
            if (tid == 0) __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

size_t persist_lds_bytes() { return kPLds; }

bool persist_supported(int H, int cells, int seqs, int num_cus) {
    return H == kPH && cells == kPC && seqs == kPS && num_cus >= 64;
}

hipError_t launch_lstm_persist(const PersistArgs& a, hipStream_t st) {
    if (a.nb <= 0 || a.T <= 0) return hipSuccess;
    if (a.G < 1 || a.G > 4 || 2 * a.nb > 128 * a.G) return hipErrorInvalidValue;
    static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(lstm_persist_kernel),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)kPLds);
    if (attr != hipSuccess) return attr;
    // Co-residency: one block per CU (LDS and registers), grid <= CUs (the caller chunks the
    // streams by the CU count).  A plain launch: hipLaunchCooperativeKernel gives the same
    // guarantee but its queue crashes rocprofv3 at process exit (AEC_CRN_PERSIST_COOP=1 selects it).
    static const int per_cu = [] {
        int n = 0;
        return hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(lstm_persist_kernel),
                                                            kPThreads, kPLds) == hipSuccess ? n : 0;
    }();
    if (per_cu < 1) return hipErrorCooperativeLaunchTooLarge;
    static const int coop = [] { const char* v = getenv("AEC_CRN_PERSIST_COOP"); return v ? atoi(v) : 0; }();
    if (!coop) {
        lstm_persist_kernel<<<dim3(64 * a.G), dim3(kPThreads), kPLds, st>>>(a);
        return hipGetLastError();
    }
    PersistArgs args = a;
    void* kargs[] = {&args};
    return hipLaunchCooperativeKernel(reinterpret_cast<const void*>(lstm_persist_kernel), dim3(64 * a.G),
                                      dim3(kPThreads), kargs, kPLds, st);
}

}  // namespace crn
