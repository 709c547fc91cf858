// crn_gemm.h — MFMA building blocks of the DCCRN path (internal).
//
// Every dense block of the reference's complex CRN is a
// GEMM whose operands are K-contiguous rows:
//   encoder ComplexConv2d (k=(5,1), s=(2,1))   dccrn.py:103-153
//   decoder ComplexConvTranspose2d (+skip)     dccrn.py:156-207, 386-395
//   LSTM input projection                      dccrn.py:423-450 / :514
//   LSTM recurrence W_hh h_{t-1}               (one launch per frame step)
// The conv kernels have time extent 1, so a conv over the frequency axis is
// an implicit GEMM over rows (frame, output bin) with k = (tap, in-channel)
// on channels-last [frame][bin][channel] maps (no im2col buffer).
//
// Element type T is float (exact f32 MFMA, v_mfma_f32_16x16x4_f32) or
// bf16 (v_mfma_f32_16x16x32_bf16, f32 accumulate).  Both read operand
// fragments as one 16-byte chunk per lane: lane l holds row (l & 15) of a
// 16-row fragment and the 16 bytes at byte offset 16 (l >> 4) of a 64-byte
// k-chunk.  For bf16 that is exactly the 16x16x32 operand map (k = 8 (l>>4)
// + j); for f32 the four elements feed four 16x16x4 steps with k = 4 (l>>4)
// + j, the same permutation on A and B, so the sum over the chunk's 16 k is
// unchanged.  Accumulator map (both): col = lane & 15, row = 4 (lane >> 4) + r.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace crn {

typedef uint16_t bf16_t;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <typename T> struct Elem;
template <> struct Elem<float> { static constexpr int kPer16 = 4; };
template <> struct Elem<bf16_t> { static constexpr int kPer16 = 8; };

__device__ __forceinline__ bf16_t f2bf(float f) { return __builtin_bit_cast(bf16_t, (__bf16)f); }
__device__ __forceinline__ float bf2f(bf16_t h) { return __uint_as_float((uint32_t)h << 16); }

template <typename T> __device__ __forceinline__ T to_elem(float v);
template <> __device__ __forceinline__ float to_elem<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16_t to_elem<bf16_t>(float v) { return f2bf(v); }
__device__ __forceinline__ float to_f32(float v) { return v; }
__device__ __forceinline__ float to_f32(bf16_t v) { return bf2f(v); }

// acc += A-chunk * B-chunk over one 64-byte k-chunk (see header)
__device__ __forceinline__ void mma_chunk(f32x4& acc, const u32x4& a, const u32x4& b, bf16_t) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), acc,
                                                 0, 0, 0);
}
__device__ __forceinline__ void mma_chunk(f32x4& acc, const u32x4& a, const u32x4& b, float) {
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[0]), __uint_as_float(b[0]), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[1]), __uint_as_float(b[1]), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[2]), __uint_as_float(b[2]), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[3]), __uint_as_float(b[3]), acc, 0, 0, 0);
}

// Output tile (mt, nt) of block `bid` in a 1-D grid of nbm x nbn tiles (a speed choice only: every
// tile is computed the same way wherever it runs).  gm == 0: row tiles in order, column tiles
// fastest.  gm > 0: blocks b, b + 8, ... are dealt to one XCD (MI355X_MICROARCH.md §Workgroup
// dispatch, observed placement); the bijective remap of cdna_hip_programming.md §5.5 T1 gives
// each such set a contiguous range of tile ids, so an XCD owns 1/8 of the rows and A is fetched
// into one L2 instead of all eight; inside that range gm row tiles are walked per column step,
// so the tiles an XCD runs together share gm A panels and 32 / gm B panels.
__device__ __forceinline__ void tile_order(int bid, int nwg, int nbm, int nbn, int gm, int64_t& mt, int& nt) {
    if (gm <= 0) {
        mt = bid / nbn;
        nt = bid % nbn;
        return;
    }
    const int q = nwg >> 3, r = nwg & 7, x = bid & 7;
    const int id = (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
    if (id >= nbm * nbn) {                          // a padded grid's spare blocks: rows past M
        mt = nbm;
        nt = 0;
        return;
    }
    const int per = gm * nbn;                       // tile ids per group of gm row tiles
    const int g = id / per, in = id - g * per;
    const int rows = min(gm, nbm - g * gm);
    mt = (int64_t)g * gm + in % rows;
    nt = in / rows;
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }
__device__ __forceinline__ float tanhf_(float x) {
    // tanh(x) = 1 - 2 / (exp(2x) + 1): saturates cleanly for |x| large
    return 1.f - 2.f / (__expf(2.f * x) + 1.f);
}

// the decoder's mask on one bin of the (mic or NLMS error) spectrum (dccrn2.py:189-210):
// shared by the batch and per-hop back kernels (crn_kernels.hip, crn_stream.hip)
template <int MODE>
__device__ __forceinline__ float2 apply_mask(float2 x, float2 mk) {
    if (MODE == 0) {   // 'E' (dccrn2.py:194-208): tanh(|M|) |X|_1e-8 * exp(i (arg X + arg M))
        const float mags = sqrtf(x.x * x.x + x.y * x.y + 1e-8f);
        const float ax = sqrtf(x.x * x.x + x.y * x.y);
        const float am = sqrtf(mk.x * mk.x + mk.y * mk.y);
        // atan2(0, 0) = 0 -> unit vector (1, 0)
        const float cx = ax > 0.f ? x.x / ax : 1.f, sx = ax > 0.f ? x.y / ax : 0.f;
        const float cm = am > 0.f ? mk.x / am : 1.f, sm = am > 0.f ? mk.y / am : 0.f;
        const float e = tanhf(am) * mags;
        return make_float2(e * (cx * cm - sx * sm), e * (sx * cm + cx * sm));
    } else if (MODE == 1) {   // 'C' (dccrn.py:575, dccrn2.py:209)
        return make_float2(x.x * mk.x - x.y * mk.y, x.x * mk.y + x.y * mk.x);
    } else {                  // 'R' (dccrn2.py:210-211)
        return make_float2(x.x * mk.x, x.y * mk.y);
    }
}

constexpr int kStageBytes = 128;   // K bytes staged per main-loop step (two 64-B k-chunks)
constexpr int kRowStride = 144;    // LDS bytes per staged row: 16 rows at one column hit 16 distinct 16-B bank slots

// Implicit-GEMM row source shared by the conv, LSTM-input and dense loaders:
//   row m -> (hi = m >> rshift, lo = m & (2^rshift - 1))
//   k     -> (tap = k >> kshift, ci = k & (2^kshift - 1))
//   element offset = hi*rs_hi + lo*rs_lo + tap*ks + ci + base_off
//   valid iff m < M, k < K and 0 <= lo*pmul + tap + padd < plim  (zero otherwise:
//   the conv's frequency padding and the K / M tails).
struct RowSrc {
    const void* src;
    int64_t M;
    int32_t K;
    int32_t rshift;
    int64_t rs_hi, rs_lo;
    int32_t kshift;
    int32_t pmul, padd, plim;
    int64_t ks, base_off;
    int64_t src_elems;          // elements of the source tensor (buffer range of the DMA path)
};

template <typename T>
__device__ __forceinline__ u32x4 rowsrc_load(const RowSrc& a, int64_t m, int kbyte) {
    constexpr int E = Elem<T>::kPer16;
    const int k = kbyte / (int)sizeof(T);
    const int64_t hi = m >> a.rshift;
    const int lo = (int)(m & ((1ll << a.rshift) - 1));
    const int tap = k >> a.kshift;
    const int ci = k & ((1 << a.kshift) - 1);
    const int pos = lo * a.pmul + tap + a.padd;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (m < a.M && k < a.K && pos >= 0 && pos < a.plim) {
        const T* p = reinterpret_cast<const T*>(a.src) + hi * a.rs_hi + (int64_t)lo * a.rs_lo + (int64_t)tap * a.ks +
                     ci + a.base_off;
        v = *reinterpret_cast<const u32x4*>(p);
    }
    (void)E;
    return v;
}

// Block-level main loop: acc[FM][FN] += A[wr0 + fm*16 + i][:] . B[wc0 + fn*16 + j][:]
// over `nstages` stages of 128 K-bytes.  A / B rows are fetched through the
// callables al(row, kbyte) / bl(row, kbyte) (block-relative rows) as 16-byte
// chunks, staged global -> registers -> LDS with the next stage's loads in
// flight during the current stage's MFMAs.  256 threads.
template <typename T, int BM, int BN, int FM, int FN, class AL, class BL>
__device__ __forceinline__ void gemm_core(f32x4 (&acc)[FM][FN], char* smem, const AL& al, const BL& bl, int nstages,
                                          int wr0, int wc0) {
    constexpr int NA = BM * 8, NB = BN * 8;                // 16-B chunks per stage
    constexpr int CA = (NA + 255) / 256, CB = (NB + 255) / 256;
    char* sA = smem;
    char* sB = smem + BM * kRowStride;
    const int tid = threadIdx.x, lane = tid & 63;
    u32x4 ra[CA], rb[CB];
    auto gload = [&](int st) {
#pragma unroll
        for (int i = 0; i < CA; ++i) {
            const int c = tid + 256 * i;
            if (NA % 256 == 0 || c < NA) ra[i] = al(c >> 3, st * kStageBytes + (c & 7) * 16);
        }
#pragma unroll
        for (int i = 0; i < CB; ++i) {
            const int c = tid + 256 * i;
            if (NB % 256 == 0 || c < NB) rb[i] = bl(c >> 3, st * kStageBytes + (c & 7) * 16);
        }
    };
    auto sstore = [&]() {
#pragma unroll
        for (int i = 0; i < CA; ++i) {
            const int c = tid + 256 * i;
            if (NA % 256 == 0 || c < NA) *reinterpret_cast<u32x4*>(sA + (c >> 3) * kRowStride + (c & 7) * 16) = ra[i];
        }
#pragma unroll
        for (int i = 0; i < CB; ++i) {
            const int c = tid + 256 * i;
            if (NB % 256 == 0 || c < NB) *reinterpret_cast<u32x4*>(sB + (c >> 3) * kRowStride + (c & 7) * 16) = rb[i];
        }
    };
    gload(0);
    sstore();
    __syncthreads();
    const int fr = lane & 15, fq = (lane >> 4) * 16;
    for (int st = 0; st < nstages; ++st) {
        const bool more = st + 1 < nstages;
        if (more) gload(st + 1);
#pragma unroll
        for (int kc = 0; kc < 2; ++kc) {
            u32x4 af[FM], bfr[FN];
#pragma unroll
            for (int fm = 0; fm < FM; ++fm)
                af[fm] = *reinterpret_cast<const u32x4*>(sA + (wr0 + fm * 16 + fr) * kRowStride + kc * 64 + fq);
#pragma unroll
            for (int fn = 0; fn < FN; ++fn)
                bfr[fn] = *reinterpret_cast<const u32x4*>(sB + (wc0 + fn * 16 + fr) * kRowStride + kc * 64 + fq);
#pragma unroll
            for (int fm = 0; fm < FM; ++fm)
#pragma unroll
                for (int fn = 0; fn < FN; ++fn) mma_chunk(acc[fm][fn], af[fm], bfr[fn], T{});
        }
        if (more) {
            __syncthreads();
            sstore();
            __syncthreads();
        }
    }
}


// --------------------------------------------------------------------------
// LDS-DMA main loop (buffer_load ... lds): no register staging, NBUF stage
// buffers, one barrier per stage, counted vmcnt.  Each stage is 128 K-bytes
// per row; LDS rows are 128 B, unpadded (the DMA writes 64 lanes x 16 B
// contiguously), with the 16-B chunk q of row r stored at slot
// q ^ ((r >> 1) & 7): the 16 rows of a fragment read then hit 16 distinct
// bank slots.  A lane of DMA instruction i fills row 8i + (lane >> 3), slot
// lane & 7, so it fetches logical chunk (lane & 7) ^ ((row >> 1) & 7).
// aoff(i, kbyte) / boff(i, kbyte): the lane's byte offset into ra / rb for
// its row of A / B instruction i (i < BM/(8 NW) resp. BN/(8 NW) per wave,
// rows 8 (NW i + wave) + lane/8, NW waves) at K-byte kbyte, or 0x80000000
// (out of range -> the hardware writes zeros).  BM, BN multiples of 8 NW.
// --------------------------------------------------------------------------
// 16-B slot of logical chunk q in LDS row `row`: 128-B rows use q ^ ((row >> 1) & 7),
// 64-B rows (4 rows per 256-B bank window) q ^ ((row >> 2) & 3): either way the 16
// rows of one fragment read land on 16 distinct bank slots.
template <int RB = 128>
__device__ __forceinline__ int swz_slot(int row, int q) {
    return RB == 128 ? (q ^ ((row >> 1) & 7)) : (q ^ ((row >> 2) & 3));
}

template <int N>
__device__ __forceinline__ void wait_vm() {
    static_assert(N >= 0 && N < 64, "vmcnt");
    // gfx9 s_waitcnt: vmcnt[3:0] | expcnt[6:4]=7 | lgkmcnt[11:8]=15 | vmcnt[5:4] << 14
    __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// RB = bytes of K per row per stage (128: two 64-B k-chunks; 64: one).  A DMA
// instruction writes 64 lanes x 16 B = 1 KiB = 1024 / RB rows.
// AUXA: cache policy bits of the A-operand DMA (2 = nt: streamed operand, keep L2 for B)
// Tail hook: at the first iteration that issues no further stage (st =
// nstages - NBUF + 1, after its barrier) the buffer of stage st - 1 is free
// for the rest of the loop; tail(buf) may issue HK DMA instructions per wave
// into it (the epilogue operands), which the remaining waits leave in flight.
struct NoTail {
    __device__ __forceinline__ void operator()(char*) const {}
};
template <typename T, int BM, int BN, int FM, int FN, int NBUF, class AO, class BO, int NW = 4, int RB = 128,
          int AUXA = 0, class TAIL = NoTail, int HK = 0>
__device__ __forceinline__ void gemm_core_dma(f32x4 (&acc)[FM][FN], char* smem, __amdgpu_buffer_rsrc_t ra,
                                              __amdgpu_buffer_rsrc_t rb, const AO& aoff, const BO& boff,
                                              int nstages, int wr0, int wc0, const TAIL& tail = TAIL{}) {
    constexpr int RPI = 1024 / RB;                       // rows per DMA instruction
    constexpr int CPR = RB / 16;                         // 16-B chunks per row
    static_assert(BM % (RPI * NW) == 0 && BN % (RPI * NW) == 0 && NBUF >= 2, "tile");
    constexpr int LA = BM / (RPI * NW), LB = BN / (RPI * NW);   // DMA instructions per wave per stage
    constexpr int STAGE = (BM + BN) * RB;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int q_l = lane & (CPR - 1);
    auto issue = [&](int st) {
        char* buf = smem + (st % NBUF) * STAGE;
#pragma unroll
        for (int i = 0; i < LA; ++i) {
            const int row = RPI * (NW * i + wave) + lane / CPR;
            const uint32_t vo = aoff(i, st * RB + swz_slot<RB>(row, q_l) * 16);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                ra, (__attribute__((address_space(3))) void*)(buf + RPI * (NW * i + wave) * RB), 16, vo, 0, 0, AUXA);
        }
#pragma unroll
        for (int i = 0; i < LB; ++i) {
            const int row = RPI * (NW * i + wave) + lane / CPR;
            const uint32_t vo = boff(i, st * RB + swz_slot<RB>(row, q_l) * 16);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rb, (__attribute__((address_space(3))) void*)(buf + BM * RB + RPI * (NW * i + wave) * RB), 16, vo, 0,
                0, 0);
        }
    };
#pragma unroll
    for (int s = 0; s < NBUF - 1; ++s)
        if (s < nstages) issue(s);
    const int fr = lane & 15, g = lane >> 4;
    const int st_tail = nstages - NBUF + 1;              // first iteration without a stage issue
    for (int st = 0; st < nstages; ++st) {
        if (st + NBUF - 2 < nstages)
            wait_vm<(NBUF - 2) * (LA + LB)>();
        else if (HK > 0 && st > st_tail)
            wait_vm<HK>();                                   // the tail DMAs stay in flight
        else
            wait_vm<0>();
        __builtin_amdgcn_s_barrier();
        if (st + NBUF - 1 < nstages) issue(st + NBUF - 1);
        if (HK > 0 && st == (st_tail > 0 ? st_tail : 0)) tail(smem + ((st + NBUF - 1) % NBUF) * STAGE);
        const char* sA = smem + (st % NBUF) * STAGE;
        const char* sB = sA + BM * RB;
#pragma unroll
        for (int kc = 0; kc < RB / 64; ++kc) {
            u32x4 af[FM], bfr[FN];
#pragma unroll
            for (int fm = 0; fm < FM; ++fm) {
                const int r = wr0 + fm * 16 + fr;
                af[fm] = *reinterpret_cast<const u32x4*>(sA + r * RB + swz_slot<RB>(r, kc * 4 + g) * 16);
            }
#pragma unroll
            for (int fn = 0; fn < FN; ++fn) {
                const int r = wc0 + fn * 16 + fr;
                bfr[fn] = *reinterpret_cast<const u32x4*>(sB + r * RB + swz_slot<RB>(r, kc * 4 + g) * 16);
            }
#pragma unroll
            for (int fm = 0; fm < FM; ++fm)
#pragma unroll
                for (int fn = 0; fn < FN; ++fn) mma_chunk(acc[fm][fn], af[fm], bfr[fn], T{});
        }
    }
}

// Software-pipelined form of gemm_core_dma for two 128-B stage buffers: a
// stage's fragments are read into registers one k-chunk ahead (set X = k-chunk
// 0, set Y = k-chunk 1), so a stage buffer is free once its second chunk is in
// registers. Iteration st:
//   read Y (stage st, chunk 1); MFMAs on X;
//   wait for this wave's DMAs and its LDS reads, barrier (stage st+1 landed
//   everywhere, nobody reads buffer st&1 again);
//   issue stage st+2 into buffer st&1; read X (stage st+1, chunk 0); MFMAs on Y.
// The LDS read latency and the DMA issue run under the other chunk's MFMAs
// instead of in front of them; the DMA still has one stage of MFMAs to land.
// Same MFMA order per accumulator as gemm_core_dma (bit-identical results).
// TRANS: the operands are swapped in every MFMA, so acc[fm][fn] holds the
// transposed 16x16 block (lane: row m = lane & 15, columns n = 4 (lane >> 4)
// + r): four adjacent output columns per lane (packed epilogue stores).
template <typename T, int BM, int BN, int FM, int FN, class AO, class BO, int NW = 8, bool TRANS = false>
__device__ __forceinline__ void gemm_core_dma_pipe(f32x4 (&acc)[FM][FN], char* smem, __amdgpu_buffer_rsrc_t ra,
                                                   __amdgpu_buffer_rsrc_t rb, const AO& aoff, const BO& boff,
                                                   int nstages, int wr0, int wc0) {
    constexpr int RB = 128, RPI = 8, CPR = 8;
    static_assert(BM % (RPI * NW) == 0 && BN % (RPI * NW) == 0, "tile");
    constexpr int LA = BM / (RPI * NW), LB = BN / (RPI * NW);
    constexpr int STAGE = (BM + BN) * RB;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int q_l = lane & (CPR - 1);
    // live = false: the same instructions with out-of-range offsets (the
    // hardware writes zeros, no memory traffic), so the loop body stays one
    // basic block the MFMAs can be interleaved with
    // offsets of stage st (computed ahead, in the MFMA phase before the barrier)
    auto offs = [&](int st, bool live, uint32_t(&vo)[LA + LB]) {
#pragma unroll
        for (int i = 0; i < LA; ++i) {
            const int row = RPI * (NW * i + wave) + lane / CPR;
            const uint32_t o = aoff(i, st * RB + swz_slot<RB>(row, q_l) * 16);
            vo[i] = live ? o : 0x80000000u;
        }
#pragma unroll
        for (int i = 0; i < LB; ++i) {
            const int row = RPI * (NW * i + wave) + lane / CPR;
            const uint32_t o = boff(i, st * RB + swz_slot<RB>(row, q_l) * 16);
            vo[LA + i] = live ? o : 0x80000000u;
        }
    };
    auto issue_at = [&](int st, const uint32_t(&vo)[LA + LB]) {
        char* buf = smem + (st & 1) * STAGE;
#pragma unroll
        for (int i = 0; i < LA; ++i)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                ra, (__attribute__((address_space(3))) void*)(buf + RPI * (NW * i + wave) * RB), 16, vo[i], 0, 0, 0);
#pragma unroll
        for (int i = 0; i < LB; ++i)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rb, (__attribute__((address_space(3))) void*)(buf + BM * RB + RPI * (NW * i + wave) * RB), 16,
                vo[LA + i], 0, 0, 0);
    };
    auto issue = [&](int st, bool live) {
        uint32_t vo[LA + LB];
        offs(st, live, vo);
        issue_at(st, vo);
    };
    const int fr = lane & 15, g = lane >> 4;
    auto rd = [&](int st, int kc, u32x4(&af)[FM], u32x4(&bf)[FN]) {
        const char* sA = smem + (st & 1) * STAGE;
        const char* sB = sA + BM * RB;
#pragma unroll
        for (int fm = 0; fm < FM; ++fm) {
            const int r = wr0 + fm * 16 + fr;
            af[fm] = *reinterpret_cast<const u32x4*>(sA + r * RB + swz_slot<RB>(r, kc * 4 + g) * 16);
        }
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
            const int r = wc0 + fn * 16 + fr;
            bf[fn] = *reinterpret_cast<const u32x4*>(sB + r * RB + swz_slot<RB>(r, kc * 4 + g) * 16);
        }
    };
    auto rda = [&](int st, int kc, int fm) -> u32x4 {
        const int r = wr0 + fm * 16 + fr;
        return *reinterpret_cast<const u32x4*>(smem + (st & 1) * STAGE + r * RB + swz_slot<RB>(r, kc * 4 + g) * 16);
    };
    auto rdb = [&](int st, int kc, u32x4(&bf)[FN]) {
        const char* sB = smem + (st & 1) * STAGE + BM * RB;
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
            const int r = wc0 + fn * 16 + fr;
            bf[fn] = *reinterpret_cast<const u32x4*>(sB + r * RB + swz_slot<RB>(r, kc * 4 + g) * 16);
        }
    };
    // MFMA row fm of one chunk, then the A fragment of the same row of the
    // next chunk into the registers that row just released
    u32x4 xa[FM], xb[FN], ya[FM], yb[FN];
    issue(0, true);
    wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    issue(1, nstages > 1);
    rd(0, 0, xa, xb);
    for (int st = 0; st < nstages; ++st) {
        uint32_t vo[LA + LB];
        offs(st + 2, st + 2 < nstages, vo);
        rdb(st, 1, yb);
#pragma unroll
        for (int fm = 0; fm < FM; ++fm) {
#pragma unroll
            for (int fn = 0; fn < FN; ++fn) {
                if constexpr (TRANS) mma_chunk(acc[fm][fn], xb[fn], xa[fm], T{});
                else mma_chunk(acc[fm][fn], xa[fm], xb[fn], T{});
            }
            ya[fm] = rda(st, 1, fm);
        }
        if constexpr (FM == 8 && FN == 4) {                 // row of MFMAs, then 2 / 1 LDS reads
#define CRN_G(n) __builtin_amdgcn_sched_group_barrier(0x008, 4, 0); __builtin_amdgcn_sched_group_barrier(0x100, n, 0);
            CRN_G(2) CRN_G(2) CRN_G(2) CRN_G(2) CRN_G(1) CRN_G(1) CRN_G(1) CRN_G(1)
#undef CRN_G
        }
        __builtin_amdgcn_sched_barrier(0);
        __builtin_amdgcn_s_waitcnt(0x0070);                 // vmcnt(0) expcnt(7) lgkmcnt(0)
        __builtin_amdgcn_s_barrier();
        __builtin_amdgcn_sched_barrier(0);
        issue_at(st + 2, vo);
        // (after the last stage these read a stale buffer; the values are unused)
        rdb(st + 1, 0, xb);
#pragma unroll
        for (int fm = 0; fm < FM; ++fm) {
#pragma unroll
            for (int fn = 0; fn < FN; ++fn) {
                if constexpr (TRANS) mma_chunk(acc[fm][fn], yb[fn], ya[fm], T{});
                else mma_chunk(acc[fm][fn], ya[fm], yb[fn], T{});
            }
            xa[fm] = rda(st + 1, 0, fm);
        }
        if constexpr (FM == 8 && FN == 4) {                 // row of MFMAs, LDS reads, one DMA
#define CRN_G(n)                                                                                   \
    __builtin_amdgcn_sched_group_barrier(0x008, 4, 0); __builtin_amdgcn_sched_group_barrier(0x100, n, 0); \
    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
            CRN_G(2) CRN_G(2) CRN_G(2) CRN_G(2) CRN_G(1) CRN_G(1) CRN_G(1) CRN_G(1)
#undef CRN_G
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    wait_vm<0>();                                          // the trailing (empty) DMAs, before the epilogue reuses LDS
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint64_t bytes) {
    const uint32_t nr = bytes > 0x7FFFFFF0ull ? 0x7FFFFFF0u : (uint32_t)bytes;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)nr, 0x00020000);
}

constexpr uint32_t kOOB = 0x80000000u;

// --------------------------------------------------------------------------
// MX-fp8 main loop: OCP e4m3 operands with an E8M0 scale per 32 k of every
// row, v_mfma_scale_f32_16x16x128_f8f6f4 (2x the bf16 MFMA rate per clock).
// Operand map, measured on gfx950 (tools/probes/mx8_probe.hip, one-hot
// probes over all 2048 lane/byte slots): lane l = (g = l >> 4, r = l & 15)
// holds row r's bytes [16g, 16g+16) in operand regs 0-3 and [64+16g,
// 64+16g+16) in regs 4-7, and its scale operand is the E8M0 of (row r,
// k-block [32g, 32g+32)); C/D as the bf16 16x16 form.  So a 128-byte K stage
// staged exactly as in gemm_core_dma feeds ONE MX MFMA per fragment pair from
// the two 16-B chunks the bf16 loop reads (slots g and 4+g).
// Stage layout: [A BM x 128 B][B BN x 128 B][A scales BM x 4 B][B scales BN x
// 4 B]; a stage's scales (bytes 4 st .. 4 st+3 of every row's scale row) come
// by one 4-byte DMA per lane: wave w, lane l fetches row 64 w + l of [A | B]
// (BM + BN == 64 NW), so every wave issues LA + LB + 1 DMAs per stage.
// rs / soff(st): the wave's scale descriptor (A or B, wave-uniform) and the
// lane's byte offset of its row's 4 scale bytes of stage st (kOOB: zero
// scales: the row, or the conv tap, is out of range).
// --------------------------------------------------------------------------
typedef int i32x8 __attribute__((ext_vector_type(8)));

template <int BM, int BN, int FM, int FN, int NBUF, class AO, class BO, int NW, class SO>
__device__ __forceinline__ void gemm_core_mx8(f32x4 (&acc)[FM][FN], char* smem, __amdgpu_buffer_rsrc_t ra,
                                              __amdgpu_buffer_rsrc_t rb, __amdgpu_buffer_rsrc_t rs, const AO& aoff,
                                              const BO& boff, const SO& soff, int nstages, int wr0, int wc0) {
    constexpr int RB = 128, RPI = 8;
    static_assert(BM % (RPI * NW) == 0 && BN % (RPI * NW) == 0 && NBUF >= 2 && BM + BN == 64 * NW, "tile");
    constexpr int LA = BM / (RPI * NW), LB = BN / (RPI * NW);
    constexpr int STAGE = (BM + BN) * (RB + 4);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int q_l = lane & 7;
    auto issue = [&](int st) {
        char* buf = smem + (st % NBUF) * STAGE;
#pragma unroll
        for (int i = 0; i < LA; ++i) {
            const int row = RPI * (NW * i + wave) + lane / 8;
            const uint32_t vo = aoff(i, st * RB + swz_slot<RB>(row, q_l) * 16);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                ra, (__attribute__((address_space(3))) void*)(buf + RPI * (NW * i + wave) * RB), 16, vo, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < LB; ++i) {
            const int row = RPI * (NW * i + wave) + lane / 8;
            const uint32_t vo = boff(i, st * RB + swz_slot<RB>(row, q_l) * 16);
            __builtin_amdgcn_raw_ptr_buffer_load_lds(
                rb, (__attribute__((address_space(3))) void*)(buf + BM * RB + RPI * (NW * i + wave) * RB), 16, vo, 0,
                0, 0);
        }
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            rs, (__attribute__((address_space(3))) void*)(buf + (BM + BN) * RB + wave * 256), 4, soff(st), 0, 0, 0);
    };
#pragma unroll
    for (int s = 0; s < NBUF - 1; ++s)
        if (s < nstages) issue(s);
    const int fr = lane & 15, g = lane >> 4;
    for (int st = 0; st < nstages; ++st) {
        if (st + NBUF - 2 < nstages)
            wait_vm<(NBUF - 2) * (LA + LB + 1)>();
        else
            wait_vm<0>();
        __builtin_amdgcn_s_barrier();
        if (st + NBUF - 1 < nstages) issue(st + NBUF - 1);
        const char* sA = smem + (st % NBUF) * STAGE;
        const char* sB = sA + BM * RB;
        const uint32_t* sS = reinterpret_cast<const uint32_t*>(sA + (BM + BN) * RB);
        i32x8 bfr[FN];
        int sb[FN];
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
            const int r = wc0 + fn * 16 + fr;
            const u32x4 lo = *reinterpret_cast<const u32x4*>(sB + r * RB + swz_slot<RB>(r, g) * 16);
            const u32x4 hi = *reinterpret_cast<const u32x4*>(sB + r * RB + swz_slot<RB>(r, 4 + g) * 16);
            bfr[fn] = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1], (int)hi[2],
                            (int)hi[3]};
            sb[fn] = (int)((sS[BM + r] >> (8 * g)) & 0xFFu);
        }
#pragma unroll
        for (int fm = 0; fm < FM; ++fm) {
            const int r = wr0 + fm * 16 + fr;
            const u32x4 lo = *reinterpret_cast<const u32x4*>(sA + r * RB + swz_slot<RB>(r, g) * 16);
            const u32x4 hi = *reinterpret_cast<const u32x4*>(sA + r * RB + swz_slot<RB>(r, 4 + g) * 16);
            const i32x8 af = i32x8{(int)lo[0], (int)lo[1], (int)lo[2], (int)lo[3], (int)hi[0], (int)hi[1],
                                   (int)hi[2], (int)hi[3]};
            const int sa = (int)((sS[r] >> (8 * g)) & 0xFFu);
#pragma unroll
            for (int fn = 0; fn < FN; ++fn)
                acc[fm][fn] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(af, bfr[fn], acc[fm][fn], 0, 0, 0, sa,
                                                                               0, sb[fn]);
        }
    }
}

// MX-fp8 shadow of one 16-B output chunk (8 bf16, columns n .. n+7) whose
// 32-column group's 4 chunks sit in lanes 4j .. 4j+3: the group's E8M0 scale
// (amax over the 4 lanes) and the chunk's 8 e4m3 bytes, by mx8_quant_kernel's
// rule on the same bf16 values (so an MX GEMM reading the shadow in place sees
// the bytes the separate quantisation pass would have written).  ok: the
// chunk is a real output (its bytes / scale are stored); every lane of the
// wave must call it (cross-lane reduction).
__device__ __forceinline__ void mx8_chunk(const u32x4& v, bool ok, uint8_t* q8, uint8_t* qs, int64_t eo, bool lead) {
    float x[8];
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        x[2 * i] = __uint_as_float(v[i] << 16);
        x[2 * i + 1] = __uint_as_float(v[i] & 0xFFFF0000u);
        amax = fmaxf(amax, fmaxf(fabsf(x[2 * i]), fabsf(x[2 * i + 1])));
    }
    if (!ok) amax = 0.f;
    amax = fmaxf(amax, __shfl_xor(amax, 1));
    amax = fmaxf(amax, __shfl_xor(amax, 2));
    const int ebits = (int)((__float_as_uint(amax) >> 23) & 0xFF);     // floor(log2 amax) + 127
    const int code = ebits > 8 ? ebits - 8 : 0;                          // E8M0: 2^(code - 127)
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
    if (ok) {
        *reinterpret_cast<uint2*>(q8 + eo) = make_uint2(pk[0], pk[1]);
        if (lead) qs[eo >> 5] = (uint8_t)code;
    }
}

}  // namespace crn
