// aec_stream.hip — the fused per-hop streaming step of the Stage-2 path on
// gfx950: ONE launch per 256-sample hop for B concurrent streams runs
//
//   frame (prev hop | hop) -> Hann -> rFFT-512 (mic, ref)        attention_ccrn.py:45-52
//   -> [FD-NLMS: E = M - sum_l W_l R_{t-l}, W update]            build-defined
//   -> |E|, |R| -> ERB (mic_erb, ref_erb) -> x = [mic, |mic-ref|]  ERB.py:277-290
//   -> one GRU step, head, mask -> est_erb                        ERB.py:293-304
//   -> gains -> irFFT-512 -> Hann -> overlap-add / WOLA -> +1e-9   ERB.py:306-316, attention_ccrn.py:82-101
//
// and emits output hop k-1 (the OLA of frames k-1 and k).  This is the
// reference's per-frame loop (Little_net.forward, ERB.py:252-334) cut at the
// frame boundary: nothing in it looks ahead, so a streamed utterance equals
// the batch result (aec_process) given the same input samples.  The
// normaliser x - mean(x)/std(x) (ERB.py:254-256) is an utterance-global
// statistic a stream cannot know: the caller passes the hops already
// normalised (or raw; serving callers use their own offset).
//
// One block of 4 waves per stream; per-stream state lives in HBM between
// calls (prev hop, NLMS taps / far-end history / power, GRU h, OLA tail) and
// is read once and written once per hop.  The arithmetic is the batch path's
// own (the aec_frame.h helpers, GRU step and head included), so a streamed
// utterance reproduces aec_process bit for bit (tests/test_gpu_stream.py).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "aec_fft.h"
#include "aec_frame.h"
#include "aec_launch.h"
#include "aec_stft.h"
#include "aec_tables.h"

namespace aec {

constexpr int kStreamThreads = 256;
constexpr int kSchedMax = 48;                 // ErbTables: L <= 48

template <int TAPS>
__global__ __launch_bounds__(kStreamThreads) void stream_step_kernel(StreamStepArgs p) {
    __shared__ __attribute__((aligned(16))) float4 sSched[kSchedMax * 16];
    __shared__ int2 sComb[32];
    __shared__ __attribute__((aligned(16))) float2 sTw512[258];
    __shared__ __attribute__((aligned(16))) float2 sTwT[256];
    __shared__ __attribute__((aligned(16))) float sHann[512];
    __shared__ __attribute__((aligned(16))) float sCoff[256];
    __shared__ __attribute__((aligned(16))) float4 sBin[257];
    __shared__ __attribute__((aligned(16))) float sStg[2][kHopStride + kHop];   // prev hop at 0, hop at 288
    __shared__ __attribute__((aligned(16))) float sScr[2][kGroupFloats];
    __shared__ __attribute__((aligned(16))) float2 sRow[3][256];                  // M, R, E rows
    __shared__ __attribute__((aligned(16))) float sMicErb[32];
    __shared__ __attribute__((aligned(16))) float sRefErb[32];
    __shared__ __attribute__((aligned(16))) float sX[64];
    __shared__ __attribute__((aligned(16))) float sGi[96];
    __shared__ __attribute__((aligned(16))) float sH[32];
    __shared__ __attribute__((aligned(16))) float sHn[32];
    __shared__ __attribute__((aligned(16))) float sO[32];
    __shared__ __attribute__((aligned(16))) float sEst[32];

    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const int gg = lane >> 4, lb = lane & 15, sw = 16 * (gg & 1);
    const int b = blockIdx.x;
    const int L = p.sched_len;
    float* st = p.state + (int64_t)b * p.state_stride;
    const float* mic = p.mic + (int64_t)b * p.ld_in;
    const float* ref = p.ref + (int64_t)b * p.ld_in;

    const float* W_ih = p.w;                  // [96][64]  (state_dict order, aec_hip.h)
    const float* W_hh = p.w + 96 * 64;        // [96][32]
    const float* b_ih = W_hh + 96 * 32;       // [96]
    const float* b_hh = b_ih + 96;            // [96]
    const float* W1 = b_hh + 96;              // [32][64]
    const float* b1 = W1 + 32 * 64;           // [32]
    const float* W2 = b1 + 32;                // [32][32]
    const float* b2 = W2 + 32 * 32;           // [32]

    // ---- P0: tables, hops, state, role weights --------------------------
    const DevTables* tb = reinterpret_cast<const DevTables*>(p.tables);
    {
        sTwT[tid] = tb->twT[tid];
        sTw512[tid] = tb->tw512[tid];
        if (tid < 2) sTw512[256 + tid] = tb->tw512[256 + tid];
        sHann[tid] = tb->hann[tid];
        sHann[tid + 256] = tb->hann[tid + 256];
        sCoff[tid] = tb->inv_coff[tid];
        const float4* bt = reinterpret_cast<const float4*>(p.bintab);
        sBin[tid] = bt[tid];
        if (tid == 0) sBin[256] = bt[256];
        const float4* sch = reinterpret_cast<const float4*>(p.sched);
        for (int i = tid; i < L * 16; i += kStreamThreads) sSched[i] = sch[i];
        if (tid < 32) sComb[tid] = reinterpret_cast<const int2*>(p.sched + 4 * 16 * L)[tid];
    }
    {
        float* prev = st + kStPrev;
        const float pm = prev[tid], pr = prev[256 + tid];
        const float cm = mic[tid], cr = ref[tid];
        sStg[0][tid] = pm;
        sStg[0][kHopStride + tid] = cm;
        sStg[1][tid] = pr;
        sStg[1][kHopStride + tid] = cr;
        prev[tid] = cm;                       // this hop is the next frame's first half
        prev[256 + tid] = cr;
        if (tid < 32) sH[tid] = st[kStH + tid];
    }
    const float tail = st[kStTail + tid];

    // NLMS bin slot k = tid (slot 0: the real pair (0, 256)); taps, power and
    // the raw far-end history r[t-1 .. t-TAPS+1] from the state
    NlmsBin<TAPS ? TAPS : 1> nb;
    float2 rh[TAPS > 1 ? TAPS - 1 : 1];
    float2* nst = reinterpret_cast<float2*>(st + kStNlms);
    if constexpr (TAPS > 0) {
        nb.reset(tid == 0);
#pragma unroll
        for (int l = 0; l < TAPS; ++l) {
            const float2 w = nst[l * 256 + tid];
            nb.w[l] = w;
        }
#pragma unroll
        for (int l = 0; l + 1 < TAPS; ++l) {
            // the operands step() derived from r when r entered (same expressions)
            const float2 r2 = nst[(TAPS + l) * 256 + tid];
            rh[l] = r2;
            nb.hist(l, r2);
        }
        const float2 pp = nst[(2 * TAPS - 1) * 256 + tid];
        nb.p = pp;
    }

    // role weights: wave 0 the recurrence (W_hh k-halves, as gru_kernel's
    // wave 0), threads 64..159 the input projection rows, wave 3 the head
    const int j = lane & 31, kh = lane >> 5;
    f2v wrz[16], wn[8];
    float bhn = 0.f;
    float wih[64];
    float gbias = 0.f;
    const int grow = tid - 64;
    float w1[64], w2[32];
    float b1j = 0.f, b2j = 0.f;
    if (wave == 0) {
        const float* rR = W_hh + j * 32 + 16 * kh;
        const float* rZ = W_hh + (32 + j) * 32 + 16 * kh;
        const float* rN = W_hh + (64 + j) * 32 + 16 * kh;
#pragma unroll
        for (int k = 0; k < 16; ++k) wrz[k] = f2v{rR[k], rZ[k]};
#pragma unroll
        for (int i = 0; i < 8; ++i) wn[i] = f2v{rN[2 * i], rN[2 * i + 1]};
        bhn = b_hh[64 + j];
    } else if (grow < 96) {
#pragma unroll
        for (int k = 0; k < 64; ++k) wih[k] = W_ih[grow * 64 + k];
        gbias = b_ih[grow] + (grow < 64 ? b_hh[grow] : 0.f);
    } else if (wave == 3 && lane < 32) {
#pragma unroll
        for (int k = 0; k < 64; ++k) w1[k] = W1[lane * 64 + k];
#pragma unroll
        for (int k = 0; k < 32; ++k) w2[k] = W2[lane * 32 + k];
        b1j = b1[lane];
        b2j = b2[lane];
    }
    __syncthreads();

    // ---- P1: wave 0, group 0 = mic, group 1 = ref: window + rFFT + ERB ----
    float2 xa[8], xb[8], x128;
    if (wave == 0 && gg < 2) {
        float2 v[16];
        load_frame(v, sStg[gg], sHann, 0, lb);
        wave_fence();
        fft256<false>(v, lb, sScr[gg], sTwT);
        rfft_unpack(v, lb, sTw512, xa, xb, x128);
        row_to_scr(reinterpret_cast<float*>(sRow[gg]), lb, xa, xb, x128);
        mags_to_scr(sScr[gg], lb, sw, xa, xb, x128);
        wave_fence();
        // ref_erb; mic_erb here is the bypass value (|M|), replaced by |E| below
        erb_project(sScr[gg], sSched, sComb, L, lb, sw, gg ? sRefErb : sMicErb);
    }
    __syncthreads();

    // ---- P2: NLMS step of every bin (E row) ----
    if constexpr (TAPS > 0) {
        const float2 e = nb.step(sRow[0][tid], sRow[1][tid], p.mu, p.beta, p.delta);
        sRow[2][tid] = e;
#pragma unroll
        for (int l = 0; l < TAPS; ++l) nst[l * 256 + tid] = nb.w[l];
        if constexpr (TAPS > 1) {
            nst[TAPS * 256 + tid] = sRow[1][tid];
#pragma unroll
            for (int l = 1; l + 1 < TAPS; ++l) nst[(TAPS + l) * 256 + tid] = rh[l - 1];
        }
        nst[(2 * TAPS - 1) * 256 + tid] = nb.p;
        __syncthreads();
    }

    // ---- P3: mic_erb from |E| (group 0 keeps E's pairs for the synthesis); x ----
    if (wave == 0 && gg == 0) {
        if constexpr (TAPS > 0) {
            row_to_pairs(sRow[2], lb, true, xa, xb, x128);
            wave_fence();
            mags_to_scr(sScr[0], lb, 0, xa, xb, x128);
            wave_fence();
            erb_project(sScr[0], sSched, sComb, L, lb, 0, sMicErb);
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int band = lb + 16 * h;
            const float m = sMicErb[band];
            sX[band] = m;
            sX[32 + band] = fabsf(m - sRefErb[band]);
        }
    }
    __syncthreads();

    // ---- P4: gi = W_ih x + b_ih (+ b_hh for r, z) — gru_kernel's helper order ----
    if (wave != 0 && grow < 96) {
        sGi[grow] = gru_gi(wih, sX, gbias);
    }
    __syncthreads();

    // ---- P5: the GRU step (gru_kernel wave 0, one frame) ----
    if (wave == 0) {
        const float hj = gru_step(wrz, wn, sH, kh, sGi[j], sGi[32 + j], sGi[64 + j], bhn, sH[j]);
        if (kh == 0) {
            sHn[j] = hj;
            st[kStH + j] = hj;
        }
    }
    __syncthreads();

    // ---- P6: head (linear1 / relu / linear2 / sigmoid) -> est_erb (gru_kernel order) ----
    if (wave == 3 && lane < 32) {
        const float mask = head_mask(w1, w2, b1j, b2j, sHn, sMicErb, sO, lane);
        sEst[lane] = mask * sMicErb[lane];
    }
    __syncthreads();

    // ---- P7: gains -> irFFT -> window (group 0 of wave 0 holds the spectrum) ----
    if (wave == 0 && gg == 0) synth_frame(xa, xb, x128, sEst, sBin, sTw512, sTwT, sHann, sScr[0], lb);
    __syncthreads();

    // ---- P8: overlap-add with the previous frame's tail, WOLA, +1e-9 ----
    const float c = sScr[0][tid];
    p.out[(int64_t)b * p.ld_out + tid] = (tail + c) * sCoff[tid] + 1e-9f;
    st[kStTail + tid] = sScr[0][256 + tid];
}

hipError_t launch_stream_step(const StreamStepArgs& a, int B, int taps, hipStream_t s) {
    if (B <= 0) return hipSuccess;
    if (a.sched_len > kSchedMax) return hipErrorInvalidValue;
    switch (taps) {
#define AEC_STREAM_CASE(T) \
        case T: hipLaunchKernelGGL(stream_step_kernel<T>, dim3(B), dim3(kStreamThreads), 0, s, a); break;
        AEC_STREAM_CASE(0) AEC_STREAM_CASE(1) AEC_STREAM_CASE(2) AEC_STREAM_CASE(3) AEC_STREAM_CASE(4)
        AEC_STREAM_CASE(5) AEC_STREAM_CASE(6) AEC_STREAM_CASE(7) AEC_STREAM_CASE(8)
#undef AEC_STREAM_CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace aec
