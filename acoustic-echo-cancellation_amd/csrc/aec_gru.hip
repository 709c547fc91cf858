// aec_gru.hip — the recurrent part of the Stage-2 post-filter on gfx950.
//
// Reference: nn.GRU(64, 32) + linear1/relu + linear2/sigmoid + mask
// (Stage2_lhm/scripts/network/ERB.py:213-217, 287-304) and the loss (:318-323).
//
// One block per stream, 7 waves:
//   wave 0      the recurrence h_{t-1} -> h_t (the only sequential dependency
//               of the whole path), one step per frame, raised issue priority,
//               k-split over the two wave halves (24 packed FMAs per lane);
//   waves 1..6  helpers, software-pipelined around it in ticks of kCH frames:
//               at tick c they stage chunk c+2's features (loaded from HBM at
//               tick c-1, so no load latency is exposed), issue the loads of
//               chunk c+3, compute gi = W_ih x + b for chunk c+1 and run the
//               head (linear1/relu/linear2/sigmoid, est_erb, loss) for chunk c-1.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "aec_fft.h"
#include "aec_frame.h"
#include "aec_launch.h"

namespace aec {

constexpr int kGruHelpers = 6;
constexpr int kGruThreads = 64 * (1 + kGruHelpers);
constexpr int kHL = 64 * kGruHelpers;                 // helper lanes (384)
constexpr int kHeadGroups = kHL / 32;                 // 12 (j, frame-group) groups of 32 lanes

__global__ __launch_bounds__(kGruThreads) void gru_kernel(GruArgs p) {
    __shared__ __attribute__((aligned(16))) float sX[2][kCH][64];
    __shared__ __attribute__((aligned(16))) float sGi[2][kCH][96];
    __shared__ __attribute__((aligned(16))) float sH[2][kCH][32];
    __shared__ __attribute__((aligned(16))) float sMic[4][kCH][32];
    __shared__ __attribute__((aligned(16))) float sNear[4][kCH][32];
    __shared__ __attribute__((aligned(16))) float sO[kHeadGroups][32];
    __shared__ float sLoss[1 + kGruHelpers];
    __shared__ __attribute__((aligned(16))) float sHb[32];   // h_{t-1} broadcast slot (recurrence wave)

    const int b = p.b0 + blockIdx.x;
    const int64_t n = p.lens[b];
    const int T = (int)(n / kHop + 1);
    const int nch = (T + kCH - 1) / kCH;
    const int tid = threadIdx.x;
    const int wave = tid >> 6, lane = tid & 63;
    const float* W_ih = p.w;                  // [96][64]
    const float* W_hh = p.w + 96 * 64;        // [96][32]
    const float* b_ih = W_hh + 96 * 32;       // [96]
    const float* b_hh = b_ih + 96;            // [96]
    const float* W1 = b_hh + 96;              // [32][64]
    const float* b1 = W1 + 32 * 64;           // [32]
    const float* W2 = b1 + 32;                // [32][32]
    const float* b2 = W2 + 32 * 32;           // [32]
    const float* fb = p.feats + (int64_t)b * p.Tmax * 96;

    if (wave == 0) {
        // ---------------- recurrence wave ----------------
        // lane l: j = l & 31, kh = l >> 5.  Each lane holds rows r_j, z_j, n_j of
        // W_hh restricted to its k-half [16 kh, 16 kh + 16): 24 packed FMAs per
        // step instead of 32 full-length (r|z, n) dots, and no row computed
        // twice.  h_{t-1} is broadcast through a 32-float LDS slot (one write,
        // four b128 reads of the lane's half) and the two halves' partial dots
        // are combined with v_permlane32_swap; h_j ends up identical in both
        // halves.
        __builtin_amdgcn_s_setprio(3);
        const bool run = p.mode != 2;
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
        float hj = 0.f;                                   // h_{-1} = 0
        float* hb = sHb;
        if (lane < 32) hb[lane] = 0.f;
        for (int c = -3; c <= nch; ++c) {
            if (run && c >= 0 && c < nch) {
                const int f_end = min(kCH, T - c * kCH);
                const float* gi = &sGi[c & 1][0][0];
                float gr = gi[j], gz = gi[32 + j], gn = gi[64 + j];
                for (int f = 0; f < f_end; ++f) {
                    // prefetch next step's input projections (independent of h)
                    const int fn = f + 1 < f_end ? f + 1 : f;
                    const float ngr = gi[fn * 96 + j], ngz = gi[fn * 96 + 32 + j], ngn = gi[fn * 96 + 64 + j];
                    // h_{t-1}[16 kh .. 16 kh + 15] (LDS ops of one wave execute in order;
                    // measured faster than a permlane16_swap + 16 DPP row_newbcast
                    // broadcast: 0.177 vs 0.197 ms recurrence-only)
                    hj = gru_step(wrz, wn, hb, kh, gr, gz, gn, bhn, hj);
                    if (kh == 0) {
                        hb[j] = hj;                            // broadcast slot for the next step
                        sH[c & 1][f][j] = hj;                  // for the head (off the chain)
                    }
                    gr = ngr; gz = ngz; gn = ngn;
                }
            }
            __syncthreads();
        }
    } else {
        // ---------------- helper waves ----------------
        const bool run = p.mode != 1;
        const int hl = tid - 64;                       // 0..383
        // gi role: row = hl % 96, frames f = fq, fq+4, fq+8, fq+12
        const int grow = hl % 96, fq = hl / 96;
        float wih[64];
#pragma unroll
        for (int k = 0; k < 64; ++k) wih[k] = W_ih[grow * 64 + k];
        const float gbias = b_ih[grow] + (grow < 64 ? b_hh[grow] : 0.f);
        // head role: j = hl & 31, frames f = fg, fg + 12
        const int hj_ = hl & 31, fg = hl >> 5;
        float w1[64], w2[32];
#pragma unroll
        for (int k = 0; k < 64; ++k) w1[k] = W1[hj_ * 64 + k];
#pragma unroll
        for (int k = 0; k < 32; ++k) w2[k] = W2[hj_ * 32 + k];
        const float b1j = b1[hj_], b2j = b2[hj_];
        float lacc = 0.f;
        // feature prefetch registers: elements e = hl and hl + kHL of a chunk's
        // [16 frames][32 bands] tile (mic, ref, near)
        float pm[2] = {0.f, 0.f}, pr[2] = {0.f, 0.f}, pn[2] = {0.f, 0.f};
        auto load_chunk = [&](int cc) {
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int e = hl + u * kHL;
                const int t = cc * kCH + (e >> 5);
                const bool ok = e < kCH * 32 && t < T;
                const float* f = fb + (int64_t)t * 96 + (e & 31);
                pm[u] = ok ? f[0] : 0.f;
                pr[u] = ok ? f[32] : 0.f;
                pn[u] = ok && p.has_near ? f[64] : 0.f;
            }
        };

        for (int c = -3; c <= nch; ++c) {
            if (run) {
                // (a) stage chunk c+2 (loaded at tick c-1) and load chunk c+3
                const int cs = c + 2;
                if (cs >= 0 && cs < nch) {
#pragma unroll
                    for (int u = 0; u < 2; ++u) {
                        const int e = hl + u * kHL;
                        if (e < kCH * 32) {
                            const int f = e >> 5, jj = e & 31;
                            sX[cs & 1][f][jj] = pm[u];
                            sX[cs & 1][f][32 + jj] = fabsf(pm[u] - pr[u]);
                            sMic[cs & 3][f][jj] = pm[u];
                            sNear[cs & 3][f][jj] = pn[u];
                        }
                    }
                }
                if (c + 3 < nch) load_chunk(c + 3);
                // (b) gi for chunk c+1
                const int cg = c + 1;
                if (cg >= 0 && cg < nch) {
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        const int f = fq + 4 * i;
                        sGi[cg & 1][f][grow] = gru_gi(wih, &sX[cg & 1][f][0], gbias);
                    }
                }
                // (c) head for chunk c-1
                const int ch = c - 1;
                if (ch >= 0 && ch < nch) {
                    for (int f = fg; f < kCH; f += kHeadGroups) {
                        const int t = ch * kCH + f;
                        if (t >= T) break;               // uniform within the 32-lane group
                        const float mask = head_mask(w1, w2, b1j, b2j, &sH[ch & 1][f][0], &sMic[ch & 3][f][0], &sO[fg][0], hj_);
                        const float me = sMic[ch & 3][f][hj_];
                        const float est = mask * me;
                        const int64_t o_idx = ((int64_t)b * p.Tmax + t) * 32 + hj_;
                        p.est[o_idx] = est;
                        if (p.dbg_h) p.dbg_h[o_idx] = sH[ch & 1][f][hj_];
                        if (p.dbg_mask) p.dbg_mask[o_idx] = mask;
                        if (p.has_near) {
                            const float d = sqrtf(sNear[ch & 3][f][hj_]) - sqrtf(est);
                            lacc += d * d;
                        }
                    }
                }
            }
            __syncthreads();
        }
        if (p.loss) {
#pragma unroll
            for (int o = 32; o > 0; o >>= 1) lacc += __shfl_xor(lacc, o);
            if (lane == 0) sLoss[wave] = lacc;
        }
    }
    if (p.loss) {
        __syncthreads();
        if (tid == 0) {
            float s = 0.f;
            for (int w = 1; w <= kGruHelpers; ++w) s += sLoss[w];
            p.loss[b] = s / (float)(T * 32);
        }
    }
}

hipError_t launch_gru(const GruArgs& a, int B, hipStream_t st) {
    hipLaunchKernelGGL(gru_kernel, dim3(B), dim3(kGruThreads), 0, st, a);
    return hipGetLastError();
}

}  // namespace aec
