// aec_train.hip — the training step of the Stage-2 post-filter on gfx950
// (SURVEY.md §8(f) row 4).
//
// Reference: scripts/train1.py:191-218 — a zero-padded batch (collate_fn,
// train1.py:43-74) through Little_net.forward with the batch-GLOBAL
// normaliser (ERB.py:254-256 over the whole [B, N] tensor), loss.backward(),
// Adam.step() (train1.py:153).  The loss (ERB.py:318-323) reaches the
// parameters only through est_erb = mask * mic_erb, so the backward is the
// head (linear1 / relu / linear2 / sigmoid) and BPTT through nn.GRU(64, 32);
// the STFT / ERB features are parameter-free (fixed buffers).
//
// Forward = the inference kernels (K1 moments, norm_global_kernel here, K2
// analysis, K3 gru_kernel writing h [B][Tmax][32], K4 synthesis).  Backward:
//   T1 train_head_kernel   frame-parallel: the gates r, z, n, W_hn h + b_hn of
//                          every frame recomputed from (x_t, h_{t-1}) — no
//                          sequential dependency once h is known — and the
//                          head forward + backward -> per-frame record
//                          rec [B*T][8][32] = dh_head, r, z, n, ghn, dz1, dz2, o
//   T2 train_bptt_kernel   one wave per stream, t = T-1 .. 0: the gate
//                          gradients and dh_{t-1} = dh z + W_hh^T dg (W_hh^T in
//                          registers, split over the wave halves as the
//                          forward step is) -> dg [B*T][4][32] = dar, daz, dan, dghn
//   T3 train_wgrad_mfma_kernel  every weight gradient is a GEMM over frames
//                          (sum of outer products of two per-frame vectors):
//                          blocks stage frame records in LDS and run them
//                          through v_mfma_f32_16x16x4_f32, 4 frames per
//                          instruction; biases are plain sums -> part
//                          [nblk][12544] (no atomics)
//   T4 train_reduce_kernel grad = grad_loss * sum over blocks (fixed order, f64)
//   adam_kernel            torch.optim.Adam's update, one thread per element
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#include "aec_fft.h"
#include "aec_frame.h"
#include "aec_launch.h"

namespace aec {

namespace {
constexpr int kRec = 8 * 32;           // per-frame record floats (T1 -> T2, T3)
constexpr int kDg = 4 * 32;            // per-frame gate gradients (T2 -> T3)
constexpr int kWgF = 32;               // frames per T3 LDS stage
constexpr int kWgRow = 452;            // T3 LDS frame row (see train_wgrad_mfma_kernel; 4 floats of padding)

__device__ __forceinline__ float sig_acc(float x) { return 1.f / (1.f + expf(-x)); }
}  // namespace

// ---------------------------------------------------------------------------
// Batch-global normaliser: c_s = mean / std (unbiased) over all B rows of
// signal s (each row contributes its kMomChunks partials over n samples), the
// same scalar for every row (ERB.py:254-256 on the padded [B, N] batch).
// grid = 3 (signal), block = 256; fixed-order sums (deterministic).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void norm_global_kernel(const double2* __restrict__ mom, int B, int64_t n,
                                                          float* __restrict__ cvals) {
    const int s = blockIdx.x, tid = threadIdx.x;
    double s1 = 0.0, s2 = 0.0;
    for (int i = tid; i < B * kMomChunks; i += 256) {
        const int b = i / kMomChunks, c = i % kMomChunks;
        const double2 v = mom[((int64_t)b * 3 + s) * kMomChunks + c];
        s1 += v.x;
        s2 += v.y;
    }
    __shared__ double r1[256], r2[256];
    r1[tid] = s1;
    r2[tid] = s2;
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
        if (tid < st) {
            r1[tid] += r1[tid + st];
            r2[tid] += r2[tid + st];
        }
        __syncthreads();
    }
    const double dn = (double)B * (double)n;
    const double mean = r1[0] / dn;
    double num = r2[0] - r1[0] * mean;
    if (num < 0.0) num = 0.0;
    const float c = (float)(mean / sqrt(num / (dn - 1.0)));
    for (int b = tid; b < B; b += 256) cvals[b * 3 + s] = c;
}

// ---------------------------------------------------------------------------
// T1: per-frame gates + head forward / backward.  One half-wave (32 lanes,
// lane j = unit / band j) per frame, grid-strided over the B*T frames.  The
// matrices sit in LDS transposed where a lane walks a row (lane j reads
// W^T[k][j]: consecutive lanes, consecutive banks) and as stored where a lane
// walks a column (do = W2^T dz2, dh = W1[:, :32]^T dz1).
// ---------------------------------------------------------------------------
namespace {
constexpr int oWihT = 0;                       // [64][96]
constexpr int oWhhT = oWihT + 64 * 96;         // [32][96]
constexpr int oW1T = oWhhT + 32 * 96;          // [64][32]
constexpr int oW2T = oW1T + 64 * 32;           // [32][32]
constexpr int oW1 = oW2T + 32 * 32;            // [32][64]
constexpr int oW2 = oW1 + 32 * 64;             // [32][32]
constexpr int oBih = oW2 + 32 * 32;            // [96]
constexpr int oBhh = oBih + 96;                // [96]
constexpr int oB1 = oBhh + 96;                 // [32]
constexpr int oB2 = oB1 + 32;                  // [32]
constexpr int oScr = oB2 + 32;                 // 8 half-waves x kScr
constexpr int kScr = 256;                      // x 64 | hp 32 | hc 64 | o 32 | dz2 32 | dz1 32
constexpr int kHeadFloats = oScr + 8 * kScr;
}  // namespace

size_t train_head_smem_bytes() { return (size_t)kHeadFloats * 4; }

__global__ __launch_bounds__(256) void train_head_kernel(TrainArgs p) {
    extern __shared__ __attribute__((aligned(16))) float smem[];
    const int tid = threadIdx.x;
    const float* W_ih = p.w;                  // [96][64]   (blob order, aec_hip.h)
    const float* W_hh = W_ih + 96 * 64;       // [96][32]
    const float* b_ih = W_hh + 96 * 32;
    const float* b_hh = b_ih + 96;
    const float* W1 = b_hh + 96;              // [32][64]
    const float* b1 = W1 + 32 * 64;
    const float* W2 = b1 + 32;                // [32][32]
    const float* b2 = W2 + 32 * 32;
    for (int i = tid; i < 96 * 64; i += 256) smem[oWihT + (i % 64) * 96 + i / 64] = W_ih[i];
    for (int i = tid; i < 96 * 32; i += 256) smem[oWhhT + (i % 32) * 96 + i / 32] = W_hh[i];
    for (int i = tid; i < 32 * 64; i += 256) {
        smem[oW1T + (i % 64) * 32 + i / 64] = W1[i];
        smem[oW1 + i] = W1[i];
    }
    for (int i = tid; i < 32 * 32; i += 256) {
        smem[oW2T + (i % 32) * 32 + i / 32] = W2[i];
        smem[oW2 + i] = W2[i];
    }
    if (tid < 96) {
        smem[oBih + tid] = b_ih[tid];
        smem[oBhh + tid] = b_hh[tid];
    }
    if (tid < 32) {
        smem[oB1 + tid] = b1[tid];
        smem[oB2 + tid] = b2[tid];
    }
    __syncthreads();
    const float* sWihT = smem + oWihT;
    const float* sWhhT = smem + oWhhT;
    const float* sW1T = smem + oW1T;
    const float* sW2T = smem + oW2T;
    const float* sW1 = smem + oW1;
    const float* sW2 = smem + oW2;
    const int hw = tid >> 5, j = tid & 31;
    float* sx = smem + oScr + hw * kScr;      // x [64]
    float* shp = sx + 64;                     // h_{t-1} [32]
    float* shc = shp + 32;                    // [h_t, mic_erb] [64]
    float* so = shc + 64;                     // relu(linear1) [32]
    float* sdz2 = so + 32;
    float* sdz1 = sdz2 + 32;
    const int T = p.T;
    const int64_t nf = (int64_t)p.B * T;
    const float inv_tf = 1.f / (float)(T * 32);
    for (int64_t g = (int64_t)blockIdx.x * 8 + hw; g < nf; g += (int64_t)gridDim.x * 8) {
        const int b = (int)(g / T), t = (int)(g % T);
        const int64_t row = (int64_t)b * p.Tmax + t;
        const float* fr = p.feats + row * 96;
        const float me = fr[j], re = fr[32 + j], ne = fr[64 + j];
        const float ht = p.h[row * 32 + j];
        const float hp = t > 0 ? p.h[(row - 1) * 32 + j] : 0.f;
        sx[j] = me;
        sx[32 + j] = fabsf(me - re);
        shp[j] = hp;
        shc[j] = ht;
        shc[32 + j] = me;
        wave_fence();
        // gates (nn.GRU: r, z, n), recomputed from x_t and h_{t-1}
        float gir = smem[oBih + j], giz = smem[oBih + 32 + j], gin = smem[oBih + 64 + j];
#pragma unroll 8
        for (int k = 0; k < 64; ++k) {
            const float xv = sx[k];
            gir = fmaf(sWihT[k * 96 + j], xv, gir);
            giz = fmaf(sWihT[k * 96 + 32 + j], xv, giz);
            gin = fmaf(sWihT[k * 96 + 64 + j], xv, gin);
        }
        float ghr = smem[oBhh + j], ghz = smem[oBhh + 32 + j], ghn = smem[oBhh + 64 + j];
#pragma unroll 8
        for (int k = 0; k < 32; ++k) {
            const float hv = shp[k];
            ghr = fmaf(sWhhT[k * 96 + j], hv, ghr);
            ghz = fmaf(sWhhT[k * 96 + 32 + j], hv, ghz);
            ghn = fmaf(sWhhT[k * 96 + 64 + j], hv, ghn);
        }
        const float r = sig_acc(gir + ghr);
        const float z = sig_acc(giz + ghz);
        const float n = tanhf(gin + r * ghn);
        // head forward (ERB.py:295-304)
        float z1 = smem[oB1 + j];
#pragma unroll 8
        for (int k = 0; k < 64; ++k) z1 = fmaf(sW1T[k * 32 + j], shc[k], z1);
        const float o = fmaxf(z1, 0.f);
        so[j] = o;
        wave_fence();
        float z2 = smem[oB2 + j];
#pragma unroll 8
        for (int k = 0; k < 32; ++k) z2 = fmaf(sW2T[k * 32 + j], so[k], z2);
        const float mask = sig_acc(z2);
        const float est = mask * me;
        // loss (ERB.py:318-323) backward with d loss = 1; grad_loss scales T4
        const float u = sqrtf(ne) - sqrtf(est);
        const float dest = -(2.f * u * inv_tf) * (0.5f / sqrtf(est));
        const float dz2 = dest * me * mask * (1.f - mask);
        sdz2[j] = dz2;
        wave_fence();
        float dov = 0.f;
#pragma unroll 8
        for (int k = 0; k < 32; ++k) dov = fmaf(sW2[k * 32 + j], sdz2[k], dov);
        const float dz1 = o > 0.f ? dov : 0.f;
        sdz1[j] = dz1;
        wave_fence();
        float dhh = 0.f;
#pragma unroll 8
        for (int k = 0; k < 32; ++k) dhh = fmaf(sW1[k * 64 + j], sdz1[k], dhh);
        float* rec = p.rec + g * kRec;
        rec[j] = dhh;
        rec[32 + j] = r;
        rec[64 + j] = z;
        rec[96 + j] = n;
        rec[128 + j] = ghn;
        rec[160 + j] = dz1;
        rec[192 + j] = dz2;
        rec[224 + j] = o;
        wave_fence();                           // scratch reused by the next frame
    }
}

// ---------------------------------------------------------------------------
// T2: BPTT, one wave per stream.  Lane l: unit j = l & 31, half kh = l >> 5.
// The lane holds W_hh[g][j] for the 48 gate rows g = 32 i + 16 kh + q
// (i = r, z, n; q < 16): dh_{t-1}[j] = dh[j] z[j] + sum_g W_hh[g][j] dgh[g],
// the two halves' partial sums combined with v_permlane32_swap (fixed order:
// half 0 + half 1, identical in both halves).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(64) void train_bptt_kernel(TrainArgs p) {
    __shared__ __attribute__((aligned(16))) float sG[96];
    const int lane = threadIdx.x, j = lane & 31, kh = lane >> 5;
    const int b = blockIdx.x;
    const float* W_hh = p.w + 96 * 64;
    float wT[48];
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int q = 0; q < 16; ++q) wT[16 * i + q] = W_hh[(32 * i + 16 * kh + q) * 32 + j];
    const int T = p.T;
    const float* rec0 = p.rec + (int64_t)b * T * kRec;
    float* dg0 = p.dg + (int64_t)b * T * kDg;
    const float* h0 = p.h + (int64_t)b * p.Tmax * 32;
    // inputs of kP steps are loaded one chunk ahead (HBM latency spans
    // several steps of the chain)
    constexpr int kP = 8;
    float cur[kP][6], nxt[kP][6];
    auto ld = [&](float (&v)[kP][6], int tc) {
#pragma unroll
        for (int i = 0; i < kP; ++i) {
            const int t = tc - i;
            const float* rc = rec0 + (int64_t)max(t, 0) * kRec;
            v[i][0] = rc[j]; v[i][1] = rc[32 + j]; v[i][2] = rc[64 + j]; v[i][3] = rc[96 + j]; v[i][4] = rc[128 + j];
            v[i][5] = t > 0 ? h0[(int64_t)(t - 1) * 32 + j] : 0.f;
        }
    };
    ld(cur, T - 1);
    float carry = 0.f;
    for (int tc = T - 1; tc >= 0; tc -= kP) {
        if (tc - kP >= 0) ld(nxt, tc - kP);
#pragma unroll
        for (int i = 0; i < kP; ++i) {
            const int t = tc - i;
            if (t < 0) break;
            const float dhh = cur[i][0], r = cur[i][1], z = cur[i][2], n = cur[i][3], ghn = cur[i][4], hp = cur[i][5];
            const float dh = dhh + carry;
            const float dn = dh * (1.f - z);
            const float dzz = dh * (hp - n);
            const float dan = dn * (1.f - n * n);
            const float dar = dan * ghn * r * (1.f - r);
            const float daz = dzz * z * (1.f - z);
            const float dghn = dan * r;
            if (kh == 0) {
                float* d = dg0 + (int64_t)t * kDg;
                d[j] = dar;
                d[32 + j] = daz;
                d[64 + j] = dan;
                d[96 + j] = dghn;
                sG[j] = dar;
                sG[32 + j] = daz;
                sG[64 + j] = dghn;
            }
            wave_fence();
            float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int g = 0; g < 3; ++g) {
                const float4* g4 = reinterpret_cast<const float4*>(sG + 32 * g + 16 * kh);
#pragma unroll
                for (int q4 = 0; q4 < 4; ++q4) {
                    const float4 v = g4[q4];
                    acc[0] = fmaf(wT[16 * g + 4 * q4], v.x, acc[0]);
                    acc[1] = fmaf(wT[16 * g + 4 * q4 + 1], v.y, acc[1]);
                    acc[2] = fmaf(wT[16 * g + 4 * q4 + 2], v.z, acc[2]);
                    acc[3] = fmaf(wT[16 * g + 4 * q4 + 3], v.w, acc[3]);
                }
            }
            const float part = (acc[0] + acc[1]) + (acc[2] + acc[3]);
            const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(part), __float_as_uint(part), false, false);
            const float other = __uint_as_float(kh ? sw[0] : sw[1]);
            const float sum = kh ? (other + part) : (part + other);
            carry = fmaf(dh, z, sum);
            wave_fence();                       // sG reads done before the next step's writes
        }
#pragma unroll
        for (int i = 0; i < kP; ++i)
#pragma unroll
            for (int q = 0; q < 6; ++q) cur[i][q] = nxt[i][q];
    }
}


// ---------------------------------------------------------------------------
// T2 as a chunked scan.  With the forward values fixed, BPTT is an AFFINE
// recurrence in g_t = dL/dh_t:
//   g_{t-1} = dh_head[t-1] + M_t g_t,
//   M_t = diag(z_t) + W_r^T diag(a_r) + W_z^T diag(a_z) + W_n^T diag(a_n),
//   a_r = (1-z)(1-n^2) ghn r(1-r),  a_z = (h_{t-1} - n) z(1-z),  a_n = (1-z)(1-n^2) r
// so the 626-step chain splits into chunks of kL steps:
//   T2a (B x chunks blocks, parallel): each chunk's map g_{t0} = P g_{t1} + q
//       composed over its steps (32x32 P, 1,536 FMAs per lane and step);
//   T2b (one wave per stream): g at every chunk start, chunks right to left
//       (C matvecs instead of T steps);
//   T2c (B x chunks blocks): each chunk's steps from its incoming g, writing
//       dg as train_bptt_kernel does.
// Same gradients up to the summation order (tests/test_train.py).
// ---------------------------------------------------------------------------
constexpr int kL = 16;                       // steps per chunk

// forward values of step t for unit j: z and the three a's (see above)
__device__ __forceinline__ void bptt_coef(const float* rc, float hp, int j, float& z, float& ar, float& az,
                                          float& an) {
    const float r = rc[32 + j], zz = rc[64 + j], n = rc[96 + j], ghn = rc[128 + j];
    const float c = (1.f - zz) * (1.f - n * n);
    z = zz;
    ar = c * ghn * r * (1.f - r);
    az = (hp - n) * zz * (1.f - zz);
    an = c * r;
}

// T2a: one wave per (stream, chunk).  The chunk's forward values are staged
// in LDS first (one load latency); per step the 32 x 32 M_{t+1} is built in
// LDS (column-major: sM[k][i] = M[i][k], 48 FMAs per lane from W_hh in
// registers), then P <- M P with a 4 x 4 output tile per lane (two b128 LDS
// reads per 16 FMAs) and q <- dh_head + M q.
__global__ __launch_bounds__(64) void bptt_chunk_map_kernel(TrainArgs p) {
    __shared__ __attribute__((aligned(16))) float sC[kL][4][32];   // z, a_r, a_z, a_n of step t0 + s + 1
    __shared__ __attribute__((aligned(16))) float sD[kL][32];      // dh_head of step t0 + s
    __shared__ __attribute__((aligned(16))) float sM[32][32];      // M^T
    __shared__ __attribute__((aligned(16))) float sP[2][32][32];
    __shared__ __attribute__((aligned(16))) float sq[2][32];
    const int lane = threadIdx.x, i = lane & 31, kh = lane >> 5;
    const int ib = lane >> 3, jb = lane & 7;       // the lane's 4 x 4 tile of P
    const int nc = (p.T + kL - 1) / kL;
    const int b = blockIdx.x / nc, c = blockIdx.x % nc;
    const int T = p.T, t0 = c * kL, t1 = min(T, t0 + kL);
    const float* rec0 = p.rec + (int64_t)b * T * kRec;
    const float* h0 = p.h + (int64_t)b * p.Tmax * 32;
    const float* W_hh = p.w + 96 * 64;
    float w[3][16];                                // W_hh[32 g + 16 kh + kk][i]
#pragma unroll
    for (int g = 0; g < 3; ++g)
#pragma unroll
        for (int kk = 0; kk < 16; ++kk) w[g][kk] = W_hh[(32 * g + 16 * kh + kk) * 32 + i];
    // stage the chunk: items (s, unit) = (e >> 5, e & 31), 8 per lane; M_T = 0 (z = a = 0)
#pragma unroll
    for (int u = 0; u < kL * 32 / 64; ++u) {
        const int e = lane + 64 * u, s = e >> 5, j = e & 31;
        const int t = t0 + s;
        float z = 0.f, ar = 0.f, az = 0.f, an = 0.f, dhh = 0.f;
        if (t < t1) {
            dhh = rec0[(int64_t)t * kRec + j];
            if (t + 1 < T) bptt_coef(rec0 + (int64_t)(t + 1) * kRec, h0[(int64_t)t * 32 + j], j, z, ar, az, an);
        }
        sD[s][j] = dhh;
        sC[s][0][j] = z;
        sC[s][1][j] = ar;
        sC[s][2][j] = az;
        sC[s][3][j] = an;
    }
    float pt[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int cc = 0; cc < 4; ++cc) pt[a][cc] = (t1 < T && 4 * ib + a == 4 * jb + cc) ? 1.f : 0.f;
#pragma unroll
    for (int a = 0; a < 4; ++a)
        *reinterpret_cast<float4*>(&sP[0][4 * ib + a][4 * jb]) = make_float4(pt[a][0], pt[a][1], pt[a][2], pt[a][3]);
    if (kh == 0) sq[0][i] = 0.f;
    wave_fence();
    int cur = 0;
    for (int s = t1 - t0 - 1; s >= 0; --s) {
        // M^T[k][i] for k = 16 kh + kk
        const float zi = sC[s][0][i];
        const float4* ar4 = reinterpret_cast<const float4*>(&sC[s][1][16 * kh]);
        const float4* az4 = reinterpret_cast<const float4*>(&sC[s][2][16 * kh]);
        const float4* an4 = reinterpret_cast<const float4*>(&sC[s][3][16 * kh]);
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4) {
            const float4 vr = ar4[k4], vz = az4[k4], vn = an4[k4];
            const float r_[4] = {vr.x, vr.y, vr.z, vr.w}, z_[4] = {vz.x, vz.y, vz.z, vz.w},
                        n_[4] = {vn.x, vn.y, vn.z, vn.w};
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) {
                const int kk = 4 * k4 + q4, k = 16 * kh + kk;
                float m = fmaf(w[0][kk], r_[q4], fmaf(w[1][kk], z_[q4], w[2][kk] * n_[q4]));
                if (k == i) m += zi;
                sM[k][i] = m;
            }
        }
        wave_fence();
        // P <- M P (4 x 4 tile), q <- dh_head + M q
        float acc[4][4] = {};
#pragma unroll
        for (int k = 0; k < 32; ++k) {
            const float4 m4 = *reinterpret_cast<const float4*>(&sM[k][4 * ib]);
            const float4 p4 = *reinterpret_cast<const float4*>(&sP[cur][k][4 * jb]);
            const float mv[4] = {m4.x, m4.y, m4.z, m4.w}, pv[4] = {p4.x, p4.y, p4.z, p4.w};
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int cc = 0; cc < 4; ++cc) acc[a][cc] = fmaf(mv[a], pv[cc], acc[a][cc]);
        }
        float qa = 0.f, qb = 0.f;
#pragma unroll
        for (int kk = 0; kk < 16; kk += 2) {
            const int k = 16 * kh + kk;
            qa = fmaf(sM[k][i], sq[cur][k], qa);
            qb = fmaf(sM[k + 1][i], sq[cur][k + 1], qb);
        }
        const float part = qa + qb;
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(part), __float_as_uint(part), false, false);
        const float other = __uint_as_float(kh ? sw[0] : sw[1]);
        const float qn = sD[s][i] + (kh ? (other + part) : (part + other));
        const int nx = cur ^ 1;
#pragma unroll
        for (int a = 0; a < 4; ++a)
            *reinterpret_cast<float4*>(&sP[nx][4 * ib + a][4 * jb]) = make_float4(acc[a][0], acc[a][1], acc[a][2], acc[a][3]);
        if (kh == 0) sq[nx][i] = qn;
        wave_fence();                              // sM / sP[cur] reads done, sP[nx] written
        cur = nx;
    }
    float* Pc = p.scan_p + ((int64_t)b * nc + c) * 1024;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int e = 4 * (lane + 64 * u);
        *reinterpret_cast<float4*>(Pc + e) = *reinterpret_cast<const float4*>(&sP[cur][0][0] + e);
    }
    if (kh == 0) p.scan_q[((int64_t)b * nc + c) * 32 + i] = sq[cur][i];
}

// T2b: G[c] = g at chunk c's first step = P_c G[c+1] + q_c, c = nc-1 .. 0
__global__ __launch_bounds__(64) void bptt_chunk_carry_kernel(TrainArgs p) {
    __shared__ __attribute__((aligned(16))) float sG[32];
    const int lane = threadIdx.x, i = lane & 31, jh = lane >> 5;
    const int b = blockIdx.x;
    const int nc = (p.T + kL - 1) / kL;
    const float* P0 = p.scan_p + (int64_t)b * nc * 1024;
    const float* q0 = p.scan_q + (int64_t)b * nc * 32;
    float* G0 = p.scan_g + (int64_t)b * nc * 32;
    float gi = q0[(int64_t)(nc - 1) * 32 + i];
    if (jh == 0) G0[(int64_t)(nc - 1) * 32 + i] = gi;
    float4 pn[4];
    auto ldp = [&](int c, float4 (&v)[4]) {
        const float4* row = reinterpret_cast<const float4*>(P0 + (int64_t)c * 1024 + i * 32 + 16 * jh);
#pragma unroll
        for (int m = 0; m < 4; ++m) v[m] = row[m];
    };
    float qn = 0.f;
    if (nc >= 2) {
        ldp(nc - 2, pn);
        qn = q0[(int64_t)(nc - 2) * 32 + i];
    }
    for (int c = nc - 2; c >= 0; --c) {
        float4 pc[4];
#pragma unroll
        for (int m = 0; m < 4; ++m) pc[m] = pn[m];
        const float qc = qn;
        if (c >= 1) {
            ldp(c - 1, pn);
            qn = q0[(int64_t)(c - 1) * 32 + i];
        }
        if (jh == 0) sG[i] = gi;
        wave_fence();
        const float4* g4 = reinterpret_cast<const float4*>(sG + 16 * jh);
        float a0 = 0.f, a1 = 0.f;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const float4 gv = g4[m];
            a0 = fmaf(pc[m].x, gv.x, a0);
            a1 = fmaf(pc[m].y, gv.y, a1);
            a0 = fmaf(pc[m].z, gv.z, a0);
            a1 = fmaf(pc[m].w, gv.w, a1);
        }
        const float part = a0 + a1;
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(part), __float_as_uint(part), false, false);
        const float other = __uint_as_float(jh ? sw[0] : sw[1]);
        gi = qc + (jh ? (other + part) : (part + other));
        if (jh == 0) G0[(int64_t)c * 32 + i] = gi;
        wave_fence();
    }
}

// T2c: chunk c's steps t1-1 .. t0 from g_{t1} = G[c+1] (the last chunk: carry 0)
__global__ __launch_bounds__(64) void bptt_chunk_fill_kernel(TrainArgs p) {
    __shared__ __attribute__((aligned(16))) float sG[96];
    const int lane = threadIdx.x, j = lane & 31, kh = lane >> 5;
    const int nc = (p.T + kL - 1) / kL;
    const int b = blockIdx.x / nc, c = blockIdx.x % nc;
    const int T = p.T, t0 = c * kL, t1 = min(T, t0 + kL);
    const float* W_hh = p.w + 96 * 64;
    float wT[48];
#pragma unroll
    for (int g = 0; g < 3; ++g)
#pragma unroll
        for (int q = 0; q < 16; ++q) wT[16 * g + q] = W_hh[(32 * g + 16 * kh + q) * 32 + j];
    const float* rec0 = p.rec + (int64_t)b * T * kRec;
    float* dg0 = p.dg + (int64_t)b * T * kDg;
    const float* h0 = p.h + (int64_t)b * p.Tmax * 32;
    // steps t1 (seed: g given, no dg) .. t0, all inputs loaded up front
    float v[kL + 1][6];
#pragma unroll
    for (int s = 0; s <= kL; ++s) {
        const int t = min(t1 - s, T - 1);
        const float* rc = rec0 + (int64_t)max(t, 0) * kRec;
        v[s][0] = rc[j]; v[s][1] = rc[32 + j]; v[s][2] = rc[64 + j]; v[s][3] = rc[96 + j]; v[s][4] = rc[128 + j];
        v[s][5] = t > 0 ? h0[(int64_t)(t - 1) * 32 + j] : 0.f;
    }
    const bool seed = t1 < T;
    float carry = 0.f;
    const float gseed = seed ? p.scan_g[((int64_t)b * nc + c + 1) * 32 + j] : 0.f;
#pragma unroll
    for (int s = 0; s <= kL; ++s) {
        const int t = t1 - s;                      // s = 0: the seed step t1
        if (s == 0 && !seed) continue;
        if (t < t0) break;
        const float r = v[s][1], z = v[s][2], n = v[s][3], ghn = v[s][4], hp = v[s][5];
        const float dh = s == 0 ? gseed : v[s][0] + carry;
        const float dn = dh * (1.f - z);
        const float dzz = dh * (hp - n);
        const float dan = dn * (1.f - n * n);
        const float dar = dan * ghn * r * (1.f - r);
        const float daz = dzz * z * (1.f - z);
        const float dghn = dan * r;
        if (kh == 0) {
            if (s > 0) {
                float* d = dg0 + (int64_t)t * kDg;
                d[j] = dar;
                d[32 + j] = daz;
                d[64 + j] = dan;
                d[96 + j] = dghn;
            }
            sG[j] = dar;
            sG[32 + j] = daz;
            sG[64 + j] = dghn;
        }
        wave_fence();
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int g = 0; g < 3; ++g) {
            const float4* g4 = reinterpret_cast<const float4*>(sG + 32 * g + 16 * kh);
#pragma unroll
            for (int q4 = 0; q4 < 4; ++q4) {
                const float4 gv = g4[q4];
                acc[0] = fmaf(wT[16 * g + 4 * q4], gv.x, acc[0]);
                acc[1] = fmaf(wT[16 * g + 4 * q4 + 1], gv.y, acc[1]);
                acc[2] = fmaf(wT[16 * g + 4 * q4 + 2], gv.z, acc[2]);
                acc[3] = fmaf(wT[16 * g + 4 * q4 + 3], gv.w, acc[3]);
            }
        }
        const float part = (acc[0] + acc[1]) + (acc[2] + acc[3]);
        const auto sw = __builtin_amdgcn_permlane32_swap(__float_as_uint(part), __float_as_uint(part), false, false);
        const float other = __uint_as_float(kh ? sw[0] : sw[1]);
        carry = fmaf(dh, z, kh ? (other + part) : (part + other));
        wave_fence();
    }
}

int train_scan_chunks(int T) { return (T + kL - 1) / kL; }

// ---------------------------------------------------------------------------
// T3: weight-gradient partials.  LDS frame row (floats):
//   [0, 96)   dgi = (dar, daz, dan)          [96, 192) dgh = (dar, daz, dghn)
//   [192,256) x = (mic_erb, |mic - ref|)      [256,288) h_{t-1}
//   [288,320) dz1   [320,384) (h_t, mic_erb)  [384,416) dz2   [416,448) o
// Block k owns the frames [k * per, (k + 1) * per) of the flattened B*T.
// ---------------------------------------------------------------------------
// T3 on the matrix cores: every weight gradient is a GEMM over frames,
// dW[g][c] = sum_f A[f][g] B[f][c] (A, B per-frame vectors of the staged rows),
// so v_mfma_f32_16x16x4_f32 takes 4 frames per instruction (lane l: A at
// row (f0 + l / 16), column g0 + l % 16; B likewise; D holds dW[g0 + 4 (l / 16)
// + r][c0 + l % 16]).  48 16x16 tiles per block: waves 0-1 W_ih (3 row tiles x
// 4 column tiles each), wave 2 W_hh (6 x 2), wave 3 linear1 (2 x 4) and
// linear2 (2 x 2); the 256 bias entries are plain sums (one per thread).
typedef float wg_f32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void train_wgrad_mfma_kernel(TrainArgs p, int64_t per) {
    __shared__ __attribute__((aligned(16))) float sR[kWgF * kWgRow];
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int fr = lane & 15, fk = lane >> 4;
    wg_f32x4 acc[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) acc[i] = wg_f32x4{0.f, 0.f, 0.f, 0.f};
    // bias entry of this thread: row offset and blob index
    const int boff = tid < 192 ? tid : (tid < 224 ? 288 + tid - 192 : 384 + tid - 224);
    const int bblob = tid < 96 ? 9216 + tid : (tid < 192 ? 9312 + tid - 96 : (tid < 224 ? 11456 + tid - 192
                                                                                       : 12512 + tid - 224));
    float bacc = 0.f;
    const int T = p.T;
    const int64_t nf = (int64_t)p.B * T;
    const int64_t g0 = (int64_t)blockIdx.x * per, g1 = min(nf, g0 + per);
    for (int64_t gs = g0; gs < g1; gs += kWgF) {
        const int nfr = (int)min((int64_t)kWgF, g1 - gs);
        __syncthreads();                                  // previous stage consumed
        for (int e = tid; e < kWgF * 32; e += 256) {
            const int f = e >> 5, j = e & 31;
            float* row = sR + f * kWgRow;
            if (f < nfr) {
                const int64_t g = gs + f;
                const int b = (int)(g / T), t = (int)(g % T);
                const int64_t fi = (int64_t)b * p.Tmax + t;
                const float* d = p.dg + g * kDg;
                const float* rc = p.rec + g * kRec;
                const float dar = d[j], daz = d[32 + j], dan = d[64 + j], dghn = d[96 + j];
                const float me = p.feats[fi * 96 + j], re = p.feats[fi * 96 + 32 + j];
                row[j] = dar; row[32 + j] = daz; row[64 + j] = dan;
                row[96 + j] = dar; row[128 + j] = daz; row[160 + j] = dghn;
                row[192 + j] = me; row[224 + j] = fabsf(me - re);
                row[256 + j] = t > 0 ? p.h[(fi - 1) * 32 + j] : 0.f;
                row[288 + j] = rc[160 + j];
                row[320 + j] = p.h[fi * 32 + j];
                row[352 + j] = me;
                row[384 + j] = rc[192 + j];
                row[416 + j] = rc[224 + j];
            } else {
                for (int c = j; c < 448; c += 32) row[c] = 0.f;
            }
        }
        __syncthreads();
#pragma unroll 2
        for (int f0 = 0; f0 < kWgF; f0 += 4) {
            const float* rk = sR + (f0 + fk) * kWgRow + fr;
            auto mm = [&](int i, float a, float b) {
                acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
            };
            if (wave < 2) {                                   // W_ih: A = dgi [0, 96), B = x [192, 256)
                float bv[4];
#pragma unroll
                for (int c = 0; c < 4; ++c) bv[c] = rk[192 + 16 * c];
#pragma unroll
                for (int r = 0; r < 3; ++r) {
                    const float av = rk[16 * (3 * wave + r)];
#pragma unroll
                    for (int c = 0; c < 4; ++c) mm(4 * r + c, av, bv[c]);
                }
            } else if (wave == 2) {                           // W_hh: A = dgh [96, 192), B = h_{t-1} [256, 288)
                const float b0 = rk[256], b1 = rk[256 + 16];
#pragma unroll
                for (int r = 0; r < 6; ++r) {
                    const float av = rk[96 + 16 * r];
                    mm(2 * r, av, b0);
                    mm(2 * r + 1, av, b1);
                }
            } else {                                          // linear1: dz1 x (h, mic); linear2: dz2 x o
                float bv[4];
#pragma unroll
                for (int c = 0; c < 4; ++c) bv[c] = rk[320 + 16 * c];
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    const float av = rk[288 + 16 * r];
#pragma unroll
                    for (int c = 0; c < 4; ++c) mm(4 * r + c, av, bv[c]);
                }
                const float o0 = rk[416], o1 = rk[416 + 16];
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    const float av = rk[384 + 16 * r];
                    mm(8 + 2 * r, av, o0);
                    mm(8 + 2 * r + 1, av, o1);
                }
            }
        }
        for (int f = 0; f < nfr; ++f) bacc += sR[f * kWgRow + boff];
    }
    float* part = p.part + (int64_t)blockIdx.x * kWeights;
    auto put = [&](int i, int base, int ld, int g0_, int c0) {
#pragma unroll
        for (int r = 0; r < 4; ++r) part[base + (g0_ + 4 * fk + r) * ld + c0 + fr] = acc[i][r];
    };
    if (wave < 2) {
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) put(4 * r + c, 0, 64, 16 * (3 * wave + r), 16 * c);
    } else if (wave == 2) {
#pragma unroll
        for (int r = 0; r < 6; ++r)
#pragma unroll
            for (int c = 0; c < 2; ++c) put(2 * r + c, 6144, 32, 16 * r, 16 * c);
    } else {
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int c = 0; c < 4; ++c) put(4 * r + c, 9408, 64, 16 * r, 16 * c);
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int c = 0; c < 2; ++c) put(8 + 2 * r + c, 11488, 32, 16 * r, 16 * c);
    }
    part[bblob] = bacc;
}

// T4: grad[e] = grad_loss * sum_k part[k][e]: block = 64 entries x 4 waves,
// wave q sums blocks k = q, q + 4, ... (8 loads in flight), then a fixed-order
// combine (deterministic).
__global__ __launch_bounds__(256) void train_reduce_kernel(TrainArgs p, int nblk, const float* __restrict__ grad_loss,
                                                           float* __restrict__ grad) {
    __shared__ double sp[4][64];
    const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
    const int e = blockIdx.x * 64 + lane;
    double s = 0.0;
    if (e < kWeights) {
        int k = q;
        for (; k + 28 < nblk; k += 32) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = p.part[(int64_t)(k + 4 * u) * kWeights + e];
#pragma unroll
            for (int u = 0; u < 8; ++u) s += (double)v[u];
        }
        for (; k < nblk; k += 4) s += (double)p.part[(int64_t)k * kWeights + e];
    }
    sp[q][lane] = s;
    __syncthreads();
    if (q == 0 && e < kWeights) {
        const float gl = grad_loss ? *grad_loss : 1.f;
        grad[e] = (float)((sp[0][lane] + sp[1][lane]) + (sp[2][lane] + sp[3][lane])) * gl;
    }
}

__global__ void loss_sum_kernel(const float* __restrict__ per_stream, int B, float* __restrict__ loss) {
    if (threadIdx.x != 0) return;
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += per_stream[b];
    *loss = s;
}

// torch.optim.Adam (amsgrad = False, maximize = False; torch/optim/adam.py):
//   g += wd p;  m = lerp(m, g, 1 - beta1);  v = beta2 v + (1 - beta2) g^2
//   p -= step_size * m / (sqrt(v) / bc2_sqrt + eps),  step_size = lr / (1 - beta1^step)
__global__ __launch_bounds__(256) void adam_kernel(float* __restrict__ prm, const float* __restrict__ grad,
                                                   float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                   float beta1, float beta2, float eps, float wd, float step_size,
                                                   float bc2_sqrt) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    float g = grad[i];
    const float pv = prm[i];
    if (wd != 0.f) g = fmaf(wd, pv, g);
    const float mv = m[i];
    const float mn = fmaf(1.f - beta1, g - mv, mv);
    const float vn = fmaf(beta2, v[i], (1.f - beta2) * g * g);
    m[i] = mn;
    v[i] = vn;
    const float denom = sqrtf(vn) / bc2_sqrt + eps;
    prm[i] = pv - step_size * (mn / denom);
}

// The same update over up to kAdamMax tensors in one launch (one optimizer
// param group): element i belongs to tensor k with off[k] <= i < off[k + 1].
__global__ __launch_bounds__(256) void adam_multi_kernel(AdamList L, float beta1, float beta2, float eps, float wd) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= L.off[L.n]) return;
    int k = 0;
    while (i >= L.off[k + 1]) ++k;
    const int64_t j = i - L.off[k];
    float g = L.g[k][j];
    const float pv = L.p[k][j];
    if (wd != 0.f) g = fmaf(wd, pv, g);
    const float mv = L.m[k][j];
    const float mn = fmaf(1.f - beta1, g - mv, mv);
    const float vn = fmaf(beta2, L.v[k][j], (1.f - beta2) * g * g);
    L.m[k][j] = mn;
    L.v[k][j] = vn;
    const float denom = sqrtf(vn) / L.bc2_sqrt[k] + eps;
    L.p[k][j] = pv - L.step_size[k] * (mn / denom);
}

hipError_t launch_adam_multi(const AdamList& L, float beta1, float beta2, float eps, float wd, hipStream_t st) {
    const int64_t n = L.off[L.n];
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(adam_multi_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, L, beta1, beta2, eps, wd);
    return hipGetLastError();
}

hipError_t launch_norm_global(const double2* mom, int B, int64_t n, float* cvals, hipStream_t st) {
    hipLaunchKernelGGL(norm_global_kernel, dim3(3), dim3(256), 0, st, mom, B, n, cvals);
    return hipGetLastError();
}

int train_wgrad_blocks(int B, int T, int num_cus) {
    const int64_t nf = (int64_t)B * T;
    const int64_t stages = (nf + kWgF - 1) / kWgF;
    return (int)std::max<int64_t>(1, std::min<int64_t>(stages, 2 * (int64_t)num_cus));
}

hipError_t launch_train_backward(const TrainArgs& a, int nblk, const float* grad_loss, float* grad, hipStream_t st) {
    static const hipError_t attr = hipFuncSetAttribute(reinterpret_cast<const void*>(train_head_kernel),
                                                       hipFuncAttributeMaxDynamicSharedMemorySize,
                                                       (int)train_head_smem_bytes());
    if (attr != hipSuccess) return attr;
    const int64_t nf = (int64_t)a.B * a.T;
    const int hblocks = (int)std::min<int64_t>((nf + 7) / 8, 2 * (int64_t)a.num_cus);
    hipLaunchKernelGGL(train_head_kernel, dim3(hblocks), dim3(256), train_head_smem_bytes(), st, a);
    // the scan does ~32x the serial recursion's FLOPs: it wins while the
    // B waves of the serial form leave most of the chip idle (measured at
    // T = 626: B = 16 62 vs 232 us, B = 256 316 vs 238 us)
    const int nc_ = (a.T + kL - 1) / kL;
    if (a.scan_p && a.T > 4 * kL && (int64_t)a.B * nc_ <= 32 * (int64_t)a.num_cus) {
        const int nc = nc_;
        hipLaunchKernelGGL(bptt_chunk_map_kernel, dim3(a.B * nc), dim3(64), 0, st, a);
        hipLaunchKernelGGL(bptt_chunk_carry_kernel, dim3(a.B), dim3(64), 0, st, a);
        hipLaunchKernelGGL(bptt_chunk_fill_kernel, dim3(a.B * nc), dim3(64), 0, st, a);
    } else {
        hipLaunchKernelGGL(train_bptt_kernel, dim3(a.B), dim3(64), 0, st, a);
    }
    const int64_t stages = (nf + kWgF - 1) / kWgF;
    const int64_t per = ((stages + nblk - 1) / nblk) * kWgF;
    hipLaunchKernelGGL(train_wgrad_mfma_kernel, dim3(nblk), dim3(256), 0, st, a, per);
    hipLaunchKernelGGL(train_reduce_kernel, dim3((kWeights + 63) / 64), dim3(256), 0, st, a, nblk, grad_loss, grad);
    return hipGetLastError();
}

hipError_t launch_loss_sum(const float* per_stream, int B, float* loss, hipStream_t st) {
    hipLaunchKernelGGL(loss_sum_kernel, dim3(1), dim3(64), 0, st, per_stream, B, loss);
    return hipGetLastError();
}

hipError_t launch_adam(float* prm, const float* grad, float* m, float* v, int64_t n, float beta1, float beta2,
                       float eps, float wd, float step_size, float bc2_sqrt, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(adam_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, prm, grad, m, v, n, beta1,
                       beta2, eps, wd, step_size, bc2_sqrt);
    return hipGetLastError();
}

}  // namespace aec
