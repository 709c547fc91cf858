// crn_stream.hip — fused kernels of the DCCRN per-hop step (aec_crn_stream_step).
//
// At one frame per stream the step's launches are latency chains: a launch
// costs ~5 us even when its work is a few hundred thousand MACs.  The front of
// the hop (the frame [prev hop | cur hop] of mic and far -> rFFT-512 ->
// FD-NLMS step -> X0 -> the narrow encoder levels) therefore runs as ONE
// launch, one block per stream, with the intermediate maps in LDS:
//
//   ConvSTFT          dccrn.py:45-52    (aec_fft.h / aec_stft.h transforms)
//   FD-NLMS           aec::NlmsBin       (build-defined, aec_hip.h)
//   encoder 0 .. n-1  dccrn2.py:49-62 / dccrn.py:463-478: ComplexConv2d k=(5,1)
//                     s=(2,1) p=(2,0) + folded (Complex)BatchNorm + PReLU, as
//                     implicit GEMMs on v_mfma_f32_16x16x32_bf16
//
// Each level is the batch path's GEMM restated: the same packed weights, the
// same 32-k chunks accumulated in the same order from zero, the same epilogue
// (v >= 0 ? v : alpha v, then bf16), so its outputs equal the row-GEMM
// kernel's (tests/test_gpu_crn.py::test_fused_stream_front_bit_exact).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "aec_fft.h"
#include "aec_frame.h"
#include "aec_stft.h"
#include "aec_tables.h"
#include "crn_gemm.h"
#include "crn_launch.h"

namespace crn {

namespace {

constexpr int kMapElems = 2048;    // bf16 elements of one level's output map (Fo x N = 8 tiles of 16 x 16)

// X0 bin k (1..256) as 8 bf16: (mic.re, far.re, mic.im, far.im, 0, 0, 0, 0) (dccrn.py:559-561)
__device__ __forceinline__ void x0_put(bf16_t* x0, int k, float2 m, float2 f) {
    u32x4 v;
    v[0] = (uint32_t)f2bf(m.x) | ((uint32_t)f2bf(f.x) << 16);
    v[1] = (uint32_t)f2bf(m.y) | ((uint32_t)f2bf(f.y) << 16);
    v[2] = 0u;
    v[3] = 0u;
    *reinterpret_cast<u32x4*>(x0 + (k - 1) * 8) = v;
}

}  // namespace

template <int TAPS>
__global__ __launch_bounds__(256) void crn_stream_enc_kernel(StreamEncArgs p) {
    __shared__ __attribute__((aligned(16))) float sTab[256 * 2 + 258 * 2 + 512];
    __shared__ __attribute__((aligned(16))) float sGrp[2][aec::kGroupFloats];
    __shared__ __attribute__((aligned(16))) float2 sRow[2][256];
    __shared__ __attribute__((aligned(16))) bf16_t sX0[256 * 8];
    __shared__ __attribute__((aligned(16))) bf16_t sMap[2][kMapElems];
    float2* sTwT = reinterpret_cast<float2*>(sTab);
    float2* sTw512 = sTwT + 256;
    float* sHann = reinterpret_cast<float*>(sTw512 + 258);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int b = blockIdx.x;

    // 1. every independent load first: the two hops of both signals (one float4 per thread;
    //    the current hop also saved to the ring), the tables, the NLMS state and the weight
    //    fragments of every level
    {
        const int s = tid >> 7, h = (tid >> 6) & 1, i = tid & 63;
        float4 v;
        if (h == 0) {
            v = reinterpret_cast<const float4*>((s ? p.prev_far : p.prev_mic) + (int64_t)b * 256)[i];
        } else {
            const float* cur = (s ? p.cur_far : p.cur_mic) + (int64_t)b * p.ld_cur;
            if ((p.ld_cur & 3) == 0 && ((reinterpret_cast<uintptr_t>(p.cur_mic) | reinterpret_cast<uintptr_t>(p.cur_far)) & 15) == 0)
                v = reinterpret_cast<const float4*>(cur)[i];
            else
                v = make_float4(cur[4 * i], cur[4 * i + 1], cur[4 * i + 2], cur[4 * i + 3]);
            float* save = s ? p.save_far : p.save_mic;
            if (save) reinterpret_cast<float4*>(save + (int64_t)b * 256)[i] = v;
        }
        reinterpret_cast<float4*>(sGrp[s] + h * aec::kHopStride)[i] = v;
    }
    const float2 t0 = p.tab->twT[tid], t1 = p.tab->tw512[tid];
    const float2 t2 = tid < 2 ? p.tab->tw512[256 + tid] : make_float2(0.f, 0.f);
    const float h0 = p.tab->hann[tid], h1 = p.tab->hann[tid + 256];
    aec::NlmsBin<(TAPS > 0 ? TAPS : 1)> nb;
    float2 rh[TAPS > 1 ? TAPS - 1 : 1];
    float2* nst = nullptr;
    if constexpr (TAPS > 0) {
        const int k = tid;
        nst = p.state + (int64_t)b * (2 * TAPS) * 256;
        nb.reset(k == 0);
#pragma unroll
        for (int l = 0; l < TAPS; ++l) {
            const float2 w = nst[l * 256 + k];
            nb.w[l] = aec::v2f{w.x, w.y};
        }
#pragma unroll
        for (int l = 0; l + 1 < TAPS; ++l) rh[l] = nst[(TAPS + l) * 256 + k];
        const float2 pp = nst[(2 * TAPS - 1) * 256 + k];
        nb.p = aec::v2f{pp.x, pp.y};
    }
    // weight fragments: level i, this wave's N tile nt = wave % NT, chunk c: row nt*16 + (lane & 15),
    // k = 32 c + 8 (lane >> 4) .. + 7 (the 16x16x32 B operand)
    u32x4 bw[3][kStreamEncChunks];
    float bias[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        if (i >= p.nlev) break;
        const StreamEncLevel& L = p.lev[i];
        const int NT = L.N >> 4;
        const int n = (wave % NT) * 16 + (lane & 15);
        bias[i] = L.bias[n];
        const bf16_t* wr = L.w + (int64_t)n * L.kpad + 8 * (lane >> 4);
#pragma unroll
        for (int c = 0; c < kStreamEncChunks; ++c)
            bw[i][c] = c < L.nchunk ? *reinterpret_cast<const u32x4*>(wr + 32 * c) : u32x4{0u, 0u, 0u, 0u};
    }
    sTwT[tid] = t0;
    sTw512[tid] = t1;
    if (tid < 2) sTw512[256 + tid] = t2;
    sHann[tid] = h0;
    sHann[tid + 256] = h1;
    __syncthreads();

    // 2. the two transforms on waves 0 (mic) and 1 (far), lanes 0-15: the batch front's
    //    transform code (bit-identical frames) -> packed spectrum rows (slot 0 = (X[0], X[256]))
    if (wave < 2 && lane < 16) {
        const int lb = lane;
        float* reg = sGrp[wave];
        float2 v[16];
        float2 xa[8], xb[8], x128;
        aec::load_frame(v, reg, sHann, 0, lb);
        aec::wave_fence();
        aec::fft256<false>(v, lb, reg, sTwT);
        aec::rfft_unpack(v, lb, sTw512, xa, xb, x128);
        float2* row = sRow[wave];
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
    __syncthreads();

    // 3. bin slot k = tid: the NLMS step (crn_stream_nlms_kernel's arithmetic) and X0
    {
        const int k = tid;
        const float2 rm = sRow[0][k], rf = sRow[1][k];
        float2 e = rm;
        if constexpr (TAPS > 0) {
#pragma unroll
            for (int l = 0; l + 1 < TAPS; ++l) {
                const aec::v2f r{rh[l].x, rh[l].y};
                nb.a[l] = r * nb.ma;
                nb.bq[l] = aec::vfma(aec::v2f{r.y, r.x}, nb.mb, r * nb.mc);
                nb.qq[l] = aec::vfma(nb.a[l], nb.a[l], nb.bq[l] * nb.bq[l]);
            }
            e = nb.step(rm, rf, p.mu, p.beta, p.delta);
#pragma unroll
            for (int l = 0; l < TAPS; ++l) nst[l * 256 + k] = make_float2(nb.w[l].x, nb.w[l].y);
            if constexpr (TAPS > 1) {
                nst[TAPS * 256 + k] = rf;
#pragma unroll
                for (int l = 1; l + 1 < TAPS; ++l) nst[(TAPS + l) * 256 + k] = rh[l - 1];
            }
            nst[(2 * TAPS - 1) * 256 + k] = make_float2(nb.p.x, nb.p.y);
            p.espec[(int64_t)b * 256 + k] = e;
        }
        if (k > 0)
            x0_put(sX0, k, e, rf);
        else   // slot 0 holds (X[0], X[256]): the Nyquist bin 256; DC is not an encoder input
            x0_put(sX0, 256, make_float2(e.y, 0.f), make_float2(rf.y, 0.f));
    }
    __syncthreads();

    // 4. encoder levels: 8 output tiles of 16 bins x 16 channels per level, two per wave (N tile
    //    nt = wave % NT, M tiles m0 = wave / NT and m0 + 4 / NT); the implicit A rows read the
    //    input map in LDS (input bin 2 j - 2 + tap, zero outside [0, Fin))
    const bf16_t* in = sX0;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        if (i >= p.nlev) break;
        const StreamEncLevel& L = p.lev[i];
        const int Fin = 256 >> i, Fo = Fin >> 1;
        const int NT = L.N >> 4;
        const int nt = wave % NT, m0 = wave / NT, m1 = m0 + 4 / NT;
        const int cs = L.cin_shift;
        f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int c = 0; c < kStreamEncChunks; ++c) {
            if (c >= L.nchunk) break;
            const int k0 = 32 * c + 8 * (lane >> 4);
            const int tap = k0 >> cs, q0 = k0 & ((1 << cs) - 1);
#pragma unroll
            for (int t = 0; t < 2; ++t) {
                const int j = (t ? m1 : m0) * 16 + (lane & 15);
                const int ib = 2 * j - 2 + tap;
                u32x4 a = {0u, 0u, 0u, 0u};
                if (tap < 5 && ib >= 0 && ib < Fin) a = *reinterpret_cast<const u32x4*>(in + (ib << cs) + q0);
                mma_chunk(acc[t], a, bw[i][c], bf16_t{});
            }
        }
        bf16_t* map = sMap[i & 1];
        const bool keep = i + 1 < p.nlev;
        bf16_t* out = L.out + (int64_t)b * Fo * L.ldo + L.choff;
        const int n = nt * 16 + (lane & 15);
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = (t ? m1 : m0) * 16 + 4 * (lane >> 4) + r;
                float v = acc[t][r] + bias[i];
                v = v >= 0.f ? v : L.alpha * v;
                const bf16_t o = f2bf(v);
                if (keep) map[row * L.N + n] = o;
                out[(int64_t)row * L.ldo + n] = o;
            }
        __syncthreads();
        in = map;
    }
}

hipError_t launch_stream_enc(const StreamEncArgs& a, int taps, hipStream_t st) {
    if (a.B <= 0) return hipSuccess;
    if (a.nlev < 1 || a.nlev > 3) return hipErrorInvalidValue;
    for (int i = 0; i < a.nlev; ++i) {
        const StreamEncLevel& L = a.lev[i];
        const int Fo = 128 >> i;
        if (L.N % 16 || (Fo / 16) * (L.N / 16) != 8 || 4 % (L.N / 16) || L.nchunk < 1 ||
            L.nchunk > kStreamEncChunks || L.cin_shift < 3 || (i > 0 && (1 << L.cin_shift) != a.lev[i - 1].N) ||
            (i == 0 && L.cin_shift != 3) || L.kpad < 32 * L.nchunk || L.kpad % 8 || !L.w || !L.bias || !L.out)
            return hipErrorInvalidValue;
    }
    switch (taps) {
#define CRN_ENC_CASE(N)                                                                               \
    case N: hipLaunchKernelGGL((crn_stream_enc_kernel<N>), dim3((unsigned)a.B), dim3(256), 0, st, a); break;
        CRN_ENC_CASE(0) CRN_ENC_CASE(1) CRN_ENC_CASE(2) CRN_ENC_CASE(3) CRN_ENC_CASE(4)
        CRN_ENC_CASE(5) CRN_ENC_CASE(6) CRN_ENC_CASE(7) CRN_ENC_CASE(8)
#undef CRN_ENC_CASE
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

}  // namespace crn
