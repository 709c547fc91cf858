// Semantics probe for the gfx950 block-scaled MFMA v_mfma_scale_f32_16x16x128_f8f6f4
// (e4m3 x e4m3, E8M0 scales) and for v_cvt_pk_fp8_f32 (f32 -> OCP e4m3):
//   hypothesis: lane l holds A[row l&15][k = 32 (l>>4) + j] (j = 0..31, one byte each),
//   B[k = 32 (l>>4) + j][col l&15], and the scale of (row / col l&15, k-block l>>4);
//   C/D: col = l&15, row = 4 (l>>4) + i.
// Exact integer data with power-of-two scales: every product and sum is exact in f32.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

static float e4m3_decode(uint8_t c) {
    const int s = c >> 7, e = (c >> 3) & 15, m = c & 7;
    if (e == 15 && m == 7) return NAN;
    const float v = e == 0 ? std::ldexp((float)m / 8.f, -6) : std::ldexp(1.f + m / 8.f, e - 7);
    return s ? -v : v;
}
// nearest code, ties to even mantissa, saturating at +-448
static uint8_t e4m3_encode(float x) {
    const float ax = std::fabs(x) > 448.f ? 448.f : std::fabs(x);
    int best = 0;
    float bd = 1e30f;
    for (int c = 0; c < 127; ++c) {
        const float d = std::fabs(e4m3_decode((uint8_t)c) - ax);
        if (d < bd || (d == bd && (c & 1) == 0)) { bd = d; best = c; }
    }
    return (uint8_t)(best | (x < 0 ? 0x80 : 0));
}

__global__ void mfma_probe(const uint8_t* A, const uint8_t* Bt, const uint8_t* sa, const uint8_t* sb, float* D) {
    const int l = threadIdx.x, r = l & 15, g = l >> 4;
    i32x8 a, b;
    for (int i = 0; i < 8; ++i) {
        a[i] = *reinterpret_cast<const int*>(A + r * 128 + 32 * g + 4 * i);
        b[i] = *reinterpret_cast<const int*>(Bt + r * 128 + 32 * g + 4 * i);
    }
    const int sca = sa[r * 4 + g], scb = sb[r * 4 + g];
    f32x4 c = {0.f, 0.f, 0.f, 0.f};
    c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, sca, 0, scb);
    for (int i = 0; i < 4; ++i) D[(4 * g + i) * 16 + r] = c[i];
}


// One-hot lane/byte probe: block w sets A (mode 0-2, 6) and / or B (mode 3-6) to a
// single 1.0 at lane w >> 5, byte w & 31 (the other operand all ones unless mode 6);
// scale codes per lane identify which lane's scale applies to the element.
__global__ void onehot_probe(int mode, float* D) {
    const int w = blockIdx.x, l = threadIdx.x, ls = w >> 5, js = w & 31;
    i32x8 a, b;
    const bool ahot = mode <= 2 || mode == 6, bhot = mode >= 3;
    for (int i = 0; i < 8; ++i) {
        const int hot = (l == ls && i == js / 4) ? (0x38 << (8 * (js % 4))) : 0;
        a[i] = ahot ? hot : 0x38383838;
        b[i] = bhot ? hot : 0x38383838;
    }
    const int code = (mode == 1 || mode == 4) ? 119 + (l & 15) : (mode == 2 || mode == 5) ? 125 + (l >> 4) : 127;
    const int sca = mode <= 2 ? code : 127, scb = (mode >= 3 && mode <= 5) ? code : 127;
    f32x4 c = {0.f, 0.f, 0.f, 0.f};
    c = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, sca, 0, scb);
    for (int i = 0; i < 4; ++i) D[(size_t)w * 256 + (4 * (l >> 4) + i) * 16 + (l & 15)] = c[i];
}

__global__ void cvt_probe(const float* x, uint8_t* o, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (2 * i + 1 >= n) return;
    const int p = __builtin_amdgcn_cvt_pk_fp8_f32(x[2 * i], x[2 * i + 1], 0, false);
    o[2 * i] = (uint8_t)(p & 0xFF);
    o[2 * i + 1] = (uint8_t)((p >> 8) & 0xFF);
}

int main() {
    srand(1);
    uint8_t A[16 * 128], Bt[16 * 128], sa[64], sb[64];
    float Af[16 * 128], Bf[16 * 128];
    for (int i = 0; i < 16 * 128; ++i) {
        Af[i] = (float)(rand() % 9 - 4);
        Bf[i] = (float)(rand() % 9 - 4) * 0.5f;
        A[i] = e4m3_encode(Af[i]);
        Bt[i] = e4m3_encode(Bf[i]);
        if (e4m3_decode(A[i]) != Af[i] || e4m3_decode(Bt[i]) != Bf[i]) { printf("encoder broken\n"); return 2; }
    }
    for (int i = 0; i < 64; ++i) { sa[i] = (uint8_t)(125 + rand() % 5); sb[i] = (uint8_t)(125 + rand() % 5); }
    uint8_t *dA, *dB, *dsa, *dsb;
    float* dD;
    hipMalloc(&dA, sizeof(A)); hipMalloc(&dB, sizeof(Bt)); hipMalloc(&dsa, 64); hipMalloc(&dsb, 64);
    hipMalloc(&dD, 256 * 4);
    hipMemcpy(dA, A, sizeof(A), hipMemcpyHostToDevice);
    hipMemcpy(dB, Bt, sizeof(Bt), hipMemcpyHostToDevice);
    hipMemcpy(dsa, sa, 64, hipMemcpyHostToDevice);
    hipMemcpy(dsb, sb, 64, hipMemcpyHostToDevice);
    mfma_probe<<<1, 64>>>(dA, dB, dsa, dsb, dD);
    float D[256];
    hipMemcpy(D, dD, sizeof(D), hipMemcpyDeviceToHost);
    int bad = 0;
    for (int r = 0; r < 16; ++r)
        for (int c = 0; c < 16; ++c) {
            double ref = 0;
            for (int k = 0; k < 128; ++k)
                ref += (double)Af[r * 128 + k] * std::ldexp(1.0, sa[r * 4 + k / 32] - 127) * Bf[c * 128 + k] *
                       std::ldexp(1.0, sb[c * 4 + k / 32] - 127);
            if ((double)D[r * 16 + c] != ref) {
                if (bad < 5) printf("D[%d][%d] = %g ref %g\n", r, c, D[r * 16 + c], ref);
                ++bad;
            }
        }
    printf("mfma_scale 16x16x128 e4m3 layout mismatches: %d / 256\n", bad);

    {
        float* dO;
        hipMalloc(&dO, (size_t)2048 * 256 * 4);
        float* O = (float*)malloc((size_t)2048 * 256 * 4);
        for (int mode = 0; mode < 7; ++mode) {
            onehot_probe<<<2048, 64>>>(mode, dO);
            hipMemcpy(O, dO, (size_t)2048 * 256 * 4, hipMemcpyDeviceToHost);
            printf("mode %d:", mode);
            for (int w = 0; w < 2048; ++w) {
                int nz = 0, fr = -1, fc = -1;
                float v = 0;
                for (int e = 0; e < 256; ++e)
                    if (O[(size_t)w * 256 + e] != 0.f) { if (!nz) { fr = e / 16; fc = e % 16; v = O[(size_t)w * 256 + e]; } ++nz; }
                // lane, byte : nonzero count, first row, first col, log2 value
                printf(" %d.%d:%d,%d,%d,%d", w >> 5, w & 31, nz, fr, fc, nz ? (int)std::lround(std::log2(std::fabs(v))) : 99);
            }
            printf("\n");
        }
    }
    // conversion: a sweep of magnitudes incl. ties, subnormals and > 448
    const int n = 4096;
    float* xs = (float*)malloc(n * 4);
    for (int i = 0; i < n; ++i) {
        const float m = std::ldexp(1.f + (float)(i % 64) / 64.f, (i / 64) % 22 - 12);
        xs[i] = (i & 1) ? -m : m;
    }
    xs[0] = 500.f; xs[1] = -1000.f; xs[2] = 448.f; xs[3] = 464.f; xs[4] = 0.f; xs[5] = 1e-9f;
    float* dx; uint8_t* dq;
    hipMalloc(&dx, n * 4); hipMalloc(&dq, n);
    hipMemcpy(dx, xs, n * 4, hipMemcpyHostToDevice);
    cvt_probe<<<n / 128, 64>>>(dx, dq, n);
    uint8_t* q = (uint8_t*)malloc(n);
    hipMemcpy(q, dq, n, hipMemcpyDeviceToHost);
    int cbad = 0, sat = 0;
    for (int i = 0; i < n; ++i) {
        const uint8_t h = e4m3_encode(xs[i]);
        if (h != q[i]) {
            if (std::fabs(xs[i]) > 448.f) { ++sat; if (sat < 4) printf("x=%g dev 0x%02x host 0x%02x\n", xs[i], q[i], h); }
            else { if (cbad < 8) printf("x=%.9g dev 0x%02x (%g) host 0x%02x (%g)\n", xs[i], q[i], e4m3_decode(q[i]), h, e4m3_decode(h)); ++cbad; }
        }
    }
    printf("cvt_pk_fp8_f32 mismatches vs RNE-saturating host encoder: %d in range, %d above 448\n", cbad, sat);
    return (bad || cbad) ? 1 : 0;
}
