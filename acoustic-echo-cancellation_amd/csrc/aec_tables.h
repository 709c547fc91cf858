// aec_tables.h — constant tables shared by host (built once in float64) and device.
#pragma once
#include <hip/hip_runtime.h>

namespace aec {

// Built by the host at aec_create (float64 math, rounded to float32).
struct DevTables {
    float2 tw256[256];   // W256^j = (cos 2pi j/256, -sin 2pi j/256)
    float2 tw512[258];   // W512^k, k = 0..256 (+1 pad)
    float hann[512];     // periodic Hann = scipy get_window('hann', 512) (attention_ccrn.py:12)
    float coffp[256];    // f32(hann[r]^2 + hann[r+256]^2) + 1e-8  (attention_ccrn.py:94-96)
};

// ERB matrix in two sparse views (the reference multiplies the dense [257,32]
// matrix, ERB.py:282-284 and :306-307; only its 483 non-zeros matter).
// Blob layout (int32 words; weights stored as float bit patterns):
//   band_ptr[33] | bin_ptr[258] | band_bin[nnz] | band_w[nnz] | bin_band[nnz] | bin_w[nnz]
struct ErbCSRView {
    const int* band_ptr;
    const int* bin_ptr;
    const int* band_bin;
    const float* band_w;
    const int* bin_band;
    const float* bin_w;
};

__host__ __device__ inline ErbCSRView erb_view(const int* blob, int nnz) {
    ErbCSRView v;
    v.band_ptr = blob;
    v.bin_ptr = blob + 33;
    v.band_bin = blob + 33 + 258;
    v.band_w = reinterpret_cast<const float*>(v.band_bin + nnz);
    v.bin_band = reinterpret_cast<const int*>(v.band_w + nnz);
    v.bin_w = reinterpret_cast<const float*>(v.bin_band + nnz);
    return v;
}

inline size_t erb_blob_words(int nnz) { return 33 + 258 + 4 * (size_t)nnz; }

}  // namespace aec
