// aec_tables.h — constant tables shared by host (built once in float64) and device.
#pragma once
#include <hip/hip_runtime.h>

#include <vector>

namespace aec {

// Built by the host at aec_create (float64 math, rounded to float32).
struct DevTables {
    float2 twT[256];     // twT[k1*16 + lb] = W256^(lb*k1), W256^j = (cos 2pi j/256, -sin 2pi j/256)
    float2 tw512[258];   // W512^k, k = 0..256 (+1 pad)
    float hann[512];     // periodic Hann = scipy get_window('hann', 512) (attention_ccrn.py:12)
    float inv_coff[256]; // 1 / (f32(hann[r]^2 + hann[r+256]^2) + 1e-8)  (attention_ccrn.py:94-96)
};

// ERB matrix views.  The reference multiplies the dense [257,32] float32
// matrix (ERB.py:282-284 forward, :306-307 transpose); only its non-zeros
// (483 for erb_conf) matter, and every bin lies in at most 2 bands.
//
// Forward (bins -> bands), analysis kernel: a per-lane schedule for the 16
// lanes of a frame group.  Bands wider than `split` bins are cut into two
// pieces; the pieces are packed (first-fit decreasing, <= 3 pieces per lane)
// so every lane runs the same L entries.  Entry = float4(bin as int bits,
// w0, w1, w2): exactly one of w0..w2 is the matrix value (the piece's slot
// in that lane), the others are 0, so the lane does 3 FMAs and no selects.
// comb[j] = (slot index of piece 0, slot index of piece 1 or -1), slot index
// = 3*lane + slot.  Blob = float4[L][16] followed by int2[32].
//
// Transpose (bands -> bins), synthesis kernel: float4[257] =
// (band_a as int bits, w_a, band_b as int bits, w_b); w_b = 0 when the bin is
// in one band, both 0 when in none (DC / Nyquist).
struct ErbTables {
    int sched_len = 0;
    int conflicts = 0;           // (step, lane) entries that could not get a distinct residue
    std::vector<float> sched;    // 16 * 4 * L floats + 64 ints (as floats)
    std::vector<float> bintab;   // 257 * 4
    bool ok = false;
    const char* why = "";
};

ErbTables build_erb_tables(const float* erb /* [257][32] */);
void build_dev_tables(DevTables& t);

}  // namespace aec
