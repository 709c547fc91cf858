// crn_launch.h — DCCRN kernel argument blocks and host launchers (internal).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "aec_knobs.h"
#include "aec_tables.h"
#include "crn_gemm.h"

namespace crn {

// Front: frame + Hann + rFFT-512 of mic and far (ConvSTFT, dccrn.py:28-59)
// -> the encoder input map X0 [Tmax][B][256][8] (bins 1..256; channels
// mic_re, far_re, mic_im, far_im, 0, 0, 0, 0 — dccrn.py:559-561).
struct FrontArgs {
    const float* mic;
    const float* far;
    int64_t ld;
    const int64_t* lens;        // device [B]
    int64_t Tmax;
    const aec::DevTables* tab;
    void* x0;
    float2* spec;               // non-null: write the complex spectrum [B][Tmax][257] of `mic` instead of X0
    float2* rows = nullptr;     // non-null (NLMS): write the packed mic / far rows [B][Tmax][2][256]
                                // (slot 0 = (X[0], X[256]), the layout aec::nlms_recursion_kernel reads)
                                // instead of X0
};

// NLMS: X0 from the error rows E [B][Tmax][256] (mic channels) and the far
// half of the packed rows (far channels); frames t >= T_b zero.
struct RowsX0Args {
    const float2* rows;         // [B][Tmax][2][256]
    const float2* espec;        // [B][Tmax][256]
    const int64_t* lens;
    int64_t Tmax;
    void* x0;                   // [Tmax][B][256][8]
    int32_t B;
};

// Back: mask [Tmax][B][256] float2 (bins 1..256) applied to the re-derived
// mic spectrum (mode 0 = 'E', 1 = 'C', 2 = 'R'; dccrn2.py:189-210), irFFT +
// WOLA (ConviSTFT, dccrn.py:80-100) -> out [B][ld_out]; optionally the
// masked spectrum [B][Tmax][257] float2 (out_spec).
struct BackArgs {
    const float* mic;
    int64_t ld;
    const int64_t* lens;
    int64_t Tmax;
    const aec::DevTables* tab;
    const float2* mask;
    float* out;
    int64_t ld_out;
    float2* spec;               // nullable
    const float2* espec = nullptr;   // non-null (NLMS): mask the error rows E [B][Tmax][256] (packed) instead
    // bf16: the mask level (decoder cl = 1, pack_decoder_fused, N = 4) computed in the kernel from
    // cat[1] [Tmax*B][128][2 ch1] instead of reading `mask` (the per-frame GEMM of the row kernel:
    // same 32-k chunks from zero, same epilogue)
    const bf16_t* dm_in = nullptr;
    const bf16_t* dm_w = nullptr;    // packed [16][kpad]
    const float* dm_bias = nullptr;
    int32_t dm_kpad = 0, dm_cin_shift = 0, dm_act = 0;
};

// Row-GEMM epilogue: out[(m >> oshift)*o_hi + (m & mask)*o_lo + o_add + n] =
// act(acc + bias[n]) for m < M, n < N; act 0 none, 1 PReLU(alpha), 2 tanh.
struct RowEpi {
    void* out;
    int64_t M;
    int32_t N;
    int32_t oshift;
    int64_t o_hi, o_lo, o_add;
    const float* bias;
    float alpha;
    int32_t act;
    int32_t mode = 0;           // timing experiments only (CRN_GEMM_MODE): bit0 skip the epilogue
    // tile order (speed only, never the result): 0 = row tiles in order, column tiles fastest;
    // g > 0 = XCD-aware: each set of blocks sharing an XCD gets a contiguous range of tile ids,
    // walked g row tiles per column step (crn_gemm.h tile_order)
    int32_t xcd_gm = 0;
    // column split (the decoder's fused parities): columns n >= nsplit are
    // stored at element offset split_add + (n - nsplit) instead of n
    int32_t nsplit = 0x7fffffff;
    int64_t split_add = 0;
    // MX-fp8 shadow of the output (bf16 outputs, N % 32 == 0): e4m3 bytes at the output's element
    // offsets (q8) and one E8M0 scale per 32-column group at element offset / 32 (qs), the
    // operand an MX GEMM consumer reads in place (launch_gemm_mx8_rows); null: none
    uint8_t* q8 = nullptr;
    uint8_t* qs = nullptr;
    // split-K (launch_gemm_mx8*): ksplit > 1 runs the 64 x 64 tile grid ksplit times over K
    // slices; skp holds the f32 partial tiles (sk_bytes >= mx8_splitk_bytes), skc one arrival
    // counter per output tile (skc_n >= mx8_splitk_tiles ints, zero between launches).  The
    // caller picks ksplit per layer (never from M), so a row's result does not depend on the
    // batch it sits in.
    int32_t ksplit = 1;
    int32_t skc_n = 0;
    float* skp = nullptr;
    int* skc = nullptr;
    int64_t sk_bytes = 0;
};
int64_t mx8_splitk_tiles(int64_t M, int N);
int64_t mx8_splitk_bytes(int64_t M, int N, int ksplit);

// One LSTM frame step for CELLS weight sets x S input sequences (v1: 1x1,
// v2 NavieComplexLSTM: 2x2), gate columns packed per 16 units (i|f|g|o).
struct StepArgs {
    const void* whh;            // [CELLS*4H][H]
    const void* gx;             // this frame's Gx rows [B][S][CELLS*4H] (input projection + both biases,
                                // the 4 gates of a unit adjacent)
    const void* y_prev;         // h_{t-1} [B][CELLS][S][H]  (unused when first)
    void* y_cur;                // h_t     [B][CELLS][S][H]
    float* cst;                 // c       [B][CELLS][S][H]  (read unless first, written)
    int32_t B, H;
    int32_t first;              // frame 0: h_{-1} = c_{-1} = 0
    int32_t mode;               // timing experiments only (CRN_STEP_MODE)
};

// MX-fp8 layer step of a NavieComplexLSTM (CELLS = S = 2): input projection,
// recurrence, cell update and combination in one launch (lstm_step_mx8_kernel),
// the per-hop streaming form.
struct StepMxArgs {
    const uint8_t* wq;          // [W_ih | W_hh] e4m3 [2*4H][2H] in W_hh's packed row order (pack_lstm),
    const uint8_t* wsc;         //   E8M0 per 32 k [2*4H][2H/32]
    const float* bias;          // b_ih + b_hh [2][H][4] (a unit's 4 gates adjacent)
    const uint8_t* xq;          // layer input x as e4m3: element (b, s, k) at
    const uint8_t* xs;          //   b*x_f + s*x_s + (k >> x_sh)*x_t + (k & (2^x_sh - 1)) + x_0 (2^x_sh % 256 == 0);
    int64_t x_f, x_s, x_t, x_0, x_elems;   //   its E8M0 per 32 k at element offset / 32
    int32_t x_sh;
    const uint8_t* hq_prev;     // h_{t-1} e4m3 [B][2][2][H], E8M0 per 32 units: hs_prev [B][2][2][H/32]
    const uint8_t* hs_prev;
    uint8_t* hq_cur;            // h_t, same layout
    uint8_t* hs_cur;
    float* cst;                 // c [B][2][2][H] (read, written)
    float* hx;                  // h_t f32 [B][2][2][H]: the cell pair's hand-off
    int* cnt;                   // lstm_step_mx8_counters(H, B) arrival counters, zero between launches
    bf16_t* dst;                // combined rows: real at b*ldf + (j >> dshift)*ldd + (j & (2^dshift - 1)),
    int64_t ldf, ldd;           //   imag at + 2^dshift (lstm_combine_kernel's map)
    int32_t dshift;
    uint8_t* q8;                // their MX-fp8 shadow (RowEpi::q8 layout), nullable
    uint8_t* qs;
    int32_t B, H;
    int32_t mode = 0;           // timing experiments only (CRN_MX_STEP_MODE; results invalid unless 0)
};
hipError_t launch_lstm_step_mx8(const StepMxArgs& a, hipStream_t st);
// the layout preconditions of lstm_step_mx8_kernel (H % 256, 128-k stages inside one x tap, 32-unit
// output groups): the pointer-free part of launch_lstm_step_mx8's argument check
bool lstm_step_mx8_layout_ok(const StepMxArgs& a);
int64_t lstm_step_mx8_counters(int H, int B);

// Streaming (one hop per stream): frame = [prev hop, cur hop] of each stream
struct StreamFrontArgs {
    const float* prev_mic;      // [B][256] (the hop ring)
    const float* cur_mic;       // [B][ld_cur]: this call's hop, read in place from the caller's buffer
    const float* prev_far;
    const float* cur_far;
    const aec::DevTables* tab;
    void* x0;                   // [B][256][8]
    int32_t B;
    float2* rows = nullptr;     // non-null (NLMS): write the packed rows [B][2][256] instead of X0
    int64_t ld_cur = 256;       // row stride of cur_mic / cur_far (elements)
    float* save_mic = nullptr;  // non-null: copy the current hops into the ring ([B][256]) for the
    float* save_far = nullptr;  //   next call's frame and the back kernel
};
// NLMS streaming step: one block per stream, bin slot per lane; state
// [B][2*TAPS][256] float2 (taps, far history r[t-1..t-TAPS+1], power — the
// aec_stream.hip layout) -> E rows [B][256] and X0.
struct StreamNlmsArgs {
    const float2* rows;         // [B][2][256]
    float2* state;
    float2* espec;              // [B][256]
    void* x0;                   // [B][256][8]
    int32_t B;
    float mu, beta, delta;
};
struct StreamBackArgs {
    const float* prev_mic;
    const float* cur_mic;
    const aec::DevTables* tab;
    const float2* mask;         // [B][256]
    float* tail;                // [B][256] overlap-add state (in / out)
    float* out;                 // [B][ld_out] output hop (the previous hop of the stream): the caller's buffer
    int32_t B;
    const float2* espec = nullptr;   // non-null (NLMS): mask the E rows [B][256] instead of the mic frame
    int64_t ld_out = 256;
};

// Fused per-hop front (crn_stream.hip): frame -> rFFT of mic and far -> [FD-NLMS step] -> X0 ->
// encoder levels 0 .. nlev-1 (bf16 implicit-GEMM MFMA, 8 tiles of 16 x 16 per level), one block
// per stream; replaces launch_stream_front + launch_stream_nlms + those levels' row GEMMs.
constexpr int kStreamEncChunks = 5;   // 32-k chunks per level 0-2 (K <= 160)
constexpr int kStreamEncChunks3 = 10; // level 3 (K <= 320)
struct StreamEncLevel {
    const bf16_t* w;            // packed [npad][kpad] (pack_encoder)
    const float* bias;
    float alpha;                // PReLU
    int32_t kpad, N, nchunk;    // nchunk = ceil(K / 32)
    int32_t cin_shift;          // log2 of the input map's channels per bin (3: X0's 8)
    bf16_t* out;                // cat[l + 1] [B][Fo][ldo]: the encoder half at channel offset choff
    int64_t ldo;
    int32_t choff;
    uint8_t* q8 = nullptr;      // level 3: the output's MX-fp8 shadow (RowEpi::q8 / qs layout) or null
    uint8_t* qs = nullptr;
};
// Optional last level of the fused front (fp8 step, AEC_CRN_STREAM_FUSE bit 4): encoder level 4
// as its MX-fp8 GEMM (scaled MFMA, 8 output bins x 256 channels, K = 5 taps x 128) on level 3's
// e4m3 shadow kept in LDS; its output (and the output's MX-fp8 shadow) -> cat[5]'s encoder half.
constexpr int kStreamEncMxStages = 5;   // 128-k stages of level 4 (K = 640)
struct StreamEncMxLevel {
    const uint8_t* wq = nullptr;  // [npad8][640] e4m3
    const uint8_t* wsc = nullptr; // [npad8][20] E8M0
    const float* bias = nullptr;
    float alpha = 0.f;
    bf16_t* out = nullptr;        // cat[5] [B][8][ldo] at channel offset choff
    int64_t ldo = 0;
    int32_t choff = 0;
    uint8_t* q8 = nullptr;        // its shadow (RowEpi::q8 / qs layout)
    uint8_t* qs = nullptr;
};
struct StreamEncArgs {
    const float* prev_mic;      // [B][256] hop ring
    const float* cur_mic;       // [B][ld_cur] this call's hop (caller's buffer)
    const float* prev_far;
    const float* cur_far;
    int64_t ld_cur;
    float* save_mic;            // [B][256]: the current hops for the next call and the back kernel
    float* save_far;
    const aec::DevTables* tab;
    int32_t B;
    float2* state;              // NLMS (taps > 0): [B][2 taps][256] (StreamNlmsArgs layout)
    float2* espec;              //   E rows [B][256]
    float mu, beta, delta;
    int32_t nlev;               // 3 or 4 (level 3: 16 output bins x 128 channels, K = 320)
    StreamEncLevel lev[4];
    StreamEncMxLevel mx4;       // mx4.wq non-null (nlev == 4): level 4 as well
};
hipError_t launch_stream_enc(const StreamEncArgs& a, int taps, hipStream_t st);

// Batch encoder front (crn_stream.hip): encoder levels 0-3 of F frames from X0 [F][256][8]
// (frame f's level-i map at lev[i].out + f * Fo_i * ldo + choff), the four levels' shapes as
// launch_stream_enc's; replaces the four row GEMMs of the batch forward's encoder front.
struct EncBatchArgs {
    const bf16_t* x0;
    int64_t F;
    StreamEncLevel lev[4];
};
bool enc_batch_ok(const EncBatchArgs& a);
hipError_t launch_enc_batch(const EncBatchArgs& a, hipStream_t st);

// Fused per-hop back (crn_stream.hip): the last three decoder levels (ComplexConvTranspose2d +
// skip, both parities per GEMM: pack_decoder_fused) with the maps in LDS, the mask, the masked
// spectrum's irFFT and the overlap-add, one block per stream; replaces those levels' row GEMMs
// + launch_stream_back.  Level i's input map = [decoder half | encoder half] of cat[cl]; the
// first map comes whole from HBM, the later ones take the previous level's output as decoder
// half and the encoder half from HBM.
constexpr int kStreamDecChunks0 = 12, kStreamDecChunks1 = 6, kStreamDecChunks2 = 3;   // K <= 384 / 192 / 96
struct StreamDecLevel {
    const bf16_t* w;            // packed [npad][kpad] (pack_decoder_fused: columns [0, Co) parity 0, [Co, 2 Co) parity 1)
    const float* bias;
    float alpha;
    int32_t act;                // 1 PReLU (levels), 0 none / 2 tanh (the mask level)
    int32_t kpad, N, nchunk;    // N = 2 Co (4 at the mask level)
    int32_t cin_shift;          // log2 of the input map's channels per bin (2 ch[cl])
    const bf16_t* src;          // cat[cl] [B][Fin][2 ch[cl]]: the whole map (level 0) or its encoder half (later levels)
};
// Optional first level of the fused back (fp8 step, AEC_CRN_STREAM_FUSE bit 3): decoder cl = 4 as
// its MX-fp8 GEMM (scaled MFMA on cat[4]'s e4m3 shadow and the e4m3 weights, 16 input bins x 128
// columns = both parities of 64 channels, K = 3 taps x 256), its output cat[3]'s decoder half kept
// in LDS.  The K slices (ksplit 1 or 2) summed as gemm_mx8_kernel's split-K reducer sums them.
constexpr int kStreamMxStages = 6;   // 128-k stages of cl = 4 (K = 768)
struct StreamDecMxLevel {
    const uint8_t* wq;          // [npad8][768] e4m3 (pack_decoder_fused order, MX)
    const uint8_t* wsc;         // [npad8][24] E8M0
    const float* bias;
    float alpha;
    const uint8_t* q8;          // cat[4]'s shadow [B][16][256] e4m3
    const uint8_t* qs;          //   and its E8M0 per 32 [B][16][8]
    int32_t ksplit;             // the row GEMM's split (conv_ksplit), 1 or 2
};
struct StreamDecArgs {
    StreamDecLevel lev[3];      // cl = 3, 2, 1 (the last is the mask level)
    StreamDecMxLevel mx;        // mx.wq non-null: cl = 4 first (then lev[0].src supplies only the encoder half)
    const aec::DevTables* tab;
    const float2* espec;        // NLMS: E rows [B][256] (the masked spectrum), else the mic frame:
    const float* prev_mic;      //   [prev hop | cur hop] from the ring
    const float* cur_mic;
    float* tail;                // [B][256] overlap-add state
    float* out;                 // [B][ld_out]
    int64_t ld_out;
    int32_t B;
};
hipError_t launch_stream_dec(const StreamDecArgs& a, int mode, hipStream_t st);

// Batch decoder levels cl = 3, 2 (crn_stream.hip): per frame, cat[3] (whole map, 32 bins x 128)
// -> level cl = 3 -> cat[2]'s decoder half (LDS only) + its encoder half from HBM -> level cl = 2
// -> cat[1]'s decoder half (out, 128 bins x 16 at row stride ldo1).  lev[0..1] as the per-hop
// back's first two levels (src = cat[3] / cat[2]); replaces those two row GEMMs of the batch forward.
struct DecBatchArgs {
    int64_t F;
    StreamDecLevel lev[2];
    bf16_t* out;                // cat[1] [F][128][ldo1], channels [0, 16)
    int64_t ldo1;
};
bool dec_batch_ok(const DecBatchArgs& a);
hipError_t launch_dec_batch(const DecBatchArgs& a, hipStream_t st);

template <typename T>
hipError_t launch_stream_front(const StreamFrontArgs& a, hipStream_t st);
hipError_t launch_stream_back(const StreamBackArgs& a, int mode, hipStream_t st);
template <typename T>
hipError_t launch_stream_nlms(const StreamNlmsArgs& a, int taps, hipStream_t st);
template <typename T>
hipError_t launch_rows_x0(const RowsX0Args& a, hipStream_t st);
hipError_t launch_unpack_rows(const float2* espec, const int64_t* lens, int B, int64_t Tmax, float2* spec,
                              hipStream_t st);

template <typename T, typename OutT>
hipError_t launch_gemm_rows(const RowSrc& a, const T* bt, int64_t ldb, int nstages, const RowEpi& e, int npad,
                            hipStream_t st);
// MX-fp8 (dtype 2): quantize bf16 rows of a RowSrc to e4m3 + E8M0 per 32 k,
// and the scaled-MFMA GEMM over such operands (B = packed weight rows)
hipError_t launch_mx8_quant(const RowSrc& a, uint8_t* q, uint8_t* s, hipStream_t st);
template <typename OutT>
hipError_t launch_gemm_mx8(const uint8_t* aq, const uint8_t* as, const uint8_t* bq, const uint8_t* bs, int K,
                           const RowEpi& e, int npad, hipStream_t st);
// the same GEMM with the A operand gathered in place from an MX-fp8 shadow map (RowEpi::q8 / qs
// of its producer): a = the bf16 GEMM's RowSrc with src = the e4m3 map (one byte per element),
// as_map = its scale map; needs 2^kshift % 128 == 0 (a 128-k stage inside one tap)
template <typename OutT>
hipError_t launch_gemm_mx8_rows(const RowSrc& a, const uint8_t* as_map, const uint8_t* bq, const uint8_t* bs, int K,
                                const RowEpi& e, int npad, hipStream_t st);
template <typename T>
hipError_t launch_front(const FrontArgs& a, int B, hipStream_t st);
hipError_t launch_back(const BackArgs& a, int B, int mode, hipStream_t st);
template <typename T>
hipError_t launch_lstm_step(const StepArgs& a, int cells, int seqs, hipStream_t st);
template <typename T>
hipError_t launch_lstm_combine(const T* y, T* dst, int64_t nframes, int H, int cells, int seqs, int dshift,
                               int64_t ldf, int64_t ldd, hipStream_t st, uint8_t* q8 = nullptr,
                               uint8_t* qs = nullptr);

// Persistent LSTM recurrence (crn_persist.hip): all T frames of one layer in
// one launch for up to 256 streams (64 G blocks, G = ceil(nb / 64) row
// groups), W_hh in AGPRs, h handed over per team through y with arrival counters.
struct PersistArgs {
    const bf16_t* whh;          // packed W_hh [CELLS*4H][H]
    const bf16_t* gx;           // [T][B][S][CELLS*4H] (frame f = t*B + b)
    bf16_t* y;                  // [T][B][CELLS][S][H]: the layer output and the h hand-off
    int* sync;                  // arrival counters (one 64-B line each, [team][half]; kPersistCounters
                                // ints, zeroed per launch), then the error word at kPersistErr (cleared
                                // once per aec_crn_process, set by a wave whose poll timed out)
    int32_t B;                  // streams of the batch (frame row stride)
    int32_t b0, nb;             // this launch's streams b0 .. b0 + nb - 1 (nb <= 256)
    int32_t T;
    int32_t G;                  // row groups (1..4)
    int32_t spin_limit;         // polls before a wave gives up (error word set)
    int32_t read_ahead = 1;     // read the next phase's counter at chunk 7 (CRN_PERSIST_RA, A/B)
    int32_t stall = 0;          // added to every poll target (tests only: a team that never arrives)
};
constexpr int kPersistCounters = 8 * 2 * 16;     // 8 teams x 2 halves, one 64-B line each
constexpr int kPersistErr = kPersistCounters;    // error word
constexpr int kPersistSyncInts = kPersistErr + 16;
constexpr int kPersistSpinLimit = 1 << 22;       // default polls before a wave gives up (AEC_CRN_SPIN_LIMIT)
bool persist_supported(int H, int cells, int seqs, int num_cus);
// the team's rows in two halves whose phases alternate, so each half's cell
// update and hand-off run under the other half's MFMAs
hipError_t launch_lstm_persist(const PersistArgs& a, hipStream_t st);

// tile width the host must pad the weight rows (N) to for a GEMM of N columns
inline int gemm_bn(int N) { return N <= 16 ? 16 : N <= 32 ? 32 : N <= 64 ? 64 : 128; }

}  // namespace crn
