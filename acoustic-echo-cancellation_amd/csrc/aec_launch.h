// aec_launch.h — kernel argument blocks and host launchers (internal).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "aec_fft.h"
#include "aec_knobs.h"

namespace aec {

constexpr int kFPB = 16;            // frames per analysis / synthesis block (16 groups x 16 lanes)
constexpr int kHopsOut = kFPB - 1;  // output hops per synthesis block
constexpr int kCH = 16;             // frames per chunk in the GRU pipeline
constexpr int kMomChunks = 8;       // moment partials per (stream, signal)

constexpr int kAnalysisBlocksPerCU = 3;
constexpr int kWeights = 12544;     // Little_net parameter blob (state_dict order, include/aec_hip.h)

// One analysis work item: 4 consecutive frames [wt, wt+4) of stream b (length n).
struct WorkItem {
    int32_t b;
    int32_t wt;
    int64_t n;
};

struct AnalysisArgs {
    const float* sig[3];
    int64_t ld;
    const WorkItem* items;   // host-built list (valid items only)
    int64_t nitems;
    int num_cus;
    const float* cvals;      // [B][3] normaliser scalars, or null: computed from mom (the NLMS split path
                             // without a look-ahead; norm_finalize_kernel's expression, the same bits)
    const double2* mom;      // [B][3][kMomChunks] moment partials (read when cvals is null)
    const int32_t* slen;     // [B][4] per-signal lengths (mic, ref, near, -); mic = the item's n
    const float* tables;     // DevTables
    const float* sched;      // ERB schedule: float4[L][16] then int2[32] (aec_tables.h)
    int sched_len;           // L (multiple of 4)
    int nsig;
    float* feats;            // [B][Tmax][96]
    int64_t Tmax;
    float2* rows;            // small-batch NLMS path: packed spectrum rows [B][Tmax][2][256] of mic and
                             // ref (slot 0 = (X[0], X[256])), or null
};

// K2n: per-stream analysis with the FD-NLMS canceller (one block per stream).
struct NlmsArgs {
    const float* sig[3];
    int64_t ld;
    const int64_t* lens;
    const int32_t* slen;     // [B][4] per-signal lengths (mic, ref, near, -)
    int b0;                  // first stream of this launch (block i runs stream b0 + i)
    const float* cvals;
    const float* tables;
    const float* sched;
    int sched_len;
    int nsig;
    float* feats;            // [B][Tmax][96]
    int64_t Tmax;
    float2* spec;            // [B][Tmax][256] error spectrum E (slot 0 = (E[0], E[256]))
    int taps;
    float mu, beta, delta;
    int prio;                // wave priorities (AEC_NLMS_PRIO, decimal digits mic|ref|nlms, 0..3 each)
    int erb_role;            // waves that run the mic_erb pass: 0 mic if no near (else ref), 1 ref, 2 nlms
    int mode;                // timing experiments only (AEC_NLMS_MODE): bit0 skip recursion,
                             // bit1 skip near transform, bit2 skip mic ERB, bit3 skip mic/ref transforms;
                             // bit4 (valid results): the ref waves' two ERB projections in two passes
};

struct GruArgs {
    const float* feats;      // [B][Tmax][96]
    int64_t Tmax;
    const int64_t* lens;
    const float* w;          // weights blob (state_dict order)
    float* est;              // [B][Tmax][32]
    float* loss;             // [B] or null
    int has_near;
    float* dbg_h;            // [B][Tmax][32] or null
    float* dbg_mask;         // [B][Tmax][32] or null
    int mode;                // timing experiments only: 0 full, 1 recurrence only, 2 helpers only
    int b0;                  // first stream of this launch (block i runs stream b0 + i)
};

struct SynthArgs {
    const float* mic;
    int64_t ld;
    const WorkItem* items;   // host-built list: (b, first output hop h0, n), h0 += 15
    int64_t nitems;
    int num_cus;
    const float* cvals;
    const float* tables;
    const float* bintab;     // float4[257]: (band_a, w_a, band_b, w_b) per bin
    const float* est;        // [B][Tmax][32]
    int64_t Tmax;
    float* out;
    int64_t ld_out;
    const float2* spec;      // NLMS error spectrum [B][Tmax][256], or null: re-derive the mic spectrum
    int fmode;               // fused kernel timing experiments only (AEC_FUSED_MODE; results invalid
                             // unless 0): bit0 skip the synthesis, bit1 skip the OLA, bit2 skip the E loads
    unsigned long long wmap; // A/B builds only: role wave of hardware wave i = (wmap >> 4 i) & 15 (0: identity)
    int64_t spec_stride;     // gru_synth: float2 per frame of `spec` (0: 256, the E rows; 512: K2's packed
                             // mic / ref rows, the bypass path's mic spectrum)
};

// Fused streaming step (aec_stream.hip): one 256-sample hop of B streams.
// Per-stream state, floats (stride = stream_state_floats(taps)):
//   [0, 512)     previous input hop: mic (256), ref (256)
//   [512, 768)   OLA tail: second half of the previous synthesis frame
//   [768, 800)   GRU h
//   [1024, ...)  NLMS, float2[2*taps][256] by field: w[0..taps-1],
//                far-end history r[t-1 .. t-taps+1], power p
constexpr int kStPrev = 0;
constexpr int kStTail = 512;
constexpr int kStH = 768;
constexpr int kStNlms = 1024;
inline int64_t stream_state_floats(int taps) { return 1024 + (int64_t)1024 * taps; }

struct StreamStepArgs {
    const float* mic;        // [B][ld_in] hop k of every stream
    const float* ref;
    int64_t ld_in;
    float* out;              // [B][ld_out] output hop k-1
    int64_t ld_out;
    float* state;            // [B][state_stride]
    int64_t state_stride;
    const float* w;          // weights blob
    const float* tables;     // DevTables
    const float* sched;
    int sched_len;
    const float* bintab;
    float mu, beta, delta;
};

// dynamic LDS bytes (must match the carve in the kernels)
inline size_t analysis_smem_bytes(int sched_len) {
    return (size_t)sched_len * 16 * 16 + 32 * 8 + (258 * 2 + 256 * 2 + 512 + (size_t)kFPB * kGroupFloats) * 4;
}
// K2n: tables + 8 wave regions (mic, ref waves; the nlms waves keep their
// state in registers) + 2 x 16 error rows of 560 floats
#ifndef AEC_NLMS_MAGROW
#define AEC_NLMS_MAGROW 1
#endif
inline size_t nlms_smem_bytes(int sched_len, int /*taps*/) {
    // error rows: |E| rows of 288 + 48 floats (AEC_NLMS_MAGROW), or E rows of 512 + 48
    return (size_t)sched_len * 16 * 16 + 32 * 8 +
           (258 * 2 + 256 * 2 + 512 + (size_t)8 * 4 * kGroupFloats + (size_t)2 * kFPB * (AEC_NLMS_MAGROW ? 336 : 560)) * 4;
}
inline size_t synthesis_smem_bytes() {
    return 260 * 16 + (258 * 2 + 256 * 2 + 512 + 256 + kFPB * 33 + 4 + (size_t)kFPB * kGroupFloats) * 4;
}

// slen: [B][4] per-signal lengths (mic, ref, near, -)
hipError_t launch_moments(const float* mic, const float* ref, const float* near, int64_t ld,
                          const int32_t* slen, double2* mom, int b0, int nb, int nsig, hipStream_t st);
hipError_t launch_norm_finalize(const double2* mom, const int32_t* slen, float* cvals, int b0, int b1, int nsig,
                                hipStream_t st);
hipError_t launch_analysis(const AnalysisArgs& a, hipStream_t st);
hipError_t launch_nlms_analysis(const NlmsArgs& a, int nb, hipStream_t st);
// small-batch NLMS path (few streams: the per-stream K2n block would leave the
// chip idle): K2 with spectrum rows, then the recursion per (stream, bin) and
// the mic_erb pass over all frames
hipError_t launch_nlms_recursion(const float2* rows, float2* spec, const int64_t* lens, int64_t Tmax, int taps,
                                 float mu, float beta, float delta, int b0, int nb, float2* dummy_rows, hipStream_t st);
hipError_t launch_mic_erb(const float2* spec, float* feats, const int64_t* lens, int64_t Tmax, const float* sched,
                          int sched_len, const WorkItem* items, int64_t nitems, hipStream_t st);
hipError_t launch_gru(const GruArgs& a, int B, hipStream_t st);
hipError_t launch_synthesis(const SynthArgs& a, hipStream_t st);
hipError_t launch_stream_step(const StreamStepArgs& a, int B, int taps, hipStream_t st);
// K3+K4 fused (aec_gru_synth.hip): GRU + head + synthesis of the NLMS error spectrum
hipError_t launch_gru_synth(const GruArgs& g, const SynthArgs& y, int B, hipStream_t st);
// Small-batch pipeline: the split path's NLMS recursion and mic_erb run in producer blocks of the
// GRU + synthesis launch (gru_synth_kernel<1, true>), chunk by chunk ahead of the recurrence
struct PipeArgs {
    const float2* rows;               // K2's packed mic / ref rows [B][Tmax][2][256]
    float2* spec;                     // E rows [B][Tmax][256] (out)
    float* feats;                     // mic_erb = feats[b][t][0:32] (out)
    const float* sched;               // ERB schedule (aec_tables.h)
    int sched_len;
    float mu, beta, delta;
    unsigned long long* progress;     // [B]: (epoch << 32) | chunks of the stream published
    unsigned long long epoch;         // this launch's epoch (per handle, increasing)
    int* err;                         // host-mapped word: a consumer wave gave up waiting
    int spin_limit;                   // polls (s_sleep 1 each) before giving up
    int stall;                        // test hook (AEC_SMALLB_PIPE_STALL): producers never publish
};
constexpr int kPipeTaps = 4;          // the one tap count the pipeline is instantiated for
hipError_t launch_gru_synth_pipe(const GruArgs& g, const SynthArgs& y, const PipeArgs& q, int B, hipStream_t st);
size_t gru_synth_smem_bytes();

// Training step (aec_train.hip): the backward of Little_net's loss through the
// head and the GRU for a padded batch of B rows of T frames each.
struct TrainArgs {
    const float* feats;      // [B][Tmax][96] mic_erb | ref_erb | near_erb (forward)
    const float* h;          // [B][Tmax][32] GRU outputs (forward)
    const float* w;          // weights blob
    float* rec;              // [B*T][8][32] per-frame record (T1)
    float* dg;               // [B*T][4][32] gate gradients (T2)
    float* part;             // [nblk][kWeights] weight-gradient partials (T3)
    int B, T;
    int64_t Tmax;
    int num_cus;
    float* scan_p;           // chunked-scan BPTT (null: the serial kernel): [B][chunks][32][32] chunk maps,
    float* scan_q;           //   [B][chunks][32] offsets,
    float* scan_g;           //   [B][chunks][32] g at each chunk's first step
};
int train_scan_chunks(int T);
hipError_t launch_norm_global(const double2* mom, int B, int64_t n, float* cvals, hipStream_t st);
int train_wgrad_blocks(int B, int T, int num_cus);
hipError_t launch_train_backward(const TrainArgs& a, int nblk, const float* grad_loss, float* grad, hipStream_t st);
hipError_t launch_loss_sum(const float* per_stream, int B, float* loss, hipStream_t st);
constexpr int kAdamMax = 16;
struct AdamList {                // up to kAdamMax tensors of one param group
    float* p[kAdamMax];
    const float* g[kAdamMax];
    float* m[kAdamMax];
    float* v[kAdamMax];
    float step_size[kAdamMax];   // lr / (1 - beta1^step)
    float bc2_sqrt[kAdamMax];    // sqrt(1 - beta2^step)
    int64_t off[kAdamMax + 1];   // element offsets (off[0] = 0)
    int n;
};
hipError_t launch_adam_multi(const AdamList& L, float beta1, float beta2, float eps, float wd, hipStream_t st);
hipError_t launch_adam(float* prm, const float* grad, float* m, float* v, int64_t n, float beta1, float beta2,
                       float eps, float wd, float step_size, float bc2_sqrt, hipStream_t st);

}  // namespace aec
