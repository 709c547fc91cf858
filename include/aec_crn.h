/*
 * aec_crn.h — C ABI of the DCCRN (complex CRN) post-filter in libaec_hip.so.
 *
 * Drop-in boundary for the reference's two complex CRNs
 * (SZU-Speech/Acoustic-Echo-Cancellation, Stage2_lhm/scripts/network/):
 *
 *   aec_crn_create / aec_crn_set_params
 *        replace  DCCRN(config) + load_state_dict(...) + eval()
 *                 (dccrn.py:453-521 — "version 1"; dccrn2.py:10-116 —
 *                 "version 2"; config dict = configs.net_conf, configs.py:29-46)
 *   aec_crn_process
 *        replaces DCCRN.forward(mic, far, near, echo) in eval mode:
 *                 v1 -> (out_wav, out_spec, near_specs, loss)  (dccrn.py:532-594)
 *                 v2 -> (out_spec, out_wav, near_specs)        (dccrn2.py:118-218)
 *                 for B utterances at batch=1 semantics (nothing couples
 *                 utterances in eval mode).  out_wav / out_spec / the mask
 *                 come from here; near_specs (and v1's echo spectrum for the
 *                 loss) from aec_crn_stft.
 *   aec_crn_stft
 *        replaces ConvSTFT.forward (dccrn.py:45-52) -> complex spectrum.
 *
 * Conventions as include/aec_hip.h: plain pointers and sizes; signal, output
 * and spectrum pointers are DEVICE pointers, params and lengths HOST
 * pointers; `stream` is a hipStream_t passed as void*; calls are
 * asynchronous on it; integer status codes (aec_status), aec_crn_last_error
 * describes the last failure.  One handle per device, calls serialised by
 * the caller.
 */
#ifndef AEC_CRN_H
#define AEC_CRN_H

#include <stddef.h>
#include <stdint.h>

#include "aec_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct aec_crn_handle aec_crn_handle;

/* Mirrors the config dict DCCRN reads (configs.net_conf, configs.py:29-46).
 * win_size 512 / hop_size 256 / kernel (5,1) / stride (2,1) / padding (2,0)
 * are fixed by the kernels.  Requirements: every conv_channels[i] a power of
 * two >= 4 (conv_channels[0] == 4: mic/far real/imag), 256 >> n_layers == 4
 * (the LSTM width the reference hard-codes), v2: hidden_dim == 4, use_clstm. */
typedef struct {
    int32_t version;            /* 1 = network/dccrn.py DCCRN, 2 = network/dccrn2.py DCCRN   */
    int32_t n_layers;           /* len(conv_channels) - 1                                    */
    int32_t conv_channels[9];
    int32_t hidden_dim;         /* v2 */
    int32_t rnn_layers;         /* v2: number of NavieComplexLSTM layers                     */
    int32_t use_cbn;            /* v2: ComplexBatchNorm (1) or BatchNorm2d (0)               */
    int32_t masking_mode;       /* v2: 'E', 'C' or 'R' (character code); v1 uses 'C'         */
    int32_t dtype;              /* compute / storage type: 0 = float32, 1 = bfloat16,
                                   2 = bfloat16 with MX-fp8 GEMMs (OCP e4m3 weights and
                                   activations, E8M0 scale per 32 k) for the LSTM input
                                   projections and every conv layer whose implicit rows
                                   allow it (input channels % 32 == 0, K % 128 == 0,
                                   output channels >= 128: encoder 4-5 and decoder levels
                                   5-6 of net_conf); needs H % 128 == 0 and
                                   H / (256 >> n_layers) % 32 == 0                         */
    /* Build-defined FD-NLMS front end (no reference counterpart; SURVEY.md §8
     * a13 + a14, the Stage-2 "NLMS -> CRN" composition).  nlms_taps = 0 is the
     * reference-parity network.  With nlms_taps > 0 every frame's mic spectrum
     * X_mic is replaced by the a-priori error E of the per-bin complex NLMS of
     * aec_hip.h (same recursion, same parameter meaning) driven by the far
     * spectrum; E feeds the encoder's mic channels AND is the spectrum the
     * decoder's mask is applied to (out_spec / out_wav).  The far channels
     * stay X_far.  Streaming carries the NLMS state per stream. */
    int32_t nlms_taps;          /* 0 = off; 1..8 */
    float   nlms_mu;            /* [0, 2)  */
    float   nlms_beta;          /* [0, 1)  */
    float   nlms_delta;         /* > 0     */
} aec_crn_config;

/* Number of floats in the parameter blob: the reference state_dict entries
 * the eval forward reads, concatenated in this order (each tensor row-major):
 *   encoder.{i}.0.{real_conv,imag_conv}.{weight,bias}, then the norm
 *     (v2 + use_cbn: encoder.{i}.1.{Wrr,Wri,Wii,Br,Bi,RMr,RMi,RVrr,RVri,RVii};
 *      otherwise encoder.{i}.1.{weight,bias,running_mean,running_var}),
 *     then encoder.{i}.2.weight (PReLU), for i = 0 .. n_layers-1;
 *   decoder.{d}.0.{real_conv,imag_conv}.{weight,bias} + norm + PReLU for
 *     d = 0 .. n_layers-2; the last decoder block: its conv, and for v1 its
 *     BatchNorm2d(2) (decoder.{d}.1.*);
 *   v1: lstm.{weight_ih_l0, weight_hh_l0, bias_ih_l0, bias_hh_l0};
 *   v2: enhance.{l}.{real_lstm,imag_lstm}.{weight_ih_l0, weight_hh_l0,
 *       bias_ih_l0, bias_hh_l0} for l = 0 .. rnn_layers-1.
 * (The STFT buffers are closed-form and num_batches_tracked is unused.)
 * Returns 0 for an unsupported config. */
size_t aec_crn_param_count(const aec_crn_config* cfg);

aec_status aec_crn_create(const aec_crn_config* cfg, const float* params, size_t n_params, int32_t device,
                          aec_crn_handle** out);
aec_status aec_crn_set_params(aec_crn_handle* h, const float* params, size_t n_params);

/* Run the CRN for B utterances.
 *   mic, far : device [B, ld] float32, row b holds lengths[b] samples
 *   lengths  : host [B] int64, each in [1, ld]; T_b = lengths[b]/256 + 1,
 *              Tmax = max T_b
 *   out      : device [B, ld_out] float32: row b receives 256*(lengths[b]/256)
 *              samples (out_wav); may be NULL when every length is < 256
 *   spec     : device [B, Tmax, 257] float2 or NULL: the masked spectrum
 *              (out_spec; frames t >= T_b unspecified)
 *   mask     : device [B, Tmax, 256, 2] float32 or NULL: the decoder output
 *              for bins 1..256 (mask_real, mask_imag before F.pad)
 * Host blocking: with the persistent LSTM recurrence (bf16 / fp8, the
 * default when the grid fits the device) the call returns only after the
 * LSTM stage has run on `stream` (its error word is read back, so a
 * timed-out grid fails this call); the decoder and back kernels are queued
 * and run asynchronously.  After two consecutive timed-out calls the handle
 * switches to the per-frame step kernel for good (AEC_CRN_PERSIST=0 does
 * that from the start). */
aec_status aec_crn_process(aec_crn_handle* h, const float* mic, const float* far, const int64_t* lengths, int32_t B,
                           int64_t ld, float* out, int64_t ld_out, float* spec, float* mask, void* stream);

/* NLMS handles (nlms_taps > 0): the FD-NLMS error spectrum E of the last
 * aec_crn_process call -> device [B, Tmax, 257] float2 (frames t >= T_b zero),
 * the spectrum the mask was applied to (the v1 loss's cRM reference,
 * dccrn.py:556-566, when the network is fed E). */
aec_status aec_crn_error_spec(aec_crn_handle* h, float* spec, void* stream);

/* ConvSTFT of B signals -> device [B, Tmax, 257] float2 (frames t >= T_b zero). */
aec_status aec_crn_stft(aec_crn_handle* h, const float* x, const int64_t* lengths, int32_t B, int64_t ld,
                        float* spec, void* stream);

/* Streaming (serving): one 256-sample hop per stream per call, the per-frame
 * loop of the same network (the DCCRN has no utterance-global statistic, so a
 * streamed utterance equals the batch result: frame t needs hops t-1 and t,
 * ConvSTFT framing dccrn.py:45-52).  Per handle, the launches of one frame
 * go out directly (mode 0, the default) or are captured once per ring parity
 * in a hipGraph and replayed (mode 1: aec_crn_stream_set_graph, or
 * AEC_CRN_GRAPH=1 in the environment when aec_crn_stream_open runs); both
 * modes give bit-identical outputs, and a graph that cannot be captured or
 * instantiated fails the step with AEC_ERR_HIP (no silent fallback).
 * 7 launches for the fp8 step at net_conf (fused front = STFT, FD-NLMS and
 * encoder levels 0-4; one MX conv level; two LSTM layer steps; two MX conv
 * levels; fused back = decoder levels 4-1, mask, iSTFT).  The fp8 step folds
 * encoder / decoder level 4 into the fused kernels only while B <= the
 * device's CU count (above that they are separate launches; the results are
 * bit-identical either way).
 *   aec_crn_stream_open(h, B)        B concurrent streams; state zeroed
 *   aec_crn_stream_reset(h, b, st)   zero stream b's state (-1: all, and the hop counter)
 *   aec_crn_stream_step(h, mic, far, ld_in, out, ld_out, st)
 *        mic, far: device [B, ld_in] float32, hop k of every stream (samples
 *        256k .. 256k+255; zero-pad a final partial hop);
 *        out: device [B, ld_out] float32 receives output hop k-1 (the
 *        reference's out_wav[256(k-1) : 256k]); the output of a stream's first
 *        step is the warm-up region the reference trims (dccrn.py:99), and
 *        one extra all-zero hop after the last input hop flushes the final
 *        output hop. */
aec_status aec_crn_stream_open(aec_crn_handle* h, int32_t B);
aec_status aec_crn_stream_reset(aec_crn_handle* h, int32_t b, void* stream);
aec_status aec_crn_stream_step(aec_crn_handle* h, const float* mic, const float* far, int64_t ld_in, float* out,
                               int64_t ld_out, void* stream);
/* Per-hop launch mode of the open streams: 0 = direct launches, 1 = hipGraph
 * replay (the per-frame step of BASELINE config 5, dccrn2.py:118-218 per hop).
 * Switching synchronises the device and drops the captured graphs; the stream
 * state is kept. */
aec_status aec_crn_stream_set_graph(aec_crn_handle* h, int32_t mode);
/* The mode in effect and how many hops ran as graph replays / direct launches
 * since aec_crn_stream_open (any pointer may be NULL). */
aec_status aec_crn_stream_stats(const aec_crn_handle* h, int32_t* graph_mode, int64_t* graph_replays,
                                int64_t* direct_hops);

/* Kernel timing (HIP events on `stream`): ms[0..4] = front, encoder,
 * lstm (input projection + steps + combine), decoder, back; summed over the
 * calls since the previous read. */
aec_status aec_crn_profile_enable(aec_crn_handle* h, int32_t enable);
aec_status aec_crn_profile_read(aec_crn_handle* h, double* ms5, int64_t* calls);

const char* aec_crn_last_error(const aec_crn_handle* h);
void aec_crn_destroy(aec_crn_handle* h);

#ifdef __cplusplus
}
#endif
#endif /* AEC_CRN_H */
