/*
 * aec_hip.h — C ABI of libaec_hip.so, the MI355X (gfx950) Stage-2 AEC hot path.
 *
 * Drop-in boundary for the reference's Stage-2 inference path
 * (SZU-Speech/Acoustic-Echo-Cancellation, Stage2_lhm/):
 *
 *   aec_create / aec_set_weights / aec_set_erb
 *        replace  Little_net.__init__ + net.load_state_dict(...)
 *                 (scripts/network/ERB.py:204-229, scripts/test.py:102-124)
 *                 and the ERB matrix upload (scripts/test.py:108-111).
 *   aec_process
 *        replaces Little_net.forward(mic, ref, near, erb) -> (out_wav, loss)
 *                 (scripts/network/ERB.py:252-334) as called at
 *                 scripts/test.py:157, with batch=1 semantics per stream
 *                 (per-stream normaliser over its true length).
 *   aec_debug_copy
 *        exposes the intermediates the reference computes inside forward
 *        (ERB.py:282-307) for parity tests.
 *
 * Conventions: plain pointers and sizes only.  Signal / output / loss
 * pointers are DEVICE pointers (e.g. torch tensor data_ptr()); weights, ERB
 * matrix and lengths are HOST pointers.  `stream` is a hipStream_t passed as
 * void* (NULL = the null stream).  Calls are asynchronous on `stream`.
 * Errors are integer status codes; no exceptions cross the ABI;
 * aec_last_error() describes the last failure on a handle.
 * One handle per device; calls on one handle must be serialised by the caller.
 */
#ifndef AEC_HIP_H
#define AEC_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    AEC_OK = 0,
    AEC_ERR_INVALID_ARG = 1,
    AEC_ERR_OOM = 2,
    AEC_ERR_HIP = 3,
    AEC_ERR_UNSUPPORTED = 4
} aec_status;

typedef struct aec_handle aec_handle;

/* Mirrors speech_conf/erb_conf (scripts/configs.py:1-8,21-27) + the
 * build-defined FD-NLMS stage (no reference counterpart; nlms_taps = 0 is the
 * reference-parity bypass). */
typedef struct {
    int32_t win_size;    /* 512  (speech_conf['win_size'])  — only 512 supported  */
    int32_t hop_size;    /* 256  (speech_conf['hop_size'])  — only 256 supported  */
    int32_t erb_bands;   /* 32   (erb_conf['total_erb_bands']); GRU hidden = bands */
    int32_t nlms_taps;   /* 0 = bypass; 1..8 taps per bin (frames of far-end history) */
    float   nlms_mu;     /* step size, [0, 2); 0 leaves the mic spectrum unchanged    */
    float   nlms_beta;   /* far-end power smoothing, [0, 1)                           */
    float   nlms_delta;  /* regulariser, > 0                                          */
    int32_t reserved;
} aec_config;

/* Number of floats in the weights blob: the reference state_dict parameters
 * concatenated in state_dict order (gru1.weight_ih_l0 [96,64],
 * gru1.weight_hh_l0 [96,32], gru1.bias_ih_l0 [96], gru1.bias_hh_l0 [96],
 * linear1.weight [32,64], linear1.bias [32], linear2.weight [32,32],
 * linear2.bias [32]) = 12,544 for 32 bands. */
size_t aec_weights_count(int32_t erb_bands);

/* Create a handle on `device`.  weights: host blob (see above, may be NULL =
 * zeros, set later); erb_257x32: host [257, bands] float32 row-major (may be
 * NULL = set later). */
aec_status aec_create(const aec_config* cfg, const float* weights, size_t n_weights,
                      const float* erb_257xbands, int32_t device, aec_handle** out);
/* With nlms_taps > 0 every frame's mic spectrum is first replaced by the
 * a-priori error of a per-bin complex NLMS driven by the ref spectrum
 *   E = D - sum_l W[l] R[t-l],  P = beta P + (1-beta) sum_l |R[t-l]|^2,
 *   W[l] += mu E conj(R[t-l]) / (P + delta)      (W, P = 0 at each stream start)
 * and the post-filter (features, gains, iSTFT) runs on E instead of the mic
 * spectrum. */

aec_status aec_set_weights(aec_handle* h, const float* weights, size_t n_weights);
aec_status aec_set_erb(aec_handle* h, const float* erb_257xbands);

/* Run the whole hot path for B streams.
 *   mic, ref : device [B, ld]   float32 (row b holds lengths[b] valid samples)
 *   near     : device [B, ld]   float32 or NULL (then no loss is computed)
 *   lengths  : host   [B]       int64, each in [1, ld]
 *   out      : device [B, ld_out] float32; row b receives 256*(lengths[b]/256)
 *              samples (the reference's output length), the rest is untouched;
 *              may be NULL when every length is < 256 (empty outputs)
 *   loss     : device [B] float32 or NULL; loss[b] = sum_{t,j}
 *              (near_erb^0.5 - est_erb^0.5)^2 / (T_b * bands)   (ERB.py:318-323)
 */
aec_status aec_process(aec_handle* h, const float* mic, const float* ref, const float* near,
                       const int64_t* lengths, int32_t B, int64_t ld,
                       float* out, int64_t ld_out, float* loss, void* stream);

/* aec_process with a length per signal, as scripts/test.py feeds the
 * reference (test.py:139: default collate at batch 1, every signal at its
 * stored length): each signal is normalised over, and zero-padded beyond, its
 * own length (ERB.py:254-256, attention_ccrn.py:48).  The mic length sets the
 * frame count and the output length; ref / near must have the same frame
 * count N//256 + 1 (the reference's frame-wise concat / loss raise otherwise,
 * ERB.py:287-290, 318-323) — AEC_ERR_INVALID_ARG here.
 *   lengths3 : host [B][3] int64 (mic, ref, near); near's entry is ignored when
 *              near is NULL */
aec_status aec_process_siglens(aec_handle* h, const float* mic, const float* ref, const float* near,
                               const int64_t* lengths3, int32_t B, int64_t ld,
                               float* out, int64_t ld_out, float* loss, void* stream);

/* Optional look-ahead (serving): queue the per-stream normaliser pass of a batch
 * (c = mean/std of each signal over its length, ERB.py:254-256 — a full read of
 * every signal before the first frame can be normalised) on `stream`, ahead of
 * the aec_process_prepared call that will take the batch.  *token (non-NULL)
 * receives the look-ahead's identity; only aec_process_prepared with that token
 * consumes it (on any stream: it waits for the pass on the device instead of
 * running it).  aec_process / aec_process_siglens never consume a look-ahead, so
 * a buffer refilled at the same address is never normalised with stale
 * constants by accident.  At most two look-aheads may be pending per handle
 * (AEC_ERR_INVALID_ARG beyond).  The caller guarantees that the signals are
 * unchanged between the two calls (the pass reads them when it runs on
 * `stream`).  Outputs are bit-identical with and without the look-ahead (the
 * same kernels).  No reference counterpart: the reference computes the
 * normaliser inside Little_net.forward (ERB.py:254-256).
 *   lengths3 : host [B][3] int64, as aec_process_siglens (aec_prepare: one
 *              length per stream, [B]) */
aec_status aec_prepare_siglens(aec_handle* h, const float* mic, const float* ref, const float* near,
                               const int64_t* lengths3, int32_t B, int64_t ld, void* stream, uint64_t* token);
aec_status aec_prepare(aec_handle* h, const float* mic, const float* ref, const float* near,
                       const int64_t* lengths, int32_t B, int64_t ld, void* stream, uint64_t* token);
/* aec_process_siglens taking the look-ahead `token` names: the pending
 * look-aheads queued before it are dropped, and the call fails
 * (AEC_ERR_INVALID_ARG, nothing launched) when the token is not pending or was
 * prepared for other signal pointers, ld, B or lengths. */
aec_status aec_process_prepared(aec_handle* h, uint64_t token, const float* mic, const float* ref, const float* near,
                                const int64_t* lengths3, int32_t B, int64_t ld, float* out, int64_t ld_out,
                                float* loss, void* stream);

/* Streaming (serving): the reference's per-frame loop (Little_net.forward,
 * ERB.py:252-334) advanced by one 256-sample hop per stream per call, as ONE
 * fused kernel launch (frame -> rFFT -> [FD-NLMS] -> ERB -> GRU step -> head
 * -> gains -> irFFT -> overlap-add).  Frame t needs hops t-1 and t
 * (ConvSTFT framing, attention_ccrn.py:45-52), so step k emits output hop
 * k-1; the first step's output is the warm-up region the reference trims
 * (attention_ccrn.py:99).  Feeding hops 0 .. n/256 (the last one zero-padded
 * past n) reproduces aec_process's out row for that stream.  The hops must
 * already be normalised: x - mean(x)/std(x) (ERB.py:254-256) needs the whole
 * utterance, which a stream does not have; near / loss are not computed.
 *   aec_stream_open(h, B)        B concurrent streams; state zeroed
 *   aec_stream_reset(h, b, st)   zero stream b's state (-1: all streams)
 *   aec_stream_step(h, mic, ref, ld_in, out, ld_out, st)
 *        mic, ref: device [B, ld_in] float32, hop k of every stream;
 *        out: device [B, ld_out] float32 receives output hop k-1 (256 samples). */
aec_status aec_stream_open(aec_handle* h, int32_t B);
aec_status aec_stream_reset(aec_handle* h, int32_t b, void* stream);
aec_status aec_stream_step(aec_handle* h, const float* mic, const float* ref, int64_t ld_in,
                           float* out, int64_t ld_out, void* stream);

/* Debug / parity: copy an intermediate of the LAST aec_process call into the
 * device buffer dst ([B, T_max, 32] float32, frames beyond a stream's T left
 * unspecified).  Requires aec_set_debug(h, 1) before that call.
 * what: 0 = mic_erb, 1 = ref_erb, 2 = near_erb, 3 = gru_out (h_t),
 *       4 = mask, 5 = est_erb. */
aec_status aec_set_debug(aec_handle* h, int32_t enable);
aec_status aec_debug_copy(aec_handle* h, int32_t what, float* dst, size_t n_floats, void* stream);

/* Kernel timing: when enabled, aec_process records a HIP event before and
 * after each of its kernels on `stream`.  aec_profile_read waits for those
 * events, returns the summed milliseconds per kernel (ms[0..3] = moments,
 * analysis, gru, synthesis) over all calls since the previous read and the
 * number of calls, and clears the record. */
aec_status aec_profile_enable(aec_handle* h, int32_t enable);
aec_status aec_profile_read(aec_handle* h, double* ms4, int64_t* calls);

/* Host-side check of the ERB tables the device uses (no GPU needed): builds
 * the forward schedule / transpose table for erb_257xbands exactly as
 * aec_set_erb does and applies them on the CPU:
 *   bands[32]  = schedule applied to mags[257]   (== mags @ erb, ERB.py:282)
 *   gains[257] = transpose table applied to est[32] (== est @ erb^T, ERB.py:306)
 * Returns the schedule length per lane in *sched_len and the number of
 * schedule entries whose LDS read could not be placed on a distinct bank
 * residue in *conflicts. */
aec_status aec_erb_tables_check(const float* erb_257xbands, const float* mags, const float* est,
                                float* bands, float* gains, int32_t* sched_len, int32_t* conflicts);

/* Training step: replaces one iteration of
 * Trainer.train (scripts/train1.py:191-218) — net(mic, far, near, erb) on a
 * collate_fn-padded batch (train1.py:43-74), loss.backward(), Adam.step()
 * (train1.py:153).
 *   aec_set_weights_device(h, w, n, st)
 *        the 12,544-float blob from DEVICE memory, copied on `stream` (the
 *        parameters of a training loop stay on the device).
 *   aec_train_forward(h, mic, ref, near, n, B, ld, out, ld_out, loss, st)
 *        Little_net.forward (ERB.py:252-334) in training semantics: B rows of
 *        n samples each (already zero-padded, as collate_fn pads), ONE
 *        normaliser scalar per signal over the whole [B, n] batch
 *        (ERB.py:254-256), *loss (device, 1 float) = the reference's batch
 *        loss (ERB.py:318-323, summed over rows).  out (nullable) receives the
 *        [B, 256*(n//256)] enhanced waveforms.  Keeps what the backward needs
 *        in the handle (nlms_taps must be 0: the reference network).
 *   aec_train_backward(h, grad_loss, grad, st)
 *        loss.backward() for the last aec_train_forward: grad (device, 12,544
 *        floats, blob order) = grad_loss * d loss / d params; grad_loss is a
 *        device scalar (NULL = 1).  An aec_process / aec_process_siglens call
 *        in between overwrites the forward's features: the backward then
 *        fails with AEC_ERR_INVALID_ARG.
 *   aec_train_generation(h)
 *        count of aec_train_forward calls (an autograd binding checks that
 *        its backward belongs to the latest forward).
 *   aec_adam_step(h, params, grad, exp_avg, exp_avg_sq, n, step, lr, beta1,
 *                 beta2, eps, weight_decay, st)
 *        torch.optim.Adam (amsgrad = False) over n device floats at 1-based
 *        `step` (train1.py:153 builds Adam(lr = train_conf['lr'])). */
aec_status aec_set_weights_device(aec_handle* h, const float* weights_dev, size_t n_weights, void* stream);
aec_status aec_train_forward(aec_handle* h, const float* mic, const float* ref, const float* near, int64_t n,
                             int32_t B, int64_t ld, float* out, int64_t ld_out, float* loss, void* stream);
aec_status aec_train_backward(aec_handle* h, const float* grad_loss, float* grad, void* stream);
int64_t aec_train_generation(const aec_handle* h);
aec_status aec_adam_step(aec_handle* h, float* params, const float* grad, float* exp_avg, float* exp_avg_sq,
                         size_t n, int64_t step, float lr, float beta1, float beta2, float eps, float weight_decay,
                         void* stream);
/* The same update over `count` tensors (one param group) in one launch per 16
 * tensors: host arrays of device pointers, element counts and 1-based steps. */
aec_status aec_adam_step_multi(aec_handle* h, float* const* params, const float* const* grads, float* const* exp_avg,
                               float* const* exp_avg_sq, const int64_t* sizes, const int64_t* steps, int32_t count,
                               float lr, float beta1, float beta2, float eps, float weight_decay, void* stream);

/* Frame / output-length integers (bit-exact framing contract). */
int64_t aec_num_frames(int64_t n_samples);   /* n//256 + 1 */
int64_t aec_out_len(int64_t n_samples);      /* 256*(n//256) */

const char* aec_last_error(const aec_handle* h);

/* Build description of this library (no reference counterpart: bench and test
 * provenance).  "arch=gfx950 ab_knobs=off mode_knobs=<names>": ab_knobs=on marks
 * an A/B build (-DAEC_AB_KNOBS) that reads timing-only / work-skipping knobs;
 * mode_knobs lists the environment variables that select tested modes. */
const char* aec_build_info(void);
void aec_destroy(aec_handle* h);

#ifdef __cplusplus
}
#endif
#endif /* AEC_HIP_H */
