/*
 * ba3c.h — C ABI of the MI355X-native BA3C learner/predictor hot path (libba3c.so).
 *
 * Plain pointers and sizes only: every data buffer is owned by the caller (the Python
 * host allocates them with PyTorch-ROCm); the handle owns static configuration, a few HIP
 * events and a few KB of device memory allocated by ba3c_create (the tagged-partial words of
 * the fused clip + optimizer launch and of the one-launch bucket clip, the chained launches'
 * signal counters; without a device they stay unallocated and those launches fall back to
 * unchained ones).  One handle serves one stream at a time.  No other call allocates
 * device memory, none synchronises the stream except ba3c_probe_read, and none throws:
 * every entry returns a BA3C_* status and
 * ba3c_last_error() holds a thread-local message.  All device pointers must be 16-byte
 * aligned.  `stream` is a hipStream_t (NULL = default stream).
 *
 * Each entry point replaces one piece of the reference TF-1.2 graph / runtime
 * (paths relative to /root/reference/src):
 *   ba3c_forward        OpenAIGym/train.py:164-299 for is_training=False (towerp0:
 *                       'logitsT', 'pred_value'), served by OnlinePredictor._do_call
 *                       tensorpack_cpu/tensorpack/predict/base.py:80-92 and
 *                       MultiThreadAsyncPredictor predict/concurrency.py:172-219
 *   ba3c_train_grads    OpenAIGym/train.py:164-327 forward + A3C loss and TF autodiff
 *                       tensorpack_cpu/tensorpack/train/multigpu.py:85-86
 *   ba3c_clip_grads     OpenAIGym/train.py:329-330 MapGradient(clip_by_average_norm(.,0.1)),
 *                       applied per replica in train/base.py:206-217, multigpu.py:157
 *   ba3c_apply_update   OpenAIGym/train.py:582-597 optimizer.apply_gradients
 *                       (multigpu.py:194): Adam / RMSProp / GD / Momentum / Adagrad / Adadelta
 *   ba3c_sample         OpenAIGym/train.py:382 np.random.choice(len(p), p=p) given its draw u
 *   (gradient mean)     OpenAIGym/train.py:598-606 SyncReplicasOptimizer: the host
 *                       all-reduces the clipped flat gradient buffer over RCCL between
 *                       ba3c_clip_grads and ba3c_apply_update (grad_scale = 1/world).
 */
#ifndef BA3C_H
#define BA3C_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BA3C_OK 0
#define BA3C_ERR_INVALID 1  /* bad argument / shape / config */
#define BA3C_ERR_HIP 2      /* a HIP runtime call failed */

/* optimizer ids (OpenAIGym/train.py:583-597, run_job.py -o choices) */
#define BA3C_OPT_ADAM 0
#define BA3C_OPT_GD 1
#define BA3C_OPT_ADAGRAD 2
#define BA3C_OPT_ADADELTA 3
#define BA3C_OPT_MOMENTUM 4
#define BA3C_OPT_RMS 5

/* scalars written by ba3c_train_grads (double[BA3C_NUM_SCALARS]); names are the
 * TfDictOp keys of train/multigpu.py:193-205 */
#define BA3C_SC_COST 0
#define BA3C_SC_POLICY_LOSS 1    /* policy_loss*128/B              train.py:311 */
#define BA3C_SC_XENTROPY_LOSS 2  /* xentropy_loss*128/B*beta       train.py:315-316 */
#define BA3C_SC_VALUE_LOSS 3     /* value_loss*128/B               train.py:320 */
#define BA3C_SC_ADVANTAGE 4      /* mean(stop_grad(V)-R)           train.py:323 */
#define BA3C_SC_PRED_REWARD 5    /* mean(V)                        train.py:321 */
#define BA3C_SC_MAX_LOGIT 6      /* max(softmax)                   train.py:291 */
#define BA3C_SC_ACTIVE_RELUS 7   /* sum count_nonzero(relu outs)   train.py:271 */
#define BA3C_NUM_SCALARS 8

/* kernel ids for the timing probe */
#define BA3C_K_CONV0_FWD 0
#define BA3C_K_CONV1_FWD 1
#define BA3C_K_CONV2_FWD 2
#define BA3C_K_CONV3_FWD 3
#define BA3C_K_FC1_FWD 4
#define BA3C_K_HEADS 5
#define BA3C_K_FC1_DGRAD 6
#define BA3C_K_CONV3_DGRAD 7
#define BA3C_K_CONV2_DGRAD 8
#define BA3C_K_CONV1_DGRAD 9
#define BA3C_K_HEAD_WGRAD 10
#define BA3C_K_FC1_WGRAD 11
#define BA3C_K_CONV3_WGRAD 12
#define BA3C_K_CONV2_WGRAD 13
#define BA3C_K_CONV1_WGRAD 14
#define BA3C_K_CONV0_WGRAD 15
#define BA3C_K_WGRAD_REDUCE 16
#define BA3C_K_CLIP 17
#define BA3C_K_UPDATE 18
#define BA3C_K_SCALARS 19   /* TfDictOp scalar reduction (its own launch or a job of conv3's input-gradient launch) */
#define BA3C_NUM_KERNELS 20

typedef struct ba3c_handle ba3c_handle;

/* Network geometry — the flag surface of OpenAIGym/parse.py:9-70 / run_job.py:13-48. */
typedef struct ba3c_config {
  int32_t max_batch;         /* largest B any call on this handle passes (workspace sizing) */
  int32_t channels;          /* real input channels C = 4*--channels (4 or 12), train.py:95 */
  int32_t fc_neurons;        /* --fc_neurons F (multiple of 4*fc_splits) */
  int32_t fc_splits;         /* --fc_splits S  (train.py:216-229) */
  int32_t num_actions;       /* A = env action count (train.py:122), 1..31 */
  int32_t replace_with_conv; /* 1: --replace_with_conv True (default); 0: --use_normal_fc */
  int32_t ps;                /* --ps: number of legacy FC splits (train.py:230-243) */
} ba3c_config;

/* Hyper-parameters of one optimizer apply. Power terms are the TF float32 variables
 * beta1_power/beta2_power BEFORE this apply (beta^t at step t). */
typedef struct ba3c_opt_params {
  float lr, beta1, beta2, epsilon;    /* Adam (train.py:584) */
  float beta1_power, beta2_power;     /* Adam bias-correction state */
  float decay, momentum;              /* RMSProp (TF defaults 0.9 / 0.0), Momentum 0.9 */
  float rho;                          /* Adadelta (0.95) */
} ba3c_opt_params;

int ba3c_create(const ba3c_config* cfg, ba3c_handle** out);
void ba3c_destroy(ba3c_handle* h);
const char* ba3c_last_error(void);
int ba3c_version(void);

/* Flat parameter layout shared by params / grads / optimizer slots.  Tensor i is
 * name (checkpoint key, e.g. "conv0/W"), at float offset `offset`, `numel` elements in
 * TF layout (HWIO conv, [in,out] FC).  Offsets are 64-float aligned; gaps are zero. */
int ba3c_num_tensors(const ba3c_handle* h);
int ba3c_tensor_info(const ba3c_handle* h, int32_t i, const char** name, int64_t* offset,
                     int64_t* numel, int32_t shape[4], int32_t* ndim);
int64_t ba3c_flat_size(const ba3c_handle* h);
/* Bytes of scratch device memory a call with batch B needs (train=1: ba3c_train_grads). */
size_t ba3c_workspace_size(const ba3c_handle* h, int32_t batch, int32_t train);
/* Introspection of the workspace a call with batch B carved (for tests / debugging): byte
 * offset and size of an intermediate — "p0","p1","p2" pooled maps [B,H,W,C] fp32, "c0".."c2"
 * argmax codes (uint8, 0..3 = first max of the 2x2 window, 255 = max <= 0), "a3" [B,1600],
 * "h" [B,F], and in training "dh","dy3","dp2","dp1","dp0" gradients. */
int ba3c_workspace_tensor(const ba3c_handle* h, int32_t batch, int32_t train, const char* name,
                          int64_t* offset_bytes, int64_t* bytes);

/* Predictor: one forward of B uint8 [B,84,84,C] states.  probs = softmax(policy)
 * ('logits', train.py:288), probsT = softmax(policy*explore_factor) ('logitsT', :299),
 * value = 'pred_value' [B].  Any output pointer may be NULL. */
int ba3c_forward(ba3c_handle* h, void* stream, const float* params, const uint8_t* state,
                 int32_t batch, float explore_factor, void* workspace, float* probs,
                 float* probsT, float* value);

/* Learner: forward + A3C loss + backward for one tower.  Writes RAW (unclipped) gradients
 * of every tensor into `grads` (flat layout, fully overwritten incl. gaps) and
 * BA3C_NUM_SCALARS doubles into `scalars` (device memory, may be NULL).
 * action: int64 [B] in [0,A); futurereward: fp32 [B]. */
int ba3c_train_grads(ba3c_handle* h, void* stream, const float* params, const uint8_t* state,
                     const int64_t* action, const float* futurereward, int32_t batch,
                     float entropy_beta, void* workspace, float* grads, double* scalars);

/* ba3c_train_grads in two phases for data-parallel bucketing: phase 1 runs the
 * forward, the loss / scalars and the backward of the heads and fc1 and leaves THEIR gradient
 * tensors (tensors ba3c_bucket_tensor(h) .. end of the flat layout) final; phase 2 (same
 * arguments, same workspace) runs conv3..conv0 and finishes the rest.  Phase 0 = both = the
 * bit-identical ba3c_train_grads.  Between the phases the caller may clip and all-reduce the
 * fc1 + heads bucket while the conv layers run (the reference's per-variable PS pushes,
 * OpenAIGym/train.py:598-606).
 * Phase 3 = phase 0 with the final weight-gradient reduction left pending: the next
 * ba3c_apply_update(_dev) with fuse_clip on the same handle, stream and `grads` runs it and the
 * clip + update as ONE chained launch (a launch fewer per step, but measured 4 us slower at
 * configs[1]: the trainer uses it only with BA3C_DEFER_REDUCE=1); any other entry
 * point on the handle (forward, train, clip, an unfused or mismatched apply, device_errors)
 * first launches it on the pass's stream (a call on another stream then waits for it).  `grads` holds the raw gradients only after that.
 * Phase 4 = phase 1 with the fc1 + heads reduction HELD: nothing launches it until
 * ba3c_launch_held(h, stream) puts it on the caller's stream (after the pass's stream), so the
 * N>1 step can run it, the bucket clip and the bucket's all-reduce on its exchange stream
 * while phase 2 runs; phase 2 does not launch it, every other entry point does (on its own
 * stream, after the pass's). */
int ba3c_train_grads_phase(ba3c_handle* h, void* stream, const float* params, const uint8_t* state,
                           const int64_t* action, const float* futurereward, int32_t batch,
                           float entropy_beta, void* workspace, float* grads, double* scalars,
                           int32_t phase);
/* Launch the reduction a phase-4 pass held back, on `stream`; no-op when none is held.  The
 * caller orders `stream` after the phase-4 pass (e.g. by waiting for the ba3c_set_phase2_event
 * event, which follows it); the implicit launches of the other entry points order themselves
 * after everything enqueued on the pass's stream.  Replaces the PS push of the fc1 + heads
 * variables' gradients of OpenAIGym/train.py:598-606 (their aggregation starts from here). */
int ba3c_launch_held(ba3c_handle* h, void* stream);
/* Record the HIP event `event` (a hipEvent_t of the caller's, NULL: none) on the pass's stream
 * in every later phase-2 pass, right after conv3's gradient launches: the N>1 step starts the
 * fc1 + heads bucket's exchange from there, so its collective's workgroups take CUs at the
 * boundary before conv2's launch (short, non-persistent workgroups the dispatcher rebalances)
 * instead of beside conv3's persistent ones. */
int ba3c_set_phase2_event(ba3c_handle* h, void* event);
/* Launch a reduction that a phase-3 pass left pending, on the pass's stream (no-op when none
 * is pending; also launches a held phase-4 reduction).  For callers that read `grads` through another API (a torch view, a gradient
 * summary) between the pass and the fused apply. */
int ba3c_flush_pending(ba3c_handle* h);
/* First tensor of the fc1 + heads bucket (tensors before it: the conv layers). */
int ba3c_bucket_tensor(const ba3c_handle* h);

/* Per-tensor tf.clip_by_average_norm(g, 0.1) in place (n = graph numel incl. padding). */
int ba3c_clip_grads(ba3c_handle* h, void* stream, float* grads, void* workspace);
/* The same clip over tensors [t0, t1) only (a bucket). */
/* ba3c_clip_grads_range with flags: BA3C_CLIP_NO_RESIDENCY makes no co-residency
 * assumption (sum-of-squares + clip launches instead of the one-launch tagged form, whose
 * workgroups wait for each other): for a clip on a stream that runs beside other kernels. */
#define BA3C_CLIP_NO_RESIDENCY 1
int ba3c_clip_grads_range2(ba3c_handle* h, void* stream, float* grads, void* workspace, int32_t t0,
                           int32_t t1, int32_t flags);
int ba3c_clip_grads_range(ba3c_handle* h, void* stream, float* grads, void* workspace, int32_t t0,
                          int32_t t1);

/* One optimizer apply over the flat buffers: g_eff = grads*grad_scale (1/world after an
 * all-reduce-sum), or, with fuse_clip=1, clip_by_average_norm(grads) fused in (single
 * replica; one launch with a grid barrier when the tensor chunks fit one workgroup per CU,
 * bit-identical to ba3c_clip_grads followed by an unfused apply).  slot0/slot1: Adam m/v,
 * RMS ms/mom, Adagrad accum, Adadelta accum/accum_update, Momentum accum; unused slots may
 * be NULL. */
int ba3c_apply_update(ba3c_handle* h, void* stream, int32_t opt, float* params,
                      const float* grads, float* slot0, float* slot1,
                      const ba3c_opt_params* hp, float grad_scale, int32_t fuse_clip,
                      void* workspace);

/* Same apply with the Adam bias-correction state on the device: dev_powers = {beta1_power,
 * beta2_power} (float32, TF's variables) is read by the update and multiplied by
 * (beta1, beta2) after it, on the stream — so a captured hipGraph of the whole step replays
 * with the correct per-step alpha.  hp->beta*_power are ignored. */
int ba3c_apply_update_dev(ba3c_handle* h, void* stream, int32_t opt, float* params,
                          const float* grads, float* slot0, float* slot1,
                          const ba3c_opt_params* hp, float* dev_powers, float grad_scale,
                          int32_t fuse_clip, void* workspace);

/* Action sampling: actions[i] = #{k : cdf_i[k] <= u[i]} with cdf_i = cumsum(double(p_i))
 * / cdf_i[A-1]  (numpy RandomState.choice).  nonfinite (device int32, may be NULL) is
 * set to 1 if any probability is not finite (train.py:381 assert). */
int ba3c_sample(void* stream, const float* probs, const double* u, int32_t batch,
                int32_t num_actions, int64_t* actions, int32_t* nonfinite);

/* Evaluation action (OpenAIGym/common.py:24-33, play_one_episode): actions[i] = first argmax of
 * probs[i] (np.argmax), or random_actions[i] (the player's action_space.sample()) when
 * u[i] < eps (`random.random() < 0.001`). */
int ba3c_greedy(void* stream, const float* probs, const double* u, const int64_t* random_actions,
                int32_t batch, int32_t num_actions, double eps, int64_t* actions);

/* Timing probe: bracket every launch of kernel `kernel_id` with HIP events (on the stream
 * it is launched on) until disabled (kernel_id = -1).  ba3c_probe_read synchronises the
 * recorded events and returns the summed milliseconds and launch count since enabling. */
int ba3c_probe_enable(ba3c_handle* h, int32_t kernel_id);
/* Device-side error flags of the handle's in-launch waits (bit 0: a fused clip+optimizer launch,
 * bit 1: a one-launch ba3c_clip_grads_range, stopped waiting for another workgroup's partial;
 * bit 2: a chained launch's conv0 workgroups stopped waiting for the zeroing of the ReLU
 * counters / max slots — the results are invalid).  0 in normal operation.  Synchronises the
 * device (diagnostics / tests only).  Once bit 2 is seen the handle zeroes its chain words and
 * stops chaining launches (the flag stays set). */
int ba3c_device_errors(ba3c_handle* h, uint32_t* flags);

int ba3c_probe_read(ba3c_handle* h, double* total_ms, int32_t* launches);
/* Bracket only the first of every `n` launches of the probed kernel (default 1: every launch),
 * counted from here / from ba3c_probe_enable.  Each bracket's two events leave 5-6 us gaps in
 * the stream, so a throughput run samples its launches (bench.py --probe-every). */
int ba3c_probe_every(ba3c_handle* h, int32_t n);
/* The synchronous gradient exchange through the C ABI (SURVEY.md §8b `ba3c_allreduce_mean`;
 * replaces the SyncReplicasOptimizer aggregation on the parameter servers,
 * OpenAIGym/train.py:598-606): an RCCL communicator owned by the handle.  RCCL is resolved at
 * run time from the process's librccl.so.1 (torch's copy when torch is loaded).
 * ba3c_comm_unique_id: rank 0 draws BA3C_UNIQUE_ID_BYTES bytes and the caller broadcasts them;
 * ba3c_comm_init is collective over the ranks; ba3c_comm_destroy(abort = 1) does not wait for
 * enqueued collectives (an exit path where a peer may be gone).  ba3c_allreduce_sum sums
 * `count` floats in place over the ranks on `stream`; ba3c_allreduce_mean also scales them by
 * 1/nranks (16-byte aligned `grads`).  The Python trainer drives the same RCCL through
 * ba3c_amd/rccl.py, with the same semantics. */
#define BA3C_UNIQUE_ID_BYTES 128
int ba3c_comm_unique_id(void* id_out);
int ba3c_comm_init(ba3c_handle* h, const void* id, int32_t nranks, int32_t rank);
int ba3c_comm_destroy(ba3c_handle* h, int32_t abort);
int ba3c_allreduce_sum(ba3c_handle* h, void* stream, float* buf, int64_t count);
int ba3c_allreduce_mean(ba3c_handle* h, void* stream, float* grads, int64_t count);
/* Diagnostic, not part of the reference's interface: enqueue on `stream` a launch of `n_cus`
 * workgroups that each hold one whole CU (all 160 KiB of its LDS) for `usec` microseconds,
 * doing nothing.  bench.py --occupy uses it on the exchange stream to stand in for RCCL's
 * channel workgroups while the conv backward runs (how persistent kernels degrade when K CUs
 * are missing). */
int ba3c_occupy_cus(void* stream, int32_t n_cus, double usec);

/* Arithmetic path of kernel `kernel_id` on this handle (for roofline accounting; no
 * reference counterpart): the number of 16-bit MFMA products it issues per fp32 product —
 * 6 for the bf16 hi/mid/lo split, 3 for the scaled fp16 hi/lo split (or conv0's u8 x bf16x3),
 * 2 for conv0's u8 x scaled-fp16 hi/lo — or 1 for fp32 MFMA (v_mfma_f32_*_f32), 0 for a
 * kernel with no matrix work; -1 on a bad id. */
int ba3c_kernel_split(const ba3c_handle* h, int32_t kernel_id);

/* Operand family of a split kernel: 3 = bf16 planes (v_mfma_*_bf16), 2 = power-of-two
 * scaled fp16 planes (v_mfma_*_f16); otherwise the value of ba3c_kernel_split (1, 0, -1). */
int ba3c_kernel_family(const ba3c_handle* h, int32_t kernel_id);

/* Kernels that ran inside kernel `kernel_id`'s launch in the last training pass (multi-job
 * launches: the probe of `kernel_id` brackets them too, and they record no launch of their own),
 * as a bitmask of kernel ids; 0 when the launch ran only that kernel, -1 on a bad id.  For
 * roofline accounting only (no reference counterpart). */
int ba3c_kernel_merged(const ba3c_handle* h, int32_t kernel_id);

/* ---- data formats either side of the path ---------------- */

/* n-step returns of MySimulatorMaster (OpenAIGym/train.py:408-437, _parse_memory) for n_envs
 * simulators at once.  Env e's memory is a ring of `slots` transitions (i-th oldest at slot
 * (start[e]+i) % slots), length[e] of them with known rewards (float64, as gym returns them)
 * and predictor values.  not over: the newest transition only bootstraps (R = its value) and
 * is not emitted; over: R = 0 and all are emitted.  Emitted in reverse time order, env by env
 * (the reference's queue order): R = clip(r,-1,1) + gamma*R in float64, stored as float32;
 * src[i] = e*slots + slot of datapoint i; init_R / over as the reference's datapoint
 * fields.  Output arrays hold n_envs*slots entries; *count (device int32) receives the
 * number written.  One workgroup: latency-bound. */
int ba3c_nstep_returns(void* stream, const double* reward, const float* value,
                       const int32_t* start, const int32_t* length, const uint8_t* is_over,
                       int32_t n_envs, int32_t slots, double gamma, float* R, int32_t* src,
                       float* init_R, uint8_t* over, int32_t* count);

/* BatchData / EnqueueThread hand-off (dataflow/common.py:64-99, train/trainer.py:116-155):
 * out[i] = rows[idx[i]] for n rows of row_bytes (a multiple of 16, e.g. 84*84*C states, or
 * exactly 8: int64 actions). */
int ba3c_gather_rows(void* stream, const void* rows, const int32_t* idx, int32_t n,
                     int64_t row_bytes, void* out);

/* HistoryFramePlayer (RL/history.py:12-55) for n_envs simulators: state[e] ([pixels][hist_len
 * * channels] uint8, oldest frame first) becomes concat(state[..., channels:], frame[e]); when
 * is_over[e] (may be NULL) the frame starts a new episode: zeros + frame. */
int ba3c_history_push(void* stream, const uint8_t* frame, uint8_t* state, const uint8_t* is_over,
                      int32_t n_envs, int32_t pixels, int32_t hist_len, int32_t channels);

#ifdef __cplusplus
}
#endif
#endif /* BA3C_H */
