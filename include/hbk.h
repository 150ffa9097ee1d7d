/*
 * hbk.h — C ABI of libhbk.so, the MI355X (gfx950) hot path of hey-buddy's
 * featurizer and wake-word trainer.
 *
 * Conventions (every entry point):
 *   - extern "C", plain pointers and sizes, no C++ or torch types.
 *   - return 0 on success, a negative hbk_status on failure; the message of the
 *     last failure on the calling thread is hbk_last_error().
 *   - every tensor pointer is a caller-owned DEVICE pointer (f32 unless noted),
 *     C-contiguous with the strides given; nothing on the hot path allocates.
 *   - work is enqueued on the caller's hipStream_t (passed as void*; NULL = the
 *     legacy default stream) and is asynchronous: the call returns once the
 *     kernels are launched.
 *
 * Each function names the reference interface it replaces (file:line under
 * src/python/heybuddy/ of therealadityashankar/hey-buddy).
 */
#ifndef HBK_H
#define HBK_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
  HBK_OK = 0,
  HBK_ERR_ARG = -1,      /* bad argument / shape */
  HBK_ERR_HIP = -2,      /* HIP runtime error (launch, alloc, copy) */
  HBK_ERR_UNSUPPORTED = -3
} hbk_status;

/* Library identity and error reporting. */
const char* hbk_version(void);
const char* hbk_last_error(void);
/* Number of HIP devices visible to the library (0 on a GPU-less host). */
int hbk_device_count(int* count);
/* A stream whose kernels run only on the compute units set in cu_mask (bit i
 * of word i / 32 = CU i; n_words 32-bit words; hipExtStreamCreateWithCUMask).
 * The pipelined train driver (heybuddy.pipeline) gives the latency-bound
 * classifier step a CU partition of its own while the next chunk of clips is
 * featurized on the rest; no reference interface (the reference runs the two
 * phases one after the other, __main__.py:245-429). */
int hbk_stream_create_cu_mask(const uint32_t* cu_mask, int n_words, void** stream);
int hbk_stream_destroy(void* stream);

/* Profiling marker (no reference counterpart): enqueues hbk_profile_mark_kernel,
 * a one-wave kernel that stores `tag`, on `stream`. bench.py brackets its timed
 * region with tags 1 / 2 (and its sequential stage-timing steps with 3 / 4),
 * each behind a device synchronize, so a rocprofv3 kernel trace or counter pass
 * can keep exactly the dispatches that fall between two markers
 * (tools/prof_summary.py). */
int hbk_profile_mark(int32_t tag, void* stream);

/* ------------------------------------------------------------------------ *
 * Mel spectrogram (STFT -> |.|^2 -> mel filterbank -> 10 log10 -> x/10 + 2)
 *
 * Replaces MelSpectrogramModel.__call__ (spectrogram.py:23-32), i.e. the ORT
 * session.run of the mel ONNX graph (util/onnx_util.py:83-96) plus the host
 * post-scale `/10 + 2` (spectrogram.py:32), as driven per 17,280-sample audio
 * window by SpeechEmbeddings.audio_to_spectrograms (embeddings.py:56-84).
 * This entry computes each UNIQUE frame of a clip once: frame f covers
 * samples [hop*f, hop*f + n_fft) (no centre padding), which is frame f - 12w
 * of the reference's audio window w (embeddings.py:190).
 * ------------------------------------------------------------------------ */
typedef struct hbk_mel_plan hbk_mel_plan;

/* window: host f32[n_fft] (the analysis window already zero-padded and centred
 *   in n_fft, as torch.stft does for win_length < n_fft);
 * fbank: host f32[(n_fft/2+1) * n_mels], row-major [freq][mel] (torchaudio
 *   melscale_fbanks layout);
 * in_scale: multiplies the PCM before framing (32767.0, embeddings.py:182);
 * log_floor: clamp before 10*log10 (1e-10, AmplitudeToDB amin);
 * out_div, out_add: y = 10*log10(max(mel, floor)) / out_div + out_add
 *   (10, 2: spectrogram.py:32).
 * Supported: n_fft == 512, n_mels <= 64 and even. */
int hbk_mel_plan_create(const float* window, const float* fbank, int n_fft,
                        int hop, int n_mels, float in_scale, float log_floor,
                        float out_div, float out_add, hbk_mel_plan** plan);
int hbk_mel_plan_destroy(hbk_mel_plan* plan);
/* The filterbank stage of hbk_mel_frames: 0 = sparse per-lane dot products on
 * the VALU (default), 1 = a dense split-f16 MFMA product (32 mels on bins < 128
 * only; HBK_MEL_MFMA=1 in the environment selects it at plan creation).
 * Same transform and outputs (within the 1e-4 tolerance). */
int hbk_mel_set_variant(hbk_mel_plan* plan, int32_t variant);

/* pcm: [n_clips, clip_stride] f32; frames f in [0, n_frames) of every clip
 *   (caller guarantees hop*(n_frames-1) + n_fft <= samples per clip);
 * out: [n_clips, n_frames, n_mels] f32. */
int hbk_mel_frames(const hbk_mel_plan* plan, const float* pcm, int64_t n_clips,
                   int64_t clip_stride, int64_t n_frames, float* out,
                   void* stream);

/* ------------------------------------------------------------------------ *
 * Speech embedding (conv stack on 76-frame mel windows -> 96-d embedding)
 *
 * Replaces SpeechEmbeddingModel.__call__ (embeddings.py:32-42), the ORT run of
 * the embedding ONNX graph (input_1 [n,76,32,1] -> conv2d_19 [n,1,1,96],
 * src/js/src/models/speech-embedding.js:125-146), as driven by
 * SpeechEmbeddings.spectrograms_to_embeddings (embeddings.py:86-151).
 * The graph is runtime data: a list of Keras-style ops (Conv2D 'valid',
 * stride 1, HWIO weights, optional LeakyReLU; MaxPool2D with stride = window),
 * NHWC with H = time (frames) and W = mel bins.
 * ------------------------------------------------------------------------ */
typedef enum { HBK_OP_CONV = 0, HBK_OP_MAXPOOL = 1 } hbk_op_kind;
typedef enum { HBK_ACT_NONE = 0, HBK_ACT_LEAKY_RELU = 1 } hbk_act;

typedef struct {
  int32_t kind;          /* hbk_op_kind */
  int32_t kh, kw;        /* conv kernel, or pool window (= stride) */
  int32_t cin, cout;     /* conv only */
  int32_t act;           /* conv only: hbk_act */
  float alpha;           /* LeakyReLU slope */
  const float* weight;   /* conv only: HOST f32 [kh][kw][cin][cout] */
  const float* bias;     /* conv only: HOST f32 [cout] */
} hbk_graph_op;

typedef struct hbk_embed_plan hbk_embed_plan;

/* in_h x in_w: the embedding window (76 x 32). win_start[n_win]: start frame of
 * each embedding window inside a clip's unique-frame sequence, in output-slot
 * order (the reference's 16 windows: 12 w + 8 q, embeddings.py:190 and
 * :136-143). Layers before the first max-pool whose time stride stops dividing
 * every start run ONCE per clip over the whole frame sequence (valid convs are
 * time-translation equivariant); the rest runs per window. */
int hbk_embed_plan_create(const hbk_graph_op* ops, int32_t n_ops, int32_t in_h, int32_t in_w,
                          const int32_t* win_start, int32_t n_win, hbk_embed_plan** plan);
int hbk_embed_plan_destroy(hbk_embed_plan* plan);

/* Arithmetic of the conv GEMMs.
 * SPLIT_F16 (default of hbk_embed_plan_create): every activation and weight is
 *   held as an fp16 pair x = hi + 2^-11 lo and each product as
 *   hi*hi + 2^-11 (hi*lo + lo*hi) on v_mfma_f32_32x32x16_f16 with f32
 *   accumulation: ~2^-21 relative per operand (f32 is 2^-24), at 16x the MFMA
 *   rate of f32 input. Requires |activations| and |weights| < 65504: a plan
 *   whose weights reach it is refused (HBK_ERR_UNSUPPORTED: use EXACT_F32), and
 *   every kernel that splits an activation raises the plan's range flag when one
 *   reaches it (hbk_embed_range_status).
 * EXACT_F32: v_mfma_f32_16x16x4f32, bitwise an fmaf chain in f32. */
typedef enum { HBK_PREC_SPLIT_F16 = 0, HBK_PREC_EXACT_F32 = 1 } hbk_precision;
int hbk_embed_plan_create_ex(const hbk_graph_op* ops, int32_t n_ops, int32_t in_h, int32_t in_w,
                             const int32_t* win_start, int32_t n_win, int32_t precision,
                             hbk_embed_plan** plan);

/* out_dim; number of ops shared per clip; fused chains (clip path); MACs per
 * clip (shared prefix, algorithmic) and per window (tail; when the tail runs
 * on deduplicated phase images -- windows whose offsets agree modulo the
 * tail's pool stride share one -- the phase images' MACs per clip / n_win). */
int hbk_embed_plan_info(const hbk_embed_plan* plan, int32_t* out_dim, int32_t* n_prefix_ops,
                        int32_t* n_chains, double* prefix_macs_per_clip,
                        double* tail_macs_per_window, int32_t* seq_frames);

/* Workspace for hbk_embed_clips / hbk_embed_windows over n items. */
int hbk_embed_workspace_size(const hbk_embed_plan* plan, int64_t n, int64_t* bytes);

/* mel: [n_clips, mel_clip_stride] f32 (unique frames x in_w, row-major; at
 * least seq_frames frames); out: [n_clips, n_win, out_dim] f32. */
int hbk_embed_clips(const hbk_embed_plan* plan, const float* mel, int64_t n_clips,
                    int64_t mel_clip_stride, float* out, void* workspace,
                    int64_t workspace_bytes, void* stream);

/* hbk_embed_clips in two calls on two streams (no reference counterpart: a
 * scheduling split, e.g. the tail of featurisation on the training stream's
 * CUs). The front runs the clip program's first n_front fused chains
 * (1 <= n_front < n_chains) and writes chain n_front - 1's output to mid
 * ([n_clips, mid_floats_per_clip] f32, hbk_embed_split_info); the back runs
 * the remaining chains from mid into out. Front + back == hbk_embed_clips.
 * Each call needs its own workspace (hbk_embed_workspace_size) when the two
 * can run concurrently. */
int hbk_embed_split_info(const hbk_embed_plan* plan, int32_t n_front, int64_t* mid_floats_per_clip);
int hbk_embed_clips_front(const hbk_embed_plan* plan, const float* mel, int64_t n_clips,
                          int64_t mel_clip_stride, int32_t n_front, float* mid, void* workspace,
                          int64_t workspace_bytes, void* stream);
int hbk_embed_clips_back(const hbk_embed_plan* plan, const float* mid, int64_t n_clips, int32_t n_front,
                         float* out, void* workspace, int64_t workspace_bytes, void* stream);

/* Per-window API of the reference: windows [n, in_h, in_w] f32 -> out [n, out_dim]. */
int hbk_embed_windows(const hbk_embed_plan* plan, const float* windows, int64_t n, float* out,
                      void* workspace, int64_t workspace_bytes, void* stream);

/* NaN rows of an embedding batch, in place (embeddings.py:209-234): rows [n, row_len] f32
 * (row_len % 4 == 0, 16-B aligned; one row = one clip's embeddings). Every row holding a NaN
 * is replaced by a NaN-free row drawn uniformly (a counter-based hash of (seed, row) in place
 * of np.random.choice), or by zeros when every row holds a NaN; NaN-free rows are unchanged.
 * No host synchronisation (the reference's warning needs the count on the host and is not
 * emitted). workspace: hbk_nan_rows_workspace_size(n) bytes. */
int64_t hbk_nan_rows_workspace_size(int64_t n);
int hbk_nan_rows_fix(float* rows, int64_t n, int64_t row_len, uint64_t seed, void* workspace,
                     int64_t workspace_bytes, void* stream);

/* Range guard of SPLIT_F16 plans (no reference counterpart: the ONNX graph runs
 * in f32). *tripped = 1 if any split kernel of this plan saw an activation with
 * |x| >= 65504 since the flag was last cleared (those outputs are not
 * f32-accurate: recompute them with an EXACT_F32 plan), else 0. Waits for the
 * work queued on `stream`; reset != 0 clears the flag. */
int hbk_embed_range_status(const hbk_embed_plan* plan, int32_t* tripped, int32_t reset, void* stream);

/* ------------------------------------------------------------------------ *
 * Wake-word classifier: gated MLP forward and the fused train step
 *
 * Replaces WakeWordMLPModel.forward (wakeword.py:334-348, gated MLP of
 * modules/multi_layer_perceptron.py:76-124) and the optimisation path of
 * WakeWordTrainer.train_epoch (trainer.py:380-494): high-loss filter
 * (:407-424), weighted BCE (:301-312), backward, the < 128-sample
 * accumulation gate (:443-465) and torch.optim.Adam (:45).
 * Parameters live in ONE flat f32 buffer (layout: hbk_mlp_layout).
 * ------------------------------------------------------------------------ */
typedef struct hbk_mlp_plan hbk_mlp_plan;

/* d_in = 16*96, layer_dim = 96, hidden = get_normalized_dim(96) = 64. */
int hbk_mlp_plan_create(int32_t d_in, int32_t layer_dim, int32_t hidden, int32_t n_layers,
                        hbk_mlp_plan** plan);
int hbk_mlp_plan_destroy(hbk_mlp_plan* plan);
/* n_params and the float offsets of: norm_in g,b; per GMLP (mlp_in,
 * layers..., mlp_out) W_hg [2H,in] (hidden rows then gate rows), b_hg [2H],
 * W_o [out,H], b_o [out]; per LN (layers..., norm_out) g, b. */
int hbk_mlp_layout(const hbk_mlp_plan* plan, int64_t* n_params, int64_t* offsets, int32_t n_offsets);
int hbk_mlp_workspace_size(const hbk_mlp_plan* plan, int64_t batch, int64_t* bytes);

/* x [batch, d_in] f32 -> prob [batch] (and pre-sigmoid logit [batch] if non-NULL).
 * dropout_p: input dropout (nn.Dropout before the first LayerNorm; the
 * reference keeps it active in training AND validation since .eval() is never
 * called), mask = f(seed, element index); 0 disables it. */
int hbk_mlp_forward(const hbk_mlp_plan* plan, const float* params, const float* x, int64_t batch,
                    float* prob, float* logit, float dropout_p, uint64_t seed, void* workspace,
                    int64_t workspace_bytes, void* stream);

/* Forward + filter + weighted BCE + backward. bucket [n_params + 8] is zeroed,
 * then receives the UNNORMALISED gradient sum over the selected samples of
 * w * dl/dz and the statistics [n_sel, sum w*l, n_neg_sel, fp_sel, n_pos_sel,
 * tp_sel, batch, 0]; data-parallel ranks all-reduce (sum) the whole bucket.
 * y: labels as f32 0/1. prob [batch] (optional) receives sigmoid outputs. */
int hbk_mlp_train_fwd_bwd(const hbk_mlp_plan* plan, const float* params, const float* x,
                          const float* y, int64_t batch, float neg_weight,
                          float high_loss_threshold, float activation_threshold, float dropout_p,
                          uint64_t seed, float* bucket, float* prob, void* workspace,
                          int64_t workspace_bytes, void* stream);

/* The accumulation gate on the (reduced) bucket statistics and, when it fires,
 * Adam on params with grads * 1/(n_sel * accumulation_steps). state[4]:
 * accumulated_samples, accumulation_steps (init 1), adam step, step index;
 * ctrl[4] scratch; history (optional, [cap, 8]): per step n_sel,
 * accumulation_steps used, fired, loss (BCE mean / accumulation_steps),
 * n_neg_sel, fp_sel, n_pos_sel, tp_sel. */
int hbk_mlp_gate_adam(const hbk_mlp_plan* plan, float* params, const float* bucket, float* m,
                      float* v, float* state, float* ctrl, float* history, int32_t history_cap,
                      float lr, float beta1, float beta2, float eps, void* stream);

/* Fused train step (default architecture: d_in 1536, layer_dim 96, hidden 64,
 * at most 4 layers; *supported = 0 for other plans, which keep the generic
 * entry points above). Four launches per step, no host synchronisation:
 * hbk_mlp_step_fwd_bwd (input gather + LayerNorm + input GEMM, the 16-row
 * chain forward/filter/BCE/backward, the weight gradients) and
 * hbk_mlp_step_update (gate + Adam + bucket zeroing), with the data-parallel
 * all-reduce of the bucket between them.
 *
 * Rows: row r of the step's batch is pool32 row idx[r] (idx[r] >= 0, f32
 *   [n32, 1536]) or pool16 row -idx[r] - 1 (f16 [n16, 1536]); an index outside
 *   its pool reads as a zero row. idx == NULL: row r = pool32 row r. The step's
 *   idx is idx + step * idx_step_stride, its labels y + step * y_step_stride
 *   (0/1 f32), where step = state[8 * parity + 3].
 * state: device float[16], two halves of [accumulated_samples,
 *   accumulation_steps (init 1), adam step t, step index, dropout salt, 0, 0, 0].
 *   A step reads half `parity` and hbk_mlp_step_update writes half 1 - parity
 *   (step + 1): successive steps alternate parity, and a hipGraph of an even
 *   number of steps replays a whole stage.
 * sched (optional, device f32 [sched_len][2]): (lr, neg_weight) of step s at
 *   row min(s, sched_len - 1), in place of the lr / neg_weight arguments.
 * bucket [n_params + 8]: must be zero before the first step (hbk_mlp_step_update
 *   zeroes it for the next one); receives the unnormalised gradients and the
 *   statistics of hbk_mlp_train_fwd_bwd. history as in hbk_mlp_gate_adam.
 * The dropout mask of element i of step s is f(seed + s + (salt << 24), i).
 *
 * The input gather + dropout + LayerNorm of a step needs no weights, so it is
 * computed one step AHEAD inside the previous step's launches:
 *   flags & HBK_STEP_PREFETCH_NEXT (with idx): this call also computes step + 1's
 *     normalised rows (rows idx[step + 1], if step + 1 < idx_steps) into the
 *     workspace, concurrently with its own chain kernel;
 *   flags & HBK_STEP_XHAT_READY: this step's rows were prefetched that way (the
 *     previous call on the same workspace set PREFETCH_NEXT) and are not
 *     recomputed. Without it the step gathers its own rows first.
 * The chain kernel reads its weight matrices as pre-split f16 hi / lo planes
 * (plain and transposed) from a cache at the start of the workspace:
 *   flags & HBK_STEP_WEIGHTS_READY: the previous hbk_mlp_step_update got the same
 *     workspace and left the cache current (it rewrites the cached matrices with
 *     every update); without it the step refreshes the cache from params first.
 * The weight gradients are written per batch split as partial slabs in the
 * workspace (plain stores; no float atomics) and summed once:
 *   flags & HBK_STEP_DEFER_PARTIALS: by the next hbk_mlp_step_update, which must
 *     get this workspace (it fails otherwise) and must follow with nothing that
 *     reads the bucket in between (one process: no all-reduce);
 *   without it: into the bucket at the end of this call (for the data-parallel
 *     all-reduce, or an update without the workspace). */
#define HBK_STEP_XHAT_READY 1
#define HBK_STEP_PREFETCH_NEXT 2
#define HBK_STEP_WEIGHTS_READY 4
#define HBK_STEP_DEFER_PARTIALS 8
int hbk_mlp_fused_supported(const hbk_mlp_plan* plan, int32_t* supported);
int hbk_mlp_step_fwd_bwd(const hbk_mlp_plan* plan, const float* params, const float* pool32, int64_t n32,
                         const void* pool16, int64_t n16, const int32_t* idx, int64_t idx_step_stride,
                         const float* y, int64_t y_step_stride, int64_t batch, const float* state,
                         int32_t parity, const float* sched, int64_t sched_len, float neg_weight,
                         float high_loss_threshold, float activation_threshold, float dropout_p,
                         uint64_t seed, float* bucket, float* prob, int64_t idx_steps, int32_t flags,
                         void* workspace, int64_t workspace_bytes, void* stream);
int hbk_mlp_step_update(const hbk_mlp_plan* plan, float* params, float* bucket, float* m, float* v,
                        float* state, int32_t parity, const float* sched, int64_t sched_len, float lr,
                        float beta1, float beta2, float eps, float* history, int32_t history_cap,
                        void* workspace, int64_t workspace_bytes, void* stream);

/* Graph-captured training steps: dev_scalars (device, double[3] = lr,
 * neg_weight, dropout seed; NULL = off) is read by the kernels of
 * hbk_mlp_train_fwd_bwd and hbk_mlp_gate_adam in place of their lr,
 * neg_weight and seed arguments, so one captured hipGraph replays every step
 * of a stage with the schedule's values written before each replay. */
int hbk_mlp_set_step_scalars(hbk_mlp_plan* plan, const double* dev_scalars);

/* Evaluation passes: the validation and testing forwards of train_epoch
 * (trainer.py:496-566; the default validation pass is 500 batches of 50
 * positives + 1,000 negatives, the testing pass 500 of 50 + 50, every
 * validation_steps = 250 steps, with dropout active as the reference never
 * calls .eval()), reduced on the device to prediction counts, and the
 * reference's bookkeeping after them (false positives per hour, recall,
 * testing rates, the dynamic negative weight of :531-536). Fused plans only.
 *
 * hbk_mlp_eval_prepare: the pass's weight planes from params (once per pass:
 *   params must not change between it and the counts).
 * hbk_mlp_eval_count: rows r = 0 .. rows-1 of ONE pool (pool_is_f16: f16 [n_pool,
 *   1536], else f32), row r = pool row idx[r] (idx != NULL) or (row_offset + r) %
 *   n_pool, all labelled `label`; counts[2 label] += #(p >= activation_threshold),
 *   counts[2 label + 1] += #(p > activation_threshold) (f32 counters, exact below
 *   2^24: the caller zeroes them). The dropout mask of element i of row r is
 *   f(seed, row_offset + r, i). prob (optional, [rows]) receives p.
 *   Replaces the per-batch `self.model(x)[:, 0]` loops of trainer.py:503-510, 542-548.
 * hbk_mlp_eval_finish: sizes (host) = {validation negatives, validation
 *   positives, testing negatives, testing positives}; counts_test may be NULL.
 *   out (device f32 [8]) = {validation false positives per hour (count / (n_neg
 *   1.44 / 3600) in f32), validation recall, testing false-positive rate,
 *   testing recall, testing accuracy, new negative weight, weight before, 0}.
 *   adjust_ratio > 0: the negative weight of step next_step - 1 (sched row) is
 *   multiplied by adjust_ratio when the rate exceeds the target, else divided
 *   by it with a floor of 1, and written to sched rows next_step .. sched_len - 1
 *   (trainer.py:531-536). */
int hbk_mlp_eval_workspace_size(const hbk_mlp_plan* plan, int64_t rows, int64_t* bytes);
int hbk_mlp_eval_prepare(const hbk_mlp_plan* plan, const float* params, void* workspace, int64_t workspace_bytes,
                         void* stream);
int hbk_mlp_eval_count(const hbk_mlp_plan* plan, const float* params, const void* pool, int32_t pool_is_f16,
                       int64_t n_pool, const int32_t* idx, int64_t rows, int64_t row_offset, int32_t label,
                       float activation_threshold, float dropout_p, uint64_t seed, float* counts, float* prob,
                       void* workspace, int64_t workspace_bytes, void* stream);
/* hbk_mlp_eval_count for n_pools (<= 4) pools of one dtype in ONE launch: pool i's rows
 * r = 0 .. rows[i]-1 are pool rows (row_offsets[i] + r) % n_pool[i], labelled labels[i], counted
 * into counts[i] with dropout seed seeds[i], each exactly as its own hbk_mlp_eval_count (no idx, no
 * prob); the workgroups of all pools share one grid, so small pools fill each other's last round.
 * Host arrays of device pointers / values; workspace sized for the largest pool. */
int hbk_mlp_eval_count_multi(const hbk_mlp_plan* plan, const float* params, int32_t n_pools,
                             const void* const* pools, int32_t pools_are_f16, const int64_t* n_pool,
                             const int64_t* rows, const int64_t* row_offsets, const int32_t* labels,
                             const uint64_t* seeds, float* const* counts, float activation_threshold,
                             float dropout_p, void* workspace, int64_t workspace_bytes, void* stream);
int hbk_mlp_eval_finish(const float* counts_val, const float* counts_test, const double* sizes,
                        float target_false_positives_per_hour, float adjust_ratio, float* sched, int64_t sched_len,
                        int64_t next_step, float* out, void* stream);

/* ------------------------------------------------------------------------ *
 * Batch augmentation: background-noise mix + impulse-response reverb
 *
 * Replaces add_background_noise_to_batch -> torchaudio.functional.add_noise
 * (dataset/augmented.py:234-276, applied :383-384) and speechbrain
 * reverberate(batch, ir, rescale_amp="avg") (:386-392) of
 * AugmentedAudioGenerator.execute_augment_batch, for clips of T = 23,040
 * samples (1.44 s, augmented.py:31).
 * ------------------------------------------------------------------------ */
typedef struct hbk_reverb_plan hbk_reverb_plan;

/* T must be 23040. */
int hbk_reverb_plan_create(int64_t T, hbk_reverb_plan** plan);
int hbk_reverb_plan_destroy(hbk_reverb_plan* plan);

/* Spectrum slots per IR: bin k (0 <= k <= T/2 = 11520) of rfft(kernel) is
 * stored at slot (k % 16) * 721 + k / 16 (16 rows of 721; 15 slots unused), so
 * that hbk_augment's pair loop reads it with coalesced loads. */
#define HBK_REVERB_SPECTRUM_SLOTS 11536

/* kernels [n_kernels, stride] f32: the ROTATED length-T kernels
 * [ir[d:], zeros(T - L), ir[:d]] (d = argmax |ir|, ir truncated to T first),
 * spectra [n_kernels, HBK_REVERB_SPECTRUM_SLOTS] complex64 (interleaved f32):
 * rfft(kernel) in the slot order above. */
int hbk_reverb_spectrum(const hbk_reverb_plan* plan, const float* kernels, int64_t n_kernels,
                        int64_t stride, float* spectra, void* stream);

/* Per clip i of x [n_clips, x_stride] (first T samples used):
 *   if gain != NULL: x = gain[i] x (torch_audiomentations Gain, applied before the
 *      noise mix as in the reference's batch chain, augmented.py:114-118, :383-392);
 *   if noise_off[i] >= 0: y = x + 10^((10 log10(|x|^2/|n|^2) - snr_db[i]) / 20) n,
 *      n = noise_ring[(noise_off[i] + t) mod ring_len], t < T (noise_off[i] < ring_len < 2^30);
 *   if spec_idx[i] >= 0: y = mean|y| * c / (mean|c| + 1e-14), c = irfft(rfft(y) * spectra[spec_idx[i]]).
 * out [n_clips, out_stride] (may equal x). All pointers are device pointers. */
int hbk_augment(const hbk_reverb_plan* plan, const float* x, int64_t n_clips, int64_t x_stride,
                const float* noise_ring, int64_t ring_len, const int64_t* noise_off,
                const float* snr_db, const float* spectra, const int32_t* spec_idx,
                const float* gain, float* out, int64_t out_stride, void* stream);

/* Colored noise: torch_audiomentations AddColoredNoise, which the reference's
 * batch chain applies per batch with p 0.25 (dataset/augmented.py:107-113,
 * constants.py:128-132). Per clip i of x [n_clips, x_stride] (first T = 23040
 * samples used), the package's _gen_noise / apply_transform, with the white
 * noise shared by each group of clips_per_noise consecutive clips, g = i /
 * clips_per_noise (per_batch mode runs the transform on the batch reshaped to
 * (1, batch, T): one noise vector for the whole batch; 1 = a vector per clip):
 *   w = white[g][0 .. 16000) (N(0,1), white_stride >= 16000) or, if white ==
 *       NULL, the counter-based N(0,1) stream: samples 2q, 2q + 1 of group g are
 *       the Box-Muller pair of hash (seed, g * 8000 + q);
 *   n1 = irfft(rfft(w) / linspace(1, sqrt(8000), 8001)^f_decay[i], n = 16000);
 *   n1 /= rms(n1) + 1e-8;  noise[t] = n1[t mod 16000] (tiled to T, not renormalised);
 *   out[i] = x[i] + rms(x[i]) / 10^(snr_db[i] / 20) * noise;
 *   snr_db[i] NaN: out[i] = x[i] (a batch whose coin came up tails).
 * sample_rate must be 16000 (the noise is one second long). out may equal x.
 * Device pointers. */
int hbk_colored_noise(const hbk_reverb_plan* plan, const float* x, int64_t n_clips, int64_t x_stride,
                      const float* white, int64_t white_stride, uint64_t seed, int64_t clips_per_noise,
                      const float* f_decay, const float* snr_db, float sample_rate, const int32_t* idx,
                      int64_t n_entries, float* out, int64_t out_stride, void* stream);
/* The same with a workspace of hbk_colored_noise_workspace_size(n_clips,
 * clips_per_noise) bytes (0 when clips_per_noise is 1): each group's coloured
 * second is made once (from its first clip's f_decay) and every clip of the
 * group with that f_decay mixes from it, bit-identical to the per-clip path
 * (per_batch mode draws one f_decay per batch). */
int64_t hbk_colored_noise_workspace_size(int64_t n_clips, int64_t clips_per_noise);
int hbk_colored_noise_ws(const hbk_reverb_plan* plan, const float* x, int64_t n_clips, int64_t x_stride,
                         const float* white, int64_t white_stride, uint64_t seed, int64_t clips_per_noise,
                         const float* f_decay, const float* snr_db, float sample_rate, const int32_t* idx,
                         int64_t n_entries, float* out, int64_t out_stride, void* workspace, int64_t workspace_bytes,
                         void* stream);

/* Colored noise followed by hbk_augment in one pass over the clips: out =
 * hbk_augment(hbk_colored_noise_ws(x)), bit-identical to the two calls (the
 * reference's batch chain runs AddColoredNoise right before the gain, noise and
 * reverb, dataset/augmented.py:107-118). The group path's mix (the clips
 * colored_mix_kernel would mix) happens in augment_kernel's prologue, so those
 * clips are read and written once; the clips the group path does not cover
 * (c_idx lists them; NULL = scan every clip) are coloured into out first and
 * augment_kernel reads them from there. Arguments as in hbk_augment and
 * hbk_colored_noise_ws (c_f_decay / c_snr_db per clip, NaN c_snr_db = no
 * colored noise). out may equal x; otherwise it must not overlap it. */
int hbk_augment_colored(const hbk_reverb_plan* plan, const float* x, int64_t n_clips, int64_t x_stride,
                        const float* noise_ring, int64_t ring_len, const int64_t* noise_off,
                        const float* snr_db, const float* spectra, const int32_t* spec_idx,
                        const float* gain, const float* white, int64_t white_stride, uint64_t seed,
                        int64_t clips_per_noise, const float* c_f_decay, const float* c_snr_db,
                        float sample_rate, const int32_t* c_idx, int64_t c_n_entries, float* out,
                        int64_t out_stride, void* workspace, int64_t workspace_bytes, void* stream);

/* Band-stop: torch_audiomentations BandStopFilter, which the reference applies
 * in its batch chain with p 0.25 per batch, one parameter set per batch
 * (center mel-uniform in [200, 4000] Hz, bandwidth fraction U[0.5, 1.99];
 * dataset/augmented.py:101-105, constants.py:127). Filter f: cutoffs f_lo[f],
 * f_hi[f] (fractions of the sample rate) and julius' half size
 * f_half[f] = int(8 / f_lo / 2); its spectra are slots f_spec0[f] .. of the
 * n_spectra listed in s_filt / s_part: ONE slot with s_part = -1 when
 * f_half <= HBK_BAND_STOP_CIRCULAR_MAX_HALF (circular convolution + direct edge
 * correction), else ceil((2 f_half + 1) / 11521) slots with s_part = 0, 1, ..
 * (overlap-save partitions). For entry e < n, clip row r = idx[e] of x
 * [*, x_stride] (first T = 23040 samples):
 *   out[r] = x[r] - julius.bandpass_filter(x[r], f_lo[filt[e]], f_hi[filt[e]])
 * (windowed-sinc lowpasses over the replicate-padded clip). Rows not listed are
 * not touched; out may equal x. workspace: hbk_band_stop_workspace_size bytes.
 * Device pointers. */
#define HBK_BAND_STOP_CIRCULAR_MAX_HALF 512
int64_t hbk_band_stop_workspace_size(int64_t n, int32_t n_filters, int32_t n_spectra, void* stream);
int hbk_band_stop(const hbk_reverb_plan* plan, const float* x, int64_t x_stride, int64_t n, const int32_t* idx,
                  const int32_t* filt, int32_t n_filters, const float* f_lo, const float* f_hi,
                  const int32_t* f_half, const int32_t* f_spec0, int32_t n_spectra, const int32_t* s_filt,
                  const int32_t* s_part, float* out, int64_t out_stride, void* workspace, int64_t workspace_bytes,
                  void* stream);

/* Pitch shift: torch_audiomentations PitchShift (+-3 semitones, mode per_batch,
 * p 0.25; dataset/augmented.py:93-100, constants.py:125-126), which calls
 * torch_pitch_shift.pitch_shift(x, Fraction(num, den), sample_rate): at 16 kHz
 * its "fast shifts" within +-3 semitones are 125/128 and 128/125. For entry
 * e < n, clip row r = idx[e] of x [*, x_stride] (first T samples):
 *   X = stft(x[r], n_fft 250, hop 7, rectangular window, center, reflect)
 *   Y = phase_vocoder(X, rate = den / num, adv = linspace(0, 7 pi, 126))
 *   out[r] = Resample(16000, 16000 den / num)(istft(Y)), cropped / zero-padded to T
 * Rows not listed are not touched; out may equal x (all reads of x precede
 * the writes). HBK_ERR_UNSUPPORTED for sample_rate != 16000 or a ratio whose
 * resampler needs more than 128 phases or HBK_PITCH_SHIFT_MAX_TAPS taps.
 * workspace: hbk_pitch_shift_workspace_size bytes (~0.2 MB per entry at
 * T = 23040; 0 for an unsupported geometry). Device pointers. */
#define HBK_PITCH_SHIFT_MAX_TAPS 144
int64_t hbk_pitch_shift_workspace_size(int64_t n, int64_t T, int32_t sample_rate, int32_t num, int32_t den);
int hbk_pitch_shift(const float* x, int64_t x_stride, int64_t n, const int32_t* idx, int64_t T, int32_t sample_rate,
                    int32_t num, int32_t den, float* out, int64_t out_stride, void* workspace,
                    int64_t workspace_bytes, void* stream);

/* Tanh distortion: audiomentations TanhDistortion, which the reference applies
 * per clip with p 0.25 and distortion ~ U[1e-4, 0.1] before the batch chain
 * (dataset/augmented.py:79-90, :325-328; constants.py:122-124). Per clip i of
 * x [n_clips, x_stride] (first T = 23040 samples used):
 *   th = percentile(|x|, 100 - 99 amount[i]) (numpy "linear");
 *   y = tanh(0.5 / (th + 1e-6) x); if rms(x) > 1e-9: y *= rms(x) / rms(y);
 *   amount[i] NaN: out[i] = x[i].
 * out may equal x. Device pointers. */
/* Seven-band parametric EQ: audiomentations SevenBandParametricEQ, which the
 * reference applies per clip with p 0.25 and gains in +-6 dB, first in its
 * per-clip Compose (dataset/augmented.py:79-84; constants.py:120-121). For
 * entry j < n_entries, clip c = idx[j] (idx NULL: every clip, c = j,
 * n_entries = n_clips) of x [., x_stride] (first T = 23040 samples): seven
 * biquads in series, coef[j][k] = (b0, b1, b2, a1, a2) normalised by a0 (f64;
 * low shelf, five peaks, high shelf from the RBJ cookbook, built by the
 * caller), each run as direct form II transposed in f64 from a zero state with
 * its output rounded to f32 (scipy sosfilt + astype(float32) per filter), into
 * out[c]. coef[j][0][0] NaN: out[c] = x[c]. Clips not listed are not touched:
 * with idx, run it in place (out == x). Rows 16-B aligned. Device pointers. */
int hbk_seven_band_eq(const float* x, int64_t n_clips, int64_t x_stride, const double* coef, const int32_t* idx,
                      int64_t n_entries, float* out, int64_t out_stride, void* stream);

/* (tanh distortion and colored noise) idx: NULL runs every clip of
 * [0, n_clips); else only the n_entries clip rows it lists (the clips or
 * batches whose coin came up, so the grid's work is balanced), in place or into
 * out's same rows (the other rows of out are not written). */
int hbk_tanh_distortion(const float* x, int64_t n_clips, int64_t x_stride, const float* amount,
                        const int32_t* idx, int64_t n_entries, float* out, int64_t out_stride, void* stream);

/* Clip placement: AugmentedAudioGenerator.to_target_length
 * (dataset/augmented.py:200-232) for a batch already on the device. Per clip i
 * of src [n_clips, src_stride] holding src_len[i] valid samples:
 *   out[i, t] = src[i, t - pre[i]] for pre[i] <= t < pre[i] + min(src_len[i], T),
 *   out[i, t] = 0 elsewhere, t < T.
 * The reference crops (pre = 0) when src_len >= T, else pads with
 * pre = np.random.randint(int(S/4), int(3S/4)) leading zeros, S = T - src_len
 * (pre = 0 when S == 1); the caller draws pre on the host with that rule.
 * T % 4 == 0, out rows 16-B aligned. One persistent launch (4,096-sample spans of the clips). */
int hbk_place_clips(const float* src, int64_t n_clips, int64_t src_stride, const int32_t* src_len,
                    const int32_t* pre, float* out, int64_t out_stride, int64_t T, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* HBK_H */
