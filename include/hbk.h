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

/* out_dim; number of ops shared per clip; fused chains (clip path); MACs per
 * clip (shared prefix, algorithmic) and per window (tail). */
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

/* Per-window API of the reference: windows [n, in_h, in_w] f32 -> out [n, out_dim]. */
int hbk_embed_windows(const hbk_embed_plan* plan, const float* windows, int64_t n, float* out,
                      void* workspace, int64_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* HBK_H */
