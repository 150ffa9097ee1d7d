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

#ifdef __cplusplus
}
#endif

#endif /* HBK_H */
