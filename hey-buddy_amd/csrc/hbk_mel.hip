// Fused STFT + power + mel filterbank + log kernel for gfx950.
//
// Replaces the mel ONNX graph run by MelSpectrogramModel.__call__
// (spectrogram.py:23-32) from SpeechEmbeddings.audio_to_spectrograms
// (embeddings.py:56-84). One frame = n_fft = 512 samples at hop 160, no centre
// padding (frame count ceil(t/160 - 3), embeddings.py:67).
//
// Work decomposition (one wave64 = 4 frames, 16 lanes per frame):
//   z[n] = xw[2n] + i xw[2n+1]  (n < 256) packs the real 512-point frame into a
//   256-point complex FFT, done four-step as 16 x 16:
//     lane n2 holds z[16 n1 + n2] for n1 = 0..15   -> FFT16 over n1 in VGPRs
//     twiddle W256^(n2 k1), transpose through LDS    -> lane k1 holds column k1
//     FFT16 over n2                                  -> Z[k1 + 16 k2]
//   real-FFT split X[k] = (Z[k] + Z*[256-k])/2 + W512^k (Z[k] - Z*[256-k])/(2i),
//   power |X[k]|^2 into LDS, then the mel filters as fixed-width sparse dot
//   products (each filter's non-zero bins are contiguous), 10 log10, /10 + 2.
// The 4 frames of a wave only exchange data through the wave's own LDS slice,
// so no workgroup barrier is needed after the table load.
#include <algorithm>
#include <cmath>
#include <vector>

#include "hbk_common.h"

namespace hbk {
namespace {

constexpr int kNfft = 512;
constexpr int kFramesPerWave = 4;
constexpr int kWaves = 4;
constexpr int kThreads = 64 * kWaves;
constexpr int kFramesPerBlock = kFramesPerWave * kWaves;
constexpr int kRow = 17;                  // transpose row: 16 complex + 1 pad (bank spread)
constexpr int kFrameC = 16 * kRow + 1;    // 273 complex = 2184 B per frame (== 8 mod 16 B)
constexpr int kMaxTaps = 16;              // widest mel filter supported
constexpr int kMaxMels = 32;
constexpr int kBlocksPerCU = 8;           // persistent grid: CUs x this

struct MelArgs {
  const float* pcm;
  float* out;
  const float* window;  // [512], in_scale folded in
  const float2* tw256;  // [256]
  const float2* tw512;  // [257]
  const int* mel_lo;    // [n_mels]
  const float* mel_w;   // [n_mels * taps]
  int64_t n_clips;
  int64_t clip_stride;
  int64_t n_frames;
  int hop;
  int n_mels;
  int taps;
  int nk2;      // number of 16-bin blocks of X[k] the filters read (k < 16*nk2)
  int need256;  // filters read bin 256
  float log_floor;
  float out_div;
  float out_add;
};

// exp(-2 pi i p / 16)
__device__ __forceinline__ cf w16(int p) {
  constexpr float c1 = 0.92387953251128674f, s1 = 0.38268343236508978f, r = 0.70710678118654757f;
  switch (p & 15) {
    case 0: return {1.f, 0.f};
    case 1: return {c1, -s1};
    case 2: return {r, -r};
    case 3: return {s1, -c1};
    case 4: return {0.f, -1.f};
    case 6: return {-r, -r};
    case 9: return {-c1, s1};
    default: return {0.f, 0.f};  // unused
  }
}

__device__ __forceinline__ void fft4(cf& a0, cf& a1, cf& a2, cf& a3) {
  const cf t0 = cadd(a0, a2), t1 = csub(a0, a2);
  const cf t2 = cadd(a1, a3), t3 = cmul_mi(csub(a1, a3));
  a0 = cadd(t0, t2);
  a2 = csub(t0, t2);
  a1 = cadd(t1, t3);
  a3 = csub(t1, t3);
}

// In-register 16-point forward DFT: v[k] <- sum_n v[n] W16^(nk), natural order.
__device__ __forceinline__ void fft16(cf (&v)[16]) {
  // n = 4 m1 + m2: radix-4 over m1 for each m2 -> v[4 l1 + m2] = A[m2][l1]
#pragma unroll
  for (int m2 = 0; m2 < 4; ++m2) fft4(v[m2], v[4 + m2], v[8 + m2], v[12 + m2]);
#pragma unroll
  for (int l1 = 1; l1 < 4; ++l1)
#pragma unroll
    for (int m2 = 1; m2 < 4; ++m2) v[4 * l1 + m2] = cmul(v[4 * l1 + m2], w16(m2 * l1));
  // radix-4 over m2 for each l1 -> v[4 l1 + l2] = X[l1 + 4 l2]
#pragma unroll
  for (int l1 = 0; l1 < 4; ++l1) fft4(v[4 * l1 + 0], v[4 * l1 + 1], v[4 * l1 + 2], v[4 * l1 + 3]);
  cf t[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) t[k] = v[4 * (k & 3) + (k >> 2)];
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = t[k];
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ void load_frame(const float* __restrict__ src, cf (&x)[16]) {
#pragma unroll
  for (int n1 = 0; n1 < 16; ++n1) x[n1] = *reinterpret_cast<const cf*>(src + 32 * n1);
}

// Persistent blocks: tables are staged into LDS once, then the block walks
// groups of 16 consecutive frames (flattened over clips) with a grid stride,
// prefetching the next group's samples while transforming the current one.
__global__ void __launch_bounds__(kThreads) mel_frames_kernel(MelArgs a) {
  __shared__ cf s_win[kNfft / 2];
  __shared__ cf s_tw256[256];
  __shared__ cf s_tw512[257];
  __shared__ int s_lo[kMaxMels];
  __shared__ float s_w[kMaxMels * kMaxTaps];
  __shared__ cf s_frame[kFramesPerBlock * kFrameC];

  const int tid = threadIdx.x;
  for (int i = tid; i < kNfft / 2; i += kThreads) s_win[i] = cf{a.window[2 * i], a.window[2 * i + 1]};
  for (int i = tid; i < 256; i += kThreads) s_tw256[i] = cf{a.tw256[i].x, a.tw256[i].y};
  for (int i = tid; i < 257; i += kThreads) s_tw512[i] = cf{a.tw512[i].x, a.tw512[i].y};
  for (int i = tid; i < a.n_mels; i += kThreads) s_lo[i] = a.mel_lo[i];
  for (int i = tid; i < a.n_mels * a.taps; i += kThreads) s_w[i] = a.mel_w[i];
  __syncthreads();

  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int slot = wave * kFramesPerWave + (lane >> 4);  // frame slot within the group
  const int j = lane & 15;                               // lane within the frame
  const uint32_t total = static_cast<uint32_t>(a.n_clips * a.n_frames);
  const uint32_t nf = static_cast<uint32_t>(a.n_frames);
  const uint32_t groups = (total + kFramesPerBlock - 1) / kFramesPerBlock;
  cf* buf = s_frame + slot * kFrameC;
  float* pbuf = reinterpret_cast<float*>(buf);

  auto frame_src = [&](uint32_t grp) {
    uint32_t g = min(grp, groups - 1) * kFramesPerBlock + slot;
    g = g < total ? g : total - 1;  // clamp: tail slots recompute a valid frame, store nothing
    const uint32_t clip = g / nf;
    const uint32_t f = g - clip * nf;
    return a.pcm + static_cast<int64_t>(clip) * a.clip_stride + static_cast<int64_t>(f) * a.hop + 2 * j;
  };

  uint32_t grp = blockIdx.x;
  cf x[16];
  if (grp < groups) load_frame(frame_src(grp), x);
  for (; grp < groups; grp += gridDim.x) {
    // 1) window: lane j holds z[16 n1 + j] = (x[32 n1 + 2 j], x[32 n1 + 2 j + 1]) * w
    cf v[16];
#pragma unroll
    for (int n1 = 0; n1 < 16; ++n1) v[n1] = x[n1] * s_win[16 * n1 + j];
    load_frame(frame_src(grp + gridDim.x), x);  // prefetch (clamped past the end)
    // 2) FFT16 over n1, twiddle W256^(j k1), transpose through LDS
    fft16(v);
#pragma unroll
    for (int k1 = 1; k1 < 16; ++k1) v[k1] = cmul(v[k1], s_tw256[j * k1]);
#pragma unroll
    for (int k1 = 0; k1 < 16; ++k1) buf[k1 * kRow + j] = v[k1];
    wave_sync();
#pragma unroll
    for (int n2 = 0; n2 < 16; ++n2) v[n2] = buf[j * kRow + n2];
    // 3) FFT16 over n2: v[k2] = Z[j + 16 k2]
    fft16(v);
    wave_sync();
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2) buf[j + 16 * k2] = v[k2];
    wave_sync();
    // 4) real-FFT split X[k] = Fe + W512^k Fo and |X[k]|^2 for the bins the filters read
    float p[16];
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2) {
      p[k2] = 0.f;
      if (k2 < a.nk2) {
        const int k = j + 16 * k2;
        const cf z = v[k2];
        const cf zc = buf[(256 - k) & 255];
        const cf fe = 0.5f * cf{z.x + zc.x, z.y - zc.y};
        const cf fo = 0.5f * cf{z.y + zc.y, zc.x - z.x};
        const cf xk = fe + cmul(s_tw512[k], fo);
        p[k2] = fmaf(xk.x, xk.x, xk.y * xk.y);
      }
    }
    float p256 = 0.f;
    if (a.need256) {
      const cf z0 = buf[0];
      p256 = (z0.x - z0.y) * (z0.x - z0.y);
    }
    wave_sync();
#pragma unroll
    for (int k2 = 0; k2 < 16; ++k2)
      if (k2 < a.nk2) pbuf[j + 16 * k2] = p[k2];
    if (a.need256 && j == 0) pbuf[256] = p256;
    wave_sync();
    // 5) mel filters: lane j owns mels 2j, 2j+1
    float y[2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int m = 2 * j + q;
      float acc = 0.f;
      if (m < a.n_mels) {
        const int lo = s_lo[m];
        const float* w = &s_w[m * a.taps];
#pragma unroll 4
        for (int t = 0; t < a.taps; ++t) acc = fmaf(w[t], pbuf[lo + t], acc);
      }
      // clamp(min=floor) that keeps NaN (torch.clamp / np.maximum semantics)
      const float c = acc < a.log_floor ? a.log_floor : acc;
      y[q] = 10.f * log10f(c) / a.out_div + a.out_add;
    }
    const uint32_t g = grp * kFramesPerBlock + slot;
    if (g < total && 2 * j < a.n_mels)
      *reinterpret_cast<float2*>(a.out + static_cast<int64_t>(g) * a.n_mels + 2 * j) = make_float2(y[0], y[1]);
    wave_sync();  // the next group's transpose overwrites pbuf
  }
}

}  // namespace
}  // namespace hbk

struct hbk_mel_plan {
  int n_fft, hop, n_mels, taps, nk2, need256;
  float log_floor, out_div, out_add;
  float* d_window = nullptr;
  float2* d_tw256 = nullptr;
  float2* d_tw512 = nullptr;
  int* d_lo = nullptr;
  float* d_w = nullptr;
};

extern "C" {

int hbk_mel_plan_create(const float* window, const float* fbank, int n_fft, int hop, int n_mels,
                        float in_scale, float log_floor, float out_div, float out_add,
                        hbk_mel_plan** plan) {
  using namespace hbk;
  if (!plan) return arg_error("plan is NULL");
  *plan = nullptr;
  if (!window || !fbank) return arg_error("window/fbank is NULL");
  if (n_fft != kNfft) return arg_error("n_fft must be 512");
  if (hop <= 0) return arg_error("hop must be positive");
  if (n_mels <= 0 || n_mels > kMaxMels || (n_mels & 1)) return arg_error("n_mels must be even and <= 32");
  if (out_div == 0.f) return arg_error("out_div must be non-zero");
  const int n_freq = n_fft / 2 + 1;

  // Sparse filterbank: each filter's non-zero bins form one contiguous run.
  std::vector<int> lo(n_mels, 0), hi(n_mels, -1);
  int taps = 1;
  for (int m = 0; m < n_mels; ++m) {
    for (int k = 0; k < n_freq; ++k) {
      if (fbank[k * n_mels + m] != 0.f) {
        if (hi[m] < 0) lo[m] = k;
        hi[m] = k;
      }
    }
    if (hi[m] < 0) { lo[m] = 0; hi[m] = 0; }  // all-zero filter: weights stay 0
    taps = std::max(taps, hi[m] - lo[m] + 1);
  }
  if (taps > kMaxTaps) {
    set_error("hbk: mel filter spans %d bins (> %d supported)", taps, kMaxTaps);
    return HBK_ERR_UNSUPPORTED;
  }
  std::vector<float> w(static_cast<size_t>(n_mels) * taps, 0.f);
  int kmax = 0;
  for (int m = 0; m < n_mels; ++m) {
    if (lo[m] + taps > n_freq) lo[m] = n_freq - taps;  // keep reads inside [0, 257)
    for (int t = 0; t < taps; ++t) w[m * taps + t] = fbank[(lo[m] + t) * n_mels + m];
    kmax = std::max(kmax, lo[m] + taps - 1);
  }
  const int need256 = kmax >= 256 ? 1 : 0;
  const int nk2 = std::min(16, (std::min(kmax, 255) + 16) / 16);

  std::vector<float> win(n_fft);
  for (int i = 0; i < n_fft; ++i) win[i] = window[i] * in_scale;
  std::vector<float2> tw256(256), tw512(257);
  for (int i = 0; i < 256; ++i) {
    const double ang = -2.0 * M_PI * i / 256.0;
    tw256[i] = make_float2(static_cast<float>(cos(ang)), static_cast<float>(sin(ang)));
  }
  for (int i = 0; i < 257; ++i) {
    const double ang = -2.0 * M_PI * i / 512.0;
    tw512[i] = make_float2(static_cast<float>(cos(ang)), static_cast<float>(sin(ang)));
  }

  hbk_mel_plan* p = new hbk_mel_plan();
  p->n_fft = n_fft;
  p->hop = hop;
  p->n_mels = n_mels;
  p->taps = taps;
  p->nk2 = nk2;
  p->need256 = need256;
  p->log_floor = log_floor;
  p->out_div = out_div;
  p->out_add = out_add;
  auto fail = [&](hipError_t e, const char* where) {
    hbk_mel_plan_destroy(p);
    return hip_error(e, where);
  };
  hipError_t e;
  if ((e = hipMalloc(&p->d_window, n_fft * sizeof(float))) != hipSuccess) return fail(e, "hipMalloc window");
  if ((e = hipMalloc(&p->d_tw256, 256 * sizeof(float2))) != hipSuccess) return fail(e, "hipMalloc tw256");
  if ((e = hipMalloc(&p->d_tw512, 257 * sizeof(float2))) != hipSuccess) return fail(e, "hipMalloc tw512");
  if ((e = hipMalloc(&p->d_lo, n_mels * sizeof(int))) != hipSuccess) return fail(e, "hipMalloc lo");
  if ((e = hipMalloc(&p->d_w, w.size() * sizeof(float))) != hipSuccess) return fail(e, "hipMalloc w");
  if ((e = hipMemcpy(p->d_window, win.data(), n_fft * sizeof(float), hipMemcpyHostToDevice)) != hipSuccess)
    return fail(e, "copy window");
  if ((e = hipMemcpy(p->d_tw256, tw256.data(), 256 * sizeof(float2), hipMemcpyHostToDevice)) != hipSuccess)
    return fail(e, "copy tw256");
  if ((e = hipMemcpy(p->d_tw512, tw512.data(), 257 * sizeof(float2), hipMemcpyHostToDevice)) != hipSuccess)
    return fail(e, "copy tw512");
  if ((e = hipMemcpy(p->d_lo, lo.data(), n_mels * sizeof(int), hipMemcpyHostToDevice)) != hipSuccess)
    return fail(e, "copy lo");
  if ((e = hipMemcpy(p->d_w, w.data(), w.size() * sizeof(float), hipMemcpyHostToDevice)) != hipSuccess)
    return fail(e, "copy w");
  *plan = p;
  return HBK_OK;
}

int hbk_mel_plan_destroy(hbk_mel_plan* p) {
  if (!p) return HBK_OK;
  (void)hipFree(p->d_window);
  (void)hipFree(p->d_tw256);
  (void)hipFree(p->d_tw512);
  (void)hipFree(p->d_lo);
  (void)hipFree(p->d_w);
  delete p;
  return HBK_OK;
}

int hbk_mel_frames(const hbk_mel_plan* plan, const float* pcm, int64_t n_clips, int64_t clip_stride,
                   int64_t n_frames, float* out, void* stream) {
  using namespace hbk;
  if (!plan) return arg_error("plan is NULL");
  if (n_clips < 0 || n_frames < 0) return arg_error("negative size");
  if (n_clips == 0 || n_frames == 0) return HBK_OK;
  if (!pcm || !out) return arg_error("pcm/out is NULL");
  if ((clip_stride & 1) || (plan->hop & 1)) return arg_error("clip_stride and hop must be even (float2 loads)");
  if ((reinterpret_cast<uintptr_t>(pcm) & 7) || (reinterpret_cast<uintptr_t>(out) & 7))
    return arg_error("pcm/out must be 8-byte aligned");
  if (plan->hop * (n_frames - 1) + plan->n_fft > clip_stride) return arg_error("frames exceed clip_stride");
  MelArgs a;
  a.pcm = pcm;
  a.out = out;
  a.window = plan->d_window;
  a.tw256 = plan->d_tw256;
  a.tw512 = plan->d_tw512;
  a.mel_lo = plan->d_lo;
  a.mel_w = plan->d_w;
  a.n_clips = n_clips;
  a.clip_stride = clip_stride;
  a.n_frames = n_frames;
  a.hop = plan->hop;
  a.n_mels = plan->n_mels;
  a.taps = plan->taps;
  a.nk2 = plan->nk2;
  a.need256 = plan->need256;
  a.log_floor = plan->log_floor;
  a.out_div = plan->out_div;
  a.out_add = plan->out_add;
  const int64_t total = n_clips * n_frames;
  if (total >= (int64_t(1) << 31)) return arg_error("more than 2^31 frames in one call");
  const int64_t groups = (total + kFramesPerBlock - 1) / kFramesPerBlock;
  const int64_t blocks = std::min<int64_t>(groups, persistent_blocks(kBlocksPerCU));
  hipLaunchKernelGGL(mel_frames_kernel, dim3(static_cast<unsigned>(blocks)), dim3(kThreads), 0,
                     as_stream(stream), a);
  HBK_LAUNCH_CHECK("mel_frames_kernel");
  return HBK_OK;
}

}  // extern "C"
