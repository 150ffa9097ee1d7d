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
#include <cstdlib>
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

// Scalar-pair complex: the same arithmetic as cf issued as single-lane f32
// ops instead of v_pk_*_f32 (the v2 kernel picks one with a template argument).
struct sc {
  float x, y;
};
using hbk::cadd;
using hbk::cmul;
using hbk::cmul_mi;
using hbk::csub;
__device__ __forceinline__ sc operator+(sc a, sc b) { return {a.x + b.x, a.y + b.y}; }
__device__ __forceinline__ sc operator-(sc a, sc b) { return {a.x - b.x, a.y - b.y}; }
__device__ __forceinline__ sc operator*(sc a, sc b) { return {a.x * b.x, a.y * b.y}; }  // elementwise
__device__ __forceinline__ sc cadd(sc a, sc b) { return a + b; }
__device__ __forceinline__ sc csub(sc a, sc b) { return a - b; }
__device__ __forceinline__ sc cmul_mi(sc a) { return {a.y, -a.x}; }
__device__ __forceinline__ sc cmul(sc a, sc b) {
  return {fmaf(a.x, b.x, -a.y * b.y), fmaf(a.x, b.y, a.y * b.x)};
}
template <class C>
__device__ __forceinline__ C cpx(cf v) { return C{v.x, v.y}; }

template <class C>
__device__ __forceinline__ void fft4(C& a0, C& a1, C& a2, C& a3) {
  const C t0 = cadd(a0, a2), t1 = csub(a0, a2);
  const C t2 = cadd(a1, a3), t3 = cmul_mi(csub(a1, a3));
  a0 = cadd(t0, t2);
  a2 = csub(t0, t2);
  a1 = cadd(t1, t3);
  a3 = csub(t1, t3);
}

// In-register 16-point forward DFT: v[k] <- sum_n v[n] W16^(nk), natural order.
template <class C>
__device__ __forceinline__ void fft16(C (&v)[16]) {
  // n = 4 m1 + m2: radix-4 over m1 for each m2 -> v[4 l1 + m2] = A[m2][l1]
#pragma unroll
  for (int m2 = 0; m2 < 4; ++m2) fft4(v[m2], v[4 + m2], v[8 + m2], v[12 + m2]);
#pragma unroll
  for (int l1 = 1; l1 < 4; ++l1)
#pragma unroll
    for (int m2 = 1; m2 < 4; ++m2) v[4 * l1 + m2] = cmul(v[4 * l1 + m2], cpx<C>(w16(m2 * l1)));
  // radix-4 over m2 for each l1 -> v[4 l1 + l2] = X[l1 + 4 l2]
#pragma unroll
  for (int l1 = 0; l1 < 4; ++l1) fft4(v[4 * l1 + 0], v[4 * l1 + 1], v[4 * l1 + 2], v[4 * l1 + 3]);
  C t[16];
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

// ------------------------------------------------------------------ v2 ----
// The same transform, specialised for the filterbanks the reference uses
// (32 mels reading only bins k < 128, e.g. H0's 60-3800 Hz bank) and cut for
// LDS traffic / bank conflicts and VALU count, the resources the v1 kernel is
// bound by (rocprofv3 SQ counters: LDS array busy ~60-75 % of the kernel):
//  - the window is a per-lane VGPR constant; W256 twiddles, split twiddles
//    -i W512^k and filter weights are a [entry][lane] LDS table whose b64
//    reads are conflict-free and broadcast to the wave's 4 frames (v1 reads
//    its tables with bank conflicts); 8-wave blocks share it, 4 waves / SIMD;
//  - the real-FFT split's partner Z[256 - k] comes from lane (16 - j) mod 16
//    of the same frame through two DPP moves (row_mirror, row_ror:1) instead
//    of a second LDS round trip; lane 0 takes its own register;
//  - only the 8 blocks of 16 bins the filters read are split and squared;
//  - a window that is zero on its first and last 32 samples (win_length 400
//    centred in 512) skips the n1 = 0 and n1 = 15 rows (EDGE0);
//  - the transpose reads are 16-B ds_read_b128 (rows of 18 complex, frame
//    regions 9 x 256 B so the two frames of a b128 lane group hit disjoint
//    banks);
//  - mel filters are balanced over lanes: lane j computes the narrow filter j
//    (8 bins) and the wide filter 31 - j (16 bins) from even start bins with
//    8-B reads; odd frames' power rows
//    sit 32 dwords up so a lane group's two frames read disjoint banks;
//  - the 1/2 of the split is folded into the filter weights (x 1/4 on |X|^2,
//    exact in binary floating point).
constexpr int kRow2 = 18;
constexpr int kFrameC2 = 16 * kRow2;  // 288 complex = 2304 B
constexpr int kTapsA = 8;             // filters 0..15
constexpr int kTapsB = 16;            // filters 16..31
constexpr int kBins2 = 128;
constexpr int kWaves2 = 8;            // 512-thread blocks sharing one constant table
constexpr int kThreads2 = 64 * kWaves2;
constexpr int kFramesPerBlock2 = kFramesPerWave * kWaves2;
constexpr int kBlocksPerCU2 = 2;      // <= 128 VGPRs, 80 KB LDS: 4 waves / SIMD

struct Mel2Args {
  const float* pcm;
  float* out;
  const float* window;  // [512], in_scale folded in
  const float2* tw256;  // [256] W256^i
  const float2* twsm;   // [128] -i W512^k
  const int* mel_lo2;   // [32]: lo(filter j), lo(filter 31 - j) at [j], [16 + j]; even, in-range
  const float* mel_w2;  // [16][kTapsA] then [16][kTapsB], x 1/4, zero-padded
  int64_t n_clips;
  int64_t clip_stride;
  int64_t n_frames;
  int hop;
  float log_floor;
  float out_scale;  // 10 / out_div
  float out_add;
};

// lane j >= 1 of each 16-lane row receives v from lane 16 - j; lane 0 keeps
// `own`: row_mirror (mirror()), then row_shr:1 (shr1_or()) whose out-of-row
// source leaves lane 0's old value in place (bound_ctrl off). All mirrors of
// a group are issued before the shifts (no DPP read-after-write nops).
__device__ __forceinline__ int mirror(float v) {
  return __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), 0x140, 0xF, 0xF, false);
}
__device__ __forceinline__ float shr1_or(int t, float own) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, own), t, 0x111,
                                                               0xF, 0xF, false));
}

// per-lane constant table in LDS, [entry][lane j] (16-lane rows: conflict-free
// b64 reads, broadcast over a wave's 4 frames)
constexpr int kCTw = 0;                   // 16 entries: W256^(j k1)
constexpr int kCWs = 16;                  // 8 entries: -i W512^(j + 16 k2)
constexpr int kCWa = 24;                  // kTapsA / 2 pairs: weights of filter j
constexpr int kCWb = kCWa + kTapsA / 2;   // kTapsB / 2 pairs: weights of filter 31 - j
constexpr int kCWin = kCWb + kTapsB / 2;  // 16 entries: window pair (w[32 n1 + 2 j], w[32 n1 + 2 j + 1])
constexpr int kCN = kCWin + 16;           // 52 entries = 6.5 KB

// (Computing the twiddles from 4 table reads + products, or the split twiddles
// from one read x W32^k2, trades LDS reads for VALU: measured 2-5 % slower.)
template <bool EDGE0, class C>
__global__ void __launch_bounds__(kThreads2) __attribute__((amdgpu_waves_per_eu(4)))
mel_frames_v2_kernel(Mel2Args a) {
  __shared__ __attribute__((aligned(16))) cf s_frame[kFramesPerBlock2 * kFrameC2];
  __shared__ __attribute__((aligned(16))) cf s_c[kCN * 16];

  const int tid = threadIdx.x;
  for (int i = tid; i < kCN * 16; i += kThreads2) {
    const int e = i >> 4, jj = i & 15;
    cf c;
    if (e < kCWs) {
      const float2 t = a.tw256[(jj * e) & 255];
      c = cf{t.x, t.y};
    } else if (e < kCWa) {
      const float2 t = a.twsm[jj + 16 * (e - kCWs)];
      c = cf{t.x, t.y};
    } else if (e < kCWb) {
      c = *reinterpret_cast<const cf*>(a.mel_w2 + jj * kTapsA + 2 * (e - kCWa));
    } else if (e < kCWin) {
      c = *reinterpret_cast<const cf*>(a.mel_w2 + 16 * kTapsA + jj * kTapsB + 2 * (e - kCWb));
    } else {
      c = *reinterpret_cast<const cf*>(a.window + 2 * (16 * (e - kCWin) + jj));
    }
    s_c[i] = c;
  }
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int slot = wave * kFramesPerWave + (lane >> 4);
  const int j = lane & 15;
  const cf* cj = s_c + j;  // entry e of this lane: cj[16 e]
  __syncthreads();

  const uint32_t total = static_cast<uint32_t>(a.n_clips * a.n_frames);
  const uint32_t nf = static_cast<uint32_t>(a.n_frames);
  const uint32_t groups = (total + kFramesPerBlock2 - 1) / kFramesPerBlock2;
  cf* buf = s_frame + slot * kFrameC2;
  float* pbuf = reinterpret_cast<float*>(buf) + (slot & 1) * 32;
  const float* pA = pbuf + a.mel_lo2[j];
  const float* pB = pbuf + a.mel_lo2[16 + j];
  constexpr int n1lo = EDGE0 ? 1 : 0, n1hi = EDGE0 ? 15 : 16;

  auto frame_src = [&](uint32_t grp) {
    uint32_t g = min(grp, groups - 1) * kFramesPerBlock2 + slot;
    g = g < total ? g : total - 1;
    const uint32_t clip = g / nf;
    const uint32_t f = g - clip * nf;
    return a.pcm + static_cast<int64_t>(clip) * a.clip_stride + static_cast<int64_t>(f) * a.hop + 2 * j;
  };
  auto load = [&](const float* src, C (&x)[16]) {
#pragma unroll
    for (int n1 = n1lo; n1 < n1hi; ++n1) x[n1] = cpx<C>(*reinterpret_cast<const cf*>(src + 32 * n1));
  };
  auto to_log = [&](float acc) {
    const float c = acc < a.log_floor ? a.log_floor : acc;  // keeps NaN
    return __log10f(c) * a.out_scale + a.out_add;  // v_log_f32 (log2) x log10(2): ~1e-7 against the 1e-4 tolerance
  };

  // one group: transform the frames in `cur`, prefetching group grp + stride into `nxt`
  auto process = [&](uint32_t grp, const C (&cur)[16], C (&nxt)[16]) {
    // window and twiddles come from the LDS table in two batches of reads
    // (one wait each) instead of VGPR-resident window + per-use twiddle reads
    C v[16];
#pragma unroll
    for (int n1 = n1lo; n1 < n1hi; ++n1) v[n1] = cpx<C>(cj[16 * (kCWin + n1)]);
    C tw[16];
#pragma unroll
    for (int k1 = 1; k1 < 16; ++k1) tw[k1] = cpx<C>(cj[16 * (kCTw + k1)]);
#pragma unroll
    for (int n1 = 0; n1 < 16; ++n1) v[n1] = (n1 < n1lo || n1 >= n1hi) ? C{0.f, 0.f} : cur[n1] * v[n1];
    load(frame_src(grp + gridDim.x), nxt);  // prefetch (clamped past the end)
    fft16(v);
#pragma unroll
    for (int k1 = 1; k1 < 16; ++k1) v[k1] = cmul(v[k1], tw[k1]);
#pragma unroll
    for (int k1 = 0; k1 < 16; ++k1) buf[k1 * kRow2 + j] = cf{v[k1].x, v[k1].y};
    wave_sync();
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float4 t = *reinterpret_cast<const float4*>(buf + j * kRow2 + 2 * q);
      v[2 * q] = C{t.x, t.y};
      v[2 * q + 1] = C{t.z, t.w};
    }
    C ws[8];
#pragma unroll
    for (int k2 = 0; k2 < 8; ++k2) ws[k2] = cpx<C>(cj[16 * (kCWs + k2)]);
    fft16(v);  // v[k2] = Z[j + 16 k2]
    // 2 X[k] = (Z[k] + Z*[256-k]) + (-i W512^k) (Z[k] - Z*[256-k]),  k = j + 16 k2
    float p[8];
    int mx[8], my[8];
#pragma unroll
    for (int k2 = 0; k2 < 8; ++k2) {
      mx[k2] = mirror(v[15 - k2].x);
      my[k2] = mirror(v[15 - k2].y);
    }
#pragma unroll
    for (int k2 = 0; k2 < 8; ++k2) {
      const C own = v[(16 - k2) & 15];  // lane 0: Z[256 - 16 k2] is its own
      const C zr = C{shr1_or(mx[k2], own.x), shr1_or(my[k2], own.y)};
      const C zc = C{zr.x, -zr.y};  // Z*[256 - k]
      const C s = v[k2] + zc;
      const C d = v[k2] - zc;
      const C X = s + cmul(d, ws[k2]);
      p[k2] = fmaf(X.x, X.x, X.y * X.y);
    }
    wave_sync();
#pragma unroll
    for (int k2 = 0; k2 < 8; ++k2) pbuf[j + 16 * k2] = p[k2];
    wave_sync();
    float accA = 0.f, accB = 0.f;
#pragma unroll
    for (int t = 0; t < kTapsA; t += 2) {
      const float2 pv = *reinterpret_cast<const float2*>(pA + t);
      const cf w = cj[16 * (kCWa + t / 2)];
      accA = fmaf(w.x, pv.x, accA);
      accA = fmaf(w.y, pv.y, accA);
    }
#pragma unroll
    for (int t = 0; t < kTapsB; t += 2) {
      const float2 pv = *reinterpret_cast<const float2*>(pB + t);
      const cf w = cj[16 * (kCWb + t / 2)];
      accB = fmaf(w.x, pv.x, accB);
      accB = fmaf(w.y, pv.y, accB);
    }
    const uint32_t g = grp * kFramesPerBlock2 + slot;
    if (g < total) {
      float* o = a.out + static_cast<int64_t>(g) * kMaxMels;
      o[j] = to_log(accA);
      o[31 - j] = to_log(accB);
    }
    wave_sync();  // the next group's transpose overwrites pbuf
  };

  // two explicit prefetch buffers (no register copies on the loop back edge)
  uint32_t grp = blockIdx.x;
  C xa[16], xb[16];
  if (grp < groups) load(frame_src(grp), xa);
  while (grp < groups) {
    process(grp, xa, xb);
    grp += gridDim.x;
    if (grp >= groups) break;
    process(grp, xb, xa);
    grp += gridDim.x;
  }
}


// ------------------------------------------------------------------ v3 ----
// The MFMA filterbank variant (BASELINE north_star: "MFMA used only for the
// mel-filterbank x power-spectrum ... contractions"): the transform of v2, then
// the 32-mel filterbank as a dense [frames x 128 bins] x [128 x 32] product on
// v_mfma_f32_16x16x32_bf16 instead of the sparse per-lane dot products.
//  - f32-range operands: the power row and the weights are split into bf16
//    hi / lo pairs (hi = bf16(x), lo = bf16(x - hi): 16 significant bits, f32's
//    exponent range). A frame's bins span more than f16's range after any one
//    scale (a DC clip: ~1e14 at bin 0 against ~1 in the upper filters, which
//    an f16 split with a per-frame scale flushed to zero), bf16 keeps them.
//    hi*hi + hi*lo + lo*hi, f32 accumulation: ~2^-16 relative per product, and
//    the sums are of non-negative terms (no cancellation): ~1e-5 of log10,
//    inside the 1e-4 output tolerance;
//  - a wave holds 4 frames, an MFMA tile 16 rows: row 4 q + f holds frame f's
//    bins of quarter q (32 bins, the 32-deep k-block q; zero elsewhere), so each
//    lane fetches ONE k-block of one frame from the power row in LDS and the
//    4 k-blocks x 2 mel tiles x 3 products = 24 MFMAs give the 4 quarters'
//    partial sums in 4 rows each; a reduce-scatter over the quarters
//    (v_permlane32_swap, v_permlane16_swap) leaves frame kq's two mels on lane
//    (n, kq), i.e. the log of v2's 2 values per lane;
//  - 6-wave blocks (2 per CU: the split weight planes take 17 KB of LDS).
// The dense product multiplies ~4x the non-zero taps, on the matrix pipe.
constexpr int kWaves3 = 6;
constexpr int kThreads3 = 64 * kWaves3;
constexpr int kFramesPerBlock3 = kFramesPerWave * kWaves3;
constexpr int kBlocksPerCU3 = 2;
constexpr int kWLd3 = kBins2 + 8;  // bf16 per mel row of a weight plane (bank spread)
typedef __bf16 h8m __attribute__((ext_vector_type(8)));
typedef __bf16 h2m __attribute__((ext_vector_type(2)));
typedef float f2m __attribute__((ext_vector_type(2)));
typedef float f4m __attribute__((ext_vector_type(4)));

struct Mel3Args {
  const float* pcm;
  float* out;
  const float* window;  // [512], in_scale folded in
  const float2* tw256;  // [256] W256^i
  const float2* twsm;   // [128] -i W512^k
  const float* fbt;     // [32][128] filterbank^T x 1/4 (the split's 1/2, squared)
  int64_t n_clips;
  int64_t clip_stride;
  int64_t n_frames;
  int hop;
  float log_floor;
  float out_scale;  // 10 / out_div
  float out_add;
};

__device__ __forceinline__ void split8m(const float (&v)[8], h8m& hi, h8m& lo) {
#pragma unroll
  for (int e = 0; e < 8; e += 2) {
    const h2m h = __builtin_convertvector(f2m{v[e], v[e + 1]}, h2m);
    const f2m r = f2m{v[e], v[e + 1]} - __builtin_convertvector(h, f2m);
    const h2m l = __builtin_convertvector(r, h2m);
    hi[e] = h[0];
    hi[e + 1] = h[1];
    lo[e] = l[0];
    lo[e + 1] = l[1];
  }
}
// reduce-scatter across lane ^ 16 / lane ^ 32 (v_permlane*_swap; see hbk_augment.hip's pv_swap_add)
template <bool kSwap16>
__device__ __forceinline__ float mel_swap_add(float x, float y) {
  if (kSwap16)
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\ts_nop 1" : "+v"(x), "+v"(y));
  else
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1" : "+v"(x), "+v"(y));
  return x + y;
}

template <bool EDGE0, class C>
__global__ void __launch_bounds__(kThreads3) __attribute__((amdgpu_waves_per_eu(3)))
mel_frames_mfma_kernel(Mel3Args a) {
  __shared__ __attribute__((aligned(16))) cf s_frame[kFramesPerBlock3 * kFrameC2];
  __shared__ __attribute__((aligned(16))) cf s_c[kCWa * 16 + 16 * 16];  // tw (16), ws (8), window (16)
  __shared__ __attribute__((aligned(16))) __bf16 s_w[2][kMaxMels][kWLd3];
  constexpr int kCWin3 = kCWa;  // window entries follow the twiddles here
  const int tid = threadIdx.x;
  for (int i = tid; i < (kCWin3 + 16) * 16; i += kThreads3) {
    const int e = i >> 4, jj = i & 15;
    cf c;
    if (e < kCWs) {
      const float2 t = a.tw256[(jj * e) & 255];
      c = cf{t.x, t.y};
    } else if (e < kCWa) {
      const float2 t = a.twsm[jj + 16 * (e - kCWs)];
      c = cf{t.x, t.y};
    } else {
      c = *reinterpret_cast<const cf*>(a.window + 2 * (16 * (e - kCWin3) + jj));
    }
    s_c[i] = c;
  }
  for (int i = tid; i < kMaxMels * kBins2 / 2; i += kThreads3) {
    const int m = i / (kBins2 / 2), k = 2 * (i % (kBins2 / 2));
    const float w0 = a.fbt[m * kBins2 + k], w1 = a.fbt[m * kBins2 + k + 1];
    const h2m h = __builtin_convertvector(f2m{w0, w1}, h2m);
    const h2m l = __builtin_convertvector(f2m{w0, w1} - __builtin_convertvector(h, f2m), h2m);
    *reinterpret_cast<h2m*>(&s_w[0][m][k]) = h;
    *reinterpret_cast<h2m*>(&s_w[1][m][k]) = l;
  }
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int slot = wave * kFramesPerWave + (lane >> 4);
  const int j = lane & 15;
  const int kq = lane >> 4;  // MFMA lane group (== the frame slot of the transform)
  const cf* cj = s_c + j;
  __syncthreads();

  const uint32_t total = static_cast<uint32_t>(a.n_clips * a.n_frames);
  const uint32_t nf = static_cast<uint32_t>(a.n_frames);
  const uint32_t groups = (total + kFramesPerBlock3 - 1) / kFramesPerBlock3;
  cf* buf = s_frame + slot * kFrameC2;
  float* pbuf = reinterpret_cast<float*>(buf) + (slot & 1) * 32;
  // MFMA operand rows: row m = 4 q + f reads frame f's quarter q
  const int mq = j >> 2, mf = j & 3;
  const float* arow = reinterpret_cast<const float*>(s_frame + (wave * kFramesPerWave + mf) * kFrameC2) +
                      (mf & 1) * 32 + 32 * mq + 8 * kq;
  constexpr int n1lo = EDGE0 ? 1 : 0, n1hi = EDGE0 ? 15 : 16;

  auto frame_src = [&](uint32_t grp) {
    uint32_t g = min(grp, groups - 1) * kFramesPerBlock3 + slot;
    g = g < total ? g : total - 1;
    const uint32_t clip = g / nf;
    const uint32_t f = g - clip * nf;
    return a.pcm + static_cast<int64_t>(clip) * a.clip_stride + static_cast<int64_t>(f) * a.hop + 2 * j;
  };
  auto load = [&](const float* src, C (&x)[16]) {
#pragma unroll
    for (int n1 = n1lo; n1 < n1hi; ++n1) x[n1] = cpx<C>(*reinterpret_cast<const cf*>(src + 32 * n1));
  };

  auto process = [&](uint32_t grp, const C (&cur)[16], C (&nxt)[16]) {
    C v[16];
#pragma unroll
    for (int n1 = n1lo; n1 < n1hi; ++n1) v[n1] = cpx<C>(cj[16 * (kCWin3 + n1)]);
    C tw[16];
#pragma unroll
    for (int k1 = 1; k1 < 16; ++k1) tw[k1] = cpx<C>(cj[16 * (kCTw + k1)]);
#pragma unroll
    for (int n1 = 0; n1 < 16; ++n1) v[n1] = (n1 < n1lo || n1 >= n1hi) ? C{0.f, 0.f} : cur[n1] * v[n1];
    load(frame_src(grp + gridDim.x), nxt);  // prefetch (clamped past the end)
    fft16(v);
#pragma unroll
    for (int k1 = 1; k1 < 16; ++k1) v[k1] = cmul(v[k1], tw[k1]);
#pragma unroll
    for (int k1 = 0; k1 < 16; ++k1) buf[k1 * kRow2 + j] = cf{v[k1].x, v[k1].y};
    wave_sync();
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const float4 t = *reinterpret_cast<const float4*>(buf + j * kRow2 + 2 * q);
      v[2 * q] = C{t.x, t.y};
      v[2 * q + 1] = C{t.z, t.w};
    }
    C ws[8];
#pragma unroll
    for (int k2 = 0; k2 < 8; ++k2) ws[k2] = cpx<C>(cj[16 * (kCWs + k2)]);
    fft16(v);
    float p[8];
    int mx[8], my[8];
#pragma unroll
    for (int k2 = 0; k2 < 8; ++k2) {
      mx[k2] = mirror(v[15 - k2].x);
      my[k2] = mirror(v[15 - k2].y);
    }
#pragma unroll
    for (int k2 = 0; k2 < 8; ++k2) {
      const C own = v[(16 - k2) & 15];
      const C zr = C{shr1_or(mx[k2], own.x), shr1_or(my[k2], own.y)};
      const C zc = C{zr.x, -zr.y};
      const C s = v[k2] + zc;
      const C d = v[k2] - zc;
      const C X = s + cmul(d, ws[k2]);
      p[k2] = fmaf(X.x, X.x, X.y * X.y);
    }
    wave_sync();
#pragma unroll
    for (int k2 = 0; k2 < 8; ++k2) pbuf[j + 16 * k2] = p[k2];
    wave_sync();
    // A: this lane's quarter of its frame (row 4 mq + mf), zero in the other k-blocks
    float av[8];
    {
      const float4 t0 = *reinterpret_cast<const float4*>(arow), t1 = *reinterpret_cast<const float4*>(arow + 4);
      av[0] = t0.x; av[1] = t0.y; av[2] = t0.z; av[3] = t0.w;
      av[4] = t1.x; av[5] = t1.y; av[6] = t1.z; av[7] = t1.w;
    }
    h8m ah, al;
    split8m(av, ah, al);
    const h8m hz = {};
    f4m acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const h8m aih = mq == i ? ah : hz, ail = mq == i ? al : hz;
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        const h8m bh = *reinterpret_cast<const h8m*>(&s_w[0][16 * ct + j][32 * i + 8 * kq]);
        const h8m bl = *reinterpret_cast<const h8m*>(&s_w[1][16 * ct + j][32 * i + 8 * kq]);
        acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aih, bh, acc[ct], 0, 0, 0);
        acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aih, bl, acc[ct], 0, 0, 0);
        acc[ct] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ail, bh, acc[ct], 0, 0, 0);
      }
    }
    // lane (n, kq) holds quarter kq of frames 0..3: reduce-scatter over the quarters -> frame kq
    float y[2];
#pragma unroll
    for (int ct = 0; ct < 2; ++ct) {
      const float w0 = mel_swap_add<false>(acc[ct][0], acc[ct][2]);  // frames 0 / 2 (lane bit 5)
      const float w1 = mel_swap_add<false>(acc[ct][1], acc[ct][3]);  // frames 1 / 3
      y[ct] = mel_swap_add<true>(w0, w1);                            // frame 2 (kq >> 1) + (kq & 1) = kq
    }
    const uint32_t g = grp * kFramesPerBlock3 + wave * kFramesPerWave + kq;
    if (g < total) {
      float* o = a.out + static_cast<int64_t>(g) * kMaxMels;
#pragma unroll
      for (int ct = 0; ct < 2; ++ct) {
        const float acc1 = y[ct];
        const float c = acc1 < a.log_floor ? a.log_floor : acc1;  // keeps NaN
        o[16 * ct + j] = __log10f(c) * a.out_scale + a.out_add;
      }
    }
    wave_sync();  // the next group's transpose overwrites the frame buffers
  };

  uint32_t grp = blockIdx.x;
  C xa[16], xb[16];
  if (grp < groups) load(frame_src(grp), xa);
  while (grp < groups) {
    process(grp, xa, xb);
    grp += gridDim.x;
    if (grp >= groups) break;
    process(grp, xb, xa);
    grp += gridDim.x;
  }
}
// ------------------------------------------------------------------ v4 ----
// The v2 transform with every float op packed: a lane carries TWO columns of
// one frame (8 lanes per frame, 8 frames per wave), as SoA pairs -- re of
// both columns in one 64-bit register pair, im of both in another -- so each
// v_pk_{add,mul,fma}_f32 does the work of two scalar ops of v2 with no
// re / im swaps (v2's AoS packed form, HBK_MEL_PACKED, spent ~20 % of its
// instructions on v_mov / v_xor to swap and negate halves; multiplying by -i
// here is a renaming). v2 runs at ~82 % VALU issue (PMC r03): the instruction
// count per frame is its bound.
//  - stage A: lane jj holds columns jj and jj + 8 of z[16 n1 + n2]; FFT16 over
//    n1, twiddles W256^(n2 k1) as (jj, jj + 8) pairs from the [entry][lane] table;
//  - transpose through LDS as re / im planes, rows stored in the order
//    0, 8, 1, 15, 2, 14, ... (row k1 beside row 16 - k1), so that in stage B
//    lane kk reads its row pair (kk, 16 - kk) (kk = 0: rows 0, 8) with
//    ds_read2_b32 at one base;
//  - FFT16 over n2: lane kk holds Z[k1 + 16 k2] for k1 = kk and 16 - kk, so the
//    real-FFT split's partner Z[256 - k] sits in the SAME lane's other half
//    (kk = 0: rows 0 and 8 are their own partners): no cross-lane moves;
//  - power to LDS, then 4 mel filters per lane (two of the <= 8-tap set, two
//    of the <= 16-tap set: v2's slots jj and jj + 8) as packed dot products.
// LDS per frame: one 280-dword buffer that carries the transpose one plane at a time
// (re, then im: half the LDS of both planes at once, so 3 blocks fit a CU) and then
// the power row. Transform row k1 sits at LDS row row5(k1) = the pair index p of
// (p, 16 - p) (rows 0, 8: pair 0), its partner 16 - p at row p + 8, so stage B's lane
// jj reads rows jj and jj + 8. Frame bases 280 = 24 mod 32 apart put the 4 frames of
// a 32-lane LDS group on disjoint banks: the stage-A stores (bank 24 f + jj), the
// stage-B reads (24 f + 17 jj + n2) and the power stores are conflict-free
// (tools/lds_bank_sim.py; the first 577-dword layout ran the stores 4-way). The power
// row sits at +24 (f & 1) + 8 (f >> 1 & 1) (8-B aligned pairs for the filter reads).
constexpr int kFramesPerWave4 = 8;
constexpr int kLdt4 = 17, kFs4 = 280;
constexpr int kBlocksPerCU4 = 3;  // 3 x (35 KB frames + 6.5 KB table) of LDS, <= 168 VGPRs
// constant table [entry][8 lanes] of float4
constexpr int kE4Win = 0;           // 16: (w[32 n1 + 2jj], w[.. + 16], w[.. + 1], w[.. + 17])
constexpr int kE4Tw = 16;           // 16 (k1 = 0 unused): (Re W^(jj k1), Re W^((jj+8) k1), Im .., Im ..)
constexpr int kE4Ws = 32;           // 8: -i W512^k for bins (ra + 16 k2, rb + 16 k2), re pair, im pair
constexpr int kE4Mel = 40;          // 12: weights of A slots jj, jj + 8 (8 each), B slots jj, jj + 8 (16 each)
constexpr int kE4N = 52;

struct P2 {
  cf r, i;
};
__device__ __forceinline__ P2 operator+(P2 a, P2 b) { return {a.r + b.r, a.i + b.i}; }
__device__ __forceinline__ P2 operator-(P2 a, P2 b) { return {a.r - b.r, a.i - b.i}; }
// a * (cr + i ci), per-half constants
__device__ __forceinline__ P2 pmul(P2 a, cf cr, cf ci) {
  return {__builtin_elementwise_fma(a.r, cr, -(a.i * ci)), __builtin_elementwise_fma(a.r, ci, a.i * cr)};
}
__device__ __forceinline__ cf bc(float v) { return cf{v, v}; }
__device__ __forceinline__ void fft4p(P2& a0, P2& a1, P2& a2, P2& a3) {
  const P2 t0 = a0 + a2, t1 = a0 - a2, t2 = a1 + a3, d = a1 - a3;
  a0 = t0 + t2;
  a2 = t0 - t2;
  a1 = P2{t1.r + d.i, t1.i - d.r};  // t1 - i d
  a3 = P2{t1.r - d.i, t1.i + d.r};  // t1 + i d
}
// a * W16^p for the products p = m2 l1 of fft16 (1, 2, 3, 4, 6, 9)
template <int p>
__device__ __forceinline__ P2 w16p(P2 a) {
  constexpr float c1 = 0.92387953251128674f, s1 = 0.38268343236508978f, r = 0.70710678118654757f;
  if constexpr (p == 4) return P2{a.i, -a.r};
  if constexpr (p == 2) return P2{bc(r) * (a.r + a.i), bc(r) * (a.i - a.r)};
  if constexpr (p == 6) return P2{bc(r) * (a.i - a.r), bc(-r) * (a.r + a.i)};
  if constexpr (p == 1) return pmul(a, bc(c1), bc(-s1));
  if constexpr (p == 3) return pmul(a, bc(s1), bc(-c1));
  return pmul(a, bc(-c1), bc(s1));  // p = 9
}
__device__ __forceinline__ void fft16p(P2 (&v)[16]) {
#pragma unroll
  for (int m2 = 0; m2 < 4; ++m2) fft4p(v[m2], v[4 + m2], v[8 + m2], v[12 + m2]);
  v[5] = w16p<1>(v[5]);
  v[6] = w16p<2>(v[6]);
  v[7] = w16p<3>(v[7]);
  v[9] = w16p<2>(v[9]);
  v[10] = w16p<4>(v[10]);
  v[11] = w16p<6>(v[11]);
  v[13] = w16p<3>(v[13]);
  v[14] = w16p<6>(v[14]);
  v[15] = w16p<9>(v[15]);
#pragma unroll
  for (int l1 = 0; l1 < 4; ++l1) fft4p(v[4 * l1 + 0], v[4 * l1 + 1], v[4 * l1 + 2], v[4 * l1 + 3]);
  P2 t[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) t[k] = v[4 * (k & 3) + (k >> 2)];
#pragma unroll
  for (int k = 0; k < 16; ++k) v[k] = t[k];
}
// LDS row of transform row k1: pair index p of rows (p, 16 - p), +8 for the second
// of the pair (row 0 -> 0, row 8 -> 8)
__device__ __forceinline__ constexpr int row5(int k1) {
  return k1 == 0 ? 0 : k1 == 8 ? 8 : k1 < 8 ? k1 : 16 - k1 + 8;
}

struct Mel4Args {
  const float* pcm;
  float* out;
  const float4* table;  // [kE4N][8]
  const int* mel_lo2;   // v2's [32]
  int64_t n_clips;
  int64_t clip_stride;
  int64_t n_frames;
  int hop;
  float log_floor;
  float out_scale;  // 10 / out_div
  float out_add;
};

// W waves per block. W = 4: the next group's samples are prefetched into a second register
// buffer (<= 168 VGPRs, 3 waves / SIMD, 3 blocks / CU); W = 8: no prefetch (<= 128 VGPRs,
// 4 waves / SIMD: two 8-wave blocks share a CU's LDS)
template <bool EDGE0, int W>
__global__ void __launch_bounds__(64 * W) __attribute__((amdgpu_waves_per_eu(W == 4 ? 3 : 4)))
mel_frames_soa_kernel(Mel4Args a) {
  constexpr int kFPB = kFramesPerWave4 * W;
  __shared__ float s_fr[kFPB * kFs4];
  __shared__ __attribute__((aligned(16))) float4 s_t[kE4N * 8];
  const int tid = threadIdx.x;
  for (int i = tid; i < kE4N * 8; i += 64 * W) s_t[i] = a.table[i];
  const int wave = tid >> 6, lane = tid & 63;
  const int f = lane >> 3, jj = lane & 7;
  const int slot = wave * kFramesPerWave4 + f;
  const float4* tj = s_t + jj;  // entry e: tj[8 e]
  float* fr = s_fr + slot * kFs4;
  float* pw = fr + 24 * (f & 1) + 8 * ((f >> 1) & 1);  // the power row (8-B aligned pairs)
  const int ra = jj == 0 ? 0 : jj, rb = jj == 0 ? 8 : 16 - jj;  // stage-B rows of this lane
  const float* rowsB = fr + jj * kLdt4;                           // LDS rows jj, jj + 8
  const int loA0 = a.mel_lo2[jj], loA1 = a.mel_lo2[jj + 8];
  const int loB0 = a.mel_lo2[16 + jj], loB1 = a.mel_lo2[16 + jj + 8];
  __syncthreads();

  const uint32_t total = static_cast<uint32_t>(a.n_clips * a.n_frames);
  const uint32_t nf = static_cast<uint32_t>(a.n_frames);
  const uint32_t groups = (total + kFPB - 1) / kFPB;
  constexpr int n1lo = EDGE0 ? 1 : 0, n1hi = EDGE0 ? 15 : 16;
  auto frame_src = [&](uint32_t grp) {
    uint32_t g = min(grp, groups - 1) * kFPB + slot;
    g = g < total ? g : total - 1;  // clamp: tail slots recompute a valid frame, store nothing
    const uint32_t clip = g / nf;
    const uint32_t fi = g - clip * nf;
    return a.pcm + static_cast<int64_t>(clip) * a.clip_stride + static_cast<int64_t>(fi) * a.hop + 2 * jj;
  };
  // samples of columns jj (x[32 n1 + 2 jj], + 1) and jj + 8 (x[.. + 16], + 17), loaded
  // straight into SoA pairs: xr = (x[2 jj], x[2 jj + 16]), xi = (x[2 jj + 1], x[2 jj + 17])
  // (4-B loads: the pair's halves land in adjacent registers with no moves)
  auto load = [&](const float* src, cf (&xr)[16], cf (&xi)[16]) {
#pragma unroll
    for (int n1 = n1lo; n1 < n1hi; ++n1) {
      const float* s = src + 32 * n1;
      xr[n1] = cf{s[0], s[16]};
      xi[n1] = cf{s[1], s[17]};
    }
  };
  auto to_log = [&](float acc) {
    const float c = acc < a.log_floor ? a.log_floor : acc;  // keeps NaN
    return __log10f(c) * a.out_scale + a.out_add;
  };

  // one group: transform the samples in (cr, ci), prefetching group grp + stride into (nr, ni)
  auto process = [&](uint32_t grp, cf (&xr)[16], cf (&xi)[16], cf (&nr)[16], cf (&ni)[16]) {
    if constexpr (W != 4) load(frame_src(grp), xr, xi);
    P2 v[16];
#pragma unroll
    for (int n1 = 0; n1 < 16; ++n1) {
      if (n1 < n1lo || n1 >= n1hi) {
        v[n1] = P2{bc(0.f), bc(0.f)};
      } else {
        const float4 w = tj[8 * (kE4Win + n1)];
        v[n1] = P2{xr[n1] * cf{w.x, w.y}, xi[n1] * cf{w.z, w.w}};
      }
    }
    if constexpr (W == 4) load(frame_src(grp + gridDim.x), nr, ni);  // prefetch (clamped past the end)
    fft16p(v);  // v[k1] = A[k1][(jj, jj + 8)]
#pragma unroll
    for (int k1 = 1; k1 < 16; ++k1) {
      const float4 t = tj[8 * (kE4Tw + k1)];
      v[k1] = pmul(v[k1], cf{t.x, t.y}, cf{t.z, t.w});
    }
    // the transpose, re plane then im plane through the frame's one buffer (wavefront-scope
    // fences: ordering only, the frame belongs to this wave)
#pragma unroll
    for (int k1 = 0; k1 < 16; ++k1) {
      float* row = fr + row5(k1) * kLdt4 + jj;
      row[0] = v[k1].r.x;
      row[8] = v[k1].r.y;
    }
    wave_sync();
    cf tr[16];
#pragma unroll
    for (int n2 = 0; n2 < 16; ++n2) tr[n2] = cf{rowsB[n2], rowsB[8 * kLdt4 + n2]};
    wave_sync();
#pragma unroll
    for (int k1 = 0; k1 < 16; ++k1) {
      float* row = fr + row5(k1) * kLdt4 + jj;
      row[0] = v[k1].i.x;
      row[8] = v[k1].i.y;
    }
    wave_sync();
#pragma unroll
    for (int n2 = 0; n2 < 16; ++n2) v[n2] = P2{tr[n2], cf{rowsB[n2], rowsB[8 * kLdt4 + n2]}};
    fft16p(v);  // v[k2] = (Z[ra + 16 k2], Z[rb + 16 k2])
    // 2 X[k] = (Z[k] + Z*[256-k]) + (-i W512^k) (Z[k] - Z*[256-k]) for the bins below 128
    cf p[8];
#pragma unroll
    for (int k2 = 0; k2 < 8; ++k2) {
      const P2 z = v[k2], z15 = v[15 - k2], z16 = v[(16 - k2) & 15];
      // partner pair: (Z[256 - lo bin], Z[256 - hi bin]): the other half of v[15 - k2];
      // lane 0 (rows 0, 8): (row 0 of v[16 - k2], row 8 of v[15 - k2])
      const cf pr = jj ? cf{z15.r.y, z15.r.x} : cf{z16.r.x, z15.r.y};
      const cf pi = jj ? cf{z15.i.y, z15.i.x} : cf{z16.i.x, z15.i.y};
      const cf sr = z.r + pr, si = z.i - pi, dr = z.r - pr, di = z.i + pi;
      const float4 w = tj[8 * (kE4Ws + k2)];
      const cf wr = cf{w.x, w.y}, wi = cf{w.z, w.w};
      const cf xr = __builtin_elementwise_fma(-di, wi, __builtin_elementwise_fma(dr, wr, sr));
      const cf xi = __builtin_elementwise_fma(dr, wi, __builtin_elementwise_fma(di, wr, si));
      p[k2] = __builtin_elementwise_fma(xr, xr, xi * xi);
    }
    wave_sync();  // every lane of the frame has read its rows: the power row may overwrite them
#pragma unroll
    for (int k2 = 0; k2 < 8; ++k2) {
      pw[ra + 16 * k2] = p[k2].x;
      pw[rb + 16 * k2] = p[k2].y;
    }
    wave_sync();
    // 4 filters: A slots jj, jj + 8 (filters jj, jj + 8), B slots jj, jj + 8 (filters 31 - jj, 23 - jj);
    // taps in pairs (even start bins), weights x 1/4 from the table
    auto dot = [&](int lo, int e0, int T) {
      cf acc = bc(0.f);
#pragma unroll
      for (int q = 0; q < T / 4; ++q) {
        const float4 w = tj[8 * (e0 + q)];
        acc = __builtin_elementwise_fma(*reinterpret_cast<const cf*>(pw + lo + 4 * q), cf{w.x, w.y}, acc);
        acc = __builtin_elementwise_fma(*reinterpret_cast<const cf*>(pw + lo + 4 * q + 2), cf{w.z, w.w}, acc);
      }
      return acc.x + acc.y;
    };
    const float yA0 = dot(loA0, kE4Mel, kTapsA), yA1 = dot(loA1, kE4Mel + 2, kTapsA);
    const float yB0 = dot(loB0, kE4Mel + 4, kTapsB), yB1 = dot(loB1, kE4Mel + 8, kTapsB);
    const uint32_t g = grp * kFPB + slot;
    if (g < total) {
      float* o = a.out + static_cast<int64_t>(g) * kMaxMels;
      o[jj] = to_log(yA0);
      o[jj + 8] = to_log(yA1);
      o[31 - jj] = to_log(yB0);
      o[23 - jj] = to_log(yB1);
    }
    wave_sync();  // the next group's transpose overwrites the power row
  };

  // two explicit prefetch buffers (no register copies on the loop back edge)
  uint32_t grp = blockIdx.x;
  cf ar[16], ai[16], br[16], bi[16];
  if (W == 4 && grp < groups) load(frame_src(grp), ar, ai);
  if constexpr (W != 4) {
    for (; grp < groups; grp += gridDim.x) process(grp, ar, ai, ar, ai);
    return;
  }
  while (grp < groups) {
    process(grp, ar, ai, br, bi);
    grp += gridDim.x;
    if (grp >= groups) break;
    process(grp, br, bi, ar, ai);
    grp += gridDim.x;
  }
}

}  // namespace
}  // namespace hbk

#ifdef HBK_MEL_PACKED
#define HBK_MEL_V2(e) (hbk::mel_frames_v2_kernel<e, hbk::cf>)
#define HBK_MEL_V3(e) (hbk::mel_frames_mfma_kernel<e, hbk::cf>)
#else
#define HBK_MEL_V2(e) (hbk::mel_frames_v2_kernel<e, hbk::sc>)
#define HBK_MEL_V3(e) (hbk::mel_frames_mfma_kernel<e, hbk::sc>)
#endif

struct hbk_mel_plan {
  int n_fft, hop, n_mels, taps, nk2, need256;
  float log_floor, out_div, out_add;
  float* d_window = nullptr;
  float2* d_tw256 = nullptr;
  float2* d_tw512 = nullptr;
  int* d_lo = nullptr;
  float* d_w = nullptr;
  // v2 (32 mels, bins < 128): -i W512^k, even start bins, x 1/4 weights
  int v2 = 0, edge0 = 0;
  float2* d_twsm = nullptr;
  int* d_lo2 = nullptr;
  float* d_w2 = nullptr;
  // v3 (hbk_mel_set_variant 1): the dense filterbank^T [32][128] x 1/4 for the MFMA variant
  int variant = 0;
  float* d_fbt = nullptr;
  // v4 (HBK_MEL_V4): 4 or 8 waves per block, 0 = v2; its per-lane constant table
  int v4 = 0;
  float4* d_t4 = nullptr;
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
  // v2 layout: 32 mels reading bins < 128 only. Lane j computes filter j from
  // kTapsA bins and filter 31 - j from kTapsB bins, each from an even start
  // (8-B LDS pairs) kept inside [0, 128); weights x 1/4, zero outside the filter.
  int kmax_all = 0;
  for (int m = 0; m < n_mels; ++m) kmax_all = std::max(kmax_all, hi[m]);
  bool v2 = n_mels == kMaxMels && kmax_all < kBins2 && !getenv("HBK_MEL_V1");
  std::vector<int> lo2(kMaxMels, 0);
  std::vector<float> w2(16 * (kTapsA + kTapsB), 0.f);
  for (int m = 0; v2 && m < n_mels; ++m) {
    const int T = m < 16 ? kTapsA : kTapsB;
    int l = lo[m] & ~1;
    if (hi[m] - l + 1 > T) {
      v2 = false;
      break;
    }
    if (l + T > kBins2) l = kBins2 - T;  // even: T is even
    const int slot_j = m < 16 ? m : 31 - m;
    lo2[m < 16 ? slot_j : 16 + slot_j] = l;
    float* w = w2.data() + (m < 16 ? slot_j * kTapsA : 16 * kTapsA + slot_j * kTapsB);
    for (int t = 0; t < T; ++t) w[t] = 0.25f * fbank[(l + t) * n_mels + m];
  }
  bool edge0 = true;
  for (int i = 0; i < 32; ++i) edge0 = edge0 && window[i] == 0.f && window[n_fft - 1 - i] == 0.f;
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
  if (v2) {
    std::vector<float2> twsm(kBins2);
    for (int k = 0; k < kBins2; ++k) {  // -i W512^k = (sin(-2 pi k/512), -cos(-2 pi k/512))
      const double ang = -2.0 * M_PI * k / 512.0;
      twsm[k] = make_float2(static_cast<float>(sin(ang)), static_cast<float>(-cos(ang)));
    }
    p->v2 = 1;
    p->edge0 = edge0 ? 1 : 0;
    if ((e = hipMalloc(&p->d_twsm, kBins2 * sizeof(float2))) != hipSuccess) return fail(e, "hipMalloc twsm");
    if ((e = hipMalloc(&p->d_lo2, kMaxMels * sizeof(int))) != hipSuccess) return fail(e, "hipMalloc lo2");
    if ((e = hipMalloc(&p->d_w2, w2.size() * sizeof(float))) != hipSuccess) return fail(e, "hipMalloc w2");
    if ((e = hipMemcpy(p->d_twsm, twsm.data(), kBins2 * sizeof(float2), hipMemcpyHostToDevice)) != hipSuccess)
      return fail(e, "copy twsm");
    if ((e = hipMemcpy(p->d_lo2, lo2.data(), kMaxMels * sizeof(int), hipMemcpyHostToDevice)) != hipSuccess)
      return fail(e, "copy lo2");
    if ((e = hipMemcpy(p->d_w2, w2.data(), w2.size() * sizeof(float), hipMemcpyHostToDevice)) != hipSuccess)
      return fail(e, "copy w2");
    std::vector<float> fbt(static_cast<size_t>(kMaxMels) * kBins2);
    for (int m = 0; m < kMaxMels; ++m)
      for (int k = 0; k < kBins2; ++k) fbt[m * kBins2 + k] = 0.25f * fbank[k * n_mels + m];
    if ((e = hipMalloc(&p->d_fbt, fbt.size() * sizeof(float))) != hipSuccess) return fail(e, "hipMalloc fbt");
    if ((e = hipMemcpy(p->d_fbt, fbt.data(), fbt.size() * sizeof(float), hipMemcpyHostToDevice)) != hipSuccess)
      return fail(e, "copy fbt");
    p->variant = getenv("HBK_MEL_MFMA") ? 1 : 0;
    // v4 table [entry][lane jj]: window, W256 twiddles, split twiddles, filter weights
    std::vector<float4> t4(static_cast<size_t>(kE4N) * 8, make_float4(0.f, 0.f, 0.f, 0.f));
    auto W = [](double num) {
      const double ang = -2.0 * M_PI * num;
      return std::pair<float, float>(static_cast<float>(cos(ang)), static_cast<float>(sin(ang)));
    };
    for (int jj = 0; jj < 8; ++jj) {
      for (int n1 = 0; n1 < 16; ++n1) {
        const int s = 32 * n1 + 2 * jj;
        t4[(kE4Win + n1) * 8 + jj] = make_float4(win[s], win[s + 16], win[s + 1], win[s + 17]);
      }
      for (int k1 = 1; k1 < 16; ++k1) {
        const auto a0 = W(double(jj * k1) / 256.0), a1 = W(double((jj + 8) * k1) / 256.0);
        t4[(kE4Tw + k1) * 8 + jj] = make_float4(a0.first, a1.first, a0.second, a1.second);
      }
      const int ra = jj == 0 ? 0 : jj, rb = jj == 0 ? 8 : 16 - jj;
      for (int k2 = 0; k2 < 8; ++k2) {
        const float2 s0 = twsm[ra + 16 * k2], s1 = twsm[rb + 16 * k2];
        t4[(kE4Ws + k2) * 8 + jj] = make_float4(s0.x, s1.x, s0.y, s1.y);
      }
      const float* wa0 = w2.data() + jj * kTapsA;
      const float* wa1 = w2.data() + (jj + 8) * kTapsA;
      const float* wb0 = w2.data() + 16 * kTapsA + jj * kTapsB;
      const float* wb1 = w2.data() + 16 * kTapsA + (jj + 8) * kTapsB;
      for (int q = 0; q < 2; ++q) t4[(kE4Mel + q) * 8 + jj] = make_float4(wa0[4 * q], wa0[4 * q + 1], wa0[4 * q + 2], wa0[4 * q + 3]);
      for (int q = 0; q < 2; ++q) t4[(kE4Mel + 2 + q) * 8 + jj] = make_float4(wa1[4 * q], wa1[4 * q + 1], wa1[4 * q + 2], wa1[4 * q + 3]);
      for (int q = 0; q < 4; ++q) t4[(kE4Mel + 4 + q) * 8 + jj] = make_float4(wb0[4 * q], wb0[4 * q + 1], wb0[4 * q + 2], wb0[4 * q + 3]);
      for (int q = 0; q < 4; ++q) t4[(kE4Mel + 8 + q) * 8 + jj] = make_float4(wb1[4 * q], wb1[4 * q + 1], wb1[4 * q + 2], wb1[4 * q + 3]);
    }
    if ((e = hipMalloc(&p->d_t4, t4.size() * sizeof(float4))) != hipSuccess) return fail(e, "hipMalloc t4");
    if ((e = hipMemcpy(p->d_t4, t4.data(), t4.size() * sizeof(float4), hipMemcpyHostToDevice)) != hipSuccess)
      return fail(e, "copy t4");
    // opt-in until measured on the GPU: HBK_MEL_V4=1 (4-wave blocks, prefetch) or 8 (8-wave blocks)
    // (0 or unset: off, as the other HBK_* knobs read their values)
    const char* v4 = getenv("HBK_MEL_V4");
    const int v4n = v4 ? atoi(v4) : 0;
    p->v4 = v4n == 0 ? 0 : (v4n == 8 ? 8 : 4);
  }
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
  (void)hipFree(p->d_twsm);
  (void)hipFree(p->d_lo2);
  (void)hipFree(p->d_w2);
  (void)hipFree(p->d_fbt);
  (void)hipFree(p->d_t4);
  delete p;
  return HBK_OK;
}

int hbk_mel_set_variant(hbk_mel_plan* plan, int32_t variant) {
  using namespace hbk;
  if (!plan) return arg_error("plan is NULL");
  if (variant != 0 && variant != 1) return arg_error("variant must be 0 (sparse VALU) or 1 (MFMA)");
  if (variant == 1 && !plan->v2) {
    set_error("hbk: the MFMA filterbank variant covers 32 mels on bins < 128");
    return HBK_ERR_UNSUPPORTED;
  }
  plan->variant = variant;
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
  const int64_t total = n_clips * n_frames;
  if (total >= (int64_t(1) << 31)) return arg_error("more than 2^31 frames in one call");
  if (plan->v2 && plan->variant == 1) {
    const int64_t groups3 = (total + kFramesPerBlock3 - 1) / kFramesPerBlock3;
    Mel3Args a;
    a.pcm = pcm;
    a.out = out;
    a.window = plan->d_window;
    a.tw256 = plan->d_tw256;
    a.twsm = plan->d_twsm;
    a.fbt = plan->d_fbt;
    a.n_clips = n_clips;
    a.clip_stride = clip_stride;
    a.n_frames = n_frames;
    a.hop = plan->hop;
    a.log_floor = plan->log_floor;
    a.out_scale = 10.f / plan->out_div;
    a.out_add = plan->out_add;
    const int64_t blocks = std::min<int64_t>(groups3, persistent_blocks(kBlocksPerCU3, stream));
    if (plan->edge0)
      hipLaunchKernelGGL(HBK_MEL_V3(true), dim3(static_cast<unsigned>(blocks)), dim3(kThreads3), 0,
                         as_stream(stream), a);
    else
      hipLaunchKernelGGL(HBK_MEL_V3(false), dim3(static_cast<unsigned>(blocks)), dim3(kThreads3), 0,
                         as_stream(stream), a);
    HBK_LAUNCH_CHECK("mel_frames_mfma_kernel");
    return HBK_OK;
  }
  if (plan->v2 && plan->v4) {
    const int W = plan->v4 == 8 ? 8 : 4;  // waves per block (hbk_mel_plan::v4)
    const int64_t fpb = kFramesPerWave4 * W;
    const int64_t groups4 = (total + fpb - 1) / fpb;
    Mel4Args a;
    a.pcm = pcm;
    a.out = out;
    a.table = plan->d_t4;
    a.mel_lo2 = plan->d_lo2;
    a.n_clips = n_clips;
    a.clip_stride = clip_stride;
    a.n_frames = n_frames;
    a.hop = plan->hop;
    a.log_floor = plan->log_floor;
    a.out_scale = 10.f / plan->out_div;
    a.out_add = plan->out_add;
    const int64_t blocks = std::min<int64_t>(groups4, persistent_blocks(W == 8 ? 2 : kBlocksPerCU4, stream));
    const dim3 grid(static_cast<unsigned>(blocks)), block(64 * W);
    if (W == 8) {
      if (plan->edge0)
        hipLaunchKernelGGL((hbk::mel_frames_soa_kernel<true, 8>), grid, block, 0, as_stream(stream), a);
      else
        hipLaunchKernelGGL((hbk::mel_frames_soa_kernel<false, 8>), grid, block, 0, as_stream(stream), a);
    } else {
      if (plan->edge0)
        hipLaunchKernelGGL((hbk::mel_frames_soa_kernel<true, 4>), grid, block, 0, as_stream(stream), a);
      else
        hipLaunchKernelGGL((hbk::mel_frames_soa_kernel<false, 4>), grid, block, 0, as_stream(stream), a);
    }
    HBK_LAUNCH_CHECK("mel_frames_soa_kernel");
    return HBK_OK;
  }
  if (plan->v2) {
    const int64_t groups2 = (total + kFramesPerBlock2 - 1) / kFramesPerBlock2;
    Mel2Args a;
    a.pcm = pcm;
    a.out = out;
    a.window = plan->d_window;
    a.tw256 = plan->d_tw256;
    a.twsm = plan->d_twsm;
    a.mel_lo2 = plan->d_lo2;
    a.mel_w2 = plan->d_w2;
    a.n_clips = n_clips;
    a.clip_stride = clip_stride;
    a.n_frames = n_frames;
    a.hop = plan->hop;
    a.log_floor = plan->log_floor;
    a.out_scale = 10.f / plan->out_div;
    a.out_add = plan->out_add;
    const int64_t blocks = std::min<int64_t>(groups2, persistent_blocks(kBlocksPerCU2, stream));
    if (plan->edge0)
      hipLaunchKernelGGL(HBK_MEL_V2(true), dim3(static_cast<unsigned>(blocks)), dim3(kThreads2), 0,
                         as_stream(stream), a);
    else
      hipLaunchKernelGGL(HBK_MEL_V2(false), dim3(static_cast<unsigned>(blocks)), dim3(kThreads2), 0,
                         as_stream(stream), a);
    HBK_LAUNCH_CHECK("mel_frames_v2_kernel");
    return HBK_OK;
  }
  const int64_t groups = (total + kFramesPerBlock - 1) / kFramesPerBlock;
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
  const int64_t blocks = std::min<int64_t>(groups, persistent_blocks(kBlocksPerCU, stream));
  hipLaunchKernelGGL(mel_frames_kernel, dim3(static_cast<unsigned>(blocks)), dim3(kThreads), 0,
                     as_stream(stream), a);
  HBK_LAUNCH_CHECK("mel_frames_kernel");
  return HBK_OK;
}

}  // extern "C"
