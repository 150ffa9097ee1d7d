// Fused batch augmentation for gfx950: gain + background-noise mix + IR reverb.
//
// Gain: torch_audiomentations Gain (per-batch dB ~ U[-18, 6], p 1.0 in the
// reference's batch chain, augmented.py:114-118), a per-clip factor applied
// to x on load.
// Replaces add_background_noise_to_batch -> torchaudio.functional.add_noise
// (augmented.py:234-276, :383-384) and speechbrain's reverberate(batch, ir)
// (augmented.py:386-392) of AugmentedAudioGenerator.execute_augment_batch.
//
// One workgroup (1024 threads) per clip, the whole clip resident in LDS:
//   x and the clip's noise segment arrive in registers (loaded after the
//   previous clip's inverse FFT) -> E_x, E_n ->
//   y = x + 10^((10 log10(E_x/E_n) - snr)/20) n -> LDS, a_in = mean|y|
//   circular convolution with the batch's IR kernel of length T = 23040:
//     z[n] = y[2n] + i y[2n+1], an 11520-point complex FFT done in place in
//     LDS as four mixed-radix decimation-in-frequency passes 16 x 16 x 9 x 5
//     (720, 720, 1280 and 2304 independent DFTs per pass, one per thread and
//     round, radix-16 / 9 / 5 in VGPRs); twiddles W_M^e = HI[e >> 7] LO[e & 127]
//     from two small LDS tables. Z lands in digit-reversed order (zaddr); the
//     real-FFT split, * H[k] and the inverse split run on (k, M-k) pairs (H and
//     W_N^k stored bin-major, [k % 16][k / 16], so those loads coalesce); the
//     inverse transform is the passes reversed (decimation in time, conjugate
//     twiddles) and lands back in natural order.
//   y <- a_in * y / (mean|y| + 1e-14), store.
// The IR spectrum H (one per batch) comes from the same transform run on the
// rotated kernel [ir[d:], 0..., ir[:d]] (hbk_reverb_spectrum).
#include <algorithm>
#include <cmath>
#include <numeric>
#include <type_traits>
#include <vector>

#include "hbk_common.h"

namespace hbk {
namespace {

constexpr int kT = 23040;        // clip length (1.44 s @ 16 kHz, augmented.py:31)
constexpr int kM = kT / 2;       // complex FFT length
constexpr int kThreads = 1024;   // 16 waves: one clip per CU (92 KB of LDS)
constexpr int kN1 = 16000;       // colored noise: torch_audiomentations' noise length = sample_rate
constexpr int kM1 = kN1 / 2;     // 8000

// ---- small DFTs in registers (constant twiddles) --------------------------
template <bool INV>
__device__ __forceinline__ cf tw_const(double frac) {  // exp(-+2 pi i frac)
  const double a = (INV ? 2.0 : -2.0) * M_PI * frac;
  return cf{static_cast<float>(cos(a)), static_cast<float>(sin(a))};
}

template <bool INV>
__device__ __forceinline__ void dft3(cf& a, cf& b, cf& c) {
  // X0 = a+b+c; X1 = a + w b + w^2 c; X2 = a + w^2 b + w c, w = exp(-+2pi i/3)
  constexpr float h = 0.5f, s = 0.86602540378443865f;
  const cf t = b + c;
  const cf d = b - c;
  const cf m = a - h * t;
  // (-+) i s d
  const cf r = INV ? cf{-s * d.y, s * d.x} : cf{s * d.y, -s * d.x};
  a = a + t;
  b = m + r;
  c = m - r;
}

template <bool INV>
__device__ __forceinline__ void dft5(cf (&x)[5]) {
  cf y[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) {
    cf acc = x[0];
#pragma unroll
    for (int n = 1; n < 5; ++n) acc = acc + cmul(x[n], tw_const<INV>(double((n * k) % 5) / 5.0));
    y[k] = acc;
  }
#pragma unroll
  for (int k = 0; k < 5; ++k) x[k] = y[k];
}

// DFT-9 as 3 x 3: n = 3u + v, k = c + 3d
template <bool INV>
__device__ __forceinline__ void dft9(cf (&x)[9]) {
#pragma unroll
  for (int v = 0; v < 3; ++v) dft3<INV>(x[v], x[3 + v], x[6 + v]);  // x[3c + v] = A[v][c]
#pragma unroll
  for (int c = 1; c < 3; ++c)
#pragma unroll
    for (int v = 1; v < 3; ++v) x[3 * c + v] = cmul(x[3 * c + v], tw_const<INV>(double(v * c) / 9.0));
#pragma unroll
  for (int c = 0; c < 3; ++c) dft3<INV>(x[3 * c + 0], x[3 * c + 1], x[3 * c + 2]);  // x[3c + d] = X[c + 3d]
  cf t[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) t[k] = x[3 * (k % 3) + k / 3];
#pragma unroll
  for (int k = 0; k < 9; ++k) x[k] = t[k];
}

// DFT-45 as 5 x 9: n = 5p + q, k = r + 9s; natural order in and out.
template <bool INV>
__device__ __forceinline__ void dft45(cf (&x)[45]) {
  cf a[5][9];
#pragma unroll
  for (int q = 0; q < 5; ++q) {
    cf col[9];
#pragma unroll
    for (int p = 0; p < 9; ++p) col[p] = x[5 * p + q];
    dft9<INV>(col);
#pragma unroll
    for (int r = 0; r < 9; ++r) a[q][r] = (q && r) ? cmul(col[r], tw_const<INV>(double(q * r) / 45.0)) : col[r];
  }
#pragma unroll
  for (int r = 0; r < 9; ++r) {
    cf v[5];
#pragma unroll
    for (int q = 0; q < 5; ++q) v[q] = a[q][r];
    dft5<INV>(v);
#pragma unroll
    for (int s = 0; s < 5; ++s) x[r + 9 * s] = v[s];
  }
}

template <bool INV>
__device__ __forceinline__ void fft4v(cf& a0, cf& a1, cf& a2, cf& a3) {
  const cf t0 = a0 + a2, t1 = a0 - a2, t2 = a1 + a3;
  const cf d = a1 - a3;
  const cf t3 = INV ? cf{-d.y, d.x} : cf{d.y, -d.x};  // (+-i) d
  a0 = t0 + t2;
  a2 = t0 - t2;
  a1 = t1 + t3;
  a3 = t1 - t3;
}

template <bool INV>
__device__ __forceinline__ void fft16v(cf (&v)[16]) {
#pragma unroll
  for (int m2 = 0; m2 < 4; ++m2) fft4v<INV>(v[m2], v[4 + m2], v[8 + m2], v[12 + m2]);
#pragma unroll
  for (int l1 = 1; l1 < 4; ++l1)
#pragma unroll
    for (int m2 = 1; m2 < 4; ++m2) v[4 * l1 + m2] = cmul(v[4 * l1 + m2], tw_const<INV>(double(m2 * l1) / 16.0));
#pragma unroll
  for (int l1 = 0; l1 < 4; ++l1) fft4v<INV>(v[4 * l1 + 0], v[4 * l1 + 1], v[4 * l1 + 2], v[4 * l1 + 3]);
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

// Two-level twiddle table in LDS: W_M^e = hi[e >> 7] * lo[e & 127], e < kM.
constexpr int kTwLo = 128, kTwHi = kM / kTwLo;  // 128 x 90
static_assert(kTwLo * kTwHi == kM, "twiddle split");

template <bool INV>
__device__ __forceinline__ cf twiddle(const cf* thi, const cf* tlo, int e) {
  const cf w = cmul(thi[e >> 7], tlo[e & (kTwLo - 1)]);
  return INV ? cf{w.x, -w.y} : w;
}

template <int R, bool INV>
__device__ __forceinline__ void dftr(cf (&v)[R]) {
  if constexpr (R == 16) fft16v<INV>(v);
  else if constexpr (R == 9) dft9<INV>(v);
  else dft5<INV>(v);
}

// One in-place pass of radix R over span L (blocks of R L elements): task
// (blk, i) owns elements blk R L + i + L m, m < R. Forward (DIF): DFT-R, then
// output k times W_M^(S i k). Inverse (DIT): input k times conj W_M^(S i k),
// then the inverse DFT-R. Independent tasks, so one barrier per pass.
template <int R, int L, int S, bool INV>
__device__ __forceinline__ void pass(cf* z, const cf* thi, const cf* tlo) {
  constexpr int kTasks = kM / R;
  // opaque copy of the thread id: keeps the per-pass index math inside the
  // clip loop instead of hoisted (as dozens of live VGPRs) out of it
  int t0;
  asm volatile("v_mov_b32 %0, %1" : "=v"(t0) : "v"(static_cast<int>(threadIdx.x)));
  for (int t = t0; t < kTasks; t += kThreads) {
    // lanes walk i (contiguous addresses) when L is large, blocks (stride R L =
    // 45 complex: conflict-free over 32 lanes) when L is the short span of 5
    constexpr int kBlocks = kM / (R * L);
    int blk, i;
    if constexpr (L < 16) {
      i = t / kBlocks;
      blk = t - i * kBlocks;
    } else {
      blk = t / L;
      i = t - blk * L;
    }
    cf* q = z + blk * (R * L) + i;
    cf v[R];
#pragma unroll
    for (int m = 0; m < R; ++m) v[m] = q[L * m];
    cf w[R];  // w[k] = W_M^(S i k) (conjugated for INV)
    if constexpr (S != 0) {
      if constexpr (R == 16) {
        // 4 table lookups (k = 1, 2, 4, 8), the other powers as products (<= 3 deep)
        w[1] = twiddle<INV>(thi, tlo, S * i);
        w[2] = twiddle<INV>(thi, tlo, 2 * S * i);
        w[4] = twiddle<INV>(thi, tlo, 4 * S * i);
        w[8] = twiddle<INV>(thi, tlo, 8 * S * i);
        w[3] = cmul(w[1], w[2]);
        w[5] = cmul(w[1], w[4]);
        w[6] = cmul(w[2], w[4]);
        w[7] = cmul(w[3], w[4]);
#pragma unroll
        for (int k = 9; k < 16; ++k) w[k] = cmul(w[k - 8], w[8]);
      } else {
#pragma unroll
        for (int k = 1; k < R; ++k) w[k] = twiddle<INV>(thi, tlo, S * i * k);
      }
    }
    if (INV && S)
#pragma unroll
      for (int k = 1; k < R; ++k) v[k] = cmul(v[k], w[k]);
    dftr<R, INV>(v);
    if (!INV && S)
#pragma unroll
      for (int k = 1; k < R; ++k) v[k] = cmul(v[k], w[k]);
#pragma unroll
    for (int m = 0; m < R; ++m) q[L * m] = v[m];
  }
}

#ifdef HBK_PHASE_TIMING
// Profiling build only (build.py variant "phase"): thread 0 of every block adds
// the s_memtime cycles of each augment phase (barrier waits included in the
// phase before them) into g_aug_phase; read by hbk_debug_aug_phase.
__device__ unsigned long long g_aug_phase[32];
#define HBK_APH(i)                                                  \
  do {                                                              \
    if (threadIdx.x == 0) {                                         \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime();   \
      atomicAdd(&g_aug_phase[i], t_ - ph_t0);                       \
      ph_t0 = t_;                                                   \
    }                                                               \
  } while (0)
#else
#define HBK_APH(i) \
  do {             \
  } while (0)
#endif

// Forward: natural z -> Z[f] at zaddr(f); inverse: the reverse (x kM).
// (ph_t0 / ph: phase-timing build only, phases ph .. ph + 3)
template <bool INV>
__device__ __forceinline__ void transform(cf* z, const cf* thi, const cf* tlo,
                                          [[maybe_unused]] unsigned long long& ph_t0,
                                          [[maybe_unused]] int ph) {
  if (!INV) {
    pass<16, 720, 1, false>(z, thi, tlo);
    __syncthreads();
    HBK_APH(ph);
    pass<16, 45, 16, false>(z, thi, tlo);
    __syncthreads();
    HBK_APH(ph + 1);
    pass<9, 5, 256, false>(z, thi, tlo);
    __syncthreads();
    HBK_APH(ph + 2);
    pass<5, 1, 0, false>(z, thi, tlo);
    __syncthreads();
    HBK_APH(ph + 3);
  } else {
    pass<5, 1, 0, true>(z, thi, tlo);
    __syncthreads();
    HBK_APH(ph);
    pass<9, 5, 256, true>(z, thi, tlo);
    __syncthreads();
    HBK_APH(ph + 1);
    pass<16, 45, 16, true>(z, thi, tlo);
    __syncthreads();
    HBK_APH(ph + 2);
    pass<16, 720, 1, true>(z, thi, tlo);
    __syncthreads();
    HBK_APH(ph + 3);
  }
}

// Position of frequency f = k1 + 16 k2 + 256 k3 + 2304 k4 after the forward
// passes: 720 k1 + 45 k2 + 5 k3 + k4 (mixed-radix digit reversal).
__device__ __forceinline__ int zaddr(int f) {
  const int k1 = f & 15, r = f >> 4;
  const int k2 = r & 15, r2 = r >> 4;
  const int k4 = r2 / 9, k3 = r2 - 9 * k4;
  return 720 * k1 + 45 * k2 + 5 * k3 + k4;
}

// Frequency stored at position p (inverse of zaddr).
__device__ __forceinline__ int zfreq(int p) {
  const int k1 = p / 720, r = p - 720 * k1;
  const int k2 = r / 45, r2 = r - 45 * k2;
  const int k3 = r2 / 5, k4 = r2 - 5 * k3;
  return k1 + 16 * k2 + 256 * k3 + 2304 * k4;
}

// the twiddle tables into LDS (after z and the reduction slots)
__device__ __forceinline__ void load_tw(cf* thi, cf* tlo, const float2* ghi, const float2* glo) {
  for (int i = threadIdx.x; i < kTwHi; i += kThreads) thi[i] = cf{ghi[i].x, ghi[i].y};
  for (int i = threadIdx.x; i < kTwLo; i += kThreads) tlo[i] = cf{glo[i].x, glo[i].y};
}

// wave sum through DPP (no lane-index VGPRs, unlike __shfl_xor's bpermute
// addresses, which the compiler hoists and spills): quad_perm [1,0,3,2],
// [2,3,0,1], row_half_mirror, row_mirror leave each 16-lane row's sum in all
// of its lanes; the four rows are added from readlane
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float wave_sum(float v) {
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0x141>(v);
  v += dpp_f<0x140>(v);
  const int b = __builtin_bit_cast(int, v);
  return (__builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 0)) +
          __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 16))) +
         (__builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 32)) +
          __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 48)));
}

// (results and the wave index are uniform: SGPRs, so nothing here takes a
// VGPR that could be spilled and reloaded behind the next clip's prefetch)
__device__ __forceinline__ float sgpr_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v)));
}
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  __syncthreads();
  if (lane == 0) red[wave] = v;
  __syncthreads();
  float s = 0.f;
  for (int w = 0; w < kThreads / 64; ++w) s += red[w];
  return sgpr_f(s);  // summed here, not sunk to the use with 16 live partials
}

// opaque copy of the thread id: index math derived from it stays inside the
// clip loop (the compiler otherwise hoists dozens of per-element offsets out of
// it and spills them)
__device__ __forceinline__ int opaque_tid() {
  int t;
  asm volatile("v_mov_b32 %0, %1" : "=v"(t) : "v"(static_cast<int>(threadIdx.x)));
  return t;
}

// two block sums in one barrier round (red holds 2 x 16 wave partials)
__device__ __forceinline__ void block_sum2(float& a, float& b, float* red) {
  a = wave_sum(a);
  b = wave_sum(b);
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  __syncthreads();
  if (lane == 0) {
    red[wave] = a;
    red[16 + wave] = b;
  }
  __syncthreads();
  a = b = 0.f;
  for (int w = 0; w < kThreads / 64; ++w) {
    a += red[w];
    b += red[16 + w];
  }
  a = sgpr_f(a);
  b = sgpr_f(b);
}

// spectrum / W_N^k slot of bin k <= kM: [k % 16][k / 16] (HBK_REVERB_SPECTRUM_SLOTS):
// the pair loop's lanes walk k in steps of 16, i.e. consecutive slots
constexpr int kHRow = kM / 16 + 1;  // 721
constexpr int kHSlots = 16 * kHRow;
static_assert(kHSlots == HBK_REVERB_SPECTRUM_SLOTS, "spectrum slot layout");
__device__ __forceinline__ int hslot(int k) { return (k & 15) * kHRow + (k >> 4); }

struct AugArgs {
  const float* x;
  int64_t x_stride;
  float* out;
  int64_t out_stride;
  int64_t n_clips;
  const float* ring;        // background-noise ring (all noise clips back to back)
  int64_t ring_len;
  const int64_t* noise_off; // per clip: ring offset of its segment, < 0 = no noise
  const float* snr_db;      // per clip
  const float2* spectra;    // [n_spec][kHSlots], bin k at hslot(k)
  const int* spec_idx;      // per clip: spectrum index, < 0 = no reverb
  const float* gain;        // per clip linear gain, or NULL
  const float2* thi;        // W_M^(128 h), h < 90
  const float2* tlo;        // W_M^l, l < 128
  const float2* twn;        // W_N^k, k <= kM, at hslot(k)
  // colored noise folded into the prologue (hbk_augment_colored; c_snr NULL: none). A clip
  // with a non-NaN c_snr whose group's coloured second was made (c_grms[g] not NaN) and
  // whose f_decay equals its group's first clip's is mixed here, exactly as
  // colored_mix_kernel mixes it; any other coloured clip was written to out by
  // colored_noise_kernel beforehand and is read from out instead of x.
  const float* c_snr;
  const float* c_fd;
  int64_t c_group;
  const float* c_gbuf;      // [groups][16000]: the coloured second x 8000
  const float* c_grms;      // [groups], NULL: no group path
};

// 0: no colored noise, 1: mixed in augment_kernel's prologue, 2: coloured by
// colored_noise_kernel into out (uniform per clip)
__device__ __forceinline__ int colored_mode(const AugArgs& a, int64_t clip) {
  if (!a.c_snr) return 0;
  const float snr = a.c_snr[clip];
  if (snr != snr) return 0;
  if (a.c_grms) {
    const int64_t g = clip / a.c_group;
    const float r = a.c_grms[g];
    if (r == r && a.c_fd[clip] == a.c_fd[g * a.c_group]) return 1;
  }
  return 2;
}

__global__ void __launch_bounds__(kThreads) augment_kernel(AugArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  cf* z = reinterpret_cast<cf*>(smem);                      // kM complex
  float* red = smem + 2 * kM;                               // 32 floats
  cf* thi = reinterpret_cast<cf*>(smem + 2 * kM + 32);
  cf* tlo = thi + kTwHi;
  load_tw(thi, tlo, a.thi, a.tlo);
  const cf* twn = reinterpret_cast<const cf*>(a.twn);
  float* zf = smem;
  const int tid = threadIdx.x;
  // the next clip's samples are loaded into registers while this clip's
  // transforms run (one clip per CU: otherwise every load is exposed); the
  // noise segment is read twice (energy, then mix; the 2nd read hits L2)
  constexpr int kPer = (kT + kThreads - 1) / kThreads;
  float xr[kPer], nr[kPer];
  // the next clip's samples and noise segment  are loaded after this clip's inverse FFT,
  // so their latency hides behind the |y| sum and the stores without holding
  // VGPRs through the FFT passes
  // (noff: the clip's noise offset, read well before, so that no branch waits
  // on a load queued behind these; vmcnt retires loads in order)
  // (cmode: colored_mode of the clip, read ahead like noff; 2 = read the clip from out)
  auto prefetch = [&](int64_t clip, int64_t noff, int cmode) {
    // uniform base + 32-bit per-lane offsets from an opaque thread id (keeps
    // the 46 per-load addresses from being hoisted out of the clip loop)
    const int t = opaque_tid();
    // one uniform element offset from a.x. (The colored fold pushes this kernel's SGPRs over
    // the limit: 2 x 8 B of VGPR spills, stored and reloaded once per clip, outside the passes.)
    const int64_t row = cmode == 2 ? (a.out - a.x) + clip * a.out_stride : clip * a.x_stride;
    const float* x = a.x + row;
    // 32-bit BYTE offsets from a uniform base: global_load's saddr form, one
    // VGPR per address (ring_len < 2^30, checked on the host)
    auto at = [](const float* base, uint32_t i) {
      return *reinterpret_cast<const float*>(reinterpret_cast<const char*>(base) + (i << 2));
    };
#pragma unroll
    for (int u = 0; u < kPer; ++u) xr[u] = at(x, static_cast<uint32_t>(min(t + u * kThreads, kT - 1)));
    if (noff >= 0) {
      const uint32_t rlen = static_cast<uint32_t>(a.ring_len), r0 = static_cast<uint32_t>(noff);
#pragma unroll
      for (int u = 0; u < kPer; ++u) {
        uint32_t r = r0 + static_cast<uint32_t>(min(t + u * kThreads, kT - 1));
        r = r >= rlen ? r - rlen : r;
        nr[u] = at(a.ring, r);
      }
    }
  };
  if (blockIdx.x < a.n_clips) prefetch(blockIdx.x, a.noise_off[blockIdx.x], colored_mode(a, blockIdx.x));
  unsigned long long ph_t0 = 0;
#ifdef HBK_PHASE_TIMING
  ph_t0 = __builtin_amdgcn_s_memtime();
#endif
  for (int64_t clip = blockIdx.x; clip < a.n_clips; clip += gridDim.x) {
    // 1) y = x + scale n (torchaudio add_noise: snr0 = 10 (log10 Ex - log10 En),
    //    scale = 10^((snr0 - snr)/20)) in registers; y goes to LDS once and
    //    a_in = mean|y| is summed on the way
    const int64_t noff = a.noise_off[clip];
    const int sp = a.spec_idx[clip];
    const float gain = a.gain ? a.gain[clip] : 1.f;
    const bool next = clip + gridDim.x < a.n_clips;
    const int64_t noff_next = __builtin_amdgcn_readfirstlane(static_cast<int>(next ? a.noise_off[clip + gridDim.x] : -1));
    const int cmode = __builtin_amdgcn_readfirstlane(colored_mode(a, clip));
    const int cmode_next = __builtin_amdgcn_readfirstlane(next ? colored_mode(a, clip + gridDim.x) : 0);
    float ex = 0.f, aa = 0.f;
    if (cmode == 1) {
      // colored noise (the group path), in colored_mix_kernel's per-thread order and block
      // sum: bit-identical to hbk_colored_noise_ws followed by hbk_augment
      const int64_t g = clip / a.c_group;
      const float* gb = a.c_gbuf + g * kN1;
      const int t = opaque_tid();
      // explicit fmaf, as colored_mix_kernel: a plain `ec += x * x` here was SLP-vectorised
      // into v_pk_mul + v_add (two roundings) and moved 1 in ~30 clips by an ulp
      float ec = 0.f, ez = 0.f;
#pragma unroll
      for (int u = 0; u < kPer; ++u)
        if (t + u * kThreads < kT) ec = fmaf(xr[u], xr[u], ec);
      block_sum2(ec, ez, red);
      const float rms_x = sqrtf(ec / kT);
      const float scale = rms_x / powf(10.f, a.c_snr[clip] / 20.f) / (a.c_grms[g] + 1e-8f) * (1.f / kM1);
      // the coloured second from L2 (64 KB per batch), loaded after the sum: held across it,
      // its 23 registers spilled
#pragma unroll
      for (int u = 0; u < kPer; ++u) {
        const int s = min(t + u * kThreads, kT - 1);
        const int sn = s < kN1 ? s : s - kN1;
        xr[u] = fmaf(scale,
                     *reinterpret_cast<const float*>(reinterpret_cast<const char*>(gb) + (static_cast<uint32_t>(sn) << 2)),
                     xr[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      xr[u] *= gain;
      if (tid + u * kThreads < kT) ex += xr[u] * xr[u];
    }
    HBK_APH(0);
    if (noff >= 0) {
      float en = 0.f;
#pragma unroll
      for (int u = 0; u < kPer; ++u)
        if (tid + u * kThreads < kT) en += nr[u] * nr[u];
      HBK_APH(1);
      block_sum2(ex, en, red);
      HBK_APH(2);
      const float snr0 = 10.f * (log10f(ex) - log10f(en));
      const float scale = powf(10.f, (snr0 - a.snr_db[clip]) / 20.f);
#pragma unroll
      for (int u = 0; u < kPer; ++u) xr[u] += scale * nr[u];
    }
    {
      const int t = opaque_tid();
#pragma unroll
      for (int u = 0; u < kPer; ++u) {
        const int s = t + u * kThreads;
        if (s < kT) {
          zf[s] = xr[u];
          aa += fabsf(xr[u]);
        }
      }
    }
    HBK_APH(3);
    float* out = a.out + clip * a.out_stride;
    if (sp < 0) {  // no reverb: each thread stores the samples it wrote
      if (next) prefetch(clip + gridDim.x, noff_next, cmode_next);
      for (int s = opaque_tid(); s < kT; s += kThreads) out[s] = zf[s];
      __syncthreads();
      continue;
    }
    // 2) a_in = mean |y| (block_sum's first barrier also publishes zf)
    const float a_in = block_sum(aa, red) / kT;
    HBK_APH(4);
    // 3) forward FFT (natural -> permuted)
    transform<false>(z, thi, tlo, ph_t0, 5);
    // 4) split, multiply by H, inverse split, on (k, M-k) pairs
    const cf* H = reinterpret_cast<const cf*>(a.spectra) + static_cast<int64_t>(sp) * kHSlots;
    // one thread per pair (k, M - k), k <= M / 2; consecutive lanes take k in
    // steps of 16 (k = c + 16 r, c = idx / 361), so their positions zaddr(k)
    // step by 45 complex instead of 720 (no 16-way bank conflicts)
    // All of a thread's H[k], H[M - k], W_N^k (L2-resident) are loaded in one
    // batch before the loop: one exposed latency instead of one per pair.
    constexpr int kRest = kM / 2 / 16 + 1;  // 361
    constexpr int kSplitIt = (16 * kRest + kThreads - 1) / kThreads;
    cf hk[kSplitIt], hc[kSplitIt], wn[kSplitIt];
    const int ts = opaque_tid();
    auto pair_k = [&](int it) {
      const int idx = min(ts + it * kThreads, 16 * kRest - 1);
      const int c = idx / kRest;
      return min(c + 16 * (idx - c * kRest), kM / 2);
    };
#pragma unroll
    for (int it = 0; it < kSplitIt; ++it) {
      const int k = pair_k(it);
      hk[it] = H[hslot(k)];
      hc[it] = H[hslot(kM - k)];
      wn[it] = twn[hslot(k)];
    }
#pragma unroll
    for (int it = 0; it < kSplitIt; ++it) {
      const int idx = ts + it * kThreads;
      const int c = idx / kRest;
      const int k = c + 16 * (idx - c * kRest);
      if (idx >= 16 * kRest || k > kM / 2) continue;
      const int kc = (kM - k) % kM;
      const int p = zaddr(k);
      const cf zk = z[p];
      const cf zc = z[zaddr(kc)];
      const cf fe = 0.5f * cf{zk.x + zc.x, zk.y - zc.y};
      const cf fo = 0.5f * cf{zk.y + zc.y, zc.x - zk.x};
      const cf wk = wn[it];
      const cf Xk = fe + cmul(wk, fo);
      // partner: Fe' = conj(fe), Fo' = conj(fo), W_N^(M-k) = -conj(W_N^k)
      const cf fe2 = cf{fe.x, -fe.y};
      const cf fo2 = cf{fo.x, -fo.y};
      const cf wk2 = cf{-wk.x, wk.y};
      const cf Xc = fe2 + cmul(wk2, fo2);  // X[M - k] (X[M] when k = 0)
      const cf Yk = cmul(Xk, hk[it]);
      const cf Yc = cmul(Xc, hc[it]);
      // inverse split: Z'[k] = (Y[k] + conj Y[M-k])/2 + i W_N^-k (Y[k] - conj Y[M-k])/2
      const cf s1 = 0.5f * cf{Yk.x + Yc.x, Yk.y - Yc.y};
      const cf d1 = 0.5f * cf{Yk.x - Yc.x, Yk.y + Yc.y};
      const cf wd = cmul(cf{wk.x, -wk.y}, d1);
      const cf zk2 = s1 + cf{-wd.y, wd.x};
      // partner k' = M - k: Y[k'] = Yc, Y[M-k'] = Yk, W_N^-(M-k) = -W_N^k
      const cf s2 = 0.5f * cf{Yc.x + Yk.x, Yc.y - Yk.y};
      const cf d2 = 0.5f * cf{Yc.x - Yk.x, Yc.y + Yk.y};
      const cf wd2 = cmul(cf{-wk.x, -wk.y}, d2);
      const cf zc2 = s2 + cf{-wd2.y, wd2.x};
      z[p] = zk2;
      if (kc != k) z[zaddr(kc)] = zc2;
    }
    __syncthreads();
    HBK_APH(9);
    // 5) inverse FFT (permuted -> natural), 1/M
    transform<true>(z, thi, tlo, ph_t0, 10);
    if (next) prefetch(clip + gridDim.x, noff_next, cmode_next);
    float ay = 0.f;
    for (int s = opaque_tid(); s < kT; s += kThreads) ay += fabsf(zf[s]);
    const float a_out = block_sum(ay, red) / kT / kM;
    HBK_APH(14);
    const float g = a_in / (a_out + 1e-14f) / kM;
    for (int s = opaque_tid(); s < kT; s += kThreads) out[s] = zf[s] * g;
    __syncthreads();
    HBK_APH(15);
  }
}

// Spectrum of one rotated IR kernel k [kT] -> H[k], k = 0..kM (natural order).
__global__ void __launch_bounds__(kThreads) spectrum_kernel(const float* kern, int64_t kern_stride,
                                                            float2* spectra, const float2* thi_,
                                                            const float2* tlo_, const float2* twn_) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  cf* z = reinterpret_cast<cf*>(smem);
  cf* thi = reinterpret_cast<cf*>(smem + 2 * kM + 32);
  cf* tlo = thi + kTwHi;
  load_tw(thi, tlo, thi_, tlo_);
  const cf* twn = reinterpret_cast<const cf*>(twn_);
  const float* k = kern + blockIdx.x * kern_stride;
  for (int s = threadIdx.x; s < kT; s += kThreads) smem[s] = k[s];
  __syncthreads();
  unsigned long long ph_t0 = 0;
  transform<false>(z, thi, tlo, ph_t0, 16);
  float2* H = spectra + static_cast<int64_t>(blockIdx.x) * kHSlots;
  for (int q = threadIdx.x; q <= kM; q += kThreads) {
    const int qq = q % kM, qc = (kM - q) % kM;
    const cf zk = z[zaddr(qq)];
    const cf zc = z[zaddr(qc)];
    const cf fe = 0.5f * cf{zk.x + zc.x, zk.y - zc.y};
    const cf fo = 0.5f * cf{zk.y + zc.y, zc.x - zk.x};
    const cf X = fe + cmul(twn[hslot(q)], fo);
    H[hslot(q)] = make_float2(X.x, X.y);
  }
}

// ---- band-stop ------------------------------------------------------------
// torch_audiomentations BandStopFilter (the reference's batch chain,
// augmented.py:101-105; p 0.25 per batch, one parameter set per batch):
//   y = x - julius.bandpass_filter(x, cut_lo, cut_hi)
// julius: the difference of two windowed-sinc lowpasses of half size
// h = int(8 / cut_lo / 2) over the clip padded by h replicated edge samples,
//   f_c[t] = 2 c hann[t + h] sinc(2 pi c t) / sum, t in [-h, h]
// (taps in float32 arithmetic, as torch computes them); g = f_hi - f_lo.
// Three launches per call: per filter (batch) the two lowpass sums and, for
// short filters, the taps g[0..h]; per filter spectrum (the reverb transform);
// per clip the convolution:
//  * h <= HBK_BAND_STOP_CIRCULAR_MAX_HALF (about 80 % of the reference's draws):
//    the clip's circular convolution with g (one forward and one inverse
//    transform, like the reverb), then the 2h edge samples corrected directly:
//    for n < h the taps that wrapped to the clip's end are replaced by the
//    replicated first sample, sum_{d < -n} g[d] (x[0] - x[T + n + d]), and
//    likewise at the other end;
//  * longer filters: overlap-save. f[k] = g[k - h], k < 2h + 1, in partitions
//    of kBsPart taps, each with its own spectrum; for partition p and output
//    half b the segment s[j] = xpad[11520 b + p kBsPart + j] (xpad[m] =
//    x[clamp(m - h, 0, T - 1)]) is transformed, multiplied, transformed back:
//    samples 0..11519 are the partition's sum for n = 11520 b + i (i + k <
//    23040: nothing wraps); the clip sits in a per-block global scratch row
//    (the output may alias the input).
constexpr int kBsHalf = kT / 2;             // outputs per overlap-save block
constexpr int kBsPart = kT - kBsHalf + 1;   // 11521 taps per partition
constexpr int kBsCirc = HBK_BAND_STOP_CIRCULAR_MAX_HALF;
static_assert(2 * kBsCirc <= kThreads, "one edge sample per thread");

// unnormalised julius lowpass tap t in [-h, h] (float32 as torch: hann from
// arange * f32(2 pi / (2h)), arg = f32(2 pi c) * t, 2c * w * sinc)
struct BsLowpass {
  float two_c, two_pi_c, wstep;
  int h;
  __device__ __forceinline__ BsLowpass(float c, int h_) : h(h_) {
    two_c = static_cast<float>(2.0 * double(c));
    two_pi_c = static_cast<float>(2.0 * double(c) * M_PI);
    wstep = static_cast<float>(2.0 * M_PI / double(2 * h_));
  }
  __device__ __forceinline__ float tap(int t) const {
    const float w = 0.5f - 0.5f * cosf(static_cast<float>(t + h) * wstep);
    const float arg = two_pi_c * static_cast<float>(t);
    const float sinc = arg == 0.f ? 1.f : sinf(arg) / arg;
    return two_c * w * sinc;
  }
};

struct BandStopArgs {
  const float* x;
  int64_t x_stride;
  float* out;
  int64_t out_stride;
  int64_t n;               // filtered clips
  const int32_t* idx;      // clip row of entry e
  const int32_t* filt;     // filter of entry e
  int n_filters;
  const float* f_lo;       // per filter: cutoffs (fraction of the sample rate), half size,
  const float* f_hi;       //   first spectrum slot
  const int32_t* f_half;
  const int32_t* f_spec0;
  int n_spectra;
  const int32_t* s_filt;   // per spectrum: filter, partition (-1: circular kernel)
  const int32_t* s_part;
  float2* sums;            // [n_filters]: the two lowpass sums (lo, hi)
  float* taps;             // [n_filters][kBsCirc + 1]: g[0..h] of circular filters
  float2* spectra;         // [n_spectra][kHSlots]
  float* scratch;          // [gridDim.x][kT]: overlap-save clips
  const float2* thi;
  const float2* tlo;
  const float2* twn;
};

// g[t] from the normalised lowpasses
__device__ __forceinline__ float bs_g(const BsLowpass& lo, const BsLowpass& hi, float2 s, int t) {
  return hi.tap(t) / s.y - lo.tap(t) / s.x;
}

// launch 1: one block per filter
__global__ void __launch_bounds__(kThreads) band_stop_sums_kernel(BandStopArgs a) {
  __shared__ float red[32];
  const int f = blockIdx.x;
  const int h = a.f_half[f];
  const BsLowpass lo(a.f_lo[f], h), hi(a.f_hi[f], h);
  double sl = 0.0, sh = 0.0;
  for (int t = static_cast<int>(threadIdx.x) - h; t <= h; t += kThreads) {
    sl += lo.tap(t);
    sh += hi.tap(t);
  }
  float fl = static_cast<float>(sl), fh = static_cast<float>(sh);
  block_sum2(fl, fh, red);
  const float2 sm = make_float2(fl, fh);
  if (threadIdx.x == 0) a.sums[f] = sm;
  if (h <= kBsCirc)
    for (int t = threadIdx.x; t <= h; t += kThreads) a.taps[int64_t(f) * (kBsCirc + 1) + t] = bs_g(lo, hi, sm, t);
}

// launch 2: one block per spectrum: circular kernel kappa[m] = g[(-m) mod T]
// (|t| <= h) or overlap-save partition p: kappa[0] = f_p[0], kappa[T - k] = f_p[k]
__global__ void __launch_bounds__(kThreads) band_stop_spectrum_kernel(BandStopArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  cf* z = reinterpret_cast<cf*>(smem);
  cf* thi = reinterpret_cast<cf*>(smem + 2 * kM + 32);
  cf* tlo = thi + kTwHi;
  load_tw(thi, tlo, a.thi, a.tlo);
  const cf* twn = reinterpret_cast<const cf*>(a.twn);
  const int sidx = blockIdx.x, f = a.s_filt[sidx], p = a.s_part[sidx];
  const int h = a.f_half[f], L = 2 * h + 1;
  const BsLowpass lo(a.f_lo[f], h), hi(a.f_hi[f], h);
  const float2 sm = a.sums[f];
  for (int m = threadIdx.x; m < kT; m += kThreads) {
    float v = 0.f;
    if (p < 0) {  // circular: tap t = -m or T - m
      const int t = m <= kT / 2 ? -m : kT - m;
      if (t >= -h && t <= h) v = bs_g(lo, hi, sm, t);
    } else {
      const int k = m == 0 ? 0 : kT - m;
      const int kk = p * kBsPart + k;
      if (k < kBsPart && kk < L) v = bs_g(lo, hi, sm, kk - h);
    }
    smem[m] = v;
  }
  __syncthreads();
  unsigned long long ph_t0 = 0;
  transform<false>(z, thi, tlo, ph_t0, 16);
  cf* H = reinterpret_cast<cf*>(a.spectra) + static_cast<int64_t>(sidx) * kHSlots;
  for (int q = threadIdx.x; q <= kM; q += kThreads) {
    const int qq = q % kM, qc = (kM - q) % kM;
    const cf zk = z[zaddr(qq)];
    const cf zc = z[zaddr(qc)];
    const cf fe = 0.5f * cf{zk.x + zc.x, zk.y - zc.y};
    const cf fo = 0.5f * cf{zk.y + zc.y, zc.x - zk.x};
    H[hslot(q)] = fe + cmul(twn[hslot(q)], fo);
  }
}

// the split, x H, inverse split on (k, M - k) pairs (as augment_kernel)
__device__ __forceinline__ void bs_multiply(cf* z, const cf* H, const cf* twn) {
  constexpr int kRest = kM / 2 / 16 + 1;
  for (int idx = opaque_tid(); idx < 16 * kRest; idx += kThreads) {
    const int c = idx / kRest;
    const int k = c + 16 * (idx - c * kRest);
    if (k > kM / 2) continue;
    const int kc = (kM - k) % kM;
    const int pz = zaddr(k);
    const cf zk = z[pz];
    const cf zc = z[zaddr(kc)];
    const cf fe = 0.5f * cf{zk.x + zc.x, zk.y - zc.y};
    const cf fo = 0.5f * cf{zk.y + zc.y, zc.x - zk.x};
    const cf wk = twn[hslot(k)];
    const cf Xk = fe + cmul(wk, fo);
    const cf Xc = cf{fe.x, -fe.y} + cmul(cf{-wk.x, wk.y}, cf{fo.x, -fo.y});
    const cf Yk = cmul(Xk, H[hslot(k)]);
    const cf Yc = cmul(Xc, H[hslot(kM - k)]);
    const cf s1 = 0.5f * cf{Yk.x + Yc.x, Yk.y - Yc.y};
    const cf d1 = 0.5f * cf{Yk.x - Yc.x, Yk.y + Yc.y};
    const cf wd = cmul(cf{wk.x, -wk.y}, d1);
    const cf s2 = 0.5f * cf{Yc.x + Yk.x, Yc.y - Yk.y};
    const cf d2 = 0.5f * cf{Yc.x - Yk.x, Yc.y + Yk.y};
    const cf wd2 = cmul(cf{-wk.x, -wk.y}, d2);
    z[pz] = s1 + cf{-wd.y, wd.x};
    if (kc != k) z[zaddr(kc)] = s2 + cf{-wd2.y, wd2.x};
  }
}

// launch 3: one block per clip (grid-strided)
__global__ void __launch_bounds__(kThreads) band_stop_kernel(BandStopArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  cf* z = reinterpret_cast<cf*>(smem);
  cf* thi = reinterpret_cast<cf*>(smem + 2 * kM + 32);
  cf* tlo = thi + kTwHi;
  float* gt = reinterpret_cast<float*>(tlo + kTwLo);  // [kBsCirc + 1] taps g[0..h]
  float* xe = gt + kBsCirc + 1;                        // [4 kBsCirc]: x[0, 2h), x[T - 2h, T)
  load_tw(thi, tlo, a.thi, a.tlo);
  const cf* twn = reinterpret_cast<const cf*>(a.twn);
  float* zf = smem;
  float* xs = a.scratch + static_cast<int64_t>(blockIdx.x) * kT;
  unsigned long long ph_t0 = 0;
  for (int64_t e = blockIdx.x; e < a.n; e += gridDim.x) {
    const int64_t clip = a.idx[e];
    const float* x = a.x + clip * a.x_stride;
    float* out = a.out + clip * a.out_stride;
    const int f = a.filt[e];
    const int h = a.f_half[f];
    const cf* H0 = reinterpret_cast<const cf*>(a.spectra) + static_cast<int64_t>(a.f_spec0[f]) * kHSlots;
    __syncthreads();  // the previous clip's readers of LDS / xs are done
    if (h <= kBsCirc) {
      // circular convolution + direct correction of the 2h edge samples
      for (int s = opaque_tid(); s < kT; s += kThreads) zf[s] = x[s];
      for (int t = threadIdx.x; t <= h; t += kThreads) gt[t] = a.taps[int64_t(f) * (kBsCirc + 1) + t];
      for (int i = threadIdx.x; i < 2 * h; i += kThreads) {
        xe[i] = x[i];
        xe[2 * kBsCirc + i] = x[kT - 2 * h + i];
      }
      __syncthreads();
      // edge sample of this thread (n < h, or n >= T - h), computed before the
      // transform overwrites nothing it needs (x edges and taps live apart from z)
      const int tid = threadIdx.x;
      float corr = 0.f;
      int n_edge = -1;
      if (tid < 2 * h) {
        const float* xb = xe + 2 * kBsCirc;  // xb[j] = x[T - 2h + j]
        if (tid < h) {  // n = tid: taps d = -h .. -n-1 wrapped to x[T + n + d]
          n_edge = tid;
          const float x0 = xe[0];
          for (int d = -h; d < -n_edge; ++d) corr += gt[-d] * (x0 - xb[2 * h + n_edge + d]);
        } else {  // n = T - 2h + tid: taps d = T - n .. h wrapped to x[n + d - T]
          n_edge = kT - 2 * h + tid;
          const float x1 = xb[2 * h - 1];
          for (int d = kT - n_edge; d <= h; ++d) corr += gt[d] * (x1 - xe[n_edge + d - kT]);
        }
      }
      transform<false>(z, thi, tlo, ph_t0, 16);
      bs_multiply(z, H0, twn);
      __syncthreads();
      transform<true>(z, thi, tlo, ph_t0, 16);
      // out = x - conv (x re-read from global: each thread reads then writes only its own samples)
      for (int s = opaque_tid(); s < kT; s += kThreads) {
        const bool edge = s < h || s >= kT - h;
        if (!edge) out[s] = x[s] - zf[s] * (1.f / kM);
      }
      if (n_edge >= 0) {
        const float xv = n_edge < h ? xe[n_edge] : xe[2 * kBsCirc + n_edge - (kT - 2 * h)];
        out[n_edge] = xv - (zf[n_edge] * (1.f / kM) + corr);
      }
      continue;
    }
    // overlap-save over partitions of kBsPart taps
    for (int s = opaque_tid(); s < kT; s += kThreads) xs[s] = x[s];
    const int parts = (2 * h + 1 + kBsPart - 1) / kBsPart;
    for (int p = 0; p < parts; ++p) {
      const cf* Hp = H0 + static_cast<int64_t>(p) * kHSlots;
      for (int b = 0; b < 2; ++b) {
        __syncthreads();  // xs published; the previous transform's readers of z are done
        const int base = b * kBsHalf + p * kBsPart - h;
        for (int j = opaque_tid(); j < kT; j += kThreads) zf[j] = xs[min(max(base + j, 0), kT - 1)];
        __syncthreads();
        transform<false>(z, thi, tlo, ph_t0, 16);
        bs_multiply(z, Hp, twn);
        __syncthreads();
        transform<true>(z, thi, tlo, ph_t0, 16);
        // y = x - sum_p c_p: each thread revisits only the samples it wrote before
        for (int i = opaque_tid(); i < kBsHalf; i += kThreads) {
          const int n = b * kBsHalf + i;
          const float c = zf[i] * (1.f / kM);
          out[n] = (p == 0 ? xs[n] : out[n]) - c;
        }
      }
    }
  }
}

// ---- colored noise --------------------------------------------------------
// torch_audiomentations AddColoredNoise (the reference's batch chain,
// augmented.py:107-113; p 0.25 per batch, snr ~ U[10, 30] dB and f_decay ~
// U[-1, 2] per clip, constants.py:128-132). Per clip:
//   w ~ N(0, 1) [T]; S = rfft(w) / linspace(1, sqrt(sr / 2), T/2 + 1)^f_decay;
//   n = irfft(S); n /= rms(n) + 1e-8; y = x + rms(x) / 10^(snr / 20) n.
// One workgroup per clip on the augment kernel's LDS transform: white noise
// into LDS, forward FFT, the real-FFT split x mask x inverse split on (k, M-k)
// pairs, inverse FFT, then rms(n) and rms(x) in one block sum and the mix.
// White noise comes from the caller (parity tests) or from a counter-based
// Box-Muller stream (seed, clip, sample): no RNG state, any grid.
struct ColoredArgs {
  const float* x;
  int64_t x_stride;
  float* out;
  int64_t out_stride;
  int64_t n_clips;
  const float* white;     // [n_clips, white_stride >= 16000] N(0,1) or NULL (generated from seed)
  int64_t white_stride;
  uint64_t seed;
  int64_t group;          // clips per white-noise vector (per_batch: the batch size)
  const float* f_decay;   // per clip
  const float* snr_db;    // per clip
  float lin_step;         // (sqrt(8000) - 1) / 8000: linspace step over the 8001 bins
  const int32_t* idx;     // NULL: every clip; else the n_entries listed clip rows (balanced launch)
  int64_t n_entries;
  const float2* thi;
  const float2* tlo;
  const float2* twn;
  // group path (clips_per_noise > 1, hbk_colored_noise_ws): colored_group_kernel writes each
  // group's coloured second (x kM1) and its rms; a clip whose f_decay equals its group's first
  // clip's mixes from it (NULL: every clip colours its own second)
  float* gbuf;            // [n_groups][kN1]
  float* grms;            // [n_groups]: rms of the coloured second, NaN where not made
  int64_t n_groups;
  int no_copy;            // hbk_augment_colored: clips this kernel does not colour are left alone
};

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
// standard normals 2i and 2i + 1 of the stream (Box-Muller on two 24-bit
// uniforms of one hash: both the cosine and the sine branch)
__device__ __forceinline__ float2 gauss2(uint64_t seed, uint64_t i) {
  const uint64_t h = mix64(seed + 0x9E3779B97F4A7C15ull * (i + 1));
  const float u1 = (static_cast<float>(h >> 40) + 0.5f) * (1.f / 16777216.f);
  const float u2 = static_cast<float>((h >> 16) & 0xFFFFFF) * (1.f / 16777216.f);
  const float r = sqrtf(-2.f * __logf(u1));
  float sn, cs;
  __sincosf(6.283185307179586f * u2, &sn, &cs);
  return make_float2(r * cs, r * sn);
}

// a clip copied through registers: all loads issued before the first store
// (a load -> store loop waits out one memory latency per element, since x and
// out may alias)
// (groups of 8 slots: few live VGPRs in the 64-VGPR tanh kernel)
__device__ __forceinline__ void copy_clip(const float* x, float* out, int tid) {
  constexpr int kPer = (kT + kThreads - 1) / kThreads, kG = 8;
#pragma unroll 1
  for (int u0 = 0; u0 < kPer; u0 += kG) {
    float v[kG];
#pragma unroll
    for (int u = 0; u < kG; ++u) {
      const int s = tid + (u0 + u) * kThreads;
      v[u] = s < kT ? *reinterpret_cast<const float*>(reinterpret_cast<const char*>(x) + (static_cast<uint32_t>(s) << 2))
                    : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kG; ++u) {
      const int s = tid + (u0 + u) * kThreads;
      if (s < kT) *reinterpret_cast<float*>(reinterpret_cast<char*>(out) + (static_cast<uint32_t>(s) << 2)) = v[u];
    }
  }
}

// ---- 8000-point complex FFT (the 16,000-sample real FFT of one second of
// noise): DIF passes 16 x 5 x 5 x 5 x 4 in LDS, twiddles W_8000^e =
// HI8[e / 100] LO8[e % 100]; frequency f = k1 + 16 k2 + 80 k3 + 400 k4 + 2000 k5
// lands at 500 k1 + 100 k2 + 20 k3 + 4 k4 + k5.
constexpr int kTw8Lo = 100, kTw8Hi = kM1 / kTw8Lo;  // 100 x 80

template <bool INV>
__device__ __forceinline__ cf twiddle8(const cf* thi, const cf* tlo, int e) {
  const int h = e / kTw8Lo;
  const cf w = cmul(thi[h], tlo[e - h * kTw8Lo]);
  return INV ? cf{w.x, -w.y} : w;
}

template <int R, int L, int S, bool INV>
__device__ __forceinline__ void pass8(cf* z, const cf* thi, const cf* tlo) {
  constexpr int kTasks = kM1 / R;
  int t0;
  asm volatile("v_mov_b32 %0, %1" : "=v"(t0) : "v"(static_cast<int>(threadIdx.x)));
  for (int t = t0; t < kTasks; t += kThreads) {
    const int blk = t / L, i = t - (t / L) * L;
    cf* q = z + blk * (R * L) + i;
    cf v[R];
#pragma unroll
    for (int m = 0; m < R; ++m) v[m] = q[L * m];
    cf w[R];
    if constexpr (S != 0) {
#pragma unroll
      for (int k = 1; k < R; ++k) w[k] = twiddle8<INV>(thi, tlo, S * i * k);
    }
    if (INV && S)
#pragma unroll
      for (int k = 1; k < R; ++k) v[k] = cmul(v[k], w[k]);
    if constexpr (R == 16) fft16v<INV>(v);
    else if constexpr (R == 4) fft4v<INV>(v[0], v[1], v[2], v[3]);
    else dft5<INV>(v);
    if (!INV && S)
#pragma unroll
      for (int k = 1; k < R; ++k) v[k] = cmul(v[k], w[k]);
#pragma unroll
    for (int m = 0; m < R; ++m) q[L * m] = v[m];
  }
}

template <bool INV>
__device__ __forceinline__ void transform8(cf* z, const cf* thi, const cf* tlo) {
  if (!INV) {
    pass8<16, 500, 1, false>(z, thi, tlo);
    __syncthreads();
    pass8<5, 100, 16, false>(z, thi, tlo);
    __syncthreads();
    pass8<5, 20, 80, false>(z, thi, tlo);
    __syncthreads();
    pass8<5, 4, 400, false>(z, thi, tlo);
    __syncthreads();
    pass8<4, 1, 0, false>(z, thi, tlo);
    __syncthreads();
  } else {
    pass8<4, 1, 0, true>(z, thi, tlo);
    __syncthreads();
    pass8<5, 4, 400, true>(z, thi, tlo);
    __syncthreads();
    pass8<5, 20, 80, true>(z, thi, tlo);
    __syncthreads();
    pass8<5, 100, 16, true>(z, thi, tlo);
    __syncthreads();
    pass8<16, 500, 1, true>(z, thi, tlo);
    __syncthreads();
  }
}

__device__ __forceinline__ int zaddr8(int f) {
  const int k1 = f & 15, r = f >> 4;  // r = k2 + 5 k3 + 25 k4 + 125 k5
  const int k2 = r % 5, r2 = r / 5;
  const int k3 = r2 % 5, r3 = r2 / 5;
  const int k4 = r3 % 5, k5 = r3 / 5;
  return 500 * k1 + 100 * k2 + 20 * k3 + 4 * k4 + k5;
}

// 1) + 2): group grp's second of white noise -> LDS, forward FFT, the real-FFT split x the
// 1 / linspace^f_decay mask x inverse split, inverse FFT: zf = the coloured second x kM1
// (natural order). Entered and left at a barrier.
__device__ __forceinline__ void colored_second(const ColoredArgs& a, cf* z, const cf* thi, const cf* tlo, int tid,
                                               int64_t grp, float fd) {
  float* zf = reinterpret_cast<float*>(z);
  // 1) one second of white noise -> LDS (the previous clip's readers finished at its last barrier)
  if (a.white) {
    const float* w = a.white + grp * a.white_stride;
    for (int s = tid; s < kN1; s += kThreads) zf[s] = w[s];
  } else {
    for (int q = tid; q < kN1 / 2; q += kThreads) {
      const float2 g = gauss2(a.seed, static_cast<uint64_t>(grp) * (kN1 / 2) + q);
      *reinterpret_cast<float2*>(zf + 2 * q) = g;
    }
  }
  __syncthreads();
  transform8<false>(z, thi, tlo);
  // 2) X = split(Z); Y = X / lin^f_decay; Z' = inverse split(Y), pairs (k, M - k), k <= M / 2
  for (int k = tid; k <= kM1 / 2; k += kThreads) {
    const int kc = (kM1 - k) % kM1;
    const int p = zaddr8(k), pc = zaddr8(kc);
    const cf zk = z[p];
    const cf zc = z[pc];
    const cf fe = 0.5f * cf{zk.x + zc.x, zk.y - zc.y};
    const cf fo = 0.5f * cf{zk.y + zc.y, zc.x - zk.x};
    const cf wk = cf{a.twn[k].x, a.twn[k].y};  // W_16000^k
    const float mk = exp2f(-fd * __log2f(fmaf(a.lin_step, static_cast<float>(k), 1.f)));
    const float mc = exp2f(-fd * __log2f(fmaf(a.lin_step, static_cast<float>(kM1 - k), 1.f)));  // bin M - k
    const cf Yk = mk * (fe + cmul(wk, fo));
    const cf Yc = mc * (cf{fe.x, -fe.y} + cmul(cf{-wk.x, wk.y}, cf{fo.x, -fo.y}));
    const cf s1 = 0.5f * cf{Yk.x + Yc.x, Yk.y - Yc.y};
    const cf d1 = 0.5f * cf{Yk.x - Yc.x, Yk.y + Yc.y};
    const cf wd = cmul(cf{wk.x, -wk.y}, d1);
    const cf s2 = 0.5f * cf{Yc.x + Yk.x, Yc.y - Yk.y};
    const cf d2 = 0.5f * cf{Yc.x - Yk.x, Yc.y + Yk.y};
    const cf wd2 = cmul(cf{-wk.x, -wk.y}, d2);
    z[p] = s1 + cf{-wd.y, wd.x};
    if (kc != k) z[pc] = s2 + cf{-wd2.y, wd2.x};
  }
  __syncthreads();
  transform8<true>(z, thi, tlo);  // natural order, x kM1
}

// torch_audiomentations AddColoredNoise (per clip, white noise w of ONE second):
//   n1 = irfft(rfft(w[:16000]) / linspace(1, sqrt(sr/2), 8001)^f_decay)      (16,000)
//   n1 /= rms(n1) + 1e-8;  noise[t] = n1[t mod 16000], t < T (tiled, not renormalised)
//   y = x + rms(x) / 10^(snr/20) noise
// The 16,000 noise samples as 8000 complex pairs in LDS, forward FFT, the
// real-FFT split x mask x inverse split on (k, M - k) pairs, inverse FFT.
__global__ void __launch_bounds__(kThreads) colored_noise_kernel(ColoredArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  cf* z = reinterpret_cast<cf*>(smem);                 // kM1 complex
  float* red = smem + 2 * kM1;                         // 32 floats
  cf* thi = reinterpret_cast<cf*>(smem + 2 * kM1 + 32);
  cf* tlo = thi + kTw8Hi;
  for (int i = threadIdx.x; i < kTw8Hi; i += kThreads) thi[i] = cf{a.thi[i].x, a.thi[i].y};
  for (int i = threadIdx.x; i < kTw8Lo; i += kThreads) tlo[i] = cf{a.tlo[i].x, a.tlo[i].y};
  float* zf = smem;
  constexpr int kPer = (kT + kThreads - 1) / kThreads;
  const int64_t n_iter = a.idx ? a.n_entries : a.n_clips;
  for (int64_t e = blockIdx.x; e < n_iter; e += gridDim.x) {
    const int64_t clip = a.idx ? a.idx[e] : e;
    const int tid = opaque_tid();
    const float snr = a.snr_db[clip];
    if (snr != snr) {  // NaN: this clip's batch drew no colored noise (uniform per block)
      if (!a.no_copy && (a.out != a.x || a.out_stride != a.x_stride))
        copy_clip(a.x + clip * a.x_stride, a.out + clip * a.out_stride, tid);
      continue;
    }
    const int64_t grp = clip / a.group;  // clips of one batch share the noise vector (per_batch)
    float rms_g = __builtin_nanf("");
    if (a.grms && a.f_decay[clip] == a.f_decay[grp * a.group]) rms_g = a.grms[grp];  // uniform per block
    if (rms_g == rms_g) continue;  // the group's coloured second is made: colored_mix_kernel mixes it
    colored_second(a, z, thi, tlo, tid, grp, a.f_decay[clip]);
    // 3) rms(n1) over 16,000 and rms(x) over T in one block sum; tile and mix
    const float* x = a.x + clip * a.x_stride;
    float xr[kPer];
    float ex = 0.f, en = 0.f;
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int s = tid + u * kThreads;
      xr[u] = 0.f;
      if (s < kT) {
        xr[u] = x[s];
        ex = fmaf(xr[u], xr[u], ex);
      }
      if (s < kN1) {
        const float nv = zf[s] * (1.f / kM1);
        en += nv * nv;
      }
    }
    block_sum2(ex, en, red);
    const float rms_x = sqrtf(ex / kT), rms_n = sqrtf(en / kN1);
    const float scale = rms_x / powf(10.f, snr / 20.f) / (rms_n + 1e-8f) * (1.f / kM1);
    float* out = a.out + clip * a.out_stride;
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int s = tid + u * kThreads;
      if (s < kT) out[s] = fmaf(scale, zf[s < kN1 ? s : s - kN1], xr[u]);
    }
    __syncthreads();  // zf is rewritten by the next clip
  }
}

// The coloured second of every group whose first clip draws noise (clips_per_noise > 1:
// per_batch mode shares the white noise and, in the reference's chain, f_decay across the
// batch), with its rms computed exactly as the clip kernel does.
__global__ void __launch_bounds__(kThreads) colored_group_kernel(ColoredArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  cf* z = reinterpret_cast<cf*>(smem);
  float* red = smem + 2 * kM1;
  cf* thi = reinterpret_cast<cf*>(smem + 2 * kM1 + 32);
  cf* tlo = thi + kTw8Hi;
  for (int i = threadIdx.x; i < kTw8Hi; i += kThreads) thi[i] = cf{a.thi[i].x, a.thi[i].y};
  for (int i = threadIdx.x; i < kTw8Lo; i += kThreads) tlo[i] = cf{a.tlo[i].x, a.tlo[i].y};
  const float* zf = smem;
  constexpr int kPer = (kT + kThreads - 1) / kThreads;
  for (int64_t g = blockIdx.x; g < a.n_groups; g += gridDim.x) {
    const int tid = opaque_tid();
    const int64_t c0 = g * a.group;
    if (a.snr_db[c0] != a.snr_db[c0]) {  // the group's first clip draws no noise: not made
      if (tid == 0) a.grms[g] = __builtin_nanf("");
      continue;
    }
    __syncthreads();  // tables loaded / the previous group's readers of zf are done
    colored_second(a, z, thi, tlo, tid, g, a.f_decay[c0]);
    float ex = 0.f, en = 0.f;
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int s = tid + u * kThreads;
      if (s < kN1) {
        const float nv = zf[s] * (1.f / kM1);
        en += nv * nv;
      }
    }
    block_sum2(ex, en, red);
    float* gb = a.gbuf + g * kN1;
    for (int s = tid; s < kN1; s += kThreads) gb[s] = zf[s];
    if (tid == 0) a.grms[g] = sqrtf(en / kN1);
    __syncthreads();
  }
}

// The clips of made groups (colored_group_kernel): rms(x) and the mix, from the group's
// coloured second in global memory (L2-resident across its clips). The same per-thread
// order and block sum as colored_noise_kernel, so the result is bit-identical; no
// transform LDS, so two 1024-thread blocks (two clips in flight) per CU.
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(8))) colored_mix_kernel(ColoredArgs a) {
  __shared__ float red[32];
  constexpr int kPer = (kT + kThreads - 1) / kThreads;
  const int64_t n_iter = a.idx ? a.n_entries : a.n_clips;
  for (int64_t e = blockIdx.x; e < n_iter; e += gridDim.x) {
    const int64_t clip = a.idx ? a.idx[e] : e;
    const int tid = opaque_tid();
    const float snr = a.snr_db[clip];
    const int64_t grp = clip / a.group;
    float rms_g = __builtin_nanf("");
    if (snr == snr && a.f_decay[clip] == a.f_decay[grp * a.group]) rms_g = a.grms[grp];
    if (rms_g != rms_g) continue;  // uniform per block: colored_noise_kernel's clip
    const float* gb = a.gbuf + grp * kN1;
    const float* x = a.x + clip * a.x_stride;
    // two passes over x (the second from the cache): nothing is held across the block sum,
    // so the kernel fits 64 VGPRs without spills; ex in colored_noise_kernel's order
    float ex = 0.f, en = 0.f;
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int s = tid + u * kThreads;
      if (s < kT) {  // 32-bit byte offsets on uniform bases
        const float v = *reinterpret_cast<const float*>(reinterpret_cast<const char*>(x) + (static_cast<uint32_t>(s) << 2));
        ex = fmaf(v, v, ex);
      }
    }
    block_sum2(ex, en, red);
    const float rms_x = sqrtf(ex / kT);
    const float scale = rms_x / powf(10.f, snr / 20.f) / (rms_g + 1e-8f) * (1.f / kM1);
    float* out = a.out + clip * a.out_stride;
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int s = tid + u * kThreads;
      if (s < kT) {
        const int sn = s < kN1 ? s : s - kN1;
        const float xv = *reinterpret_cast<const float*>(reinterpret_cast<const char*>(x) + (static_cast<uint32_t>(s) << 2));
        const float nv =
            *reinterpret_cast<const float*>(reinterpret_cast<const char*>(gb) + (static_cast<uint32_t>(sn) << 2));
        *reinterpret_cast<float*>(reinterpret_cast<char*>(out) + (static_cast<uint32_t>(s) << 2)) = fmaf(scale, nv, xv);
      }
    }
    __syncthreads();  // red is reused by the next clip
  }
}

// ---- tanh distortion ------------------------------------------------------
// audiomentations TanhDistortion (the reference's per-clip Compose,
// augmented.py:79-90; p 0.25, distortion ~ U[1e-4, 0.1], constants.py:122-124):
//   q = 100 - 99 amount; th = percentile(|x|, q) (numpy's linear interpolation);
//   y = tanh(0.5 / (th + 1e-6) x); if rms(x) > 1e-9: y *= rms(x) / rms(y).
// One workgroup per clip, the clip in registers. The two order statistics of
// |x| around the percentile come from an LDS radix select over the f32 bit
// patterns (non-negative floats order like their bits): four 8-bit histogram
// passes for rank lo, then its successor from one count + min reduction.
struct TanhArgs {
  const float* x;
  int64_t x_stride;
  float* out;
  int64_t out_stride;
  int64_t n_clips;
  const float* amount;  // per clip; NaN = clip unchanged
  const int32_t* idx;   // NULL: every clip; else the n_entries listed clip rows (balanced launch)
  int64_t n_entries;
};

// |x| bits of slot u (u < kPer), or ~0 past the end of the clip (above every value);
// recomputed per pass instead of held (2 blocks / CU need <= 64 VGPRs)
__device__ __forceinline__ unsigned abs_bits(float v, int s) {
  return s < kT ? (__builtin_bit_cast(unsigned, v) & 0x7FFFFFFFu) : 0xFFFFFFFFu;
}

__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(8)))
tanh_distortion_kernel(TanhArgs a) {
  // radix-select digits over |x|'s bits 30..0 (bit 31 is 0): 12 + 10 + 9 bits. The first
  // digit spans the exponent and 4 mantissa bits, so a clip's values spread over ~200 bins
  // instead of crowding the ~9 of an 8-bit top digit (LDS atomics to one address serialise)
  __shared__ unsigned hist[4096];
  __shared__ float red[32];
  __shared__ unsigned pick[2];  // selected digit, rank left within it
  constexpr int kPer = (kT + kThreads - 1) / kThreads;
  const int64_t n_iter = a.idx ? a.n_entries : a.n_clips;
  for (int64_t e = blockIdx.x; e < n_iter; e += gridDim.x) {
    const int64_t clip = a.idx ? a.idx[e] : e;
    const int tid = opaque_tid();
    const float* x = a.x + clip * a.x_stride;
    float* out = a.out + clip * a.out_stride;
    const float amt = a.amount[clip];
    if (amt != amt) {
      if (out != x) copy_clip(x, out, tid);
      continue;
    }
    // uniform base + 32-bit byte offsets (global_load's saddr form): one VGPR per
    // address instead of a hoisted 64-bit pointer per slot
    float xr[kPer];
    {
    const int t = opaque_tid();
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int s = t + u * kThreads;
      xr[u] = s < kT ? *reinterpret_cast<const float*>(reinterpret_cast<const char*>(x) + (static_cast<uint32_t>(s) << 2))
                     : 0.f;
    }
    }
    // numpy percentile, method "linear": position q/100 (N - 1)
    const double pos = (100.0 - 99.0 * static_cast<double>(amt)) / 100.0 * (kT - 1);
    const int lo = min(max(static_cast<int>(floor(pos)), 0), kT - 1);
    const double frac = pos - lo;
    unsigned prefix = 0, mask = 0, rank = static_cast<unsigned>(lo);
#pragma unroll 1
    for (int p = 0; p < 3; ++p) {
      const int shift = p == 0 ? 19 : (p == 1 ? 9 : 0), bins = p == 0 ? 4096 : (p == 1 ? 1024 : 512);
      const int per_lane = bins >> 6;  // bins per lane of wave 0's scan
      for (int i = tid; i < bins; i += kThreads) hist[i] = 0;
      __syncthreads();
      const int t = opaque_tid();
#pragma unroll
      for (int u = 0; u < kPer; ++u) {
        const unsigned b = abs_bits(xr[u], t + u * kThreads);
        if ((b & mask) == prefix && b != 0xFFFFFFFFu) atomicAdd(&hist[(b >> shift) & (bins - 1)], 1u);
      }
      __syncthreads();
      if (tid < 64) {  // wave 0: per_lane bins per lane, inclusive scan over lanes, first lane past rank
        unsigned own = 0;
        for (int i = 0; i < per_lane; ++i) own += hist[per_lane * tid + i];
        unsigned inc = own;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const unsigned v = __shfl_up(inc, d, 64);
          if (tid >= d) inc += v;
        }
        const unsigned long long hit = __ballot(inc > rank);
        const int l = __ffsll(static_cast<long long>(hit)) - 1;
        if (tid == l) {
          unsigned r = rank - (inc - own), dsel = per_lane * l;
          for (int i = 0; i < per_lane - 1; ++i) {
            const unsigned h = hist[dsel];
            if (r < h) break;
            r -= h;
            ++dsel;
          }
          pick[0] = dsel;
          pick[1] = r;
        }
      }
      __syncthreads();
      prefix |= pick[0] << shift;
      mask |= static_cast<unsigned>(bins - 1) << shift;
      rank = pick[1];
    }
    // successor: v_lo again if more than lo + 1 values are <= v_lo, else min{|x| > v_lo}
    float cnt = 0.f, mg = __builtin_inff();
    const int t2 = opaque_tid();
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const unsigned b = abs_bits(xr[u], t2 + u * kThreads);
      if (b == 0xFFFFFFFFu) continue;
      if (b <= prefix) cnt += 1.f;
      else mg = fminf(mg, __builtin_bit_cast(float, b));
    }
    cnt = block_sum(cnt, red);
    {  // block min (wave min through shuffles, then the 16 partials)
      for (int d = 32; d >= 1; d >>= 1) mg = fminf(mg, __shfl_xor(mg, d, 64));
      __syncthreads();
      if ((tid & 63) == 0) red[tid >> 6] = mg;
      __syncthreads();
      mg = red[0];
      for (int w = 1; w < kThreads / 64; ++w) mg = fminf(mg, red[w]);
    }
    const double v_lo = __builtin_bit_cast(float, prefix);
    const double v_hi = (cnt >= lo + 2 || lo + 1 >= kT) ? v_lo : static_cast<double>(mg);
    const double d = v_hi - v_lo;
    const double th = frac >= 0.5 ? v_hi - d * (1.0 - frac) : v_lo + d * frac;  // numpy _lerp
    const float g = static_cast<float>(0.5 / (th + 1e-6));
    float ex = 0.f, ey = 0.f;
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      ex += xr[u] * xr[u];
      // tanh(v) = 1 - 2 / (e^(2v) + 1) on the transcendental unit (+-1 at the
      // overflow ends; absolute error ~1e-7, tanhf's polynomial cost ~4x more);
      // past-the-end slots hold 0 -> 0
      xr[u] = 1.f - __fdividef(2.f, __expf(2.f * g * xr[u]) + 1.f);
      ey += xr[u] * xr[u];
    }
    block_sum2(ex, ey, red);
    const float rms_x = sqrtf(ex / kT);
    const float post = rms_x > 1e-9f ? rms_x / sqrtf(ey / kT) : 1.f;
    const int t3 = opaque_tid();
#pragma unroll
    for (int u = 0; u < kPer; ++u) {
      const int s = t3 + u * kThreads;
      if (s < kT) *reinterpret_cast<float*>(reinterpret_cast<char*>(out) + (static_cast<uint32_t>(s) << 2)) = xr[u] * post;
    }
    __syncthreads();  // red / hist reuse by the next clip
  }
}

// Clip placement (AugmentedAudioGenerator.to_target_length, augmented.py:200-232):
// out[i, t] = src[i, t - pre[i]] for pre[i] <= t < pre[i] + min(len[i], T), else 0.
// One 256-thread block per (clip, 4096-sample span): every thread writes one
// float4 of out (T % 4 == 0); the shifted source is read with scalar loads
// (pre[i] is arbitrary, so the 4 samples are not 16-B aligned in src).
constexpr int kPlaceSpan = 4096;
__global__ void __launch_bounds__(256) place_kernel(const float* __restrict__ src, int64_t src_stride,
                                                    const int32_t* __restrict__ src_len,
                                                    const int32_t* __restrict__ pre, float* __restrict__ out,
                                                    int64_t out_stride, int64_t n_clips, int T) {
  // workgroup b takes (clip, span) item b (one 4,096-sample span of one clip; a 1-D grid, so
  // no 65,535-clip launch limit); every load is unconditional (clamped into the clip, zeroed by
  // a select), so a thread's 16 loads are in flight together instead of each behind its own
  // branch
  const int spans = (T + kPlaceSpan - 1) / kPlaceSpan;
  const int64_t items = n_clips * spans;
  constexpr int kR = kPlaceSpan / 1024;
  // (measured: the same 3.1 ms per 100 k clips, 4.85 TB/s, as the round-4 2-D grid with
  // predicated loads, tools/probe_place.py: the kernel is bound by HBM's write rate)
  for (int64_t it = blockIdx.x; it < items; it += gridDim.x) {  // (one pass: grid = items)
    const int64_t clip = it / spans;
    const int sp = static_cast<int>(it - clip * spans);
    const int p = pre[clip];
    const int n = min(src_len[clip], T);
    const int last = max(n - 1, 0);
    const float* s = src + clip * src_stride;
    float* o = out + clip * out_stride;
    const int t0 = sp * kPlaceSpan + 4 * static_cast<int>(threadIdx.x);
    float v[kR][4];
#pragma unroll
    for (int r = 0; r < kR; ++r)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int u = t0 + r * 1024 + q - p;
        const float x = n > 0 ? s[min(max(u, 0), last)] : 0.f;  // (n: uniform per item)
        v[r][q] = (u >= 0 && u < n) ? x : 0.f;
      }
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      const int t = t0 + r * 1024;
      if (t < T) *reinterpret_cast<float4*>(o + t) = make_float4(v[r][0], v[r][1], v[r][2], v[r][3]);
    }
  }
}


// ---------------------------------------------------------------------------
// Seven-band parametric EQ: audiomentations SevenBandParametricEQ, the
// reference's per-clip transform ahead of tanh (dataset/augmented.py:79-84):
// seven RBJ biquads in series (low shelf, five peaks, high shelf), each the
// direct form II transposed recursion of scipy sosfilt in float64 with its
// output rounded to float32 before the next stage (audiomentations casts each
// filter's output). One lane per clip: the recursion is sequential in time,
// and clips are the parallel axis. A wave owns 64 clips; 64-sample tiles are
// loaded coalesced (16 lanes per clip row, float4), transposed through LDS to
// [sample][clip] (conflict-free column reads), filtered in place and stored
// back the same way; the next tile's loads are issued before the current one
// is filtered. A clip whose first b0 is NaN is copied.
constexpr int kEqTile = 64;
struct EqArgs {
  const float* x;
  int64_t x_stride;
  const double* coef;  // [n][7][5]: b0, b1, b2, a1, a2 (a0 = 1)
  const int32_t* idx;  // clip of entry j (NULL: j)
  float* out;
  int64_t out_stride;
  int64_t n;
};

// Systolic over the cascade: a wave filters 8 clips, 8 lanes per clip; lane
// s < 7 holds section s's coefficients and state and, at step t, filters sample
// t - s: its input is section s - 1's output of step t - 1 (DPP row_shr:1),
// section 0 reads x[t] from the LDS tile, section 6's output is y[t - 6]. Each
// section runs the same float64 recursion, in the same order, as a one-lane
// cascade (float32 between sections), so the result is bitwise that of the
// sequential filter; eight times as many waves fill the chip (the filter is
// sequential in time, so one lane per clip left most SIMDs idle). A clip whose
// coefficients are NaN passes through an identity cascade (a copy).
constexpr int kEqClips = 8;  // clips per wave
__global__ void __launch_bounds__(64) eq_kernel(EqArgs a) {
  constexpr int kRow = kEqTile + 4;  // 16-B aligned rows (b128 reads / writes of 8 steps)
  __shared__ __attribute__((aligned(16))) float tin[kEqClips][kRow];
  __shared__ __attribute__((aligned(16))) float tout[kEqClips][kRow];
  const int lane = threadIdx.x, c = lane >> 3, sec = lane & 7;
  const int64_t j0 = static_cast<int64_t>(blockIdx.x) * kEqClips;
  const int64_t jc = min(j0 + c, a.n - 1);
  const double* cf0 = a.coef + jc * 35;
  const bool copy = cf0[0] != cf0[0];
  const int k = min(sec, 6);
  double b0 = cf0[5 * k], b1 = cf0[5 * k + 1], b2 = cf0[5 * k + 2], a1 = cf0[5 * k + 3], a2 = cf0[5 * k + 4];
  if (copy) b0 = 1.0, b1 = b2 = a1 = a2 = 0.0;
  double s1 = 0.0, s2 = 0.0;
  // tile I/O mapping: lane -> clip lc = lane >> 3, float4 column lq = lane & 7 (samples 4 lq, 32 + 4 lq)
  const int lc = lane >> 3, lq = lane & 7;
  const int64_t jl = min(j0 + lc, a.n - 1);
  const int64_t clip_l = a.idx ? static_cast<int64_t>(a.idx[jl]) : jl;
  const float* xl = a.x + clip_l * a.x_stride;
  float* ol = a.out + clip_l * a.out_stride;
  const bool store_l = j0 + lc < a.n;
  float4 p0 = *reinterpret_cast<const float4*>(xl + 4 * lq);
  float4 p1 = *reinterpret_cast<const float4*>(xl + 32 + 4 * lq);
  float prev = 0.f;
  for (int t0 = 0; t0 <= kT; t0 += kEqTile) {  // the last tile only drains the pipeline
    tin[lc][4 * lq] = p0.x;
    tin[lc][4 * lq + 1] = p0.y;
    tin[lc][4 * lq + 2] = p0.z;
    tin[lc][4 * lq + 3] = p0.w;
    tin[lc][32 + 4 * lq] = p1.x;
    tin[lc][32 + 4 * lq + 1] = p1.y;
    tin[lc][32 + 4 * lq + 2] = p1.z;
    tin[lc][32 + 4 * lq + 3] = p1.w;
    __syncthreads();
    const int tn = min(t0 + kEqTile, kT - kEqTile);  // next tile (clamped: the drain re-reads the last)
    p0 = *reinterpret_cast<const float4*>(xl + tn + 4 * lq);
    p1 = *reinterpret_cast<const float4*>(xl + tn + 32 + 4 * lq);
    // 8 steps per group: their section-0 inputs read ahead (two b128 reads, one
    // wait), section 6's outputs written after (branch-free steps in between)
    for (int st0 = 0; st0 < kEqTile; st0 += 8) {
      const float4 ia = *reinterpret_cast<const float4*>(&tin[c][st0]);
      const float4 ib = *reinterpret_cast<const float4*>(&tin[c][st0 + 4]);
      const float in8[8] = {ia.x, ia.y, ia.z, ia.w, ib.x, ib.y, ib.z, ib.w};
      float o8[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float u = sec == 0 ? in8[q] : prev;
        const double vd = u;
        const double y = fma(b0, vd, s1);
        s1 = fma(b1, vd, fma(-a1, y, s2));
        s2 = fma(b2, vd, -a2 * y);
        const float v = static_cast<float>(y);
        o8[q] = v;  // section 6: sample t0 + st0 + q - 6
        prev = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, prev),
                                                                     __builtin_bit_cast(int, v), 0x111, 0xF, 0xF,
                                                                     false));
      }
      if (sec == 6) {
        *reinterpret_cast<float4*>(&tout[c][st0]) = float4{o8[0], o8[1], o8[2], o8[3]};
        *reinterpret_cast<float4*>(&tout[c][st0 + 4]) = float4{o8[4], o8[5], o8[6], o8[7]};
      }
    }
    __syncthreads();
    if (store_l) {
#pragma unroll
      for (int m = 0; m < 8; ++m) {
        const int kk = lq + 8 * m;
        const int n = t0 - 6 + kk;
        if (n >= 0 && n < kT) ol[n] = tout[lc][kk];
      }
    }
    __syncthreads();
  }
}

// ----------------------------------------------------------------------------
// PitchShift (torch_audiomentations PitchShift -> torch_pitch_shift.pitch_shift,
// augmented.py:93-100): stft (n_fft 250, hop 7, rectangular window, center,
// reflect) -> phase vocoder (torchaudio TimeStretch, rate = 1 / shift) ->
// istft -> sinc resample (torchaudio Resample(sr, int(sr / shift))), cropped or
// zero-padded to the clip length. One ratio per call (per_batch mode).
//
// ps_vocoder_kernel: ONE pass per clip, 128 lanes = 126 bins, sequential over
// the clip's frames (kPvClips clips per workgroup in lockstep: every clip of a
// call has the same frame geometry). No spectrogram is stored, no segment is
// recomputed:
//  * analysis: a sliding DFT (hop 7: X_f = w^-7 (X_{f-1} + sum_j d_j w^j),
//    d_j = xp[7f+243+j] - xp[7f-7+j], w = e^{-2 pi i k/250}) whose state X is
//    float64 and whose increment sum_j d_j w^j is float32 (packed FMAs); a
//    direct float64 DFT restarts it every kPvRestart frames. A frame whose 250
//    samples are all zero is exactly 0 (angle 0) as in the FFT (a running
//    count of non-zero samples);
//  * vocoder without angles: the accumulated phase e^{i phi_t} is kept as a unit
//    complex P_t = u_0 prod (u_{i0+1} conj u_{i0}) of the frames' unit vectors
//    u = X / |X| (u = 1 for X = 0, angle 0 as in torch), since
//    e^{i (angle(X1) - angle(X0))} = u_1 conj u_0 whatever 2 pi wrap the
//    reference applies. The product telescopes while the source frame steps by
//    one: P_t = R u_{i0(t)} with R constant, changed only by a repeated source
//    frame (R *= u_{i0+1} conj u_{i0}) or a double step. The phase advance
//    2 pi 7k/250 cancels against the istft's frame rotation, so
//    Z_t = Y_t e^{-2 pi i 7kt/250} = m_t P_t e^{-2 pi i qz_t/250} with
//    qz_t = 7kt mod 250 an exact integer counter (no atan2, no sin / cos; R is
//    renormalised once per frame group);
//  * synthesis without inverse transforms: with Q_t = sum_{t' <= t} Z_t' (a
//    prefix per bin) and G(t, s) = Re sum_k c_k e^{2 pi i k (7t + s)/250} Q_t[k],
//    s < 7, the overlap-added istft sample p = 7t + r is
//      (G(t, r) - G(t - 36, r + 2)) / (250 env)   r <= 4 (frames t-35 .. t)
//      (G(t, r) - G(t - 35, r - 5)) / (250 env)   r = 5, 6 (frames t-34 .. t)
//    so a bin keeps no window of past frames. The 7 G(t, .) of a frame are
//    reduced over the bins in registers: lane k forms its 7 products
//    Re(Q_t e^{2 pi i 7kt/250} c_k e^{2 pi i ks/250}) and an 8-lane
//    reduce-scatter by DPP leaves s = g(lane & 7) on each lane; after the
//    group's 8 frames a reduce-scatter over the octets (DPP row_ror:8,
//    v_permlane16/32_swap) leaves frame u of the wave's 64 bins on octet u. No
//    LDS in the per-frame path; per kPvGroup frames one float per lane goes to
//    LDS for the istft samples.
// ps_resample_kernel (frame group, clip): polyphase sinc, taps in registers.
constexpr int kPsFft = 250, kPsHop = 7, kPsBins = kPsFft / 2 + 1, kPsPad = kPsFft / 2;
constexpr int kPsTapMax = HBK_PITCH_SHIFT_MAX_TAPS;    // 2 width + orig (142 / 139 at 16 kHz)
constexpr int kPsPhaseMax = 128;                       // new (resampler phases)
constexpr int kPsResFrames = 32;                       // resampler frames per workgroup
#ifndef HBK_PV_ABLATE
#define HBK_PV_ABLATE 0  // profiling builds: 1 skips the bin reduction, 2 the per-bin vocoder
#endif
#ifndef HBK_PV_CLIPS
#define HBK_PV_CLIPS 2  // measured: 1.79 us/clip at 2, 1.95 at 4, 2.33 at 1 (12,800 clips)
#endif
constexpr int kPvClips = HBK_PV_CLIPS;                 // clips per workgroup (128 lanes each)
constexpr int kPvGroup = 8;                            // output frames per istft step (lane 8u + .: frame u)
constexpr int kPvRows = 64;                            // input frames of d rows held in LDS
constexpr int kPvGh = 64;                              // ring of G(t, .) rows (>= 36 + kPvGroup)
#ifndef HBK_PV_F32STATE
#define HBK_PV_F32STATE 0  // 1: the sliding DFT's state in float32, restarted every 128 frames (variant pv32)
#endif
#ifndef HBK_PV_RESTART
#if HBK_PV_F32STATE
#define HBK_PV_RESTART 128
#else
#define HBK_PV_RESTART 1024  // measured L2 vs the float64 oracle: 3.8e-5 at 128, 5.6e-5 at 256, 6.5e-5 at 1024
#endif
#endif
constexpr int kPvRestart = HBK_PV_RESTART;             // sliding-DFT frames between direct DFTs
#if HBK_PV_F32STATE
typedef float pv_t;   // sliding-DFT state
#else
typedef double pv_t;
#endif

struct PitchArgs {
  const float* x;
  int64_t x_stride;
  const int32_t* idx;
  int n;
  float* out;
  int64_t out_stride;
  int L, f_in, f_out, l1, orig, nw, width, target;
  double rate;
  float* y;       // [n][l1]: istft output (resampler input)
  float* taps;    // [nw][kPsTapMax]
};

__device__ __forceinline__ int ps_i0(const PitchArgs& a, int t, float& alpha) {
  // torch.arange(0, f_in, rate, dtype=float32): start + step * i in double, cast
  const float ts = static_cast<float>(static_cast<double>(t) * a.rate);
  const float fl = floorf(ts);
  alpha = ts - fl;
  return static_cast<int>(fl);
}

struct PvClip {
  float d[kPvRows][8];        // row f - fb: d_j (j < 7) of frame f, [7] = the non-zero-count change
  float xs[256];              // xp[0, 250) (frame 0's direct DFT)
  float gh[2][kPvGh][8];      // G(t, s) over wave w's 64 bins, row t mod kPvGh (s = 7: unused)
  int cnt0;
};
struct PvShared {
  cf tw[256];                 // e^{+2 pi i q / 250}
  double tw64[256][2];        // e^{-2 pi i q / 250}, float64
  float4 wt[3][128];          // w^j, w^{j+1} (j = 1, 3, 5) of bin lane, lane-major (one ds_read_b128 per wave)
  PvClip c[kPvClips];
};

// the s of register r on lane b (b = lane & 7) is r ^ pv_g(b): with partners
// b ^ 1, b ^ 2, b ^ 7 (DPP quad_perm / row_half_mirror) each reduce-scatter step
// pairs equal s (pv_g(1) = 1, pv_g(2) = 2, pv_g(7) = 4), and lane b ends with s = pv_g(b)
__device__ __forceinline__ int pv_g(int b) { return (b & 3) ^ ((b & 4) ? 7 : 0); }

template <int kCtrl>
__device__ __forceinline__ float pv_dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), kCtrl, 0xF, 0xF, true));
}

// reduce-scatter of (x, y) across lane ^ 16 (kSwap16) or lane ^ 32: lanes with
// that bit clear get x + x', the others y + y'. (inline asm: the compiler's
// builtin for the swap returns one register for both results in this
// toolchain; s_nop covers the VALU-write -> permlane hazard)
template <bool kSwap16>
__device__ __forceinline__ float pv_swap_add(float x, float y) {
  if (kSwap16)
    asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1\n\ts_nop 1" : "+v"(x), "+v"(y));
  else
    asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1\n\ts_nop 1" : "+v"(x), "+v"(y));
  return x + y;
}

// Complex products as two packed instructions with the operand swaps and the sign in the
// VOP3P op_sel / neg modifiers (the compiler materialises a negated or swapped pair with
// extra moves): a b = (a.x b.x - a.y b.y, a.x b.y + a.y b.x) and a conj(b)
__device__ __forceinline__ cf pv_cmul(cf a, cf b) {
  cf t, r;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1]" : "=v"(t) : "v"(a), "v"(b));  // (a.x b.x, a.x b.y)
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1] neg_lo:[0,1,0]" : "=v"(r) : "v"(a), "v"(b), "v"(t));
  return r;
}
__device__ __forceinline__ cf pv_cmul_conj(cf a, cf b) {
  cf t, r;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel_hi:[0,1] neg_hi:[0,1]" : "=v"(t) : "v"(a), "v"(b));  // (a.x b.x, -a.x b.y)
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[1,0,1]" : "=v"(r) : "v"(a), "v"(b), "v"(t));
  return r;
}

typedef float pv_v4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const pv_v4 pv_lds_v4;  // an LDS float4 (32-bit address)
__device__ __forceinline__ float4 pv_f4(pv_v4 v) { return float4{v.x, v.y, v.z, v.w}; }

// sum_{j = 1..6} d_j w^j of a slide (d_j in da.yzw, db.xyz; w^j pairs in w12, w34, w56): one packed
// product and five packed FMAs, each d_j broadcast by op_sel (no register copies)
__device__ __forceinline__ cf pv_inc(float4 da, float4 db, float4 w12, float4 w34, float4 w56) {
  const cf dxy = {da.x, da.y}, dzw = {da.z, da.w}, exy = {db.x, db.y}, ez = {db.z, db.w};
  const cf w1 = {w12.x, w12.y}, w2 = {w12.z, w12.w}, w3 = {w34.x, w34.y}, w4 = {w34.z, w34.w};
  const cf w5 = {w56.x, w56.y}, w6 = {w56.z, w56.w};
  cf acc;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1]" : "=v"(acc) : "v"(dxy), "v"(w1));
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,0,0] op_sel_hi:[0,1,1]" : "+v"(acc) : "v"(dzw), "v"(w2));
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,0,0] op_sel_hi:[1,1,1]" : "+v"(acc) : "v"(dzw), "v"(w3));
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,0,0] op_sel_hi:[0,1,1]" : "+v"(acc) : "v"(exy), "v"(w4));
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[1,0,0] op_sel_hi:[1,1,1]" : "+v"(acc) : "v"(exy), "v"(w5));
  asm("v_pk_fma_f32 %0, %1, %2, %0 op_sel:[0,0,0] op_sel_hi:[0,1,1]" : "+v"(acc) : "v"(ez), "v"(w6));
  return acc;
}

// padded sample p of clip row xr (reflect padding by n_fft / 2)
__device__ __forceinline__ float ps_xp(const float* xr, int L, int p) {
  int i = p - kPsPad;
  i = i < 0 ? -i : i;
  i = i >= L ? 2 * (L - 1) - i : i;
  return xr[i];
}

// rows [fb, fb + kPvRows) of every clip of the workgroup (frames >= f_in: zero rows)
__device__ __forceinline__ void pv_load_rows(const PitchArgs& a, PvShared& sh, const float* xr, int cl, int lane,
                                             int fb) {
  for (int q = lane; q < 2 * kPvRows; q += 128) {
    const int row = q >> 1, h = q & 1, f = fb + row;
    float* dr = sh.c[cl].d[row];
    if (f >= a.f_in) {
      for (int j = 4 * h; j < 4 * h + 4; ++j) dr[j] = 0.f;
      continue;
    }
    if (h == 0) {
      for (int j = 0; j < 4; ++j) dr[j] = ps_xp(xr, a.L, 7 * f + 243 + j) - ps_xp(xr, a.L, 7 * f - 7 + j);
    } else {
      int delta = 0;
      for (int j = 0; j < 7; ++j) {
        const float vin = ps_xp(xr, a.L, 7 * f + 243 + j), vout = ps_xp(xr, a.L, 7 * f - 7 + j);
        delta += (vin != 0.f) - (vout != 0.f);
        if (j >= 4) dr[j] = vin - vout;
      }
      dr[7] = __builtin_bit_cast(float, delta);  // the count change as int bits (read by SALU)
    }
  }
}

#ifdef HBK_PHASE_TIMING
// profiling build: wave 0 of each block sums the s_memtime cycles of the
// vocoder's phases locally, adds them to g_aug_phase[16 + i] at the end
#define HBK_PVT(i)                                     \
  do {                                                 \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime(); \
    pvt[i] += t_ - pvt_t0;                             \
    pvt_t0 = t_;                                       \
  } while (0)
#else
#define HBK_PVT(i) \
  do {             \
  } while (0)
#endif

#ifndef HBK_PV_UNROLL_TAIL
#define HBK_PV_UNROLL_TAIL 1  // 0: the non-FULL groups' frames in a loop (A/B)
#endif
#ifndef HBK_PV_WAVES
#define HBK_PV_WAVES 4  // waves per SIMD the vocoder is register-limited to
#endif
__global__ void __launch_bounds__(128 * kPvClips) __attribute__((amdgpu_waves_per_eu(HBK_PV_WAVES)))
ps_vocoder_kernel(PitchArgs a) {
#ifdef HBK_PHASE_TIMING
  unsigned long long pvt[5] = {0, 0, 0, 0, 0}, pvt_t0 = __builtin_amdgcn_s_memtime();
#endif
  extern __shared__ __attribute__((aligned(16))) unsigned char pv_smem[];
  PvShared& sh = *reinterpret_cast<PvShared*>(pv_smem);
  const int tid = threadIdx.x, cl = tid >> 7, lane = tid & 127;
  const int e = min(static_cast<int>(blockIdx.x) * kPvClips + cl, a.n - 1);  // padding slots repeat the last clip
  const bool live = static_cast<int>(blockIdx.x) * kPvClips + cl < a.n;
  const float* xr = a.x + static_cast<int64_t>(a.idx[e]) * a.x_stride;
  PvClip& C = sh.c[cl];
  // tables
  for (int q = tid; q < 256; q += blockDim.x) {
    double sn, cs;
    sincospi(2.0 * q / kPsFft, &sn, &cs);
    sh.tw[q] = cf{static_cast<float>(cs), static_cast<float>(sn)};
    sh.tw64[q][0] = cs;
    sh.tw64[q][1] = -sn;
  }
  if (lane == 0) C.cnt0 = 0;
  __syncthreads();
  int nz = 0;
  for (int q = lane; q < kPsFft; q += 128) {
    const float v = ps_xp(xr, a.L, q);
    C.xs[q] = v;
    nz += v != 0.f;
  }
  if (nz) atomicAdd(&C.cnt0, nz);
  for (int q = tid; q < 3 * 128; q += blockDim.x) {
    const int j = 2 * (q / 128) + 1, kk = min(q % 128, kPsBins - 1), q1 = (kk * j) % kPsFft,
              q2 = (kk * (j + 1)) % kPsFft;
    sh.wt[q / 128][q % 128] = float4{static_cast<float>(sh.tw64[q1][0]), static_cast<float>(sh.tw64[q1][1]),
                                     static_cast<float>(sh.tw64[q2][0]), static_cast<float>(sh.tw64[q2][1])};
  }
  int fb = 1;
  pv_load_rows(a, sh, xr, cl, lane, fb);
  __syncthreads();

  const int k = min(lane, kPsBins - 1);
  // per-bin constants: w^-7 in float64 (w^j, j < 7, read from sh.wt per slide), the synthesis weight
  const int q7 = (7 * k) % kPsFft;
  const pv_t rr = static_cast<pv_t>(sh.tw64[q7][0]), ri = static_cast<pv_t>(-sh.tw64[q7][1]);
  const float ck = lane < kPsBins ? ((lane == 0 || lane == kPsBins - 1) ? 1.f : 2.f) : 0.f;
  // synthesis weights c_k e^{2 pi i k s / 250} of the lane's registers (s = r ^ pv_g(lane & 7); s = 7: 0)
  const int gb = pv_g(lane & 7), w = lane >> 6, ou = (lane >> 3) & 7;
  cf esr[4], esi[4];  // (re, im) of registers 2j, 2j + 1 as pairs (packed products)
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const int sr = r ^ gb;
    const cf ev = sr < kPsHop ? ck * sh.tw[(k * sr) % kPsFft] : cf{0.f, 0.f};
    esr[r >> 1][r & 1] = ev.x;
    esi[r >> 1][r & 1] = -ev.y;
  }
  const bool b3 = lane & 8;
  // direct DFT (float64) of the frame staged in C.xs: frame 0, and every
  // kPvRestart frames a restart of the sliding DFT (its float32 increments'
  // rounding then accumulates over at most kPvRestart frames)
  auto direct = [&](double& re, double& im) {
    re = im = 0.0;
    int q = 0;
    for (int n = 0; n < kPsFft; ++n) {
      const double v = static_cast<double>(C.xs[n]);
      re = fma(v, sh.tw64[q][0], re);
      im = fma(v, sh.tw64[q][1], im);
      q += k;
      q -= q >= kPsFft ? kPsFft : 0;
    }
  };
  pv_t xre, xim;
  {
    double dre, dim;
    direct(dre, dim);
    xre = static_cast<pv_t>(dre);
    xim = static_cast<pv_t>(dim);
  }
  int cnt = __builtin_amdgcn_readfirstlane(C.cnt0);
  if (cnt == 0) xre = xim = pv_t(0);
  int sf = 0;  // last slid frame
  int anchor = 0;  // frame of the last direct DFT
  static_assert(sizeof(sh.wt[0]) == 128 * sizeof(float4), "wt rows of 128 lanes");
  uint32_t wt_addr = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((const pv_lds_v4*)&sh.wt[0][lane]));
  // the sliding DFT's next frame (sf + 1) from the current state, as a candidate
  // (xre, xim, cnt are committed by the caller): two partial sums per component
  // keep the float64 dependency chain short
  // drow: frame sf + 1's d row (C.d[sf + 1 - fb]; a FULL group passes its rows at constant offsets)
  auto slide_to = [&](pv_t& nre, pv_t& nim, int& ncnt, const float* drow) {
    const int f = sf + 1;
    if (f >= a.f_in) {
      nre = nim = pv_t(0);
      ncnt = cnt;
      return;
    }
    // the increment sum_j d_j w^j in float32 (packed; d_j rounded once to float32): its
    // rounding enters the float64 state as a random walk far below the state's level
    // the (loop-invariant) table reads stay in the loop, out of VGPRs: the lane's LDS address is
    // made opaque in place (no copy, no address arithmetic per frame: ds_read_b128 wt_addr offset:..)
    asm volatile("" : "+v"(wt_addr));
    const pv_lds_v4* wtp = (const pv_lds_v4*)static_cast<uintptr_t>(wt_addr);
    const float4 w12 = pv_f4(wtp[0]), w34 = pv_f4(wtp[128]), w56 = pv_f4(wtp[256]);
    const float4* drv = reinterpret_cast<const float4*>(drow);
    const float4 da = drv[0], db = drv[1];
    cf acc = pv_inc(da, db, w12, w34, w56);
    acc.x += da.x;  // w^0 = 1
    ncnt = cnt + __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, db.w));  // a clip's count: wave-uniform
    const pv_t ar = xre + static_cast<pv_t>(acc.x), ai = xim + static_cast<pv_t>(acc.y);
    nre = ar * rr - ai * ri;
    nim = ar * ri + ai * rr;
    if (ncnt == 0) nre = nim = pv_t(0);
  };
  auto commit = [&](pv_t nre, pv_t nim, int ncnt) {
    xre = nre;
    xim = nim;
    cnt = ncnt;
    ++sf;
  };
  // unit vector and magnitude of a frame's bin (X = 0: u = 1, |X| = 0)
  auto polar_of = [&](pv_t re, pv_t im, cf& u, float& mag) {
    const float fr = static_cast<float>(re), fi = static_cast<float>(im);
    const float n2 = fmaf(fr, fr, fi * fi);
    // no selects: for X = 0, rs = rsq(2^-126) = 2^63 and (0 + 2^-63, 0) rs = (1, 0), n2 rs = 0; elsewhere
    // (|X| > 2^-38) both offsets are below half an ulp, so rs and u are those of X itself
    const float rs = __builtin_amdgcn_rsqf(n2 + 0x1p-126f);  // v_rsq_f32 (1 ulp)
    u = cf{fr + 0x1p-63f, fi} * rs;
    mag = n2 * rs;
  };
  auto polar = [&](cf& u, float& mag) { polar_of(xre, xim, u, mag); };
  // frames c, c + 1 in (ca, cm), (na, nm); frame c + 2 = sf ahead in (pa, pm)
  cf ca, na, pa;
  float cm, nm, pm;
  polar(ca, cm);
  {
    pv_t nre, nim;
    int ncnt;
    slide_to(nre, nim, ncnt, C.d[sf + 1 - fb]);
    commit(nre, nim, ncnt);
    polar(na, nm);
    slide_to(nre, nim, ncnt, C.d[sf + 1 - fb]);
    commit(nre, nim, ncnt);
    polar(pa, pm);
  }
  int c = 0;
  // The accumulated phase at frame t is e^{i phi_t} = P_t e^{-2 pi i qz_t / 250} with
  // P_t = R u_c (P_0 = u_0: R = 1); R changes only when the source frame repeats or
  // double-steps (the float32 products' rounding is a random walk; |R| is reset to 1
  // once per group), and t * 7k / 250 mod 1 = qz_t / 250 comes from the integer
  // counter qz exactly.
  cf R = {1.f, 0.f};
  cf Q = {0.f, 0.f};
  int qz = 0;
  const int dq = q7;
  // the istft rotation tw[qz] advances by e7 = tw[7k mod 250] per frame: rotated in registers
  // (tz and i tz), re-read from the table once per group (no drift, no scattered LDS read per frame)
  const cf e7 = sh.tw[q7];
  const int jmax = (a.l1 + kPsPad - 1) / kPsHop;  // the frame of the last istft sample
  float* y = a.y + static_cast<int64_t>(e) * a.l1;
  HBK_PVT(0);  // init: tables, frame 0, the first rows

  for (int t0 = 0; t0 <= jmax; t0 += kPvGroup) {
    // the group's source frames (and one ahead) must be resident: refill the d rows
    {
      float al;
      const int tl = min(t0 + kPvGroup - 1, a.f_out - 1);
      const int need = t0 < a.f_out ? min(ps_i0(a, tl, al) + 3, a.f_in - 1) : 0;
      if (need >= fb + kPvRows) {  // uniform across the workgroup
        __syncthreads();
        fb = sf + 1;
        pv_load_rows(a, sh, xr, cl, lane, fb);
        __syncthreads();
      }
    }
    if (sf - anchor >= kPvRestart && sf < a.f_in) {  // uniform across the workgroup
      __syncthreads();
      for (int q = lane; q < kPsFft; q += 128) C.xs[q] = ps_xp(xr, a.L, kPsHop * sf + q);
      __syncthreads();
      double dre, dim;
      direct(dre, dim);
      xre = static_cast<pv_t>(dre);
      xim = static_cast<pv_t>(dim);
      if (cnt == 0) xre = xim = pv_t(0);
      anchor = sf;
    }
    HBK_PVT(1);  // row refills, restarts
    R *= __builtin_amdgcn_rsqf(fmaf(R.x, R.x, R.y * R.y));
    cf tz = sh.tw[qz];  // tw[qz]; i tw[qz] = (-y, x) is read through the packed ops' neg / op_sel modifiers
    const float* dg = C.d[0] + 8 * (sf + 1 - fb);  // FULL groups: frame u slides to row sf + 1 + u
    float gr[kPvGroup];  // frame u: G(t0 + u, pv_g(lane & 7)) over the lane's octet
    float al_lane = 0.f;  // the source frame i0 and alpha of frame t0 + (lane & 7), read by frame u as lane u
    int i0_lane = 0;
    // one output frame; FULL: t < f_out and i0(t) = c + 1 are known for the whole group
    auto frame = [&](int u, auto full) {
      constexpr bool FULL = decltype(full)::value;
      const int t = t0 + u;
#if HBK_PV_ABLATE & 2  // profiling build: the per-bin vocoder replaced by a stand-in
      if (t < a.f_out) {
        float al;
        ps_i0(a, t, al);
        Q.x += al * tz.x;
      }
      if (false) {
#else
      if (FULL || t < a.f_out) {
#endif
        float al;
        int i0;
        if (FULL) {  // i0 = c + 1; the group's alphas were computed once, lane u -> frame u
          i0 = c + 1;
          al = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, al_lane), u));
        } else {
          i0 = __builtin_amdgcn_readlane(i0_lane, u);
          al = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, al_lane), u));
        }
        if (!FULL && i0 > c + 1) {  // rate > 1: a second source frame this step (rare)
          ++c;
          ca = na;
          cm = nm;
          na = pa;
          nm = pm;
          R = cmul(R, cmul_conj(ca, na));  // P_t = P_{t-1} u_{c+1} conj u_c = R u_{c+1}, and c + 2 becomes the frame
          pv_t nre, nim;
          int ncnt;
          slide_to(nre, nim, ncnt, C.d[sf + 1 - fb]);
          commit(nre, nim, ncnt);
          polar(pa, pm);
        }
        // the common step (i0 = c + 1): in a FULL group every frame steps (the source
        // frames rename through the unrolled frames: no selects), elsewhere selects
        const bool step = FULL || i0 > c;
        if (!FULL && !step && t > 0) R = cmul(R, cmul_conj(na, ca));  // the source frame repeats (uniform)
        c += step ? 1 : 0;
        ca = step ? na : ca;
        cm = step ? nm : cm;
        na = step ? pa : na;
        nm = step ? pm : nm;
        pv_t nre, nim;
        int ncnt;
        // candidate frame sf + 1 and its polar form, kept only when stepping (FULL: frame u
        // slides to the group's first row + u)
        slide_to(nre, nim, ncnt, FULL ? dg + 8 * u : C.d[sf + 1 - fb]);
        cf qa;
        float qm;
        polar_of(nre, nim, qa, qm);
        const float m = fmaf(al, nm - cm, cm);
        const cf P = pv_cmul(R, ca);
        // Z_t = m P e^{-2 pi i qz / 250} = m (P.x (x, -y) + P.y (y, x))
        const cf Z = pv_cmul_conj(P, tz);
        Q = __builtin_elementwise_fma(cf{m, m}, Z, Q);
        xre = step ? nre : xre;
        xim = step ? nim : xim;
        cnt = step ? ncnt : cnt;
        sf += step ? 1 : 0;
        pa = step ? qa : pa;
        pm = step ? qm : pm;
      }
      // G(t, .) over the wave's bins: 7 products, reduce-scatter over the lane octet,
      // all-reduce over the 8 octets
      const cf vq = pv_cmul(Q, tz);  // Q tw[qz]
#if HBK_PV_ABLATE & 1  // profiling build: no bin reduction
      gr[u] = vq.x * esr[u & 3].x;
#else
      cf pr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) pr[j] = __builtin_elementwise_fma(cf{vq.x, vq.x}, esr[j], cf{vq.y, vq.y} * esi[j]);
      const float q0 = pr[0].x + pv_dpp<0xB1>(pr[0].y), q1 = pr[1].x + pv_dpp<0xB1>(pr[1].y);  // lane ^ 1
      const float q2 = pr[2].x + pv_dpp<0xB1>(pr[2].y), q3 = pr[3].x + pv_dpp<0xB1>(pr[3].y);
      const float h0 = q0 + pv_dpp<0x4E>(q1), h1 = q2 + pv_dpp<0x4E>(q3);                     // lane ^ 2
      const float gv = h0 + pv_dpp<0x141>(h1);                                                 // lane ^ 7
      if (FULL) {
        gr[u] = gv;  // u is a constant of the unrolled group
      } else {
#pragma unroll
        for (int j = 0; j < kPvGroup; ++j) gr[j] = j == u ? gv : gr[j];
      }
#endif
      tz = pv_cmul(tz, e7);
    };
    bool full = t0 + kPvGroup <= a.f_out;
    if (full) {  // per-frame advances are all >= 1 (rate > 1) or all <= 1 (rate < 1): a total of
      float al;  // kPvGroup means every frame of the group steps exactly once
      full = ps_i0(a, t0 + kPvGroup - 1, al) - c == kPvGroup;
    }
    i0_lane = ps_i0(a, t0 + (lane & 7), al_lane);
    if (full) {
#pragma unroll
      for (int u = 0; u < kPvGroup; ++u) frame(u, std::true_type{});
    } else {  // tail, repeat or double-step group (about a fifth of the groups at 125/128, 128/125)
#if HBK_PV_UNROLL_TAIL  // unrolled too: the frame's result lands in gr[u] without a select chain
#pragma unroll
#else
#pragma unroll 1
#endif
      for (int u = 0; u < kPvGroup; ++u) frame(u, std::false_type{});
    }
    qz = (qz + kPvGroup * dq) % kPsFft;  // the next group's first frame
    // reduce-scatter over the octets: octet o keeps frame o (lane ^ 8, ^ 16, ^ 32)
    float h[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float keep = b3 ? gr[2 * i + 1] : gr[2 * i], send = b3 ? gr[2 * i] : gr[2 * i + 1];
      h[i] = keep + pv_dpp<0x128>(send);  // frame 2i + b3
    }
    const float h02 = pv_swap_add<true>(h[0], h[1]), h13 = pv_swap_add<true>(h[2], h[3]);
    const float gsum = pv_swap_add<false>(h02, h13);
    HBK_PVT(2);  // the group's frames
    // rows t0 .. t0 + 7 of the ring; the previous group's istft step read other rows
    if (gb < kPsHop) C.gh[w][(t0 + ou) % kPvGh][gb] = gsum;
    __syncthreads();
    HBK_PVT(3);  // G rows to LDS + barrier wait
    // the group's istft samples p = 7 t + r
    if (lane < kPsHop * kPvGroup && live) {
      const int t = t0 + lane / kPsHop, r = lane % kPsHop;
      const int m = kPsHop * t + r - kPsPad;
      if (t <= jmax && m >= 0 && m < a.l1) {
        const float g1 = C.gh[0][t % kPvGh][r] + C.gh[1][t % kPvGh][r];
        float g2 = 0.f;
        if (r <= 4) {
          if (t >= 36) g2 = C.gh[0][(t - 36) % kPvGh][r + 2] + C.gh[1][(t - 36) % kPvGh][r + 2];
        } else if (t >= 35) {
          g2 = C.gh[0][(t - 35) % kPvGh][r - 5] + C.gh[1][(t - 35) % kPvGh][r - 5];
        }
        const int lo = max(0, t - 35 + (r >= 5 ? 1 : 0)), hi = min(a.f_out - 1, t);
        // / (250 env) as a product with v_rcp_f32 (1 ulp; the IEEE division's scale / fixup
        // sequence is ~10 VALU per sample)
        y[m] = (g1 - g2) * __builtin_amdgcn_rcpf(static_cast<float>(kPsFft) * static_cast<float>(hi - lo + 1));
      }
    }
    HBK_PVT(4);  // istft samples
  }
#ifdef HBK_PHASE_TIMING
  if (tid == 0)
    for (int i = 0; i < 5; ++i) atomicAdd(&g_aug_phase[16 + i], pvt[i]);
#endif
}

__global__ void ps_taps_kernel(PitchArgs a) {
  // torchaudio _get_sinc_resample_kernel: sinc_interp_hann, width 6, rolloff 0.99
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= a.nw * kPsTapMax) return;
  const int ph = i / kPsTapMax, q = i % kPsTapMax;
  float v = 0.f;
  if (q < 2 * a.width + a.orig) {
    const double lpw = 6.0, base = min(a.orig, a.nw) * 0.99;
    double t = static_cast<double>(static_cast<float>(-ph) / static_cast<float>(a.nw)) +
               static_cast<double>(q - a.width) / a.orig;
    t = fmin(fmax(t * base, -lpw), lpw);
    const double c = cos(t * M_PI / lpw / 2);
    t *= M_PI;
    v = static_cast<float>((t == 0.0 ? 1.0 : sin(t) / t) * c * c * (base / a.orig));
  }
  a.taps[i] = v;
}

__global__ void __launch_bounds__(128) ps_resample_kernel(PitchArgs a) {
  // frames in pairs (f, f + 1): ys2[p] interleaves their windows, (f q, f+1 q, f q+1, f+1 q+1) per
  // float4, so one packed FMA per tap serves both frames (the taps of a phase are the same)
  static_assert(kPsTapMax % 2 == 0 && kPsResFrames % 2 == 0, "resampler pairs");
  constexpr int kPairs = kPsResFrames / 2;
  __shared__ __attribute__((aligned(16))) float ys2[kPairs][2 * kPsTapMax];
  const int ph = threadIdx.x, e = blockIdx.y;
  const int f0 = blockIdx.x * kPsResFrames;
  const float* y = a.y + static_cast<int64_t>(e) * a.l1;
  // y padded by (width, width + orig) zeros; frame f reads ypad[f orig + q]
  // (the window is read to kPsTapMax, past 2 width + orig, against zero taps)
  const int j0 = f0 * a.orig - a.width;
  for (int el = ph; el < kPsResFrames * kPsTapMax; el += 128) {
    const int fr = el / kPsTapMax, q = el - fr * kPsTapMax;  // q fastest: coalesced reads
    const int src = j0 + fr * a.orig + q;
    ys2[fr >> 1][2 * q + (fr & 1)] = (src >= 0 && src < a.l1) ? y[src] : 0.f;
  }
  float tp[kPsTapMax];
  const float* tr = a.taps + min(ph, a.nw - 1) * kPsTapMax;
#pragma unroll
  for (int q = 0; q < kPsTapMax; ++q) tp[q] = tr[q];
  __syncthreads();
  if (ph >= a.nw) return;
  float* out = a.out + static_cast<int64_t>(a.idx[e]) * a.out_stride;
  for (int p = 0; p < kPairs; ++p) {
    const int i = (f0 + 2 * p) * a.nw + ph, i1 = i + a.nw;
    if (i >= a.L) break;
    cf v = {0.f, 0.f};
    if (i < a.target) {
      const float4* w = reinterpret_cast<const float4*>(ys2[p]);
#pragma unroll
      for (int q2 = 0; q2 < kPsTapMax / 2; ++q2) {
        const float4 ww = w[q2];
        v = __builtin_elementwise_fma(cf{tp[2 * q2], tp[2 * q2]}, cf{ww.x, ww.y}, v);
        v = __builtin_elementwise_fma(cf{tp[2 * q2 + 1], tp[2 * q2 + 1]}, cf{ww.z, ww.w}, v);
      }
    }
    out[i] = v.x;
    if (i1 < a.L) out[i1] = i1 < a.target ? v.y : 0.f;
  }
}


// The resampler as a GEMM on the matrix cores: out[f nw + ph] = sum_q taps[ph][q]
// ypad[f orig - width + q] is [frames x 160] x [160 x nw] per clip (K = the taps,
// zero-padded from kPsTapMax to 5 blocks of 32). v_mfma_f32_16x16x32_f16 in split
// f16 (hi*hi + hi*lo + lo*hi, f32 accumulation: ~2^-22 relative per product, as
// the f32 FMAs it replaces). A workgroup takes 64 frames of one clip: their
// windows are staged once into LDS as f16 hi / lo planes (one row per frame, the
// overlapping samples duplicated so every A fragment is one aligned 16-B read)
// after a power-of-two scale that puts the block's largest |sample| in
// [2^14, 2^15); the taps (x 2^10) are each wave's B fragments in VGPRs, two
// 16-phase tiles per wave.
constexpr int kRsFrames = 64, kRsK = 160, kRsLd = kRsK + 8;  // 336-B rows (odd 16-B count)
static_assert(kPsTapMax <= kRsK && kPsPhaseMax <= 128, "the MFMA resampler's K padding and 8 phase tiles");
typedef _Float16 rs_h8 __attribute__((ext_vector_type(8)));
typedef float rs_f4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void rs_split(float v, _Float16& h, _Float16& l) {
  h = static_cast<_Float16>(v);
  l = static_cast<_Float16>(v - static_cast<float>(h));
}
__global__ void __launch_bounds__(256) ps_resample_mfma_kernel(PitchArgs a) {
  __shared__ __attribute__((aligned(16))) _Float16 wh[kRsFrames][kRsLd];
  __shared__ __attribute__((aligned(16))) _Float16 wl[kRsFrames][kRsLd];
  __shared__ float red[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int e = blockIdx.y, f0 = blockIdx.x * kRsFrames;
  const float* y = a.y + static_cast<int64_t>(e) * a.l1;
  // staging: pair p = tid + 256 u of (frame p / 80, taps 2 (p % 80) and + 1)
  constexpr int kPairs = kRsFrames * kRsK / 2, kPer = kPairs / 256;
  float v0[kPer], v1[kPer];
  float mx = 0.f;
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int p = tid + 256 * u, fr = p / (kRsK / 2), q = 2 * (p - fr * (kRsK / 2));
    const int src = (f0 + fr) * a.orig - a.width + q;
    const int s0 = min(max(src, 0), a.l1 - 1), s1 = min(max(src + 1, 0), a.l1 - 1);
    const float x0 = y[s0], x1 = y[s1];
    v0[u] = (src >= 0 && src < a.l1 && q < kPsTapMax) ? x0 : 0.f;
    v1[u] = (src + 1 >= 0 && src + 1 < a.l1 && q + 1 < kPsTapMax) ? x1 : 0.f;
    mx = fmaxf(mx, fmaxf(fabsf(v0[u]), fabsf(v1[u])));
  }
  // B fragments: phases 16 (2 wave + t) + (lane & 15), taps 32 ks + 8 (lane >> 4) ..
  const int n = lane & 15, kq = lane >> 4;
  rs_h8 bh[2][5], bl[2][5];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    const int ph = min(16 * (2 * wave + t) + n, a.nw - 1);
    const float* tr = a.taps + ph * kPsTapMax;
#pragma unroll
    for (int ks = 0; ks < 5; ++ks)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int q = 32 * ks + 8 * kq + j;
        const float tv = tr[min(q, kPsTapMax - 1)];
        _Float16 h, l;
        rs_split(q < kPsTapMax ? tv * 1024.f : 0.f, h, l);
        bh[t][ks][j] = h;
        bl[t][ks][j] = l;
      }
  }
  for (int o = 32; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  if (lane == 0) red[wave] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  const int ex = mx > 0.f ? min(14 - ilogbf(mx), 100) : 0;
  const float scale = ldexpf(1.f, ex), unscale = ldexpf(1.f, -ex - 10);
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int p = tid + 256 * u, fr = p / (kRsK / 2), q = 2 * (p - fr * (kRsK / 2));
    _Float16 h0, l0, h1, l1;
    rs_split(v0[u] * scale, h0, l0);
    rs_split(v1[u] * scale, h1, l1);
    wh[fr][q] = h0;
    wh[fr][q + 1] = h1;
    wl[fr][q] = l0;
    wl[fr][q + 1] = l1;
  }
  __syncthreads();
  float* out = a.out + static_cast<int64_t>(a.idx[e]) * a.out_stride;
#pragma unroll
  for (int ft = 0; ft < kRsFrames / 16; ++ft) {
    rs_f4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int ks = 0; ks < 5; ++ks) {
      const rs_h8 ah = *reinterpret_cast<const rs_h8*>(&wh[16 * ft + n][32 * ks + 8 * kq]);
      const rs_h8 al = *reinterpret_cast<const rs_h8*>(&wl[16 * ft + n][32 * ks + 8 * kq]);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh[t][ks], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl[t][ks], acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh[t][ks], acc[t], 0, 0, 0);
      }
    }
    // lane (n, kq) holds frames 16 ft + 4 kq + j of phase 16 (2 wave + t) + n
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int ph = 16 * (2 * wave + t) + n;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int i = (f0 + 16 * ft + 4 * kq + j) * a.nw + ph;
        if (ph < a.nw && i < a.L) out[i] = i < a.target ? acc[t][j] * unscale : 0.f;
      }
    }
  }
}

}  // namespace
}  // namespace hbk

struct hbk_reverb_plan {
  float2* thi = nullptr;
  float2* tlo = nullptr;
  float2* twn = nullptr;
  float2* thi8 = nullptr;  // colored noise: W_8000^(100 h), W_8000^l, W_16000^k (k <= 4000)
  float2* tlo8 = nullptr;
  float2* twn16 = nullptr;
};

namespace {
constexpr size_t kAugLds = (size_t(2 * hbk::kM + 32) * sizeof(float)) + (hbk::kTwHi + hbk::kTwLo) * sizeof(float2);
constexpr size_t kBandStopLds = kAugLds + (5 * hbk::kBsCirc + 1) * sizeof(float);  // + taps g[0..h], the edges
constexpr size_t kColoredLds = (size_t(2 * hbk::kM1 + 32) * sizeof(float)) + (hbk::kTw8Hi + hbk::kTw8Lo) * sizeof(float2);
}

extern "C" {

int hbk_reverb_plan_create(int64_t T, hbk_reverb_plan** plan) {
  using namespace hbk;
  if (!plan) return arg_error("plan is NULL");
  *plan = nullptr;
  if (T != kT) {
    set_error("hbk: reverb supports clips of %d samples (1.44 s @ 16 kHz), got %lld", kT, (long long)T);
    return HBK_ERR_UNSUPPORTED;
  }
  std::vector<float2> th(kTwHi), tl(kTwLo), tn(kHSlots, make_float2(0.f, 0.f));
  for (int i = 0; i < kTwHi; ++i) {
    const double a = -2.0 * M_PI * (double(i) * kTwLo) / double(kM);
    th[i] = make_float2(float(cos(a)), float(sin(a)));
  }
  for (int i = 0; i < kTwLo; ++i) {
    const double a = -2.0 * M_PI * i / double(kM);
    tl[i] = make_float2(float(cos(a)), float(sin(a)));
  }
  for (int i = 0; i <= kM; ++i) {  // W_N^k at the spectrum slot of bin k
    const double a = -2.0 * M_PI * i / double(kT);
    tn[(i % 16) * kHRow + i / 16] = make_float2(float(cos(a)), float(sin(a)));
  }
  std::vector<float2> th8(kTw8Hi), tl8(kTw8Lo), tn16(kM1 / 2 + 1);
  for (int i = 0; i < kTw8Hi; ++i) {
    const double a = -2.0 * M_PI * (double(i) * kTw8Lo) / double(kM1);
    th8[i] = make_float2(float(cos(a)), float(sin(a)));
  }
  for (int i = 0; i < kTw8Lo; ++i) {
    const double a = -2.0 * M_PI * i / double(kM1);
    tl8[i] = make_float2(float(cos(a)), float(sin(a)));
  }
  for (int i = 0; i <= kM1 / 2; ++i) {
    const double a = -2.0 * M_PI * i / double(kN1);
    tn16[i] = make_float2(float(cos(a)), float(sin(a)));
  }
  auto* p = new hbk_reverb_plan();
  hipError_t e;
  if ((e = hipMalloc(&p->thi, kTwHi * sizeof(float2))) != hipSuccess ||
      (e = hipMalloc(&p->tlo, kTwLo * sizeof(float2))) != hipSuccess ||
      (e = hipMalloc(&p->twn, kHSlots * sizeof(float2))) != hipSuccess ||
      (e = hipMemcpy(p->thi, th.data(), kTwHi * sizeof(float2), hipMemcpyHostToDevice)) != hipSuccess ||
      (e = hipMemcpy(p->tlo, tl.data(), kTwLo * sizeof(float2), hipMemcpyHostToDevice)) != hipSuccess ||
      (e = hipMemcpy(p->twn, tn.data(), kHSlots * sizeof(float2), hipMemcpyHostToDevice)) != hipSuccess ||
      (e = hipMalloc(&p->thi8, kTw8Hi * sizeof(float2))) != hipSuccess ||
      (e = hipMalloc(&p->tlo8, kTw8Lo * sizeof(float2))) != hipSuccess ||
      (e = hipMalloc(&p->twn16, tn16.size() * sizeof(float2))) != hipSuccess ||
      (e = hipMemcpy(p->thi8, th8.data(), kTw8Hi * sizeof(float2), hipMemcpyHostToDevice)) != hipSuccess ||
      (e = hipMemcpy(p->tlo8, tl8.data(), kTw8Lo * sizeof(float2), hipMemcpyHostToDevice)) != hipSuccess ||
      (e = hipMemcpy(p->twn16, tn16.data(), tn16.size() * sizeof(float2), hipMemcpyHostToDevice)) != hipSuccess) {
    hbk_reverb_plan_destroy(p);
    return hip_error(e, "reverb plan tables");
  }
  const size_t lds = kAugLds;
  if ((e = hipFuncSetAttribute(reinterpret_cast<const void*>(augment_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, int(lds))) != hipSuccess ||
      (e = hipFuncSetAttribute(reinterpret_cast<const void*>(spectrum_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, int(lds))) != hipSuccess ||
      (e = hipFuncSetAttribute(reinterpret_cast<const void*>(band_stop_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, int(kBandStopLds))) != hipSuccess ||
      (e = hipFuncSetAttribute(reinterpret_cast<const void*>(band_stop_spectrum_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, int(lds))) != hipSuccess ||
      (e = hipFuncSetAttribute(reinterpret_cast<const void*>(colored_noise_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, int(kColoredLds))) != hipSuccess ||
      (e = hipFuncSetAttribute(reinterpret_cast<const void*>(colored_group_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, int(kColoredLds))) != hipSuccess) {
    hbk_reverb_plan_destroy(p);
    return hip_error(e, "hipFuncSetAttribute(augment LDS)");
  }
  *plan = p;
  return HBK_OK;
}

int hbk_reverb_plan_destroy(hbk_reverb_plan* p) {
  if (!p) return HBK_OK;
  (void)hipFree(p->thi);
  (void)hipFree(p->tlo);
  (void)hipFree(p->twn);
  (void)hipFree(p->thi8);
  (void)hipFree(p->tlo8);
  (void)hipFree(p->twn16);
  delete p;
  return HBK_OK;
}

int hbk_reverb_spectrum(const hbk_reverb_plan* p, const float* kernels, int64_t n_kernels, int64_t stride,
                        float* spectra, void* stream) {
  using namespace hbk;
  if (!p) return arg_error("plan is NULL");
  if (n_kernels < 0) return arg_error("negative n_kernels");
  if (n_kernels == 0) return HBK_OK;
  if (!kernels || !spectra) return arg_error("NULL pointer");
  if (stride < kT) return arg_error("kernel stride < 23040");
  hipLaunchKernelGGL(spectrum_kernel, dim3(unsigned(n_kernels)), dim3(kThreads), kAugLds, as_stream(stream),
                     kernels, stride, reinterpret_cast<float2*>(spectra), p->thi, p->tlo, p->twn);
  HBK_LAUNCH_CHECK("spectrum_kernel");
  return HBK_OK;
}

static int augment_args(const hbk_reverb_plan* p, const float* x, int64_t n_clips, int64_t x_stride,
                        const float* noise_ring, int64_t ring_len, const int64_t* noise_off, const float* snr_db,
                        const float* spectra, const int32_t* spec_idx, const float* gain, float* out,
                        int64_t out_stride, hbk::AugArgs& a) {
  using namespace hbk;
  if (!p) return arg_error("plan is NULL");
  if (n_clips < 0) return arg_error("negative n_clips");
  if (!x || !out || !noise_off || !snr_db || !spec_idx) return arg_error("NULL pointer");
  if (x_stride < kT || out_stride < kT) return arg_error("stride < 23040");
  if (!noise_ring && ring_len > 0) return arg_error("noise ring is NULL");
  if (ring_len >= (int64_t(1) << 30)) return arg_error("noise ring longer than 2^30 samples");
  a = AugArgs{};
  a.x = x;
  a.x_stride = x_stride;
  a.out = out;
  a.out_stride = out_stride;
  a.n_clips = n_clips;
  a.ring = noise_ring;
  a.ring_len = ring_len;
  a.noise_off = noise_off;
  a.snr_db = snr_db;
  a.spectra = reinterpret_cast<const float2*>(spectra);
  a.spec_idx = spec_idx;
  a.gain = gain;
  a.thi = p->thi;
  a.tlo = p->tlo;
  a.twn = p->twn;
  return HBK_OK;
}

static void augment_launch(const hbk::AugArgs& a, void* stream) {
  using namespace hbk;
  const int64_t blocks = std::min<int64_t>(a.n_clips, persistent_blocks(1, stream));
  hipLaunchKernelGGL(augment_kernel, dim3(unsigned(blocks)), dim3(kThreads), kAugLds, as_stream(stream), a);
}

int hbk_augment(const hbk_reverb_plan* p, const float* x, int64_t n_clips, int64_t x_stride,
                const float* noise_ring, int64_t ring_len, const int64_t* noise_off, const float* snr_db,
                const float* spectra, const int32_t* spec_idx, const float* gain, float* out,
                int64_t out_stride, void* stream) {
  using namespace hbk;
  if (n_clips == 0 && p) return HBK_OK;
  AugArgs a;
  const int st = augment_args(p, x, n_clips, x_stride, noise_ring, ring_len, noise_off, snr_db, spectra, spec_idx,
                              gain, out, out_stride, a);
  if (st != HBK_OK) return st;
  augment_launch(a, stream);
  HBK_LAUNCH_CHECK("augment_kernel");
  return HBK_OK;
}

static int64_t colored_groups(int64_t n_clips, int64_t clips_per_noise) {
  return clips_per_noise > 1 && n_clips > 0 ? (n_clips + clips_per_noise - 1) / clips_per_noise : 0;
}

int64_t hbk_colored_noise_workspace_size(int64_t n_clips, int64_t clips_per_noise) {
  const int64_t g = colored_groups(n_clips, clips_per_noise);
  return g ? g * hbk::kN1 * int64_t(sizeof(float)) + ((g * int64_t(sizeof(float)) + 255) & ~int64_t(255)) : 0;
}

int hbk_colored_noise(const hbk_reverb_plan* p, const float* x, int64_t n_clips, int64_t x_stride,
                      const float* white, int64_t white_stride, uint64_t seed, int64_t clips_per_noise,
                      const float* f_decay, const float* snr_db, float sample_rate, const int32_t* idx,
                      int64_t n_entries, float* out, int64_t out_stride, void* stream) {
  return hbk_colored_noise_ws(p, x, n_clips, x_stride, white, white_stride, seed, clips_per_noise, f_decay, snr_db,
                              sample_rate, idx, n_entries, out, out_stride, nullptr, 0, stream);
}

static int colored_args(const hbk_reverb_plan* p, const float* x, int64_t n_clips, int64_t x_stride,
                        const float* white, int64_t white_stride, uint64_t seed, int64_t clips_per_noise,
                        const float* f_decay, const float* snr_db, float sample_rate, const int32_t* idx,
                        int64_t n_entries, float* out, int64_t out_stride, void* workspace, int64_t workspace_bytes,
                        hbk::ColoredArgs& a) {
  using namespace hbk;
  if (!p) return arg_error("plan is NULL");
  if (n_clips < 0) return arg_error("negative n_clips");
  if (!x || !out || !f_decay || !snr_db) return arg_error("NULL pointer");
  if (x_stride < kT || out_stride < kT) return arg_error("stride < 23040");
  if (white && white_stride < kN1) return arg_error("white_stride < 16000");
  if (clips_per_noise < 1) return arg_error("clips_per_noise < 1");
  if (idx && n_entries < 0) return arg_error("negative n_entries");
  if (sample_rate != float(kN1)) {
    set_error("hbk: colored noise is generated at 16 kHz (one second = 16000 samples), got %g", double(sample_rate));
    return HBK_ERR_UNSUPPORTED;
  }
  a = ColoredArgs{};
  a.x = x;
  a.x_stride = x_stride;
  a.out = out;
  a.out_stride = out_stride;
  a.n_clips = n_clips;
  a.white = white;
  a.white_stride = white_stride;
  a.seed = seed;
  a.group = clips_per_noise;
  a.f_decay = f_decay;
  a.snr_db = snr_db;
  a.lin_step = static_cast<float>((std::sqrt(double(kN1) / 2.0) - 1.0) / double(kM1));
  a.idx = idx;
  a.n_entries = idx ? n_entries : n_clips;
  a.thi = p->thi8;
  a.tlo = p->tlo8;
  a.twn = p->twn16;
  a.gbuf = a.grms = nullptr;
  a.n_groups = 0;
  a.no_copy = 0;
  const int64_t need = hbk_colored_noise_workspace_size(n_clips, clips_per_noise);
  if (workspace && need > 0) {
    if (workspace_bytes < need) return arg_error("workspace too small (hbk_colored_noise_workspace_size)");
    a.n_groups = colored_groups(n_clips, clips_per_noise);
    a.gbuf = static_cast<float*>(workspace);
    a.grms = a.gbuf + a.n_groups * kN1;
  }
  return HBK_OK;
}

static void colored_group_launch(const hbk::ColoredArgs& a, void* stream) {
  using namespace hbk;
  const int64_t gblocks = std::min<int64_t>(a.n_groups, persistent_blocks(1, stream));
  hipLaunchKernelGGL(colored_group_kernel, dim3(unsigned(gblocks)), dim3(kThreads), kColoredLds, as_stream(stream), a);
}

static void colored_clip_launch(const hbk::ColoredArgs& a, void* stream) {
  using namespace hbk;
  const int64_t blocks = std::min<int64_t>(a.n_entries, persistent_blocks(1, stream));
  hipLaunchKernelGGL(colored_noise_kernel, dim3(unsigned(blocks)), dim3(kThreads), kColoredLds, as_stream(stream), a);
}

int hbk_colored_noise_ws(const hbk_reverb_plan* p, const float* x, int64_t n_clips, int64_t x_stride,
                         const float* white, int64_t white_stride, uint64_t seed, int64_t clips_per_noise,
                         const float* f_decay, const float* snr_db, float sample_rate, const int32_t* idx,
                         int64_t n_entries, float* out, int64_t out_stride, void* workspace, int64_t workspace_bytes,
                         void* stream) {
  using namespace hbk;
  if (n_clips == 0 && p) return HBK_OK;
  ColoredArgs a;
  const int st = colored_args(p, x, n_clips, x_stride, white, white_stride, seed, clips_per_noise, f_decay, snr_db,
                              sample_rate, idx, n_entries, out, out_stride, workspace, workspace_bytes, a);
  if (st != HBK_OK) return st;
  if (a.n_entries <= 0) return HBK_OK;
  if (a.grms) {
    colored_group_launch(a, stream);
    HBK_LAUNCH_CHECK("colored_group_kernel");
    const int64_t mblocks = std::min<int64_t>(a.n_entries, persistent_blocks(2, stream));
    hipLaunchKernelGGL(colored_mix_kernel, dim3(unsigned(mblocks)), dim3(kThreads), 0, as_stream(stream), a);
    HBK_LAUNCH_CHECK("colored_mix_kernel");
  }
  colored_clip_launch(a, stream);
  HBK_LAUNCH_CHECK("colored_noise_kernel");
  return HBK_OK;
}

int hbk_augment_colored(const hbk_reverb_plan* p, const float* x, int64_t n_clips, int64_t x_stride,
                        const float* noise_ring, int64_t ring_len, const int64_t* noise_off, const float* snr_db,
                        const float* spectra, const int32_t* spec_idx, const float* gain, const float* white,
                        int64_t white_stride, uint64_t seed, int64_t clips_per_noise, const float* c_f_decay,
                        const float* c_snr_db, float sample_rate, const int32_t* c_idx, int64_t c_n_entries,
                        float* out, int64_t out_stride, void* workspace, int64_t workspace_bytes, void* stream) {
  using namespace hbk;
  if (n_clips == 0 && p) return HBK_OK;
  AugArgs a;
  int st = augment_args(p, x, n_clips, x_stride, noise_ring, ring_len, noise_off, snr_db, spectra, spec_idx, gain,
                        out, out_stride, a);
  if (st != HBK_OK) return st;
  ColoredArgs c;
  st = colored_args(p, x, n_clips, x_stride, white, white_stride, seed, clips_per_noise, c_f_decay, c_snr_db,
                    sample_rate, c_idx, c_n_entries, out, out_stride, workspace, workspace_bytes, c);
  if (st != HBK_OK) return st;
  if (out != x && out + n_clips * out_stride > x && x + n_clips * x_stride > out)
    return arg_error("out overlaps x without being x");
  c.no_copy = 1;
  if (c.grms) {
    colored_group_launch(c, stream);
    HBK_LAUNCH_CHECK("colored_group_kernel");
  }
  if (c.n_entries > 0) {  // the clips the group path does not cover, coloured into out
    colored_clip_launch(c, stream);
    HBK_LAUNCH_CHECK("colored_noise_kernel");
  }
  a.c_snr = c_snr_db;
  a.c_fd = c_f_decay;
  a.c_group = clips_per_noise;
  a.c_gbuf = c.gbuf;
  a.c_grms = c.grms;
  augment_launch(a, stream);
  HBK_LAUNCH_CHECK("augment_kernel");
  return HBK_OK;
}

int64_t hbk_band_stop_workspace_size(int64_t n, int32_t n_filters, int32_t n_spectra, void* stream) {
  using namespace hbk;
  if (n <= 0) return 0;
  const int64_t blocks = std::min<int64_t>(n, persistent_blocks(1, stream));
  int64_t b = ((int64_t(n_filters) * 8 + 255) & ~int64_t(255));                          // sums
  b += ((int64_t(n_filters) * (kBsCirc + 1) * 4 + 255) & ~int64_t(255));                 // taps
  b += int64_t(n_spectra) * kHSlots * 8;                                                  // spectra
  b += blocks * kT * 4;                                                                   // clips
  return b;
}

int hbk_band_stop(const hbk_reverb_plan* p, const float* x, int64_t x_stride, int64_t n, const int32_t* idx,
                  const int32_t* filt, int32_t n_filters, const float* f_lo, const float* f_hi,
                  const int32_t* f_half, const int32_t* f_spec0, int32_t n_spectra, const int32_t* s_filt,
                  const int32_t* s_part, float* out, int64_t out_stride, void* workspace, int64_t workspace_bytes,
                  void* stream) {
  using namespace hbk;
  if (!p) return arg_error("plan is NULL");
  if (n < 0 || n_filters < 0 || n_spectra < 0) return arg_error("negative count");
  if (n == 0) return HBK_OK;
  if (n_filters == 0 || n_spectra < n_filters) return arg_error("every filter needs at least one spectrum");
  if (!x || !idx || !filt || !f_lo || !f_hi || !f_half || !f_spec0 || !s_filt || !s_part || !out || !workspace)
    return arg_error("NULL pointer");
  if (x_stride < kT || out_stride < kT) return arg_error("stride < 23040");
  if (workspace_bytes < hbk_band_stop_workspace_size(n, n_filters, n_spectra, stream))
    return arg_error("workspace too small (hbk_band_stop_workspace_size)");
  const int64_t blocks = std::min<int64_t>(n, persistent_blocks(1, stream));
  BandStopArgs a;
  a.x = x;
  a.x_stride = x_stride;
  a.out = out;
  a.out_stride = out_stride;
  a.n = n;
  a.idx = idx;
  a.filt = filt;
  a.n_filters = n_filters;
  a.f_lo = f_lo;
  a.f_hi = f_hi;
  a.f_half = f_half;
  a.f_spec0 = f_spec0;
  a.n_spectra = n_spectra;
  a.s_filt = s_filt;
  a.s_part = s_part;
  unsigned char* w = static_cast<unsigned char*>(workspace);
  a.sums = reinterpret_cast<float2*>(w);
  w += (int64_t(n_filters) * 8 + 255) & ~int64_t(255);
  a.taps = reinterpret_cast<float*>(w);
  w += (int64_t(n_filters) * (kBsCirc + 1) * 4 + 255) & ~int64_t(255);
  a.spectra = reinterpret_cast<float2*>(w);
  w += int64_t(n_spectra) * kHSlots * 8;
  a.scratch = reinterpret_cast<float*>(w);
  a.thi = p->thi;
  a.tlo = p->tlo;
  a.twn = p->twn;
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(band_stop_sums_kernel, dim3(unsigned(n_filters)), dim3(kThreads), 0, st, a);
  HBK_LAUNCH_CHECK("band_stop_sums_kernel");
  hipLaunchKernelGGL(band_stop_spectrum_kernel, dim3(unsigned(n_spectra)), dim3(kThreads), kAugLds, st, a);
  HBK_LAUNCH_CHECK("band_stop_spectrum_kernel");
  hipLaunchKernelGGL(band_stop_kernel, dim3(unsigned(blocks)), dim3(kThreads), kBandStopLds, st, a);
  HBK_LAUNCH_CHECK("band_stop_kernel");
  return HBK_OK;
}

int hbk_place_clips(const float* src, int64_t n_clips, int64_t src_stride, const int32_t* src_len,
                    const int32_t* pre, float* out, int64_t out_stride, int64_t T, void* stream) {
  using namespace hbk;
  if (n_clips < 0) return arg_error("negative n_clips");
  if (n_clips == 0) return HBK_OK;
  if (!src || !src_len || !pre || !out) return arg_error("NULL pointer");
  if (T <= 0 || T % 4 || T > (int64_t(1) << 30)) return arg_error("T must be a positive multiple of 4");
  if (out_stride < T || out_stride % 4 || (reinterpret_cast<uintptr_t>(out) & 15))
    return arg_error("out rows must be 16-B aligned with stride >= T");
  const int64_t items = n_clips * ((T + kPlaceSpan - 1) / kPlaceSpan);
  if (items >= (int64_t(1) << 31)) return arg_error("too many clips for one launch");
  const int64_t blocks = items;
  hipLaunchKernelGGL(place_kernel, dim3(unsigned(blocks)), dim3(256), 0, as_stream(stream), src, src_stride, src_len,
                     pre, out, out_stride, n_clips, int(T));
  HBK_LAUNCH_CHECK("place_kernel");
  return HBK_OK;
}

int hbk_tanh_distortion(const float* x, int64_t n_clips, int64_t x_stride, const float* amount,
                        const int32_t* idx, int64_t n_entries, float* out, int64_t out_stride, void* stream) {
  using namespace hbk;
  if (n_clips < 0) return arg_error("negative n_clips");
  if (n_clips == 0) return HBK_OK;
  if (!x || !out || !amount) return arg_error("NULL pointer");
  if (x_stride < kT || out_stride < kT) return arg_error("stride < 23040");
  TanhArgs a;
  a.x = x;
  a.x_stride = x_stride;
  a.out = out;
  a.out_stride = out_stride;
  a.n_clips = n_clips;
  a.amount = amount;
  a.idx = idx;
  a.n_entries = idx ? n_entries : n_clips;
  if (a.n_entries <= 0) return n_entries < 0 ? arg_error("negative n_entries") : HBK_OK;
  const int64_t blocks = std::min<int64_t>(a.n_entries, persistent_blocks(2, stream));
  hipLaunchKernelGGL(tanh_distortion_kernel, dim3(unsigned(blocks)), dim3(kThreads), 0, as_stream(stream), a);
  HBK_LAUNCH_CHECK("tanh_distortion_kernel");
  return HBK_OK;
}

int hbk_seven_band_eq(const float* x, int64_t n_clips, int64_t x_stride, const double* coef, const int32_t* idx,
                      int64_t n_entries, float* out, int64_t out_stride, void* stream) {
  using namespace hbk;
  if (n_clips < 0 || n_entries < 0) return arg_error("negative count");
  if (!idx) n_entries = n_clips;
  if (n_entries == 0) return HBK_OK;
  if (!x || !out || !coef) return arg_error("NULL pointer");
  if (x_stride < kT || out_stride < kT) return arg_error("stride < 23040");
  if ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(out)) % 16 || x_stride % 4 || out_stride % 4)
    return arg_error("x / out rows must be 16-B aligned");
  EqArgs a;
  a.x = x;
  a.x_stride = x_stride;
  a.coef = coef;
  a.idx = idx;
  a.out = out;
  a.out_stride = out_stride;
  a.n = n_entries;
  hipLaunchKernelGGL(eq_kernel, dim3(unsigned((n_entries + kEqClips - 1) / kEqClips)), dim3(64), 0,
                     as_stream(stream), a);
  HBK_LAUNCH_CHECK("eq_kernel");
  return HBK_OK;
}

static int ps_geometry(int64_t L, int32_t sample_rate, int32_t num, int32_t den, hbk::PitchArgs& a) {
  using namespace hbk;
  if (sample_rate != 16000) {
    set_error("hbk: pitch shift supports 16 kHz (n_fft 250, hop 7), got %d", sample_rate);
    return HBK_ERR_UNSUPPORTED;
  }
  if (num <= 0 || den <= 0) return arg_error("shift num / den must be positive");
  if (L <= kPsPad || L > (int64_t(1) << 24)) return arg_error("clip length must be in (125, 2^24]");
  a.L = static_cast<int>(L);
  a.rate = double(den) / double(num);
  a.f_in = 1 + a.L / kPsHop;
  a.f_out = static_cast<int>(std::ceil(double(a.f_in) / a.rate));
  a.l1 = kPsHop * (a.f_out - 1);
  const int64_t new_sr = int64_t(sample_rate) * den / num;
  const int64_t g = std::gcd(int64_t(sample_rate), new_sr);
  if (new_sr <= 0 || g <= 0) return arg_error("shift out of range");
  a.orig = static_cast<int>(sample_rate / g);
  a.nw = static_cast<int>(new_sr / g);
  a.width = static_cast<int>(std::ceil(6.0 * a.orig / (std::min(a.orig, a.nw) * 0.99)));
  a.target = static_cast<int>(std::ceil(double(a.nw) * a.l1 / a.orig));
  // a group of kPvGroup output frames reads at most rate * kPvGroup + 2 new source frames
  if (a.nw > kPsPhaseMax || 2 * a.width + a.orig > kPsTapMax || a.l1 <= 0 ||
      a.rate * kPvGroup + 3 > kPvRows) {
    set_error("hbk: pitch shift %d/%d resamples %d -> %d (%d taps): the kernel holds <= %d phases of <= %d taps "
              "(torch_pitch_shift's fast shifts at 16 kHz)", num, den, a.orig, a.nw, 2 * a.width + a.orig,
              kPsPhaseMax, kPsTapMax);
    return HBK_ERR_UNSUPPORTED;
  }
  return HBK_OK;
}

static int64_t ps_bytes(const hbk::PitchArgs& a, int64_t n, int64_t* off) {
  using namespace hbk;
  auto up = [](int64_t b) { return (b + 255) & ~int64_t(255); };
  off[0] = off[1] = off[2] = off[3] = 0;           // y
  off[4] = up(n * a.l1 * 4);                       // taps
  return off[4] + up(int64_t(kPsPhaseMax) * kPsTapMax * 4);
}

int64_t hbk_pitch_shift_workspace_size(int64_t n, int64_t T, int32_t sample_rate, int32_t num, int32_t den) {
  hbk::PitchArgs a{};
  if (n <= 0 || ps_geometry(T, sample_rate, num, den, a) != HBK_OK) return 0;
  int64_t off[5];
  return ps_bytes(a, n, off);
}

int hbk_pitch_shift(const float* x, int64_t x_stride, int64_t n, const int32_t* idx, int64_t T, int32_t sample_rate,
                    int32_t num, int32_t den, float* out, int64_t out_stride, void* workspace,
                    int64_t workspace_bytes, void* stream) {
  using namespace hbk;
  if (n < 0) return arg_error("negative n");
  if (n == 0) return HBK_OK;
  if (n > 65535) return arg_error("n > 65535 per call");
  if (!x || !idx || !out || !workspace) return arg_error("NULL pointer");
  PitchArgs a{};
  const int rc = ps_geometry(T, sample_rate, num, den, a);
  if (rc != HBK_OK) return rc;
  if (x_stride < T || out_stride < T) return arg_error("stride < T");
  int64_t off[5];
  if (workspace_bytes < ps_bytes(a, n, off)) return arg_error("workspace too small (hbk_pitch_shift_workspace_size)");
  unsigned char* w = static_cast<unsigned char*>(workspace);
  a.x = x;
  a.x_stride = x_stride;
  a.idx = idx;
  a.out = out;
  a.out_stride = out_stride;
  a.n = static_cast<int>(n);
  a.y = reinterpret_cast<float*>(w + off[3]);
  a.taps = reinterpret_cast<float*>(w + off[4]);
  hipStream_t st = as_stream(stream);
  hipLaunchKernelGGL(ps_taps_kernel, dim3(unsigned((a.nw * kPsTapMax + 255) / 256)), dim3(256), 0, st, a);
  HBK_LAUNCH_CHECK("ps_taps_kernel");
  static bool lds_set = false;  // > 64 KB of dynamic LDS needs the opt-in (per process, idempotent)
  if (!lds_set) {
    HBK_HIP(hipFuncSetAttribute(reinterpret_cast<const void*>(ps_vocoder_kernel),
                                hipFuncAttributeMaxDynamicSharedMemorySize, int(sizeof(PvShared))));
    lds_set = true;
  }
  hipLaunchKernelGGL(ps_vocoder_kernel, dim3(unsigned((n + kPvClips - 1) / kPvClips)), dim3(128 * kPvClips),
                     sizeof(PvShared), st, a);
  HBK_LAUNCH_CHECK("ps_vocoder_kernel");
  const int res_frames = (a.L + a.nw - 1) / a.nw;
  static const bool valu_rs = getenv("HBK_PS_RESAMPLE_VALU") != nullptr;  // the f32 VALU resampler (A/B)
  if (valu_rs || a.nw > 128) {
    hipLaunchKernelGGL(ps_resample_kernel, dim3(unsigned((res_frames + kPsResFrames - 1) / kPsResFrames), unsigned(n)),
                       dim3(128), 0, st, a);
    HBK_LAUNCH_CHECK("ps_resample_kernel");
  } else {
    hipLaunchKernelGGL(ps_resample_mfma_kernel, dim3(unsigned((res_frames + kRsFrames - 1) / kRsFrames), unsigned(n)),
                       dim3(256), 0, st, a);
    HBK_LAUNCH_CHECK("ps_resample_mfma_kernel");
  }
  return HBK_OK;
}

}  // extern "C"

#ifdef HBK_PHASE_TIMING
extern "C" int hbk_debug_aug_phase(unsigned long long* out) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(hbk::g_aug_phase), sizeof(unsigned long long) * 32) != hipSuccess)
    return -2;
  unsigned long long z[32] = {};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(hbk::g_aug_phase), z, sizeof(z));
  return 0;
}
#endif
