// Speech-embedding conv stack for gfx950: fused conv chains on MFMA (f32).
//
// Replaces the speech-embedding ONNX graph run by SpeechEmbeddingModel.__call__
// (embeddings.py:32-42) over the 76-frame windows that
// SpeechEmbeddings.spectrograms_to_embeddings cuts (embeddings.py:86-151).
//
// Execution model
//   * The graph (Keras Conv2D 'valid' stride 1 + LeakyReLU, MaxPool2D) is cut
//     into CHAINS: [optional input pool] conv ... conv [optional output pool].
//     One launch runs a whole chain; its activations live in LDS.
//   * A task = G images x one band of output rows. The band's input rows are
//     staged into LDS once (NHWC, channels padded to an odd count so that the
//     16 rows of an MFMA A-fragment hit 16 different banks), then every conv
//     runs as an implicit GEMM  out[m, n] = sum_k A[m, k] W[k, n]  with
//     m = (image, y, x), k = (dh, dw, ci) gathered from LDS through a per-stage
//     offset table, on v_mfma_f32_16x16x4f32 (exact f32, fmaf-chain numerics).
//   * Clip path: layers before the first pool that breaks the alignment of the
//     window starts run ONCE per clip over the whole 136-frame sequence
//     ("prefix"); windows are then cut from the prefix output (row offsets) for
//     the per-window "tail". The per-window API runs every layer per window.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>
#include <vector>

#include "hbk_common.h"

namespace hbk {
namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kMaxStages = 10;
constexpr int kMaxWin = 32;
constexpr int kLdsBudget = 78 * 1024;     // bytes per block: 2 blocks per CU
constexpr int kLdsBudgetCU = 156 * 1024;  // one block per CU
constexpr int kChunkClips = 16384;     // clips per workspace chunk (default; HBK_EMBED_CHUNK overrides)
// clips per workspace chunk (HBK_EMBED_CHUNK: 256 .. 32,768): every chain kernel runs once per chunk (its last round of waves
// partly filled); measured: 100 k clips in 16,384-clip chunks 24.30 ms, in 32,768-clip chunks
// 24.43 ms, bit-identical (tools/embed_chunk_check.py), so the smaller workspace stays
inline int64_t chunk_clips() {
  static const int64_t c = [] {
    const char* e = getenv("HBK_EMBED_CHUNK");
    const long long v = e ? atoll(e) : 0;
    // (capped at 32,768, the size tools/embed_chunk_check.py validated: the chain kernels'
    // task counts are 32-bit and assume at most that many clips x windows x bands)
    return v >= 256 && v <= 32768 ? int64_t(v) : int64_t(kChunkClips);
  }();
  return c;
}

typedef float f4 __attribute__((ext_vector_type(4)));

struct StageDesc {
  int kh, kw, cin, cinp, cout, coutp;
  int K, ksteps, act;
  float alpha;
  int w_off, b_off;  // floats into the chain's weight blob
};

struct ChainArgs {
  const float* in;
  float* out;
  const float* wblob;
  int64_t n_img;            // images (clips or windows)
  int64_t src_clip_stride;  // floats between source clips
  int src_row_stride;       // floats between source rows
  int ipc;                  // images per source clip
  int row_off[kMaxWin];     // source row offset of image (i % ipc)
  int C_src;
  int in_ph, in_pw;         // input max-pool
  int W_in;                 // chain input width after the input pool
  int out_ph, out_pw;       // output max-pool
  int H_out, W_out, C_out;  // chain output per image
  int64_t out_img_stride;   // floats between output images
  int G;                    // images per task
  int band;                 // output rows per task
  int n_bands;
  int shrink;               // sum over stages of kh - 1
  int n_stages;
  StageDesc st[kMaxStages];
  int wblob_floats;
  int wstride;              // row stride of packed weights
  int lds_x, lds_y, lds_w, lds_k;  // float offsets into dynamic LDS
};

template <int NB, int RB, bool WG>
__device__ __forceinline__ void conv_stage(const float* __restrict__ X, float* __restrict__ Y,
                                           const float* __restrict__ Wst,
                                           const int* __restrict__ ktab,
                                           const float* __restrict__ bias, int G, int hin, int win,
                                           const StageDesc& S, int wstride, int lane, int wave) {
  const int ho = hin - S.kh + 1, wo = win - S.kw + 1;
  const int img_pos = ho * wo, M = G * img_pos;
  const int nrb = (M + 15) >> 4;
  const int r16 = lane & 15, kq = lane >> 4;
  // output channels in groups of NB 16-column blocks (more than NB * 16 channels: several passes)
  const int nblk = (S.cout + 15) >> 4;
  for (int cb = 0; cb < nblk; cb += NB)
  for (int rb0 = wave * RB; rb0 < nrb; rb0 += kWaves * RB) {
    int moff[RB];
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      int m = min((rb0 + r) * 16 + r16, M - 1);
      const int g = m / img_pos;
      const int rem = m - g * img_pos;
      const int y = rem / wo;
      const int x = rem - y * wo;
      moff[r] = ((g * hin + y) * win + x) * S.cinp;
    }
    f4 acc[RB][NB];
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
      for (int c = 0; c < NB; ++c) acc[r][c] = f4{0.f, 0.f, 0.f, 0.f};
    const float* wp = Wst + kq * wstride + cb * 16 + r16;
#pragma unroll 2
    for (int ks = 0; ks < S.ksteps; ++ks) {
      const int koff = ktab[ks * 4 + kq];
      float av[RB], bv[NB];
#pragma unroll
      for (int r = 0; r < RB; ++r) av[r] = X[moff[r] + koff];
#pragma unroll
      for (int c = 0; c < NB; ++c) bv[c] = wp[ks * 4 * wstride + min(c, nblk - 1 - cb) * 16];
#pragma unroll
      for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int c = 0; c < NB; ++c)
          acc[r][c] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[r], bv[c], acc[r][c], 0, 0, 0);
    }
    // C/D layout: row (lane >> 4) * 4 + i, column lane & 15
#pragma unroll
    for (int c = 0; c < NB; ++c) {
      const int n = (cb + c) * 16 + r16;
      if (n >= S.cout) continue;
      const float bb = bias[n];
#pragma unroll
      for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = (rb0 + r) * 16 + kq * 4 + i;
          if (m < M) {
            float v = acc[r][c][i] + bb;
            if (S.act) v = v >= 0.f ? v : v * S.alpha;
            Y[m * S.coutp + n] = v;
          }
        }
    }
  }
  (void)WG;
}

template <int NB, int RB, bool WG>
__global__ void __launch_bounds__(kThreads) conv_chain_kernel(ChainArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* X = smem + a.lds_x;
  float* Y = smem + a.lds_y;
  float* Wl = smem + a.lds_w;
  int* ktab = reinterpret_cast<int*>(smem + a.lds_k);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (!WG)
    for (int i = tid; i < a.wblob_floats; i += kThreads) Wl[i] = a.wblob[i];  // resident weights

  const int64_t n_groups = (a.n_img + a.G - 1) / a.G;
  const int64_t n_tasks = n_groups * a.n_bands;
  const int C = a.C_src;
  const int cinp0 = a.st[0].cinp;
  for (int64_t task = blockIdx.x; task < n_tasks; task += gridDim.x) {
    const int64_t grp = task / a.n_bands;
    const int band = static_cast<int>(task - grp * a.n_bands);
    const int64_t img0 = grp * a.G;
    const int G = static_cast<int>(min<int64_t>(a.G, a.n_img - img0));
    const int orow0 = band * a.band;
    const int orows = min(a.band, a.H_out - orow0);
    const int r0 = orow0 * a.out_ph;           // first chain-input row of the band
    const int rows_in = orows * a.out_ph + a.shrink;

    // 1) stage the band's input rows (max-pooled on the fly) into X
    const int row_elems = a.W_in * C;
    const int per_img = rows_in * row_elems;
    for (int e = tid; e < G * per_img; e += kThreads) {
      const int g = e / per_img;
      int rem = e - g * per_img;
      const int r = rem / row_elems;
      rem -= r * row_elems;
      const int w = rem / C;
      const int c = rem - w * C;
      const int64_t im = img0 + g;
      const int64_t clip = im / a.ipc;
      const int roff = a.row_off[im - clip * a.ipc];
      const float* src = a.in + clip * a.src_clip_stride +
                         static_cast<int64_t>(roff + (r0 + r) * a.in_ph) * a.src_row_stride +
                         (w * a.in_pw) * C + c;
      float v = src[0];
      for (int i = 0; i < a.in_ph; ++i)
        for (int j = 0; j < a.in_pw; ++j) v = nan_max(v, src[i * a.src_row_stride + j * C]);
      X[((g * rows_in + r) * a.W_in + w) * cinp0 + c] = v;
    }

    // 2) the chain's convs, ping-ponging between X and Y
    int hin = rows_in, win = a.W_in;
    float* cur = X;
    float* nxt = Y;
    for (int s = 0; s < a.n_stages; ++s) {
      const StageDesc S = a.st[s];
      __syncthreads();  // stage input complete; previous stage done with ktab
      for (int k = tid; k < S.ksteps * 4; k += kThreads) {
        int v = 0;  // padded k: weight 0, read the (finite) own-position value
        if (k < S.K) {
          const int tap = k / S.cin;
          const int ci = k - tap * S.cin;
          const int dh = tap / S.kw;
          const int dw = tap - dh * S.kw;
          v = (dh * win + dw) * S.cinp + ci;
        }
        ktab[k] = v;
      }
      __syncthreads();
      const float* Wst = WG ? a.wblob + S.w_off : Wl + S.w_off;
      conv_stage<NB, RB, WG>(cur, nxt, Wst, ktab, a.wblob + S.b_off, G, hin, win, S, a.wstride,
                             lane, wave);
      float* t = cur;
      cur = nxt;
      nxt = t;
      hin -= S.kh - 1;
      win -= S.kw - 1;
    }
    __syncthreads();

    // 3) store the band (max-pooled on the fly)
    const int coutp = a.st[a.n_stages - 1].coutp;
    const int orow_elems = a.W_out * a.C_out;
    const int per_out = orows * orow_elems;
    for (int e = tid; e < G * per_out; e += kThreads) {
      const int g = e / per_out;
      int rem = e - g * per_out;
      const int r = rem / orow_elems;
      rem -= r * orow_elems;
      const int w = rem / a.C_out;
      const int c = rem - w * a.C_out;
      const float* p = cur + ((g * hin + r * a.out_ph) * win + w * a.out_pw) * coutp + c;
      float v = p[0];
      for (int i = 0; i < a.out_ph; ++i)
        for (int j = 0; j < a.out_pw; ++j) v = nan_max(v, p[(i * win + j) * coutp]);
      a.out[(img0 + g) * a.out_img_stride + static_cast<int64_t>(orow0 + r) * orow_elems + w * a.C_out + c] = v;
    }
    __syncthreads();  // the next task restages X
  }
}

// ------------------------------------------------- split-f16 conv chain ----
// Same task structure as conv_chain_kernel; the arithmetic is an fp16 pair per
// value, x = hi + lo (hi = x with its 13 low mantissa bits cleared, i.e. x
// rounded toward zero to fp16's 11 bits; lo = fp16(x - hi)), and each GEMM is
//   acc = W_hi X_hi + W_hi X_lo + W_lo X_hi
// on v_mfma_f32_32x32x16_f16 (f32 accumulation): ~2^-22 relative per operand
// (lo loses bits only below fp16's subnormal step, 2^-24 absolute; the
// dropped W_lo X_lo is 2^-22 relative). WEIGHTS are the A
// operand (32 output channels) and 32 output POSITIONS as the B operand, so a
// lane of the accumulator holds 4 consecutive channels of one position: the
// epilogue packs them (v_cvt_pkrtz) and stores 8 B per plane.
// Activations live in LDS as two fp16 planes [pos][cs] (cs = channels rounded
// to 8, with cs / 8 odd so the 16-B fragment reads of 32 consecutive positions
// are conflict-free); a K-group is 8 consecutive channels of one tap, the unit
// of one lane's ds_read_b128. Weights are [n][wrow] fp16 planes (k contiguous
// per output channel). A first stage whose cin is not a multiple of 8 (the
// mel input, cin 1) is expanded im2col-style during staging and runs as a
// 1x1 conv. Staging / store loops use a per-kernel 2-D thread mapping (row x
// unit) so no integer division runs per element.
constexpr int kXThreads = 256;
constexpr int kXWaves = kXThreads / 64;

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef __fp16 h2 __attribute__((ext_vector_type(2)));
typedef float f16x __attribute__((ext_vector_type(16)));

struct XStage {
  int kh, kw, cin, cout;
  int coutr;          // output channels written (cout rounded up to 8; the pad is exactly 0)
  int cs_in, cs_out;  // fp16 elements per position of the input / output tensor
  int ksteps;         // K steps of 16 (two 8-channel groups)
  int nblk;           // 32-wide output-channel blocks
  int act;
  float alpha;
  int w_off;          // fp16 offset of the hi plane [nblk * 32][wrow]
  int w_lo;           // fp16 distance hi -> lo plane
  int wrow;
  int b_off;          // float offset into the bias blob
  int kt_off;         // int offset of the stage's group-offset table
};

struct XArgs {
  const float* in;
  float* out;
  const _Float16* wblob;   // global weights (WG mode reads them here)
  const float* bblob;      // biases [per stage nblk * 32]
  const int* ktab;         // group offsets, all stages
  const int* i2c_off;      // im2col: raw-row offset of tap k = (dh kw + dw) C + ci
  int i2c_n;
  int64_t n_img;
  int64_t src_clip_stride;
  int src_row_stride;
  int ipc;
  int row_off[kMaxWin];
  int C_src, cs0;          // source channels; fp16 stride of the staged tensor
  int im2col;              // stage 0 input is the im2col expansion (K0 = kh kw cin)
  int in_ph, in_pw, W_in;
  int out_ph, out_pw, H_out, W_out, C_out;
  int64_t out_img_stride;
  int vec_out;             // C_out % 4 == 0 and 16-B aligned output: float4 stores
  int raw_vec;             // im2col staging reads float4 (in_pw == 1, aligned rows)
  int G, band, n_bands, shrink, n_stages;
  XStage st[kMaxStages];
  int w_halfs;             // resident weights (0: WG mode)
  int b_floats, kt_n;
  int lds_x, lds_y, lds_w, lds_b, lds_k;  // byte offsets into dynamic LDS
  int dbg_slot;            // phase-timing slot (chain index mod 4; profiling build only)
  int dbg_skip;            // profiling build only: bit 0 stages, 1 im2col, 2 store, 3 staging
  int* range_flag;         // set to 1 when an f16-split value reaches kF16Max
};

#if defined(HBK_PHASE_TIMING) || defined(HBK_ABLATE)
#define HBK_SKIP(bit) (a.dbg_skip & (1 << (bit)))
#else
#define HBK_SKIP(bit) false
#endif
#ifdef HBK_PHASE_TIMING
// Profiling build only (build.py --phase-timing): wave 0 of every block adds
// the s_memtime cycles of each task phase (staging, im2col, stage s, store;
// barrier waits included in the phase before them) into g_phase_cycles.
__device__ unsigned long long g_phase_cycles[64];  // [chain slot (4)][phase (16)]
#define HBK_PHASE(i)                                                          \
  do {                                                                        \
    if (threadIdx.x == 0) {                                                   \
      const unsigned long long t_ = __builtin_amdgcn_s_memtime();             \
      atomicAdd(&g_phase_cycles[a.dbg_slot * 16 + (i)], t_ - phase_t0);      \
      phase_t0 = t_;                                                          \
    }                                                                         \
  } while (0)
#else
#define HBK_PHASE(i) \
  do {               \
  } while (0)
#endif

#ifdef HBK_TRACE
// Tracing build only: lane 0 of waves of the first 4 blocks records
// s_memtime at marks of the first tasks into g_trace[block][wave][event].
__device__ unsigned long long g_trace[4][4][256];
__device__ int g_trace_n[4][4];
#define HBK_MARK(id)                                                                        \
  do {                                                                                      \
    if (blockIdx.x < 4 && (threadIdx.x & 63) == 0) {                                        \
      const int w_ = threadIdx.x >> 6, b_ = blockIdx.x;                                     \
      const int n_ = g_trace_n[b_][w_];                                                     \
      if (n_ < 255) {                                                                       \
        g_trace[b_][w_][n_] = (__builtin_amdgcn_s_memtime() << 8) | static_cast<unsigned>(id); \
        g_trace_n[b_][w_] = n_ + 1;                                                         \
      }                                                                                     \
    }                                                                                       \
  } while (0)
#else
#define HBK_MARK(id) \
  do {               \
  } while (0)
#endif

constexpr int kXStageInts = sizeof(XStage) / 4;
constexpr int kI2cLds = 256;  // im2col tap table entries kept in LDS

// A stage descriptor from the block's LDS copy, as uniform (scalar) values.
__device__ __forceinline__ XStage lds_stage(const int* p) {
  XStage S;
  int* d = reinterpret_cast<int*>(&S);
#pragma unroll
  for (int i = 0; i < kXStageInts; ++i) d[i] = __builtin_amdgcn_readfirstlane(p[i]);
  return S;
}

// q = n / d for 0 <= n < 2^24, d >= 1, from a float reciprocal (one
// correction step covers its rounding); inv = 1.f / d
__device__ __forceinline__ int div_small(int n, int d, float inv) {
  int q = static_cast<int>(static_cast<float>(n) * inv);
  const int r = n - q * d;
  q += (r >= d) ? 1 : 0;
  q -= (r < 0) ? 1 : 0;
  return q;
}

// hi = v rounded toward zero to fp16 (11 significant bits in fp16's normal
// range), lo = (v - hi) rounded to fp16 by v_fma_mix{lo,hi}_f16 (v - hi is
// exact in f32); two values, packed: 3 VALU instructions per pair
// The f16 planes hold |v| < 65504 (kF16Max): amax keeps the largest |v| a
// thread split (one v_max3 per pair; fmaxf drops NaN, which is not a range
// fault) and the kernel raises its plan's range flag when it reaches kF16Max.
constexpr float kF16Max = 65504.f;
// (one v_max3 through asm: fmaxf / fabsf put canonicalising v_max ops in front)
__device__ __forceinline__ void track(float& amax, float a, float b) {
  asm("v_max3_f32 %0, %0, |%1|, |%2|" : "+v"(amax) : "v"(a), "v"(b));
}
__device__ __forceinline__ void raise_range(int* flag, float amax) {
  if (amax >= kF16Max) *flag = 1;  // vector store: any writer, same value
}
// (the generic kernel runs at its VGPR cap: it checks each group of values
// where it splits them instead of carrying amax, guard4)
__device__ __forceinline__ void guard4(int* flag, float a, float b, float c, float d) {
  float m = 0.f;
  track(m, a, b);
  track(m, c, d);
  if (m >= kF16Max) *flag = 1;
}
__device__ __forceinline__ void split2(float a, float b, h2& hi, h2& lo) {
  hi = __builtin_amdgcn_cvt_pkrtz(a, b);
  const uint32_t hb = __builtin_bit_cast(uint32_t, hi);
  uint32_t l;  // mixlo writes bits 15:0, mixhi bits 31:16: no initial value needed
  asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=v"(l) : "v"(a), "v"(hb));
  asm("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(l) : "v"(b), "v"(hb));
  lo = __builtin_bit_cast(h2, l);
}

// max(v, alpha v) through asm: fmaxf on MFMA results gets a canonicalising
// v_max in front of it; both operands are NaN for a NaN v, so NaN propagates
__device__ __forceinline__ float leaky_max(float v, float alpha) {
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(v), "v"(v * alpha));
  return r;
}

__device__ __forceinline__ uint32_t h2_bits(h2 v) { return __builtin_bit_cast(uint32_t, v); }

// 2-D mapping of kXThreads threads onto rows of `units` work items: rpp rows
// per pass; this thread takes unit t_u of row t_row (+ rpp per pass). When a
// row has more units than threads, rpp = 1 and the unit loop strides by
// kXThreads.
struct RowMap {
  int rpp, t_row, t_u, u_step;
  __device__ __forceinline__ RowMap(int units, int tid) {
    if (units <= kXThreads) {
      rpp = kXThreads / units;
      t_row = tid / units;
      t_u = tid - t_row * units;
      u_step = units;  // one unit per row per thread
      if (t_row >= rpp) t_row = 1 << 30;  // idle thread
    } else {
      rpp = 1;
      t_row = 0;
      t_u = tid;
      u_step = kXThreads;
    }
  }
};

// Yf != nullptr: the chain's last stage, written as f32 [m][coutr] for the
// pooled store (no split / reconstruct).
template <int NB, int RB>
__device__ __forceinline__ void xstage(const _Float16* __restrict__ Xh, const _Float16* __restrict__ Xl,
                                       _Float16* __restrict__ Yh, _Float16* __restrict__ Yl,
                                       float* __restrict__ Yf, const _Float16* __restrict__ Wh,
                                       const int* __restrict__ kt, const float* __restrict__ bias, int M,
                                       int hA, int wA, int ho, int wo, const XStage& S, int lane, int wave,
                                       int* flag, int cb) {
  // output channels 32 (cb + c) + ..., c < NB: one group of at most 3 blocks of a wider stage
  const int img_pos = ho * wo;
  const int nrb = (M + 31) >> 5;
  const int r32 = lane & 31, khalf = lane >> 5;
  const int cstride = 32 * S.wrow;
  const _Float16* wp = Wh + cb * cstride + r32 * S.wrow + khalf * 8;
  // input position of output m = (g, y, x): with ytot = g ho + y = m / wo,
  // (g hA + y) wA + x = m + ytot (wA - wo) + g (hA - ho) wA
  const float inv_wo = 1.f / static_cast<float>(wo), inv_ho = 1.f / static_cast<float>(ho);
  const bool one_img = M <= img_pos;
  // this lane's biases, channels n = 32 c + 8 q + 4 khalf + j (register 4 q + j)
  f16x bl[NB];
#pragma unroll
  for (int c = 0; c < NB; ++c)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float4 b = *reinterpret_cast<const float4*>(bias + (cb + c) * 32 + 8 * q + 4 * khalf);
      bl[c][4 * q] = b.x;
      bl[c][4 * q + 1] = b.y;
      bl[c][4 * q + 2] = b.z;
      bl[c][4 * q + 3] = b.w;
    }
  for (int rb0 = wave * RB; rb0 < nrb; rb0 += kXWaves * RB) {
    HBK_MARK(10);
    int xoff[RB];
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const int m = min((rb0 + r) * 32 + r32, M - 1);
      const int ytot = div_small(m, wo, inv_wo);
      const int g = one_img ? 0 : div_small(ytot, ho, inv_ho);
      xoff[r] = (m + ytot * (wA - wo) + g * (hA - ho) * wA) * S.cs_in;
    }
    (void)img_pos;
    f16x acc[RB][NB];
    // software-pipelined K loop over two fragment sets: the LDS reads of step
    // ks + 1 are in flight while the MFMAs of step ks run (the prefetch index
    // is clamped, so the last step re-reads its own fragments harmlessly)
    struct Frag {
      h8 xh[RB], xl[RB], wh[NB], wl[NB];
    };
    auto load = [&](Frag& f, int ks) {
      const int ko = kt[2 * ks + khalf];
#pragma unroll
      for (int r = 0; r < RB; ++r) {
        f.xh[r] = *reinterpret_cast<const h8*>(Xh + xoff[r] + ko);
        f.xl[r] = *reinterpret_cast<const h8*>(Xl + xoff[r] + ko);
      }
#pragma unroll
      for (int c = 0; c < NB; ++c) {
        f.wh[c] = *reinterpret_cast<const h8*>(wp + c * cstride + ks * 16);
        f.wl[c] = *reinterpret_cast<const h8*>(wp + S.w_lo + c * cstride + ks * 16);
      }
    };
    // three products per tile, the tiles interleaved so that consecutive
    // MFMAs never chain on one accumulator
    auto mma = [&](const Frag& f, bool first) {
#pragma unroll
      for (int c = 0; c < NB; ++c) {
#pragma unroll
        for (int r = 0; r < RB; ++r)
          acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.wh[c], f.xh[r], first ? bl[c] : acc[r][c], 0, 0,
                                                              0);
#pragma unroll
        for (int r = 0; r < RB; ++r)
          acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.wh[c], f.xl[r], acc[r][c], 0, 0, 0);
#pragma unroll
        for (int r = 0; r < RB; ++r)
          acc[r][c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.wl[c], f.xh[r], acc[r][c], 0, 0, 0);
      }
    };
    HBK_MARK(11);
    const int last = S.ksteps - 1;
    Frag fa, fb;
    load(fa, 0);
    load(fb, min(1, last));
    mma(fa, true);
    int ks = 1;
    for (; ks < last; ks += 2) {
      load(fa, ks + 1);
      mma(fb, false);
      load(fb, min(ks + 2, last));
      mma(fa, false);
    }
    if (ks == last) mma(fb, false);
#ifdef HBK_TRACE
    // make the mark wait for the accumulators (MFMA completion)
    asm volatile("" ::"v"(acc[0][0][0]));
#endif
    HBK_MARK(12);
    // D[n][m]: this lane holds position m = tile + (lane & 31) and channels
    // n = 32 c + 8 q + 4 (lane >> 5) + j for register i = 4 q + j
    float m4 = 0.f;  // range guard over this epilogue's split values
#pragma unroll
    for (int r = 0; r < RB; ++r) {
      const int m = (rb0 + r) * 32 + r32;
      if (m >= M) continue;
      _Float16* yh = Yh + m * S.cs_out;
      _Float16* yl = Yl + m * S.cs_out;
#pragma unroll
      for (int c = 0; c < NB; ++c)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          // coutr is a multiple of 8, so this test is the same for both lane halves (uniform)
          if ((cb + c) * 32 + 8 * q >= S.coutr) continue;
          const int n0 = (cb + c) * 32 + 8 * q + 4 * khalf;
          // (the bias is the first MFMA's accumulator input)
          float v[4] = {acc[r][c][4 * q], acc[r][c][4 * q + 1], acc[r][c][4 * q + 2], acc[r][c][4 * q + 3]};
          if (S.act == 1) {  // LeakyReLU, 0 <= alpha <= 1: max(v, alpha v) (NaN stays NaN)
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = leaky_max(v[j], S.alpha);
          } else if (S.act == 2) {
#pragma unroll
            for (int j = 0; j < 4; ++j) v[j] = v[j] >= 0.f ? v[j] : v[j] * S.alpha;
          }
          if (Yf) {
            *reinterpret_cast<float4*>(Yf + m * S.coutr + n0) = float4{v[0], v[1], v[2], v[3]};
            continue;
          }
          h2 h01, l01, h23, l23;
          track(m4, v[0], v[1]);
          track(m4, v[2], v[3]);
          split2(v[0], v[1], h01, l01);
          split2(v[2], v[3], h23, l23);
          *reinterpret_cast<uint2*>(yh + n0) = uint2{h2_bits(h01), h2_bits(h23)};
          *reinterpret_cast<uint2*>(yl + n0) = uint2{h2_bits(l01), h2_bits(l23)};
        }
    }
    if (m4 >= kF16Max) *flag = 1;
    HBK_MARK(13);
  }
}

#ifndef HBK_X3_WAVES_PER_EU
#define HBK_X3_WAVES_PER_EU 2
#endif
template <int NBMAX, bool WG>
__global__ void __launch_bounds__(kXThreads) __attribute__((amdgpu_waves_per_eu(HBK_X3_WAVES_PER_EU)))
conv_chain_x3_kernel(XArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char xsmem[];
  unsigned char* Xb = xsmem + a.lds_x;
  unsigned char* Yb = xsmem + a.lds_y;
  _Float16* Wl = reinterpret_cast<_Float16*>(xsmem + a.lds_w);
  float* Bl = reinterpret_cast<float*>(xsmem + a.lds_b);
  int* kt = reinterpret_cast<int*>(xsmem + a.lds_k);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // per-block LDS copies of the stage descriptors and the im2col tap table
  // (read every task; kernel arguments are not re-read in the task loop)
  __shared__ int s_st[kMaxStages * kXStageInts];
  __shared__ int s_i2c[kI2cLds];
  for (int i = tid; i < a.n_stages * kXStageInts; i += kXThreads)
    s_st[i] = reinterpret_cast<const int*>(a.st)[i];
  for (int i = tid; i < kI2cLds; i += kXThreads) s_i2c[i] = a.i2c_off[min(i, a.i2c_n - 1)];
  if (!WG)
    for (int i = tid; i < a.w_halfs / 8; i += kXThreads)
      reinterpret_cast<h8*>(Wl)[i] = reinterpret_cast<const h8*>(a.wblob)[i];
  for (int i = tid; i < a.b_floats; i += kXThreads) Bl[i] = a.bblob[i];
  for (int i = tid; i < a.kt_n; i += kXThreads) kt[i] = a.ktab[i];

  // task indices fit in 32 bits (at most kChunkClips x 32 windows x bands)
  const int n_tasks = static_cast<int>((a.n_img + a.G - 1) / a.G) * a.n_bands;
  const int C = a.C_src;
  const XStage& S0 = a.st[0];
  // per-kernel thread mappings
  //  staging (no im2col): units of 8 channels, W_in * C / 8 per row
  //  staging (im2col):    raw f32, W_in * C per row
  //  im2col expansion:    positions, wo0 per row
  //  store:               units of 4 channels (vec_out) or 1, W_out * C_out / (4|1) per row
  const int st_units = a.im2col ? (a.raw_vec ? a.W_in * C / 4 : a.W_in * C) : a.W_in * (C / 8);
  const int raw_len = a.W_in * C;  // floats per raw row (im2col)
  const RowMap ms(st_units, tid);
  const int st_w = a.im2col ? 0 : ms.t_u / (C / 8);
  const int wo0 = a.W_in - S0.kw + 1;
  const RowMap mi(wo0, tid);
  const int cu = a.vec_out ? 4 : 1;
  const RowMap mo(a.W_out * a.C_out / cu, tid);
  const int o_w = mo.t_u / (a.C_out / cu), o_c = (mo.t_u - o_w * (a.C_out / cu)) * cu;

  struct Geo {
    int64_t img0;
    int G, orow0, orows, r0, rows_in, nrows;
  };
  auto geo = [&](int task) {
    Geo t;
    const int grp = task / a.n_bands;
    const int band = task - grp * a.n_bands;
    t.img0 = static_cast<int64_t>(grp) * a.G;
    t.G = static_cast<int>(min<int64_t>(a.G, a.n_img - t.img0));
    t.orow0 = band * a.band;
    t.orows = min(a.band, a.H_out - t.orow0);
    t.r0 = t.orow0 * a.out_ph;
    t.rows_in = t.orows * a.out_ph + a.shrink;
    t.nrows = t.G * t.rows_in;
    return t;
  };
  // one staging unit of row `row` (image g, band row r), max-pooled on load:
  // im2col: 4 raw floats (raw_vec) or 1; otherwise 8 channels of position w
  auto load_unit = [&](const Geo& t, int row, int u, float4& v0, float4& v1) {
    const int g = row / t.rows_in;
    const int r = row - g * t.rows_in;
    const int64_t im = t.img0 + g;
    const int64_t clip = im / a.ipc;
    const int roff = a.row_off[im - clip * a.ipc];
    const float* srow = a.in + clip * a.src_clip_stride +
                        static_cast<int64_t>(roff + (t.r0 + r) * a.in_ph) * a.src_row_stride;
    if (a.im2col) {
      if (a.raw_vec) {  // in_pw == 1
        const float* src = srow + u * 4;
        v0 = *reinterpret_cast<const float4*>(src);
        for (int i = 1; i < a.in_ph; ++i) {
          const float4 q = *reinterpret_cast<const float4*>(src + i * a.src_row_stride);
          v0 = float4{nan_max(v0.x, q.x), nan_max(v0.y, q.y), nan_max(v0.z, q.z), nan_max(v0.w, q.w)};
        }
      } else {
        const int w = u / C, c = u - w * C;
        const float* src = srow + (w * a.in_pw) * C + c;
        float v = src[0];
        for (int i = 0; i < a.in_ph; ++i)
          for (int j = 0; j < a.in_pw; ++j) v = nan_max(v, src[i * a.src_row_stride + j * C]);
        v0.x = v;
      }
      return;
    }
    const int w = (ms.u_step == st_units) ? st_w : u / (C / 8);
    const int c8 = (u - w * (C / 8)) * 8;
    const float* src = srow + (w * a.in_pw) * C + c8;
    if (a.in_ph <= 2 && a.in_pw <= 2) {
      // window of at most 2 x 2: all four taps are loaded unconditionally (a tap
      // outside the window re-reads tap (0, 0); the max is idempotent), so no
      // load sits in a predicated branch or a runtime loop that would wait on it
      const int di = a.in_ph > 1 ? a.src_row_stride : 0, dj = a.in_pw > 1 ? C : 0;
      const float4 p00 = *reinterpret_cast<const float4*>(src), q00 = *reinterpret_cast<const float4*>(src + 4);
      const float4 p01 = *reinterpret_cast<const float4*>(src + dj);
      const float4 q01 = *reinterpret_cast<const float4*>(src + dj + 4);
      const float4 p10 = *reinterpret_cast<const float4*>(src + di);
      const float4 q10 = *reinterpret_cast<const float4*>(src + di + 4);
      const float4 p11 = *reinterpret_cast<const float4*>(src + di + dj);
      const float4 q11 = *reinterpret_cast<const float4*>(src + di + dj + 4);
      auto mx = [](const float4& x, const float4& y) {
        return float4{nan_max(x.x, y.x), nan_max(x.y, y.y), nan_max(x.z, y.z), nan_max(x.w, y.w)};
      };
      v0 = mx(mx(p00, p01), mx(p10, p11));
      v1 = mx(mx(q00, q01), mx(q10, q11));
      return;
    }
    v0 = *reinterpret_cast<const float4*>(src);
    v1 = *reinterpret_cast<const float4*>(src + 4);
    for (int i = 0; i < a.in_ph; ++i)
      for (int j = 0; j < a.in_pw; ++j) {
        if (i == 0 && j == 0) continue;
        const float* q = src + i * a.src_row_stride + j * C;
        const float4 p0 = *reinterpret_cast<const float4*>(q);
        const float4 p1 = *reinterpret_cast<const float4*>(q + 4);
        v0 = float4{nan_max(v0.x, p0.x), nan_max(v0.y, p0.y), nan_max(v0.z, p0.z), nan_max(v0.w, p0.w)};
        v1 = float4{nan_max(v1.x, p1.x), nan_max(v1.y, p1.y), nan_max(v1.z, p1.z), nan_max(v1.w, p1.w)};
      }
  };
  auto store_unit = [&](const Geo& t, int row, int u, const float4& v0, const float4& v1) {
    if (a.im2col) {
      float* R = reinterpret_cast<float*>(Yb) + row * raw_len;
      if (a.raw_vec)
        *reinterpret_cast<float4*>(R + u * 4) = v0;
      else
        R[u] = v0.x;
      return;
    }
    const int w = (ms.u_step == st_units) ? st_w : u / (C / 8);
    const int c8 = (u - w * (C / 8)) * 8;
    h2 a0, b0, a1, b1, a2, b2, a3, b3;
    guard4(a.range_flag, v0.x, v0.y, v0.z, v0.w);
    guard4(a.range_flag, v1.x, v1.y, v1.z, v1.w);
    split2(v0.x, v0.y, a0, b0);
    split2(v0.z, v0.w, a1, b1);
    split2(v1.x, v1.y, a2, b2);
    split2(v1.z, v1.w, a3, b3);
    _Float16* Sh = reinterpret_cast<_Float16*>(Xb);
    const int idx = (row * a.W_in + w) * a.cs0 + c8;
    *reinterpret_cast<uint4*>(Sh + idx) = uint4{h2_bits(a0), h2_bits(a1), h2_bits(a2), h2_bits(a3)};
    *reinterpret_cast<uint4*>(Sh + t.nrows * a.W_in * a.cs0 + idx) =
        uint4{h2_bits(b0), h2_bits(b1), h2_bits(b2), h2_bits(b3)};
  };
  // The first kPF row passes of a task's staging are loaded into registers
  // one task ahead (their global loads overlap the current task's compute);
  // further passes, or rows wider than the block, load synchronously.
#ifndef HBK_X3_PF
#define HBK_X3_PF (NBMAX == 1 ? 4 : 2)
#endif
  constexpr int kPF = HBK_X3_PF;
  const bool pf_ok = ms.u_step == st_units;
  float4 pv0[kPF], pv1[kPF];
  auto prefetch = [&](const Geo& t) {
#pragma unroll
    for (int p = 0; p < kPF; ++p) {
      // clamped, not predicated: rows past the task re-read its last row (unused)
      const int row = min(ms.t_row + p * ms.rpp, t.nrows - 1);
      load_unit(t, row, ms.t_u, pv0[p], pv1[p]);
    }
  };

  int task = blockIdx.x;
  Geo tg{};
  if (task < n_tasks) {
    tg = geo(task);
    if (pf_ok) prefetch(tg);
  }
  for (; task < n_tasks; task += gridDim.x) {
    const Geo t = tg;
    const int64_t img0 = t.img0;
    const int G = t.G, orow0 = t.orow0, orows = t.orows, rows_in = t.rows_in;

    // 1) stage the band's input rows (max-pooled on the fly)
    __syncthreads();  // previous task's readers of X / Y are done (kt, Wl, Bl on the first task)
#ifdef HBK_PHASE_TIMING
    unsigned long long phase_t0 = __builtin_amdgcn_s_memtime();
#endif
    HBK_MARK(1);
    if (HBK_SKIP(3)) {
    } else if (pf_ok) {
#pragma unroll
      for (int p = 0; p < kPF; ++p) {
        const int row = ms.t_row + p * ms.rpp;
        if (row < t.nrows) store_unit(t, row, ms.t_u, pv0[p], pv1[p]);
      }
      for (int row = ms.t_row + kPF * ms.rpp; row < t.nrows; row += ms.rpp) {
        float4 v0, v1;
        load_unit(t, row, ms.t_u, v0, v1);
        store_unit(t, row, ms.t_u, v0, v1);
      }
    } else {
      for (int row = ms.t_row; row < t.nrows; row += ms.rpp)
        for (int u = ms.t_u; u < st_units; u += ms.u_step) {
          float4 v0, v1;
          load_unit(t, row, u, v0, v1);
          store_unit(t, row, u, v0, v1);
        }
    }
    if (task + static_cast<int>(gridDim.x) < n_tasks) {
      tg = geo(task + gridDim.x);
      if (pf_ok && !HBK_SKIP(3)) prefetch(tg);  // in flight during this task's compute
    }
    int hin = rows_in, win = a.W_in;
    if (a.im2col && !HBK_SKIP(1)) {
      // expand stage 0's taps: position (g, y, x) of its OUTPUT holds k = (dh kw + dw) C + ci
      __syncthreads();
      HBK_PHASE(0);
      const int ho = hin - S0.kh + 1;
      const int K0 = S0.kh * S0.kw * C, K8 = (K0 + 7) & ~7;
      const float* R = reinterpret_cast<const float*>(Yb);
      _Float16* Ih = reinterpret_cast<_Float16*>(Xb);
      _Float16* Il = Ih + G * ho * wo0 * a.cs0;
      for (int prow = mi.t_row; prow < G * ho; prow += mi.rpp)
      for (int x = mi.t_u; x < wo0; x += mi.u_step) {
        const int g = prow / ho, y = prow - g * ho;
        const float* base = R + ((g * rows_in + y) * win + x) * C;
        _Float16* dh_ = Ih + (prow * wo0 + x) * a.cs0;
        _Float16* dl_ = Il + (prow * wo0 + x) * a.cs0;
        for (int k8 = 0; k8 < K8; k8 += 8) {  // one 8-channel group: 16 B per plane
          uint32_t hb[4], lb[4];
          float m = 0.f;
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            const int k = k8 + 2 * p;  // tap offsets: uniform table (scalar loads)
            const int o0 = k < kI2cLds ? s_i2c[k] : a.i2c_off[k];
            const int o1 = k + 1 < kI2cLds ? s_i2c[k + 1] : a.i2c_off[k + 1];
            const float v0 = k < K0 ? base[o0] : 0.f;
            const float v1 = k + 1 < K0 ? base[o1] : 0.f;
            h2 hh, ll;
            track(m, v0, v1);
            split2(v0, v1, hh, ll);
            hb[p] = h2_bits(hh);
            lb[p] = h2_bits(ll);
          }
          if (m >= kF16Max) *a.range_flag = 1;
          *reinterpret_cast<uint4*>(dh_ + k8) = uint4{hb[0], hb[1], hb[2], hb[3]};
          *reinterpret_cast<uint4*>(dl_ + k8) = uint4{lb[0], lb[1], lb[2], lb[3]};
        }
      }
    }

    // 2) the chain's convs, ping-ponging between X and Y
    unsigned char* cur = Xb;
    unsigned char* nxt = Yb;
    for (int s = 0; s < a.n_stages; ++s) {
      const XStage S = lds_stage(s_st + s * kXStageInts);
      const int ho = hin - S.kh + 1, wo = win - S.kw + 1;
      const bool i2c = a.im2col && s == 0;
      const int hA = i2c ? ho : hin, wA = i2c ? wo : win;
      const int M = G * ho * wo;
      HBK_MARK(19);
      __syncthreads();  // stage input complete
      HBK_PHASE(s == 0 ? 1 : 1 + s);
      HBK_MARK(20 + s);
      const _Float16* Xh = reinterpret_cast<const _Float16*>(cur);
      const _Float16* Xl = Xh + G * hA * wA * S.cs_in;
      _Float16* Yh = reinterpret_cast<_Float16*>(nxt);
      _Float16* Yl = Yh + M * S.cs_out;
      const _Float16* Wst = WG ? a.wblob + S.w_off : Wl + S.w_off;
      const int* kts = kt + S.kt_off;
      const float* bs = Bl + S.b_off;
      float* Yf = s + 1 == a.n_stages ? reinterpret_cast<float*>(nxt) : nullptr;
      // RB x NB tiles of one 16-register accumulator each. NBMAX 4 (plans with
      // a stage wider than 96 channels): groups of 3 blocks, each re-reading
      // the stage input (a separate instantiation: the loop costs the others
      // spills)
      if (HBK_SKIP(0)) {
      } else if constexpr (NBMAX > 3) {
        for (int cb = 0; cb < S.nblk; cb += 3) {
          const int nb = min(3, S.nblk - cb);
          if (nb == 3)
            xstage<3, 1>(Xh, Xl, Yh, Yl, Yf, Wst, kts, bs, M, hA, wA, ho, wo, S, lane, wave, a.range_flag, cb);
          else if (nb == 2)
            xstage<2, 2>(Xh, Xl, Yh, Yl, Yf, Wst, kts, bs, M, hA, wA, ho, wo, S, lane, wave, a.range_flag, cb);
          else
            xstage<1, 2>(Xh, Xl, Yh, Yl, Yf, Wst, kts, bs, M, hA, wA, ho, wo, S, lane, wave, a.range_flag, cb);
        }
      } else if (NBMAX >= 3 && S.nblk == 3) {
        xstage<3, 1>(Xh, Xl, Yh, Yl, Yf, Wst, kts, bs, M, hA, wA, ho, wo, S, lane, wave, a.range_flag, 0);
      } else if (NBMAX >= 2 && S.nblk == 2) {
        xstage<2, 2>(Xh, Xl, Yh, Yl, Yf, Wst, kts, bs, M, hA, wA, ho, wo, S, lane, wave, a.range_flag, 0);
      } else {
        xstage<1, 2>(Xh, Xl, Yh, Yl, Yf, Wst, kts, bs, M, hA, wA, ho, wo, S, lane, wave, a.range_flag, 0);
      }
      unsigned char* t = cur;
      cur = nxt;
      nxt = t;
      hin = ho;
      win = wo;
    }
    HBK_MARK(19);
    __syncthreads();
    HBK_PHASE(1 + a.n_stages);
    HBK_MARK(5);

    // 3) store the band (max-pooled on the fly) from the last stage's f32 output
    const int cso = __builtin_amdgcn_readfirstlane(s_st[(a.n_stages - 1) * kXStageInts + 4]);  // coutr
    const float* O = reinterpret_cast<const float*>(cur);
    const int units = a.W_out * a.C_out / cu;
    for (int orow = HBK_SKIP(2) ? (1 << 30) : mo.t_row; orow < G * orows; orow += mo.rpp) {
      const int g = orow / orows, r = orow - g * orows;
      float* drow = a.out + (img0 + g) * a.out_img_stride + static_cast<int64_t>(orow0 + r) * a.W_out * a.C_out;
      for (int u = mo.t_u; u < units; u += mo.u_step) {
        const int w = (mo.u_step == units) ? o_w : u / (a.C_out / cu);
        const int c = (mo.u_step == units) ? o_c : (u - w * (a.C_out / cu)) * cu;
        const int base = ((g * hin + r * a.out_ph) * win + w * a.out_pw) * cso + c;
        if (a.vec_out) {
          float4 v = *reinterpret_cast<const float4*>(O + base);
          for (int i = 0; i < a.out_ph; ++i)
            for (int j = 0; j < a.out_pw; ++j) {
              if (i == 0 && j == 0) continue;
              const float4 t = *reinterpret_cast<const float4*>(O + base + (i * win + j) * cso);
              v = float4{nan_max(v.x, t.x), nan_max(v.y, t.y), nan_max(v.z, t.z), nan_max(v.w, t.w)};
            }
          *reinterpret_cast<float4*>(drow + w * a.C_out + c) = v;
        } else {
          float v = O[base];
          for (int i = 0; i < a.out_ph; ++i)
            for (int j = 0; j < a.out_pw; ++j) v = nan_max(v, O[base + (i * win + j) * cso]);
          drow[w * a.C_out + c] = v;
        }
      }
    }
    HBK_PHASE(2 + a.n_stages);
    HBK_MARK(6);
  }
}

// ------------------------------------------------------------------- p0 ----
// Pattern kernel for the chain  conv 3x3 (1 -> C) . conv 1x3 (C -> C) .
// conv 3x1 (C -> C) . max-pool 2x2  on a fixed input width WI (the SE20
// prefix's first group: 136 x 32 mel rows -> 66 x 14 x 24, ~55 % of the
// embedding MACs). Same split-f16 numerics as conv_chain_x3_kernel (3 fp16
// products per f32-accurate MAC on v_mfma_f32_32x32x16_f16, f32 accumulate),
// but every shape is a compile-time constant, so the position / tap address
// math folds to shifts and immediates (the generic kernel spends ~20 VALU
// instructions per MFMA on runtime index math and SGPR spills):
//   * stage 0 builds its B fragments straight from the f32 input rows in LDS
//     (taps 0-4 in the lane's first K half, 5-8 in the second): no im2col
//     buffer;
//   * every stage's A fragments (weights) and bias are loaded once per block
//     and stay in VGPRs (4-wave blocks, 2 waves / SIMD); the bias is the first
//     MFMA's accumulator input;
//   * the hi/lo split of each output is v_cvt_pkrtz (hi, round toward zero)
//     plus v_fma_mix{lo,hi}_f16 (lo = x - hi rounded to fp16);
//   * one task = one image x BAND pooled rows (4 waves, 32-position tiles
//     round-robin over the waves), 2 blocks / CU.
constexpr int kP0Waves = 4;
constexpr int kP0Threads = 64 * kP0Waves;

struct P0Args {
  const float* in;          // [img][rows][WI] f32, row stride WI
  float* out;               // [img][H_out][W2 / 2][C] f32
  const _Float16* w;        // stage s: hi [32][16 ks_s], lo [32][16 ks_s]
  const float* bias;        // [3][32] (rows >= C are 0)
  int64_t n_img;
  int64_t src_img_stride;   // floats
  int H_in;                 // valid input rows per image
  int H_out;                // pooled output rows per image
  int n_bands;
  float alpha;              // LeakyReLU slope of all three convs (LEAKY kernels)
  int* range_flag;          // set to 1 when an f16-split value reaches kF16Max
};

template <int WI, int C, int BAND>
struct P0Geo {
  static constexpr int W0 = WI - 2, W1 = W0 - 2, W2 = W1;
  static constexpr int R2 = 2 * BAND, R1 = R2 + 2, R0 = R1, RI = R0 + 2;
  static constexpr int CS = ((C / 8) % 2 == 0) ? C + 8 : C;  // odd number of 16-B groups per position
  static constexpr int M0 = R0 * W0, M1 = R1 * W1, M2 = R2 * W2;
  static constexpr int T0 = (M0 + 31) / 32, T1 = (M1 + 31) / 32, T2 = (M2 + 31) / 32;
  static constexpr int KS = (3 * C + 15) / 16;  // K steps of stages 1 and 2
  static constexpr int RAW = RI * WI * 4;
  static constexpr int S0B = M0 * CS * 4, S1B = M1 * CS * 4, S2B = M2 * C * 4;
  static constexpr int XB = ((RAW > S1B ? RAW : S1B) + 15) & ~15;  // raw input, then stage-1 output
  static constexpr int YB = ((S0B > S2B ? S0B : S2B) + 15) & ~15;  // stage-0 output, then stage-2 f32
  static constexpr int LDS = XB + YB;
  static constexpr int WOFF1 = 2 * 32 * 16, WOFF2 = WOFF1 + 2 * 32 * 16 * KS;  // fp16 offsets
  static constexpr int WHALFS = WOFF2 + 2 * 32 * 16 * KS;
};

// hi = v rounded toward zero to fp16, lo = (v - hi) rounded to fp16; two values, packed
__device__ __forceinline__ void split2_mix(float a, float b, uint32_t& hi, uint32_t& lo, float& amax) {
  track(amax, a, b);
  hi = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pkrtz(a, b));
  uint32_t l;  // mixlo writes bits 15:0, mixhi bits 31:16: no initial value needed
  asm("v_fma_mixlo_f16 %0, %1, 1.0, -%2 op_sel_hi:[0,0,1]" : "=v"(l) : "v"(a), "v"(hi));
  asm("v_fma_mixhi_f16 %0, %1, 1.0, -%2 op_sel:[0,0,1] op_sel_hi:[0,0,1]" : "+v"(l) : "v"(b), "v"(hi));
  lo = l;
}

// LEAKY: every conv of the chain is LeakyReLU with 0 <= alpha <= 1 (max(v, alpha v)); else identity
// (v_max_f32 through asm: fmaxf on MFMA results gets a canonicalising v_max in
// front of it; both operands are NaN for a NaN input, so NaN propagates)
template <bool LEAKY>
__device__ __forceinline__ float p0_act(float v, float alpha) {
  if (!LEAKY) return v;
  float r;
  asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(v), "v"(v * alpha));
  return r;
}

// bias of this lane's accumulator rows (channels 8 q + 4 khalf + j, register 4 q + j)
__device__ __forceinline__ f16x p0_bias(const float* b, int khalf) {
  f16x v;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4 t = *reinterpret_cast<const float4*>(b + 8 * q + 4 * khalf);
    v[4 * q] = t.x;
    v[4 * q + 1] = t.y;
    v[4 * q + 2] = t.z;
    v[4 * q + 3] = t.w;
  }
  return v;
}

// activation + split of a finished tile into the hi / lo planes at position p
template <int C, int CS, bool LEAKY>
__device__ __forceinline__ void p0_store_planes(const f16x& acc, int p, int khalf, _Float16* oh, _Float16* ol,
                                                float alpha, float& amax) {
#pragma unroll
  for (int q = 0; q < C / 8; ++q) {
    float v[4];
#pragma unroll
    for (int jj = 0; jj < 4; ++jj) v[jj] = p0_act<LEAKY>(acc[4 * q + jj], alpha);
    uint32_t h01, l01, h23, l23;
    split2_mix(v[0], v[1], h01, l01, amax);
    split2_mix(v[2], v[3], h23, l23, amax);
    const int o = p * CS + 8 * q + 4 * khalf;
    *reinterpret_cast<uint2*>(oh + o) = uint2{h01, h23};
    *reinterpret_cast<uint2*>(ol + o) = uint2{l01, l23};
  }
}

// Stage 1 (1x3, ST = 1: grid R0 x W0 -> R1 x W1, planes out) or stage 2
// (3x1, ST = 2: R1 x W1 -> R2 x W2, f32 out) of a task; K = tap * C + ci.
// A fragments (hi, lo) and bias of stage ST for this lane, loaded ahead of use
template <int KS>
struct P0W {
  h8 ah[KS], al[KS];
  f16x bias;
};
template <int WI, int C, int BAND, int ST>
__device__ __forceinline__ P0W<P0Geo<WI, C, BAND>::KS> p0_load_w(const P0Args& a, int r32, int khalf) {
  using G = P0Geo<WI, C, BAND>;
  P0W<G::KS> w;
  const _Float16* wp = a.w + (ST == 1 ? G::WOFF1 : G::WOFF2) + r32 * (16 * G::KS) + 8 * khalf;
#pragma unroll
  for (int ks = 0; ks < G::KS; ++ks) {
    w.ah[ks] = *reinterpret_cast<const h8*>(wp + 16 * ks);
    w.al[ks] = *reinterpret_cast<const h8*>(wp + 32 * 16 * G::KS + 16 * ks);
  }
  w.bias = p0_bias(a.bias + 32 * ST, khalf);
  return w;
}

template <int WI, int C, int BAND, int ST, bool LEAKY>
__device__ __forceinline__ void p0_stage12(const P0Args& a, const P0W<P0Geo<WI, C, BAND>::KS>& W,
                                           const _Float16* xh_, const _Float16* xl_, _Float16* oh, _Float16* ol,
                                           float* of, int wave, int r32, int khalf, float& amax) {
  using G = P0Geo<WI, C, BAND>;
  constexpr int M = ST == 1 ? G::M1 : G::M2, T = ST == 1 ? G::T1 : G::T2;
  constexpr int Wout = ST == 1 ? G::W1 : G::W2, Win = ST == 1 ? G::W0 : G::W1;
  constexpr int TAPSTRIDE = ST == 1 ? G::CS : G::W1 * G::CS;  // fp16 between taps in the input grid
  const float alpha = a.alpha;
  // Software pipeline over this wave's tiles: the epilogue (activation, split,
  // LDS stores) of tile t - 1 is issued in the same block as tile t's MFMA
  // chain, so its VALU work fills the MFMA issue gaps.
  auto load = [&](int t, int ks, h8& xh, h8& xl) {
    const int p = min(t * 32 + r32, M - 1);
    const int y = p / Wout, x = p - y * Wout;
    // this lane's 8-channel group: K = 16 ks + 8 khalf (groups past 3 C read group 0; weights 0)
    const int ka = 16 * ks < 3 * C ? 16 * ks : 0;
    const int kb = 16 * ks + 8 < 3 * C ? 16 * ks + 8 : 0;
    const int oa = (ka / C) * TAPSTRIDE + ka % C, ob = (kb / C) * TAPSTRIDE + kb % C;
    const int o = (y * Win + x) * G::CS + (khalf ? ob : oa);
    xh = *reinterpret_cast<const h8*>(xh_ + o);
    xl = *reinterpret_cast<const h8*>(xl_ + o);
  };
  auto epilogue = [&](int t, const f16x& acc) {
    const int pp = t * 32 + r32;
    if (pp >= M) return;
    if (ST == 1) {
      p0_store_planes<C, G::CS, LEAKY>(acc, pp, khalf, oh, ol, alpha, amax);
    } else {
#pragma unroll
      for (int q = 0; q < C / 8; ++q) {
        float4 v;
        v.x = p0_act<LEAKY>(acc[4 * q], alpha);
        v.y = p0_act<LEAKY>(acc[4 * q + 1], alpha);
        v.z = p0_act<LEAKY>(acc[4 * q + 2], alpha);
        v.w = p0_act<LEAKY>(acc[4 * q + 3], alpha);
        *reinterpret_cast<float4*>(of + pp * C + 8 * q + 4 * khalf) = v;
      }
    }
  };
  f16x prev;
  int tprev = -1;
  for (int t = wave; t < T; t += kP0Waves) {
    h8 xh[G::KS], xl[G::KS];
#pragma unroll
    for (int ks = 0; ks < G::KS; ++ks) load(t, ks, xh[ks], xl[ks]);
    f16x acc = W.bias;
#pragma unroll
    for (int ks = 0; ks < G::KS; ++ks) {
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(W.ah[ks], xh[ks], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(W.ah[ks], xl[ks], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(W.al[ks], xh[ks], acc, 0, 0, 0);
    }
    if (tprev >= 0) epilogue(tprev, prev);
    prev = acc;
    tprev = t;
  }
  if (tprev >= 0) epilogue(tprev, prev);
}

template <int WI, int C, int BAND, bool LEAKY>
__global__ void __launch_bounds__(kP0Threads) __attribute__((amdgpu_waves_per_eu(2)))
p0_chain_kernel(P0Args a) {
  using G = P0Geo<WI, C, BAND>;
  extern __shared__ __attribute__((aligned(16))) unsigned char p0mem[];
  float* raw = reinterpret_cast<float*>(p0mem);
  _Float16* s1h = reinterpret_cast<_Float16*>(p0mem);
  _Float16* s1l = s1h + G::M1 * G::CS;
  _Float16* s0h = reinterpret_cast<_Float16*>(p0mem + G::XB);
  _Float16* s0l = s0h + G::M0 * G::CS;
  float* s2 = reinterpret_cast<float*>(p0mem + G::XB);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r32 = lane & 31, khalf = lane >> 5;
  const int n_tasks = static_cast<int>(a.n_img) * a.n_bands;

  // the task's input rows (RI x WI floats = RI * WI / 4 float4, one per thread
  // while it fits) are loaded one task ahead into registers
  constexpr int kRawV = G::RI * WI / 4;
  constexpr int kRawPer = (kRawV + kP0Threads - 1) / kP0Threads;
  float4 rawv[kRawPer];
  auto load_raw = [&](int task) {
    const int img = task / a.n_bands, band = task - img * a.n_bands;
    const float* src = a.in + static_cast<int64_t>(img) * a.src_img_stride;
#pragma unroll
    for (int u = 0; u < kRawPer; ++u) {
      const int i = tid + u * kP0Threads;
      if (i < kRawV) {
        const int r = i / (WI / 4), c4 = i - r * (WI / 4);
        const int rr = min(band * G::R2 + r, a.H_in - 1);
        rawv[u] = *reinterpret_cast<const float4*>(src + static_cast<int64_t>(rr) * WI + 4 * c4);
      }
    }
  };
  if (static_cast<int>(blockIdx.x) < n_tasks) load_raw(blockIdx.x);
  // every stage's A fragments and bias stay in VGPRs for the whole kernel
  const _Float16* wp0 = a.w + r32 * 16 + 8 * khalf;
  const h8 a0h = *reinterpret_cast<const h8*>(wp0), a0l = *reinterpret_cast<const h8*>(wp0 + 32 * 16);
  const f16x b0 = p0_bias(a.bias, khalf);
  const auto W1 = p0_load_w<WI, C, BAND, 1>(a, r32, khalf);
  const auto W2 = p0_load_w<WI, C, BAND, 2>(a, r32, khalf);
  float amax = 0.f;

  for (int task = blockIdx.x; task < n_tasks; task += gridDim.x) {
    const int img = task / a.n_bands, band = task - img * a.n_bands;
    HBK_MARK(1);
    __syncthreads();  // the previous task's readers are done
    // 1) input rows [row0, row0 + RI) (clamped to the image) -> raw; prefetch the next task's
#pragma unroll
    for (int u = 0; u < kRawPer; ++u) {
      const int i = tid + u * kP0Threads;
      if (i < kRawV) *reinterpret_cast<float4*>(raw + 4 * i) = rawv[u];
    }
    if (task + static_cast<int>(gridDim.x) < n_tasks) load_raw(task + gridDim.x);
    __syncthreads();
    HBK_MARK(40);
    // 2) stage 0: 3x3, 1 -> C; B fragments straight from the f32 rows
    //    (taps 0-4 in the first K half, 5-8 and a zero in the second)
    {
      for (int t = wave; t < G::T0; t += kP0Waves) {
        const int pp = t * 32 + r32, p = min(pp, G::M0 - 1);
        const int y = p / G::W0, x = p - y * G::W0;
        const float* rp = raw + y * WI + x;
        float v[8];
#pragma unroll
        for (int i = 0; i < 5; ++i) {
          const int t1 = 5 + i < 9 ? 5 + i : 0;
          v[i] = rp[khalf ? (t1 / 3) * WI + t1 % 3 : (i / 3) * WI + i % 3];
        }
        if (khalf) v[4] = 0.f;
        v[5] = v[6] = v[7] = 0.f;
        uint32_t hb[4], lb[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) split2_mix(v[2 * i], v[2 * i + 1], hb[i], lb[i], amax);
        const h8 xh = __builtin_bit_cast(h8, uint4{hb[0], hb[1], hb[2], hb[3]});
        const h8 xl = __builtin_bit_cast(h8, uint4{lb[0], lb[1], lb[2], lb[3]});
        f16x acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0h, xh, b0, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0h, xl, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a0l, xh, acc, 0, 0, 0);
        if (pp < G::M0) p0_store_planes<C, G::CS, LEAKY>(acc, p, khalf, s0h, s0l, a.alpha, amax);
      }
    }
    HBK_MARK(50);
    __syncthreads();
    HBK_MARK(41);
    p0_stage12<WI, C, BAND, 1, LEAKY>(a, W1, s0h, s0l, s1h, s1l, nullptr, wave, r32, khalf, amax);
    HBK_MARK(51);
    __syncthreads();
    HBK_MARK(42);
    p0_stage12<WI, C, BAND, 2, LEAKY>(a, W2, s1h, s1l, nullptr, nullptr, s2, wave, r32, khalf, amax);
    HBK_MARK(52);
    __syncthreads();
    HBK_MARK(43);
    // 3) 2x2 max-pool of the stage-2 rows -> the band's BAND output rows
    {
      constexpr int PW = G::W2 / 2, C4 = C / 4;
      float* dst = a.out + static_cast<int64_t>(img) * a.H_out * PW * C;
      for (int i = tid; i < BAND * PW * C4; i += kP0Threads) {
        const int c4 = i % C4, rest = i / C4, px = rest % PW, py = rest / PW;
        const int orow = band * BAND + py;
        if (orow >= a.H_out) continue;
        const float* q0 = s2 + ((2 * py) * G::W2 + 2 * px) * C + 4 * c4;
        const float4 v00 = *reinterpret_cast<const float4*>(q0);
        const float4 v01 = *reinterpret_cast<const float4*>(q0 + C);
        const float4 v10 = *reinterpret_cast<const float4*>(q0 + G::W2 * C);
        const float4 v11 = *reinterpret_cast<const float4*>(q0 + G::W2 * C + C);
        float4 m;
        m.x = nan_max(nan_max(v00.x, v01.x), nan_max(v10.x, v11.x));
        m.y = nan_max(nan_max(v00.y, v01.y), nan_max(v10.y, v11.y));
        m.z = nan_max(nan_max(v00.z, v01.z), nan_max(v10.z, v11.z));
        m.w = nan_max(nan_max(v00.w, v01.w), nan_max(v10.w, v11.w));
        *reinterpret_cast<float4*>(dst + (static_cast<int64_t>(orow) * PW + px) * C + 4 * c4) = m;
      }
    }
    HBK_MARK(6);
  }
  raise_range(a.range_flag, amax);
}

// ------------------------------------------------------------------- p1 ----
// Pattern kernel for the chain  conv 1x3 (CI -> 32) . conv 3x1 (32 -> 32) .
// conv 1x3 (32 -> 32) . conv 3x1 (32 -> 32) . max-pool 2x2  on an NHWC f32
// input of fixed width WI (SE20 chain 1: 66 x 14 x 24 -> 31 x 5 x 32). Same
// split-f16 numerics and tile / epilogue scheme as p0_chain_kernel; the
// stage weights do not all fit in VGPRs, so each stage's A fragments are
// loaded (from L2) one stage ahead, while the previous stage runs.
constexpr int kP1C = 32;

struct P1Args {
  const float* in;          // [img][H_in][WI][CI] f32
  float* out;               // [img][H_out][W4 / 2][32] f32
  const _Float16* w;        // stage s at woff[s]: hi [32][16 ks_s], lo [32][16 ks_s]
  const float* bias;        // [4][32]
  int64_t n_img;
  int64_t src_img_stride;   // floats
  int H_in, H_out, n_bands;
  float alpha;
  int* range_flag;          // set to 1 when an f16-split value reaches kF16Max
};

template <int WI, int CI, int BAND>
struct P1Geo {
  static constexpr int C = kP1C;
  static constexpr int W0 = WI, W1 = WI - 2, W2 = W1, W3 = W1 - 2, W4 = W3;
  static constexpr int R4 = 2 * BAND, R3 = R4 + 2, R2 = R3, R1 = R2 + 2, R0 = R1;
  static constexpr int CSI = ((CI / 8) % 2 == 0) ? CI + 8 : CI;
  static constexpr int CS = ((C / 8) % 2 == 0) ? C + 8 : C;
  static constexpr int M1 = R1 * W1, M2 = R2 * W2, M3 = R3 * W3, M4 = R4 * W4;
  static constexpr int KS1 = (3 * CI + 15) / 16, KS = (3 * C + 15) / 16;
  static constexpr int KSMAX = KS1 > KS ? KS1 : KS;
  static constexpr int INB = R0 * W0 * CSI * 4, S1B = M1 * CS * 4, S2B = M2 * CS * 4, S3B = M3 * CS * 4,
                       S4B = M4 * C * 4;
  static constexpr int mx(int a, int b) { return a > b ? a : b; }
  static constexpr int XB = (mx(mx(INB, S2B), S4B) + 15) & ~15;  // input, stage-2 out, stage-4 out (f32)
  static constexpr int YB = (mx(S1B, S3B) + 15) & ~15;            // stage-1 out, stage-3 out
  static constexpr int LDS = XB + YB;
  static constexpr int WOFF1 = 0, WOFF2 = WOFF1 + 2 * 32 * 16 * KS1, WOFF3 = WOFF2 + 2 * 32 * 16 * KS,
                       WOFF4 = WOFF3 + 2 * 32 * 16 * KS, WHALFS = WOFF4 + 2 * 32 * 16 * KS;
};

template <int KS>
__device__ __forceinline__ P0W<KS> p1_load_w(const _Float16* w, const float* bias, int r32, int khalf) {
  P0W<KS> W;
  const _Float16* wp = w + r32 * (16 * KS) + 8 * khalf;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    W.ah[ks] = *reinterpret_cast<const h8*>(wp + 16 * ks);
    W.al[ks] = *reinterpret_cast<const h8*>(wp + 32 * 16 * KS + 16 * ks);
  }
  W.bias = p0_bias(bias, khalf);
  return W;
}

// One conv stage on LDS planes: kernel KH x KW over CIN channels (fp16 stride
// CSI per position, input grid width WIN), output grid (M positions, width
// WOUT), 32 output channels -> planes (CSO) or f32 (F32OUT, stride 32).
template <int KH, int KW, int CIN, int CSI, int WIN, int WOUT, int M, int KS, int CSO, bool F32OUT, bool LEAKY>
__device__ __forceinline__ void p1_stage(const P0W<KS>& W, const _Float16* xh_, const _Float16* xl_,
                                         _Float16* oh, _Float16* ol, float* of, float alpha, int wave, int r32,
                                         int khalf, float& amax) {
  constexpr int T = (M + 31) / 32;
  auto epilogue = [&](int t, const f16x& acc) {
    const int pp = t * 32 + r32;
    if (pp >= M) return;
    if (!F32OUT) {
      p0_store_planes<kP1C, CSO, LEAKY>(acc, pp, khalf, oh, ol, alpha, amax);
    } else {
#pragma unroll
      for (int q = 0; q < kP1C / 8; ++q) {
        float4 v;
        v.x = p0_act<LEAKY>(acc[4 * q], alpha);
        v.y = p0_act<LEAKY>(acc[4 * q + 1], alpha);
        v.z = p0_act<LEAKY>(acc[4 * q + 2], alpha);
        v.w = p0_act<LEAKY>(acc[4 * q + 3], alpha);
        *reinterpret_cast<float4*>(of + pp * kP1C + 8 * q + 4 * khalf) = v;
      }
    }
  };
  f16x prev;
  int tprev = -1;
  for (int t = wave; t < T; t += kP0Waves) {
    const int p = min(t * 32 + r32, M - 1);
    const int y = p / WOUT, x = p - y * WOUT;
    const int base = (y * WIN + x) * CSI;
    h8 xh[KS], xl[KS];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      // K = tap * CIN + ci, tap = dy * KW + dx; groups past KH KW CIN read group 0 (weights 0)
      const int ka = 16 * ks < KH * KW * CIN ? 16 * ks : 0;
      const int kb = 16 * ks + 8 < KH * KW * CIN ? 16 * ks + 8 : 0;
      const int ta = ka / CIN, tb = kb / CIN;
      const int oa = ((ta / KW) * WIN + ta % KW) * CSI + ka % CIN;
      const int ob = ((tb / KW) * WIN + tb % KW) * CSI + kb % CIN;
      const int o = base + (khalf ? ob : oa);
      xh[ks] = *reinterpret_cast<const h8*>(xh_ + o);
      xl[ks] = *reinterpret_cast<const h8*>(xl_ + o);
    }
    f16x acc = W.bias;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(W.ah[ks], xh[ks], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(W.ah[ks], xl[ks], acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(W.al[ks], xh[ks], acc, 0, 0, 0);
    }
    if (tprev >= 0) epilogue(tprev, prev);
    prev = acc;
    tprev = t;
  }
  if (tprev >= 0) epilogue(tprev, prev);
}

template <int WI, int CI, int BAND, bool LEAKY>
__global__ void __launch_bounds__(kP0Threads) __attribute__((amdgpu_waves_per_eu(2)))
p1_chain_kernel(P1Args a) {
  using G = P1Geo<WI, CI, BAND>;
  constexpr int C = kP1C;
  extern __shared__ __attribute__((aligned(16))) unsigned char p1mem[];
  _Float16* inh = reinterpret_cast<_Float16*>(p1mem);
  _Float16* inl = inh + G::R0 * G::W0 * G::CSI;
  _Float16* s2h = reinterpret_cast<_Float16*>(p1mem);
  _Float16* s2l = s2h + G::M2 * G::CS;
  float* s4 = reinterpret_cast<float*>(p1mem);
  _Float16* s1h = reinterpret_cast<_Float16*>(p1mem + G::XB);
  _Float16* s1l = s1h + G::M1 * G::CS;
  _Float16* s3h = reinterpret_cast<_Float16*>(p1mem + G::XB);
  _Float16* s3l = s3h + G::M3 * G::CS;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r32 = lane & 31, khalf = lane >> 5;
  const int n_tasks = static_cast<int>(a.n_img) * a.n_bands;
  const float alpha = a.alpha;

  P0W<G::KS1> W1 = p1_load_w<G::KS1>(a.w + G::WOFF1, a.bias, r32, khalf);
  float amax = 0.f;
  for (int task = blockIdx.x; task < n_tasks; task += gridDim.x) {
    const int img = task / a.n_bands, band = task - img * a.n_bands;
    const int row0 = band * G::R4;
    __syncthreads();  // the previous task's readers are done
    // 1) input rows [row0, row0 + R0) (clamped) -> hi / lo planes, 8 channels per unit
    {
      const float* src = a.in + static_cast<int64_t>(img) * a.src_img_stride;
      constexpr int U = G::R0 * WI * (CI / 8);
      for (int u = tid; u < U; u += kP0Threads) {
        const int c8 = u % (CI / 8), pos = u / (CI / 8);
        const int r = pos / WI, x = pos - r * WI;
        const int rr = min(row0 + r, a.H_in - 1);
        const float* q = src + (static_cast<int64_t>(rr) * WI + x) * CI + 8 * c8;
        const float4 v0 = *reinterpret_cast<const float4*>(q), v1 = *reinterpret_cast<const float4*>(q + 4);
        uint32_t h[4], l[4];
        split2_mix(v0.x, v0.y, h[0], l[0], amax);
        split2_mix(v0.z, v0.w, h[1], l[1], amax);
        split2_mix(v1.x, v1.y, h[2], l[2], amax);
        split2_mix(v1.z, v1.w, h[3], l[3], amax);
        const int o = pos * G::CSI + 8 * c8;
        *reinterpret_cast<uint4*>(inh + o) = uint4{h[0], h[1], h[2], h[3]};
        *reinterpret_cast<uint4*>(inl + o) = uint4{l[0], l[1], l[2], l[3]};
      }
    }
    __syncthreads();
    P0W<G::KS> W2 = p1_load_w<G::KS>(a.w + G::WOFF2, a.bias + 32, r32, khalf);
    p1_stage<1, 3, CI, G::CSI, G::W0, G::W1, G::M1, G::KS1, G::CS, false, LEAKY>(W1, inh, inl, s1h, s1l, nullptr,
                                                                                  alpha, wave, r32, khalf, amax);
    __syncthreads();
    P0W<G::KS> W3 = p1_load_w<G::KS>(a.w + G::WOFF3, a.bias + 64, r32, khalf);
    p1_stage<3, 1, C, G::CS, G::W1, G::W2, G::M2, G::KS, G::CS, false, LEAKY>(W2, s1h, s1l, s2h, s2l, nullptr,
                                                                               alpha, wave, r32, khalf, amax);
    __syncthreads();
    P0W<G::KS> W4 = p1_load_w<G::KS>(a.w + G::WOFF4, a.bias + 96, r32, khalf);
    p1_stage<1, 3, C, G::CS, G::W2, G::W3, G::M3, G::KS, G::CS, false, LEAKY>(W3, s2h, s2l, s3h, s3l, nullptr,
                                                                               alpha, wave, r32, khalf, amax);
    __syncthreads();
    W1 = p1_load_w<G::KS1>(a.w + G::WOFF1, a.bias, r32, khalf);  // the next task's stage 1
    p1_stage<3, 1, C, G::CS, G::W3, G::W4, G::M4, G::KS, G::CS, true, LEAKY>(W4, s3h, s3l, nullptr, nullptr, s4,
                                                                              alpha, wave, r32, khalf, amax);
    __syncthreads();
    // 2x2 max-pool of the stage-4 rows -> BAND output rows
    {
      constexpr int PW = G::W4 / 2, C4 = C / 4;
      float* dst = a.out + static_cast<int64_t>(img) * a.H_out * PW * C;
      for (int i = tid; i < BAND * PW * C4; i += kP0Threads) {
        const int c4 = i % C4, rest = i / C4, px = rest % PW, py = rest / PW;
        const int orow = band * BAND + py;
        if (orow >= a.H_out) continue;
        const float* q0 = s4 + ((2 * py) * G::W4 + 2 * px) * C + 4 * c4;
        const float4 v00 = *reinterpret_cast<const float4*>(q0);
        const float4 v01 = *reinterpret_cast<const float4*>(q0 + C);
        const float4 v10 = *reinterpret_cast<const float4*>(q0 + G::W4 * C);
        const float4 v11 = *reinterpret_cast<const float4*>(q0 + G::W4 * C + C);
        float4 m;
        m.x = nan_max(nan_max(v00.x, v01.x), nan_max(v10.x, v11.x));
        m.y = nan_max(nan_max(v00.y, v01.y), nan_max(v10.y, v11.y));
        m.z = nan_max(nan_max(v00.z, v01.z), nan_max(v10.z, v11.z));
        m.w = nan_max(nan_max(v00.w, v01.w), nan_max(v10.w, v11.w));
        *reinterpret_cast<float4*>(dst + (static_cast<int64_t>(orow) * PW + px) * C + 4 * c4) = m;
      }
    }
  }
  raise_range(a.range_flag, amax);
}

// ------------------------------------------------------------------ p0s ----
// Streaming form of the p0 chain (SE20 chain 0 on a 32-wide mel image:
// 3x3 1 -> 24, 1x3 24 -> 24, 3x1 24 -> 24, max-pool 2x2): ONE WAVE PER CLIP,
// the clip's rows streamed top to bottom, no halo recomputation and no
// workgroup barrier. A tile is one row (32 positions; 30 / 28 / 28 valid).
// Iteration y runs three independent MFMA chains:
//   stage 0 of row y      B from the raw rows in registers      -> s0[y & 1]
//   stage 1 of row y - 1  B from s0[(y - 1) & 1] (LDS)          -> s1[(y - 1) & 3]
//   stage 2 of row y - 4  B from s1 rows y - 4 .. y - 2 (LDS)   -> registers
// Every LDS row an iteration reads was written by an earlier iteration of the
// same wave, and a wave's LDS instructions execute in order, so a compiler
// barrier between iterations is the only synchronisation. Stage-2 rows 2i and
// 2i + 1 are max-pooled in registers, the column pairs by a DPP lane swap,
// and the pooled row is stored as f32 [66][14][24] (the p1 chain's input).
// Raw rows: one dword per lane per row, loaded 8-11 rows ahead; the three
// column taps come from two DPP wave shifts. Biases ride in a padding slot
// of K whose B value is 1 (hi 1, lo 0), so every accumulator starts at 0.
constexpr int kP0sWaves = 4;
constexpr int kP0sThreads = 64 * kP0sWaves;
constexpr int kP0sCS = 24;                         // fp16 per position (3 odd 16-B groups)
constexpr int kP0sS0Plane = 34 * kP0sCS;           // positions 0..33 (x + tap <= 33)
constexpr int kP0sS1Plane = 32 * kP0sCS;
constexpr int kP0sOnes = 4 * kP0sS0Plane + 8 * kP0sS1Plane;  // fp16 offset of the ones / zeros slots
constexpr int kP0sWaveHalfs = kP0sOnes + 16;
constexpr int kP0sLds = kP0sWaves * kP0sWaveHalfs * 2;
constexpr int kP0sKS = 5;                          // K steps of stages 1 and 2 (72 + bias slot)
constexpr int kP0sRows = 136, kP0sHout = 66, kP0sWout = 14, kP0sC = 24;

struct P0sW {
  h8 h[kP0sKS], l[kP0sKS];
};

__device__ __forceinline__ float wave_shl1(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x130, 0xf, 0xf, false));
}

typedef float f2v __attribute__((ext_vector_type(2)));

// LeakyReLU of two values: one packed multiply, two maxes (NaN stays NaN)
template <bool LEAKY>
__device__ __forceinline__ void p0s_act2(float& a, float& b, float alpha) {
  if (!LEAKY) return;
  const f2v m = f2v{a, b} * alpha;
  asm("v_max_f32 %0, %0, %1" : "+v"(a) : "v"(m.x));
  asm("v_max_f32 %0, %0, %1" : "+v"(b) : "v"(m.y));
}

// activation, split and LDS store of one finished stage-0 / stage-1 tile
template <bool LEAKY>
__device__ __forceinline__ void p0s_store(const f16x& acc, _Float16* oh, int x, int khalf, float alpha, bool track_it,
                                          float& amax, int plane) {
  float m = 0.f;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    float v[4] = {acc[4 * q], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]};
    p0s_act2<LEAKY>(v[0], v[1], alpha);
    p0s_act2<LEAKY>(v[2], v[3], alpha);
    uint32_t h01, l01, h23, l23;
    split2_mix(v[0], v[1], h01, l01, m);
    split2_mix(v[2], v[3], h23, l23, m);
    const int o = x * kP0sCS + 8 * q + 4 * khalf;
    *reinterpret_cast<uint2*>(oh + o) = uint2{h01, h23};
    *reinterpret_cast<uint2*>(oh + plane + o) = uint2{l01, l23};
  }
  asm("v_max_f32 %0, %0, %1" : "+v"(amax) : "v"(track_it ? m : 0.f));
}

template <bool LEAKY>
struct P0sCtx {
  h8 a0h, a0l;
  P0sW w1, w2;
  float r[2][3];   // raw rows y + khalf, y + 1 + khalf at columns x, x + 1, x + 2
  float q[8];      // raw rows loaded ahead (column x; row + khalf)
  f16x pool;       // stage-2 row 2i (even) awaiting its partner
  float amax;
  float alpha;
};

template <int PAR, bool LEAKY>
__device__ __forceinline__ void p0s_iter(P0sCtx<LEAKY>& c, int y, int qi, _Float16* wl, float* orow_base, int x,
                                         int khalf) {
  // raw window: rows y + khalf, y + 1 + khalf (the second from the load queue)
  c.r[0][0] = c.r[1][0]; c.r[0][1] = c.r[1][1]; c.r[0][2] = c.r[1][2];
  c.r[1][0] = c.q[qi];
  c.r[1][1] = wave_shl1(c.r[1][0]);
  c.r[1][2] = wave_shl1(c.r[1][1]);

  _Float16* s0w = wl + (PAR & 1) * 2 * kP0sS0Plane;        // stage 0 writes row y
  _Float16* s0r = wl + ((PAR + 1) & 1) * 2 * kP0sS0Plane;  // stage 1 reads row y - 1
  _Float16* s1 = wl + 4 * kP0sS0Plane;

  // B fragments of stage 1 (row y - 1) and stage 2 (row y - 4), one K step
  // ahead of their MFMAs. Stage 1: K group g = 2 ks + khalf = tap * 3 + c sits
  // at s0 fp16 offset 24 (x + tap) + 8 c = 24 x + 8 g, one per-lane base plus
  // immediates; group 9 is the bias slot (B = 1). Stage 2: the groups (dy, c)
  // are paired within a row for ks < 3 (khalf = c), then (0, 2) | (1, 2) and
  // (2, 2) | bias (mirrored by plan_p0s's packing).
  const _Float16* base1 = s0r + x * kP0sCS + 8 * khalf;
  const _Float16* base2 = s1 + x * kP0sCS + 8 * khalf;
  auto load1 = [&](int ks, h8& bh, h8& bl) {
    const bool one = ks == 4 && khalf;
    const _Float16* p1 = one ? wl + kP0sOnes : base1 + 16 * ks;
    bh = *reinterpret_cast<const h8*>(p1);
    bl = *reinterpret_cast<const h8*>(p1 + (one ? 8 : kP0sS0Plane));
  };
  auto load2 = [&](int ks, h8& bh, h8& bl) {
    const _Float16* p2;
    if (ks < 3) {
      p2 = base2 + ((PAR + ks) & 3) * 2 * kP0sS1Plane;
    } else if (ks == 3) {
      p2 = s1 + x * kP0sCS + 16 + (khalf ? ((PAR + 1) & 3) : (PAR & 3)) * 2 * kP0sS1Plane;
    } else {
      p2 = khalf ? wl + kP0sOnes : s1 + x * kP0sCS + 16 + ((PAR + 2) & 3) * 2 * kP0sS1Plane;
    }
    const bool one = ks == 4 && khalf;
    bh = *reinterpret_cast<const h8*>(p2);
    bl = *reinterpret_cast<const h8*>(p2 + (one ? 8 : kP0sS1Plane));
  };
  h8 f[2][2];
  load1(0, f[0][0], f[0][1]);

  // stage 0 (row y): K slots {r0[0..2], r1[0..2], 1, 0} in both lane halves, the
  // window one row lower in the upper half (taps (0, *), (1, 0), (1, 1) and the
  // bias in the lower half's weights, (1, 2), (2, *) in the upper half's)
  uint32_t hb[3], lb[3];
  float m0 = 0.f;
  split2_mix(c.r[0][0], c.r[0][1], hb[0], lb[0], m0);
  split2_mix(c.r[0][2], c.r[1][0], hb[1], lb[1], m0);
  split2_mix(c.r[1][1], c.r[1][2], hb[2], lb[2], m0);
  const h8 xh = __builtin_bit_cast(h8, uint4{hb[0], hb[1], hb[2], 0x3C00u});  // slot 6 = 1.0 (f16)
  const h8 xl = __builtin_bit_cast(h8, uint4{lb[0], lb[1], lb[2], 0u});
  const f16x zero = {};
  f16x acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(c.a0h, xh, zero, 0, 0, 0);
  acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(c.a0h, xl, acc0, 0, 0, 0);
  acc0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(c.a0l, xh, acc0, 0, 0, 0);
  const bool raw_ok = y < kP0sRows - 2;

  // The three stages' MFMA chains run one after another (stage 1, then stage
  // 2), and each finished stage's epilogue is issued between the next stage's
  // MFMAs (sched_group_barrier: 1 MFMA, then up to 5 VALU), so a wave keeps its
  // own matrix pipe busy while it activates, splits and stores: stage 0's
  // epilogue beside stage 1's MFMAs, stage 1's beside stage 2's.
  f16x acc1 = zero;
#pragma unroll
  for (int ks = 0; ks < kP0sKS; ++ks) {
    h8* cur = f[ks & 1];
    if (ks + 1 < kP0sKS) load1(ks + 1, f[(ks + 1) & 1][0], f[(ks + 1) & 1][1]);
    else load2(0, f[(ks + 1) & 1][0], f[(ks + 1) & 1][1]);
    acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(c.w1.h[ks], cur[0], acc1, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(c.w1.h[ks], cur[1], acc1, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(c.w1.l[ks], cur[0], acc1, 0, 0, 0);
    if (ks == 1) {
      asm("v_max_f32 %0, %0, %1" : "+v"(c.amax) : "v"(raw_ok ? m0 : 0.f));
      p0s_store<LEAKY>(acc0, s0w, x, khalf, c.alpha, raw_ok && x < 30, c.amax, kP0sS0Plane);
    }
#pragma unroll
    for (int g = 0; g < 3; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
      __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
    }
  }
  // stage 2 accumulates into c.pool for an even row y - 4 (held for its odd partner)
  f16x acc2 = zero;
  f16x& a2 = (PAR & 1) == 0 ? c.pool : acc2;
  a2 = zero;
#pragma unroll
  for (int ks = 0; ks < kP0sKS; ++ks) {
    h8* cur = f[(ks + kP0sKS) & 1];
    if (ks + 1 < kP0sKS) load2(ks + 1, f[(ks + 1 + kP0sKS) & 1][0], f[(ks + 1 + kP0sKS) & 1][1]);
    a2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(c.w2.h[ks], cur[0], a2, 0, 0, 0);
    a2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(c.w2.h[ks], cur[1], a2, 0, 0, 0);
    a2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(c.w2.l[ks], cur[0], a2, 0, 0, 0);
    if (ks == 0)
      p0s_store<LEAKY>(acc1, s1 + ((PAR + 3) & 3) * 2 * kP0sS1Plane, x, khalf, c.alpha,
                       y >= 1 && y <= kP0sRows - 2 && x < 28, c.amax, kP0sS1Plane);
#pragma unroll
    for (int g = 0; g < 3; ++g) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x002, 5, 0);
      __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
    }
  }

  // stage 2 (row y - 4): rows 2i and 2i + 1 pooled (max commutes with the
  // monotone activation; v_maximum3 propagates NaN, as the reference's max-pool)
  if ((PAR & 1) == 1) {
    float pv[12];
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      const float t = __builtin_elementwise_maximum(c.pool[i], acc2[i]);
      // column pair (x, x ^ 1): DPP quad_perm [1, 0, 3, 2]
      const float u = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, t), 0xB1, 0xf, 0xf,
                                                                         false));
      pv[i] = __builtin_elementwise_maximum(t, u);
    }
#pragma unroll
    for (int i = 0; i < 12; i += 2) p0s_act2<LEAKY>(pv[i], pv[i + 1], c.alpha);
    if (y >= 5 && !(x & 1) && x < 28) {
      float* o = orow_base + static_cast<int64_t>((y - 4) >> 1) * (kP0sWout * kP0sC) + (x >> 1) * kP0sC + 4 * khalf;
#pragma unroll
      for (int q = 0; q < 3; ++q)
        *reinterpret_cast<float4*>(o + 8 * q) = float4{pv[4 * q], pv[4 * q + 1], pv[4 * q + 2], pv[4 * q + 3]};
    }
  }
  asm volatile("" ::: "memory");  // this iteration's LDS writes before the next one's reads (in-order LDS)
}

template <bool LEAKY>
__global__ void __launch_bounds__(kP0sThreads) __attribute__((amdgpu_waves_per_eu(2)))
p0s_chain_kernel(P0Args a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char p0smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int x = lane & 31, khalf = lane >> 5;
  _Float16* wl = reinterpret_cast<_Float16*>(p0smem) + wave * kP0sWaveHalfs;
  // constant slots: hi {1, 0, ..} and lo {0, ..}; s0 positions 32, 33 (never written) = 0
  if (lane < 16) wl[kP0sOnes + lane] = static_cast<_Float16>(lane == 0 ? 1.f : 0.f);
  for (int i = lane; i < 2 * 2 * 2 * kP0sCS; i += 64) {  // [buffer][plane][pos 32, 33][24]
    const int b = i / (4 * kP0sCS), rest = i - b * 4 * kP0sCS, pl = rest / (2 * kP0sCS);
    wl[b * 2 * kP0sS0Plane + pl * kP0sS0Plane + 32 * kP0sCS + rest % (2 * kP0sCS)] = static_cast<_Float16>(0.f);
  }
  P0sCtx<LEAKY> c;
  c.alpha = a.alpha;
  c.amax = 0.f;
  {
    const _Float16* w0 = a.w + x * 16 + 8 * khalf;
    c.a0h = *reinterpret_cast<const h8*>(w0);
    c.a0l = *reinterpret_cast<const h8*>(w0 + 32 * 16);
    const _Float16* w1 = a.w + 2 * 32 * 16 + x * (16 * kP0sKS) + 8 * khalf;
    const _Float16* w2 = w1 + 2 * 32 * 16 * kP0sKS;
#pragma unroll
    for (int ks = 0; ks < kP0sKS; ++ks) {
      c.w1.h[ks] = *reinterpret_cast<const h8*>(w1 + 16 * ks);
      c.w1.l[ks] = *reinterpret_cast<const h8*>(w1 + 32 * 16 * kP0sKS + 16 * ks);
      c.w2.h[ks] = *reinterpret_cast<const h8*>(w2 + 16 * ks);
      c.w2.l[ks] = *reinterpret_cast<const h8*>(w2 + 32 * 16 * kP0sKS + 16 * ks);
    }
  }
  asm volatile("" ::: "memory");
  const int64_t stride_w = static_cast<int64_t>(gridDim.x) * kP0sWaves;
  for (int64_t img = static_cast<int64_t>(blockIdx.x) * kP0sWaves + wave; img < a.n_img; img += stride_w) {
    const float* src = a.in + img * a.src_img_stride + x;
    const int hmax = a.H_in - 1;
    auto raw = [&](int row) { return src[min(row, hmax) * 32]; };
    float* orow_base = a.out + img * (static_cast<int64_t>(kP0sHout) * kP0sWout * kP0sC);
    // window row khalf (the first iteration shifts it down and brings row 1 + khalf); queue rows 1 .. 4 (+ khalf)
    c.r[1][0] = raw(khalf);
    c.r[1][1] = wave_shl1(c.r[1][0]);
    c.r[1][2] = wave_shl1(c.r[1][1]);
#pragma unroll
    for (int i = 0; i < 4; ++i) c.q[i] = raw(1 + khalf + i);
    for (int y0 = 0; y0 < kP0sRows; y0 += 4) {
      // rows y0 + 5 .. y0 + 8 (+ khalf; the next four iterations') into the queue's second half
#pragma unroll
      for (int i = 0; i < 4; ++i) c.q[4 + i] = raw(y0 + 5 + khalf + i);
      p0s_iter<0, LEAKY>(c, y0, 0, wl, orow_base, x, khalf);
      p0s_iter<1, LEAKY>(c, y0 + 1, 1, wl, orow_base, x, khalf);
      p0s_iter<2, LEAKY>(c, y0 + 2, 2, wl, orow_base, x, khalf);
      p0s_iter<3, LEAKY>(c, y0 + 3, 3, wl, orow_base, x, khalf);
#pragma unroll
      for (int i = 0; i < 4; ++i) c.q[i] = c.q[i + 4];
    }
  }
  raise_range(a.range_flag, c.amax);
}

// ------------------------------------------------------------------ p1s ----
// Streaming form of the p1 chain (SE20 chain 1 on the 66 x 14 x 24 chain-0
// output: 1x3 24 -> 32, 3x1, 1x3, 3x1 32 -> 32, max-pool 2x2 -> 31 x 5 x 32),
// rows streamed top to bottom through a TWO-WAVE STAGE PIPELINE per clip:
// wave 0 runs stages a and b, wave 1 stages c and d, so each wave keeps only
// its two stages' weights in VGPRs (96) and a CU runs two waves per SIMD.
// v_mfma_f32_16x16x32_f16 with a tile of one row (16 positions; 12 / 12 /
// 10 / 10 valid: a 32-position tile would be under half full) and two
// 16-channel output blocks. Iteration y (one workgroup barrier after it):
//   wave 0: stage input row y + 1; a(y) -> A[y & 3]; b(y - 3) -> B[(y - 3) & 1]
//   wave 1: c(y - 4) from B[(y - 4) & 1] -> C[(y - 4) & 3]; d(y - 7), pooled
// Every row a wave reads was written before the previous barrier or earlier
// by itself (a wave's LDS instructions execute in order). Stage a's bias
// rides in its K padding (slot 72, B = 1); b, c and d start their
// accumulators at the bias. K groups of 8 (g = 4 ks + kq, kq = lane / 16):
//   a: g = tap * 3 + c   -> input position x + tap, channels 8 c   (24 x + 8 g)
//   b: g = dy * 4 + c    -> A row (r + dy), position x, channels 8 c
//   c: g = dx * 4 + c    -> B position x + dx, channels 8 c
//   d: g = dy * 4 + c    -> C row (r + dy), position x, channels 8 c
constexpr int kP1sThreads = 128;
constexpr int kP1sCSI = 24, kP1sCS = 40;          // fp16 per position: input (24 ch), stage outputs (32 ch)
constexpr int kP1sInPlane = 18 * kP1sCSI;         // 18 positions (14 valid; x + tap <= 17)
constexpr int kP1sInSlot = 2 * kP1sInPlane + 32;  // hi, lo, then ones (hi 8, lo 8) and zeros (hi 8, lo 8)
constexpr int kP1sPlane = 16 * kP1sCS;            // A / C rows
constexpr int kP1sBPlane = 18 * kP1sCS;           // B rows (c reads x + dx <= 17)
constexpr int kP1sIn = 0, kP1sA = kP1sIn + 2 * kP1sInSlot, kP1sB = kP1sA + 4 * 2 * kP1sPlane,
              kP1sCr = kP1sB + 2 * 2 * kP1sBPlane;
constexpr int kP1sHalfs = kP1sCr + 4 * 2 * kP1sPlane;
constexpr int kP1sLds = kP1sHalfs * 2;
constexpr int kP1sHin = 66, kP1sHout = 31, kP1sWi = 14, kP1sWo = 5, kP1sCo = 32;
constexpr int kP1sStageHalfs = 2 * 32 * 96;       // weights per stage: hi [32][96], lo [32][96]

struct P1sW {
  h8 h[2][3], l[2][3];  // [output block][K step]
};

struct P1sCtx {
  P1sW w[2];           // this wave's two stages
  f4 bias[2][2];       // wave 0: [b][mb] in bias[1]; wave 1: c, d
  float4 q[4][2];      // wave 0: input rows y + 1 .. y + 4 (two float4 per lane)
  f4 pool[2];          // wave 1: stage-d row 2i awaiting its partner
  float amax, alpha;
};

// one stage of one row: 2 output blocks x 3 K steps x 3 products
__device__ __forceinline__ void p1s_mma(f4 (&acc)[2], const P1sW& w, const h8 (&bh)[3], const h8 (&bl)[3]) {
#pragma unroll
  for (int ks = 0; ks < 3; ++ks)
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
      acc[mb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w.h[mb][ks], bh[ks], acc[mb], 0, 0, 0);
      acc[mb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w.h[mb][ks], bl[ks], acc[mb], 0, 0, 0);
      acc[mb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w.l[mb][ks], bh[ks], acc[mb], 0, 0, 0);
    }
}

// activation, split and LDS store of a finished stage row (channels 16 mb + 4 kq + j at position x)
template <bool LEAKY>
__device__ __forceinline__ void p1s_store(const f4 (&acc)[2], _Float16* oh, int plane, int x, int kq, float alpha,
                                          bool track_it, float& amax) {
  float m = 0.f;
#pragma unroll
  for (int mb = 0; mb < 2; ++mb) {
    float v[4] = {acc[mb][0], acc[mb][1], acc[mb][2], acc[mb][3]};
    p0s_act2<LEAKY>(v[0], v[1], alpha);
    p0s_act2<LEAKY>(v[2], v[3], alpha);
    uint32_t h01, l01, h23, l23;
    split2_mix(v[0], v[1], h01, l01, m);
    split2_mix(v[2], v[3], h23, l23, m);
    const int o = x * kP1sCS + 16 * mb + 4 * kq;
    *reinterpret_cast<uint2*>(oh + o) = uint2{h01, h23};
    *reinterpret_cast<uint2*>(oh + plane + o) = uint2{l01, l23};
  }
  asm("v_max_f32 %0, %0, %1" : "+v"(amax) : "v"(track_it ? m : 0.f));
}

// the input row in registers (two float4 per lane: entries lane, lane + 64 of 84) -> hi / lo planes
__device__ __forceinline__ void p1s_stage_row(const float4 (&v)[2], _Float16* in_w, int lane, float& amx) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = lane + 64 * u;
    if (u == 0 || lane < kP1sWi * 6 - 64) {
      uint32_t h01, l01, h23, l23;
      split2_mix(v[u].x, v[u].y, h01, l01, amx);
      split2_mix(v[u].z, v[u].w, h23, l23, amx);
      const int o = (i / 6) * kP1sCSI + (i % 6) * 4;
      *reinterpret_cast<uint2*>(in_w + o) = uint2{h01, h23};
      *reinterpret_cast<uint2*>(in_w + kP1sInPlane + o) = uint2{l01, l23};
    }
  }
}

// wave 0, iteration y: stage input row y + 1, a(y), b(y - 3)
template <int PAR, bool LEAKY>
__device__ __forceinline__ void p1s_iter0(P1sCtx& c, int y, _Float16* sm, const float* src, int hmax, int x, int kq,
                                          int lane, int a2h, int a2l) {
  const _Float16* in_r = sm + kP1sIn + (PAR & 1) * kP1sInSlot;
  _Float16* A = sm + kP1sA;
  h8 bh[2][3], bl[2][3];
#pragma unroll
  for (int ks = 0; ks < 3; ++ks) {
    const int oa = ks < 2 ? x * kP1sCSI + 32 * ks + 8 * kq : a2h;  // 24 x + 8 g; ks 2: the lane's slot
    const int la = ks < 2 ? kP1sInPlane : a2l;
    bh[0][ks] = *reinterpret_cast<const h8*>(in_r + oa);
    bl[0][ks] = *reinterpret_cast<const h8*>(in_r + oa + la);
    const _Float16* pb = A + ((PAR + 1 + ks) & 3) * 2 * kP1sPlane + x * kP1sCS + 8 * kq;  // row y - 3 + ks
    bh[1][ks] = *reinterpret_cast<const h8*>(pb);
    bl[1][ks] = *reinterpret_cast<const h8*>(pb + kP1sPlane);
  }
  {  // input row y + 1 (loaded four iterations ago) -> the other input slot; load row y + 5
    const int slot = (PAR + 1) & 3;
    float amx = 0.f;
    p1s_stage_row(c.q[slot], sm + kP1sIn + ((PAR + 1) & 1) * kP1sInSlot, lane, amx);
    asm("v_max_f32 %0, %0, %1" : "+v"(c.amax) : "v"(y + 1 < kP1sHin ? amx : 0.f));
    const float* r = src + static_cast<int64_t>(min(y + 5, hmax)) * (kP1sWi * kP1sCSI);
    c.q[slot][0] = *reinterpret_cast<const float4*>(r + 4 * lane);
    c.q[slot][1] = *reinterpret_cast<const float4*>(r + 4 * min(lane + 64, kP1sWi * 6 - 1));
  }
  const f4 zero = {};
  f4 acca[2] = {zero, zero}, accb[2] = {c.bias[1][0], c.bias[1][1]};
  p1s_mma(acca, c.w[0], bh[0], bl[0]);
  p1s_mma(accb, c.w[1], bh[1], bl[1]);
  p1s_store<LEAKY>(acca, A + (PAR & 3) * 2 * kP1sPlane, kP1sPlane, x, kq, c.alpha, y < kP1sHin && x < 12, c.amax);
  p1s_store<LEAKY>(accb, sm + kP1sB + ((PAR + 1) & 1) * 2 * kP1sBPlane, kP1sBPlane, x, kq, c.alpha,
                   y >= 3 && y - 3 < kP1sHin - 2 && x < 12, c.amax);
}

// wave 1, iteration y: c(y - 4), d(y - 7) pooled with row y - 8 when y - 7 is odd
template <int PAR, bool LEAKY>
__device__ __forceinline__ void p1s_iter1(P1sCtx& c, int y, _Float16* sm, float* obase, int x, int kq) {
  const _Float16* B = sm + kP1sB + (PAR & 1) * 2 * kP1sBPlane;  // row y - 4
  _Float16* C = sm + kP1sCr;
  h8 bh[2][3], bl[2][3];
#pragma unroll
  for (int ks = 0; ks < 3; ++ks) {
    const _Float16* pc = B + (x + ks) * kP1sCS + 8 * kq;
    bh[0][ks] = *reinterpret_cast<const h8*>(pc);
    bl[0][ks] = *reinterpret_cast<const h8*>(pc + kP1sBPlane);
    const _Float16* pd = C + ((PAR + 1 + ks) & 3) * 2 * kP1sPlane + x * kP1sCS + 8 * kq;  // row y - 7 + ks
    bh[1][ks] = *reinterpret_cast<const h8*>(pd);
    bl[1][ks] = *reinterpret_cast<const h8*>(pd + kP1sPlane);
  }
  f4 accc[2] = {c.bias[0][0], c.bias[0][1]};
  f4 accd_odd[2] = {c.bias[1][0], c.bias[1][1]};
  f4(&accd)[2] = ((PAR & 1) == 1) ? c.pool : accd_odd;  // row y - 7 even (y odd): accumulate into the pool
  if ((PAR & 1) == 1) {
    c.pool[0] = c.bias[1][0];
    c.pool[1] = c.bias[1][1];
  }
  p1s_mma(accc, c.w[0], bh[0], bl[0]);
  p1s_mma(accd, c.w[1], bh[1], bl[1]);
  p1s_store<LEAKY>(accc, C + (PAR & 3) * 2 * kP1sPlane, kP1sPlane, x, kq, c.alpha,
                   y >= 4 && y - 4 < kP1sHin - 2 && x < 10, c.amax);
  if ((PAR & 1) == 0) {  // row y - 7 odd: pool with row y - 8, store pooled row (y - 8) / 2
    float pv[2][4];
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float t = __builtin_elementwise_maximum(c.pool[mb][j], accd[mb][j]);
        const float u = __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, t), 0xB1, 0xf, 0xf,
                                                                           false));
        pv[mb][j] = __builtin_elementwise_maximum(t, u);
      }
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
      p0s_act2<LEAKY>(pv[mb][0], pv[mb][1], c.alpha);
      p0s_act2<LEAKY>(pv[mb][2], pv[mb][3], c.alpha);
    }
    if (y >= 8 && y - 8 < 2 * kP1sHout && !(x & 1) && x < 2 * kP1sWo) {
      float* o = obase + static_cast<int64_t>((y - 8) >> 1) * (kP1sWo * kP1sCo) + (x >> 1) * kP1sCo + 4 * kq;
#pragma unroll
      for (int mb = 0; mb < 2; ++mb)
        *reinterpret_cast<float4*>(o + 16 * mb) = float4{pv[mb][0], pv[mb][1], pv[mb][2], pv[mb][3]};
    }
  }
}

template <bool LEAKY>
__global__ void __launch_bounds__(kP1sThreads) __attribute__((amdgpu_waves_per_eu(2)))
p1s_chain_kernel(P1Args a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char p1smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int x = lane & 15, kq = lane >> 4;
  _Float16* sm = reinterpret_cast<_Float16*>(p1smem);
  // never-written positions: input 14 .. 17 (both slots, planes), B 16, 17; the ones / zeros slots
  for (int i = threadIdx.x; i < 2 * 2 * 4 * kP1sCSI; i += kP1sThreads) {
    const int s = i / (8 * kP1sCSI), rest = i - s * 8 * kP1sCSI, pl = rest / (4 * kP1sCSI);
    sm[kP1sIn + s * kP1sInSlot + pl * kP1sInPlane + 14 * kP1sCSI + rest % (4 * kP1sCSI)] = static_cast<_Float16>(0.f);
  }
  for (int i = threadIdx.x; i < 2 * 2 * 2 * kP1sCS; i += kP1sThreads) {
    const int s = i / (4 * kP1sCS), rest = i - s * 4 * kP1sCS, pl = rest / (2 * kP1sCS);
    sm[kP1sB + s * 2 * kP1sBPlane + pl * kP1sBPlane + 16 * kP1sCS + rest % (2 * kP1sCS)] = static_cast<_Float16>(0.f);
  }
  if (threadIdx.x < 64) {
    const int s = lane >> 5, k = lane & 31;
    sm[kP1sIn + s * kP1sInSlot + 2 * kP1sInPlane + k] = static_cast<_Float16>(k == 0 ? 1.f : 0.f);
  }
  // stage a's K step 2: lanes kq 0 read group 8 (tap 2, c 2), kq 1 the ones slot (bias), kq 2, 3 zeros
  const int a2h = kq == 0 ? x * kP1sCSI + 64 : 2 * kP1sInPlane + (kq == 1 ? 0 : 16);
  const int a2l = kq == 0 ? kP1sInPlane : 8;
  P1sCtx c;
  c.alpha = a.alpha;
  c.amax = 0.f;
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) {
        const _Float16* wp = a.w + (2 * wave + s) * kP1sStageHalfs + (16 * mb + x) * 96 + 32 * ks + 8 * kq;
        c.w[s].h[mb][ks] = *reinterpret_cast<const h8*>(wp);
        c.w[s].l[mb][ks] = *reinterpret_cast<const h8*>(wp + 32 * 96);
      }
  // biases of stages b, c, d ([3][32]): wave 0 keeps b's in bias[1], wave 1 c's and d's
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
      const int st = wave == 0 ? 0 : s + 1;
      const float4 b = *reinterpret_cast<const float4*>(a.bias + 32 * st + 16 * mb + 4 * kq);
      c.bias[wave == 0 ? 1 : s][mb] = f4{b.x, b.y, b.z, b.w};
    }
  __syncthreads();
  const int hmax = a.H_in - 1;
  for (int64_t img = blockIdx.x; img < a.n_img; img += gridDim.x) {
    const float* src = a.in + img * a.src_img_stride;
    float* obase = a.out + img * (static_cast<int64_t>(kP1sHout) * kP1sWo * kP1sCo);
    if (wave == 0) {  // input row 0 straight into slot 0; rows 1 .. 4 into the queue (slot = row & 3)
      float4 v[2];
      v[0] = *reinterpret_cast<const float4*>(src + 4 * lane);
      v[1] = *reinterpret_cast<const float4*>(src + 4 * min(lane + 64, kP1sWi * 6 - 1));
      float amx = 0.f;
      p1s_stage_row(v, sm + kP1sIn, lane, amx);
      asm("v_max_f32 %0, %0, %1" : "+v"(c.amax) : "v"(amx));
#pragma unroll
      for (int r = 1; r <= 4; ++r) {
        const float* rp = src + static_cast<int64_t>(min(r, hmax)) * (kP1sWi * kP1sCSI);
        c.q[r & 3][0] = *reinterpret_cast<const float4*>(rp + 4 * lane);
        c.q[r & 3][1] = *reinterpret_cast<const float4*>(rp + 4 * min(lane + 64, kP1sWi * 6 - 1));
      }
    }
    __syncthreads();
    for (int y0 = 0; y0 < 72; y0 += 4) {
#define HBK_P1S_STEP(P)                                                              \
  if (wave == 0)                                                                     \
    p1s_iter0<P, LEAKY>(c, y0 + P, sm, src, hmax, x, kq, lane, a2h, a2l);            \
  else                                                                               \
    p1s_iter1<P, LEAKY>(c, y0 + P, sm, obase, x, kq);                                \
  __syncthreads();
      HBK_P1S_STEP(0)
      HBK_P1S_STEP(1)
      HBK_P1S_STEP(2)
      HBK_P1S_STEP(3)
#undef HBK_P1S_STEP
    }
  }
  raise_range(a.range_flag, c.amax);
}

// ------------------------------------------------------------------ p2s ----
// Streaming form of SE20's chain 2 (the prefix's last chain, no output pool:
// 31 x 5 x 32 -> 1x3 32 -> 48 -> 3x1 -> 1x3 -> 3x1 48 -> 48 -> 27 x 1 x 48).
// Its rows are 3 or 1 positions wide, so a tile packs CLIPS: a workgroup
// streams the rows of 16 clips at once, and a 16-position tile of
// v_mfma_f32_16x16x32_f16 is (clip, column) for stages a, b (48 positions: 3
// tiles) and the clip for stages c, d (1 tile). Eight waves, one unit each,
// with that unit's weights in VGPRs: waves 0-2 stage a tiles 0-2, waves 3-5
// stage b tiles 0-2, wave 6 stage c, wave 7 stage d. Tick y (one workgroup
// barrier after it): a(y), b(y - 3), c(y - 4), d(y - 7), and every wave
// stages its share of input row y + 1. Rings as in p1s. K groups of 8
// (g = 4 ks + kq): a: g = dx * 4 + c (32 input channels); b, c, d: g = tap * 6
// + c (48 channels), g = 18 the bias slot (B = 1), g = 19 zeros; stage a
// starts its accumulators at the bias.
constexpr int kP2sThreads = 512, kP2sClips = 16;
constexpr int kP2sHin = 31, kP2sWi = 5, kP2sCi = 32, kP2sCo = 48, kP2sHout = 27;
constexpr int kP2sCSI = 40, kP2sCS = 56;                      // fp16 per position (odd 16-B groups)
constexpr int kP2sInPlane = kP2sClips * kP2sWi * kP2sCSI;     // one input row of 16 clips
constexpr int kP2sAPlane = kP2sClips * 3 * kP2sCS;            // stage a / b output rows (3 columns)
constexpr int kP2sCPlane = kP2sClips * kP2sCS;                // stage c output rows (1 column)
constexpr int kP2sIn = 0, kP2sA = kP2sIn + 2 * 2 * kP2sInPlane, kP2sB = kP2sA + 4 * 2 * kP2sAPlane,
              kP2sC = kP2sB + 2 * 2 * kP2sAPlane, kP2sOnes = kP2sC + 4 * 2 * kP2sCPlane;
constexpr int kP2sHalfs = kP2sOnes + 32;
constexpr int kP2sLds = kP2sHalfs * 2;
constexpr int kP2sKa = 96, kP2sK = 160;                       // packed K of stage a / stages b, c, d
constexpr int kP2sTicks = 36;                                 // rows 0 .. 30 through a 7-tick pipeline

struct P2sArgs {
  const float* in;        // [img][31][5][32] f32
  float* out;             // [img][27][48] f32
  const _Float16* w;      // a: hi / lo [48][96]; b, c, d: hi / lo [48][160]
  const float* bias_a;    // [48]
  int64_t n_img, src_img_stride;
  float alpha;
  int* range_flag;
};

// the wave's weights: [output block][K step] hi / lo
template <int KS>
struct P2sW {
  h8 h[3][KS], l[3][KS];
};

template <int KS>
__device__ __forceinline__ void p2s_mma(f4 (&acc)[3], const P2sW<KS>& w, int ks, const h8& bh, const h8& bl) {
#pragma unroll
  for (int mb = 0; mb < 3; ++mb) {
    acc[mb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w.h[mb][ks], bh, acc[mb], 0, 0, 0);
    acc[mb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w.h[mb][ks], bl, acc[mb], 0, 0, 0);
    acc[mb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w.l[mb][ks], bh, acc[mb], 0, 0, 0);
  }
}

// activation, split and LDS store of a finished tile (channels 16 mb + 4 kq + j at position p)
template <bool LEAKY>
__device__ __forceinline__ void p2s_store(const f4 (&acc)[3], _Float16* oh, int plane, int p, int kq, float alpha,
                                          bool track_it, float& amax) {
  float m = 0.f;
#pragma unroll
  for (int mb = 0; mb < 3; ++mb) {
    float v[4] = {acc[mb][0], acc[mb][1], acc[mb][2], acc[mb][3]};
    p0s_act2<LEAKY>(v[0], v[1], alpha);
    p0s_act2<LEAKY>(v[2], v[3], alpha);
    uint32_t h01, l01, h23, l23;
    split2_mix(v[0], v[1], h01, l01, m);
    split2_mix(v[2], v[3], h23, l23, m);
    const int o = p * kP2sCS + 16 * mb + 4 * kq;
    *reinterpret_cast<uint2*>(oh + o) = uint2{h01, h23};
    *reinterpret_cast<uint2*>(oh + plane + o) = uint2{l01, l23};
  }
  asm("v_max_f32 %0, %0, %1" : "+v"(amax) : "v"(track_it ? m : 0.f));
}

// every thread's share of input row `row` of the group's clips (640 float4): load / stage
struct P2sRow {
  float4 v[2];
};
__device__ __forceinline__ void p2s_load_row(P2sRow& r, const P2sArgs& a, int64_t img0, int row, int tid) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = min(tid + kP2sThreads * u, kP2sClips * kP2sWi * kP2sCi / 4 - 1);
    const int c = i / 40, rem = i - 40 * c;
    const int64_t img = min(img0 + c, a.n_img - 1);
    r.v[u] = *reinterpret_cast<const float4*>(a.in + img * a.src_img_stride + min(row, kP2sHin - 1) *
                                              (kP2sWi * kP2sCi) + 4 * rem);
  }
}
__device__ __forceinline__ void p2s_stage_row(const P2sRow& r, _Float16* slot, int tid, float& amax) {
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = tid + kP2sThreads * u;
    if (u == 0 || i < kP2sClips * kP2sWi * kP2sCi / 4) {
      const int c = i / 40, rem = i - 40 * c, col = rem >> 3, c4 = rem & 7;
      uint32_t h01, l01, h23, l23;
      split2_mix(r.v[u].x, r.v[u].y, h01, l01, amax);
      split2_mix(r.v[u].z, r.v[u].w, h23, l23, amax);
      const int o = (c * kP2sWi + col) * kP2sCSI + 4 * c4;
      *reinterpret_cast<uint2*>(slot + o) = uint2{h01, h23};
      *reinterpret_cast<uint2*>(slot + kP2sInPlane + o) = uint2{l01, l23};
    }
  }
}

template <bool LEAKY>
__global__ void __launch_bounds__(kP2sThreads) __attribute__((amdgpu_waves_per_eu(2)))
p2s_chain_kernel(P2sArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char p2smem[];
  _Float16* sm = reinterpret_cast<_Float16*>(p2smem);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int pl = lane & 15, kq = lane >> 4;
  if (tid < 32) sm[kP2sOnes + tid] = static_cast<_Float16>(tid == 0 ? 1.f : 0.f);  // ones (hi, lo), zeros
  const int64_t n_groups = (a.n_img + kP2sClips - 1) / kP2sClips;
  float amax = 0.f;
  const float alpha = a.alpha;
  const _Float16* ones = sm + kP2sOnes;
  // K groups g = 4 ks + kq of stages b, c, d: tap g / 6, channel group g % 6; g >= 18: bias / zeros slot
  auto tap_of = [&](int ks) { return (4 * ks + kq) / 6; };
  auto cg_of = [&](int ks) { return (4 * ks + kq) % 6; };

  if (wave < 3) {  // ---------------- stage a, tile t = wave: positions p = 3 clip + column
    const int t = wave, p = 16 * t + pl, c = p / 3, x = p - 3 * c;
    P2sW<3> W;
#pragma unroll
    for (int mb = 0; mb < 3; ++mb)
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) {
        const _Float16* wp = a.w + (16 * mb + pl) * kP2sKa + 32 * ks + 8 * kq;
        W.h[mb][ks] = *reinterpret_cast<const h8*>(wp);
        W.l[mb][ks] = *reinterpret_cast<const h8*>(wp + kP2sCo * kP2sKa);
      }
    f4 bias[3];
#pragma unroll
    for (int mb = 0; mb < 3; ++mb) {
      const float4 b = *reinterpret_cast<const float4*>(a.bias_a + 16 * mb + 4 * kq);
      bias[mb] = f4{b.x, b.y, b.z, b.w};
    }
    const int base = (c * kP2sWi + x) * kP2sCSI + 8 * kq;  // + 40 ks: column x + ks, channels 8 kq
    for (int64_t gi = blockIdx.x; gi < n_groups; gi += gridDim.x) {
      const int64_t img0 = gi * kP2sClips;
      P2sRow q0, q1;
      p2s_load_row(q0, a, img0, 0, tid);
      p2s_load_row(q1, a, img0, 1, tid);
      p2s_stage_row(q0, sm + kP2sIn, tid, amax);
      p2s_load_row(q0, a, img0, 2, tid);
      __syncthreads();
      for (int y = 0; y < kP2sTicks; ++y) {
        const _Float16* in = sm + kP2sIn + (y & 1) * 2 * kP2sInPlane;
        h8 bh[3], bl[3];
#pragma unroll
        for (int ks = 0; ks < 3; ++ks) {
          bh[ks] = *reinterpret_cast<const h8*>(in + base + kP2sCSI * ks);
          bl[ks] = *reinterpret_cast<const h8*>(in + kP2sInPlane + base + kP2sCSI * ks);
        }
        {  // input row y + 1 (loaded a tick ago) -> the other slot; load row y + 3
          float m = 0.f;
          p2s_stage_row((y & 1) ? q0 : q1, sm + kP2sIn + ((y + 1) & 1) * 2 * kP2sInPlane, tid, m);
          asm("v_max_f32 %0, %0, %1" : "+v"(amax) : "v"(y + 1 < kP2sHin ? m : 0.f));
          if (y & 1) p2s_load_row(q0, a, img0, y + 3, tid);
          else p2s_load_row(q1, a, img0, y + 3, tid);
        }
        f4 acc[3] = {bias[0], bias[1], bias[2]};
#pragma unroll
        for (int ks = 0; ks < 3; ++ks) p2s_mma<3>(acc, W, ks, bh[ks], bl[ks]);
        p2s_store<LEAKY>(acc, sm + kP2sA + (y & 3) * 2 * kP2sAPlane, kP2sAPlane, p, kq, alpha, y < kP2sHin, amax);
        __syncthreads();
      }
    }
  } else if (wave < 6) {  // ---------------- stage b (3x1 on the A ring), tile t = wave - 3
    const int t = wave - 3, p = 16 * t + pl;
    P2sW<5> W;
#pragma unroll
    for (int mb = 0; mb < 3; ++mb)
#pragma unroll
      for (int ks = 0; ks < 5; ++ks) {
        const _Float16* wp = a.w + 2 * kP2sCo * kP2sKa + (16 * mb + pl) * kP2sK + 32 * ks + 8 * kq;
        W.h[mb][ks] = *reinterpret_cast<const h8*>(wp);
        W.l[mb][ks] = *reinterpret_cast<const h8*>(wp + kP2sCo * kP2sK);
      }
    for (int64_t gi = blockIdx.x; gi < n_groups; gi += gridDim.x) {
      const int64_t img0 = gi * kP2sClips;
      P2sRow q0, q1;
      p2s_load_row(q0, a, img0, 0, tid);
      p2s_load_row(q1, a, img0, 1, tid);
      p2s_stage_row(q0, sm + kP2sIn, tid, amax);
      p2s_load_row(q0, a, img0, 2, tid);
      __syncthreads();
      for (int y = 0; y < kP2sTicks; ++y) {
        f4 acc[3] = {};
#pragma unroll
        for (int ks = 0; ks < 5; ++ks) {
          const int tap = tap_of(ks), cg = cg_of(ks);
          const bool bias_slot = 4 * ks + kq >= 18;
          const _Float16* pb = bias_slot ? ones + (kq == 2 ? 0 : 16)
                                         : sm + kP2sA + ((y + 1 + tap) & 3) * 2 * kP2sAPlane + p * kP2sCS + 8 * cg;
          const int lo = bias_slot ? 8 : kP2sAPlane;
          const h8 bh = *reinterpret_cast<const h8*>(pb), bl = *reinterpret_cast<const h8*>(pb + lo);
          p2s_mma<5>(acc, W, ks, bh, bl);
        }
        {
          float m = 0.f;
          p2s_stage_row((y & 1) ? q0 : q1, sm + kP2sIn + ((y + 1) & 1) * 2 * kP2sInPlane, tid, m);
          asm("v_max_f32 %0, %0, %1" : "+v"(amax) : "v"(y + 1 < kP2sHin ? m : 0.f));
          if (y & 1) p2s_load_row(q0, a, img0, y + 3, tid);
          else p2s_load_row(q1, a, img0, y + 3, tid);
        }
        p2s_store<LEAKY>(acc, sm + kP2sB + ((y + 1) & 1) * 2 * kP2sAPlane, kP2sAPlane, p, kq, alpha,
                         y >= 3 && y - 3 < kP2sHin - 2, amax);
        __syncthreads();
      }
    }
  } else {  // ---------------- stage c (wave 6: 1x3 on B) or d (wave 7: 3x1 on the C ring); position = clip
    const bool is_c = wave == 6;
    P2sW<5> W;
#pragma unroll
    for (int mb = 0; mb < 3; ++mb)
#pragma unroll
      for (int ks = 0; ks < 5; ++ks) {
        const _Float16* wp = a.w + 2 * kP2sCo * kP2sKa + (is_c ? 1 : 2) * 2 * kP2sCo * kP2sK + (16 * mb + pl) * kP2sK +
                             32 * ks + 8 * kq;
        W.h[mb][ks] = *reinterpret_cast<const h8*>(wp);
        W.l[mb][ks] = *reinterpret_cast<const h8*>(wp + kP2sCo * kP2sK);
      }
    for (int64_t gi = blockIdx.x; gi < n_groups; gi += gridDim.x) {
      const int64_t img0 = gi * kP2sClips;
      P2sRow q0, q1;
      p2s_load_row(q0, a, img0, 0, tid);
      p2s_load_row(q1, a, img0, 1, tid);
      p2s_stage_row(q0, sm + kP2sIn, tid, amax);
      p2s_load_row(q0, a, img0, 2, tid);
      __syncthreads();
      for (int y = 0; y < kP2sTicks; ++y) {
        f4 acc[3] = {};
#pragma unroll
        for (int ks = 0; ks < 5; ++ks) {
          const int tap = tap_of(ks), cg = cg_of(ks);
          const bool bias_slot = 4 * ks + kq >= 18;
          const _Float16* src;
          int lo;
          if (is_c) {  // B row y - 4, position (clip, tap), channels 8 cg
            src = sm + kP2sB + (y & 1) * 2 * kP2sAPlane + (3 * pl + tap) * kP2sCS + 8 * cg;
            lo = kP2sAPlane;
          } else {     // C ring row y - 7 + tap, position clip
            src = sm + kP2sC + ((y + 1 + tap) & 3) * 2 * kP2sCPlane + pl * kP2sCS + 8 * cg;
            lo = kP2sCPlane;
          }
          const _Float16* pb = bias_slot ? ones + (kq == 2 ? 0 : 16) : src;
          if (bias_slot) lo = 8;
          const h8 bh = *reinterpret_cast<const h8*>(pb), bl = *reinterpret_cast<const h8*>(pb + lo);
          p2s_mma<5>(acc, W, ks, bh, bl);
        }
        {
          float m = 0.f;
          p2s_stage_row((y & 1) ? q0 : q1, sm + kP2sIn + ((y + 1) & 1) * 2 * kP2sInPlane, tid, m);
          asm("v_max_f32 %0, %0, %1" : "+v"(amax) : "v"(y + 1 < kP2sHin ? m : 0.f));
          if (y & 1) p2s_load_row(q0, a, img0, y + 3, tid);
          else p2s_load_row(q1, a, img0, y + 3, tid);
        }
        if (is_c) {
          p2s_store<LEAKY>(acc, sm + kP2sC + (y & 3) * 2 * kP2sCPlane, kP2sCPlane, pl, kq, alpha,
                           y >= 4 && y - 4 < kP2sHin - 2, amax);
        } else if (y >= 7 && y - 7 < kP2sHout && img0 + pl < a.n_img) {
          float* o = a.out + (img0 + pl) * (kP2sHout * kP2sCo) + (y - 7) * kP2sCo + 4 * kq;
#pragma unroll
          for (int mb = 0; mb < 3; ++mb) {
            float v[4] = {acc[mb][0], acc[mb][1], acc[mb][2], acc[mb][3]};
            p0s_act2<LEAKY>(v[0], v[1], alpha);
            p0s_act2<LEAKY>(v[2], v[3], alpha);
            *reinterpret_cast<float4*>(o + 16 * mb) = float4{v[0], v[1], v[2], v[3]};
          }
        }
        __syncthreads();
      }
    }
  }
  raise_range(a.range_flag, amax);
}

// ------------------------------------------------------------------ t3s ----
// Streaming form of SE20's tail (chain 3 over the phase images of the tail
// deduplication): the input pool 2x1 over p2s's 27 x 1 x 48 rows, then
// 3x1 (48 -> 64), 1x1, 3x1, 1x1 (64), 2x1 (64 -> 96), four 1x1 (96; the last
// without activation): 8 x 1 x 96 per phase image. The rows are one position
// wide, so a tile packs IMAGES: 16 positions = 8 clips x 2 phase images
// (position p = image img0 + p, image = 2 clip + phase). The weights are the A
// operand in VGPRs (hi / lo f16), the activations the B operand from LDS rings
// (hi / lo planes [position][channel]); the bias starts the accumulator. Waves
// 0-3 run the four 64-channel stages for output block mb = wave, waves 4-9 the
// five 96-channel stages for mb = wave - 4. Tick y (one barrier after it):
// pooled row y is staged (waves 0-2, loaded a tick ahead), stage s computes its
// row y - kT3Delay[s] (each stage reads only rows written in earlier ticks).
constexpr int kT3Waves = 10, kT3Threads = 64 * kT3Waves, kT3Pos = 16;
constexpr int kT3Hin = 27, kT3C0 = 48, kT3Hp = 13, kT3C1 = 64, kT3C2 = 96, kT3Hout = 8;
constexpr int kT3Ticks = 22;
constexpr int kT3CS0 = 56, kT3CS1 = 72, kT3CS2 = 104;  // f16 per position (odd 16-B groups)
// ring slots (rows) and LDS offsets (f16): P (pooled, 4), A1 (2), A2 (4), A3 (2), A4 (4), A5..A8 (2 each)
constexpr int kT3PlP = kT3Pos * kT3CS0, kT3Pl1 = kT3Pos * kT3CS1, kT3Pl2 = kT3Pos * kT3CS2;
constexpr int kT3P = 0, kT3A1 = kT3P + 4 * 2 * kT3PlP, kT3A2 = kT3A1 + 2 * 2 * kT3Pl1,
              kT3A3 = kT3A2 + 4 * 2 * kT3Pl1, kT3A4 = kT3A3 + 2 * 2 * kT3Pl1, kT3A5 = kT3A4 + 4 * 2 * kT3Pl1;
constexpr int kT3Zero = kT3A5 + 4 * 2 * 2 * kT3Pl2;  // 16 zero halfs (stage 1's K padding)
constexpr int kT3Halfs = kT3Zero + 16;
constexpr int kT3BiasOff = kT3Halfs * 2;            // bytes: biases [4][64] then [5][96] f32
constexpr int kT3Lds = kT3BiasOff + (4 * kT3C1 + 5 * kT3C2) * 4;
// weights (f16, hi plane then lo plane per stage, [cout][K], K = tap * cin + ci)
constexpr int kT3K[9] = {160, 64, 192, 64, 128, 96, 96, 96, 96};  // stage 1: 144 + 16 zero
constexpr int kT3W[9] = {0,
                         2 * 64 * 160,
                         2 * 64 * (160 + 64),
                         2 * 64 * (160 + 64 + 192),
                         2 * 64 * (160 + 64 + 192 + 64),
                         2 * 64 * 480 + 2 * 96 * 128,
                         2 * 64 * 480 + 2 * 96 * (128 + 96),
                         2 * 64 * 480 + 2 * 96 * (128 + 192),
                         2 * 64 * 480 + 2 * 96 * (128 + 288)};
constexpr int kT3WHalfs = 2 * 64 * 480 + 2 * 96 * 512;

struct T3sArgs {
  const float* in;      // [clip][27][48] f32 (p2s output)
  float* out;           // [image][8][96] f32, image = 2 clip + phase
  const _Float16* w;    // kT3WHalfs
  const float* bias;    // [4][64] + [5][96]
  int64_t n_img, src_clip_stride, out_img_stride;
  float alpha;
  int* range_flag;
};

// one output block (16 channels) of one row: KS K-steps of 32, B from the
// ring rows `rows` (tap t -> rows[t]), channel group 8 cg of tap g / (CIN / 8)
template <int KS, int CIN, int CS, int PL>
__device__ __forceinline__ f4 t3_block(const h8 (&wh)[KS], const h8 (&wl)[KS], f4 acc, const _Float16* sm,
                                       const int (&rowoff)[3], int pos, int kq, const _Float16* zero) {
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    const int g = 4 * ks + kq, tap = g / (CIN / 8), cg = g - tap * (CIN / 8);
    const bool pad = tap >= 3;  // stage 1's K padding (groups 18, 19)
    const _Float16* src = pad ? zero : sm + rowoff[tap < 3 ? tap : 0] + pos * CS + 8 * cg;
    const h8 bh = *reinterpret_cast<const h8*>(src), bl = *reinterpret_cast<const h8*>(pad ? zero : src + PL);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[ks], bh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wh[ks], bl, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(wl[ks], bh, acc, 0, 0, 0);
  }
  return acc;
}

// activation, split and ring store of one block's tile (channels 16 mb + 4 kq + j of position pos)
template <bool ACT, int CS, int PL>
__device__ __forceinline__ void t3_store(f4 acc, _Float16* oh, int pos, int mb, int kq, float alpha, float& amax) {
  float v[4] = {acc[0], acc[1], acc[2], acc[3]};
  p0s_act2<ACT>(v[0], v[1], alpha);
  p0s_act2<ACT>(v[2], v[3], alpha);
  uint32_t h01, l01, h23, l23;
  split2_mix(v[0], v[1], h01, l01, amax);
  split2_mix(v[2], v[3], h23, l23, amax);
  const int o = pos * CS + 16 * mb + 4 * kq;
  *reinterpret_cast<uint2*>(oh + o) = uint2{h01, h23};
  *reinterpret_cast<uint2*>(oh + PL + o) = uint2{l01, l23};
}

template <int KS, int K>
__device__ __forceinline__ void t3_load_w(h8 (&wh)[KS], h8 (&wl)[KS], const _Float16* w, int cout, int n, int kq) {
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    wh[ks] = *reinterpret_cast<const h8*>(w + n * K + 32 * ks + 8 * kq);
    wl[ks] = *reinterpret_cast<const h8*>(w + cout * K + n * K + 32 * ks + 8 * kq);
  }
}

__device__ __forceinline__ f4 t3_bias(const float* b) {
  const float4 v = *reinterpret_cast<const float4*>(b);
  return f4{v.x, v.y, v.z, v.w};
}

template <bool LEAKY>
__global__ void __launch_bounds__(kT3Threads) __attribute__((amdgpu_waves_per_eu(3)))
t3s_chain_kernel(T3sArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char t3smem[];
  _Float16* sm = reinterpret_cast<_Float16*>(t3smem);
  float* sb = reinterpret_cast<float*>(t3smem + kT3BiasOff);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int pos = lane & 15, kq = lane >> 4;
  for (int i = tid; i < 16; i += kT3Threads) sm[kT3Zero + i] = static_cast<_Float16>(0.f);
  for (int i = tid; i < 4 * kT3C1 + 5 * kT3C2; i += kT3Threads) sb[i] = a.bias[i];
  const _Float16* zero = sm + kT3Zero;
  const int64_t n_groups = (a.n_img + kT3Pos - 1) / kT3Pos;
  const float alpha = a.alpha;
  float amax = 0.f;
  // staging: threads 0..191 take 4 channels (c4) of position sp
  const int sp = tid / 12, c4 = tid - 12 * sp;
  const bool stager = tid < kT3Pos * 12;
  float4 r0 = {0.f, 0.f, 0.f, 0.f}, r1 = r0;
  auto load_row = [&](int64_t img0, int y) {  // pooled row y's two source rows, this thread's share
    const int64_t img = min(img0 + sp, a.n_img - 1);
    const int64_t clip = img >> 1;
    const int row = static_cast<int>(img & 1) + 2 * min(y, kT3Hp - 1);
    const float* src = a.in + clip * a.src_clip_stride + row * kT3C0 + 4 * c4;
    r0 = *reinterpret_cast<const float4*>(src);
    r1 = *reinterpret_cast<const float4*>(src + kT3C0);
  };
  auto stage_row = [&](int y) {
    const float4 v = {nan_max(r0.x, r1.x), nan_max(r0.y, r1.y), nan_max(r0.z, r1.z), nan_max(r0.w, r1.w)};
    uint32_t h01, l01, h23, l23;
    split2_mix(v.x, v.y, h01, l01, amax);
    split2_mix(v.z, v.w, h23, l23, amax);
    _Float16* d = sm + kT3P + (y & 3) * 2 * kT3PlP + sp * kT3CS0 + 4 * c4;
    *reinterpret_cast<uint2*>(d) = uint2{h01, h23};
    *reinterpret_cast<uint2*>(d + kT3PlP) = uint2{l01, l23};
  };
  __syncthreads();

  if (wave < 4) {  // ---------------- the 64-channel stages, block mb = wave
    const int mb = wave, n = 16 * mb + pos;
    h8 w1h[5], w1l[5], w2h[2], w2l[2], w3h[6], w3l[6], w4h[2], w4l[2];
    t3_load_w<5, 160>(w1h, w1l, a.w + kT3W[0], kT3C1, n, kq);
    t3_load_w<2, 64>(w2h, w2l, a.w + kT3W[1], kT3C1, n, kq);
    t3_load_w<6, 192>(w3h, w3l, a.w + kT3W[2], kT3C1, n, kq);
    t3_load_w<2, 64>(w4h, w4l, a.w + kT3W[3], kT3C1, n, kq);
    const int bo = 16 * mb + 4 * kq;
    for (int64_t gi = blockIdx.x; gi < n_groups; gi += gridDim.x) {
      const int64_t img0 = gi * kT3Pos;
      if (stager) load_row(img0, 0);
      for (int y = 0; y < kT3Ticks; ++y) {
        if (stager && y < kT3Hp) {
          stage_row(y);
          load_row(img0, y + 1);
        }
        if (y >= 3 && y < 3 + 11) {  // stage 1: row r from pooled rows r .. r + 2
          const int r = y - 3;
          const int ro[3] = {kT3P + (r & 3) * 2 * kT3PlP, kT3P + ((r + 1) & 3) * 2 * kT3PlP,
                             kT3P + ((r + 2) & 3) * 2 * kT3PlP};
          const f4 acc = t3_block<5, kT3C0, kT3CS0, kT3PlP>(w1h, w1l, t3_bias(sb + bo), sm, ro, pos, kq, zero);
          t3_store<LEAKY, kT3CS1, kT3Pl1>(acc, sm + kT3A1 + (r & 1) * 2 * kT3Pl1, pos, mb, kq, alpha, amax);
        }
        if (y >= 4 && y < 4 + 11) {  // stage 2 (1x1)
          const int r = y - 4;
          const int ro[3] = {kT3A1 + (r & 1) * 2 * kT3Pl1, 0, 0};
          const f4 acc = t3_block<2, kT3C1, kT3CS1, kT3Pl1>(w2h, w2l, t3_bias(sb + kT3C1 + bo), sm, ro, pos, kq, zero);
          t3_store<LEAKY, kT3CS1, kT3Pl1>(acc, sm + kT3A2 + (r & 3) * 2 * kT3Pl1, pos, mb, kq, alpha, amax);
        }
        if (y >= 7 && y < 7 + 9) {  // stage 3 (3x1)
          const int r = y - 7;
          const int ro[3] = {kT3A2 + (r & 3) * 2 * kT3Pl1, kT3A2 + ((r + 1) & 3) * 2 * kT3Pl1,
                             kT3A2 + ((r + 2) & 3) * 2 * kT3Pl1};
          const f4 acc = t3_block<6, kT3C1, kT3CS1, kT3Pl1>(w3h, w3l, t3_bias(sb + 2 * kT3C1 + bo), sm, ro, pos, kq,
                                                           zero);
          t3_store<LEAKY, kT3CS1, kT3Pl1>(acc, sm + kT3A3 + (r & 1) * 2 * kT3Pl1, pos, mb, kq, alpha, amax);
        }
        if (y >= 8 && y < 8 + 9) {  // stage 4 (1x1)
          const int r = y - 8;
          const int ro[3] = {kT3A3 + (r & 1) * 2 * kT3Pl1, 0, 0};
          const f4 acc = t3_block<2, kT3C1, kT3CS1, kT3Pl1>(w4h, w4l, t3_bias(sb + 3 * kT3C1 + bo), sm, ro, pos, kq,
                                                           zero);
          t3_store<LEAKY, kT3CS1, kT3Pl1>(acc, sm + kT3A4 + (r & 3) * 2 * kT3Pl1, pos, mb, kq, alpha, amax);
        }
        __syncthreads();
      }
    }
  } else {  // ---------------- the 96-channel stages, block mb = wave - 4
    const int mb = wave - 4, n = 16 * mb + pos;
    h8 w5h[4], w5l[4], w6h[3], w6l[3], w7h[3], w7l[3], w8h[3], w8l[3], w9h[3], w9l[3];
    t3_load_w<4, 128>(w5h, w5l, a.w + kT3W[4], kT3C2, n, kq);
    t3_load_w<3, 96>(w6h, w6l, a.w + kT3W[5], kT3C2, n, kq);
    t3_load_w<3, 96>(w7h, w7l, a.w + kT3W[6], kT3C2, n, kq);
    t3_load_w<3, 96>(w8h, w8l, a.w + kT3W[7], kT3C2, n, kq);
    t3_load_w<3, 96>(w9h, w9l, a.w + kT3W[8], kT3C2, n, kq);
    const float* bb = sb + 4 * kT3C1 + 16 * mb + 4 * kq;
    constexpr int A5 = kT3A5, A6 = A5 + 2 * 2 * kT3Pl2, A7 = A6 + 2 * 2 * kT3Pl2, A8 = A7 + 2 * 2 * kT3Pl2;
    for (int64_t gi = blockIdx.x; gi < n_groups; gi += gridDim.x) {
      const int64_t img0 = gi * kT3Pos;
      for (int y = 0; y < kT3Ticks; ++y) {
        if (y >= 10 && y < 10 + 8) {  // stage 5 (2x1, 64 -> 96) from rows r, r + 1 of A4
          const int r = y - 10;
          const int ro[3] = {kT3A4 + (r & 3) * 2 * kT3Pl1, kT3A4 + ((r + 1) & 3) * 2 * kT3Pl1, 0};
          const f4 acc = t3_block<4, kT3C1, kT3CS1, kT3Pl1>(w5h, w5l, t3_bias(bb), sm, ro, pos, kq, zero);
          t3_store<LEAKY, kT3CS2, kT3Pl2>(acc, sm + A5 + (r & 1) * 2 * kT3Pl2, pos, mb, kq, alpha, amax);
        }
        if (y >= 11 && y < 11 + 8) {  // stage 6
          const int r = y - 11;
          const int ro[3] = {A5 + (r & 1) * 2 * kT3Pl2, 0, 0};
          const f4 acc = t3_block<3, kT3C2, kT3CS2, kT3Pl2>(w6h, w6l, t3_bias(bb + kT3C2), sm, ro, pos, kq, zero);
          t3_store<LEAKY, kT3CS2, kT3Pl2>(acc, sm + A6 + (r & 1) * 2 * kT3Pl2, pos, mb, kq, alpha, amax);
        }
        if (y >= 12 && y < 12 + 8) {  // stage 7
          const int r = y - 12;
          const int ro[3] = {A6 + (r & 1) * 2 * kT3Pl2, 0, 0};
          const f4 acc = t3_block<3, kT3C2, kT3CS2, kT3Pl2>(w7h, w7l, t3_bias(bb + 2 * kT3C2), sm, ro, pos, kq, zero);
          t3_store<LEAKY, kT3CS2, kT3Pl2>(acc, sm + A7 + (r & 1) * 2 * kT3Pl2, pos, mb, kq, alpha, amax);
        }
        if (y >= 13 && y < 13 + 8) {  // stage 8
          const int r = y - 13;
          const int ro[3] = {A7 + (r & 1) * 2 * kT3Pl2, 0, 0};
          const f4 acc = t3_block<3, kT3C2, kT3CS2, kT3Pl2>(w8h, w8l, t3_bias(bb + 3 * kT3C2), sm, ro, pos, kq, zero);
          t3_store<LEAKY, kT3CS2, kT3Pl2>(acc, sm + A8 + (r & 1) * 2 * kT3Pl2, pos, mb, kq, alpha, amax);
        }
        if (y >= 14 && y < 14 + 8) {  // stage 9 (no activation) -> out
          const int r = y - 14;
          const int ro[3] = {A8 + (r & 1) * 2 * kT3Pl2, 0, 0};
          const f4 acc = t3_block<3, kT3C2, kT3CS2, kT3Pl2>(w9h, w9l, t3_bias(bb + 4 * kT3C2), sm, ro, pos, kq, zero);
          if (img0 + pos < a.n_img) {
            float* o = a.out + (img0 + pos) * a.out_img_stride + r * kT3C2 + 16 * mb + 4 * kq;
            *reinterpret_cast<float4*>(o) = float4{acc[0], acc[1], acc[2], acc[3]};
          }
        }
        __syncthreads();
      }
    }
  }
  raise_range(a.range_flag, amax);
}

// ------------------------------------------------------------------ host ----

struct OpInfo {
  int kind, kh, kw, cin, cout, act;
  float alpha;
  std::vector<float> w, b;  // HWIO, [cout]
};

struct Dims {
  int h, w, c;
};

using KernelFn = void (*)(ChainArgs);

struct ChainPlan {
  ChainArgs args{};
  bool split = false;        // split-f16 kernel (XArgs x) instead of the exact one
  XArgs x{};
  int nb = 1;
  bool wg = false;
  KernelFn fn = nullptr;
  void (*xfn)(XArgs) = nullptr;
  size_t lds_bytes = 0;
  float* d_blob = nullptr;
  int src_buf = -1;          // -1: the call's input, else workspace buffer index
  int dst_buf = -1;          // -1: the call's output
  int64_t out_floats = 0;    // per source clip (clip path) or per window
  double macs_per_img = 0;   // algorithmic MACs per image of this chain
  // pattern kernel (p0_chain_kernel) for this chain, if it matches; the split
  // plan above stays as the fallback for unaligned buffers
  void (*p0fn)(P0Args) = nullptr;
  P0Args p0{};
  bool p0s = false;  // p0fn is the streaming p0s_chain_kernel (one wave per image)
  bool p1s = false;  // p1fn is the streaming p1s_chain_kernel (one wave per image)
  void (*p2fn)(P2sArgs) = nullptr;  // p2s pattern (SE20 chain 2; shares d_p0 / p0_lds / p0_blocks_per_cu)
  P2sArgs p2{};
  void (*p1fn)(P1Args) = nullptr;  // p1 pattern (shares d_p0 / p0_lds / p0_blocks_per_cu)
  P1Args p1{};
  void (*t3fn)(T3sArgs) = nullptr;  // t3s pattern (SE20's deduplicated tail; shares d_p0 / p0_lds / ...)
  T3sArgs t3{};
  size_t p0_lds = 0;
  int p0_blocks_per_cu = 0;
  void* d_p0 = nullptr;
};

struct Program {
  std::vector<ChainPlan> chains;
  int64_t buf_floats[2] = {0, 0};  // per unit (clip or window)
  // phase-deduplicated tail: the last chain writes [n_src rows][out_dim] per clip
  // into workspace buffer gather_buf; output row i is source row gather_src[i]
  int gather_buf = -1, n_src = 0;
  std::vector<int> gather_src;
  int* d_gather = nullptr;
};

template <int NB, int RB, bool WG>
KernelFn kernel_for() {
  return conv_chain_kernel<NB, RB, WG>;
}

KernelFn pick_kernel(int nb, bool wg) {
  // RB x NB accumulators of 4 VGPRs: keep RB * NB <= 12
  switch (nb) {
    case 1: return wg ? kernel_for<1, 4, true>() : kernel_for<1, 4, false>();
    case 2: return wg ? kernel_for<2, 4, true>() : kernel_for<2, 4, false>();
    case 3: return wg ? kernel_for<3, 4, true>() : kernel_for<3, 4, false>();
    case 4: return wg ? kernel_for<4, 2, true>() : kernel_for<4, 2, false>();
    case 5: return wg ? kernel_for<5, 2, true>() : kernel_for<5, 2, false>();
    default: return wg ? kernel_for<6, 2, true>() : kernel_for<6, 2, false>();
  }
}

inline int odd_pad(int c) { return (c % 2 == 0) ? c + 1 : c; }

}  // namespace
}  // namespace hbk

struct hbk_embed_plan {
  std::vector<hbk::OpInfo> ops;
  int in_h = 0, in_w = 0, out_dim = 0;
  std::vector<int> starts;
  int n_prefix = 0;
  int seq_frames = 0;
  int split_stride = 1;
  bool split_f16 = true;
  double prefix_macs = 0, tail_macs = 0;
  hbk::Program clip_prog, win_prog;
  int* d_range = nullptr;  // range flag of the split-f16 kernels (hbk_embed_range_status)
};

namespace hbk {
namespace {

// fp16 elements per position for c channels: rounded up to 8, with an odd
// number of 16-B groups (conflict-free ds_read_b128 over consecutive positions).
inline int x_cs(int c) {
  int cs = (c + 7) & ~7;
  if ((cs / 8) % 2 == 0) cs += 8;
  return cs;
}

using XKernelFn = void (*)(XArgs);

template <int NBMAX, bool WG>
XKernelFn xkernel_for() {
  return conv_chain_x3_kernel<NBMAX, WG>;
}

XKernelFn pick_xkernel(int nb, bool wg) {
  switch (nb) {
    case 1: return wg ? xkernel_for<1, true>() : xkernel_for<1, false>();
    case 2: return wg ? xkernel_for<2, true>() : xkernel_for<2, false>();
    case 3: return wg ? xkernel_for<3, true>() : xkernel_for<3, false>();
    default: return wg ? xkernel_for<4, true>() : xkernel_for<4, false>();  // > 3 blocks: groups of 3
  }
}

// Dynamic-LDS limit of a kernel raised to what the CU holds beside its static
// LDS (set once to the maximum, so plans sharing the kernel never lower it).
hipError_t set_max_dynamic_lds(const void* fn) {
  hipFuncAttributes at;
  hipError_t e = hipFuncGetAttributes(&at, fn);
  if (e != hipSuccess) return e;
  return hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                             int(160 * 1024 - static_cast<int>(at.sharedSizeBytes)));
}

// Split-f16 layout of one chain whose source / pooling fields are already in
// `a`: packs the fp16 weight planes, biases and group-offset tables, and picks
// images-per-task and band for the LDS budget.
int layout_split(const std::vector<OpInfo>& ops, const std::vector<int>& stage_ops, Dims d,
                 const ChainArgs& a, ChainPlan& cp, Dims& od_out) {
  XArgs& x = cp.x;
  // LDS per block (default 78 KB: two blocks per CU); HBK_EMBED_LDS_KB for tuning
  // (a chain that fits fewer than kMinG whole images per task at that budget
  // takes a whole CU instead: measured on SE20's chain 2, 2 -> 6 images,
  // 0.96 -> 0.81 ms per 16384 clips; the tail chain, 30 images, keeps 2 / CU)
  constexpr int kMinG = 8;
  const char* lds_env = getenv("HBK_EMBED_LDS_KB");
  int64_t lds_budget = kLdsBudget;
  if (lds_env) lds_budget = std::min<int64_t>(160, std::max(16, atoi(lds_env))) * 1024;
  x.ipc = a.ipc;
  for (int k = 0; k < kMaxWin; ++k) x.row_off[k] = a.row_off[k];
  x.src_clip_stride = a.src_clip_stride;
  x.src_row_stride = a.src_row_stride;
  x.C_src = a.C_src;
  x.in_ph = a.in_ph;
  x.in_pw = a.in_pw;
  x.W_in = a.W_in;
  x.out_ph = a.out_ph;
  x.out_pw = a.out_pw;
  x.n_stages = static_cast<int>(stage_ops.size());
  x.shrink = 0;
  x.im2col = (d.c % 8) != 0;

  std::vector<_Float16> wb;  // hi/lo planes per stage
  std::vector<float> bb;
  std::vector<int> kt;
  int cin = d.c, h = d.h, w = d.w, nbmax = 1;
  double macs = 0;
  for (int s = 0; s < x.n_stages; ++s) {
    const OpInfo& op = ops[stage_ops[s]];
    if (op.cin != cin) {
      set_error("hbk: graph channel mismatch at op %d (%d != %d)", stage_ops[s], op.cin, cin);
      return HBK_ERR_ARG;
    }
    XStage& S = x.st[s];
    S.kh = op.kh;
    S.kw = op.kw;
    S.cin = op.cin;
    S.cout = op.cout;
    S.coutr = (op.cout + 7) & ~7;
    S.act = op.act ? ((op.alpha >= 0.f && op.alpha <= 1.f) ? 1 : 2) : 0;
    S.alpha = op.alpha;
    const bool i2c = x.im2col && s == 0;
    const int K0 = op.kh * op.kw * op.cin;
    const int cin8 = (op.cin + 7) & ~7;
    const int groups = i2c ? (K0 + 7) / 8 : op.kh * op.kw * cin8 / 8;
    S.cs_in = i2c ? x_cs(K0) : x_cs(op.cin);
    S.cs_out = x_cs(op.cout);
    S.ksteps = (groups + 1) / 2;
    S.nblk = (op.cout + 31) / 32;
    nbmax = std::max(nbmax, S.nblk);
    S.wrow = S.ksteps * 16 + 8;
    const int wo_in = w;  // this stage's input width (group offsets)
    h -= op.kh - 1;
    w -= op.kw - 1;
    x.shrink += op.kh - 1;
    if (h <= 0 || w <= 0) {
      set_error("hbk: graph collapses the image at op %d", stage_ops[s]);
      return HBK_ERR_ARG;
    }
    macs += double(h) * w * op.cout * K0;
    // weights [n][k] (k = group * 8 + j), hi then lo plane
    const int rows = S.nblk * 32;
    S.w_off = static_cast<int>(wb.size());
    S.w_lo = rows * S.wrow;
    wb.resize(wb.size() + size_t(2) * rows * S.wrow, static_cast<_Float16>(0.f));
    for (int n = 0; n < op.cout; ++n)
      for (int k = 0; k < S.ksteps * 16; ++k) {
        const int g = k / 8, j = k - g * 8;
        int src = -1;  // index into HWIO weights (k' = tap * cin + ci)
        if (i2c) {
          if (k < K0) src = k;
        } else if (g < groups) {
          const int tap = g / (cin8 / 8), ci = (g - tap * (cin8 / 8)) * 8 + j;
          if (ci < op.cin) src = tap * op.cin + ci;
        }
        if (src < 0) continue;
        const float v = op.w[size_t(src) * op.cout + n];
        uint32_t bits;
        memcpy(&bits, &v, 4);
        bits &= 0xFFFFE000u;  // hi: v rounded toward zero to 11 bits, as on the device
        float hv;
        memcpy(&hv, &bits, 4);
        wb[S.w_off + size_t(n) * S.wrow + k] = static_cast<_Float16>(hv);
        wb[S.w_off + S.w_lo + size_t(n) * S.wrow + k] = static_cast<_Float16>(v - hv);
      }
    S.b_off = static_cast<int>(bb.size());
    for (int n = 0; n < rows; ++n) bb.push_back(n < op.cout ? op.b[n] : 0.f);
    // group offsets (fp16 elements into the stage's input tensor); pad groups read offset 0
    S.kt_off = static_cast<int>(kt.size());
    for (int g = 0; g < 2 * S.ksteps; ++g) {
      int v = 0;
      if (g < groups) {
        if (i2c) {
          v = g * 8;
        } else {
          const int tap = g / (cin8 / 8), cg = g - tap * (cin8 / 8);
          const int dh = tap / op.kw, dw = tap - dh * op.kw;
          v = (dh * wo_in + dw) * S.cs_in + cg * 8;
        }
      }
      kt.push_back(v);
    }
    cin = op.cout;
  }
  x.cs0 = x.st[0].cs_in;
  cp.nb = nbmax;
  std::vector<int> i2c;  // im2col tap offsets into the raw rows (stage-0 input width)
  if (x.im2col) {
    const XStage& S = x.st[0];
    for (int dh = 0; dh < S.kh; ++dh)
      for (int dw = 0; dw < S.kw; ++dw)
        for (int ci = 0; ci < S.cin; ++ci) i2c.push_back((dh * d.w + dw) * S.cin + ci);
  }
  i2c.push_back(0);
  const Dims od{h / x.out_ph, w / x.out_pw, cin};
  if (od.h <= 0 || od.w <= 0) {
    set_error("hbk: pooling collapses the image");
    return HBK_ERR_ARG;
  }
  x.H_out = od.h;
  x.W_out = od.w;
  x.C_out = od.c;
  x.out_img_stride = int64_t(od.h) * od.w * od.c;
  x.kt_n = static_cast<int>(kt.size());
  while (wb.size() % 8) wb.push_back(static_cast<_Float16>(0.f));

  // LDS: tensor t (stage t input; t = n_stages: last output) alternates X / Y
  auto region_bytes = [&](int G, int band, int64_t& xb, int64_t& yb) {
    const int n = x.n_stages;
    std::vector<int> rows(n + 1), wid(n + 1);
    rows[n] = band * x.out_ph;
    wid[0] = d.w;
    for (int s = 0; s < n; ++s) wid[s + 1] = wid[s] - (x.st[s].kw - 1);
    for (int s = n - 1; s >= 0; --s) rows[s] = rows[s + 1] + x.st[s].kh - 1;
    xb = yb = 0;
    for (int t = 0; t <= n; ++t) {
      int64_t bytes;
      if (t == 0 && x.im2col)  // stage 0 input = im2col tensor at its output geometry
        bytes = int64_t(G) * rows[1] * wid[1] * x.st[0].cs_in * 4;
      else
        bytes = int64_t(G) * rows[t] * wid[t] * (t == 0 ? x.st[0].cs_in : x.st[t - 1].cs_out) * 4;
      int64_t& r = (t % 2 == 0) ? xb : yb;
      r = std::max(r, bytes);
    }
    if (x.im2col) yb = std::max(yb, int64_t(G) * rows[0] * wid[0] * d.c * 4);  // raw f32 rows
    xb = (xb + 15) & ~int64_t(15);
    yb = (yb + 15) & ~int64_t(15);
  };
  const int64_t w_bytes = int64_t(wb.size()) * 2, k_bytes = (int64_t(kt.size()) * 4 + 15) & ~int64_t(15);
  const int64_t b_bytes = int64_t(bb.size()) * 4;  // multiple of 128
  auto lds_total = [&](int G, int band, bool resident) {
    int64_t xb, yb;
    region_bytes(G, band, xb, yb);
    return xb + yb + (resident ? w_bytes : 0) + b_bytes + k_bytes;
  };
  // MACs computed per output row of the whole image for a band of b rows
  // (halo rows recomputed by every band): useful / computed = efficiency.
  auto efficiency = [&](int b) {
    const int n = x.n_stages, nb = (od.h + b - 1) / b;
    double useful = 0, done = 0;
    int rows_b = b * x.out_ph, rows_full = od.h * x.out_ph;
    for (int s = n - 1; s >= 0; --s) {
      const XStage& S = x.st[s];
      int wo = d.w;
      for (int q = 0; q <= s; ++q) wo -= x.st[q].kw - 1;
      const double per_row = double(wo) * S.cout * S.kh * S.kw * S.cin;
      useful += per_row * rows_full;
      done += per_row * rows_b * nb;
      rows_b += S.kh - 1;
      rows_full += S.kh - 1;
    }
    return useful / done;
  };
  auto best_band = [&](bool res) {
    for (int b = od.h; b >= 1; --b)
      if (lds_total(1, b, res) <= lds_budget) return b;
    return 0;
  };
  bool resident = false;
  int band = 0, G = 1;
  for (int attempt = 0; attempt < 2; ++attempt) {
    // resident weights unless they cost more than 5 % of the work in halo rows
    // (HBK_EMBED_WEIGHTS=lds|global overrides, for tuning)
    const int band_r = lds_total(1, 1, true) <= lds_budget ? best_band(true) : 0;
    const int band_g = best_band(false);
    resident = band_r > 0 && (band_g == 0 || efficiency(band_r) >= 0.95 * efficiency(band_g));
    if (const char* wp = getenv("HBK_EMBED_WEIGHTS")) {
      if (!strcmp(wp, "global") && band_g > 0) resident = false;
      if (!strcmp(wp, "lds") && band_r > 0) resident = true;
    }
    band = resident ? band_r : band_g;
    G = 1;
    if (band == 0) {
      set_error("hbk: one output row of a chain does not fit in LDS");
      return HBK_ERR_UNSUPPORTED;
    }
    if (band == od.h)
      while (G < 64 && lds_total(G + 1, band, resident) <= lds_budget) ++G;  // any G: fill the LDS budget
    if (attempt == 0 && !lds_env && band == od.h && G < kMinG) {
      lds_budget = kLdsBudgetCU;
      continue;
    }
    break;
  }
  x.G = G;
  x.band = band;
  x.n_bands = (od.h + band - 1) / band;
  int64_t xb, yb;
  region_bytes(G, band, xb, yb);
  x.lds_x = 0;
  x.lds_y = static_cast<int>(xb);
  x.lds_w = static_cast<int>(xb + yb);
  x.lds_b = x.lds_w + static_cast<int>(resident ? w_bytes : 0);
  x.lds_k = x.lds_b + static_cast<int>(b_bytes);
  x.w_halfs = resident ? static_cast<int>(wb.size()) : 0;
  x.b_floats = static_cast<int>(bb.size());
  x.vec_out = od.c % 4 == 0;  // cleared at launch for an unaligned output
  x.raw_vec = x.im2col && x.in_pw == 1 && (x.W_in * x.C_src) % 4 == 0;  // and at launch: alignment
  cp.lds_bytes = size_t(x.lds_k + k_bytes);
  cp.wg = !resident;
  cp.split = true;
  cp.xfn = pick_xkernel(nbmax, cp.wg);
  // device blob: weights (fp16), biases (f32), group offsets (int)
  const size_t wsz = wb.size() * 2, bsz = ((bb.size() * 4 + 15) & ~size_t(15));
  const size_t ksz = (kt.size() * 4 + 15) & ~size_t(15), isz = i2c.size() * 4;
  hipError_t e = hipMalloc(reinterpret_cast<void**>(&cp.d_blob), wsz + bsz + ksz + isz);
  if (e != hipSuccess) return hip_error(e, "hipMalloc chain weights");
  unsigned char* base = reinterpret_cast<unsigned char*>(cp.d_blob);
  e = hipMemcpy(base, wb.data(), wsz, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(base + wsz, bb.data(), bb.size() * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(base + wsz + bsz, kt.data(), kt.size() * 4, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(base + wsz + bsz + ksz, i2c.data(), isz, hipMemcpyHostToDevice);
  if (e != hipSuccess) return hip_error(e, "copy chain weights");
  x.wblob = reinterpret_cast<const _Float16*>(base);
  x.bblob = reinterpret_cast<const float*>(base + wsz);
  x.ktab = reinterpret_cast<const int*>(base + wsz + bsz);
  x.i2c_off = reinterpret_cast<const int*>(base + wsz + bsz + ksz);
  x.i2c_n = static_cast<int>(i2c.size());
  if (cp.lds_bytes > 64 * 1024) {  // the CU maximum: chains sharing a kernel never lower it
    e = set_max_dynamic_lds(reinterpret_cast<const void*>(cp.xfn));
    if (e != hipSuccess) return hip_error(e, "hipFuncSetAttribute(max dynamic LDS)");
  }
  cp.macs_per_img = macs;
  od_out = od;
  if (getenv("HBK_DEBUG_EMBED"))
    fprintf(stderr, "hbk split chain: %d stages, in %dx%dx%d (pool %dx%d, im2col %d) -> %dx%dx%d (pool %dx%d); "
            "G %d band %d/%d (eff %.3f), weights %s %lld B, LDS %zu B, nb %d\n",
            x.n_stages, d.h, d.w, d.c, x.in_ph, x.in_pw, x.im2col, od.h, od.w, od.c, x.out_ph, x.out_pw, G,
            band, od.h, efficiency(band), resident ? "LDS" : "global", (long long)w_bytes, cp.lds_bytes, nbmax);
  return HBK_OK;
}

// The p0 pattern: [3x3 (1 -> C), 1x3 (C -> C), 3x1 (C -> C)] + output pool 2x2
// on input width 32, C = 24, one image per source clip; all convs LeakyReLU
// with one slope in [0, 1], or all linear. Packs the weights / biases and
// sizes the grid; returns false (generic kernel) when the chain differs.
constexpr int kP0W = 32, kP0C = 24;

template <int kP0Band>
bool plan_p0_band(const std::vector<OpInfo>& ops, const std::vector<int>& st, const ChainArgs& a, Dims d, Dims od,
                  ChainPlan& cp) {
  using P0G = P0Geo<kP0W, kP0C, kP0Band>;
  if (st.size() != 3 || a.ipc != 1 || a.C_src != 1 || a.in_ph != 1 || a.in_pw != 1) return false;
  if (a.out_ph != 2 || a.out_pw != 2 || d.w != kP0W || a.src_row_stride != kP0W) return false;
  const OpInfo &o0 = ops[st[0]], &o1 = ops[st[1]], &o2 = ops[st[2]];
  const int C = kP0C;
  if (!(o0.kh == 3 && o0.kw == 3 && o0.cin == 1 && o0.cout == C)) return false;
  if (!(o1.kh == 1 && o1.kw == 3 && o1.cin == C && o1.cout == C)) return false;
  if (!(o2.kh == 3 && o2.kw == 1 && o2.cin == C && o2.cout == C)) return false;
  const bool leaky = o0.act != 0;
  for (const OpInfo* o : {&o0, &o1, &o2}) {
    if ((o->act != 0) != leaky) return false;
    if (leaky && (o->alpha != o0.alpha || !(o->alpha >= 0.f && o->alpha <= 1.f))) return false;
  }
  if (od.h != (d.h - 4) / 2 || od.w != (d.w - 4) / 2 || od.c != C) return false;
  // weights: stage s = hi [32][16 ks_s] then lo; K of stage 0 = taps 0-4 | pad | taps 5-8 | pad
  std::vector<_Float16> w(P0G::WHALFS, static_cast<_Float16>(0.f));
  auto put = [&](int off, int ks, int n, int k, float v) {
    uint32_t bits;
    memcpy(&bits, &v, 4);
    bits &= 0xFFFFE000u;
    float hv;
    memcpy(&hv, &bits, 4);
    w[off + n * 16 * ks + k] = static_cast<_Float16>(hv);
    w[off + 32 * 16 * ks + n * 16 * ks + k] = static_cast<_Float16>(v - hv);
  };
  for (int n = 0; n < C; ++n) {
    for (int k = 0; k < 16; ++k) {
      const int tap = k < 5 ? k : (k >= 8 && k < 12 ? k - 3 : -1);
      if (tap >= 0) put(0, 1, n, k, o0.w[size_t(tap) * C + n]);
    }
    for (int k = 0; k < 3 * C; ++k) {
      put(P0G::WOFF1, P0G::KS, n, k, o1.w[size_t(k) * C + n]);  // HWIO: (tap * C + ci) * C + n
      put(P0G::WOFF2, P0G::KS, n, k, o2.w[size_t(k) * C + n]);
    }
  }
  std::vector<float> b(96, 0.f);
  for (int n = 0; n < C; ++n) {
    b[n] = o0.b[n];
    b[32 + n] = o1.b[n];
    b[64 + n] = o2.b[n];
  }
  const size_t wbytes = (w.size() * 2 + 15) & ~size_t(15);
  hipError_t e = hipMalloc(&cp.d_p0, wbytes + b.size() * 4);
  if (e == hipSuccess) e = hipMemcpy(cp.d_p0, w.data(), w.size() * 2, hipMemcpyHostToDevice);
  if (e == hipSuccess)
    e = hipMemcpy(static_cast<unsigned char*>(cp.d_p0) + wbytes, b.data(), b.size() * 4, hipMemcpyHostToDevice);
  cp.p0fn = leaky ? p0_chain_kernel<kP0W, kP0C, kP0Band, true> : p0_chain_kernel<kP0W, kP0C, kP0Band, false>;
  cp.p0_lds = P0G::LDS;
  if (e == hipSuccess)
    e = hipFuncSetAttribute(reinterpret_cast<const void*>(cp.p0fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                            int(cp.p0_lds));
  int per_cu = 0;
  if (e == hipSuccess)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(cp.p0fn), kP0Threads,
                                                     cp.p0_lds);
  if (e != hipSuccess || per_cu < 1) {
    (void)hipGetLastError();
    if (cp.d_p0) (void)hipFree(cp.d_p0);
    cp.d_p0 = nullptr;
    cp.p0fn = nullptr;
    return false;
  }
  cp.p0_blocks_per_cu = per_cu;
  P0Args& p = cp.p0;
  p.w = static_cast<const _Float16*>(cp.d_p0);
  p.bias = reinterpret_cast<const float*>(static_cast<unsigned char*>(cp.d_p0) + wbytes);
  p.H_in = d.h;
  p.H_out = od.h;
  p.n_bands = (od.h + kP0Band - 1) / kP0Band;
  p.alpha = leaky ? o0.alpha : 0.f;
  if (getenv("HBK_DEBUG_EMBED"))
    fprintf(stderr, "hbk p0 chain: %dx%dx1 -> %dx%dx%d, band %d (%d bands), LDS %zu B, %d blocks/CU\n", d.h, d.w,
            od.h, od.w, od.c, kP0Band, p.n_bands, cp.p0_lds, per_cu);
  return true;
}

// The streaming p0 form (p0s_chain_kernel): the same chain on a 136-row input,
// one wave per clip. Weights as plan_p0_band's (hi / lo of 16 W rounded toward
// zero), with each stage's bias in K slot 12 (stage 0) or 72 (stages 1, 2).
bool plan_p0s(const std::vector<OpInfo>& ops, const std::vector<int>& st, const ChainArgs& a, Dims d, Dims od,
              ChainPlan& cp) {
  if (getenv("HBK_EMBED_NO_P0S")) return false;
  if (st.size() != 3 || a.ipc != 1 || a.C_src != 1 || a.in_ph != 1 || a.in_pw != 1) return false;
  if (a.out_ph != 2 || a.out_pw != 2 || d.w != kP0W || a.src_row_stride != kP0W || d.h != kP0sRows) return false;
  const OpInfo &o0 = ops[st[0]], &o1 = ops[st[1]], &o2 = ops[st[2]];
  const int C = kP0C;
  if (!(o0.kh == 3 && o0.kw == 3 && o0.cin == 1 && o0.cout == C)) return false;
  if (!(o1.kh == 1 && o1.kw == 3 && o1.cin == C && o1.cout == C)) return false;
  if (!(o2.kh == 3 && o2.kw == 1 && o2.cin == C && o2.cout == C)) return false;
  const bool leaky = o0.act != 0;
  for (const OpInfo* o : {&o0, &o1, &o2}) {
    if ((o->act != 0) != leaky) return false;
    if (leaky && (o->alpha != o0.alpha || !(o->alpha >= 0.f && o->alpha <= 1.f))) return false;
  }
  if (od.h != kP0sHout || od.w != kP0sWout || od.c != C) return false;
  const int woff1 = 2 * 32 * 16, woff2 = woff1 + 2 * 32 * 16 * kP0sKS, total = woff2 + 2 * 32 * 16 * kP0sKS;
  std::vector<_Float16> w(total, static_cast<_Float16>(0.f));
  auto put = [&](int off, int ks, int n, int k, float v) {
    uint32_t bits;
    memcpy(&bits, &v, 4);
    bits &= 0xFFFFE000u;
    float hv;
    memcpy(&hv, &bits, 4);
    w[off + n * 16 * ks + k] = static_cast<_Float16>(hv);
    w[off + 32 * 16 * ks + n * 16 * ks + k] = static_cast<_Float16>(v - hv);
  };
  for (int n = 0; n < C; ++n) {
    // K slots (p0s_iter): lower half 0-5 = window (y, y + 1) x (dx 0-2), upper half 8-13 = window
    // (y + 1, y + 2); taps 0-4 in the lower half, 5-8 in the upper, the bias in slot 6 (B = 1)
    for (int k = 0; k < 16; ++k) {
      const int tap = k < 5 ? k : (k >= 10 && k < 14 ? k - 5 : -1);
      if (tap >= 0) put(0, 1, n, k, o0.w[size_t(tap) * C + n]);
    }
    put(0, 1, n, 6, o0.b[n]);
    for (int k = 0; k < 3 * C; ++k) put(woff1, kP0sKS, n, k, o1.w[size_t(k) * C + n]);  // HWIO: (tap C + ci) C + n
    put(woff1, kP0sKS, n, 3 * C, o1.b[n]);
    // stage 2: K step ks, lane half h holds group (dy, c) = G2[ks][h] (p0s_iter), channels 8 c .. 8 c + 7
    static const int G2[5][2][2] = {{{0, 0}, {0, 1}}, {{1, 0}, {1, 1}}, {{2, 0}, {2, 1}}, {{0, 2}, {1, 2}},
                                    {{2, 2}, {-1, -1}}};
    for (int ks = 0; ks < kP0sKS; ++ks)
      for (int h = 0; h < 2; ++h)
        for (int i = 0; i < 8; ++i) {
          const int k = 16 * ks + 8 * h + i, dy = G2[ks][h][0], cg = G2[ks][h][1];
          put(woff2, kP0sKS, n, k, dy < 0 ? (i == 0 ? o2.b[n] : 0.f) : o2.w[size_t(dy * C + 8 * cg + i) * C + n]);
        }
  }
  hipError_t e = hipMalloc(&cp.d_p0, w.size() * 2);
  if (e == hipSuccess) e = hipMemcpy(cp.d_p0, w.data(), w.size() * 2, hipMemcpyHostToDevice);
  cp.p0fn = leaky ? p0s_chain_kernel<true> : p0s_chain_kernel<false>;
  cp.p0_lds = kP0sLds;
  if (e == hipSuccess)
    e = hipFuncSetAttribute(reinterpret_cast<const void*>(cp.p0fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                            int(cp.p0_lds));
  int per_cu = 0;
  if (e == hipSuccess)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(cp.p0fn), kP0sThreads,
                                                     cp.p0_lds);
  if (e != hipSuccess || per_cu < 1) {
    (void)hipGetLastError();
    if (cp.d_p0) (void)hipFree(cp.d_p0);
    cp.d_p0 = nullptr;
    cp.p0fn = nullptr;
    return false;
  }
  cp.p0s = true;
  cp.p0_blocks_per_cu = per_cu;
  P0Args& p = cp.p0;
  p.w = static_cast<const _Float16*>(cp.d_p0);
  p.bias = nullptr;
  p.H_in = d.h;
  p.H_out = od.h;
  p.n_bands = 1;
  p.alpha = leaky ? o0.alpha : 0.f;
  if (getenv("HBK_DEBUG_EMBED"))
    fprintf(stderr, "hbk p0s chain: %dx%dx1 -> %dx%dx%d, one wave per clip, LDS %zu B, %d blocks/CU\n", d.h, d.w,
            od.h, od.w, od.c, cp.p0_lds, per_cu);
  return true;
}

// pooled rows per task: 6 (78 KB of LDS, two blocks per CU); HBK_P0_BAND=5|7 for tuning
bool plan_p0(const std::vector<OpInfo>& ops, const std::vector<int>& st, const ChainArgs& a, Dims d, Dims od,
             ChainPlan& cp) {
  if (getenv("HBK_EMBED_NO_P0")) return false;
  if (plan_p0s(ops, st, a, d, od, cp)) return true;
  const char* bs = getenv("HBK_P0_BAND");
  const int band = bs ? atoi(bs) : 6;
  if (band == 5) return plan_p0_band<5>(ops, st, a, d, od, cp);
  if (band == 7) return plan_p0_band<7>(ops, st, a, d, od, cp);
  return plan_p0_band<6>(ops, st, a, d, od, cp);
}

// The p1 pattern: [1x3 (CI -> 32), 3x1, 1x3, 3x1 (32 -> 32)] + output pool 2x2,
// NHWC input of width 14 with CI = 24, one image per source image.
constexpr int kP1W = 14, kP1CI = 24, kP1Band = 8;
using P1G = P1Geo<kP1W, kP1CI, kP1Band>;

// The streaming p1 form (p1s_chain_kernel) for a 66-row input: weights per
// stage s as hi / lo [32][96] (K = tap * cin + ci; stage a's bias at K 72),
// biases of stages b, c, d as [3][32] f32.
bool plan_p1s(const std::vector<OpInfo>& ops, const std::vector<int>& st, const ChainArgs& a, Dims d, Dims od,
              ChainPlan& cp) {
  if (getenv("HBK_EMBED_NO_P1S")) return false;
  if (st.size() != 4 || a.ipc != 1 || a.in_ph != 1 || a.in_pw != 1 || a.out_ph != 2 || a.out_pw != 2) return false;
  if (d.h != kP1sHin || d.w != kP1sWi || d.c != kP1sCSI || a.C_src != kP1sCSI || a.src_row_stride != kP1sWi * kP1sCSI)
    return false;
  const int kh[4] = {1, 3, 1, 3}, kw[4] = {3, 1, 3, 1};
  const bool leaky = ops[st[0]].act != 0;
  for (int i = 0; i < 4; ++i) {
    const OpInfo& o = ops[st[i]];
    if (o.kh != kh[i] || o.kw != kw[i] || o.cin != (i ? kP1sCo : kP1sCSI) || o.cout != kP1sCo) return false;
    if ((o.act != 0) != leaky) return false;
    if (leaky && (o.alpha != ops[st[0]].alpha || !(o.alpha >= 0.f && o.alpha <= 1.f))) return false;
  }
  if (od.h != kP1sHout || od.w != kP1sWo || od.c != kP1sCo) return false;
  std::vector<_Float16> w(4 * kP1sStageHalfs, static_cast<_Float16>(0.f));
  auto put = [&](int s, int n, int k, float v) {
    uint32_t bits;
    memcpy(&bits, &v, 4);
    bits &= 0xFFFFE000u;
    float hv;
    memcpy(&hv, &bits, 4);
    w[s * kP1sStageHalfs + n * 96 + k] = static_cast<_Float16>(hv);
    w[s * kP1sStageHalfs + 32 * 96 + n * 96 + k] = static_cast<_Float16>(v - hv);
  };
  for (int s = 0; s < 4; ++s) {
    const OpInfo& o = ops[st[s]];
    const int K = 3 * o.cin;
    for (int n = 0; n < kP1sCo; ++n) {
      for (int k = 0; k < K; ++k) put(s, n, k, o.w[size_t(k) * kP1sCo + n]);  // HWIO: (tap cin + ci) cout + n
      if (s == 0) put(0, n, K, o.b[n]);
    }
  }
  std::vector<float> b(3 * 32, 0.f);
  for (int s = 1; s < 4; ++s)
    for (int n = 0; n < kP1sCo; ++n) b[32 * (s - 1) + n] = ops[st[s]].b[n];
  const size_t wbytes = (w.size() * 2 + 15) & ~size_t(15);
  hipError_t e = hipMalloc(&cp.d_p0, wbytes + b.size() * 4);
  if (e == hipSuccess) e = hipMemcpy(cp.d_p0, w.data(), w.size() * 2, hipMemcpyHostToDevice);
  if (e == hipSuccess)
    e = hipMemcpy(static_cast<unsigned char*>(cp.d_p0) + wbytes, b.data(), b.size() * 4, hipMemcpyHostToDevice);
  cp.p1fn = leaky ? p1s_chain_kernel<true> : p1s_chain_kernel<false>;
  cp.p0_lds = kP1sLds;
  if (e == hipSuccess)
    e = hipFuncSetAttribute(reinterpret_cast<const void*>(cp.p1fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                            int(cp.p0_lds));
  int per_cu = 0;
  if (e == hipSuccess)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(cp.p1fn), kP1sThreads,
                                                     cp.p0_lds);
  if (e != hipSuccess || per_cu < 1) {
    (void)hipGetLastError();
    if (cp.d_p0) (void)hipFree(cp.d_p0);
    cp.d_p0 = nullptr;
    cp.p1fn = nullptr;
    return false;
  }
  cp.p1s = true;
  cp.p0_blocks_per_cu = per_cu;
  P1Args& p = cp.p1;
  p.w = static_cast<const _Float16*>(cp.d_p0);
  p.bias = reinterpret_cast<const float*>(static_cast<unsigned char*>(cp.d_p0) + wbytes);
  p.H_in = d.h;
  p.H_out = od.h;
  p.n_bands = 1;
  p.alpha = leaky ? ops[st[0]].alpha : 0.f;
  if (getenv("HBK_DEBUG_EMBED"))
    fprintf(stderr, "hbk p1s chain: %dx%dx%d -> %dx%dx%d, two-wave stage pipeline per clip, LDS %zu B, %d blocks/CU\n",
            d.h, d.w,
            d.c, od.h, od.w, od.c, cp.p0_lds, per_cu);
  return true;
}

// The p2s pattern (SE20 chain 2): [1x3 (32 -> 48), 3x1, 1x3, 3x1 (48 -> 48)] on a
// 31 x 5 x 32 input, no output pool, one image per source image. Weights hi /
// lo [48][96] (stage a) and [48][160] (b, c, d: K = tap * 48 + ci, the bias at
// K 144); stage a's bias as f32.
bool plan_p2s(const std::vector<OpInfo>& ops, const std::vector<int>& st, const ChainArgs& a, Dims d, Dims od,
              ChainPlan& cp) {
  if (getenv("HBK_EMBED_NO_P2S")) return false;
  if (st.size() != 4 || a.ipc != 1 || a.in_ph != 1 || a.in_pw != 1 || a.out_ph != 1 || a.out_pw != 1) return false;
  if (d.h != kP2sHin || d.w != kP2sWi || d.c != kP2sCi || a.C_src != kP2sCi || a.src_row_stride != kP2sWi * kP2sCi)
    return false;
  const int kh[4] = {1, 3, 1, 3}, kw[4] = {3, 1, 3, 1};
  const bool leaky = ops[st[0]].act != 0;
  for (int i = 0; i < 4; ++i) {
    const OpInfo& o = ops[st[i]];
    if (o.kh != kh[i] || o.kw != kw[i] || o.cin != (i ? kP2sCo : kP2sCi) || o.cout != kP2sCo) return false;
    if ((o.act != 0) != leaky) return false;
    if (leaky && (o.alpha != ops[st[0]].alpha || !(o.alpha >= 0.f && o.alpha <= 1.f))) return false;
  }
  if (od.h != kP2sHout || od.w != 1 || od.c != kP2sCo) return false;
  const size_t wa = size_t(2) * kP2sCo * kP2sKa, wsz = size_t(2) * kP2sCo * kP2sK;
  std::vector<_Float16> w(wa + 3 * wsz, static_cast<_Float16>(0.f));
  auto put = [&](size_t off, int Kp, int n, int k, float v) {
    uint32_t bits;
    memcpy(&bits, &v, 4);
    bits &= 0xFFFFE000u;
    float hv;
    memcpy(&hv, &bits, 4);
    w[off + size_t(n) * Kp + k] = static_cast<_Float16>(hv);
    w[off + size_t(kP2sCo) * Kp + size_t(n) * Kp + k] = static_cast<_Float16>(v - hv);
  };
  for (int s2 = 0; s2 < 4; ++s2) {
    const OpInfo& o = ops[st[s2]];
    const size_t off = s2 == 0 ? 0 : wa + (s2 - 1) * wsz;
    const int Kp = s2 == 0 ? kP2sKa : kP2sK, K = 3 * o.cin;
    for (int n = 0; n < kP2sCo; ++n) {
      for (int k = 0; k < K; ++k) put(off, Kp, n, k, o.w[size_t(k) * kP2sCo + n]);  // HWIO: (tap cin + ci) cout + n
      if (s2 > 0) put(off, Kp, n, K, o.b[n]);
    }
  }
  const size_t wbytes = (w.size() * 2 + 15) & ~size_t(15);
  hipError_t e = hipMalloc(&cp.d_p0, wbytes + kP2sCo * 4);
  if (e == hipSuccess) e = hipMemcpy(cp.d_p0, w.data(), w.size() * 2, hipMemcpyHostToDevice);
  if (e == hipSuccess)
    e = hipMemcpy(static_cast<unsigned char*>(cp.d_p0) + wbytes, ops[st[0]].b.data(), kP2sCo * 4,
                  hipMemcpyHostToDevice);
  cp.p2fn = leaky ? p2s_chain_kernel<true> : p2s_chain_kernel<false>;
  cp.p0_lds = kP2sLds;
  if (e == hipSuccess)
    e = hipFuncSetAttribute(reinterpret_cast<const void*>(cp.p2fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                            int(cp.p0_lds));
  int per_cu = 0;
  if (e == hipSuccess)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(cp.p2fn), kP2sThreads,
                                                     cp.p0_lds);
  if (e != hipSuccess || per_cu < 1) {
    (void)hipGetLastError();
    if (cp.d_p0) (void)hipFree(cp.d_p0);
    cp.d_p0 = nullptr;
    cp.p2fn = nullptr;
    return false;
  }
  cp.p0_blocks_per_cu = per_cu;
  P2sArgs& p = cp.p2;
  p.w = static_cast<const _Float16*>(cp.d_p0);
  p.bias_a = reinterpret_cast<const float*>(static_cast<unsigned char*>(cp.d_p0) + wbytes);
  p.alpha = leaky ? ops[st[0]].alpha : 0.f;
  if (getenv("HBK_DEBUG_EMBED"))
    fprintf(stderr, "hbk p2s chain: %dx%dx%d -> %dx%dx%d, %d clips per workgroup, LDS %zu B, %d blocks/CU\n", d.h,
            d.w, d.c, od.h, od.w, od.c, kP2sClips, cp.p0_lds, per_cu);
  return true;
}

// The t3s pattern (SE20's tail over its two phase images per clip): an input
// pool 2x1 of the 27 x 1 x 48 chain-2 rows, 3x1 (48 -> 64), 1x1, 3x1, 1x1 (64),
// 2x1 (64 -> 96), four 1x1 (96), the last without activation. Weights hi / lo
// [cout][K] per stage (K = tap * cin + ci; stage 1 zero-padded to 160), biases f32.
bool plan_t3s(const std::vector<OpInfo>& ops, const std::vector<int>& st, const ChainArgs& a, Dims d, Dims od,
              ChainPlan& cp) {
  if (getenv("HBK_EMBED_NO_T3S")) return false;
  if (st.size() != 9 || a.ipc != 2 || a.row_off[0] != 0 || a.row_off[1] != 1 || a.in_ph != 2 || a.in_pw != 1 ||
      a.out_ph != 1 || a.out_pw != 1)
    return false;
  if (d.h != kT3Hp || d.w != 1 || d.c != kT3C0 || a.C_src != kT3C0 || a.src_row_stride != kT3C0 ||
      a.src_clip_stride != int64_t(kT3Hin) * kT3C0)
    return false;
  if (od.h != kT3Hout || od.w != 1 || od.c != kT3C2 || cp.x.out_img_stride != int64_t(kT3Hout) * kT3C2) return false;
  const int kh[9] = {3, 1, 3, 1, 2, 1, 1, 1, 1};
  const int cin[9] = {kT3C0, kT3C1, kT3C1, kT3C1, kT3C1, kT3C2, kT3C2, kT3C2, kT3C2};
  const bool leaky = ops[st[0]].act != 0;
  for (int i = 0; i < 9; ++i) {
    const OpInfo& o = ops[st[i]];
    if (o.kh != kh[i] || o.kw != 1 || o.cin != cin[i] || o.cout != (i < 4 ? kT3C1 : kT3C2)) return false;
    if ((o.act != 0) != (leaky && i < 8)) return false;
    if (o.act != 0 && (o.alpha != ops[st[0]].alpha || !(o.alpha >= 0.f && o.alpha <= 1.f))) return false;
  }
  std::vector<_Float16> w(kT3WHalfs, static_cast<_Float16>(0.f));
  std::vector<float> b(4 * kT3C1 + 5 * kT3C2, 0.f);
  int boff = 0;
  for (int i = 0; i < 9; ++i) {
    const OpInfo& o = ops[st[i]];
    const int K = o.kh * o.cin, Kp = kT3K[i];
    for (int n = 0; n < o.cout; ++n) {
      for (int k = 0; k < K; ++k) {
        const float v = o.w[size_t(k) * o.cout + n];  // HWIO: (tap cin + ci) cout + n
        uint32_t bits;
        memcpy(&bits, &v, 4);
        bits &= 0xFFFFE000u;
        float hv;
        memcpy(&hv, &bits, 4);
        w[kT3W[i] + size_t(n) * Kp + k] = static_cast<_Float16>(hv);
        w[kT3W[i] + size_t(o.cout) * Kp + size_t(n) * Kp + k] = static_cast<_Float16>(v - hv);
      }
      b[boff + n] = o.b[n];
    }
    boff += o.cout;
  }
  const size_t wbytes = (w.size() * 2 + 15) & ~size_t(15);
  hipError_t e = hipMalloc(&cp.d_p0, wbytes + b.size() * 4);
  if (e == hipSuccess) e = hipMemcpy(cp.d_p0, w.data(), w.size() * 2, hipMemcpyHostToDevice);
  if (e == hipSuccess)
    e = hipMemcpy(static_cast<unsigned char*>(cp.d_p0) + wbytes, b.data(), b.size() * 4, hipMemcpyHostToDevice);
  cp.t3fn = leaky ? t3s_chain_kernel<true> : t3s_chain_kernel<false>;
  cp.p0_lds = kT3Lds;
  if (e == hipSuccess)
    e = hipFuncSetAttribute(reinterpret_cast<const void*>(cp.t3fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                            int(cp.p0_lds));
  int per_cu = 0;
  if (e == hipSuccess)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(cp.t3fn), kT3Threads,
                                                     cp.p0_lds);
  if (e != hipSuccess || per_cu < 1) {
    (void)hipGetLastError();
    if (cp.d_p0) (void)hipFree(cp.d_p0);
    cp.d_p0 = nullptr;
    cp.t3fn = nullptr;
    return false;
  }
  cp.p0_blocks_per_cu = per_cu;
  T3sArgs& p = cp.t3;
  p.w = static_cast<const _Float16*>(cp.d_p0);
  p.bias = reinterpret_cast<const float*>(static_cast<unsigned char*>(cp.d_p0) + wbytes);
  p.out_img_stride = cp.x.out_img_stride;
  p.alpha = leaky ? ops[st[0]].alpha : 0.f;
  if (getenv("HBK_DEBUG_EMBED"))
    fprintf(stderr, "hbk t3s chain: %dx%dx%d (pool 2x1) -> %dx%dx%d, %d images per workgroup, LDS %zu B, %d blocks/CU\n",
            d.h, d.w, d.c, od.h, od.w, od.c, kT3Pos, cp.p0_lds, per_cu);
  return true;
}

bool plan_p1(const std::vector<OpInfo>& ops, const std::vector<int>& st, const ChainArgs& a, Dims d, Dims od,
             ChainPlan& cp) {
  if (getenv("HBK_EMBED_NO_P1")) return false;
  if (plan_p1s(ops, st, a, d, od, cp)) return true;
  if (st.size() != 4 || a.ipc != 1 || a.in_ph != 1 || a.in_pw != 1 || a.out_ph != 2 || a.out_pw != 2) return false;
  if (d.w != kP1W || d.c != kP1CI || a.C_src != kP1CI || a.src_row_stride != kP1W * kP1CI) return false;
  const int C = kP1C;
  const int kh[4] = {1, 3, 1, 3}, kw[4] = {3, 1, 3, 1};
  bool leaky = ops[st[0]].act != 0;
  for (int i = 0; i < 4; ++i) {
    const OpInfo& o = ops[st[i]];
    if (o.kh != kh[i] || o.kw != kw[i] || o.cin != (i ? C : kP1CI) || o.cout != C) return false;
    if ((o.act != 0) != leaky) return false;
    if (leaky && (o.alpha != ops[st[0]].alpha || !(o.alpha >= 0.f && o.alpha <= 1.f))) return false;
  }
  if (od.h != (d.h - 4) / 2 || od.w != (d.w - 4) / 2 || od.c != C) return false;
  std::vector<_Float16> w(P1G::WHALFS, static_cast<_Float16>(0.f));
  const int woff[4] = {P1G::WOFF1, P1G::WOFF2, P1G::WOFF3, P1G::WOFF4};
  for (int i = 0; i < 4; ++i) {
    const OpInfo& o = ops[st[i]];
    const int ks = i ? P1G::KS : P1G::KS1, K = 3 * o.cin;
    for (int n = 0; n < C; ++n)
      for (int k = 0; k < K; ++k) {
        const float v = o.w[size_t(k) * C + n];  // HWIO: (tap * cin + ci) * cout + n
        uint32_t bits;
        memcpy(&bits, &v, 4);
        bits &= 0xFFFFE000u;
        float hv;
        memcpy(&hv, &bits, 4);
        w[woff[i] + n * 16 * ks + k] = static_cast<_Float16>(hv);
        w[woff[i] + 32 * 16 * ks + n * 16 * ks + k] = static_cast<_Float16>(v - hv);
      }
  }
  std::vector<float> b(128, 0.f);
  for (int i = 0; i < 4; ++i)
    for (int n = 0; n < C; ++n) b[32 * i + n] = ops[st[i]].b[n];
  const size_t wbytes = (w.size() * 2 + 15) & ~size_t(15);
  hipError_t e = hipMalloc(&cp.d_p0, wbytes + b.size() * 4);
  if (e == hipSuccess) e = hipMemcpy(cp.d_p0, w.data(), w.size() * 2, hipMemcpyHostToDevice);
  if (e == hipSuccess)
    e = hipMemcpy(static_cast<unsigned char*>(cp.d_p0) + wbytes, b.data(), b.size() * 4, hipMemcpyHostToDevice);
  cp.p1fn = leaky ? p1_chain_kernel<kP1W, kP1CI, kP1Band, true> : p1_chain_kernel<kP1W, kP1CI, kP1Band, false>;
  cp.p0_lds = P1G::LDS;
  if (e == hipSuccess)
    e = hipFuncSetAttribute(reinterpret_cast<const void*>(cp.p1fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                            int(cp.p0_lds));
  int per_cu = 0;
  if (e == hipSuccess)
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(cp.p1fn), kP0Threads,
                                                     cp.p0_lds);
  if (e != hipSuccess || per_cu < 1) {
    (void)hipGetLastError();
    if (cp.d_p0) (void)hipFree(cp.d_p0);
    cp.d_p0 = nullptr;
    cp.p1fn = nullptr;
    return false;
  }
  cp.p0_blocks_per_cu = per_cu;
  P1Args& p = cp.p1;
  p.w = static_cast<const _Float16*>(cp.d_p0);
  p.bias = reinterpret_cast<const float*>(static_cast<unsigned char*>(cp.d_p0) + wbytes);
  p.H_in = d.h;
  p.H_out = od.h;
  p.n_bands = (od.h + kP1Band - 1) / kP1Band;
  p.alpha = leaky ? ops[st[0]].alpha : 0.f;
  if (getenv("HBK_DEBUG_EMBED"))
    fprintf(stderr, "hbk p1 chain: %dx%dx%d -> %dx%dx%d, band %d (%d bands), LDS %zu B, %d blocks/CU\n", d.h, d.w,
            d.c, od.h, od.w, od.c, kP1Band, p.n_bands, cp.p0_lds, per_cu);
  return true;
}

// Builds the chains for ops [o0, o1) applied to images of dims `in`, reading
// image i from row_off[i % ipc] of source clip i / ipc.
int build_segment(const std::vector<OpInfo>& ops, int o0, int o1, Dims in, int ipc,
                  const std::vector<int>& row_off, int64_t src_clip_floats, int src_row_floats,
                  int first_src_buf, bool split, Program& prog, std::vector<Dims>* out_dims_per_chain) {
  int i = o0;
  Dims cur = in;
  int src_buf = first_src_buf;
  bool first = true;
  while (i < o1) {
    ChainPlan cp;
    ChainArgs& a = cp.args;
    a.ipc = first ? ipc : 1;
    for (int k = 0; k < kMaxWin; ++k) a.row_off[k] = 0;
    if (first)
      for (size_t k = 0; k < row_off.size(); ++k) a.row_off[k] = row_off[k];
    a.src_clip_stride = first ? src_clip_floats : int64_t(cur.h) * cur.w * cur.c;
    a.src_row_stride = first ? src_row_floats : cur.w * cur.c;
    a.C_src = cur.c;
    a.in_ph = a.in_pw = 1;
    if (ops[i].kind == HBK_OP_MAXPOOL) {
      a.in_ph = ops[i].kh;
      a.in_pw = ops[i].kw;
      ++i;
    }
    Dims d{cur.h / a.in_ph, cur.w / a.in_pw, cur.c};
    a.W_in = d.w;
    const int H_in = d.h;
    std::vector<int> stage_ops;
    while (i < o1 && ops[i].kind == HBK_OP_CONV && int(stage_ops.size()) < kMaxStages) {
      stage_ops.push_back(i);
      ++i;
    }
    if (stage_ops.empty()) {
      set_error("hbk: unsupported graph: a max-pool must be followed by a conv");
      return HBK_ERR_UNSUPPORTED;
    }
    a.out_ph = a.out_pw = 1;
    if (i < o1 && ops[i].kind == HBK_OP_MAXPOOL && (i + 1 >= o1 || ops[i + 1].kind == HBK_OP_CONV)) {
      // keep the pool as this chain's output pool unless the next chain needs it as input pool
      a.out_ph = ops[i].kh;
      a.out_pw = ops[i].kw;
      ++i;
    }
    if (split) {
      Dims od;
      const int rc = layout_split(ops, stage_ops, d, a, cp, od);
      if (rc) return rc;
      if (!plan_p0(ops, stage_ops, a, d, od, cp) && !plan_p1(ops, stage_ops, a, d, od, cp) &&
          !plan_p2s(ops, stage_ops, a, d, od, cp))
        plan_t3s(ops, stage_ops, a, d, od, cp);
      cp.x.dbg_slot = static_cast<int>(prog.chains.size() % 4);
      if (const char* e = getenv("HBK_DEBUG_SKIP")) cp.x.dbg_skip = atoi(e);
      cp.src_buf = src_buf;
      cp.out_floats = cp.x.out_img_stride * (first ? ipc : 1);
      prog.chains.push_back(cp);
      if (out_dims_per_chain) out_dims_per_chain->push_back(od);
      src_buf = -2;
      cur = od;
      first = false;
      continue;
    }
    // stages
    int nb = 1;
    int cin = d.c, h = H_in, w = d.w;
    a.n_stages = static_cast<int>(stage_ops.size());
    a.shrink = 0;
    double macs = 0;
    std::vector<Dims> tens;  // stage input/output tensors (per image, padded channels)
    for (int s = 0; s < a.n_stages; ++s) {
      const OpInfo& op = ops[stage_ops[s]];
      if (op.cin != cin) {
        set_error("hbk: graph channel mismatch at op %d (%d != %d)", stage_ops[s], op.cin, cin);
        return HBK_ERR_ARG;
      }
      StageDesc& S = a.st[s];
      S.kh = op.kh;
      S.kw = op.kw;
      S.cin = op.cin;
      S.cinp = odd_pad(op.cin);
      S.cout = op.cout;
      S.coutp = odd_pad(op.cout);
      S.K = op.kh * op.kw * op.cin;
      S.ksteps = (S.K + 3) / 4;
      S.act = op.act;
      S.alpha = op.alpha;
      nb = std::max(nb, (op.cout + 15) / 16);
      a.shrink += op.kh - 1;
      h -= op.kh - 1;
      w -= op.kw - 1;
      if (h <= 0 || w <= 0) {
        set_error("hbk: graph collapses the image at op %d", stage_ops[s]);
        return HBK_ERR_ARG;
      }
      macs += double(h) * w * op.cout * S.K;
      cin = op.cout;
    }
    cp.nb = nb;  // > 6 blocks: the 6-block kernel loops over channel groups
    a.wstride = nb * 16 + ((nb * 16) % 32 == 0 ? 16 : 0);  // kq rows on different bank halves
    // pack weights: per stage [ksteps*4][wstride] then bias [nb*16]
    std::vector<float> blob;
    int max_stage_w = 0, max_k = 0;
    for (int s = 0; s < a.n_stages; ++s) {
      const OpInfo& op = ops[stage_ops[s]];
      StageDesc& S = a.st[s];
      S.w_off = static_cast<int>(blob.size());
      const int rows = S.ksteps * 4;
      blob.resize(blob.size() + size_t(rows) * a.wstride, 0.f);
      for (int k = 0; k < S.K; ++k)
        for (int n = 0; n < op.cout; ++n) blob[S.w_off + size_t(k) * a.wstride + n] = op.w[size_t(k) * op.cout + n];
      max_stage_w = std::max(max_stage_w, rows * a.wstride);
      max_k = std::max(max_k, rows);
    }
    for (int s = 0; s < a.n_stages; ++s) {
      const OpInfo& op = ops[stage_ops[s]];
      a.st[s].b_off = static_cast<int>(blob.size());
      for (int n = 0; n < nb * 16; ++n) blob.push_back(n < op.cout ? op.b[n] : 0.f);
    }
    a.wblob_floats = static_cast<int>(blob.size());
    // output dims
    Dims od{h / a.out_ph, w / a.out_pw, cin};
    a.H_out = od.h;
    a.W_out = od.w;
    a.C_out = od.c;
    a.out_img_stride = int64_t(od.h) * od.w * od.c;
    if (od.h <= 0 || od.w <= 0) {
      set_error("hbk: pooling collapses the image");
      return HBK_ERR_ARG;
    }
    // choose G (images per task) and band (output rows per task) for the LDS budget
    auto lds_floats = [&](int G, int band, bool resident) -> int64_t {
      int rows = band * a.out_ph;  // rows of the last conv output
      std::vector<int64_t> t(a.n_stages + 1);
      for (int s = a.n_stages - 1; s >= 0; --s) {
        const StageDesc& S = a.st[s];
        int wo = d.w;
        for (int q = 0; q <= s; ++q) wo -= a.st[q].kw - 1;
        t[s + 1] = int64_t(G) * rows * wo * S.coutp;
        rows += S.kh - 1;
      }
      t[0] = int64_t(G) * rows * d.w * a.st[0].cinp;
      int64_t x = 0, y = 0;
      for (int s = 0; s <= a.n_stages; ++s) (s % 2 == 0 ? x : y) = std::max(s % 2 == 0 ? x : y, t[s]);
      int64_t wf = resident ? a.wblob_floats : 0;
      return ((x + 3) & ~3) + ((y + 3) & ~3) + ((wf + 3) & ~3) + ((max_k + 3) & ~3);
    };
    const int64_t budget = kLdsBudget / 4;
    bool resident = lds_floats(1, 1, true) <= budget;
    int band = 0, G = 1;
    for (int b = od.h; b >= 1; --b)
      if (lds_floats(1, b, resident) <= budget) { band = b; break; }
    if (band == 0) {
      set_error("hbk: one output row of a chain does not fit in LDS");
      return HBK_ERR_UNSUPPORTED;
    }
    if (band == od.h)
      while (G < 64 && lds_floats(G * 2, band, resident) <= budget) G *= 2;
    a.G = G;
    a.band = band;
    a.n_bands = (od.h + band - 1) / band;
    int64_t xf = 0, yf = 0;
    {
      int rows = band * a.out_ph;
      std::vector<int64_t> t(a.n_stages + 1);
      for (int s = a.n_stages - 1; s >= 0; --s) {
        int wo = d.w;
        for (int q = 0; q <= s; ++q) wo -= a.st[q].kw - 1;
        t[s + 1] = int64_t(G) * rows * wo * a.st[s].coutp;
        rows += a.st[s].kh - 1;
      }
      t[0] = int64_t(G) * rows * d.w * a.st[0].cinp;
      for (int s = 0; s <= a.n_stages; ++s) (s % 2 == 0 ? xf : yf) = std::max(s % 2 == 0 ? xf : yf, t[s]);
    }
    a.lds_x = 0;
    a.lds_y = static_cast<int>((xf + 3) & ~3);
    a.lds_w = a.lds_y + static_cast<int>((yf + 3) & ~3);
    a.lds_k = a.lds_w + (resident ? ((a.wblob_floats + 3) & ~3) : 0);
    cp.lds_bytes = size_t(a.lds_k + ((max_k + 3) & ~3)) * 4;
    cp.wg = !resident;
    cp.fn = pick_kernel(nb, cp.wg);
    (void)max_stage_w;
    // device weights
    hipError_t e = hipMalloc(&cp.d_blob, blob.size() * sizeof(float));
    if (e != hipSuccess) return hip_error(e, "hipMalloc chain weights");
    e = hipMemcpy(cp.d_blob, blob.data(), blob.size() * sizeof(float), hipMemcpyHostToDevice);
    if (e != hipSuccess) return hip_error(e, "copy chain weights");
    a.wblob = cp.d_blob;
    if (cp.lds_bytes > 64 * 1024) {
      e = set_max_dynamic_lds(reinterpret_cast<const void*>(cp.fn));  // see layout_split
      if (e != hipSuccess) return hip_error(e, "hipFuncSetAttribute(max dynamic LDS)");
    }
    cp.macs_per_img = macs;
    cp.src_buf = src_buf;
    cp.out_floats = a.out_img_stride * (first ? ipc : 1);
    prog.chains.push_back(cp);
    if (out_dims_per_chain) out_dims_per_chain->push_back(od);
    src_buf = -2;  // placeholder: assigned by the caller
    cur = od;
    first = false;
  }
  return HBK_OK;
}

// Assign ping-pong workspace buffers: chain k writes buffer k % 2, the last
// writes the call's output; record per-unit buffer sizes.
void assign_buffers(Program& prog, int64_t units_per_first_img_ratio) {
  (void)units_per_first_img_ratio;
  const size_t n = prog.chains.size();
  for (size_t k = 0; k < n; ++k) {
    ChainPlan& c = prog.chains[k];
    c.src_buf = (k == 0) ? -1 : int((k - 1) % 2);
    c.dst_buf = (k + 1 == n && prog.gather_src.empty()) ? -1 : int(k % 2);
  }
  if (!prog.gather_src.empty()) prog.gather_buf = int((n - 1) % 2);
}

// out[u][i][:] = src[u][gather_src[i]][:] (rows of `row` floats, row % 4 == 0);
// one wave per unit, all of a unit's reads ahead of its writes (distinct buffers)
__global__ void __launch_bounds__(256) embed_gather_kernel(const float* __restrict__ src, float* __restrict__ out,
                                                           const int* __restrict__ map, int64_t n_units, int n_src,
                                                           int n_out, int row) {
  const int lane = threadIdx.x & 63;
  const int64_t u = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (u >= n_units) return;
  const int r4 = row / 4, n4 = n_out * r4;
  const float4* s = reinterpret_cast<const float4*>(src + u * n_src * row);
  float4* d = reinterpret_cast<float4*>(out + u * n_out * row);
  for (int f = lane; f < n4; f += 64) {
    const int i = f / r4, c = f - i * r4;
    d[f] = s[map[i] * r4 + c];
  }
}

// Runs chains [k_begin, k_end) of the program (k_end < 0: to the end). The
// first chain run reads `in` (the call's input, or for k_begin > 0 the output
// of chain k_begin - 1 in its workspace layout); the last writes `out` (for
// k_end < n: chain k_end - 1's output in its workspace layout, no gather).
int run_program(const Program& prog, const float* in, int64_t n_units, int64_t in_unit_stride,
                float* out, int64_t out_unit_floats, float* ws, int64_t chunk, hipStream_t stream,
                const std::vector<int64_t>& imgs_per_unit, const std::vector<int64_t>& buf_unit_floats,
                int* range_flag, int k_begin = 0, int k_end = -1) {
  const int n_ch = static_cast<int>(prog.chains.size());
  if (k_end < 0) k_end = n_ch;
  for (int64_t u0 = 0; u0 < n_units; u0 += chunk) {
    const int64_t nu = std::min(chunk, n_units - u0);
    float* bufs[2] = {ws, ws + chunk * buf_unit_floats[0]};
    for (int k = k_begin; k < k_end; ++k) {
      ChainPlan c = prog.chains[k];
      if (k == k_begin && k_begin > 0) c.src_buf = -1;  // the caller's copy of chain k - 1's output
      if (k == k_end - 1 && k_end < n_ch) c.dst_buf = -1;  // handed to the caller (no gather)
      if (c.p0fn) {
        P0Args pa = c.p0;
        pa.range_flag = range_flag;
        pa.in = c.src_buf < 0 ? in + u0 * in_unit_stride : bufs[c.src_buf];
        pa.src_img_stride = c.src_buf < 0 ? in_unit_stride : c.x.src_clip_stride;  // (in_unit_stride == it past chain 0)
        pa.out = c.dst_buf < 0 ? out + u0 * out_unit_floats : bufs[c.dst_buf];
        pa.n_img = nu * imgs_per_unit[k];
        const bool aligned = !(reinterpret_cast<uintptr_t>(pa.in) & 15) && !(pa.src_img_stride & 3) &&
                             !(reinterpret_cast<uintptr_t>(pa.out) & 15);
        if (aligned && pa.n_img * pa.n_bands < (int64_t(1) << 31)) {
          const int64_t tasks = c.p0s ? (pa.n_img + kP0sWaves - 1) / kP0sWaves : pa.n_img * pa.n_bands;
          const int64_t blocks = std::min<int64_t>(tasks, persistent_blocks(c.p0_blocks_per_cu, stream));
          if (blocks <= 0) continue;
          hipLaunchKernelGGL(c.p0fn, dim3(unsigned(blocks)), dim3(kP0Threads), c.p0_lds, stream, pa);
          HBK_LAUNCH_CHECK("p0_chain_kernel");
          continue;
        }
      }
      if (c.p1fn) {
        P1Args pa = c.p1;
        pa.range_flag = range_flag;
        pa.in = c.src_buf < 0 ? in + u0 * in_unit_stride : bufs[c.src_buf];
        pa.src_img_stride = c.src_buf < 0 ? in_unit_stride : c.x.src_clip_stride;  // (in_unit_stride == it past chain 0)
        pa.out = c.dst_buf < 0 ? out + u0 * out_unit_floats : bufs[c.dst_buf];
        pa.n_img = nu * imgs_per_unit[k];
        const bool aligned = !(reinterpret_cast<uintptr_t>(pa.in) & 15) && !(pa.src_img_stride & 3) &&
                             !(reinterpret_cast<uintptr_t>(pa.out) & 15);
        if (aligned && pa.n_img * pa.n_bands < (int64_t(1) << 31)) {
          const int64_t tasks = c.p1s ? pa.n_img : pa.n_img * pa.n_bands;
          const int64_t blocks = std::min<int64_t>(tasks, persistent_blocks(c.p0_blocks_per_cu, stream));
          if (blocks <= 0) continue;
          hipLaunchKernelGGL(c.p1fn, dim3(unsigned(blocks)), dim3(c.p1s ? kP1sThreads : kP0Threads), c.p0_lds, stream, pa);
          HBK_LAUNCH_CHECK("p1_chain_kernel");
          continue;
        }
      }
      if (c.p2fn) {
        P2sArgs pa = c.p2;
        pa.range_flag = range_flag;
        pa.in = c.src_buf < 0 ? in + u0 * in_unit_stride : bufs[c.src_buf];
        pa.src_img_stride = c.src_buf < 0 ? in_unit_stride : c.x.src_clip_stride;  // (in_unit_stride == it past chain 0)
        pa.out = c.dst_buf < 0 ? out + u0 * out_unit_floats : bufs[c.dst_buf];
        pa.n_img = nu * imgs_per_unit[k];
        const bool aligned = !(reinterpret_cast<uintptr_t>(pa.in) & 15) && !(pa.src_img_stride & 3) &&
                             !(reinterpret_cast<uintptr_t>(pa.out) & 15);
        if (aligned) {
          const int64_t groups = (pa.n_img + kP2sClips - 1) / kP2sClips;
          const int64_t blocks = std::min<int64_t>(groups, persistent_blocks(c.p0_blocks_per_cu, stream));
          if (blocks <= 0) continue;
          hipLaunchKernelGGL(c.p2fn, dim3(unsigned(blocks)), dim3(kP2sThreads), c.p0_lds, stream, pa);
          HBK_LAUNCH_CHECK("p2s_chain_kernel");
          continue;
        }
      }
      if (c.t3fn) {
        T3sArgs pa = c.t3;
        pa.range_flag = range_flag;
        pa.in = c.src_buf < 0 ? in + u0 * in_unit_stride : bufs[c.src_buf];
        pa.src_clip_stride = c.src_buf < 0 ? in_unit_stride : c.x.src_clip_stride;
        pa.out = c.dst_buf < 0 ? out + u0 * out_unit_floats : bufs[c.dst_buf];
        pa.n_img = nu * imgs_per_unit[k];
        const bool aligned = !(reinterpret_cast<uintptr_t>(pa.in) & 15) && !(pa.src_clip_stride & 3) &&
                             !(reinterpret_cast<uintptr_t>(pa.out) & 15) && !(pa.out_img_stride & 3);
        if (aligned && pa.src_clip_stride >= int64_t(kT3Hin) * kT3C0) {
          const int64_t groups = (pa.n_img + kT3Pos - 1) / kT3Pos;
          const int64_t blocks = std::min<int64_t>(groups, persistent_blocks(c.p0_blocks_per_cu, stream));
          if (blocks <= 0) continue;
          hipLaunchKernelGGL(c.t3fn, dim3(unsigned(blocks)), dim3(kT3Threads), c.p0_lds, stream, pa);
          HBK_LAUNCH_CHECK("t3s_chain_kernel");
          continue;
        }
      }
      if (c.split) {
        XArgs x = c.x;
        x.range_flag = range_flag;
        if (c.src_buf < 0) {
          x.in = in + u0 * in_unit_stride;
          x.src_clip_stride = in_unit_stride;
        } else {
          x.in = bufs[c.src_buf];
        }
        x.out = c.dst_buf < 0 ? out + u0 * out_unit_floats : bufs[c.dst_buf];
        if ((reinterpret_cast<uintptr_t>(x.out) & 15) || (x.out_img_stride & 3)) x.vec_out = 0;
        if ((reinterpret_cast<uintptr_t>(x.in) & 15) || (x.src_clip_stride & 3) || (x.src_row_stride & 3))
          x.raw_vec = 0;
        x.n_img = nu * imgs_per_unit[k];
        const int64_t tasks = ((x.n_img + x.G - 1) / x.G) * x.n_bands;
        const int per_cu = std::max<int>(1, std::min<int>(4, int((160 * 1024) / std::max<size_t>(c.lds_bytes, 1))));
        const int64_t blocks = std::min<int64_t>(tasks, persistent_blocks(per_cu, stream));
        if (blocks <= 0) continue;
        hipLaunchKernelGGL(c.xfn, dim3(unsigned(blocks)), dim3(kXThreads), c.lds_bytes, stream, x);
        HBK_LAUNCH_CHECK("conv_chain_x3_kernel");
        continue;
      }
      ChainArgs a = c.args;
      if (c.src_buf < 0) {
        a.in = in + u0 * in_unit_stride;
        a.src_clip_stride = in_unit_stride;
      } else {
        a.in = bufs[c.src_buf];
      }
      a.out = c.dst_buf < 0 ? out + u0 * out_unit_floats : bufs[c.dst_buf];
      a.n_img = nu * imgs_per_unit[k];
      const int64_t tasks = ((a.n_img + a.G - 1) / a.G) * a.n_bands;
      const int64_t blocks = std::min<int64_t>(tasks, persistent_blocks(2, stream));
      if (blocks <= 0) continue;
      hipLaunchKernelGGL(c.fn, dim3(unsigned(blocks)), dim3(kThreads), c.lds_bytes, stream, a);
      HBK_LAUNCH_CHECK("conv_chain_kernel");
    }
    if (prog.gather_buf >= 0 && k_end == n_ch) {
      const int n_out = static_cast<int>(prog.gather_src.size());
      const int row = static_cast<int>(out_unit_floats / n_out);
      hipLaunchKernelGGL(embed_gather_kernel, dim3(unsigned((nu + 3) / 4)), dim3(256), 0, stream,
                         bufs[prog.gather_buf], out + u0 * out_unit_floats, prog.d_gather, nu, prog.n_src, n_out, row);
      HBK_LAUNCH_CHECK("embed_gather_kernel");
    }
  }
  return HBK_OK;
}

}  // namespace
}  // namespace hbk

extern "C" {

int hbk_embed_plan_create(const hbk_graph_op* ops, int32_t n_ops, int32_t in_h, int32_t in_w,
                          const int32_t* win_start, int32_t n_win, hbk_embed_plan** plan) {
  return hbk_embed_plan_create_ex(ops, n_ops, in_h, in_w, win_start, n_win, HBK_PREC_SPLIT_F16, plan);
}

int hbk_embed_plan_create_ex(const hbk_graph_op* ops, int32_t n_ops, int32_t in_h, int32_t in_w,
                             const int32_t* win_start, int32_t n_win, int32_t precision,
                             hbk_embed_plan** plan) {
  using namespace hbk;
  if (!plan) return arg_error("plan is NULL");
  *plan = nullptr;
  if (precision != HBK_PREC_SPLIT_F16 && precision != HBK_PREC_EXACT_F32) return arg_error("unknown precision");
  if (!ops || n_ops <= 0) return arg_error("empty graph");
  if (in_h <= 0 || in_w <= 0) return arg_error("bad window size");
  if (!win_start || n_win <= 0 || n_win > kMaxWin) return arg_error("n_win must be in [1, 32]");
  auto* p = new hbk_embed_plan();
  auto fail = [&](int rc) {
    hbk_embed_plan_destroy(p);
    return rc;
  };
  p->in_h = in_h;
  p->in_w = in_w;
  p->split_f16 = precision == HBK_PREC_SPLIT_F16;
  {
    hipError_t e = hipMalloc(reinterpret_cast<void**>(&p->d_range), sizeof(int));
    if (e == hipSuccess) e = hipMemset(p->d_range, 0, sizeof(int));
    if (e != hipSuccess) return fail(hip_error(e, "hipMalloc range flag"));
  }
  for (int i = 0; i < n_win; ++i) {
    if (win_start[i] < 0) return fail(arg_error("negative window start"));
    p->starts.push_back(win_start[i]);
  }
  Dims d{in_h, in_w, 1};
  std::vector<Dims> dims;  // per op, for one window
  for (int i = 0; i < n_ops; ++i) {
    const hbk_graph_op& o = ops[i];
    OpInfo op{o.kind, o.kh, o.kw, o.cin, o.cout, o.act, o.alpha, {}, {}};
    if (o.kh <= 0 || o.kw <= 0) return fail(arg_error("kernel / pool size must be positive"));
    if (o.kind == HBK_OP_CONV) {
      if (o.cin != d.c || o.cout <= 0 || !o.weight || !o.bias) return fail(arg_error("bad conv op"));
      op.w.assign(o.weight, o.weight + size_t(o.kh) * o.kw * o.cin * o.cout);
      op.b.assign(o.bias, o.bias + o.cout);
      if (p->split_f16)
        for (float w : op.w)
          if (!(std::fabs(w) < kF16Max)) {
            set_error("hbk: op %d has a weight |w| >= 65504 (or NaN), outside the split-f16 range; "
                      "use HBK_PREC_EXACT_F32", i);
            return fail(HBK_ERR_UNSUPPORTED);
          }
      d = Dims{d.h - o.kh + 1, d.w - o.kw + 1, o.cout};
    } else if (o.kind == HBK_OP_MAXPOOL) {
      d = Dims{d.h / o.kh, d.w / o.kw, d.c};
    } else {
      return fail(arg_error("unknown op kind"));
    }
    if (d.h <= 0 || d.w <= 0) return fail(arg_error("graph collapses the window"));
    p->ops.push_back(std::move(op));
    dims.push_back(d);
  }
  if (d.h != 1 || d.w != 1) return fail(arg_error("graph output must be 1 x 1 x C"));
  p->out_dim = d.c;

  // prefix: ops shared across the windows of a clip. A pool of height ph keeps
  // the windows aligned iff the cumulative time stride divides every start.
  int g = 0;
  for (int s : p->starts) g = std::gcd(g, s);
  // If every pool keeps the alignment, split at the last pool (any earlier
  // split is equally valid; the tail must start with a pool).
  int stride = 1, split = n_ops, last_pool = -1, stride_before_last = 1;
  for (int i = 0; i < n_ops; ++i) {
    if (p->ops[i].kind == HBK_OP_MAXPOOL) {
      const int ns = stride * p->ops[i].kh;
      if (g % ns != 0) {
        split = i;
        break;
      }
      last_pool = i;
      stride_before_last = stride;
      stride = ns;
    }
  }
  if (split == n_ops && last_pool > 0) {
    split = last_pool;
    stride = stride_before_last;
  }
  // the tail must start with a pool (its input pool) and contain a conv
  if (split == n_ops || split == 0) {
    set_error("hbk: graph has no window-splitting pool; use hbk_embed_windows");
    return fail(HBK_ERR_UNSUPPORTED);
  }
  p->n_prefix = split;
  p->split_stride = stride;
  const int max_start = *std::max_element(p->starts.begin(), p->starts.end());
  p->seq_frames = max_start + in_h;

  int rc;
  // ---- clip program: prefix over [seq_frames, in_w, 1] per clip ----
  {
    std::vector<Dims> od;
    rc = build_segment(p->ops, 0, split, Dims{p->seq_frames, in_w, 1}, 1, {0}, 0, in_w, -1,
                       p->split_f16, p->clip_prog, &od);
    if (rc) return fail(rc);
    const Dims pre = od.back();
    // window rows at the split, for one window
    const Dims wd = dims[split - 1];
    std::vector<int> roff;
    for (int s : p->starts) roff.push_back(s / stride);
    for (int r : roff)
      if (r + wd.h > pre.h) return fail(arg_error("window start beyond the frame sequence"));
    const size_t n_pre = p->clip_prog.chains.size();
    // Phase deduplication of the tail: with S = the tail's cumulative pool
    // stride, windows whose prefix-row offsets are congruent mod S see the same
    // pool grid, and the tail's valid convs are translation-equivariant, so
    // ONE "phase image" per residue (rows [phi, phi + H)) yields every such
    // window as output row (r - phi) / S. Used when the phase images' output
    // fits the per-clip output (n_phase x rows <= n_win) and HBK_EMBED_NO_DEDUP
    // is unset; the output rows are gathered into window order afterwards.
    std::vector<int> phases, win_src;
    int H = 0;
    {
      int S = 1;
      for (int i = split; i < n_ops; ++i)
        if (p->ops[i].kind == HBK_OP_MAXPOOL) S *= p->ops[i].kh;
      for (int r : roff)
        if (std::find(phases.begin(), phases.end(), r % S) == phases.end()) phases.push_back(r % S);
      std::sort(phases.begin(), phases.end());
      for (int r : roff) H = std::max(H, r - r % S + wd.h);
      bool ok = S > 1 && !getenv("HBK_EMBED_NO_DEDUP") && int(phases.size()) < n_win;
      for (int ph : phases) ok = ok && ph + H <= pre.h;
      // tail output rows for an H-row phase image
      Dims t{H, wd.w, wd.c};
      for (int i = split; i < n_ops && ok; ++i) {
        const OpInfo& o = p->ops[i];
        t = o.kind == HBK_OP_CONV ? Dims{t.h - o.kh + 1, t.w - o.kw + 1, o.cout} : Dims{t.h / o.kh, t.w / o.kw, t.c};
        ok = t.h > 0 && t.w > 0;
      }
      ok = ok && t.w == 1 && int(phases.size()) * t.h <= n_win;
      if (ok) {
        for (int r : roff) {
          const int ph = int(std::find(phases.begin(), phases.end(), r % S) - phases.begin());
          const int row = (r - r % S) / S;
          ok = ok && row < t.h;
          win_src.push_back(ph * t.h + row);
        }
        p->clip_prog.n_src = int(phases.size()) * t.h;
      }
      if (!ok) phases.clear();
    }
    if (!phases.empty()) {
      p->clip_prog.gather_src = win_src;
      hipError_t e = hipMalloc(reinterpret_cast<void**>(&p->clip_prog.d_gather), win_src.size() * sizeof(int));
      if (e == hipSuccess)
        e = hipMemcpy(p->clip_prog.d_gather, win_src.data(), win_src.size() * sizeof(int), hipMemcpyHostToDevice);
      if (e != hipSuccess) return fail(hip_error(e, "embed gather map"));
      rc = build_segment(p->ops, split, n_ops, Dims{H, wd.w, wd.c}, int(phases.size()), phases,
                         int64_t(pre.h) * pre.w * pre.c, pre.w * pre.c, 0, p->split_f16, p->clip_prog, nullptr);
      if (getenv("HBK_DEBUG_EMBED"))
        fprintf(stderr, "hbk tail dedup: %zu phase images of %d rows per clip for %d windows\n", phases.size(), H,
                n_win);
    } else {
      rc = build_segment(p->ops, split, n_ops, Dims{wd.h, wd.w, wd.c}, n_win, roff,
                         int64_t(pre.h) * pre.w * pre.c, pre.w * pre.c, 0, p->split_f16, p->clip_prog,
                         nullptr);
    }
    if (rc) return fail(rc);
    for (size_t k = 0; k < p->clip_prog.chains.size(); ++k) {
      if (k < n_pre) p->prefix_macs += p->clip_prog.chains[k].macs_per_img;
      else p->tail_macs += p->clip_prog.chains[k].macs_per_img;
    }
    // tail_macs is reported per window: with phase images, their MACs per clip / n_win
    if (!phases.empty()) p->tail_macs *= double(phases.size()) / double(n_win);
    assign_buffers(p->clip_prog, 1);
  }
  // ---- window program: every op per window ----
  {
    std::vector<Dims> od;
    rc = build_segment(p->ops, 0, n_ops, Dims{in_h, in_w, 1}, 1, {0}, int64_t(in_h) * in_w, in_w,
                       -1, p->split_f16, p->win_prog, &od);
    if (rc) return fail(rc);
    assign_buffers(p->win_prog, 1);
  }
  *plan = p;
  return HBK_OK;
}

int hbk_embed_plan_destroy(hbk_embed_plan* p) {
  if (!p) return HBK_OK;
  for (auto* prog : {&p->clip_prog, &p->win_prog}) {
    for (auto& c : prog->chains) {
      (void)hipFree(c.d_blob);
      if (c.d_p0) (void)hipFree(c.d_p0);
    }
    if (prog->d_gather) (void)hipFree(prog->d_gather);
  }
  if (p->d_range) (void)hipFree(p->d_range);
  delete p;
  return HBK_OK;
}

int hbk_embed_plan_info(const hbk_embed_plan* p, int32_t* out_dim, int32_t* n_prefix_ops,
                        int32_t* n_chains, double* prefix_macs, double* tail_macs,
                        int32_t* seq_frames) {
  if (!p) return hbk::arg_error("plan is NULL");
  if (out_dim) *out_dim = p->out_dim;
  if (n_prefix_ops) *n_prefix_ops = p->n_prefix;
  if (n_chains) *n_chains = static_cast<int32_t>(p->clip_prog.chains.size());
  if (prefix_macs) *prefix_macs = p->prefix_macs;
  if (tail_macs) *tail_macs = p->tail_macs;
  if (seq_frames) *seq_frames = p->seq_frames;
  return HBK_OK;
}

}  // extern "C"

namespace hbk {
namespace {

// Per-unit (clip or window) workspace floats of each ping-pong buffer and the
// images per unit of each chain.
void program_geometry(const Program& prog, bool clip_path, int n_win, std::vector<int64_t>& imgs,
                      std::vector<int64_t>& bufs) {
  imgs.clear();
  bufs.assign(2, 0);
  bool tail = false;
  int tail_imgs = n_win;
  for (size_t k = 0; k < prog.chains.size(); ++k) {
    const ChainPlan& c = prog.chains[k];
    const int ipc = c.split ? c.x.ipc : c.args.ipc;
    const int64_t ois = c.split ? c.x.out_img_stride : c.args.out_img_stride;
    if (clip_path && ipc > 1 && !tail) {
      tail = true;
      tail_imgs = ipc;  // n_win, or the phase images of a deduplicated tail
    }
    imgs.push_back(tail ? tail_imgs : 1);
    if (c.dst_buf >= 0) bufs[c.dst_buf] = std::max(bufs[c.dst_buf], ois * imgs.back());
  }
}

}  // namespace

// ---- NaN rows (embeddings.py:209-234): in place, no host synchronisation ----
// Three grid-wide launches, each a no-op past one load when the batch has no NaN row:
// nan_flags_kernel: block b owns the contiguous rows [b*per, (b+1)*per) (one wave per row,
//   float4 loads): flags[r] = 1 for a NaN row, which is appended to bad[] (meta[0] counts
//   them; the order is free, a row's draw depends on (seed, row) only), and blk_good[b] counts
//   the block's NaN-free rows.
// nan_list_kernel: block b lists its NaN-free rows in order at the offset sum(blk_good[< b])
//   (ballot scans over 256-row slices), so good[] is every NaN-free row, ascending.
// nan_patch_kernel: one wave per NaN row copies good[h % n_good], h a hash of (seed, row) — a
//   uniformly drawn NaN-free clip, as the reference's np.random.choice — or writes zeros when
//   every row is NaN.
constexpr int kNanBlocks = 2048;  // flags / list blocks at most (blk_good's length)
constexpr int kNanPatchBlocks = 512;

__global__ void __launch_bounds__(256) nan_flags_kernel(const float* __restrict__ rows, int64_t n, int64_t row_len,
                                                        int64_t per, int32_t* __restrict__ flags,
                                                        int32_t* __restrict__ blk_good, int32_t* __restrict__ bad,
                                                        int32_t* __restrict__ meta) {
  __shared__ int32_t s_good;
  if (threadIdx.x == 0) s_good = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t lo = static_cast<int64_t>(blockIdx.x) * per, hi = min<int64_t>(n, lo + per);
  int32_t n_good = 0;
  for (int64_t r = lo + wave; r < hi; r += 4) {
    const float4* p = reinterpret_cast<const float4*>(rows + r * row_len);
    bool nan = false;
    for (int64_t j = lane; j < row_len / 4; j += 64) {
      const float4 v = p[j];
      nan |= (v.x != v.x) | (v.y != v.y) | (v.z != v.z) | (v.w != v.w);
    }
    const bool any = __ballot(nan) != 0;
    if (lane == 0) {
      flags[r] = any ? 1 : 0;
      if (any)
        bad[atomicAdd(meta, 1)] = static_cast<int32_t>(r);
      else
        ++n_good;
    }
  }
  if (lane == 0) atomicAdd(&s_good, n_good);
  __syncthreads();
  if (threadIdx.x == 0) blk_good[blockIdx.x] = s_good;
}

__global__ void __launch_bounds__(256) nan_list_kernel(int64_t n, int64_t per, const int32_t* __restrict__ flags,
                                                       const int32_t* __restrict__ blk_good,
                                                       int32_t* __restrict__ good, const int32_t* __restrict__ meta) {
  __shared__ int32_t s_w[4];
  __shared__ int32_t s_off;
  if (meta[0] == 0) return;  // uniform: the common case
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int32_t off = 0;  // NaN-free rows of the blocks before this one
  for (int i = tid; i < static_cast<int>(blockIdx.x); i += 256) off += blk_good[i];
  for (int o = 32; o > 0; o >>= 1) off += __shfl_xor(off, o, 64);
  if (lane == 0) s_w[wave] = off;
  __syncthreads();
  if (tid == 0) s_off = s_w[0] + s_w[1] + s_w[2] + s_w[3];
  __syncthreads();
  off = s_off;
  const int64_t lo = static_cast<int64_t>(blockIdx.x) * per, hi = min<int64_t>(n, lo + per);
  for (int64_t base = lo; base < hi; base += 256) {
    const int64_t r = base + tid;
    const bool keep = r < hi && flags[r] == 0;
    const uint64_t m = __ballot(keep);
    const int32_t below = __popcll(m & ((uint64_t(1) << lane) - 1));
    __syncthreads();  // s_w of the previous slice has been read
    if (lane == 0) s_w[wave] = __popcll(m);
    __syncthreads();
    int32_t pre = 0;
    for (int w = 0; w < wave; ++w) pre += s_w[w];
    if (keep) good[off + pre + below] = static_cast<int32_t>(r);
    off += s_w[0] + s_w[1] + s_w[2] + s_w[3];
  }
}

__device__ __forceinline__ uint64_t nan_hash(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void __launch_bounds__(256) nan_patch_kernel(float* __restrict__ rows, int64_t n, int64_t row_len,
                                                        const int32_t* __restrict__ bad,
                                                        const int32_t* __restrict__ good,
                                                        const int32_t* __restrict__ meta, uint64_t seed) {
  const int64_t n_bad = meta[0];
  if (n_bad == 0) return;
  const int64_t n_good = n - n_bad;
  const int lane = threadIdx.x & 63;
  const int64_t nw = static_cast<int64_t>(gridDim.x) * 4;
  for (int64_t i = (static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x) >> 6; i < n_bad; i += nw) {
    const int64_t r = bad[i];
    float4* dst = reinterpret_cast<float4*>(rows + r * row_len);
    if (n_good == 0) {
      for (int64_t j = lane; j < row_len / 4; j += 64) dst[j] = float4{0.f, 0.f, 0.f, 0.f};
      continue;
    }
    const uint64_t h = nan_hash(seed ^ (0x9E3779B97F4A7C15ull * static_cast<uint64_t>(r + 1)));
    const int64_t src = good[static_cast<int64_t>((static_cast<unsigned __int128>(h) * static_cast<uint64_t>(n_good)) >> 64)];
    const float4* sp = reinterpret_cast<const float4*>(rows + src * row_len);
    for (int64_t j = lane; j < row_len / 4; j += 64) dst[j] = sp[j];
  }
}

}  // namespace hbk

extern "C" {

int hbk_embed_workspace_size(const hbk_embed_plan* p, int64_t n, int64_t* bytes) {
  using namespace hbk;
  if (!p || !bytes) return arg_error("plan/bytes is NULL");
  if (n < 0) return arg_error("negative n");
  const int64_t chunk = std::max<int64_t>(1, std::min<int64_t>(n, chunk_clips()));
  std::vector<int64_t> imgs, bc, bw;
  program_geometry(p->clip_prog, true, int(p->starts.size()), imgs, bc);
  const int64_t chunk_w = std::max<int64_t>(1, std::min<int64_t>(n, chunk_clips()));
  program_geometry(p->win_prog, false, 1, imgs, bw);
  const int64_t fc = chunk * (bc[0] + bc[1]);
  const int64_t fw = chunk_w * (bw[0] + bw[1]);
  *bytes = std::max(fc, fw) * int64_t(sizeof(float)) + 256;
  return HBK_OK;
}

int hbk_embed_clips(const hbk_embed_plan* p, const float* mel, int64_t n_clips, int64_t mel_clip_stride,
                    float* out, void* workspace, int64_t workspace_bytes, void* stream) {
  using namespace hbk;
  if (!p) return arg_error("plan is NULL");
  if (n_clips < 0) return arg_error("negative n_clips");
  if (n_clips == 0) return HBK_OK;
  if (!mel || !out || !workspace) return arg_error("NULL pointer");
  if (mel_clip_stride < int64_t(p->seq_frames) * p->in_w) return arg_error("mel_clip_stride < seq_frames * in_w");
  int64_t need = 0;
  hbk_embed_workspace_size(p, n_clips, &need);
  if (workspace_bytes < need) return arg_error("workspace too small");
  std::vector<int64_t> imgs, bufs;
  program_geometry(p->clip_prog, true, int(p->starts.size()), imgs, bufs);
  const int64_t chunk = std::min<int64_t>(n_clips, chunk_clips());
  return run_program(p->clip_prog, mel, n_clips, mel_clip_stride, out,
                     int64_t(p->starts.size()) * p->out_dim, static_cast<float*>(workspace), chunk,
                     as_stream(stream), imgs, bufs, p->d_range);
}

int hbk_embed_split_info(const hbk_embed_plan* p, int32_t n_front, int64_t* mid_floats_per_clip) {
  using namespace hbk;
  if (!p || !mid_floats_per_clip) return arg_error("plan/mid_floats_per_clip is NULL");
  const int n = static_cast<int>(p->clip_prog.chains.size());
  if (n_front < 1 || n_front >= n) return arg_error("n_front must be in [1, n_chains - 1]");
  std::vector<int64_t> imgs, bufs;
  program_geometry(p->clip_prog, true, int(p->starts.size()), imgs, bufs);
  const ChainPlan& c = p->clip_prog.chains[n_front - 1];
  *mid_floats_per_clip = (c.split ? c.x.out_img_stride : c.args.out_img_stride) * imgs[n_front - 1];
  return HBK_OK;
}

int hbk_embed_clips_front(const hbk_embed_plan* p, const float* mel, int64_t n_clips, int64_t mel_clip_stride,
                          int32_t n_front, float* mid, void* workspace, int64_t workspace_bytes, void* stream) {
  using namespace hbk;
  int64_t mid_floats = 0;
  int rc = hbk_embed_split_info(p, n_front, &mid_floats);
  if (rc) return rc;
  if (n_clips < 0) return arg_error("negative n_clips");
  if (n_clips == 0) return HBK_OK;
  if (!mel || !mid || !workspace) return arg_error("NULL pointer");
  if (mel_clip_stride < int64_t(p->seq_frames) * p->in_w) return arg_error("mel_clip_stride < seq_frames * in_w");
  int64_t need = 0;
  hbk_embed_workspace_size(p, n_clips, &need);
  if (workspace_bytes < need) return arg_error("workspace too small");
  std::vector<int64_t> imgs, bufs;
  program_geometry(p->clip_prog, true, int(p->starts.size()), imgs, bufs);
  const int64_t chunk = std::min<int64_t>(n_clips, chunk_clips());
  return run_program(p->clip_prog, mel, n_clips, mel_clip_stride, mid, mid_floats, static_cast<float*>(workspace),
                     chunk, as_stream(stream), imgs, bufs, p->d_range, 0, n_front);
}

int hbk_embed_clips_back(const hbk_embed_plan* p, const float* mid, int64_t n_clips, int32_t n_front, float* out,
                         void* workspace, int64_t workspace_bytes, void* stream) {
  using namespace hbk;
  int64_t mid_floats = 0;
  int rc = hbk_embed_split_info(p, n_front, &mid_floats);
  if (rc) return rc;
  if (n_clips < 0) return arg_error("negative n_clips");
  if (n_clips == 0) return HBK_OK;
  if (!mid || !out || !workspace) return arg_error("NULL pointer");
  int64_t need = 0;
  hbk_embed_workspace_size(p, n_clips, &need);
  if (workspace_bytes < need) return arg_error("workspace too small");
  std::vector<int64_t> imgs, bufs;
  program_geometry(p->clip_prog, true, int(p->starts.size()), imgs, bufs);
  const int64_t chunk = std::min<int64_t>(n_clips, chunk_clips());
  return run_program(p->clip_prog, mid, n_clips, mid_floats, out, int64_t(p->starts.size()) * p->out_dim,
                     static_cast<float*>(workspace), chunk, as_stream(stream), imgs, bufs, p->d_range, n_front, -1);
}

int hbk_embed_windows(const hbk_embed_plan* p, const float* windows, int64_t n, float* out,
                      void* workspace, int64_t workspace_bytes, void* stream) {
  using namespace hbk;
  if (!p) return arg_error("plan is NULL");
  if (n < 0) return arg_error("negative n");
  if (n == 0) return HBK_OK;
  if (!windows || !out || !workspace) return arg_error("NULL pointer");
  int64_t need = 0;
  hbk_embed_workspace_size(p, n, &need);
  if (workspace_bytes < need) return arg_error("workspace too small");
  std::vector<int64_t> imgs, bufs;
  program_geometry(p->win_prog, false, 1, imgs, bufs);
  const int64_t chunk = std::min<int64_t>(n, chunk_clips());
  return run_program(p->win_prog, windows, n, int64_t(p->in_h) * p->in_w, out, p->out_dim,
                     static_cast<float*>(workspace), chunk, as_stream(stream), imgs, bufs, p->d_range);
}

int64_t hbk_nan_rows_workspace_size(int64_t n) {
  return n < 0 ? 0 : (3 * n + hbk::kNanBlocks + 1) * int64_t(sizeof(int32_t));
}

int hbk_nan_rows_fix(float* rows, int64_t n, int64_t row_len, uint64_t seed, void* workspace,
                     int64_t workspace_bytes, void* stream) {
  using namespace hbk;
  if (n < 0 || row_len <= 0 || row_len % 4) return arg_error("n >= 0, row_len a positive multiple of 4");
  if (n == 0) return HBK_OK;
  if (n >= (int64_t(1) << 31)) return arg_error("n >= 2^31 rows");
  if (!rows || !workspace) return arg_error("NULL pointer");
  if ((reinterpret_cast<uintptr_t>(rows) & 15)) return arg_error("rows must be 16-B aligned");
  if (workspace_bytes < hbk_nan_rows_workspace_size(n)) return arg_error("workspace too small");
  int32_t* flags = static_cast<int32_t*>(workspace);  // [n]
  int32_t* good = flags + n;                          // [n]
  int32_t* bad = good + n;                            // [n]
  int32_t* blk_good = bad + n;                        // [kNanBlocks]
  int32_t* meta = blk_good + kNanBlocks;              // [1]: NaN rows
  hipStream_t st = as_stream(stream);
  hipError_t e = hipMemsetAsync(meta, 0, sizeof(int32_t), st);
  if (e != hipSuccess) return hip_error(e, "hbk_nan_rows_fix");
  const int64_t blocks = std::min<int64_t>(kNanBlocks, (n + 3) / 4);
  const int64_t per = (n + blocks - 1) / blocks;
  const int64_t used = (n + per - 1) / per;  // every launched block owns at least one row
  hipLaunchKernelGGL(nan_flags_kernel, dim3(unsigned(used)), dim3(256), 0, st, rows, n, row_len, per, flags,
                     blk_good, bad, meta);
  HBK_LAUNCH_CHECK("nan_flags_kernel");
  hipLaunchKernelGGL(nan_list_kernel, dim3(unsigned(used)), dim3(256), 0, st, n, per, flags, blk_good, good, meta);
  HBK_LAUNCH_CHECK("nan_list_kernel");
  const int64_t pblocks = std::min<int64_t>(kNanPatchBlocks, (n + 3) / 4);
  hipLaunchKernelGGL(nan_patch_kernel, dim3(unsigned(pblocks)), dim3(256), 0, st, rows, n, row_len, bad, good, meta,
                     seed);
  HBK_LAUNCH_CHECK("nan_patch_kernel");
  return HBK_OK;
}

int hbk_embed_range_status(const hbk_embed_plan* p, int32_t* tripped, int32_t reset, void* stream) {
  using namespace hbk;
  if (!p || !tripped) return arg_error("plan/tripped is NULL");
  int32_t h = 0;
  hipError_t e = hipMemcpyAsync(&h, p->d_range, sizeof(int32_t), hipMemcpyDeviceToHost, as_stream(stream));
  if (e == hipSuccess) e = hipStreamSynchronize(as_stream(stream));
  if (e == hipSuccess && reset && h) e = hipMemsetAsync(p->d_range, 0, sizeof(int32_t), as_stream(stream));
  if (e != hipSuccess) return hip_error(e, "hbk_embed_range_status");
  *tripped = h;
  return HBK_OK;
}

}  // extern "C"

#ifdef HBK_PHASE_TIMING
extern "C" int hbk_debug_phase_cycles(unsigned long long* out, int n) {
  unsigned long long h[64];
  if (hipMemcpyFromSymbol(h, HIP_SYMBOL(hbk::g_phase_cycles), sizeof(h)) != hipSuccess) return -2;
  for (int i = 0; i < n && i < 64; ++i) out[i] = h[i];
  unsigned long long z[64] = {};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(hbk::g_phase_cycles), z, sizeof(z));
  return 0;
}
#endif

#ifdef HBK_TRACE
extern "C" int hbk_debug_trace(unsigned long long* out, int* counts) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(hbk::g_trace), sizeof(unsigned long long) * 4 * 4 * 256) != hipSuccess)
    return -2;
  if (hipMemcpyFromSymbol(counts, HIP_SYMBOL(hbk::g_trace_n), sizeof(int) * 16) != hipSuccess) return -2;
  int z[16] = {};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(hbk::g_trace_n), z, sizeof(z));
  return 0;
}
#endif
