// Fused wake-word classifier train step for gfx950 (default architecture:
// d_in = 16 x 96 = 1536, layer_dim 96, hidden get_normalized_dim(96) = 64,
// 0..2 layers; other plans use the generic GEMM path of hbk_mlp.hip).
//
// Replaces, per optimisation step of WakeWordTrainer.train_epoch
// (trainer.py:380-494), the reference's forward (wakeword.py:334-348), the
// high-loss filter and weighted BCE (:407-445), autograd backward and
// torch.optim.Adam (:45, :460-462), with FOUR launches and no host sync:
//
//   k1a        gather the batch rows from the embedding pools by index (f32
//              or f16 pool), input dropout, LayerNorm(1536) -> xhat^T in HBM.
//              It needs no weights, so step s + 1's k1a runs as extra
//              workgroups of step s's k2 launch, two row tiles each (k2 fills
//              35 of 256 CUs at B = 1100, two workgroups per CU) and is off
//              the critical path; a standalone launch covers the first step
//              and steps without a known successor
//   k1b        the input GEMM HG0 = (xhat g + b) W_hg0^T as split-K partial
//              slabs (row tiles of 16 x K-chunks: ~576 workgroups at B = 1100)
//   k2_rows    per 16-row tile, the whole rest of the network in LDS:
//              sum of the HG0 partials + bias, SiLU gate, every gated MLP and
//              LayerNorm forward, sigmoid, the high-loss filter, weighted BCE
//              statistics and dL/dz, then the backward chain down to dHG0;
//              bias and LayerNorm(96) gradients as per-tile column sums
//              (float atomics); activations for the weight gradients to HBM
//   k3_wgrad   every weight gradient dW = dY^T X as split-K MFMA tiles with
//              atomic accumulation into the gradient bucket; the input layer's
//              tiles also produce the norm_in gamma/beta gradients from the
//              same product (dW_hg0 = g o (dHG0^T xhat) + beta (x) colsum dHG0,
//              dgamma = sum_j W o (dHG0^T xhat), dbeta = colsum(dHG0) W_hg0;
//              colsum dHG0 itself = the hidden/gate bias gradient, from k2)
//   [RCCL all-reduce of the bucket between k3 and k4 when data-parallel]
//   k4_update  the < 128-sample accumulation gate, Adam, and zeroing of the
//              bucket for the next step
//
// GEMMs are split-f16 products (hi*hi + hi*lo + lo*hi of f16 hi / lo parts,
// f32 accumulation, operands power-of-two scaled into the f16 range): ~22-bit
// products, so results differ from the f32 reference at the level of its own
// summation-order differences; everything else is f32.
//
// Step state lives on the device and is PING-PONGED: state[2][8] floats
// (acc_samples, acc_steps, adam_t, step, -, -, -, -); step s reads half
// (s & 1) and k4 writes half 1 - (s & 1). No kernel of a step therefore writes
// anything another workgroup of the same step reads, and a hipGraph of an even
// number of steps replays them all. The step index selects the batch's row
// indices (idx + step * idx_stride) and the LR / negative weight
// (sched[step]), so one captured graph covers a whole stage.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <initializer_list>
#include <utility>
#include <cmath>
#include <cstdio>

#include "hbk_common.h"
#include "hbk_mlp_internal.h"

namespace hbk {
namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));

constexpr int kD = 1536, kL = 96, kH = 64, kH2 = 128;
constexpr int kR = 16;            // rows per tile = MFMA M
constexpr int kMaxG = 4;          // gated MLPs held by k2 (n_layers <= 2: the LDS budget)
constexpr int kStats = 8;
constexpr float kLnEps = 1e-5f;
constexpr int kLd = 132;          // LDS row stride of [16][<=128] activation tiles
constexpr int kChunkMax = 384;    // k1 K-chunk

__device__ __forceinline__ f4 mma(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
// wave sum through DPP: quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror,
// row_mirror leave each 16-lane row's sum in all of its lanes (rsum16); the
// four rows are then added from readlane (a bpermute-based __shfl_xor chain
// costs an LDS round trip per step)
template <int CTRL>
__device__ __forceinline__ float dpp_f(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float rsum16(float v) {
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0x141>(v);
  v += dpp_f<0x140>(v);
  return v;
}
__device__ __forceinline__ float wsum(float v) {
  v = rsum16(v);
  const int b = __builtin_bit_cast(int, v);
  return (__builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 0)) +
          __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 16))) +
         (__builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 32)) +
          __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 48)));
}
__device__ __forceinline__ float wmax(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x141>(v));
  v = fmaxf(v, dpp_f<0x140>(v));
  const int b = __builtin_bit_cast(int, v);
  return fmaxf(fmaxf(__builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 0)),
                     __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 16))),
               fmaxf(__builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 32)),
                     __builtin_bit_cast(float, __builtin_amdgcn_readlane(b, 48))));
}
__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }
// The gates (train step and evaluation) and the evaluation's output: the hardware
// exp2 and reciprocal (1 ulp each) instead of expf's range reduction and the IEEE
// division sequence (~20 VALU instructions per sigmoid, on k2's dependent
// stages); values move by ~1e-7 relative (the tests' tolerances are >= 1e-5, and
// their counts allow predictions that near the threshold). The train step's loss
// stage keeps sigm (its high-loss filter compares p with thresholds).
__device__ __forceinline__ float sigm_fast(float x) {
  return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-1.44269504088896341f * x));
}

// Barrier of a loop with global->LDS DMA in flight (its waits counted by hand
// before it): a fenced barrier would wait vmcnt(0), as the DMA writes LDS. The
// empty asm statements keep the compiler from moving memory accesses across.
__device__ __forceinline__ void dma_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
// Workgroup barrier for LDS traffic only (the evaluation network's stages):
// the release / acquire fences are restricted to the local address space, so
// the barrier waits for the wave's LDS operations (lgkmcnt) but not for the
// next stage's weight loads in flight (a plain __syncthreads() waits vmcnt(0)
// too). Its waves hand nothing to each other through global memory. (In the
// train step's k2 the same change measured no difference: 36.89 vs 36.89 us.)
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}


#ifdef HBK_TRACE
// Tracing build only (lib/libhbk_trace.so, tools/probe_mlp.py): lane 0 of every
// wave of block 0 records (mark << 56 | s_memtime) at stage marks of k1 / k2 / k3.
// Slots: kTraceKerns kernels x kTraceWaves waves. Every mark is bound-checked on
// both (r04: the k4 marks at kernel slots 4 and 5 wrote past a [4]-kernel array --
// the hipErrorIllegalAddress of gpurun_out/trace64.log -- until the array grew to 6).
constexpr int kTraceKerns = 6, kTraceWaves = 4;
static_assert(kTraceWaves * 64 >= 256, "every traced kernel runs <= 256 threads (4 waves)");
__device__ unsigned long long g_mlp_trace[kTraceKerns][kTraceWaves][128];
__device__ int g_mlp_trace_n[kTraceKerns][kTraceWaves];
#define HBK_MTB(kern, id, blk)                                                                       \
  do {                                                                                         \
    static_assert((kern) >= 0 && (kern) < kTraceKerns, "trace kernel slot out of range");     \
    if (blockIdx.x == (blk) && (threadIdx.x & 63) == 0 && (threadIdx.x >> 6) < kTraceWaves) {   \
      const int w_ = threadIdx.x >> 6;                                                          \
      const int n_ = g_mlp_trace_n[kern][w_];                                                   \
      if (n_ < 128) {                                                                           \
        g_mlp_trace[kern][w_][n_] = (static_cast<unsigned long long>(id) << 56) |               \
                                    (__builtin_amdgcn_s_memtime() & 0xFFFFFFFFFFFFFFull);       \
        g_mlp_trace_n[kern][w_] = n_ + 1;                                                       \
      }                                                                                         \
    }                                                                                           \
  } while (0)
#define HBK_MT(kern, id) HBK_MTB(kern, id, 0)
// per-block spans of one kernel (k3s): {start, end} s_memrealtime (100 MHz, device-wide) and
// the block's job / split
__device__ unsigned long long g_span[1024][3];
#define HBK_SPAN(slot, v)                                                               \
  do {                                                                                  \
    if (threadIdx.x == 0 && blockIdx.x < 1024) g_span[blockIdx.x][slot] = (v);           \
  } while (0)
#else
#define HBK_SPAN(slot, v) \
  do {                    \
  } while (0)
#define HBK_MT(kern, id) \
  do {                   \
  } while (0)
#define HBK_MTB(kern, id, blk) \
  do {                         \
  } while (0)
#endif

#ifdef HBK_BOUNDS
// Bounds-checked build (lib/libhbk_bounds.so, tools/probe_bounds.py): the step
// kernels' global accesses go through BCK, which checks them against the ranges
// the host registered for the call (workspace, parameters, pools, ...); the first
// violation is recorded (source line, block, thread, address) and the access is
// redirected to a scratch buffer, so a bad index shows up as a record instead of
// a GPU memory fault.
constexpr int kBMax = 16;
__device__ unsigned long long g_brange[kBMax][2];
__device__ int g_bn;
__device__ unsigned long long g_berr[4];
__device__ __attribute__((aligned(16))) char g_bsafe[1 << 16];
template <typename T>
__device__ __forceinline__ T* bck_(T* p, int nbytes, int line) {
  const unsigned long long c = reinterpret_cast<unsigned long long>(p);
  bool ok = false;
  for (int i = 0; i < kBMax; ++i) ok |= i < g_bn && c >= g_brange[i][0] && c + nbytes <= g_brange[i][1];
  if (ok) return p;
  if (atomicCAS(&g_berr[0], 0ull, static_cast<unsigned long long>(line)) == 0ull) {
    g_berr[1] = blockIdx.x;
    g_berr[2] = threadIdx.x;
    g_berr[3] = c;
  }
  return reinterpret_cast<T*>(g_bsafe);
}
#define BCK(p, n) bck_((p), (n), __LINE__)
#else
#define BCK(p, n) (p)
#endif

__device__ __forceinline__ int step_of(const float* state, int parity) {
  return state ? static_cast<int>(state[parity * 8 + 3]) : 0;
}

// ------------------------------------------------------------------ k1 ----
struct K1aArgs {
  const float* pool32;
  const _Float16* pool16;
  int64_t n32, n16;    // pool rows; an index outside its pool reads as a zero row
  const int32_t* idx;  // row r of the step's batch: >= 0 pool32 row, < 0 pool16 row -idx-1; NULL = r
  int64_t idx_stride;
  int64_t idx_steps;   // rows of idx (steps) available: no prefetch past the last
  const float* state;
  int parity;
  int B;
  float drop_p;
  uint64_t seed;
  float* xhat[2];      // TRANSPOSED [1536][Bp] (rows >= B zero), by step parity (v1 step)
  int64_t Bp;
  // v2 step (the default): per row of the step, by parity, its LayerNorm statistics
  // and the row's address {mu, rs, addr lo, addr hi} (mu / rs as float bits; addr =
  // the row's first byte in its pool with bit 0 set for an f16 row: consumers address
  // rows without branches; a zero row points at a valid row of its pool) and its
  // dropout mask (bit c of word c / 32 set = element c dropped; a zero row has every
  // bit set, and mu = 0); no xhat^T
  uint4* rinfo[2];     // [Bp]
  uint32_t* mask[2];   // [Bp][48]
};

struct K1bArgs {
  const float* P;
  int64_t g_in, b_in, w0;
  int B;
  const float* xhat;  // this step's xhat^T
  int64_t Bp;
  float* hg_part;     // [KS][B][128]
  float* stats;       // bucket tail, zeroed here (k2 accumulates into it); may be NULL
};

// 32-bit counter hash for the input dropout mask (murmur3's finaliser over
// the element-pair index mixed with the step's 64-bit seed): one hash gives
// the 16-bit uniforms of elements 2 i and 2 i + 1 (p resolved to 2^-16).
__device__ __forceinline__ uint32_t drop_hash(uint32_t s0, uint32_t s1, uint32_t i) {
  uint32_t h = i * 0x9E3779B1u + s0;
  h ^= s1;
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

// k1a: one 16-row tile, full width. Every loop is unrolled and every global
// load unconditional (a row outside its pool reads a valid fallback row and is
// zeroed afterwards), so the vmcnt waits are exact and a wave's four rows are
// in flight together: one 16-B load per lane per 256 f32 / 512 f16 elements,
// the f16 row re-reading its first half for slots 3..5. Lane value j holds
// element 4 (lane + 64 (j / 4)) + j % 4 (f32 rows) or 8 (lane + 64 (j / 8)) +
// j % 8 (f16 rows): either way values 8 t .. 8 t + 7 fall in columns
// [512 t, 512 t + 512), so xhat^T is written in three 512-column slabs staged
// through LDS (slab: [16][516] floats) as 64-B column runs.
constexpr int kSlabLd = 516;
constexpr int kPreTiles = 2;    // k1a row tiles per prefetch workgroup of k2 (v1)
constexpr int kPreTiles2 = 3;   // k1s (v2: statistics and mask only) row tiles per prefetch workgroup (2: 84.0, 3: 83.6, 4: 86.0 us per step)
constexpr int kMaskW = kD / 32;  // mask words per row
// kV2: the row statistics and dropout mask (rinfo, mask) instead of xhat^T; slab is then
// >= 4 waves x 4 rows x 1536 bytes of LDS scratch (the mask's byte image)
template <bool kIdx, bool kV2 = false>
__device__ __forceinline__ void k1a_tile(const K1aArgs& a, int rt, int step, float* __restrict__ xout,
                                         float* slab, int dpar = 0) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const uint64_t seed = a.seed + static_cast<uint64_t>(step) +
                        (a.state ? static_cast<uint64_t>(a.state[a.parity * 8 + 4]) << 24 : 0);
  const uint32_t s0 = static_cast<uint32_t>(seed), s1 = static_cast<uint32_t>(seed >> 32) * 0x27D4EB2Fu;
  const char* fallback = a.pool32 ? reinterpret_cast<const char*>(a.pool32) : reinterpret_cast<const char*>(a.pool16);
  int ixs[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    ixs[i] = min(rt * kR + wave * 4 + i, a.B - 1);
    if (kIdx) ixs[i] = *BCK(&a.idx[static_cast<int64_t>(step) * a.idx_stride + ixs[i]], 4);
  }
  uint4 raw[4][6];
  bool is16[4], ok[4];
  const char* rowptr[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = rt * kR + wave * 4 + i;
    const int ix = __builtin_amdgcn_readfirstlane(ixs[i]);
    is16[i] = ix < 0;
    const int64_t row16 = -static_cast<int64_t>(ix) - 1;
    ok[i] = r < a.B && (is16[i] ? row16 < a.n16 : ix < a.n32);
    const char* bp = !ok[i] ? fallback
                     : is16[i] ? reinterpret_cast<const char*>(a.pool16 + row16 * kD)
                               : reinterpret_cast<const char*>(a.pool32 + static_cast<int64_t>(ix) * kD);
    rowptr[i] = bp;
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      const int slot = is16[i] ? u % 3 : u;
      raw[i][u] = *BCK(reinterpret_cast<const uint4*>(bp + 16 * (lane + 64 * slot)), 16);
    }
  }
  const float keep = a.drop_p > 0.f ? 1.f / (1.f - a.drop_p) : 1.f;
  const uint32_t thr = static_cast<uint32_t>(a.drop_p * 65536.f + 0.5f);
  float xh[4][kV2 ? 1 : 24];
  unsigned char* mimg = reinterpret_cast<unsigned char*>(slab) + (wave * 4) * kD;  // v2: [4 rows][1536] flag bytes
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = rt * kR + wave * 4 + i;
    float v[24];
    int c[24];
    bool dr[24];  // element dropped (v2's mask; a zero row drops everything)
#pragma unroll
    for (int j = 0; j < 24; ++j) {
      const uint4 w16 = raw[i][j >> 3];
      const uint32_t word16 = (&w16.x)[(j & 7) >> 1];
      const _Float16 h = __builtin_bit_cast(_Float16, static_cast<uint16_t>((j & 1) ? word16 >> 16 : word16));
      const uint4 w32 = raw[i][j >> 2];
      const float f = __builtin_bit_cast(float, (&w32.x)[j & 3]);
      v[j] = ok[i] ? (is16[i] ? static_cast<float>(h) : f) : 0.f;
      c[j] = is16[i] ? 8 * (lane + 64 * (j >> 3)) + (j & 7) : 4 * (lane + 64 * (j >> 2)) + (j & 3);
      dr[j] = !ok[i];
    }
    if (a.drop_p > 0.f) {  // nn.Dropout on the input (wakeword.py:197, :338): one hash per element pair
      const uint32_t base = static_cast<uint32_t>(r) * (kD / 2);
#pragma unroll
      for (int j = 0; j < 24; j += 2) {
        const uint32_t hsh = drop_hash(s0, s1, base + (c[j] >> 1));
        const bool d0 = (hsh & 0xFFFFu) < thr, d1 = (hsh >> 16) < thr;
        v[j] = d0 ? 0.f : v[j] * keep;
        v[j + 1] = d1 ? 0.f : v[j + 1] * keep;
        dr[j] = dr[j] || d0;
        dr[j + 1] = dr[j + 1] || d1;
      }
    }
    float sm = 0.f;
#pragma unroll
    for (int j = 0; j < 24; ++j) sm += v[j];
    const float mu = wsum(sm) * (1.f / kD);
    float sq = 0.f;
#pragma unroll
    for (int j = 0; j < 24; ++j) sq += (v[j] - mu) * (v[j] - mu);
    const float rs = __builtin_amdgcn_rsqf(wsum(sq) * (1.f / kD) + kLnEps);
    const bool live = r < a.B;
    if constexpr (kV2) {
      // the flag bytes of this row: lane's elements are 4 (f32) / 8 (f16) consecutive per slot
      unsigned char* row = mimg + i * kD;
#pragma unroll
      for (int q = 0; q < 6; ++q) {
        const uint32_t b4 = (dr[4 * q] ? 1u : 0u) | (dr[4 * q + 1] ? 0x100u : 0u) | (dr[4 * q + 2] ? 0x10000u : 0u) |
                            (dr[4 * q + 3] ? 0x1000000u : 0u);
        const int off = is16[i] ? 8 * lane + 512 * (q >> 1) + 4 * (q & 1) : 4 * lane + 256 * q;
        *reinterpret_cast<uint32_t*>(row + off) = b4;
      }
      if (lane == 0) {
        // a zero row's loads read its fallback row as that pool's dtype (in bounds either way)
        const bool h = ok[i] ? is16[i] : a.pool32 == nullptr;
        const uint64_t addr = reinterpret_cast<uint64_t>(rowptr[i]) | (h ? 1u : 0u);
        *BCK(&a.rinfo[dpar][r], 16) =
            uint4{__float_as_uint(live ? mu : 0.f), __float_as_uint(live ? rs : 0.f), static_cast<uint32_t>(addr),
                  static_cast<uint32_t>(addr >> 32)};
      }
    } else {
#pragma unroll
      for (int j = 0; j < 24; ++j) xh[i][j] = live ? (v[j] - mu) * rs : 0.f;
    }
  }
  if constexpr (kV2) {
    // 32 flag bytes -> one mask word per lane (lanes 0..47), four rows
    __syncthreads();
    uint32_t* mdst = a.mask[dpar];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = rt * kR + wave * 4 + i;
      if (lane < kMaskW) {
        const uint4* src = reinterpret_cast<const uint4*>(mimg + i * kD + 32 * lane);
        const uint4 b0 = src[0], b1 = src[1];
        const uint32_t d[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
        uint32_t wd = 0;
#pragma unroll
        for (int e = 0; e < 8; ++e) wd |= ((d[e] * 0x01020408u) >> 24 & 0xFu) << (4 * e);  // 4 flag bytes -> 4 bits
        *BCK(&mdst[static_cast<int64_t>(r) * kMaskW + lane], 4) = wd;
      }
    }
    return;
  }
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    __syncthreads();  // the slab's previous readers are done
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float* row = slab + (wave * 4 + i) * kSlabLd;
#pragma unroll
      for (int jj = 0; jj < 8; ++jj) {
        const int j = 8 * t + jj;
        const int col = is16[i] ? 8 * lane + jj : 4 * lane + (jj & 3) + 256 * (jj >> 2);
        row[col] = xh[i][j];
      }
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int col = tid + 256 * h;
      float* dst = xout + static_cast<int64_t>(512 * t + col) * a.Bp + rt * kR;
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4)
        *reinterpret_cast<f4*>(dst + 4 * q4) =
            f4{slab[(4 * q4) * kSlabLd + col], slab[(4 * q4 + 1) * kSlabLd + col],
               slab[(4 * q4 + 2) * kSlabLd + col], slab[(4 * q4 + 3) * kSlabLd + col]};
    }
  }
}

// Standalone k1a: the step's own xhat (next = 0) or its successor's (next = 1).
template <bool kIdx>
__global__ void __launch_bounds__(256) k1a_kernel(K1aArgs a, int next) {
  __shared__ __attribute__((aligned(16))) float slab[kR * kSlabLd];
  const int step = step_of(a.state, a.parity) + next;
  if (kIdx && next && step >= a.idx_steps) return;
  HBK_MT(0, 1);
  k1a_tile<kIdx>(a, blockIdx.x, step, a.xhat[a.parity ^ next], slab);
  HBK_MT(0, 2);
}
// Standalone k1s (v2): the step's (next = 0) or its successor's (next = 1) row
// statistics and dropout mask.
static_assert(kR * kSlabLd * 4 >= 16 * kD, "k1s: the mask image fits the slab");
template <bool kIdx>
__global__ void __launch_bounds__(256) k1s_kernel(K1aArgs a, int next) {
  __shared__ __attribute__((aligned(16))) float slab[kR * kSlabLd];
  const int step = step_of(a.state, a.parity) + next;
  if (kIdx && next && step >= a.idx_steps) return;
  k1a_tile<kIdx, true>(a, blockIdx.x, step, nullptr, slab, a.parity ^ next);
}

// Split-f16 products on v_mfma_f32_16x16x32_f16: v = hi + lo with hi = f16(v)
// and lo = f16(v - hi) (v - hi is exact in f32), so
// a . b ~ hi_a hi_b + hi_a lo_b + lo_a hi_b: three f16 MFMAs (16 cycles each
// per 16x16x32) for the 8 f32 MFMAs (32 cycles each) of the same 32-deep
// product. hi is rounded to nearest (v_cvt_pk_f16_f32), so |lo| <= 2^-11 |x|
// with either sign and the dropped lo_a lo_b is an unbiased ~2^-22 relative
// term (a round-toward-zero hi makes it up to 2^-20 and one-signed, a bias that
// survives long sums). lo = x - hi is exact in f32 before its rounding to f16.
// Plain vector code (cvt_pk, two cvt back, pk_fma, cvt_pk per pair): the
// compiler sees every operand and places the wait states itself. Callers keep
// |x| < 2^15.
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
typedef float f2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void split_pair(float a, float b, uint32_t& hi, uint32_t& lo) {
  const h2v h = __builtin_convertvector(f2v{a, b}, h2v);
  const f2v r = f2v{a, b} - __builtin_convertvector(h, f2v);
  hi = __builtin_bit_cast(uint32_t, h);
  lo = __builtin_bit_cast(uint32_t, __builtin_convertvector(r, h2v));
}
// 8 floats (two f4) -> hi / lo h8
__device__ __forceinline__ void split8(const f4& x0, const f4& x1, h8& hi, h8& lo) {
  uint32_t h[4], l[4];
  split_pair(x0[0], x0[1], h[0], l[0]);
  split_pair(x0[2], x0[3], h[1], l[1]);
  split_pair(x1[0], x1[1], h[2], l[2]);
  split_pair(x1[2], x1[3], h[3], l[3]);
  typedef uint32_t u4 __attribute__((ext_vector_type(4)));
  hi = __builtin_bit_cast(h8, u4{h[0], h[1], h[2], h[3]});
  lo = __builtin_bit_cast(h8, u4{l[0], l[1], l[2], l[3]});
}
__device__ __forceinline__ f4 mma3(const h8& ah, const h8& al, const h8& bh, const h8& bl, f4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah, bl, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(al, bh, c, 0, 0, 0);
}

// k1b: HG0 partials for 64 rows x one K-chunk per workgroup (4 MFMA row tiles
// share each W fragment: W is read from L2 ceil(B / 64) times per step, not
// ceil(B / 16)). Grid: the KS chunks of one 64-row block run on ONE XCD
// (blocks b and b + 8 share an XCD under round-robin dispatch; speed only).
// KS is a template argument: all loads unconditional and issued together (the
// xhat^T tile, norm_in's gamma / beta, the chunk's W_hg0 fragments), then the
// unrolled split-f16 chain. W is scaled by 16 before the split (keeps lo of
// |W| ~ 1e-2 in f16's normal range); the sums are scaled back exactly.
constexpr int kRB = 64;
template <int KS>
__global__ void __launch_bounds__(256) k1b_kernel(K1bArgs a) {
  constexpr int kChunk = kD / KS, kN32 = kChunk / 32, kXl = kChunk / 16;  // xhat^T f4 loads per thread
  __shared__ __attribute__((aligned(16))) float xn[kRB][kChunk + 4];  // xhat of the chunk
  __shared__ __attribute__((aligned(16))) float gb[2][kChunk];        // norm_in gamma, beta of the chunk
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q = blockIdx.x >> 3;
  const int ks = q % KS, rb = (q / KS) * 8 + (blockIdx.x & 7);
  const int r0 = rb * kRB;
  if (r0 >= a.B) return;
  HBK_MT(3, 1);
  const int k0 = ks * kChunk;
  if (a.stats && rb == 0 && ks == 0 && tid < kStats) a.stats[tid] = 0.f;
  // xhat^T: column c holds the block's 64 rows as 16 float4; rows past Bp read
  // a clamped (valid) run, their outputs are never stored
  f4 xt[kXl];
#pragma unroll
  for (int h = 0; h < kXl; ++h) {
    const int e = tid + 256 * h, col = e >> 4;
    const int row = min(r0 + 4 * (e & 15), static_cast<int>(a.Bp) - 4);
    xt[h] = *reinterpret_cast<const f4*>(a.xhat + static_cast<int64_t>(k0 + col) * a.Bp + row);
  }
  float gv[2], bv[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int c = min(tid + 256 * h, kChunk - 1);
    gv[h] = a.P[a.g_in + k0 + c];
    bv[h] = a.P[a.b_in + k0 + c];
  }
  // W fragments: lane (n = m, kq) of column tile c holds W[32 w + 16 c + m][k0 + 32 i + 8 kq .. + 7]
  const int m = lane & 15, kq = lane >> 4;
  f4 wr[2][kN32][2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const float* wp = a.P + a.w0 + static_cast<int64_t>(32 * wave + 16 * c + m) * kD + k0 + 8 * kq;
#pragma unroll
    for (int i = 0; i < kN32; ++i) {
      wr[c][i][0] = *reinterpret_cast<const f4*>(wp + 32 * i);
      wr[c][i][1] = *reinterpret_cast<const f4*>(wp + 32 * i + 4);
    }
  }
#pragma unroll
  for (int h = 0; h < kXl; ++h) {
    const int e = tid + 256 * h, col = e >> 4, r4 = 4 * (e & 15);
#pragma unroll
    for (int u = 0; u < 4; ++u) xn[r4 + u][col] = xt[h][u];
  }
#pragma unroll
  for (int h = 0; h < 2; ++h)
    if (tid + 256 * h < kChunk) {
      gb[0][tid + 256 * h] = gv[h];
      gb[1][tid + 256 * h] = bv[h];
    }
  h8 whi[2][kN32], wlo[2][kN32];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int i = 0; i < kN32; ++i) split8(wr[c][i][0] * 16.f, wr[c][i][1] * 16.f, whi[c][i], wlo[c][i]);
  __syncthreads();
  HBK_MT(3, 2);
  // wave w -> output columns [32 w, 32 w + 32) of all 64 rows: 4 row tiles x 2
  // column tiles, A = LN output = xhat g + b from LDS (k = 32 i + 8 kq ..)
  f4 acc[4][2];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t][0] = acc[t][1] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i < kN32; ++i) {
    const int kk = 32 * i + 8 * kq;
    const f4 g0 = *reinterpret_cast<const f4*>(&gb[0][kk]), g1 = *reinterpret_cast<const f4*>(&gb[0][kk + 4]);
    const f4 b0 = *reinterpret_cast<const f4*>(&gb[1][kk]), b1 = *reinterpret_cast<const f4*>(&gb[1][kk + 4]);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float* xr = &xn[16 * t + m][kk];
      const f4 a0 = *reinterpret_cast<const f4*>(xr) * g0 + b0;
      const f4 a1 = *reinterpret_cast<const f4*>(xr + 4) * g1 + b1;
      h8 ah, al;
      split8(a0, a1, ah, al);
      acc[t][0] = mma3(ah, al, whi[0][i], wlo[0][i], acc[t][0]);
      acc[t][1] = mma3(ah, al, whi[1][i], wlo[1][i], acc[t][1]);
    }
  }
  float* out = a.hg_part + static_cast<int64_t>(ks) * a.B * kH2;
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int r = r0 + 16 * t + 4 * kq + e;
      if (r < a.B) {
        out[static_cast<int64_t>(r) * kH2 + 32 * wave + m] = acc[t][0][e] * (1.f / 16.f);
        out[static_cast<int64_t>(r) * kH2 + 32 * wave + 16 + m] = acc[t][1][e] * (1.f / 16.f);
      }
    }
  HBK_MT(3, 3);
}

// ------------------------------------------------------------ k1c (v2) ----
// The input GEMM from the embedding pools themselves: no xhat^T round trip
// through HBM (k1a wrote 6.8 MB per step at B = 1,100 and k1b and k3 read it
// back). Workgroup = 16 RT rows x one KC-deep K chunk, 8 waves; grid = row blocks
// x KS chunks, blockIdx = row block * KS + chunk, so the blocks of one chunk
// share an XCD (when KS % 8 == 0) and its W slice is read from that XCD's L2.
// Each thread stages 8-element runs of the block's rows: the raw pool values
// (f16 or f32 row, by k1s's source), the dropout mask bits, xhat = (v - mu) rs
// with k1s's statistics (the formula k1a used), then a = xhat g + b split into
// f16 hi / lo planes in LDS ONCE (k1b split per wave and fragment); wave w then
// multiplies every row tile by W's column tile w (16 W, pre-split in registers).
struct K1cArgs {
  const float* P;
  int64_t g_in, b_in, w0;
  int B, RT, KS;
  const float* pool32;
  const _Float16* pool16;
  const uint4* rinfo;     // this step's rows (k1s)
  const uint32_t* mask;   // [Bp][48]
  float keep;             // 1 / (1 - p), or 1
  float* hg_part;         // [KS][B][128]
  float* stats;           // bucket tail, zeroed here (k2 accumulates into it); may be NULL
};
template <int KC>
constexpr int k1c_rt_max() {
  return 16 * (KC + 16) * 4 * 9 <= 150 * 1024 ? 9 : (150 * 1024) / (16 * (KC + 16) * 4);
}
// A load through a pointer the compiler cannot trace to a kernel argument (a row address
// read from memory) is emitted as a FLAT load, which counts in both vmcnt and lgkmcnt and
// is waited for with vmcnt(0) lgkmcnt(0) -- it serialised k3s's gathers. ldg: the same
// load in the global address space.
typedef uint32_t u4v_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 ldg(const uint4* p) {
  typedef const __attribute__((address_space(1))) u4v_t* gp_t;
  const u4v_t v = *(gp_t)(uintptr_t)p;
  return uint4{v.x, v.y, v.z, v.w};
}
__device__ __forceinline__ uint32_t ldg(const uint32_t* p) {
  typedef const __attribute__((address_space(1))) uint32_t* gp_t;
  return *(gp_t)(uintptr_t)p;
}
// a row's first byte and dtype from k1s's row information (bit 0 of the address: f16)
__device__ __forceinline__ const char* row_addr(const uint4& inf, bool& is16) {
  const uint64_t ad = static_cast<uint64_t>(inf.z) | (static_cast<uint64_t>(inf.w) << 32);
  is16 = (ad & 1u) != 0;
  return reinterpret_cast<const char*>(ad & ~uint64_t(15));
}
template <int KC>
__global__ void __launch_bounds__(512) k1c_kernel(K1cArgs a) {
  constexpr int kNI = KC / 32, kLdA = KC + 16, kU8 = KC / 8;  // (KC + 16 halves: conflict-free b128 reads)
  constexpr int kRTM = k1c_rt_max<KC>();
  constexpr int kUPT = (kRTM * 16 * kU8 + 511) / 512;  // staging units per thread
  static_assert(KC % 32 == 0 && kD % KC == 0 && KC <= 512, "K chunk");
  __shared__ __attribute__((aligned(16))) _Float16 ahS[kRTM * 16 * kLdA];
  __shared__ __attribute__((aligned(16))) _Float16 alS[kRTM * 16 * kLdA];
  __shared__ __attribute__((aligned(16))) float gb[2][KC];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, m = lane & 15, kq = lane >> 4;
  const int ks = blockIdx.x % a.KS, rb = blockIdx.x / a.KS;
  const int RT = a.RT, rows = 16 * RT, r0 = rb * rows;
  if (r0 >= a.B) return;
  HBK_MT(3, 1);
  const int k0 = ks * KC;
  if (a.stats && rb == 0 && ks == 0 && tid < kStats) *BCK(&a.stats[tid], 4) = 0.f;
  // every load issued up front: W's column tile, gamma / beta, the rows' statistics and mask words
  f4 wr[kNI][2];
  {
    const float* wp = a.P + a.w0 + static_cast<int64_t>(16 * wave + m) * kD + k0 + 8 * kq;
#pragma unroll
    for (int i = 0; i < kNI; ++i) {
      wr[i][0] = *BCK(reinterpret_cast<const f4*>(wp + 32 * i), 16);
      wr[i][1] = *BCK(reinterpret_cast<const f4*>(wp + 32 * i + 4), 16);
    }
  }
  const int cg = min(tid, KC - 1);
  const float gv = *BCK(&a.P[a.g_in + k0 + cg], 4), bv = *BCK(&a.P[a.b_in + k0 + cg], 4);
  // (the rows' information as uint4: clang miscompiles a bit_cast of an ext_vector element,
  // __builtin_bit_cast(int, v[2]) / (int, v.z) read element 0 -- ROCm 7.2, gfx950)
  uint4 info[kUPT];
  uint32_t mw[kUPT];
#pragma unroll
  for (int j = 0; j < kUPT; ++j) {
    const int q = tid + 512 * j, rr = min(q / kU8, rows - 1), c8 = q % kU8;
    const int64_t r = min(r0 + rr, a.B - 1);
    info[j] = *BCK(&a.rinfo[r], 16);
    mw[j] = *BCK(&a.mask[r * kMaskW + (k0 + 8 * c8) / 32], 4);
  }
  uint4 lo[kUPT], hi[kUPT];
#pragma unroll
  for (int j = 0; j < kUPT; ++j) {
    const int q = tid + 512 * j, c8 = q % kU8;
    bool is16;
    const char* base = row_addr(info[j], is16);
    const char* p = base + (static_cast<int64_t>(k0 + 8 * c8) << (is16 ? 1 : 2));
    lo[j] = ldg(BCK(reinterpret_cast<const uint4*>(p), 16));
    hi[j] = ldg(BCK(reinterpret_cast<const uint4*>(p + (is16 ? 0 : 16)), 16));
  }
  if (tid < KC) {
    gb[0][tid] = gv;
    gb[1][tid] = bv;
  }
  __syncthreads();
  // stage: a = ((v - mu) rs) g + b, split once into the hi / lo planes
#pragma unroll
  for (int j = 0; j < kUPT; ++j) {
    const int q = tid + 512 * j;
    if (q >= rows * kU8) break;
    const int rr = q / kU8, c8 = q % kU8;
    const bool is16 = (info[j].z & 1u) != 0;
    const uint32_t bits = mw[j] >> (8 * (((k0 >> 3) + c8) & 3));
    const float mu = __uint_as_float(info[j].x), rs = __uint_as_float(info[j].y);
    const uint32_t hw[4] = {lo[j].x, lo[j].y, lo[j].z, lo[j].w};
    const uint32_t fw[8] = {lo[j].x, lo[j].y, lo[j].z, lo[j].w, hi[j].x, hi[j].y, hi[j].z, hi[j].w};
    float av[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float x = is16 ? static_cast<float>(__builtin_bit_cast(
                                 _Float16, static_cast<uint16_t>((e & 1) ? hw[e >> 1] >> 16 : hw[e >> 1])))
                           : __builtin_bit_cast(float, fw[e]);
      const float v = (bits >> e) & 1u ? 0.f : x * a.keep;
      const float xh = (v - mu) * rs;
      av[e] = xh * gb[0][8 * c8 + e] + gb[1][8 * c8 + e];
    }
    h8 ahv, alv;
    split8(f4{av[0], av[1], av[2], av[3]}, f4{av[4], av[5], av[6], av[7]}, ahv, alv);
    *reinterpret_cast<h8*>(&ahS[rr * kLdA + 8 * c8]) = ahv;
    *reinterpret_cast<h8*>(&alS[rr * kLdA + 8 * c8]) = alv;
  }
  h8 whi[kNI], wlo[kNI];
#pragma unroll
  for (int i = 0; i < kNI; ++i) split8(wr[i][0] * 16.f, wr[i][1] * 16.f, whi[i], wlo[i]);
  __syncthreads();
  HBK_MT(3, 2);
  f4 acc[kRTM];
#pragma unroll
  for (int t = 0; t < kRTM; ++t) {
    acc[t] = f4{0.f, 0.f, 0.f, 0.f};
    if (t < RT) {
#pragma unroll
      for (int i = 0; i < kNI; ++i) {
        const h8 ah = *reinterpret_cast<const h8*>(&ahS[(16 * t + m) * kLdA + 32 * i + 8 * kq]);
        const h8 al = *reinterpret_cast<const h8*>(&alS[(16 * t + m) * kLdA + 32 * i + 8 * kq]);
        acc[t] = mma3(ah, al, whi[i], wlo[i], acc[t]);
      }
    }
  }
  float* out = a.hg_part + static_cast<int64_t>(ks) * a.B * kH2 + 16 * wave + m;
#pragma unroll
  for (int t = 0; t < kRTM; ++t)
    if (t < RT) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = r0 + 16 * t + 4 * kq + e;
        if (r < a.B) *BCK(&out[static_cast<int64_t>(r) * kH2], 4) = acc[t][e] * (1.f / 16.f);
      }
    }
  HBK_MT(3, 3);
}

// ------------------------------------------------------------------ k2 ----
// One 16-row tile per workgroup, 4 waves. Every matrix stage is
// C[16][N] = A[16][K] . op(W) with A in LDS, as split-f16 products on
// v_mfma_f32_16x16x32_f16 (hi*hi + hi*lo + lo*hi, f32 accumulation, as in k1b
// and k3: a fifth of the MFMA cycles of the f32 16x16x4 chain). Wave w owns
// the 16-column tiles w and w + 4, so a gated MLP's hidden column j and gate
// column 64 + j land in the same wave and the SiLU gate (forward) and its
// derivative (backward) run in the GEMM epilogue. The B operands (weights) of
// the NEXT matrix stage are loaded into registers while the current one runs
// (one workgroup per CU: the whole 512-VGPR file is available) and split just
// before use. NT: W [N][K] row-major (forward, y = x W^T); NN: W [K][N] in LDS
// (backward, dx = dy W). MFMA block i covers k = 32 i + 8 kq .. + 7 for lane
// group kq.
// Range: every wave reads the whole A tile (16 rows x K) for its fragments, so
// it takes the tile's max |A| itself (DPP + readlane, no LDS round trip) and
// scales A by a power of two into [2^14, 2^15) before the split; W is scaled by
// 16 (as in k1b). The sums are scaled back exactly. Gradients (multiples of dz)
// can be arbitrarily small and activations large: neither leaves f16's range.
// Weight fragments come pre-split from the step's weight cache (WSplit below:
// f16 hi / lo planes of 16 W, written by k4 with every update): T tiles of a
// [N][K] matrix (k contiguous), lane (n, kq) of block i holding k = 32 i + 8 kq
// .. + 7 of row n. Loads are unconditional: a tile past N reads a clamped
// (valid) row and its product is discarded by the caller. A load under a lane
// predicate becomes a branch whose join copies the value, i.e. an s_waitcnt
// vmcnt(0) right after the load, which serialises the whole prefetch.
template <int K, int T>
struct WFrag {
  h8 h[T][K / 32], l[T][K / 32];
};
template <int K, int N, int T>
__device__ __forceinline__ void load_wf(WFrag<K, T>& w, const _Float16* __restrict__ hi, int wave, int lane) {
  const int m = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int tt = 0; tt < T; ++tt) {
    const int n = min(16 * (wave + 4 * tt) + m, N - 1);
#pragma unroll
    for (int i = 0; i < K / 32; ++i) {
      w.h[tt][i] = *reinterpret_cast<const h8*>(hi + n * K + 32 * i + 8 * kq);
      w.l[tt][i] = *reinterpret_cast<const h8*>(hi + N * K + n * K + 32 * i + 8 * kq);
    }
  }
}

// 2^p and 2^-p with max |a| 2^p in [2^14, 2^15) (p clamped to +-100: a zero tile
// gets 2^100; inf / NaN propagate through the products)
__device__ __forceinline__ void pow2_scale(float amax, float& s, float& inv) {
  const int e = (__builtin_bit_cast(int, amax) >> 23) & 255;
  const int p = max(-100, min(100, 141 - e));
  s = __builtin_bit_cast(float, (127 + p) << 23);
  inv = __builtin_bit_cast(float, (127 - p) << 23);
}

// split-f16 A fragments of a [16][kLd] f32 LDS tile; inv undoes the A scale and
// the 16 on W
template <int K>
struct AFrag {
  h8 h[K / 32], l[K / 32];
  float inv;
};
template <int K, int LD = kLd>
__device__ __forceinline__ AFrag<K> load_a(const float* A, int lane) {
  const int m = lane & 15, kq = lane >> 4;
  f4 v[K / 32][2];
  float mx = 0.f;
#pragma unroll
  for (int i = 0; i < K / 32; ++i) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      v[i][h] = *reinterpret_cast<const f4*>(A + m * LD + 32 * i + 8 * kq + 4 * h);
#pragma unroll
      for (int s = 0; s < 4; ++s) mx = fmaxf(mx, fabsf(v[i][h][s]));
    }
  }
  float sc, inv;
  pow2_scale(wmax(mx), sc, inv);
  AFrag<K> f;
  f.inv = inv * (1.f / 16.f);
#pragma unroll
  for (int i = 0; i < K / 32; ++i) split8(v[i][0] * sc, v[i][1] * sc, f.h[i], f.l[i]);
  return f;
}

// two tiles (w, w + 4), two interleaved accumulation chains
template <int K>
__device__ __forceinline__ void gemm2(const WFrag<K, 2>& w, const AFrag<K>& a, f4& c0, f4& c1) {
  c0 = f4{0.f, 0.f, 0.f, 0.f};
  c1 = c0;
#pragma unroll
  for (int i = 0; i < K / 32; ++i) {
    c0 = mma3(a.h[i], a.l[i], w.h[0][i], w.l[0][i], c0);
    c1 = mma3(a.h[i], a.l[i], w.h[1][i], w.l[1][i], c1);
  }
  c0 *= a.inv;
  c1 *= a.inv;
}
// one tile (w), two chains over the even / odd k blocks
template <int K>
__device__ __forceinline__ f4 gemm1(const WFrag<K, 1>& w, const AFrag<K>& a) {
  f4 c[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int i = 0; i < K / 32; ++i) c[i & 1] = mma3(a.h[i], a.l[i], w.h[0][i], w.l[0][i], c[i & 1]);
  return (c[0] + c[1]) * a.inv;
}

// The step's weight cache: the matrices k2 multiplies by (W_o_k, k < NG - 1:
// [96][64]; W_hg_k, k >= 1: [128][96]) as f16 hi / lo planes of 16 W, each
// twice: as stored ([N][K], the forward's NT operand) and transposed (the
// backward's NN operand dx = dy W, again with k contiguous). Segment s at
// halves dst: hi [R][C], lo [R][C], hi^T [C][R], lo^T [C][R]. Written from the
// parameters by k0_wsplit (a step whose predecessor did not run k4 on this
// workspace) and by k4 with every update, so k2 reads its fragments with no
// conversion (the split of the f32 weights used to cost each of the ~70
// workgroups ~700 VALU cycles per matrix stage).
constexpr int kMaxSeg = 2 * kMaxG;
struct WSeg {
  int64_t src;  // float offset of the matrix in the parameters
  int rows, cols;
  int64_t dst;  // halves from the cache base
  int64_t q0;   // first float4 of the segment in the k0 grid
};
struct WSplit {
  int n;
  WSeg s[kMaxSeg];
};
__device__ __forceinline__ void wsplit_store4(const WSplit& w, _Float16* __restrict__ base, int64_t i4, f4 p) {
#pragma unroll
  for (int sg = 0; sg < kMaxSeg; ++sg) {
    if (sg >= w.n) break;
    const WSeg g = w.s[sg];
    const int64_t rc = int64_t(g.rows) * g.cols, off = i4 - g.src;
    if (off < 0 || off >= rc) continue;
    uint32_t h[2], l[2];
    split_pair(16.f * p[0], 16.f * p[1], h[0], l[0]);
    split_pair(16.f * p[2], 16.f * p[3], h[1], l[1]);
    _Float16* d = base + g.dst;
    *reinterpret_cast<uint2*>(d + off) = uint2{h[0], h[1]};
    *reinterpret_cast<uint2*>(d + rc + off) = uint2{l[0], l[1]};
    const int r = static_cast<int>(off / g.cols), c = static_cast<int>(off - int64_t(r) * g.cols);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t he = (e & 1) ? h[e >> 1] >> 16 : h[e >> 1] & 0xFFFFu;
      const uint32_t le = (e & 1) ? l[e >> 1] >> 16 : l[e >> 1] & 0xFFFFu;
      d[2 * rc + int64_t(c + e) * g.rows + r] = __builtin_bit_cast(_Float16, static_cast<uint16_t>(he));
      d[3 * rc + int64_t(c + e) * g.rows + r] = __builtin_bit_cast(_Float16, static_cast<uint16_t>(le));
    }
  }
}
// k0: the cache from the parameters (grid-stride over the segments' float4s)
__global__ void __launch_bounds__(256) k0_wsplit_kernel(WSplit w, const float* __restrict__ P,
                                                         _Float16* __restrict__ base, int64_t n4) {
  for (int64_t q = blockIdx.x * int64_t(256) + threadIdx.x; q < n4; q += int64_t(gridDim.x) * 256) {
    int sg = 0;
#pragma unroll
    for (int t = 1; t < kMaxSeg; ++t)
      if (t < w.n && q >= w.s[t].q0) sg = t;
    const int64_t i4 = w.s[sg].src + 4 * (q - w.s[sg].q0);
    wsplit_store4(w, base, i4, *reinterpret_cast<const f4*>(P + i4));
  }
}

struct K2Args {
  const float* P;
  int B, NG, KS;
  int64_t w_hg[kMaxG], b_hg[kMaxG], w_o[kMaxG], b_o[kMaxG];
  int64_t ln_g[kMaxG], ln_b[kMaxG];  // LN k sits between GMLP k and k + 1
  const float* hg_part;
  const float* y;  // labels (0/1 f32) of row r: y[step * y_stride + r]; NULL in inference
  int64_t y_stride;
  const float* state;
  int parity;
  const float* sched;  // [sched_len][2] (lr, neg_weight) or NULL
  int sched_len;
  float neg_weight, thr, act_thr;
  float* prob;   // [B] or NULL
  float* logit;  // [B] or NULL
  float* G;      // gradient bucket (params layout)
  float* stats;  // its statistics tail (8 floats)
  // activations for k3, TRANSPOSED [NG][width][Bp] (Bp = B rounded up to 16, pad rows zero):
  // U 64, Xn 96 (k >= 1), dS 96 (k = NG-1: row 0 = dz), dHG 128
  int64_t Bp;
  float* U;
  float* Xn;
  float* dS;
  float* dHG;
  // workgroups n_rt .. 2 n_rt - 1 (when prefetch): k1a of the NEXT step
  int n_rt, prefetch;
  K1aArgs pre;
  // weight cache (WSplit): hi planes of W_o_k / W_hg_k as stored and transposed
  const _Float16* wc;
  int64_t c_o[kMaxG], c_hg[kMaxG], c_oT[kMaxG], c_hgT[kMaxG];
  // inference only (evaluation passes): counts[2 label] += #(p >= act_thr),
  // counts[2 label + 1] += #(p > act_thr) over the live rows (float counters)
  float* counts;
  int count_label;
  // v2: the prefetch workgroups run k1s (statistics + mask, kPreTiles2 tiles each),
  // and every wave publishes the max |value| of the gradient tiles it stores
  // (maxS[mat][row tile][wave], mat k = dHG_k, NG + k = dS_k: k3s's scales)
  int v2;
  float* maxS;
  int pre_tiles;  // v2: k1s row tiles per prefetch workgroup (kPreTiles2; HBK_PRE_TILES)
};

#ifdef HBK_TRACE
#define K2_MARK(id)                                                                \
  do {                                                                             \
    if (blockIdx.x == 0 && lane == 0 && wave < kTraceWaves && trn < 48)            \
      trS[wave][trn++] = (static_cast<unsigned long long>(id) << 56) |             \
                         (__builtin_amdgcn_s_memtime() & 0xFFFFFFFFFFFFFFull);     \
  } while (0)
#else
#define K2_MARK(id) \
  do {              \
  } while (0)
#endif

#ifndef HBK_K2_ABLATE
#define HBK_K2_ABLATE 0  // profiling builds (wrong results): 1 loads each matrix's fragments once, 2 sums one slab group
#endif
// NG (= n_layers + 2 gated MLPs) is a template argument: every stage below is
// straight-line code, so the register prefetches and their waits are exact.
template <bool kTrain, int NG>
__global__ void __launch_bounds__(256) k2_rows_kernel(K2Args a) {
  // hgS, or the k1a slab of a prefetch workgroup (<= 80 KB in all: two
  // workgroups per CU, so the 2 n_rt-workgroup launch fits n_rt CUs)
  constexpr int kHgF = NG * kR * kLd > kR * kSlabLd ? NG * kR * kLd : kR * kSlabLd;
  __shared__ __attribute__((aligned(16))) float hgRaw[kHgF];
  float (*hgS)[kR][kLd] = reinterpret_cast<float (*)[kR][kLd]>(hgRaw);
  __shared__ __attribute__((aligned(16))) float xhS[NG - 1][kR][kL + 4];
  __shared__ __attribute__((aligned(16))) float bX[kR][kLd];   // LN output (forward) / dHG (backward)
  __shared__ __attribute__((aligned(16))) float bU[kR][kLd];   // gate output (forward) / dXn (backward)
  __shared__ __attribute__((aligned(16))) float bS[kR][kLd];   // GMLP output (forward) / dS (backward)
  __shared__ float rsS[NG][kR];
  __shared__ float zS[kR], dzS[kR];
  __shared__ float red[kStats];
  __shared__ float sBhg[NG][kH2], sWo[kH];
#ifdef HBK_TRACE
  __shared__ unsigned long long trS[4][48];
  int trn = 0;
#endif
  if (kTrain && static_cast<int>(blockIdx.x) >= a.n_rt) {  // next step's k1a (weights not needed)
    // kPreTiles row tiles per workgroup: about as long as a chain workgroup, and
    // the launch needs n_rt + n_rt / kPreTiles slots (two per CU)
    const int step = step_of(a.pre.state, a.pre.parity) + 1;
    if (step < a.pre.idx_steps) {
      if (a.v2) {
        for (int t = 0; t < a.pre_tiles; ++t) {
          const int rt = (blockIdx.x - a.n_rt) * a.pre_tiles + t;
          if (rt >= a.n_rt) break;
          if (t) __syncthreads();  // the mask image's previous readers are done
          k1a_tile<true, true>(a.pre, rt, step, nullptr, hgRaw, a.pre.parity ^ 1);
        }
      } else {
        for (int t = 0; t < kPreTiles; ++t) {
          const int rt = (blockIdx.x - a.n_rt) * kPreTiles + t;
          if (rt >= a.n_rt) break;
          if (t) __syncthreads();  // the slab's previous readers are done
          k1a_tile<true>(a.pre, rt, step, a.pre.xhat[a.pre.parity ^ 1], hgRaw);
        }
      }
    }
    return;
  }
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m = lane & 15, kq = lane >> 4;
  const int r0 = blockIdx.x * kR;
  const int nrow = min(kR, a.B - r0);
  const float* P = a.P;
  const int64_t B = a.B;
  const int64_t Bp = a.Bp;
  K2_MARK(1);
  // step, label and negative weight of this workgroup's rows (used by the loss,
  // loaded now so their two dependent latencies hide under the forward pass)
  const int step = step_of(a.state, a.parity);
  float y_pre = 0.f, nw_pre = a.neg_weight;
  if (kTrain) {
    y_pre = *BCK(&a.y[static_cast<int64_t>(step) * a.y_stride + min(r0 + (tid & 15), a.B - 1)], 4);
    if (a.sched) nw_pre = *BCK(&a.sched[2 * min(step, a.sched_len - 1) + 1], 4);
  }
  WFrag<kH, 2> wa;
  WFrag<kL, 2> wb;
  load_wf<kH, kL, 2>(wa, a.wc + a.c_o[0], wave, lane);
  // small parameters, all loads issued unconditionally: the HG biases and the
  // output weights to LDS; this lane's output biases (columns n0, n1 of the
  // S GEMMs) and LayerNorm gamma / beta (columns c0 .. c0 + 5) to registers
  const int lc0 = 6 * (lane & 15);
  float bo0[NG], bo1[NG], lg[NG][6], lb[NG][6];
  {
    const int c2 = tid & (kH2 - 1);
    float vbhg[NG];
#pragma unroll
    for (int k = 0; k < NG; ++k) {
      vbhg[k] = P[a.b_hg[k] + c2];
      bo0[k] = P[a.b_o[k] + (k + 1 < NG ? 16 * wave + m : 0)];
      bo1[k] = P[a.b_o[k] + (k + 1 < NG ? min(16 * (wave + 4) + m, kL - 1) : 0)];
#pragma unroll
      for (int e = 0; e < 6; ++e) {
        lg[k][e] = k + 1 < NG ? P[a.ln_g[k] + lc0 + e] : 0.f;
        lb[k][e] = k + 1 < NG ? P[a.ln_b[k] + lc0 + e] : 0.f;
      }
    }
    const float vwo = P[a.w_o[NG - 1] + (tid & (kH - 1))];
#pragma unroll
    for (int k = 0; k < NG; ++k)
      if (tid < kH2) sBhg[k][tid] = vbhg[k];
    if (tid < kH) sWo[tid] = vwo;
  }
  // HG0 = sum of k1b's KS partial slabs + bias; U0 = silu(H) G. Thread ->
  // 4 (row, j) pairs; up to 12 slabs' loads are issued together (unrolled,
  // clamped: slabs past KS are re-reads weighted 0; rows past B read row B - 1,
  // whose values are finite and whose every gradient is multiplied by dz = 0).
  {
    float h[4] = {0.f, 0.f, 0.f, 0.f}, g[4] = {0.f, 0.f, 0.f, 0.f};
    // rounds of U slabs (U = 12 for KS = 12 / 24, else 8: k1c's KS = 8 read 12 clamped slabs per round)
    auto sum_slabs = [&](auto U_) {
      constexpr int U = decltype(U_)::value;
      for (int s0 = 0; s0 < a.KS; s0 += U) {
        float lh[U][4], lg[U][4];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int sl = (HBK_K2_ABLATE & 2) ? 0 : min(s0 + u, a.KS - 1);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int e = tid + 256 * q, r = min(e >> 6, nrow - 1), j = e & 63;
            const float* src = a.hg_part + (sl * B + r0 + r) * kH2;
            lh[u][q] = *BCK(&src[j], 4);
            lg[u][q] = *BCK(&src[kH + j], 4);
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const float on = s0 + u < a.KS ? 1.f : 0.f;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            h[q] += on * lh[u][q];
            g[q] += on * lg[u][q];
          }
        }
      }
    };
    if (a.KS % 12 == 0)
      sum_slabs(std::integral_constant<int, 12>{});
    else
      sum_slabs(std::integral_constant<int, 8>{});
    const float bh = P[a.b_hg[0] + (tid & 63)], bg = P[a.b_hg[0] + kH + (tid & 63)];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int e = tid + 256 * q, r = e >> 6, j = e & 63;
      const float hh = h[q] + bh, gg = g[q] + bg;
      hgS[0][r][j] = hh;
      hgS[0][r][kH + j] = gg;
      bU[r][j] = hh * sigm_fast(hh) * gg;
    }
  }
  __syncthreads();
  K2_MARK(2);
  // transposed activation stores: 4 consecutive rows of one column per float4
  auto st4 = [&](float* base, int col, int row4, f4 v) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (r0 + row4 + e >= a.B) v[e] = 0.f;
    *BCK(reinterpret_cast<f4*>(base + col * Bp + r0 + row4), 16) = v;
  };
  // a [16][kLd] LDS tile's first ncols columns -> base^T (4 rows per float4);
  // returns the max |value| stored (dead rows are stored as zeros)
  auto amax4 = [&](f4 v, int row4) {
    float x = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e) x = fmaxf(x, r0 + row4 + e < a.B ? fabsf(v[e]) : 0.f);
    return x;
  };
  auto store_t = [&](float* base, const float* src, int ncols) {
    float mx = 0.f;
    for (int e = tid; e < 4 * ncols; e += 256) {
      const int col = e >> 2, r4 = 4 * (e & 3);
      const f4 v = f4{src[r4 * kLd + col], src[(r4 + 1) * kLd + col], src[(r4 + 2) * kLd + col],
                      src[(r4 + 3) * kLd + col]};
      mx = fmaxf(mx, amax4(v, r4));
      st4(base, col, r4, v);
    }
    return mx;
  };
  // v2: this wave's max |gradient| of matrix mat over this row tile
  auto pub_max = [&](int mat, float mx) {
    if (a.maxS) {
      mx = wmax(mx);
      if (lane == 0) *BCK(&a.maxS[(static_cast<int64_t>(mat) * a.n_rt + blockIdx.x) * 4 + wave], 4) = mx;
    }
  };
  if (kTrain) {  // U_0 from bU: thread -> column tid & 63, rows 4 (tid >> 6) ..
    const int j = tid & 63, rg = 4 * (tid >> 6);
    st4(a.U, j, rg, f4{bU[rg][j], bU[rg + 1][j], bU[rg + 2][j], bU[rg + 3][j]});
  }
  // ---------------------------------------------------------- forward ----
#pragma unroll
  for (int k = 0; k + 1 < NG; ++k) {
    // S_k = U_k W_o_k^T + b_o_k  -> bS   (weights in wa; prefetch HG_{k+1}'s into wb)
    if (!(HBK_K2_ABLATE & 1) || k == 0) load_wf<kL, kH2, 2>(wb, a.wc + a.c_hg[k + 1], wave, lane);
    {
      f4 c0, c1;
      gemm2<kH>(wa, load_a<kH>(&bU[0][0], lane), c0, c1);
      const int n0 = 16 * wave + m, n1 = 16 * (wave + 4) + m;
      const float bo0_ = bo0[k], bo1_ = bo1[k];
#pragma unroll
      for (int e = 0; e < 4; ++e) bS[4 * kq + e][n0] = c0[e] + bo0_;
      if (n1 < kL) {
#pragma unroll
        for (int e = 0; e < 4; ++e) bS[4 * kq + e][n1] = c1[e] + bo1_;
      }
    }
    __syncthreads();
    K2_MARK(10 + k);
    // LayerNorm k over 96 columns: 16 lanes per row (wave w -> rows 4w..4w+3,
    // lane -> row 4w + lane / 16, columns 6 (lane % 16) ..), both reductions of
    // the four rows in parallel within 16-lane DPP rows (rsum16: no cross-row
    // steps); Xn^T goes to HBM from LDS in the next stage
    if (!(HBK_K2_ABLATE & 1) && k + 2 < NG) load_wf<kH, kL, 2>(wa, a.wc + a.c_o[k + 1], wave, lane);
    {
      const int r = wave * 4 + (lane >> 4), c0 = 6 * (lane & 15);
      float v[6];
#pragma unroll
      for (int e = 0; e < 6; ++e) v[e] = bS[r][c0 + e];
      const float mu = rsum16(((v[0] + v[1]) + (v[2] + v[3])) + (v[4] + v[5])) * (1.f / kL);
      float sq = 0.f;
#pragma unroll
      for (int e = 0; e < 6; ++e) sq += (v[e] - mu) * (v[e] - mu);
      const float rs = __builtin_amdgcn_rsqf(rsum16(sq) * (1.f / kL) + kLnEps);
#pragma unroll
      for (int e = 0; e < 6; ++e) {
        const float x = (v[e] - mu) * rs;
        xhS[k][r][c0 + e] = x;
        bX[r][c0 + e] = x * lg[k][e] + lb[k][e];
      }
      if ((lane & 15) == 0) rsS[k][r] = rs;
    }
    __syncthreads();
    K2_MARK(20 + k);
    // HG_{k+1} = Xn W_hg^T + b, gate in the epilogue -> hgS[k+1], U_{k+1} -> bU
    if (kTrain) store_t(a.Xn + (k + 1) * kL * Bp, &bX[0][0], kL);
    {
      f4 ch, cg;
      gemm2<kL>(wb, load_a<kL>(&bX[0][0], lane), ch, cg);
      const int j = 16 * wave + m;
      const float bh = sBhg[k + 1][j], bg = sBhg[k + 1][kH + j];
      f4 uo;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = 4 * kq + e;
        const float h = ch[e] + bh, g = cg[e] + bg;
        hgS[k + 1][r][j] = h;
        hgS[k + 1][r][kH + j] = g;
        const float u = h * sigm_fast(h) * g;
        bU[r][j] = u;
        uo[e] = u;
      }
      if (kTrain) st4(a.U + (k + 1) * kH * Bp, j, 4 * kq, uo);
    }
    __syncthreads();
    K2_MARK(30 + k);
  }
  // backward weight fragments of the first two backward matrix stages (from
  // the transposed cache): W_hg_{NG-1}, W_o_{NG-2}
  WFrag<kH2, 2> fx;
  WFrag<kL, 1> fy;
  if (kTrain) {
    load_wf<kH2, kL, 2>(fx, a.wc + a.c_hgT[NG - 1], wave, lane);
    load_wf<kL, kH, 1>(fy, a.wc + a.c_oT[NG - 2], wave, lane);
  }
  // output unit: z = U . w_o + b_o (wave w -> rows 4w..4w+3)
  {
    const float bo = bo0[NG - 1];
    const float wl = sWo[lane];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = wave * 4 + i;
      const float z = wsum(bU[r][lane] * wl) + bo;
      if (lane == 0) zS[r] = z;
    }
  }
  __syncthreads();
  K2_MARK(40);
  // sigmoid, high-loss filter (trainer.py:407-424), weighted BCE (:301-312, torch
  // formulas incl. the log clamp at -100 and the 1e-12 in BCE's backward)
  if (tid < kR) {
    const int r = tid;
    float loc[kStats] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float dz = 0.f;
    if (r < nrow) {
      const float z = zS[r], p = sigm(z);
      if (a.prob) *BCK(&a.prob[r0 + r], 4) = p;
      if (a.logit) *BCK(&a.logit[r0 + r], 4) = z;
      if (kTrain) {
        const float nw = nw_pre;
        const float yy = y_pre;
        const bool pos = yy == 1.f;
        const bool sel = pos ? (p < 1.f - a.thr) : (p >= a.thr);
        if (sel) {
          const float w = pos ? 1.f : nw;
          const float lp = fmaxf(logf(p), -100.f), l1p = fmaxf(logf(1.f - p), -100.f);
          loc[0] = 1.f;
          loc[1] = -w * (yy * lp + (1.f - yy) * l1p);
          dz = w * (p - yy) / fmaxf((1.f - p) * p, 1e-12f) * ((1.f - p) * p);
          if (pos) {
            loc[4] = 1.f;
            loc[5] = p > a.act_thr ? 1.f : 0.f;  // recall numerator (preds > threshold)
          } else {
            loc[2] = 1.f;
            loc[3] = (yy - p <= -a.act_thr) ? 1.f : 0.f;  // num_false_positives (trainer.py:287-296)
          }
        }
        loc[6] = 1.f;
      }
    }
    dzS[r] = dz;
    if (!kTrain && a.counts) {  // evaluation pass: predictions at the activation threshold
      float pge = 0.f, pgt = 0.f;
      if (r < nrow) {
        const float p = sigm(zS[r]);
        pge = p >= a.act_thr ? 1.f : 0.f;
        pgt = p > a.act_thr ? 1.f : 0.f;
      }
      pge = rsum16(pge);
      pgt = rsum16(pgt);
      if (tid == 0) {
        if (pge != 0.f) atomicAdd(BCK(a.counts + 2 * a.count_label, 4), pge);
        if (pgt != 0.f) atomicAdd(BCK(a.counts + 2 * a.count_label + 1, 4), pgt);
      }
    }
    if (kTrain) {
#pragma unroll
      for (int s = 0; s < kStats; ++s) {
        const float v = rsum16(loc[s]);  // lanes 0..15 of wave 0
        if (tid == 0) red[s] = v;
      }
    }
  }
  if constexpr (!kTrain) return;
  __syncthreads();
  K2_MARK(41);
  if (tid < kStats && red[tid] != 0.f) atomicAdd(BCK(a.stats + tid, 4), red[tid]);
  // ---------------------------------------------------------- backward ---
  float* G = a.G;
  {
    const f4 dz4 = f4{dzS[4 * (tid & 3)], dzS[4 * (tid & 3) + 1], dzS[4 * (tid & 3) + 2], dzS[4 * (tid & 3) + 3]};
    if (tid < 4) st4(a.dS + (NG - 1) * kL * Bp, 0, 4 * tid, dz4);
    pub_max(2 * NG - 1, tid < 4 ? amax4(dz4, 4 * tid) : 0.f);
  }
  if (tid == 64) {  // output bias gradient = sum dz
    float s = 0.f;
    for (int r = 0; r < kR; ++r) s += dzS[r];
    if (s != 0.f) atomicAdd(BCK(G + a.b_o[NG - 1], 4), s);
  }
  // output unit: dU = dz w_o, gate backward -> dHG (bX)
  {
    const int k = NG - 1;
    const int j = tid & 63, rg = 4 * (tid >> 6);
    const float wj = sWo[j];
    f4 dho, dgo;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int r = rg + e;
      const float h = hgS[k][r][j], gg = hgS[k][r][kH + j], du = dzS[r] * wj;
      const float sg = sigm_fast(h);
      const float dh = du * gg * (sg * (1.f + h * (1.f - sg))), dg = du * h * sg;
      bX[r][j] = dh;
      bX[r][kH + j] = dg;
      dho[e] = dh;
      dgo[e] = dg;
    }
    st4(a.dHG + k * kH2 * Bp, j, rg, dho);
    st4(a.dHG + k * kH2 * Bp, kH + j, rg, dgo);
    pub_max(k, fmaxf(amax4(dho, rg), amax4(dgo, rg)));
  }
  __syncthreads();
  K2_MARK(42);
#pragma unroll
  for (int k = NG - 1; k >= 1; --k) {
    // bias gradient of hidden + gate k: column sums of dHG_k (bX)
    if (tid < kH2) {
      float s = 0.f;
      for (int r = 0; r < kR; ++r) s += bX[r][tid];
      atomicAdd(BCK(G + a.b_hg[k] + tid, 4), s);
    }
    // dXn = dHG_k W_hg_k (NN: K 128 -> N 96, fragments fx) -> bU; then W_hg_{k-1}'s
    {
      f4 c0, c1;
      gemm2<kH2>(fx, load_a<kH2>(&bX[0][0], lane), c0, c1);
      if (!(HBK_K2_ABLATE & 1) && k - 1 >= 1) load_wf<kH2, kL, 2>(fx, a.wc + a.c_hgT[k - 1], wave, lane);
      const int n0 = 16 * wave + m, n1 = 16 * (wave + 4) + m;
#pragma unroll
      for (int e = 0; e < 4; ++e) bU[4 * kq + e][n0] = c0[e];
      if (n1 < kL) {
#pragma unroll
        for (int e = 0; e < 4; ++e) bU[4 * kq + e][n1] = c1[e];
      }
    }
    __syncthreads();
    K2_MARK(50 + k);
    // LayerNorm k-1 backward: gamma / beta column sums, dS_{k-1} per row -> bS
    {
      const int l = k - 1;
      if (tid < kL) {
        float sg = 0.f, sb = 0.f;
        for (int r = 0; r < kR; ++r) {
          sg += bU[r][tid] * xhS[l][r][tid];
          sb += bU[r][tid];
        }
        atomicAdd(BCK(G + a.ln_g[l] + tid, 4), sg);
        atomicAdd(BCK(G + a.ln_b[l] + tid, 4), sb);
      }
      // 16 lanes per row, as in the forward LayerNorm; dS^T goes to HBM from
      // LDS in the next stage
      const int r = wave * 4 + (lane >> 4), c0 = 6 * (lane & 15);
      float t[6], x[6];
      float p1 = 0.f, p2 = 0.f;
#pragma unroll
      for (int e = 0; e < 6; ++e) {
        t[e] = bU[r][c0 + e] * lg[l][e];
        x[e] = xhS[l][r][c0 + e];
        p1 += t[e];
        p2 += t[e] * x[e];
      }
      const float s1 = rsum16(p1) * (1.f / kL), s2 = rsum16(p2) * (1.f / kL);
      const float rs = rsS[l][r];
#pragma unroll
      for (int e = 0; e < 6; ++e) bS[r][c0 + e] = rs * (t[e] - s1 - x[e] * s2);
    }
    __syncthreads();
    K2_MARK(60 + k);
    // GMLP k-1: output bias gradient (column sums of dS), dU = dS W_o (NN: K 96 -> N 64,
    // fragments fy) with the gate backward in the epilogue -> dHG_{k-1} (bX)
    {
      const int kk = k - 1;
      pub_max(NG + kk, store_t(a.dS + kk * kL * Bp, &bS[0][0], kL));
      if (tid < kL) {
        float s = 0.f;
        for (int r = 0; r < kR; ++r) s += bS[r][tid];
        atomicAdd(BCK(G + a.b_o[kk] + tid, 4), s);
      }
      const f4 du = gemm1<kL>(fy, load_a<kL>(&bS[0][0], lane));
      if (!(HBK_K2_ABLATE & 1) && k - 2 >= 0) load_wf<kL, kH, 1>(fy, a.wc + a.c_oT[k - 2], wave, lane);
      const int j = 16 * wave + m;
      f4 dho, dgo;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = 4 * kq + e;
        const float h = hgS[kk][r][j], gg = hgS[kk][r][kH + j];
        const float sg = sigm_fast(h);
        const float dh = du[e] * gg * (sg * (1.f + h * (1.f - sg))), dg = du[e] * h * sg;
        bX[r][j] = dh;
        bX[r][kH + j] = dg;
        dho[e] = dh;
        dgo[e] = dg;
      }
      st4(a.dHG + kk * kH2 * Bp, j, 4 * kq, dho);
      st4(a.dHG + kk * kH2 * Bp, kH + j, 4 * kq, dgo);
      pub_max(kk, fmaxf(amax4(dho, 4 * kq), amax4(dgo, 4 * kq)));
    }
    __syncthreads();
    K2_MARK(70 + k);
  }
  // bias gradient of mlp_in's hidden + gate
  if (tid < kH2) {
    float s = 0.f;
    for (int r = 0; r < kR; ++r) s += bX[r][tid];
    atomicAdd(BCK(G + a.b_hg[0] + tid, 4), s);
  }
  K2_MARK(99);
#ifdef HBK_TRACE
  if (blockIdx.x == 0 && lane == 0 && wave < kTraceWaves) {
    for (int i = 0; i < trn; ++i) g_mlp_trace[1][wave][i] = trS[wave][i];
    g_mlp_trace_n[1][wave] = trn;
  }
#endif
}

// ------------------------------------------------------------------ k3 ----
// dW [M][N] += X^T Y over a split of batch rows, from k1a/k2's TRANSPOSED
// activations X^T [M][Bp] (a gradient: dHG or dS), Y^T [N][Bp] (an
// activation: xhat, Xn or U); rows of b contiguous, pad rows zero. Split-f16
// products on v_mfma_f32_16x16x32_f16 (hi*hi + hi*lo + lo*hi, f32
// accumulation): lane (m, kq) of step u holds b = 32 u + 8 kq .. + 7, so A and B
// are two float4 runs along b. Gradients can be arbitrarily small, so X is
// scaled by a power of two per workgroup (its tile's max |X| into [2^14, 2^15):
// no f16 overflow, lo parts in f16's normal range) and the sums are scaled
// back exactly. Tile 128 x 32: wave w owns M rows 32 w .. 32 w + 31 (two MFMA
// row tiles, X in registers, all loads in flight together) and both 16-column
// halves; the split's Y^T tile (32 x 288) is loaded once per workgroup, split
// into f16 hi / lo planes in LDS and shared by the four waves. Split-K partials
// are added with float atomics into the bucket (zeroed by the previous k4).
constexpr int kTM = 128, kTN = 32, kMaxJobs = 2 * kMaxG;
// batch rows per split: measured 4 / 5 / 6 / 9 steps (124 / 152 / 180 / 248 VGPRs) at 60.2 / 60.3 /
// 61.6 / 58.9 us per step on 256 CUs and 88.7 / 88.9 / 94.8 / 92.1 on a 64-CU stream
#ifndef HBK_K3_STEPS
#define HBK_K3_STEPS 9
#endif
constexpr int kK3Steps = HBK_K3_STEPS, kK3Rows = 32 * kK3Steps;  // batch rows per split (B = 1100: 4 splits)
constexpr int kYLdH = kK3Rows + 8;                    // LDS row stride (halves) of the Y planes
constexpr int kK3StepsNarrow = 4, kK3NarrowCUs = 96;
// narrow streams: one workgroup may walk this many consecutive 128-row splits
// (one partial slab per group). Measured at 3 on a 64-CU stream: k3 23.8 ->
// 38.9 us (256 VGPRs, two workgroups per CU, the splits' latencies in series)
// and k4 unchanged at 11.7 us with 3 slabs instead of 9, so it stays 1.
#ifndef HBK_K3_GROUP
#define HBK_K3_GROUP 1
#endif
constexpr int kK3GroupNarrow = HBK_K3_GROUP;
struct WJob {
  const float* X;  // [M][Bp]
  const float* Y;  // [N][Bp]
  int64_t c_off;   // the gradient [M][ldc] at this offset of the parameter layout
  int ldc, M, N, tn;
};
// The covered parameter ranges (k3's weight gradients, norm_in's gamma / beta):
// k3 writes them as one partial slab per batch split, part[split][n_params],
// with plain stores (float atomics run at the memory side, ~1 TB/s chip-wide,
// and were most of k3's time); k4 adds the slabs while it reads the bucket
// (or k3_fold_kernel adds them into the bucket first, for the all-reduce).
constexpr int kMaxRng = 2 + 2 * kMaxG;
struct Ranges {
  int n;
  int64_t lo[kMaxRng], hi[kMaxRng];
};
__device__ __forceinline__ bool in_ranges(const Ranges& r, int64_t i) {
  bool c = false;
#pragma unroll
  for (int k = 0; k < kMaxRng; ++k) c |= k < r.n && i >= r.lo[k] && i < r.hi[k];
  return c;
}
struct K3Args {
  WJob job[kMaxJobs];
  int start[kMaxJobs + 1];
  int n_jobs, KS;
  int64_t Bp;
  // input-layer job (job 0): post-op with norm_in's affine and W_hg0
  const float* g_in;
  const float* b_in;
  const float* W0;
  int64_t g_off, b_off;  // norm_in gamma / beta in the parameter layout
  float* part;           // [KS][pstride] partial slabs
  int64_t pstride;
};

// STEPS: batch rows per split / 32 (the grid's split count follows); the launch
// takes kK3Steps on a wide stream and kK3StepsNarrow on a CU-masked one of at
// most kK3NarrowCUs CUs (fewer, longer workgroups: see kK3Steps' sweep)
template <int STEPS, int G>
__global__ void __launch_bounds__(256) k3_wgrad_kernel(K3Args a) {
  constexpr int kK3Steps = STEPS, kK3Rows = 32 * STEPS, kYLdH = kK3Rows + 8;
  __shared__ __attribute__((aligned(16))) _Float16 yh[kTN * kYLdH];
  __shared__ __attribute__((aligned(16))) _Float16 yl[kTN * kYLdH];
  __shared__ float sS[kTM];
  __shared__ float red[2][4][kTN];
  __shared__ float smax[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int blk = blockIdx.x;
  int j = 0;
  while (j + 1 < a.n_jobs && blk >= a.start[j + 1]) ++j;
  const WJob jb = a.job[j];
  const int local = blk - a.start[j];
  const int split = local % a.KS, tile = local / a.KS;  // split: a group of G consecutive batch splits
  float* const C = a.part + split * a.pstride + jb.c_off;
  const int tm = tile / jb.tn, tn = tile - tm * jb.tn;
  HBK_MT(2, 1);
  const int Bp = static_cast<int>(a.Bp);
  const int m = lane & 15, kq = lane >> 4;
  const int mrow = tm * kTM + 32 * wave;  // first M row of this wave (two 16-row tiles)
  const int n0 = tn * kTN;
  // Y^T tile of a split: 32 columns x kK3Rows rows; rows past Bp are zeroed
  // (their loads read a clamped valid run). Columns past N read a clamped row:
  // their products only reach outputs that are never stored.
  constexpr int kYv = kTN * kK3Rows / 4 / 256;  // float4 per thread
  f4 yv[kYv];
  auto load_y = [&](int rb0) {
#pragma unroll
    for (int h = 0; h < kYv; ++h) {
      const int e = tid + 256 * h, col = e / (kK3Rows / 4), off = 4 * (e % (kK3Rows / 4));
      const int b = min(rb0 + off, Bp - 4);
      yv[h] = *reinterpret_cast<const f4*>(jb.Y + static_cast<int64_t>(min(n0 + col, jb.N - 1)) * Bp + b);
    }
  };
  // X: rows past M read a clamped row (discarded outputs); this lane's 8 batch
  // rows past Bp (8-row granularity: Bp is a multiple of 16) read the last 8
  // rows and are zeroed
  const float* X0 = jb.X + static_cast<int64_t>(min(mrow + m, jb.M - 1)) * Bp;
  const float* X1 = jb.X + static_cast<int64_t>(min(mrow + 16 + m, jb.M - 1)) * Bp;
  f4 rx[2][kK3Steps][2];
  auto load_x = [&](int rb0, int u) {
    const int b = min(rb0 + 32 * u + 8 * kq, Bp - 8);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      rx[0][u][h] = *reinterpret_cast<const f4*>(X0 + b + 4 * h);
      rx[1][u][h] = *reinterpret_cast<const f4*>(X1 + b + 4 * h);
    }
  };
  const int rbase = split * G * kK3Rows;
  load_y(rbase);
#pragma unroll
  for (int u = 0; u < kK3Steps; ++u) load_x(rbase, u);
  const f4 z = {0.f, 0.f, 0.f, 0.f};
  f4 ssum[2] = {z, z};
  f4 acc[2][2] = {{z, z}, {z, z}};
  const _Float16* y0h = &yh[m * kYLdH + 8 * kq];
  const _Float16* y0l = &yl[m * kYLdH + 8 * kq];
  const _Float16* y1h = &yh[(16 + m) * kYLdH + 8 * kq];
  const _Float16* y1l = &yl[(16 + m) * kYLdH + 8 * kq];
  // the group's splits one after the other, each with its own power-of-two
  // scale; the next split's Y loads are issued once this one's tile is in LDS,
  // its X loads step by step as this one's products release the registers
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const int rb0 = rbase + g * kK3Rows;
    if (g) lds_barrier();  // the previous split's readers of yh / yl (and smax) are done
#pragma unroll
    for (int h = 0; h < kYv; ++h) {
      const int e = tid + 256 * h, col = e / (kK3Rows / 4), off = 4 * (e % (kK3Rows / 4));
      const f4 v = rb0 + off < Bp ? yv[h] : z;
      uint32_t h0, l0, h1, l1;
      split_pair(v[0], v[1], h0, l0);
      split_pair(v[2], v[3], h1, l1);
      *reinterpret_cast<uint2*>(&yh[col * kYLdH + off]) = uint2{h0, h1};
      *reinterpret_cast<uint2*>(&yl[col * kYLdH + off]) = uint2{l0, l1};
    }
    // zero the dead batch rows of X, row sums (input job) and the split's max |X|
    float mx = 0.f;
#pragma unroll
    for (int u = 0; u < kK3Steps; ++u) {
      const bool live = rb0 + 32 * u + 8 * kq < Bp;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          rx[t][u][h] = live ? rx[t][u][h] : z;
          ssum[t] += rx[t][u][h];
#pragma unroll
          for (int e = 0; e < 4; ++e) mx = fmaxf(mx, fabsf(rx[t][u][h][e]));
        }
    }
    mx = wmax(mx);
    if (lane == 0) smax[wave] = mx;
    lds_barrier();  // (LDS only: the next split's loads issued below stay in flight)
    if (g + 1 < G) load_y(rb0 + kK3Rows);
    mx = fmaxf(fmaxf(smax[0], smax[1]), fmaxf(smax[2], smax[3]));
    // scale = 2^(14 - floor(log2 max)): max |X| * scale in [2^14, 2^15)
    const int ex = mx > 0.f ? min(14 - ilogbf(mx), 126) : 0;
    const float scale = ldexpf(1.f, ex), unscale = ldexpf(1.f, -ex);
    f4 as[2][2] = {{z, z}, {z, z}};
#pragma unroll
    for (int u = 0; u < kK3Steps; ++u) {
      const h8 bh0 = *reinterpret_cast<const h8*>(y0h + 32 * u), bl0 = *reinterpret_cast<const h8*>(y0l + 32 * u);
      const h8 bh1 = *reinterpret_cast<const h8*>(y1h + 32 * u), bl1 = *reinterpret_cast<const h8*>(y1l + 32 * u);
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        h8 ah, al;
        split8(rx[t][u][0] * scale, rx[t][u][1] * scale, ah, al);
        as[t][0] = mma3(ah, al, bh0, bl0, as[t][0]);
        as[t][1] = mma3(ah, al, bh1, bl1, as[t][1]);
      }
      if (g + 1 < G) load_x(rb0 + kK3Rows, u);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      acc[t][0] += as[t][0] * unscale;
      acc[t][1] += as[t][1] * unscale;
    }
  }
  const bool nok0 = n0 + m < jb.N, nok1 = n0 + 16 + m < jb.N;
  HBK_MT(2, 2);
  if (j != 0) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = mrow + 16 * t + 4 * kq + e;
        if (row < jb.M) {
          if (nok0) C[static_cast<int64_t>(row) * jb.ldc + n0 + m] = acc[t][0][e];
          if (nok1) C[static_cast<int64_t>(row) * jb.ldc + n0 + 16 + m] = acc[t][1][e];
        }
      }
    return;
  }
  // input layer: s_j = sum over the split's rows of dHG0[b][j] (lanes m + 16 q hold parts)
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    float sj_part = (ssum[t][0] + ssum[t][1]) + (ssum[t][2] + ssum[t][3]);
    sj_part += __shfl_xor(sj_part, 16, 64);
    sj_part += __shfl_xor(sj_part, 32, 64);
    if (kq == 0) sS[32 * wave + 16 * t + m] = sj_part;
  }
  __syncthreads();
  float dg0 = 0.f, dg1 = 0.f, dbt0 = 0.f, dbt1 = 0.f;
  const int c0 = n0 + m, c1 = n0 + 16 + m;
  // every epilogue load is issued up front at clamped (valid) addresses, so none
  // sits behind an atomic in a predicated branch
  const int c0c = min(c0, jb.N - 1), c1c = min(c1, jb.N - 1);
  const float g0 = a.g_in[c0c], g1 = a.g_in[c1c];
  const float be0 = a.b_in[c0c], be1 = a.b_in[c1c];
  float w0[2][4], w1[2][4];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float* wr = a.W0 + static_cast<int64_t>(min(mrow + 16 * t + 4 * kq + e, jb.M - 1)) * jb.ldc;
      w0[t][e] = wr[c0c];
      w1[t][e] = wr[c1c];
    }
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = mrow + 16 * t + 4 * kq + e;  // j
      if (row >= jb.M) continue;
      const float sj = sS[32 * wave + 16 * t + 4 * kq + e];
      if (nok0) {
        C[static_cast<int64_t>(row) * jb.ldc + c0] = g0 * acc[t][0][e] + be0 * sj;
        dg0 += w0[t][e] * acc[t][0][e];
        dbt0 += w0[t][e] * sj;
      }
      if (nok1) {
        C[static_cast<int64_t>(row) * jb.ldc + c1] = g1 * acc[t][1][e] + be1 * sj;
        dg1 += w1[t][e] * acc[t][1][e];
        dbt1 += w1[t][e] * sj;
      }
    }
  // reduce over kq (lanes m + 16 q) then over waves
#pragma unroll
  for (int o = 16; o < 64; o <<= 1) {
    dg0 += __shfl_xor(dg0, o, 64);
    dg1 += __shfl_xor(dg1, o, 64);
    dbt0 += __shfl_xor(dbt0, o, 64);
    dbt1 += __shfl_xor(dbt1, o, 64);
  }
  if (kq == 0) {
    red[0][wave][m] = dg0;
    red[0][wave][16 + m] = dg1;
    red[1][wave][m] = dbt0;
    red[1][wave][16 + m] = dbt1;
  }
  __syncthreads();
  if (tid < kTN) {
    const int c = n0 + tid;
    if (c < jb.N) {
      float* P = a.part + split * a.pstride;
      P[a.g_off + c] = red[0][0][tid] + red[0][1][tid] + red[0][2][tid] + red[0][3][tid];
      P[a.b_off + c] = red[1][0][tid] + red[1][1][tid] + red[1][2][tid] + red[1][3][tid];
    }
  }
}

// ------------------------------------------------------------ k3s (v2) ---
// The weight gradients dW [M][N] = dY^T X over S batch splits of R rows, with
// wide N tiles: tile = 128 (M) x 16 NBT (N), kK3sWaves waves of 128 / kK3sWaves M rows, so the
// gradient operand dY^T is read from HBM / L2 once per N tile (the v1 kernel's
// 32-column tiles re-read dHG0 48 times per split: 27 MB of its 47 MB per step at
// B = 1,100). The batch streams through in 32-row steps: the activation chunk X
// (16 NBT columns x 32 rows) is converted to f16 hi / lo planes in a double-
// buffered LDS image (one barrier per step), the gradient chunk is loaded three steps
// ahead into registers. The gradient's power-of-two scale comes from k2's per-tile
// maxima (maxS), so the whole split accumulates in one scale. The input layer's X
// is not stored anywhere: it is recomputed from the pool rows, k1s's statistics and
// dropout mask (xhat = (v - mu) rs, the formula of k1a) as the chunk is staged.
constexpr int kK3sMaxR = 512;  // rows per split
// 8 waves of one 16-row M tile each: two waves per SIMD hide each other's latency (4 waves
// of two M tiles ran one wave per SIMD at 256 VGPRs + AGPRs, 4.2 k cycles per 32-row step
// against 1.9 k of issue). (4 M groups of two tiles x 2 column halves -- each B fragment read
// from LDS feeding two M tiles, the gradient split twice -- measured slower: 24.2 vs 22.1 us)
constexpr int kK3sWaves = 8, kK3sThr = 64 * kK3sWaves, kK3sMT = 1, kK3sMG = 8;
static_assert(kK3sMG * kK3sMT * 16 == 128 && kK3sWaves == kK3sMG, "k3s wave layout");
struct K3sJob {
  const float* X;  // the gradient dY^T [M][Bp]
  const float* Y;  // the activation X^T [N][Bp]; NULL: the input layer's pool rows
  int64_t c_off;
  int ldc, M, N, tn, mat;
  int S, R;  // this job's batch splits, of R = 32 x (its compiled step count) rows
};
struct K3sArgs {
  K3sJob job[kMaxJobs];
  int start[kMaxJobs + 1];
  int n_jobs, S, n_rt, B;  // S: the slabs (the largest job split; a job with fewer zeroes the rest)
  int64_t Bp;
  const float* maxS;  // [2 NG][n_rt][4]
  const float* pool32;
  const _Float16* pool16;
  const uint4* rinfo;
  const uint32_t* mask;
  float keep;
  // input-layer post-op (job 0)
  const float* g_in;
  const float* b_in;
  const float* W0;
  int64_t g_off, b_off;
  float* part;  // [S][pstride]
  int64_t pstride;
};
// XOR swizzle of the 16-B chunks of a 256-B row (the input layer's [32][128] half images):
// conflict-free ds_write_b128 of whole chunks and ds_read_b64_tr_b16 of the B operand
__device__ __forceinline__ int k3s_swz(int row, int ch) { return ch ^ (((row & 3) << 2) | ((row >> 2) & 3)); }
// N tile widths: the input layer's 256 columns (each gradient chunk, loaded and split once,
// feeds 16 column tiles: its 12x re-read of dHG0 per split became 6x, the split's VALU is
// amortised over twice the MFMAs; 22.1 against 24.5 us), the generic jobs' 128. k3s is bound
// per CU (two workgroups on one CU each ran 2.2x slower), not by a chip-wide resource, and
// neither fewer VALU, half the LDS fragment traffic nor contiguous row loads moved it
// (profiles/r06_ab_step.log)
constexpr int kK3sNbtRaw = 16, kK3sNbtGen = 8;
static_assert(kD % (16 * kK3sNbtRaw) == 0, "the input layer's tiles are all live");
struct K3sShared {
  static constexpr int kLdY = 48;  // generic: LDS column of 32 rows + 16 pad halves (conflict-free b128 reads)
  static constexpr int kPlane = 32 * 16 * kK3sNbtRaw > 16 * kK3sNbtGen * kLdY ? 32 * 16 * kK3sNbtRaw
                                                                             : 16 * kK3sNbtGen * kLdY;
  _Float16 ys[2][2][kPlane];  // [buf][hi, lo]: generic [col][row]; input layer two [32][128] halves
  float sS[128];
  float red[2][kK3sWaves][16 * kK3sNbtRaw];
  uint4 rinfoS[kK3sMaxR];                          // input layer: the split's rows' {mu, rs, address}
  uint32_t maskS[kK3sMaxR * kK3sNbtRaw / 2];       // ... and their mask words of this N tile
};
// one workgroup's tile; kRaw: the input layer (X from the pool rows). NST steps of 32 rows,
// fully unrolled, the prefetches unconditional (clamped to the last step: a redundant
// reload at the tail): straight-line code, so the compiler's vmcnt waits are exact (a
// rolled loop made it wait vmcnt(0) at the top of every step, i.e. for the loads issued
// one step earlier: 8 k cycles per step). A split shorter than NST steps (the last)
// computes zero rows in its tail steps.
template <int NBT, bool kRaw, int NST>
__device__ __forceinline__ void k3s_body(const K3sArgs& a, const K3sJob& jb, int split, int tm, int tnn,
                                         K3sShared& sh) {
  constexpr int NT = 16 * NBT, kLdY = K3sShared::kLdY;
  constexpr int kYU = NT * 8 / kK3sThr;  // float4 units per thread and step (transposed X)
  constexpr int MT = kK3sMT, NBW = NBT;  // M tiles and column tiles per wave
  static_assert(!kRaw || NT == 256, "the input layer's image is two [32][128] halves (the swizzle's 256-B rows)");
  static_assert(kRaw || NT * kLdY <= K3sShared::kPlane, "a generic image fits a buffer plane");
  static_assert(NT <= 16 * kK3sNbtRaw && NT / 32 <= kK3sNbtRaw / 2, "red / maskS sizes");
  // input-layer image offset (halves) of row r, 16-B chunk c (0 .. NT / 8)
  auto raw_off = [](int r, int c) { return (c >> 4) * (32 * 128) + r * 128 + 8 * k3s_swz(r, c & 15); };
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, m = lane & 15, kq = lane >> 4;
  const int Bp = static_cast<int>(a.Bp);
  const int rb0 = split * jb.R;
  constexpr int nst = NST;
  const int n0 = tnn * NT;
  const int mg = wave, nt0 = 0;  // this wave's M group, first column tile
  const int mrow = tm * 128 + 16 * MT * mg;
  // gradient chunk of step u: MT 16-row M tiles x 8 batch rows (b = 32 u + 8 kq ..)
  const float* Xt[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) Xt[t] = jb.X + static_cast<int64_t>(min(mrow + 16 * t + m, jb.M - 1)) * Bp;
  // (unclamped: rows past Bp read the next row, or past the last row of the workspace array the
  // arrays after it, <= R floats; they are zeroed at use. One base address per tile and
  // immediate offsets per step: a clamp per step held a 64-bit address per unrolled step)
  auto load_g = [&](int u, f4 (&d)[MT][2]) {
    const int b = rb0 + 32 * u + 8 * kq;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int t = 0; t < MT; ++t) d[t][h] = *BCK(reinterpret_cast<const f4*>(Xt[t] + b + 4 * h), 16);
  };
  // activation chunk of step u into registers ...
  // (input layer: thread -> 16-B chunks q = tid + kK3sThr j of the step's [32 rows][NT] image, row
  // q / (NT / 8), columns 8 (q % (NT / 8)) ..: the pool rows as they lie, 16 / 32 B per chunk)
  constexpr int kCPR = NT / 8, kCPT = 32 * kCPR / kK3sThr;  // chunks per row, per thread
  // two register sets: step v's loads are issued at step v - 3 and converted at step v - 1
  f4 yv[2][kRaw ? 1 : kYU];
  uint4 ylo[2][kRaw ? kCPT : 1], yhi[2][kRaw ? kCPT : 1];
  auto issue_raw = [&](int u, int j, const uint4& inf) {  // chunk j of step u, its row's info inf
    bool is16;
    const char* base = row_addr(inf, is16);
    const char* p = base + (static_cast<int64_t>(n0 + 8 * ((tid + kK3sThr * j) % kCPR)) << (is16 ? 1 : 2));
    ylo[u & 1][j] = ldg(BCK(reinterpret_cast<const uint4*>(p), 16));
    yhi[u & 1][j] = ldg(BCK(reinterpret_cast<const uint4*>(p + (is16 ? 0 : 16)), 16));
  };
  auto load_y = [&](int u) {
    const int ys_ = u & 1;
    if constexpr (kRaw) {
#pragma unroll
      for (int j = 0; j < kCPT; ++j) issue_raw(u, j, sh.rinfoS[32 * u + (tid + kK3sThr * j) / kCPR]);
    } else {
#pragma unroll
      for (int jj = 0; jj < kYU; ++jj) {
        const int q = tid + kK3sThr * jj, col = min(n0 + (q >> 3), jb.N - 1);
        const int b = rb0 + 32 * u + 4 * (q & 7);  // (unclamped, as the gradient's)
        yv[ys_][jj] = *BCK(reinterpret_cast<const f4*>(jb.Y + static_cast<int64_t>(col) * Bp + b), 16);
      }
    }
  };
  // ... converted into LDS buffer buf
  auto write_y = [&](int u, int buf) {
    _Float16* yh = &sh.ys[buf][0][0];
    _Float16* yl = &sh.ys[buf][1][0];
    const int ys_ = u & 1;
    if constexpr (kRaw) {
      // xhat = (v - mu) rs of the chunk's 8 elements, split, into the row-major hi / lo images
      // ([32][NT] halves, 16-B chunks XOR-swizzled: conflict-free b128 writes and tr reads)
#pragma unroll
      for (int j = 0; j < kCPT; ++j) {
        const int q = tid + kK3sThr * j, row = q / kCPR, ch = q % kCPR, rl = 32 * u + row;
        const uint4 inf = sh.rinfoS[rl];
        const bool is16 = (inf.z & 1u) != 0;
        const uint32_t bits = sh.maskS[rl * (NT / 32) + (ch >> 2)] >> (8 * (ch & 3));
        const float mu = __uint_as_float(inf.x), rs = rb0 + rl < a.B ? __uint_as_float(inf.y) : 0.f;
        const uint4 lo = ylo[ys_][j], hi = yhi[ys_][j];
        const uint32_t hw[4] = {lo.x, lo.y, lo.z, lo.w};
        const uint32_t fw[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
        // xhat = (keep x - mu) rs as one fma per element, (keep rs) x + (-mu rs), a dropped element
        // the constant -mu rs (2 VALU fewer per element than the sub / mul form; f32 rounding)
        const float k2 = a.keep * rs, c0 = -mu * rs;
        float xs[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float x = is16 ? static_cast<float>(__builtin_bit_cast(
                                     _Float16, static_cast<uint16_t>((e & 1) ? hw[e >> 1] >> 16 : hw[e >> 1])))
                               : __builtin_bit_cast(float, fw[e]);
          xs[e] = (bits >> e) & 1u ? c0 : fmaf(x, k2, c0);  // (rows past B: rs = 0 and a finite x -> 0)
        }
        h8 hv, lv;
        split8(f4{xs[0], xs[1], xs[2], xs[3]}, f4{xs[4], xs[5], xs[6], xs[7]}, hv, lv);
        const int off = raw_off(row, ch);
        *reinterpret_cast<h8*>(yh + off) = hv;
        *reinterpret_cast<h8*>(yl + off) = lv;
      }
    } else {
#pragma unroll
      for (int jj = 0; jj < kYU; ++jj) {
        const int q = tid + kK3sThr * jj, col = q >> 3, b4 = 4 * (q & 7);
        const f4 v = rb0 + 32 * u + b4 < Bp ? yv[ys_][jj] : f4{0.f, 0.f, 0.f, 0.f};
        uint32_t h0, l0, h1, l1;
        split_pair(v[0], v[1], h0, l0);
        split_pair(v[2], v[3], h1, l1);
        *reinterpret_cast<uint2*>(yh + col * kLdY + b4) = uint2{h0, h1};
        *reinterpret_cast<uint2*>(yl + col * kLdY + b4) = uint2{l0, l1};
      }
    }
  };
  const f4 z = {0.f, 0.f, 0.f, 0.f};
  f4 acc[MT][NBW];
  f4 ssum[MT];
#pragma unroll
  for (int t = 0; t < MT; ++t) {
    ssum[t] = z;
#pragma unroll
    for (int i = 0; i < NBW; ++i) acc[t][i] = z;
  }
  f4 ga[3][MT][2];  // gradient ring: [slot][tile][half], step v in slot v % 3 (loaded 3 steps ahead)
  constexpr int last = NST - 1;
  // prologue, every independent load issued at once (the serial round trips were 4.6 us of a
  // 12-step workgroup's 24): the gradient's per-tile maxima, the gradient of steps 0 .. 2,
  // the input layer's row information and mask words (for LDS), and the activation of steps 0
  // and 1 (the input layer's through row information loaded into registers here as well)
  static_assert(kK3sMaxR / 16 * 4 <= 128, "maxS: two entries per lane");
  float mxv[2];
  {
    const int t0 = rb0 / 16, n4 = 4 * (min(a.n_rt, (rb0 + 32 * nst) / 16) - t0);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = lane + 64 * i;
      const float v = *BCK(&a.maxS[(static_cast<int64_t>(jb.mat) * a.n_rt + t0) * 4 + min(q, n4 - 1)], 4);
      mxv[i] = q < n4 ? v : 0.f;
    }
  }
  load_g(0, ga[0]);
  load_g(min(1, last), ga[1]);
  load_g(min(2, last), ga[2]);
  float sc, inv;
  if constexpr (kRaw) {  // the split's row information and mask words (rows past B: row B - 1's, zeroed below)
    // (unrolled, every load unconditional at a clamped row: all in flight together)
    const int nr = 32 * nst;
    constexpr int kRI = kK3sMaxR / kK3sThr, kMI = kK3sMaxR * (NT / 32) / kK3sThr;
    uint4 ri[kRI], r01[2][kCPT];
    uint32_t mi[kMI];
#pragma unroll
    for (int it = 0; it < kRI; ++it)
      ri[it] = *BCK(&a.rinfo[min(rb0 + min(tid + kK3sThr * it, nr - 1), a.B - 1)], 16);
#pragma unroll
    for (int v = 0; v < 2; ++v)
#pragma unroll
      for (int j = 0; j < kCPT; ++j)
        r01[v][j] = *BCK(&a.rinfo[min(rb0 + 32 * min(v, last) + (tid + kK3sThr * j) / kCPR, a.B - 1)], 16);
#pragma unroll
    for (int it = 0; it < kMI; ++it) {
      const int q = min(tid + kK3sThr * it, nr * (NT / 32) - 1);
      mi[it] = *BCK(&a.mask[static_cast<int64_t>(min(rb0 + q / (NT / 32), a.B - 1)) * kMaskW + n0 / 32 + q % (NT / 32)], 4);
    }
#pragma unroll
    for (int v = 0; v < 2; ++v)
#pragma unroll
      for (int j = 0; j < kCPT; ++j) issue_raw(min(v, last), j, r01[v][j]);
    pow2_scale(wmax(fmaxf(mxv[0], mxv[1])), sc, inv);
#pragma unroll
    for (int it = 0; it < kRI; ++it)
      if (tid + kK3sThr * it < nr) sh.rinfoS[tid + kK3sThr * it] = ri[it];
#pragma unroll
    for (int it = 0; it < kMI; ++it)
      if (tid + kK3sThr * it < nr * (NT / 32)) sh.maskS[tid + kK3sThr * it] = mi[it];
    __syncthreads();
  } else {
    load_y(0);
    load_y(min(1, last));
    pow2_scale(wmax(fmaxf(mxv[0], mxv[1])), sc, inv);
  }
  HBK_MT(2, 3);
  // step 0 staged; steps 1, 2 of X and 0, 1, 2 of the gradient in flight
  write_y(0, 0);
  load_y(min(2, last));
  __syncthreads();
  HBK_MT(2, 4);
  auto step = [&](int u, f4 (&g)[MT][2]) {
    // this step's gradient: dead batch rows zeroed, row sums (input layer), scaled split
    const bool live = rb0 + 32 * u + 8 * kq < Bp;
    h8 ah[MT], al[MT];
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const f4 g0 = live ? g[t][0] : z, g1 = live ? g[t][1] : z;
      ssum[t] += g0 + g1;
      split8(g0 * sc, g1 * sc, ah[t], al[t]);
    }
    const _Float16* yh = &sh.ys[u & 1][0][0];
    const _Float16* yl = &sh.ys[u & 1][1][0];
    // every column tile, live or not (a generic job's dead tiles hold clamped columns: finite,
    // never stored; a uniform branch per tile made each wait for its own LDS reads), in groups
    // of kGrp tiles: group g + 1's B fragments are read while group g's MFMAs run (fenced:
    // unfenced, all 16 tiles' reads were hoisted to the top, 128 VGPRs)
    constexpr int kGrp = 4, nGrp = NBW / kGrp;
    static_assert(NBW % kGrp == 0, "column-tile groups");
    h8 fb[2][kGrp][2];  // [slot][tile][hi, lo]
    auto read_grp = [&](int gi, h8 (&d)[kGrp][2]) {
#pragma unroll
      for (int i = 0; i < kGrp; ++i) {
        const int nt = nt0 + gi * kGrp + i;
        if constexpr (kRaw) {
          // rows 8 kq .. 8 kq + 7 of column 16 nt + m, by two transposed reads (rows 8 kq + q
          // and 8 kq + 4 + q supplied by lane 4 q + p of the 16-lane group, columns 16 nt + 4 p ..)
          const int qq = (lane & 15) >> 2, pp = lane & 3;
          const int r0 = 8 * kq + qq, r1 = r0 + 4, c2 = 2 * nt + (pp >> 1);
          const int o0 = raw_off(r0, c2) + 4 * (pp & 1);
          const int o1 = raw_off(r1, c2) + 4 * (pp & 1);
          typedef __fp16 hv4 __attribute__((__vector_size__(4 * sizeof(__fp16))));
          typedef __attribute__((address_space(3))) hv4* lp_t;
          const hv4 h0 = __builtin_amdgcn_ds_read_tr16_b64_v4f16((lp_t)const_cast<_Float16*>(yh + o0));
          const hv4 h1 = __builtin_amdgcn_ds_read_tr16_b64_v4f16((lp_t)const_cast<_Float16*>(yh + o1));
          const hv4 l0 = __builtin_amdgcn_ds_read_tr16_b64_v4f16((lp_t)const_cast<_Float16*>(yl + o0));
          const hv4 l1 = __builtin_amdgcn_ds_read_tr16_b64_v4f16((lp_t)const_cast<_Float16*>(yl + o1));
          typedef uint32_t u2v __attribute__((ext_vector_type(2)));
          typedef uint32_t u4v __attribute__((ext_vector_type(4)));
          const u2v h0b = __builtin_bit_cast(u2v, h0), h1b = __builtin_bit_cast(u2v, h1);
          const u2v l0b = __builtin_bit_cast(u2v, l0), l1b = __builtin_bit_cast(u2v, l1);
          d[i][0] = __builtin_bit_cast(h8, u4v{h0b.x, h0b.y, h1b.x, h1b.y});
          d[i][1] = __builtin_bit_cast(h8, u4v{l0b.x, l0b.y, l1b.x, l1b.y});
        } else {
          d[i][0] = *reinterpret_cast<const h8*>(yh + (16 * nt + m) * kLdY + 8 * kq);
          d[i][1] = *reinterpret_cast<const h8*>(yl + (16 * nt + m) * kLdY + 8 * kq);
        }
      }
    };
    read_grp(0, fb[0]);
#pragma unroll
    for (int gi = 0; gi < nGrp; ++gi) {
      if (gi + 1 < nGrp) read_grp(gi + 1, fb[(gi + 1) & 1]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < kGrp; ++i)
#pragma unroll
        for (int t = 0; t < MT; ++t)
          acc[t][gi * kGrp + i] = mma3(ah[t], al[t], fb[gi & 1][i][0], fb[gi & 1][i][1], acc[t][gi * kGrp + i]);
      __builtin_amdgcn_sched_barrier(0);
    }
    // step u + 1's X into the other buffer (read by nobody now: the barrier that ended step
    // u - 1 passed), then step u + 2's loads (clamped: past the end they reload the last step)
    if (u < 4) HBK_MT(2, 40 + 3 * u);
    write_y(min(u + 1, last), (u + 1) & 1);
    if (u < 4) HBK_MT(2, 41 + 3 * u);
    load_y(min(u + 3, last));
    load_g(min(u + 3, last), g);
    if (u < 4) HBK_MT(2, 42 + 3 * u);
    lds_barrier();  // (LDS only: the prefetched loads stay in flight)
    HBK_MT(2, 16 + u);
    // a scheduling fence per step: unfenced, the scheduler hoisted every step's (address-
    // independent) gradient loads to the top, ~11 VGPRs per unrolled step
    __builtin_amdgcn_sched_barrier(0);
  };
#pragma unroll
  for (int u = 0; u < NST; ++u) step(u, ga[u % 3]);  // (a runtime step bound, as a break or
  // a guard per step, cost 35 us against 24: rolled loop / per-step branch joins)
  HBK_MT(2, 2);
  float* const C = a.part + split * a.pstride + jb.c_off;
  if constexpr (!kRaw) {
#pragma unroll
    for (int t = 0; t < MT; ++t)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = mrow + 16 * t + 4 * kq + e;
        if (row >= jb.M) continue;
#pragma unroll
        for (int i = 0; i < NBW; ++i) {
          const int c = n0 + 16 * (nt0 + i) + m;
          if (c < jb.N) {
            *BCK(&C[static_cast<int64_t>(row) * jb.ldc + c], 4) = acc[t][i][e] * inv;
            // slabs past this job's splits (the launch's S is the largest job's): zeros
            for (int z = split + jb.S; z < a.S; z += jb.S)
              *BCK(&C[(z - split) * a.pstride + static_cast<int64_t>(row) * jb.ldc + c], 4) = 0.f;
          }
        }
      }
    return;
  } else {
    // input layer: dW = g o (dHG0^T xhat) + s (x) b, dgamma = sum_j W o (dHG0^T xhat),
    // dbeta = sum_j W s_j, with s_j = the split's sum of dHG0[b][j]
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      float sj = (ssum[t][0] + ssum[t][1]) + (ssum[t][2] + ssum[t][3]);
      sj += __shfl_xor(sj, 16, 64);
      sj += __shfl_xor(sj, 32, 64);
      if (kq == 0) sh.sS[16 * MT * mg + 16 * t + m] = sj;
    }
    // (the input layer's N is a multiple of the tile: every column live.) W0, gamma and beta
    // are loaded before the first store (a store may alias them: interleaved, each load
    // waited behind the one before)
    float wv[NBW][MT][4], gcv[NBW], bcv[NBW];
#pragma unroll
    for (int i = 0; i < NBW; ++i) {
      const int c = n0 + 16 * (nt0 + i) + m;
      gcv[i] = *BCK(&a.g_in[c], 4);
      bcv[i] = *BCK(&a.b_in[c], 4);
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          wv[i][t][e] = *BCK(&a.W0[static_cast<int64_t>(mrow + 16 * t + 4 * kq + e) * jb.ldc + c], 4);
    }
    __syncthreads();
    float dg[NBW], db[NBW];
#pragma unroll
    for (int i = 0; i < NBW; ++i) {
      dg[i] = db[i] = 0.f;
#pragma unroll
      for (int t = 0; t < MT; ++t)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = mrow + 16 * t + 4 * kq + e;  // j (< 128 = M)
          const float s = sh.sS[16 * MT * mg + 16 * t + 4 * kq + e];
          const float v = acc[t][i][e] * inv;
          *BCK(&C[static_cast<int64_t>(row) * jb.ldc + n0 + 16 * (nt0 + i) + m], 4) = gcv[i] * v + bcv[i] * s;
          dg[i] += wv[i][t][e] * v;
          db[i] += wv[i][t][e] * s;
        }
    }
    // per column, the M groups' partials: red[.][M group][column]
#pragma unroll
    for (int i = 0; i < NBW; ++i) {
#pragma unroll
      for (int o = 16; o < 64; o <<= 1) {
        dg[i] += __shfl_xor(dg[i], o, 64);
        db[i] += __shfl_xor(db[i], o, 64);
      }
      if (kq == 0) {
        sh.red[0][mg][16 * (nt0 + i) + m] = dg[i];
        sh.red[1][mg][16 * (nt0 + i) + m] = db[i];
      }
    }
    __syncthreads();
    if (tid < NT) {
      float* P = a.part + split * a.pstride;
      float rg = 0.f, rb = 0.f;
#pragma unroll
      for (int w = 0; w < kK3sMG; ++w) {
        rg += sh.red[0][w][tid];
        rb += sh.red[1][w][tid];
      }
      *BCK(&P[a.g_off + n0 + tid], 4) = rg;
      *BCK(&P[a.b_off + n0 + tid], 4) = rb;
    }
  }
}
// NST0: the input layer's steps per split, NST1: the generic jobs'; kOcc waves per SIMD
// (4: two workgroups per CU, <= 128 VGPRs -- the short-step pairs only: the unrolled steps'
// registers grow with the step count)
template <int NST0, int NST1, int kOcc>
__global__ void __launch_bounds__(kK3sThr, kOcc) k3s_kernel(K3sArgs a) {
  __shared__ __attribute__((aligned(16))) K3sShared sh;
  const int blk = blockIdx.x;
  int j = 0;
  while (j + 1 < a.n_jobs && blk >= a.start[j + 1]) ++j;
  const K3sJob jb = a.job[j];
  const int local = blk - a.start[j];
  const int split = local % jb.S, tile = local / jb.S;
  const int tm = tile / jb.tn, tnn = tile - tm * jb.tn;
  HBK_MT(2, 1);
  HBK_SPAN(0, __builtin_amdgcn_s_memrealtime());
  if (jb.Y == nullptr)
    k3s_body<kK3sNbtRaw, true, NST0>(a, jb, split, tm, tnn, sh);
  else
    k3s_body<kK3sNbtGen, false, NST1>(a, jb, split, tm, tnn, sh);
  HBK_SPAN(1, __builtin_amdgcn_s_memrealtime());
  HBK_SPAN(2, (static_cast<unsigned long long>(j) << 32) | split);
}

// Steps whose update does not get the workspace (or is preceded by the
// data-parallel all-reduce): the slabs added into the bucket's covered ranges
// float4 per thread, 8 slabs' loads issued together per round (clamped; the ones past ns weigh
// 0): a scalar loop over the slabs waited for each load in turn (+9 us per step before the
// data-parallel all-reduce at B = 1,100 on 64 CUs, 7 slabs)
__global__ void __launch_bounds__(256) k3_fold_kernel(Ranges rg, const float* __restrict__ part, int64_t pstride,
                                                      int ns, float* __restrict__ G, int64_t n) {
  constexpr int kR = 8;
  const int64_t n4 = n >> 2, ps4 = pstride >> 2;
  const f4* P4 = reinterpret_cast<const f4*>(part);
  f4* G4 = reinterpret_cast<f4*>(G);
  for (int64_t q = blockIdx.x * int64_t(256) + threadIdx.x; q < n4; q += int64_t(gridDim.x) * 256) {
    bool in[4], any = false;
#pragma unroll
    for (int e = 0; e < 4; ++e) any |= in[e] = in_ranges(rg, 4 * q + e);
    if (!any) continue;
    const f4 g0 = *BCK(&G4[q], 16);
    f4 acc = g0;
    for (int s0 = 0; s0 < ns; s0 += kR) {
      f4 v[kR];
#pragma unroll
      for (int u = 0; u < kR; ++u) v[u] = *BCK(&P4[min(s0 + u, ns - 1) * ps4 + q], 16);
#pragma unroll
      for (int u = 0; u < kR; ++u)
        if (s0 + u < ns) acc += v[u];
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) acc[e] = in[e] ? acc[e] : g0[e];
    *BCK(&G4[q], 16) = acc;
  }
  for (int64_t i = 4 * n4 + blockIdx.x * int64_t(256) + threadIdx.x; i < n; i += int64_t(gridDim.x) * 256) {
    if (!in_ranges(rg, i)) continue;
    float g = *BCK(&G[i], 4);
    for (int sp = 0; sp < ns; ++sp) g += *BCK(&part[sp * pstride + i], 4);
    *BCK(&G[i], 4) = g;
  }
}

// ------------------------------------------------------------------ k4 ----
constexpr int kTileR = 16, kMaxTiles = 48;
struct K4Args {
  float* P;
  float* G;  // gradient bucket; the statistics follow at G[n]
  float* m;
  float* v;
  int64_t n;
  float* state;
  int parity;
  const float* sched;
  int sched_len;
  float lr, b1, b2, eps;
  float* hist;
  int hist_cap;
  WSplit w;       // weight cache kept current with the update (wc NULL: not kept)
  _Float16* wc;
  // with wc: workgroups 0 .. n_tiles - 1 update the cached matrices in tiles of
  // kTileR rows (tile t: segment tile_seg[t], first row tile_r0[t]) and write the
  // transposed planes from LDS as 16-B column runs; the rest do everything else
  int n_tiles;
  int tile_seg[kMaxTiles], tile_r0[kMaxTiles];
  // k3's partial slabs left for this update (ns of them; 0: none)
  const float* part;
  int64_t pstride;
  int ns;
  // 32-bit forms of the per-element tests (n < 2^31; fewer scalar registers than the int64
  // WSplit / Ranges: those spilled 135 SGPRs): the cached matrices in float4 units [lo, hi),
  // the tile workgroups' share; the slab-covered ranges in floats
  int n_skip, n_cov;
  int32_t skip_lo[kMaxSeg], skip_hi[kMaxSeg];
  int32_t cov_lo[kMaxRng], cov_hi[kMaxRng];
};
__device__ __forceinline__ bool k4_covered(const K4Args& a, int32_t i) {
  bool c = false;
#pragma unroll
  for (int k = 0; k < kMaxRng; ++k) c |= k < a.n_cov && i >= a.cov_lo[k] && i < a.cov_hi[k];
  return c;
}

// The accumulation gate (trainer.py:443-465), computed identically by every
// workgroup from the step's read-only state half; workgroup 0 writes the other
// half and the history row. Then torch.optim.Adam (foreach, no weight decay) on
// grads * 1 / (n_sel * accumulation_steps) when it fires; the bucket's
// gradients are zeroed either way (zero_grad every step, :404).
__global__ void __launch_bounds__(256) k4_update_kernel(K4Args a) {
  const float* st = a.state + a.parity * 8;
  const float* stats = a.G + a.n;
  // statistics read before any store (the history row copies them)
  const float n_sel = stats[0], s_loss = stats[1], s_neg = stats[2], s_fp = stats[3], s_pos = stats[4],
              s_tp = stats[5];
  float acc_samples = st[0], acc_steps = st[1], t = st[2];
  const float stepf = st[3];
  const int step = static_cast<int>(stepf);
  float fire = 0.f, scale = 0.f, loss = 0.f;
  const float used = acc_steps;
  if (n_sel > 0.f) {
    loss = s_loss / n_sel / acc_steps;
    acc_samples += n_sel;
    if (acc_samples < 128.f) {
      acc_steps += 1.f;
    } else {
      fire = 1.f;
      scale = 1.f / (n_sel * acc_steps);
      acc_steps = 1.f;
      acc_samples = 0.f;
      t += 1.f;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    float* nx = a.state + (1 - a.parity) * 8;
    nx[0] = acc_samples;
    nx[1] = acc_steps;
    nx[2] = t;
    nx[3] = stepf + 1.f;
    nx[4] = st[4];  // dropout salt of the epoch
    if (a.hist && step < a.hist_cap) {
      float* h = a.hist + static_cast<int64_t>(step) * 8;
      h[0] = n_sel;
      h[1] = used;
      h[2] = fire;
      h[3] = loss;
      h[4] = s_neg;
      h[5] = s_fp;
      h[6] = s_pos;
      h[7] = s_tp;
    }
  }
  float lr = a.lr;
  if (a.sched) lr = a.sched[2 * min(step, a.sched_len - 1)];
  const int64_t n4 = a.n >> 2;
  f4* G4 = reinterpret_cast<f4*>(a.G);
  f4* P4 = reinterpret_cast<f4*>(a.P);
  f4* M4 = reinterpret_cast<f4*>(a.m);
  f4* V4 = reinterpret_cast<f4*>(a.v);
  const f4 z4 = {0.f, 0.f, 0.f, 0.f};
  const int ns = a.part ? a.ns : 0;
  const f4* PT4 = reinterpret_cast<const f4*>(a.part);
  const int64_t ps4 = a.pstride >> 2;
  // the step's gradient of float4 i: the bucket (k2's atomics) and zero it, or, in a range
  // covered by k3's deferred slabs (where the bucket holds zeros), the slabs' sum
  auto grad4 = [&](int64_t i, bool covered, bool zero) -> f4 {
    if (!covered) {
      const f4 g = G4[i];
      if (zero) G4[i] = z4;
      return g;
    }
    f4 q[4] = {z4, z4, z4, z4};
    int sp = 0;
    for (; sp + 4 <= ns; sp += 4) {
#pragma unroll
      for (int u = 0; u < 4; ++u) q[u] += PT4[(sp + u) * ps4 + i];
    }
    for (; sp < ns; ++sp) q[0] += PT4[sp * ps4 + i];
    return (q[0] + q[1]) + (q[2] + q[3]);
  };
  const float bc1 = 1.f - powf(a.b1, t), bc2s = sqrtf(1.f - powf(a.b2, t));
  const float step_size = lr / bc1, inv_bc2s = 1.f / bc2s;
  const bool on = fire != 0.f;
  // float4 body (the bucket, params and moments are 16-B aligned torch buffers), scalar tail

  // one float4: all four loads unconditional (issued together, no wait behind
  // the gate decision, which itself waits on the statistics); the parameters
  // after the step are returned
  auto adam4 = [&](int64_t i) -> f4 {
    const f4 g = grad4(i, ns > 0 && k4_covered(a, static_cast<int32_t>(4 * i)), true), m0 = M4[i], v0 = V4[i];
    f4 p = P4[i];
    if (on) {
      const f4 gi = g * scale;
      const f4 mi = a.b1 * m0 + (1.f - a.b1) * gi;
      const f4 vi = a.b2 * v0 + (1.f - a.b2) * gi * gi;
      M4[i] = mi;
      V4[i] = vi;
#pragma unroll
      for (int e = 0; e < 4; ++e) p[e] -= adam_step(mi[e], vi[e], step_size, inv_bc2s, a.eps);
      P4[i] = p;
    }
    return p;
  };
  const int t0 = a.wc ? a.n_tiles : 0;
  if (static_cast<int>(blockIdx.x) < t0) {  // a tile of a cached matrix
    __shared__ float tileS[kTileR][kL + 1];
    const WSeg g = a.w.s[a.tile_seg[blockIdx.x]];
    const int r0 = a.tile_r0[blockIdx.x], C = g.cols, C4 = g.cols / 4;
    const int rows = min(kTileR, g.rows - r0);
    const int64_t rc = int64_t(g.rows) * C;
    _Float16* d = a.wc + g.dst;
    // <= kTileR * kL / 4 / 256 float4s per thread (2), all loads issued first
    // (clamped indices) so the tile costs one memory latency, not several
    constexpr int kIt = (kTileR * kL / 4 + 255) / 256;
    f4 lg_[kIt], lm_[kIt], lv_[kIt], lp_[kIt];
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int q = min(static_cast<int>(threadIdx.x) + 256 * it, rows * C4 - 1);
      const int r = q / C4, c4 = q - r * C4;
      const int64_t i = (g.src + int64_t(r0 + r) * C + 4 * c4) >> 2;
      lg_[it] = grad4(i, ns > 0, false);  // the cached matrices are k3's (covered); zeroed by the owner below
      lm_[it] = M4[i];
      lv_[it] = V4[i];
      lp_[it] = P4[i];
    }
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const int q = static_cast<int>(threadIdx.x) + 256 * it;
      if (q >= rows * C4) break;
      const int r = q / C4, c4 = q - r * C4;
      const int64_t off = int64_t(r0 + r) * C + 4 * c4;
      const int64_t i = (g.src + off) >> 2;
      f4 p = lp_[it];
      if (ns == 0) G4[i] = z4;  // (with slabs the bucket holds zeros here)
      if (on) {
        const f4 gi = lg_[it] * scale;
        const f4 mi = a.b1 * lm_[it] + (1.f - a.b1) * gi;
        const f4 vi = a.b2 * lv_[it] + (1.f - a.b2) * gi * gi;
        M4[i] = mi;
        V4[i] = vi;
#pragma unroll
        for (int e = 0; e < 4; ++e) p[e] -= adam_step(mi[e], vi[e], step_size, inv_bc2s, a.eps);
        P4[i] = p;
      }
      if (on) {
        uint32_t h[2], l[2];
        split_pair(16.f * p[0], 16.f * p[1], h[0], l[0]);
        split_pair(16.f * p[2], 16.f * p[3], h[1], l[1]);
        *reinterpret_cast<uint2*>(d + off) = uint2{h[0], h[1]};
        *reinterpret_cast<uint2*>(d + rc + off) = uint2{l[0], l[1]};
#pragma unroll
        for (int e = 0; e < 4; ++e) tileS[r][4 * c4 + e] = p[e];
      }
    }
    if (!on) return;  // the gate is the same in every thread: parameters and cache unchanged
    __syncthreads();
    for (int u = threadIdx.x; u < C * (kTileR / 8); u += 256) {
      const int c = u / (kTileR / 8), rb = 8 * (u % (kTileR / 8));
      if (rb >= rows) continue;
      h8 hi, lo;
      split8(f4{tileS[rb][c], tileS[rb + 1][c], tileS[rb + 2][c], tileS[rb + 3][c]} * 16.f,
             f4{tileS[rb + 4][c], tileS[rb + 5][c], tileS[rb + 6][c], tileS[rb + 7][c]} * 16.f, hi, lo);
      const int64_t o = int64_t(c) * g.rows + r0 + rb;
      *reinterpret_cast<h8*>(d + 2 * rc + o) = hi;
      *reinterpret_cast<h8*>(d + 3 * rc + o) = lo;
    }
    return;
  }
  const int64_t b0 = static_cast<int64_t>(blockIdx.x) - t0, nb = static_cast<int64_t>(gridDim.x) - t0;
  for (int64_t i = b0 * 256 + threadIdx.x; i < n4; i += nb * 256) {
    if (t0) {  // cached matrices are the tile workgroups'
      bool cached = false;
      const int32_t i32 = static_cast<int32_t>(i);
#pragma unroll
      for (int sg = 0; sg < kMaxSeg; ++sg) cached |= sg < a.n_skip && i32 >= a.skip_lo[sg] && i32 < a.skip_hi[sg];
      if (cached) continue;
    }
    adam4(i);
  }
  for (int64_t i = 4 * n4 + b0 * 256 + threadIdx.x; i < a.n; i += nb * 256) {
    float g = a.G[i];
    if (ns > 0 && k4_covered(a, static_cast<int32_t>(i)))
      for (int sp = 0; sp < ns; ++sp) g += a.part[sp * a.pstride + i];
    a.G[i] = 0.f;
    if (on) {
      const float gi = g * scale;
      const float mi = a.b1 * a.m[i] + (1.f - a.b1) * gi;
      const float vi = a.b2 * a.v[i] + (1.f - a.b2) * gi * gi;
      a.m[i] = mi;
      a.v[i] = vi;
      a.P[i] -= adam_step(mi, vi, step_size, inv_bc2s, a.eps);
    }
  }
}


// ---------------------------------------------------------- evaluation ----
// The validation / testing passes of train_epoch (trainer.py:496-566): a
// forward with input dropout over hundreds of thousands of rows (the default
// validation pass is 500 batches of 50 + 1,000 rows, the testing pass 500 of
// 50 + 50), reduced to prediction counts. The input layer is a real GEMM here
// ([rows, 1536] x [1536, 128]), so it gets a throughput kernel of its own,
// kv_gemm: the LayerNorm is folded into the GEMM's epilogue,
//   (LN(x) g + b) W^T = rs (x W'^T - mu c1) + c0,  W' = W o g (columns scaled),
//   c1[n] = sum_k W'[n][k],  c0[n] = sum_k b[k] W[n][k],
// so the product runs on the raw (dropped-out) rows: an f16 pool row is exact
// in f16 (its hi part; no lo), two products per 32-deep block instead of
// three. mu / rs come from the same loaded values (per-lane float sums of 8,
// accumulated in double). W' (f16 hi / lo planes of 16 W') is staged through
// LDS in 64-deep chunks, double-buffered, shared by 8 waves of 32 rows each;
// the rows stream from HBM straight into MFMA A fragments, prefetched two
// chunks ahead. The pre-bias HG0 rows go to a slab that k2_rows_kernel
// <false> (the inference chain, with its counters) reads as its one K-split.
constexpr int kKvKC = 64, kKvChunks = kD / kKvKC;
constexpr int kKvMaxSeg = kEvalMaxSeg;
struct KvArgs {
  const void* pool;      // f32 or f16 rows of 1536
  int64_t n_pool;
  const int32_t* idx;    // row r -> pool row idx[r]; NULL: r0 + r modulo n_pool
  int64_t rows, r0;      // this launch's rows; r0 = their first index in the pass (dropout counter)
  const _Float16* wq;    // [2][128][1536] hi / lo planes of 16 W'
  const float* c0;
  const float* c1;
  float drop_p;
  uint64_t seed;
  // the rest of the network (parameter offsets; weight cache planes as k2 reads them)
  const float* P;
  int64_t b_hg[kMaxG], b_o[kMaxG], w_o[kMaxG], ln_g[kMaxG], ln_b[kMaxG];
  const _Float16* wc;
  int64_t c_o[kMaxG], c_hg[kMaxG];
  float act_thr;
  float* counts;  // [4]: counts[2 label] += #(p >= act_thr), counts[2 label + 1] += #(p > act_thr)
  int label;
  float* prob;    // [rows] or NULL
  // several pools in one launch (hbk_mlp_eval_count_multi; nseg = 0: the fields above): workgroup
  // b of segment s = the first segment with b < seg_tile0[s + 1] takes pool s's tile b - seg_tile0[s]
  int nseg;
  int seg_tile0[kKvMaxSeg + 1];
  const void* seg_pool[kKvMaxSeg];
  int64_t seg_npool[kKvMaxSeg], seg_rows[kKvMaxSeg], seg_r0[kKvMaxSeg];
  uint64_t seg_seed[kKvMaxSeg];
  float* seg_counts[kKvMaxSeg];
  int seg_label[kKvMaxSeg];
};

__global__ void __launch_bounds__(256) kv_prep_kernel(const float* __restrict__ P, int64_t w0, int64_t g_in,
                                                      int64_t b_in, _Float16* __restrict__ wq, float* c0,
                                                      float* c1) {
  __shared__ double red[2][4];
  const int n = blockIdx.x, tid = threadIdx.x;
  const float* W = P + w0 + int64_t(n) * kD;
  double s0 = 0.0, s1 = 0.0;
  for (int k = 2 * tid; k < kD; k += 512) {
    const float wa = W[k], wb = W[k + 1];
    const float ga = wa * P[g_in + k], gb = wb * P[g_in + k + 1];
    uint32_t hi, lo;
    split_pair(16.f * ga, 16.f * gb, hi, lo);
    *reinterpret_cast<uint32_t*>(wq + int64_t(n) * kD + k) = hi;
    *reinterpret_cast<uint32_t*>(wq + int64_t(kH2) * kD + int64_t(n) * kD + k) = lo;
    s1 += double(ga) + double(gb);
    s0 += double(P[b_in + k]) * wa + double(P[b_in + k + 1]) * wb;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) {
    s0 += __shfl_xor(s0, o, 64);
    s1 += __shfl_xor(s1, o, 64);
  }
  if ((tid & 63) == 0) {
    red[0][tid >> 6] = s0;
    red[1][tid >> 6] = s1;
  }
  __syncthreads();
  if (tid == 0) {
    c0[n] = static_cast<float>((red[0][0] + red[0][1]) + (red[0][2] + red[0][3]));
    c1[n] = static_cast<float>((red[1][0] + red[1][1]) + (red[1][2] + red[1][3]));
  }
}

#ifndef HBK_KV_ABLATE
#define HBK_KV_ABLATE 0  // profiling builds: 1 skips the network phase, 2 the dropout mask
#endif
// The streamed rows are read once: non-temporal loads (HBK_KV_NT, default on)
// keep them from evicting W', which every tile re-reads, from the XCD's L2.
#ifndef HBK_KV_NT
#define HBK_KV_NT 1
#endif
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 load_rows4(const uint4* p) {
#if HBK_KV_NT
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return uint4{v[0], v[1], v[2], v[3]};
#else
  return *p;
#endif
}

// kF16: the rows are f16 (exact in hi); else f32 (split hi / lo).
// W' chunks reach LDS by global->LDS DMA (global_load_lds_dwordx4: no register
// staging, so no spills at 8 waves x ~240 VGPRs), issued two chunks ahead. The
// DMA writes a wave's 64 x 16 B contiguously, so the image is unpadded
// [plane][n][64 halves] rows with the 16-B pieces XOR-swizzled by (n >> 1) & 7
// on the SOURCE address (the B-fragment reads of 16 lanes then hit 16
// distinct 4-bank groups). The chunk's barrier waits with a counted vmcnt
// (the DMA retired, the next rows' loads still in flight) and a raw s_barrier:
// __syncthreads() would emit vmcnt(0) and drain the row prefetch.
constexpr int kKvPiece = 8;  // 16-B pieces per 64-deep row of a chunk
__device__ __forceinline__ int kv_swz(int n) { return (n >> 1) & 7; }
constexpr int kNetWLd = 104, kAld = 100;  // LDS row strides: weight halves (K <= 96), activation floats
// W: waves per workgroup, 8 (f16 rows: two 16-row tiles per wave) or 16 (one tile per wave:
// twice the waves per CU to hide the stream's latency, at most 128 VGPRs each)
template <bool kF16, int NG, int W>
__global__ void __launch_bounds__(64 * W) kv_gemm_kernel(KvArgs a0) {
  // this workgroup's pool (segment): its fields replace the single-pool ones (uniform)
  KvArgs a = a0;
  int blk = static_cast<int>(blockIdx.x);
  if (a0.nseg > 0) {
    int sg = 0;
#pragma unroll
    for (int q = 1; q < kKvMaxSeg; ++q) sg += (q < a0.nseg && blk >= a0.seg_tile0[q]) ? 1 : 0;
    blk -= a0.seg_tile0[sg];
    a.pool = a0.seg_pool[sg];
    a.n_pool = a0.seg_npool[sg];
    a.idx = nullptr;
    a.rows = a0.seg_rows[sg];
    a.r0 = a0.seg_r0[sg];
    a.seed = a0.seg_seed[sg];
    a.counts = a0.seg_counts[sg];
    a.label = a0.seg_label[sg];
    a.prob = nullptr;
  }
  // ONE __shared__ object: beside a second one hipcc drains the DMA (vmcnt(0))
  // before every chunk's first LDS read. GEMM phase: the W' ring (the row
  // statistics reuse buffer 0 after it); network phase: a stage's weight planes
  // at 0, the waves' activation tiles after them, two counters last.
  constexpr int kWBuf = 3;  // W' ring: chunk c + 2's DMA is issued during chunk c (kWBuf - 1 == 2 assumed below)
  constexpr int kRT = (kF16 && W == 8) ? 2 : 1;  // 16-row tiles per wave (f32 rows: one, for the split's registers)
  constexpr int kThr = 64 * W;
  constexpr int kGemmBytes = kWBuf * 2 * kH2 * kKvKC * 2;
  constexpr int kWsBytes = 2 * kH2 * kNetWLd * 2;
  constexpr int kActBytes = W * 16 * kRT * kAld * 4;
  constexpr int kLdsBytes = (kGemmBytes > kWsBytes + kActBytes ? kGemmBytes : kWsBytes + kActBytes) + 16;
  static_assert(kLdsBytes <= 160 * 1024, "one workgroup's LDS");
  __shared__ __attribute__((aligned(16))) unsigned char smem[kLdsBytes];
  auto wb = reinterpret_cast<_Float16 (*)[2][kH2][kKvKC]>(smem);  // [buf][hi / lo][n][k] (swizzled pieces)
  float (*stS)[16 * kRT][2] = reinterpret_cast<float (*)[16 * kRT][2]>(smem);
  static_assert(sizeof(float) * W * 16 * kRT * 2 <= kWsBytes, "statistics: below the activation tiles");
#ifndef HBK_KV_DEPTH
#define HBK_KV_DEPTH 2
#endif
  constexpr int kDepth = kF16 ? HBK_KV_DEPTH : 2;  // A chunks in flight (this one + kDepth - 1 ahead)
  constexpr int kBGroup = kDepth > 2 ? 2 : 4;       // column tiles whose B fragments may be in flight together
  constexpr int kU = kF16 ? 1 : 2;  // 16-B loads per 8 elements
  constexpr int kALoads = kRT * 2 * kU;  // per chunk
  constexpr int kTile = W * 16 * kRT;
  constexpr int kDma = 32 / W;  // W' DMA instructions per wave and chunk (2 planes x 128 rows of 128 B)
  static_assert(kALoads * (kDepth - 1) + kDma < 16, "the counted waits use vmcnt's low field");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, m = lane & 15, kq = lane >> 4;
  const int64_t tile0 = int64_t(blk) * kTile;
  const char* rp[kRT];
  uint32_t rid[kRT];
#pragma unroll
  for (int rt = 0; rt < kRT; ++rt) {
    const int64_t r = min(tile0 + 16 * kRT * wave + 16 * rt + m, a.rows - 1);
    int64_t pr = a.idx ? static_cast<int64_t>(a.idx[r]) : (a.r0 + r) % a.n_pool;
    pr = min(max(pr, int64_t(0)), a.n_pool - 1);
    rp[rt] = static_cast<const char*>(a.pool) + pr * kD * (kF16 ? 2 : 4);
    rid[rt] = static_cast<uint32_t>(a.r0 + r);
  }
  const uint64_t seed = a.seed;
  const uint32_t s0 = static_cast<uint32_t>(seed), s1 = static_cast<uint32_t>(seed >> 32) * 0x27D4EB2Fu;
  const uint32_t thr = static_cast<uint32_t>(a.drop_p * 65536.f + 0.5f);
  const float keep = a.drop_p > 0.f ? 1.f / (1.f - a.drop_p) : 1.f;
  uint4 ar[kDepth][kRT][2][kU];
  auto load_rows = [&](int c, int slot) {
#pragma unroll
    for (int rt = 0; rt < kRT; ++rt)
#pragma unroll
      for (int kb = 0; kb < 2; ++kb) {
        const int k = kKvKC * c + 32 * kb + 8 * kq;
#pragma unroll
        for (int u = 0; u < kU; ++u)
          ar[slot][rt][kb][u] = load_rows4(reinterpret_cast<const uint4*>(rp[rt] + int64_t(k) * (kF16 ? 2 : 4) + 16 * u));
      }
  };
  // W' chunk c -> buffer buf: 2 planes x 128 rows x 8 pieces = 2,048 pieces, 4 DMA
  // instructions per wave (8 rows each); lane l of instruction j writes piece
  // (row 8 (4 wave + j) + l / 8, slot l % 8), reading the source piece slot ^ swz(row)
  auto dma_w = [&](int c, int buf) {
#pragma unroll
    for (int j = 0; j < kDma; ++j) {
      const int row8 = kDma * wave + j;              // 0 .. 31: plane row8 / 16, rows 8 (row8 % 16) ..
      const int pl = row8 >> 4, n = 8 * (row8 & 15) + (lane >> 3), pc = (lane & 7) ^ kv_swz(n);
      const _Float16* src = a.wq + int64_t(pl) * kH2 * kD + int64_t(n) * kD + kKvKC * c + kKvPiece * pc;
      __builtin_amdgcn_global_load_lds(src, &wb[buf][pl][8 * (row8 & 15)][0], 16, 0, 0);
    }
  };
  // prologue: chunks 0 and 1 (W' buffers 0, 1; A slots 0, 1); chunk 0 waited for here,
  // chunk 1 at the end of chunk 0
  dma_w(0, 0);
  load_rows(0, 0);
  dma_w(1, 1);
#pragma unroll
  for (int d = 1; d < kDepth; ++d) load_rows(d, d);
  __builtin_amdgcn_s_waitcnt((kALoads * (kDepth - 1) + kDma) | (0x7 << 4) | (0xF << 8));  // chunk 0 in (the later chunks' DMA and rows may fly)
  dma_barrier();
  f4 acc[kRT][8];
#pragma unroll
  for (int rt = 0; rt < kRT; ++rt)
#pragma unroll
    for (int ct = 0; ct < 8; ++ct) acc[rt][ct] = f4{0.f, 0.f, 0.f, 0.f};
  double sd1[kRT], sd2[kRT];
#pragma unroll
  for (int rt = 0; rt < kRT; ++rt) sd1[rt] = sd2[rt] = 0.0;
  static_assert(kKvChunks % kDepth == 0, "the A ring's slots must be compile-time");
  int buf = 0;  // W' buffer of chunk c (c % kWBuf; a run-time LDS offset, the A slot is unrolled)
#pragma unroll 1
  for (int cb = 0; cb < kKvChunks; cb += kDepth)
#pragma unroll
  for (int slot = 0; slot < kDepth; ++slot) {
    const int c = cb + slot;
    const int bnext = buf == 0 ? kWBuf - 1 : buf - 1;  // (c + 2) % kWBuf
    // this chunk's A values (dropout mask, row sums, split) first: their loads are
    // ordinary global loads, so no DMA may be outstanding when they are used
    h8 ah[kRT][2], al[kRT][2];
    float t1[kRT], t2[kRT];
#pragma unroll
    for (int rt = 0; rt < kRT; ++rt) t1[rt] = t2[rt] = 0.f;
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int rt = 0; rt < kRT; ++rt) {
        float v[8];
        if (kF16) {
          const h8 hv = __builtin_bit_cast(h8, ar[slot][rt][kb][0]);
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = static_cast<float>(hv[e]);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) v[e] = __builtin_bit_cast(float, (&ar[slot][rt][kb][e >> 2].x)[e & 3]);
        }
        if (!(HBK_KV_ABLATE & 2) && a.drop_p > 0.f) {  // nn.Dropout's mask (the 1 / (1 - p) scale is applied after the GEMM)
          const uint32_t base = rid[rt] * (kD / 2) + ((kKvKC * c + 32 * kb + 8 * kq) >> 1);
#pragma unroll
          for (int e = 0; e < 8; e += 2) {
            const uint32_t hsh = drop_hash(s0, s1, base + (e >> 1));
            v[e] = (hsh & 0xFFFFu) < thr ? 0.f : v[e];
            v[e + 1] = (hsh >> 16) < thr ? 0.f : v[e + 1];
          }
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          t1[rt] += v[e];
          t2[rt] += v[e] * v[e];
        }
        if (kF16) {
#pragma unroll
          for (int e = 0; e < 8; ++e) ah[rt][kb][e] = static_cast<_Float16>(v[e]);  // exact
        } else {
          split8(f4{v[0], v[1], v[2], v[3]}, f4{v[4], v[5], v[6], v[7]}, ah[rt][kb], al[rt][kb]);
        }
      }
#pragma unroll
    for (int rt = 0; rt < kRT; ++rt) {
      sd1[rt] += double(t1[rt]);
      sd2[rt] += double(t2[rt]);
    }
    // unconditional (past the end: a clamped re-read) so that the loop has no
    // branches and hipcc's counted waits stay exact across the back edge
    dma_w(min(c + 2, kKvChunks - 1), bnext);  // its readers (chunk c - 1) passed the last barrier
    load_rows(min(c + kDepth, kKvChunks - 1), slot);
#pragma unroll
    for (int kb = 0; kb < 2; ++kb)
#pragma unroll
      for (int ct = 0; ct < 8; ++ct) {
        const int n = 16 * ct + m, pc = (4 * kb + kq) ^ kv_swz(n);
        const h8 bh = *reinterpret_cast<const h8*>(&wb[buf][0][n][kKvPiece * pc]);
        const h8 bl = *reinterpret_cast<const h8*>(&wb[buf][1][n][kKvPiece * pc]);
#pragma unroll
        for (int rt = 0; rt < kRT; ++rt) {
          acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[rt][kb], bh, acc[rt][ct], 0, 0, 0);
          acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[rt][kb], bl, acc[rt][ct], 0, 0, 0);
          if (!kF16) acc[rt][ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[rt][kb], bh, acc[rt][ct], 0, 0, 0);
        }
        if ((ct & (kBGroup - 1)) == kBGroup - 1) __builtin_amdgcn_sched_barrier(0);  // bound the B fragments in flight (registers)
      }
    // chunk c + 1's DMA and rows retired (chunk c + 2's, issued above, may still fly), then the barrier.
    // The sched_barriers keep the next chunk's conversions below the counted wait: hoisted
    // above it, hipcc guards them with vmcnt(0) (DMA and row loads pending together)
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt((kALoads * (kDepth - 1) + kDma) | (0x7 << 4) | (0xF << 8));  // chunk c + 1 in
    __builtin_amdgcn_s_waitcnt((0x3F & 0xF) | ((0x3F >> 4) << 14) | (0x7 << 4) | (0x0 << 8));  // lgkmcnt(0)
    dma_barrier();
    __builtin_amdgcn_sched_barrier(0);
    buf = buf == kWBuf - 1 ? 0 : buf + 1;
  }
  __builtin_amdgcn_s_waitcnt((0x7 << 4) | (0xF << 8));  // vmcnt(0): the clamped re-reads (into buffers 0, 1) in
  dma_barrier();
  // row statistics: the 4 lanes m + 16 kq hold a row's parts
  // (buffer 0's last readers, chunk kKvChunks - 2, passed that chunk's barrier)
#pragma unroll
  for (int rt = 0; rt < kRT; ++rt) {
#pragma unroll
    for (int o = 16; o < 64; o <<= 1) {
      sd1[rt] += __shfl_xor(sd1[rt], o, 64);
      sd2[rt] += __shfl_xor(sd2[rt], o, 64);
    }
    if (kq == 0) {
      const double mu = sd1[rt] * (1.0 / kD);
      const double var = fmax(sd2[rt] * (1.0 / kD) - mu * mu, 0.0);
      const double kp = double(keep);
      stS[wave][16 * rt + m][0] = static_cast<float>(kp * mu);                              // mean of the dropped-out row
      stS[wave][16 * rt + m][1] = static_cast<float>(1.0 / sqrt(kp * kp * var + double(kLnEps)));  // its 1 / std
    }
  }
  dma_barrier();
#if HBK_KV_ABLATE & 1  // profiling build: the input GEMM only (no network, no counts)
  if (a.rows > 0) return;
#endif
  // ---- the rest of the network, per wave on its kRT row tiles ----
  // HG0 = rs (acc / 16 keep - mu c1) + c0 + b; U0 = silu(H) G into the wave's
  // activation tile (the lane holds hidden column j = 16 ct + m and gate column
  // 64 + j: ct and ct + 4)
  float* A = reinterpret_cast<float*>(smem + kWsBytes) + wave * (16 * kRT * kAld);
  {
    const float ks = keep * (1.f / 16.f);
    float mu[kRT][4], rs[kRT][4];
#pragma unroll
    for (int rt = 0; rt < kRT; ++rt)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        mu[rt][e] = stS[wave][16 * rt + 4 * kq + e][0];
        rs[rt][e] = stS[wave][16 * rt + 4 * kq + e][1];
      }
    lds_barrier();  // every wave has its statistics: the activation tiles may overwrite them
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      const int j = 16 * ct + m;
      const float c0h = a.c0[j] + a.P[a.b_hg[0] + j], c0g = a.c0[kH + j] + a.P[a.b_hg[0] + kH + j];
      const float c1h = a.c1[j], c1g = a.c1[kH + j];
#pragma unroll
      for (int rt = 0; rt < kRT; ++rt)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float h = rs[rt][e] * (acc[rt][ct][e] * ks - mu[rt][e] * c1h) + c0h;
          const float g = rs[rt][e] * (acc[rt][ct + 4][e] * ks - mu[rt][e] * c1g) + c0g;
          A[(16 * rt + 4 * kq + e) * kAld + j] = h * sigm_fast(h) * g;
        }
    }
  }
  // weight stages: W_o_0, W_hg_1, W_o_1, ..., W_hg_{NG-1}: (cache offset, N, K); each
  // stage's f16 hi / lo planes staged into LDS once for the 8 waves, the next
  // stage's loaded into registers while the current one runs
  _Float16 (*wS)[kH2][kNetWLd] = reinterpret_cast<_Float16 (*)[kH2][kNetWLd]>(smem);
  constexpr int kStages = 2 * (NG - 1);
  auto st_off = [&](int st) { return (st & 1) ? a.c_hg[st / 2 + 1] : a.c_o[st / 2]; };
  auto st_n = [](int st) { return (st & 1) ? kH2 : kL; };
  auto st_k = [](int st) { return (st & 1) ? kL : kH; };
  // (six named registers, not an array: an array here stays in scratch memory
  // beside the GEMM phase's register pressure)
  uint4 wr0, wr1, wr2, wr3, wr4, wr5;
  constexpr int kWr = 3072 / kThr;  // staged 16-B pieces per thread (W_hg: 2 planes x 1,536)
  auto piece = [&](int st, int j, int& pl, int& n, int& k) {
    const int N = st_n(st), K = st_k(st), pieces = N * K / 8;  // per plane
    const int q = min(tid + kThr * j, 2 * pieces - 1), e0 = q % pieces;
    pl = q / pieces;
    n = (8 * e0) / K;
    k = 8 * e0 - n * K;
  };
  auto load1 = [&](int st, int j, uint4& v) {
    int pl, n, k;
    piece(st, j, pl, n, k);
    v = *reinterpret_cast<const uint4*>(a.wc + st_off(st) + int64_t(pl) * st_n(st) * st_k(st) + n * st_k(st) + k);
  };
  auto store1 = [&](int st, int j, const uint4& v) {  // (threads past the pieces repeat the last one)
    int pl, n, k;
    piece(st, j, pl, n, k);
    *reinterpret_cast<uint4*>(&wS[pl][n][k]) = v;
  };
  auto load_w = [&](int st) {
    load1(st, 0, wr0);
    load1(st, 1, wr1);
    load1(st, 2, wr2);
    if constexpr (kWr > 3) {
      load1(st, 3, wr3);
      load1(st, 4, wr4);
      load1(st, 5, wr5);
    }
  };
  auto store_w = [&](int st) {
    store1(st, 0, wr0);
    store1(st, 1, wr1);
    store1(st, 2, wr2);
    if constexpr (kWr > 3) {
      store1(st, 3, wr3);
      store1(st, 4, wr4);
      store1(st, 5, wr5);
    }
  };
  load_w(0);
  store_w(0);
  lds_barrier();
  const float* P = a.P;
#pragma unroll
  for (int st = 0; st < kStages; ++st) {
    if (st + 1 < kStages) load_w(st + 1);  // the next stage's planes, in flight during this one
    if ((st & 1) == 0) {
      // S = U W_o^T + b_o (K 64, N 96: 6 column tiles), then LayerNorm k -> X (A, K 96)
      const int k = st / 2;
      AFrag<kH> af[kRT];
#pragma unroll
      for (int rt = 0; rt < kRT; ++rt) af[rt] = load_a<kH, kAld>(A + 16 * rt * kAld, lane);
      f4 c[kRT][6];
#pragma unroll
      for (int ct = 0; ct < 6; ++ct) {
#pragma unroll
        for (int rt = 0; rt < kRT; ++rt) c[rt][ct] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < kH / 32; ++i) {
          const h8 bh = *reinterpret_cast<const h8*>(&wS[0][16 * ct + m][32 * i + 8 * kq]);
          const h8 bl = *reinterpret_cast<const h8*>(&wS[1][16 * ct + m][32 * i + 8 * kq]);
#pragma unroll
          for (int rt = 0; rt < kRT; ++rt) c[rt][ct] = mma3(af[rt].h[i], af[rt].l[i], bh, bl, c[rt][ct]);
        }
      }
      float bo[6], gm[6], bt[6];
#pragma unroll
      for (int ct = 0; ct < 6; ++ct) {
        bo[ct] = P[a.b_o[k] + 16 * ct + m];
        gm[ct] = P[a.ln_g[k] + 16 * ct + m];
        bt[ct] = P[a.ln_b[k] + 16 * ct + m];
      }
#pragma unroll
      for (int rt = 0; rt < kRT; ++rt) {
        float sm[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ct = 0; ct < 6; ++ct)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            c[rt][ct][e] = c[rt][ct][e] * af[rt].inv + bo[ct];
            sm[e] += c[rt][ct][e];
          }
        float mu[4], sq[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int e = 0; e < 4; ++e) mu[e] = rsum16(sm[e]) * (1.f / kL);
#pragma unroll
        for (int ct = 0; ct < 6; ++ct)
#pragma unroll
          for (int e = 0; e < 4; ++e) sq[e] += (c[rt][ct][e] - mu[e]) * (c[rt][ct][e] - mu[e]);
#pragma unroll
        for (int e = 0; e < 4; ++e) sq[e] = __builtin_amdgcn_rsqf(rsum16(sq[e]) * (1.f / kL) + kLnEps);
#pragma unroll
        for (int ct = 0; ct < 6; ++ct)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            A[(16 * rt + 4 * kq + e) * kAld + 16 * ct + m] = (c[rt][ct][e] - mu[e]) * sq[e] * gm[ct] + bt[ct];
      }
    } else {
      // HG = X W_hg^T + b (K 96, N 128), gate in the epilogue -> U (A, K 64)
      const int k = st / 2 + 1;
      AFrag<kL> af[kRT];
#pragma unroll
      for (int rt = 0; rt < kRT; ++rt) af[rt] = load_a<kL, kAld>(A + 16 * rt * kAld, lane);
      f4 c[kRT][8];
#pragma unroll
      for (int ct = 0; ct < 8; ++ct) {
#pragma unroll
        for (int rt = 0; rt < kRT; ++rt) c[rt][ct] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int i = 0; i < kL / 32; ++i) {
          const h8 bh = *reinterpret_cast<const h8*>(&wS[0][16 * ct + m][32 * i + 8 * kq]);
          const h8 bl = *reinterpret_cast<const h8*>(&wS[1][16 * ct + m][32 * i + 8 * kq]);
#pragma unroll
          for (int rt = 0; rt < kRT; ++rt) c[rt][ct] = mma3(af[rt].h[i], af[rt].l[i], bh, bl, c[rt][ct]);
        }
      }
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        const int col = 16 * ct + m;
        const float bh = P[a.b_hg[k] + col], bg = P[a.b_hg[k] + kH + col];
#pragma unroll
        for (int rt = 0; rt < kRT; ++rt)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float h = c[rt][ct][e] * af[rt].inv + bh, g = c[rt][ct + 4][e] * af[rt].inv + bg;
            A[(16 * rt + 4 * kq + e) * kAld + col] = h * sigm_fast(h) * g;
          }
      }
    }
    if (st + 1 < kStages) {
      lds_barrier();  // every wave is done with this stage's planes
      store_w(st + 1);
      lds_barrier();
    }
  }
  // z = U w_out + b_out: lane -> row lane / 4 of a tile, 16 columns; sigmoid, counts
  float* cntS = reinterpret_cast<float*>(smem + kWsBytes + kActBytes);
  if (tid < 2) cntS[tid] = 0.f;
  lds_barrier();
  {
    const int r = lane >> 2, c0 = 16 * (lane & 3);
    float wo[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) wo[q] = P[a.w_o[NG - 1] + c0 + q];
    const float bz = P[a.b_o[NG - 1]];
    int ge = 0, gt = 0;
#pragma unroll
    for (int rt = 0; rt < kRT; ++rt) {
      float z = 0.f;
#pragma unroll
      for (int q = 0; q < 16; ++q) z = fmaf(A[(16 * rt + r) * kAld + c0 + q], wo[q], z);
      z += dpp_f<0xB1>(z);  // quad_perm: lanes ^ 1, ^ 2 hold the row's other columns
      z += dpp_f<0x4E>(z);
      z += bz;
      const int64_t row = tile0 + 16 * kRT * wave + 16 * rt + r;
      const bool live = row < a.rows && (lane & 3) == 0;
      const float p = sigm_fast(z);
      if (live && a.prob) a.prob[row] = p;
      ge += __popcll(__ballot(live && p >= a.act_thr));
      gt += __popcll(__ballot(live && p > a.act_thr));
    }
    if (lane == 0) {
      if (ge) atomicAdd(&cntS[0], static_cast<float>(ge));
      if (gt) atomicAdd(&cntS[1], static_cast<float>(gt));
    }
  }
  lds_barrier();
  if (tid < 2 && cntS[tid] != 0.f) atomicAdd(a.counts + 2 * a.label + tid, cntS[tid]);
}


// After the passes (trainer.py:509-536, :549-566): the validation false
// positives per hour (count / hours in float32, as torch divides an integer
// count tensor by a Python float), recall, the testing rates, and the dynamic
// negative weight (x ratio above the target rate, / ratio with a floor of 1
// otherwise) written into the schedule rows of every later step.
struct EvalFinish {
  const float* cv;  // validation counts [4] (label 0: >=, >; label 1: >=, >)
  const float* ct;  // testing counts [4] or NULL
  float n_neg_v, n_pos_v, n_neg_t, n_pos_t;
  float hours_v;    // n_neg_v * 1.44 / 3600, rounded to float32 on the host
  float target, ratio;  // ratio <= 0: no dynamic adjustment
  float* sched;
  int64_t sched_len, next_step;
  float* out;       // [8]
};
__global__ void __launch_bounds__(256) kv_finish_kernel(EvalFinish f) {
  const float cur = f.sched ? f.sched[2 * max(int64_t(0), min(f.next_step - 1, f.sched_len - 1)) + 1] : 1.f;
  float fph = 0.f, rec = 0.f, nw = cur;
  if (f.cv) {
    fph = f.cv[0] / f.hours_v;  // float32 division (x / 0 -> inf, 0 / 0 -> nan, as torch)
    rec = f.n_pos_v > 0.f ? f.cv[3] / f.n_pos_v : 0.f;
    if (f.ratio > 0.f) nw = fph > f.target ? cur * f.ratio : fmaxf(1.f, cur / f.ratio);
  }
  if (threadIdx.x == 0 && f.out) {
    f.out[0] = fph;
    f.out[1] = rec;
    if (f.ct) {
      f.out[2] = f.ct[0] / fmaxf(f.n_neg_t, 1.f);
      f.out[3] = f.n_pos_t > 0.f ? f.ct[3] / f.n_pos_t : 0.f;
      f.out[4] = (f.ct[3] + (f.n_neg_t - f.ct[1])) / fmaxf(f.n_neg_t + f.n_pos_t, 1.f);
    } else {
      f.out[2] = f.out[3] = f.out[4] = 0.f;
    }
    f.out[5] = nw;
    f.out[6] = cur;
    f.out[7] = 0.f;
  }
  if (f.cv && f.ratio > 0.f && f.sched)
    for (int64_t s = f.next_step + threadIdx.x; s < f.sched_len; s += blockDim.x) f.sched[2 * s + 1] = nw;
}

// --------------------------------------------------------- workspace ------
struct FusedWs {
  int64_t wsplit, part, pstride, hg_part, xhat[2], U, Xn, dS, dHG, rinfo[2], mask[2], maxS, total;  // float offsets
};
// the weight cache's segments (WSplit) for plan p: W_o_k (k < NG - 1), then W_hg_k (k >= 1)
WSplit make_wsplit(const hbk_mlp_plan& p) {
  const int NG = static_cast<int>(p.g.size());
  WSplit w{};
  int64_t dst = 0, q = 0;
  auto add = [&](int64_t src, int rows, int cols) {
    WSeg& g = w.s[w.n++];
    g.src = src;
    g.rows = rows;
    g.cols = cols;
    g.dst = dst;
    g.q0 = q;
    dst += 4 * int64_t(rows) * cols;
    q += int64_t(rows) * cols / 4;
  };
  for (int k = 0; k + 1 < NG; ++k) add(p.g[k].w_o, p.g[k].out, p.g[k].hid);
  for (int k = 1; k < NG; ++k) add(p.g[k].w_hg, 2 * p.g[k].hid, p.g[k].in);
  return w;
}
int64_t wsplit_halves(int NG) { return int64_t(NG - 1) * 4 * (kL * kH + kH2 * kL); }
int k1_blocks(int B) { return ((B + kRB - 1) / kRB + 7) / 8 * 8; }  // row blocks, XCD-aware
int k1_splits(int B) {  // (one round of three per CU on a 64-CU stream, KS 8, measured 92.1 vs 88.4 us per step)
  static const int forced = getenv("HBK_K1_KS") ? atoi(getenv("HBK_K1_KS")) : 0;  // (A/B: 4 6 8 12 16 24)
  if (forced == 4 || forced == 6 || forced == 8 || forced == 12 || forced == 16 || forced == 24) return forced;
  static const int ks_opts[] = {4, 6, 8, 12, 16, 24};
  for (int ks : ks_opts)
    if (k1_blocks(B) * ks >= 256) return ks;
  return 24;
}
// k3's batch splits: rows per split by the stream's width (see kK3Steps)
int k3_rows(const void* stream) {
  static const bool k3_wide = getenv("HBK_K3_WIDE") != nullptr;
  const bool narrow = !k3_wide && persistent_blocks(1, stream) <= kK3NarrowCUs;
  return 32 * (narrow ? kK3StepsNarrow * kK3GroupNarrow : kK3Steps);
}
FusedWs fused_layout(int64_t B, int NG, int64_t n_params = 0) {
  FusedWs w;
  int64_t o = 0;
  auto take = [&](int64_t n) { const int64_t r = o; o += (n + 63) & ~int64_t(63); return r; };
  const int64_t Bp = (B + kR - 1) / kR * kR;
  w.wsplit = take(wsplit_halves(NG) / 2);  // first: its offset does not depend on B
  // k3's partial slabs (the most splits either width takes), at a fixed offset too
  w.pstride = (n_params + 63) & ~int64_t(63);
  w.part = take(w.pstride * ((Bp + 32 * std::min(kK3StepsNarrow, kK3Steps) - 1) /
                             (32 * std::min(kK3StepsNarrow, kK3Steps))));
  w.hg_part = take(int64_t(24) * B * kH2);
  w.xhat[0] = take(Bp * kD);
  w.xhat[1] = take(Bp * kD);
  w.U = take(int64_t(NG) * Bp * kH);
  w.Xn = take(int64_t(NG) * Bp * kL);
  w.dS = take(int64_t(NG) * Bp * kL);
  w.dHG = take(int64_t(NG) * Bp * kH2);
  w.rinfo[0] = take(Bp * 4);
  w.rinfo[1] = take(Bp * 4);
  w.mask[0] = take(Bp * kMaskW);
  w.mask[1] = take(Bp * kMaskW);
  w.maxS = take(int64_t(2) * NG * (Bp / kR) * 4);
  w.total = o;
  return w;
}

// HBK_STEP=2: the v2 step (k1s -> k1c / k3s from the pool rows); 1: the k1a -> xhat^T ->
// k1b / k3 path. By default the faster one as measured for the batch (tools/ab_step.sh, 64
// CUs, r06: B = 1,100 v2 83.2 / v1 87.3 us; 550 65.1 / 63.5; 273 59.8 / 56.7; 138 57.2 /
// 51.4 -- k3s's fixed prologue and its 2 splits at ceil(Bp / 128) slabs cost it the small
// batches): v2 from kStepV2MinB rows (HBK_STEP_V2_MIN_B), on a stream of at most
// kStepV2MaxCUs CUs -- on the whole GPU v1 is faster (B = 1,100: 59.1 against 66.1 us; its
// 288-row splits and 32-column tiles spread over 256 CUs, where k3s's 256-column tiles and
// fixed prologue do not)
constexpr int kStepV2MinB = 800, kStepV2MaxCUs = 128;
bool step_v2(int64_t B, const void* stream) {
  static const int forced = getenv("HBK_STEP") ? atoi(getenv("HBK_STEP")) : 0;
  static const int min_b = getenv("HBK_STEP_V2_MIN_B") ? atoi(getenv("HBK_STEP_V2_MIN_B")) : kStepV2MinB;
  if (forced) return forced == 2;
  return B >= min_b && persistent_blocks(1, stream) <= kStepV2MaxCUs;
}
int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}
// k1c's geometry: K chunk KC (KS = 1536 / KC chunks) and row tiles RT per block, by a
// per-CU byte model: the block's pool rows (~2.2 B per element at the training mix),
// its W slice and its partial slab, times the rounds of blocks per CU, plus the KS
// slabs each k2 row tile sums first (HBK_K1_KC / HBK_K1_RT override)
struct K1cGeom {
  int KC, RT, KS, blocks;
};
int k1c_rtmax(int KC) {
  switch (KC) {
    case 64: return k1c_rt_max<64>();
    case 96: return k1c_rt_max<96>();
    case 192: return k1c_rt_max<192>();
    default: return k1c_rt_max<384>();
  }
}
K1cGeom k1c_geom(int B, const void* stream) {
  const int cus = static_cast<int>(std::max<int64_t>(1, persistent_blocks(1, stream)));
  const int fkc = env_int("HBK_K1_KC", 0), frt = env_int("HBK_K1_RT", 0);
  K1cGeom best{192, 9, 8, 0};
  double best_cost = 1e30;
  for (int KC : {64, 96, 192, 384}) {
    if (fkc && KC != fkc) continue;
    const int rtm = k1c_rtmax(KC);
    const double lds = 16.0 * rtm * (KC + 16) * 4 + 8.0 * KC;
    const int per_cu = std::max(1, std::min(2, static_cast<int>(160.0 * 1024 / lds)));
    for (int RT = 1; RT <= rtm; ++RT) {
      if (frt && RT != std::min(frt, rtm)) continue;
      const int KS = kD / KC, nrb = (B + 16 * RT - 1) / (16 * RT), blocks = nrb * KS;
      const int rounds = (blocks + cus * per_cu - 1) / (cus * per_cu);
      const int on_cu = std::min(per_cu, (blocks + cus - 1) / cus);
      const double rows = std::min(16 * RT, B);
      const double per_wg = rows * KC * 2.2 + 128.0 * KC * 4 + rows * 128 * 4;
      const double cost = per_wg * on_cu * rounds + KS * 16.0 * 128 * 4;
      if (cost < best_cost) {
        best_cost = cost;
        best = K1cGeom{KC, RT, KS, blocks};
      }
    }
  }
  return best;
}
// k3s's batch splits: the input layer's job (12 of the launch's tiles and the bulk of its
// FLOPs) gets S0 splits of NST0 32-row steps, the small generic jobs S1 <= S0 of NST1, so
// that the launch fits the CUs in one round and its longest workgroup (steps x the job's
// relative step cost: the generic tiles have 4 or 6 of 8 column tiles live) is shortest.
// The step counts are compile-time (fully unrolled steps), one of kK3sPairs; at most
// ceil(Bp / 128) splits (the workspace's slabs). HBK_K3_R forces one pair by its rows.
constexpr int kK3sPairs[][2] = {{1, 1}, {2, 2}, {3, 3}, {3, 5}, {4, 4}, {4, 9}, {4, 12}, {5, 12},
                                {6, 14}, {7, 16}, {8, 8}, {9, 16}, {12, 12}, {16, 16}};
constexpr int kK3sNPairs = sizeof(kK3sPairs) / sizeof(kK3sPairs[0]);
constexpr int k3s_occ(int) { return 2; }  // (two workgroups per CU measured no faster: the
                                          // CU's load rate binds, r06)
struct K3sPlan {
  int S0, S1, pair;
};
// per-workgroup time model (units of ~0.78 us, the generic jobs' 32-row step of r06, fitted
// to the traced spans): the input layer's 3 + 1.6 x steps, a generic job's 2.5 + 0.65 x steps
K3sPlan k3s_plan(int64_t Bp, int tiles0, int tiles1, const void* stream) {
  const int cus = static_cast<int>(std::max<int64_t>(1, persistent_blocks(1, stream)));
  const int64_t max_s = (Bp + 127) / 128;
  const int fr = env_int("HBK_K3_R", 0), fq = env_int("HBK_K3_PAIR", -1);
  auto splits = [&](int st) { return static_cast<int>((Bp + 32 * st - 1) / (32 * st)); };
  K3sPlan best{splits(16), splits(16), kK3sNPairs - 1};
  double best_cost = 1e30;
  for (int q = 0; q < kK3sNPairs; ++q) {
    const int st0 = kK3sPairs[q][0], st1 = kK3sPairs[q][1];
    if (fr > 0 && 32 * st0 < fr) continue;
    if (fq >= 0 && q != fq) continue;
    const int s0 = splits(st0), s1 = splits(st1);
    if (s0 > max_s && st0 < 16) continue;  // (the workspace's slabs)
    const int wgs = tiles0 * s0 + tiles1 * s1, rounds = (wgs + cus - 1) / cus;
    const double cost = rounds * std::max(3.0 + 1.6 * st0, 2.5 + 0.65 * st1) + 1e-3 * wgs;
    if (cost < best_cost) {
      best_cost = cost;
      best = K3sPlan{s0, s1, q};
    }
    if (fr > 0) break;
  }
  return best;
}
template <int Q = 0>
void launch_k3s(int q, dim3 grid, hipStream_t s, const K3sArgs& k3) {
  if constexpr (Q < kK3sNPairs) {
    if (q == Q)
      hipLaunchKernelGGL((k3s_kernel<kK3sPairs[Q][0], kK3sPairs[Q][1], k3s_occ(Q)>), grid, dim3(kK3sThr), 0, s, k3);
    else
      launch_k3s<Q + 1>(q, grid, s, k3);
  }
}

void fill_k2(const hbk_mlp_plan& p, K2Args& k) {
  const int NG = static_cast<int>(p.g.size());
  k.NG = NG;
  for (int i = 0; i < NG; ++i) {
    k.w_hg[i] = p.g[i].w_hg;
    k.b_hg[i] = p.g[i].b_hg;
    k.w_o[i] = p.g[i].w_o;
    k.b_o[i] = p.g[i].b_o;
  }
  for (int i = 0; i + 1 < NG; ++i) {
    k.ln_g[i] = p.ln[i].g;
    k.ln_b[i] = p.ln[i].b;
  }
}

// the weight cache's plane offsets as k2 reads them
void set_k2_cache(const WSplit& wsp, int NG, const _Float16* wc, K2Args& k2) {
  k2.wc = wc;
  for (int k = 0; k < NG; ++k) k2.c_o[k] = k2.c_oT[k] = k2.c_hg[k] = k2.c_hgT[k] = 0;
  for (int sg = 0; sg < wsp.n; ++sg) {
    const WSeg& g = wsp.s[sg];
    const int64_t rc = int64_t(g.rows) * g.cols;
    const bool is_o = sg < NG - 1;
    const int k = is_o ? sg : sg - (NG - 1) + 1;
    (is_o ? k2.c_o : k2.c_hg)[k] = g.dst;
    (is_o ? k2.c_oT : k2.c_hgT)[k] = g.dst + 2 * rc;
  }
}

// k3's covered parameter ranges: norm_in gamma / beta, every W_hg and W_o
Ranges make_ranges(const hbk_mlp_plan& p) {
  Ranges r{};
  auto add = [&](int64_t lo, int64_t n) {
    r.lo[r.n] = lo;
    r.hi[r.n++] = lo + n;
  };
  add(p.ln_in.g, p.ln_in.d);
  add(p.ln_in.b, p.ln_in.d);
  for (const Gmlp& g : p.g) {
    add(g.w_hg, int64_t(2) * g.hid * g.in);
    add(g.w_o, int64_t(g.out) * g.hid);
  }
  return r;
}

// evaluation workspace: the weight cache (as the fused layout's first region),
// W' planes, c0, c1
struct EvalWs {
  int64_t wsplit, wq, c0, c1, total;  // float offsets
};
EvalWs eval_layout(int NG) {
  EvalWs w;
  int64_t o = 0;
  auto take = [&](int64_t n) { const int64_t r = o; o += (n + 63) & ~int64_t(63); return r; };
  w.wsplit = take(wsplit_halves(NG) / 2);
  w.wq = take(int64_t(kH2) * kD);  // 2 planes of halves
  w.c0 = take(kH2);
  w.c1 = take(kH2);
  w.total = o;
  return w;
}

}  // namespace

bool mlp_fused_supported(const hbk_mlp_plan& p) {
  return p.d_in == kD && p.layer == kL && p.hid == kH && static_cast<int>(p.g.size()) <= kMaxG &&
         p.g.size() >= 2;
}

int64_t mlp_fused_ws_floats(const hbk_mlp_plan& p, int64_t B) {
  return fused_layout(std::max<int64_t>(B, 1), static_cast<int>(p.g.size()), p.n_params).total;
}

// k1 + k2 (+ k3): the forward (inference) or forward/backward half of a step.
#ifdef HBK_BOUNDS
void bounds_set(std::initializer_list<std::pair<const void*, int64_t>> rs) {
  unsigned long long h[kBMax][2] = {};
  int n = 0;
  for (const auto& r : rs)
    if (r.first && r.second > 0 && n < kBMax) {
      h[n][0] = reinterpret_cast<unsigned long long>(r.first);
      h[n][1] = h[n][0] + static_cast<unsigned long long>(r.second);
      ++n;
    }
  (void)hipDeviceSynchronize();
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_brange), h, sizeof(h));
  (void)hipMemcpyToSymbol(HIP_SYMBOL(g_bn), &n, sizeof(n));
}
#endif
int mlp_fused_run(const hbk_mlp_plan& p, const float* params, const float* pool32, int64_t n32,
                  const void* pool16, int64_t n16, const int32_t* idx, int64_t idx_stride, int64_t idx_steps,
                  const float* y, int64_t y_stride, int B, const float* state, int parity, const float* sched,
                  int sched_len, float neg_weight, float thr, float act_thr, float drop_p, uint64_t seed,
                  float* bucket, float* prob, float* logit, float* ws, bool train, int flags, hipStream_t s) {
  const int NG = static_cast<int>(p.g.size());
  const FusedWs w = fused_layout(B, NG, p.n_params);
#ifdef HBK_BOUNDS
  bounds_set({{params, p.n_params * 4},
              {pool32, n32 * kD * 4},
              {pool16, n16 * kD * 2},
              {idx, (std::max<int64_t>(idx_steps, 1) * idx_stride + B) * 4},
              {y, (std::max<int64_t>(idx_steps, 1) * y_stride + B) * 4},
              {state, 64},
              {sched, int64_t(sched_len) * 8},
              {bucket, (p.n_params + kStats) * 4},
              {prob, int64_t(B) * 4},
              {logit, int64_t(B) * 4},
              {ws, w.total * 4}});
#endif

  const int64_t Bp = (B + kR - 1) / kR * kR;
  const int rt = (B + kR - 1) / kR;
  K1aArgs ka;
  ka.pool32 = pool32;
  ka.pool16 = static_cast<const _Float16*>(pool16);
  ka.n32 = pool32 ? n32 : 0;
  ka.n16 = pool16 ? n16 : 0;
  ka.idx = idx;
  ka.idx_stride = idx_stride;
  ka.idx_steps = idx ? idx_steps : 0;
  ka.state = state;
  ka.parity = parity;
  ka.B = B;
  ka.drop_p = drop_p;
  ka.seed = seed;
  ka.xhat[0] = ws + w.xhat[0];
  ka.xhat[1] = ws + w.xhat[1];
  ka.Bp = Bp;
  for (int i = 0; i < 2; ++i) {
    ka.rinfo[i] = reinterpret_cast<uint4*>(ws + w.rinfo[i]);
    ka.mask[i] = reinterpret_cast<uint32_t*>(ws + w.mask[i]);
  }
  const bool v2 = step_v2(B, s);
  const float keep = drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f;
  const float* xhat = ws + w.xhat[parity];
  const WSplit wsp = make_wsplit(p);
  _Float16* wc = reinterpret_cast<_Float16*>(ws + w.wsplit);
  if (!(flags & HBK_STEP_WEIGHTS_READY)) {  // the previous step's k4 did not leave the cache current
    const int64_t n4 = wsplit_halves(NG) / 16;  // float4s of the segments
    hipLaunchKernelGGL(k0_wsplit_kernel, dim3(unsigned(std::min<int64_t>((n4 + 255) / 256, 256))), dim3(256), 0,
                       s, wsp, params, wc, n4);
    HBK_LAUNCH_CHECK("k0_wsplit_kernel");
  }
  if (!(flags & HBK_STEP_XHAT_READY)) {  // this step's rows were not prefetched by the previous step
    if (v2) {
      if (idx)
        hipLaunchKernelGGL(k1s_kernel<true>, dim3(rt), dim3(256), 0, s, ka, 0);
      else
        hipLaunchKernelGGL(k1s_kernel<false>, dim3(rt), dim3(256), 0, s, ka, 0);
      HBK_LAUNCH_CHECK("k1s_kernel");
    } else {
      if (idx)
        hipLaunchKernelGGL(k1a_kernel<true>, dim3(rt), dim3(256), 0, s, ka, 0);
      else
        hipLaunchKernelGGL(k1a_kernel<false>, dim3(rt), dim3(256), 0, s, ka, 0);
      HBK_LAUNCH_CHECK("k1a_kernel");
    }
  }
  int KS = k1_splits(B);
  if (v2) {
    const K1cGeom g1 = k1c_geom(B, s);
    KS = g1.KS;
    K1cArgs kc;
    kc.P = params;
    kc.g_in = p.ln_in.g;
    kc.b_in = p.ln_in.b;
    kc.w0 = p.g[0].w_hg;
    kc.B = B;
    kc.RT = g1.RT;
    kc.KS = g1.KS;
    kc.pool32 = pool32;
    kc.pool16 = static_cast<const _Float16*>(pool16);
    kc.rinfo = ka.rinfo[parity];
    kc.mask = ka.mask[parity];
    kc.keep = keep;
    kc.hg_part = ws + w.hg_part;
    kc.stats = train ? bucket + p.n_params : nullptr;
    auto launch = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(g1.blocks), dim3(512), 0, s, kc); };
    switch (g1.KC) {
      case 64: launch(k1c_kernel<64>); break;
      case 96: launch(k1c_kernel<96>); break;
      case 192: launch(k1c_kernel<192>); break;
      default: launch(k1c_kernel<384>);
    }
    HBK_LAUNCH_CHECK("k1c_kernel");
  } else {
  K1bArgs kb;
  kb.P = params;
  kb.g_in = p.ln_in.g;
  kb.b_in = p.ln_in.b;
  kb.w0 = p.g[0].w_hg;
  kb.B = B;
  kb.xhat = xhat;
  kb.Bp = Bp;
  kb.hg_part = ws + w.hg_part;
  kb.stats = train ? bucket + p.n_params : nullptr;
  {
    auto launch = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(k1_blocks(B) * KS), dim3(256), 0, s, kb); };
    switch (KS) {
      case 4: launch(k1b_kernel<4>); break;
      case 6: launch(k1b_kernel<6>); break;
      case 8: launch(k1b_kernel<8>); break;
      case 12: launch(k1b_kernel<12>); break;
      case 16: launch(k1b_kernel<16>); break;
      default: launch(k1b_kernel<24>);
    }
    HBK_LAUNCH_CHECK("k1b_kernel");
  }
  }
  K2Args k2;
  k2.P = params;
  k2.B = B;
  k2.KS = KS;
  fill_k2(p, k2);
  k2.hg_part = ws + w.hg_part;
  k2.y = y;
  k2.y_stride = y_stride;
  k2.state = state;
  k2.parity = parity;
  k2.sched = sched;
  k2.sched_len = sched_len;
  k2.neg_weight = neg_weight;
  k2.thr = thr;
  k2.act_thr = act_thr;
  k2.prob = prob;
  k2.logit = logit;
  k2.counts = nullptr;
  k2.count_label = 0;
  k2.G = bucket;
  k2.stats = bucket ? bucket + p.n_params : nullptr;
  k2.U = ws + w.U;
  k2.Xn = ws + w.Xn;
  k2.dS = ws + w.dS;
  k2.dHG = ws + w.dHG;
  k2.Bp = Bp;
  k2.n_rt = rt;
  k2.prefetch = train && idx && (flags & HBK_STEP_PREFETCH_NEXT);
  k2.pre = ka;
  k2.v2 = v2 ? 1 : 0;
  k2.maxS = v2 && train ? ws + w.maxS : nullptr;
  set_k2_cache(wsp, NG, wc, k2);
  {
    k2.pre_tiles = std::max(1, env_int("HBK_PRE_TILES", kPreTiles2));
    const int pt = v2 ? k2.pre_tiles : kPreTiles;
    const int grid = k2.prefetch ? rt + (rt + pt - 1) / pt : rt;
    auto launch = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, s, k2); };
    if (train) {
      if (NG == 2) launch(k2_rows_kernel<true, 2>);
      else if (NG == 3) launch(k2_rows_kernel<true, 3>);
      else launch(k2_rows_kernel<true, 4>);
    } else {
      if (NG == 2) launch(k2_rows_kernel<false, 2>);
      else if (NG == 3) launch(k2_rows_kernel<false, 3>);
      else launch(k2_rows_kernel<false, 4>);
    }
    HBK_LAUNCH_CHECK("k2_rows_kernel");
  }
  if (!train) return HBK_OK;
  if (v2) {  // k3s: job 0 = input layer (pool rows), then dW_hg of GMLPs 1.., then dW_o of every GMLP
    constexpr int kNtRaw = 16 * kK3sNbtRaw, kNtGen = 16 * kK3sNbtGen;
    K3sArgs k3;
    int nj = 0, tiles = 0;
    auto add = [&](const float* X, const float* Y, int64_t c_off, int ldc, int M, int N, int mat) {
      K3sJob& j = k3.job[nj];
      j.X = X;
      j.Y = Y;
      j.c_off = c_off;
      j.ldc = ldc;
      j.M = M;
      j.N = N;
      const int nt = Y ? kNtGen : kNtRaw;
      j.tn = (N + nt - 1) / nt;
      j.mat = mat;
      k3.start[nj] = ((M + 127) / 128) * j.tn;  // (tiles; scaled by the job's splits below)
      tiles += k3.start[nj];
      ++nj;
    };
    add(ws + w.dHG, nullptr, p.g[0].w_hg, kD, kH2, kD, 0);
    for (int k = 1; k < NG; ++k)
      add(ws + w.dHG + int64_t(k) * kH2 * Bp, ws + w.Xn + int64_t(k) * kL * Bp, p.g[k].w_hg, kL, kH2, kL, k);
    for (int k = 0; k < NG; ++k)
      add(ws + w.dS + int64_t(k) * kL * Bp, ws + w.U + int64_t(k) * kH * Bp, p.g[k].w_o, kH, p.g[k].out, kH, NG + k);
    const K3sPlan pl = k3s_plan(Bp, k3.start[0], tiles - k3.start[0], s);
    const int S = pl.S0;
    if (getenv("HBK_PLAN_LOG")) {  // (tuning aid) the plan of each distinct batch, once
      static int64_t logged = -1;
      if (logged != Bp) {
        logged = Bp;
        fprintf(stderr, "hbk k3s plan: Bp %lld, CUs %lld, S0 %d x %d steps, S1 %d x %d steps\n",
                static_cast<long long>(Bp), static_cast<long long>(persistent_blocks(1, s)), pl.S0,
                kK3sPairs[pl.pair][0], pl.S1, kK3sPairs[pl.pair][1]);
      }
    }
    int wgs = 0;
    for (int i = 0; i < nj; ++i) {
      k3.job[i].S = i == 0 ? pl.S0 : pl.S1;
      k3.job[i].R = 32 * kK3sPairs[pl.pair][i == 0 ? 0 : 1];
      const int t = k3.start[i];
      k3.start[i] = wgs;
      wgs += t * k3.job[i].S;
    }
    k3.start[nj] = wgs;
    k3.n_jobs = nj;
    k3.S = S;
    k3.n_rt = rt;
    k3.B = B;
    k3.Bp = Bp;
    k3.maxS = ws + w.maxS;
    k3.pool32 = pool32;
    k3.pool16 = static_cast<const _Float16*>(pool16);
    k3.rinfo = ka.rinfo[parity];
    k3.mask = ka.mask[parity];
    k3.keep = keep;
    k3.g_in = params + p.ln_in.g;
    k3.b_in = params + p.ln_in.b;
    k3.W0 = params + p.g[0].w_hg;
    k3.g_off = p.ln_in.g;
    k3.b_off = p.ln_in.b;
    k3.part = ws + w.part;
    k3.pstride = w.pstride;
    launch_k3s(pl.pair, dim3(wgs), s, k3);
    HBK_LAUNCH_CHECK("k3s_kernel");
    if (flags & HBK_STEP_DEFER_PARTIALS) {
      p.deferred_ws = ws;
      p.deferred_ks = S;
    } else {
      p.deferred_ws = nullptr;
      hipLaunchKernelGGL(k3_fold_kernel, dim3(unsigned(std::min<int64_t>((p.n_params / 4 + 255) / 256, 1024))), dim3(256),
                         0, s, make_ranges(p), ws + w.part, w.pstride, S, bucket, p.n_params);
      HBK_LAUNCH_CHECK("k3_fold_kernel");
    }
    return HBK_OK;
  }
  // k3: job 0 = input layer, then dW_hg of GMLPs 1.., then dW_o of every GMLP
  K3Args k3;
  int nj = 0, blocks = 0;
  // HBK_K3_WIDE=1: the 288-row splits on narrow streams too (4 instead of 9
  // splits at B = 1100: fewer partial slabs, more time on a small partition)
  const int rows3 = k3_rows(s);
  const bool narrow = rows3 == 32 * kK3StepsNarrow * kK3GroupNarrow;
  const int KS3 = static_cast<int>((Bp + rows3 - 1) / rows3);
  auto add = [&](const float* X, const float* Y, int64_t c_off, int ldc, int M, int N) {
    WJob& j = k3.job[nj];
    j.X = X;
    j.Y = Y;
    j.c_off = c_off;
    j.ldc = ldc;
    j.M = M;
    j.N = N;
    j.tn = (N + kTN - 1) / kTN;
    k3.start[nj] = blocks;
    blocks += ((M + kTM - 1) / kTM) * j.tn * KS3;
    ++nj;
  };
  add(ws + w.dHG, xhat, p.g[0].w_hg, kD, kH2, kD);
  for (int k = 1; k < NG; ++k)
    add(ws + w.dHG + int64_t(k) * kH2 * Bp, ws + w.Xn + int64_t(k) * kL * Bp, p.g[k].w_hg, kL, kH2, kL);
  for (int k = 0; k < NG; ++k)
    add(ws + w.dS + int64_t(k) * kL * Bp, ws + w.U + int64_t(k) * kH * Bp, p.g[k].w_o, kH, p.g[k].out, kH);
  k3.start[nj] = blocks;
  k3.n_jobs = nj;
  k3.KS = KS3;
  k3.Bp = Bp;
  k3.g_in = params + p.ln_in.g;
  k3.b_in = params + p.ln_in.b;
  k3.W0 = params + p.g[0].w_hg;
  k3.g_off = p.ln_in.g;
  k3.b_off = p.ln_in.b;
  k3.part = ws + w.part;
  k3.pstride = w.pstride;
  if (narrow)
    hipLaunchKernelGGL((k3_wgrad_kernel<kK3StepsNarrow, kK3GroupNarrow>), dim3(blocks), dim3(256), 0, s, k3);
  else
    hipLaunchKernelGGL((k3_wgrad_kernel<kK3Steps, 1>), dim3(blocks), dim3(256), 0, s, k3);
  HBK_LAUNCH_CHECK("k3_wgrad_kernel");
  if (flags & HBK_STEP_DEFER_PARTIALS) {  // the update adds the slabs
    p.deferred_ws = ws;
    p.deferred_ks = KS3;
  } else {
    p.deferred_ws = nullptr;
    hipLaunchKernelGGL(k3_fold_kernel, dim3(unsigned(std::min<int64_t>((p.n_params / 4 + 255) / 256, 1024))), dim3(256),
                       0, s, make_ranges(p), ws + w.part, w.pstride, KS3, bucket, p.n_params);
    HBK_LAUNCH_CHECK("k3_fold_kernel");
  }
  return HBK_OK;
}

int mlp_fused_update(const hbk_mlp_plan& p, float* params, float* bucket, float* m, float* v, float* state,
                     int parity, const float* sched, int sched_len, float lr, float b1, float b2, float eps,
                     float* hist, int hist_cap, float* ws, hipStream_t s) {
  if (p.deferred_ws && p.deferred_ws != ws) {
    set_error("hbk: the previous hbk_mlp_step_fwd_bwd deferred its weight-gradient partials to its workspace: "
              "pass that workspace to hbk_mlp_step_update");
    return HBK_ERR_ARG;
  }
  K4Args k;
  k.w = make_wsplit(p);
  const FusedWs fl = fused_layout(1, static_cast<int>(p.g.size()), p.n_params);
  k.wc = ws ? reinterpret_cast<_Float16*>(ws + fl.wsplit) : nullptr;
  k.part = p.deferred_ws ? ws + fl.part : nullptr;
  k.pstride = fl.pstride;
  k.ns = p.deferred_ws ? p.deferred_ks : 0;
  if (p.n_params >= (int64_t(1) << 31) - 4) {
    set_error("hbk: hbk_mlp_step_update: parameter count >= 2^31");
    return HBK_ERR_ARG;
  }
  const Ranges rg = make_ranges(p);
  k.n_cov = rg.n;
  for (int i = 0; i < kMaxRng; ++i) {
    k.cov_lo[i] = i < rg.n ? static_cast<int32_t>(rg.lo[i]) : 0;
    k.cov_hi[i] = i < rg.n ? static_cast<int32_t>(rg.hi[i]) : 0;
  }
  k.n_skip = k.w.n;
  for (int sg = 0; sg < kMaxSeg; ++sg) {  // 4 i in [src, src + rows cols) <=> i in [ceil(src / 4), ceil(end / 4))
    const int64_t lo = sg < k.w.n ? k.w.s[sg].src : 0, hi = sg < k.w.n ? lo + int64_t(k.w.s[sg].rows) * k.w.s[sg].cols : 0;
    k.skip_lo[sg] = static_cast<int32_t>((lo + 3) / 4);
    k.skip_hi[sg] = static_cast<int32_t>((hi + 3) / 4);
  }
  p.deferred_ws = nullptr;
  k.n_tiles = 0;
  for (int sg = 0; sg < k.w.n; ++sg)
    for (int r0 = 0; r0 < k.w.s[sg].rows && k.n_tiles < kMaxTiles; r0 += kTileR) {
      k.tile_seg[k.n_tiles] = sg;
      k.tile_r0[k.n_tiles++] = r0;
    }
  k.P = params;
  k.G = bucket;
  k.m = m;
  k.v = v;
  k.n = p.n_params;
  k.state = state;
  k.parity = parity;
  k.sched = sched;
  k.sched_len = sched_len;
  k.lr = lr;
  k.b1 = b1;
  k.b2 = b2;
  k.eps = eps;
  k.hist = hist;
  k.hist_cap = hist_cap;
  const int64_t blocks = (k.wc ? k.n_tiles : 0) + std::min<int64_t>((p.n_params / 4 + 255) / 256, 1024);
  hipLaunchKernelGGL(k4_update_kernel, dim3(unsigned(blocks)), dim3(256), 0, s, k);
  HBK_LAUNCH_CHECK("k4_update_kernel");
  return HBK_OK;
}

int64_t mlp_eval_ws_floats(const hbk_mlp_plan& p, int64_t rows) {
  (void)rows;  // the passes need no per-row workspace
  return eval_layout(static_cast<int>(p.g.size())).total;
}

int mlp_eval_prepare(const hbk_mlp_plan& p, const float* params, float* ws, hipStream_t s) {
  const int NG = static_cast<int>(p.g.size());
  const EvalWs w = eval_layout(NG);
  const WSplit wsp = make_wsplit(p);
  const int64_t n4 = wsplit_halves(NG) / 16;
  hipLaunchKernelGGL(k0_wsplit_kernel, dim3(unsigned(std::min<int64_t>((n4 + 255) / 256, 256))), dim3(256), 0, s,
                     wsp, params, reinterpret_cast<_Float16*>(ws + w.wsplit), n4);
  HBK_LAUNCH_CHECK("k0_wsplit_kernel");
  hipLaunchKernelGGL(kv_prep_kernel, dim3(kH2), dim3(256), 0, s, params, p.g[0].w_hg, p.ln_in.g, p.ln_in.b,
                     reinterpret_cast<_Float16*>(ws + w.wq), ws + w.c0, ws + w.c1);
  HBK_LAUNCH_CHECK("kv_prep_kernel");
  return HBK_OK;
}

// One kv_gemm_kernel launch over nseg pools of one dtype (nseg = 1: the single-pool fields,
// which also allow idx / prob; nseg > 1: the segment table, workgroups in pool order).
static int mlp_eval_launch(const hbk_mlp_plan& p, const float* params, bool f16, const EvalSeg* seg, int nseg,
                           const int32_t* idx, float act_thr, float drop_p, float* prob, float* ws, hipStream_t s) {
  const int NG = static_cast<int>(p.g.size());
  const EvalWs w = eval_layout(NG);
  const WSplit wsp = make_wsplit(p);
  K2Args kc{};  // the weight cache's plane offsets as k2 reads them
  set_k2_cache(wsp, NG, reinterpret_cast<const _Float16*>(ws + w.wsplit), kc);
  KvArgs ka{};
  ka.pool = seg[0].pool;
  ka.n_pool = seg[0].n_pool;
  ka.idx = idx;
  ka.rows = seg[0].rows;
  ka.r0 = seg[0].r0;
  ka.wq = reinterpret_cast<const _Float16*>(ws + w.wq);
  ka.c0 = ws + w.c0;
  ka.c1 = ws + w.c1;
  ka.drop_p = drop_p;
  ka.seed = seg[0].seed;
  ka.P = params;
  for (int i = 0; i < kMaxG; ++i) {
    const int g = std::min(i, NG - 1);
    ka.b_hg[i] = p.g[g].b_hg;
    ka.b_o[i] = p.g[g].b_o;
    ka.w_o[i] = p.g[g].w_o;
    ka.ln_g[i] = i + 1 < NG ? p.ln[i].g : 0;
    ka.ln_b[i] = i + 1 < NG ? p.ln[i].b : 0;
    ka.c_o[i] = kc.c_o[i];
    ka.c_hg[i] = kc.c_hg[i];
  }
  ka.wc = kc.wc;
  ka.act_thr = act_thr;
  ka.counts = seg[0].counts;
  ka.label = seg[0].label;
  ka.prob = prob;
  // f16 rows: 16 waves of one 16-row tile each (126 VGPRs); f32 rows (the split's registers
  // spill at 128): 8 waves. HBK_KV_WAVES=8: 8 waves of two tiles for f16 rows too (A/B)
  static const bool w8 = getenv("HBK_KV_WAVES") && atoi(getenv("HBK_KV_WAVES")) == 8;
  const int waves = f16 && !w8 ? 16 : 8;
  const int tile = (f16 ? 256 : 128);  // kv_gemm_kernel's rows per workgroup
  int64_t tiles = (seg[0].rows + tile - 1) / tile;
  ka.nseg = 0;
  if (nseg > 1) {
    ka.nseg = nseg;
    tiles = 0;
    for (int i = 0; i < nseg; ++i) {
      ka.seg_tile0[i] = static_cast<int>(tiles);
      ka.seg_pool[i] = seg[i].pool;
      ka.seg_npool[i] = seg[i].n_pool;
      ka.seg_rows[i] = seg[i].rows;
      ka.seg_r0[i] = seg[i].r0;
      ka.seg_seed[i] = seg[i].seed;
      ka.seg_counts[i] = seg[i].counts;
      ka.seg_label[i] = seg[i].label;
      tiles += (seg[i].rows + tile - 1) / tile;
    }
    ka.seg_tile0[nseg] = static_cast<int>(tiles);
  }
  const dim3 grid(static_cast<unsigned>(tiles));
  auto launch = [&](auto kern) { hipLaunchKernelGGL(kern, grid, dim3(64 * waves), 0, s, ka); };
  if (waves == 16) {
    if (NG == 2) launch(kv_gemm_kernel<true, 2, 16>);
    else if (NG == 3) launch(kv_gemm_kernel<true, 3, 16>);
    else launch(kv_gemm_kernel<true, 4, 16>);
  } else if (f16) {
    if (NG == 2) launch(kv_gemm_kernel<true, 2, 8>);
    else if (NG == 3) launch(kv_gemm_kernel<true, 3, 8>);
    else launch(kv_gemm_kernel<true, 4, 8>);
  } else {
    if (NG == 2) launch(kv_gemm_kernel<false, 2, 8>);
    else if (NG == 3) launch(kv_gemm_kernel<false, 3, 8>);
    else launch(kv_gemm_kernel<false, 4, 8>);
  }
  HBK_LAUNCH_CHECK("kv_gemm_kernel");
  return HBK_OK;
}

int mlp_eval_count(const hbk_mlp_plan& p, const float* params, const void* pool, bool f16, int64_t n_pool,
                   const int32_t* idx, int64_t rows, int64_t r0, int label, float act_thr, float drop_p,
                   uint64_t seed, float* counts, float* prob, float* ws, hipStream_t s) {
  if (rows <= 0) return HBK_OK;
  const EvalSeg seg{pool, n_pool, rows, r0, seed, counts, label};
  return mlp_eval_launch(p, params, f16, &seg, 1, idx, act_thr, drop_p, prob, ws, s);
}

int mlp_eval_count_multi(const hbk_mlp_plan& p, const float* params, bool f16, const EvalSeg* seg, int nseg,
                         float act_thr, float drop_p, float* ws, hipStream_t s) {
  EvalSeg live[kKvMaxSeg];
  int n = 0;
  for (int i = 0; i < nseg; ++i)
    if (seg[i].rows > 0) live[n++] = seg[i];
  if (n == 0) return HBK_OK;
  return mlp_eval_launch(p, params, f16, live, n, nullptr, act_thr, drop_p, nullptr, ws, s);
}

int mlp_eval_finish(const float* cv, const float* ct, const double* sizes, float target, float ratio, float* sched,
                    int64_t sched_len, int64_t next_step, float* out, hipStream_t s) {
  EvalFinish f;
  f.cv = cv;
  f.ct = ct;
  f.n_neg_v = static_cast<float>(sizes[0]);
  f.n_pos_v = static_cast<float>(sizes[1]);
  f.n_neg_t = static_cast<float>(sizes[2]);
  f.n_pos_t = static_cast<float>(sizes[3]);
  f.hours_v = static_cast<float>(sizes[0] * 1.44 / 3600.0);
  f.target = target;
  f.ratio = ratio;
  f.sched = sched;
  f.sched_len = sched_len;
  f.next_step = next_step;
  f.out = out;
  hipLaunchKernelGGL(kv_finish_kernel, dim3(1), dim3(256), 0, s, f);
  HBK_LAUNCH_CHECK("kv_finish_kernel");
  return HBK_OK;
}

}  // namespace hbk

#ifdef HBK_BOUNDS
extern "C" int hbk_debug_bounds(unsigned long long* out) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(hbk::g_berr), 4 * sizeof(unsigned long long)) != hipSuccess) return -2;
  unsigned long long z[4] = {};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(hbk::g_berr), z, sizeof(z));
  return 0;
}
#endif

#ifdef HBK_TRACE
extern "C" int hbk_debug_mlp_trace(unsigned long long* out, int* counts) {
  static_assert(sizeof(hbk::g_mlp_trace) == sizeof(unsigned long long) * 6 * 4 * 128, "probe_mlp.py's buffer");
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(hbk::g_mlp_trace), sizeof(hbk::g_mlp_trace)) != hipSuccess) return -2;
  if (hipMemcpyFromSymbol(counts, HIP_SYMBOL(hbk::g_mlp_trace_n), sizeof(hbk::g_mlp_trace_n)) != hipSuccess)
    return -2;
  int z[hbk::kTraceKerns * hbk::kTraceWaves] = {};
  (void)hipMemcpyToSymbol(HIP_SYMBOL(hbk::g_mlp_trace_n), z, sizeof(z));
  return 0;
}
// k3s's per-block spans of the last launch: [1024][3] {start, end, job << 32 | split}
extern "C" int hbk_debug_spans(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(hbk::g_span), sizeof(hbk::g_span)) == hipSuccess ? 0 : -2;
}
#endif
