// Fused wake-word classifier train step for gfx950 (default architecture:
// d_in = 16 x 96 = 1536, layer_dim 96, hidden get_normalized_dim(96) = 64, any
// number of layers up to kMaxG - 2).
//
// Replaces, per optimisation step of WakeWordTrainer.train_epoch
// (trainer.py:380-494), the reference's forward (wakeword.py:334-348), the
// high-loss filter and weighted BCE (:407-445), autograd backward and
// torch.optim.Adam (:45, :460-462), with FOUR launches and no host sync:
//
//   k1_input   gather the batch rows from the embedding pools by index (f32
//              or f16 pool), input dropout, LayerNorm(1536) -> xhat, and the
//              input GEMM HG0 = LN(x) W_hg0^T as split-K partial slabs
//              (row tiles of 16 x K-chunks: ~280 workgroups at B = 1100)
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
// All arithmetic is f32 (GEMMs on v_mfma_f32_16x16x4_f32, bitwise an fmaf
// chain); results differ from the reference only in summation order.
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
#include <cmath>

#include "hbk_common.h"
#include "hbk_mlp_internal.h"

namespace hbk {
namespace {

typedef float f4 __attribute__((ext_vector_type(4)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));

constexpr int kD = 1536, kL = 96, kH = 64, kH2 = 128;
constexpr int kR = 16;            // rows per tile = MFMA M
constexpr int kMaxG = 6;          // gated MLPs held by k2 (n_layers <= 4)
constexpr int kStats = 8;
constexpr float kLnEps = 1e-5f;
constexpr int kLd = 132;          // LDS row stride of [16][<=128] activation tiles
constexpr int kChunkMax = 384;    // k1 K-chunk

__device__ __forceinline__ f4 mma(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float wsum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float sigm(float x) { return 1.f / (1.f + expf(-x)); }

__device__ __forceinline__ int step_of(const float* state, int parity) {
  return state ? static_cast<int>(state[parity * 8 + 3]) : 0;
}

// ------------------------------------------------------------------ k1 ----
struct K1Args {
  const float* P;
  int64_t g_in, b_in, w0;
  const float* pool32;
  const _Float16* pool16;
  int64_t n32, n16;    // pool rows; an index outside its pool reads as a zero row
  const int32_t* idx;  // row r of the step's batch: >= 0 pool32 row, < 0 pool16 row -idx-1; NULL = r
  int64_t idx_stride;
  const float* state;
  int parity;
  int B, chunk;
  float drop_p;
  uint64_t seed;
  float* hg_part;  // [KS][B][128]
  float* xhat;     // [B][1536]
  float* stats;    // bucket tail, zeroed here (k2 accumulates into it); may be NULL
};

__global__ void __launch_bounds__(256) k1_input_kernel(K1Args a) {
  __shared__ __attribute__((aligned(16))) float xn[kR][kChunkMax + 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int rt = blockIdx.x, ks = blockIdx.y;
  const int k0 = ks * a.chunk;
  const int step = step_of(a.state, a.parity);
  if (a.stats && rt == 0 && ks == 0 && tid < kStats) a.stats[tid] = 0.f;
  const int32_t* idx = a.idx ? a.idx + static_cast<int64_t>(step) * a.idx_stride : nullptr;
  // per-step dropout stream: base seed + step + the epoch salt (state[4])
  const uint64_t seed = a.seed + static_cast<uint64_t>(step) +
                        (a.state ? static_cast<uint64_t>(a.state[a.parity * 8 + 4]) << 24 : 0);
  const float* g = a.P + a.g_in;
  const float* bb = a.P + a.b_in;
  const float keep = a.drop_p > 0.f ? 1.f / (1.f - a.drop_p) : 1.f;
  // LayerNorm: wave w normalises rows 4w..4w+3; lane holds elements
  // c = 4 lane + 256 u + e (u < 6, e < 4)
  for (int i = 0; i < 4; ++i) {
    const int rl = wave * 4 + i, r = rt * kR + rl;
    if (r >= a.B) {
      for (int c = lane; c < a.chunk; c += 64) xn[rl][c] = 0.f;
      continue;
    }
    const int ix = idx ? idx[r] : r;
    f4 v[6];
    if (ix >= 0 ? ix >= a.n32 : -static_cast<int64_t>(ix) - 1 >= a.n16) {
#pragma unroll
      for (int u = 0; u < 6; ++u) v[u] = f4{0.f, 0.f, 0.f, 0.f};
    } else if (ix >= 0) {
      const f4* src = reinterpret_cast<const f4*>(a.pool32 + static_cast<int64_t>(ix) * kD);
#pragma unroll
      for (int u = 0; u < 6; ++u) v[u] = src[lane + 64 * u];
    } else {
      const h4* src = reinterpret_cast<const h4*>(a.pool16 + static_cast<int64_t>(-ix - 1) * kD);
#pragma unroll
      for (int u = 0; u < 6; ++u) v[u] = __builtin_convertvector(src[lane + 64 * u], f4);
    }
    if (a.drop_p > 0.f) {  // nn.Dropout on the input (wakeword.py:197, :338)
      const uint64_t base = static_cast<uint64_t>(r) * kD;
#pragma unroll
      for (int u = 0; u < 6; ++u)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const uint64_t c = 4 * lane + 256 * u + e;
          v[u][e] = uniform01(seed, base + c) < a.drop_p ? 0.f : v[u][e] * keep;
        }
    }
    float s = 0.f;
#pragma unroll
    for (int u = 0; u < 6; ++u) s += (v[u][0] + v[u][1]) + (v[u][2] + v[u][3]);
    const float mu = wsum(s) * (1.f / kD);
    float q = 0.f;
#pragma unroll
    for (int u = 0; u < 6; ++u)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = v[u][e] - mu;
        q += d * d;
      }
    const float rs = 1.f / sqrtf(wsum(q) * (1.f / kD) + kLnEps);
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      const int c = 4 * lane + 256 * u;
      if (c >= k0 && c < k0 + a.chunk) {
        const f4 xh = (v[u] - mu) * rs;
        *reinterpret_cast<f4*>(a.xhat + static_cast<int64_t>(r) * kD + c) = xh;
        const f4 gg = *reinterpret_cast<const f4*>(g + c), b4 = *reinterpret_cast<const f4*>(bb + c);
        *reinterpret_cast<f4*>(&xn[rl][c - k0]) = xh * gg + b4;
      }
    }
  }
  __syncthreads();
  // HG0 partial over this K chunk: wave w -> output columns [32 w, 32 w + 32).
  // MFMA step (i, s) covers k = 16 i + 4 kq + s for lane group kq: A and B
  // both read float4 runs along k.
  const int m = lane & 15, kq = lane >> 4;
  const float* w0 = a.P + a.w0 + static_cast<int64_t>(32 * wave + m) * kD + k0 + 4 * kq;
  const float* w1 = w0 + 16 * kD;
  const float* xr = &xn[m][4 * kq];
  f4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
  const int n16 = a.chunk / 16;
#pragma unroll 4
  for (int i = 0; i < n16; ++i) {
    const f4 av = *reinterpret_cast<const f4*>(xr + 16 * i);
    const f4 b0 = *reinterpret_cast<const f4*>(w0 + 16 * i);
    const f4 b1 = *reinterpret_cast<const f4*>(w1 + 16 * i);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      acc0 = mma(av[s], b0[s], acc0);
      acc1 = mma(av[s], b1[s], acc1);
    }
  }
  float* out = a.hg_part + static_cast<int64_t>(ks) * a.B * kH2;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int r = rt * kR + 4 * kq + e;
    if (r < a.B) {
      out[static_cast<int64_t>(r) * kH2 + 32 * wave + m] = acc0[e];
      out[static_cast<int64_t>(r) * kH2 + 32 * wave + 16 + m] = acc1[e];
    }
  }
}

// ------------------------------------------------------------------ k2 ----
// C[16][N] = A[16][K] (LDS, stride kLd) . op(W) (+ bias), op(W) = W^T for
// W [N][K] row-major (NT, the forward) or W for W [K][N] (NN, the backward).
// Waves take 16-column tiles round robin; two accumulation chains per tile.
template <int K, int N, bool NT>
__device__ __forceinline__ void rows_gemm(const float* A, const float* __restrict__ W,
                                          const float* __restrict__ bias, float* C, int wave, int lane) {
  constexpr int kTiles = (N + 15) / 16;
  const int m = lane & 15, kq = lane >> 4;
  for (int t = wave; t < kTiles; t += 4) {
    const int n = 16 * t + m;
    const bool nok = n < N;
    f4 acc[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int i = 0; i < K / 16; ++i) {
      const f4 av = *reinterpret_cast<const f4*>(A + m * kLd + 16 * i + 4 * kq);
      f4 bv = {0.f, 0.f, 0.f, 0.f};
      if (nok) {
        if (NT) {
          bv = *reinterpret_cast<const f4*>(W + n * K + 16 * i + 4 * kq);
        } else {
#pragma unroll
          for (int s = 0; s < 4; ++s) bv[s] = W[(16 * i + 4 * kq + s) * N + n];
        }
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) acc[i & 1] = mma(av[s], bv[s], acc[i & 1]);
    }
    const f4 r = acc[0] + acc[1];
    if (nok) {
      const float b = bias ? bias[n] : 0.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) C[(4 * kq + e) * kLd + n] = r[e] + b;
    }
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
  // activations for k3, [NG][B][width]: U 64, Xn 96 (k >= 1), dS 96 (k = NG-1: column 0), dHG 128
  float* U;
  float* Xn;
  float* dS;
  float* dHG;
};

template <bool kTrain>
__global__ void __launch_bounds__(256) k2_rows_kernel(K2Args a) {
  __shared__ __attribute__((aligned(16))) float hgS[kMaxG][kR][kLd];
  __shared__ __attribute__((aligned(16))) float xhS[kMaxG - 1][kR][kL + 4];
  __shared__ __attribute__((aligned(16))) float bufA[kR][kLd];
  __shared__ __attribute__((aligned(16))) float bufB[kR][kLd];
  __shared__ __attribute__((aligned(16))) float bufS[kR][kLd];
  __shared__ float rsS[kMaxG][kR];
  __shared__ float zS[kR], dzS[kR];
  __shared__ float red[4][kStats];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r0 = blockIdx.x * kR;
  const int nrow = min(kR, a.B - r0);
  const float* P = a.P;
  const int NG = a.NG;
  const int64_t B = a.B;
  // HG0 = sum of k1's partials + bias
  for (int e = tid; e < kR * kH2; e += 256) {
    const int r = e >> 7, j = e & 127;
    float v = 0.f;
    if (r < nrow)
      for (int s = 0; s < a.KS; ++s) v += a.hg_part[(s * B + r0 + r) * kH2 + j];
    hgS[0][r][j] = v + P[a.b_hg[0] + j];
  }
  __syncthreads();
  // ---------------------------------------------------------- forward ----
  for (int k = 0; k < NG; ++k) {
    // U = silu(H) * G
    for (int e = tid; e < kR * kH; e += 256) {
      const int r = e >> 6, j = e & 63;
      const float h = hgS[k][r][j], gg = hgS[k][r][kH + j];
      const float u = h * sigm(h) * gg;
      bufA[r][j] = u;
      if (kTrain && r < nrow) a.U[(k * B + r0 + r) * kH + j] = u;
    }
    __syncthreads();
    if (k == NG - 1) break;
    rows_gemm<kH, kL, true>(&bufA[0][0], P + a.w_o[k], P + a.b_o[k], &bufB[0][0], wave, lane);
    __syncthreads();
    // LayerNorm k over 96 columns: wave w -> rows 4w..4w+3, lane -> c, c + 64
    const float* lg = P + a.ln_g[k];
    const float* lb = P + a.ln_b[k];
    for (int i = 0; i < 4; ++i) {
      const int r = wave * 4 + i;
      const float v0 = bufB[r][lane], v1 = lane < kL - 64 ? bufB[r][64 + lane] : 0.f;
      const float mu = wsum(v0 + v1) * (1.f / kL);
      const float d0 = v0 - mu, d1 = lane < kL - 64 ? v1 - mu : 0.f;
      const float rs = 1.f / sqrtf(wsum(d0 * d0 + d1 * d1) * (1.f / kL) + kLnEps);
      const float x0 = d0 * rs, x1 = d1 * rs;
      xhS[k][r][lane] = x0;
      const float n0 = x0 * lg[lane] + lb[lane];
      bufA[r][lane] = n0;
      if (kTrain && r < nrow) a.Xn[((k + 1) * B + r0 + r) * kL + lane] = n0;
      if (lane < kL - 64) {
        xhS[k][r][64 + lane] = x1;
        const float n1 = x1 * lg[64 + lane] + lb[64 + lane];
        bufA[r][64 + lane] = n1;
        if (kTrain && r < nrow) a.Xn[((k + 1) * B + r0 + r) * kL + 64 + lane] = n1;
      }
      if (lane == 0) rsS[k][r] = rs;
    }
    __syncthreads();
    rows_gemm<kL, kH2, true>(&bufA[0][0], P + a.w_hg[k + 1], P + a.b_hg[k + 1], &hgS[k + 1][0][0], wave, lane);
    __syncthreads();
  }
  // output unit: z = U . w_o + b_o (wave w -> rows 4w..4w+3)
  {
    const float* wo = P + a.w_o[NG - 1];
    const float bo = P[a.b_o[NG - 1]];
    for (int i = 0; i < 4; ++i) {
      const int r = wave * 4 + i;
      const float z = wsum(bufA[r][lane] * wo[lane]) + bo;
      if (lane == 0) zS[r] = z;
    }
  }
  __syncthreads();
  const int step = step_of(a.state, a.parity);
  // sigmoid, high-loss filter (trainer.py:407-424), weighted BCE (:301-312, torch
  // formulas incl. the log clamp at -100 and the 1e-12 in BCE's backward)
  if (tid < kR) {
    const int r = tid;
    float loc[kStats] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    float dz = 0.f;
    if (r < nrow) {
      const float z = zS[r], p = sigm(z);
      if (a.prob) a.prob[r0 + r] = p;
      if (a.logit) a.logit[r0 + r] = z;
      if (kTrain) {
        float nw = a.neg_weight;
        if (a.sched) nw = a.sched[2 * min(step, a.sched_len - 1) + 1];
        const float yy = a.y[static_cast<int64_t>(step) * a.y_stride + r0 + r];
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
    if (kTrain) {
#pragma unroll
      for (int s = 0; s < kStats; ++s) {
        float v = loc[s];
#pragma unroll
        for (int o = 8; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);  // 16-lane sum
        if (tid == 0) red[0][s] = v;
      }
    }
  }
  if (!kTrain) return;
  __syncthreads();
  if (tid < kStats && red[0][tid] != 0.f) atomicAdd(a.stats + tid, red[0][tid]);
  // ---------------------------------------------------------- backward ---
  float* G = a.G;
  // dS of the output unit = dz (column 0), its bias gradient = sum dz
  if (tid < kR) {
    bufS[tid][0] = dzS[tid];
    if (tid < nrow) a.dS[((NG - 1) * B + r0 + tid) * kL] = dzS[tid];
  }
  if (tid == 0) {
    float s = 0.f;
    for (int r = 0; r < kR; ++r) s += dzS[r];
    if (s != 0.f) atomicAdd(G + a.b_o[NG - 1], s);
  }
  __syncthreads();
  for (int k = NG - 1; k >= 0; --k) {
    // dU = dS_k . W_o_k
    if (k == NG - 1) {
      const float* wo = P + a.w_o[k];
      for (int e = tid; e < kR * kH; e += 256) {
        const int r = e >> 6, j = e & 63;
        bufA[r][j] = bufS[r][0] * wo[j];
      }
    } else {
      rows_gemm<kL, kH, false>(&bufS[0][0], P + a.w_o[k], nullptr, &bufA[0][0], wave, lane);
      // bias gradient of output k: column sums of dS_k
      if (tid < kL) {
        float s = 0.f;
        for (int r = 0; r < kR; ++r) s += bufS[r][tid];
        atomicAdd(G + a.b_o[k] + tid, s);
      }
    }
    __syncthreads();
    // gate backward: dH = dU G silu'(H), dG = dU silu(H)
    for (int e = tid; e < kR * kH; e += 256) {
      const int r = e >> 6, j = e & 63;
      const float h = hgS[k][r][j], gg = hgS[k][r][kH + j], du = bufA[r][j];
      const float sg = sigm(h);
      const float dh = du * gg * (sg * (1.f + h * (1.f - sg))), dg = du * h * sg;
      bufB[r][j] = dh;
      bufB[r][kH + j] = dg;
      if (r < nrow) {
        a.dHG[(k * B + r0 + r) * kH2 + j] = dh;
        a.dHG[(k * B + r0 + r) * kH2 + kH + j] = dg;
      }
    }
    __syncthreads();
    if (tid < kH2) {  // bias gradient of hidden + gate k
      float s = 0.f;
      for (int r = 0; r < kR; ++r) s += bufB[r][tid];
      atomicAdd(G + a.b_hg[k] + tid, s);
    }
    if (k == 0) break;
    // dXn (input of GMLP k = output of LayerNorm k - 1) = dHG . W_hg_k
    rows_gemm<kH2, kL, false>(&bufB[0][0], P + a.w_hg[k], nullptr, &bufA[0][0], wave, lane);
    __syncthreads();
    // LayerNorm k - 1 backward: gamma / beta column sums, dS_{k-1} per row
    {
      const int l = k - 1;
      if (tid < kL) {
        float sg = 0.f, sb = 0.f;
        for (int r = 0; r < kR; ++r) {
          sg += bufA[r][tid] * xhS[l][r][tid];
          sb += bufA[r][tid];
        }
        atomicAdd(G + a.ln_g[l] + tid, sg);
        atomicAdd(G + a.ln_b[l] + tid, sb);
      }
      const float* lg = P + a.ln_g[l];
      for (int i = 0; i < 4; ++i) {
        const int r = wave * 4 + i;
        const float t0 = bufA[r][lane] * lg[lane];
        const float t1 = lane < kL - 64 ? bufA[r][64 + lane] * lg[64 + lane] : 0.f;
        const float x0 = xhS[l][r][lane], x1 = lane < kL - 64 ? xhS[l][r][64 + lane] : 0.f;
        const float s1 = wsum(t0 + t1) * (1.f / kL);
        const float s2 = wsum(t0 * x0 + t1 * x1) * (1.f / kL);
        const float rs = rsS[l][r];
        const float d0 = rs * (t0 - s1 - x0 * s2);
        bufS[r][lane] = d0;
        if (r < nrow) a.dS[(l * B + r0 + r) * kL + lane] = d0;
        if (lane < kL - 64) {
          const float d1 = rs * (t1 - s1 - x1 * s2);
          bufS[r][64 + lane] = d1;
          if (r < nrow) a.dS[(l * B + r0 + r) * kL + 64 + lane] = d1;
        }
      }
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ k3 ----
// dW [M][N] += X^T Y over a chunk of batch rows: X [B][ldx] (columns = M),
// Y [B][ldy] (columns = N). Tile 64 x 32, wave w -> rows 16 w..16 w + 15.
constexpr int kTM = 64, kTN = 32, kMaxJobs = 2 * kMaxG;
struct WJob {
  const float* X;
  const float* Y;
  float* C;
  int ldx, ldy, ldc, M, N, tn;
};
struct K3Args {
  WJob job[kMaxJobs];
  int start[kMaxJobs + 1];
  int n_jobs, B, Kc, KS;
  // input-layer job (job 0): post-op with norm_in's affine and W_hg0
  const float* g_in;
  const float* b_in;
  const float* W0;
  float* dg_in;
  float* db_in;
};

__global__ void __launch_bounds__(256) k3_wgrad_kernel(K3Args a) {
  __shared__ float sS[kTM];
  __shared__ float red[2][4][kTN];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int blk = blockIdx.x;
  int j = 0;
  while (j + 1 < a.n_jobs && blk >= a.start[j + 1]) ++j;
  const WJob jb = a.job[j];
  const int local = blk - a.start[j];
  const int split = local % a.KS, tile = local / a.KS;
  const int tm = tile / jb.tn, tn = tile - tm * jb.tn;
  const int rb0 = split * a.Kc, rb1 = min(a.B, rb0 + a.Kc);
  const int m = lane & 15, kq = lane >> 4;
  const int mrow = tm * kTM + 16 * wave;   // first M row of this wave
  const int n0 = tn * kTN;
  const bool mok = mrow + m < jb.M;
  const bool nok0 = n0 + m < jb.N, nok1 = n0 + 16 + m < jb.N;
  f4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
  float ssum = 0.f;
  const float* X = jb.X + mrow + m;
  const float* Y0 = jb.Y + n0 + m;
  const float* Y1 = Y0 + 16;
  for (int b = rb0; b < rb1; b += 32) {
    float xa[8], ya[8], yb[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int rb = b + 4 * u + kq;
      const bool ok = rb < rb1;
      xa[u] = (ok && mok) ? X[static_cast<int64_t>(rb) * jb.ldx] : 0.f;
      ya[u] = (ok && nok0) ? Y0[static_cast<int64_t>(rb) * jb.ldy] : 0.f;
      yb[u] = (ok && nok1) ? Y1[static_cast<int64_t>(rb) * jb.ldy] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      acc0 = mma(xa[u], ya[u], acc0);
      acc1 = mma(xa[u], yb[u], acc1);
      ssum += xa[u];
    }
  }
  if (j != 0) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int row = mrow + 4 * kq + e;
      if (row < jb.M) {
        if (nok0) atomicAdd(jb.C + static_cast<int64_t>(row) * jb.ldc + n0 + m, acc0[e]);
        if (nok1) atomicAdd(jb.C + static_cast<int64_t>(row) * jb.ldc + n0 + 16 + m, acc1[e]);
      }
    }
    return;
  }
  // input layer: s_j = sum over the chunk's rows of dHG0[b][j] (lanes m, m+16, m+32, m+48 hold parts)
  ssum += __shfl_xor(ssum, 16, 64);
  ssum += __shfl_xor(ssum, 32, 64);
  if (kq == 0) sS[16 * wave + m] = ssum;
  __syncthreads();
  float dg0 = 0.f, dg1 = 0.f, dbt0 = 0.f, dbt1 = 0.f;
  const int c0 = n0 + m, c1 = n0 + 16 + m;
  const float g0 = nok0 ? a.g_in[c0] : 0.f, g1 = nok1 ? a.g_in[c1] : 0.f;
  const float be0 = nok0 ? a.b_in[c0] : 0.f, be1 = nok1 ? a.b_in[c1] : 0.f;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int row = mrow + 4 * kq + e;  // j
    if (row >= jb.M) continue;
    const float sj = sS[16 * wave + 4 * kq + e];
    const float* wr = a.W0 + static_cast<int64_t>(row) * jb.ldc;
    if (nok0) {
      atomicAdd(jb.C + static_cast<int64_t>(row) * jb.ldc + c0, g0 * acc0[e] + be0 * sj);
      const float w = wr[c0];
      dg0 += w * acc0[e];
      dbt0 += w * sj;
    }
    if (nok1) {
      atomicAdd(jb.C + static_cast<int64_t>(row) * jb.ldc + c1, g1 * acc1[e] + be1 * sj);
      const float w = wr[c1];
      dg1 += w * acc1[e];
      dbt1 += w * sj;
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
      atomicAdd(a.dg_in + c, red[0][0][tid] + red[0][1][tid] + red[0][2][tid] + red[0][3][tid]);
      atomicAdd(a.db_in + c, red[1][0][tid] + red[1][1][tid] + red[1][2][tid] + red[1][3][tid]);
    }
  }
}

// ------------------------------------------------------------------ k4 ----
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
};

// The accumulation gate (trainer.py:443-465), computed identically by every
// workgroup from the step's read-only state half; workgroup 0 writes the other
// half and the history row. Then torch.optim.Adam (foreach, no weight decay) on
// grads * 1 / (n_sel * accumulation_steps) when it fires; the bucket's
// gradients are zeroed either way (zero_grad every step, :404).
__global__ void __launch_bounds__(256) k4_update_kernel(K4Args a) {
  const float* st = a.state + a.parity * 8;
  const float* stats = a.G + a.n;
  const float n_sel = stats[0];
  float acc_samples = st[0], acc_steps = st[1], t = st[2];
  const float stepf = st[3];
  const int step = static_cast<int>(stepf);
  float fire = 0.f, scale = 0.f, loss = 0.f;
  const float used = acc_steps;
  if (n_sel > 0.f) {
    loss = stats[1] / n_sel / acc_steps;
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
      h[4] = stats[2];
      h[5] = stats[3];
      h[6] = stats[4];
      h[7] = stats[5];
    }
  }
  float lr = a.lr;
  if (a.sched) lr = a.sched[2 * min(step, a.sched_len - 1)];
  const float bc1 = 1.f - powf(a.b1, t), bc2s = sqrtf(1.f - powf(a.b2, t));
  const float step_size = lr / bc1;
  for (int64_t i = blockIdx.x * int64_t(256) + threadIdx.x; i < a.n; i += int64_t(gridDim.x) * 256) {
    const float g = a.G[i];
    a.G[i] = 0.f;
    if (fire != 0.f) {
      const float gi = g * scale;
      const float mi = a.b1 * a.m[i] + (1.f - a.b1) * gi;
      const float vi = a.b2 * a.v[i] + (1.f - a.b2) * gi * gi;
      a.m[i] = mi;
      a.v[i] = vi;
      a.P[i] -= step_size * mi / (sqrtf(vi) / bc2s + a.eps);
    }
  }
}

// --------------------------------------------------------- workspace ------
struct FusedWs {
  int64_t hg_part, xhat, U, Xn, dS, dHG, total;  // float offsets
};
int k1_splits(int B) {
  const int rt = (B + kR - 1) / kR;
  static const int ks_opts[] = {4, 6, 8, 12, 16, 24};
  for (int ks : ks_opts)
    if (rt * ks >= 240) return ks;
  return 24;
}
FusedWs fused_layout(int64_t B, int NG) {
  FusedWs w;
  int64_t o = 0;
  auto take = [&](int64_t n) { const int64_t r = o; o += (n + 63) & ~int64_t(63); return r; };
  w.hg_part = take(int64_t(24) * B * kH2);
  w.xhat = take(B * kD);
  w.U = take(int64_t(NG) * B * kH);
  w.Xn = take(int64_t(NG) * B * kL);
  w.dS = take(int64_t(NG) * B * kL);
  w.dHG = take(int64_t(NG) * B * kH2);
  w.total = o;
  return w;
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

}  // namespace

bool mlp_fused_supported(const hbk_mlp_plan& p) {
  return p.d_in == kD && p.layer == kL && p.hid == kH && static_cast<int>(p.g.size()) <= kMaxG &&
         p.g.size() >= 2;
}

int64_t mlp_fused_ws_floats(const hbk_mlp_plan& p, int64_t B) {
  return fused_layout(std::max<int64_t>(B, 1), static_cast<int>(p.g.size())).total;
}

// k1 + k2 (+ k3): the forward (inference) or forward/backward half of a step.
int mlp_fused_run(const hbk_mlp_plan& p, const float* params, const float* pool32, int64_t n32,
                  const void* pool16, int64_t n16, const int32_t* idx, int64_t idx_stride, const float* y, int64_t y_stride, int B,
                  const float* state, int parity, const float* sched, int sched_len, float neg_weight,
                  float thr, float act_thr, float drop_p, uint64_t seed, float* bucket, float* prob,
                  float* logit, float* ws, bool train, hipStream_t s) {
  const int NG = static_cast<int>(p.g.size());
  const FusedWs w = fused_layout(B, NG);
  const int KS = k1_splits(B);
  K1Args k1;
  k1.P = params;
  k1.g_in = p.ln_in.g;
  k1.b_in = p.ln_in.b;
  k1.w0 = p.g[0].w_hg;
  k1.pool32 = pool32;
  k1.pool16 = static_cast<const _Float16*>(pool16);
  k1.n32 = pool32 ? n32 : 0;
  k1.n16 = pool16 ? n16 : 0;
  k1.idx = idx;
  k1.idx_stride = idx_stride;
  k1.state = state;
  k1.parity = parity;
  k1.B = B;
  k1.chunk = kD / KS;
  k1.drop_p = drop_p;
  k1.seed = seed;
  k1.hg_part = ws + w.hg_part;
  k1.xhat = ws + w.xhat;
  k1.stats = train ? bucket + p.n_params : nullptr;
  const int rt = (B + kR - 1) / kR;
  hipLaunchKernelGGL(k1_input_kernel, dim3(rt, KS), dim3(256), 0, s, k1);
  HBK_LAUNCH_CHECK("k1_input_kernel");
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
  k2.G = bucket;
  k2.stats = bucket ? bucket + p.n_params : nullptr;
  k2.U = ws + w.U;
  k2.Xn = ws + w.Xn;
  k2.dS = ws + w.dS;
  k2.dHG = ws + w.dHG;
  if (!train) {
    hipLaunchKernelGGL(k2_rows_kernel<false>, dim3(rt), dim3(256), 0, s, k2);
    HBK_LAUNCH_CHECK("k2_rows_kernel");
    return HBK_OK;
  }
  hipLaunchKernelGGL(k2_rows_kernel<true>, dim3(rt), dim3(256), 0, s, k2);
  HBK_LAUNCH_CHECK("k2_rows_kernel");
  // k3: job 0 = input layer, then dW_hg of GMLPs 1.., then dW_o of every GMLP
  K3Args k3;
  int nj = 0, blocks = 0;
  const int KS3 = std::max(1, std::min((B + 127) / 128, 8));
  const int Kc = ((B + KS3 - 1) / KS3 + 3) / 4 * 4;
  auto add = [&](const float* X, int ldx, const float* Y, int ldy, float* C, int ldc, int M, int N) {
    WJob& j = k3.job[nj];
    j.X = X;
    j.ldx = ldx;
    j.Y = Y;
    j.ldy = ldy;
    j.C = C;
    j.ldc = ldc;
    j.M = M;
    j.N = N;
    j.tn = (N + kTN - 1) / kTN;
    k3.start[nj] = blocks;
    blocks += ((M + kTM - 1) / kTM) * j.tn * KS3;
    ++nj;
  };
  float* G = bucket;
  add(ws + w.dHG, kH2, ws + w.xhat, kD, G + p.g[0].w_hg, kD, kH2, kD);
  for (int k = 1; k < NG; ++k)
    add(ws + w.dHG + int64_t(k) * B * kH2, kH2, ws + w.Xn + int64_t(k) * B * kL, kL, G + p.g[k].w_hg, kL, kH2,
        kL);
  for (int k = 0; k < NG; ++k)
    add(ws + w.dS + int64_t(k) * B * kL, kL, ws + w.U + int64_t(k) * B * kH, kH, G + p.g[k].w_o, kH,
        p.g[k].out, kH);
  k3.start[nj] = blocks;
  k3.n_jobs = nj;
  k3.B = B;
  k3.Kc = Kc;
  k3.KS = KS3;
  k3.g_in = params + p.ln_in.g;
  k3.b_in = params + p.ln_in.b;
  k3.W0 = params + p.g[0].w_hg;
  k3.dg_in = G + p.ln_in.g;
  k3.db_in = G + p.ln_in.b;
  hipLaunchKernelGGL(k3_wgrad_kernel, dim3(blocks), dim3(256), 0, s, k3);
  HBK_LAUNCH_CHECK("k3_wgrad_kernel");
  return HBK_OK;
}

int mlp_fused_update(const hbk_mlp_plan& p, float* params, float* bucket, float* m, float* v, float* state,
                     int parity, const float* sched, int sched_len, float lr, float b1, float b2, float eps,
                     float* hist, int hist_cap, hipStream_t s) {
  K4Args k;
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
  const int64_t blocks = std::min<int64_t>((p.n_params + 1023) / 1024, 1024);
  hipLaunchKernelGGL(k4_update_kernel, dim3(unsigned(blocks)), dim3(256), 0, s, k);
  HBK_LAUNCH_CHECK("k4_update_kernel");
  return HBK_OK;
}

}  // namespace hbk
