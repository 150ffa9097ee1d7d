// Wake-word classifier (gated MLP) forward + fused train step for gfx950.
//
// Replaces WakeWordMLPModel.forward (wakeword.py:334-348) and the optimisation
// path of WakeWordTrainer.train_epoch (trainer.py:380-494): high-loss filter,
// weighted BCE, backward, the < 128-sample accumulation gate and Adam
// (trainer.py:45). Numerics are f32 throughout (GEMMs on
// v_mfma_f32_16x16x4f32), so logits match the reference within 1e-4.
//
// Parameter layout (one flat f32 buffer; the Python module exposes state_dict
// views into it):
//   norm_in.{weight,bias} [D_in] x2
//   per GMLP g in (mlp_in, layers.l.1 ..., mlp_out):
//     W_hg [2H, in] (rows 0..H-1 = hidden.weight, H..2H-1 = gate.weight)
//     b_hg [2H]     (hidden.bias, gate.bias)
//     W_o  [out, H] (output.weight), b_o [out] (output.bias)
//   per LN before layers / norm_out: weight, bias [L]
// The order of blocks follows the forward pass.
//
// One train step, without a single host synchronisation:
//   hbk_mlp_train_fwd_bwd   forward, filter + BCE terms, backward into an
//                           UNNORMALISED gradient bucket (sum over selected
//                           samples of w * dl/dz), plus 8 statistics at the
//                           bucket's tail (n_sel, sum w*l, ...)
//   [optional RCCL all-reduce of the bucket across data-parallel ranks]
//   hbk_mlp_gate_adam       the reference's accumulation gate on the reduced
//                           statistics (device-resident state), then Adam on
//                           grads * 1 / (n_sel * accumulation_steps) iff it fires.
#include <algorithm>
#include <cmath>
#include <vector>

#include "hbk_common.h"
#include "hbk_mlp_internal.h"

namespace hbk {
namespace {

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int kStats = 8;  // bucket tail: see hbk.h
constexpr float kLnEps = 1e-5f;

// ------------------------------------------------------------- GEMM -------
// C[M,N] (+)= sum_k A(m,k) B(k,n) (+ bias[n]); A(m,k) = TA ? A[k*lda+m] : A[m*lda+k],
// B(k,n) = TB ? B[n*ldb+k] : B[k*ldb+n]. Tile 64x64x16, 4 waves as 2x2 of 32x32.
constexpr int GBM = 64, GBN = 64, GBK = 16;

template <bool TA, bool TB>
__global__ void __launch_bounds__(256) gemm_kernel(const float* __restrict__ A, const float* __restrict__ B,
                                                   float* __restrict__ C, const float* __restrict__ bias,
                                                   int M, int N, int K, int lda, int ldb, int ldc,
                                                   int accumulate, int k_split) {
  // split-K: block z covers K rows [z k_split, (z + 1) k_split) and atomically
  // adds its partial product (C pre-zeroed by the host; bias from split 0)
  __shared__ float As[GBK][GBM + 4];
  __shared__ float Bs[GBK][GBN + 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const int m0 = blockIdx.y * GBM, n0 = blockIdx.x * GBN;
  const int r16 = lane & 15, kq = lane >> 4;
  f4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
  const int kb = blockIdx.z * k_split, ke = min(K, kb + k_split);
  for (int k0 = kb; k0 < ke; k0 += GBK) {
    // stage A: 64 x 16 -> As[k][m]; B: 16 x 64 -> Bs[k][n]
#pragma unroll
    for (int e = tid; e < GBM * GBK; e += 256) {
      int m, k;
      if (TA) { k = e / GBM; m = e - k * GBM; } else { m = e / GBK; k = e - m * GBK; }
      const int gm = m0 + m, gk = k0 + k;
      float v = 0.f;
      if (gm < M && gk < ke) v = TA ? A[static_cast<int64_t>(gk) * lda + gm] : A[static_cast<int64_t>(gm) * lda + gk];
      As[k][m] = v;
    }
#pragma unroll
    for (int e = tid; e < GBN * GBK; e += 256) {
      int n, k;
      if (TB) { n = e / GBK; k = e - n * GBK; } else { k = e / GBN; n = e - k * GBN; }
      const int gn = n0 + n, gk = k0 + k;
      float v = 0.f;
      if (gn < N && gk < ke) v = TB ? B[static_cast<int64_t>(gn) * ldb + gk] : B[static_cast<int64_t>(gk) * ldb + gn];
      Bs[k][n] = v;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < GBK; kk += 4) {
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[kk + kq][32 * wr + 16 * i + r16];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[kk + kq][32 * wc + 16 * j + r16];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = n0 + 32 * wc + 16 * j + r16;
      if (n >= N) continue;
      const float bb = (bias && blockIdx.z == 0) ? bias[n] : 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int m = m0 + 32 * wr + 16 * i + kq * 4 + q;
        if (m < M) {
          float* c = C + static_cast<int64_t>(m) * ldc + n;
          const float v = acc[i][j][q] + bb;
          if (gridDim.z > 1)
            atomicAdd(c, v);
          else
            *c = accumulate ? *c + v : v;
        }
      }
    }
}

// ----------------------------------------------------- row kernels --------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Input dropout (nn.Dropout, wakeword.py:197/338: zero with prob p, scale by
// 1/(1-p)) folded into the first LayerNorm's load.
__device__ __forceinline__ float dropped(const float* xr, int64_t base, int i, float p, float keep_scale,
                                         uint64_t seed) {
  const float v = xr[i];
  if (p <= 0.f) return v;
  return uniform01(seed, static_cast<uint64_t>(base + i)) < p ? 0.f : v * keep_scale;
}

// LayerNorm forward, one wave per row: y = xhat * g + b; keeps xhat, rstd.
__global__ void __launch_bounds__(256) ln_fwd_kernel(const float* __restrict__ x, const float* __restrict__ g,
                                                     const float* __restrict__ b, float* __restrict__ y,
                                                     float* __restrict__ xhat, float* __restrict__ rstd,
                                                     int rows, int D, float drop_p, uint64_t seed,
                                                     const double* __restrict__ step_sc) {
  if (step_sc) seed = static_cast<uint64_t>(step_sc[2]);  // graph replays: per-step seed from the device
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float* xr = x + static_cast<int64_t>(row) * D;
  const int64_t base = static_cast<int64_t>(row) * D;
  const float ks = drop_p > 0.f ? 1.f / (1.f - drop_p) : 1.f;
  float s = 0.f;
  for (int i = lane; i < D; i += 64) s += dropped(xr, base, i, drop_p, ks, seed);
  const float mu = wave_sum(s) / D;
  float v = 0.f;
  for (int i = lane; i < D; i += 64) {
    const float d = dropped(xr, base, i, drop_p, ks, seed) - mu;
    v += d * d;
  }
  const float rs = 1.f / sqrtf(wave_sum(v) / D + kLnEps);
  for (int i = lane; i < D; i += 64) {
    const float h = (dropped(xr, base, i, drop_p, ks, seed) - mu) * rs;
    xhat[static_cast<int64_t>(row) * D + i] = h;
    y[static_cast<int64_t>(row) * D + i] = h * g[i] + b[i];
  }
  if (lane == 0) rstd[row] = rs;
}

// LayerNorm backward. dx (optional) per row; dgamma/dbeta accumulated with
// per-block partial sums over 4 rows then atomics (one per column per block).
__global__ void __launch_bounds__(256) ln_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ xhat,
                                                     const float* __restrict__ rstd, const float* __restrict__ g,
                                                     float* __restrict__ dx, float* __restrict__ dg,
                                                     float* __restrict__ db, int rows, int D,
                                                     int rows_per_block) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r0 = blockIdx.x * rows_per_block;
  // dgamma / dbeta: thread owns columns c = tid, tid+256, ...
  for (int c = threadIdx.x; c < D; c += 256) {
    float sg = 0.f, sb = 0.f;
    for (int r = r0; r < min(r0 + rows_per_block, rows); ++r) {
      const float d = dy[static_cast<int64_t>(r) * D + c];
      sg += d * xhat[static_cast<int64_t>(r) * D + c];
      sb += d;
    }
    atomicAdd(dg + c, sg);
    atomicAdd(db + c, sb);
  }
  if (!dx) return;
  for (int r = r0 + wave; r < min(r0 + rows_per_block, rows); r += 4) {
    const float* dyr = dy + static_cast<int64_t>(r) * D;
    const float* xr = xhat + static_cast<int64_t>(r) * D;
    float s1 = 0.f, s2 = 0.f;
    for (int i = lane; i < D; i += 64) {
      const float t = dyr[i] * g[i];
      s1 += t;
      s2 += t * xr[i];
    }
    s1 = wave_sum(s1) / D;
    s2 = wave_sum(s2) / D;
    const float rs = rstd[r];
    for (int i = lane; i < D; i += 64) dx[static_cast<int64_t>(r) * D + i] = rs * (dyr[i] * g[i] - s1 - xr[i] * s2);
  }
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + expf(-x)); }

// U = silu(H) * G from HG [rows, 2H]
__global__ void gate_fwd_kernel(const float* __restrict__ hg, float* __restrict__ u, int rows, int H) {
  const int64_t n = static_cast<int64_t>(rows) * H;
  for (int64_t e = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; e < n; e += int64_t(gridDim.x) * blockDim.x) {
    const int64_t r = e / H;
    const int j = static_cast<int>(e - r * H);
    const float h = hg[r * 2 * H + j], g = hg[r * 2 * H + H + j];
    u[e] = h * sigmoidf_(h) * g;
  }
}

// dHG from dU: dH = dU * G * silu'(H), dG = dU * silu(H)
__global__ void gate_bwd_kernel(const float* __restrict__ du, const float* __restrict__ hg,
                                float* __restrict__ dhg, int rows, int H) {
  const int64_t n = static_cast<int64_t>(rows) * H;
  for (int64_t e = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; e < n; e += int64_t(gridDim.x) * blockDim.x) {
    const int64_t r = e / H;
    const int j = static_cast<int>(e - r * H);
    const float h = hg[r * 2 * H + j], g = hg[r * 2 * H + H + j];
    const float s = sigmoidf_(h);
    const float d = du[e];
    dhg[r * 2 * H + j] = d * g * (s * (1.f + h * (1.f - s)));
    dhg[r * 2 * H + H + j] = d * h * s;
  }
}

// column sums of X [rows, N] accumulated into out [N] (bias gradients)
__global__ void colsum_kernel(const float* __restrict__ x, float* __restrict__ out, int rows, int N,
                              int rows_per_block) {
  const int r0 = blockIdx.x * rows_per_block;
  for (int c = threadIdx.x; c < N; c += blockDim.x) {
    float s = 0.f;
    for (int r = r0; r < min(r0 + rows_per_block, rows); ++r) s += x[static_cast<int64_t>(r) * N + c];
    atomicAdd(out + c, s);
  }
}

// sigmoid, high-loss filter (trainer.py:407-424), weighted BCE terms and dl/dz
// for the selected samples (torch formulas); block-reduced statistics into the
// bucket tail: [n_sel, sum w*l, n_neg_sel, fp_sel, n_pos_sel, tp_sel, n, 0].
__global__ void __launch_bounds__(256) loss_kernel(const float* __restrict__ z, const float* __restrict__ y,
                                                   float* __restrict__ prob, float* __restrict__ dz,
                                                   float* __restrict__ stats, int rows, float neg_weight,
                                                   float thr, float act_thr, const double* __restrict__ step_sc) {
  if (step_sc) neg_weight = static_cast<float>(step_sc[1]);
  __shared__ float red[4][kStats];
  float loc[kStats] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < rows; i += gridDim.x * blockDim.x) {
    const float p = sigmoidf_(z[i]);
    prob[i] = p;
    const float yy = y[i];
    const bool pos = yy == 1.f;
    const bool sel = pos ? (p < 1.f - thr) : (p >= thr);
    float d = 0.f;
    if (sel) {
      const float w = pos ? 1.f : neg_weight;
      const float lp = fmaxf(logf(p), -100.f), l1p = fmaxf(logf(1.f - p), -100.f);
      const float l = -(yy * lp + (1.f - yy) * l1p);
      const float dp = w * (p - yy) / fmaxf((1.f - p) * p, 1e-12f);
      d = dp * (1.f - p) * p;
      loc[0] += 1.f;
      loc[1] += w * l;
      if (pos) {
        loc[4] += 1.f;
        if (p > act_thr) loc[5] += 1.f;  // recall numerator (torchmetrics: preds > threshold)
      } else {
        loc[2] += 1.f;
        if (yy - p <= -act_thr) loc[3] += 1.f;  // num_false_positives (trainer.py:287-296)
      }
    }
    dz[i] = d;
    loc[6] += 1.f;
  }
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
#pragma unroll
  for (int s = 0; s < kStats; ++s) {
    const float v = wave_sum(loc[s]);
    if (lane == 0) red[wave][s] = v;
  }
  __syncthreads();
  if (threadIdx.x < kStats) {
    const float v = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    atomicAdd(stats + threadIdx.x, v);
  }
}

// sigmoid only (inference)
__global__ void sigmoid_kernel(const float* __restrict__ z, float* __restrict__ p, int rows) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < rows; i += gridDim.x * blockDim.x) p[i] = sigmoidf_(z[i]);
}

// Accumulation gate (trainer.py:443-465), one thread. state:
// [0] accumulated_samples [1] accumulation_steps [2] adam t [3] step index
// ctrl (written): [0] fire [1] grad scale [2] bias-correction 1 [3] bias-correction 2
// hist (per step, 8 floats): n_sel, acc_steps used, fired, loss, n_neg_sel, fp, n_pos_sel, tp
__global__ void gate_kernel(const float* __restrict__ stats, float* __restrict__ state, float* __restrict__ ctrl,
                            float* __restrict__ hist, int hist_cap, float beta1, float beta2) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const float n_sel = stats[0];
  float acc_samples = state[0], acc_steps = state[1], t = state[2];
  const int step = static_cast<int>(state[3]);
  float fire = 0.f, scale = 0.f, loss = 0.f;
  const float used_steps = acc_steps;
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
  state[0] = acc_samples;
  state[1] = acc_steps;
  state[2] = t;
  state[3] = static_cast<float>(step + 1);
  ctrl[0] = fire;
  ctrl[1] = scale;
  ctrl[2] = 1.f - powf(beta1, t);
  ctrl[3] = 1.f - powf(beta2, t);
  if (hist && step < hist_cap) {
    float* h = hist + static_cast<int64_t>(step) * 8;
    h[0] = n_sel;
    h[1] = used_steps;
    h[2] = fire;
    h[3] = loss;
    h[4] = stats[2];  // selected negatives
    h[5] = stats[3];  // false positives among them
    h[6] = stats[4];  // selected positives
    h[7] = stats[5];  // true positives among them
  }
}

// torch.optim.Adam (foreach, amsgrad off, no weight decay):
// m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2;
// p -= lr / bc1 * m / (sqrt(v) / sqrt(bc2) + eps)
__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, const float* __restrict__ ctrl, int64_t n, float lr,
                            float beta1, float beta2, float eps, const double* __restrict__ step_sc) {
  if (ctrl[0] == 0.f) return;
  if (step_sc) lr = static_cast<float>(step_sc[0]);
  const float scale = ctrl[1], bc1 = ctrl[2], bc2s = sqrtf(ctrl[3]);
  const float step_size = lr / bc1, inv_bc2s = 1.f / bc2s;
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n; i += int64_t(gridDim.x) * blockDim.x) {
    const float gi = g[i] * scale;
    const float mi = beta1 * m[i] + (1.f - beta1) * gi;
    const float vi = beta2 * v[i] + (1.f - beta2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    p[i] -= adam_step(mi, vi, step_size, inv_bc2s, eps);
  }
}

}  // namespace
}  // namespace hbk

namespace hbk {
namespace {

// Workspace layout for a batch of B rows (floats).
struct Ws {
  int64_t xn_in, xhat_in, rstd_in;  // [B, D_in] x2, [B]
  std::vector<int64_t> hg, u, s;    // per GMLP: [B,2H], [B,H], [B,out]
  std::vector<int64_t> xn, xhat, rstd;  // per LN (layers + norm_out): [B,L], [B,L], [B]
  int64_t z, dz, prob, dtmp_a, dtmp_b, dhg, total;
};

Ws ws_layout(const hbk_mlp_plan& p, int64_t B) {
  Ws w;
  int64_t o = 0;
  auto take = [&](int64_t n) { const int64_t r = o; o += (n + 63) & ~int64_t(63); return r; };
  w.xn_in = take(B * p.d_in);
  w.xhat_in = take(B * p.d_in);
  w.rstd_in = take(B);
  for (const auto& gm : p.g) {
    w.hg.push_back(take(B * 2 * gm.hid));
    w.u.push_back(take(B * gm.hid));
    w.s.push_back(take(B * gm.out));
  }
  for (const auto& l : p.ln) {
    w.xn.push_back(take(B * l.d));
    w.xhat.push_back(take(B * l.d));
    w.rstd.push_back(take(B));
  }
  w.z = w.s.back();
  w.dz = take(B);
  w.prob = take(B);
  const int64_t wide = std::max<int64_t>(p.d_in, 2 * p.hid);
  w.dtmp_a = take(B * std::max<int64_t>(wide, p.layer));
  w.dtmp_b = take(B * std::max<int64_t>(wide, p.layer));
  w.dhg = take(B * 2 * p.hid);
  w.total = o;
  return w;
}

template <bool TA, bool TB>
int gemm(const float* A, const float* B, float* C, const float* bias, int M, int N, int K, int lda,
         int ldb, int ldc, bool acc, hipStream_t s) {
  if (M <= 0 || N <= 0) return HBK_OK;
  dim3 grid((N + GBN - 1) / GBN, (M + GBM - 1) / GBM);
  // Split-K when the output has too few tiles to fill the chip (the weight
  // gradients: K = batch; the input layer: K = 1536), >= 16 K rows per split.
  int splits = 1;
  const int tiles = int(grid.x * grid.y);
  if (tiles < 256 && K >= 256 && (ldc == N || acc)) splits = std::min(std::max(1, 512 / tiles), K / 16);
  const int k_split = ((K + splits - 1) / splits + GBK - 1) / GBK * GBK;
  splits = (K + k_split - 1) / k_split;
  if (splits > 1 && !acc) {
    hipError_t e = hipMemsetAsync(C, 0, size_t(M) * N * sizeof(float), s);
    if (e != hipSuccess) return hip_error(e, "hipMemsetAsync (split-K)");
  }
  grid.z = splits;
  hipLaunchKernelGGL((gemm_kernel<TA, TB>), grid, dim3(256), 0, s, A, B, C, bias, M, N, K, lda, ldb, ldc,
                     acc ? 1 : 0, k_split);
  HBK_LAUNCH_CHECK("gemm_kernel");
  return HBK_OK;
}

inline unsigned ew_grid(int64_t n) { return static_cast<unsigned>(std::min<int64_t>((n + 255) / 256, 4096)); }

#define HBK_RC(x)            \
  do {                       \
    int rc_ = (x);           \
    if (rc_) return rc_;     \
  } while (0)

// Forward pass; fills the workspace (activations kept for backward).
int forward(const hbk_mlp_plan& p, const float* P, const float* x, int B, float* ws, const Ws& w,
            float drop_p, uint64_t seed, hipStream_t s, const double* step_sc = nullptr) {
  const unsigned lnb = (B + 3) / 4;
  hipLaunchKernelGGL(ln_fwd_kernel, dim3(lnb), dim3(256), 0, s, x, P + p.ln_in.g, P + p.ln_in.b, ws + w.xn_in,
                     ws + w.xhat_in, ws + w.rstd_in, B, p.d_in, drop_p, seed, step_sc);
  HBK_LAUNCH_CHECK("ln_fwd_kernel");
  const float* in = ws + w.xn_in;
  for (size_t k = 0; k < p.g.size(); ++k) {
    const Gmlp& gm = p.g[k];
    if (k > 0) {
      const Ln& l = p.ln[k - 1];
      hipLaunchKernelGGL(ln_fwd_kernel, dim3(lnb), dim3(256), 0, s, ws + w.s[k - 1], P + l.g, P + l.b,
                         ws + w.xn[k - 1], ws + w.xhat[k - 1], ws + w.rstd[k - 1], B, l.d, 0.f,
                         uint64_t(0), static_cast<const double*>(nullptr));
      HBK_LAUNCH_CHECK("ln_fwd_kernel");
      in = ws + w.xn[k - 1];
    }
    // HG = in . W_hg^T + b_hg
    HBK_RC((gemm<false, true>(in, P + gm.w_hg, ws + w.hg[k], P + gm.b_hg, B, 2 * gm.hid, gm.in, gm.in, gm.in,
                              2 * gm.hid, false, s)));
    hipLaunchKernelGGL(gate_fwd_kernel, dim3(ew_grid(int64_t(B) * gm.hid)), dim3(256), 0, s, ws + w.hg[k],
                       ws + w.u[k], B, gm.hid);
    HBK_LAUNCH_CHECK("gate_fwd_kernel");
    HBK_RC((gemm<false, true>(ws + w.u[k], P + gm.w_o, ws + w.s[k], P + gm.b_o, B, gm.out, gm.hid, gm.hid,
                              gm.hid, gm.out, false, s)));
  }
  return HBK_OK;
}

}  // namespace
}  // namespace hbk

extern "C" {

int hbk_mlp_plan_create(int32_t d_in, int32_t layer_dim, int32_t hidden, int32_t n_layers, hbk_mlp_plan** plan) {
  using namespace hbk;
  if (!plan) return arg_error("plan is NULL");
  *plan = nullptr;
  if (d_in <= 0 || layer_dim <= 0 || hidden <= 0 || n_layers < 0) return arg_error("bad MLP dims");
  auto* p = new hbk_mlp_plan();
  p->d_in = d_in;
  p->layer = layer_dim;
  p->hid = hidden;
  p->n_layers = n_layers;
  int64_t o = 0;
  p->ln_in = Ln{d_in, o, o + d_in};
  o += 2 * int64_t(d_in);
  auto add_gmlp = [&](int in, int out) {
    Gmlp gm{in, hidden, out, 0, 0, 0, 0};
    gm.w_hg = o; o += int64_t(2) * hidden * in;
    gm.b_hg = o; o += 2 * hidden;
    gm.w_o = o; o += int64_t(out) * hidden;
    gm.b_o = o; o += out;
    p->g.push_back(gm);
  };
  auto add_ln = [&](int d) {
    p->ln.push_back(Ln{d, o, o + d});
    o += 2 * int64_t(d);
  };
  add_gmlp(d_in, layer_dim);
  for (int l = 0; l < n_layers; ++l) {
    add_ln(layer_dim);
    add_gmlp(layer_dim, layer_dim);
  }
  add_ln(layer_dim);
  add_gmlp(layer_dim, 1);
  p->n_params = o;
  *plan = p;
  return HBK_OK;
}

int hbk_mlp_plan_destroy(hbk_mlp_plan* p) {
  delete p;
  return HBK_OK;
}

int hbk_mlp_layout(const hbk_mlp_plan* p, int64_t* n_params, int64_t* offsets, int32_t n_offsets) {
  using namespace hbk;
  if (!p || !n_params) return arg_error("NULL");
  *n_params = p->n_params;
  // offsets (if given): ln_in g,b; then per GMLP k: w_hg, b_hg, w_o, b_o, and per
  // LN k (after GMLP k): g, b  -> 2 + 4*n_gmlp + 2*n_ln entries
  const int need = 2 + 4 * int(p->g.size()) + 2 * int(p->ln.size());
  if (offsets) {
    if (n_offsets < need) return arg_error("offsets array too small");
    int i = 0;
    offsets[i++] = p->ln_in.g;
    offsets[i++] = p->ln_in.b;
    for (const auto& gm : p->g) {
      offsets[i++] = gm.w_hg;
      offsets[i++] = gm.b_hg;
      offsets[i++] = gm.w_o;
      offsets[i++] = gm.b_o;
    }
    for (const auto& l : p->ln) {
      offsets[i++] = l.g;
      offsets[i++] = l.b;
    }
  }
  return HBK_OK;
}

int hbk_mlp_workspace_size(const hbk_mlp_plan* p, int64_t batch, int64_t* bytes) {
  if (!p || !bytes) return hbk::arg_error("NULL");
  int64_t floats = hbk::ws_layout(*p, std::max<int64_t>(batch, 1)).total;
  if (hbk::mlp_fused_supported(*p)) floats = std::max(floats, hbk::mlp_fused_ws_floats(*p, batch));
  *bytes = floats * int64_t(sizeof(float));
  return HBK_OK;
}

int hbk_mlp_forward(const hbk_mlp_plan* p, const float* params, const float* x, int64_t batch, float* prob,
                    float* logit, float dropout_p, uint64_t seed, void* workspace, int64_t ws_bytes,
                    void* stream) {
  using namespace hbk;
  if (!p) return arg_error("plan is NULL");
  if (batch < 0 || batch > (1 << 24)) return arg_error("batch out of range");
  if (batch == 0) return HBK_OK;
  if (!params || !x || !prob || !workspace) return arg_error("NULL pointer");
  const Ws w = ws_layout(*p, batch);
  if (ws_bytes < w.total * int64_t(sizeof(float))) return arg_error("workspace too small");
  hipStream_t s = as_stream(stream);
  float* ws = static_cast<float*>(workspace);
  const int B = static_cast<int>(batch);
  if (dropout_p < 0.f || dropout_p >= 1.f) return arg_error("dropout_p must be in [0, 1)");
  if (mlp_fused_supported(*p)) {
    if (ws_bytes < mlp_fused_ws_floats(*p, batch) * int64_t(sizeof(float))) return arg_error("workspace too small");
    return mlp_fused_run(*p, params, x, batch, nullptr, 0, nullptr, 0, 0, nullptr, 0, B, nullptr, 0, nullptr, 0, 1.f,
                         0.f, 0.f, dropout_p, seed, nullptr, prob, logit, ws, false, 0, s);
  }
  HBK_RC(forward(*p, params, x, B, ws, w, dropout_p, seed, s));
  hipLaunchKernelGGL(sigmoid_kernel, dim3(ew_grid(B)), dim3(256), 0, s, ws + w.z, prob, B);
  HBK_LAUNCH_CHECK("sigmoid_kernel");
  if (logit) HBK_HIP(hipMemcpyAsync(logit, ws + w.z, sizeof(float) * B, hipMemcpyDeviceToDevice, s));
  return HBK_OK;
}

int hbk_mlp_train_fwd_bwd(const hbk_mlp_plan* p, const float* params, const float* x, const float* y,
                          int64_t batch, float neg_weight, float high_loss_threshold,
                          float activation_threshold, float dropout_p, uint64_t seed, float* bucket,
                          float* prob, void* workspace, int64_t ws_bytes, void* stream) {
  using namespace hbk;
  if (!p) return arg_error("plan is NULL");
  if (batch < 0 || batch > (1 << 24)) return arg_error("batch out of range");
  if (!bucket || !workspace || !params) return arg_error("NULL pointer");
  hipStream_t s = as_stream(stream);
  HBK_HIP(hipMemsetAsync(bucket, 0, sizeof(float) * (p->n_params + kStats), s));
  if (batch == 0) return HBK_OK;
  if (!x || !y) return arg_error("NULL x/y");
  const Ws w = ws_layout(*p, batch);
  if (ws_bytes < w.total * int64_t(sizeof(float))) return arg_error("workspace too small");
  float* ws = static_cast<float*>(workspace);
  const int B = static_cast<int>(batch);
  if (dropout_p < 0.f || dropout_p >= 1.f) return arg_error("dropout_p must be in [0, 1)");
  HBK_RC(forward(*p, params, x, B, ws, w, dropout_p, seed, s, p->step_scalars));
  float* G = bucket;  // gradients, same layout as params
  float* stats = bucket + p->n_params;
  float* pr = prob ? prob : ws + w.prob;
  hipLaunchKernelGGL(loss_kernel, dim3(std::min<unsigned>((B + 255) / 256, 64)), dim3(256), 0, s, ws + w.z, y, pr,
                     ws + w.dz, stats, B, neg_weight, high_loss_threshold, activation_threshold, p->step_scalars);
  HBK_LAUNCH_CHECK("loss_kernel");
  // backward: dS = d(output of GMLP k) [B, out]
  const float* dS = ws + w.dz;  // [B,1] for mlp_out
  // rows per block of the column reductions (LN dgamma/dbeta, bias grads): ~256
  // blocks at the stage batch sizes (32 rows gave 35 blocks at B = 1100)
  const int rpb = std::max(4, (B + 255) / 256);
  const unsigned cs_grid = (B + rpb - 1) / rpb;
  float* bufA = ws + w.dtmp_a;
  float* bufB = ws + w.dtmp_b;
  for (int k = static_cast<int>(p->g.size()) - 1; k >= 0; --k) {
    const Gmlp& gm = p->g[k];
    const float* X = (k == 0) ? ws + w.xn_in : ws + w.xn[k - 1];
    // dW_o [out, H] = dS^T U ; db_o = colsum dS
    // (weight gradients accumulate into the bucket zeroed above: acc = true spares
    // split-K its own memset of C)
    HBK_RC((gemm<true, false>(dS, ws + w.u[k], G + gm.w_o, nullptr, gm.out, gm.hid, B, gm.out, gm.hid, gm.hid,
                              true, s)));
    hipLaunchKernelGGL(colsum_kernel, dim3(cs_grid), dim3(128), 0, s, dS, G + gm.b_o, B, gm.out, rpb);
    HBK_LAUNCH_CHECK("colsum_kernel");
    // dU [B, H] = dS W_o
    HBK_RC((gemm<false, false>(dS, params + gm.w_o, bufA, nullptr, B, gm.hid, gm.out, gm.out, gm.hid, gm.hid,
                               false, s)));
    hipLaunchKernelGGL(gate_bwd_kernel, dim3(ew_grid(int64_t(B) * gm.hid)), dim3(256), 0, s, bufA, ws + w.hg[k],
                       ws + w.dhg, B, gm.hid);
    HBK_LAUNCH_CHECK("gate_bwd_kernel");
    // dW_hg [2H, in] = dHG^T X ; db_hg = colsum dHG
    HBK_RC((gemm<true, false>(ws + w.dhg, X, G + gm.w_hg, nullptr, 2 * gm.hid, gm.in, B, 2 * gm.hid, gm.in,
                              gm.in, true, s)));
    hipLaunchKernelGGL(colsum_kernel, dim3(cs_grid), dim3(128), 0, s, ws + w.dhg, G + gm.b_hg, B, 2 * gm.hid, rpb);
    HBK_LAUNCH_CHECK("colsum_kernel");
    // dX [B, in] = dHG W_hg
    HBK_RC((gemm<false, false>(ws + w.dhg, params + gm.w_hg, bufB, nullptr, B, gm.in, 2 * gm.hid, 2 * gm.hid,
                               gm.in, gm.in, false, s)));
    // LayerNorm in front of this GMLP
    const Ln& l = (k == 0) ? p->ln_in : p->ln[k - 1];
    const float* xh = (k == 0) ? ws + w.xhat_in : ws + w.xhat[k - 1];
    const float* rs = (k == 0) ? ws + w.rstd_in : ws + w.rstd[k - 1];
    float* dx = (k == 0) ? nullptr : bufA;  // input-layer dX is not needed
    hipLaunchKernelGGL(ln_bwd_kernel, dim3(cs_grid), dim3(256), 0, s, bufB, xh, rs, params + l.g, dx, G + l.g,
                       G + l.b, B, l.d, rpb);
    HBK_LAUNCH_CHECK("ln_bwd_kernel");
    dS = bufA;
    std::swap(bufA, bufB);
  }
  return HBK_OK;
}

int hbk_mlp_set_step_scalars(hbk_mlp_plan* p, const double* dev_scalars) {
  if (!p) return hbk::arg_error("plan is NULL");
  p->step_scalars = dev_scalars;
  return HBK_OK;
}

int hbk_mlp_gate_adam(const hbk_mlp_plan* p, float* params, const float* bucket, float* m, float* v,
                      float* state, float* ctrl, float* history, int32_t history_cap, float lr, float beta1,
                      float beta2, float eps, void* stream) {
  using namespace hbk;
  if (!p || !params || !bucket || !m || !v || !state || !ctrl) return arg_error("NULL pointer");
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(gate_kernel, dim3(1), dim3(64), 0, s, bucket + p->n_params, state, ctrl, history,
                     history_cap, beta1, beta2);
  HBK_LAUNCH_CHECK("gate_kernel");
  hipLaunchKernelGGL(adam_kernel, dim3(ew_grid(p->n_params)), dim3(256), 0, s, params, bucket, m, v, ctrl,
                     p->n_params, lr, beta1, beta2, eps, p->step_scalars);
  HBK_LAUNCH_CHECK("adam_kernel");
  return HBK_OK;
}

int hbk_mlp_fused_supported(const hbk_mlp_plan* p, int32_t* supported) {
  if (!p || !supported) return hbk::arg_error("NULL");
  *supported = hbk::mlp_fused_supported(*p) ? 1 : 0;
  return HBK_OK;
}

int hbk_mlp_step_fwd_bwd(const hbk_mlp_plan* p, const float* params, const float* pool32, int64_t n32,
                         const void* pool16, int64_t n16, const int32_t* idx, int64_t idx_step_stride, const float* y, int64_t y_step_stride,
                         int64_t batch, const float* state, int32_t parity, const float* sched, int64_t sched_len,
                         float neg_weight, float high_loss_threshold, float activation_threshold, float dropout_p,
                         uint64_t seed, float* bucket, float* prob, int64_t idx_steps, int32_t flags,
                         void* workspace, int64_t ws_bytes, void* stream) {
  using namespace hbk;
  if (!p) return arg_error("plan is NULL");
  if (!mlp_fused_supported(*p)) {
    set_error("hbk: the fused train step covers d_in 1536, layer 96, hidden 64, <= 4 layers");
    return HBK_ERR_UNSUPPORTED;
  }
  if (batch <= 0 || batch > (1 << 22)) return arg_error("batch out of range");
  if (!params || !y || !bucket || !workspace || !state) return arg_error("NULL pointer");
  if (!idx && !pool32) return arg_error("no rows: idx and pool32 are NULL");
  if (parity != 0 && parity != 1) return arg_error("parity must be 0 or 1");
  if (sched && sched_len <= 0) return arg_error("sched_len must be > 0");
  if (dropout_p < 0.f || dropout_p >= 1.f) return arg_error("dropout_p must be in [0, 1)");
  if (ws_bytes < mlp_fused_ws_floats(*p, batch) * int64_t(sizeof(float))) return arg_error("workspace too small");
  if (n32 < 0 || n16 < 0) return arg_error("negative pool size");
  if (!idx && n32 < batch) return arg_error("idx NULL: pool32 must hold the batch rows");
  if (flags & ~(HBK_STEP_XHAT_READY | HBK_STEP_PREFETCH_NEXT | HBK_STEP_WEIGHTS_READY | HBK_STEP_DEFER_PARTIALS))
    return arg_error("unknown flags");
  if (!pool32 && !pool16) return arg_error("no embedding pool");
  return mlp_fused_run(*p, params, pool32, n32, pool16, n16, idx, idx_step_stride, idx_steps, y, y_step_stride,
                       static_cast<int>(batch), state, parity, sched,
                       static_cast<int>(std::min<int64_t>(sched_len, 1 << 30)), neg_weight, high_loss_threshold,
                       activation_threshold, dropout_p, seed, bucket, prob, nullptr, static_cast<float*>(workspace),
                       true, flags, as_stream(stream));
}

int hbk_mlp_step_update(const hbk_mlp_plan* p, float* params, float* bucket, float* m, float* v, float* state,
                        int32_t parity, const float* sched, int64_t sched_len, float lr, float beta1, float beta2,
                        float eps, float* history, int32_t history_cap, void* workspace, int64_t ws_bytes,
                        void* stream) {
  using namespace hbk;
  if (!p) return arg_error("plan is NULL");
  if (!params || !bucket || !m || !v || !state) return arg_error("NULL pointer");
  if (parity != 0 && parity != 1) return arg_error("parity must be 0 or 1");
  if (sched && sched_len <= 0) return arg_error("sched_len must be > 0");
  if (workspace && (!mlp_fused_supported(*p) || ws_bytes < mlp_fused_ws_floats(*p, 1) * int64_t(sizeof(float))))
    return arg_error("workspace: fused plans only, and at least the weight cache");
  return mlp_fused_update(*p, params, bucket, m, v, state, parity, sched,
                          static_cast<int>(std::min<int64_t>(sched_len, 1 << 30)), lr, beta1, beta2, eps, history,
                          history ? history_cap : 0, static_cast<float*>(workspace), as_stream(stream));
}

int hbk_mlp_eval_workspace_size(const hbk_mlp_plan* p, int64_t rows, int64_t* bytes) {
  using namespace hbk;
  if (!p || !bytes) return arg_error("NULL");
  if (!mlp_fused_supported(*p)) {
    set_error("hbk: the evaluation pass covers the fused plans (d_in 1536, layer 96, hidden 64, <= 4 layers)");
    return HBK_ERR_UNSUPPORTED;
  }
  *bytes = mlp_eval_ws_floats(*p, std::max<int64_t>(rows, 1)) * int64_t(sizeof(float));
  return HBK_OK;
}

int hbk_mlp_eval_prepare(const hbk_mlp_plan* p, const float* params, void* workspace, int64_t ws_bytes,
                         void* stream) {
  using namespace hbk;
  if (!p || !params || !workspace) return arg_error("NULL pointer");
  if (!mlp_fused_supported(*p)) {
    set_error("hbk: the evaluation pass covers the fused plans");
    return HBK_ERR_UNSUPPORTED;
  }
  if (ws_bytes < mlp_eval_ws_floats(*p, 1) * int64_t(sizeof(float))) return arg_error("workspace too small");
  return mlp_eval_prepare(*p, params, static_cast<float*>(workspace), as_stream(stream));
}

int hbk_mlp_eval_count(const hbk_mlp_plan* p, const float* params, const void* pool, int32_t pool_is_f16,
                       int64_t n_pool, const int32_t* idx, int64_t rows, int64_t row_offset, int32_t label,
                       float activation_threshold, float dropout_p, uint64_t seed, float* counts, float* prob,
                       void* workspace, int64_t ws_bytes, void* stream) {
  using namespace hbk;
  if (!p || !params || !workspace || !counts) return arg_error("NULL pointer");
  if (!mlp_fused_supported(*p)) {
    set_error("hbk: the evaluation pass covers the fused plans");
    return HBK_ERR_UNSUPPORTED;
  }
  if (rows < 0 || row_offset < 0 || rows + row_offset > (int64_t(1) << 31) / 768) return arg_error("rows out of range");
  if (rows == 0) return HBK_OK;
  if (!pool || n_pool <= 0) return arg_error("empty pool");
  if (label != 0 && label != 1) return arg_error("label must be 0 or 1");
  if (dropout_p < 0.f || dropout_p >= 1.f) return arg_error("dropout_p must be in [0, 1)");
  if (ws_bytes < mlp_eval_ws_floats(*p, rows) * int64_t(sizeof(float))) return arg_error("workspace too small");
  return mlp_eval_count(*p, params, pool, pool_is_f16 != 0, n_pool, idx, rows, row_offset, label,
                        activation_threshold, dropout_p, seed, counts, prob, static_cast<float*>(workspace),
                        as_stream(stream));
}

int hbk_mlp_eval_count_multi(const hbk_mlp_plan* p, const float* params, int32_t n_pools,
                             const void* const* pools, int32_t pools_are_f16, const int64_t* n_pool,
                             const int64_t* rows, const int64_t* row_offsets, const int32_t* labels,
                             const uint64_t* seeds, float* const* counts, float activation_threshold,
                             float dropout_p, void* workspace, int64_t ws_bytes, void* stream) {
  using namespace hbk;
  if (!p || !params || !workspace) return arg_error("NULL pointer");
  if (!mlp_fused_supported(*p)) {
    set_error("hbk: the evaluation pass covers the fused plans");
    return HBK_ERR_UNSUPPORTED;
  }
  if (n_pools < 0 || n_pools > kEvalMaxSeg) return arg_error("n_pools must be in [0, 4]");
  if (n_pools == 0) return HBK_OK;
  if (!pools || !n_pool || !rows || !row_offsets || !labels || !seeds || !counts) return arg_error("NULL array");
  if (dropout_p < 0.f || dropout_p >= 1.f) return arg_error("dropout_p must be in [0, 1)");
  EvalSeg seg[kEvalMaxSeg];
  int64_t max_rows = 0;
  for (int i = 0; i < n_pools; ++i) {
    if (rows[i] < 0 || row_offsets[i] < 0 || rows[i] + row_offsets[i] > (int64_t(1) << 31) / 768)
      return arg_error("rows out of range");
    if (rows[i] > 0 && (!pools[i] || n_pool[i] <= 0)) return arg_error("empty pool");
    if (labels[i] != 0 && labels[i] != 1) return arg_error("label must be 0 or 1");
    if (rows[i] > 0 && !counts[i]) return arg_error("counts is NULL");
    seg[i] = EvalSeg{pools[i], n_pool[i], rows[i], row_offsets[i], seeds[i], counts[i], labels[i]};
    max_rows = std::max(max_rows, rows[i]);
  }
  if (ws_bytes < mlp_eval_ws_floats(*p, max_rows) * int64_t(sizeof(float))) return arg_error("workspace too small");
  return mlp_eval_count_multi(*p, params, pools_are_f16 != 0, seg, n_pools, activation_threshold, dropout_p,
                              static_cast<float*>(workspace), as_stream(stream));
}

int hbk_mlp_eval_finish(const float* counts_val, const float* counts_test, const double* sizes,
                        float target_false_positives_per_hour, float adjust_ratio, float* sched, int64_t sched_len,
                        int64_t next_step, float* out, void* stream) {
  using namespace hbk;
  if (!sizes) return arg_error("sizes is NULL");
  if (sched && (sched_len <= 0 || next_step < 0)) return arg_error("schedule range");
  return mlp_eval_finish(counts_val, counts_test, sizes, target_false_positives_per_hour, adjust_ratio, sched,
                         sched_len, next_step, out, as_stream(stream));
}

}  // extern "C"
