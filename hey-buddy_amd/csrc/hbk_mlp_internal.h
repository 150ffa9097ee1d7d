// The classifier plan shared by hbk_mlp.hip (generic GEMM path, any dims) and
// hbk_mlp_fused.hip (fused train step for the default architecture).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

namespace hbk {

struct Gmlp {
  int in, hid, out;
  int64_t w_hg, b_hg, w_o, b_o;  // float offsets into the flat parameter buffer
};
struct Ln {
  int d;
  int64_t g, b;
};

}  // namespace hbk

struct hbk_mlp_plan {
  int d_in = 0, layer = 0, hid = 0, n_layers = 0;
  hbk::Ln ln_in;
  std::vector<hbk::Gmlp> g;  // mlp_in, layers..., mlp_out
  std::vector<hbk::Ln> ln;   // layers' LNs..., norm_out
  int64_t n_params = 0;
  // hbk_mlp_set_step_scalars: device [lr, neg_weight, seed] read by the train
  // kernels in place of their by-value arguments (graph-captured steps)
  const double* step_scalars = nullptr;
  // hbk_mlp_step_fwd_bwd with HBK_STEP_DEFER_PARTIALS left its weight-gradient
  // slabs (deferred_ks of them) in this workspace for the next hbk_mlp_step_update
  mutable const void* deferred_ws = nullptr;
  mutable int deferred_ks = 0;
};

namespace hbk {
// Counter-based uniform in [0, 1) (splitmix64 of seed ^ index): the input
// dropout mask of element i of a step is a pure function of (seed, i).
__device__ __forceinline__ float uniform01(uint64_t seed, uint64_t i) {
  uint64_t z = seed + 0x9E3779B97F4A7C15ull * (i + 1);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return static_cast<float>(z >> 40) * (1.f / 16777216.f);
}

// Adam's parameter step, torch's step_size * m / (sqrt(v) / bc2s + eps), on the
// hardware v_sqrt_f32 / v_rcp_f32 (1 ulp each) instead of the IEEE square root
// and two IEEE divisions; shared by k4 and the generic adam_kernel so that the
// two update paths stay bit-identical (k4: 12.0 -> 10.9 us per step on 64 CUs)
__device__ __forceinline__ float adam_step(float mi, float vi, float step_size, float inv_bc2s, float eps) {
  return step_size * mi * __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(vi) * inv_bc2s + eps);
}

// True when the fused kernels of hbk_mlp_fused.hip cover this plan.
bool mlp_fused_supported(const hbk_mlp_plan& p);
int64_t mlp_fused_ws_floats(const hbk_mlp_plan& p, int64_t B);
int mlp_fused_run(const hbk_mlp_plan& p, const float* params, const float* pool32, int64_t n32,
                  const void* pool16, int64_t n16, const int32_t* idx, int64_t idx_stride, int64_t idx_steps,
                  const float* y, int64_t y_stride, int B, const float* state, int parity, const float* sched,
                  int sched_len, float neg_weight, float thr, float act_thr, float drop_p, uint64_t seed,
                  float* bucket, float* prob, float* logit, float* ws, bool train, int flags, hipStream_t s);
int mlp_fused_update(const hbk_mlp_plan& p, float* params, float* bucket, float* m, float* v, float* state,
                     int parity, const float* sched, int sched_len, float lr, float b1, float b2, float eps,
                     float* hist, int hist_cap, float* ws, hipStream_t s);
// Evaluation passes (validation / testing forwards reduced to prediction counts)
int64_t mlp_eval_ws_floats(const hbk_mlp_plan& p, int64_t rows);
int mlp_eval_prepare(const hbk_mlp_plan& p, const float* params, float* ws, hipStream_t s);
int mlp_eval_count(const hbk_mlp_plan& p, const float* params, const void* pool, bool f16, int64_t n_pool,
                   const int32_t* idx, int64_t rows, int64_t r0, int label, float act_thr, float drop_p,
                   uint64_t seed, float* counts, float* prob, float* ws, hipStream_t s);
// one pool of an evaluation launch (mlp_eval_count_multi: several pools of one dtype in one launch)
struct EvalSeg {
  const void* pool;
  int64_t n_pool, rows, r0;
  uint64_t seed;
  float* counts;
  int label;
};
constexpr int kEvalMaxSeg = 4;
int mlp_eval_count_multi(const hbk_mlp_plan& p, const float* params, bool f16, const EvalSeg* seg, int nseg,
                         float act_thr, float drop_p, float* ws, hipStream_t s);
int mlp_eval_finish(const float* cv, const float* ct, const double* sizes, float target, float ratio, float* sched,
                    int64_t sched_len, int64_t next_step, float* out, hipStream_t s);
}  // namespace hbk
