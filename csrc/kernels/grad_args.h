// Arguments of the fused learner-gradient kernels (mlp_grad.hip, value_grad.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace rrl {

enum GradHead : int {
  HEAD_PG_CAT = 0,     // REINFORCE: loss = -mean(logp(a) * adv)
  HEAD_VALUE_MSE = 1,  // baseline: loss = mean((v - ret)^2)
  HEAD_PPO_CAT = 2,    // PPO clipped surrogate, categorical
  HEAD_PPO_GAUSS = 3,  // PPO clipped surrogate, diagonal Gaussian
  HEAD_PG_GAUSS = 4,   // REINFORCE / A2C with a Gaussian policy
};

struct GradArgs {
  const float* params;
  const float* X;  // [B][D]
  int B, D, A;
  const float* mask;       // [B][A] or null
  const int* act;          // [B]
  const float* actc;       // [B][A]
  const float* adv;        // [B]
  const float* ret;        // [B]
  const float* logp_old;   // [B] or null
  const float* adv_stats;  // [3] = {sum, sumsq, count} -> normalise adv, or null
  float inv_B;             // 1 / (global batch)
  float clip_eps;
  float ent_coef;
  float* grad_slab;  // [grid][P]
  float* loss_slab;  // [grid][8]
  int P;
  int tune = 0;      // value_grad.hip scheduling variant (set by its launcher)
  unsigned long long* stamps = nullptr;  // diagnostic stamp sums (value_grad.hip STAMP build)
  // Device-side batch shape (graph capture with a batch that changes between replays): rows
  // >= *nvalid are inert (no loss, zero gradient; B stays the allocated capacity the grid and
  // the clamped loads use), and *inv_B_dev replaces inv_B.  Null = the host values.
  const int* nvalid = nullptr;
  const float* inv_B_dev = nullptr;
  float* vout = nullptr;  // value forward (value_grad.hip FWD instance): V of every row
};

// Weight-stationary bf16x6 gradient kernels (value_grad.hip): value head for H = 128,
// D <= 24; categorical policy heads (PG / PPO) for H = 128, D <= 8, A = 2..4; Gaussian
// policy heads for H = 128, D <= 20, A = 1 or 6.
bool value_grad_split_supported(int D, int H);
int launch_value_grad_split(const GradArgs& a, int grid, hipStream_t s);
bool policy_grad_split_supported(int D, int H, int A, int head);
int launch_policy_grad_split(const GradArgs& a, int head, int grid, hipStream_t s);
// Value forward V(x) on the same weight-stationary bf16x6 layers (fp32-accurate), p.vout.
int launch_value_fwd_split(const GradArgs& a, int grid, hipStream_t s);

}  // namespace rrl
