// Partial-gradient slab reduction + fused multi-tensor Adam over one flat fp32
// parameter buffer (K13 of SURVEY §2.6; reference uses torch.optim.Adam with default
// betas (0.9, 0.999), eps 1e-8 over the policy and value nets, REINFORCE.py:47-50).
//
// The step counter lives on the device so that an optimisation loop (e.g. the 80
// value iterations, REINFORCE.py:110-115) can be captured into one hipGraph: every
// block reads the counter s0 and uses t = s0 + step_add + 1; the last block to finish
// (arrival ticket) sets the counter to s0 + step_inc.  A loop of K updates passes
// step_add = k and step_inc = 0 (no ticket at all) for k < K - 1 and step_inc = K on the last
// one: the ticket's 271-way serialised device-scope atomic (~3 us at the end of every update,
// MI355X_MICROARCH.md fanin) is paid once per loop instead of once per update.
#include "common.h"

namespace rrl {

struct AdamArgs {
  float* param;
  float* m;
  float* v;
  const float* grad;  // [P] flat gradient, or null when reducing slabs
  const float* slab;  // [nslab][P] partial gradients
  int nslab;
  float* grad_out;    // optional: write the reduced gradient here
  int* step;          // device step counter
  unsigned* ticket;   // device arrival counter (zeroed by the last block); null: step_inc == 0
  int P;
  int step_add, step_inc;
  float lr, beta1, beta2, eps, grad_scale, weight_decay;
};

// Block = 64 parameters x 16 slab groups (1024 threads): the slab sum is split over
// 16 waves (coalesced 256-B rows per wave-load) and combined through LDS, so reducing
// ~256 slabs of a 17k-parameter net is bandwidth- not latency-bound (was 23 us).
constexpr int kAdamCols = 64;
constexpr int kAdamGroups = 16;

// Partial sum of column p over the slabs k = grp, grp + 16, ... (one of 16 groups).  Up to 8
// loads in flight per thread: at the small-batch value step (128 slabs, 8 per thread) the
// whole sum is one HBM latency instead of two.
RRL_DEV float slab_group_sum(const float* __restrict__ slab, int nslab, int P, int p, int grp) {
  const float* s = slab + p;
  float g = 0.f;
  int k = grp;
  for (; k + 7 * kAdamGroups < nslab; k += 8 * kAdamGroups) {
    float q[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) q[i] = s[(size_t)(k + i * kAdamGroups) * P];
    g += ((q[0] + q[1]) + (q[2] + q[3])) + ((q[4] + q[5]) + (q[6] + q[7]));
  }
  if (k + 3 * kAdamGroups < nslab) {
    const float g0 = s[(size_t)k * P], g1 = s[(size_t)(k + kAdamGroups) * P];
    const float g2 = s[(size_t)(k + 2 * kAdamGroups) * P], g3 = s[(size_t)(k + 3 * kAdamGroups) * P];
    g += (g0 + g1) + (g2 + g3);
    k += 4 * kAdamGroups;
  }
  for (; k < nslab; k += kAdamGroups) g += s[(size_t)k * P];
  return g;
}

__global__ __launch_bounds__(1024) void adam_kernel(AdamArgs a) {
  __shared__ float part[kAdamGroups][kAdamCols];
  const int s0 = *a.step;
  const int t = s0 + a.step_add + 1;
  const int col = threadIdx.x & (kAdamCols - 1);
  const int grp = threadIdx.x / kAdamCols;
  const int p = blockIdx.x * kAdamCols + col;
  // the update's own operands are loaded before the slab sum, so their latency hides under it
  float w = 0.f, m0 = 0.f, v0 = 0.f;
  if (grp == 0 && p < a.P) {
    w = a.param[p];
    m0 = a.m[p];
    v0 = a.v[p];
  }
  float g = 0.f;
  if (p < a.P) {
    if (a.grad) {
      if (grp == 0) g = a.grad[p];
    } else {
      g = slab_group_sum(a.slab, a.nslab, a.P, p, grp);
    }
  }
  part[grp][col] = g;
  __syncthreads();
  if (grp == 0 && p < a.P) {
    float gs = 0.f;
#pragma unroll
    for (int q = 0; q < kAdamGroups; ++q) gs += part[q][col];
    gs *= a.grad_scale;
    if (a.grad_out) a.grad_out[p] = gs;
    const float bc1 = 1.f - __powf(a.beta1, (float)t);
    const float bc2 = 1.f - __powf(a.beta2, (float)t);
    if (a.weight_decay != 0.f) gs += a.weight_decay * w;
    const float m = a.beta1 * m0 + (1.f - a.beta1) * gs;
    const float v = a.beta2 * v0 + (1.f - a.beta2) * gs * gs;
    a.m[p] = m;
    a.v[p] = v;
    // torch.optim.Adam: p -= lr/bc1 * m / (sqrt(v)/sqrt(bc2) + eps)
    w -= (a.lr / bc1) * m / (sqrtf(v) * rsqrtf(bc2) + a.eps);
    a.param[p] = w;
  }
  // arrival ticket: the last block bumps the step counter (every block read `step`
  // above, before its __syncthreads / ticket)
  if (a.ticket && threadIdx.x == 0) {
    const unsigned prev = atomicAdd(a.ticket, 1u);
    if (prev == gridDim.x - 1) {
      *a.ticket = 0u;
      *a.step = s0 + a.step_inc;
    }
  }
}

// Plain slab reduction (used before a data-parallel all-reduce): the same 64-column x
// 16-group layout as the Adam kernel (the per-thread serial loop over ~256 slabs it
// replaces was latency-bound, and runs once per optimiser step when world > 1).
__global__ __launch_bounds__(1024) void reduce_slabs_kernel(const float* slab, int nslab, int P, float scale,
                                                            float* out) {
  __shared__ float part[kAdamGroups][kAdamCols];
  const int col = threadIdx.x & (kAdamCols - 1);
  const int grp = threadIdx.x / kAdamCols;
  const int p = blockIdx.x * kAdamCols + col;
  part[grp][col] = p < P ? slab_group_sum(slab, nslab, P, p, grp) : 0.f;
  __syncthreads();
  if (grp == 0 && p < P) {
    float gs = 0.f;
#pragma unroll
    for (int q = 0; q < kAdamGroups; ++q) gs += part[q][col];
    out[p] = gs * scale;
  }
}

}  // namespace rrl

using namespace rrl;

extern "C" int rrl_adam(float* param, float* m, float* v, const float* grad, const float* slab, int nslab,
                        float* grad_out, int* step, unsigned* ticket, int P, float lr, float beta1,
                        float beta2, float eps, float grad_scale, float weight_decay, int step_add, int step_inc,
                        void* stream) {
  if (step_inc != 0 && ticket == nullptr) return -1;
  AdamArgs a{param, m, v, grad, slab, nslab, grad_out, step, step_inc != 0 ? ticket : nullptr, P, step_add,
             step_inc, lr, beta1, beta2, eps, grad_scale, weight_decay};
  const int grid = (P + kAdamCols - 1) / kAdamCols;
  hipLaunchKernelGGL(adam_kernel, dim3(grid < 1 ? 1 : grid), dim3(kAdamCols * kAdamGroups), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

extern "C" int rrl_reduce_slabs(const float* slab, int nslab, int P, float scale, float* out, void* stream) {
  const int grid = (P + kAdamCols - 1) / kAdamCols;
  hipLaunchKernelGGL(reduce_slabs_kernel, dim3(grid < 1 ? 1 : grid), dim3(kAdamCols * kAdamGroups), 0,
                     (hipStream_t)stream, slab, nslab, P, scale, out);
  return (int)hipGetLastError();
}
