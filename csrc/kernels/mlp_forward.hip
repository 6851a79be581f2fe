// Batched fused MLP forward + head (K1-K6, K16 of SURVEY §2.6).
//
// One launch evaluates a Linear-ReLU-Linear-ReLU-Linear net for B rows with the
// weights staged once per workgroup into LDS and the activations kept in registers
// (transposed MFMA tiles, see common.h).  The head runs in the epilogue:
//   MODE_VALUE      : v[b]                         (BaselineValueNetwork, kernel.py:78-84)
//   MODE_CAT_SAMPLE : act[b], logp[b], ent[b]      (step(), kernel.py:99-107 / 127-135)
//   MODE_CAT_EVAL   : logp[b | act], ent[b]        (forward(obs, mask, act), kernel.py:39-46)
//   MODE_LOGITS     : logits[b][A] (masked)        (debug / oracle checks)
//   MODE_GAUSS_SAMPLE / MODE_GAUSS_EVAL: continuous policy (the reference's incomplete
//                     ContinuousPolicyNetwork, kernel.py:49-75, completed).
#include "common.h"
#include "grad_args.h"
#include "heads.h"

namespace rrl {

enum FwdMode : int {
  MODE_VALUE = 0,
  MODE_CAT_SAMPLE = 1,
  MODE_CAT_EVAL = 2,
  MODE_LOGITS = 3,
  MODE_GAUSS_SAMPLE = 4,
  MODE_GAUSS_EVAL = 5,
};

struct FwdArgs {
  const float* params;
  const float* X;        // [B][D]
  int B, D, A, H;
  const float* mask;     // [B][A] or null
  const int* act_in;     // [B] (CAT_EVAL)
  const float* actc_in;  // [B][A] (GAUSS_EVAL)
  int* act_out;          // [B]
  float* actc_out;       // [B][A]
  float* out0;           // v / logp
  float* out1;           // entropy (may be null)
  float* logits_out;     // [B][A] (MODE_LOGITS) or mean for Gaussian (may be null)
  uint32_t seed_lo, seed_hi;
  uint32_t step_lo, step_hi;
  uint32_t row_offset;   // stream id of row 0 (global env index)
  const float* gate;     // MODE_VALUE: [B] done codes; only 16-row tiles holding a code 2
                         // (time-limit truncation) are evaluated, or null = every row
  // host-env rollout (runtime/host_rollout.cpp): X may be PINNED HOST memory read over PCIe
  // (zero-copy); x_copy gets the rows in HBM for the learner and act_host / actc_host the
  // sampled actions in pinned host memory for the env threads -- one launch per half-step,
  // no H2D / D2H copies.  All null on the ordinary path.
  float* x_copy;         // [B][D] or null
  int* act_host;         // [B] or null (CAT_SAMPLE)
  float* actc_host;      // [B][A] or null (GAUSS_SAMPLE)
};

template <int DT, int HT, int MODE>
__global__ __launch_bounds__(256, 2) void mlp_forward_kernel(FwdArgs p) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  using L = LdsNet<DT, HT>;
  constexpr int H = L::H;
  const bool gauss = (MODE == MODE_GAUSS_SAMPLE || MODE == MODE_GAUSS_EVAL);
  const int A = (MODE == MODE_VALUE) ? 1 : p.A;
  stage_net<DT, HT>(lds, p.params, p.D, A, gauss);
  __syncthreads();

  const int l = lane_id();
  const int j = l & 15, g = l >> 4;
  const int waves_per_block = blockDim.x >> 6;
  const int wave = (threadIdx.x >> 6) + blockIdx.x * waves_per_block;
  const int total_waves = gridDim.x * waves_per_block;
  const int ntiles = (p.B + kTileB - 1) / kTileB;

  for (int tile = wave; tile < ntiles; tile += total_waves) {
    const int row0 = tile * kTileB;
    const int nrows = min(kTileB, p.B - row0);
    const int row = row0 + j;
    const bool valid = j < nrows;
    if (MODE == MODE_VALUE && p.gate != nullptr) {
      // truncation bootstraps are rare (CartPole: one per 500 steps): skip tiles without one
      if (__ballot(valid && p.gate[row] > 1.5f) == 0) continue;
    }

    floatx4 x[DT], h1[HT], h2[HT];
    load_x_tile<DT>(p.X, p.D, p.D, row0, nrows, x);
    if (p.x_copy != nullptr && valid) {  // every (row, feature) is held by exactly one lane
      float* xr = p.x_copy + (size_t)row * p.D;
#pragma unroll
      for (int t = 0; t < DT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int f = 16 * t + 4 * r + g;
          if (f < p.D) xr[f] = x[t][r];
        }
    }
    dense_fwd<DT, HT, true>(lds + L::W1, L::S1, lds + L::B1, x, h1, input_kr_last(p.D, DT));
    dense_fwd<HT, HT, true>(lds + L::W2, L::S2, lds + L::B2, h1, h2);

    if (MODE == MODE_VALUE) {
      const float v = head_dot<HT>(lds + L::W3, lds[L::B3], h2);
      if (valid && g == 0) p.out0[row] = v;
    } else if (MODE == MODE_CAT_SAMPLE || MODE == MODE_CAT_EVAL || MODE == MODE_LOGITS) {
      float logits[kMaxAct];
      policy_logits<HT>(lds + L::W3, lds + L::B3, A, H, h2, logits);
      if (valid) apply_mask(p.mask ? p.mask + (size_t)row * A : nullptr, A, logits);
      const CatStats cs = cat_stats(A, logits);
      if (MODE == MODE_LOGITS) {
        if (valid) {
          // lane group g writes actions g, g+4, g+8, g+12
#pragma unroll
          for (int a = 0; a < kMaxAct; ++a)
            if (a < A && (a & 3) == g) p.logits_out[(size_t)row * A + a] = logits[a];
        }
      } else if (MODE == MODE_CAT_SAMPLE) {
        const uint4 rnd = philox4x32(make_uint4(p.row_offset + (uint32_t)row, p.step_lo, p.step_hi, 0u),
                                     make_uint2(p.seed_lo, p.seed_hi));
        const int a = cat_sample(A, logits, cs.lse, u01(rnd.x));
        if (valid && g == 0) {
          p.act_out[row] = a;
          if (p.act_host != nullptr) p.act_host[row] = a;
          p.out0[row] = pick_logit(A, logits, a) - cs.lse;
          if (p.out1) p.out1[row] = cs.entropy;
        }
      } else {
        const int a = valid ? p.act_in[row] : 0;
        if (valid && g == 0) {
          p.out0[row] = pick_logit(A, logits, a) - cs.lse;
          if (p.out1) p.out1[row] = cs.entropy;
        }
      }
    } else {  // Gaussian
      float lp = 0.f, ent = 0.f;
      uint4 rnd = make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int a = 0; a < kMaxAct; ++a) {
        if (a < A) {
          const float mu = head_dot<HT>(lds + L::W3 + a * H, lds[L::B3 + a], h2);
          const float ls = lds[L::LOGSTD + a];
          const float sd = __expf(ls);
          float xa;
          if (MODE == MODE_GAUSS_SAMPLE) {
            if ((a & 1) == 0)
              rnd = philox4x32(make_uint4(p.row_offset + (uint32_t)row, p.step_lo, p.step_hi, 16u + (uint32_t)a),
                               make_uint2(p.seed_lo, p.seed_hi));
            // Box-Muller on (rnd.x, rnd.y) / (rnd.z, rnd.w)
            const float u1 = fmaxf(u01((a & 1) ? rnd.z : rnd.x), 1e-7f);
            const float u2 = u01((a & 1) ? rnd.w : rnd.y);
            const float z = sqrtf(-2.f * __logf(u1)) * __cosf(6.2831853071795864f * u2);
            xa = mu + sd * z;
            if (valid && g == 0) {
              p.actc_out[(size_t)row * A + a] = xa;
              if (p.actc_host != nullptr) p.actc_host[(size_t)row * A + a] = xa;
            }
          } else {
            xa = valid ? p.actc_in[(size_t)row * A + a] : mu;
          }
          const float zz = (xa - mu) / sd;
          lp += -0.5f * zz * zz - ls - kHalfLog2Pi;
          ent += 0.5f + kHalfLog2Pi + ls;
          if (p.logits_out && valid && g == 0) p.logits_out[(size_t)row * A + a] = mu;
        }
      }
      if (valid && g == 0) {
        p.out0[row] = lp;
        if (p.out1) p.out1[row] = ent;
      }
    }
  }
}

}  // namespace rrl

using namespace rrl;

template <int DT, int HT, int MODE>
static int launch_fwd(const FwdArgs& a, int grid, hipStream_t s) {
  using L = LdsNet<DT, HT>;
  const int A = (MODE == MODE_VALUE) ? 1 : a.A;
  const size_t lds = (size_t)L::floats(A) * sizeof(float);
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)mlp_forward_kernel<DT, HT, MODE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              163840);
    attr_set = true;
  }
  hipLaunchKernelGGL((mlp_forward_kernel<DT, HT, MODE>), dim3(grid), dim3(256), lds, s, a);
  return (int)hipGetLastError();
}

template <int DT, int HT>
static int dispatch_mode(int mode, const FwdArgs& a, int grid, hipStream_t s) {
  switch (mode) {
    case MODE_VALUE: return launch_fwd<DT, HT, MODE_VALUE>(a, grid, s);
    case MODE_CAT_SAMPLE: return launch_fwd<DT, HT, MODE_CAT_SAMPLE>(a, grid, s);
    case MODE_CAT_EVAL: return launch_fwd<DT, HT, MODE_CAT_EVAL>(a, grid, s);
    case MODE_LOGITS: return launch_fwd<DT, HT, MODE_LOGITS>(a, grid, s);
    case MODE_GAUSS_SAMPLE: return launch_fwd<DT, HT, MODE_GAUSS_SAMPLE>(a, grid, s);
    case MODE_GAUSS_EVAL: return launch_fwd<DT, HT, MODE_GAUSS_EVAL>(a, grid, s);
  }
  return -1;
}

extern "C" int rrl_set_value_grad_mode(int mode);  // mlp_grad.hip (-1 queries)

// Value forward on the bf16x6 weight-stationary kernel (value_grad.hip FWD instance, ~0.6x the
// fp32-MFMA kernel's time at H = 128) -- 1 -- or the fp32-MFMA kernel below -- 0.  The split
// kernel also needs the bf16x6 gradient mode (rrl_set_value_grad_mode 1).
static int g_value_fwd_mode = 1;
extern "C" int rrl_set_value_fwd_mode(int mode) {
  const int old = g_value_fwd_mode;
  if (mode == 0 || mode == 1) g_value_fwd_mode = mode;
  return old;
}

extern "C" int rrl_mlp_forward(int mode, const float* params, const float* X, int B, int D, int A,
                               int H, const float* mask, const int* act_in, const float* actc_in,
                               int* act_out, float* actc_out, float* out0, float* out1,
                               float* logits_out, uint64_t seed, uint64_t step, uint32_t row_offset,
                               const float* gate, float* x_copy, int* act_host, float* actc_host, int num_cu,
                               void* stream) {
  if (B <= 0) return 0;
  if (A < 1 || A > kMaxAct || D < 1 || D > 32) return -2;
  FwdArgs a{params, X, B, D, A, H, mask, act_in, actc_in, act_out, actc_out, out0, out1, logits_out,
            (uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)step, (uint32_t)(step >> 32), row_offset, gate,
            x_copy, act_host, actc_host};
  if (mode == MODE_VALUE && gate == nullptr && x_copy == nullptr && H == 128 && D <= 24 && g_value_fwd_mode == 1 &&
      rrl_set_value_grad_mode(-1) == 1) {
    GradArgs g{};
    g.params = params;
    g.X = X;
    g.B = B;
    g.D = D;
    g.A = 1;
    g.vout = out0;
    int sg = (B + 63) / 64;
    const int scap = num_cu > 0 ? num_cu : 256;
    if (sg > scap) sg = scap;
    return launch_value_fwd_split(g, sg, (hipStream_t)stream);
  }
  const int tiles = (B + kTileB - 1) / kTileB;
  const int waves_needed = tiles;
  int grid = (waves_needed + 3) / 4;
  const int cap = 2 * (num_cu > 0 ? num_cu : 256);
  if (grid > cap) grid = cap;
  hipStream_t s = (hipStream_t)stream;
  const int DT = (D <= 16) ? 1 : 2;
  if (H == 128) return DT == 1 ? dispatch_mode<1, 8>(mode, a, grid, s) : dispatch_mode<2, 8>(mode, a, grid, s);
  if (H == 64) return DT == 1 ? dispatch_mode<1, 4>(mode, a, grid, s) : dispatch_mode<2, 4>(mode, a, grid, s);
  return -3;
}
