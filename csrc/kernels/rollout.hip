// Fused on-device actor: T steps of {policy MLP forward -> masked softmax -> Philox
// categorical sample -> log-prob -> env physics -> auto-reset} for N vectorised envs
// in ONE launch, writing a time-major SoA rollout into HBM.
//
// This replaces the reference's per-step agent path (request_for_action ->
// TorchScript step() at batch 1 -> safetensors encode -> ZMQ push; SURVEY §3.3,
// agent_zmq.rs:458-571) for the on-GPU actor.  Each wave owns 16 envs; every lane
// of an env column keeps a replica of that env's state in registers, so the whole
// step needs no cross-lane traffic except the two head reductions.
#include "common.h"
#include "heads.h"
#include "envs.h"

namespace rrl {

struct RolloutArgs {
  const float* params;
  int N, T, H;
  float* state;     // [N][NS]
  int* ep_len;      // [N]
  float* ep_ret;    // [N]
  float* obs_buf;   // [T+1][N][D]
  int* act_buf;     // [T][N]
  float* logp_buf;  // [T][N]
  float* rew_buf;   // [T][N]
  float* done_buf;  // [T][N]: 0 running, 1 terminal, 2 time-limit truncation (needs tobs_buf)
  float* tobs_buf;  // [T][N][D] pre-reset observation where done == 2, or null (truncation -> 1)
  float* ep_stats;  // [grid][8]: n_done, sum_ret, sumsq_ret, max_ret, min_ret, sum_len
  uint32_t seed_lo, seed_hi;
  uint32_t step_lo, step_hi;  // global step of t = 0 (RNG counter)
  int reset_all;
  int max_steps;
};

template <class Env, int HT>
__global__ __launch_bounds__(256, 2) void rollout_kernel(RolloutArgs p) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int DT = 1;
  using L = LdsNet<DT, HT>;
  constexpr int H = L::H;
  constexpr int D = Env::D, A = Env::A, NS = Env::NS;
  static_assert(D <= 16, "device envs use one input tile");
  stage_net<DT, HT>(lds, p.params, D, A, false);
  __syncthreads();

  const int l = lane_id();
  const int j = l & 15, g = l >> 4;
  const int wave_in_block = threadIdx.x >> 6;
  const int waves_per_block = blockDim.x >> 6;
  const int wave = wave_in_block + blockIdx.x * waves_per_block;
  const int total_waves = gridDim.x * waves_per_block;
  const int ntiles = (p.N + kTileB - 1) / kTileB;
  const uint2 key = make_uint2(p.seed_lo, p.seed_hi);
  const uint64_t step0 = ((uint64_t)p.step_hi << 32) | p.step_lo;

  float st_n = 0.f, st_sum = 0.f, st_sq = 0.f, st_max = -INFINITY, st_min = INFINITY, st_len = 0.f;

  for (int tile = wave; tile < ntiles; tile += total_waves) {
    const int env = tile * kTileB + j;
    const bool valid = env < p.N;
    const int envc = valid ? env : p.N - 1;
    float s[NS];
    int len;
    float ret;
    if (p.reset_all) {
      const uint4 r = philox4x32(make_uint4((uint32_t)envc, (uint32_t)step0, (uint32_t)(step0 >> 32), 1u), key);
      Env::reset(s, r);
      len = 0;
      ret = 0.f;
    } else {
#pragma unroll
      for (int k = 0; k < NS; ++k) s[k] = p.state[(size_t)envc * NS + k];
      len = p.ep_len[envc];
      ret = p.ep_ret[envc];
    }

    for (int t = 0; t < p.T; ++t) {
      const uint64_t gstep = step0 + (uint64_t)t;
      const size_t base = (size_t)t * p.N + env;
      // observation tile, interleaved layout: feature f of env j lives in lane group
      // f&3, register f>>2 (so the 4 CartPole features are ONE MFMA k-step)
      floatx4 x[1];
      x[0] = zero4();
#pragma unroll
      for (int f = 0; f < D; ++f) {
        const float o = Env::obs(s, f);
        if ((f & 3) == g) x[0][f >> 2] = o;
      }
      if (valid) {
#pragma unroll
        for (int f = 0; f < D; ++f)
          if ((f & 3) == g) p.obs_buf[base * D + f] = x[0][f >> 2];
      }
      floatx4 h1[HT], h2[HT];
      dense_fwd<DT, HT, true>(lds + L::W1, L::S1, lds + L::B1, x, h1, (D + 3) >> 2);
      dense_fwd<HT, HT, true>(lds + L::W2, L::S2, lds + L::B2, h1, h2);
      float logits[kMaxAct];
      policy_logits<HT>(lds + L::W3, lds + L::B3, A, H, h2, logits);
      const CatStats cs = cat_stats(A, logits);
      const uint4 rnd = philox4x32(make_uint4((uint32_t)envc, (uint32_t)gstep, (uint32_t)(gstep >> 32), 0u), key);
      const int a = cat_sample(A, logits, cs.lse, u01(rnd.x));
      const float logp = pick_logit(A, logits, a) - cs.lse;

      bool term;
      const float r = Env::step(s, a, term, u01(rnd.y));
      len += 1;
      ret += r;
      const bool trunc = len >= p.max_steps;
      const bool done = term || trunc;
      const bool boot = trunc && !term && p.tobs_buf != nullptr;  // cut path: bootstrap V(s_t+1)
      if (valid && g == 0) {
        p.act_buf[base] = a;
        p.logp_buf[base] = logp;
        p.rew_buf[base] = r;
        p.done_buf[base] = boot ? 2.f : (done ? 1.f : 0.f);
      }
      if (boot && valid) {
#pragma unroll
        for (int f = 0; f < D; ++f)
          if ((f & 3) == g) p.tobs_buf[base * D + f] = Env::obs(s, f);
      }
      if (done) {
        if (valid && g == 0) {
          st_n += 1.f;
          st_sum += ret;
          st_sq += ret * ret;
          st_max = fmaxf(st_max, ret);
          st_min = fminf(st_min, ret);
          st_len += (float)len;
        }
        const uint4 rr = philox4x32(make_uint4((uint32_t)envc, (uint32_t)gstep, (uint32_t)(gstep >> 32), 1u), key);
        Env::reset(s, rr);
        len = 0;
        ret = 0.f;
      }
    }
    // final observation (bootstrap row T) and persistent env state
    if (valid) {
      const size_t base = (size_t)p.T * p.N + env;
#pragma unroll
      for (int f = 0; f < D; ++f)
        if ((f & 3) == g) p.obs_buf[base * D + f] = Env::obs(s, f);
      if (g == 0) {
#pragma unroll
        for (int k = 0; k < NS; ++k) p.state[(size_t)env * NS + k] = s[k];
        p.ep_len[env] = len;
        p.ep_ret[env] = ret;
      }
    }
  }

  // workgroup reduction of episode statistics
  __syncthreads();
  float* red = lds;  // weights no longer needed
  float v0 = wave_sum(st_n), v1 = wave_sum(st_sum), v2 = wave_sum(st_sq), v5 = wave_sum(st_len);
  float v3 = st_max, v4 = st_min;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    v3 = fmaxf(v3, __shfl_xor(v3, o, 64));
    v4 = fminf(v4, __shfl_xor(v4, o, 64));
  }
  if (l == 0) {
    red[wave_in_block * 8 + 0] = v0;
    red[wave_in_block * 8 + 1] = v1;
    red[wave_in_block * 8 + 2] = v2;
    red[wave_in_block * 8 + 3] = v3;
    red[wave_in_block * 8 + 4] = v4;
    red[wave_in_block * 8 + 5] = v5;
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    const int q = threadIdx.x;
    float v = red[q];
    for (int w = 1; w < waves_per_block; ++w) {
      const float u = red[w * 8 + q];
      v = (q == 3) ? fmaxf(v, u) : (q == 4) ? fminf(v, u) : v + u;
    }
    p.ep_stats[blockIdx.x * 8 + q] = v;
  }
}

// ------------------------------------------------------------------ small-N variant
// rollout_kernel gives each wave 16 envs and a whole 128x128 layer per step, so a short
// rollout over few envs (the time-to-threshold config: 1,024 envs = 64 tiles) runs 64 long
// serial chains on 16 CUs.  Here a workgroup's WPT = 4 waves share ONE 16-env tile: every
// wave keeps the env replica and the full layer 1 (HT MFMAs), computes HT/WPT output tiles of layer 2 and their partial logits, and the partials meet in LDS
// (double-buffered by step parity: one barrier per step).  All waves then sum the WPT
// partials in the same order, so they draw the same action and step identical env
// replicas; wave 0 writes.  Measured at 1,024 envs x 64 steps: 340 us (rollout_kernel),
// 166 us (4 waves per tile), 187 us (8 waves per tile: the per-step barrier and the
// redundant layer 1 outweigh the shorter layer-2 slice).
template <class Env, int HT, int WPT>
__global__ __launch_bounds__(64 * WPT, 1) void rollout_wide_kernel(RolloutArgs p) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int DT = 1;
  using L = LdsNet<DT, HT>;
  constexpr int H = L::H;
  constexpr int D = Env::D, A = Env::A, NS = Env::NS;
  constexpr int QT = HT / WPT;  // layer-2 output tiles per wave
  static_assert(D <= 16 && HT % WPT == 0, "one input tile, layer 2 split over the tile's waves");
  stage_net<DT, HT>(lds, p.params, D, A, false);
  float* part = lds + ((L::floats(A) + 3) & ~3);  // [2 parity][WPT waves][kMaxAct][16 envs]
  __syncthreads();

  const int l = lane_id();
  const int j = l & 15, g = l >> 4;
  const int w = threadIdx.x >> 6;
  const int to0 = w * QT;
  const int ntiles = (p.N + kTileB - 1) / kTileB;
  const uint2 key = make_uint2(p.seed_lo, p.seed_hi);
  const uint64_t step0 = ((uint64_t)p.step_hi << 32) | p.step_lo;
  const bool writer = (w == 0) && (g == 0);
  int parity = 0;

  float st_n = 0.f, st_sum = 0.f, st_sq = 0.f, st_max = -INFINITY, st_min = INFINITY, st_len = 0.f;

  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int env = tile * kTileB + j;
    const bool valid = env < p.N;
    const int envc = valid ? env : p.N - 1;
    float s[NS];
    int len;
    float ret;
    if (p.reset_all) {
      const uint4 r = philox4x32(make_uint4((uint32_t)envc, (uint32_t)step0, (uint32_t)(step0 >> 32), 1u), key);
      Env::reset(s, r);
      len = 0;
      ret = 0.f;
    } else {
#pragma unroll
      for (int k = 0; k < NS; ++k) s[k] = p.state[(size_t)envc * NS + k];
      len = p.ep_len[envc];
      ret = p.ep_ret[envc];
    }

    for (int t = 0; t < p.T; ++t) {
      const uint64_t gstep = step0 + (uint64_t)t;
      const size_t base = (size_t)t * p.N + env;
      floatx4 x[1];
      x[0] = zero4();
#pragma unroll
      for (int f = 0; f < D; ++f) {
        const float o = Env::obs(s, f);
        if ((f & 3) == g) x[0][f >> 2] = o;
      }
      if (valid && w == 0) {
#pragma unroll
        for (int f = 0; f < D; ++f)
          if ((f & 3) == g) p.obs_buf[base * D + f] = x[0][f >> 2];
      }
      floatx4 h1[HT], h2[QT];
      dense_fwd<DT, HT, true>(lds + L::W1, L::S1, lds + L::B1, x, h1, (D + 3) >> 2);
      dense_fwd<HT, QT, true>(lds + L::W2 + 16 * to0 * L::S2, L::S2, lds + L::B2 + 16 * to0, h1, h2);
      float* pp = part + parity * (WPT * kMaxAct * 16);
#pragma unroll
      for (int a = 0; a < A; ++a) {
        const float v = head_dot<QT>(lds + L::W3 + a * H + 16 * to0, 0.f, h2);
        if (g == 0) pp[(w * kMaxAct + a) * 16 + j] = v;
      }
      __syncthreads();
      float logits[kMaxAct];
#pragma unroll
      for (int a = 0; a < kMaxAct; ++a) {
        if (a < A) {
          const float* q = pp + a * 16 + j;
          float z = q[0];
#pragma unroll
          for (int v = 1; v < WPT; ++v) z += q[v * kMaxAct * 16];  // same order in every wave
          logits[a] = z + lds[L::B3 + a];
        } else {
          logits[a] = -INFINITY;
        }
      }
      parity ^= 1;
      const CatStats cs = cat_stats(A, logits);
      const uint4 rnd = philox4x32(make_uint4((uint32_t)envc, (uint32_t)gstep, (uint32_t)(gstep >> 32), 0u), key);
      const int a = cat_sample(A, logits, cs.lse, u01(rnd.x));
      const float logp = pick_logit(A, logits, a) - cs.lse;

      bool term;
      const float r = Env::step(s, a, term, u01(rnd.y));
      len += 1;
      ret += r;
      const bool trunc = len >= p.max_steps;
      const bool done = term || trunc;
      const bool boot = trunc && !term && p.tobs_buf != nullptr;
      if (valid && writer) {
        p.act_buf[base] = a;
        p.logp_buf[base] = logp;
        p.rew_buf[base] = r;
        p.done_buf[base] = boot ? 2.f : (done ? 1.f : 0.f);
      }
      if (boot && valid && w == 0) {
#pragma unroll
        for (int f = 0; f < D; ++f)
          if ((f & 3) == g) p.tobs_buf[base * D + f] = Env::obs(s, f);
      }
      if (done) {
        if (valid && writer) {
          st_n += 1.f;
          st_sum += ret;
          st_sq += ret * ret;
          st_max = fmaxf(st_max, ret);
          st_min = fminf(st_min, ret);
          st_len += (float)len;
        }
        const uint4 rr = philox4x32(make_uint4((uint32_t)envc, (uint32_t)gstep, (uint32_t)(gstep >> 32), 1u), key);
        Env::reset(s, rr);
        len = 0;
        ret = 0.f;
      }
    }
    if (valid && w == 0) {
      const size_t base = (size_t)p.T * p.N + env;
#pragma unroll
      for (int f = 0; f < D; ++f)
        if ((f & 3) == g) p.obs_buf[base * D + f] = Env::obs(s, f);
      if (g == 0) {
#pragma unroll
        for (int k = 0; k < NS; ++k) p.state[(size_t)env * NS + k] = s[k];
        p.ep_len[env] = len;
        p.ep_ret[env] = ret;
      }
    }
  }

  // workgroup statistics: only wave 0 accumulated, so its wave reduction is the answer
  if (w == 0) {
    float v0 = wave_sum(st_n), v1 = wave_sum(st_sum), v2 = wave_sum(st_sq), v5 = wave_sum(st_len);
    float v3 = st_max, v4 = st_min;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      v3 = fmaxf(v3, __shfl_xor(v3, o, 64));
      v4 = fminf(v4, __shfl_xor(v4, o, 64));
    }
    if (l == 0) {
      float* e = p.ep_stats + blockIdx.x * 8;
      e[0] = v0;
      e[1] = v1;
      e[2] = v2;
      e[3] = v3;
      e[4] = v4;
      e[5] = v5;
    }
  }
}

// ------------------------------------------------------------------ continuous envs
// Same structure for a diagonal-Gaussian policy (PPO / REINFORCE on HalfCheetahSynth):
// mu = MLP(obs), a = mu + exp(log_std) * n with n from Box-Muller over Philox draws
// (tags 0 and 2), logp = sum(-n^2/2 - log_std - log(2 pi)/2) -- the learner's GAUSS_EVAL
// formula.  Env constant tables (system matrices) are staged in LDS after the net.
struct RolloutContArgs {
  const float* params;
  const float* env_consts;
  int N, T;
  float* state;     // [N][NS]
  int* ep_len;      // [N]
  float* ep_ret;    // [N]
  float* obs_buf;   // [T+1][N][D]
  float* act_buf;   // [T][N][A]
  float* logp_buf;  // [T][N]
  float* rew_buf;   // [T][N]
  float* done_buf;  // [T][N]: 0 running, 2 time-limit truncation (1 without tobs_buf)
  float* tobs_buf;  // [T][N][D] pre-reset observation where done == 2, or null
  float* ep_stats;  // [grid][8]
  uint32_t seed_lo, seed_hi;
  uint32_t step_lo, step_hi;
  int reset_all;
  int max_steps;
};

template <class Env, int HT>
__global__ __launch_bounds__(256, 2) void rollout_cont_kernel(RolloutContArgs p) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  constexpr int DT = (Env::D + 15) / 16;
  using L = LdsNet<DT, HT>;
  constexpr int H = L::H;
  constexpr int D = Env::D, A = Env::A, NS = Env::NS;
  static_assert(NS == D, "continuous device envs observe their full state");
  const int net_floats = (L::floats(A) + 3) & ~3;
  float* cst = lds + net_floats;
  stage_net<DT, HT>(lds, p.params, D, A, true);
  for (int i = threadIdx.x; i < Env::kConsts; i += blockDim.x) cst[i] = p.env_consts[i];
  __syncthreads();

  const int l = lane_id();
  const int j = l & 15, g = l >> 4;
  const int wave_in_block = threadIdx.x >> 6;
  const int waves_per_block = blockDim.x >> 6;
  const int wave = wave_in_block + blockIdx.x * waves_per_block;
  const int total_waves = gridDim.x * waves_per_block;
  const int ntiles = (p.N + kTileB - 1) / kTileB;
  const uint2 key = make_uint2(p.seed_lo, p.seed_hi);
  const uint64_t step0 = ((uint64_t)p.step_hi << 32) | p.step_lo;
  const int kr1 = input_kr_last(D, DT);

  float st_n = 0.f, st_sum = 0.f, st_sq = 0.f, st_max = -INFINITY, st_min = INFINITY, st_len = 0.f;

  for (int tile = wave; tile < ntiles; tile += total_waves) {
    const int env = tile * kTileB + j;
    const bool valid = env < p.N;
    const int envc = valid ? env : p.N - 1;
    float s[NS];
    int len;
    float ret;
    if (p.reset_all) {
      Env::reset(s, key, (uint32_t)envc, step0);
      len = 0;
      ret = 0.f;
    } else {
#pragma unroll
      for (int k = 0; k < NS; ++k) s[k] = p.state[(size_t)envc * NS + k];
      len = p.ep_len[envc];
      ret = p.ep_ret[envc];
    }
    for (int t = 0; t < p.T; ++t) {
      const uint64_t gstep = step0 + (uint64_t)t;
      const size_t base = (size_t)t * p.N + env;
      floatx4 x[DT];
#pragma unroll
      for (int q = 0; q < DT; ++q) x[q] = zero4();
#pragma unroll
      for (int f = 0; f < D; ++f)
        if ((f & 3) == g) x[f >> 4][(f >> 2) & 3] = s[f];
      if (valid) {
#pragma unroll
        for (int f = 0; f < D; ++f)
          if ((f & 3) == g) p.obs_buf[base * D + f] = s[f];
      }
      floatx4 h1[HT], h2[HT];
      dense_fwd<DT, HT, true>(lds + L::W1, L::S1, lds + L::B1, x, h1, kr1);
      dense_fwd<HT, HT, true>(lds + L::W2, L::S2, lds + L::B2, h1, h2);
      float mu[kMaxAct];
      policy_logits<HT>(lds + L::W3, lds + L::B3, A, H, h2, mu);
      const uint4 r0 = philox4x32(make_uint4((uint32_t)envc, (uint32_t)gstep, (uint32_t)(gstep >> 32), 0u), key);
      const uint4 r1 = philox4x32(make_uint4((uint32_t)envc, (uint32_t)gstep, (uint32_t)(gstep >> 32), 2u), key);
      const float uu[8] = {u01(r0.x), u01(r0.y), u01(r0.z), u01(r0.w), u01(r1.x), u01(r1.y), u01(r1.z), u01(r1.w)};
      float nrm[8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float rad = sqrtf(-2.f * __logf(1.f - uu[2 * q]));
        float sn, cs;
        __sincosf(6.283185307179586f * uu[2 * q + 1], &sn, &cs);
        nrm[2 * q] = rad * cs;
        nrm[2 * q + 1] = rad * sn;
      }
      float act[kMaxAct];
      float logp = 0.f;
#pragma unroll
      for (int a = 0; a < kMaxAct; ++a) {
        act[a] = 0.f;
        if (a < A) {
          const float ls = lds[L::LOGSTD + a];
          const float n = nrm[a < 8 ? a : 0];
          act[a] = mu[a] + __expf(ls) * n;
          logp += -0.5f * n * n - ls - kHalfLog2Pi;
        }
      }
      const float r = Env::step(s, act, cst, key, (uint32_t)envc, gstep);
      len += 1;
      ret += r;
      const bool done = len >= p.max_steps;  // this env only truncates (time limit)
      const bool boot = done && p.tobs_buf != nullptr;
      if (valid && g == 0) {
#pragma unroll
        for (int a = 0; a < A; ++a) p.act_buf[base * A + a] = act[a];
        p.logp_buf[base] = logp;
        p.rew_buf[base] = r;
        p.done_buf[base] = boot ? 2.f : (done ? 1.f : 0.f);
      }
      if (boot && valid) {
#pragma unroll
        for (int f = 0; f < D; ++f)
          if ((f & 3) == g) p.tobs_buf[base * D + f] = s[f];
      }
      if (done) {
        if (valid && g == 0) {
          st_n += 1.f;
          st_sum += ret;
          st_sq += ret * ret;
          st_max = fmaxf(st_max, ret);
          st_min = fminf(st_min, ret);
          st_len += (float)len;
        }
        Env::reset(s, key, (uint32_t)envc, gstep + 0x100000000ull);
        len = 0;
        ret = 0.f;
      }
    }
    if (valid) {
      const size_t base = (size_t)p.T * p.N + env;
#pragma unroll
      for (int f = 0; f < D; ++f)
        if ((f & 3) == g) p.obs_buf[base * D + f] = s[f];
      if (g == 0) {
#pragma unroll
        for (int k = 0; k < NS; ++k) p.state[(size_t)env * NS + k] = s[k];
        p.ep_len[env] = len;
        p.ep_ret[env] = ret;
      }
    }
  }
  __syncthreads();
  float* red = lds;
  float v0 = wave_sum(st_n), v1 = wave_sum(st_sum), v2 = wave_sum(st_sq), v5 = wave_sum(st_len);
  float v3 = st_max, v4 = st_min;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    v3 = fmaxf(v3, __shfl_xor(v3, o, 64));
    v4 = fminf(v4, __shfl_xor(v4, o, 64));
  }
  if (l == 0) {
    red[wave_in_block * 8 + 0] = v0;
    red[wave_in_block * 8 + 1] = v1;
    red[wave_in_block * 8 + 2] = v2;
    red[wave_in_block * 8 + 3] = v3;
    red[wave_in_block * 8 + 4] = v4;
    red[wave_in_block * 8 + 5] = v5;
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    const int q = threadIdx.x;
    float v = red[q];
    for (int w = 1; w < waves_per_block; ++w) {
      const float u = red[w * 8 + q];
      v = (q == 3) ? fmaxf(v, u) : (q == 4) ? fminf(v, u) : v + u;
    }
    p.ep_stats[blockIdx.x * 8 + q] = v;
  }
}

}  // namespace rrl

using namespace rrl;

enum EnvId : int { ENV_CARTPOLE = 0, ENV_MOUNTAINCAR = 1, ENV_ACROBOT = 2, ENV_LUNARLANDER = 3, ENV_HALFCHEETAH = 4 };

extern "C" int rrl_env_dims(int env, int* D, int* A, int* NS, int* max_steps) {
  switch (env) {
    case ENV_CARTPOLE: *D = CartPoleEnv::D; *A = CartPoleEnv::A; *NS = CartPoleEnv::NS; *max_steps = CartPoleEnv::kMaxSteps; return 0;
    case ENV_MOUNTAINCAR: *D = MountainCarEnv::D; *A = MountainCarEnv::A; *NS = MountainCarEnv::NS; *max_steps = MountainCarEnv::kMaxSteps; return 0;
    case ENV_ACROBOT: *D = AcrobotEnv::D; *A = AcrobotEnv::A; *NS = AcrobotEnv::NS; *max_steps = AcrobotEnv::kMaxSteps; return 0;
    case ENV_LUNARLANDER:
      *D = LunarLanderSynthEnv::D;
      *A = LunarLanderSynthEnv::A;
      *NS = LunarLanderSynthEnv::NS;
      *max_steps = LunarLanderSynthEnv::kMaxSteps;
      return 0;
    case ENV_HALFCHEETAH:
      *D = HalfCheetahSynthEnv::D;
      *A = HalfCheetahSynthEnv::A;
      *NS = HalfCheetahSynthEnv::NS;
      *max_steps = HalfCheetahSynthEnv::kMaxSteps;
      return 0;
  }
  return -1;
}

// Few envs (at most two 16-env tiles per CU): one workgroup per tile, layer 2 split over
// its waves (rollout_wide_kernel); otherwise 4 tiles per workgroup, one per wave.
static bool rollout_wide(int N, int num_cu) {
  const int tiles = (N + kTileB - 1) / kTileB;
  return tiles <= 2 * (num_cu > 0 ? num_cu : 256);
}

extern "C" int rrl_rollout_grid(int N, int num_cu) {
  const int tiles = (N + kTileB - 1) / kTileB;
  if (rollout_wide(N, num_cu)) return tiles < 1 ? 1 : tiles;
  int grid = (tiles + 3) / 4;
  const int cap = 2 * (num_cu > 0 ? num_cu : 256);
  if (grid > cap) grid = cap;
  return grid < 1 ? 1 : grid;
}

template <class Env, int HT>
static int launch_rollout(const RolloutArgs& a, int grid, bool wide, hipStream_t s) {
  using L = LdsNet<1, HT>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)rollout_kernel<Env, HT>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              163840);
    (void)hipFuncSetAttribute((const void*)rollout_wide_kernel<Env, HT, 4>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    attr = true;
  }
  if (wide) {
    constexpr int WPT = 4;  // 8 waves per tile (one layer-2 output tile each) measured slower: 187 vs 166 us
    const size_t bytes = ((size_t)((L::floats(Env::A) + 3) & ~3) + 2 * WPT * kMaxAct * 16) * sizeof(float);
    hipLaunchKernelGGL((rollout_wide_kernel<Env, HT, WPT>), dim3(grid), dim3(64 * WPT), bytes, s, a);
  } else {
    const size_t bytes = (size_t)L::floats(Env::A) * sizeof(float);
    hipLaunchKernelGGL((rollout_kernel<Env, HT>), dim3(grid), dim3(256), bytes, s, a);
  }
  return (int)hipGetLastError();
}

extern "C" int rrl_rollout(int env, const float* params, int N, int T, int H, float* state, int* ep_len,
                           float* ep_ret, float* obs_buf, int* act_buf, float* logp_buf, float* rew_buf,
                           float* done_buf, float* tobs_buf, float* ep_stats, uint64_t seed, uint64_t step0,
                           int reset_all, int max_steps, int num_cu, void* stream) {
  if (N <= 0 || T <= 0) return -2;
  RolloutArgs a{params, N, T, H, state, ep_len, ep_ret, obs_buf, act_buf, logp_buf, rew_buf, done_buf, tobs_buf, ep_stats,
                (uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)step0, (uint32_t)(step0 >> 32), reset_all,
                max_steps};
  const int grid = rrl_rollout_grid(N, num_cu);
  const bool wide = rollout_wide(N, num_cu);
  hipStream_t s = (hipStream_t)stream;
  if (H == 128) {
    switch (env) {
      case ENV_CARTPOLE: return launch_rollout<CartPoleEnv, 8>(a, grid, wide, s);
      case ENV_MOUNTAINCAR: return launch_rollout<MountainCarEnv, 8>(a, grid, wide, s);
      case ENV_ACROBOT: return launch_rollout<AcrobotEnv, 8>(a, grid, wide, s);
      case ENV_LUNARLANDER: return launch_rollout<LunarLanderSynthEnv, 8>(a, grid, wide, s);
    }
  } else if (H == 64) {
    switch (env) {
      case ENV_CARTPOLE: return launch_rollout<CartPoleEnv, 4>(a, grid, wide, s);
      case ENV_MOUNTAINCAR: return launch_rollout<MountainCarEnv, 4>(a, grid, wide, s);
      case ENV_ACROBOT: return launch_rollout<AcrobotEnv, 4>(a, grid, wide, s);
      case ENV_LUNARLANDER: return launch_rollout<LunarLanderSynthEnv, 4>(a, grid, wide, s);
    }
  }
  return -3;
}

template <class Env, int HT>
static int launch_rollout_cont(const RolloutContArgs& a, int grid, hipStream_t s) {
  constexpr int DT = (Env::D + 15) / 16;
  using L = LdsNet<DT, HT>;
  const size_t bytes = ((size_t)((L::floats(Env::A) + 3) & ~3) + Env::kConsts) * sizeof(float);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)rollout_cont_kernel<Env, HT>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    attr = true;
  }
  hipLaunchKernelGGL((rollout_cont_kernel<Env, HT>), dim3(grid), dim3(256), bytes, s, a);
  return (int)hipGetLastError();
}

// Continuous-action device envs (env id ENV_HALFCHEETAH); env_consts = env_constants(name).
extern "C" int rrl_rollout_cont(int env, const float* params, const float* env_consts, int N, int T, int H,
                                float* state, int* ep_len, float* ep_ret, float* obs_buf, float* act_buf,
                                float* logp_buf, float* rew_buf, float* done_buf, float* tobs_buf, float* ep_stats,
                                uint64_t seed, uint64_t step0, int reset_all, int max_steps, int num_cu, void* stream) {
  if (N <= 0 || T <= 0 || env != ENV_HALFCHEETAH || env_consts == nullptr) return -2;
  RolloutContArgs a{params, env_consts, N, T, state, ep_len, ep_ret, obs_buf, act_buf, logp_buf, rew_buf, done_buf,
                    tobs_buf, ep_stats, (uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)step0, (uint32_t)(step0 >> 32),
                    reset_all, max_steps};
  const int grid = rrl_rollout_grid(N, num_cu);
  hipStream_t s = (hipStream_t)stream;
  if (H == 128) return launch_rollout_cont<HalfCheetahSynthEnv, 8>(a, grid, s);
  if (H == 64) return launch_rollout_cont<HalfCheetahSynthEnv, 4>(a, grid, s);
  return -3;
}
