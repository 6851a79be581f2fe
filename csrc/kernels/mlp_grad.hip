// Fused learner kernel: MLP forward recompute + loss head + full backward + weight
// gradients, one launch per optimisation step (K10, K11, K12 of SURVEY §2.6).
//
// Reference hot path: REINFORCE.compute_loss_pi / compute_loss_vf + loss.backward()
// (REINFORCE.py:97-125, 141-160), i.e. three nn.Linear layers forward and backward on
// the whole epoch batch.  Here one persistent workgroup per CU walks the batch in
// 64-row slabs (16 rows per wave):
//
//   forward   : h1 = relu(W1 x + b1), h2 = relu(W2 h1 + b2)       (MFMA, registers)
//   head      : dout = dLoss/d(out) for PG / value-MSE / PPO heads  (VALU epilogue)
//   bwd data  : dh2 = W3^T dout * (h2>0) (VALU), dh1 = W2^T dh2 * (h1>0) (MFMA)
//   bwd weight: dW3, dW2, dW1 as MFMA products that sum over the batch.  The batch
//               index lives on the lane axis of the activation tiles, so each
//               operand pair is transposed once through a [feature][64 batch] LDS
//               staging image (b32 writes, b128 reads) and the 4 waves split the
//               output tiles of each weight gradient between them.
//   bias grads: accumulated from the A-operand values already in registers.
//
// Each workgroup writes one partial-gradient slab (flat parameter order); the
// reduce+Adam kernel (adam.hip) sums the slabs, so the result is deterministic.
#include "common.h"
#include "heads.h"
#include "grad_args.h"

namespace rrl {

constexpr int kStageLd = 68;  // [feature][64 batch + 4 pad]

// acc[to][ti] += sum_b At[16*(to0+to)+i][b] * Bt[16*(ti0+ti)+i][b], b over the 64-row slab.
// Operands of batch block bb+1 are loaded while block bb's MFMAs issue.
template <int NTO, int NTI>
RRL_DEV void wgrad(const float* __restrict__ At, const float* __restrict__ Bt, int to0, int ti0,
                   floatx4 (&acc)[NTO][NTI], float (&bacc)[NTO]) {
  const int l = lane_id();
  const int i = l & 15, g = l >> 4;
  floatx4 a[NTO], b[NTI], an[NTO], bn[NTI];
#pragma unroll
  for (int to = 0; to < NTO; ++to)
    a[to] = *reinterpret_cast<const floatx4*>(At + (16 * (to0 + to) + i) * kStageLd + 4 * g);
#pragma unroll
  for (int ti = 0; ti < NTI; ++ti)
    b[ti] = *reinterpret_cast<const floatx4*>(Bt + (16 * (ti0 + ti) + i) * kStageLd + 4 * g);
#pragma unroll
  for (int bb = 0; bb < 4; ++bb) {
    if (bb < 3) {
#pragma unroll
      for (int to = 0; to < NTO; ++to)
        an[to] = *reinterpret_cast<const floatx4*>(At + (16 * (to0 + to) + i) * kStageLd + 16 * (bb + 1) + 4 * g);
#pragma unroll
      for (int ti = 0; ti < NTI; ++ti)
        bn[ti] = *reinterpret_cast<const floatx4*>(Bt + (16 * (ti0 + ti) + i) * kStageLd + 16 * (bb + 1) + 4 * g);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int to = 0; to < NTO; ++to) {
#pragma unroll
        for (int ti = 0; ti < NTI; ++ti) acc[to][ti] = mfma4(a[to][r], b[ti][r], acc[to][ti]);
      }
    }
#pragma unroll
    for (int to = 0; to < NTO; ++to) bacc[to] += (a[to][0] + a[to][1]) + (a[to][2] + a[to][3]);
    __builtin_amdgcn_sched_barrier(0);
    if (bb < 3) {
#pragma unroll
      for (int to = 0; to < NTO; ++to) a[to] = an[to];
#pragma unroll
      for (int ti = 0; ti < NTI; ++ti) b[ti] = bn[ti];
    }
  }
}

// Write NT transposed tiles of this wave (16 batch columns) into a staging image.
template <int NT>
RRL_DEV void stage_tiles(float* __restrict__ St, int wave, const floatx4 (&v)[NT]) {
  const int l = lane_id();
  const int j = l & 15, g = l >> 4;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
#pragma unroll
    for (int r = 0; r < 4; ++r) St[(16 * t + 4 * g + r) * kStageLd + 16 * wave + j] = v[t][r];
  }
}

// Interleaved input tile (load_x_tile layout: reg r of group g = feature 16t + 4r + g)
// written into the staging image in natural feature order.
template <int NT>
RRL_DEV void stage_x_tiles(float* __restrict__ St, int wave, const floatx4 (&v)[NT]) {
  const int l = lane_id();
  const int j = l & 15, g = l >> 4;
#pragma unroll
  for (int t = 0; t < NT; ++t) {
#pragma unroll
    for (int r = 0; r < 4; ++r) St[(16 * t + 4 * r + g) * kStageLd + 16 * wave + j] = v[t][r];
  }
}

// A3 > 0: the last layer has A3 (<= 2) outputs and its weight gradient is accumulated on
// the VALU in registers (dout x h2 outer products, reduced once at the end) instead of
// a 16-row MFMA tile that would be 1/16 (value) or 1/8 (CartPole policy) useful; this
// also removes one staging phase and two workgroup barriers per 64-row slab.
template <int DT, int HT, int HEAD, int A3, int EARLY>
__global__ __launch_bounds__(256, 1) void mlp_grad_kernel(GradArgs p) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  using L = LdsNet<DT, HT>;
  constexpr int H = L::H;
  constexpr bool kGauss = (HEAD == HEAD_PPO_GAUSS || HEAD == HEAD_PG_GAUSS);
  constexpr bool kCat = (HEAD == HEAD_PG_CAT || HEAD == HEAD_PPO_CAT);
  constexpr int TO = HT / 4;  // dW2 / dW1 output tiles per wave
  constexpr int TI3 = HT / 4; // dW3 input tiles per wave
  const int A = (HEAD == HEAD_VALUE_MSE) ? 1 : p.A;
  const int net_floats = (L::floats(A) + 3) & ~3;
  float* st0 = lds + net_floats;        // [H][68]
  float* st1 = st0 + H * kStageLd;      // [H][68]

  stage_net<DT, HT>(lds, p.params, p.D, A, kGauss);

  const int l = lane_id();
  const int j = l & 15, g = l >> 4;
  const int wave = threadIdx.x >> 6;

  float adv_mean = 0.f, adv_rstd = 1.f;
  if (p.adv_stats != nullptr) {
    const float n = fmaxf(p.adv_stats[2], 1.f);
    adv_mean = p.adv_stats[0] / n;
    const float var = fmaxf(p.adv_stats[1] / n - adv_mean * adv_mean, 0.f);
    adv_rstd = 1.f / (sqrtf(var) + 1e-8f);
  }

  floatx4 acc2[TO][HT], acc1[TO][DT], acc3[1][TI3];
  float bacc2[TO], bacc1[TO], bacc3[1];
#pragma unroll
  for (int a = 0; a < TO; ++a) {
    bacc2[a] = 0.f;
    bacc1[a] = 0.f;
#pragma unroll
    for (int b = 0; b < HT; ++b) acc2[a][b] = zero4();
#pragma unroll
    for (int b = 0; b < DT; ++b) acc1[a][b] = zero4();
  }
#pragma unroll
  for (int b = 0; b < TI3; ++b) acc3[0][b] = zero4();
  bacc3[0] = 0.f;
  float dls_acc[kMaxAct];  // Gaussian d(log_std) accumulators (per lane)
#pragma unroll
  for (int a = 0; a < kMaxAct; ++a) dls_acc[a] = 0.f;
  float s_loss = 0.f, s_ent = 0.f, s_kl = 0.f, s_clip = 0.f, s_val = 0.f, s_cnt = 0.f;
  constexpr int A3N = A3 > 0 ? A3 : 1;
  floatx4 acc3v[A3N][HT];  // VALU dW3 partials (A3 > 0)
  float bacc3v[A3N];
#pragma unroll
  for (int a = 0; a < A3N; ++a) {
    bacc3v[a] = 0.f;
#pragma unroll
    for (int t = 0; t < HT; ++t) acc3v[a][t] = zero4();
  }
  const int kr1 = input_kr_last(p.D, DT);
  // device-side batch shape (grad_args.h): rows >= Bv inert, inv_B from memory
  const int Bv = p.nvalid ? min(*p.nvalid, p.B) : p.B;
  const float invB = p.inv_B_dev ? *p.inv_B_dev : p.inv_B;

  __syncthreads();

  for (int base = blockIdx.x * 64; base < Bv; base += gridDim.x * 64) {
    const int row0 = base + 16 * wave;
    const int nrows = max(0, min(16, Bv - row0));
    const bool valid = j < nrows;
    const int row = row0 + j;

    floatx4 x[DT], h1[HT], h2[HT];
    load_x_tile<DT>(p.X, p.D, p.D, row0, nrows, x);
    dense_fwd<DT, HT, true>(lds + L::W1, L::S1, lds + L::B1, x, h1, kr1);
    dense_fwd<HT, HT, true>(lds + L::W2, L::S2, lds + L::B2, h1, h2);

    // ------------------------------------------------------------ head + dLoss/dout
    float dout[kMaxAct];
#pragma unroll
    for (int a = 0; a < kMaxAct; ++a) dout[a] = 0.f;
    const bool count = valid && g == 0;
    if (HEAD == HEAD_VALUE_MSE) {
      const float v = head_dot<HT>(lds + L::W3, lds[L::B3], h2);
      const float target = valid ? p.ret[row] : 0.f;
      const float diff = v - target;
      dout[0] = valid ? 2.f * diff * invB : 0.f;
      if (count) {
        s_loss += diff * diff;
        s_val += v;
        s_cnt += 1.f;
      }
    } else if (kCat) {
      float logits[kMaxAct];
      policy_logits<HT>(lds + L::W3, lds + L::B3, A, H, h2, logits);
      if (valid) apply_mask(p.mask ? p.mask + (size_t)row * A : nullptr, A, logits);
      const CatStats cs = cat_stats(A, logits);
      const int act = valid ? p.act[row] : 0;
      const float logp = pick_logit(A, logits, act) - cs.lse;
      float adv = valid ? p.adv[row] : 0.f;
      adv = (adv - adv_mean) * adv_rstd;
      float dlogp;  // dLoss_i / dlogp_i  (before the 1/B mean)
      float loss_i;
      if (HEAD == HEAD_PG_CAT) {
        dlogp = -adv;
        loss_i = -logp * adv;
      } else {
        const float lpo = valid ? p.logp_old[row] : logp;
        const float ratio = __expf(logp - lpo);
        const float s1 = ratio * adv;
        const float s2 = fminf(fmaxf(ratio, 1.f - p.clip_eps), 1.f + p.clip_eps) * adv;
        dlogp = (s1 <= s2) ? -adv * ratio : 0.f;
        loss_i = -fminf(s1, s2);
        if (count) s_clip += (fabsf(ratio - 1.f) > p.clip_eps) ? 1.f : 0.f;
      }
      const float scale = valid ? invB : 0.f;
#pragma unroll
      for (int a = 0; a < kMaxAct; ++a) {
        if (a < A) {
          const float pa = __expf(logits[a] - cs.lse);
          const float lpa = logits[a] - cs.lse;
          // d(logp_act)/dlogit_a = onehot - p ;  dH/dlogit_a = -p (log p_a + H)
          const float dpg = dlogp * ((a == act ? 1.f : 0.f) - pa);
          const float dent = pa > 0.f ? p.ent_coef * pa * (lpa + cs.entropy) : 0.f;
          dout[a] = scale * (dpg + dent);
        }
      }
      if (count) {
        s_loss += loss_i;
        s_ent += cs.entropy;
        if (p.logp_old) s_kl += p.logp_old[row] - logp;
        s_cnt += 1.f;
      }
    } else {  // Gaussian heads
      float adv = valid ? p.adv[row] : 0.f;
      adv = (adv - adv_mean) * adv_rstd;
      float mu[kMaxAct];
      float logp = 0.f;
#pragma unroll
      for (int a = 0; a < kMaxAct; ++a) {
        mu[a] = 0.f;
        if (a < A) {
          mu[a] = head_dot<HT>(lds + L::W3 + a * H, lds[L::B3 + a], h2);
          const float ls = lds[L::LOGSTD + a];
          const float xa = valid ? p.actc[(size_t)row * A + a] : mu[a];
          const float z = (xa - mu[a]) * __expf(-ls);
          logp += -0.5f * z * z - ls - kHalfLog2Pi;
        }
      }
      float dlogp, loss_i;
      if (HEAD == HEAD_PG_GAUSS) {
        dlogp = -adv;
        loss_i = -logp * adv;
      } else {
        const float lpo = valid ? p.logp_old[row] : logp;
        const float ratio = __expf(logp - lpo);
        const float s1 = ratio * adv;
        const float s2 = fminf(fmaxf(ratio, 1.f - p.clip_eps), 1.f + p.clip_eps) * adv;
        dlogp = (s1 <= s2) ? -adv * ratio : 0.f;
        loss_i = -fminf(s1, s2);
        if (count) s_clip += (fabsf(ratio - 1.f) > p.clip_eps) ? 1.f : 0.f;
      }
      const float scale = valid ? invB : 0.f;
      float ent = 0.f;
#pragma unroll
      for (int a = 0; a < kMaxAct; ++a) {
        if (a < A) {
          const float ls = lds[L::LOGSTD + a];
          const float inv_var = __expf(-2.f * ls);
          const float xa = valid ? p.actc[(size_t)row * A + a] : mu[a];
          const float d = xa - mu[a];
          // dlogp/dmu = d / var ; dlogp/dls = d^2/var - 1 ; dH/dls = 1
          dout[a] = scale * dlogp * d * inv_var;
          if (g == 0) dls_acc[a] += scale * (dlogp * (d * d * inv_var - 1.f) - p.ent_coef);
          ent += 0.5f + kHalfLog2Pi + ls;
        }
      }
      if (count) {
        s_loss += loss_i;
        s_ent += ent;
        if (p.logp_old) s_kl += p.logp_old[row] - logp;
        s_cnt += 1.f;
      }
    }

    // ------------------------------------------------------------ dh2 = W3^T dout * relu'
    floatx4 dh2[HT];
#pragma unroll
    for (int t = 0; t < HT; ++t) dh2[t] = zero4();
#pragma unroll
    for (int a = 0; a < kMaxAct; ++a) {
      if (a < A) {
#pragma unroll
        for (int t = 0; t < HT; ++t) {
          const floatx4 w = *reinterpret_cast<const floatx4*>(lds + L::W3 + a * H + 16 * t + 4 * g);
#pragma unroll
          for (int r = 0; r < 4; ++r) dh2[t][r] = fmaf(w[r], dout[a], dh2[t][r]);
        }
      }
    }
#pragma unroll
    for (int t = 0; t < HT; ++t) {
#pragma unroll
      for (int r = 0; r < 4; ++r) dh2[t][r] = h2[t][r] > 0.f ? dh2[t][r] : 0.f;
    }

    // ------------------------------------------------------------ phase A: dW3, db3
    if (A3 > 0) {
#pragma unroll
      for (int a = 0; a < A3N; ++a) {
        bacc3v[a] += dout[a];
#pragma unroll
        for (int t = 0; t < HT; ++t) {
#pragma unroll
          for (int r = 0; r < 4; ++r) acc3v[a][t][r] = fmaf(dout[a], h2[t][r], acc3v[a][t][r]);
        }
      }
    } else {
      __syncthreads();  // previous slab's phase-C readers are done with st0/st1
      stage_tiles<HT>(st0, wave, h2);
#pragma unroll
      for (int a = 0; a < kMaxAct; ++a)
        if ((a >> 2) == g) st1[a * kStageLd + 16 * wave + j] = (a < A) ? dout[a] : 0.f;
      __syncthreads();
      wgrad<1, TI3>(st1, st0, 0, wave * TI3, acc3, bacc3);
    }

    // ------------------------------------------------------------ phase B: dW2, db2
    __syncthreads();
    stage_tiles<HT>(st0, wave, h1);
    stage_tiles<HT>(st1, wave, dh2);
    floatx4 dh1[HT];
    if (EARLY) {
      // dh1 needs only registers + W2: issuing its 256 MFMAs before the barrier hides the
      // staging-write latency and the wave skew at the barrier
      dense_bwd_data<HT, HT, true>(lds + L::W2, L::S2, dh2, h1, dh1);
    }
    __syncthreads();
    wgrad<TO, HT>(st1, st0, wave * TO, 0, acc2, bacc2);
    if (!EARLY) dense_bwd_data<HT, HT, true>(lds + L::W2, L::S2, dh2, h1, dh1);

    // ------------------------------------------------------------ phase C: dW1, db1
    __syncthreads();
    stage_x_tiles<DT>(st0, wave, x);
    stage_tiles<HT>(st1, wave, dh1);
    __syncthreads();
    wgrad<TO, DT>(st1, st0, wave * TO, 0, acc1, bacc1);
  }

  // ------------------------------------------------------------------ epilogue
  const FlatOffsets o = flat_offsets(p.D, H, A);
  float* slab = p.grad_slab + (size_t)blockIdx.x * p.P;
  // dW2 / db2
#pragma unroll
  for (int to = 0; to < TO; ++to) {
    const int ot = wave * TO + to;
#pragma unroll
    for (int ti = 0; ti < HT; ++ti) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        slab[o.w2 + (16 * ot + 4 * g + r) * H + 16 * ti + j] = acc2[to][ti][r];
    }
    const float b2 = group_sum(bacc2[to]);
    if (g == 0) slab[o.b2 + 16 * ot + j] = b2;
#pragma unroll
    for (int ti = 0; ti < DT; ++ti) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int col = 16 * ti + j;
        if (col < p.D) slab[o.w1 + (16 * ot + 4 * g + r) * p.D + col] = acc1[to][ti][r];
      }
    }
    const float b1 = group_sum(bacc1[to]);
    if (g == 0) slab[o.b1 + 16 * ot + j] = b1;
  }
  // dW3 / db3
  if (A3 > 0) {
    // reduce the per-lane partials over the 16 batch columns, then over the 4 waves
    __syncthreads();
    float* red3 = st1;  // [4 waves][A3 * H + A3]
#pragma unroll
    for (int a = 0; a < A3N; ++a) {
#pragma unroll
      for (int t = 0; t < HT; ++t) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float v = col_sum(acc3v[a][t][r]);
          if (j == 0) red3[wave * (A3N * H + A3N) + a * H + 16 * t + 4 * g + r] = v;
        }
      }
      const float bv = col_sum(bacc3v[a]);
      if (l == 0) red3[wave * (A3N * H + A3N) + A3N * H + a] = bv;
    }
    __syncthreads();
    for (int q = threadIdx.x; q < A3N * H + A3N; q += blockDim.x) {
      const int stride = A3N * H + A3N;
      const float v = red3[q] + red3[stride + q] + red3[2 * stride + q] + red3[3 * stride + q];
      if (q < A3N * H) {
        if (q / H < A) slab[o.w3 + q] = v;
      } else if (q - A3N * H < A) {
        slab[o.b3 + (q - A3N * H)] = v;
      }
    }
  } else {
#pragma unroll
    for (int ti = 0; ti < TI3; ++ti) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int a = 4 * g + r;
        if (a < A) slab[o.w3 + a * H + 16 * (wave * TI3 + ti) + j] = acc3[0][ti][r];
      }
    }
    const float b3 = group_sum(bacc3[0]);
    if (wave == 0 && g == 0 && j < A) slab[o.b3 + j] = b3;
  }

  // Gaussian log_std grads and loss statistics: reduce over the workgroup via LDS
  __syncthreads();
  float* red = st0;  // reuse staging: [4 waves][32]
  float stats[6] = {s_loss, s_ent, s_kl, s_clip, s_val, s_cnt};
#pragma unroll
  for (int s = 0; s < 6; ++s) {
    const float v = wave_sum(stats[s]);
    if (l == 0) red[wave * 32 + s] = v;
  }
  if (kGauss) {
#pragma unroll
    for (int a = 0; a < kMaxAct; ++a) {
      const float v = wave_sum(dls_acc[a]);
      if (l == 0) red[wave * 32 + 8 + a] = v;
    }
  }
  __syncthreads();
  if (threadIdx.x < 32) {
    const int s = threadIdx.x;
    const float v = red[s] + red[32 + s] + red[64 + s] + red[96 + s];
    if (s < 6) p.loss_slab[blockIdx.x * 8 + s] = v;
    if (kGauss && s >= 8 && s - 8 < A) slab[o.log_std + (s - 8)] = v;
  }
}

}  // namespace rrl

using namespace rrl;

template <int DT, int HT, int HEAD, int A3, int EARLY>
static int launch_grad_v(const GradArgs& a, int grid, hipStream_t s) {
  using L = LdsNet<DT, HT>;
  const int A = (HEAD == HEAD_VALUE_MSE) ? 1 : a.A;
  const size_t floats = (size_t)((L::floats(A) + 3) & ~3) + 2 * (size_t)L::H * kStageLd;
  const size_t bytes = floats * sizeof(float);
  if (bytes > 163840) return -4;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)mlp_grad_kernel<DT, HT, HEAD, A3, EARLY>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    attr_set = true;
  }
  hipLaunchKernelGGL((mlp_grad_kernel<DT, HT, HEAD, A3, EARLY>), dim3(grid), dim3(256), bytes, s, a);
  return (int)hipGetLastError();
}

template <int DT, int HT, int HEAD, int A3>
static int launch_grad(const GradArgs& a, int grid, hipStream_t s) {
  return launch_grad_v<DT, HT, HEAD, A3, 1>(a, grid, s);
}

template <int DT, int HT, int HEAD>
static int dispatch_a3(const GradArgs& a, int grid, hipStream_t s) {
  if (HEAD == HEAD_VALUE_MSE || a.A == 1) return launch_grad<DT, HT, HEAD, 1>(a, grid, s);
  if (a.A == 2) return launch_grad<DT, HT, HEAD, 2>(a, grid, s);
  return launch_grad<DT, HT, HEAD, 0>(a, grid, s);
}

template <int DT, int HT>
static int dispatch_head(int head, const GradArgs& a, int grid, hipStream_t s) {
  switch (head) {
    case HEAD_PG_CAT: return dispatch_a3<DT, HT, HEAD_PG_CAT>(a, grid, s);
    case HEAD_VALUE_MSE: return launch_grad<DT, HT, HEAD_VALUE_MSE, 1>(a, grid, s);
    case HEAD_PPO_CAT: return dispatch_a3<DT, HT, HEAD_PPO_CAT>(a, grid, s);
    case HEAD_PPO_GAUSS: return dispatch_a3<DT, HT, HEAD_PPO_GAUSS>(a, grid, s);
    case HEAD_PG_GAUSS: return dispatch_a3<DT, HT, HEAD_PG_GAUSS>(a, grid, s);
  }
  return -1;
}

// Value-MSE and policy gradient path: 1 = weight-stationary bf16x6 kernels (value_grad.hip)
// where they apply (value: H = 128, D <= 24; categorical: D <= 8, A = 2..4; Gaussian: D <= 24,
// A = 1 or 6), 0 = the fp32-MFMA kernel above for every shape.
static int g_value_grad_mode = 1;
extern "C" int rrl_set_value_grad_mode(int mode) {
  const int old = g_value_grad_mode;
  if (mode == 0 || mode == 1) g_value_grad_mode = mode;
  return old;
}

// Number of partial-gradient slabs (== grid size) the launcher will use.
extern "C" int rrl_mlp_grad_slabs(int B, int num_cu) {
  int grid = (B + 63) / 64;
  const int cap = num_cu > 0 ? num_cu : 256;
  if (grid > cap) grid = cap;
  if (grid < 1) grid = 1;
  return grid;
}

extern "C" int rrl_mlp_grad(int head, const float* params, const float* X, int B, int D, int A, int H,
                            const float* mask, const int* act, const float* actc, const float* adv,
                            const float* ret, const float* logp_old, const float* adv_stats,
                            float inv_B, float clip_eps, float ent_coef, float* grad_slab,
                            float* loss_slab, int P, const int* nvalid, const float* inv_B_dev, int num_cu,
                            void* stream) {
  if (A < 1 || A > kMaxAct || D < 1 || D > 32) return -2;
  GradArgs a{params, X, B, D, A, mask, act, actc, adv, ret, logp_old, adv_stats, inv_B, clip_eps,
             ent_coef, grad_slab, loss_slab, P};
  a.nvalid = nvalid;
  a.inv_B_dev = inv_B_dev;
  const int grid = rrl_mlp_grad_slabs(B, num_cu);
  hipStream_t s = (hipStream_t)stream;
  if (head == HEAD_VALUE_MSE && g_value_grad_mode == 1 && value_grad_split_supported(D, H))
    return launch_value_grad_split(a, grid, s);
  if (head != HEAD_VALUE_MSE && g_value_grad_mode == 1 && policy_grad_split_supported(D, H, A, head))
    return launch_policy_grad_split(a, head, grid, s);
  const int DT = (D <= 16) ? 1 : 2;
  if (H == 128) return DT == 1 ? dispatch_head<1, 8>(head, a, grid, s) : dispatch_head<2, 8>(head, a, grid, s);
  if (H == 64) return DT == 1 ? dispatch_head<1, 4>(head, a, grid, s) : dispatch_head<2, 4>(head, a, grid, s);
  return -3;
}
