// Policy / value heads fused into the MLP epilogue (K2-K6 of SURVEY §2.6).
//
// Reference semantics (kernel.py:23-37): logits += (mask - 1) * 1e8, softmax,
// torch.multinomial sample.  Unlike the reference (which gathers the raw logit and
// calls it a log-prob) we return the true log_softmax[a]; the
// entropy is the true -sum p log p.
#pragma once
#include "common.h"

namespace rrl {

// Full logits (every lane of column j ends up with all A values).
template <int HT>
RRL_DEV void policy_logits(const float* __restrict__ W3, const float* __restrict__ b3, int A, int H,
                           const floatx4 (&h)[HT], float (&logits)[kMaxAct]) {
#pragma unroll
  for (int a = 0; a < kMaxAct; ++a) {
    if (a < A) logits[a] = head_dot<HT>(W3 + a * H, b3[a], h);
    else logits[a] = -INFINITY;
  }
}

RRL_DEV void apply_mask(const float* __restrict__ mrow, int A, float (&logits)[kMaxAct]) {
  if (mrow == nullptr) return;
#pragma unroll
  for (int a = 0; a < kMaxAct; ++a)
    if (a < A) logits[a] = logits[a] + (mrow[a] - 1.f) * 1e8f;
}

struct CatStats {
  float lse;      // log-sum-exp of logits
  float entropy;  // -sum p log p
};

RRL_DEV CatStats cat_stats(int A, const float (&logits)[kMaxAct]) {
  float m = -INFINITY;
#pragma unroll
  for (int a = 0; a < kMaxAct; ++a)
    if (a < A) m = fmaxf(m, logits[a]);
  float s = 0.f, sx = 0.f;
#pragma unroll
  for (int a = 0; a < kMaxAct; ++a)
    if (a < A) {
      const float e = __expf(logits[a] - m);
      s += e;
      sx += e * (logits[a] - m);
    }
  CatStats c;
  c.lse = m + __logf(s);
  // H = lse - sum p*logit = log s - sx/s   (shifted by m)
  c.entropy = __logf(s) - sx / s;
  return c;
}

// Inverse-CDF categorical draw with uniform u in [0,1).
RRL_DEV int cat_sample(int A, const float (&logits)[kMaxAct], float lse, float u) {
  float c = 0.f;
  int pick = -1;
#pragma unroll
  for (int a = 0; a < kMaxAct; ++a)
    if (a < A) {
      const float p = __expf(logits[a] - lse);
      c += p;
      if (pick < 0 && u < c && p > 0.f) pick = a;
    }
  if (pick < 0) {  // u beyond the rounded cdf: take the last action with p > 0
#pragma unroll
    for (int a = 0; a < kMaxAct; ++a)
      if (a < A && __expf(logits[a] - lse) > 0.f) pick = a;
  }
  return pick < 0 ? 0 : pick;
}

RRL_DEV float pick_logit(int A, const float (&logits)[kMaxAct], int act) {
  float v = 0.f;
#pragma unroll
  for (int a = 0; a < kMaxAct; ++a)
    if (a == act) v = logits[a];
  return v;
}

// Gaussian head: log N(x; mu, sigma) summed over dims.
constexpr float kHalfLog2Pi = 0.91893853320467274f;

}  // namespace rrl
