// The A2C policy / value head of the pixel model (Nature CNN fc 512 -> A logits + value):
// the kernel arguments and the per-row rollout math shared by cnn.hip's a2c_head_kernel and
// pong.hip's fused head + env step kernel.
#pragma once
#include "common.h"
#include "gemm_bf16.h"
#include "heads.h"

namespace rrl {

// One wave per row: lane owns features 8*lane .. 8*lane+7 of h (F = 512 -> 64 lanes x 8);
// head parameters: A policy rows of F fp32, A biases, the value row, its bias.
constexpr int kHeadF = 512;

struct HeadArgs {
  const uint16_t* h;      // [B][F] post-ReLU fc output
  const float* w;         // [A][F] policy rows; value row at w_v
  const float* bias;      // [A]
  const float* w_v;       // [F]
  const float* b_v;       // [1]
  int B, A;
  // rollout outputs
  int32_t* act;
  float* logp;
  float* value;
  float* logits_out;      // optional [B][A]
  uint32_t seed_lo, seed_hi, step_lo, step_hi;
  const unsigned long long* step_base;  // optional device counter added to the step (graph replays)
  int row_offset;
  // training inputs / outputs
  const int32_t* act_in;
  const float* adv;
  const float* ret;
  float inv_B, vf_coef, ent_coef;
  uint16_t* dh;           // [B][F] grad wrt fc pre-activation (masked), bf16
  float* dhead;           // [B][A+1] fp32: dlogits, dv
  float* stats;           // [gridDim.x][4]: pg loss, vf loss, entropy, count
  // rollout mode straight from the fc GEMM's split-K partials (fc.hip): h = bf16(relu(
  // fc_b + sum_z part[z][row][:])) is formed here and written to h_out for the backward
  const float* part;      // [splits][B][F] or null (then h is read)
  int splits;
  const float* fc_b;      // [F]
  uint16_t* h_out;        // [B][F]
};

// fp32 split-K partial sum of one lane's 8 features (S > 0: compile-time split count)
template <int S>
__device__ __forceinline__ void head_sum_part(float (&v)[8], const float* pr, size_t zs, int splits) {
  if constexpr (S > 0) {  // compile-time split count: every load issued before the adds
    float4 p[S][2];
#pragma unroll
    for (int z = 0; z < S; ++z) {
      p[z][0] = *reinterpret_cast<const float4*>(pr + z * zs);
      p[z][1] = *reinterpret_cast<const float4*>(pr + z * zs + 4);
    }
#pragma unroll
    for (int z = 0; z < S; ++z) {
      v[0] += p[z][0].x; v[1] += p[z][0].y; v[2] += p[z][0].z; v[3] += p[z][0].w;
      v[4] += p[z][1].x; v[5] += p[z][1].y; v[6] += p[z][1].z; v[7] += p[z][1].w;
    }
  } else {
    for (int z = 0; z < splits; ++z) {
      const float4 p0 = *reinterpret_cast<const float4*>(pr + z * zs);
      const float4 p1 = *reinterpret_cast<const float4*>(pr + z * zs + 4);
      v[0] += p0.x; v[1] += p0.y; v[2] += p0.z; v[3] += p0.w;
      v[4] += p1.x; v[5] += p1.y; v[6] += p1.z; v[7] += p1.w;
    }
  }
}

// Rollout mode, one wave per row, head weights STREAMED from global (L2) per output instead of
// held in registers (the fused Pong kernel runs at <= 64 VGPRs): h = bf16(relu(fc_b + sum_z
// part[z][row])) stored to h_out, then the same logits / value / sample arithmetic, in the same
// order, as a2c_head_kernel<false, AMAX> -- so the two paths agree bitwise.  Lane 0 writes
// act / logp / value and returns the action; other lanes return -1.
// (WV / WP: where the value / policy weight rows are read -- a.w_v / a.w, or an LDS copy)
template <int AMAX>
RRL_DEV int a2c_rollout_row_streamed(const HeadArgs& a, int row, int lane, const float* WV, const float* WP) {
  const int A = a.A, F = kHeadF;
  const float4 b0 = *reinterpret_cast<const float4*>(a.fc_b + 8 * lane);
  const float4 b1 = *reinterpret_cast<const float4*>(a.fc_b + 8 * lane + 4);
  float v[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
  const float* pr = a.part + (size_t)row * F + 8 * lane;
  const size_t zs = (size_t)a.B * F;
  switch (a.splits) {
    case 4: head_sum_part<4>(v, pr, zs, 4); break;
    case 2: head_sum_part<2>(v, pr, zs, 2); break;
    case 1: head_sum_part<1>(v, pr, zs, 1); break;
    default: head_sum_part<0>(v, pr, zs, a.splits); break;
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] = fmaxf(v[e], 0.f);
  const uint4 hv = pack_bf16x8(v);
  *reinterpret_cast<uint4*>(a.h_out + (size_t)row * F + 8 * lane) = hv;
  const uint32_t hw[4] = {hv.x, hv.y, hv.z, hv.w};
  float x[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    x[2 * i] = bf2f((uint16_t)(hw[i] & 0xffff));
    x[2 * i + 1] = bf2f((uint16_t)(hw[i] >> 16));
  }
  float logits[kMaxAct];
#pragma unroll
  for (int o = 0; o < kMaxAct; ++o) logits[o] = -INFINITY;
  float vsum = 0.f;
  {
    const float4 w0 = *reinterpret_cast<const float4*>(WV + 8 * lane);
    const float4 w1 = *reinterpret_cast<const float4*>(WV + 8 * lane + 4);
    const float wv[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
    for (int i = 0; i < 8; ++i) vsum += wv[i] * x[i];
  }
  const float value = wave_sum(vsum) + a.b_v[0];
#pragma unroll
  for (int o = 0; o < AMAX; ++o) {
    if (o < A) {
      const float4 w0 = *reinterpret_cast<const float4*>(WP + o * F + 8 * lane);
      const float4 w1 = *reinterpret_cast<const float4*>(WP + o * F + 8 * lane + 4);
      const float wp[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < 8; ++i) s += wp[i] * x[i];
      logits[o] = wave_sum(s) + a.bias[o];
    }
  }
  const CatStats cs = cat_stats(A, logits);
  int pick = -1;
  if (lane == 0) {
    unsigned long long st = ((unsigned long long)a.step_hi << 32) | a.step_lo;
    if (a.step_base) st += *a.step_base;
    const uint4 r = philox4x32(make_uint4((uint32_t)(row + a.row_offset), (uint32_t)st, (uint32_t)(st >> 32), 0x50u),
                               make_uint2(a.seed_lo, a.seed_hi));
    pick = cat_sample(A, logits, cs.lse, u01(r.x));
    if (a.act) a.act[row] = pick;
    if (a.logp) a.logp[row] = pick_logit(A, logits, pick) - cs.lse;
    if (a.value) a.value[row] = value;
  }
  return pick;
}
template <int AMAX>
RRL_DEV int a2c_rollout_row_streamed(const HeadArgs& a, int row, int lane) {
  return a2c_rollout_row_streamed<AMAX>(a, row, lane, a.w_v, a.w);
}

}  // namespace rrl
