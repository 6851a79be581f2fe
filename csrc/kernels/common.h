// Shared device helpers for the relayrl_prototype_amd HIP kernels (gfx950 / CDNA4 only).
//
// Design notes (see docs/KERNELS.md for the full write-up):
//   * Every MLP in the reference (REINFORCE kernel.py:15-21, BaseKernel.py:25-39) is
//     Linear(D,H)-ReLU-Linear(H,H)-ReLU-Linear(H,A) with H = 128.  We run them on the
//     exact-fp32 matrix cores (v_mfma_f32_16x16x4_f32) so numerics match the reference's
//     fp32 libtorch CPU math.
//   * Activations are kept TRANSPOSED in the MFMA C/D layout: a 16x16 tile holds 16
//     features (rows, 4 per lane-group) x 16 batch columns (lane & 15).  In that layout
//     the output of one layer is directly the B operand of the next (the product sums
//     over the tile's row index), so a whole MLP forward never leaves registers.
//   * Weights live in LDS, row-major with a +4 float pad (stride = 4 mod 16 floats):
//       - forward A operand W[o][k..k+3] is one ds_read_b128 (near conflict-free),
//       - backward-data A operand W^T[i][k] = W[k][i] is a ds_read_b32 that is
//         bank-conflict free for the 32-lane halves (bank = 16*g + i).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef float floatx4 __attribute__((ext_vector_type(4)));

#define RRL_DEV __device__ __forceinline__

namespace rrl {

constexpr int kWave = 64;
constexpr int kTileB = 16;      // batch columns per wave tile
constexpr int kMaxAct = 16;     // max action dim supported by the fused heads

RRL_DEV int lane_id() { return threadIdx.x & 63; }

RRL_DEV floatx4 mfma4(float a, float b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

RRL_DEV floatx4 zero4() { floatx4 z = {0.f, 0.f, 0.f, 0.f}; return z; }

// Sum over the 4 lane groups (lanes j, j+16, j+32, j+48) that share batch column j.
RRL_DEV float group_sum(float v) {
  v += __shfl_xor(v, 16, 64);
  v += __shfl_xor(v, 32, 64);
  return v;
}
RRL_DEV float group_max(float v) {
  v = fmaxf(v, __shfl_xor(v, 16, 64));
  v = fmaxf(v, __shfl_xor(v, 32, 64));
  return v;
}
// Sum over the 16 batch columns (lanes with equal lane>>4).
RRL_DEV float col_sum(float v) {
  v += __shfl_xor(v, 1, 64);
  v += __shfl_xor(v, 2, 64);
  v += __shfl_xor(v, 4, 64);
  v += __shfl_xor(v, 8, 64);
  return v;
}
RRL_DEV float wave_sum(float v) {
  v = col_sum(v);
  return group_sum(v);
}

// ---------------------------------------------------------------- Philox4x32-10
// Counter-based RNG (Salmon et al. 2011).  key = run seed, counter = (stream id,
// step, tag, 0): every draw is a pure function of its coordinates, so the rollout
// kernel, the batched step kernel and the host-side oracle (ops/philox.py) agree
// bit for bit.
RRL_DEV uint4 philox4x32(uint4 c, uint2 k) {
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t lo0 = 0xD2511F53u * c.x;
    const uint32_t hi0 = __umulhi(0xD2511F53u, c.x);
    const uint32_t lo1 = 0xCD9E8D57u * c.z;
    const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
    k.x += 0x9E3779B9u;
    k.y += 0xBB67AE85u;
  }
  return c;
}
RRL_DEV float u01(uint32_t x) { return (float)(x >> 8) * (1.0f / 16777216.0f); }

// ---------------------------------------------------------------- MLP geometry
// Flat parameter layout of one Linear-ReLU-Linear-ReLU-Linear net (same order as
// nn.Sequential(...).parameters()): W1[H*D] b1[H] W2[H*H] b2[H] W3[A*H] b3[A]
// [+ log_std[A] for Gaussian policies].
struct FlatOffsets {
  int w1, b1, w2, b2, w3, b3, log_std, total;
};
RRL_DEV FlatOffsets flat_offsets(int D, int H, int A) {
  FlatOffsets o;
  o.w1 = 0;
  o.b1 = o.w1 + H * D;
  o.w2 = o.b1 + H;
  o.b2 = o.w2 + H * H;
  o.w3 = o.b2 + H;
  o.b3 = o.w3 + A * H;
  o.log_std = o.b3 + A;
  o.total = o.log_std + A;
  return o;
}

// LDS image of one net.  DT = input tiles (D <= 16*DT), HT = hidden tiles (H = 16*HT).
template <int DT, int HT>
struct LdsNet {
  static constexpr int H = 16 * HT;
  static constexpr int S1 = 16 * DT + 4;   // W1 row stride (floats)
  static constexpr int S2 = H + 4;         // W2 row stride (floats)
  static constexpr int W1 = 0;
  static constexpr int W2 = W1 + H * S1;
  static constexpr int B1 = W2 + H * S2;
  static constexpr int B2 = B1 + H;
  static constexpr int B3 = B2 + H;        // kMaxAct floats
  static constexpr int LOGSTD = B3 + kMaxAct;
  static constexpr int W3 = LOGSTD + kMaxAct;  // [A][H]
  static constexpr int fixed_floats() { return W3; }
  static constexpr int floats(int A) { return W3 + A * H; }
};

// Cooperative global->LDS staging of a flat parameter vector into the padded image.
template <int DT, int HT>
RRL_DEV void stage_net(float* __restrict__ lds, const float* __restrict__ flat, int D, int A,
                       bool has_log_std) {
  using L = LdsNet<DT, HT>;
  constexpr int H = L::H;
  const FlatOffsets o = flat_offsets(D, H, A);
  const int tid = threadIdx.x, nt = blockDim.x;
  // W1 columns are stored in the interleaved-input order (see load_x_tile): LDS column
  // c = 16t + 4g + r holds input feature f = 16t + 4r + g.
  for (int idx = tid; idx < H * L::S1; idx += nt) {
    const int row = idx / L::S1, c = idx - row * L::S1;
    const int t = c >> 4, rem = c & 15;
    const int f = 16 * t + 4 * (rem & 3) + (rem >> 2);
    lds[L::W1 + idx] = (c < 16 * DT && f < D) ? flat[o.w1 + row * D + f] : 0.f;
  }
  // W2: float4 copies (row length H is a multiple of 16)
  for (int idx = tid; idx < H * (H / 4); idx += nt) {
    const int r = idx / (H / 4), c4 = idx - r * (H / 4);
    const floatx4 v = *reinterpret_cast<const floatx4*>(flat + o.w2 + r * H + 4 * c4);
    *reinterpret_cast<floatx4*>(lds + L::W2 + r * L::S2 + 4 * c4) = v;
  }
  for (int idx = tid; idx < H; idx += nt) {
    lds[L::B1 + idx] = flat[o.b1 + idx];
    lds[L::B2 + idx] = flat[o.b2 + idx];
  }
  for (int idx = tid; idx < kMaxAct; idx += nt) {
    lds[L::B3 + idx] = (idx < A) ? flat[o.b3 + idx] : 0.f;
    lds[L::LOGSTD + idx] = (has_log_std && idx < A) ? flat[o.log_std + idx] : 0.f;
  }
  for (int idx = tid; idx < A * H; idx += nt) lds[L::W3 + idx] = flat[o.w3 + idx];
}

// out = W * in + b  (transposed-activation tiles), optional ReLU.
//   in : NI tiles, rows = input features (16*ti + 4g + r), col = batch (lane & 15)
//   out: NO tiles, rows = output features
// W is row-major [NO*16][S] in LDS, b is [NO*16] in LDS.  The A-operand loads of input
// tile ti+1 are issued before the MFMAs of tile ti (register double buffer), and a
// sched_barrier per tile stops the compiler from hoisting every load (register blow-up).
// KR_LAST < 4 skips the k-steps of the last input tile that only see zero padding
// (interleaved input layer: feature 4r+g lives in k-step r).
template <int NI, int NO, bool RELU>
RRL_DEV void dense_fwd(const float* __restrict__ W, int S, const float* __restrict__ b,
                       const floatx4 (&in)[NI], floatx4 (&out)[NO], int kr_last = 4) {
  const int l = lane_id();
  const int i = l & 15, g = l >> 4;
#pragma unroll
  for (int to = 0; to < NO; ++to) out[to] = *reinterpret_cast<const floatx4*>(b + 16 * to + 4 * g);
  floatx4 wc[NO], wn[NO];
#pragma unroll
  for (int to = 0; to < NO; ++to) wc[to] = *reinterpret_cast<const floatx4*>(W + (16 * to + i) * S + 4 * g);
#pragma unroll
  for (int ti = 0; ti < NI; ++ti) {
    if (ti + 1 < NI) {
#pragma unroll
      for (int to = 0; to < NO; ++to)
        wn[to] = *reinterpret_cast<const floatx4*>(W + (16 * to + i) * S + 16 * (ti + 1) + 4 * g);
    }
    const int kr = (ti == NI - 1) ? kr_last : 4;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (r < kr) {
#pragma unroll
        for (int to = 0; to < NO; ++to) out[to] = mfma4(wc[to][r], in[ti][r], out[to]);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (ti + 1 < NI) {
#pragma unroll
      for (int to = 0; to < NO; ++to) wc[to] = wn[to];
    }
  }
  if (RELU) {
#pragma unroll
    for (int to = 0; to < NO; ++to) {
#pragma unroll
      for (int r = 0; r < 4; ++r) out[to][r] = fmaxf(out[to][r], 0.f);
    }
  }
}

// k-steps of the last interleaved input tile that carry real features.
RRL_DEV int input_kr_last(int D, int DT) {
  const int rem = D - 16 * (DT - 1);
  return rem >= 16 ? 4 : (rem + 3) >> 2;
}

// dIn = W^T * dOut  (sum over output features), no bias.  Optionally masked by
// relu'(act) where act are the forward activations of the *input* side.
template <int NI, int NO, bool MASK>
RRL_DEV void dense_bwd_data(const float* __restrict__ W, int S, const floatx4 (&dout)[NO],
                            const floatx4 (&act_in)[NI], floatx4 (&din)[NI]) {
  const int l = lane_id();
  const int i = l & 15, g = l >> 4;
#pragma unroll
  for (int ti = 0; ti < NI; ++ti) din[ti] = zero4();
  float wc[4][NI], wn[4][NI];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
#pragma unroll
    for (int ti = 0; ti < NI; ++ti) wc[r][ti] = W[(4 * g + r) * S + i + 16 * ti];
  }
#pragma unroll
  for (int to = 0; to < NO; ++to) {
    if (to + 1 < NO) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int ti = 0; ti < NI; ++ti) wn[r][ti] = W[(16 * (to + 1) + 4 * g + r) * S + i + 16 * ti];
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int ti = 0; ti < NI; ++ti) din[ti] = mfma4(wc[r][ti], dout[to][r], din[ti]);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (to + 1 < NO) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
#pragma unroll
        for (int ti = 0; ti < NI; ++ti) wc[r][ti] = wn[r][ti];
      }
    }
  }
  if (MASK) {
#pragma unroll
    for (int ti = 0; ti < NI; ++ti) {
#pragma unroll
      for (int r = 0; r < 4; ++r) din[ti][r] = act_in[ti][r] > 0.f ? din[ti][r] : 0.f;
    }
  }
}

// Head: out[a] (a < A) for this lane's batch column, fully reduced over lane groups.
// W3 is [A][H] row-major in LDS, b3 [A].
template <int HT>
RRL_DEV float head_dot(const float* __restrict__ W3row, float b, const floatx4 (&h)[HT]) {
  const int g = lane_id() >> 4;
  float acc = 0.f;
#pragma unroll
  for (int t = 0; t < HT; ++t) {
    const floatx4 w = *reinterpret_cast<const floatx4*>(W3row + 16 * t + 4 * g);
    acc = fmaf(w[0], h[t][0], acc);
    acc = fmaf(w[1], h[t][1], acc);
    acc = fmaf(w[2], h[t][2], acc);
    acc = fmaf(w[3], h[t][3], acc);
  }
  return group_sum(acc) + b;
}

// Load a [16 batch x D] observation tile in the INTERLEAVED input layout: lane (j, g)
// reg r of tile t holds feature 16t + 4r + g of row j, so features 0..3 form k-step 0
// of the first layer's MFMA (D = 4 needs 1 k-step instead of 4).  Rows >= nrows are 0.
template <int DT>
RRL_DEV void load_x_tile(const float* __restrict__ X, int ldx, int D, int row0, int nrows,
                         floatx4 (&x)[DT]) {
  const int l = lane_id();
  const int j = l & 15, g = l >> 4;
  const bool ok = j < nrows;
  const float* row = X + (size_t)(row0 + j) * ldx;
#pragma unroll
  for (int t = 0; t < DT; ++t) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int f = 16 * t + 4 * r + g;
      x[t][r] = (ok && f < D) ? row[f] : 0.f;
    }
  }
}

}  // namespace rrl
