// Pixel-policy (Nature-CNN actor-critic) kernels for the A2C / Pong configuration
// (BASELINE.json config 4; SURVEY §2.6 "New: CNN encoder (Pong) -- implicit-GEMM conv on
// MFMA").  The reference has no pixel model; this family is new.
//
// Compute dtype: bf16 operands on v_mfma_f32_16x16x32_bf16 with fp32 accumulation,
// fp32 master weights / Adam state, bf16 shadow weights written by the optimizer.
// Activations are NHWC bf16 (post-ReLU), weights [Cout][KH][KW][Cin] so that a conv's
// reduction index k = (kh, kw, c) is contiguous in both operands.
//
//   forward   Y  = relu(im2col(X) . W^T + b)        A = ConvLoader/FrameLoader, B = W   [NT]
//   dgrad     dXc = dY . W                          A = dY, B = W (transposed LDS read) [NN]
//             dX = col2im(dXc) * (X > 0)            gather form, no atomics
//   wgrad     dW = dY^T . im2col(X)                 both operands via transposed reads,
//                                                   split over batch x spatial -> fp32 partials
#include "gemm_bf16.h"
#include "heads.h"
#include "a2c_head.h"

namespace rrl {

struct ConvGeom {
  int N, H, W, C, KH, KW, S, OH, OW, Cout;
  __host__ __device__ int M() const { return N * OH * OW; }
  __host__ __device__ int K() const { return KH * KW * C; }
};

// ----------------------------------------------------------------------------- epilogues
struct BiasReluStore {  // bf16 [M][N] = act(scale * acc + b[n])
  uint16_t* y;
  const float* b;
  int M, N;
  bool relu;
  float scale;
  static constexpr bool kVec8 = true;
  __device__ __forceinline__ void store8(int m, int n, const float (&v)[8], int) const {
    float o[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float t = scale * v[e] + (b ? b[n + e] : 0.f);
      o[e] = relu ? fmaxf(t, 0.f) : t;
    }
    *reinterpret_cast<uint4*>(y + (size_t)m * N + n) = pack_bf16x8(o);
  }
  __device__ __forceinline__ void operator()(int m, int n, f32x4_t acc, int) const {
    if (n >= N) return;
    const float bb = b ? b[n] : 0.f;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (m + r < M) {
        float v = scale * acc[r] + bb;
        if (relu) v = fmaxf(v, 0.f);
        y[(size_t)(m + r) * N + n] = f2bf(v);
      }
    }
  }
};

struct MaskStore {  // bf16 [M][N] = acc * (mask[m][n] > 0)   (mask == null: plain store)
  uint16_t* y;
  const uint16_t* mask;
  int M, N;
  static constexpr bool kVec8 = true;
  __device__ __forceinline__ void store8(int m, int n, const float (&v)[8], int) const {
    const size_t i = (size_t)m * N + n;
    float o[8];
    const uint4 mk = mask ? *reinterpret_cast<const uint4*>(mask + i) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (!mask || bf16x8_at(mk, e) > 0.f) ? v[e] : 0.f;
    *reinterpret_cast<uint4*>(y + i) = pack_bf16x8(o);
  }
  __device__ __forceinline__ void operator()(int m, int n, f32x4_t acc, int) const {
    if (n >= N) return;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (m + r < M) {
        const size_t i = (size_t)(m + r) * N + n;
        float v = acc[r];
        if (mask && !(bf2f(mask[i]) > 0.f)) v = 0.f;
        y[i] = f2bf(v);
      }
    }
  }
};

struct PartialStore {  // fp32 [split][M][N]
  float* out;
  int M, N;
  static constexpr bool kVec8 = true;
  __device__ __forceinline__ void store8(int m, int n, const float (&v)[8], int z) const {
    float* o = out + (size_t)z * M * N + (size_t)m * N + n;
    *reinterpret_cast<f32x4_t*>(o) = f32x4_t{v[0], v[1], v[2], v[3]};
    *reinterpret_cast<f32x4_t*>(o + 4) = f32x4_t{v[4], v[5], v[6], v[7]};
  }
  __device__ __forceinline__ void operator()(int m, int n, f32x4_t acc, int z) const {
    if (n >= N) return;
    float* o = out + (size_t)z * M * N;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      if (m + r < M) o[(size_t)(m + r) * N + n] = acc[r];
  }
};

struct PartialStoreT {  // fp32 [split][N][M] = scale * acc: the GEMM computed the transpose (rows = k, cols = cout)
  float* out;
  int M, N;  // GEMM dims: M = K of the conv (rows), N = Cout
  float scale;
  __device__ __forceinline__ void operator()(int m, int n, f32x4_t acc, int z) const {
    if (n >= N) return;
    float* o = out + (size_t)z * M * N + (size_t)n * M;
    if (m + 3 < M) {
      *reinterpret_cast<float4*>(o + m) =
          make_float4(scale * acc[0], scale * acc[1], scale * acc[2], scale * acc[3]);
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (m + r < M) o[m + r] = scale * acc[r];
    }
  }
};

template <int BM, int BN, bool A_TR, bool B_TR, class LA, class LB, class Epi>
static int launch_gemm(LA la, LB lb, Epi epi, int M, int N, int K, int splits, hipStream_t st) {
  using S = GemmShape<BM, BN, A_TR, B_TR>;
  auto kern = gemm_bf16_kernel<BM, BN, A_TR, B_TR, LA, LB, Epi>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, S::LDS_BYTES);
    attr = true;
  }
  splits = splits < 1 ? 1 : splits;
  int kps = (K + splits - 1) / splits;
  kps = (kps + kGemmBK - 1) / kGemmBK * kGemmBK;
  splits = (K + kps - 1) / kps;
  dim3 grid((M + BM - 1) / BM, (N + BN - 1) / BN, splits);
  hipLaunchKernelGGL(kern, grid, dim3(256), S::LDS_BYTES, st, la, lb, epi, M, N, K, kps);
  return (int)hipGetLastError();
}

// Calls f(loader) with the fastest im2col loader for the geometry: compile-time
// variants for the Nature-CNN layers, plain row loader for 1x1 (fc), runtime otherwise.
template <class F>
static int with_im2col(const ConvGeom& g, const void* x, bool u8, F&& f) {
  const int M = g.M(), K = g.K();
  if (u8) {
    const uint8_t* xu = (const uint8_t*)x;
    if (g.C % 8 == 0) {  // space-to-depth frames (the PongSynth layout: 21 x 21 x 64)
      if (g.H == 21 && g.W == 21 && g.C == 64 && g.KH == 2 && g.KW == 2 && g.S == 1)
        return f(U8ConvLoaderT<21, 21, 64, 2, 1, 20, 20>{xu, M, K});
      return f(U8ConvLoader{xu, g.H, g.W, g.C, g.KW, g.S, g.OH, g.OW, M, K});
    }
    if (g.C != 4 || (g.KW & 1)) return -1;  // plain NHWC stacked frames
    if (g.H == 84 && g.W == 84 && g.KH == 8 && g.KW == 8 && g.S == 4)
      return f(FrameLoaderT<84, 84, 8, 4, 20, 20>{xu, M, K});
    return f(FrameLoader{xu, g.H, g.W, g.KW, g.S, g.OH, g.OW, M, K});
  }
  if (g.C % 8) return -1;
  const uint16_t* xb = (const uint16_t*)x;
  if (g.H == 1 && g.W == 1 && g.KH == 1 && g.KW == 1) return f(RowLoader{xb, M, K});
  if (g.H == 20 && g.W == 20 && g.C == 32 && g.KH == 4 && g.KW == 4 && g.S == 2)
    return f(ConvLoaderT<20, 20, 32, 4, 2, 9, 9>{xb, M, K});
  if (g.H == 9 && g.W == 9 && g.C == 64 && g.KH == 3 && g.KW == 3 && g.S == 1)
    return f(ConvLoaderT<9, 9, 64, 3, 1, 7, 7>{xb, M, K});
  return f(ConvLoader{xb, g.H, g.W, g.C, g.KW, g.S, g.OH, g.OW, M, K});
}

// ----------------------------------------------------------------------------- col2im
// dX[n][ih][iw][c] = sum over (kh, kw) with ih = oh*S + kh, iw = ow*S + kw of
// dXc[(n, oh, ow)][(kh, kw, c)], then * (X > 0).  One thread per 8 channels.
__global__ void col2im_mask_kernel(const uint16_t* __restrict__ dcol, const uint16_t* __restrict__ xact,
                                   uint16_t* __restrict__ dx, ConvGeom g) {
  const int C8 = g.C / 8;
  const size_t total = (size_t)g.N * g.H * g.W * C8;
  const int K = g.K();
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < total; t += (size_t)gridDim.x * blockDim.x) {
    const int c8 = (int)(t % C8);
    size_t r = t / C8;
    const int iw = (int)(r % g.W);
    r /= g.W;
    const int ih = (int)(r % g.H);
    const int n = (int)(r / g.H);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int kh = 0; kh < g.KH; ++kh) {
      const int th = ih - kh;
      if (th < 0 || th % g.S) continue;
      const int oh = th / g.S;
      if (oh >= g.OH) continue;
      for (int kw = 0; kw < g.KW; ++kw) {
        const int tw = iw - kw;
        if (tw < 0 || tw % g.S) continue;
        const int ow = tw / g.S;
        if (ow >= g.OW) continue;
        const size_t m = ((size_t)n * g.OH + oh) * g.OW + ow;
        const uint4 v = *reinterpret_cast<const uint4*>(dcol + m * K + (kh * g.KW + kw) * g.C + c8 * 8);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          acc[2 * i] += bf2f((uint16_t)(w[i] & 0xffff));
          acc[2 * i + 1] += bf2f((uint16_t)(w[i] >> 16));
        }
      }
    }
    const size_t o = t * 8;
    const uint4 xm = *reinterpret_cast<const uint4*>(xact + o);
    const uint32_t xw[4] = {xm.x, xm.y, xm.z, xm.w};
    uint32_t ow4[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float a = bf2f((uint16_t)(xw[i] & 0xffff)) > 0.f ? acc[2 * i] : 0.f;
      const float b = bf2f((uint16_t)(xw[i] >> 16)) > 0.f ? acc[2 * i + 1] : 0.f;
      ow4[i] = (uint32_t)f2bf(a) | ((uint32_t)f2bf(b) << 16);
    }
    *reinterpret_cast<uint4*>(dx + o) = make_uint4(ow4[0], ow4[1], ow4[2], ow4[3]);
  }
}

// Split-K forward epilogue: y[m][n] = act(sum_z part[z][m][n] + b[n]) -> bf16.
__global__ void bias_act_kernel(const float* __restrict__ part, int splits, int M, int N, const float* __restrict__ b,
                                uint16_t* __restrict__ y, int relu) {
  const size_t total = (size_t)M * N;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    float v = b ? b[i % N] : 0.f;
    for (int z = 0; z < splits; ++z) v += part[(size_t)z * total + i];
    if (relu) v = fmaxf(v, 0.f);
    y[i] = f2bf(v);
  }
}

// ----------------------------------------------------------------------------- reductions
// part [splits][n] fp32 -> out[n].  Block = 16 float4 columns x 16 split phases (LDS
// fold), so a few thousand outputs with hundreds of splits still spread over the chip.
__global__ void __launch_bounds__(256) sum_splits_kernel(const float* __restrict__ part, int splits, size_t n,
                                                         float* __restrict__ out) {
  __shared__ float4 red[16][16];
  const int col = threadIdx.x & 15, ph = threadIdx.x >> 4;
  const size_t i4 = (size_t)blockIdx.x * 16 + col;  // float4 index
  const size_t n4 = n / 4;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i4 < n4) {
    // 8 slab loads in flight per thread (the fused conv backward kernels leave 256-512
    // slabs of 8-37 K floats: one load per iteration was latency-bound)
    int z = ph;
    for (; z + 7 * 16 < splits; z += 8 * 16) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = reinterpret_cast<const float4*>(part + (size_t)(z + 16 * u) * n)[i4];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a.x += v[u].x;
        a.y += v[u].y;
        a.z += v[u].z;
        a.w += v[u].w;
      }
    }
    for (; z < splits; z += 16) {
      const float4 v = reinterpret_cast<const float4*>(part + (size_t)z * n)[i4];
      a.x += v.x;
      a.y += v.y;
      a.z += v.z;
      a.w += v.w;
    }
  }
  red[ph][col] = a;
  __syncthreads();
  if (ph == 0 && i4 < n4) {
    for (int k = 1; k < 16; ++k) {
      a.x += red[k][col].x;
      a.y += red[k][col].y;
      a.z += red[k][col].z;
      a.w += red[k][col].w;
    }
    reinterpret_cast<float4*>(out)[i4] = a;
  }
  // tail (n % 4) handled by block 0
  if (blockIdx.x == 0 && threadIdx.x < (int)(n & 3)) {
    const size_t i = n4 * 4 + threadIdx.x;
    float t = 0.f;
    for (int z = 0; z < splits; ++z) t += part[(size_t)z * n + i];
    out[i] = t;
  }
}

// Several split sums in ONE launch (the conv layers' weight and bias partials at the end of
// the backward: 6 launches -> 1, and the 32 / 64-float bias sums no longer run as single-
// block kernels of their own).  Segment q covers blocks [first[q], first[q + 1]); each block
// is the sum_splits_kernel block shape (16 float4 columns x 16 split phases).
constexpr int kMaxSumSegs = 8;
struct SumSegs {
  const float* part[kMaxSumSegs];
  float* out[kMaxSumSegs];
  long long n[kMaxSumSegs];
  int splits[kMaxSumSegs];
  int first[kMaxSumSegs + 1];
  int count;
};
__global__ void __launch_bounds__(256) sum_splits_multi_kernel(SumSegs sg) {
  __shared__ float4 red[16][16];
  int q = 0;
#pragma unroll 1
  while (q + 1 < sg.count && (int)blockIdx.x >= sg.first[q + 1]) ++q;
  const float* part = sg.part[q];
  const int splits = sg.splits[q];
  const size_t n = (size_t)sg.n[q];
  const int col = threadIdx.x & 15, ph = threadIdx.x >> 4;
  const size_t i4 = (size_t)(blockIdx.x - sg.first[q]) * 16 + col;
  const size_t n4 = n / 4;
  float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i4 < n4) {
    int z = ph;
    for (; z + 7 * 16 < splits; z += 8 * 16) {
      float4 v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) v[u] = reinterpret_cast<const float4*>(part + (size_t)(z + 16 * u) * n)[i4];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a.x += v[u].x;
        a.y += v[u].y;
        a.z += v[u].z;
        a.w += v[u].w;
      }
    }
    for (; z < splits; z += 16) {
      const float4 v = reinterpret_cast<const float4*>(part + (size_t)z * n)[i4];
      a.x += v.x;
      a.y += v.y;
      a.z += v.z;
      a.w += v.w;
    }
  }
  red[ph][col] = a;
  __syncthreads();
  if (ph == 0 && i4 < n4) {
    for (int k = 1; k < 16; ++k) {
      a.x += red[k][col].x;
      a.y += red[k][col].y;
      a.z += red[k][col].z;
      a.w += red[k][col].w;
    }
    reinterpret_cast<float4*>(sg.out[q])[i4] = a;
  }
}

// Few splits (<= 8, e.g. the fc weight gradient's 5): one float4 column per thread, its splits
// summed in order -- the 16-phase block above left 11 of 16 phases idle there and moved
// 25 k blocks for the 1.6 M fc weights (15 us; this shape ~7 us).
constexpr int kFewSplits = 8;
__global__ void __launch_bounds__(256) sum_splits_few_kernel(SumSegs sg) {
  int q = 0;
#pragma unroll 1
  while (q + 1 < sg.count && (int)blockIdx.x >= sg.first[q + 1]) ++q;
  const size_t n4 = (size_t)sg.n[q] / 4;
  const size_t i4 = (size_t)(blockIdx.x - sg.first[q]) * 256 + threadIdx.x;
  if (i4 >= n4) return;
  const float4* part = reinterpret_cast<const float4*>(sg.part[q]);
  const int splits = sg.splits[q];
  float4 v[kFewSplits];
#pragma unroll
  for (int z = 0; z < kFewSplits; ++z)
    if (z < splits) v[z] = part[(size_t)z * n4 + i4];
  float4 a = v[0];
#pragma unroll
  for (int z = 1; z < kFewSplits; ++z)
    if (z < splits) {
      a.x += v[z].x;
      a.y += v[z].y;
      a.z += v[z].z;
      a.w += v[z].w;
    }
  reinterpret_cast<float4*>(sg.out[q])[i4] = a;
}

// Unaligned / odd-length split sums (e.g. the A2C head, n = 512 (A+1) + A+1): a block
// owns 64 consecutive columns and splits the slab sum over 16 row groups (coalesced 256-B
// rows per wave), folded through LDS -- the one-thread-per-column serial loop it replaces
// was latency-bound (61 us for 256 slabs of 3.6 K floats).
__global__ void __launch_bounds__(1024) sum_splits_scalar_kernel(const float* __restrict__ part, int splits, size_t n,
                                                                 float* __restrict__ out) {
  __shared__ float red[16][64];
  const int col = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const size_t i = (size_t)blockIdx.x * 64 + col;
  float t = 0.f;
  if (i < n) {
    for (int z = grp; z < splits; z += 16) t += part[(size_t)z * n + i];
  }
  red[grp][col] = t;
  __syncthreads();
  if (grp == 0 && i < n) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) s += red[q][col];
    out[i] = s;
  }
}

// Column sums of a bf16 [M][C] matrix (C % 8 == 0, C <= 2048): partial [gridDim.x][C].
// A thread owns 8 consecutive columns of one row per pass (one 16-byte load); the
// 256 / (C/8) row lanes of a block are folded through LDS at the end.
__global__ void __launch_bounds__(256) colsum_kernel(const uint16_t* __restrict__ y, int M, int C,
                                                     float* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) float cred[];  // [256][8]
  const int cg = C / 8;
  const int lanes_per_row = cg < 256 ? cg : 256;
  const int row_lanes = 256 / lanes_per_row;
  const int tid = threadIdx.x;
  const int c8 = tid % lanes_per_row, rl = tid / lanes_per_row;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (rl < row_lanes) {
    for (int cc = c8; cc < cg; cc += lanes_per_row) {
      for (int r = blockIdx.x * row_lanes + rl; r < M; r += gridDim.x * row_lanes) {
        const uint4 v = *reinterpret_cast<const uint4*>(y + (size_t)r * C + 8 * cc);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          acc[2 * i] += bf2f((uint16_t)(w[i] & 0xffff));
          acc[2 * i + 1] += bf2f((uint16_t)(w[i] >> 16));
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) cred[tid * 8 + i] = acc[i];
  __syncthreads();
  if (rl == 0) {
    for (int k = 1; k < row_lanes; ++k)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += cred[(k * lanes_per_row + c8) * 8 + i];
#pragma unroll
    for (int i = 0; i < 8; ++i) part[(size_t)blockIdx.x * C + 8 * c8 + i] = acc[i];
  }
}

// Sum of squares of an fp32 vector: two-pass, deterministic.
// (VEC: 16-byte loads of a 16-byte aligned x, the n % 4 tail on block 0 -- 5.6 -> ~3 us for the
// 1.7 M Nature-CNN gradient)
template <bool VEC>
__global__ void sumsq_partial_kernel(const float* __restrict__ x, size_t n, float* __restrict__ part) {
  __shared__ float red[4];
  float s = 0.f;
  if (VEC) {
    const size_t n4 = n / 4;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n4; i += (size_t)gridDim.x * blockDim.x) {
      const float4 v = reinterpret_cast<const float4*>(x)[i];
      s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
    }
    if (blockIdx.x == 0 && threadIdx.x < (int)(n & 3)) {
      const float v = x[n4 * 4 + threadIdx.x];
      s += v * v;
    }
  } else {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
      const float v = x[i];
      s += v * v;
    }
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}
__global__ void sum_small_kernel(const float* __restrict__ part, int n, float* __restrict__ out) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += part[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = red[0] + red[1] + red[2] + red[3];
}

// The squared norm from the sum-of-squares partials, reduced inside every clip + Adam block in
// sum_small_kernel's exact order (256 threads): the same float, one launch fewer per update.
__device__ __forceinline__ float block_sum_parts(const float* __restrict__ part, int n) {
  __shared__ float red[4];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += part[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

// Adam with global-norm clipping (scale = min(1, max_norm / ||g||), norm from the device)
// and a bf16 shadow copy of the updated parameters for the next forward.
__global__ void adam_clip_kernel(float* __restrict__ p, float* __restrict__ m, float* __restrict__ v,
                                 const float* __restrict__ g, uint16_t* __restrict__ shadow, size_t n,
                                 const float* __restrict__ norm_sq, float max_norm, float lr, float b1, float b2,
                                 float eps, float bc1, float bc2, const long long* __restrict__ step_dev, int norm_parts) {
  if (step_dev) {  // bias corrections from the device step counter (capturable in a hipGraph)
    const float t = (float)(*step_dev);
    bc1 = 1.f - powf(b1, t);
    bc2 = 1.f - powf(b2, t);
  }
  float scale = 1.f;
  if (norm_sq != nullptr && max_norm > 0.f) {
    const float nrm = sqrtf(norm_parts > 0 ? block_sum_parts(norm_sq, norm_parts) : norm_sq[0]);
    scale = nrm > max_norm ? max_norm / (nrm + 1e-6f) : 1.f;
  }
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float gi = g[i] * scale;
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float denom = sqrtf(vi / bc2) + eps;
    const float pi = p[i] - lr * (mi / bc1) / denom;
    p[i] = pi;
    if (shadow) shadow[i] = f2bf(pi);
  }
}

// The same update four elements per thread: 16-byte loads / stores of p, m, v, g and one 8-byte
// store of the four bf16 shadow values (the scalar form above moved 4-byte words: 17.5 us for the
// 1.7 M Nature-CNN parameters, ~2x its HBM time).  The n % 4 tail is block 0's.
__global__ void adam_clip4_kernel(float* __restrict__ p, float* __restrict__ m, float* __restrict__ v,
                                  const float* __restrict__ g, uint16_t* __restrict__ shadow, size_t n,
                                  const float* __restrict__ norm_sq, float max_norm, float lr, float b1, float b2,
                                  float eps, float bc1, float bc2, const long long* __restrict__ step_dev, int norm_parts) {
  // this thread's first float4 of p / m / v / g is loaded before the norm reduction and the
  // bias corrections, so the two latencies overlap (one float4 per thread at the Pong size)
  const size_t n4 = n / 4, stride = (size_t)gridDim.x * blockDim.x;
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  float4 pv = make_float4(0.f, 0.f, 0.f, 0.f), mv = pv, vv = pv, gv = pv;
  if (i < n4) {
    pv = reinterpret_cast<const float4*>(p)[i];
    mv = reinterpret_cast<const float4*>(m)[i];
    vv = reinterpret_cast<const float4*>(v)[i];
    gv = reinterpret_cast<const float4*>(g)[i];
  }
  if (step_dev) {
    const float t = (float)(*step_dev);
    bc1 = 1.f - powf(b1, t);
    bc2 = 1.f - powf(b2, t);
  }
  float scale = 1.f;
  if (norm_sq != nullptr && max_norm > 0.f) {
    const float nrm = sqrtf(norm_parts > 0 ? block_sum_parts(norm_sq, norm_parts) : norm_sq[0]);
    scale = nrm > max_norm ? max_norm / (nrm + 1e-6f) : 1.f;
  }
  auto upd = [&](float pi, float mi, float vi, float gi, float& po, float& mo, float& vo) {
    gi *= scale;
    mo = b1 * mi + (1.f - b1) * gi;
    vo = b2 * vi + (1.f - b2) * gi * gi;
    const float denom = sqrtf(vo / bc2) + eps;
    po = pi - lr * (mo / bc1) / denom;
  };
  for (; i < n4; i += stride) {
    if (i != blockIdx.x * (size_t)blockDim.x + threadIdx.x) {
      pv = reinterpret_cast<const float4*>(p)[i];
      mv = reinterpret_cast<const float4*>(m)[i];
      vv = reinterpret_cast<const float4*>(v)[i];
      gv = reinterpret_cast<const float4*>(g)[i];
    }
    float4 po, mo, vo;
    upd(pv.x, mv.x, vv.x, gv.x, po.x, mo.x, vo.x);
    upd(pv.y, mv.y, vv.y, gv.y, po.y, mo.y, vo.y);
    upd(pv.z, mv.z, vv.z, gv.z, po.z, mo.z, vo.z);
    upd(pv.w, mv.w, vv.w, gv.w, po.w, mo.w, vo.w);
    reinterpret_cast<float4*>(m)[i] = mo;
    reinterpret_cast<float4*>(v)[i] = vo;
    reinterpret_cast<float4*>(p)[i] = po;
    if (shadow)
      reinterpret_cast<uint2*>(shadow)[i] =
          make_uint2((uint32_t)f2bf(po.x) | ((uint32_t)f2bf(po.y) << 16), (uint32_t)f2bf(po.z) | ((uint32_t)f2bf(po.w) << 16));
  }
  if (blockIdx.x == 0 && threadIdx.x < (int)(n & 3)) {
    const size_t i = n4 * 4 + threadIdx.x;
    float po, mo, vo;
    upd(p[i], m[i], v[i], g[i], po, mo, vo);
    m[i] = mo;
    v[i] = vo;
    p[i] = po;
    if (shadow) shadow[i] = f2bf(po);
  }
}

__global__ void to_bf16_kernel(const float* __restrict__ x, uint16_t* __restrict__ y, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    y[i] = f2bf(x[i]);
}

// ----------------------------------------------------------------------------- A2C head
// (HeadArgs, head_sum_part: a2c_head.h, shared with the fused Pong head + step kernel)

// Head weights live in REGISTERS: lane l holds features 8 l .. 8 l + 7 of every policy row
// and of the value row, loaded once per wave before its rows (L2 hits after the first
// wave), so there is no per-block LDS staging pass and no barrier in front of the rows --
// at 2,048 rollout rows a block has one row per wave and that staging was most of the
// launch.  AMAX = compile-time cap on A (8 covers Pong's 6; 16 = kMaxAct otherwise).
template <bool TRAIN, int AMAX>
__global__ void __launch_bounds__(256) a2c_head_kernel(HeadArgs a) {
  __shared__ float red[16];
  const int A = a.A, F = kHeadF;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float wv[8], wp[AMAX][8], bp[AMAX];
  {
    const float4 v0 = *reinterpret_cast<const float4*>(a.w_v + 8 * lane);
    const float4 v1 = *reinterpret_cast<const float4*>(a.w_v + 8 * lane + 4);
    wv[0] = v0.x; wv[1] = v0.y; wv[2] = v0.z; wv[3] = v0.w; wv[4] = v1.x; wv[5] = v1.y; wv[6] = v1.z; wv[7] = v1.w;
#pragma unroll
    for (int o = 0; o < AMAX; ++o) {  // rows past A: a clamped duplicate, never used
      const int oc = o < A ? o : A - 1;
      const float4 w0 = *reinterpret_cast<const float4*>(a.w + oc * F + 8 * lane);
      const float4 w1 = *reinterpret_cast<const float4*>(a.w + oc * F + 8 * lane + 4);
      wp[o][0] = w0.x; wp[o][1] = w0.y; wp[o][2] = w0.z; wp[o][3] = w0.w;
      wp[o][4] = w1.x; wp[o][5] = w1.y; wp[o][6] = w1.z; wp[o][7] = w1.w;
      bp[o] = a.bias[oc];
    }
  }
  const float bv = a.b_v[0];
  float st_pg = 0.f, st_vf = 0.f, st_ent = 0.f, st_n = 0.f;
  // TRAIN: the next row's inputs are loaded before this row's math (one row-load latency per
  // wave instead of one per row; the backward runs ~4 rows per wave)
  const int rstride = gridDim.x * 4;
  uint4 hv_n = make_uint4(0u, 0u, 0u, 0u);
  int act_n = 0;
  float adv_n = 0.f, ret_n = 0.f;
  if (TRAIN && blockIdx.x * 4 + wave < a.B) {
    const int r0 = blockIdx.x * 4 + wave;
    hv_n = *reinterpret_cast<const uint4*>(a.h + (size_t)r0 * F + 8 * lane);
    act_n = a.act_in[r0];
    adv_n = a.adv[r0];
    ret_n = a.ret[r0];
  }
  for (int row = blockIdx.x * 4 + wave; row < a.B; row += rstride) {
    uint4 hv;
    int act_c = 0;
    float adv_c = 0.f, ret_c = 0.f;
    if (TRAIN) {
      hv = hv_n;
      act_c = act_n;
      adv_c = adv_n;
      ret_c = ret_n;
      const int nr = row + rstride;
      if (nr < a.B) {
        hv_n = *reinterpret_cast<const uint4*>(a.h + (size_t)nr * F + 8 * lane);
        act_n = a.act_in[nr];
        adv_n = a.adv[nr];
        ret_n = a.ret[nr];
      }
    } else if (a.part) {
      // split-K reduction + bias + ReLU + bf16 rounding (the order bias_act_kernel uses)
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
      hv = pack_bf16x8(v);
      *reinterpret_cast<uint4*>(a.h_out + (size_t)row * F + 8 * lane) = hv;
    } else {
      hv = *reinterpret_cast<const uint4*>(a.h + (size_t)row * F + 8 * lane);
    }
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
#pragma unroll
    for (int i = 0; i < 8; ++i) vsum += wv[i] * x[i];
    const float value = wave_sum(vsum) + bv;
#pragma unroll
    for (int o = 0; o < AMAX; ++o) {
      if (o < A) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) s += wp[o][i] * x[i];
        logits[o] = wave_sum(s) + bp[o];
      }
    }
    const CatStats cs = cat_stats(A, logits);
    if (!TRAIN) {
      if (lane == 0) {
        unsigned long long st = ((unsigned long long)a.step_hi << 32) | a.step_lo;
        if (a.step_base) st += *a.step_base;
        const uint4 r = philox4x32(make_uint4((uint32_t)(row + a.row_offset), (uint32_t)st, (uint32_t)(st >> 32), 0x50u),
                                   make_uint2(a.seed_lo, a.seed_hi));
        const int pick = cat_sample(A, logits, cs.lse, u01(r.x));
        if (a.act) a.act[row] = pick;
        if (a.logp) a.logp[row] = pick_logit(A, logits, pick) - cs.lse;
        if (a.value) a.value[row] = value;
        if (a.logits_out)
          for (int o = 0; o < A; ++o) a.logits_out[(size_t)row * A + o] = logits[o];
      }
    } else {
      const int act = act_c;
      const float adv = adv_c, ret = ret_c;
      const float lp = pick_logit(A, logits, act) - cs.lse;
      // d/dz of  -adv*logp(a) - ent_coef*H  (mean over B), d/dv of vf_coef*(v-ret)^2
      float dz[kMaxAct];
#pragma unroll
      for (int o = 0; o < kMaxAct; ++o) {
        dz[o] = 0.f;
        if (o < A) {
          const float lpo = logits[o] - cs.lse;
          const float p = __expf(lpo);
          dz[o] = a.inv_B * (-adv * ((o == act ? 1.f : 0.f) - p) + a.ent_coef * p * (lpo + cs.entropy));
        }
      }
      const float dv = a.inv_B * 2.f * a.vf_coef * (value - ret);
      float g[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) g[i] = dv * wv[i];
#pragma unroll
      for (int o = 0; o < AMAX; ++o)
        if (o < A) {
#pragma unroll
          for (int i = 0; i < 8; ++i) g[i] += dz[o] * wp[o][i];
        }
      uint32_t ow[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float lo = x[2 * i] > 0.f ? g[2 * i] : 0.f, hi = x[2 * i + 1] > 0.f ? g[2 * i + 1] : 0.f;
        ow[i] = (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
      }
      *reinterpret_cast<uint4*>(a.dh + (size_t)row * F + 8 * lane) = make_uint4(ow[0], ow[1], ow[2], ow[3]);
      float mine = dv;
#pragma unroll
      for (int o = 0; o < kMaxAct; ++o)
        if (o < A && lane == o) mine = dz[o];
      if (lane <= A) a.dhead[(size_t)row * (A + 1) + lane] = mine;
      if (lane == 0) {
        st_pg += -adv * lp;
        st_vf += (value - ret) * (value - ret);
        st_ent += cs.entropy;
        st_n += 1.f;
      }
    }
  }
  if (TRAIN) {
    if (lane == 0) {
      red[wave * 4 + 0] = st_pg;
      red[wave * 4 + 1] = st_vf;
      red[wave * 4 + 2] = st_ent;
      red[wave * 4 + 3] = st_n;
    }
    __syncthreads();
    if (threadIdx.x < 4)
      a.stats[blockIdx.x * 4 + threadIdx.x] = red[threadIdx.x] + red[4 + threadIdx.x] + red[8 + threadIdx.x] +
                                              red[12 + threadIdx.x];
  }
}

// Head weight gradients: part[blk][ (A+1)*F + (A+1) ] = sum over the block's rows of
// dhead[r][o] * h[r][f] (and dhead[r][o] for the biases).  Thread t owns f = 2t, 2t+1.
__global__ void __launch_bounds__(256) head_wgrad_kernel(const uint16_t* __restrict__ h,
                                                         const float* __restrict__ dhead, int B, int A,
                                                         float* __restrict__ part) {
  const int F = kHeadF, O = A + 1;
  const int rows = (B + gridDim.x - 1) / gridDim.x;
  const int r0 = blockIdx.x * rows, r1 = min(B, r0 + rows);
  const int f = 2 * threadIdx.x;
  float acc[kMaxAct + 1][2];
  float bacc[kMaxAct + 1];
#pragma unroll
  for (int o = 0; o <= kMaxAct; ++o) acc[o][0] = acc[o][1] = bacc[o] = 0.f;
  // 4 rows per step with every load issued before the FMAs (the per-row loop waited for
  // each row's hidden units and head gradients in turn: a latency chain of ~40 rows)
  // (heads with <= 8 outputs; the head-gradient loads are clamped, never branched around)
  constexpr int kO = 8;
  int r = r0;
  for (; O <= kO && r + 4 <= r1; r += 4) {
    uint32_t hv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) hv[u] = *reinterpret_cast<const uint32_t*>(h + (size_t)(r + u) * F + f);
    float d[4][kO];
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int o = 0; o < kO; ++o) d[u][o] = dhead[(size_t)(r + u) * O + min(o, O - 1)];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float x0 = bf2f((uint16_t)(hv[u] & 0xffff)), x1 = bf2f((uint16_t)(hv[u] >> 16));
#pragma unroll
      for (int o = 0; o < kO; ++o)
        if (o < O) {
          acc[o][0] += d[u][o] * x0;
          acc[o][1] += d[u][o] * x1;
          bacc[o] += d[u][o];
        }
    }
  }
  for (; r < r1; ++r) {
    const uint32_t hv = *reinterpret_cast<const uint32_t*>(h + (size_t)r * F + f);
    const float x0 = bf2f((uint16_t)(hv & 0xffff)), x1 = bf2f((uint16_t)(hv >> 16));
#pragma unroll
    for (int o = 0; o <= kMaxAct; ++o)
      if (o < O) {
        const float d = dhead[(size_t)r * O + o];
        acc[o][0] += d * x0;
        acc[o][1] += d * x1;
        bacc[o] += d;
      }
  }
  float* out = part + (size_t)blockIdx.x * (O * F + O);
  // layout = flat param order: policy W [A][F], policy b [A], value W [F], value b [1]
#pragma unroll
  for (int o = 0; o <= kMaxAct; ++o)
    if (o < O) {
      float* wdst = o < A ? out + o * F : out + A * F + A;
      wdst[f] = acc[o][0];
      wdst[f + 1] = acc[o][1];
    }
  if (threadIdx.x == 0) {
    for (int o = 0; o < A; ++o) out[A * F + o] = bacc[o];
    out[A * F + A + F] = bacc[A];
  }
}


// ----------------------------------------------------------------------------- conv1 wgrad
// dW1[cout][kh][kw][c] = sum over images and 20x20 output pixels p of
//   dY[p][cout] * X[p + (kh, kw)][c]
// for the space-to-depth first layer (21x21x64 uint8 frames, 2x2 stride-1 taps, 32
// outputs).  The implicit-GEMM path re-reads and re-converts every input byte once per
// tap and dY once per 128-row tile (~1.7 GB for a 2048-env update).  Here a workgroup
// streams whole images: the frame (converted to bf16 once) and dY go into LDS, and wave
// w computes tap (kh, kw) = (w >> 1, w & 1) as a 32 x 64 GEMM over the image's 400 pixels
// whose B operand is the SHIFTED frame, read by row offset from the same LDS image
// (~550 MB of traffic, one pass).  The next image is prefetched into registers.
//
// MFMA k-order: lane group g of a 32-pixel chunk takes pixels 4g..4g+3 and 16+4g..16+4g+3
// (a 4-pixel run never crosses an output row, so its frame rows are consecutive); with
// rows of 80 bf16 the 8 rows one transposed read touches land in distinct bank octets.
constexpr int kW1Ld = 80;
constexpr int kW1XRows = 448;  // 441 frame pixels (+ pad)
constexpr int kW1YRows = 416;  // 400 output pixels + 16 zero rows (13 chunks of 32)
constexpr int kW1Lds = (kW1XRows + kW1YRows) * kW1Ld * 2;

__device__ __forceinline__ bf16x8_t tr8(const uint16_t* a0, const uint16_t* a1) {
  typedef __attribute__((address_space(3))) s16x4_t lds_v4;
  s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(a0));
  s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(a1));
  typedef short s16x8_t __attribute__((ext_vector_type(8)));
  s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

__global__ __launch_bounds__(256, 1) void conv1_wgrad_s2d_kernel(const uint8_t* __restrict__ x,
                                                                 const uint16_t* __restrict__ dy,
                                                                 float* __restrict__ part,
                                                                 float* __restrict__ bias_part, int N) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* Xi = smem;                   // [kW1XRows][kW1Ld] frame, bf16 integers 0..255
  uint16_t* Yi = smem + kW1XRows * kW1Ld;  // [kW1YRows][kW1Ld] dY
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int kh = w >> 1, kw = w & 1;
  const int n0 = (int)(((long long)N * blockIdx.x) / gridDim.x);
  const int n1 = (int)(((long long)N * (blockIdx.x + 1)) / gridDim.x);
  for (int q = tid; q < 16 * (kW1Ld / 8); q += 256)
    *reinterpret_cast<uint4*>(Yi + (400 + q / (kW1Ld / 8)) * kW1Ld + 8 * (q % (kW1Ld / 8))) = make_uint4(0, 0, 0, 0);

  f32x4_t acc[2][4], accb[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    accb[mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }
  // bias gradient db[co] = sum_p dY[p][co] rides along on wave 0 as one more MFMA column
  // block whose B operand is 1 in column 0 (the separate column-sum pass re-read dY)
  const bool do_bias = bias_part != nullptr && w == 0;
  bf16x8_t ones;
  {
    typedef short s16x8_t __attribute__((ext_vector_type(8)));
    const short one = (lane & 15) == 0 ? (short)0x3f80 : (short)0;  // bf16 1.0 in column 0
    s16x8_t v = {one, one, one, one, one, one, one, one};
    ones = __builtin_bit_cast(bf16x8_t, v);
  }

  constexpr int XC = 441 * 4, YC = 400 * 4;  // 16-byte chunks per image
  constexpr int XPT = (XC + 255) / 256, YPT = (YC + 255) / 256;
  uint4 rx[XPT], ry[YPT];
  auto gload = [&](int n) {
    const uint4* xs = reinterpret_cast<const uint4*>(x + (size_t)n * 441 * 64);
    const uint4* ys = reinterpret_cast<const uint4*>(dy + (size_t)n * 400 * 32);
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int q = tid + 256 * i;
      rx[i] = q < XC ? xs[q] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < YPT; ++i) {
      const int q = tid + 256 * i;
      ry[i] = q < YC ? ys[q] : make_uint4(0, 0, 0, 0);
    }
  };
  auto lstore = [&]() {
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int q = tid + 256 * i;
      if (q < XC) {
        uint16_t* d = Xi + (q >> 2) * kW1Ld + (q & 3) * 16;
        *reinterpret_cast<uint4*>(d) = u8x8_to_bf16x8(make_uint2(rx[i].x, rx[i].y));
        *reinterpret_cast<uint4*>(d + 8) = u8x8_to_bf16x8(make_uint2(rx[i].z, rx[i].w));
      }
    }
#pragma unroll
    for (int i = 0; i < YPT; ++i) {
      const int q = tid + 256 * i;
      if (q < YC) *reinterpret_cast<uint4*>(Yi + (q >> 2) * kW1Ld + (q & 3) * 8) = ry[i];
    }
  };

  const int g = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
  if (n0 < n1) gload(n0);
  for (int n = n0; n < n1; ++n) {
    __syncthreads();  // the previous image's fragment reads are done
    lstore();
    if (n + 1 < n1) gload(n + 1);
    __syncthreads();
#pragma unroll 1
    for (int kc = 0; kc < kW1YRows / 32; ++kc) {
      const int pa = 32 * kc + 4 * g, pb = pa + 16;
      // frame row of output pixel p under this wave's tap (0 past the last pixel: dY is 0 there)
      const int ra = (pa < 400 ? (pa / 20 + kh) * 21 + pa % 20 + kw : 0) + qq;
      const int rb = (pb < 400 ? (pb / 20 + kh) * 21 + pb % 20 + kw : 0) + qq;
      bf16x8_t af[2], bfr[4];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
        af[mt] = tr8(Yi + (pa + qq) * kW1Ld + 16 * mt + 4 * pp, Yi + (pb + qq) * kW1Ld + 16 * mt + 4 * pp);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        bfr[nt] = tr8(Xi + ra * kW1Ld + 16 * nt + 4 * pp, Xi + rb * kW1Ld + 16 * nt + 4 * pp);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
          acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], bfr[nt], acc[mt][nt], 0, 0, 0);
      if (do_bias) {
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) accb[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], ones, accb[mt], 0, 0, 0);
      }
    }
  }
  if (do_bias && (lane & 15) == 0) {
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) bias_part[(size_t)blockIdx.x * 32 + 16 * mt + 4 * g + r] = accb[mt][r];
  }
  // part[split][cout][kh][kw][c], raw-byte products scaled by 1/255
  float* o = part + (size_t)blockIdx.x * 32 * 256 + kh * 128 + kw * 64;
  const int j = lane & 15;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[(16 * mt + 4 * g + r) * 256 + 16 * nt + j] = acc[mt][nt][r] * kU8Scale;
}


// ----------------------------------------------------------------------------- conv1 forward
// y[n][p][co] = act(scale * sum_{kh,kw,c} X[n][p + (kh, kw)][c] W[co][kh][kw][c] + b[co]) for the
// space-to-depth first layer (21x21x64 uint8 frame -> 20x20x32).  Persistent workgroups
// walk the frames with the next frame prefetched into registers; each frame is converted
// to bf16 ONCE into LDS (the implicit-GEMM loader converted every byte once per tap),
// each tap reads its shifted rows from that image, W stays in registers, and the 400 x 32
// output goes back through LDS as one contiguous 25.6 KB block.
constexpr int kF1Lds = kW1XRows * kW1Ld * 2;

__global__ __launch_bounds__(256, 2) void conv1_fwd_s2d_kernel(const uint8_t* __restrict__ x,
                                                               const uint16_t* __restrict__ w,
                                                               const float* __restrict__ b, uint16_t* __restrict__ y,
                                                               int N, float scale, int relu) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* Xi = smem;  // [441][kW1Ld] frame (bf16 integers 0..255); later [400][40] output
  uint16_t* O = smem;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i = lane & 15, g = lane >> 4;
  // weights -> registers: B fragment (k-step ks, cout tile nt) = W[16nt + i][32ks + 8g .. +7]
  bf16x8_t wf[8][2];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) wf[ks][nt] = *reinterpret_cast<const bf16x8_t*>(w + (16 * nt + i) * 256 + 32 * ks + 8 * g);
  const float b0 = b[i], b1 = b[16 + i];
  constexpr int XC = 441 * 4, XPT = (XC + 255) / 256;
  uint4 rx[XPT];
  auto gload = [&](size_t n) {
    const uint4* xs = reinterpret_cast<const uint4*>(x + n * 441 * 64);
#pragma unroll
    for (int k = 0; k < XPT; ++k) {
      const int q = tid + 256 * k;
      rx[k] = q < XC ? xs[q] : make_uint4(0, 0, 0, 0);
    }
  };
  // persistent over frames; the next frame is prefetched into registers
  if ((int)blockIdx.x < N) gload(blockIdx.x);
  for (int n = blockIdx.x; n < N; n += gridDim.x) {
    __syncthreads();  // the previous frame's output tile has been copied out
#pragma unroll
    for (int k = 0; k < XPT; ++k) {
      const int q = tid + 256 * k;
      if (q < XC) {
        uint16_t* d = Xi + (q >> 2) * kW1Ld + (q & 3) * 16;
        *reinterpret_cast<uint4*>(d) = u8x8_to_bf16x8(make_uint2(rx[k].x, rx[k].y));
        *reinterpret_cast<uint4*>(d + 8) = u8x8_to_bf16x8(make_uint2(rx[k].z, rx[k].w));
      }
    }
    if (n + (int)gridDim.x < N) gload((size_t)n + gridDim.x);
    __syncthreads();
    // 25 pixel tiles of 16; wave w takes tiles w, w + 4, ...
    constexpr int MT = 7;
    f32x4_t acc[MT][2];
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      acc[t][0] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      acc[t][1] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      const int mt = wave + 4 * t;
      if (mt < 25) {
        const int p = 16 * mt + i;
        const int r0 = (p / 20) * 21 + p % 20;  // frame row of tap (0, 0)
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
          const int tap = ks >> 1;  // (kh, kw) = (tap >> 1, tap & 1); 2 k-steps of 32 channels each
          const int row = r0 + (tap >> 1) * 21 + (tap & 1);
          const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(Xi + row * kW1Ld + 32 * (ks & 1) + 8 * g);
          acc[t][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wf[ks][0], acc[t][0], 0, 0, 0);
          acc[t][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wf[ks][1], acc[t][1], 0, 0, 0);
        }
      }
    }
    __syncthreads();  // the frame image is dead: reuse the LDS for the output tile [400][40]
#pragma unroll
    for (int t = 0; t < MT; ++t) {
      const int mt = wave + 4 * t;
      if (mt < 25) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int p = 16 * mt + 4 * g + r;
          float v0 = scale * acc[t][0][r] + b0, v1 = scale * acc[t][1][r] + b1;
          if (relu) {
            v0 = fmaxf(v0, 0.f);
            v1 = fmaxf(v1, 0.f);
          }
          O[p * 40 + i] = f2bf(v0);
          O[p * 40 + 16 + i] = f2bf(v1);
        }
      }
    }
    __syncthreads();
    uint4* yd = reinterpret_cast<uint4*>(y + (size_t)n * 400 * 32);
    for (int q = tid; q < 400 * 4; q += 256) yd[q] = *reinterpret_cast<const uint4*>(O + (q >> 2) * 40 + (q & 3) * 8);
  }
}

// ----------------------------------------------------------------------------- conv2 dgrad
// da1 = conv^T(da2, W2) * (a1 > 0) for the Nature CNN's second layer (20x20x32 input, 4x4
// stride-2 taps, 9x9x64 output).  Persistent workgroups walk the images; wave w owns the
// phase class (ph, pw) = (w >> 1, w & 1) of input pixels (ih, iw) = (ph + 2a, pw + 2b), a
// 100 x 32 GEMM over (tap (i, j), co) whose A operand reads da2[a - i][b - j] straight out
// of a zero-bordered 11x11 LDS image of the output gradient (no per-tap global re-reads:
// the implicit-GEMM path fetched every da2 element 16 times), B = this class's W2 taps held
// in registers.  The 400 x 32 result goes through LDS and leaves as contiguous 16-byte
// chunks, masked by a1 on the way out.
constexpr int kD2Ld = 72;                  // da2 image row: 64 co + 8 pad (bf16)
constexpr int kD2Rows = 121;               // (oh + 1) * 11 + (ow + 1), oh, ow in -1 .. 9
constexpr int kD2OutLd = 40;               // staging row: 32 c + 8 pad
constexpr int kD2Lds = (kD2Rows * kD2Ld + 400 * kD2OutLd) * 2;

__global__ __launch_bounds__(256, 2) void conv2_dgrad_kernel(const uint16_t* __restrict__ dy,
                                                             const uint16_t* __restrict__ w,
                                                             const uint16_t* __restrict__ xact,
                                                             uint16_t* __restrict__ dx, int N) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* Yi = smem;                      // [121][72] da2, zero border
  uint16_t* O = smem + kD2Rows * kD2Ld;      // [400][40] unmasked da1
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i16 = lane & 15, g = lane >> 4;
  const int ph = wave >> 1, pw = wave & 1;
  // B fragments: k-step ks = (tap t = ks >> 1, co block (ks & 1) * 32), n tile nt:
  // W2[co0 + 8g + e][ph + 2 (t >> 1)][pw + 2 (t & 1)][16 nt + i16], e = 0..7
  bf16x8_t wf[8][2];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) {
    const int t = ks >> 1, kh = ph + 2 * (t >> 1), kw = pw + 2 * (t & 1), co0 = (ks & 1) * 32 + 8 * g;
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      typedef short s16x8_t __attribute__((ext_vector_type(8)));
      s16x8_t v;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (short)w[(((co0 + e) * 4 + kh) * 4 + kw) * 32 + 16 * nt + i16];
      wf[ks][nt] = __builtin_bit_cast(bf16x8_t, v);
    }
  }
  // zero the border rows of the da2 image once (the interior is rewritten per image)
  for (int q = tid; q < kD2Rows * (kD2Ld / 8); q += 256) {
    const int r = q / (kD2Ld / 8), oh = r / 11 - 1, ow = r % 11 - 1;
    if (oh < 0 || oh > 8 || ow < 0 || ow > 8)
      *reinterpret_cast<uint4*>(Yi + r * kD2Ld + 8 * (q % (kD2Ld / 8))) = make_uint4(0, 0, 0, 0);
  }
  constexpr int YC = 81 * 8, YPT = (YC + 255) / 256;  // 16-byte chunks of one da2 image
  uint4 ry[YPT];
  auto gload = [&](int n) {
    const uint4* ys = reinterpret_cast<const uint4*>(dy + (size_t)n * 81 * 64);
#pragma unroll
    for (int k = 0; k < YPT; ++k) {
      const int q = tid + 256 * k;
      ry[k] = q < YC ? ys[q] : make_uint4(0, 0, 0, 0);
    }
  };
  if ((int)blockIdx.x < N) gload(blockIdx.x);
  for (int n = blockIdx.x; n < N; n += gridDim.x) {
    __syncthreads();  // the previous image's staging tile has been copied out
#pragma unroll
    for (int k = 0; k < YPT; ++k) {
      const int q = tid + 256 * k;
      if (q < YC) {
        const int pix = q >> 3, oh = pix / 9, ow = pix - oh * 9;
        *reinterpret_cast<uint4*>(Yi + ((oh + 1) * 11 + ow + 1) * kD2Ld + (q & 7) * 8) = ry[k];
      }
    }
    if (n + (int)gridDim.x < N) gload(n + gridDim.x);
    // this image's activation mask, fetched now so its latency hides behind the MFMAs
    constexpr int XC = 400 * 4, XPT = (XC + 255) / 256;
    uint4 rm[XPT];
    const uint4* xa = reinterpret_cast<const uint4*>(xact + (size_t)n * 400 * 32);
#pragma unroll
    for (int k = 0; k < XPT; ++k) {
      const int q = tid + 256 * k;
      rm[k] = q < XC ? xa[q] : make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    // class GEMM: 7 tiles of 16 pixels (a, b) = (p / 10, p % 10), p < 100, in two batches of
    // 4 and 3 tiles.  k-step outer, tiles inner: 8 / 6 independent accumulators per k-step
    // with their fragment reads batched ahead (a tile-outer loop chained 8 dependent MFMAs
    // per accumulator); all 7 tiles at once spilled
    auto class_tiles = [&](auto tag) {
      constexpr int T0 = decltype(tag)::value, NT = T0 == 0 ? 4 : 3;
      f32x4_t acc0[NT], acc1[NT];
      int rb[NT];
#pragma unroll
      for (int u = 0; u < NT; ++u) {
        acc0[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        acc1[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        const int p = 16 * (T0 + u) + i16;
        const int pc = p < 100 ? p : 0;  // rows past the class are computed and discarded
        const int a = pc / 10, b = pc - a * 10;
        rb[u] = (a + 1) * 11 + (b + 1);
      }
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        const int t = ks >> 1, ti = t >> 1, tj = t & 1;
        const int off = -(ti * 11 + tj) * kD2Ld + (ks & 1) * 32 + 8 * g;
        bf16x8_t af[NT];
#pragma unroll
        for (int u = 0; u < NT; ++u) af[u] = *reinterpret_cast<const bf16x8_t*>(Yi + rb[u] * kD2Ld + off);
#pragma unroll
        for (int u = 0; u < NT; ++u) {
          acc0[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[u], wf[ks][0], acc0[u], 0, 0, 0);
          acc1[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[u], wf[ks][1], acc1[u], 0, 0, 0);
        }
      }
#pragma unroll
      for (int u = 0; u < NT; ++u)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int q = 16 * (T0 + u) + 4 * g + r;
          if (q < 100) {
            const int aa = q / 10, bb = q - aa * 10;
            const int pix = (ph + 2 * aa) * 20 + pw + 2 * bb;
            O[pix * kD2OutLd + i16] = f2bf(acc0[u][r]);
            O[pix * kD2OutLd + 16 + i16] = f2bf(acc1[u][r]);
          }
        }
    };
    class_tiles(std::integral_constant<int, 0>{});
    class_tiles(std::integral_constant<int, 4>{});
    __syncthreads();
    uint4* xd = reinterpret_cast<uint4*>(dx + (size_t)n * 400 * 32);
#pragma unroll
    for (int k = 0; k < XPT; ++k) {
      const int q = tid + 256 * k;
      if (q < XC) {
        const uint4 v = *reinterpret_cast<const uint4*>(O + (q >> 2) * kD2OutLd + (q & 3) * 8);
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = bf16x8_at(rm[k], e) > 0.f ? bf16x8_at(v, e) : 0.f;
        xd[q] = pack_bf16x8(o);
      }
    }
  }
}


// ----------------------------------------------------------------------------- conv2/3 forward
// y = relu(conv(x, W) + b) for the Nature CNN's bf16 layers (20x20x32 -> 9x9x64, 4x4 s2;
// 9x9x64 -> 7x7x64, 3x3 s1).  Persistent workgroups walk the images with the next image
// prefetched into registers: the input image goes into LDS once (the implicit-GEMM loader
// fetched each input element once per overlapping tap), wave w computes output channels
// 16w..16w+15 with its W slice in registers (K / 32 fragments), and the OHxOWx64 result
// leaves through LDS as one contiguous block.
template <int H, int W, int C, int KH, int KW, int S, int OH, int OW>
__global__ __launch_bounds__(256, 2) void conv_fwd_img_kernel(const uint16_t* __restrict__ x,
                                                              const uint16_t* __restrict__ w,
                                                              const float* __restrict__ b, uint16_t* __restrict__ y,
                                                              int N, int relu) {
  constexpr int CO = 64, K = KH * KW * C, KS = K / 32, CB = C / 32;
  constexpr int P = OH * OW, MT = (P + 15) / 16;
  constexpr int XLD = C + 8, OLD = CO + 8;
  constexpr int XC = H * W * C / 8, XPT = (XC + 255) / 256;  // 16-byte chunks of one input image
  static_assert(C % 32 == 0, "k-steps of 32 channels");
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* Xi = smem;  // [H*W][XLD]
  uint16_t* O = smem;   // [P][OLD] after the MFMAs (aliases the input image)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i = lane & 15, g = lane >> 4;
  bf16x8_t wf[KS];  // B operand: W[16 wave + i][8g .. 8g+7 of k-step ks]
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) wf[ks] = *reinterpret_cast<const bf16x8_t*>(w + (size_t)(16 * wave + i) * K + 32 * ks + 8 * g);
  const float bias = b[16 * wave + i];
  uint4 rx[XPT];
  auto gload = [&](int n) {
    const uint4* xs = reinterpret_cast<const uint4*>(x + (size_t)n * H * W * C);
#pragma unroll
    for (int k = 0; k < XPT; ++k) {
      const int q = tid + 256 * k;
      rx[k] = q < XC ? xs[q] : make_uint4(0, 0, 0, 0);
    }
  };
  if ((int)blockIdx.x < N) gload(blockIdx.x);
  for (int n = blockIdx.x; n < N; n += gridDim.x) {
    __syncthreads();  // the previous image's output has been copied out
#pragma unroll
    for (int k = 0; k < XPT; ++k) {
      const int q = tid + 256 * k;
      if (q < XC) *reinterpret_cast<uint4*>(Xi + (q / (C / 8)) * XLD + (q % (C / 8)) * 8) = rx[k];
    }
    if (n + (int)gridDim.x < N) gload(n + gridDim.x);
    __syncthreads();
    f32x4_t acc[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      acc[mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      const int p = 16 * mt + i;
      const int pc = p < P ? p : 0;  // rows past the image are computed and discarded
      const int oh = pc / OW, ow = pc - oh * OW;
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const int tap = ks / CB, kh = tap / KW, kw = tap - kh * KW;
        const int row = (oh * S + kh) * W + ow * S + kw;
        const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(Xi + row * XLD + 32 * (ks % CB) + 8 * g);
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wf[ks], acc[mt], 0, 0, 0);
      }
    }
    __syncthreads();  // the input image is dead: reuse the LDS for the output tile
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int p = 16 * mt + 4 * g + r;
        if (p < P) {
          float v = acc[mt][r] + bias;
          if (relu) v = fmaxf(v, 0.f);
          O[p * OLD + 16 * wave + i] = f2bf(v);
        }
      }
    }
    __syncthreads();
    uint4* yd = reinterpret_cast<uint4*>(y + (size_t)n * P * CO);
    for (int q = tid; q < P * CO / 8; q += 256)
      yd[q] = *reinterpret_cast<const uint4*>(O + (q / (CO / 8)) * OLD + (q % (CO / 8)) * 8);
  }
}

template <int H, int W, int C, int KH, int KW, int S, int OH, int OW>
static int launch_conv_fwd_img(const uint16_t* x, const uint16_t* w, const float* b, uint16_t* y, int N, int relu,
                               hipStream_t st) {
  constexpr int lds = (H * W * (C + 8) > OH * OW * 72 ? H * W * (C + 8) : OH * OW * 72) * 2;
  auto kern = conv_fwd_img_kernel<H, W, C, KH, KW, S, OH, OW>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = true;
  }
  if (N < 1) return 0;
  const int grid = N < 512 ? N : 512;  // 2 resident workgroups per CU
  hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, st, x, w, b, y, N, relu);
  return (int)hipGetLastError();
}


// ----------------------------------------------------------------------------- conv3 dgrad
// da2 = conv^T(da3, W3) * (a2 > 0) for the third layer (9x9x64 input, 3x3 stride-1 taps,
// 7x7x64 output): per image an 81 x 64 GEMM over (tap, co) whose A operand reads da3 from
// an LDS image with a 2-pixel zero border; wave w owns input channels 16w..16w+15 with its
// W3 taps in registers; the mask is prefetched and the result leaves as 16-byte chunks.
constexpr int kD3Ld = 72;    // [121 bordered da3 pixels][64 co + 8]
constexpr int kD3OutLd = 72;  // [81][64 c + 8]
constexpr int kD3Lds = (121 * kD3Ld + 81 * kD3OutLd) * 2;

__global__ __launch_bounds__(256, 2) void conv3_dgrad_kernel(const uint16_t* __restrict__ dy,
                                                             const uint16_t* __restrict__ w,
                                                             const uint16_t* __restrict__ xact,
                                                             uint16_t* __restrict__ dx, int N) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* Yi = smem;                 // (oh + 2) * 11 + (ow + 2), oh, ow in -2 .. 8
  uint16_t* O = smem + 121 * kD3Ld;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i16 = lane & 15, g = lane >> 4;
  // B fragments: k-step ks = (tap t = ks >> 1, co block (ks & 1) * 32):
  // W3[co0 + 8g + e][t / 3][t % 3][16 wave + i16]
  bf16x8_t wf[18];
#pragma unroll
  for (int ks = 0; ks < 18; ++ks) {
    const int t = ks >> 1, co0 = (ks & 1) * 32 + 8 * g;
    typedef short s16x8_t __attribute__((ext_vector_type(8)));
    s16x8_t v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (short)w[((co0 + e) * 9 + t) * 64 + 16 * wave + i16];
    wf[ks] = __builtin_bit_cast(bf16x8_t, v);
  }
  for (int q = tid; q < 121 * (kD3Ld / 8); q += 256) {
    const int r = q / (kD3Ld / 8), oh = r / 11 - 2, ow = r % 11 - 2;
    if (oh < 0 || oh > 6 || ow < 0 || ow > 6)
      *reinterpret_cast<uint4*>(Yi + r * kD3Ld + 8 * (q % (kD3Ld / 8))) = make_uint4(0, 0, 0, 0);
  }
  constexpr int YC = 49 * 8, YPT = (YC + 255) / 256, XC = 81 * 8, XPT = (XC + 255) / 256;
  uint4 ry[YPT];
  auto gload = [&](int n) {
    const uint4* ys = reinterpret_cast<const uint4*>(dy + (size_t)n * 49 * 64);
#pragma unroll
    for (int k = 0; k < YPT; ++k) {
      const int q = tid + 256 * k;
      ry[k] = q < YC ? ys[q] : make_uint4(0, 0, 0, 0);
    }
  };
  if ((int)blockIdx.x < N) gload(blockIdx.x);
  for (int n = blockIdx.x; n < N; n += gridDim.x) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < YPT; ++k) {
      const int q = tid + 256 * k;
      if (q < YC) {
        const int pix = q >> 3, oh = pix / 7, ow = pix - oh * 7;
        *reinterpret_cast<uint4*>(Yi + ((oh + 2) * 11 + ow + 2) * kD3Ld + (q & 7) * 8) = ry[k];
      }
    }
    if (n + (int)gridDim.x < N) gload(n + gridDim.x);
    uint4 rm[XPT];
    const uint4* xa = reinterpret_cast<const uint4*>(xact + (size_t)n * 81 * 64);
#pragma unroll
    for (int k = 0; k < XPT; ++k) {
      const int q = tid + 256 * k;
      rm[k] = q < XC ? xa[q] : make_uint4(0, 0, 0, 0);
    }
    __syncthreads();
    // k-step outer, 6 independent tile accumulators inner (reads batched ahead)
    {
      f32x4_t acc[6];
      int rb[6];
#pragma unroll
      for (int mt = 0; mt < 6; ++mt) {
        acc[mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        const int p = 16 * mt + i16;
        const int pc = p < 81 ? p : 0;
        const int ih = pc / 9, iw = pc - ih * 9;
        rb[mt] = (ih + 2) * 11 + (iw + 2);
      }
#pragma unroll
      for (int ks = 0; ks < 18; ++ks) {
        const int t = ks >> 1, kh = t / 3, kw = t - kh * 3;
        const int off = -(kh * 11 + kw) * kD3Ld + (ks & 1) * 32 + 8 * g;
        bf16x8_t af[6];
#pragma unroll
        for (int mt = 0; mt < 6; ++mt) af[mt] = *reinterpret_cast<const bf16x8_t*>(Yi + rb[mt] * kD3Ld + off);
#pragma unroll
        for (int mt = 0; mt < 6; ++mt) acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], wf[ks], acc[mt], 0, 0, 0);
      }
#pragma unroll
      for (int mt = 0; mt < 6; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int q = 16 * mt + 4 * g + r;
          if (q < 81) O[q * kD3OutLd + 16 * wave + i16] = f2bf(acc[mt][r]);
        }
    }
    __syncthreads();
    uint4* xd = reinterpret_cast<uint4*>(dx + (size_t)n * 81 * 64);
#pragma unroll
    for (int k = 0; k < XPT; ++k) {
      const int q = tid + 256 * k;
      if (q < XC) {
        const uint4 v = *reinterpret_cast<const uint4*>(O + (q >> 3) * kD3OutLd + (q & 7) * 8);
        float o[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = bf16x8_at(rm[k], e) > 0.f ? bf16x8_at(v, e) : 0.f;
        xd[q] = pack_bf16x8(o);
      }
    }
  }
}

}  // namespace rrl

using namespace rrl;

static int rrl_gemm_splits_impl(int R, int splits) {
  splits = splits < 1 ? 1 : splits;
  int kps = (R + splits - 1) / splits;
  kps = (kps + kGemmBK - 1) / kGemmBK * kGemmBK;
  return (R + kps - 1) / kps;
}

static int grid_for(size_t n, int per_block = 256, int cap = 4096) {
  size_t g = (n + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > (size_t)cap) g = cap;
  return (int)g;
}

// Rollout head with the weights streamed from L1 / L2 per row (a2c_rollout_row_streamed,
// bitwise the a2c_head_kernel<false> result) instead of held in 80 registers: 79 VGPRs, 6 waves
// per SIMD instead of a2c_head_kernel's 3 (139 VGPRs) -- the rollout head from 4,096 rows.
template <int AMAX>
__global__ void __launch_bounds__(256) a2c_head_streamed_kernel(HeadArgs a) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  for (int row = blockIdx.x * 4 + wave; row < a.B; row += gridDim.x * 4)
    (void)a2c_rollout_row_streamed<AMAX>(a, row, lane);
}

// The head backward with the same streamed weights (float4 pairs re-read per row from L1 for
// the logits and again for dh, 107 VGPRs instead of 160): bitwise the a2c_head_kernel<true>
// result (same products, same order), 4 waves per SIMD instead of 3 -- and slower (the L1
// re-reads cost more than the waves gain), so opt-in: RRL_HEAD_STREAMED=1.
template <int AMAX>
__global__ void __launch_bounds__(256) a2c_head_train_streamed_kernel(HeadArgs a) {
  __shared__ float red[16];
  const int A = a.A, F = kHeadF;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float st_pg = 0.f, st_vf = 0.f, st_ent = 0.f, st_n = 0.f;
  for (int row = blockIdx.x * 4 + wave; row < a.B; row += gridDim.x * 4) {
    const uint4 hv = *reinterpret_cast<const uint4*>(a.h + (size_t)row * F + 8 * lane);
    const int act = a.act_in[row];
    const float adv = a.adv[row], ret = a.ret[row];
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
    float wv[8];
    {
      const float4 v0 = *reinterpret_cast<const float4*>(a.w_v + 8 * lane);
      const float4 v1 = *reinterpret_cast<const float4*>(a.w_v + 8 * lane + 4);
      wv[0] = v0.x; wv[1] = v0.y; wv[2] = v0.z; wv[3] = v0.w; wv[4] = v1.x; wv[5] = v1.y; wv[6] = v1.z; wv[7] = v1.w;
    }
    float vsum = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) vsum += wv[i] * x[i];
    const float value = wave_sum(vsum) + a.b_v[0];
#pragma unroll
    for (int o = 0; o < AMAX; ++o) {
      if (o < A) {
        const float4 w0 = *reinterpret_cast<const float4*>(a.w + o * F + 8 * lane);
        const float4 w1 = *reinterpret_cast<const float4*>(a.w + o * F + 8 * lane + 4);
        const float wp[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) s += wp[i] * x[i];
        logits[o] = wave_sum(s) + a.bias[o];
      }
    }
    const CatStats cs = cat_stats(A, logits);
    const float lp = pick_logit(A, logits, act) - cs.lse;
    float dz[kMaxAct];
#pragma unroll
    for (int o = 0; o < kMaxAct; ++o) {
      dz[o] = 0.f;
      if (o < A) {
        const float lpo = logits[o] - cs.lse;
        const float p = __expf(lpo);
        dz[o] = a.inv_B * (-adv * ((o == act ? 1.f : 0.f) - p) + a.ent_coef * p * (lpo + cs.entropy));
      }
    }
    const float dv = a.inv_B * 2.f * a.vf_coef * (value - ret);
    float g[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) g[i] = dv * wv[i];
#pragma unroll
    for (int o = 0; o < AMAX; ++o)
      if (o < A) {
        const float4 w0 = *reinterpret_cast<const float4*>(a.w + o * F + 8 * lane);
        const float4 w1 = *reinterpret_cast<const float4*>(a.w + o * F + 8 * lane + 4);
        const float wp[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
        for (int i = 0; i < 8; ++i) g[i] += dz[o] * wp[i];
      }
    uint32_t ow[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float lo = x[2 * i] > 0.f ? g[2 * i] : 0.f, hi = x[2 * i + 1] > 0.f ? g[2 * i + 1] : 0.f;
      ow[i] = (uint32_t)f2bf(lo) | ((uint32_t)f2bf(hi) << 16);
    }
    *reinterpret_cast<uint4*>(a.dh + (size_t)row * F + 8 * lane) = make_uint4(ow[0], ow[1], ow[2], ow[3]);
    float mine = dv;
#pragma unroll
    for (int o = 0; o < kMaxAct; ++o)
      if (o < A && lane == o) mine = dz[o];
    if (lane <= A) a.dhead[(size_t)row * (A + 1) + lane] = mine;
    if (lane == 0) {
      st_pg += -adv * lp;
      st_vf += (value - ret) * (value - ret);
      st_ent += cs.entropy;
      st_n += 1.f;
    }
  }
  if (lane == 0) {
    red[wave * 4 + 0] = st_pg;
    red[wave * 4 + 1] = st_vf;
    red[wave * 4 + 2] = st_ent;
    red[wave * 4 + 3] = st_n;
  }
  __syncthreads();
  if (threadIdx.x < 4)
    a.stats[blockIdx.x * 4 + threadIdx.x] = red[threadIdx.x] + red[4 + threadIdx.x] + red[8 + threadIdx.x] +
                                            red[12 + threadIdx.x];
}

// The head backward on fp32 MFMA (v_mfma_f32_16x16x4_f32: exact f32 products): one wave per
// 16-row tile.  The register kernel above spends its time in 7 wave-wide reductions and
// ~400 VALU ops per row; here
//   (1) logits + value of 16 rows = hid[16 x 512] . [W; w_v]^T    (128 MFMAs, 4 accumulators),
//       hid staged in LDS (16 x 1,040 B rows), [W; w_v] once per workgroup (16 KiB);
//   (2) 16 lanes (one per row) form the softmax, the loss gradients dz / dv and the stats;
//   (3) dh[16 x 512] = [dz | dv][16 x 8] . [W; w_v]   (32 column tiles x 2 MFMAs), masked by
//       hid > 0 and rounded to bf16 IN PLACE of the hid tile, which then leaves as 16-B rows.
// Same math as a2c_head_kernel<true>; the sums run in another order (fp32-accurate, not
// bitwise).  A <= 7 (A + 1 outputs in one 8-wide k block).
constexpr int kHmRow = 520;                       // hid / dh tile row stride, bf16 elements (1,040 B)
constexpr int kHmWave = 16 * kHmRow * 2 + 16 * 17 * 4 + 16 * 8 * 4;  // 18,240 B of LDS per wave
constexpr int kHmW = 8 * kHeadF * 4;  // [W; w_v; 0] as f32 rows, 16 KiB per workgroup
__global__ void __launch_bounds__(256) a2c_head_train_mfma_kernel(HeadArgs a, int stats_rows) {
  extern __shared__ __attribute__((aligned(16))) unsigned char hm_smem[];
  const int A = a.A, F = kHeadF, B = a.B;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float* Wl = reinterpret_cast<float*>(hm_smem);  // row o < A: W[o]; o == A: w_v; else zeros
  uint16_t* H = reinterpret_cast<uint16_t*>(hm_smem + kHmW + wave * kHmWave);
  float* Lg = reinterpret_cast<float*>(hm_smem + kHmW + wave * kHmWave + 16 * kHmRow * 2);
  float* G = Lg + 16 * 17;
  const int li = lane & 15, q = lane >> 4;
  for (int i = threadIdx.x; i < 8 * F / 4; i += 256) {
    const int o = i / (F / 4), c = i % (F / 4);
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (o < A) v = *reinterpret_cast<const float4*>(a.w + o * F + 4 * c);
    else if (o == A) v = *reinterpret_cast<const float4*>(a.w_v + 4 * c);
    *reinterpret_cast<float4*>(Wl + o * F + 4 * c) = v;
  }
  __syncthreads();
  // this lane's weight row for the B operand of (1): output j = li (rows 8..15 are zero outputs)
  const float* wrow = li < 8 ? Wl + li * F : nullptr;
  float st_pg = 0.f, st_vf = 0.f, st_ent = 0.f, st_n = 0.f;
  const int ntiles = (B + 15) >> 4;
  for (int tile = blockIdx.x * 4 + wave; tile < ntiles; tile += gridDim.x * 4) {
    const int row0 = tile * 16;
    // stage hid rows row0 .. row0 + 15 (rows past B: a clamped duplicate, never stored)
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int c = lane + 64 * t, r = c >> 6, c16 = c & 63;
      const int gr = min(row0 + r, B - 1);
      *reinterpret_cast<uint4*>(H + r * kHmRow + c16 * 8) =
          *reinterpret_cast<const uint4*>(a.h + (size_t)gr * F + c16 * 8);
    }
    // per-row inputs for (2), loaded early
    int act = 0;
    float adv = 0.f, ret = 0.f;
    const int myrow = row0 + li;
    if (lane < 16 && myrow < B) {
      act = a.act_in[myrow];
      adv = a.adv[myrow];
      ret = a.ret[myrow];
    }
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    // (1): lane (li, q) covers k = 128 q .. 128 q + 127 of row li (A operand) and of output li (B)
    f32x4_t acc[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
    const uint16_t* hr = H + li * kHmRow + 128 * q;
#pragma unroll 2
    for (int s8 = 0; s8 < 16; ++s8) {
      const uint4 hv = *reinterpret_cast<const uint4*>(hr + 8 * s8);
      float4 w0 = make_float4(0.f, 0.f, 0.f, 0.f), w1 = w0;
      if (wrow) {
        w0 = *reinterpret_cast<const float4*>(wrow + 128 * q + 8 * s8);
        w1 = *reinterpret_cast<const float4*>(wrow + 128 * q + 8 * s8 + 4);
      }
      const uint32_t hw[4] = {hv.x, hv.y, hv.z, hv.w};
      const float wk[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xv = bf2f((uint16_t)(e & 1 ? hw[e >> 1] >> 16 : hw[e >> 1] & 0xffff));
        acc[e & 3] = __builtin_amdgcn_mfma_f32_16x16x4f32(xv, wk[e], acc[e & 3], 0, 0, 0);
      }
    }
    // D[row = 4 q + r][out = li]
#pragma unroll
    for (int r = 0; r < 4; ++r) Lg[(4 * q + r) * 17 + li] = (acc[0][r] + acc[1][r]) + (acc[2][r] + acc[3][r]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    // (2): lane li < 16 owns row row0 + li
    if (lane < 16) {
      float gz[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if (myrow < B) {
        float logits[kMaxAct];
#pragma unroll
        for (int o = 0; o < kMaxAct; ++o) logits[o] = o < A ? Lg[li * 17 + o] + a.bias[o] : -INFINITY;
        const float value = Lg[li * 17 + A] + a.b_v[0];
        const CatStats cs = cat_stats(A, logits);
        const float lp = pick_logit(A, logits, act) - cs.lse;
#pragma unroll
        for (int o = 0; o < 8; ++o)
          if (o < A) {
            const float lpo = logits[o] - cs.lse;
            const float p = __expf(lpo);
            gz[o] = a.inv_B * (-adv * ((o == act ? 1.f : 0.f) - p) + a.ent_coef * p * (lpo + cs.entropy));
          }
        const float dv = a.inv_B * 2.f * a.vf_coef * (value - ret);
#pragma unroll
        for (int o = 0; o < 8; ++o)
          if (o == A) gz[o] = dv;
#pragma unroll
        for (int o = 0; o < 8; ++o)
          if (o <= A) a.dhead[(size_t)myrow * (A + 1) + o] = gz[o];
        st_pg += -adv * lp;
        st_vf += (value - ret) * (value - ret);
        st_ent += cs.entropy;
        st_n += 1.f;
      }
#pragma unroll
      for (int o = 0; o < 8; ++o) G[li * 8 + o] = gz[o];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
    // (3): A operand G[row li][o = q | 4 + q], B operand [W; w_v][o][k = 16 kt + li]
    const float g0 = G[li * 8 + q], g1 = G[li * 8 + 4 + q];
    const float* b0row = Wl + q * F;
    const float* b1row = Wl + (4 + q) * F;
#pragma unroll 4
    for (int kt = 0; kt < 32; ++kt) {
      const int k = 16 * kt + li;
      const float b0 = b0row[k], b1 = b1row[k];
      f32x4_t d = f32x4_t{0.f, 0.f, 0.f, 0.f};
      d = __builtin_amdgcn_mfma_f32_16x16x4f32(g0, b0, d, 0, 0, 0);
      d = __builtin_amdgcn_mfma_f32_16x16x4f32(g1, b1, d, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 4; ++r) {  // D[row = 4 q + r][k]: keep where hid > 0, bf16, in place
        uint16_t* p = H + (4 * q + r) * kHmRow + k;
        const float xv = bf2f(*p);
        *p = f2bf(xv > 0.f ? d[r] : 0.f);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int t = 0; t < 16; ++t) {
      const int c = lane + 64 * t, r = c >> 6, c16 = c & 63;
      if (row0 + r < B)
        *reinterpret_cast<uint4*>(a.dh + (size_t)(row0 + r) * F + c16 * 8) =
            *reinterpret_cast<const uint4*>(H + r * kHmRow + c16 * 8);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();  // the next tile's staging overwrites H
  }
  __shared__ float red[16];
  st_pg = wave_sum(st_pg);
  st_vf = wave_sum(st_vf);
  st_ent = wave_sum(st_ent);
  st_n = wave_sum(st_n);
  if (lane == 0) {
    red[wave * 4 + 0] = st_pg;
    red[wave * 4 + 1] = st_vf;
    red[wave * 4 + 2] = st_ent;
    red[wave * 4 + 3] = st_n;
  }
  __syncthreads();
  if (threadIdx.x < 4)
    a.stats[blockIdx.x * 4 + threadIdx.x] = red[threadIdx.x] + red[4 + threadIdx.x] + red[8 + threadIdx.x] +
                                            red[12 + threadIdx.x];
  if (blockIdx.x == 0)  // stats rows past this grid (the caller sums stats_rows rows)
    for (int i = threadIdx.x; i < (stats_rows - (int)gridDim.x) * 4; i += 256) a.stats[gridDim.x * 4 + i] = 0.f;
}

static bool head_mfma() {  // RRL_HEAD_MFMA=1: the MFMA head backward (A/B), read per call
  const char* e = getenv("RRL_HEAD_MFMA");
  return e && e[0] == '1';
}

// RRL_HEAD_STREAMED (read per call): unset = the streamed rollout head from 4,096 rows (20.0 vs
// 24.5 us per 8,192 rows; 11.1 vs 10.7 us at 2,048) and the register backward; 1 = both
// streamed (the backward measured slower: 80.6 vs 68.3 us at 40,960 rows, 28.6 vs 24.2 at
// 10,240 -- profiles/r5_head_streamed_ab.txt); 0 = neither.
static bool head_streamed(bool train, int B) {
  const char* e = getenv("RRL_HEAD_STREAMED");
  if (e && e[0] == '1') return true;
  if (e && e[0] == '0') return false;
  return !train && B >= 4096;
}

extern "C" {

// Forward conv (or fc as a 1x1 conv on H = W = 1): y bf16 [N*OH*OW][Cout].  When the
// output has too few tiles to fill the chip (the fc layer at rollout batch sizes) and a
// workspace is given, the reduction is split over workgroups into fp32 partials and a
// second kernel applies bias + ReLU.
int rrl_conv_fwd(const void* x, int x_u8, const uint16_t* w, const float* b, uint16_t* y, int N, int H, int W,
                 int C, int KH, int KW, int S, int Cout, int relu, float* work, long long work_elems,
                 void* stream_) {
  hipStream_t st = (hipStream_t)stream_;
  ConvGeom g{N, H, W, C, KH, KW, S, (H - KH) / S + 1, (W - KW) / S + 1, Cout};
  const int M = g.M(), K = g.K();
  if (x_u8 && H == 21 && W == 21 && C == 64 && KH == 2 && KW == 2 && S == 1 && Cout == 32) {
    // PongSynth's space-to-depth first layer: one workgroup per frame (conv1_fwd_s2d_kernel)
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)conv1_fwd_s2d_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                kF1Lds);
      attr = true;
    }
    if (N < 1) return 0;
    const int grid = N < 512 ? N : 512;  // 2 resident workgroups per CU
    hipLaunchKernelGGL(conv1_fwd_s2d_kernel, dim3(grid), dim3(256), kF1Lds, st, (const uint8_t*)x, w, b, y, N,
                       kU8Scale, relu);
    return (int)hipGetLastError();
  }
  if (!x_u8 && H == 20 && W == 20 && C == 32 && KH == 4 && KW == 4 && S == 2 && Cout == 64)
    return launch_conv_fwd_img<20, 20, 32, 4, 4, 2, 9, 9>((const uint16_t*)x, w, b, y, N, relu, st);
  if (!x_u8 && H == 9 && W == 9 && C == 64 && KH == 3 && KW == 3 && S == 1 && Cout == 64)
    return launch_conv_fwd_img<9, 9, 64, 3, 3, 1, 7, 7>((const uint16_t*)x, w, b, y, N, relu, st);
  RowLoader lw{w, Cout, K};
  BiasReluStore epi{y, b, M, Cout, relu != 0, x_u8 ? kU8Scale : 1.0f};
  const int tiles = ((M + 127) / 128) * ((Cout + 63) / 64);
  int splits = 1;
  if (!x_u8 && work != nullptr && Cout >= 64 && tiles < 160 && K >= 1024) {
    splits = (320 + tiles - 1) / tiles;
    if (splits > K / 256) splits = K / 256;
    while (splits > 1 && (long long)splits * M * Cout > work_elems) --splits;
    splits = rrl_gemm_splits_impl(K, splits);
  }
  return with_im2col(g, x, x_u8 != 0, [&](auto lx) -> int {
    if (splits > 1) {
      PartialStore pe{work, M, Cout};
      int rc = launch_gemm<128, 64, false, false>(lx, lw, pe, M, Cout, K, splits, st);
      if (rc) return rc;
      const size_t total = (size_t)M * Cout;
      hipLaunchKernelGGL(bias_act_kernel, dim3(grid_for(total, 256, 8192)), dim3(256), 0, st, work, splits, M,
                         Cout, b, y, relu);
      return (int)hipGetLastError();
    }
    return Cout >= 64 ? launch_gemm<128, 64, false, false>(lx, lw, epi, M, Cout, K, 1, st)
                      : launch_gemm<128, 32, false, false>(lx, lw, epi, M, Cout, K, 1, st);
  });
}

// dY [M][Cout] . W [Cout][K] -> bf16 [M][K] (masked by mask[M][K] > 0 when given).
int rrl_gemm_dgrad(const uint16_t* dy, const uint16_t* w, const uint16_t* mask, uint16_t* out, int M, int Cout,
                   int K, void* stream_) {
  hipStream_t st = (hipStream_t)stream_;
  if (Cout % 8 || K % 8) return -1;
  RowLoader la{dy, M, Cout};
  RowLoader lb{w, Cout, K};
  MaskStore epi{out, mask, M, K};
  return launch_gemm<128, 64, false, true>(la, lb, epi, M, K, Cout, 1, st);
}

// Implicit dgrad + ReLU mask for the supported geometries (-1 otherwise: callers fall
// back to gemm_dgrad + col2im_mask).
int rrl_conv_dgrad(const uint16_t* dy, const uint16_t* w, const uint16_t* xact, uint16_t* dx, int N, int H, int W,
                   int C, int KH, int KW, int S, int Cout, void* stream_) {
  hipStream_t st = (hipStream_t)stream_;
  if (H == 20 && W == 20 && C == 32 && KH == 4 && KW == 4 && S == 2 && Cout == 64) {
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)conv2_dgrad_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, kD2Lds);
      attr = true;
    }
    if (N < 1) return 0;
    const int grid = N < 512 ? N : 512;  // 2 resident workgroups per CU (190 VGPRs)
    hipLaunchKernelGGL(conv2_dgrad_kernel, dim3(grid), dim3(256), kD2Lds, st, dy, w, xact, dx, N);
    return (int)hipGetLastError();
  }
  if (H == 9 && W == 9 && C == 64 && KH == 3 && KW == 3 && S == 1 && Cout == 64) {
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)conv3_dgrad_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, kD3Lds);
      attr = true;
    }
    if (N < 1) return 0;
    const int grid = N < 512 ? N : 512;
    hipLaunchKernelGGL(conv3_dgrad_kernel, dim3(grid), dim3(256), kD3Lds, st, dy, w, xact, dx, N);
    return (int)hipGetLastError();
  }
  return -1;
}

int rrl_col2im_mask(const uint16_t* dcol, const uint16_t* xact, uint16_t* dx, int N, int H, int W, int C, int KH,
                    int KW, int S, void* stream_) {
  hipStream_t st = (hipStream_t)stream_;
  ConvGeom g{N, H, W, C, KH, KW, S, (H - KH) / S + 1, (W - KW) / S + 1, 0};
  if (C % 8) return -1;
  const size_t total = (size_t)N * H * W * (C / 8);
  hipLaunchKernelGGL(col2im_mask_kernel, dim3(grid_for(total, 256, 16384)), dim3(256), 0, st, dcol, xact, dx, g);
  return (int)hipGetLastError();
}

// dW partials: part [splits][Cout][K] = dY^T . im2col(X) over each split's rows.
// The GEMM is computed transposed -- rows = the conv's K (long), cols = Cout (32 / 64 /
// 512) -- so the wide im2col operand gets the 128-row tile and the epilogue stores 4
// consecutive k of one output channel as one 16-byte write.
int rrl_conv_wgrad(const uint16_t* dy, const void* x, int x_u8, float* part, float* bias_part, int splits, int N,
                   int H, int W, int C, int KH, int KW, int S, int Cout, void* stream_) {
  hipStream_t st = (hipStream_t)stream_;
  ConvGeom g{N, H, W, C, KH, KW, S, (H - KH) / S + 1, (W - KW) / S + 1, Cout};
  const int M = g.M(), K = g.K();
  if (x_u8 && H == 21 && W == 21 && C == 64 && KH == 2 && KW == 2 && S == 1 && Cout == 32) {
    // PongSynth's space-to-depth first layer: one streaming pass (conv1_wgrad_s2d_kernel);
    // same number of partial slabs as the GEMM path would use
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)conv1_wgrad_s2d_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                kW1Lds);
      attr = true;
    }
    const int grid = rrl_gemm_splits_impl(M, splits);
    hipLaunchKernelGGL(conv1_wgrad_s2d_kernel, dim3(grid), dim3(256), kW1Lds, st, (const uint8_t*)x, dy, part,
                       bias_part, N);
    return (int)hipGetLastError();
  }
  if (bias_part != nullptr) {  // bias partials [splits][Cout] from the column-sum kernel
    if (Cout % 8 || Cout > 2048) return -1;
    hipLaunchKernelGGL(colsum_kernel, dim3(rrl_gemm_splits_impl(M, splits)), dim3(256), 256 * 8 * sizeof(float), st,
                       dy, M, Cout, bias_part);
    const int rc = (int)hipGetLastError();
    if (rc) return rc;
  }
  RowLoader ly{dy, M, Cout};
  PartialStoreT epi{part, K, Cout, x_u8 ? kU8Scale : 1.0f};
  return with_im2col(g, x, x_u8 != 0, [&](auto lx) -> int {
    return Cout >= 64 ? launch_gemm<128, 64, true, true>(lx, ly, epi, K, Cout, M, splits, st)
                      : launch_gemm<128, 32, true, true>(lx, ly, epi, K, Cout, M, splits, st);
  });
}

// Actual number of splits launch_gemm uses for a reduction of length R.
int rrl_gemm_splits(int R, int splits) { return rrl_gemm_splits_impl(R, splits); }

// count segments (<= 8), each part / out 16-byte aligned with n % 4 == 0
int rrl_sum_splits_multi(const float* const* parts, const int* splits, const long long* ns, float* const* outs,
                         int count, void* stream_) {
  if (count < 1 || count > kMaxSumSegs) return -1;
  SumSegs sg{};
  sg.count = count;
  bool few = true;
  for (int q = 0; q < count; ++q) few = few && splits[q] <= kFewSplits;
  int blocks = 0;
  for (int q = 0; q < count; ++q) {
    if (((uintptr_t)parts[q] & 15) || ((uintptr_t)outs[q] & 15) || (ns[q] & 3) || splits[q] < 1) return -1;
    sg.part[q] = parts[q];
    sg.out[q] = outs[q];
    sg.n[q] = ns[q];
    sg.splits[q] = splits[q];
    sg.first[q] = blocks;
    blocks += few ? (int)((ns[q] / 4 + 255) / 256) : (int)((ns[q] / 4 + 15) / 16);
  }
  sg.first[count] = blocks;
  if (few)
    hipLaunchKernelGGL(sum_splits_few_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream_, sg);
  else
    hipLaunchKernelGGL(sum_splits_multi_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream_, sg);
  return (int)hipGetLastError();
}

int rrl_sum_splits(const float* part, int splits, long long n, float* out, void* stream_) {
  hipStream_t st = (hipStream_t)stream_;
  if (((uintptr_t)part & 15) || ((uintptr_t)out & 15) || (n & 3)) {  // float4 path needs aligned rows
    hipLaunchKernelGGL(sum_splits_scalar_kernel, dim3((unsigned)((n + 63) / 64)), dim3(1024), 0, st, part, splits,
                       (size_t)n, out);
    return (int)hipGetLastError();
  }
  const size_t blocks = ((size_t)n / 4 + 15) / 16;
  hipLaunchKernelGGL(sum_splits_kernel, dim3((unsigned)(blocks < 1 ? 1 : blocks)), dim3(256), 0, st, part, splits,
                     (size_t)n, out);
  return (int)hipGetLastError();
}

int rrl_colsum(const uint16_t* y, int M, int C, float* part, int splits, void* stream_) {
  hipStream_t st = (hipStream_t)stream_;
  if (C % 8 || C > 2048 || splits < 1) return -1;
  hipLaunchKernelGGL(colsum_kernel, dim3(splits), dim3(256), 256 * 8 * sizeof(float), st, y, M, C, part);
  return (int)hipGetLastError();
}

int rrl_sumsq(const float* x, long long n, float* work, int work_n, float* out, void* stream_) {
  hipStream_t st = (hipStream_t)stream_;
  const int g = work_n < 1 ? 1 : (work_n > 1024 ? 1024 : work_n);
  if ((reinterpret_cast<uintptr_t>(x) & 15) == 0)
    hipLaunchKernelGGL(sumsq_partial_kernel<true>, dim3(g), dim3(256), 0, st, x, (size_t)n, work);
  else
    hipLaunchKernelGGL(sumsq_partial_kernel<false>, dim3(g), dim3(256), 0, st, x, (size_t)n, work);
  hipLaunchKernelGGL(sum_small_kernel, dim3(1), dim3(256), 0, st, work, g, out);
  return (int)hipGetLastError();
}

// sum-of-squares partials only (the clip + Adam launch reduces them itself, norm_parts = the return)
int rrl_sumsq_partial(const float* x, long long n, float* work, int work_n, void* stream_) {
  hipStream_t st = (hipStream_t)stream_;
  const int g = work_n < 1 ? 1 : (work_n > 1024 ? 1024 : work_n);
  if ((reinterpret_cast<uintptr_t>(x) & 15) == 0)
    hipLaunchKernelGGL(sumsq_partial_kernel<true>, dim3(g), dim3(256), 0, st, x, (size_t)n, work);
  else
    hipLaunchKernelGGL(sumsq_partial_kernel<false>, dim3(g), dim3(256), 0, st, x, (size_t)n, work);
  const int rc = (int)hipGetLastError();
  return rc != 0 ? -rc : g;
}

// norm_parts > 0: norm_sq holds that many sum-of-squares partials (rrl_sumsq_partial)
int rrl_adam_clip(float* p, float* m, float* v, const float* g, uint16_t* shadow, long long n, const float* norm_sq,
                  float max_norm, float lr, float b1, float b2, float eps, int step, const long long* step_dev,
                  int norm_parts, void* stream_) {
  hipStream_t st = (hipStream_t)stream_;
  const float bc1 = 1.f - powf(b1, (float)step), bc2 = 1.f - powf(b2, (float)step);
  const bool vec = ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(m) | reinterpret_cast<uintptr_t>(v) |
                     reinterpret_cast<uintptr_t>(g)) & 15) == 0 && (reinterpret_cast<uintptr_t>(shadow) & 7) == 0;
  if (vec)
    hipLaunchKernelGGL(adam_clip4_kernel, dim3(grid_for((size_t)(n / 4 + 1), 256, 8192)), dim3(256), 0, st, p, m, v, g,
                       shadow, (size_t)n, norm_sq, max_norm, lr, b1, b2, eps, bc1, bc2, step_dev, norm_parts);
  else
    hipLaunchKernelGGL(adam_clip_kernel, dim3(grid_for((size_t)n, 256, 8192)), dim3(256), 0, st, p, m, v, g, shadow,
                       (size_t)n, norm_sq, max_norm, lr, b1, b2, eps, bc1, bc2, step_dev, norm_parts);
  return (int)hipGetLastError();
}

struct CounterAdds {
  long long* c[4];
  long long inc[4];
  int n;
};
__global__ void counter_add_kernel(CounterAdds a) {
  if ((int)threadIdx.x < a.n) a.c[threadIdx.x][0] += a.inc[threadIdx.x];
}

// Device-side step counters advanced inside captured graphs (up to 4 in one launch: the Pong
// update's sampling, env and Adam counters were three single-thread launches).
int rrl_counter_add_n(long long* const* c, const long long* inc, int n, void* stream_) {
  if (n < 1 || n > 4) return -1;
  CounterAdds a{};
  for (int i = 0; i < n; ++i) {
    a.c[i] = c[i];
    a.inc[i] = inc[i];
  }
  a.n = n;
  hipLaunchKernelGGL(counter_add_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream_, a);
  return (int)hipGetLastError();
}

int rrl_counter_add(long long* c, long long inc, void* stream_) { return rrl_counter_add_n(&c, &inc, 1, stream_); }

int rrl_to_bf16(const float* x, uint16_t* y, long long n, void* stream_) {
  hipStream_t st = (hipStream_t)stream_;
  hipLaunchKernelGGL(to_bf16_kernel, dim3(grid_for((size_t)n, 256, 8192)), dim3(256), 0, st, x, y, (size_t)n);
  return (int)hipGetLastError();
}

// mode 0: rollout (sample act / logp / value), 1: training (dh, dhead, stats).
int rrl_a2c_head(int mode, const uint16_t* h, const float* head_params, int B, int A, int32_t* act, float* logp,
                 float* value, float* logits_out, unsigned long long seed, unsigned long long step,
                 const unsigned long long* step_base, int row_offset,
                 const int32_t* act_in, const float* adv, const float* ret, float inv_B, float vf_coef,
                 float ent_coef, uint16_t* dh, float* dhead, float* stats, int grid, const float* part,
                 int splits, const float* fc_b, uint16_t* h_out, void* stream_) {
  hipStream_t st = (hipStream_t)stream_;
  if (A < 1 || A > kMaxAct) return -1;
  if (part && (mode != 0 || !fc_b || !h_out || splits < 1)) return -1;
  HeadArgs a;
  a.part = part;
  a.splits = splits;
  a.fc_b = fc_b;
  a.h_out = h_out;
  a.h = h;
  a.w = head_params;
  a.bias = head_params + A * kHeadF;
  a.w_v = a.bias + A;
  a.b_v = a.w_v + kHeadF;
  a.B = B;
  a.A = A;
  a.act = act;
  a.logp = logp;
  a.value = value;
  a.logits_out = logits_out;
  a.seed_lo = (uint32_t)seed;
  a.seed_hi = (uint32_t)(seed >> 32);
  a.step_lo = (uint32_t)step;
  a.step_hi = (uint32_t)(step >> 32);
  a.step_base = step_base;
  a.row_offset = row_offset;
  a.act_in = act_in;
  a.adv = adv;
  a.ret = ret;
  a.inv_B = inv_B;
  a.vf_coef = vf_coef;
  a.ent_coef = ent_coef;
  a.dh = dh;
  a.dhead = dhead;
  a.stats = stats;
  if (mode != 0 && A <= 7 && head_mfma()) {
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)a2c_head_train_mfma_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                kHmW + 4 * kHmWave);
      attr = true;
    }
    const int ntiles = (B + 15) / 16;
    const int g = std::max(1, std::min(grid, (ntiles + 3) / 4));
    hipLaunchKernelGGL(a2c_head_train_mfma_kernel, dim3(g), dim3(256), kHmW + 4 * kHmWave, st, a, grid);
    return (int)hipGetLastError();
  }
  if (A <= 8 && head_streamed(mode != 0, B)) {
    if (mode == 0 && part && !logits_out) {
      hipLaunchKernelGGL((a2c_head_streamed_kernel<8>), dim3(grid), dim3(256), 0, st, a);
      return (int)hipGetLastError();
    }
    if (mode != 0) {
      hipLaunchKernelGGL((a2c_head_train_streamed_kernel<8>), dim3(grid), dim3(256), 0, st, a);
      return (int)hipGetLastError();
    }
  }
  if (A <= 8) {
    if (mode == 0) hipLaunchKernelGGL((a2c_head_kernel<false, 8>), dim3(grid), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((a2c_head_kernel<true, 8>), dim3(grid), dim3(256), 0, st, a);
  } else {
    if (mode == 0) hipLaunchKernelGGL((a2c_head_kernel<false, kMaxAct>), dim3(grid), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((a2c_head_kernel<true, kMaxAct>), dim3(grid), dim3(256), 0, st, a);
  }
  return (int)hipGetLastError();
}

int rrl_head_wgrad(const uint16_t* h, const float* dhead, int B, int A, float* part, int nblk, void* stream_) {
  hipStream_t st = (hipStream_t)stream_;
  hipLaunchKernelGGL(head_wgrad_kernel, dim3(nblk), dim3(256), 0, st, h, dhead, B, A, part);
  return (int)hipGetLastError();
}

}  // extern "C"
