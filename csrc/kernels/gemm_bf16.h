// LDS-tiled bf16 MFMA GEMM core for the pixel (CNN) model family.
//
//   C[m][n] = sum_k A[m][k] * B[k][n]      fp32 accumulate, v_mfma_f32_16x16x32_bf16
//
// Operands are never materialised in a fixed layout: each side is read through a
// *loader* that returns one 16-byte chunk (8 bf16) of the operand's LDS image, where an
// image is [rows][contiguous cols].  Two image orientations per operand:
//   A  !A_TR: image [BM][BK]  (row = m, contiguous = k)  -> fragments by ds_read_b128
//       A_TR: image [BK][BM]  (row = k, contiguous = m)  -> fragments by ds_read_b64_tr_b16
//   B  !B_TR: image [BN][BK]  (row = n, contiguous = k)  -> ds_read_b128
//       B_TR: image [BK][BN]  (row = k, contiguous = n)  -> ds_read_b64_tr_b16
// so forward (X_col . W^T), data-gradient (dY . W) and weight-gradient (dY^T . X_col)
// GEMMs all stream their operands with 16-byte global loads in the layout they already
// have (NHWC activations, [Cout][KH][KW][C] weights) and transpose for free in the LDS
// read.  Implicit im2col lives in the loader (ConvLoader), so convolutions never write
// a column buffer in the forward or weight-gradient pass.
//
// Block = 256 threads (4 waves), tile BM x BN x 64, one LDS buffer with register staging
// of the next tile (kGemmStages); split-K over gridDim.z for reductions that dwarf the
// output (weight gradients over batch x spatial).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace rrl {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef short s16x4_t __attribute__((ext_vector_type(4)));
typedef float f32x4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint16_t f2bf(float f) {  // round-to-nearest-even
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u) return (uint16_t)((u >> 16) | ((u & 0xffff) ? 0x40 : 0));
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float(((uint32_t)h) << 16); }
__device__ __forceinline__ uint4 pack_bf16x8(const float (&v)[8]) {
  return make_uint4(f2bf(v[0]) | ((uint32_t)f2bf(v[1]) << 16), f2bf(v[2]) | ((uint32_t)f2bf(v[3]) << 16),
                    f2bf(v[4]) | ((uint32_t)f2bf(v[5]) << 16), f2bf(v[6]) | ((uint32_t)f2bf(v[7]) << 16));
}
// element e (0..7) of 8 bf16 packed in a uint4, as float
__device__ __forceinline__ float bf16x8_at(uint4 u, int e) {
  const uint32_t w = e < 2 ? u.x : (e < 4 ? u.y : (e < 6 ? u.z : u.w));
  return __uint_as_float((e & 1) ? (w & 0xffff0000u) : (w << 16));
}

// uint8 inputs are fed to the MFMA as exact integers 0..255 in bf16 (8 significant bits
// fit the bf16 mantissa, so the conversion is a byte->f32 convert plus taking the high
// half -- no rounding); the 1/255 input scale is applied to the fp32 accumulator in the
// epilogue instead (kU8Scale).  uint8 NHWC input with C % 8 == 0 (space-to-depth
// frames): 8 consecutive k = 8 consecutive channels of one pixel = 8 contiguous bytes.
constexpr float kU8Scale = 1.0f / 255.0f;
__device__ __forceinline__ uint32_t pack_hi16(float lo, float hi) {
  return (__float_as_uint(lo) >> 16) | (__float_as_uint(hi) & 0xffff0000u);
}
__device__ __forceinline__ uint4 u8x8_to_bf16x8(uint2 b) {
  return make_uint4(pack_hi16((float)(b.x & 0xff), (float)((b.x >> 8) & 0xff)),
                    pack_hi16((float)((b.x >> 16) & 0xff), (float)(b.x >> 24)),
                    pack_hi16((float)(b.y & 0xff), (float)((b.y >> 8) & 0xff)),
                    pack_hi16((float)((b.y >> 16) & 0xff), (float)(b.y >> 24)));
}


// ----------------------------------------------------------------------------- loaders
// Plain row-major bf16 matrix [rows][cols] (cols % 8 == 0).
struct RowLoader {
  const uint16_t* p;
  int rows, cols;
  __device__ __forceinline__ uint4 operator()(int r, int c) const {
    if (r >= rows || c >= cols) return make_uint4(0, 0, 0, 0);
    return *reinterpret_cast<const uint4*>(p + (size_t)r * cols + c);
  }
};

// Implicit im2col over an NHWC bf16 activation (C % 8 == 0).  Image coordinates are
// (m, k) for A/!TR or (k-row = m, col = k) for the weight-gradient B/TR image -- the
// caller passes (m, k) either way.  k is ordered (kh, kw, c) like the weights.
struct ConvLoader {
  const uint16_t* x;
  int H, W, C, KW, S, OH, OW, M, K;
  __device__ __forceinline__ uint4 operator()(int m, int k) const {
    if (m >= M || k >= K) return make_uint4(0, 0, 0, 0);
    const int ohw = OH * OW;
    const int n = m / ohw, p = m - n * ohw;
    const int oh = p / OW, ow = p - oh * OW;
    const int kc = KW * C;
    const int kh = k / kc, r = k - kh * kc;
    const int kw = r / C, c = r - kw * C;
    const size_t off = (((size_t)n * H + (oh * S + kh)) * W + (ow * S + kw)) * C + c;
    return *reinterpret_cast<const uint4*>(x + off);
  }
};

// Implicit im2col over uint8 NHWC frames with C == 4 (stacked grayscale frames): 8
// consecutive k are 2 adjacent pixels x 4 channels = 8 contiguous bytes (raw 0..255, see kU8Scale).
struct FrameLoader {
  const uint8_t* x;
  int H, W, KW, S, OH, OW, M, K;
  __device__ __forceinline__ uint4 operator()(int m, int k) const {
    if (m >= M || k >= K) return make_uint4(0, 0, 0, 0);
    const int ohw = OH * OW;
    const int n = m / ohw, p = m - n * ohw;
    const int oh = p / OW, ow = p - oh * OW;
    const int kc = KW * 4;
    const int kh = k / kc, kw = (k - kh * kc) >> 2;
    const size_t off = (((size_t)n * H + (oh * S + kh)) * W + (ow * S + kw)) * 4;
    return u8x8_to_bf16x8(*reinterpret_cast<const uint2*>(x + off));
  }
};

// Compile-time-geometry variants: every index division becomes a multiply-shift, which
// matters because the loader runs once per 16-byte chunk (the Nature-CNN layers use
// these; other shapes fall back to the runtime-geometry loaders above).
template <int H, int W, int C, int KW, int S, int OH, int OW>
struct ConvLoaderT {
  const uint16_t* x;
  int M, K;
  __device__ __forceinline__ uint4 operator()(int m, int k) const {
    if (m >= M || k >= K) return make_uint4(0, 0, 0, 0);
    const unsigned um = (unsigned)m, uk = (unsigned)k;
    const unsigned n = um / (OH * OW), p = um - n * (OH * OW);
    const unsigned oh = p / OW, ow = p - oh * OW;
    const unsigned kh = uk / (KW * C), r = uk - kh * (KW * C);
    const unsigned kw = r / C, c = r - kw * C;
    const size_t off = (((size_t)n * H + (oh * S + kh)) * W + (ow * S + kw)) * C + c;
    return *reinterpret_cast<const uint4*>(x + off);
  }
};

template <int H, int W, int KW, int S, int OH, int OW>
struct FrameLoaderT {
  const uint8_t* x;
  int M, K;
  __device__ __forceinline__ uint4 operator()(int m, int k) const {
    if (m >= M || k >= K) return make_uint4(0, 0, 0, 0);
    const unsigned um = (unsigned)m, uk = (unsigned)k;
    const unsigned n = um / (OH * OW), p = um - n * (OH * OW);
    const unsigned oh = p / OW, ow = p - oh * OW;
    const unsigned kh = uk / (KW * 4), kw = (uk - kh * (KW * 4)) >> 2;
    const size_t off = (((size_t)n * H + (oh * S + kh)) * W + (ow * S + kw)) * 4;
    return u8x8_to_bf16x8(*reinterpret_cast<const uint2*>(x + off));
  }
};

template <int H, int W, int C, int KW, int S, int OH, int OW>
struct U8ConvLoaderT {
  const uint8_t* x;
  int M, K;
  __device__ __forceinline__ uint4 operator()(int m, int k) const {
    if (m >= M || k >= K) return make_uint4(0, 0, 0, 0);
    const unsigned um = (unsigned)m, uk = (unsigned)k;
    const unsigned n = um / (OH * OW), p = um - n * (OH * OW);
    const unsigned oh = p / OW, ow = p - oh * OW;
    const unsigned kh = uk / (KW * C), r = uk - kh * (KW * C);
    const unsigned kw = r / C, c = r - kw * C;
    const size_t off = (((size_t)n * H + (oh * S + kh)) * W + (ow * S + kw)) * C + c;
    return u8x8_to_bf16x8(*reinterpret_cast<const uint2*>(x + off));
  }
};

struct U8ConvLoader {
  const uint8_t* x;
  int H, W, C, KW, S, OH, OW, M, K;
  __device__ __forceinline__ uint4 operator()(int m, int k) const {
    if (m >= M || k >= K) return make_uint4(0, 0, 0, 0);
    const int ohw = OH * OW;
    const int n = m / ohw, p = m - n * ohw;
    const int oh = p / OW, ow = p - oh * OW;
    const int kc = KW * C;
    const int kh = k / kc, r = k - kh * kc;
    const int kw = r / C, c = r - kw * C;
    const size_t off = (((size_t)n * H + (oh * S + kh)) * W + (ow * S + kw)) * C + c;
    return u8x8_to_bf16x8(*reinterpret_cast<const uint2*>(x + off));
  }
};

// ----------------------------------------------------------------------------- kernel
constexpr int kGemmBK = 64;
constexpr int kGemmPad = 8;  // bf16 elements of row padding (16 B)
// LDS buffers per workgroup.  The next k-tile is always staged in registers while the
// current one is consumed, so one LDS buffer (two barriers per k-tile) suffices, and it
// halves the LDS footprint: 3 -> 6 resident 128x32 workgroups per CU and 2 -> 4 for
// 128x64, which hides the global-load latency of the short-K conv GEMMs better
// (PongSynth A2C, 2048 envs: 2.66 -> 3.21 M env-steps/s; docs/PERF_NOTES.md).
#ifndef RRL_GEMM_STAGES
#define RRL_GEMM_STAGES 1
#endif
constexpr int kGemmStages = RRL_GEMM_STAGES;

template <int BM, int BN, bool A_TR, bool B_TR>
struct GemmShape {
  static constexpr int BK = kGemmBK;
  // image dims (rows x padded contiguous cols)
  static constexpr int A_ROWS = A_TR ? BK : BM, A_COLS = A_TR ? BM : BK;
  static constexpr int B_ROWS = B_TR ? BK : BN, B_COLS = B_TR ? BN : BK;
  static constexpr int A_LD = A_COLS + kGemmPad, B_LD = B_COLS + kGemmPad;
  static constexpr int A_ELEMS = A_ROWS * A_LD, B_ELEMS = B_ROWS * B_LD;
  static constexpr int STAGE = A_ELEMS + B_ELEMS;                 // bf16 elements per stage
  static constexpr int OUT_LD = BN + 4;                           // fp32 output tile row (vec8 epilogues)
  static constexpr int OUT_BYTES = BM * OUT_LD * 4;
  static constexpr int LDS_BYTES = (kGemmStages * STAGE * 2 > OUT_BYTES) ? kGemmStages * STAGE * 2 : OUT_BYTES;
  static constexpr int A_CHUNKS = A_ROWS * A_COLS / 8, B_CHUNKS = B_ROWS * B_COLS / 8;
  static constexpr int A_PER_T = (A_CHUNKS + 255) / 256, B_PER_T = (B_CHUNKS + 255) / 256;
  // wave grid: 2x2 when both dims >= 32 per wave, else 4x1
  static constexpr int WN = (BN >= 64) ? 2 : 1, WM = 4 / WN;
  static constexpr int WAVE_M = BM / WM, WAVE_N = BN / WN;
  static constexpr int TM = WAVE_M / 16, TN = WAVE_N / 16;
  static_assert(TM >= 1 && TN >= 1, "tile too small for the wave grid");
};

// Fragment of 8 consecutive k for one row/col from a [row][k] image (b128 read).
__device__ __forceinline__ bf16x8_t frag_rowk(const uint16_t* img, int ld, int row, int k) {
  return *reinterpret_cast<const bf16x8_t*>(img + row * ld + k);
}
// Fragment from a [k][col] image via two transposed reads: rows k0..k0+3 and k0+4..k0+7
// of columns col0..col0+15; lane 4q+p of each 16-lane group addresses row q, cols 4p..4p+3.
__device__ __forceinline__ bf16x8_t frag_tr(const uint16_t* img, int ld, int k0, int col0, int lane) {
  const int q = (lane >> 2) & 3, p = lane & 3;
  typedef __attribute__((address_space(3))) s16x4_t lds_v4;
  const uint16_t* a0 = img + (k0 + q) * ld + col0 + 4 * p;
  const uint16_t* a1 = a0 + 4 * ld;
  s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(a0));
  s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(a1));
  typedef short s16x8_t __attribute__((ext_vector_type(8)));
  s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

// Epilogues that define `static constexpr bool kVec8 = true` and
//   store8(m, n, const float (&v)[8], split)      (columns n .. n+7 of row m, n % 8 == 0)
// get the output tile through LDS: the MFMA C layout (4 rows x 1 column per lane) is
// re-read as 8 consecutive columns of one row per thread, so NHWC bf16 outputs (and the
// masks / skip inputs they read) move as 16-byte accesses instead of 2-byte ones.
template <class Epi, class = void>
struct EpiVec8 : std::false_type {};
template <class Epi>
struct EpiVec8<Epi, std::void_t<decltype(Epi::kVec8)>> : std::integral_constant<bool, Epi::kVec8> {};

// Loaders are called with global IMAGE coordinates (row, contiguous col):
//   A !TR: (m, k)   A TR: (k, m)   B !TR: (n, k)   B TR: (k, n)
// Epilogue functor: operator()(m, n, acc, split) with acc[r] the value of row m + r,
// column n -- the four values a lane owns (rows 4*(lane>>4)+r of one 16x16 tile).
template <int BM, int BN, bool A_TR, bool B_TR, class LA, class LB, class Epi>
__global__ void __launch_bounds__(256, 2)
gemm_bf16_kernel(LA la, LB lb, Epi epi, int M, int N, int K, int k_per_split) {
  using S = GemmShape<BM, BN, A_TR, B_TR>;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
  const int kb = blockIdx.z * k_per_split;
  const int ke = min(K, kb + k_per_split);
  const int wm = wave / S::WN, wn = wave % S::WN;
  const int wm0 = wm * S::WAVE_M, wn0 = wn * S::WAVE_N;

  f32x4_t acc[S::TM][S::TN];
#pragma unroll
  for (int i = 0; i < S::TM; ++i)
#pragma unroll
    for (int j = 0; j < S::TN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  uint4 ra[S::A_PER_T], rb[S::B_PER_T];
  auto gload = [&](int k0) {
#pragma unroll
    for (int i = 0; i < S::A_PER_T; ++i) {
      const int ch = tid + 256 * i;
      const int r = ch / (S::A_COLS / 8), c = (ch % (S::A_COLS / 8)) * 8;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (ch < S::A_CHUNKS) {
        if (A_TR) {  // image row = k, col = m
          if (k0 + r < ke) v = la(k0 + r, m0 + c);
        } else {
          if (k0 + c < ke) v = la(m0 + r, k0 + c);
        }
      }
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < S::B_PER_T; ++i) {
      const int ch = tid + 256 * i;
      const int r = ch / (S::B_COLS / 8), c = (ch % (S::B_COLS / 8)) * 8;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (ch < S::B_CHUNKS) {
        if (B_TR) {  // image row = k, col = n
          if (k0 + r < ke) v = lb(k0 + r, n0 + c);
        } else {
          if (k0 + c < ke) v = lb(n0 + r, k0 + c);
        }
      }
      rb[i] = v;
    }
  };
  auto lstore = [&](int buf) {
    uint16_t* A = smem + buf * S::STAGE;
    uint16_t* B = A + S::A_ELEMS;
#pragma unroll
    for (int i = 0; i < S::A_PER_T; ++i) {
      const int ch = tid + 256 * i;
      if (ch < S::A_CHUNKS) {
        const int r = ch / (S::A_COLS / 8), c = (ch % (S::A_COLS / 8)) * 8;
        *reinterpret_cast<uint4*>(A + r * S::A_LD + c) = ra[i];
      }
    }
#pragma unroll
    for (int i = 0; i < S::B_PER_T; ++i) {
      const int ch = tid + 256 * i;
      if (ch < S::B_CHUNKS) {
        const int r = ch / (S::B_COLS / 8), c = (ch % (S::B_COLS / 8)) * 8;
        *reinterpret_cast<uint4*>(B + r * S::B_LD + c) = rb[i];
      }
    }
  };

  const int g = lane >> 4, li = lane & 15;
  int buf = 0;
  if (kb < ke) {
    gload(kb);
    lstore(0);
  }
  __syncthreads();
  for (int k0 = kb; k0 < ke; k0 += S::BK) {
    const bool more = k0 + S::BK < ke;
    if (more) gload(k0 + S::BK);
    const uint16_t* A = smem + buf * S::STAGE;
    const uint16_t* B = A + S::A_ELEMS;
#pragma unroll
    for (int s = 0; s < S::BK / 32; ++s) {
      bf16x8_t af[S::TM], bfr[S::TN];
#pragma unroll
      for (int i = 0; i < S::TM; ++i) {
        if (A_TR) af[i] = frag_tr(A, S::A_LD, 32 * s + 8 * g, wm0 + 16 * i, lane);
        else af[i] = frag_rowk(A, S::A_LD, wm0 + 16 * i + li, 32 * s + 8 * g);
      }
#pragma unroll
      for (int j = 0; j < S::TN; ++j) {
        if (B_TR) bfr[j] = frag_tr(B, S::B_LD, 32 * s + 8 * g, wn0 + 16 * j, lane);
        else bfr[j] = frag_rowk(B, S::B_LD, wn0 + 16 * j + li, 32 * s + 8 * g);
      }
#pragma unroll
      for (int i = 0; i < S::TM; ++i)
#pragma unroll
        for (int j = 0; j < S::TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (more) {
      if (kGemmStages == 1) {
        __syncthreads();  // every wave is done reading the tile
        lstore(0);
        __syncthreads();
      } else {
        lstore(buf ^ 1);
        __syncthreads();
        buf ^= 1;
      }
    }
  }
  if constexpr (EpiVec8<Epi>::value) {
    float* T = reinterpret_cast<float*>(smem);  // [BM][OUT_LD] fp32 tile
    __syncthreads();                            // every wave is done reading the operand tiles
#pragma unroll
    for (int i = 0; i < S::TM; ++i)
#pragma unroll
      for (int j = 0; j < S::TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) T[(wm0 + 16 * i + 4 * g + r) * S::OUT_LD + wn0 + 16 * j + li] = acc[i][j][r];
    __syncthreads();
    for (int q = tid; q < BM * (BN / 8); q += 256) {
      const int row = q / (BN / 8), c = (q % (BN / 8)) * 8;
      if (m0 + row >= M || n0 + c >= N) continue;
      const f32x4_t lo = *reinterpret_cast<const f32x4_t*>(T + row * S::OUT_LD + c);
      const f32x4_t hi = *reinterpret_cast<const f32x4_t*>(T + row * S::OUT_LD + c + 4);
      const float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      epi.store8(m0 + row, n0 + c, v, blockIdx.z);
    }
  } else {
#pragma unroll
    for (int i = 0; i < S::TM; ++i)
#pragma unroll
      for (int j = 0; j < S::TN; ++j) {
        const int m = m0 + wm0 + 16 * i + 4 * g;
        const int n = n0 + wn0 + 16 * j + li;
        epi(m, n, acc[i][j], blockIdx.z);
      }
  }
}

}  // namespace rrl
