// Fully connected layers of the pixel model (Nature CNN fc: 3136 -> 512) as one "NT"
// bf16 MFMA GEMM on gfx950:
//
//   C[m][n] = sum_k A[m][k] * B[n][k]        A [M][K], B [N][K], both K-contiguous bf16
//
// The fc forward is A = a3 [rows][3136], B = Wfc [512][3136]; the fc data gradient is
// A = dh [rows][512], B = Wfc^T [3136][512] (the transposed bf16 shadow the optimiser
// writes next to the weights), so both stream 16-byte K-chunks of rows they already have.
//
// Why not gemm_bf16.h: that core stages operand tiles through registers into ONE LDS
// buffer (two barriers per k-tile, loads exposed at every tile) and tiles 128x64 over 4
// waves -- fine for the short-K implicit-im2col conv GEMMs, but the fc GEMMs are long-K
// (3136) or wide-N (3136) streaming problems: at 2,048 rows the split-K fc forward ran at
// ~0.3 PFLOP/s (21 us per call, profiles/r3_pong_a2c_kernels_fused.txt).  Here:
//   * operand tiles go global -> LDS by DMA (global_load_lds_dwordx4): no staging
//     registers, no ds_write pass; 3 LDS stages, two tiles in flight across ONE raw
//     s_barrier per k-tile (counted vmcnt, never vmcnt(0) inside the loop);
//   * the LDS image is lane-linear (the DMA writes base + 16 * lane) with an XOR swizzle
//     applied on the SOURCE side: chunk (row, kc) of a [rows][8 x 16 B] image lives at
//     row * 8 + (kc ^ ((row >> 1) & 7)), which makes every ds_read_b128 fragment read of
//     16 rows x one k-chunk conflict-free (each of the instruction's four 16-lane groups
//     touches 16 distinct 16-byte bank quads);
//   * 128 x 128 x 64 tiles on 8 waves (2 x 4, 64 x 32 per wave), 96 KB of LDS: one
//     workgroup of 8 waves per CU, two per SIMD;
//   * operands swapped in the MFMA (A-operand = B rows, B-operand = A rows) so each lane
//     owns 4 CONSECUTIVE n of one row m: 16-byte fp32 / 8-byte bf16 epilogue stores with
//     no LDS round trip;
//   * XCD-aware block order: consecutive logical tiles (m fastest) land on one XCD, so the
//     workgroups sharing a B tile (the weights) share that XCD's L2.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <type_traits>

#include "gemm_bf16.h"

namespace rrl {

constexpr int kFcBM = 128, kFcBN = 128, kFcBK = 64;
constexpr int kFcImg = kFcBM * kFcBK;                        // bf16 elements per operand image
constexpr int kFcStage = 2 * kFcImg;                         // A image + B image (32 KB)
constexpr int kFcThreads = 512;
template <int STAGES>
constexpr int fc_lds_bytes() { return STAGES * kFcStage * 2; }

// position (in 16-byte chunks) of chunk kc (0..7) of image row `row`
__device__ __forceinline__ int fc_swz(int row, int kc) { return row * 8 + (kc ^ ((row >> 1) & 7)); }

// fp32 split-K partials: part[z][m][n]
struct FcPartEpi {
  float* part;
  int M, N;
  typedef int Pre;  // nothing to prefetch
  __device__ __forceinline__ Pre prefetch(int, int) const { return 0; }
  __device__ __forceinline__ void operator()(int m, int n, f32x4_t v, int z, Pre) const {
    if (m < M && n < N)
      *reinterpret_cast<f32x4_t*>(part + ((size_t)z * M + m) * N + n) = v;
  }
};

// bf16 data gradient with the ReLU mask of the layer input: out[m][n] = v * (mask[m][n] > 0)
struct FcMaskEpi {
  uint16_t* out;
  const uint16_t* mask;
  int M, N;
  typedef uint2 Pre;  // the 4 mask values, loaded before the last k-tile's MFMAs
  __device__ __forceinline__ Pre prefetch(int m, int n) const {
    return (m < M && n < N) ? *reinterpret_cast<const uint2*>(mask + (size_t)m * N + n) : make_uint2(0, 0);
  }
  __device__ __forceinline__ void operator()(int m, int n, f32x4_t v, int, Pre mk) const {
    if (m >= M || n >= N) return;
    const size_t i = (size_t)m * N + n;
    const float o0 = bf2f((uint16_t)(mk.x & 0xffff)) > 0.f ? v[0] : 0.f;
    const float o1 = bf2f((uint16_t)(mk.x >> 16)) > 0.f ? v[1] : 0.f;
    const float o2 = bf2f((uint16_t)(mk.y & 0xffff)) > 0.f ? v[2] : 0.f;
    const float o3 = bf2f((uint16_t)(mk.y >> 16)) > 0.f ? v[3] : 0.f;
    *reinterpret_cast<uint2*>(out + i) =
        make_uint2((uint32_t)f2bf(o0) | ((uint32_t)f2bf(o1) << 16), (uint32_t)f2bf(o2) | ((uint32_t)f2bf(o3) << 16));
  }
};

// Same product, but the tile leaves through LDS: the accumulators are packed to bf16 into a
// [128][136] image in the (now idle) stage buffers, then each thread moves 8 consecutive
// columns of one row (16-byte mask load + 16-byte store, 256 contiguous bytes per 16 lanes)
// -- the direct epilogue wrote 32-byte pieces of 16 rows per instruction, which left the
// 0.26 GB data-gradient output / mask streams of a 40,960-row update at ~1.2 TB/s.
// N % 8 == 0.
struct FcMaskStagedEpi {
  uint16_t* out;
  const uint16_t* mask;
  int M, N;
  static constexpr int kLd = 136;  // bf16 row stride of the staging image
};
template <class Epi, class = void>
struct FcStaged : std::false_type {};
template <>
struct FcStaged<FcMaskStagedEpi> : std::true_type {};

// One k-tile of one operand into its LDS image: the wave's two DMA instructions fill image
// rows 16 w .. 16 w + 15 (8 rows x 8 chunks = the instruction's 64 lanes x 16 B each).
__device__ __forceinline__ void fc_stage(const uint16_t* __restrict__ X, int rows, int K, int row0, int k0,
                                         uint16_t* img, int wave, int lane) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int r0 = 16 * wave + 8 * j;
    const int r = r0 + (lane >> 3);
    const int kc = (lane & 7) ^ ((r >> 1) & 7);
    const int gr = min(row0 + r, rows - 1);  // rows past the end: a duplicate, masked in the epilogue
    const uint16_t* src = X + (size_t)gr * K + k0 + 8 * kc;
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(img + r0 * kFcBK), 16, 0, 0);
  }
}

// STAGES = 3: two k-tiles in flight, one 8-wave workgroup per CU (96 KB); STAGES = 2: one
// k-tile in flight, two workgroups per CU (64 KB each), so one workgroup's epilogue and
// prologue overlap the other's main loop (short-K problems: the data gradient, K = 512).
template <class Epi, int STAGES, bool SP = false>  // SP: s_setprio 1 around the k-tile's MFMAs (A/B)
__global__ void __launch_bounds__(kFcThreads, STAGES == 2 ? 2 : 1)
fc_nt_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B, Epi epi, int M, int N, int K,
             int tiles_m, int tiles_n, int ktiles_per_split, int m_fast) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // XCD-aware order: hardware block b runs on XCD b % 8; logical tile ids handed out so that
  // each XCD takes a contiguous run of them (bijective for any grid size)
  const int nwg = gridDim.x, b = blockIdx.x;
  const int q = nwg >> 3, rem = nwg & 7, xcd = b & 7;
  const int lid = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (b >> 3);
  // n fastest: an XCD's run of tiles shares the A rows (the activations, read from HBM once)
  // and cycles through the B tiles (the weights, small enough to stay in its L2)
  int tm, tn, z;
  if (m_fast) {  // (A/B alternative: an XCD's run shares the B tiles instead)
    tm = lid % tiles_m;
    const int rest = lid / tiles_m;
    tn = rest % tiles_n, z = rest / tiles_n;
  } else {
    tn = lid % tiles_n;
    const int rest = lid / tiles_n;
    tm = rest % tiles_m, z = rest / tiles_m;
  }
  const int m0 = tm * kFcBM, n0 = tn * kFcBN;
  const int kt0 = z * ktiles_per_split;
  const int nk = min(K / kFcBK - kt0, ktiles_per_split);

  const int wm = wave & 1, wn = wave >> 1;  // 2 x 4 waves: 64 rows (m) x 32 cols (n) each
  const int g = lane >> 4, li = lane & 15;
  f32x4_t acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};

  typedef typename std::conditional<FcStaged<Epi>::value, FcPartEpi, Epi>::type DirectEpi;
  typename DirectEpi::Pre pre[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) pre[i][j] = typename DirectEpi::Pre{};
  uint4 spre[4] = {};  // staged epilogue: this thread's 4 mask chunks
  auto issue = [&](int t) {
    uint16_t* st = smem + (t % STAGES) * kFcStage;
    const int k0 = (kt0 + t) * kFcBK;
    fc_stage(A, M, K, m0, k0, st, wave, lane);
    fc_stage(B, N, K, n0, k0, st + kFcImg, wave, lane);
  };
#pragma unroll
  for (int t = 0; t < STAGES - 1; ++t)
    if (t < nk) issue(t);
  for (int t = 0; t < nk; ++t) {
    // tile t landed (this wave's 4 DMAs of it; the up to STAGES - 2 tiles issued after it may
    // stay in flight), then a barrier publishes every wave's DMAs and retires every wave's
    // reads of tile t - 1, whose stage the next issue overwrites
    const int ahead = min(STAGES - 2, nk - 1 - t);
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + STAGES - 1 < nk) issue(t + STAGES - 1);
    if (t + 1 == nk) {  // no DMA in flight any more: the epilogue's own loads go out now
      if constexpr (FcStaged<Epi>::value) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int c = tid + kFcThreads * k;
          const int m = min(m0 + (c >> 4), M - 1), n = min(n0 + (c & 15) * 8, N - 8);  // clamped: no branch
          spre[k] = *reinterpret_cast<const uint4*>(epi.mask + (size_t)m * N + n);
        }
      } else {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j)
            pre[i][j] = epi.prefetch(m0 + 64 * wm + 16 * i + li, n0 + 32 * wn + 16 * j + 4 * g);
      }
    }
    const uint16_t* Ai = smem + (t % STAGES) * kFcStage;
    const uint16_t* Bi = Ai + kFcImg;
    if constexpr (SP) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < kFcBK / 32; ++s) {
      const int kc = 4 * s + g;
      bf16x8_t af[4], bfr[2];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        af[i] = *reinterpret_cast<const bf16x8_t*>(Ai + 8 * fc_swz(64 * wm + 16 * i + li, kc));
#pragma unroll
      for (int j = 0; j < 2; ++j)
        bfr[j] = *reinterpret_cast<const bf16x8_t*>(Bi + 8 * fc_swz(32 * wn + 16 * j + li, kc));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)  // D[n][m]: lane (g, li) holds n = 4 g .. 4 g + 3 of row m = li
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
    if constexpr (SP) __builtin_amdgcn_s_setprio(0);
  }
  if constexpr (FcStaged<Epi>::value) {
    constexpr int LD = FcMaskStagedEpi::kLd;
    uint16_t* T = smem;  // [128][LD] bf16 = 34,816 B over the idle stage buffers
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave is done reading the operand stages
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        *reinterpret_cast<uint2*>(T + (64 * wm + 16 * i + li) * LD + 32 * wn + 16 * j + 4 * g) =
            make_uint2((uint32_t)f2bf(acc[i][j][0]) | ((uint32_t)f2bf(acc[i][j][1]) << 16),
                       (uint32_t)f2bf(acc[i][j][2]) | ((uint32_t)f2bf(acc[i][j][3]) << 16));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = tid + kFcThreads * k, r = c >> 4, cc = (c & 15) * 8;
      const int m = m0 + r, n = n0 + cc;
      if (m >= M || n >= N) continue;
      const uint4 v = *reinterpret_cast<const uint4*>(T + r * LD + cc);
      const uint32_t vw[4] = {v.x, v.y, v.z, v.w}, mw[4] = {spre[k].x, spre[k].y, spre[k].z, spre[k].w};
      uint32_t ow[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {  // keep where the layer input was > 0 (bf16 -> f32 is exact)
        const uint32_t lo = bf2f((uint16_t)(mw[e] & 0xffff)) > 0.f ? 0x0000ffffu : 0u;
        const uint32_t hi = bf2f((uint16_t)(mw[e] >> 16)) > 0.f ? 0xffff0000u : 0u;
        ow[e] = vw[e] & (lo | hi);
      }
      *reinterpret_cast<uint4*>(epi.out + (size_t)m * N + n) = make_uint4(ow[0], ow[1], ow[2], ow[3]);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        epi(m0 + 64 * wm + 16 * i + li, n0 + 32 * wn + 16 * j + 4 * g, acc[i][j], z, pre[i][j]);
  }
}

static int fc_m_fast() {
  const char* e = getenv("RRL_FC_MFAST");
  return e && e[0] == '1';
}

// LDS stage count per call site (0 = forward partials, 1 = data gradient); RRL_FC_STAGES =
// "<fwd><dgrad>" (e.g. "32") overrides the defaults for A/B measurements.
static int fc_stages(int site, int dflt) {
  const char* e = getenv("RRL_FC_STAGES");  // read per call (A/B variants in one process)
  if (!e || (int)strlen(e) <= site) return dflt;
  return e[site] == '4' ? 4 : (e[site] == '3' ? 3 : (e[site] == '2' ? 2 : dflt));
}

static bool fc_setprio() {  // RRL_FC_SETPRIO=1: the s_setprio forms (A/B), read per call
  const char* e = getenv("RRL_FC_SETPRIO");
  return e && e[0] == '1';
}

template <class Epi, int STAGES, bool SP = false>
static int launch_fc_nt_sp(const uint16_t* A, const uint16_t* B, Epi epi, int M, int N, int K, int splits,
                           hipStream_t st);

template <class Epi, int STAGES>
static int launch_fc_nt(const uint16_t* A, const uint16_t* B, Epi epi, int M, int N, int K, int splits,
                        hipStream_t st) {
  return fc_setprio() ? launch_fc_nt_sp<Epi, STAGES, true>(A, B, epi, M, N, K, splits, st)
                      : launch_fc_nt_sp<Epi, STAGES, false>(A, B, epi, M, N, K, splits, st);
}

template <class Epi, int STAGES, bool SP>
static int launch_fc_nt_sp(const uint16_t* A, const uint16_t* B, Epi epi, int M, int N, int K, int splits,
                           hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)fc_nt_kernel<Epi, STAGES, SP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              fc_lds_bytes<STAGES>());
    attr = true;
  }
  const int tiles_m = (M + kFcBM - 1) / kFcBM, tiles_n = (N + kFcBN - 1) / kFcBN;
  const int kt = K / kFcBK;
  const int kps = (kt + splits - 1) / splits;
  splits = (kt + kps - 1) / kps;
  const int grid = tiles_m * tiles_n * splits;
  if (grid < 1) return 0;
  hipLaunchKernelGGL((fc_nt_kernel<Epi, STAGES, SP>), dim3(grid), dim3(kFcThreads), fc_lds_bytes<STAGES>(), st, A, B,
                     epi, M, N, K, tiles_m, tiles_n, kps, fc_m_fast());
  return (int)hipGetLastError();
}

// ----------------------------------------------------------------------------- TN (weight gradient)
//   C[i][j] = sum_r X[r][i] * Y[r][j]      X [R][I], Y [R][J] row-major bf16, R % 64 == 0
// (the fc weight gradient: X = dh [rows][512], Y = a3 [rows][3136], C = dW [512][3136]).
// Both operands are streamed as [64 r][128 col] images (256-B rows, 16 chunks of 16 B) and
// their MFMA fragments come out of ds_read_b64_tr_b16 transposed reads.  The 32 lanes of a
// b64 read touch 8 image rows x 32 B; with 256-B rows every row starts on bank 0, so the
// chunks are XOR-swizzled by an even mask of (row & 3, row >> 3 & 1):
//   chunk c of row r lives at r * 16 + (c ^ 2 * ((r & 3) | (r >> 3 & 1) << 2))
// which spreads those 8 rows x 2 chunks over 16 distinct chunk slots (conflict-free).
__device__ __forceinline__ int fc_tn_swz(int row, int c) { return row * 16 + (c ^ (2 * ((row & 3) | (((row >> 3) & 1) << 2)))); }

// Columns past the end read a duplicate chunk (masked in the epilogue) -- or, with ``ones``
// (16 bytes of bf16 1.0), a column of ones, so the padded output columns of the last tile
// carry sum_r X[r][i]: the bias gradient of the layer for free.
__device__ __forceinline__ void fc_tn_stage(const uint16_t* __restrict__ X, int ld, int r0g, int col0, uint16_t* img,
                                            int wave, int lane, const uint16_t* __restrict__ ones = nullptr) {
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int r0 = 8 * wave + 4 * j;  // image rows r0 .. r0 + 3 (4 x 256 B = the instruction's 1 KB)
    const int r = r0 + (lane >> 4);
    const int c = (lane & 15) ^ (2 * ((r & 3) | (((r >> 3) & 1) << 2)));
    const int col = min(col0 + 8 * c, ld - 8);
    const uint16_t* src = (ones && col0 + 8 * c >= ld) ? ones : X + (size_t)(r0g + r) * ld + col;
    __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)(img + r0 * 128), 16, 0, 0);
  }
}

// MFMA operand fragment (8 consecutive r for image column col0 + (lane & 15)) from a swizzled
// [64][128] image: two ds_read_b64_tr_b16, rows k0 .. k0 + 3 and k0 + 4 .. k0 + 7.  Inline asm: the
// ds_read_tr16_b64 builtin makes hipcc wait vmcnt(0) before
// every read while an LDS-DMA is in flight (it cannot tell which LDS the read touches), which
// drains the whole ring each k-tile.  The asm reads are invisible to the compiler's counters, so
// fcp_lgkm_wait retires them (tied to the fragments) before the MFMAs use them.
__device__ __forceinline__ s16x4_t fcp_tr_b64(const uint16_t* p) {
  s16x4_t v;
  const uint32_t a = (uint32_t)(size_t)(const __attribute__((address_space(3))) uint16_t*)p;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(a));
  return v;
}
__device__ __forceinline__ bf16x8_t fcp_tn_frag(const uint16_t* img, int k0, int col0, int lane) {
  const int q = (lane >> 2) & 3, p = lane & 3;
  const int c = (col0 + 4 * p) >> 3, half = (p & 1) * 4;
  const s16x4_t lo = fcp_tr_b64(img + 8 * fc_tn_swz(k0 + q, c) + half);
  const s16x4_t hi = fcp_tr_b64(img + 8 * fc_tn_swz(k0 + 4 + q, c) + half);
  typedef short s16x8_t __attribute__((ext_vector_type(8)));
  const s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}
template <int FI, int FJ>
__device__ __forceinline__ void fcp_lgkm_wait(bf16x8_t (&x)[FI], bf16x8_t (&y)[FJ]) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  // empty volatile asms stay after the wait and make every fragment an output of it, so no MFMA
  // that reads one can be scheduled above the wait
#pragma unroll
  for (int a = 0; a < FI; ++a) asm volatile("" : "+v"(x[a]));
#pragma unroll
  for (int c = 0; c < FJ; ++c) asm volatile("" : "+v"(y[c]));
}

// 128 (i) x 128 (j) output tile per workgroup, 8 waves (2 x 4: 64 i x 32 j each), the R
// reduction split over gridDim (split z takes r-tiles [z * kps, (z + 1) * kps)); fp32
// partials part[z][I][J], 4 consecutive j per lane (16-byte stores).
template <int STAGES, bool SP = false>
__global__ void __launch_bounds__(kFcThreads, STAGES == 2 ? 2 : 1)
fc_tn_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ Y, float* __restrict__ part, int R, int I,
             int J, int tiles_i, int tiles_j, int rtiles_per_split, const uint16_t* __restrict__ ones,
             float* __restrict__ bias_part) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nwg = gridDim.x, b = blockIdx.x;
  const int q = nwg >> 3, rem = nwg & 7, xcd = b & 7;
  const int lid = (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (b >> 3);
  // i fastest: an XCD's run shares the Y tile (the activations, the big operand) across the
  // dh column tiles
  const int ti = lid % tiles_i, rest = lid / tiles_i;
  const int tj = rest % tiles_j, z = rest / tiles_j;
  const int i0 = ti * 128, j0 = tj * 128;
  const int rt0 = z * rtiles_per_split;
  const int nk = min(R / 64 - rt0, rtiles_per_split);
  const int wi = wave & 1, wj = wave >> 1;
  const int g = lane >> 4, li = lane & 15;
  f32x4_t acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c) acc[a][c] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  auto issue = [&](int t) {
    uint16_t* st = smem + (t % STAGES) * kFcStage;
    const int r0g = (rt0 + t) * 64;
    fc_tn_stage(X, I, r0g, i0, st, wave, lane);
    fc_tn_stage(Y, J, r0g, j0, st + kFcImg, wave, lane, ones);
  };
#pragma unroll
  for (int t = 0; t < STAGES - 1; ++t)
    if (t < nk) issue(t);
  for (int t = 0; t < nk; ++t) {
    const int ahead = min(STAGES - 2, nk - 1 - t);
    if (ahead >= 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (ahead == 1) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (t + STAGES - 1 < nk) issue(t + STAGES - 1);
    const uint16_t* Xi = smem + (t % STAGES) * kFcStage;
    const uint16_t* Yi = Xi + kFcImg;
    if constexpr (SP) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8_t xf[4], yf[2];
#pragma unroll
      for (int a = 0; a < 4; ++a) xf[a] = fcp_tn_frag(Xi, 32 * s + 8 * g, 64 * wi + 16 * a, lane);
#pragma unroll
      for (int c = 0; c < 2; ++c) yf[c] = fcp_tn_frag(Yi, 32 * s + 8 * g, 32 * wj + 16 * c, lane);
      fcp_lgkm_wait<4, 2>(xf, yf);
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int c = 0; c < 2; ++c)  // D[j][i]: lane (g, li) holds j = 4 g .. 4 g + 3 of i = li
          acc[a][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(yf[c], xf[a], acc[a][c], 0, 0, 0);
    }
    if constexpr (SP) __builtin_amdgcn_s_setprio(0);
  }
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int i = i0 + 64 * wi + 16 * a + li, j = j0 + 32 * wj + 16 * c + 4 * g;
      if (i < I && j < J) *reinterpret_cast<f32x4_t*>(part + ((size_t)z * I + i) * J + j) = acc[a][c];
      if (bias_part && i < I && j == J) bias_part[(size_t)z * I + i] = acc[a][c][0];  // the ones column
    }
}

// RRL_FC_TN_LDS_KB (A/B runs, read per call): launch the weight-gradient GEMM with this much
// dynamic LDS (at least its own), e.g. 84 KB = one resident workgroup per CU, leaving a 75 KB
// conv3-backward workgroup room beside it on the side stream
static int fc_tn_lds(int own) {
  const char* e = getenv("RRL_FC_TN_LDS_KB");
  const int kb = (e && e[0]) ? atoi(e) : 0;
  return kb * 1024 > own ? min(kb, 160) * 1024 : own;
}

template <int STAGES, bool SP>
static int launch_fc_tn_sp(const uint16_t* X, const uint16_t* Y, float* part, int R, int I, int J, int splits,
                           const uint16_t* ones, float* bias_part, hipStream_t st) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)fc_tn_kernel<STAGES, SP>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    attr = true;
  }
  const int ti = (I + 127) / 128, tj = (J + 127) / 128, rt = R / 64;
  const int kps = (rt + splits - 1) / splits;
  splits = (rt + kps - 1) / kps;
  hipLaunchKernelGGL((fc_tn_kernel<STAGES, SP>), dim3(ti * tj * splits), dim3(kFcThreads),
                     fc_tn_lds(fc_lds_bytes<STAGES>()), st, X, Y, part, R, I, J, ti, tj, kps, ones, bias_part);
  return (int)hipGetLastError();
}

template <int STAGES>
static int launch_fc_tn(const uint16_t* X, const uint16_t* Y, float* part, int R, int I, int J, int splits,
                        const uint16_t* ones, float* bias_part, hipStream_t st) {
  return fc_setprio() ? launch_fc_tn_sp<STAGES, true>(X, Y, part, R, I, J, splits, ones, bias_part, st)
                      : launch_fc_tn_sp<STAGES, false>(X, Y, part, R, I, J, splits, ones, bias_part, st);
}

// Transposed bf16 copy: out[c][r] = in[r][c] (the fc weight's [3136][512] shadow for the
// data-gradient GEMM).  64 x 64 tiles through LDS, 16-byte loads and stores.
__global__ void __launch_bounds__(256) transpose_bf16_kernel(const uint16_t* __restrict__ in, uint16_t* __restrict__ out,
                                                             int R, int C) {
  __shared__ uint16_t t[64][66];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  for (int q = threadIdx.x; q < 64 * 8; q += 256) {
    const int r = q >> 3, c = (q & 7) * 8;
    if (r0 + r < R && c0 + c < C) {
      const uint4 v = *reinterpret_cast<const uint4*>(in + (size_t)(r0 + r) * C + c0 + c);
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        t[r][c + 2 * e] = (uint16_t)(w[e] & 0xffff);
        t[r][c + 2 * e + 1] = (uint16_t)(w[e] >> 16);
      }
    }
  }
  __syncthreads();
  for (int q = threadIdx.x; q < 64 * 8; q += 256) {
    const int c = q >> 3, r = (q & 7) * 8;
    if (c0 + c < C && r0 + r < R) {
      uint32_t w[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) w[e] = (uint32_t)t[r + 2 * e][c] | ((uint32_t)t[r + 2 * e + 1][c] << 16);
      *reinterpret_cast<uint4*>(out + (size_t)(c0 + c) * R + r0 + r) = make_uint4(w[0], w[1], w[2], w[3]);
    }
  }
}


// ----------------------------------------------------------------------------- persistent big tiles
// The kernels above run 128 x 128 tiles, 64 x 32 per wave, one tile per workgroup: per k-tile
// each workgroup pulls 32 KB through L2 for 2.1 MFLOP (64 FLOP/B), and every tile pays its own
// prologue (first DMA latency) and epilogue (store tail) -- at the Pong shapes 0.5-0.8 PFLOP/s
// (profiles/r3_fc_kbench.jsonl).  These are PERSISTENT: one 512-thread workgroup per CU walks
// a flat sequence of (tile, k-tile) steps, so the LDS ring runs straight across tile
// boundaries (the next tile's first k-tiles are in flight during this tile's epilogue), with
// 256 x 128 tiles (85 FLOP/B) and 64 x 64 per wave (16 MFMAs per 8 fragment reads).
//
// vmcnt accounting: LDS-DMA, the epilogue's stores and its prefetch loads all count on one
// in-order counter, so the wait for step u's DMA must know how many vector-memory ops were
// issued after it: the next step's DMA (D per wave) and the epilogue of a tile that ended at
// step u - 1 or u - 2 (E per wave).  Every wave issues EXACTLY E epilogue ops -- lanes with
// nothing to store write a private dummy slot instead of branching around the store -- and
// every item has >= 2 k-tiles, so at most one epilogue sits in that window.
template <int N>
__device__ __forceinline__ void fcp_vm_wait() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

template <int D, int E>
__device__ __forceinline__ void fcp_wait_window(bool next_dma, bool epi) {
  if (next_dma) {
    if (epi) fcp_vm_wait<D + E>();
    else fcp_vm_wait<D>();
  } else {
    if (epi) fcp_vm_wait<E>();
    else fcp_vm_wait<0>();
  }
}

// XCD-aware logical id of a persistent block (bijective for any grid size)
__device__ __forceinline__ int fcp_lid() {
  const int G = gridDim.x, b = blockIdx.x;
  const int q = G >> 3, rem = G & 7, xcd = b & 7;
  return (xcd < rem ? xcd * (q + 1) : rem * (q + 1) + (xcd - rem) * q) + (b >> 3);
}

// rows row0 .. row0 + R - 1 of a K-contiguous operand, k-tile k0, into a swizzled [R][64] image
// (the fc_swz layout): R / 64 DMA instructions per wave, 8 rows each
template <int R>
__device__ __forceinline__ void fcp_stage(const uint16_t* __restrict__ X, int rows, int K, int row0, int k0,
                                          uint16_t* img, int wave, int lane) {
#pragma unroll
  for (int jj = 0; jj < R / 64; ++jj) {
    const int r0 = 8 * (wave + 8 * jj);
    const int r = r0 + (lane >> 3);
    const int kc = (lane & 7) ^ ((r >> 1) & 7);
    const int gr = min(row0 + r, rows - 1);  // past the end: a duplicate row, never stored
    __builtin_amdgcn_global_load_lds(X + (size_t)gr * K + k0 + 8 * kc,
                                     (__attribute__((address_space(3))) void*)(img + r0 * kFcBK), 16, 0, 0);
  }
}

// 64 lanes x 16 B that epilogue lanes with nothing to store write (a device global: no allocation,
// nothing to do inside a graph capture)
__device__ __attribute__((aligned(16))) float fcp_dummy[64 * 4];

struct FcpPart {  // fp32 split-K partials part[z][M][N]
  float* part;
  static constexpr int kOpsPerFrag = 1;
  static constexpr bool kPrefetch = false;
};
struct FcpMask {  // bf16 out = product * (mask > 0), mask loads prefetched during the last k-tile
  uint16_t* out;
  const uint16_t* mask;
  static constexpr int kOpsPerFrag = 2;
  static constexpr bool kPrefetch = true;
};

template <int BM, int BN, int WGM, int STAGES>
struct FcpCfg {
  static constexpr int WGN = 8 / WGM;
  static constexpr int TM = BM / WGM, TN = BN / WGN;  // per-wave tile
  static constexpr int FM = TM / 16, FN = TN / 16;
  static constexpr int ImgA = BM * kFcBK, ImgB = BN * kFcBK;
  static constexpr int Stage = ImgA + ImgB;
  static constexpr int LdsBytes = STAGES * Stage * 2;
  static constexpr int D = (BM + BN) / 64;  // DMA instructions per wave per k-tile
  static_assert(WGM * WGN == 8 && TM % 16 == 0 && TN % 16 == 0 && BM % 64 == 0 && BN % 64 == 0, "tile shape");
  static_assert(STAGES == 2 || STAGES == 3, "ring depth");
  static_assert(LdsBytes <= 160 * 1024, "LDS");
};

// One 16-byte LDS-DMA piece.  Kept in a __device__ function: an amdgcn builtin called directly in
// a lambda inside a kernel template makes hipcc's HOST pass drop the kernel's launch stub
// without a diagnostic (the .so then fails to load with an undefined symbol).
__device__ __forceinline__ void fcp_glds(const uint16_t* src, uint16_t* dst) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
}

// bf16 pair (round to nearest even, NaN kept) in one v_cvt_pk_bf16_f32
__device__ __forceinline__ uint32_t fcp_pk_bf16(float a, float b) {
  typedef __bf16 bf2 __attribute__((ext_vector_type(2)));
  typedef float f2 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f2){a, b}, bf2));
}
// keep-mask of a word of two bf16: 0xffff per half whose value is > 0 (sign clear, not zero;
// the layer input is a ReLU output)
__device__ __forceinline__ uint32_t fcp_pos_mask(uint32_t w) {
  return (((int32_t)(w << 16) > 0) ? 0x0000ffffu : 0u) | (((int32_t)w > 0xffff) ? 0xffff0000u : 0u);
}

// C[m][n] = sum_k A[m][k] B[n][k]; items = (n-tile fastest, m-tile, split z), block lid takes
// items lid, lid + G, ...  Per-item work (the tile decode, the lanes' DMA source rows) is done
// once per item; a k-step adds only the k offset.
template <int BM, int BN, int WGM, int STAGES, class Epi>
__global__ void __launch_bounds__(kFcThreads, 1)
fcp_nt_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B, Epi epi, int M, int N, int K,
              int tiles_m, int tiles_n, int kps, int items) {
  using C = FcpCfg<BM, BN, WGM, STAGES>;
  constexpr int FM = C::FM, FN = C::FN, E = Epi::kOpsPerFrag * FM * FN;
  constexpr int JA = BM / 64, JB = BN / 64;  // DMA instructions per wave per operand
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int G = gridDim.x, lid = fcp_lid();
  const int ktot = K / kFcBK, tmn = tiles_m * tiles_n;
  int S = 0;
  for (int it = lid; it < items; it += G) S += min(ktot - (it / tmn) * kps, kps);

  // issue cursor: the current item's lane source rows (k offset added per step)
  const uint16_t* pa[JA];
  const uint16_t* pb[JB];
  int i_it = lid, i_kt = 0, i_nk = 0, i_k = 0, i_slot = 0, i_u = 0;
  auto issue_item = [&](int it) {
    const int tn = it % tiles_n, rest = it / tiles_n, tm = rest % tiles_m, z = rest / tiles_m;
    i_nk = min(ktot - z * kps, kps);
    i_k = z * kps * kFcBK;
#pragma unroll
    for (int jj = 0; jj < JA; ++jj) {
      const int r = 8 * (wave + 8 * jj) + (lane >> 3), kc = (lane & 7) ^ ((r >> 1) & 7);
      pa[jj] = A + (size_t)min(tm * BM + r, M - 1) * K + 8 * kc;  // past the end: a duplicate row
    }
#pragma unroll
    for (int jj = 0; jj < JB; ++jj) {
      const int r = 8 * (wave + 8 * jj) + (lane >> 3), kc = (lane & 7) ^ ((r >> 1) & 7);
      pb[jj] = B + (size_t)min(tn * BN + r, N - 1) * K + 8 * kc;
    }
  };
  if (S) issue_item(lid);
  auto issue = [&]() {
    uint16_t* st = smem + i_slot * C::Stage;
#pragma unroll
    for (int jj = 0; jj < JA; ++jj)
      fcp_glds(pa[jj] + i_k, st + 8 * (wave + 8 * jj) * kFcBK);
#pragma unroll
    for (int jj = 0; jj < JB; ++jj)
      fcp_glds(pb[jj] + i_k, st + C::ImgA + 8 * (wave + 8 * jj) * kFcBK);
    ++i_u;
    i_slot = i_slot + 1 == STAGES ? 0 : i_slot + 1;
    i_k += kFcBK;
    if (++i_kt == i_nk) {
      i_kt = 0;
      i_it += G;
      if (i_it < items) issue_item(i_it);
    }
  };
#pragma unroll
  for (int t = 0; t < STAGES - 1; ++t)
    if (i_u < S) issue();

  const int wm = wave % WGM, wn = wave / WGM;
  const int g = lane >> 4, li = lane & 15;
  f32x4_t acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  uint2 pre[FM][FN];
  // compute cursor
  int c_it = lid, c_kt = 0, c_nk = 0, c_z = 0, mb = 0, nb = 0, c_slot = 0;
  auto compute_item = [&](int it) {
    const int tn = it % tiles_n, rest = it / tiles_n, tm = rest % tiles_m;
    c_z = rest / tiles_m;
    c_nk = min(ktot - c_z * kps, kps);
    mb = tm * BM + C::TM * wm + li;
    nb = tn * BN + C::TN * wn + 4 * g;
  };
  if (S) compute_item(lid);
  bool e1 = false, e2 = false;  // an epilogue ran at step u - 1 / u - 2
  for (int u = 0; u < S; ++u) {
    if constexpr (STAGES == 3) fcp_wait_window<C::D, E>(u + 1 < S, e1 || e2);
    else fcp_wait_window<C::D, E>(false, e1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();  // DMA(u) visible to all; every wave done reading step u - 1's stage
    asm volatile("" ::: "memory");
    if (i_u < S) issue();
    const bool last = c_kt + 1 == c_nk;
    const uint16_t* Ai = smem + c_slot * C::Stage;
    const uint16_t* Bi = Ai + C::ImgA;
    c_slot = c_slot + 1 == STAGES ? 0 : c_slot + 1;
    auto compute = [&]() {
#pragma unroll
      for (int s = 0; s < kFcBK / 32; ++s) {
        const int kc = 4 * s + g;
        bf16x8_t af[FM], bfr[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i)
          af[i] = *reinterpret_cast<const bf16x8_t*>(Ai + 8 * fc_swz(C::TM * wm + 16 * i + li, kc));
#pragma unroll
        for (int j = 0; j < FN; ++j)
          bfr[j] = *reinterpret_cast<const bf16x8_t*>(Bi + 8 * fc_swz(C::TN * wn + 16 * j + li, kc));
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
      }
    };
    e2 = e1;
    e1 = last;
    if (!last) {
      compute();
      ++c_kt;
      continue;
    }
    // the tile's last k-tile: (mask prefetch,) MFMAs, epilogue -- on ONE path, so the compiler's
    // wait for the prefetched mask sits at its use, not at every later load
    if constexpr (Epi::kPrefetch) {
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const uint16_t* mrow = epi.mask + (size_t)min(mb + 16 * i, M - 1) * N;
#pragma unroll
        for (int j = 0; j < FN; ++j) pre[i][j] = *reinterpret_cast<const uint2*>(mrow + min(nb + 16 * j, N - 4));
      }
    }
    compute();
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int m = mb + 16 * i;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = nb + 16 * j;
        const bool ok = m < M && n < N;
        const f32x4_t v = acc[i][j];
        if constexpr (Epi::kPrefetch) {
          const uint2 o = make_uint2(fcp_pk_bf16(v[0], v[1]) & fcp_pos_mask(pre[i][j].x),
                                     fcp_pk_bf16(v[2], v[3]) & fcp_pos_mask(pre[i][j].y));
          uint2* dst = ok ? reinterpret_cast<uint2*>(epi.out + (size_t)m * N + n)
                          : reinterpret_cast<uint2*>(fcp_dummy + 4 * lane);
          *dst = o;
        } else {
          f32x4_t* dst = ok ? reinterpret_cast<f32x4_t*>(epi.part + ((size_t)c_z * M + m) * N + n)
                            : reinterpret_cast<f32x4_t*>(fcp_dummy + 4 * lane);
          *dst = v;
        }
        acc[i][j] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      }
    }
    c_kt = 0;
    c_it += G;
    if (c_it < items) compute_item(c_it);
  }
}

// X^T . Y (the fc weight gradient) on the same persistent ring: items = (i-tile fastest, j-tile,
// split z) over [64 r] x [128 col] sub-images (the fc_tn layout: ds_read_b64_tr_b16 fragments);
// with BIAS the padded columns past J read ``ones`` and column J's sums land in bias_part.
template <int BI, int BJ, int WGI, int STAGES, bool BIAS>
__global__ void __launch_bounds__(kFcThreads, 1)
fcp_tn_kernel(const uint16_t* __restrict__ X, const uint16_t* __restrict__ Y, float* __restrict__ part, int R, int I,
              int J, int tiles_i, int tiles_j, int kps, int items, const uint16_t* __restrict__ ones,
              float* __restrict__ bias_part) {
  constexpr int WGJ = 8 / WGI, TI = BI / WGI, TJ = BJ / WGJ, FI = TI / 16, FJ = TJ / 16;
  constexpr int HX = BI / 128, HY = BJ / 128;  // sub-images per operand, 2 DMA instructions each per wave
  constexpr int ImgX = BI * 64, ImgY = BJ * 64, Stage = ImgX + ImgY;
  constexpr int D = 2 * (HX + HY), E = FI * FJ * (BIAS ? 2 : 1);
  static_assert(BI % 128 == 0 && BJ % 128 == 0 && TI % 16 == 0 && TJ % 16 == 0 && (TI <= 128) && (TJ <= 128), "tile");
  static_assert(STAGES * Stage * 2 <= 160 * 1024, "LDS");
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int G = gridDim.x, lid = fcp_lid();
  const int rtot = R / 64, tij = tiles_i * tiles_j;
  int S = 0;
  for (int it = lid; it < items; it += G) S += min(rtot - (it / tij) * kps, kps);

  // lane sources: image rows r0 + (lane >> 4), r0 = 8 wave + 4 jj; 16-byte chunk (lane & 15)
  // XOR-swizzled (fc_tn_swz); a step moves 64 rows down (ones-column lanes stay put)
  const uint16_t* px[HX][2];
  const uint16_t* py[HY][2];
  size_t ystep[HY][2];
  int i_it = lid, i_kt = 0, i_nk = 0, i_slot = 0, i_u = 0;
  const size_t xstep = (size_t)64 * I;
  auto issue_item = [&](int it) {
    const int ti = it % tiles_i, rest = it / tiles_i, tj = rest % tiles_j, z = rest / tiles_j;
    i_nk = min(rtot - z * kps, kps);
    const size_t r0g = (size_t)z * kps * 64;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int r = 8 * wave + 4 * jj + (lane >> 4);
      const int c = (lane & 15) ^ (2 * ((r & 3) | (((r >> 3) & 1) << 2)));
#pragma unroll
      for (int h = 0; h < HX; ++h) px[h][jj] = X + (r0g + r) * I + min(ti * BI + 128 * h + 8 * c, I - 8);
#pragma unroll
      for (int h = 0; h < HY; ++h) {
        const int col = tj * BJ + 128 * h + 8 * c;
        const bool one = BIAS && col >= J;
        py[h][jj] = one ? ones : Y + (r0g + r) * J + min(col, J - 8);
        ystep[h][jj] = one ? 0 : (size_t)64 * J;
      }
    }
  };
  if (S) issue_item(lid);
  auto issue = [&]() {
    uint16_t* st = smem + i_slot * Stage;
#pragma unroll
    for (int jj = 0; jj < 2; ++jj) {
      const int r0 = 8 * wave + 4 * jj;
#pragma unroll
      for (int h = 0; h < HX; ++h) {
        fcp_glds(px[h][jj], st + h * kFcImg + r0 * 128);
        px[h][jj] += xstep;
      }
#pragma unroll
      for (int h = 0; h < HY; ++h) {
        fcp_glds(py[h][jj], st + ImgX + h * kFcImg + r0 * 128);
        py[h][jj] += ystep[h][jj];
      }
    }
    ++i_u;
    i_slot = i_slot + 1 == STAGES ? 0 : i_slot + 1;
    if (++i_kt == i_nk) {
      i_kt = 0;
      i_it += G;
      if (i_it < items) issue_item(i_it);
    }
  };
#pragma unroll
  for (int t = 0; t < STAGES - 1; ++t)
    if (i_u < S) issue();

  const int wi = wave % WGI, wj = wave / WGI;
  const int g = lane >> 4, li = lane & 15;
  f32x4_t acc[FI][FJ];
#pragma unroll
  for (int a = 0; a < FI; ++a)
#pragma unroll
    for (int c = 0; c < FJ; ++c) acc[a][c] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  int c_it = lid, c_kt = 0, c_nk = 0, c_slot = 0, ib = 0, jb = 0, c_z = 0;
  auto compute_item = [&](int it) {
    const int ti = it % tiles_i, rest = it / tiles_i, tj = rest % tiles_j;
    c_z = rest / tiles_j;
    c_nk = min(rtot - c_z * kps, kps);
    ib = ti * BI + TI * wi + li;
    jb = tj * BJ + TJ * wj + 4 * g;
  };
  if (S) compute_item(lid);
  bool e1 = false, e2 = false;
  // the wave's columns inside its operand images: sub-image (TI * wi) / 128, offset (TI * wi) % 128
  const int xo = (TI * wi / 128) * kFcImg, xc = TI * wi % 128;
  const int yo = ImgX + (TJ * wj / 128) * kFcImg, yc = TJ * wj % 128;
  for (int u = 0; u < S; ++u) {
    if constexpr (STAGES == 3) fcp_wait_window<D, E>(u + 1 < S, e1 || e2);
    else fcp_wait_window<D, E>(false, e1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (i_u < S) issue();
    const bool last = c_kt + 1 == c_nk;
    const uint16_t* st = smem + c_slot * Stage;
    c_slot = c_slot + 1 == STAGES ? 0 : c_slot + 1;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8_t xf[FI], yf[FJ];
#pragma unroll
      for (int a = 0; a < FI; ++a) xf[a] = fcp_tn_frag(st + xo, 32 * s + 8 * g, xc + 16 * a, lane);
#pragma unroll
      for (int c = 0; c < FJ; ++c) yf[c] = fcp_tn_frag(st + yo, 32 * s + 8 * g, yc + 16 * c, lane);
      fcp_lgkm_wait<FI, FJ>(xf, yf);
#pragma unroll
      for (int a = 0; a < FI; ++a)
#pragma unroll
        for (int c = 0; c < FJ; ++c) acc[a][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(yf[c], xf[a], acc[a][c], 0, 0, 0);
    }
    e2 = e1;
    e1 = last;
    if (!last) {
      ++c_kt;
      continue;
    }
#pragma unroll
    for (int a = 0; a < FI; ++a) {
      const int i = ib + 16 * a;
#pragma unroll
      for (int c = 0; c < FJ; ++c) {
        const int j = jb + 16 * c;
        f32x4_t* dst = (i < I && j < J) ? reinterpret_cast<f32x4_t*>(part + ((size_t)c_z * I + i) * J + j)
                                        : reinterpret_cast<f32x4_t*>(fcp_dummy + 4 * lane);
        *dst = acc[a][c];
        if constexpr (BIAS) {  // the ones column
          float* bd = (i < I && j == J) ? bias_part + (size_t)c_z * I + i : fcp_dummy + 4 * lane;
          *bd = acc[a][c][0];
        }
        acc[a][c] = f32x4_t{0.f, 0.f, 0.f, 0.f};
      }
    }
    c_kt = 0;
    c_it += G;
    if (c_it < items) compute_item(c_it);
  }
}

static int fcp_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
  }
  return cus;
}

// split count for a persistent launch: the largest s <= max_splits whose items (tiles x s) fit
// one round of CUs, each split keeping >= 2 k-tiles; returns (kps, used splits)
static void fcp_splits(int tiles, int ktiles, int max_splits, int cus, int* kps, int* used) {
  int s = 1;
  for (int c = 2; c <= max_splits; ++c)
    if (tiles * c <= cus && ktiles / c >= 2) s = c;
  // rebalance until the splits actually used (ceil(ktiles / k), which can be < s: kt = 13 with
  // s = 5 gives k = 3 and splits 3,3,3,3,1) all keep >= 2 k-tiles, the last one included
  int k = (ktiles + s - 1) / s;
  while (s > 1 && ktiles - ((ktiles + k - 1) / k - 1) * k < 2) {
    s -= 1;
    k = (ktiles + s - 1) / s;
  }
  *kps = k;
  *used = (ktiles + k - 1) / k;
}

// 0 = the 128 x 128 kernels above, 1 = persistent big tiles.  RRL_FC_BIG (read per call) forces
// one; unset, each call site takes the kernel that measured faster at its size
// (tools/fc_kbench.py, profiles/r5_fc_persistent_kbench.jsonl): the persistent tiles for the
// forward at >= 4,096 rows and the weight gradient at >= 20,480 rows, never for the data gradient.
static int fc_big(bool auto_big = false) {
  const char* e = getenv("RRL_FC_BIG");
  if (!e || !e[0]) return auto_big ? 1 : 0;
  return e[0] != '0';
}

template <int BM, int BN, int WGM, int STAGES, class Epi>
static int launch_fcp_nt(const uint16_t* A, const uint16_t* B, Epi epi, int M, int N, int K, int kps, int used,
                         hipStream_t st) {
  using C = FcpCfg<BM, BN, WGM, STAGES>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)fcp_nt_kernel<BM, BN, WGM, STAGES, Epi>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, C::LdsBytes);
    attr = true;
  }
  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const int items = tiles_m * tiles_n * used;
  const int grid = min(items, fcp_cus());
  hipLaunchKernelGGL((fcp_nt_kernel<BM, BN, WGM, STAGES, Epi>), dim3(grid), dim3(kFcThreads), C::LdsBytes, st, A, B,
                     epi, M, N, K, tiles_m, tiles_n, kps, items);
  return (int)hipGetLastError();
}

template <int BI, int BJ, int WGI, int STAGES, bool BIAS>
static int launch_fcp_tn(const uint16_t* X, const uint16_t* Y, float* part, int R, int I, int J, int kps, int used,
                         const uint16_t* ones, float* bias_part, hipStream_t st) {
  constexpr int lds = STAGES * (BI + BJ) * 64 * 2;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)fcp_tn_kernel<BI, BJ, WGI, STAGES, BIAS>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr = true;
  }
  const int ti = (I + BI - 1) / BI, tj = (J + BJ - 1) / BJ, items = ti * tj * used;
  const int grid = min(items, fcp_cus());
  hipLaunchKernelGGL((fcp_tn_kernel<BI, BJ, WGI, STAGES, BIAS>), dim3(grid), dim3(kFcThreads), lds, st, X, Y, part, R,
                     I, J, ti, tj, kps, items, ones, bias_part);
  return (int)hipGetLastError();
}

}  // namespace rrl

using namespace rrl;

extern "C" {

// fp32 split-K partials part[splits][M][N] of A[M][K] . B[N][K]^T (K % 64 == 0, N % 4 == 0).
// Returns the number of splits actually used (<= splits), negative on a bad shape.
int rrl_fc_nt_part(const uint16_t* a, const uint16_t* b, float* part, int M, int N, int K, int splits,
                   void* stream_) {
  if (K % kFcBK || N % 4 || M < 1 || N < 1 || splits < 1) return -1;
  const int kt = K / kFcBK;
  const int kps = (kt + splits - 1) / splits;
  const int used = (kt + kps - 1) / kps;
  const FcPartEpi epi{part, M, N};
  hipStream_t st = (hipStream_t)stream_;
  const int big = fc_big(M >= 4096);
  if (big && kt >= 2) {  // 256 x 128 persistent tiles
    const int tiles = ((M + 255) / 256) * ((N + 127) / 128);
    int kps2, used2;
    fcp_splits(tiles, kt, splits, fcp_cus(), &kps2, &used2);
    const int rc = launch_fcp_nt<256, 128, 4, 3>(a, b, FcpPart{part}, M, N, K, kps2, used2, st);
    return rc ? -rc - 1000 : used2;
  }
  const int v = fc_stages(0, 4);
  const int rc = v == 4 ? launch_fc_nt<FcPartEpi, 4>(a, b, epi, M, N, K, used, st)
                        : (v == 3 ? launch_fc_nt<FcPartEpi, 3>(a, b, epi, M, N, K, used, st)
                                  : launch_fc_nt<FcPartEpi, 2>(a, b, epi, M, N, K, used, st));
  return rc ? -rc - 1000 : used;
}

// bf16 out[M][N] = (A[M][K] . B[N][K]^T) * (mask[M][N] > 0)   (K % 64 == 0, N % 4 == 0)
int rrl_fc_nt_mask(const uint16_t* a, const uint16_t* b, const uint16_t* mask, uint16_t* out, int M, int N, int K,
                   void* stream_) {
  if (K % kFcBK || N % 4 || M < 1 || N < 1) return -1;
  hipStream_t st = (hipStream_t)stream_;
  if (fc_big(false) && K / kFcBK >= 2)  // 256 x 128 persistent tiles, whole K per item
    return launch_fcp_nt<256, 128, 4, 3>(a, b, FcpMask{out, mask}, M, N, K, K / kFcBK, 1, st);
  // The LDS-staged epilogue (16-byte mask loads and stores): 276 -> 220 us at 40,960 x 3,136 in
  // tools/fc_kbench.py, and since the round-5 weight-gradient change (its transposed reads no
  // longer drain the DMA ring, so the side-stream GEMM beside this one is shorter) also faster
  // at 10,240 rows inside the Pong update: +1.0 % end to end (profiles/r5_pong_side_epi_ab.txt;
  // round 3 had measured the direct epilogue 0.7 % faster there).  RRL_FC_DIRECT_EPI = 1 forces
  // the direct epilogue.
  const char* e = getenv("RRL_FC_DIRECT_EPI");
  if (N % 8 == 0 && !(e && e[0] == '1')) {
    const FcMaskStagedEpi epi{out, mask, M, N};
    return fc_stages(1, 2) == 3 ? launch_fc_nt<FcMaskStagedEpi, 3>(a, b, epi, M, N, K, 1, st)
                                : launch_fc_nt<FcMaskStagedEpi, 2>(a, b, epi, M, N, K, 1, st);
  }
  const FcMaskEpi epi{out, mask, M, N};
  return fc_stages(1, 2) == 3 ? launch_fc_nt<FcMaskEpi, 3>(a, b, epi, M, N, K, 1, st)
                              : launch_fc_nt<FcMaskEpi, 2>(a, b, epi, M, N, K, 1, st);
}

// fp32 partials part[splits][I][J] of X[R][I]^T . Y[R][J] (R % 64 == 0, I, J % 8 == 0);
// returns the number of splits used.
// With ``ones`` + ``bias_part`` (J % 128 != 0 and J % 4 == 0: the last column tile has a pad
// column, J itself): bias_part[splits][I] = the row sums of X, i.e. the layer's bias gradient.
int rrl_fc_tn_part(const uint16_t* x, const uint16_t* y, float* part, int R, int I, int J, int splits,
                   const uint16_t* ones, float* bias_part, void* stream_) {
  if (R % 64 || I % 8 || J % 8 || R < 64 || splits < 1) return -1;
  if ((ones == nullptr) != (bias_part == nullptr) || (bias_part && J % 128 == 0)) return -1;
  hipStream_t st = (hipStream_t)stream_;
  // RRL_FC_TN_BIG (read per call) forces this site's choice alone; unset, RRL_FC_BIG / the size rule
  const char* tb = getenv("RRL_FC_TN_BIG");
  const bool big = (tb && tb[0]) ? tb[0] != '0' : fc_big(R >= 20480);
  if (big && R / 64 >= 2 && I % 4 == 0) {  // 256 x 128 persistent tiles
    const int tiles = ((I + 255) / 256) * ((J + 127) / 128);
    int kps2, used2;
    fcp_splits(tiles, R / 64, splits, fcp_cus(), &kps2, &used2);
    const int rc = bias_part ? launch_fcp_tn<256, 128, 4, 3, true>(x, y, part, R, I, J, kps2, used2, ones, bias_part, st)
                             : launch_fcp_tn<256, 128, 4, 3, false>(x, y, part, R, I, J, kps2, used2, ones, bias_part, st);
    return rc ? -rc - 1000 : used2;
  }
  const int rt = R / 64, kps = (rt + splits - 1) / splits, used = (rt + kps - 1) / kps;
  const int rc = fc_stages(2, 2) == 2 ? launch_fc_tn<2>(x, y, part, R, I, J, used, ones, bias_part, st)
                                      : launch_fc_tn<3>(x, y, part, R, I, J, used, ones, bias_part, st);
  return rc ? -rc - 1000 : used;
}

int rrl_transpose_bf16(const uint16_t* in, uint16_t* out, int R, int C, void* stream_) {
  if (R % 8 || C % 8) return -1;
  hipLaunchKernelGGL(transpose_bf16_kernel, dim3((C + 63) / 64, (R + 63) / 64), dim3(256), 0, (hipStream_t)stream_,
                     in, out, R, C);
  return (int)hipGetLastError();
}

}  // extern "C"
