// Fused Nature-CNN conv stack for the pixel A2C model (BASELINE.json config 4).
//
// Forward: conv1 (space-to-depth 2x2/1 over 21x21x64 uint8 frames -> 20x20x32) -> ReLU ->
// conv2 (4x4/2 -> 9x9x64) -> ReLU -> conv3 (3x3/1 -> 7x7x64) -> ReLU in ONE persistent
// launch, every intermediate activation resident in LDS.  The per-layer kernels this
// replaces (conv1_fwd_s2d_kernel and conv_fwd_img_kernel x 2 in cnn.hip) each streamed
// their input image from HBM and paid their own launch fill / drain; here a frame is read
// once and a1 / a2 / a3 are written once (the backward pass needs them) and never re-read.
//
// Geometry per frame (bf16 activations, fp32 accumulate on v_mfma_f32_16x16x32_bf16):
//   conv1  400 px x 32 co, K = 256 (4 taps x 64 s2d channels)   25 x 2 (px tile, co tile) units
//   conv2   81 px x 64 co, K = 512 (16 taps x 32 channels)         6 x 4 units
//   conv3   49 px x 64 co, K = 576 (9 taps x 64 channels)          4 x 4 units
//
// Eight waves, two per SIMD, split by LAYER so that each wave keeps only one layer's
// weights in registers besides conv1's (all three layers' fragments are 168 VGPRs per
// wave, which spilled at two waves per SIMD and starved the fragment reads at one):
//   every wave        conv1 co tile (w & 1), pixel tiles (w >> 1) + 4 t       (32 VGPRs of W1)
//   waves 0-3 ("A")   conv2 co tile w over all 6 pixel tiles of frame j       (64 VGPRs of W2)
//   waves 4-7 ("B")   conv3 co tile w - 4 over all 4 pixel tiles of frame j-1 (72 VGPRs of W3)
// so conv2 of frame j and conv3 of frame j-1 run side by side between the same two
// barriers (a2 is double-buffered).  Each layer's k-step order matches the per-layer
// kernels', so the fused outputs equal theirs up to fma contraction in the epilogue.
//
// Per iteration j (frame n_j = blockIdx.x + j * gridDim.x):
//   store frame n_j (prefetched into registers) -> LDS; prefetch frame n_{j+1}      | B0 .. B1
//   copy out a2(n_{j-1}) and a3(n_{j-2}); conv1(n_j) -> A1                          | B1 .. B2
//   copy out a1(n_j); A: conv2(n_j) -> A2[j & 1]; B: conv3(n_{j-1}) -> A3          | B2 .. B0
#include "gemm_bf16.h"
#include "pong_render.h"

namespace rrl {

// Two fp32 -> packed bf16 pair (round to nearest even), a in the low half.  A vector
// conversion, not inline asm: it lowers to gfx950's v_cvt_pk_bf16_f32 AND stays visible to
// the hazard recognizer -- an asm cvt reading an MFMA result directly got no wait states
// and read the accumulator registers before the MFMA had written them.
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  typedef float f32x2_t __attribute__((ext_vector_type(2)));
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t{a, b}), bf16x2_t));
}
// The MFMAs below run with the weights as the A operand and the activation rows as B, so
// D = out^T: lane (i, g) holds 4 consecutive output channels 4g..4g+3 of pixel i, stored
// as ONE 8-byte LDS write (2 cvt_pk) instead of 4 scalar bf16 conversions and 2-byte writes.
__device__ __forceinline__ void store4_bf16(uint16_t* dst, float v0, float v1, float v2, float v3) {
  *reinterpret_cast<uint2*>(dst) = make_uint2(pk_bf16(v0, v1), pk_bf16(v2, v3));
}

// v where the ReLU mask m (8 packed bf16 activations) is > 0, else 0 -- bitwise on the packed
// halves (the masked values are already bf16: no round trip through fp32)
__device__ __forceinline__ uint32_t relu_mask2(uint32_t v, uint32_t m) {
  const uint32_t lo = ((m & 0x8000u) == 0u && (m & 0xffffu) != 0u) ? 0x0000ffffu : 0u;
  const uint32_t hi = ((m & 0x80000000u) == 0u && (m >> 16) != 0u) ? 0xffff0000u : 0u;
  return v & (lo | hi);
}
__device__ __forceinline__ uint4 relu_mask8(uint4 v, uint4 m) {
  return make_uint4(relu_mask2(v.x, m.x), relu_mask2(v.y, m.y), relu_mask2(v.z, m.z), relu_mask2(v.w, m.w));
}

namespace cs {
constexpr int kThreads = 512;
constexpr int kFrameLd = 80;                  // frame row: 64 channels + 16 pad (bf16)
constexpr int kFrameRows = 441;               // 21 x 21 s2d pixels
// the frame's 21 x 21 positions sit in LDS rows of 28 (position (a, b) at row 28 a + b): the
// conv1 fragment reads of 16 consecutive output pixels then hit disjoint banks, 1.6 -> 1.0
// LDS cycles per conflict-free cycle (tools/lds_bank_model.py --fwd)
constexpr int kFrameW = 28;
constexpr int kXiRows = 20 * kFrameW + 24;      // last position read: (20, 20) at row 580
constexpr int kA2Ld = 80;  // a2 / a3 rows: 64 co + 16 pad (72 measured 2.5x conflict cycles on the conv3 reads, 80 1.75x)
// Measured and not shipped (FwdLayout PROBE bits, profiles/r4_fwd_layouts.txt):
//  bit 4: a1 as four stride-2 phase images, (y, x) at row 100 (2 (y & 1) + (x & 1)) +
//   10 (y >> 1) + (x >> 1), rows of 48 elements, conv2 over a 9 x 10 grid -- its fragment reads
//   model conflict-free (2.0 -> 1.0; 40-element rows stay at 2.0 in any row order) and PMC
//   counted -37 % bank-conflict cycles, but the kernel ran 58.9 -> 67.2 us (SQ_WAIT_ANY +80 %);
//  bit 5: conv3 over a 7 x 9 grid (consecutive a2 rows, 1.75 -> 1.0 modelled): 54.8 -> 58.7 us
//   per 2,048 frames, Pong -1 to -2 % in an ABBA run on one box.
constexpr int kXi = 0;                                    // element offsets into LDS
constexpr int kA1 = kXi + kXiRows * kFrameLd;             // 46,720
// the largest variant (phase a1, its frame image cut to the 581 rows read): 163,552 bytes
constexpr int kLds = ((kXiRows - 3) * kFrameLd + 400 * 48 + 2 * 81 * kA2Ld + 49 * 64) * 2;
static_assert(kLds <= 160 * 1024, "LDS per workgroup");
__device__ __forceinline__ int a1_row(int p) {  // a1 pixel p = 20 y + x -> phase-image row
  const int y = p / 20, x = p - 20 * (p / 20);
  return 100 * (2 * (y & 1) + (x & 1)) + 10 * (y >> 1) + (x >> 1);
}
// layout of a PROBE variant: bit 4 = a1 as phase images in 48-element rows and conv2 over a
// 9 x 10 grid (a3 rows of 64 to fit), bit 5 = conv3 over a 7 x 9 grid; default = a1 as one
// 20 x 20 image in 40-element rows (conv2 over its 81 output pixels), conv3 over its 49 output
// pixels, a3 rows of 80
template <int PROBE>
struct FwdLayout {
  static constexpr bool kPhaseA1 = (PROBE & 16) != 0, kGrid3 = (PROBE & 32) != 0;
  static constexpr int kA1Ld = kPhaseA1 ? 48 : 40, kA3Ld = kPhaseA1 ? 64 : 80;
  static constexpr int kA1 = kPhaseA1 ? cs::kA1 - 3 * cs::kFrameLd : cs::kA1;
  static constexpr int kA2 = kA1 + 400 * kA1Ld, kA3 = kA2 + 2 * 81 * cs::kA2Ld;
  static_assert((kA3 + 49 * kA3Ld) * 2 <= cs::kLds, "variant fits in LDS");
  // discarded grid positions read past their image -- conv2 up to phase row 406, conv3 up to
  // buffer row 83 -- garbage in discarded output rows only, always inside the allocation
  static_assert(!kPhaseA1 || kA1 + 407 * kA1Ld <= kA3, "conv2 over-read stays below a3");
  static_assert(!kGrid3 || kA2 + (81 + 84) * cs::kA2Ld <= cs::kLds / 2, "conv3 over-read stays in LDS");
  static_assert(kA1 % 8 == 0 && kA2 % 8 == 0 && kA3 % 8 == 0, "16-byte aligned LDS regions");
};
constexpr int kXChunks = kFrameRows * 64 / 16;           // 16-byte chunks of one uint8 frame (1,764)
constexpr int kXPerT = (kXChunks + kThreads - 1) / kThreads;
}  // namespace cs

// PROBE (tools/cnn_kbench.py --probe, timing only -- outputs are garbage when bits 0-2 are set):
// bit 0 skips the MFMAs, bit 1 the global stores, bit 2 re-reads frame 0 (L2-hot), bit 3
// runs conv1 with one co tile per wave, bits 4-6 select earlier LDS layouts (FwdLayout)
template <int PROBE>
__global__ __launch_bounds__(cs::kThreads, 1) void conv_stack_fwd_kernel(
    const uint8_t* __restrict__ x, const uint16_t* __restrict__ w1, const float* __restrict__ b1,
    const uint16_t* __restrict__ w2, const float* __restrict__ b2, const uint16_t* __restrict__ w3,
    const float* __restrict__ b3, uint16_t* __restrict__ y1, uint16_t* __restrict__ y2,
    uint16_t* __restrict__ y3, int N) {
  using namespace cs;
  using L = FwdLayout<PROBE>;
  constexpr int kA1Ld = L::kA1Ld, kA3Ld = L::kA3Ld, kA1 = L::kA1, kA2 = L::kA2, kA3 = L::kA3;
  auto a1r = [](int p) { return L::kPhaseA1 ? a1_row(p) : p; };
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* Xi = smem + kXi;  // [21 x 28][80] frame as bf16 integers 0..255
  uint16_t* A1 = smem + kA1;  // [400][40] conv1 output (PROBE bit 4: 4 x [100][48] phase images)
  uint16_t* A3 = smem + kA3;  // [49][64]  conv3 output
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i = lane & 15, g = lane >> 4;
  const bool role_a = wave < 4;
  const int ct = wave & 3;  // co tile of conv2 (A) / conv3 (B)

  // stationary weights: B fragment = W[co][8 consecutive k], co = 16 * tile + i
  // conv1: with C1BOTH (default) every wave computes both co tiles of its pixel tiles (each
  // frame fragment read feeds two MFMAs; W1 for both tiles in registers): 63.6 -> 59.2 us per
  // 2,048 frames; PROBE bit 3 selects the one-co-tile-per-wave split for comparison
  constexpr bool C1BOTH = (PROBE & 8) == 0;
  const int c1 = C1BOTH ? 0 : (wave & 1);
  bf16x8_t f1[8], f1b[C1BOTH ? 8 : 1], fw[18];  // fw: W2 (16 k-steps) on A waves, W3 (18) on B waves
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) f1[ks] = *reinterpret_cast<const bf16x8_t*>(w1 + (16 * c1 + i) * 256 + 32 * ks + 8 * g);
  if (C1BOTH) {
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) f1b[C1BOTH ? ks : 0] = *reinterpret_cast<const bf16x8_t*>(w1 + (16 + i) * 256 + 32 * ks + 8 * g);
  }
  if (role_a) {
#pragma unroll
    for (int ks = 0; ks < 16; ++ks) fw[ks] = *reinterpret_cast<const bf16x8_t*>(w2 + (16 * ct + i) * 512 + 32 * ks + 8 * g);
    fw[16] = fw[17] = fw[0];
  } else {
#pragma unroll
    for (int ks = 0; ks < 18; ++ks) fw[ks] = *reinterpret_cast<const bf16x8_t*>(w3 + (16 * ct + i) * 576 + 32 * ks + 8 * g);
  }
  // biases of this lane's 4 output channels (co = 16 tile + 4 g + r)
  const f32x4_t bias1 = *reinterpret_cast<const f32x4_t*>(b1 + 16 * c1 + 4 * g);
  const f32x4_t bias1b = *reinterpret_cast<const f32x4_t*>(b1 + 16 + 4 * g);  // co tile 1 (C1BOTH)
  const f32x4_t bias23 = *reinterpret_cast<const f32x4_t*>((role_a ? b2 : b3) + 16 * ct + 4 * g);

  const int G = gridDim.x, n0 = blockIdx.x;
  uint4 rx[kXPerT];
  auto gload = [&](size_t n) {
    if (PROBE & 4) n = 0;
    const uint4* xs = reinterpret_cast<const uint4*>(x + n * (kFrameRows * 64));
#pragma unroll
    for (int k = 0; k < kXPerT; ++k) {
      const int q = tid + kThreads * k;
      rx[k] = q < kXChunks ? xs[q] : make_uint4(0, 0, 0, 0);
    }
  };
  if (n0 < N) gload(n0);
  // j runs two frames past this workgroup's last one to drain conv3 and the a3 copy-out
  for (int j = 0; n0 + (j - 2) * G < N; ++j) {
    const int n = n0 + j * G;        // conv1 / conv2 frame
    const bool cur = n < N;
    const bool prev = j >= 1 && n - G < N;  // conv3 frame
    __syncthreads();  // B0: conv1 / conv2 / conv3 of the previous iteration are done
    if (cur) {
#pragma unroll
      for (int k = 0; k < kXPerT; ++k) {
        const int q = tid + kThreads * k;
        if (q < kXChunks) {
          const int pix = q >> 2, pa = pix / 21;
          uint16_t* d = Xi + (pix + (kFrameW - 21) * pa) * kFrameLd + (q & 3) * 16;
          *reinterpret_cast<uint4*>(d) = u8x8_to_bf16x8(make_uint2(rx[k].x, rx[k].y));
          *reinterpret_cast<uint4*>(d + 8) = u8x8_to_bf16x8(make_uint2(rx[k].z, rx[k].w));
        }
      }
      if (n + G < N) gload((size_t)n + G);  // lands while this frame computes
    }
    __syncthreads();  // B1
    // copy-outs of the previous iterations' a2 / a3 (conv1 touches neither buffer)
    if (prev && y2 && !(PROBE & 2)) {  // y2 / y1 null: a forward whose activations no backward reads
      const uint16_t* A2p = smem + kA2 + ((j - 1) & 1) * 81 * kA2Ld;
      uint4* yd = reinterpret_cast<uint4*>(y2 + (size_t)(n - G) * 81 * 64);
      for (int q = tid; q < 81 * 8; q += kThreads) yd[q] = *reinterpret_cast<const uint4*>(A2p + (q >> 3) * kA2Ld + (q & 7) * 8);
    }
    if (j >= 2 && !(PROBE & 2)) {
      uint4* yd = reinterpret_cast<uint4*>(y3 + (size_t)(n - 2 * G) * 49 * 64);
      for (int q = tid; q < 49 * 8; q += kThreads) yd[q] = *reinterpret_cast<const uint4*>(A3 + (q >> 3) * kA3Ld + (q & 7) * 8);
    }
    // ---- conv1, C1BOTH: pixel tiles wave + 8 t (t < 3, and t = 3 on wave 0), both co tiles
    if (cur && C1BOTH) {
      constexpr int MT = 4;
      f32x4_t acc0[MT], acc1[MT];
      int r0[MT];
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        acc0[t] = acc1[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        const int p = 16 * min(wave + 8 * t, 24) + i;
        r0[t] = (p / 20) * kFrameW + p % 20;
      }
      const int nt = wave == 0 ? 4 : 3;  // wave-uniform
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        const int tap = ks >> 1;
        const int off = ((tap >> 1) * kFrameW + (tap & 1)) * kFrameLd + 32 * (ks & 1) + 8 * g;
        bf16x8_t a[MT];
#pragma unroll
        for (int t = 0; t < MT; ++t)
          if (t < nt) a[t] = *reinterpret_cast<const bf16x8_t*>(Xi + r0[t] * kFrameLd + off);
#pragma unroll
        for (int t = 0; t < MT; ++t)
          if (t < nt) {
            acc0[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f1[ks], a[t], acc0[t], 0, 0, 0);
            acc1[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f1b[C1BOTH ? ks : 0], a[t], acc1[t], 0, 0, 0);
          }
      }
#pragma unroll
      for (int t = 0; t < MT; ++t)
        if (t < nt) {
          uint16_t* dst = A1 + a1r(16 * (wave + 8 * t) + i) * kA1Ld + 4 * g;
          store4_bf16(dst, fmaxf(kU8Scale * acc0[t][0] + bias1[0], 0.f), fmaxf(kU8Scale * acc0[t][1] + bias1[1], 0.f),
                      fmaxf(kU8Scale * acc0[t][2] + bias1[2], 0.f), fmaxf(kU8Scale * acc0[t][3] + bias1[3], 0.f));
          store4_bf16(dst + 16, fmaxf(kU8Scale * acc1[t][0] + bias1b[0], 0.f),
                      fmaxf(kU8Scale * acc1[t][1] + bias1b[1], 0.f), fmaxf(kU8Scale * acc1[t][2] + bias1b[2], 0.f),
                      fmaxf(kU8Scale * acc1[t][3] + bias1b[3], 0.f));
        }
    }
    // ---- conv1 (all waves): pixel tiles (wave >> 1) + 4 t, co tile c1
    if (cur && !C1BOTH) {
      constexpr int MT = 7;
      f32x4_t acc[MT];
      int r0[MT];
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        acc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        const int mt = min((wave >> 1) + 4 * t, 24);  // a tile past the frame recomputes tile 24
        const int p = 16 * mt + i;
        r0[t] = (p / 20) * kFrameW + p % 20;  // frame row of tap (0, 0)
      }
      // k-step outer, tiles inner: MT independent MFMAs per k-step, their reads batched ahead
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        const int tap = ks >> 1;
        const int off = ((tap >> 1) * kFrameW + (tap & 1)) * kFrameLd + 32 * (ks & 1) + 8 * g;
        bf16x8_t a[MT];
#pragma unroll
        for (int t = 0; t < MT; ++t) a[t] = *reinterpret_cast<const bf16x8_t*>(Xi + r0[t] * kFrameLd + off);
#pragma unroll
        for (int t = 0; t < MT; ++t) if (!(PROBE & 1)) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f1[ks], a[t], acc[t], 0, 0, 0);
        else acc[t][0] += (float)a[t][0];
      }
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int mt = (wave >> 1) + 4 * t;
        if (mt < 25) {
          float v[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = fmaxf(kU8Scale * acc[t][r] + bias1[r], 0.f);
          store4_bf16(A1 + a1r(16 * mt + i) * kA1Ld + 16 * c1 + 4 * g, v[0], v[1], v[2], v[3]);
        }
      }
    }
    __syncthreads();  // B2: a1(n) complete
    if (cur && y1 && !(PROBE & 2)) {
      uint4* yd = reinterpret_cast<uint4*>(y1 + (size_t)n * 400 * 32);
      for (int q = tid; q < 400 * 4; q += kThreads) yd[q] = *reinterpret_cast<const uint4*>(A1 + a1r(q >> 2) * kA1Ld + (q & 3) * 8);
    }
    if (role_a) {
      // ---- conv2(n): co tile ct, all 6 pixel tiles (81 px; rows past the image are discarded)
      if (cur) {
        uint16_t* A2c = smem + kA2 + (j & 1) * 81 * kA2Ld;
        constexpr int MT = 6;
        f32x4_t acc[MT];
        int r0[MT];
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          acc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
          if (L::kPhaseA1) {
            r0[t] = 16 * t + i;  // grid position p = 10 oh + ow: phase row 10 oh + ow of tap (0, 0)
          } else {
            const int p = 16 * t + i, pc = p < 81 ? p : 0, oh = pc / 9, ow = pc - oh * 9;
            r0[t] = 2 * oh * 20 + 2 * ow;
          }
        }
#pragma unroll
        for (int ks = 0; ks < 16; ++ks) {
          const int kh = ks >> 2, kw = ks & 3;
          const int off = (L::kPhaseA1 ? 100 * (2 * (kh & 1) + (kw & 1)) + 10 * (kh >> 1) + (kw >> 1) : kh * 20 + kw) * kA1Ld + 8 * g;
          bf16x8_t a[MT];
#pragma unroll
          for (int t = 0; t < MT; ++t) a[t] = *reinterpret_cast<const bf16x8_t*>(A1 + r0[t] * kA1Ld + off);
#pragma unroll
          for (int t = 0; t < MT; ++t) if (!(PROBE & 1)) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[ks], a[t], acc[t], 0, 0, 0);
          else acc[t][0] += (float)a[t][0];
        }
#pragma unroll
        for (int t = 0; t < MT; ++t) {
          const int p = 16 * t + i, oh = p / 10, ow = p - 10 * (p / 10);
          if (L::kPhaseA1 ? (p < 90 && ow < 9) : p < 81)
            store4_bf16(A2c + (L::kPhaseA1 ? 9 * oh + ow : p) * kA2Ld + 16 * ct + 4 * g, fmaxf(acc[t][0] + bias23[0], 0.f),
                        fmaxf(acc[t][1] + bias23[1], 0.f), fmaxf(acc[t][2] + bias23[2], 0.f),
                        fmaxf(acc[t][3] + bias23[3], 0.f));
        }
      }
    } else if (prev) {
      // ---- conv3(n - G): co tile ct, all 4 pixel tiles (49 px), input a2 from the other buffer
      const uint16_t* A2p = smem + kA2 + ((j - 1) & 1) * 81 * kA2Ld;
      constexpr int MT = 4;
      f32x4_t acc[MT];
      int r0[MT];
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        acc[t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        if (L::kGrid3) {
          r0[t] = 16 * t + i;  // grid position p = 9 oh + ow = the a2 row of tap (0, 0)
        } else {
          const int p = 16 * t + i, pc = p < 49 ? p : 0, oh = pc / 7, ow = pc - oh * 7;
          r0[t] = oh * 9 + ow;
        }
      }
#pragma unroll
      for (int ks = 0; ks < 18; ++ks) {
        const int tap = ks >> 1, kh = tap / 3, kw = tap - kh * 3;
        const int off = (kh * 9 + kw) * kA2Ld + 32 * (ks & 1) + 8 * g;
        bf16x8_t a[MT];
#pragma unroll
        for (int t = 0; t < MT; ++t) a[t] = *reinterpret_cast<const bf16x8_t*>(A2p + r0[t] * kA2Ld + off);
#pragma unroll
        for (int t = 0; t < MT; ++t) if (!(PROBE & 1)) acc[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[ks], a[t], acc[t], 0, 0, 0);
          else acc[t][0] += (float)a[t][0];
      }
#pragma unroll
      for (int t = 0; t < MT; ++t) {
        const int p = 16 * t + i, oh = p / 9, ow = p - 9 * (p / 9);
        if (L::kGrid3 ? (oh < 7 && ow < 7) : p < 49)
          store4_bf16(A3 + (L::kGrid3 ? 7 * oh + ow : p) * kA3Ld + 16 * ct + 4 * g, fmaxf(acc[t][0] + bias23[0], 0.f),
                      fmaxf(acc[t][1] + bias23[1], 0.f), fmaxf(acc[t][2] + bias23[2], 0.f),
                      fmaxf(acc[t][3] + bias23[3], 0.f));
      }
    }
  }
}

// ============================================================================= 16-wave forward
// The same conv stack as a THREE-stage layer pipeline over 16 waves (4 per SIMD):
//   waves 0-7   conv1 of frame n_j        (both co tiles, pixel tiles w + 8 t)
//   waves 8-11  conv2 of frame n_{j-1}    (co tile w - 8, all 6 pixel tiles)
//   waves 12-15 conv3 of frame n_{j-2}    (co tile w - 12, all 4 pixel tiles)
// all between the same two barriers, so every SIMD holds two conv1 waves, one conv2 and one
// conv3 wave and interleaves their MFMAs and LDS reads (conv_stack_fwd_kernel above has two
// waves per SIMD and runs conv1 alone between its own barriers).  What makes it fit:
//   * the frame stays uint8 in LDS (55.8 KB instead of 93 KB as bf16): each lane reads 16
//     channels of one position per tap (ONE ds_read_b128 feeds both k-steps of the tap: lane
//     group g carries channels 16 g + 8 h .. + 7 in k-step h, the weight fragments use the same
//     order) and widens them to bf16 in registers -- exact, 0..255 fit the bf16 mantissa;
//     96-byte position rows make those reads conflict-free (tools/lds_bank_model.py --fwd16);
//   * a1 / a2 double-buffered (stage j writes one buffer while stage j + 1 reads the other);
//   * a1 / a2 / a3 leave for HBM straight from the epilogue registers (8 bytes per lane), so
//     no copy-out pass reads LDS and a3 needs no LDS image at all;
//   * one fragment array serves every role's stationary weights (72 VGPRs: conv3's 18 k-steps;
//     conv1 uses 16, conv2 16), each role's tiles in passes small enough for 128 registers.
// Per iteration j: B0 | frame n_j: registers -> LDS, next frame's loads issued | B1 | the
// three stages.  j runs two frames past this workgroup's last one to drain conv2 / conv3.
#ifndef CS16_C2_MT
#define CS16_C2_MT 2
#endif
#ifndef CS16_C3_MT
#define CS16_C3_MT 2
#endif
namespace cs16 {
constexpr int kThreads = 1024;
constexpr int kFW = 28;                       // frame positions per LDS row group (as cs::kFrameW)
constexpr int kFS = 96;                       // bytes per frame position: 64 channels + 32 pad
constexpr int kFRows = 20 * kFW + 21;         // last position read: (20, 20)
constexpr int kFBytes = kFRows * kFS;         // 55,776
constexpr int kXChunks = 441 * 4;              // 16-byte chunks of one uint8 frame
constexpr int kXPerT = (kXChunks + kThreads - 1) / kThreads;
// a1 / a2 images per layout V (the 8-wave kernel's FwdLayout bits): default -- a1 as one 20 x 20
// image in 40-element rows, conv2 over its 81 output pixels (stride-2 reads: 2.0 LDS cycles per
// conflict-free cycle in tools/lds_bank_model.py), conv3 over its 49; bit 16 -- a1 as four
// stride-2 phase images in 48-element rows, conv2 over a 9 x 10 grid (1.0); bit 32 -- conv3
// over a 7 x 9 grid of a2 (1.75 -> 1.0).  Discarded grid positions read past the image into rows
// that stay inside their buffer (garbage in discarded outputs only).
// Measured slower and removed: the activations copied out through LDS with 16-byte stores one
// iteration later (a double-buffered a3 image, a third pipeline stage): 58.8 / 214.0 us against
// 51.8 / 177.3 us per 2,048 / 8,192 frames (profiles/r5_cnn16_kbench.jsonl) -- the epilogue's
// 8-byte stores are not what bounds this kernel.
// bit 2 -- fused render: the frames are drawn in the kernel from 16-float PongSynth frame
// histories (pong_render.h) instead of read from an observation tensor
template <int V>
struct L16 {
  static constexpr bool kPhaseA1 = (V & 16) != 0, kGrid3 = (V & 32) != 0, kRender = (V & 2) != 0;
  // bit 64 -- frame ring: the frame's 4 frames are read from the PongSynth frame store through
  // the observation's frame rows fidx[n][4] (pong_render.h) and interleaved into the same LDS image
  static constexpr bool kRing = (V & 64) != 0;
  // bit 128 (with 64) -- the ring's frames as one 16-byte load per (position, frame) on a pair of
  // lanes (frames 0, 1 / 2, 3), which swap the rows the other one stores through DPP: half the
  // load instructions of the 8-byte row pieces (A/B, tools/cnn_kbench.py fwd16_ring16)
  static constexpr bool kRing16 = kRing && (V & 128) != 0;
  // bit 256 (with 64) -- only the conv1 waves (tid < 441) load and store the frame: one 16-byte
  // load per frame per position, every load instruction 1 KB of one frame; the conv2 / conv3 waves
  // hold no frame registers (A/B, tools/cnn_kbench.py fwd16_ring_wide)
  static constexpr bool kRingWide = kRing && (V & 256) != 0;
  static constexpr bool kSetprio = (V & 4) != 0;  // s_setprio 1 around each role's MFMA clusters
  // static wave priority for the whole kernel (A/B): bit 1 raises the conv2 role, bit 8 the conv3 role
  static constexpr int kPrioRole2 = (V & 1) ? 2 : 0, kPrioRole3 = (V & 8) ? 2 : 0;
  static constexpr int kA1Ld = kPhaseA1 ? 48 : 40, kA2Ld = 80;
  static constexpr int kA1Rows = kPhaseA1 ? 407 : 400, kA2Rows = kGrid3 ? 84 : 81;
  static constexpr int kA1Elems = kA1Rows * kA1Ld, kA2Elems = kA2Rows * kA2Ld;
  // fused render: TWO frame buffers (the conv1 waves draw frame j + 1 while frame j is read) of
  // 441 positions x 64 B, 16-byte chunks XOR-swizzled (rfs_chunk: 2.0 -> 1.6 LDS cycles per
  // conflict-free cycle on the conv1 reads, tools/lds_bank_model.py)
  static constexpr int kRFBytes = 441 * 64;
  static constexpr int kA1Off = kRender ? 2 * kRFBytes : kFBytes;  // byte offsets
  static constexpr int kA2Off = kA1Off + 2 * kA1Elems * 2;
  static constexpr int kLds = kA2Off + 2 * kA2Elems * 2;  // 145,696 bytes (default) .. 160,800 (bits 16 | 32)
  static_assert(kLds <= 160 * 1024, "LDS per workgroup");
  // frame ring: the table of this workgroup's images' frame rows after the images (16 KB)
  static constexpr int kLdsTotal = kLds + (kRing ? kRingTab * 16 : 0);
  static_assert(kLdsTotal <= 160 * 1024, "LDS per workgroup with the frame-row table");
  static_assert(kA1Off % 16 == 0 && kA2Off % 16 == 0, "16-byte aligned LDS regions");
};
}  // namespace cs16

// The frame ring's load / store unit of thread tid in the 16-wave forward: position
// 32 (tid / 64) + tid % 32, rows 2h, 2h + 1 with h = (tid / 32) % 2 -- the two halves of a wave
// take the two row pairs of the same 32 positions, so each 16-byte LDS store instruction's lanes
// land 96 bytes apart in distinct bank groups (the pairing of adjacent lanes on one position put
// lanes 1 and 6 of every 8 on the same banks: 2-way conflicts in the store phase every barrier
// waits for); each load instruction still reads 512 contiguous bytes of a frame
__device__ __forceinline__ int ring_pos(int tid) { return 32 * (tid >> 6) + (tid & 31); }
__device__ __forceinline__ int ring_half(int tid) { return (tid >> 5) & 1; }

// chunk c of frame position r in the fused-render frame buffer (positions contiguous, 64 B each)
__device__ __forceinline__ int rfs_chunk(int r, int c) { return r * 64 + 16 * (c ^ (2 * ((r >> 2) & 1))); }

// A frame-history row every lane reads in full: loaded once per wave and kept in SGPRs
// (readfirstlane), so the fused render adds no vector registers to the conv waves.
__device__ __forceinline__ void uniform_row(const float* __restrict__ row, float (&hv)[kPongHist]) {
#pragma unroll
  for (int i = 0; i < kPongHist; i += 4) {
    const float4 v = *reinterpret_cast<const float4*>(row + i);
    hv[i] = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v.x)));
    hv[i + 1] = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v.y)));
    hv[i + 2] = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v.z)));
    hv[i + 3] = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, v.w)));
  }
}

__device__ __forceinline__ bf16x8_t u8x8_frag(uint32_t lo, uint32_t hi) {
  return __builtin_bit_cast(bf16x8_t, u8x8_to_bf16x8(make_uint2(lo, hi)));
}

struct Stack16Args {
  const uint8_t* x;
  const float* hist;  // fused render: [N][16] frame histories (x unused)
  const uint8_t* frames;  // frame ring: [R][E][7056] frame store and the frame rows fidx[N][4] (x unused)
  const int32_t* fidx;
  const uint16_t *w1, *w2, *w3;
  const float *b1, *b2, *b3;
  uint16_t *y1, *y2, *y3;
  int N;
};

// One role's whole loop (stationary weights, per-iteration stage), so each role's registers are
// allocated on their own; every role meets the same two barriers per iteration.
template <int ROLE, int V>
__device__ __forceinline__ void stack16_role(const Stack16Args& A, uint16_t* smem, int tid, int wave) {
  using namespace cs16;
  using L = L16<V>;
  constexpr int kA1Ld = L::kA1Ld, kA2Ld = L::kA2Ld, kA1Elems = L::kA1Elems, kA2Elems = L::kA2Elems;
  constexpr int kA1Off = L::kA1Off, kA2Off = L::kA2Off;
  uint8_t* F = reinterpret_cast<uint8_t*>(smem);
  const int lane = tid & 63, i = lane & 15, g = lane >> 4;
  const int ct = wave & 3;  // co tile of conv2 / conv3
  if constexpr (ROLE == 2 && L::kPrioRole2) __builtin_amdgcn_s_setprio(L::kPrioRole2);
  if constexpr (ROLE == 3 && L::kPrioRole3) __builtin_amdgcn_s_setprio(L::kPrioRole3);
  // stationary weights, A fragments W[co = 16 tile + i][8 consecutive k]:
  //   conv1 fw[8 c + 2 tap + h] = W1[16 c + i][64 tap + 16 g + 8 h ..]; conv2 / conv3 fw[ks] = W[..][32 ks + 8 g ..]
  constexpr int NF = ROLE == 3 ? 18 : 16;
  bf16x8_t fw[NF];
  f32x4_t bias0, bias1;
  if constexpr (ROLE == 1) {
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int ks = 0; ks < 8; ++ks)
        fw[8 * c + ks] = *reinterpret_cast<const bf16x8_t*>(A.w1 + (16 * c + i) * 256 + 64 * (ks >> 1) + 16 * g + 8 * (ks & 1));
    bias0 = *reinterpret_cast<const f32x4_t*>(A.b1 + 4 * g);
    bias1 = *reinterpret_cast<const f32x4_t*>(A.b1 + 16 + 4 * g);
  } else {
    const uint16_t* w = ROLE == 2 ? A.w2 : A.w3;
    constexpr int K = ROLE == 2 ? 512 : 576;
#pragma unroll
    for (int ks = 0; ks < NF; ++ks) fw[ks] = *reinterpret_cast<const bf16x8_t*>(w + (16 * ct + i) * K + 32 * ks + 8 * g);
    bias0 = bias1 = *reinterpret_cast<const f32x4_t*>((ROLE == 2 ? A.b2 : A.b3) + 16 * ct + 4 * g);
  }

  const int G = gridDim.x, n0 = blockIdx.x, N = A.N;
  uint4 rx[L::kRender ? 1 : (L::kRingWide ? (ROLE == 1 ? 4 : 1) : kXPerT)];
  static_assert(kXPerT >= 2, "the ring form keeps 4 x 8 raw bytes per thread in rx[0..1]");
  const int4* rtab = reinterpret_cast<const int4*>(reinterpret_cast<const uint8_t*>(smem) + L::kLds);
  // frame ring: unit tid < 882 loads position tid >> 1, rows 2 (tid & 1) .. + 1 of frames 0..3 (8
  // bytes each) of the image with frame rows fr, kept raw until the LDS store (the loads stay in
  // flight while this frame computes)
  auto gload_ring = [&](int4 fr) {
    if constexpr (L::kRingWide) {
      if constexpr (ROLE == 1) {
        if (tid < kPongFramePos) {  // position tid of frames 0..3
          const size_t off = (size_t)tid * 16;
          rx[0] = *reinterpret_cast<const uint4*>(A.frames + (size_t)fr.x * kPongFrameBytes + off);
          rx[1] = *reinterpret_cast<const uint4*>(A.frames + (size_t)fr.y * kPongFrameBytes + off);
          rx[2] = *reinterpret_cast<const uint4*>(A.frames + (size_t)fr.z * kPongFrameBytes + off);
          rx[3] = *reinterpret_cast<const uint4*>(A.frames + (size_t)fr.w * kPongFrameBytes + off);
        }
      }
    } else if constexpr (L::kRing16) {
      if (tid < 2 * kPongFramePos) {  // position tid >> 1, frames 2 fp and 2 fp + 1, all 4 rows
        const int fp = tid & 1;
        const size_t off = (size_t)(tid >> 1) * 16;
        const int ra = fp ? fr.z : fr.x, rb = fp ? fr.w : fr.y;
        rx[0] = *reinterpret_cast<const uint4*>(A.frames + (size_t)ra * kPongFrameBytes + off);
        rx[1] = *reinterpret_cast<const uint4*>(A.frames + (size_t)rb * kPongFrameBytes + off);
      }
    } else if constexpr (L::kRing) {
      if (ring_pos(tid) < kPongFramePos) {
        const size_t off = (size_t)ring_pos(tid) * 16 + 8 * ring_half(tid);
        const uint2 f0 = *reinterpret_cast<const uint2*>(A.frames + (size_t)fr.x * kPongFrameBytes + off);
        const uint2 f1 = *reinterpret_cast<const uint2*>(A.frames + (size_t)fr.y * kPongFrameBytes + off);
        const uint2 f2 = *reinterpret_cast<const uint2*>(A.frames + (size_t)fr.z * kPongFrameBytes + off);
        const uint2 f3 = *reinterpret_cast<const uint2*>(A.frames + (size_t)fr.w * kPongFrameBytes + off);
        rx[0] = make_uint4(f0.x, f0.y, f1.x, f1.y);
        rx[1] = make_uint4(f2.x, f2.y, f3.x, f3.y);
      }
    }
  };
  auto gload = [&](size_t n) {
    if constexpr (L::kRender || L::kRing) return;
    const uint4* xs = reinterpret_cast<const uint4*>(A.x + n * (441 * 64));
#pragma unroll
    for (int k = 0; k < kXPerT; ++k) {
      const int q = tid + kThreads * k;
      rx[k] = q < kXChunks ? xs[q] : make_uint4(0, 0, 0, 0);
    }
  };
  // fused render: the conv1 waves draw frame n into buffer b (the history row has a wave-uniform
  // address: its 16 floats go to SGPRs); they do it for frame n + G right after their conv1 of
  // frame n, beside the longer conv2 / conv3 work of the other waves, so the pipeline keeps ONE
  // barrier per iteration
  auto render = [&](int nn, int b) {
    float hv[kPongHist];
    uniform_row(A.hist + (size_t)nn * kPongHist, hv);
    uint8_t* Fb = F + b * L::kRFBytes;
    for (int q = tid; q < kXChunks; q += 512) *reinterpret_cast<uint4*>(Fb + rfs_chunk(q >> 2, q & 3)) = pong_render_chunk(hv, q);
  };
  if constexpr (L::kRender) {
    if (ROLE == 1 && n0 < N) render(n0, 0);
  }
  if constexpr (L::kRing) {
    // the first image's rows straight from fidx and its frame loads issued first; then this
    // workgroup's images' rows staged in LDS (first read, image 1's, after barrier B0) -- staged
    // before, the table's global loads and LDS stores sat in front of the first frame loads
    if (n0 < N) gload_ring(uniform_int4(*reinterpret_cast<const int4*>(A.fidx + 4 * (size_t)n0)));
    ring_stage_table(const_cast<int4*>(rtab), A.fidx, N, n0, G, tid, kThreads);
  } else if (n0 < N) {
    gload(n0);
  }
  for (int j = 0; n0 + (j - 2) * G < N; ++j) {
    const int n = n0 + j * G;
    __syncthreads();  // B0: the previous iteration's stages are done (F free, a1 / a2 buffers complete)
    if constexpr (L::kRender) {
      // (fused render: frame n is already in buffer j & 1)
    } else if constexpr (L::kRing) {
      if (n < N) {
        // the next image's frame rows: read from the table before this image's stores
        const int4 frn = n + G < N ? ring_row(rtab, A.fidx, n0, G, j + 1) : make_int4(0, 0, 0, 0);
        if constexpr (L::kRingWide) {
          if constexpr (ROLE == 1) {
            if (tid < kPongFramePos) {  // the 4 observation chunks (dy = 0..3) of position tid
              const int pa = tid / 21;
              uint8_t* d = F + (tid + (kFW - 21) * pa) * kFS;
              *reinterpret_cast<uint4*>(d) = pong_interleave_row(rx[0].x, rx[1].x, rx[2].x, rx[3].x);
              *reinterpret_cast<uint4*>(d + 16) = pong_interleave_row(rx[0].y, rx[1].y, rx[2].y, rx[3].y);
              *reinterpret_cast<uint4*>(d + 32) = pong_interleave_row(rx[0].z, rx[1].z, rx[2].z, rx[3].z);
              *reinterpret_cast<uint4*>(d + 48) = pong_interleave_row(rx[0].w, rx[1].w, rx[2].w, rx[3].w);
            }
          }
        } else if constexpr (L::kRing16) {
          if (tid < 2 * kPongFramePos) {
            // lane fp (of an adjacent pair) holds frames 2 fp, 2 fp + 1 and stores rows 2 fp, 2 fp + 1:
            // it keeps those rows of its frames and swaps the other two rows with its partner
            const int pix = tid >> 1, pa = pix / 21, fp = tid & 1;
            const uint32_t s0 = fp ? rx[0].x : rx[0].z, s1 = fp ? rx[0].y : rx[0].w;
            const uint32_t s2 = fp ? rx[1].x : rx[1].z, s3 = fp ? rx[1].y : rx[1].w;
            const uint32_t k0 = fp ? rx[0].z : rx[0].x, k1 = fp ? rx[0].w : rx[0].y;
            const uint32_t k2 = fp ? rx[1].z : rx[1].x, k3 = fp ? rx[1].w : rx[1].y;
            // quad_perm [1, 0, 3, 2]: each lane reads its pair partner
            const uint32_t r0 = (uint32_t)__builtin_amdgcn_mov_dpp((int)s0, 0xB1, 0xF, 0xF, false);
            const uint32_t r1 = (uint32_t)__builtin_amdgcn_mov_dpp((int)s1, 0xB1, 0xF, 0xF, false);
            const uint32_t r2 = (uint32_t)__builtin_amdgcn_mov_dpp((int)s2, 0xB1, 0xF, 0xF, false);
            const uint32_t r3 = (uint32_t)__builtin_amdgcn_mov_dpp((int)s3, 0xB1, 0xF, 0xF, false);
            uint8_t* d = F + (pix + (kFW - 21) * pa) * kFS + 32 * fp;
            *reinterpret_cast<uint4*>(d) = fp ? pong_interleave_row(r0, r2, k0, k2) : pong_interleave_row(k0, k2, r0, r2);
            *reinterpret_cast<uint4*>(d + 16) =
                fp ? pong_interleave_row(r1, r3, k1, k3) : pong_interleave_row(k1, k3, r1, r3);
          }
        } else if (ring_pos(tid) < kPongFramePos) {  // rows 2h, 2h + 1 of position pix, interleaved across the 4 frames
          const int pix = ring_pos(tid), pa = pix / 21, h = ring_half(tid);
          uint8_t* d = F + (pix + (kFW - 21) * pa) * kFS + 32 * h;
          *reinterpret_cast<uint4*>(d) = pong_interleave_row(rx[0].x, rx[0].z, rx[1].x, rx[1].z);
          *reinterpret_cast<uint4*>(d + 16) = pong_interleave_row(rx[0].y, rx[0].w, rx[1].y, rx[1].w);
        }
        if (n + G < N) gload_ring(frn);
      }
    } else if (n < N) {
#pragma unroll
      for (int k = 0; k < kXPerT; ++k) {
        const int q = tid + kThreads * k;
        if (q < kXChunks) {
          const int pix = q >> 2, pa = pix / 21;
          *reinterpret_cast<uint4*>(F + (pix + (kFW - 21) * pa) * kFS + (q & 3) * 16) = rx[k];
        }
      }
      if (n + G < N) gload((size_t)n + G);  // lands while this frame computes
    }
    if constexpr (!L::kRender) __syncthreads();  // B1: F holds frame n
    if constexpr (ROLE == 1) {
      // ---- conv1(n): pixel tiles wave + 8 t, one tile at a time, both co tiles
      if (n < N) {
        uint16_t* A1c = smem + kA1Off / 2 + (j & 1) * kA1Elems;
        const int ntile = wave == 0 ? 4 : 3;  // 25 tiles over 8 waves (wave-uniform)
        for (int t = 0; t < ntile; ++t) {
          const int p = 16 * (wave + 8 * t) + i;
          const uint8_t* src = F + ((p / 20) * kFW + p % 20) * kFS + 16 * g;
          const uint8_t* Fb = F + (j & 1) * L::kRFBytes;
          const int r0 = (p / 20) * 21 + p % 20;  // fused render: positions in rows of 21
          f32x4_t acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
          if constexpr (L::kSetprio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int tap = 0; tap < 4; ++tap) {
            uint4 raw;
            if constexpr (L::kRender)
              raw = *reinterpret_cast<const uint4*>(Fb + rfs_chunk(r0 + (tap >> 1) * 21 + (tap & 1), g));
            else
              raw = *reinterpret_cast<const uint4*>(src + ((tap >> 1) * kFW + (tap & 1)) * kFS);
            const bf16x8_t lo = u8x8_frag(raw.x, raw.y), hi = u8x8_frag(raw.z, raw.w);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[2 * tap], lo, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[8 + 2 * tap], lo, acc1, 0, 0, 0);
            acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[2 * tap + 1], hi, acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[8 + 2 * tap + 1], hi, acc1, 0, 0, 0);
          }
          if constexpr (L::kSetprio) __builtin_amdgcn_s_setprio(0);
          const uint2 v0 = make_uint2(pk_bf16(fmaxf(kU8Scale * acc0[0] + bias0[0], 0.f), fmaxf(kU8Scale * acc0[1] + bias0[1], 0.f)),
                                      pk_bf16(fmaxf(kU8Scale * acc0[2] + bias0[2], 0.f), fmaxf(kU8Scale * acc0[3] + bias0[3], 0.f)));
          const uint2 v1 = make_uint2(pk_bf16(fmaxf(kU8Scale * acc1[0] + bias1[0], 0.f), fmaxf(kU8Scale * acc1[1] + bias1[1], 0.f)),
                                      pk_bf16(fmaxf(kU8Scale * acc1[2] + bias1[2], 0.f), fmaxf(kU8Scale * acc1[3] + bias1[3], 0.f)));
          const int ar = L::kPhaseA1 ? cs::a1_row(p) : p;
          *reinterpret_cast<uint2*>(A1c + ar * kA1Ld + 4 * g) = v0;
          *reinterpret_cast<uint2*>(A1c + ar * kA1Ld + 16 + 4 * g) = v1;
          if (A.y1) {
            uint16_t* yd = A.y1 + ((size_t)n * 400 + p) * 32;
            *reinterpret_cast<uint2*>(yd + 4 * g) = v0;
            *reinterpret_cast<uint2*>(yd + 16 + 4 * g) = v1;
          }
        }
      }
      if constexpr (L::kRender) {
        if (n + G < N) render(n + G, (j + 1) & 1);
      }
    } else if constexpr (ROLE == 2) {
      // ---- conv2(n - G): co tile ct, 6 pixel tiles in passes (81 px; the rest discarded)
      if (j >= 1 && n - G < N) {
        const uint16_t* A1p = smem + kA1Off / 2 + ((j - 1) & 1) * kA1Elems;
        uint16_t* A2c = smem + kA2Off / 2 + ((j - 1) & 1) * kA2Elems;
        constexpr int MT = CS16_C2_MT;
#pragma unroll
        for (int pass = 0; pass < 6 / MT; ++pass) {
          f32x4_t acc[MT];
          int r0[MT];
#pragma unroll
          for (int u = 0; u < MT; ++u) {
            acc[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
            const int p = 16 * (MT * pass + u) + i, pc = p < 81 ? p : 0, oh = pc / 9, ow = pc - oh * 9;
            r0[u] = L::kPhaseA1 ? p : 2 * oh * 20 + 2 * ow;  // phase: grid position 10 oh + ow = row of tap (0, 0)
          }
          if constexpr (L::kSetprio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int ks = 0; ks < 16; ++ks) {
            const int kh = ks >> 2, kw = ks & 3;
            const int off = (L::kPhaseA1 ? 100 * (2 * (kh & 1) + (kw & 1)) + 10 * (kh >> 1) + (kw >> 1) : kh * 20 + kw) * kA1Ld + 8 * g;
            bf16x8_t a[MT];
#pragma unroll
            for (int u = 0; u < MT; ++u) a[u] = *reinterpret_cast<const bf16x8_t*>(A1p + r0[u] * kA1Ld + off);
#pragma unroll
            for (int u = 0; u < MT; ++u) acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[ks], a[u], acc[u], 0, 0, 0);
          }
          if constexpr (L::kSetprio) __builtin_amdgcn_s_setprio(0);
#pragma unroll
          for (int u = 0; u < MT; ++u) {
            const int p = 16 * (MT * pass + u) + i, oh = p / 10, ow = p - 10 * (p / 10);
            if (L::kPhaseA1 ? (p < 90 && ow < 9) : p < 81) {
              const int q = L::kPhaseA1 ? 9 * oh + ow : p;
              const uint2 v = make_uint2(pk_bf16(fmaxf(acc[u][0] + bias0[0], 0.f), fmaxf(acc[u][1] + bias0[1], 0.f)),
                                         pk_bf16(fmaxf(acc[u][2] + bias0[2], 0.f), fmaxf(acc[u][3] + bias0[3], 0.f)));
              *reinterpret_cast<uint2*>(A2c + q * kA2Ld + 16 * ct + 4 * g) = v;
              if (A.y2) *reinterpret_cast<uint2*>(A.y2 + ((size_t)(n - G) * 81 + q) * 64 + 16 * ct + 4 * g) = v;
            }
          }
        }
      }
    } else {
      // ---- conv3(n - 2G): co tile ct, 4 pixel tiles in passes (49 px), straight to HBM
      if (j >= 2 && n - 2 * G < N) {
        const uint16_t* A2p = smem + kA2Off / 2 + ((j - 2) & 1) * kA2Elems;
        constexpr int MT = CS16_C3_MT;
#pragma unroll
        for (int pass = 0; pass < 4 / MT; ++pass) {
          f32x4_t acc[MT];
          int r0[MT];
#pragma unroll
          for (int u = 0; u < MT; ++u) {
            acc[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
            const int p = 16 * (MT * pass + u) + i, pc = p < 49 ? p : 0, oh = pc / 7, ow = pc - oh * 7;
            r0[u] = L::kGrid3 ? p : oh * 9 + ow;  // grid: position 9 oh + ow = the a2 row of tap (0, 0)
          }
          if constexpr (L::kSetprio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int ks = 0; ks < 18; ++ks) {
            const int tap = ks >> 1, kh = tap / 3, kw = tap - kh * 3;
            const int off = (kh * 9 + kw) * kA2Ld + 32 * (ks & 1) + 8 * g;
            bf16x8_t a[MT];
#pragma unroll
            for (int u = 0; u < MT; ++u) a[u] = *reinterpret_cast<const bf16x8_t*>(A2p + r0[u] * kA2Ld + off);
#pragma unroll
            for (int u = 0; u < MT; ++u) acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[ks], a[u], acc[u], 0, 0, 0);
          }
          if constexpr (L::kSetprio) __builtin_amdgcn_s_setprio(0);
#pragma unroll
          for (int u = 0; u < MT; ++u) {
            const int p = 16 * (MT * pass + u) + i, oh = p / 9, ow = p - 9 * (p / 9);
            if (L::kGrid3 ? (oh < 7 && ow < 7) : p < 49) {
              const int q = L::kGrid3 ? 7 * oh + ow : p;
              const uint2 v = make_uint2(pk_bf16(fmaxf(acc[u][0] + bias0[0], 0.f), fmaxf(acc[u][1] + bias0[1], 0.f)),
                                         pk_bf16(fmaxf(acc[u][2] + bias0[2], 0.f), fmaxf(acc[u][3] + bias0[3], 0.f)));
              *reinterpret_cast<uint2*>(A.y3 + ((size_t)(n - 2 * G) * 49 + q) * 64 + 16 * ct + 4 * g) = v;
            }
          }
        }
      }
    }
  }
}

template <int V>
__global__ __launch_bounds__(cs16::kThreads, 1) void conv_stack16_fwd_kernel(Stack16Args args) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (wave < 8) stack16_role<1, V>(args, smem, tid, wave);
  else if (wave < 12) stack16_role<2, V>(args, smem, tid, wave);
  else stack16_role<3, V>(args, smem, tid, wave);
}

}  // namespace rrl

using namespace rrl;

template <int PROBE>
static int launch_conv_stack_fwd(const uint8_t* x, const uint16_t* w1, const float* b1, const uint16_t* w2,
                                 const float* b2, const uint16_t* w3, const float* b3, uint16_t* y1, uint16_t* y2,
                                 uint16_t* y3, int N, int max_grid, hipStream_t stream) {
  using L = cs::FwdLayout<PROBE>;
  constexpr int lds = (L::kA3 + 49 * L::kA3Ld) * 2;  // 159,200 bytes for the shipped layout
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv_stack_fwd_kernel<PROBE>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              lds);
    attr = true;
  }
  if (N < 1) return 0;
  const int grid = N < max_grid ? N : max_grid;  // one 155 KB-LDS workgroup per CU
  hipLaunchKernelGGL(conv_stack_fwd_kernel<PROBE>, dim3(grid), dim3(cs::kThreads), lds, stream, x, w1, b1, w2,
                     b2, w3, b3, y1, y2, y3, N);
  return (int)hipGetLastError();
}

template <int V>
static int launch_conv_stack16_fwd(const uint8_t* x, const float* hist, const uint16_t* w1, const float* b1,
                                   const uint16_t* w2, const float* b2, const uint16_t* w3, const float* b3,
                                   uint16_t* y1, uint16_t* y2, uint16_t* y3, int N, int max_grid, hipStream_t stream,
                                   const uint8_t* frames = nullptr, const int32_t* fidx = nullptr) {
  using L = cs16::L16<V>;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv_stack16_fwd_kernel<V>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    attr = true;
  }
  if (N < 1) return 0;
  const int grid = N < max_grid ? N : max_grid;  // one 146-161 KB-LDS workgroup per CU
  const int lds = L::kLdsTotal;
  if (L::kRender && !hist) return -2;
  if (L::kRing && (!frames || !fidx)) return -2;
  const Stack16Args args{x, hist, frames, fidx, w1, w2, w3, b1, b2, b3, y1, y2, y3, N};
  hipLaunchKernelGGL(conv_stack16_fwd_kernel<V>, dim3(grid), dim3(cs16::kThreads), lds, stream, args);
  return (int)hipGetLastError();
}

// RRL_CONV_FWD = 8 / 16 picks the 8-wave or the 16-wave kernel; default 16 (Pong A2C +2.3 % at
// 2,048 envs, +3.4 % at 8,192 in ABBA runs: profiles/r5_pong_16wave_ab_*.jsonl)
static bool conv_fwd16() {
  static int v = -1;
  if (v < 0) {
    const char* e = getenv("RRL_CONV_FWD");
    v = (e && e[0]) ? (atoi(e) == 16) : 1;
  }
  return v == 1;
}

extern "C" int rrl_conv_stack_fwd(const uint8_t* x, const float* hist, const uint8_t* frames, const int32_t* fidx,
                                  const uint16_t* w1, const float* b1,
                                  const uint16_t* w2, const float* b2, const uint16_t* w3, const float* b3,
                                  uint16_t* y1, uint16_t* y2, uint16_t* y3, int N, int max_grid, void* stream) {
  // max_grid < 0: timing probe variant -max_grid >> 16 (tools/cnn_kbench.py), grid = -max_grid & 0xffff;
  // probe 64 (+ 16 / 32 / 48: its layout bits) = the 16-wave kernel, probe 128 = the 8-wave kernel
  // (whatever RRL_CONV_FWD says).  hist (PongSynth frame histories [N][16]): the 16-wave kernel
  // draws the frames itself (fused render), x is not read.
  hipStream_t st = (hipStream_t)stream;
  if (frames) {  // frame ring (frames [R][E][7056] + fidx [N][4]): the default 16-wave layout only
    const int g = max_grid >= 0 ? max_grid : ((-max_grid) & 0xffff);
    const int probe = max_grid >= 0 ? 64 : ((-max_grid) >> 16);
    if (probe == 64 + 256)  // the conv1-waves-only, 1 KB-per-load form (A/B)
      return launch_conv_stack16_fwd<64 + 256>(nullptr, nullptr, w1, b1, w2, b2, w3, b3, y1, y2, y3, N, g, st, frames, fidx);
    if (probe == 64 + 128)  // the 16-byte-load + DPP form (A/B)
      return launch_conv_stack16_fwd<64 + 128>(nullptr, nullptr, w1, b1, w2, b2, w3, b3, y1, y2, y3, N, g, st, frames, fidx);
    if (probe != 64) return -4;
    return launch_conv_stack16_fwd<64>(nullptr, nullptr, w1, b1, w2, b2, w3, b3, y1, y2, y3, N, g, st, frames, fidx);
  }
  if (hist) {
    const int g = max_grid >= 0 ? max_grid : ((-max_grid) & 0xffff);
    const int probe = max_grid >= 0 ? 64 : ((-max_grid) >> 16);
    if (probe != 64) return -4;  // the fused render exists for the default 16-wave layout only
    return launch_conv_stack16_fwd<2>(x, hist, w1, b1, w2, b2, w3, b3, y1, y2, y3, N, g, st);
  }
  if (max_grid >= 0) {
    if (conv_fwd16()) return launch_conv_stack16_fwd<0>(x, nullptr, w1, b1, w2, b2, w3, b3, y1, y2, y3, N, max_grid, st);
    return launch_conv_stack_fwd<0>(x, w1, b1, w2, b2, w3, b3, y1, y2, y3, N, max_grid, st);
  }
  const int probe = (-max_grid) >> 16, g = (-max_grid) & 0xffff;
  switch (probe) {
    case 64: return launch_conv_stack16_fwd<0>(x, nullptr, w1, b1, w2, b2, w3, b3, y1, y2, y3, N, g, st);
    case 64 + 16: return launch_conv_stack16_fwd<16>(x, nullptr, w1, b1, w2, b2, w3, b3, y1, y2, y3, N, g, st);
    case 64 + 32: return launch_conv_stack16_fwd<32>(x, nullptr, w1, b1, w2, b2, w3, b3, y1, y2, y3, N, g, st);
    case 64 + 48: return launch_conv_stack16_fwd<48>(x, nullptr, w1, b1, w2, b2, w3, b3, y1, y2, y3, N, g, st);
    case 64 + 4: return launch_conv_stack16_fwd<4>(x, nullptr, w1, b1, w2, b2, w3, b3, y1, y2, y3, N, g, st);
    case 64 + 1: return launch_conv_stack16_fwd<1>(x, nullptr, w1, b1, w2, b2, w3, b3, y1, y2, y3, N, g, st);
    case 64 + 8: return launch_conv_stack16_fwd<8>(x, nullptr, w1, b1, w2, b2, w3, b3, y1, y2, y3, N, g, st);
    case 64 + 9: return launch_conv_stack16_fwd<9>(x, nullptr, w1, b1, w2, b2, w3, b3, y1, y2, y3, N, g, st);
    case 128: return launch_conv_stack_fwd<0>(x, w1, b1, w2, b2, w3, b3, y1, y2, y3, N, g, st);
    case 1: return launch_conv_stack_fwd<1>(x, w1, b1, w2, b2, w3, b3, y1, y2, y3, N, g, st);
    case 2: return launch_conv_stack_fwd<2>(x, w1, b1, w2, b2, w3, b3, y1, y2, y3, N, g, st);
    case 3: return launch_conv_stack_fwd<3>(x, w1, b1, w2, b2, w3, b3, y1, y2, y3, N, g, st);
    case 4: return launch_conv_stack_fwd<4>(x, w1, b1, w2, b2, w3, b3, y1, y2, y3, N, g, st);
    case 7: return launch_conv_stack_fwd<7>(x, w1, b1, w2, b2, w3, b3, y1, y2, y3, N, g, st);
    case 8: return launch_conv_stack_fwd<8>(x, w1, b1, w2, b2, w3, b3, y1, y2, y3, N, g, st);
    case 16: return launch_conv_stack_fwd<16>(x, w1, b1, w2, b2, w3, b3, y1, y2, y3, N, g, st);
    case 32: return launch_conv_stack_fwd<32>(x, w1, b1, w2, b2, w3, b3, y1, y2, y3, N, g, st);
    case 48: return launch_conv_stack_fwd<48>(x, w1, b1, w2, b2, w3, b3, y1, y2, y3, N, g, st);
    default: return launch_conv_stack_fwd<0>(x, w1, b1, w2, b2, w3, b3, y1, y2, y3, N, g, st);
  }
}

// ============================================================================= conv3 backward
// dgrad + wgrad + bias gradient of the third conv layer (9x9x64 -> 3x3/1 -> 7x7x64) in ONE
// pass per image.  Both halves read the same two inputs -- the output gradient da3 [49][64]
// and the input activation a2 [81][64] (also the ReLU mask of da2) -- so each is fetched
// from HBM once instead of once per GEMM (the split-K implicit-GEMM wgrad + its partial
// sums, the column-sum bias pass and conv3_dgrad_kernel in cnn.hip), and the weight
// gradient accumulates in registers across all of a workgroup's images: one fp32 partial
// per workgroup instead of one per split-K slice.
//
// LDS, two buffers (image j computes from buffer j & 1 while image j + 1, prefetched into
// registers one iteration earlier, is written into the other and image j + 2's loads are in
// flight: ONE barrier per image, as conv2_bwd_kernel): da3 in a zero-bordered 11x11 image (row
// (oh + 2) * 11 + ow + 2), a2 as a 9 x 9 image in rows of 12 positions (ih * 12 + iw; pad
// columns and rows zero, so an 8-position run of one lane group and the next group's run land
// on disjoint banks: the wgrad transposed reads 2.0 -> 1.0 LDS cycles per conflict-free cycle
// in tools/lds_bank_model.py), rows of 64 channels + 16 pad.  (The single-buffered form with
// 72-element rows, three barriers per image and the dgrad tile staged through LDS spent 59 %
// of its wave cycles parked, SQ_WAIT_ANY, and 58 % of its LDS cycles on bank conflicts:
// profiles/r4_cnn_pmc.txt.  A chunk-swizzled da3 image cut the conflicts a further 84 % but
// its per-read address arithmetic doubled the VALU work and the kernel did not speed up:
// profiles/r4_cnn_swizzle_ab.txt.)
namespace c3b {
constexpr int kThreads = 512;
#ifndef C3B_LD
#define C3B_LD 80
#endif
constexpr int kLd = C3B_LD;
constexpr int kD = 0;                        // da3 bordered [121][kLd]
constexpr int kXW = 12;                      // a2 positions per LDS image row
constexpr int kX = kD + 121 * kLd;           // a2 [120][kLd]: (ih, iw) at ih * 12 + iw
constexpr int kBuf = kX + 120 * kLd;         // elements per buffer
constexpr int kLds = 2 * kBuf * 2;           // 74,880 bytes at kLd = 80
constexpr int kYC = 49 * 8, kXC = 81 * 8;  // 16-byte chunks per image
constexpr int kYPT = (kYC + kThreads - 1) / kThreads, kXPT = (kXC + kThreads - 1) / kThreads;
static_assert(kBuf % 8 == 0, "16-byte aligned buffers");
}  // namespace c3b

__device__ __forceinline__ bf16x8_t tr_frag(const uint16_t* a0, int ld) {
  typedef __attribute__((address_space(3))) s16x4_t lds_v4;
  s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(a0));
  s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(a0 + 4 * ld));
  typedef short s16x8_t __attribute__((ext_vector_type(8)));
  s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

// SP (wave priority): 1 = s_setprio 1 around each MFMA cluster (cdna_hip_programming.md T5: keeps
// the compiler from moving MFMAs across the clusters' boundaries; also the form without the 8-byte
// per-image spill reload of SP 0) -- the shipped kernel; 0 = without; 2 = the static form, waves
// 4-7 (the younger half) at priority 1 for the whole kernel
template <int SP = 0>
__global__ __launch_bounds__(c3b::kThreads, 1) void conv3_bwd_kernel(const uint16_t* __restrict__ dy,
                                                                     const uint16_t* __restrict__ w,
                                                                     const uint16_t* __restrict__ xact,
                                                                     uint16_t* __restrict__ dx,
                                                                     float* __restrict__ part,
                                                                     float* __restrict__ bias_part, int N) {
  using namespace c3b;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i16 = lane & 15, g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  const int ct = wave & 3, half = wave >> 2;

  // dgrad B fragments: k-step ks = (tap t = ks >> 1, co block (ks & 1) * 32):
  // W3[co0 + 8g + e][t][16 ct + i16], e = 0..7
  bf16x8_t wf[18];
#pragma unroll
  for (int ks = 0; ks < 18; ++ks) {
    const int t = ks >> 1, co0 = (ks & 1) * 32 + 8 * g;
    typedef short s16x8_t __attribute__((ext_vector_type(8)));
    s16x8_t v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (short)w[((co0 + e) * 9 + t) * 64 + 16 * ct + i16];
    wf[ks] = __builtin_bit_cast(bf16x8_t, v);
  }
  // zero both buffers once: the da3 border and the a2 pad rows are never rewritten
  for (int q = tid; q < 2 * kBuf / 8; q += kThreads) *reinterpret_cast<uint4*>(smem + 8 * q) = make_uint4(0, 0, 0, 0);

  constexpr int NTAP = 5;  // taps of this wave's wgrad k tiles (4 on the second half)
  const int tap0 = half * 5, ntap = half ? 4 : 5;
  f32x4_t wacc[4][NTAP];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int t = 0; t < NTAP; ++t) wacc[c][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;  // db3[tid & 63] over positions (tid >> 6) + 8 k

  uint4 ry[kYPT], rx[kXPT];
  auto gload = [&](int n) {
    const uint4* ys = reinterpret_cast<const uint4*>(dy + (size_t)n * 49 * 64);
    const uint4* xs = reinterpret_cast<const uint4*>(xact + (size_t)n * 81 * 64);
#pragma unroll
    for (int k = 0; k < kYPT; ++k) {
      const int q = tid + kThreads * k;
      ry[k] = q < kYC ? ys[q] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < kXPT; ++k) {
      const int q = tid + kThreads * k;
      rx[k] = q < kXC ? xs[q] : make_uint4(0, 0, 0, 0);
    }
  };
  auto lstore = [&](int buf) {
    uint16_t* Y = smem + buf * kBuf + kD;
    uint16_t* X = smem + buf * kBuf + kX;
#pragma unroll
    for (int k = 0; k < kYPT; ++k) {
      const int q = tid + kThreads * k;
      if (q < kYC) {
        const int pix = q >> 3, oh = pix / 7, ow = pix - oh * 7;
        *reinterpret_cast<uint4*>(Y + ((oh + 2) * 11 + ow + 2) * kLd + (q & 7) * 8) = ry[k];
      }
    }
#pragma unroll
    for (int k = 0; k < kXPT; ++k) {
      const int q = tid + kThreads * k;
      if (q < kXC) {
        const int pix = q >> 3, ih = pix / 9, iw = pix - ih * 9;
        *reinterpret_cast<uint4*>(X + (ih * kXW + iw) * kLd + (q & 7) * 8) = rx[k];
      }
    }
  };

  const int G = gridDim.x, n0 = blockIdx.x;
  __syncthreads();  // zeroing done before the first image lands in buffer 0
  if (n0 < N) {
    gload(n0);
    lstore(0);
  }
  if (n0 + G < N) gload(n0 + G);
  if constexpr (SP == 2) {
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);
  }
  for (int j = 0; n0 + j * G < N; ++j) {
    const int n = n0 + j * G;
    __syncthreads();  // buffer j & 1 holds image n; buffer (j + 1) & 1 is no longer read
    if (n + G < N) {
      lstore((j + 1) & 1);
      if (n + 2 * G < N) gload(n + 2 * G);
    }
    const uint16_t* Yi = smem + (j & 1) * kBuf + kD;
    const uint16_t* Xi = smem + (j & 1) * kBuf + kX;

    // ---- wgrad: 2 position k-steps x (4 co tiles x ntap taps)
    if constexpr (SP == 1 || SP == 3) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const int oh = 4 * s + g;  // this lane group's output row (7 = zero border)
      bf16x8_t af[4], bfr[NTAP];
#pragma unroll
      for (int c = 0; c < 4; ++c) af[c] = tr_frag(Yi + ((oh + 2) * 11 + 2 + q4) * kLd + 16 * c + 4 * p4, kLd);
#pragma unroll
      for (int t = 0; t < NTAP; ++t) {
        const int tap = min(tap0 + t, 8), kh = tap / 3, kw = tap - kh * 3;
        bfr[t] = tr_frag(Xi + ((oh + kh) * kXW + kw + q4) * kLd + 16 * ct + 4 * p4, kLd);
      }
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int t = 0; t < NTAP; ++t) wacc[c][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[c], bfr[t], wacc[c][t], 0, 0, 0);
    }
    if constexpr (SP == 1 || SP == 3) __builtin_amdgcn_s_setprio(0);
    // ---- dgrad: k-step outer, this wave's 3 pixel tiles inner
    {
      f32x4_t acc[3];
      int rb[3];
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        acc[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        const int p = 16 * (3 * half + u) + i16;
        const int pc = p < 81 ? p : 0;
        const int ih = pc / 9, iw = pc - ih * 9;
        rb[u] = (ih + 2) * 11 + (iw + 2);
      }
      if constexpr (SP == 1 || SP == 4) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 18; ++ks) {
        const int t = ks >> 1, kh = t / 3, kw = t - kh * 3;
        const int off = -(kh * 11 + kw) * kLd + (ks & 1) * 32 + 8 * g;
        bf16x8_t a[3];
#pragma unroll
        for (int u = 0; u < 3; ++u) a[u] = *reinterpret_cast<const bf16x8_t*>(Yi + rb[u] * kLd + off);
#pragma unroll
        for (int u = 0; u < 3; ++u) acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ks], a[u], acc[u], 0, 0, 0);
      }
      if constexpr (SP == 1 || SP == 4) __builtin_amdgcn_s_setprio(0);
      // D = da2^T: lane (i16, g) holds channels 16 ct + 4g .. + 3 of pixel q, masked by a2 > 0
#pragma unroll
      for (int u = 0; u < 3; ++u) {
        const int q = 16 * (3 * half + u) + i16;
        if (q < 81) {
          const uint2 m = *reinterpret_cast<const uint2*>(Xi + ((q / 9) * kXW + q % 9) * kLd + 16 * ct + 4 * g);
          *reinterpret_cast<uint2*>(dx + ((size_t)n * 81 + q) * 64 + 16 * ct + 4 * g) =
              make_uint2(relu_mask2(pk_bf16(acc[u][0], acc[u][1]), m.x), relu_mask2(pk_bf16(acc[u][2], acc[u][3]), m.y));
        }
      }
    }
    // ---- db3
    for (int pos = tid >> 6; pos < 49; pos += 8) {
      const int oh = pos / 7, ow = pos - oh * 7;
      bsum += bf2f(Yi[((oh + 2) * 11 + ow + 2) * kLd + (tid & 63)]);
    }
  }
  // this workgroup's weight-gradient partial: part[blk][co][tap][c]
  float* o = part + (size_t)blockIdx.x * 64 * 576;
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int t = 0; t < NTAP; ++t)
      if (t < ntap) {
#pragma unroll
        for (int r = 0; r < 4; ++r) o[(16 * c + 4 * g + r) * 576 + (tap0 + t) * 64 + 16 * ct + i16] = wacc[c][t][r];
      }
  // the bias partial folded over the 8 waves in LDS: 64 values per workgroup (the end-of-backward
  // slab sum's bias segments had 8 x the splits and were its longest blocks)
  __syncthreads();  // every wave is past its last LDS read of the image buffers
  float* red = reinterpret_cast<float*>(smem);
  red[tid] = bsum;
  __syncthreads();
  if (tid < 64) {
    float sb = 0.f;
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) sb += red[w * 64 + tid];
    bias_part[(size_t)blockIdx.x * 64 + tid] = sb;
  }
}

// 16-wave form of conv3_bwd_kernel (the conv2_bwd16_kernel split): waves 0-7 the dgrad (co tile
// w & 3, pixel tiles 3 (w >> 2) ..: W3 fragments, and they stage the next image), waves 8-15 the
// wgrad (c tile w & 3, taps 5 ((w - 8) >> 2) ..: the 20 weight-gradient accumulators).  Same LDS
// images, k-orders and partial layout as conv3_bwd_kernel: its outputs bitwise.
#ifndef C3B16_MT
#define C3B16_MT 3
#endif
#ifndef C3B16_SCHED
#define C3B16_SCHED 0
#endif
namespace c3b16 {
constexpr int kThreads = 1024;
constexpr int kStage = 512;
constexpr int kYPT = (c3b::kYC + kStage - 1) / kStage, kXPT = (c3b::kXC + kStage - 1) / kStage;
}  // namespace c3b16

template <int ROLE, int SP = 0>  // 0 = dgrad, 1 = wgrad; SP 1: s_setprio around the MFMA clusters
__device__ __forceinline__ void conv3_bwd16_role(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ w,
                                                 const uint16_t* __restrict__ xact, uint16_t* __restrict__ dx,
                                                 float* __restrict__ part, float* __restrict__ bias_part, int N,
                                                 uint16_t* smem, int tid, int wave) {
  using namespace c3b;
  constexpr int T = c3b16::kStage;
  const int lane = tid & 63;
  const int ct = wave & 3, half = (wave >> 2) & 1;
  bf16x8_t wf[ROLE == 0 ? 18 : 1];
  constexpr int NTAP = 5;
  const int tap0 = half * 5, ntap = half ? 4 : 5;
  f32x4_t wacc[ROLE == 1 ? 4 : 1][NTAP];
  if constexpr (ROLE == 0) {
    const int i16 = lane & 15, g = lane >> 4;
#pragma unroll
    for (int ks = 0; ks < 18; ++ks) {
      const int t = ks >> 1, co0 = (ks & 1) * 32 + 8 * g;
      typedef short s16x8_t __attribute__((ext_vector_type(8)));
      s16x8_t v;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (short)w[((co0 + e) * 9 + t) * 64 + 16 * ct + i16];
      wf[ks] = __builtin_bit_cast(bf16x8_t, v);
      __builtin_amdgcn_sched_barrier(0);  // one fragment's 8 loads at a time (all 144 at once spill)
    }
  } else {
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int t = 0; t < NTAP; ++t) wacc[c][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }
  for (int q = tid; q < 2 * kBuf / 8; q += c3b16::kThreads) *reinterpret_cast<uint4*>(smem + 8 * q) = make_uint4(0, 0, 0, 0);
  float bsum = 0.f;  // dgrad waves: db3[tid & 63] over positions (tid >> 6) + 8 k

  int tv = tid;  // behind an empty asm each iteration: addresses recomputed, not hoisted into registers
  uint4 ry[ROLE == 0 ? c3b16::kYPT : 1], rx[ROLE == 0 ? c3b16::kXPT : 1];
  auto gload = [&](int n) {
    if constexpr (ROLE == 1) return;
    const uint4* ys = reinterpret_cast<const uint4*>(dy + (size_t)n * 49 * 64);
    const uint4* xs = reinterpret_cast<const uint4*>(xact + (size_t)n * 81 * 64);
#pragma unroll
    for (int k = 0; k < c3b16::kYPT; ++k) {
      const int q = tv + T * k;
      ry[k] = q < kYC ? ys[q] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < c3b16::kXPT; ++k) {
      const int q = tv + T * k;
      rx[k] = q < kXC ? xs[q] : make_uint4(0, 0, 0, 0);
    }
  };
  auto lstore = [&](int buf) {
    if constexpr (ROLE == 1) return;
    uint16_t* Y = smem + buf * kBuf + kD;
    uint16_t* X = smem + buf * kBuf + kX;
#pragma unroll
    for (int k = 0; k < c3b16::kYPT; ++k) {
      const int q = tv + T * k;
      if (q < kYC) {
        const int pix = q >> 3, oh = pix / 7, ow = pix - oh * 7;
        *reinterpret_cast<uint4*>(Y + ((oh + 2) * 11 + ow + 2) * kLd + (q & 7) * 8) = ry[k];
      }
    }
#pragma unroll
    for (int k = 0; k < c3b16::kXPT; ++k) {
      const int q = tv + T * k;
      if (q < kXC) {
        const int pix = q >> 3, ih = pix / 9, iw = pix - ih * 9;
        *reinterpret_cast<uint4*>(X + (ih * kXW + iw) * kLd + (q & 7) * 8) = rx[k];
      }
    }
  };

  const int G = gridDim.x, n0 = blockIdx.x;
  __syncthreads();  // zeroing done before the first image lands in buffer 0
  if (n0 < N) {
    gload(n0);
    lstore(0);
  }
  if (n0 + G < N) gload(n0 + G);
  for (int j = 0; n0 + j * G < N; ++j) {
    const int n = n0 + j * G;
    __syncthreads();  // buffer j & 1 holds image n; buffer (j + 1) & 1 is no longer read
    asm volatile("" : "+v"(tv));
    const int i16 = tv & 15, g = (tv >> 4) & 3, q4 = (tv >> 2) & 3, p4 = tv & 3;
    if (n + G < N) {
      lstore((j + 1) & 1);
      if (n + 2 * G < N) gload(n + 2 * G);
    }
    const uint16_t* Yi = smem + (j & 1) * kBuf + kD;
    const uint16_t* Xi = smem + (j & 1) * kBuf + kX;
    if constexpr (ROLE == 1) {
      // ---- wgrad: 2 position k-steps x (4 co tiles x ntap taps)
      if constexpr (SP == 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int oh = 4 * s + g;  // this lane group's output row (7 = zero border)
        bf16x8_t af[4], bfr[NTAP];
#pragma unroll
        for (int c = 0; c < 4; ++c) af[c] = tr_frag(Yi + ((oh + 2) * 11 + 2 + q4) * kLd + 16 * c + 4 * p4, kLd);
#pragma unroll
        for (int t = 0; t < NTAP; ++t) {
          const int tap = min(tap0 + t, 8), kh = tap / 3, kw = tap - kh * 3;
          bfr[t] = tr_frag(Xi + ((oh + kh) * kXW + kw + q4) * kLd + 16 * ct + 4 * p4, kLd);
        }
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int t = 0; t < NTAP; ++t) wacc[c][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[c], bfr[t], wacc[c][t], 0, 0, 0);
      }
      if constexpr (SP == 1) __builtin_amdgcn_s_setprio(0);
    } else {
      // ---- dgrad: this wave's 3 pixel tiles, C3B16_MT at a time (k-step outer, tiles inner)
      auto tiles = [&](auto tag) {
        constexpr int U0 = decltype(tag)::value, MT = U0 + C3B16_MT <= 3 ? C3B16_MT : 3 - U0;
        f32x4_t acc[MT];
        int rb[MT];
#pragma unroll
        for (int u = 0; u < MT; ++u) {
          acc[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
          const int p = 16 * (3 * half + U0 + u) + i16;
          const int pc = p < 81 ? p : 0;
          const int ih = pc / 9, iw = pc - ih * 9;
          rb[u] = (ih + 2) * 11 + (iw + 2);
        }
        if constexpr (SP == 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int ks = 0; ks < 18; ++ks) {
          const int t = ks >> 1, kh = t / 3, kw = t - kh * 3;
          const int off = -(kh * 11 + kw) * kLd + (ks & 1) * 32 + 8 * g;
          bf16x8_t a[MT];
#pragma unroll
          for (int u = 0; u < MT; ++u) a[u] = *reinterpret_cast<const bf16x8_t*>(Yi + rb[u] * kLd + off);
#pragma unroll
          for (int u = 0; u < MT; ++u) acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ks], a[u], acc[u], 0, 0, 0);
          if (C3B16_SCHED && (ks % C3B16_SCHED) == C3B16_SCHED - 1) __builtin_amdgcn_sched_barrier(0);  // bound the reads in flight
        }
        if constexpr (SP == 1) __builtin_amdgcn_s_setprio(0);
#pragma unroll
        for (int u = 0; u < MT; ++u) {
          const int q = 16 * (3 * half + U0 + u) + i16;
          if (q < 81) {
            const uint2 m = *reinterpret_cast<const uint2*>(Xi + ((q / 9) * kXW + q % 9) * kLd + 16 * ct + 4 * g);
            *reinterpret_cast<uint2*>(dx + ((size_t)n * 81 + q) * 64 + 16 * ct + 4 * g) =
                make_uint2(relu_mask2(pk_bf16(acc[u][0], acc[u][1]), m.x), relu_mask2(pk_bf16(acc[u][2], acc[u][3]), m.y));
          }
        }
      };
      tiles(std::integral_constant<int, 0>{});
      if constexpr (C3B16_MT < 3) tiles(std::integral_constant<int, C3B16_MT>{});
      if constexpr (C3B16_MT == 1) tiles(std::integral_constant<int, 2>{});
      // ---- db3
      for (int pos = tid >> 6; pos < 49; pos += 8) {
        const int oh = pos / 7, ow = pos - oh * 7;
        bsum += bf2f(Yi[((oh + 2) * 11 + ow + 2) * kLd + (tid & 63)]);
      }
    }
  }
  if constexpr (ROLE == 1) {  // this workgroup's weight-gradient partial: part[blk][co][tap][c]
    const int i16 = lane & 15, g = lane >> 4;
    float* o = part + (size_t)blockIdx.x * 64 * 576;
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int t = 0; t < NTAP; ++t)
        if (t < ntap) {
#pragma unroll
          for (int r = 0; r < 4; ++r) o[(16 * c + 4 * g + r) * 576 + (tap0 + t) * 64 + 16 * ct + i16] = wacc[c][t][r];
        }
  }
  __syncthreads();  // every wave is past its last LDS read of the image buffers
  float* red = reinterpret_cast<float*>(smem);
  if (ROLE == 0) red[tid] = bsum;
  __syncthreads();
  if (tid < 64) {
    float sb = 0.f;
#pragma unroll
    for (int w8 = 0; w8 < 8; ++w8) sb += red[w8 * 64 + tid];
    bias_part[(size_t)blockIdx.x * 64 + tid] = sb;
  }
}

template <int SP = 0>
__global__ __launch_bounds__(c3b16::kThreads, 1) void conv3_bwd16_kernel(const uint16_t* __restrict__ dy,
                                                                         const uint16_t* __restrict__ w,
                                                                         const uint16_t* __restrict__ xact,
                                                                         uint16_t* __restrict__ dx,
                                                                         float* __restrict__ part,
                                                                         float* __restrict__ bias_part, int N) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (wave < 8) conv3_bwd16_role<0, SP>(dy, w, xact, dx, part, bias_part, N, smem, tid, wave);
  else conv3_bwd16_role<1, SP>(dy, w, xact, dx, part, bias_part, N, smem, tid, wave);
}

// variant 1: the 16-wave kernel
extern "C" int rrl_conv3_bwd(const uint16_t* dy, const uint16_t* w, const uint16_t* xact, uint16_t* dx, float* part,
                             float* bias_part, int N, int grid, int variant, void* stream) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv3_bwd_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize, c3b::kLds);
    (void)hipFuncSetAttribute((const void*)conv3_bwd_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, c3b::kLds);
    (void)hipFuncSetAttribute((const void*)conv3_bwd_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, c3b::kLds);
    (void)hipFuncSetAttribute((const void*)conv3_bwd16_kernel<0>, hipFuncAttributeMaxDynamicSharedMemorySize, c3b::kLds);
    (void)hipFuncSetAttribute((const void*)conv3_bwd16_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize, c3b::kLds);
    attr = true;
  }
  if (N < 1 || grid < 1) return 0;
  // RRL_CNN_BWD3_LDS_KB (A/B runs, read per call): launch the 8-wave kernel with this much dynamic
  // LDS (at least its own); 82 KB keeps it at one workgroup per CU, so a grid of 2 x CUs runs as
  // two rounds of workgroups the dispatcher places where CUs are free (static image sets: the
  // result does not depend on the placement)
  int lds = c3b::kLds;
  if (const char* e = getenv("RRL_CNN_BWD3_LDS_KB")) {
    const int kb = atoi(e);
    if (kb * 1024 > lds) {
      lds = min(kb, 160) * 1024;
      static bool attr_big = false;
      if (!attr_big) {
        (void)hipFuncSetAttribute((const void*)conv3_bwd_kernel<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  160 * 1024);
        attr_big = true;
      }
    }
  }
  if (variant == 1 || variant == 6) {  // the 16-wave kernel (6: with s_setprio around its MFMA clusters)
    hipLaunchKernelGGL(variant == 6 ? conv3_bwd16_kernel<1> : conv3_bwd16_kernel<0>, dim3(grid), dim3(c3b16::kThreads),
                       c3b::kLds, (hipStream_t)stream, dy, w, xact, dx, part, bias_part, N);
    return (int)hipGetLastError();
  }
  // variant 0 (default): s_setprio 1 around the MFMA clusters (SP 1): 163.6 -> 144.7 us per
  // 10,240 images, Pong +1.3 % / +1.4 % at 2,048 / 8,192 envs (profiles/r5_setprio_ab.txt);
  // 2 = without it (SP 0), 3 = the static form (SP 2)
  if (variant == 2)
    hipLaunchKernelGGL(conv3_bwd_kernel<0>, dim3(grid), dim3(c3b::kThreads), c3b::kLds, (hipStream_t)stream, dy, w,
                       xact, dx, part, bias_part, N);
  else if (variant == 3)
    hipLaunchKernelGGL(conv3_bwd_kernel<2>, dim3(grid), dim3(c3b::kThreads), c3b::kLds, (hipStream_t)stream, dy, w,
                       xact, dx, part, bias_part, N);
  else if (variant == 4 || variant == 5) {  // the priority pair around the wgrad / dgrad cluster only
    static bool attr_sp = false;
    if (!attr_sp) {
      (void)hipFuncSetAttribute((const void*)conv3_bwd_kernel<3>, hipFuncAttributeMaxDynamicSharedMemorySize, c3b::kLds);
      (void)hipFuncSetAttribute((const void*)conv3_bwd_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize, c3b::kLds);
      attr_sp = true;
    }
    hipLaunchKernelGGL(variant == 4 ? conv3_bwd_kernel<3> : conv3_bwd_kernel<4>, dim3(grid), dim3(c3b::kThreads),
                       c3b::kLds, (hipStream_t)stream, dy, w, xact, dx, part, bias_part, N);
  }
  else
    hipLaunchKernelGGL(conv3_bwd_kernel<1>, dim3(grid), dim3(c3b::kThreads), lds, (hipStream_t)stream, dy, w, xact,
                       dx, part, bias_part, N);
  return (int)hipGetLastError();
}

// ============================================================================= conv2 backward
// dgrad + wgrad + bias gradient of the second conv layer (20x20x32 -> 4x4/2 -> 9x9x64) in ONE
// pass per image, software-pipelined with ONE barrier per image: while image j computes from
// LDS buffer j & 1, image j + 1 (prefetched into registers one iteration earlier) is written
// into the other buffer and image j + 2's loads are in flight.
//
// LDS images per buffer:
//   da2  zero-bordered 12 x 12 (row (oh + 1) * 12 + ow + 1; 64 co + 16 pad: tools/lds_bank_model.py
//        --conv2; unpadded chunk-swizzled images cut the modelled LDS cycles 46 % more but their
//        per-read address arithmetic made the kernel 25 % slower, profiles/r4_cnn_swizzle_ab.txt)
//   a1   split into its four stride-2 phase images (ph, pw) = (ih & 1, iw & 1), each 10 x 10
//        positions (row (ih >> 1) * 10 + (iw >> 1), rows 100..115 zero; 32 c + 8 pad)
//   dgrad  da1[ph + 2a][pw + 2b][c] = sum_(i, j, co) da2[a - i][b - j][co] W2[co][ph + 2i][pw + 2j][c]
//          per phase class a 100 px x 32 c GEMM over K = (4 taps x 64 co); wave w: class w >> 1,
//          c tile w & 1, W2 fragments in registers.  The weights are the MFMA's A operand, so a
//          lane ends with 4 consecutive channels of one pixel: masked by a1 (from the phase
//          image) and stored straight to HBM as 8 bytes.
//   wgrad  dW2[64 co][(kh, kw, c) 512] += da2^T (co x pos) . im2col(a1) (pos x k): positions
//          in runs of 4 output columns (9 per row -> runs at ow 0, 4, 8; the run past ow 8 reads
//          the zero border), so each half of a transposed fragment read is 4 consecutive rows
//          of the da2 image AND of one a1 phase image (stride-2 taps land on unit-stride phase
//          rows); wave w: c block w & 1 of taps 4 (w >> 1) .. + 3, all 4 co tiles.
namespace c2b {
constexpr int kThreads = 512;
constexpr int kDLd = 80, kPLd = 40;  // 80: the dgrad b128 reads 2.71 -> 1.86 LDS cycles per conflict-free cycle (tools/lds_bank_model.py --conv2)
constexpr int kDRows = 144, kPRows = 116;
constexpr int kBuf = kDRows * kDLd + 4 * kPRows * kPLd;  // elements per buffer (30,080)
constexpr int kLds = 2 * kBuf * 2;                       // 120,320 bytes
constexpr int kYC = 81 * 8, kXC = 400 * 4;               // 16-byte chunks per image
constexpr int kYPT = (kYC + kThreads - 1) / kThreads, kXPT = (kXC + kThreads - 1) / kThreads;
}  // namespace c2b

__device__ __forceinline__ bf16x8_t tr_frag2(const uint16_t* a0, const uint16_t* a1) {
  typedef __attribute__((address_space(3))) s16x4_t lds_v4;
  s16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(a0));
  s16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(a1));
  typedef short s16x8_t __attribute__((ext_vector_type(8)));
  s16x8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

// STAGED: da1 goes through an LDS tile [400][40] and leaves as 16-byte row chunks after a
// second barrier, instead of 8-byte stores straight from the MFMA registers.  GRID12: the dgrad
// over a 10 x 12 grid per phase class (p = 12 a + b, columns 10, 11 and rows past 9 computed and
// discarded), 8 tiles: the 16 pixels of a fragment read 16 consecutive da2 rows, 1.86 -> 1.0
// modelled LDS factor (tools/lds_bank_model.py --conv2) -- measured 203.7 -> 205.8 us and Pong
// -0.1 to -0.4 % in an ABBA run (profiles/r4_bwd2_grid_ab.txt): not shipped
template <bool STAGED, bool GRID12 = false, int SP = 0>  // SP: wave priority, as conv3_bwd_kernel
__global__ __launch_bounds__(c2b::kThreads, 1) void conv2_bwd_kernel(const uint16_t* __restrict__ dy,
                                                                     const uint16_t* __restrict__ w,
                                                                     const uint16_t* __restrict__ xact,
                                                                     uint16_t* __restrict__ dx,
                                                                     float* __restrict__ part,
                                                                     float* __restrict__ bias_part, int N) {
  using namespace c2b;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int i16 = lane & 15, g = lane >> 4, q4 = (lane >> 2) & 3, p4 = lane & 3;
  // dgrad role: phase class (ph, pw), c tile
  const int cls = wave >> 1, ph = cls >> 1, pw = cls & 1, ct = wave & 1;
  // wgrad role: c block, taps tau0 .. tau0 + 3
  const int cb = wave & 1, tau0 = 4 * (wave >> 1);

  // dgrad A fragments (weights): k-step ks = (tap t = ks >> 1 -> (ti, tj), co block (ks & 1) * 32):
  // W2[co0 + 8g + e][ph + 2 ti][pw + 2 tj][16 ct + i16]
  bf16x8_t wf[8];
#pragma unroll
  for (int ks = 0; ks < 8; ++ks) {
    const int t = ks >> 1, kh = ph + 2 * (t >> 1), kw = pw + 2 * (t & 1), co0 = (ks & 1) * 32 + 8 * g;
    typedef short s16x8_t __attribute__((ext_vector_type(8)));
    s16x8_t v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (short)w[(((co0 + e) * 4 + kh) * 4 + kw) * 32 + 16 * ct + i16];
    wf[ks] = __builtin_bit_cast(bf16x8_t, v);
  }
  // zero both buffers once: the da2 border and the phase-image pad rows are never rewritten
  for (int q = tid; q < 2 * kBuf / 8; q += kThreads) *reinterpret_cast<uint4*>(smem + 8 * q) = make_uint4(0, 0, 0, 0);

  f32x4_t wacc[4][4];
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int t = 0; t < 4; ++t) wacc[c][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;  // db2[tid & 63] over positions (tid >> 6) + 8 k

  uint4 ry[kYPT], rx[kXPT];
  auto gload = [&](int n) {
    const uint4* ys = reinterpret_cast<const uint4*>(dy + (size_t)n * 81 * 64);
    const uint4* xs = reinterpret_cast<const uint4*>(xact + (size_t)n * 400 * 32);
#pragma unroll
    for (int k = 0; k < kYPT; ++k) {
      const int q = tid + kThreads * k;
      ry[k] = q < kYC ? ys[q] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < kXPT; ++k) {
      const int q = tid + kThreads * k;
      rx[k] = q < kXC ? xs[q] : make_uint4(0, 0, 0, 0);
    }
  };
  auto lstore = [&](int buf) {
    uint16_t* D = smem + buf * kBuf;
    uint16_t* P = D + kDRows * kDLd;
#pragma unroll
    for (int k = 0; k < kYPT; ++k) {
      const int q = tid + kThreads * k;
      if (q < kYC) {
        const int pix = q >> 3, oh = pix / 9, ow = pix - oh * 9;
        *reinterpret_cast<uint4*>(D + ((oh + 1) * 12 + ow + 1) * kDLd + (q & 7) * 8) = ry[k];
      }
    }
#pragma unroll
    for (int k = 0; k < kXPT; ++k) {
      const int q = tid + kThreads * k;
      if (q < kXC) {
        const int pix = q >> 2, ih = pix / 20, iw = pix - ih * 20;
        const int phase = (ih & 1) * 2 + (iw & 1);
        *reinterpret_cast<uint4*>(P + (phase * kPRows + (ih >> 1) * 10 + (iw >> 1)) * kPLd + (q & 3) * 8) = rx[k];
      }
    }
  };

  const int G = gridDim.x, n0 = blockIdx.x;
  __syncthreads();  // zeroing done before the first image lands in buffer 0
  if (n0 < N) {
    gload(n0);
    lstore(0);
  }
  if (n0 + G < N) gload(n0 + G);
  if constexpr (SP == 2) {
    if (wave >= 4) __builtin_amdgcn_s_setprio(1);
  }
  for (int j = 0; n0 + j * G < N; ++j) {
    const int n = n0 + j * G;
    __syncthreads();  // buffer j & 1 holds image n; buffer (j + 1) & 1 is no longer read
    if (n + G < N) {
      lstore((j + 1) & 1);
      if (n + 2 * G < N) gload(n + 2 * G);
    }
    const uint16_t* D = smem + (j & 1) * kBuf;
    const uint16_t* P = D + kDRows * kDLd;

    // ---- wgrad: 4 position k-steps (8 runs of 4 columns each), 4 co tiles x 4 taps
    if constexpr (SP == 1 || SP == 3) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      int oh[2], ow0[2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int R = 2 * (4 * s + g) + h;  // run index; runs >= 27 read zero rows
        oh[h] = R < 27 ? R / 3 : 9;
        ow0[h] = R < 27 ? 4 * (R % 3) : 0;
      }
      bf16x8_t af[4], bfr[4];
#pragma unroll
      for (int c = 0; c < 4; ++c)
        af[c] = tr_frag2(D + ((oh[0] + 1) * 12 + ow0[0] + 1 + q4) * kDLd + 16 * c + 4 * p4,
                         D + ((oh[1] + 1) * 12 + ow0[1] + 1 + q4) * kDLd + 16 * c + 4 * p4);
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int tau = tau0 + t, kh = tau >> 2, kw = tau & 3;
        const uint16_t* Pp = P + ((kh & 1) * 2 + (kw & 1)) * kPRows * kPLd + 16 * cb + 4 * p4;
        bfr[t] = tr_frag2(Pp + ((oh[0] + (kh >> 1)) * 10 + ow0[0] + (kw >> 1) + q4) * kPLd,
                          Pp + ((oh[1] + (kh >> 1)) * 10 + ow0[1] + (kw >> 1) + q4) * kPLd);
      }
#pragma unroll
      for (int c = 0; c < 4; ++c)
#pragma unroll
        for (int t = 0; t < 4; ++t) wacc[c][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[c], bfr[t], wacc[c][t], 0, 0, 0);
    }
    if constexpr (SP == 1 || SP == 3) __builtin_amdgcn_s_setprio(0);
    // ---- dgrad of phase class (ph, pw), c tile ct: 7 pixel tiles in two batches (rows past the
    // class are computed and discarded; GRID12: 8 tiles of the 10 x 12 grid)
    auto class_tiles = [&](auto tag) {
      constexpr int T0 = decltype(tag)::value, NT = (GRID12 || T0 == 0) ? 4 : 3;
      constexpr int W = GRID12 ? 12 : 10;  // grid width
      f32x4_t acc[NT];
      int rb[NT];
#pragma unroll
      for (int u = 0; u < NT; ++u) {
        acc[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
        if (GRID12) {
          rb[u] = 16 * (T0 + u) + i16 + 13;  // (a + 1) * 12 + (b + 1); at most row 140 of 144
        } else {
          const int p = 16 * (T0 + u) + i16, pc = p < 100 ? p : 0, a = pc / 10, b = pc - a * 10;
          rb[u] = (a + 1) * 12 + (b + 1);
        }
      }
      if constexpr (SP == 1 || SP == 4) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) {
        const int t = ks >> 1, ti = t >> 1, tj = t & 1;
        const int off = -(ti * 12 + tj) * kDLd + (ks & 1) * 32 + 8 * g;
        bf16x8_t bv[NT];
#pragma unroll
        for (int u = 0; u < NT; ++u) bv[u] = *reinterpret_cast<const bf16x8_t*>(D + rb[u] * kDLd + off);
#pragma unroll
        for (int u = 0; u < NT; ++u) acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ks], bv[u], acc[u], 0, 0, 0);
      }
      if constexpr (SP == 1 || SP == 4) __builtin_amdgcn_s_setprio(0);
      // D = da1^T: lane (i16, g) holds channels 16 ct + 4g .. + 3 of class pixel p
      if constexpr (SP == 8 && !STAGED && !GRID12) {
        // 16-byte stores (A/B): lanes g and g ^ 1 (same pixel row i16) swap halves through
        // ds_swizzle, so the even lane stores channels 4g .. 4g + 7 of tile u's pixel and the odd
        // lane those of tile u + 1's pixel -- one 16-byte store instruction per pair of tiles
        uint2 v[NT];
        int pix[NT];
        bool okp[NT];
#pragma unroll
        for (int u = 0; u < NT; ++u) {
          const int p = 16 * (T0 + u) + i16;
          okp[u] = p < 100;
          const int pc = okp[u] ? p : 0, a = pc / 10, b = pc - a * 10;
          const uint2 m = *reinterpret_cast<const uint2*>(P + (cls * kPRows + a * 10 + b) * kPLd + 16 * ct + 4 * g);
          v[u] = make_uint2(relu_mask2(pk_bf16(acc[u][0], acc[u][1]), m.x), relu_mask2(pk_bf16(acc[u][2], acc[u][3]), m.y));
          pix[u] = (ph + 2 * a) * 20 + pw + 2 * b;
        }
        const bool odd = (g & 1) != 0;
        const int ch = 16 * ct + 4 * (g & ~1);
#pragma unroll
        for (int u = 0; u + 1 < NT; u += 2) {
          const uint2 send = odd ? v[u] : v[u + 1];
          const uint32_t rx = (uint32_t)__builtin_amdgcn_ds_swizzle((int)send.x, 0x401F);
          const uint32_t ry = (uint32_t)__builtin_amdgcn_ds_swizzle((int)send.y, 0x401F);
          const uint4 o = odd ? make_uint4(rx, ry, v[u + 1].x, v[u + 1].y) : make_uint4(v[u].x, v[u].y, rx, ry);
          if (odd ? okp[u + 1] : okp[u])
            *reinterpret_cast<uint4*>(dx + ((size_t)n * 400 + (odd ? pix[u + 1] : pix[u])) * 32 + ch) = o;
        }
        if constexpr (NT & 1) {
          if (okp[NT - 1]) *reinterpret_cast<uint2*>(dx + ((size_t)n * 400 + pix[NT - 1]) * 32 + 16 * ct + 4 * g) = v[NT - 1];
        }
        return;
      }
#pragma unroll
      for (int u = 0; u < NT; ++u) {
        const int p = 16 * (T0 + u) + i16;
        if (GRID12 ? (p / 12 < 10 && p % 12 < 10) : p < 100) {
          const int a = p / W, b = p - a * W;
          const uint2 m = *reinterpret_cast<const uint2*>(P + (cls * kPRows + a * 10 + b) * kPLd + 16 * ct + 4 * g);
          const uint2 v = make_uint2(relu_mask2(pk_bf16(acc[u][0], acc[u][1]), m.x),
                                     relu_mask2(pk_bf16(acc[u][2], acc[u][3]), m.y));
          const int pix = (ph + 2 * a) * 20 + pw + 2 * b;
          if (STAGED) *reinterpret_cast<uint2*>(smem + 2 * kBuf + pix * 40 + 16 * ct + 4 * g) = v;
          else *reinterpret_cast<uint2*>(dx + ((size_t)n * 400 + pix) * 32 + 16 * ct + 4 * g) = v;
        }
      }
    };
    class_tiles(std::integral_constant<int, 0>{});
    class_tiles(std::integral_constant<int, 4>{});
    // ---- db2
    for (int pos = tid >> 6; pos < 81; pos += 8) {
      const int oh = pos / 9, ow = pos - oh * 9;
      bsum += bf2f(D[((oh + 1) * 12 + ow + 1) * kDLd + (tid & 63)]);
    }
    if (STAGED) {
      __syncthreads();  // staging tile complete (rewritten only after the next top barrier)
      const uint16_t* O = smem + 2 * kBuf;
      uint4* xd = reinterpret_cast<uint4*>(dx + (size_t)n * 400 * 32);
      for (int q = tid; q < 400 * 4; q += kThreads) xd[q] = *reinterpret_cast<const uint4*>(O + (q >> 2) * 40 + (q & 3) * 8);
    }
  }
  // weight-gradient partial of this workgroup: part[blk][co][kh][kw][c]
  float* o = part + (size_t)blockIdx.x * 64 * 512;
#pragma unroll
  for (int c = 0; c < 4; ++c)
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[(16 * c + 4 * g + r) * 512 + (tau0 + t) * 32 + 16 * cb + i16] = wacc[c][t][r];
  // the bias partial folded over the 8 waves in LDS: 64 values per workgroup (the end-of-backward
  // slab sum's bias segments had 8 x the splits and were its longest blocks)
  __syncthreads();  // every wave is past its last LDS read of the image buffers
  float* red = reinterpret_cast<float*>(smem);
  red[tid] = bsum;
  __syncthreads();
  if (tid < 64) {
    float sb = 0.f;
#pragma unroll
    for (int w = 0; w < kThreads / 64; ++w) sb += red[w * 64 + tid];
    bias_part[(size_t)blockIdx.x * 64 + tid] = sb;
  }
}

// 16-wave form of conv2_bwd_kernel (4 waves per SIMD instead of 2): the dgrad and the wgrad of
// an image run on DIFFERENT waves -- waves 0-7 the dgrad (phase class w >> 1, c tile w & 1: W2
// fragments + 4 accumulators), waves 8-15 the wgrad (c block w & 1, taps 4 ((w - 8) >> 1) ..
// + 3: the 16 weight-gradient accumulators) -- instead of one after the other on the same 8
// waves, so neither role carries the other's registers (<= 128 each) and a SIMD interleaves two
// dgrad and two wgrad waves.  Same LDS images, k-orders, partial layout and one barrier per image
// as conv2_bwd_kernel: its outputs bitwise.  All 1,024 threads stage the next image.
#ifndef C2B16_SCHED
#define C2B16_SCHED 0
#endif
#ifndef C2B16_NT
#define C2B16_NT 4
#endif
namespace c2b16 {
constexpr int kThreads = 1024;
constexpr int kStage = 512;  // the dgrad waves stage the next image (the wgrad waves' registers are full)
constexpr int kYPT = (c2b::kYC + kStage - 1) / kStage, kXPT = (c2b::kXC + kStage - 1) / kStage;
}  // namespace c2b16

template <int ROLE>  // 0 = dgrad, 1 = wgrad
__device__ __forceinline__ void conv2_bwd16_role(const uint16_t* __restrict__ dy, const uint16_t* __restrict__ w,
                                                 const uint16_t* __restrict__ xact, uint16_t* __restrict__ dx,
                                                 float* __restrict__ part, float* __restrict__ bias_part, int N,
                                                 uint16_t* smem, int tid, int wave) {
  using namespace c2b;
  constexpr int T = c2b16::kStage;
  const int lane = tid & 63;
  const int i16 = lane & 15, g = lane >> 4;
  const int cls = wave >> 1, ph = cls >> 1, pw = cls & 1, ct = wave & 1;  // dgrad role (waves 0-7)
  const int cb = wave & 1, tau0 = 4 * ((wave - 8) >> 1);                 // wgrad role (waves 8-15)
  bf16x8_t wf[ROLE == 0 ? 8 : 1];
  f32x4_t wacc[ROLE == 1 ? 4 : 1][4];
  if constexpr (ROLE == 0) {
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const int t = ks >> 1, kh = ph + 2 * (t >> 1), kw = pw + 2 * (t & 1), co0 = (ks & 1) * 32 + 8 * g;
      typedef short s16x8_t __attribute__((ext_vector_type(8)));
      s16x8_t v;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (short)w[(((co0 + e) * 4 + kh) * 4 + kw) * 32 + 16 * ct + i16];
      wf[ks] = __builtin_bit_cast(bf16x8_t, v);
    }
  } else {
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int t = 0; t < 4; ++t) wacc[c][t] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }
  for (int q = tid; q < 2 * kBuf / 8; q += c2b16::kThreads) *reinterpret_cast<uint4*>(smem + 8 * q) = make_uint4(0, 0, 0, 0);
  float bsum = 0.f;  // dgrad waves: db2[tid & 63] over positions (tid >> 6) + 8 k

  // tv: tid behind an empty asm each iteration, so the loop-invariant staging / fragment addresses
  // are recomputed (a few VALU) instead of hoisted out of the loop into registers this 4-wave-per-SIMD
  // kernel does not have
  int tv = tid;
  uint4 ry[ROLE == 0 ? c2b16::kYPT : 1], rx[ROLE == 0 ? c2b16::kXPT : 1];
  auto gload = [&](int n) {
    if constexpr (ROLE == 1) return;
    const uint4* ys = reinterpret_cast<const uint4*>(dy + (size_t)n * 81 * 64);
    const uint4* xs = reinterpret_cast<const uint4*>(xact + (size_t)n * 400 * 32);
#pragma unroll
    for (int k = 0; k < c2b16::kYPT; ++k) {
      const int q = tv + T * k;
      ry[k] = q < kYC ? ys[q] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int k = 0; k < c2b16::kXPT; ++k) {
      const int q = tv + T * k;
      rx[k] = q < kXC ? xs[q] : make_uint4(0, 0, 0, 0);
    }
  };
  auto lstore = [&](int buf) {
    if constexpr (ROLE == 1) return;
    uint16_t* D = smem + buf * kBuf;
    uint16_t* P = D + kDRows * kDLd;
#pragma unroll
    for (int k = 0; k < c2b16::kYPT; ++k) {
      const int q = tv + T * k;
      if (q < kYC) {
        const int pix = q >> 3, oh = pix / 9, ow = pix - oh * 9;
        *reinterpret_cast<uint4*>(D + ((oh + 1) * 12 + ow + 1) * kDLd + (q & 7) * 8) = ry[k];
      }
    }
#pragma unroll
    for (int k = 0; k < c2b16::kXPT; ++k) {
      const int q = tv + T * k;
      if (q < kXC) {
        const int pix = q >> 2, ih = pix / 20, iw = pix - ih * 20;
        const int phase = (ih & 1) * 2 + (iw & 1);
        *reinterpret_cast<uint4*>(P + (phase * kPRows + (ih >> 1) * 10 + (iw >> 1)) * kPLd + (q & 3) * 8) = rx[k];
      }
    }
  };

  const int G = gridDim.x, n0 = blockIdx.x;
  __syncthreads();  // zeroing done before the first image lands in buffer 0
  if (n0 < N) {
    gload(n0);
    lstore(0);
  }
  if (n0 + G < N) gload(n0 + G);
  for (int j = 0; n0 + j * G < N; ++j) {
    const int n = n0 + j * G;
    __syncthreads();  // buffer j & 1 holds image n; buffer (j + 1) & 1 is no longer read
    asm volatile("" : "+v"(tv));
    const int i16 = tv & 15, g = (tv >> 4) & 3, q4 = (tv >> 2) & 3, p4 = tv & 3;
    if (n + G < N) {
      lstore((j + 1) & 1);
      if (n + 2 * G < N) gload(n + 2 * G);
    }
    const uint16_t* D = smem + (j & 1) * kBuf;
    const uint16_t* P = D + kDRows * kDLd;
    if constexpr (ROLE == 1) {
      // ---- wgrad: 4 position k-steps (8 runs of 4 columns each), 4 co tiles x 4 taps
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        int oh[2], ow0[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int R = 2 * (4 * s + g) + h;  // run index; runs >= 27 read zero rows
          oh[h] = R < 27 ? R / 3 : 9;
          ow0[h] = R < 27 ? 4 * (R % 3) : 0;
        }
        bf16x8_t af[4], bfr[4];
#pragma unroll
        for (int c = 0; c < 4; ++c)
          af[c] = tr_frag2(D + ((oh[0] + 1) * 12 + ow0[0] + 1 + q4) * kDLd + 16 * c + 4 * p4,
                           D + ((oh[1] + 1) * 12 + ow0[1] + 1 + q4) * kDLd + 16 * c + 4 * p4);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const int tau = tau0 + t, kh = tau >> 2, kw = tau & 3;
          const uint16_t* Pp = P + ((kh & 1) * 2 + (kw & 1)) * kPRows * kPLd + 16 * cb + 4 * p4;
          bfr[t] = tr_frag2(Pp + ((oh[0] + (kh >> 1)) * 10 + ow0[0] + (kw >> 1) + q4) * kPLd,
                            Pp + ((oh[1] + (kh >> 1)) * 10 + ow0[1] + (kw >> 1) + q4) * kPLd);
        }
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int t = 0; t < 4; ++t) wacc[c][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[c], bfr[t], wacc[c][t], 0, 0, 0);
      }
    } else {
      // ---- dgrad of phase class (ph, pw), c tile ct: 7 pixel tiles in batches of C2B16_NT (+ 1)
      auto class_tiles = [&](auto tag) {
        constexpr int T0 = decltype(tag)::value, NT = T0 == 6 ? 1 : (C2B16_NT == 4 && T0 == 4 ? 3 : C2B16_NT);
        f32x4_t acc[NT];
        int rb[NT];
#pragma unroll
        for (int u = 0; u < NT; ++u) {
          acc[u] = f32x4_t{0.f, 0.f, 0.f, 0.f};
          const int p = 16 * (T0 + u) + i16, pc = p < 100 ? p : 0, a = pc / 10, b = pc - a * 10;
          rb[u] = (a + 1) * 12 + (b + 1);
        }
#pragma unroll
        for (int ks = 0; ks < 8; ++ks) {
          const int t = ks >> 1, ti = t >> 1, tj = t & 1;
          const int off = -(ti * 12 + tj) * kDLd + (ks & 1) * 32 + 8 * g;
          bf16x8_t bv[NT];
#pragma unroll
          for (int u = 0; u < NT; ++u) bv[u] = *reinterpret_cast<const bf16x8_t*>(D + rb[u] * kDLd + off);
#pragma unroll
          for (int u = 0; u < NT; ++u) acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[ks], bv[u], acc[u], 0, 0, 0);
          if (C2B16_SCHED) __builtin_amdgcn_sched_barrier(0);  // keep the reads of later k-steps from piling up in registers
        }
#pragma unroll
        for (int u = 0; u < NT; ++u) {
          const int p = 16 * (T0 + u) + i16;
          if (p < 100) {
            const int a = p / 10, b = p - a * 10;
            const uint2 m = *reinterpret_cast<const uint2*>(P + (cls * kPRows + a * 10 + b) * kPLd + 16 * ct + 4 * g);
            const uint2 v = make_uint2(relu_mask2(pk_bf16(acc[u][0], acc[u][1]), m.x),
                                       relu_mask2(pk_bf16(acc[u][2], acc[u][3]), m.y));
            const int pix = (ph + 2 * a) * 20 + pw + 2 * b;
            *reinterpret_cast<uint2*>(dx + ((size_t)n * 400 + pix) * 32 + 16 * ct + 4 * g) = v;
          }
        }
      };
      if constexpr (C2B16_NT == 2) {
        class_tiles(std::integral_constant<int, 0>{});
        class_tiles(std::integral_constant<int, 2>{});
        class_tiles(std::integral_constant<int, 4>{});
        class_tiles(std::integral_constant<int, 6>{});
      } else if constexpr (C2B16_NT == 3) {
        class_tiles(std::integral_constant<int, 0>{});
        class_tiles(std::integral_constant<int, 3>{});
        class_tiles(std::integral_constant<int, 6>{});
      } else {
        class_tiles(std::integral_constant<int, 0>{});
        class_tiles(std::integral_constant<int, 4>{});
      }
      // ---- db2
      for (int pos = tid >> 6; pos < 81; pos += 8) {
        const int oh = pos / 9, ow = pos - oh * 9;
        bsum += bf2f(D[((oh + 1) * 12 + ow + 1) * kDLd + (tid & 63)]);
      }
    }
  }
  if constexpr (ROLE == 1) {  // weight-gradient partial of this workgroup: part[blk][co][kh][kw][c]
    float* o = part + (size_t)blockIdx.x * 64 * 512;
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) o[(16 * c + 4 * g + r) * 512 + (tau0 + t) * 32 + 16 * cb + i16] = wacc[c][t][r];
  }
  __syncthreads();  // every wave is past its last LDS read of the image buffers
  float* red = reinterpret_cast<float*>(smem);
  if (ROLE == 0) red[tid] = bsum;
  __syncthreads();
  if (tid < 64) {
    float sb = 0.f;
#pragma unroll
    for (int w8 = 0; w8 < 8; ++w8) sb += red[w8 * 64 + tid];
    bias_part[(size_t)blockIdx.x * 64 + tid] = sb;
  }
}

__global__ __launch_bounds__(c2b16::kThreads, 1) void conv2_bwd16_kernel(const uint16_t* __restrict__ dy,
                                                                         const uint16_t* __restrict__ w,
                                                                         const uint16_t* __restrict__ xact,
                                                                         uint16_t* __restrict__ dx,
                                                                         float* __restrict__ part,
                                                                         float* __restrict__ bias_part, int N) {
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  if (wave < 8) conv2_bwd16_role<0>(dy, w, xact, dx, part, bias_part, N, smem, tid, wave);
  else conv2_bwd16_role<1>(dy, w, xact, dx, part, bias_part, N, smem, tid, wave);
}

// variant 1: da1 through the LDS staging tile (measured slower: 229 vs 214 us, tools/cnn_kbench.py
// bwd2 / bwd2_direct); 2: the dgrad over the 10 x 12 grid (measured no faster); 3: the
// 16-wave kernel (conv2_bwd16_kernel)
extern "C" int rrl_conv2_bwd(const uint16_t* dy, const uint16_t* w, const uint16_t* xact, uint16_t* dx, float* part,
                             float* bias_part, int N, int grid, int staged, void* stream) {
  static bool attr = false;
  constexpr int kStagedLds = c2b::kLds + 400 * 40 * 2;  // 152,320 bytes
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv2_bwd_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              c2b::kLds);
    (void)hipFuncSetAttribute((const void*)conv2_bwd_kernel<false, true>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, c2b::kLds);
    (void)hipFuncSetAttribute((const void*)conv2_bwd_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              kStagedLds);
    (void)hipFuncSetAttribute((const void*)conv2_bwd_kernel<false, false, 1>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, c2b::kLds);
    (void)hipFuncSetAttribute((const void*)conv2_bwd_kernel<false, false, 2>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, c2b::kLds);
    attr = true;
  }
  if (N < 1 || grid < 1) return 0;
  if (staged == 3) {
    static bool attr16 = false;
    if (!attr16) {
      (void)hipFuncSetAttribute((const void*)conv2_bwd16_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, c2b::kLds);
      attr16 = true;
    }
    hipLaunchKernelGGL(conv2_bwd16_kernel, dim3(grid), dim3(c2b16::kThreads), c2b::kLds, (hipStream_t)stream, dy, w,
                       xact, dx, part, bias_part, N);
  } else if (staged >= 4 && staged <= 7) {  // wave-priority A/B forms: SP 1 (both clusters) / 2 (static) /
    // 3 (the wgrad cluster only) / 4 (the dgrad cluster only)
    static bool attr_sp = false;
    if (!attr_sp) {
      (void)hipFuncSetAttribute((const void*)conv2_bwd_kernel<false, false, 3>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, c2b::kLds);
      (void)hipFuncSetAttribute((const void*)conv2_bwd_kernel<false, false, 4>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, c2b::kLds);
      attr_sp = true;
    }
    auto* k = staged == 4 ? conv2_bwd_kernel<false, false, 1>
                          : (staged == 5 ? conv2_bwd_kernel<false, false, 2>
                                         : (staged == 6 ? conv2_bwd_kernel<false, false, 3> : conv2_bwd_kernel<false, false, 4>));
    hipLaunchKernelGGL(k, dim3(grid), dim3(c2b::kThreads), c2b::kLds, (hipStream_t)stream, dy, w, xact, dx, part,
                       bias_part, N);
  } else if (staged == 8) {  // 16-byte da1 stores through lane swaps (A/B)
    static bool attr8 = false;
    if (!attr8) {
      (void)hipFuncSetAttribute((const void*)conv2_bwd_kernel<false, false, 8>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, c2b::kLds);
      attr8 = true;
    }
    auto* k = conv2_bwd_kernel<false, false, 8>;
    hipLaunchKernelGGL(k, dim3(grid), dim3(c2b::kThreads), c2b::kLds, (hipStream_t)stream, dy, w, xact, dx, part,
                       bias_part, N);
  } else if (staged == 1)
    hipLaunchKernelGGL(conv2_bwd_kernel<true>, dim3(grid), dim3(c2b::kThreads), kStagedLds, (hipStream_t)stream, dy, w,
                       xact, dx, part, bias_part, N);
  else if (staged == 2)
    hipLaunchKernelGGL((conv2_bwd_kernel<false, true>), dim3(grid), dim3(c2b::kThreads), c2b::kLds,
                       (hipStream_t)stream, dy, w, xact, dx, part, bias_part, N);
  else
    hipLaunchKernelGGL(conv2_bwd_kernel<false>, dim3(grid), dim3(c2b::kThreads), c2b::kLds, (hipStream_t)stream, dy,
                       w, xact, dx, part, bias_part, N);
  return (int)hipGetLastError();
}

// ============================================================================= conv1 wgrad
// dW1[co][kh][kw][c] (+ db1) of the space-to-depth first layer, 8 waves per workgroup (two per
// SIMD, where cnn.hip's conv1_wgrad_s2d_kernel ran one): wave w computes tap (kh, kw) =
// ((w & 3) >> 1, w & 1) over HALF of the 13 position chunks (w >> 2 picks the half), so the
// two waves of a SIMD hide each other's transposed-read latency; each half leaves its own
// partial slab (2 per workgroup).  Frame (as exact bf16 integers) and dY go through LDS once
// per image with the next image prefetched into registers.
namespace c1w {
constexpr int kThreads = 512;
// frame positions in LDS rows of 28 (as the fused forward) and dY rows of 48 elements: the
// transposed fragment reads of both images conflict-free in tools/lds_bank_model.py (the frame
// in 21-wide rows: 1.19 LDS cycles per conflict-free cycle)
constexpr int kLd = 80, kYLd = 48, kXW = 28;
constexpr int kXRows = 20 * kXW + 24, kYRows = 416;
constexpr int kLds = (kXRows * kLd + kYRows * kYLd) * 2;  // 133,632 bytes
constexpr int kLdsRing = kLds + kRingTab * 16;              // + the frame ring's frame-row table
static_assert(kLds % 16 == 0 && kLdsRing <= 160 * 1024, "LDS per workgroup");
constexpr int kXC = 441 * 4, kYC = 400 * 4;       // 16-byte chunks per image
constexpr int kXPT = (kXC + kThreads - 1) / kThreads, kYPT = (kYC + kThreads - 1) / kThreads;
}  // namespace c1w

// RENDER: the frames are drawn from PongSynth frame histories hist[N][16] (pong_render.h)
// instead of read from an observation tensor
// RING: the frames are read from the PongSynth frame store through the frame rows fidx[N][4]
// (pong_render.h) and interleaved into the observation's channel order -- the same LDS image
template <bool RENDER, bool SP = false, bool RING = false>  // SP: s_setprio 1 around each chunk's MFMAs (A/B)
__global__ __launch_bounds__(c1w::kThreads, 1) void conv1_wgrad8_kernel(const uint8_t* __restrict__ x,
                                                                        const float* __restrict__ hist,
                                                                        const uint16_t* __restrict__ dy,
                                                                        float* __restrict__ part,
                                                                        float* __restrict__ bias_part, int N,
                                                                        const uint8_t* __restrict__ frames = nullptr,
                                                                        const int32_t* __restrict__ fidx = nullptr,
                                                                        int T = 0) {
  using namespace c1w;
  extern __shared__ __attribute__((aligned(16))) uint16_t smem[];
  uint16_t* Xi = smem;                // [21 x 28][80] frame, bf16 integers 0..255
  uint16_t* Yi = smem + kXRows * kLd;  // [416][48] dY (rows 400.. zero)
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int tap = wave & 3, kh = tap >> 1, kw = tap & 1, half = wave >> 2;
  const int kc0 = half ? 7 : 0, kc1 = half ? 13 : 7;
  for (int q = tid; q < 16 * (kYLd / 8); q += kThreads)
    *reinterpret_cast<uint4*>(Yi + (400 + q / (kYLd / 8)) * kYLd + 8 * (q % (kYLd / 8))) = make_uint4(0, 0, 0, 0);

  f32x4_t acc[2][4], accb[2];
#pragma unroll
  for (int mt = 0; mt < 2; ++mt) {
    accb[mt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = f32x4_t{0.f, 0.f, 0.f, 0.f};
  }
  // db[co] = sum_p dY[p][co] rides on the tap-(0, 0) waves as an MFMA whose B is 1 in column 0
  const bool do_bias = tap == 0;
  bf16x8_t ones;
  {
    typedef short s16x8_t __attribute__((ext_vector_type(8)));
    const short one = (lane & 15) == 0 ? (short)0x3f80 : (short)0;
    s16x8_t v = {one, one, one, one, one, one, one, one};
    ones = __builtin_bit_cast(bf16x8_t, v);
  }
  uint4 rx[kXPT], ry[kYPT];
  // the next image's frame chunks: loaded (observations) or drawn (RENDER: the history row's 16
  // floats in SGPRs) into the same registers
  static_assert(kXPT >= 4, "the ring form keeps one position's 4 x 16 raw bytes per thread");
  // This workgroup's images, in order k = 0 .. K - 1: n0 + k G, or (T > 1, rows t E + e of a
  // T-step rollout over E envs) env-major -- the T rows of env e = n0 + q G back to back, so with
  // the frame ring the 4-frame observations of consecutive images share 3 frames and those are
  // re-read from this CU's L2 (the weight gradient is a sum over images: the order only
  // reassociates it)
  const int n0 = blockIdx.x, G = gridDim.x;
  const int E = T > 1 ? N / T : N;
  const int K = T > 1 ? (n0 < E ? T * ((E - n0 + G - 1) / G) : 0) : ring_images(N, n0, G);
  auto img = [&](int k) -> int {
    if (T > 1) {
      const int q = k / T, t = k - q * T;
      return t * E + n0 + q * G;
    }
    return n0 + k * G;
  };
  // frame ring: this workgroup's images' frame rows, staged in LDS after the images once (read
  // from the table a stage ahead; images past it read fidx directly)
  int4* rtab = reinterpret_cast<int4*>(reinterpret_cast<uint8_t*>(smem) + kLds);
  auto ring_entry = [&](int k) -> int4 {
    return uniform_int4(k < kRingTab ? rtab[k] : *reinterpret_cast<const int4*>(fidx + 4 * (size_t)img(k)));
  };
  // the frame rows of the image xload reads next (RING): read from the table a stage ahead
  int4 fr_next = make_int4(0, 0, 0, 0);
  auto xload = [&](int n) {
    if constexpr (RING) {
      // thread tid < 441: position tid, all 16 bytes of frames 0..3 (one 16-byte load per frame:
      // half the load instructions of 8-byte row pieces; the 4 registers the s2d path uses)
      const int4 fr = fr_next;
      (void)n;
      if (tid < kPongFramePos) {
        const size_t off = (size_t)tid * 16;
        rx[0] = *reinterpret_cast<const uint4*>(frames + (size_t)fr.x * kPongFrameBytes + off);
        rx[1] = *reinterpret_cast<const uint4*>(frames + (size_t)fr.y * kPongFrameBytes + off);
        rx[2] = *reinterpret_cast<const uint4*>(frames + (size_t)fr.z * kPongFrameBytes + off);
        rx[3] = *reinterpret_cast<const uint4*>(frames + (size_t)fr.w * kPongFrameBytes + off);
      }
    } else if constexpr (RENDER) {
      float hv[kPongHist];
      uniform_row(hist + (size_t)n * kPongHist, hv);
#pragma unroll
      for (int i = 0; i < kXPT; ++i) {
        const int q = tid + kThreads * i;
        rx[i] = q < kXC ? pong_render_chunk(hv, q) : make_uint4(0, 0, 0, 0);
      }
    } else {
      const uint4* xs = reinterpret_cast<const uint4*>(x + (size_t)n * 441 * 64);
#pragma unroll
      for (int i = 0; i < kXPT; ++i) {
        const int q = tid + kThreads * i;
        rx[i] = q < kXC ? xs[q] : make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto gload = [&](int n) {
    const uint4* ys = reinterpret_cast<const uint4*>(dy + (size_t)n * 400 * 32);
#pragma unroll
    for (int i = 0; i < kYPT; ++i) {
      const int q = tid + kThreads * i;
      ry[i] = q < kYC ? ys[q] : make_uint4(0, 0, 0, 0);
    }
  };
  // RENDER: the first half of the waves draws the next frame before its MFMAs, the second half
  // (the other wave of each SIMD) after them, so one wave's VALU drawing runs beside the other's
  // matrix work
  const bool draw_late = RENDER && half;
  const int g = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
  if (K > 0) {
    const int n = img(0);
    gload(n);
    // the first image's rows straight from fidx (the table is first read after the loop's barrier)
    if constexpr (RING) fr_next = uniform_int4(*reinterpret_cast<const int4*>(fidx + 4 * (size_t)n));
    xload(n);
  }
  if constexpr (RING) {  // staged after the first image's loads are in flight
    for (int k = tid; k < min(K, kRingTab); k += kThreads) rtab[k] = *reinterpret_cast<const int4*>(fidx + 4 * (size_t)img(k));
  }
  for (int k = 0; k < K; ++k) {
    const bool more = k + 1 < K;
    const int nn = more ? img(k + 1) : 0;  // the next image
    __syncthreads();  // the previous image's fragment reads are done
    if constexpr (RING) {
      if (more) fr_next = ring_entry(k + 1);  // before this image's stores
    }
    if constexpr (RING) {
      if (tid < kPongFramePos) {  // the 4 observation chunks (dy = 0..3) of position tid, as bf16
        const uint32_t f0[4] = {rx[0].x, rx[0].y, rx[0].z, rx[0].w}, f1[4] = {rx[1].x, rx[1].y, rx[1].z, rx[1].w};
        const uint32_t f2[4] = {rx[2].x, rx[2].y, rx[2].z, rx[2].w}, f3[4] = {rx[3].x, rx[3].y, rx[3].z, rx[3].w};
        uint16_t* d = Xi + (tid + (kXW - 21) * (tid / 21)) * kLd;
#pragma unroll
        for (int dy = 0; dy < 4; ++dy) {
          const uint4 c = pong_interleave_row(f0[dy], f1[dy], f2[dy], f3[dy]);
          *reinterpret_cast<uint4*>(d + 16 * dy) = u8x8_to_bf16x8(make_uint2(c.x, c.y));
          *reinterpret_cast<uint4*>(d + 16 * dy + 8) = u8x8_to_bf16x8(make_uint2(c.z, c.w));
        }
      }
    }
#pragma unroll
    for (int i = 0; i < (RING ? 0 : kXPT); ++i) {
      const int q = tid + kThreads * i;
      if (q < kXC) {
        const int pix = q >> 2;
        uint16_t* d = Xi + (pix + (kXW - 21) * (pix / 21)) * kLd + (q & 3) * 16;
        *reinterpret_cast<uint4*>(d) = u8x8_to_bf16x8(make_uint2(rx[i].x, rx[i].y));
        *reinterpret_cast<uint4*>(d + 8) = u8x8_to_bf16x8(make_uint2(rx[i].z, rx[i].w));
      }
    }
#pragma unroll
    for (int i = 0; i < kYPT; ++i) {
      const int q = tid + kThreads * i;
      if (q < kYC) *reinterpret_cast<uint4*>(Yi + (q >> 2) * kYLd + (q & 3) * 8) = ry[i];
    }
    if (more) {
      gload(nn);
      if (!draw_late) xload(nn);
    }
    __syncthreads();
    // MFMA k-order: lane group g of a 32-pixel chunk takes pixels 4g..4g+3 and 16+4g..16+4g+3
    // (a 4-pixel run never crosses an output row, so its frame rows are consecutive)
#pragma unroll 1
    for (int kc = kc0; kc < kc1; ++kc) {
      const int pa = 32 * kc + 4 * g, pb = pa + 16;
      const int ra = (pa < 400 ? (pa / 20 + kh) * kXW + pa % 20 + kw : 0) + qq;
      const int rb = (pb < 400 ? (pb / 20 + kh) * kXW + pb % 20 + kw : 0) + qq;
      bf16x8_t af[2], bfr[4];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
        af[mt] = tr_frag2(Yi + (pa + qq) * kYLd + 16 * mt + 4 * pp, Yi + (pb + qq) * kYLd + 16 * mt + 4 * pp);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt)
        bfr[nt] = tr_frag2(Xi + ra * kLd + 16 * nt + 4 * pp, Xi + rb * kLd + 16 * nt + 4 * pp);
      if constexpr (SP) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], bfr[nt], acc[mt][nt], 0, 0, 0);
      if (do_bias) {
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) accb[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], ones, accb[mt], 0, 0, 0);
      }
      if constexpr (SP) __builtin_amdgcn_s_setprio(0);
    }
    if (draw_late && more) xload(nn);
  }
  const int slab = 2 * blockIdx.x + half;
  if (do_bias && (lane & 15) == 0) {
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
      for (int r = 0; r < 4; ++r) bias_part[(size_t)slab * 32 + 16 * mt + 4 * g + r] = accb[mt][r];
  }
  // part[slab][cout][kh][kw][c], raw-byte products scaled by 1/255
  float* o = part + (size_t)slab * 32 * 256 + kh * 128 + kw * 64;
  const int j = lane & 15;
#pragma unroll
  for (int mt = 0; mt < 2; ++mt)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[(16 * mt + 4 * g + r) * 256 + 16 * nt + j] = acc[mt][nt][r] * kU8Scale;
}

// returns the number of partial slabs written (2 per workgroup); hist (PongSynth frame histories
// [N][16]): the frames are drawn in the kernel, x is not read
// T > 1 (frame ring only): the N = T E rows are a T-step rollout over E envs, visited env-major
extern "C" int rrl_conv1_wgrad8(const uint8_t* x, const float* hist, const uint8_t* frames, const int32_t* fidx,
                                const uint16_t* dy, float* part, float* bias_part, int N, int grid, int T,
                                void* stream) {
  static bool attr = false;
  if (frames) {  // frame ring: frames [R][E][7056], fidx [N][4]
    static bool attr_ring = false;
    if (!attr_ring) {
      (void)hipFuncSetAttribute((const void*)conv1_wgrad8_kernel<false, false, true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, c1w::kLdsRing);
      attr_ring = true;
    }
    if (N < 1 || grid < 1) return 0;
    if (!fidx || (T > 1 && N % T != 0)) return -2;
    hipLaunchKernelGGL((conv1_wgrad8_kernel<false, false, true>), dim3(grid), dim3(c1w::kThreads), c1w::kLdsRing,
                       (hipStream_t)stream, nullptr, nullptr, dy, part, bias_part, N, frames, fidx, T);
    return (int)hipGetLastError();
  }
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)conv1_wgrad8_kernel<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              c1w::kLds);
    (void)hipFuncSetAttribute((const void*)conv1_wgrad8_kernel<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              160 * 1024);
    attr = true;
  }
  if (N < 1 || grid < 1) return 0;
  const char* sp = getenv("RRL_CNN_WGRAD1_SETPRIO");  // A/B: 1 = the s_setprio form (read per call)
  if (!hist && sp && sp[0] == '1') {
    static bool attr_sp = false;
    if (!attr_sp) {
      (void)hipFuncSetAttribute((const void*)conv1_wgrad8_kernel<false, true>,
                                hipFuncAttributeMaxDynamicSharedMemorySize, c1w::kLds);
      attr_sp = true;
    }
    hipLaunchKernelGGL((conv1_wgrad8_kernel<false, true>), dim3(grid), dim3(c1w::kThreads), c1w::kLds,
                       (hipStream_t)stream, x, hist, dy, part, bias_part, N);
    return (int)hipGetLastError();
  }
  if (hist) {
    hipLaunchKernelGGL(conv1_wgrad8_kernel<true>, dim3(grid), dim3(c1w::kThreads), c1w::kLds, (hipStream_t)stream, x,
                       hist, dy, part, bias_part, N);
  } else {
    hipLaunchKernelGGL(conv1_wgrad8_kernel<false>, dim3(grid), dim3(c1w::kThreads), c1w::kLds, (hipStream_t)stream, x,
                       hist, dy, part, bias_part, N);
  }
  return (int)hipGetLastError();
}
