// Weight-stationary value-function gradient on bf16 matrix cores with fp32 accuracy
// (K12 of SURVEY §2.6: compute_loss_vf + backward, REINFORCE.py:110-115,158-160).
//
// The value step runs train_vf_iters = 80 times per epoch (REINFORCE.py:110-115), so on the
// CartPole flagship it is ~96 % of the learner's GPU time.  mlp_grad.hip runs it on the
// fp32 MFMA (v_mfma_f32_16x16x4_f32: 1,024 MAC per 32 cycles); this kernel runs the three
// 128x128 products on v_mfma_f32_16x16x32_bf16 (8,192 MAC per 16 cycles) with every fp32
// operand split into three bf16 pieces, x = hi + mid + lo (each rounded to nearest, so
// |x - hi - mid - lo| <= 2^-24 |x|), and the six products whose weight is >= 2^-16 summed
// in the fp32 accumulator (small terms first):
//     a b ~ al bh + ah bl + am bm + am bh + ah bm + ah bh      (dropped: am bl, al bm, al bl <= 2^-23)
// i.e. fp32-level products (the bf16 x bf16 products are exact in fp32) at 6 x 16 = 96
// cycles per 16x16x32 step instead of 8 x 32 = 256.  tests/test_value_grad_gpu.py checks
// it against float64 and against the fp32-MFMA kernel.
//
// Work split (one persistent 8-wave workgroup per CU, 64-row batch slabs, 2 waves per
// SIMD): wave w OWNS hidden features [16w, 16w + 16) of both layers and computes them for all
// 64 rows, so its slices of W2 stay in registers for the whole launch, pre-split:
//     wA = W2[own rows][all 128]     (forward  h2 = W2 h1)
//     wB = W2[all 128][own cols]^T   (backward dh1 = W2^T dh2)
// (hi + mid pieces in registers; the lo pieces of W2 sit in one LDS image [o][i] that
// both fragment kinds read once per 32-wide k-chunk).  Activations cross waves through LDS
// as pre-split bf16 images [64 batch][128 feature] (row stride 144 elements with an XOR
// chunk swizzle: conflict-free b128 reads and transposed reads, 2-way stores):
//     h1 image  -> B operand of the forward (b128) and of dW2 (ds_read_b64_tr_b16)
//     dh2 image -> B operand of dh1 (b128) and A operand of dW2 (transposed)
// Each MFMA loop loads the next step's fragment before issuing the current step's six
// MFMAs.  dW2 for the wave's 16 rows accumulates in registers across all slabs; layer 1
// (K = D <= 24) is DP / 4 fp32 MFMA k-steps; dW1 / dW3 / biases are VALU outer products
// folded over the 16 batch lanes once per slab by a DPP reduce-scatter (lane j keeps entry
// j), which keeps their accumulators at one register each.  The head's NA dot products are
// reduced over the 8 waves through LDS.  4 workgroup barriers per slab.  The same body serves
// the value step and the policy steps (categorical and Gaussian heads, PG and PPO).
//
// Measured (tools/kbench.py grad, B = 2,097,152 rows, CartPole D = 4): 1.06 ms vs 1.91 ms for
// the fp32-MFMA kernel.  A ds_bpermute-based reduce-scatter gave run-to-run different dW1
// entries in one lane at D = 4 (tests/test_value_grad_gpu.py::test_deterministic); the DPP
// form is bitwise reproducible.
#include "common.h"
#include "grad_args.h"
#include "heads.h"

namespace rrl {

typedef __bf16 vbf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 vbf16x4 __attribute__((ext_vector_type(4)));
typedef short vs16x4 __attribute__((ext_vector_type(4)));

constexpr int kVgH = 128;
#ifndef VG_MT2
#define VG_MT2 1
#endif
constexpr int kVgLd = 144;          // bf16 row stride of the activation images
constexpr int kVgImg = 64 * kVgLd;  // elements per image piece
// LDS: h1 + dh2 images (3 pieces each), head partials [8 waves][NA][64], x slabs [2][64][DP],
// b1 / b2 / w3[NA], then the W2 lo image.  When the head partials do not fit beside the rest
// (Gaussian NA = 6 at DP >= 20) they live inside the dh2 image, which is free from the start
// of a slab until its dh2 stores -- one extra barrier orders their last read before those.
constexpr int vg_red_bytes(int NA) { return 8 * 64 * NA * 4; }
constexpr int vg_base_bytes(int DP, int NA) {
  return 6 * kVgImg * 2 + 2 * 64 * DP * 4 + (2 + NA) * 128 * 4 + 32 * 4 + kVgH * kVgLd * 2;
}
constexpr bool vg_red_in_image(int DP, int NA) { return vg_base_bytes(DP, NA) + vg_red_bytes(NA) > 160 * 1024; }
constexpr int vg_lds_bytes(int DP, int NA) {
  return vg_base_bytes(DP, NA) + (vg_red_in_image(DP, NA) ? 0 : vg_red_bytes(NA));
}
// Factored (rank-1) heads (see the kernel): the value head (DP <= 8), and the 2-action
// categorical policy heads, whose logit gradients sum to zero per row (dlogit0 = -dlogit1),
// so dh2 = dlogit1 (w3[1] - w3[0]) relu'(h2) is rank 1 like the value head's.  After the W2 lo
// image: the relu'(h2) mask of the slab as bytes [64 rows][4 lane groups][4 k-chunks] (byte =
// 8 features) and the table byte -> 8 bf16 {0, 1} [256][8] that turns a byte into a dh1 B
// fragment.
constexpr bool vg_factor(int DP, int HEAD, int NA) {
  // (the policy heads' DMA'd inputs leave room for the mask plan at DP = 4 only: CartPole)
  return (HEAD == HEAD_VALUE_MSE && DP <= 8) || ((HEAD == HEAD_PG_CAT || HEAD == HEAD_PPO_CAT) && NA == 2 && DP <= 4);
}
constexpr int vg_mask_bytes(int DP, int HEAD, int NA) { return vg_factor(DP, HEAD, NA) ? 64 * 16 + 256 * 16 : 0; }
// The slab's head inputs, DMA'd from global memory: ret, or adv / logp_old / act (actc [64][NA]
// for a Gaussian head).  Inside the dh2 image after the head partials when those live there.
// (Policy heads only: the value head keeps its x slab and ret prefetched in registers, which
// measured ~1-3 % faster there; the DMA path won 6 % on the register-starved Gaussian head.)
constexpr int vg_hbuf_bytes(int HEAD, int NA) {
  return HEAD == HEAD_VALUE_MSE ? 0 : 64 * 4 * (2 + ((HEAD == HEAD_PG_GAUSS || HEAD == HEAD_PPO_GAUSS) ? NA : 1));
}
// Gaussian heads with NA > 1 compute the head once per row (lane = (row, output), spread over
// the 8 waves) and hand dout to the dh2 phase through a [64][NA] table after the head inputs.
constexpr bool vg_split_head(int HEAD, int NA) {
  return (HEAD == HEAD_PG_GAUSS || HEAD == HEAD_PPO_GAUSS) && NA > 1;
}
// (+ the per-wave db3 / dlog_std sums [8][2 NA], accumulated in LDS across the slabs)
constexpr int vg_dtab_bytes(int HEAD, int NA) { return vg_split_head(HEAD, NA) ? (64 + 16) * NA * 4 : 0; }
// Factored heads: each wave's copy of the slab's dout [8 waves][64 rows] (the wave reads its
// own rows back as b128 / b32 LDS reads instead of 20 ds_bpermutes per slab), last in LDS.
// (Other value heads too, where LDS allows: 4 ds_bpermutes per slab there.)
constexpr int vg_dw_bytes(int DP, int HEAD, int NA) {
  return (vg_factor(DP, HEAD, NA) || (HEAD == HEAD_VALUE_MSE && vg_lds_bytes(DP, 1) + 8 * 64 * 4 <= 160 * 1024))
             ? 8 * 64 * 4
             : 0;
}
// Outside the image the head inputs are double-buffered (DMA'd a slab ahead) when LDS allows.
constexpr bool vg_hbuf2(int DP, int HEAD, int NA) {
  return !vg_red_in_image(DP, NA) && vg_lds_bytes(DP, NA) + vg_mask_bytes(DP, HEAD, NA) +
                                             2 * vg_hbuf_bytes(HEAD, NA) + vg_dtab_bytes(HEAD, NA) +
                                             vg_dw_bytes(DP, HEAD, NA) <=
                                         160 * 1024;
}
constexpr int vg_total_bytes(int DP, int HEAD, int NA) {
  return vg_lds_bytes(DP, NA) + vg_mask_bytes(DP, HEAD, NA) +
         (vg_red_in_image(DP, NA) ? 0 : (vg_hbuf2(DP, HEAD, NA) ? 2 : 1) * vg_hbuf_bytes(HEAD, NA)) +
         vg_dtab_bytes(HEAD, NA) + vg_dw_bytes(DP, HEAD, NA);
}
static_assert(vg_red_bytes(6) + vg_hbuf_bytes(HEAD_PPO_GAUSS, 6) <= 3 * kVgImg * 2, "head inputs in the dh2 image");
static_assert(vg_total_bytes(8, HEAD_VALUE_MSE, 1) <= 160 * 1024, "factored LDS plan");
static_assert(vg_total_bytes(4, HEAD_PG_CAT, 2) <= 160 * 1024 && vg_total_bytes(4, HEAD_PPO_CAT, 2) <= 160 * 1024,
              "factored binary policy LDS plan");
static_assert(vg_dw_bytes(20, HEAD_VALUE_MSE, 1) > 0 && vg_total_bytes(20, HEAD_VALUE_MSE, 1) <= 160 * 1024,
              "dout table of the D = 17..20 value kernel");
static_assert(vg_lds_bytes(24, 1) <= 160 * 1024 && !vg_red_in_image(24, 1), "value-grad LDS plan");
static_assert(vg_lds_bytes(20, 6) <= 160 * 1024, "value-grad LDS plan exceeds 160 KB");
static_assert(vg_red_bytes(6) <= 3 * kVgImg * 2, "head partials must fit in the dh2 image");

struct Split8 {
  vbf16x8 h, m, l;
};

struct Split8HM {  // hi + mid pieces (the lo piece of a stationary weight fragment lives in LDS)
  vbf16x8 h, m;
};

typedef float vf32x2 __attribute__((ext_vector_type(2)));

// Two fp32 -> packed bf16 pair (round to nearest even), a in the low half.  A vector
// conversion (lowers to v_cvt_pk_bf16_f32 on gfx950), not inline asm: the compiler's hazard
// recognizer does not see into asm, and an asm convert that reads an MFMA result got no
// wait states (a NaN-producing bug in cnn_fused.hip's first conv2 backward).
RRL_DEV uint32_t cvt_pk_bf16(float a, float b) {
  typedef __bf16 vbf16x2_cvt __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((vf32x2{a, b}), vbf16x2_cvt));
}
// The packed pair back as two fp32 (exact).
RRL_DEV vf32x2 unpack_bf16(uint32_t p) {
  vf32x2 f;
  f.x = __uint_as_float(p << 16);
  f.y = __uint_as_float(p & 0xffff0000u);
  return f;
}
// x = hi + mid + lo, each piece rounded to nearest: 3 converts, 2 unpacks and 2 packed
// subtracts per pair of values.
// (Scalar subtracts, not a packed v_pk_add_f32: packed f32 VALU beside MFMAs costs more.)
RRL_DEV void split2(vf32x2 v, uint32_t& h, uint32_t& m, uint32_t& lo) {
  h = cvt_pk_bf16(v.x, v.y);
  const float r1x = v.x - __uint_as_float(h << 16), r1y = v.y - __uint_as_float(h & 0xffff0000u);
  m = cvt_pk_bf16(r1x, r1y);
  const float r2x = r1x - __uint_as_float(m << 16), r2y = r1y - __uint_as_float(m & 0xffff0000u);
  lo = cvt_pk_bf16(r2x, r2y);
}
RRL_DEV void split4(const floatx4 v, vbf16x4& h, vbf16x4& m, vbf16x4& lo) {
  uint32_t h0, m0, l0, h1, m1, l1;
  split2(vf32x2{v[0], v[1]}, h0, m0, l0);
  split2(vf32x2{v[2], v[3]}, h1, m1, l1);
  h = __builtin_bit_cast(vbf16x4, make_uint2(h0, h1));
  m = __builtin_bit_cast(vbf16x4, make_uint2(m0, m1));
  lo = __builtin_bit_cast(vbf16x4, make_uint2(l0, l1));
}

RRL_DEV Split8 split8(const floatx4 v0, const floatx4 v1) {
  vbf16x4 h0, m0, l0, h1, m1, l1;
  split4(v0, h0, m0, l0);
  split4(v1, h1, m1, l1);
  Split8 s;
  s.h = __builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7);
  s.m = __builtin_shufflevector(m0, m1, 0, 1, 2, 3, 4, 5, 6, 7);
  s.l = __builtin_shufflevector(l0, l1, 0, 1, 2, 3, 4, 5, 6, 7);
  return s;
}


// max(x, 0) as ONE v_max_i32 on the bit pattern (negative floats, -0 included, are negative
// ints): fmaxf / fmed3 get a NaN-canonicalising max per value, a compare + select an SGPR pair.
// (Not inline asm: the compiler inserts no MFMA -> VALU wait states in front of an asm block,
// and these inputs come straight out of MFMAs.)
RRL_DEV float relu1(float x) { return __int_as_float(max(__float_as_int(x), 0)); }
// 1 if a relu1 output is non-zero, as an integer bit (no compare mask)
RRL_DEV uint32_t nonzero_bit(float x) { return min(__float_as_uint(x), 1u); }

RRL_DEV floatx4 mfma_bf16(vbf16x8 a, vbf16x8 b, floatx4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// fp32-accurate 16x16x32 step from split operands
RRL_DEV floatx4 mma6(const Split8& a, const Split8& b, floatx4 c) {
  c = mfma_bf16(a.l, b.h, c);
  c = mfma_bf16(a.h, b.l, c);
  c = mfma_bf16(a.m, b.m, c);
  c = mfma_bf16(a.m, b.h, c);
  c = mfma_bf16(a.h, b.m, c);
  return mfma_bf16(a.h, b.h, c);
}

// The same six products with the roles of the operands exchanged: the transposed tile
// (b supplies the A operand), e.g. dh1 with batch rows along the registers.
RRL_DEV floatx4 mma6t(const Split8& a, const Split8& b, floatx4 c) {
  c = mfma_bf16(b.h, a.l, c);
  c = mfma_bf16(b.l, a.h, c);
  c = mfma_bf16(b.m, a.m, c);
  c = mfma_bf16(b.h, a.m, c);
  c = mfma_bf16(b.m, a.h, c);
  return mfma_bf16(b.h, a.h, c);
}

// Element (row, col) of an activation image.  The 16-byte chunk index (col / 8) is XORed with
// (row / 4) mod 4: the C-layout stores (16 lanes = 16 consecutive rows, one 8-byte half chunk
// each) then fall 2-way on the 32 store banks instead of 4-way at the plain 72-dword row
// stride, while the b128 row reads stay conflict-free and the transposed reads (rows 4g + q,
// two half chunks per row) stay conflict-free too (bank maps in docs/KERNELS.md).
RRL_DEV int img_off(int row, int col) { return row * kVgLd + (((col >> 3) ^ ((row >> 2) & 3)) << 3) + (col & 7); }

// Sum over the 4 lane groups (lanes j, j+16, j+32, j+48) with VALU lane swaps (no LDS
// round trip, unlike __shfl_xor): a wave-uniform call site only (EXEC all ones).
RRL_DEV float group_sum_swap(float v) {
  const auto a = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  const float s = __uint_as_float(a[0]) + __uint_as_float(a[1]);
  const auto b = __builtin_amdgcn_permlane32_swap(__float_as_uint(s), __float_as_uint(s), false, false);
  return __uint_as_float(b[0]) + __uint_as_float(b[1]);
}

// Bitwise OR over the 4 lane groups (same lane swaps as group_sum_swap; wave-uniform call site).
RRL_DEV uint32_t group_or_swap(uint32_t v) {
  const auto a = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  const uint32_t s = a[0] | a[1];
  const auto b = __builtin_amdgcn_permlane32_swap(s, s, false, false);
  return b[0] | b[1];
}

// Sum over the whole wave on the VALU (DPP within 16-lane rows, lane swaps across rows):
// every lane gets the total; wave-uniform call sites only.
RRL_DEV float wave_sum_vl(float v);

// 8 consecutive features of batch row `row` (b128 read of each piece).
RRL_DEV Split8 frag_row(const uint16_t* img, int row, int col) {
  Split8 s;
  const uint16_t* a = img + img_off(row, col);
  s.h = *reinterpret_cast<const vbf16x8*>(a);
  s.m = *reinterpret_cast<const vbf16x8*>(a + kVgImg);
  s.l = *reinterpret_cast<const vbf16x8*>(a + 2 * kVgImg);
  return s;
}

// Batch-contracted fragment of column col0 + (lane & 15) from a [batch][feature] image:
// lane group g gets batch rows k0 + 4g + {0..3} and k0 + 16 + 4g + {0..3} (two transposed
// reads; rows 4 apart in one 32-lane half fall in disjoint bank halves at stride 144).
RRL_DEV vbf16x8 frag_tr1(const uint16_t* img, int k0, int col0, int lane) {
  typedef __attribute__((address_space(3))) vs16x4 lds_v4;
  const int q = (lane >> 2) & 3, pp = lane & 3, g = lane >> 4;
  const uint16_t* a0 = img + img_off(k0 + 4 * g + q, col0 + 4 * pp);  // row + 16: same swizzle
  const vs16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(a0));
  const vs16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(a0 + 16 * kVgLd));
  typedef short vs16x8 __attribute__((ext_vector_type(8)));
  const vs16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(vbf16x8, v);
}
// Rows k0 .. k0 + 7 of column col0 + (lane & 15) of a plain [k][col] image (k0 includes 8g).
RRL_DEV vbf16x8 frag_tr8(const uint16_t* img, int k0, int col0, int lane) {
  typedef __attribute__((address_space(3))) vs16x4 lds_v4;
  const int q = (lane >> 2) & 3, pp = lane & 3;
  const uint16_t* a0 = img + (k0 + q) * kVgLd + col0 + 4 * pp;
  const vs16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(a0));
  const vs16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4*)(a0 + 4 * kVgLd));
  typedef short vs16x8 __attribute__((ext_vector_type(8)));
  const vs16x8 v = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(vbf16x8, v);
}
RRL_DEV Split8 frag_tr(const uint16_t* img, int k0, int col0, int lane) {
  Split8 s;
  s.h = frag_tr1(img, k0, col0, lane);
  s.m = frag_tr1(img + kVgImg, k0, col0, lane);
  s.l = frag_tr1(img + 2 * kVgImg, k0, col0, lane);
  return s;
}

// Store a wave's C-layout tile (rows = 4 consecutive features of this lane, col = batch
// row) into the three pieces of a [batch][feature] image.
RRL_DEV void store_split(uint16_t* img, int row, int col, const floatx4 v) {
  vbf16x4 h, m, lo;
  split4(v, h, m, lo);
  uint16_t* a = img + img_off(row, col);
  *reinterpret_cast<vbf16x4*>(a) = h;
  *reinterpret_cast<vbf16x4*>(a + kVgImg) = m;
  *reinterpret_cast<vbf16x4*>(a + 2 * kVgImg) = lo;
}

// A C-layout tile's three packed bf16 pieces, and their store into an image.
struct Pieces {
  vbf16x4 h, m, l;
};
RRL_DEV void store_pieces(uint16_t* img, int row, int col, const Pieces& pc) {
  uint16_t* a = img + img_off(row, col);
  *reinterpret_cast<vbf16x4*>(a) = pc.h;
  *reinterpret_cast<vbf16x4*>(a + kVgImg) = pc.m;
  *reinterpret_cast<vbf16x4*>(a + 2 * kVgImg) = pc.l;
}

// Value of v from the partner lane selected by a DPP control (VALU cross-lane move, no LDS).
template <int CTRL>
RRL_DEV float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, true));
}
constexpr int kDppXor8 = 0x128;     // row_ror:8 (16-lane rows: lane ^ 8)
constexpr int kDppMirror8 = 0x141;  // row_half_mirror (lane ^ 7 within 8: flips bit 2)
constexpr int kDppXor2 = 0x4e;      // quad_perm [2,3,0,1]
constexpr int kDppXor1 = 0xb1;      // quad_perm [1,0,3,2]

// Sum of v[q] over the 16 lanes of this lane's row, for q = j only: recursive halving with
// DPP partner moves; at each step the partner differs in the bit that decides which half of
// the remaining entries a lane keeps, so lane j ends with entry j.
RRL_DEV float reduce_scatter16(const float (&v)[16], int j) {
  float u[8], w4[4], w2[2];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const bool hi = j & 8;
    const float send = hi ? v[k] : v[k + 8], keep = hi ? v[k + 8] : v[k];
    u[k] = keep + dpp_f<kDppXor8>(send);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const bool hi = j & 4;
    const float send = hi ? u[k] : u[k + 4], keep = hi ? u[k + 4] : u[k];
    w4[k] = keep + dpp_f<kDppMirror8>(send);
  }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const bool hi = j & 2;
    const float send = hi ? w4[k] : w4[k + 2], keep = hi ? w4[k + 2] : w4[k];
    w2[k] = keep + dpp_f<kDppXor2>(send);
  }
  const bool hi = j & 1;
  const float send = hi ? w2[0] : w2[1], keep = hi ? w2[1] : w2[0];
  return keep + dpp_f<kDppXor1>(send);
}

RRL_DEV float wave_sum_vl(float v) {
  v += dpp_f<kDppXor1>(v);
  v += dpp_f<kDppXor2>(v);
  v += dpp_f<kDppMirror8>(v);
  v += dpp_f<kDppXor8>(v);
  return group_sum_swap(v);
}

// HEAD: HEAD_VALUE_MSE (one output), a categorical policy head (HEAD_PG_CAT / HEAD_PPO_CAT,
// NA = 2..4 actions) or a diagonal-Gaussian policy head (HEAD_PG_GAUSS / HEAD_PPO_GAUSS, NA
// action dims, state-independent log_std): the same three 128x128 products, only the head
// (NA outputs reduced over the 8 waves, loss gradient, dW3 / db3 / dlog_std) differs.
// Diagnostic in-kernel stamps (STAMP = true builds only, tools/kbench.py --stamps): per-wave
// cycle sums of the slab's segments, written to p.stamps; never part of a timed run.
#define VG_STAMP(k)                                                                     \
  if (STAMP) {                                                                          \
    __builtin_amdgcn_sched_barrier(0);                                                  \
    unsigned long long t_;                                                              \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");          \
    __builtin_amdgcn_sched_barrier(0);                                                  \
    if ((k) > 0) st_sum[(k) > 0 ? (k)-1 : 0] += t_ - st_prev;                           \
    st_prev = t_;                                                                       \
  }

// Structural variants of the factored value head (template V, A/B-selectable at run time with
// tune bit 7, V = tune bits 4..6, tools/kbench.py --tunes): bit 0 = dh1 from the mask table without the dh2 barrier
// (else from the hi piece of dh2', rescaled by dout / hi(dout), after a barrier); bit 1 (with
// bit 0) = the dh2 tiles' vector work runs between dh1's MFMAs and dW1's between dW2's, so each
// wave's own matrix instructions cover it (otherwise the phases run one after the other).  (A
// bit-2 variant with fp32-MFMA dW1 at DP = 4 measured 905 vs 839 us and was removed.)
// production variant per input width (DP = 8 spills 4 VGPRs with the interleave)
constexpr int vg_prod_v(int DP) { return DP <= 4 ? 3 : 1; }

// FWD: the value forward only (layers 1 and 2 and the head dot product on the same
// weight-stationary bf16x6 layout, V written to p.vout; no loss, no backward, no slabs).
template <int DP, int HEAD, int NA, bool STAMP = false, int V = vg_prod_v(DP), bool FWD = false>
__global__ __launch_bounds__(512, 1) void value_grad_split_kernel(GradArgs p) {
  unsigned long long st_prev = 0, st_sum[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long st_entry = 0;  // STAMP: slots 10 / 11 = prologue / epilogue cycles per workgroup
  if (STAMP) asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_entry)::"memory");
  extern __shared__ __attribute__((aligned(16))) uint16_t vg_lds[];
  constexpr bool kValue = HEAD == HEAD_VALUE_MSE;
  constexpr bool kGauss = HEAD == HEAD_PG_GAUSS || HEAD == HEAD_PPO_GAUSS;
  constexpr bool kPPO = HEAD == HEAD_PPO_CAT || HEAD == HEAD_PPO_GAUSS;
  static_assert(!kValue || NA == 1, "the value head has one output");
  static_assert(!FWD || kValue, "the forward-only instance is the value head's");
  static_assert(NA >= 1 && NA <= 6, "NA <= 6 (LDS plan, two field groups)");
  static_assert(!vg_split_head(HEAD, NA) || (NA % 2 == 0 && NA <= 6),
                "the dout table is read in output pairs; head MFMA lanes g = 0, 1 hold outputs 0..7");
  // batch-summed 4-feature fields of the head / bias gradients, folded over the 16 batch
  // lanes by the DPP reduce-scatter: field 0 db2, 1 dW3 row 0, 2 (unused: db1 is summed in
  // the lane), 3 dW3 row 1, 4.. rows 2..
  // Value head, DP <= 8 (the flagship): dh2 = w3 (x) (relu'(h2) * dout) is rank-1 per row.
  // w3 folds into a stationary A' = W2^T diag(w3) and into the epilogue of dW2 / db2, so
  //  * dh1 = dout * (A' x mask) with the exact 0/1 mask relu'(h2): 3 MFMAs per step instead of
  //    6.  The mask goes to LDS as bits right after layer 2, so the head's barrier publishes it
  //    and dh1 needs no barrier of its own; a byte of 8 mask bits becomes a B fragment through
  //    a 256-entry table;
  //  * dW2 needs dh2' = mask * dout of the wave's OWN 16 features only (A operand): its image
  //    pieces are mask * the pieces of the row's dout (one split per row, not per element),
  //    written and read back by the same wave.
  constexpr bool kFactor = vg_factor(DP, HEAD, NA) && !FWD;
  // 2-action categorical heads: the factored path runs on w3' = w3[1] - w3[0] and the row
  // scalar d' = (dlogit1 - dlogit0) / 2 (their sum is zero up to fp32 rounding of p0 + p1 = 1)
  constexpr bool kBin = kFactor && !kValue;
  constexpr bool kMaskB = kFactor && (V & 1);
  constexpr bool kInterleave = kMaskB && (V & 2);
  constexpr int NF = NA + 2;
  constexpr int NG = (NF + 3) / 4;  // 16-slot groups (one register each)
  constexpr bool kRedImg = vg_red_in_image(DP, NA);
  constexpr bool kSplitHead = vg_split_head(HEAD, NA);
  uint16_t* h1img = vg_lds;
  uint16_t* dhimg = vg_lds + 3 * kVgImg;
  float* tail = reinterpret_cast<float*>(vg_lds + 6 * kVgImg);
  // [8 waves][NA][64 rows], or [8 waves][64 rows][NA] under kSplitHead
  float* red = kRedImg ? reinterpret_cast<float*>(dhimg) : tail;
  float* xsb = kRedImg ? tail : tail + 8 * NA * 64;                // [2][64 rows][DP]
  float* vecs = xsb + 2 * 64 * DP;                                 // b1[128] b2[128] w3[NA][128]
  uint16_t* w2lo = reinterpret_cast<uint16_t*>(vecs + (2 + NA) * kVgH + 32);  // [128][kVgLd]
  uint32_t* mk = reinterpret_cast<uint32_t*>(w2lo + kVgH * kVgLd);  // kFactor: mask bytes [64][4][4]
  const vbf16x8* mtab = reinterpret_cast<const vbf16x8*>(mk + 64 * 4);  // kFactor: [256]
  // head inputs of the current slab: [0, 64) ret or adv, [64, 128) logp_old, [128, ..) act
  // (int bits) or actc [64][NA]
  float* hbuf0 = kRedImg ? red + 8 * NA * 64
                         : reinterpret_cast<float*>(reinterpret_cast<char*>(mk) + vg_mask_bytes(DP, HEAD, NA));
  // kSplitHead: the slab's dout [64 rows][NA] (outside both images: read while dh2 is stored)
  float* dtab = reinterpret_cast<float*>(
      reinterpret_cast<char*>(mk) + vg_mask_bytes(DP, HEAD, NA) +
      (kRedImg ? 0 : (vg_hbuf2(DP, HEAD, NA) ? 2 : 1) * vg_hbuf_bytes(HEAD, NA)));
  float* hacc = dtab + 64 * NA;  // kSplitHead: [8 waves][db3[NA], dlog_std[NA]]
  if (kSplitHead && lane_id() < 2 * NA) hacc[(threadIdx.x >> 6) * 2 * NA + lane_id()] = 0.f;
  if (kMaskB) {
    // entry i: element e (feature 8 g + e of a fragment) = 1.0 if bit e of i is set
    for (int q = threadIdx.x; q < 256 * 4; q += blockDim.x) {
      const int i = q >> 2, e = 2 * (q & 3);
      mk[64 * 4 + q] = (((i >> e) & 1) ? 0x3F80u : 0u) | (((i >> (e + 1)) & 1) ? 0x3F800000u : 0u);
    }
  }
  int parity = 0;
  constexpr int KS1 = DP / 4;
  const int l = lane_id();
  const int j = l & 15, g = l >> 4, w = threadIdx.x >> 6;
  const int D = p.D;
  // rows >= Bv are inert (p.nvalid: a batch shape that changes between graph replays); p.B
  // stays the allocated capacity that every clamped load is bounded by
  const int Bv = p.nvalid ? min(*p.nvalid, p.B) : p.B;
  const int Bc = max(Bv, 1);  // x rows past Bv load duplicates of row Bv - 1 (finite data)
  const float invB = p.inv_B_dev ? *p.inv_B_dev : p.inv_B;
  const FlatOffsets o = flat_offsets(D, kVgH, NA);
  float adv_mean = 0.f, adv_rstd = 1.f;
  if (!kValue && p.adv_stats != nullptr) {
    const float n = fmaxf(p.adv_stats[2], 1.f);
    adv_mean = p.adv_stats[0] / n;
    const float var = fmaxf(p.adv_stats[1] / n - adv_mean * adv_mean, 0.f);
    adv_rstd = 1.f / (sqrtf(var) + 1e-8f);
  }
  const float* __restrict__ P = p.params;
  const int own = 16 * w;  // this wave's 16 hidden features

  // Global inputs go straight to LDS by DMA (global_load_lds_dword: lane l's dword lands at
  // the wave-uniform destination + 4 l), so no register holds them across the slab (held in
  // registers they were spilled under the Gaussian heads' pressure, and every spill store
  // waited for its HBM load).  The x slab [64][D] (compact, row stride D) is issued one slab
  // ahead into the other half of the double buffer; the head inputs at the top of their own
  // slab, behind ~6,000 cycles of layer 1 + layer 2.  The issuing waves wait for their DMAs
  // (vmcnt) before the barrier that publishes them.  Rows past B load clamped duplicates:
  // finite, and their dout is 0.
  constexpr int NC = kGauss ? NA : 1;
  const int wu = __builtin_amdgcn_readfirstlane(w);
  auto dma = [&](const void* src, long n, long first, float* dst, int chunks, int w0) {
    for (int k = 0; k < chunks; ++k) {
      if (((k + w0) & 7) == wu) {
        const long e = min(first + 64L * k + l, n - 1);
        __builtin_amdgcn_global_load_lds(static_cast<const uint32_t*>(src) + e,
                                         (__attribute__((address_space(3))) void*)(dst + 64 * k), 4, 0, 0);
      }
    }
  };
  // x slab by DMA in the [64][DP] layout: chunk k covers LDS floats 64 k .. 64 k + 63 and lane
  // l loads element (row q / DP, column min(q % DP, D - 1)) of q = 64 k + l, so a padding
  // column holds a finite duplicate -- layer 1 multiplies it by W1's zero padding and dW1's
  // padding outputs are never written.  (A compact stride-D layout needed per-read address
  // arithmetic and selects: +2,500 cycles per slab at D = 17.)
  // Value heads instead prefetch the x slab (XQ values per thread) and ret into registers a
  // slab ahead (issued right after the head, stored to LDS at the next slab's top).
  constexpr bool kDmaIn = !kValue;
  constexpr int XQ = (64 * DP + 511) / 512;
  float xr[kDmaIn ? 1 : XQ];
  float hin_r = 0.f;
  auto prefetch_x = [&](int b0, float* dst) {
    if (kDmaIn) {
      // this wave's chunks k = w, w + 8, ..: a runtime loop, so no per-chunk address is
      // hoisted out of the slab loop into a live register
      for (int k = wu; k < DP; k += 8) {
        const int q = 64 * k + l, row = q / DP, d = q % DP;
        const long e = (long)min(b0 + row, Bc - 1) * D + min(d, D - 1);
        __builtin_amdgcn_global_load_lds(static_cast<const uint32_t*>(static_cast<const void*>(p.X)) + e,
                                         (__attribute__((address_space(3))) void*)(dst + 64 * k), 4, 0, 0);
      }
    } else {
      // unconditional loads from clamped addresses: nothing here consumes a loaded value (a
      // select on it would make the compiler wait for the load right away)
#pragma unroll
      for (int i = 0; i < (kDmaIn ? 1 : XQ); ++i) {
        const int q = min((int)threadIdx.x + 512 * i, 64 * DP - 1);
        const int rl = q / DP, d = q % DP, b = b0 + rl;
        xr[i] = p.X[(size_t)min(b, Bc - 1) * D + min(d, D - 1)];
      }
      if (!FWD) hin_r = p.ret[min(b0 + l, p.B - 1)];
    }
  };
  constexpr bool kHb2 = kDmaIn && vg_hbuf2(DP, HEAD, NA);
  constexpr int HBF = vg_hbuf_bytes(HEAD, NA) / 4;  // floats per head-input buffer
  auto dma_head = [&](int b0, float* hbuf) {
    if (kDmaIn) {
      dma(p.adv, p.B, b0, hbuf, 1, 3);
      if (p.logp_old) dma(p.logp_old, p.B, b0, hbuf + 64, 1, 4);
      if (kGauss) dma(p.actc, (long)p.B * NA, (long)b0 * NA, hbuf + 128, NA, 5);
      else dma(p.act, p.B, b0, hbuf + 128, 1, 5);
    }
  };
  auto vm_wait0 = []() { __builtin_amdgcn_s_waitcnt(0x0F70); };  // vmcnt(0) only
  // the first slab's inputs go out before the weight loads of the prologue (which then hide
  // their latency) rather than after them
  prefetch_x(blockIdx.x * 64, xsb);
  if (kHb2) dma_head(blockIdx.x * 64, hbuf0);

  // ---------------------------------------------------------------- stationary weights
  // W2 is staged once in fp32 through the activation images (free until the first slab's
  // barrier): 8 b128 global loads per thread instead of ~130 element loads (the strided wB
  // columns and the w3 scale were one 4-byte load per lane each), and its lo pieces go to the
  // W2 lo image from the same registers.  Then each wave reads its fragments from LDS.
  // (Element loads when the params slice is not 16-byte aligned.)
  constexpr int kW2Ld = kVgH + 4;  // fp32 row stride of the staged W2 (16-byte rows, 2-way bank split)
  static_assert(kVgH * kW2Ld * 4 <= 6 * kVgImg * 2, "staged W2 must fit in the activation images");
  float* w2s = reinterpret_cast<float*>(vg_lds);
  // head scalars b3[NA], log_std[NA], 1/std[NA] in LDS after w3 (read once per slab by the head)
  float* hsc = vecs + (2 + NA) * kVgH;
  // (the other weights' loads go out with W2's, ahead of the staging barrier)
  float w1a[KS1];  // layer-1 A operand: W1[own + j][4s + g]
#pragma unroll
  for (int s = 0; s < KS1; ++s) {
    const int k = 4 * s + g;
    w1a[s] = (k < D) ? P[o.w1 + (own + j) * D + k] : 0.f;
  }
  {
    const float* gw2 = P + o.w2;
    const bool al16 = (reinterpret_cast<uintptr_t>(gw2) & 15) == 0;
    floatx4 v[kVgH * kVgH / 4 / 512];
#pragma unroll
    for (int it = 0; it < kVgH * kVgH / 4 / 512; ++it) {
      const int q = (int)threadIdx.x + 512 * it;  // float4 q: row q >> 5, columns 4 (q & 31) ..
      if (al16) {
        v[it] = *reinterpret_cast<const floatx4*>(gw2 + 4 * q);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[it][e] = gw2[4 * q + e];
      }
    }
    for (int q = threadIdx.x; q < (2 + NA) * kVgH; q += blockDim.x) {
      const int k = q >> 7, f = q & (kVgH - 1);
      vecs[q] = P[(k == 0 ? o.b1 : k == 1 ? o.b2 : o.w3 + (k - 2) * kVgH) + f];
    }
    if (threadIdx.x < NA) {
      const int a = threadIdx.x;
      const float lsa = kGauss ? P[o.log_std + a] : 0.f;
      hsc[a] = P[o.b3 + a];
      hsc[NA + a] = lsa;
      hsc[2 * NA + a] = __expf(-lsa);
    }
#pragma unroll
    for (int it = 0; it < kVgH * kVgH / 4 / 512; ++it) {
      const int q = (int)threadIdx.x + 512 * it;
      *reinterpret_cast<floatx4*>(w2s + (q >> 5) * kW2Ld + 4 * (q & 31)) = v[it];
      vbf16x4 h, m, lo;
      split4(v[it], h, m, lo);
      *reinterpret_cast<vbf16x4*>(w2lo + (q >> 5) * kVgLd + 4 * (q & 31)) = lo;
    }
  }
  __syncthreads();  // staged W2 and b1 / b2 / w3 visible
  // hi + mid pieces in registers; the lo pieces of W2 sit in the LDS image [o][i] that both
  // fragment kinds read once per 32-wide k-chunk (b128 for wA, transposed for wB)
  Split8HM wA[4], wB[4];
  // the factored path's w3' (value head: w3; 2-action policy: w3[1] - w3[0]), from LDS
  auto w3f = [&](int k) { return kBin ? vecs[3 * kVgH + k] - vecs[2 * kVgH + k] : vecs[2 * kVgH + k]; };
  vbf16x8 wBl[kFactor ? 4 : 1];  // lo pieces of A' (kFactor)
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    // wA: A[m = own + j][k = 32c + 8g + e] = W2[m][k]      (forward)
    const floatx4 a0 = *reinterpret_cast<const floatx4*>(w2s + (own + j) * kW2Ld + 32 * c + 8 * g);
    const floatx4 a1 = *reinterpret_cast<const floatx4*>(w2s + (own + j) * kW2Ld + 32 * c + 8 * g + 4);
    const Split8 sa = split8(a0, a1);
    wA[c].h = sa.h;
    wA[c].m = sa.m;
    if constexpr (!FWD) {
      floatx4 b0, b1;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        // wB: A[m = own + j][k = 32c + 8g + e] = W2[k][m]      (backward data)
        //     (kFactor: A'[m][k] = W2[k][m] * w3'[k])
        b0[e] = w2s[(32 * c + 8 * g + e) * kW2Ld + own + j];
        b1[e] = w2s[(32 * c + 8 * g + 4 + e) * kW2Ld + own + j];
        if (kFactor) {
          b0[e] *= w3f(32 * c + 8 * g + e);
          b1[e] *= w3f(32 * c + 8 * g + 4 + e);
        }
      }
      const Split8 sb = split8(b0, b1);
      wB[c].h = sb.h;
      wB[c].m = sb.m;
      if (kFactor) wBl[c % (kFactor ? 4 : 1)] = sb.l;
    }
  }
  // per C-layout row own + 4g + r (re-read from LDS where used)
  const float* b1p = vecs + own + 4 * g;
  const float* b2p = vecs + kVgH + own + 4 * g;
  const float* w3p = vecs + 2 * kVgH + own + 4 * g;

  floatx4 acc2[8];
  float accv[NG];      // slot j of each 16-slot group of fields (4 features each), batch-summed
  // dW1 / db1 from the TRANSPOSED dh1 tile (lane (j, g) holds rows 16 bt + 4 g + i of
  // feature own + j): summed inside the lane over the slabs, over the 4 lane groups once in
  // the epilogue.  DP = 4: vector FMAs on broadcast x rows; wider inputs: fp32 MFMA tiles.
  constexpr bool kDw1Mfma = DP > 4;
  // DP = 20 (D = 17..20): inputs 16..19 on the VALU beside the first tile's MFMAs (a second
  // 16-wide tile would be 3/4 padding and cost as much MFMA time as the first)
  constexpr int kTail1 = (DP > 16 && DP % 16 == 4) ? 4 : 0;
  constexpr int NT1 = kTail1 ? DP / 16 : (DP + 15) / 16;
  constexpr int NA1 = kDw1Mfma ? (kTail1 ? kTail1 : 1) : DP;
  float acc1[NA1];                    // dW1[own + j][d] (kTail1: d = 16 NT1 + e), this lane's rows
  floatx4 acc1m[kDw1Mfma ? NT1 : 1];  // dW1[own + 4 g + i][16 nt + j]
  float db1acc = 0.f;                 // db1[own + j], this lane's rows
#pragma unroll
  for (int it = 0; it < 8; ++it) acc2[it] = zero4();
#pragma unroll
  for (int q = 0; q < NG; ++q) accv[q] = 0.f;
#pragma unroll
  for (int d = 0; d < NA1; ++d) acc1[d] = 0.f;
#pragma unroll
  for (int nt = 0; nt < (kDw1Mfma ? NT1 : 1); ++nt) acc1m[nt] = zero4();
  // db3 / dlog_std: wave w owns output a = w (NA <= 8 waves) and keeps its batch sum in one
  // wave-uniform register, folded over the 64 rows of every slab on the VALU.  kSplitHead:
  // the wave folds its lanes (r, a) per output a and adds the sums to its slots of hacc.
  float bacc3 = 0.f, dls = 0.f;
  // factored value head: this lane's partials of the fields db2' (x w3 in the epilogue) and
  // dW3 row 0 for its 4 features, summed over all its slabs and folded over the 16 batch lanes
  // once, after the loop (a DPP reduce-scatter per slab cost ~45 vector instructions)
  // (DP = 4 only: at DP = 8 the kernel is at 253 VGPRs and the extra live partials measured
  // 122 -> 133 us at 262 k rows, while DP = 4 gained 826 -> 810 us at 2.1 M rows)
  constexpr bool kTvPersist = kFactor && DP == 4;
  float tvs[kFactor ? 16 : 1];
#pragma unroll
  for (int e = 0; e < (kFactor ? 16 : 1); ++e) tvs[e] = 0.f;
  // fields: 0 db2' (x w3' in the epilogue), 1 dW3 row 0, 3 dW3 row 1.  kBin: tvs[4..7] hold
  // sum d' h2 = dW3 row 1, and row 0 is its negative
  auto fold_tvs = [&]() {
    float tf[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      constexpr int TN = kFactor ? 16 : 1;
      if (!kFactor) tf[e] = 0.f;
      else if (!kBin) tf[e] = tvs[e % TN];
      else tf[e] = e < 4 ? tvs[e % TN] : e < 8 ? -tvs[e % TN] : e < 12 ? 0.f : tvs[(e - 8) % TN];
    }
    return reduce_scatter16(tf, j);
  };
  float s_loss = 0.f, s_val = 0.f, s_cnt = 0.f, s_ent = 0.f, s_kl = 0.f, s_clip = 0.f;

  if ((p.tune & 1) && __builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
  if ((p.tune & 2) && __builtin_amdgcn_readfirstlane(threadIdx.x) < 256) __builtin_amdgcn_s_setprio(1);

  VG_STAMP(0);
  if (STAMP) st_sum[10] = st_prev - st_entry;
  for (int base = blockIdx.x * 64; base < Bv; base += gridDim.x * 64) {
    VG_STAMP(0);
    // ------------------------------------------------------------ x slab (DMA'd a slab ago)
    // (double-buffered by slab parity: the next slab's DMA targets the other half)
    float* xs = xsb + (parity & 1) * 64 * DP;
    float* hbuf = hbuf0 + (kHb2 ? (parity & 1) * HBF : 0);
    parity ^= 1;
    if (kDmaIn) {
      vm_wait0();
    } else {
#pragma unroll
      for (int i = 0; i < (kDmaIn ? 1 : XQ); ++i) {
        const int q = (int)threadIdx.x + 512 * i;
        const int rl = q / DP, d = q % DP;
        if (q < 64 * DP) xs[q] = (base + rl < Bv && d < D) ? xr[i] : 0.f;
      }
    }
    __syncthreads();  // x (and kHb2 head inputs) visible; the previous slab's readers are done
    VG_STAMP(1);

    // ------------------------------------------------------------ layer 1 (fp32 MFMA)
    {
      // all x reads first, then the 4 tiles' MFMAs back to back, then relu + split + stores
      // (a read placed after the previous tile's image stores would wait for them: LDS alias)
      float xv[4][KS1];
#pragma unroll
      for (int bt = 0; bt < 4; ++bt) {
#pragma unroll
        for (int s = 0; s < KS1; ++s) xv[bt][s] = xs[(16 * bt + j) * DP + 4 * s + g];
      }
      const floatx4 b1v = *reinterpret_cast<const floatx4*>(b1p);
      floatx4 a1[4];
#pragma unroll
      for (int bt = 0; bt < 4; ++bt) {
        a1[bt] = b1v;
#pragma unroll
        for (int s = 0; s < KS1; ++s) a1[bt] = mfma4(w1a[s], xv[bt][s], a1[bt]);
      }
#pragma unroll
      for (int bt = 0; bt < 4; ++bt) {
#pragma unroll
        for (int r = 0; r < 4; ++r) a1[bt][r] = relu1(a1[bt][r]);
        store_split(h1img, 16 * bt + j, own + 4 * g, a1[bt]);
      }
    }
    __syncthreads();
    // this slab's head inputs (not double-buffered): issued after layer 1's barrier, which would
    // otherwise wait for them (vmcnt 0), and landed behind layer 2 (vm_wait0 before the head's)
    if (kDmaIn && !kHb2) dma_head(base, hbuf);

    VG_STAMP(2);
    // ------------------------------------------------------------ layer 2 (bf16x6 MFMA)
    floatx4 h2[4];
#pragma unroll
    for (int bt = 0; bt < 4; ++bt) h2[bt] = *reinterpret_cast<const floatx4*>(b2p);
    {
      // 16 steps (c, bt); the next step's B fragment (and W2-lo piece) load before this one's MFMAs
      Split8 cur = frag_row(h1img, j, 8 * g);
      vbf16x8 al = *reinterpret_cast<const vbf16x8*>(w2lo + (own + j) * kVgLd + 8 * g);
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        const int c = it >> 2, bt = it & 3;
        Split8 nxt;
        vbf16x8 aln;
        if (it + 1 < 16) nxt = frag_row(h1img, 16 * ((it + 1) & 3) + j, 32 * ((it + 1) >> 2) + 8 * g);
        if (bt == 3 && it + 1 < 16)
          aln = *reinterpret_cast<const vbf16x8*>(w2lo + (own + j) * kVgLd + 32 * (c + 1) + 8 * g);
        const Split8 a{wA[c].h, wA[c].m, al};
        h2[bt] = mma6(a, cur, h2[bt]);
        __builtin_amdgcn_sched_barrier(0);
        if (it + 1 < 16) cur = nxt;
        if (bt == 3 && it + 1 < 16) al = aln;
      }
    }
#pragma unroll
    for (int bt = 0; bt < 4; ++bt) {
#pragma unroll
      for (int r = 0; r < 4; ++r) h2[bt][r] = relu1(h2[bt][r]);
    }
    if (kMaskB) {
      // relu'(h2) bits for dh1's B fragments.  Byte (row, g', c') holds features 32 c' + 8 g' +
      // {0..7}; this wave's features own + {0..7} / {8..15} are bytes (c' = w / 2, g' = 2 (w & 1)
      // + 0 / 1).  The 4 lane groups' nibbles of rows 16 bt + j are OR-ed together, then lane
      // group g writes the 16 bits of row 16 g + j.
      uint32_t x01 = 0, x23 = 0;
#pragma unroll
      for (int bt = 0; bt < 4; ++bt) {
        uint32_t nib = 0;
#pragma unroll
        for (int r = 0; r < 4; ++r) nib |= (h2[bt][r] > 0.f ? 1u : 0u) << r;
        const uint32_t sh = 4 * g + 16 * (bt & 1);
        if (bt < 2) x01 |= nib << sh;
        else x23 |= nib << sh;
      }
      x01 = group_or_swap(x01);
      x23 = group_or_swap(x23);
      const uint32_t u = ((g < 2 ? x01 : x23) >> (16 * (g & 1))) & 0xffffu;
      uint8_t* mb = reinterpret_cast<uint8_t*>(mk) + (16 * g + j) * 16 + 8 * (w & 1) + (w >> 1);
      mb[0] = (uint8_t)(u & 0xffu);
      mb[4] = (uint8_t)(u >> 8);
    }

    VG_STAMP(3);
    // ------------------------------------------------------------ head
    // partial dot products over this wave's 16 features -> LDS, reduced over the 8 waves
    if constexpr (kSplitHead) {
      // on fp32 MFMA (exact fp32 products): C[a][row] = sum_k W3[a][k] h2[row][k] over the
      // wave's features k, A = W3 row a = lane & 15 (zero past NA), B = the h2 tile as it sits
      // in C layout (k = own + 4 g + r over the 4 steps r, n = row 16 bt + j).  Lane (j, g)
      // gets outputs 4 g + i of row 16 bt + j: one sum over the lane groups per MFMA instead
      // of NA dot products + lane-swap sums on the VALU
      floatx4 w3m = zero4();
      if (j < NA) w3m = *reinterpret_cast<const floatx4*>(w3p + j * kVgH);
#pragma unroll
      for (int bt = 0; bt < 4; ++bt) {
        floatx4 c = zero4();
#pragma unroll
        for (int r = 0; r < 4; ++r) c = mfma4(w3m[r], h2[bt][r], c);
        float* dst = red + (w * 64 + 16 * bt + j) * NA + 4 * g;
        if (g == 0) {
          *reinterpret_cast<vf32x2*>(dst) = vf32x2{c[0], c[1]};
          *reinterpret_cast<vf32x2*>(dst + 2) = vf32x2{c[2], c[3]};
        } else if (4 * g < NA) {
          *reinterpret_cast<vf32x2*>(dst) = vf32x2{c[0], c[1]};
        }
      }
    } else {
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      const floatx4 w3a = *reinterpret_cast<const floatx4*>(w3p + a * kVgH);
#pragma unroll
      for (int bt = 0; bt < 4; ++bt) {
        float pv = w3a[0] * h2[bt][0];
        pv = fmaf(w3a[1], h2[bt][1], pv);
        pv = fmaf(w3a[2], h2[bt][2], pv);
        pv = fmaf(w3a[3], h2[bt][3], pv);
        pv = group_sum_swap(pv);
        if (g == bt) red[(w * NA + a) * 64 + 16 * bt + j] = pv;
      }
      if (NA > 2) __builtin_amdgcn_sched_barrier(0);
    }
    }
    VG_STAMP(4);
    if (kDmaIn && !kHb2) vm_wait0();  // this wave's head-input DMAs
    __syncthreads();
    VG_STAMP(5);
    if constexpr (FWD) {
      // V of row l (wave 0): the 8 waves' partials in the grad kernel's summation order + b3
      if (w == 0 && base + l < Bv) {
        const float* r = red + l;
        p.vout[base + l] = (((r[0] + r[64]) + (r[128] + r[192])) + ((r[256] + r[320]) + (r[384] + r[448]))) + hsc[0];
      }
      // next slab's x into registers (nothing else of this slab is read after the barrier
      // above; the next slab's own barriers order its LDS writes after these reads)
      if (base + (int)gridDim.x * 64 < Bv) prefetch_x(base + gridDim.x * 64, xsb + (parity & 1) * 64 * DP);
      continue;
    }
    // loss head: lane l handles batch row l (every wave computes the same 64 rows; wave 0's
    // lanes count each row once in the batch statistics and the head gradient sums)
    const bool lead = w == 0;
    float dout[NA];
    float dls_row[kGauss ? NA : 1];  // this row's dLoss/dlog_std terms (Gaussian heads)
    if constexpr (kSplitHead) {
      // Gaussian head, NA > 1: lane (r, a) = (l >> 3, l & 7) of wave w takes output a of row
      // 8 w + r, so each of the 64 x NA terms is computed once instead of in every wave; a
      // row's log-prob / entropy is summed over its 8 lanes by DPP, and dout goes to the
      // table that the barrier below publishes to every wave's dh2 phase
      const int a8 = l & 7, R = 8 * w + (l >> 3);
      const bool va = a8 < NA;
      const int ac = min(a8, NA - 1);
      const bool ok = base + R < Bv;
      const float* rr = red + R * NA + ac;
      constexpr int S = 64 * NA;  // wave stride
      const float outv = (((rr[0] + rr[S]) + (rr[2 * S] + rr[3 * S])) + ((rr[4 * S] + rr[5 * S]) + (rr[6 * S] + rr[7 * S]))) +
                         hsc[ac];
      const float hin = hbuf[R], hlp = hbuf[64 + R];
      const float lsd = hsc[NA + ac], istd = hsc[2 * NA + ac];
      // dlogp/dmu = d / var ; dlogp/dlog_std = d^2 / var - 1 ; dH/dlog_std = 1
      const float d = (ok ? hbuf[128 + R * NA + ac] : outv) - outv;
      const float z = d * istd;
      float logp = va ? -0.5f * z * z - lsd - kHalfLog2Pi : 0.f;
      float ent = va ? 0.5f + kHalfLog2Pi + lsd : 0.f;
      logp += dpp_f<kDppXor1>(logp);
      ent += dpp_f<kDppXor1>(ent);
      logp += dpp_f<kDppXor2>(logp);
      ent += dpp_f<kDppXor2>(ent);
      logp += dpp_f<kDppMirror8>(logp);
      ent += dpp_f<kDppMirror8>(ent);
      const float adv = ((ok ? hin : 0.f) - adv_mean) * adv_rstd;
      float dlogp, loss_i;
      if (!kPPO) {
        dlogp = -adv;
        loss_i = -logp * adv;
      } else {
        const float lpo = (ok && p.logp_old) ? hlp : logp;
        const float ratio = __expf(logp - lpo);
        const float s1 = ratio * adv;
        const float s2 = fminf(fmaxf(ratio, 1.f - p.clip_eps), 1.f + p.clip_eps) * adv;
        dlogp = (s1 <= s2) ? -adv * ratio : 0.f;
        loss_i = -fminf(s1, s2);
        if (a8 == 0 && ok) s_clip += (fabsf(ratio - 1.f) > p.clip_eps) ? 1.f : 0.f;
      }
      const float scale = (ok && va) ? invB : 0.f;
      const float iv = istd * istd;
      const float da = scale * dlogp * d * iv;
      const float dl = scale * (dlogp * (d * d * iv - 1.f) - p.ent_coef);
      if (va) dtab[R * NA + a8] = da;
      // this wave's sums of output a (lanes a + 8 r) into its LDS slots (a VGPR accumulator per
      // lane would cost registers the DP = 20 kernel spills for; the wave-uniform ones did not)
      const float hb = group_sum_swap(da + dpp_f<kDppXor8>(da));
      const float hl = group_sum_swap(dl + dpp_f<kDppXor8>(dl));
      if (l < NA) {
        hacc[w * 2 * NA + l] += hb;
        hacc[w * 2 * NA + NA + l] += hl;
      }
      if (a8 == 0 && ok) {
        s_loss += loss_i;
        s_ent += ent;
        if (p.logp_old) s_kl += hlp - logp;
        s_cnt += 1.f;
      }
    } else {
      const int b = base + l;
      const bool ok = b < Bv;
      const int bc = min(b, p.B - 1);
      const float hin = kDmaIn ? hbuf[l] : hin_r;
      const float hlp = kValue ? 0.f : hbuf[64 + l];
      const int hact = (kValue || kGauss) ? 0 : __float_as_int(hbuf[128 + l]);
      float hac[NC];
#pragma unroll
      for (int a = 0; a < NC; ++a) hac[a] = kGauss ? hbuf[128 + l * NC + a] : 0.f;
      float outv[NA];
#pragma unroll
      for (int a = 0; a < NA; ++a) {
        const float* r = red + a * 64 + l;
        constexpr int S = NA * 64;  // wave stride
        outv[a] = (((r[0] + r[S]) + (r[2 * S] + r[3 * S])) + ((r[4 * S] + r[5 * S]) + (r[6 * S] + r[7 * S]))) + hsc[a];
      }
      if (kValue) {
        const float v = outv[0];
        const float diff = v - (ok ? hin : 0.f);
        dout[0] = ok ? 2.f * diff * invB : 0.f;
        if (lead && ok) {
          s_loss += diff * diff;
          s_val += v;
          s_cnt += 1.f;
        }
      } else {
        // policy heads (mlp_grad.hip HEAD_PG_* / HEAD_PPO_*, REINFORCE.py:141-152)
        const float adv = ((ok ? hin : 0.f) - adv_mean) * adv_rstd;
        float logp = 0.f, ent = 0.f;
        float logits[kMaxAct];
        CatStats cs{0.f, 0.f};
        int act = 0;
        if (kGauss) {
#pragma unroll
          for (int a = 0; a < NA; ++a) {
            const float xa = ok ? hac[a % NC] : outv[a];
            const float z = (xa - outv[a]) * hsc[2 * NA + a];
            logp += -0.5f * z * z - hsc[NA + a] - kHalfLog2Pi;
            ent += 0.5f + kHalfLog2Pi + hsc[NA + a];
          }
        } else {
#pragma unroll
          for (int a = 0; a < kMaxAct; ++a) logits[a] = a < NA ? outv[a] : -INFINITY;
          if (ok) apply_mask(p.mask ? p.mask + (size_t)bc * NA : nullptr, NA, logits);
          cs = cat_stats(NA, logits);
          act = ok ? hact : 0;
          logp = pick_logit(NA, logits, act) - cs.lse;
          ent = cs.entropy;
        }
        float dlogp, loss_i;
        if (!kPPO) {
          dlogp = -adv;
          loss_i = -logp * adv;
        } else {
          const float lpo = (ok && p.logp_old) ? hlp : logp;
          const float ratio = __expf(logp - lpo);
          const float s1 = ratio * adv;
          const float s2 = fminf(fmaxf(ratio, 1.f - p.clip_eps), 1.f + p.clip_eps) * adv;
          dlogp = (s1 <= s2) ? -adv * ratio : 0.f;
          loss_i = -fminf(s1, s2);
          if (lead && ok) s_clip += (fabsf(ratio - 1.f) > p.clip_eps) ? 1.f : 0.f;
        }
        const float scale = ok ? invB : 0.f;
#pragma unroll
        for (int a = 0; a < NA; ++a) {
          if (kGauss) {
            // dlogp/dmu = d / var ; dlogp/dlog_std = d^2 / var - 1 ; dH/dlog_std = 1
            const float d = (ok ? hac[a % NC] : outv[a]) - outv[a];
            const float iv = hsc[2 * NA + a] * hsc[2 * NA + a];
            dout[a] = scale * dlogp * d * iv;
            dls_row[a % NC] = scale * (dlogp * (d * d * iv - 1.f) - p.ent_coef);
          } else {
            const float lpa = logits[a] - cs.lse;
            const float pa = __expf(lpa);
            const float dpg = dlogp * ((a == act ? 1.f : 0.f) - pa);
            const float dent = pa > 0.f ? p.ent_coef * pa * (lpa + cs.entropy) : 0.f;
            dout[a] = scale * (dpg + dent);
          }
        }
        if (lead && ok) {
          s_loss += loss_i;
          s_ent += ent;
          if (p.logp_old) s_kl += hlp - logp;
          s_cnt += 1.f;
        }
      }
      float mb = 0.f, ml = 0.f;  // this wave's output
#pragma unroll
      for (int a = 0; a < NA; ++a) {
        if (a == w) {
          mb = dout[a];
          if (kGauss) ml = dls_row[a % NC];
        }
      }
      if (w < NA) {  // wave-uniform
        bacc3 += wave_sum_vl(mb);
        if (kGauss) dls += wave_sum_vl(ml);
      }
    }
    // the head consumed this slab's inputs: issue the next slab's x DMA now -- after the barrier
    // below where there is one: __syncthreads waits for every outstanding vector memory op
    // (vmcnt 0), so a DMA issued just before it would stall the slab for its HBM latency
    auto prefetch_next = [&]() {
      if (base + (int)gridDim.x * 64 < Bv) {
        prefetch_x(base + gridDim.x * 64, xsb + (parity & 1) * 64 * DP);
        if (kHb2) dma_head(base + gridDim.x * 64, hbuf0 + (parity & 1) * HBF);
      }
    };
    constexpr bool kHeadBar = kRedImg || kSplitHead;
    if (!kHeadBar && kFactor) prefetch_next();  // (V1 / V3: no barrier before the next slab's)
    // every wave read the partials before dh2 overwrites them (kSplitHead: the dout table is visible)
    if (kHeadBar) {
      __syncthreads();
      prefetch_next();
    }

    VG_STAMP(6);
    // ------------------------------------------------------------ dh2, dW3, db2 / dh1, db1
    // dh1 comes out TRANSPOSED (its MFMAs take the batch-side fragment as the A operand): lane
    // (j, g) holds dh1[row 16 bt + 4 g + i][feature own + j], i = 0..3.
    floatx4 dh1[4];
#pragma unroll
    for (int bt = 0; bt < 4; ++bt) dh1[bt] = zero4();
    // relu'(h1) of the transposed tile from the h1 image's hi piece (h1 >= 0: hi != 0 iff
    // h1 > 0), two transposed reads give this lane's 16 rows; then the db1 partial
    auto dh1_relu = [&]() {
#pragma unroll
      for (int cc = 0; cc < 2; ++cc) {
        typedef unsigned short vu16x8 __attribute__((ext_vector_type(8)));
        const vu16x8 hb = __builtin_bit_cast(vu16x8, frag_tr1(h1img, 32 * cc, own, l));
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int bt = 2 * cc + (e >> 2), i = e & 3;
          dh1[bt][i] = hb[e] != 0 ? dh1[bt][i] : 0.f;
          db1acc += dh1[bt][i];
        }
      }
    };
    // the wave's dout table (lane l writes row l; only this wave reads it back): kMaskB and the
    // non-factored value heads
    constexpr bool kDwTab = vg_dw_bytes(DP, HEAD, NA) > 0 && (kMaskB || !kFactor);
    float* dtw = reinterpret_cast<float*>(reinterpret_cast<char*>(vg_lds) + vg_total_bytes(DP, HEAD, NA) -
                                          vg_dw_bytes(DP, HEAD, NA)) + 64 * w;
    if (kFactor) {
      // the row scalar of the rank-1 dh2: dout (value) or (dlogit1 - dlogit0) / 2 (kBin)
      const float dfac = kBin ? 0.5f * (dout[NA - 1] - dout[0]) : dout[0];
      float dv[4];  // dfac of C-layout row 16 bt + j (the dh2' tiles)
      if (kMaskB) {
        dtw[l] = dfac;
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int bt = 0; bt < 4; ++bt) dv[bt] = dtw[16 * bt + j];
      } else {
#pragma unroll
        for (int bt = 0; bt < 4; ++bt) dv[bt] = __shfl(dfac, 16 * bt + j, 64);
      }
      float* tv = tvs;  // fields: db2' (x w3 in the epilogue), dW3 row 0 (kTvPersist: kept over slabs)
      if (!kTvPersist) {
#pragma unroll
        for (int e = 0; e < 16; ++e) tvs[e % (kFactor ? 16 : 1)] = 0.f;
      }
      // dh2' pieces of batch tile bt (stores) and its field partials
      auto kf_tile = [&](const int bt) {
        const float v = dv[bt];
        // the row's dout split once: v = vh + vm + vl
        uint32_t ph, pm, pl;
        split2(vf32x2{v, v}, ph, pm, pl);
        uint32_t mw[2];  // relu'(h2) of this lane's 4 features as bf16 lane masks
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const bool p0 = h2[bt][2 * q] > 0.f, p1 = h2[bt][2 * q + 1] > 0.f;
          mw[q] = (p0 ? 0x0000ffffu : 0u) | (p1 ? 0xffff0000u : 0u);
        }
        Pieces pc;
        pc.h = __builtin_bit_cast(vbf16x4, make_uint2(mw[0] & ph, mw[1] & ph));
        pc.m = __builtin_bit_cast(vbf16x4, make_uint2(mw[0] & pm, mw[1] & pm));
        pc.l = __builtin_bit_cast(vbf16x4, make_uint2(mw[0] & pl, mw[1] & pl));
        store_pieces(dhimg, 16 * bt + j, own + 4 * g, pc);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          tv[r] += h2[bt][r] > 0.f ? v : 0.f;
          tv[4 + r] = fmaf(v, h2[bt][r], tv[4 + r]);
        }
      };
      auto kf_finish = [&]() {
        if (!kTvPersist) accv[0] += fold_tvs();
        if (kMaskB) {
          // the dh2' image is read back (dW2) only by the wave that wrote it: in-order LDS
          __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
          __builtin_amdgcn_wave_barrier();
        }
      };
      auto kf_dh2 = [&]() {
#pragma unroll
        for (int bt = 0; bt < 4; ++bt) kf_tile(bt);
        kf_finish();
      };
      auto kf_dh1 = [&]() {
        if (kMaskB) {
          // dh1^T = dout * (mask x A'^T), exact: the mask fragment of (k-chunk c, batch tile
          // bt) is the table entry of byte (row 16 bt + j, g, c); a row's 4 bytes are one dword
          uint32_t mrow[4];
#pragma unroll
          for (int bt = 0; bt < 4; ++bt) mrow[bt] = mk[(16 * bt + j) * 4 + g];
          // table fragments read two steps ahead (VG_MT2): one step of 3 MFMAs did not cover
          // the LDS latency (an lgkmcnt(0) wait before every step)
          constexpr int kAhead = VG_MT2 ? 2 : 1;
          auto mfrag = [&](int it) { return mtab[(mrow[it & 3] >> (8 * (it >> 2))) & 0xffu]; };
          vbf16x8 q0 = mfrag(0), q1;
          if (kAhead == 2) q1 = mfrag(1);
#pragma unroll
          for (int it = 0; it < 16; ++it) {
            const int c = it >> 2, bt = it & 3;
            vbf16x8 nxt;
            if (it + kAhead < 16) nxt = mfrag(it + kAhead);
            dh1[bt] = mfma_bf16(q0, wBl[c % (kFactor ? 4 : 1)], dh1[bt]);
            dh1[bt] = mfma_bf16(q0, wB[c].m, dh1[bt]);
            dh1[bt] = mfma_bf16(q0, wB[c].h, dh1[bt]);
            if (kInterleave) {  // this wave's dh2 work beside its own MFMAs
              if ((it & 3) == 1) kf_tile(it >> 2);
              if (it == 15) kf_finish();
            }
            __builtin_amdgcn_sched_barrier(0);
            if (kAhead == 2) {
              q0 = q1;
              if (it + 2 < 16) q1 = nxt;
            } else if (it + 1 < 16) {
              q0 = nxt;
            }
          }
        } else {
          // dh1^T = rr * (hi(dh2') x A'^T): the hi piece alone is exact (mask * hi(dout))
          vbf16x8 cur = *reinterpret_cast<const vbf16x8*>(dhimg + img_off(j, 8 * g));
#pragma unroll
          for (int it = 0; it < 16; ++it) {
            const int c = it >> 2, bt = it & 3;
            vbf16x8 nxt;
            if (it + 1 < 16)
              nxt = *reinterpret_cast<const vbf16x8*>(
                  dhimg + img_off(16 * ((it + 1) & 3) + j, 32 * ((it + 1) >> 2) + 8 * g));
            dh1[bt] = mfma_bf16(cur, wBl[c % (kFactor ? 4 : 1)], dh1[bt]);
            dh1[bt] = mfma_bf16(cur, wB[c].m, dh1[bt]);
            dh1[bt] = mfma_bf16(cur, wB[c].h, dh1[bt]);
            __builtin_amdgcn_sched_barrier(0);
            if (it + 1 < 16) cur = nxt;
          }
        }
        // per-row scale of the transposed tile (rows 16 bt + 4 g + i): dfac, or dfac / hi(dfac)
        float sr = dfac;  // lane l: row l
        if (!kMaskB) {
          const float vh = __uint_as_float(cvt_pk_bf16(sr, sr) << 16);
          sr = vh != 0.f ? sr * __builtin_amdgcn_rcpf(vh) : 0.f;  // 1 ulp: within fp32 accuracy
        }
        if (kMaskB) {
          // rows 16 bt + 4 g .. + 3 of the wave's dout table: one b128 read per batch tile
#pragma unroll
          for (int bt = 0; bt < 4; ++bt) {
            const floatx4 d4 = *reinterpret_cast<const floatx4*>(dtw + 16 * bt + 4 * g);
#pragma unroll
            for (int i = 0; i < 4; ++i) dh1[bt][i] *= d4[i];
          }
        } else {
#pragma unroll
          for (int bt = 0; bt < 4; ++bt) {
#pragma unroll
            for (int i = 0; i < 4; ++i) dh1[bt][i] *= __shfl(sr, 16 * bt + 4 * g + i, 64);
          }
        }
        dh1_relu();
      };
      if (kInterleave) {
        VG_STAMP(7);
        kf_dh1();  // (with the dh2 tiles inside)
      } else {
        kf_dh2();
        if (!kMaskB) __syncthreads();  // dh1 reads every wave's hi(dh2') features
        VG_STAMP(7);
        kf_dh1();
      }
    } else {
      // dout of batch row 16 bt + j comes from lane 16 bt + j (ds_bpermute, no barrier).  Field
      // group 0 (db2, dW3 rows 0 / 1) is folded first; the rows of outputs 2.. (group 1) in a
      // second pass, so only 16 partials are live at a time.
      // kSplitHead: dout comes from the table instead, as pairs (a, a + 1) of rows 16 bt + j (b64
      // reads), one pair at a time (sched barrier: hoisted together the reads held 24 registers
      // and the DP = 20 kernel spilled for them; a pair read ahead spilled too)
      floatx4 dd[4];
      if constexpr (kSplitHead) {
        // dd = dout x W3 on fp32 MFMA over k = outputs 4 s + g: A = W3[4 s + g][own + j], B =
        // dout[row 16 bt + j][4 s + g] from the table; C comes out in h2's layout (lane (j, g):
        // features own + 4 g + i of row 16 bt + j)
        const float* w3v = vecs + 2 * kVgH + own + j;
        const float wk0 = g < NA ? w3v[g * kVgH] : 0.f;
        const float wk1 = 4 + g < NA ? w3v[(4 + g) * kVgH] : 0.f;
#pragma unroll
        for (int bt = 0; bt < 4; ++bt) {
          const float* dr = dtab + (16 * bt + j) * NA;
          const float b0 = g < NA ? dr[g] : 0.f;
          const float b1 = 4 + g < NA ? dr[4 + g] : 0.f;
          dd[bt] = mfma4(wk1, b1, mfma4(wk0, b0, zero4()));
        }
      } else {
#pragma unroll
        for (int bt = 0; bt < 4; ++bt) dd[bt] = zero4();
      }
      auto tab_pair = [&](int a2, vf32x2(&q)[4]) {
#pragma unroll
        for (int bt = 0; bt < 4; ++bt) q[bt] = *reinterpret_cast<const vf32x2*>(dtab + (16 * bt + j) * NA + a2);
      };
      vf32x2 vq[4];
      if (kDwTab) {
        dtw[l] = dout[0];
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
      }
      {
        float tv[16];  // this slab's field partials of features own + 4g + r
#pragma unroll
        for (int e = 0; e < 16; ++e) tv[e] = 0.f;
#pragma unroll
        for (int a = 0; a < NA; ++a) {
          if (kSplitHead && (a & 1) == 0) tab_pair(a, vq);
          const floatx4 w3a = kSplitHead ? zero4() : *reinterpret_cast<const floatx4*>(w3p + a * kVgH);
          const int f = a == 0 ? 1 : 3;
#pragma unroll
          for (int bt = 0; bt < 4; ++bt) {
            const float v = kSplitHead ? vq[bt][a & 1] : kDwTab ? dtw[16 * bt + j] : __shfl(dout[a], 16 * bt + j, 64);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              if (!kSplitHead) dd[bt][r] = fmaf(w3a[r], v, dd[bt][r]);
              if (a < 2) tv[4 * f + r] = fmaf(v, h2[bt][r], tv[4 * f + r]);
            }
          }
          if (kSplitHead && (a & 1)) __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int bt = 0; bt < 4; ++bt) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            dd[bt][r] = h2[bt][r] > 0.f ? dd[bt][r] : 0.f;
            tv[r] += dd[bt][r];
          }
          store_split(dhimg, 16 * bt + j, own + 4 * g, dd[bt]);
        }
        accv[0] += reduce_scatter16(tv, j);
      }
      if (NA > 2) {
        float tv[16];
#pragma unroll
        for (int e = 0; e < 16; ++e) tv[e] = 0.f;
#pragma unroll
        for (int a = 2; a < NA; ++a) {
          if (kSplitHead && (a & 1) == 0) tab_pair(a, vq);
          const int f = a + 2;  // fields 4 .. NA + 1 -> group 1 (NA <= 6)
#pragma unroll
          for (int bt = 0; bt < 4; ++bt) {
            const float v = kSplitHead ? vq[bt][a & 1] : __shfl(dout[a], 16 * bt + j, 64);
#pragma unroll
            for (int r = 0; r < 4; ++r) tv[4 * (f & 3) + r] = fmaf(v, h2[bt][r], tv[4 * (f & 3) + r]);
          }
          if (kSplitHead && (a & 1)) __builtin_amdgcn_sched_barrier(0);
        }
        accv[1] += reduce_scatter16(tv, j);
      }
      __syncthreads();
      if (!kHeadBar) prefetch_next();  // after the dh2 barrier, for the same reason
      VG_STAMP(7);
      // dh1^T (own features) = dh2 x W2
      Split8 cur = frag_row(dhimg, j, 8 * g);
      vbf16x8 bl = frag_tr8(w2lo, 8 * g, own, l);
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        const int c = it >> 2, bt = it & 3;
        Split8 nxt;
        vbf16x8 bln;
        if (it + 1 < 16) nxt = frag_row(dhimg, 16 * ((it + 1) & 3) + j, 32 * ((it + 1) >> 2) + 8 * g);
        if (bt == 3 && it + 1 < 16) bln = frag_tr8(w2lo, 32 * (c + 1) + 8 * g, own, l);
        const Split8 a{wB[c].h, wB[c].m, bl};
        dh1[bt] = mma6t(a, cur, dh1[bt]);
        __builtin_amdgcn_sched_barrier(0);
        if (it + 1 < 16) cur = nxt;
        if (bt == 3 && it + 1 < 16) bl = bln;
      }
      dh1_relu();
    }
    // dW1 row (16 bt + 4 g + i) of the transposed dh1 tile
    auto dw1_rows_valu = [&](int bt, int i, const floatx4 (&x)[DP / 4]) {
#pragma unroll
      for (int d4 = 0; d4 < DP / 4; ++d4) {
#pragma unroll
        for (int e = 0; e < 4; ++e) acc1[(4 * d4 + e) % NA1] = fmaf(dh1[bt][i], x[d4][e], acc1[(4 * d4 + e) % NA1]);
      }
    };
    auto load_xrow = [&](int row, floatx4 (&x)[DP / 4]) {
#pragma unroll
      for (int d4 = 0; d4 < DP / 4; ++d4) x[d4] = *reinterpret_cast<const floatx4*>(xs + row * DP + 4 * d4);
    };
    auto do_dw1 = [&]() {
      VG_STAMP(8);
      if (kDw1Mfma) {
        // dW1 tile [own features][16 inputs] += dh1^T row block x x: A = the transposed dh1
        // value (feature own + j, row 16 bt + 4 g + i), B = x[that row][16 nt + j]
#pragma unroll
        for (int bt = 0; bt < 4; ++bt) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int row = 16 * bt + 4 * g + i;
#pragma unroll
            for (int nt = 0; nt < (kDw1Mfma ? NT1 : 1); ++nt) {
              const int d = 16 * nt + j;
              const float xb = d < DP ? xs[row * DP + d] : 0.f;
              acc1m[nt] = mfma4(dh1[bt][i], xb, acc1m[nt]);
            }
            if (kTail1) {
              const floatx4 xt = *reinterpret_cast<const floatx4*>(xs + row * DP + 16 * NT1);
#pragma unroll
              for (int e = 0; e < 4; ++e) acc1[e % NA1] = fmaf(dh1[bt][i], xt[e], acc1[e % NA1]);
            }
          }
        }
      } else {
#pragma unroll
        for (int bt = 0; bt < 4; ++bt) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            floatx4 x[DP / 4];
            load_xrow(16 * bt + 4 * g + i, x);
            dw1_rows_valu(bt, i, x);
          }
        }
      }
    };
    // ------------------------------------------------------------ dW2 += dh2 h1^T
    auto do_dw2 = [&]() {
      VG_STAMP(9);
      Split8 a = frag_tr(dhimg, 0, own, l);
      Split8 cur = frag_tr(h1img, 0, 0, l);
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        const int t = it & 7;
        Split8 nxt, an;
        if (it + 1 < 16) nxt = frag_tr(h1img, 32 * ((it + 1) >> 3), 16 * ((it + 1) & 7), l);
        if (it == 7) an = frag_tr(dhimg, 32, own, l);
        acc2[t] = mma6(a, cur, acc2[t]);
        __builtin_amdgcn_sched_barrier(0);
        if (it + 1 < 16) cur = nxt;
        if (it == 7) a = an;
      }
    };
    // dW2 MFMAs with dW1 vector work between them (kInterleave, DP = 4): one dh1 row per
    // step, its x row read one step ahead
    auto do_dw2_dw1 = [&]() {
      VG_STAMP(8);
      VG_STAMP(9);
      Split8 a = frag_tr(dhimg, 0, own, l);
      Split8 cur = frag_tr(h1img, 0, 0, l);
      floatx4 xq[DP / 4];
      load_xrow(4 * g, xq);
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        const int t = it & 7;
        Split8 nxt, an;
        if (it + 1 < 16) nxt = frag_tr(h1img, 32 * ((it + 1) >> 3), 16 * ((it + 1) & 7), l);
        if (it == 7) an = frag_tr(dhimg, 32, own, l);
        acc2[t] = mma6(a, cur, acc2[t]);
        {
          floatx4 xc[DP / 4];
#pragma unroll
          for (int d4 = 0; d4 < DP / 4; ++d4) xc[d4] = xq[d4];
          if (it + 1 < 16) load_xrow(16 * ((it + 1) >> 2) + 4 * g + ((it + 1) & 3), xq);
          dw1_rows_valu(it >> 2, it & 3, xc);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (it + 1 < 16) cur = nxt;
        if (it == 7) a = an;
      }
    };
    if (kInterleave && !kDw1Mfma) {
      do_dw2_dw1();
    } else {
      do_dw1();
      do_dw2();
    }
    VG_STAMP(10);
  }

  // ------------------------------------------------------------------ epilogue
  if constexpr (FWD) return;
  if (kTvPersist) accv[0] += fold_tvs();
  float* slab = p.grad_slab + (size_t)blockIdx.x * p.P;
  // kFactor: dW2 rows / db2 are w3' x the accumulated dh2' sums (w3' = w3, or w3[1] - w3[0])
  auto w3g = [&](int f) { return kBin ? P[o.w3 + kVgH + f] - P[o.w3 + f] : P[o.w3 + f]; };
  floatx4 w3s;
#pragma unroll
  for (int r = 0; r < 4; ++r) w3s[r] = kFactor ? w3g(own + 4 * g + r) : 1.f;
#pragma unroll
  for (int it = 0; it < 8; ++it) {
#pragma unroll
    for (int r = 0; r < 4; ++r) slab[o.w2 + (own + 4 * g + r) * kVgH + 16 * it + j] = acc2[it][r] * w3s[r];
  }
#pragma unroll
  for (int q = 0; q < NG; ++q) {
    const int f = 4 * q + (j >> 2), feat = own + 4 * g + (j & 3);
    if (f < NF) {
      const int off = f == 0 ? o.b2 : f == 1 ? o.w3 : f == 2 ? o.b1 : o.w3 + (f == 3 ? 1 : f - 2) * kVgH;
      if (f != 2) slab[off + feat] = (kFactor && f == 0) ? accv[q] * w3g(feat) : accv[q];
    }
  }
  if (kDw1Mfma) {
#pragma unroll
    for (int nt = 0; nt < (kDw1Mfma ? NT1 : 1); ++nt) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int d = 16 * nt + j;
        if (d < D) slab[o.w1 + (own + 4 * g + i) * D + d] = acc1m[nt][i];
      }
    }
#pragma unroll
    for (int e = 0; e < kTail1; ++e) {
      const float sd = group_sum_swap(acc1[e % NA1]);  // over the 4 lane groups (all lanes call)
      const int d = 16 * NT1 + e;
      if (g == e && d < D) slab[o.w1 + (own + j) * D + d] = sd;
    }
  } else {
#pragma unroll
    for (int d = 0; d < NA1; ++d) {
      const float sd = group_sum_swap(acc1[d]);  // over the 4 lane groups (all lanes call)
      if (g == (d & 3) && d < D) slab[o.w1 + (own + j) * D + d] = sd;
    }
  }
  {
    const float sb = group_sum_swap(db1acc);
    if (g == 0) slab[o.b1 + own + j] = sb;
  }
  if constexpr (kSplitHead) {
    // db3 / dlog_std: the waves' hacc slots; loss sums: lanes 8 r of every wave, folded in the
    // wave and then over the 8 waves through LDS (fixed order)
    const float st[6] = {wave_sum_vl(s_loss), wave_sum_vl(s_ent), wave_sum_vl(s_kl),
                         wave_sum_vl(s_clip), wave_sum_vl(s_val), wave_sum_vl(s_cnt)};
    __syncthreads();  // every wave is past its last dh2 phase: the dout table is free
    float* ep = dtab;  // [8 waves][6]: loss sums
    if (l == 0) {
#pragma unroll
      for (int k = 0; k < 6; ++k) ep[w * 6 + k] = st[k];
    }
    __syncthreads();
    const int t = threadIdx.x;
    if (t < 2 * NA) {
      float v = 0.f;
#pragma unroll
      for (int ww = 0; ww < 8; ++ww) v += hacc[ww * 2 * NA + t];
      slab[(t < NA ? o.b3 : o.log_std - NA) + t] = v;
    } else if (t >= 64 && t < 70) {
      float v = 0.f;
#pragma unroll
      for (int ww = 0; ww < 8; ++ww) v += ep[ww * 6 + t - 64];
      p.loss_slab[blockIdx.x * 8 + t - 64] = v;
    }
  }
  if (!kSplitHead && w < NA && l == 0) {
    slab[o.b3 + w] = bacc3;
    if (kGauss) slab[o.log_std + w] = dls;
  }
  if (!kSplitHead && w == 0) {
    const float sl = wave_sum(s_loss), sv = wave_sum(s_val), sc = wave_sum(s_cnt);
    const float se = wave_sum(s_ent), sk = wave_sum(s_kl), scl = wave_sum(s_clip);
    if (l == 0) {
      float* lsl = p.loss_slab + blockIdx.x * 8;
      lsl[0] = sl;
      lsl[1] = se;
      lsl[2] = sk;
      lsl[3] = scl;
      lsl[4] = sv;
      lsl[5] = sc;
    }
  }
  if (STAMP && p.stamps != nullptr) {
    unsigned long long t_end;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_end)::"memory");
    st_sum[11] = t_end - st_prev;
    if (l == 0) {
#pragma unroll
      for (int k = 0; k < 12; ++k) p.stamps[(blockIdx.x * 8 + w) * 16 + k] = st_sum[k];
    }
  }
}

bool value_grad_split_supported(int D, int H) { return H == kVgH && D >= 1 && D <= 24; }

// (head, A, D) combinations with a bf16x6 instance (the rest run the fp32-MFMA mlp_grad kernel)
bool policy_grad_split_supported(int D, int H, int A, int head) {
  if (H != kVgH || D < 1) return false;
  if (head == HEAD_PG_CAT || head == HEAD_PPO_CAT) return D <= 8 && A >= 2 && A <= 4;
  if (head == HEAD_PG_GAUSS || head == HEAD_PPO_GAUSS) return D <= 20 && (A == 1 || A == 6);
  return false;
}

static int g_vg_tune = 0;  // experiments (bit 0: waves 4-7 at prio 1, bit 1: waves 0-3, bit 3: stamps,
                           // bit 7: variant V = bits 4..6 of the DP = 4 / 8 value kernels)
static unsigned long long* g_vg_stamps = nullptr;

template <int DP, int HEAD, int NA, bool STAMP, int V>
static int launch_inst(const GradArgs& a, int grid, hipStream_t s) {
  constexpr int bytes = vg_total_bytes(DP, HEAD, NA);
  static_assert(bytes <= 160 * 1024, "value-grad LDS plan exceeds 160 KB");
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)value_grad_split_kernel<DP, HEAD, NA, STAMP, V>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    attr_set = true;
  }
  hipLaunchKernelGGL((value_grad_split_kernel<DP, HEAD, NA, STAMP, V>), dim3(grid), dim3(512), bytes, s, a);
  return (int)hipGetLastError();
}

template <int DP, int HEAD, int NA, bool STAMP>
static int launch_var(const GradArgs& a, int grid, hipStream_t s) {
  if constexpr (HEAD == HEAD_VALUE_MSE && DP <= 8) {
    if (a.tune & 128) {  // structural A/B (vg_prod_v): V = tune bits 4..6
      switch ((a.tune >> 4) & 7) {
        case 0: return launch_inst<DP, HEAD, NA, STAMP, 0>(a, grid, s);
        case 1: return launch_inst<DP, HEAD, NA, STAMP, 1>(a, grid, s);
        case 3: return launch_inst<DP, HEAD, NA, STAMP, 3>(a, grid, s);
        default: break;
      }
    }
  }
  return launch_inst<DP, HEAD, NA, STAMP, vg_prod_v(DP)>(a, grid, s);
}

template <int DP, int HEAD, int NA>
static int launch_vg(const GradArgs& a0, int grid, hipStream_t s) {
  GradArgs a = a0;
  a.tune = g_vg_tune;
  a.stamps = g_vg_stamps;
  if (a.tune & 8) return launch_var<DP, HEAD, NA, true>(a, grid, s);  // diagnostic stamps build
  return launch_var<DP, HEAD, NA, false>(a, grid, s);
}

int launch_value_grad_split(const GradArgs& a, int grid, hipStream_t s) {
  if (a.D <= 4) return launch_vg<4, HEAD_VALUE_MSE, 1>(a, grid, s);
  if (a.D <= 8) return launch_vg<8, HEAD_VALUE_MSE, 1>(a, grid, s);
  if (a.D <= 16) return launch_vg<16, HEAD_VALUE_MSE, 1>(a, grid, s);
  if (a.D <= 20) return launch_vg<20, HEAD_VALUE_MSE, 1>(a, grid, s);  // HalfCheetahSynth (D = 17)
  return launch_vg<24, HEAD_VALUE_MSE, 1>(a, grid, s);
}

template <int DP>
static int launch_fwd(const GradArgs& a0, int grid, hipStream_t s) {
  constexpr int bytes = vg_total_bytes(DP, HEAD_VALUE_MSE, 1);
  static_assert(bytes <= 160 * 1024, "value-forward LDS plan exceeds 160 KB");
  auto* kern = value_grad_split_kernel<DP, HEAD_VALUE_MSE, 1, false, vg_prod_v(DP), true>;
  static bool attr_set = false;
  if (!attr_set) {
    (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    attr_set = true;
  }
  GradArgs a = a0;
  a.tune = 0;
  a.stamps = nullptr;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(512), bytes, s, a);
  return (int)hipGetLastError();
}

int launch_value_fwd_split(const GradArgs& a, int grid, hipStream_t s) {
  if (a.vout == nullptr) return -2;
  if (a.D <= 4) return launch_fwd<4>(a, grid, s);
  if (a.D <= 8) return launch_fwd<8>(a, grid, s);
  if (a.D <= 16) return launch_fwd<16>(a, grid, s);
  if (a.D <= 20) return launch_fwd<20>(a, grid, s);
  return launch_fwd<24>(a, grid, s);
}

template <int HEAD, int NA>
static int launch_cat(const GradArgs& a, int grid, hipStream_t s) {
  return a.D <= 4 ? launch_vg<4, HEAD, NA>(a, grid, s) : launch_vg<8, HEAD, NA>(a, grid, s);
}

template <int HEAD>
static int launch_cat_a(const GradArgs& a, int grid, hipStream_t s) {
  switch (a.A) {
    case 2: return launch_cat<HEAD, 2>(a, grid, s);  // CartPole
    case 3: return launch_cat<HEAD, 3>(a, grid, s);  // MountainCar, Acrobot
    case 4: return launch_cat<HEAD, 4>(a, grid, s);  // LunarLander
    default: return -2;
  }
}

template <int HEAD, int NA>
static int launch_gauss(const GradArgs& a, int grid, hipStream_t s) {
  if (a.D <= 4) return launch_vg<4, HEAD, NA>(a, grid, s);  // Pendulum (D = 3, A = 1)
  if (a.D <= 8) return launch_vg<8, HEAD, NA>(a, grid, s);
  return launch_vg<20, HEAD, NA>(a, grid, s);  // HalfCheetahSynth (D = 17, A = 6)
}

template <int HEAD>
static int launch_gauss_a(const GradArgs& a, int grid, hipStream_t s) {
  switch (a.A) {
    case 1: return launch_gauss<HEAD, 1>(a, grid, s);
    case 6: return launch_gauss<HEAD, 6>(a, grid, s);
    default: return -2;
  }
}

// Policy-gradient step on the bf16x6 kernel (categorical A = 2..4, Gaussian A = 1 or 6).
int launch_policy_grad_split(const GradArgs& a, int head, int grid, hipStream_t s) {
  switch (head) {
    case HEAD_PG_CAT: return launch_cat_a<HEAD_PG_CAT>(a, grid, s);
    case HEAD_PPO_CAT: return launch_cat_a<HEAD_PPO_CAT>(a, grid, s);
    case HEAD_PG_GAUSS: return launch_gauss_a<HEAD_PG_GAUSS>(a, grid, s);
    case HEAD_PPO_GAUSS: return launch_gauss_a<HEAD_PPO_GAUSS>(a, grid, s);
    default: return -2;
  }
}

}  // namespace rrl

extern "C" void rrl_set_value_grad_stamps(void* buf) { rrl::g_vg_stamps = (unsigned long long*)buf; }

extern "C" int rrl_set_value_grad_tune(int t) {
  const int old = rrl::g_vg_tune;
  rrl::g_vg_tune = t;
  return old;
}
