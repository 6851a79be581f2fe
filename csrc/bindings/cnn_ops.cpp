// PyTorch bindings for the pixel-model kernels (csrc/kernels/cnn.hip, pong.hip).
// Same contract as hip_ops.cpp: every tensor is validated (device, dtype, contiguity,
// size) before a launch, launches go to the current HIP stream.
#include <ATen/hip/HIPContext.h>
#include <pybind11/stl.h>
#include <torch/extension.h>

#include <cstdint>
#include <optional>
#include <tuple>
#include <vector>

extern "C" {
int rrl_conv_fwd(const void* x, int x_u8, const uint16_t* w, const float* b, uint16_t* y, int N, int H, int W,
                 int C, int KH, int KW, int S, int Cout, int relu, float* work, long long work_elems, void* stream);
int rrl_gemm_dgrad(const uint16_t* dy, const uint16_t* w, const uint16_t* mask, uint16_t* out, int M, int Cout,
                   int K, void* stream);
int rrl_col2im_mask(const uint16_t* dcol, const uint16_t* xact, uint16_t* dx, int N, int H, int W, int C, int KH,
                    int KW, int S, void* stream);
int rrl_conv_wgrad(const uint16_t* dy, const void* x, int x_u8, float* part, float* bias_part, int splits, int N,
                   int H, int W, int C,
                   int KH, int KW, int S, int Cout, void* stream);
int rrl_gemm_splits(int R, int splits);
int rrl_conv_dgrad(const uint16_t* dy, const uint16_t* w, const uint16_t* xact, uint16_t* dx, int N, int H, int W,
                   int C, int KH, int KW, int S, int Cout, void* stream);
int rrl_sum_splits(const float* part, int splits, long long n, float* out, void* stream);
int rrl_sum_splits_multi(const float* const* parts, const int* splits, const long long* ns, float* const* outs,
                         int count, void* stream);
int rrl_colsum(const uint16_t* y, int M, int C, float* part, int splits, void* stream);
int rrl_sumsq(const float* x, long long n, float* work, int work_n, float* out, void* stream);
int rrl_adam_clip(float* p, float* m, float* v, const float* g, uint16_t* shadow, long long n, const float* norm_sq,
                  float max_norm, float lr, float b1, float b2, float eps, int step, const long long* step_dev, int norm_parts,
                  void* stream);
int rrl_sumsq_partial(const float* x, long long n, float* work, int work_n, void* stream);
int rrl_counter_add(long long* c, long long inc, void* stream);
int rrl_counter_add_n(long long* const* c, const long long* inc, int n, void* stream);
int rrl_to_bf16(const float* x, uint16_t* y, long long n, void* stream);
int rrl_a2c_head(int mode, const uint16_t* h, const float* head_params, int B, int A, int32_t* act, float* logp,
                 float* value, float* logits_out, unsigned long long seed, unsigned long long step,
                 const unsigned long long* step_base, int row_offset,
                 const int32_t* act_in, const float* adv, const float* ret, float inv_B, float vf_coef,
                 float ent_coef, uint16_t* dh, float* dhead, float* stats, int grid, const float* part,
                 int splits, const float* fc_b, uint16_t* h_out, void* stream);
int rrl_fc_nt_part(const uint16_t* a, const uint16_t* b, float* part, int M, int N, int K, int splits, void* stream);

int rrl_fc_nt_mask(const uint16_t* a, const uint16_t* b, const uint16_t* mask, uint16_t* out, int M, int N, int K,
                   void* stream);
int rrl_transpose_bf16(const uint16_t* in, uint16_t* out, int R, int C, void* stream);
int rrl_fc_tn_part(const uint16_t* x, const uint16_t* y, float* part, int R, int I, int J, int splits,
                   const uint16_t* ones, float* bias_part, void* stream);
int rrl_head_wgrad(const uint16_t* h, const float* dhead, int B, int A, float* part, int nblk, void* stream);
int rrl_pong_state_size();
int rrl_pong_step(float* state, const int32_t* act, float* rew, float* done, float* fin_ret, float* fin_len,
                  float* ep_acc, int N, unsigned long long seed, unsigned long long step,
                  const unsigned long long* step_base, int max_steps, int reset_all, float* hist_out, void* stream);
int rrl_pong_render(const float* state, uint8_t* obs, int N, void* stream);
int rrl_pong_step_render(float* state, const int32_t* act, float* rew, float* done, float* fin_ret, float* fin_len,
                         float* ep_acc, uint8_t* obs, int N, unsigned long long seed, unsigned long long step,
                         const unsigned long long* step_base, int max_steps, int reset_all, uint8_t* frames,
                         int32_t* fidx, int R, void* stream);
int rrl_pong_ring_fill(float* state, uint8_t* frames, int32_t* fidx, int N, int R, unsigned long long step,
                       const unsigned long long* step_base, void* stream);
int rrl_conv_stack_fwd(const uint8_t* x, const float* hist, const uint8_t* frames, const int32_t* fidx,
                       const uint16_t* w1, const float* b1,
                       const uint16_t* w2, const float* b2, const uint16_t* w3, const float* b3, uint16_t* y1,
                       uint16_t* y2, uint16_t* y3, int N, int max_grid, void* stream);
int rrl_conv3_bwd(const uint16_t* dy, const uint16_t* w, const uint16_t* xact, uint16_t* dx, float* part,
                  float* bias_part, int N, int grid, int variant, void* stream);
int rrl_conv2_bwd(const uint16_t* dy, const uint16_t* w, const uint16_t* xact, uint16_t* dx, float* part,
                  float* bias_part, int N, int grid, int staged, void* stream);
int rrl_conv1_wgrad8(const uint8_t* x, const float* hist, const uint8_t* frames, const int32_t* fidx,
                     const uint16_t* dy, float* part, float* bias_part, int N, int grid, int T, void* stream);
int rrl_pong_render_hist(const float* hist, uint8_t* obs, int N, void* stream);
int rrl_pong_head_step_render(const float* part, int splits, const float* fc_b, const float* head_params, int A,
                              uint16_t* h_out, int32_t* act, float* logp, float* value, unsigned long long sample_seed,
                              unsigned long long sample_step, const unsigned long long* sample_base, float* state,
                              float* rew, float* done, float* fin_ret, float* fin_len, float* ep_acc, uint8_t* obs,
                              int N, unsigned long long seed, unsigned long long step,
                              const unsigned long long* step_base, int max_steps, uint8_t* frames, int32_t* fidx,
                              int R, void* stream);

}

namespace {

using at::Tensor;
using OptT = std::optional<Tensor>;

void* stream() { return (void*)at::hip::getCurrentHIPStream().stream(); }

void check(const Tensor& t, const char* name, at::ScalarType dt, int64_t min_numel) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == dt, name, " has dtype ", t.scalar_type(), ", expected ", dt);
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
  TORCH_CHECK(t.numel() >= min_numel, name, " has ", t.numel(), " elements, need >= ", min_numel);
}
template <class T>
T* opt_ptr(const OptT& t, const char* name, at::ScalarType dt, int64_t n) {
  if (!t.has_value() || !t->defined()) return nullptr;
  check(*t, name, dt, n);
  return reinterpret_cast<T*>(t->data_ptr());
}
void rc_check(int rc, const char* what) {
  TORCH_CHECK(rc == 0, what, " failed with code ", rc,
              " (", (rc > 0 ? hipGetErrorString((hipError_t)rc) : "unsupported shape"), ")");
}
uint16_t* bf(const Tensor& t) { return reinterpret_cast<uint16_t*>(t.data_ptr()); }

constexpr int64_t kFrameBytes = 7056;  // one PongSynth frame in the ring (pong_render.h)

// A frame-ring store written by a step launch over N envs: frames [R][N][7056] uint8, fidx [N][4]
uint8_t* ring_store(const OptT& frames, const OptT& fidx, int64_t N, int64_t R) {
  TORCH_CHECK(R >= 5, "frame ring: ring_slots >= 5 (a rollout's T + 4)");
  TORCH_CHECK(R * N < (int64_t(1) << 31), "frame ring: R * N must fit int32 frame rows");
  check(*frames, "frames", at::kByte, R * N * kFrameBytes);
  TORCH_CHECK(fidx.has_value() && fidx->defined(), "frame ring: fidx is required with frames");
  check(*fidx, "fidx", at::kInt, 4 * N);
  return frames->data_ptr<uint8_t>();
}

// A frame ring read by the conv kernels for N observations: every fidx row must index a whole
// frame of the store (its values come from pong_step / pong_ring_fill, which write rows < R * E)
const uint8_t* ring_frames(const OptT& frames, const OptT& fidx, int64_t N) {
  if (!frames.has_value() || !frames->defined()) return nullptr;
  check(*frames, "frames", at::kByte, kFrameBytes);
  TORCH_CHECK(frames->numel() % kFrameBytes == 0, "frames: whole 7056-byte frames");
  TORCH_CHECK(fidx.has_value() && fidx->defined(), "frame ring: fidx is required with frames");
  check(*fidx, "fidx", at::kInt, 4 * N);
  return frames->data_ptr<uint8_t>();
}

struct Geo {
  int64_t N, H, W, C, KH, KW, S;
  int64_t OH() const { return (H - KH) / S + 1; }
  int64_t OW() const { return (W - KW) / S + 1; }
};
void check_geo(const Geo& g) {
  TORCH_CHECK(g.N > 0 && g.H >= g.KH && g.W >= g.KW && g.S > 0 && g.C > 0, "bad conv geometry");
}

void conv_fwd(const Tensor& x, const Tensor& w, const Tensor& b, const Tensor& y, int64_t N, int64_t H, int64_t W,
              int64_t C, int64_t KH, int64_t KW, int64_t S, int64_t Cout, bool relu, const OptT& work) {
  Geo g{N, H, W, C, KH, KW, S};
  check_geo(g);
  const bool u8 = x.scalar_type() == at::kByte;
  check(x, "x", u8 ? at::kByte : at::kBFloat16, N * H * W * C);
  TORCH_CHECK(u8 ? ((C == 4 && KW % 2 == 0) || C % 8 == 0) : (C % 8 == 0), "conv_fwd: unsupported channel layout");
  TORCH_CHECK(Cout % 8 == 0, "conv_fwd: Cout must be a multiple of 8 (16-byte epilogue stores)");
  check(w, "w", at::kBFloat16, Cout * KH * KW * C);
  check(b, "b", at::kFloat, Cout);
  check(y, "y", at::kBFloat16, N * g.OH() * g.OW() * Cout);
  float* wk = opt_ptr<float>(work, "work", at::kFloat, 0);
  const long long wn = wk ? work->numel() : 0;
  rc_check(rrl_conv_fwd(x.data_ptr(), u8, bf(w), b.data_ptr<float>(), bf(y), N, H, W, C, KH, KW, S, Cout, relu, wk,
                        wn, stream()),
           "conv_fwd");
}

// Fused Nature-CNN conv stack (cnn_fused.hip): uint8 s2d frames [N][21][21][64] ->
// a1 [N][20][20][32], a2 [N][9][9][64], a3 [N][7][7][64] (bf16, post-ReLU).
void conv_stack_fwd(const OptT& x, const Tensor& w1, const Tensor& b1, const Tensor& w2, const Tensor& b2,
                    const Tensor& w3, const Tensor& b3, const Tensor& y1, const Tensor& y2, const Tensor& y3,
                    int64_t N, int64_t probe, int64_t grid, bool store12, const OptT& hist, const OptT& frames,
                    const OptT& fidx) {
  TORCH_CHECK(N > 0, "conv_stack_fwd: N must be positive");
  // fused render: PongSynth frame histories [N][16] instead of s2d frames (cnn_fused.hip)
  const float* hp = opt_ptr<const float>(hist, "hist", at::kFloat, N * 16);
  const uint8_t* xp = opt_ptr<const uint8_t>(x, "x", at::kByte, N * 21 * 21 * 64);
  // frame ring: the PongSynth frame store + the observations' frame rows fidx [N][4]
  const uint8_t* fp = ring_frames(frames, fidx, N);
  const int32_t* ip = fp ? fidx->data_ptr<int32_t>() : nullptr;
  TORCH_CHECK(hp || xp || fp, "conv_stack_fwd: x (s2d frames), hist (frame histories) or frames + fidx is required");
  check(w1, "w1", at::kBFloat16, 32 * 256);
  check(w2, "w2", at::kBFloat16, 64 * 512);
  check(w3, "w3", at::kBFloat16, 64 * 576);
  check(b1, "b1", at::kFloat, 32);
  check(b2, "b2", at::kFloat, 64);
  check(b3, "b3", at::kFloat, 64);
  check(y1, "y1", at::kBFloat16, N * 400 * 32);
  check(y2, "y2", at::kBFloat16, N * 81 * 64);
  check(y3, "y3", at::kBFloat16, N * 49 * 64);
  int dev = 0, cus = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  rc_check(rrl_conv_stack_fwd(xp, hp, fp, ip, bf(w1), b1.data_ptr<float>(), bf(w2), b2.data_ptr<float>(),
                              bf(w3), b3.data_ptr<float>(), store12 ? bf(y1) : nullptr, store12 ? bf(y2) : nullptr,
                              bf(y3), (int)N,
                              probe > 0 ? -(int)((probe << 16) | (grid > 0 ? grid : cus))
                                        : (grid > 0 ? (int)grid : cus),
                              stream()),
           "conv_stack_fwd");
}

// Fused conv3 backward (cnn_fused.hip): da3 [N][49][64], W3 [64][3][3][64], a2 [N][81][64] ->
// da2 = dgrad * (a2 > 0), dW3 partials [grid][64 * 576], db3 partials [grid * 8][64].
void conv3_bwd(const Tensor& dy, const Tensor& w, const Tensor& xact, const Tensor& dx, const Tensor& part,
               const Tensor& bias_part, int64_t N, int64_t grid, int64_t variant) {
  TORCH_CHECK(N > 0 && grid > 0 && grid <= N, "conv3_bwd: need 0 < grid <= N");
  check(dy, "dy", at::kBFloat16, N * 49 * 64);
  check(w, "w", at::kBFloat16, 64 * 576);
  check(xact, "xact", at::kBFloat16, N * 81 * 64);
  check(dx, "dx", at::kBFloat16, N * 81 * 64);
  check(part, "part", at::kFloat, grid * 64 * 576);
  check(bias_part, "bias_part", at::kFloat, grid * 512);
  rc_check(rrl_conv3_bwd(bf(dy), bf(w), bf(xact), bf(dx), part.data_ptr<float>(), bias_part.data_ptr<float>(),
                         (int)N, (int)grid, (int)variant, stream()),
           "conv3_bwd");
}

// Fused conv2 backward (cnn_fused.hip): da2 [N][81][64], W2 [64][4][4][32], a1 [N][400][32] ->
// da1 = dgrad * (a1 > 0), dW2 partials [grid][64 * 512], db2 partials [grid * 8][64].
void conv2_bwd(const Tensor& dy, const Tensor& w, const Tensor& xact, const Tensor& dx, const Tensor& part,
               const Tensor& bias_part, int64_t N, int64_t grid, int64_t staged) {
  TORCH_CHECK(N > 0 && grid > 0 && grid <= N, "conv2_bwd: need 0 < grid <= N");
  check(dy, "dy", at::kBFloat16, N * 81 * 64);
  check(w, "w", at::kBFloat16, 64 * 512);
  check(xact, "xact", at::kBFloat16, N * 400 * 32);
  check(dx, "dx", at::kBFloat16, N * 400 * 32);
  check(part, "part", at::kFloat, grid * 64 * 512);
  check(bias_part, "bias_part", at::kFloat, grid * 512);
  rc_check(rrl_conv2_bwd(bf(dy), bf(w), bf(xact), bf(dx), part.data_ptr<float>(), bias_part.data_ptr<float>(),
                         (int)N, (int)grid, (int)staged, stream()),
           "conv2_bwd");
}

// conv1 weight + bias gradient, 8-wave kernel (cnn_fused.hip): s2d frames [N][21][21][64], da1
// [N][400][32] -> partials [2 grid][32 * 256] and [2 grid][32]; returns the slab count (2 grid).
int64_t conv1_wgrad8(const OptT& x, const Tensor& dy, const Tensor& part, const Tensor& bias_part, int64_t N,
                     int64_t grid, const OptT& hist, const OptT& frames, const OptT& fidx, int64_t env_major_T) {
  TORCH_CHECK(N > 0 && grid > 0 && grid <= N, "conv1_wgrad8: need 0 < grid <= N");
  const float* hp = opt_ptr<const float>(hist, "hist", at::kFloat, N * 16);
  const uint8_t* xp = opt_ptr<const uint8_t>(x, "x", at::kByte, N * 441 * 64);
  const uint8_t* fp = ring_frames(frames, fidx, N);
  const int32_t* ip = fp ? fidx->data_ptr<int32_t>() : nullptr;
  TORCH_CHECK(hp || xp || fp, "conv1_wgrad8: x (s2d frames), hist (frame histories) or frames + fidx is required");
  check(dy, "dy", at::kBFloat16, N * 400 * 32);
  check(part, "part", at::kFloat, 2 * grid * 32 * 256);
  check(bias_part, "bias_part", at::kFloat, 2 * grid * 32);
  // env_major_T > 1 (frame ring): the rows are a T-step rollout, visited env-major (rows of one env
  // back to back share 3 of their 4 frames)
  TORCH_CHECK(env_major_T <= 1 || (fp && N % env_major_T == 0), "conv1_wgrad8: env_major_T needs the ring and T | N");
  rc_check(rrl_conv1_wgrad8(xp, hp, fp, ip, bf(dy), part.data_ptr<float>(), bias_part.data_ptr<float>(), (int)N, (int)grid,
                            (int)env_major_T, stream()),
           "conv1_wgrad8");
  return 2 * grid;
}

void gemm_dgrad(const Tensor& dy, const Tensor& w, const OptT& mask, const Tensor& out, int64_t M, int64_t Cout,
                int64_t K) {
  TORCH_CHECK(Cout % 8 == 0 && K % 8 == 0, "gemm_dgrad: Cout and K must be multiples of 8");
  check(dy, "dy", at::kBFloat16, M * Cout);
  check(w, "w", at::kBFloat16, Cout * K);
  check(out, "out", at::kBFloat16, M * K);
  const uint16_t* mp = opt_ptr<uint16_t>(mask, "mask", at::kBFloat16, M * K);
  rc_check(rrl_gemm_dgrad(bf(dy), bf(w), mp, bf(out), M, Cout, K, stream()), "gemm_dgrad");
}

void col2im_mask(const Tensor& dcol, const Tensor& xact, const Tensor& dx, int64_t N, int64_t H, int64_t W,
                 int64_t C, int64_t KH, int64_t KW, int64_t S) {
  Geo g{N, H, W, C, KH, KW, S};
  check_geo(g);
  TORCH_CHECK(C % 8 == 0, "col2im_mask: C must be a multiple of 8");
  check(dcol, "dcol", at::kBFloat16, N * g.OH() * g.OW() * KH * KW * C);
  check(xact, "xact", at::kBFloat16, N * H * W * C);
  check(dx, "dx", at::kBFloat16, N * H * W * C);
  rc_check(rrl_col2im_mask(bf(dcol), bf(xact), bf(dx), N, H, W, C, KH, KW, S, stream()), "col2im_mask");
}

// Returns false (nothing launched) for geometries without an implicit-dgrad kernel.
bool conv_dgrad(const Tensor& dy, const Tensor& w, const Tensor& xact, const Tensor& dx, int64_t N, int64_t H,
                int64_t W, int64_t C, int64_t KH, int64_t KW, int64_t S, int64_t Cout) {
  Geo g{N, H, W, C, KH, KW, S};
  check_geo(g);
  check(dy, "dy", at::kBFloat16, N * g.OH() * g.OW() * Cout);
  check(w, "w", at::kBFloat16, Cout * KH * KW * C);
  check(xact, "xact", at::kBFloat16, N * H * W * C);
  check(dx, "dx", at::kBFloat16, N * H * W * C);
  const int rc = rrl_conv_dgrad(bf(dy), bf(w), bf(xact), bf(dx), N, H, W, C, KH, KW, S, Cout, stream());
  if (rc == -1) return false;
  rc_check(rc, "conv_dgrad");
  return true;
}

int64_t gemm_splits(int64_t R, int64_t splits) { return rrl_gemm_splits((int)R, (int)splits); }



int64_t conv_wgrad(const Tensor& dy, const Tensor& x, const Tensor& part, int64_t splits, int64_t N, int64_t H,
                   int64_t W, int64_t C, int64_t KH, int64_t KW, int64_t S, int64_t Cout, const OptT& bias_part) {
  Geo g{N, H, W, C, KH, KW, S};
  check_geo(g);
  const bool u8 = x.scalar_type() == at::kByte;
  const int64_t M = N * g.OH() * g.OW(), K = KH * KW * C;
  TORCH_CHECK(u8 ? ((C == 4 && KW % 2 == 0) || C % 8 == 0) : (C % 8 == 0), "conv_wgrad: unsupported channel layout");
  check(dy, "dy", at::kBFloat16, M * Cout);
  check(x, "x", u8 ? at::kByte : at::kBFloat16, N * H * W * C);
  const int64_t s = gemm_splits(M, splits);
  check(part, "part", at::kFloat, s * Cout * K);
  float* bp = nullptr;
  if (bias_part.has_value()) {  // also the bias gradient: partials [s][Cout]
    check(*bias_part, "bias_part", at::kFloat, s * Cout);
    bp = bias_part->data_ptr<float>();
  }
  rc_check(rrl_conv_wgrad(bf(dy), x.data_ptr(), u8, part.data_ptr<float>(), bp, (int)splits, N, H, W, C, KH, KW, S,
                          Cout, stream()),
           "conv_wgrad");
  return s;
}

void sum_splits(const Tensor& part, int64_t splits, int64_t n, const Tensor& out) {
  check(part, "part", at::kFloat, splits * n);
  check(out, "out", at::kFloat, n);
  rc_check(rrl_sum_splits(part.data_ptr<float>(), (int)splits, n, out.data_ptr<float>(), stream()), "sum_splits");
}

// [(part, splits, n, out), ...] (<= 8 segments) summed in one launch
void sum_splits_multi(const std::vector<std::tuple<Tensor, int64_t, int64_t, Tensor>>& segs) {
  TORCH_CHECK(!segs.empty() && segs.size() <= 8, "sum_splits_multi: 1..8 segments");
  std::vector<const float*> parts;
  std::vector<float*> outs;
  std::vector<int> splits;
  std::vector<long long> ns;
  for (const auto& sgm : segs) {
    const Tensor& part = std::get<0>(sgm);
    const int64_t s = std::get<1>(sgm), n = std::get<2>(sgm);
    const Tensor& out = std::get<3>(sgm);
    TORCH_CHECK(s >= 1 && n >= 4 && n % 4 == 0, "sum_splits_multi: splits >= 1, n % 4 == 0");
    check(part, "part", at::kFloat, s * n);
    check(out, "out", at::kFloat, n);
    parts.push_back(part.data_ptr<float>());
    outs.push_back(out.data_ptr<float>());
    splits.push_back((int)s);
    ns.push_back(n);
  }
  rc_check(rrl_sum_splits_multi(parts.data(), splits.data(), ns.data(), outs.data(), (int)segs.size(), stream()),
           "sum_splits_multi (16-byte aligned part / out needed)");
}

void colsum(const Tensor& y, int64_t M, int64_t C, const Tensor& part, int64_t splits) {
  check(y, "y", at::kBFloat16, M * C);
  check(part, "part", at::kFloat, splits * C);
  rc_check(rrl_colsum(bf(y), M, C, part.data_ptr<float>(), (int)splits, stream()), "colsum");
}

void sumsq(const Tensor& x, const Tensor& work, const Tensor& out) {
  check(x, "x", at::kFloat, 0);
  check(work, "work", at::kFloat, 1);
  check(out, "out", at::kFloat, 1);
  rc_check(rrl_sumsq(x.data_ptr<float>(), x.numel(), work.data_ptr<float>(), (int)work.numel(),
                     out.data_ptr<float>(), stream()),
           "sumsq");
}

void adam_clip(const Tensor& p, const Tensor& m, const Tensor& v, const Tensor& g, const OptT& shadow,
               const OptT& norm_sq, double max_norm, double lr, double b1, double b2, double eps, int64_t step,
               const OptT& step_dev, int64_t norm_parts) {
  const int64_t n = p.numel();
  check(p, "p", at::kFloat, n);
  check(m, "m", at::kFloat, n);
  check(v, "v", at::kFloat, n);
  check(g, "g", at::kFloat, n);
  const long long* sd = opt_ptr<const long long>(step_dev, "step_dev", at::kLong, 1);
  TORCH_CHECK(sd != nullptr || step >= 1, "adam step must be >= 1");
  uint16_t* sh = opt_ptr<uint16_t>(shadow, "shadow", at::kBFloat16, n);
  TORCH_CHECK(norm_parts >= 0 && norm_parts <= 1024, "adam_clip: norm_parts in 0..1024");
  // norm_parts > 0: norm_sq holds that many sum-of-squares partials, else the squared norm
  const float* ns = opt_ptr<const float>(norm_sq, "norm_sq", at::kFloat, norm_parts > 0 ? norm_parts : 1);
  rc_check(rrl_adam_clip(p.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), g.data_ptr<float>(), sh, n,
                         ns, (float)max_norm, (float)lr, (float)b1, (float)b2, (float)eps, (int)step, sd,
                         (int)norm_parts, stream()),
           "adam_clip");
}

// sum-of-squares partials of x into work (the clip + Adam launch reduces them: norm_parts)
int64_t sumsq_partial(const Tensor& x, const Tensor& work) {
  check(x, "x", at::kFloat, 0);
  check(work, "work", at::kFloat, 0);
  const int g = rrl_sumsq_partial(x.data_ptr<float>(), x.numel(), work.data_ptr<float>(), (int)work.numel(), stream());
  TORCH_CHECK(g > 0, "sumsq_partial failed");
  return g;
}

// several device counters in one launch: [(counter, inc), ...], at most 4 (distinct tensors)
void counter_add_many(const std::vector<std::tuple<Tensor, int64_t>>& adds) {
  TORCH_CHECK(!adds.empty() && adds.size() <= 4, "counter_add_many: 1..4 counters");
  long long* cs[4];
  long long incs[4];
  for (size_t i = 0; i < adds.size(); ++i) {
    const Tensor& c = std::get<0>(adds[i]);
    check(c, "counter", at::kLong, 1);
    cs[i] = (long long*)c.data_ptr();
    incs[i] = std::get<1>(adds[i]);
    for (size_t j = 0; j < i; ++j) TORCH_CHECK(cs[j] != cs[i], "counter_add_many: counters must be distinct");
  }
  rc_check(rrl_counter_add_n(cs, incs, (int)adds.size(), stream()), "counter_add_many");
}

void counter_add(const Tensor& c, int64_t inc) {
  check(c, "counter", at::kLong, 1);
  rc_check(rrl_counter_add((long long*)c.data_ptr(), inc, stream()),
           "counter_add");
}

void to_bf16(const Tensor& x, const Tensor& y) {
  check(x, "x", at::kFloat, 0);
  check(y, "y", at::kBFloat16, x.numel());
  rc_check(rrl_to_bf16(x.data_ptr<float>(), bf(y), x.numel(), stream()), "to_bf16");
}

void a2c_head(int64_t mode, const Tensor& h, const Tensor& head_params, int64_t B, int64_t A, const OptT& act,
              const OptT& logp, const OptT& value, const OptT& logits, int64_t seed, int64_t step,
              int64_t row_offset, const OptT& act_in, const OptT& adv, const OptT& ret, double inv_B, double vf_coef,
              double ent_coef, const OptT& dh, const OptT& dhead, const OptT& stats, int64_t grid,
              const OptT& step_base, const OptT& part, int64_t splits, const OptT& fc_b) {
  constexpr int64_t F = 512;
  TORCH_CHECK(A >= 1 && A <= 16, "a2c_head: 1 <= A <= 16");
  TORCH_CHECK(mode == 0 || mode == 1, "a2c_head: mode must be 0 (rollout) or 1 (train)");
  TORCH_CHECK(grid >= 1, "a2c_head: grid >= 1");
  check(h, "h", at::kBFloat16, B * F);
  check(head_params, "head_params", at::kFloat, (A + 1) * F + A + 1);
  int32_t* ap = opt_ptr<int32_t>(act, "act", at::kInt, B);
  float* lp = opt_ptr<float>(logp, "logp", at::kFloat, B);
  float* vp = opt_ptr<float>(value, "value", at::kFloat, B);
  float* lo = opt_ptr<float>(logits, "logits", at::kFloat, B * A);
  const int32_t* ai = opt_ptr<const int32_t>(act_in, "act_in", at::kInt, mode == 1 ? B : 0);
  const float* ad = opt_ptr<const float>(adv, "adv", at::kFloat, mode == 1 ? B : 0);
  const float* re = opt_ptr<const float>(ret, "ret", at::kFloat, mode == 1 ? B : 0);
  uint16_t* dhp = opt_ptr<uint16_t>(dh, "dh", at::kBFloat16, mode == 1 ? B * F : 0);
  float* dhd = opt_ptr<float>(dhead, "dhead", at::kFloat, mode == 1 ? B * (A + 1) : 0);
  float* st = opt_ptr<float>(stats, "stats", at::kFloat, mode == 1 ? grid * 4 : 0);
  if (mode == 1)
    TORCH_CHECK(ai && ad && re && dhp && dhd && st, "a2c_head train mode needs act_in, adv, ret, dh, dhead, stats");
  const unsigned long long* sb = opt_ptr<const unsigned long long>(step_base, "step_base", at::kLong, 1);
  // part given: h is an OUTPUT, bf16(relu(fc_b + sum of the split-K partials)) (fc.hip)
  const float* pp = opt_ptr<const float>(part, "part", at::kFloat, splits * B * F);
  const float* fb = opt_ptr<const float>(fc_b, "fc_b", at::kFloat, pp ? F : 0);
  if (pp) TORCH_CHECK(mode == 0 && fb && splits >= 1, "a2c_head: part needs mode 0, fc_b and splits >= 1");
  rc_check(rrl_a2c_head((int)mode, bf(h), head_params.data_ptr<float>(), B, A, ap, lp, vp, lo, (uint64_t)seed,
                        (uint64_t)step, sb, (int)row_offset, ai, ad, re, (float)inv_B, (float)vf_coef, (float)ent_coef,
                        dhp, dhd, st, (int)grid, pp, (int)splits, fb, pp ? bf(h) : nullptr, stream()),
           "a2c_head");
}

// fp32 split-K partials part[splits][M][N] of a[M][K] . b[N][K]^T (fc.hip); returns the
// number of splits used.
int64_t fc_nt_part(const Tensor& a, const Tensor& b, const Tensor& part, int64_t M, int64_t N, int64_t K,
                   int64_t splits) {
  TORCH_CHECK(M > 0 && N > 0 && K > 0 && K % 64 == 0 && N % 4 == 0 && splits >= 1, "fc_nt_part: bad shape");
  check(a, "a", at::kBFloat16, M * K);
  check(b, "b", at::kBFloat16, N * K);
  const int64_t kt = K / 64, kps = (kt + splits - 1) / splits, used = (kt + kps - 1) / kps;
  check(part, "part", at::kFloat, used * M * N);
  const int rc = rrl_fc_nt_part(bf(a), bf(b), part.data_ptr<float>(), M, N, K, (int)splits, stream());
  TORCH_CHECK(rc > 0, "fc_nt_part failed with code ", rc);
  return rc;
}

// out[M][N] = (a[M][K] . b[N][K]^T) * (mask[M][N] > 0), bf16 (fc.hip)
void fc_nt_mask(const Tensor& a, const Tensor& b, const Tensor& mask, const Tensor& out, int64_t M, int64_t N,
                int64_t K) {
  TORCH_CHECK(M > 0 && N > 0 && K > 0 && K % 64 == 0 && N % 4 == 0, "fc_nt_mask: bad shape");
  check(a, "a", at::kBFloat16, M * K);
  check(b, "b", at::kBFloat16, N * K);
  check(mask, "mask", at::kBFloat16, M * N);
  check(out, "out", at::kBFloat16, M * N);
  rc_check(rrl_fc_nt_mask(bf(a), bf(b), bf(mask), bf(out), M, N, K, stream()), "fc_nt_mask");
}

// fp32 partials part[splits][I][J] of x[R][I]^T . y[R][J] (fc.hip, the fc weight gradient);
// returns the number of splits used.
int64_t fc_tn_part(const Tensor& x, const Tensor& y, const Tensor& part, int64_t R, int64_t I, int64_t J,
                   int64_t splits, const OptT& ones, const OptT& bias_part) {
  TORCH_CHECK(R >= 64 && R % 64 == 0 && I > 0 && J > 0 && I % 8 == 0 && J % 8 == 0 && splits >= 1,
              "fc_tn_part: bad shape");
  check(x, "x", at::kBFloat16, R * I);
  check(y, "y", at::kBFloat16, R * J);
  const int64_t rt = R / 64, kps = (rt + splits - 1) / splits, used = (rt + kps - 1) / kps;
  check(part, "part", at::kFloat, used * I * J);
  // optional: bias gradient (row sums of x) through a column of ones in the padded last tile
  const uint16_t* on = ones.has_value() && ones->defined() ? (check(*ones, "ones", at::kBFloat16, 8), bf(*ones))
                                                           : nullptr;
  float* bp = opt_ptr<float>(bias_part, "bias_part", at::kFloat, used * I);
  TORCH_CHECK((on == nullptr) == (bp == nullptr) && (!bp || J % 128 != 0),
              "fc_tn_part: ones and bias_part go together and need J % 128 != 0");
  const int rc = rrl_fc_tn_part(bf(x), bf(y), part.data_ptr<float>(), R, I, J, (int)splits, on, bp, stream());
  TORCH_CHECK(rc > 0, "fc_tn_part failed with code ", rc);
  return rc;
}

void transpose_bf16(const Tensor& in, const Tensor& out, int64_t R, int64_t C) {
  TORCH_CHECK(R > 0 && C > 0 && R % 8 == 0 && C % 8 == 0, "transpose_bf16: R, C must be multiples of 8");
  check(in, "in", at::kBFloat16, R * C);
  check(out, "out", at::kBFloat16, R * C);
  rc_check(rrl_transpose_bf16(bf(in), bf(out), R, C, stream()), "transpose_bf16");
}

void head_wgrad(const Tensor& h, const Tensor& dhead, int64_t B, int64_t A, const Tensor& part, int64_t nblk) {
  constexpr int64_t F = 512;
  TORCH_CHECK(A >= 1 && A <= 16 && nblk >= 1, "head_wgrad: bad arguments");
  check(h, "h", at::kBFloat16, B * F);
  check(dhead, "dhead", at::kFloat, B * (A + 1));
  check(part, "part", at::kFloat, nblk * ((A + 1) * F + A + 1));
  rc_check(rrl_head_wgrad(bf(h), dhead.data_ptr<float>(), B, A, part.data_ptr<float>(), nblk, stream()),
           "head_wgrad");
}

int64_t pong_state_size() { return rrl_pong_state_size(); }

void pong_step(const Tensor& state, const Tensor& act, const Tensor& rew, const Tensor& done, const Tensor& fin_ret,
               const Tensor& fin_len, const OptT& ep_acc, int64_t N, int64_t seed, int64_t step, int64_t max_steps,
               bool reset_all, const OptT& step_base, const OptT& obs, const OptT& hist, const OptT& frames,
               const OptT& fidx, int64_t ring_slots) {
  check(state, "state", at::kFloat, N * pong_state_size());
  check(act, "act", at::kInt, reset_all ? 0 : N);
  check(rew, "rew", at::kFloat, N);
  check(done, "done", at::kFloat, N);
  check(fin_ret, "fin_ret", at::kFloat, N);
  check(fin_len, "fin_len", at::kFloat, N);
  float* acc = opt_ptr<float>(ep_acc, "ep_acc", at::kFloat, 4 * N);
  const unsigned long long* sb = opt_ptr<const unsigned long long>(step_base, "step_base", at::kLong, 1);
  if (frames.has_value() && frames->defined()) {  // step + ONE new frame into the frame ring (pong.hip)
    uint8_t* fp = ring_store(frames, fidx, N, ring_slots);
    rc_check(rrl_pong_step_render(state.data_ptr<float>(), act.data_ptr<int32_t>(), rew.data_ptr<float>(),
                                  done.data_ptr<float>(), fin_ret.data_ptr<float>(), fin_len.data_ptr<float>(), acc,
                                  nullptr, (int)N, (uint64_t)seed, (uint64_t)step, sb, (int)max_steps,
                                  reset_all ? 1 : 0, fp, fidx->data_ptr<int32_t>(), (int)ring_slots, stream()),
             "pong_step_render (frame ring)");
    return;
  }
  if (obs.has_value() && obs->defined()) {  // step + render in one launch (pong.hip)
    check(*obs, "obs", at::kByte, N * 84 * 84 * 4);
    rc_check(rrl_pong_step_render(state.data_ptr<float>(), act.data_ptr<int32_t>(), rew.data_ptr<float>(),
                                  done.data_ptr<float>(), fin_ret.data_ptr<float>(), fin_len.data_ptr<float>(), acc,
                                  obs->data_ptr<uint8_t>(), (int)N, (uint64_t)seed, (uint64_t)step, sb,
                                  (int)max_steps, reset_all ? 1 : 0, nullptr, nullptr, 0, stream()),
             "pong_step_render");
    return;
  }
  float* hout = opt_ptr<float>(hist, "hist", at::kFloat, N * 16);  // the new frame histories (fused render)
  rc_check(rrl_pong_step(state.data_ptr<float>(), act.data_ptr<int32_t>(), rew.data_ptr<float>(),
                         done.data_ptr<float>(), fin_ret.data_ptr<float>(), fin_len.data_ptr<float>(), acc, (int)N,
                         (uint64_t)seed, (uint64_t)step, sb, (int)max_steps, reset_all ? 1 : 0, hout, stream()),
           "pong_step");
}

// Fused rollout step (pong.hip): the policy head from the fc split-K partials + env step +
// render, one workgroup per env.  Same outputs as a2c_head(mode 0, part=...) then pong_step(obs=...).
void pong_head_step(const Tensor& part, int64_t splits, const Tensor& fc_b, const Tensor& head_params, int64_t A,
                    const Tensor& h_out, const Tensor& act, const Tensor& logp, const Tensor& value, int64_t sample_seed,
                    int64_t sample_step, const OptT& sample_base, const Tensor& state, const Tensor& rew,
                    const Tensor& done, const Tensor& fin_ret, const Tensor& fin_len, const OptT& ep_acc,
                    const OptT& obs, int64_t N, int64_t seed, int64_t step, const OptT& step_base,
                    int64_t max_steps, const OptT& frames, const OptT& fidx, int64_t ring_slots) {
  constexpr int64_t F = 512;
  TORCH_CHECK(A >= 1 && A <= 8 && splits >= 1 && N >= 1, "pong_head_step: 1 <= A <= 8, splits >= 1");
  check(part, "part", at::kFloat, splits * N * F);
  check(fc_b, "fc_b", at::kFloat, F);
  check(head_params, "head_params", at::kFloat, A * F + A + F + 1);
  check(h_out, "h_out", at::kBFloat16, N * F);
  check(act, "act", at::kInt, N);
  check(logp, "logp", at::kFloat, N);
  check(value, "value", at::kFloat, N);
  check(state, "state", at::kFloat, N * pong_state_size());
  check(rew, "rew", at::kFloat, N);
  check(done, "done", at::kFloat, N);
  check(fin_ret, "fin_ret", at::kFloat, N);
  check(fin_len, "fin_len", at::kFloat, N);
  uint8_t* fp = nullptr;
  uint8_t* op = nullptr;
  if (frames.has_value() && frames->defined()) {
    fp = ring_store(frames, fidx, N, ring_slots);
  } else {
    TORCH_CHECK(obs.has_value() && obs->defined(), "pong_head_step: obs or frames + fidx is required");
    check(*obs, "obs", at::kByte, N * 84 * 84 * 4);
    op = obs->data_ptr<uint8_t>();
  }
  float* acc = opt_ptr<float>(ep_acc, "ep_acc", at::kFloat, 4 * N);
  const unsigned long long* sb = opt_ptr<const unsigned long long>(step_base, "step_base", at::kLong, 1);
  const unsigned long long* ssb = opt_ptr<const unsigned long long>(sample_base, "sample_base", at::kLong, 1);
  rc_check(rrl_pong_head_step_render(part.data_ptr<float>(), (int)splits, fc_b.data_ptr<float>(),
                                     head_params.data_ptr<float>(), (int)A, bf(h_out), act.data_ptr<int32_t>(),
                                     logp.data_ptr<float>(), value.data_ptr<float>(), (uint64_t)sample_seed,
                                     (uint64_t)sample_step, ssb, state.data_ptr<float>(), rew.data_ptr<float>(),
                                     done.data_ptr<float>(), fin_ret.data_ptr<float>(), fin_len.data_ptr<float>(), acc,
                                     op, (int)N, (uint64_t)seed, (uint64_t)step, sb, (int)max_steps, fp,
                                     fp ? fidx->data_ptr<int32_t>() : nullptr, (int)ring_slots, stream()),
           "pong_head_step");
}

// The frame ring rebuilt from the env state (a restore): frames of steps st - 3 .. st, fidx [N][4]
void pong_ring_fill(const Tensor& state, const Tensor& frames, const Tensor& fidx, int64_t N, int64_t ring_slots,
                    int64_t step, const OptT& step_base) {
  check(state, "state", at::kFloat, N * pong_state_size());
  uint8_t* fp = ring_store(frames, fidx, N, ring_slots);
  const unsigned long long* sb = opt_ptr<const unsigned long long>(step_base, "step_base", at::kLong, 1);
  rc_check(rrl_pong_ring_fill(state.data_ptr<float>(), fp, fidx.data_ptr<int32_t>(), (int)N, (int)ring_slots,
                              (uint64_t)step, sb, stream()),
           "pong_ring_fill");
}

// s2d observations drawn from frame histories [N][16] (the fused-render path's reference)
void pong_render_hist(const Tensor& hist, const Tensor& obs, int64_t N) {
  check(hist, "hist", at::kFloat, N * 16);
  check(obs, "obs", at::kByte, N * 84 * 84 * 4);
  rc_check(rrl_pong_render_hist(hist.data_ptr<float>(), obs.data_ptr<uint8_t>(), (int)N, stream()), "pong_render_hist");
}

void pong_render(const Tensor& state, const Tensor& obs, int64_t N) {
  check(state, "state", at::kFloat, N * pong_state_size());
  check(obs, "obs", at::kByte, N * 84 * 84 * 4);  // [N][21][21][64] space-to-depth
  rc_check(rrl_pong_render(state.data_ptr<float>(), obs.data_ptr<uint8_t>(), (int)N, stream()), "pong_render");
}

}  // namespace

void register_cnn_ops(pybind11::module_& m) {
  m.def("conv_fwd", &conv_fwd, pybind11::arg("x"), pybind11::arg("w"), pybind11::arg("b"), pybind11::arg("y"),
        pybind11::arg("N"), pybind11::arg("H"), pybind11::arg("W"), pybind11::arg("C"), pybind11::arg("KH"),
        pybind11::arg("KW"), pybind11::arg("S"), pybind11::arg("Cout"), pybind11::arg("relu"),
        pybind11::arg("work") = pybind11::none());
  m.def("gemm_dgrad", &gemm_dgrad);
  m.def("conv_stack_fwd", &conv_stack_fwd, pybind11::arg("x"), pybind11::arg("w1"), pybind11::arg("b1"),
        pybind11::arg("w2"), pybind11::arg("b2"), pybind11::arg("w3"), pybind11::arg("b3"), pybind11::arg("y1"),
        pybind11::arg("y2"), pybind11::arg("y3"), pybind11::arg("N"), pybind11::arg("probe") = 0,
        pybind11::arg("grid") = 0, pybind11::arg("store12") = true, pybind11::arg("hist") = pybind11::none(),
        pybind11::arg("frames") = pybind11::none(), pybind11::arg("fidx") = pybind11::none());
  m.def("conv3_bwd", &conv3_bwd, pybind11::arg("dy"), pybind11::arg("w"), pybind11::arg("xact"), pybind11::arg("dx"),
        pybind11::arg("part"), pybind11::arg("bias_part"), pybind11::arg("N"), pybind11::arg("grid"),
        pybind11::arg("variant") = 0);
  m.def("conv2_bwd", &conv2_bwd, pybind11::arg("dy"), pybind11::arg("w"), pybind11::arg("xact"), pybind11::arg("dx"),
        pybind11::arg("part"), pybind11::arg("bias_part"), pybind11::arg("N"), pybind11::arg("grid"),
        pybind11::arg("staged") = 0);
  m.def("conv1_wgrad8", &conv1_wgrad8, pybind11::arg("x"), pybind11::arg("dy"), pybind11::arg("part"),
        pybind11::arg("bias_part"), pybind11::arg("N"), pybind11::arg("grid"), pybind11::arg("hist") = pybind11::none(),
        pybind11::arg("frames") = pybind11::none(), pybind11::arg("fidx") = pybind11::none(),
        pybind11::arg("env_major_T") = 0);
  m.def("col2im_mask", &col2im_mask);
  m.def("conv_dgrad", &conv_dgrad);
  m.def("gemm_splits", &gemm_splits);
  m.def("conv_wgrad", &conv_wgrad, pybind11::arg("dy"), pybind11::arg("x"), pybind11::arg("part"),
        pybind11::arg("splits"), pybind11::arg("N"), pybind11::arg("H"), pybind11::arg("W"), pybind11::arg("C"),
        pybind11::arg("KH"), pybind11::arg("KW"), pybind11::arg("S"), pybind11::arg("Cout"),
        pybind11::arg("bias_part") = pybind11::none());
  m.def("sum_splits", &sum_splits);
  m.def("colsum", &colsum);
  m.def("sum_splits_multi", &sum_splits_multi);
  m.def("sumsq", &sumsq);
  m.def("adam_clip", &adam_clip, pybind11::arg("p"), pybind11::arg("m"), pybind11::arg("v"), pybind11::arg("g"),
        pybind11::arg("shadow"), pybind11::arg("norm_sq"), pybind11::arg("max_norm"), pybind11::arg("lr"),
        pybind11::arg("b1"), pybind11::arg("b2"), pybind11::arg("eps"), pybind11::arg("step"),
        pybind11::arg("step_dev") = pybind11::none(), pybind11::arg("norm_parts") = 0);
  m.def("sumsq_partial", &sumsq_partial);
  m.def("counter_add", &counter_add);
  m.def("counter_add_many", &counter_add_many);
  m.def("to_bf16", &to_bf16);
  m.def("a2c_head", &a2c_head, pybind11::arg("mode"), pybind11::arg("h"), pybind11::arg("head_params"),
        pybind11::arg("B"), pybind11::arg("A"), pybind11::arg("act"), pybind11::arg("logp"), pybind11::arg("value"),
        pybind11::arg("logits"), pybind11::arg("seed"), pybind11::arg("step"), pybind11::arg("row_offset"),
        pybind11::arg("act_in"), pybind11::arg("adv"), pybind11::arg("ret"), pybind11::arg("inv_B"),
        pybind11::arg("vf_coef"), pybind11::arg("ent_coef"), pybind11::arg("dh"), pybind11::arg("dhead"),
        pybind11::arg("stats"), pybind11::arg("grid"), pybind11::arg("step_base") = pybind11::none(),
        pybind11::arg("part") = pybind11::none(), pybind11::arg("splits") = 0,
        pybind11::arg("fc_b") = pybind11::none());
  m.def("fc_nt_part", &fc_nt_part);
  m.def("fc_nt_mask", &fc_nt_mask);
  m.def("transpose_bf16", &transpose_bf16);
  m.def("fc_tn_part", &fc_tn_part, pybind11::arg("x"), pybind11::arg("y"), pybind11::arg("part"), pybind11::arg("R"),
        pybind11::arg("I"), pybind11::arg("J"), pybind11::arg("splits"), pybind11::arg("ones") = pybind11::none(),
        pybind11::arg("bias_part") = pybind11::none());
  m.def("head_wgrad", &head_wgrad);
  m.def("pong_state_size", &pong_state_size);
  m.def("pong_step", &pong_step, pybind11::arg("state"), pybind11::arg("act"), pybind11::arg("rew"),
        pybind11::arg("done"), pybind11::arg("fin_ret"), pybind11::arg("fin_len"), pybind11::arg("ep_acc"),
        pybind11::arg("N"), pybind11::arg("seed"), pybind11::arg("step"), pybind11::arg("max_steps"),
        pybind11::arg("reset_all"), pybind11::arg("step_base") = pybind11::none(),
        pybind11::arg("obs") = pybind11::none(), pybind11::arg("hist") = pybind11::none(),
        pybind11::arg("frames") = pybind11::none(), pybind11::arg("fidx") = pybind11::none(),
        pybind11::arg("ring_slots") = 0);
  m.def("pong_head_step", &pong_head_step, pybind11::arg("part"), pybind11::arg("splits"), pybind11::arg("fc_b"),
        pybind11::arg("head_params"), pybind11::arg("A"), pybind11::arg("h_out"), pybind11::arg("act"),
        pybind11::arg("logp"), pybind11::arg("value"), pybind11::arg("sample_seed"), pybind11::arg("sample_step"),
        pybind11::arg("sample_base"), pybind11::arg("state"), pybind11::arg("rew"), pybind11::arg("done"),
        pybind11::arg("fin_ret"), pybind11::arg("fin_len"), pybind11::arg("ep_acc"), pybind11::arg("obs"),
        pybind11::arg("N"), pybind11::arg("seed"), pybind11::arg("step"), pybind11::arg("step_base"),
        pybind11::arg("max_steps"), pybind11::arg("frames") = pybind11::none(), pybind11::arg("fidx") = pybind11::none(),
        pybind11::arg("ring_slots") = 0);
  m.def("pong_ring_fill", &pong_ring_fill, pybind11::arg("state"), pybind11::arg("frames"), pybind11::arg("fidx"),
        pybind11::arg("N"), pybind11::arg("ring_slots"), pybind11::arg("step"), pybind11::arg("step_base") = pybind11::none());
  m.def("pong_render", &pong_render);
  m.def("pong_render_hist", &pong_render_hist);
}
