// PyTorch bindings for the gfx950 HIP kernels (csrc/kernels/*.hip).
//
// The kernels are compiled by hipcc into plain objects with a C ABI; this file is
// compiled by the host C++ compiler against the PyTorch-ROCm headers, validates every
// tensor (device, dtype, contiguity, shape) BEFORE a launch so that a bad call raises a
// Python exception instead of faulting the GPU, and launches on the current HIP stream
// (so everything here is capturable into a hipGraph via torch.cuda.graph).
#include <ATen/hip/HIPContext.h>
#include <torch/extension.h>

#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstdint>
#include <optional>
#include <vector>

extern "C" {
int rrl_mlp_forward(int mode, const float* params, const float* X, int B, int D, int A, int H,
                    const float* mask, const int* act_in, const float* actc_in, int* act_out,
                    float* actc_out, float* out0, float* out1, float* logits_out, uint64_t seed,
                    uint64_t step, uint32_t row_offset, const float* gate, float* x_copy, int* act_host,
                    float* actc_host, int num_cu, void* stream);
int rrl_mlp_grad_slabs(int B, int num_cu);
int rrl_set_value_grad_mode(int mode);
int rrl_set_value_fwd_mode(int mode);
int rrl_set_value_grad_tune(int tune);
void rrl_set_value_grad_stamps(void* buf);
int rrl_mlp_grad(int head, const float* params, const float* X, int B, int D, int A, int H,
                 const float* mask, const int* act, const float* actc, const float* adv, const float* ret,
                 const float* logp_old, const float* adv_stats, float inv_B, float clip_eps, float ent_coef,
                 float* grad_slab, float* loss_slab, int P, const int* nvalid, const float* inv_B_dev, int num_cu, void* stream);
int rrl_scan_tm_parts(int N);
int rrl_gae_scan_tm(const float* rew, const float* done, const float* val, const float* tval, float* adv,
                    float* ret, float* stats_part, float* stats_out, int K, int T, int N, float gamma,
                    float lam, long long* const* cnt, const long long* inc, int ncnt, void* stream);
int rrl_scan_flat_blocks(int L);
int rrl_scan_flat(const float* rew, const float* done, const float* val, const float* boot, float* adv,
                  float* ret, float* work, float* stats_out, int L, float gamma, float lam, void* stream);
int rrl_stats_reduce(const float* part, int nparts, float* out, void* stream);
int rrl_column_sums(const float* part, int rows, int ld, int cols, double* out, void* stream);
int rrl_adam(float* param, float* m, float* v, const float* grad, const float* slab, int nslab,
             float* grad_out, int* step, unsigned* ticket, int P, float lr, float beta1, float beta2,
             float eps, float grad_scale, float weight_decay, int step_add, int step_inc, void* stream);
int rrl_reduce_slabs(const float* slab, int nslab, int P, float scale, float* out, void* stream);
int rrl_env_dims(int env, int* D, int* A, int* NS, int* max_steps);
int rrl_rollout_cont(int env, const float* params, const float* env_consts, int N, int T, int H, float* state,
                     int* ep_len, float* ep_ret, float* obs_buf, float* act_buf, float* logp_buf, float* rew_buf,
                     float* done_buf, float* tobs_buf, float* ep_stats, uint64_t seed, uint64_t step0,
                     int reset_all, int max_steps, int num_cu, void* stream);
int rrl_rollout_grid(int N, int num_cu);
int rrl_rollout(int env, const float* params, int N, int T, int H, float* state, int* ep_len, float* ep_ret,
                float* obs_buf, int* act_buf, float* logp_buf, float* rew_buf, float* done_buf,
                float* tobs_buf, float* ep_stats, uint64_t seed, uint64_t step0, int reset_all, int max_steps,
                int num_cu, void* stream);
}

namespace {

using at::Tensor;
using OptT = std::optional<Tensor>;

int g_cu_limit = 0;  // > 0: size every grid for this many CUs (set_cu_limit)

int device_cus() {
  static int n = -1;
  if (n < 0) n = at::cuda::getCurrentDeviceProperties()->multiProcessorCount;
  return n;
}

// CUs the grids of this process are sized for: all of them, or the learner's share when the
// host-env trainer partitions the chip between its actor and learner streams.
int num_cus() { return g_cu_limit > 0 ? std::min(g_cu_limit, device_cus()) : device_cus(); }

int64_t set_cu_limit(int64_t n) {
  const int64_t prev = g_cu_limit;
  g_cu_limit = (int)std::max<int64_t>(n, 0);
  return prev;
}

// A stream whose kernels run only on the listed CUs (hipExtStreamCreateWithCUMask): the
// actor / learner partition of the overlapped host-env trainer, so the rollout's sampling
// launches never queue behind the learner's persistent one-workgroup-per-CU kernels.
int64_t cu_masked_stream(const std::vector<int64_t>& cus) {
  const int n = device_cus();
  std::vector<uint32_t> mask((n + 31) / 32, 0u);
  for (int64_t c : cus) {
    TORCH_CHECK(c >= 0 && c < n, "CU index ", c, " out of range [0, ", n, ")");
    mask[c / 32] |= 1u << (c % 32);
  }
  hipStream_t st = nullptr;
  const hipError_t e = hipExtStreamCreateWithCUMask(&st, (uint32_t)mask.size(), mask.data());
  TORCH_CHECK(e == hipSuccess, "hipExtStreamCreateWithCUMask: ", hipGetErrorString(e));
  return (int64_t)(uintptr_t)st;
}

void destroy_stream(int64_t st) {
  if (st) (void)hipStreamDestroy((hipStream_t)(uintptr_t)st);
}

void* cur_stream() { return (void*)at::hip::getCurrentHIPStream().stream(); }

void check_dev(const Tensor& t, const char* name, at::ScalarType dt) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.scalar_type() == dt, name, " has dtype ", t.scalar_type(), ", expected ", dt);
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}
void check_numel(const Tensor& t, const char* name, int64_t n) {
  TORCH_CHECK(t.numel() >= n, name, " has ", t.numel(), " elements, need >= ", n);
}
const float* fptr(const OptT& t, const char* name, int64_t n) {
  if (!t.has_value() || !t->defined()) return nullptr;
  check_dev(*t, name, at::kFloat);
  check_numel(*t, name, n);
  return t->data_ptr<float>();
}
float* fptr_mut(const OptT& t, const char* name, int64_t n) { return const_cast<float*>(fptr(t, name, n)); }
const int* iptr(const OptT& t, const char* name, int64_t n) {
  if (!t.has_value() || !t->defined()) return nullptr;
  check_dev(*t, name, at::kInt);
  check_numel(*t, name, n);
  return t->data_ptr<int>();
}

int64_t flat_size(int64_t D, int64_t H, int64_t A, bool log_std) {
  return H * D + H + H * H + H + A * H + A + (log_std ? A : 0);
}

void check_rc(int rc, const char* what) {
  TORCH_CHECK(rc == 0, what, " failed with code ", rc, " (", (rc > 0 ? hipGetErrorString((hipError_t)rc) : "bad argument"), ")");
}

void mlp_forward(int64_t mode, const Tensor& params, const Tensor& X, int64_t A, int64_t H, const OptT& mask,
                 const OptT& act_in, const OptT& actc_in, const OptT& act_out, const OptT& actc_out,
                 const Tensor& out0, const OptT& out1, const OptT& logits_out, int64_t seed, int64_t step,
                 int64_t row_offset, const OptT& gate) {
  check_dev(params, "params", at::kFloat);
  check_dev(X, "X", at::kFloat);
  TORCH_CHECK(X.dim() == 2, "X must be [B, D]");
  const int64_t B = X.size(0), D = X.size(1);
  TORCH_CHECK(H == 64 || H == 128, "hidden size must be 64 or 128");
  TORCH_CHECK(D >= 1 && D <= 32, "obs dim must be in [1, 32]");
  TORCH_CHECK(A >= 1 && A <= 16, "act dim must be in [1, 16]");
  TORCH_CHECK(mode >= 0 && mode <= 5, "bad mode");
  const bool gauss = mode == 4 || mode == 5;
  const int64_t Aeff = mode == 0 ? 1 : A;
  check_numel(params, "params", flat_size(D, H, Aeff, gauss));
  check_dev(out0, "out0", at::kFloat);
  check_numel(out0, "out0", B);
  const float* m = fptr(mask, "mask", B * A);
  const int* ai = iptr(act_in, "act_in", mode == 2 ? B : 0);
  const float* ci = fptr(actc_in, "actc_in", mode == 5 ? B * A : 0);
  if (mode == 2) TORCH_CHECK(ai != nullptr, "act_in required for CAT_EVAL");
  if (mode == 5) TORCH_CHECK(ci != nullptr, "actc_in required for GAUSS_EVAL");
  int* ao = const_cast<int*>(iptr(act_out, "act_out", mode == 1 ? B : 0));
  if (mode == 1) TORCH_CHECK(ao != nullptr, "act_out required for CAT_SAMPLE");
  float* co = fptr_mut(actc_out, "actc_out", mode == 4 ? B * A : 0);
  if (mode == 4) TORCH_CHECK(co != nullptr, "actc_out required for GAUSS_SAMPLE");
  float* o1 = fptr_mut(out1, "out1", B);
  float* lo = fptr_mut(logits_out, "logits_out", B * A);
  if (mode == 3) TORCH_CHECK(lo != nullptr, "logits_out required for LOGITS");
  const float* gt = fptr(gate, "gate", B);
  TORCH_CHECK(gt == nullptr || mode == 0, "gate applies to the VALUE mode only");
  const int rc = rrl_mlp_forward((int)mode, params.data_ptr<float>(), X.data_ptr<float>(), (int)B, (int)D, (int)A,
                                 (int)H, m, ai, ci, ao, co, out0.data_ptr<float>(), o1, lo, (uint64_t)seed,
                                 (uint64_t)step, (uint32_t)row_offset, gt, nullptr, nullptr, nullptr, num_cus(),
                                 cur_stream());
  check_rc(rc, "mlp_forward");
}

int64_t mlp_grad_slabs(int64_t B) { return rrl_mlp_grad_slabs((int)B, num_cus()); }

void mlp_grad(int64_t head, const Tensor& params, const Tensor& X, int64_t A, int64_t H, const OptT& mask,
              const OptT& act, const OptT& actc, const OptT& adv, const OptT& ret, const OptT& logp_old,
              const OptT& adv_stats, double inv_B, double clip_eps, double ent_coef, const Tensor& grad_slab,
              const Tensor& loss_slab, const OptT& nvalid, const OptT& inv_B_dev) {
  check_dev(params, "params", at::kFloat);
  check_dev(X, "X", at::kFloat);
  TORCH_CHECK(X.dim() == 2, "X must be [B, D]");
  const int64_t B = X.size(0), D = X.size(1);
  TORCH_CHECK(H == 64 || H == 128, "hidden size must be 64 or 128");
  TORCH_CHECK(D >= 1 && D <= 32, "obs dim must be in [1, 32]");
  TORCH_CHECK(A >= 1 && A <= 16, "act dim must be in [1, 16]");
  TORCH_CHECK(head >= 0 && head <= 4, "bad head");
  TORCH_CHECK(B * std::max<int64_t>(D, A) < (int64_t)INT32_MAX, "batch too large for 32-bit row indexing");
  const bool gauss = head == 3 || head == 4;
  const bool cat = head == 0 || head == 2;
  const int64_t Aeff = head == 1 ? 1 : A;
  const int64_t P = flat_size(D, H, Aeff, gauss);
  check_numel(params, "params", P);
  const int64_t nslab = mlp_grad_slabs(B);
  check_dev(grad_slab, "grad_slab", at::kFloat);
  check_numel(grad_slab, "grad_slab", nslab * P);
  check_dev(loss_slab, "loss_slab", at::kFloat);
  check_numel(loss_slab, "loss_slab", nslab * 8);
  const float* m = fptr(mask, "mask", B * A);
  const int* a = iptr(act, "act", cat ? B : 0);
  if (cat) TORCH_CHECK(a != nullptr, "act required for categorical heads");
  const float* ac = fptr(actc, "actc", gauss ? B * A : 0);
  if (gauss) TORCH_CHECK(ac != nullptr, "actc required for Gaussian heads");
  const float* ad = fptr(adv, "adv", B);
  if (head != 1) TORCH_CHECK(ad != nullptr, "adv required for policy heads");
  const float* rt = fptr(ret, "ret", B);
  if (head == 1) TORCH_CHECK(rt != nullptr, "ret required for the value head");
  const float* lpo = fptr(logp_old, "logp_old", B);
  if (head == 2 || head == 3) TORCH_CHECK(lpo != nullptr, "logp_old required for PPO heads");
  const float* st = fptr(adv_stats, "adv_stats", 3);
  // device-side batch shape (graph replays with a changing batch): valid rows / 1 / global rows
  const int* nv = iptr(nvalid, "nvalid", 1);
  const float* ibd = fptr(inv_B_dev, "inv_B_dev", 1);
  const int rc = rrl_mlp_grad((int)head, params.data_ptr<float>(), X.data_ptr<float>(), (int)B, (int)D, (int)A,
                              (int)H, m, a, ac, ad, rt, lpo, st, (float)inv_B, (float)clip_eps, (float)ent_coef,
                              grad_slab.data_ptr<float>(), loss_slab.data_ptr<float>(), (int)P, nv, ibd, num_cus(),
                              cur_stream());
  check_rc(rc, "mlp_grad");
}

int64_t scan_tm_parts(int64_t N) { return rrl_scan_tm_parts((int)N); }

void gae_scan_tm(const Tensor& rew, const Tensor& done, const OptT& val, const OptT& tval, const Tensor& adv,
                 const Tensor& ret, const Tensor& stats_part, const OptT& stats_out, double gamma, double lam,
                 const std::vector<std::tuple<Tensor, int64_t>>& counters) {
  // rew [T, N] or [K, T, N] (K actor blocks of one learner shard); val [K*T*N + K*N]
  check_dev(rew, "rew", at::kFloat);
  TORCH_CHECK(rew.dim() == 2 || rew.dim() == 3, "rew must be [T, N] or [K, T, N]");
  const int64_t K = rew.dim() == 3 ? rew.size(0) : 1;
  const int64_t T = rew.size(rew.dim() - 2), N = rew.size(rew.dim() - 1);
  check_dev(done, "done", at::kFloat);
  check_numel(done, "done", K * T * N);
  const float* v = fptr(val, "val", K * (T + 1) * N);
  const float* tv = fptr(tval, "tval", K * T * N);
  check_dev(adv, "adv", at::kFloat);
  check_numel(adv, "adv", K * T * N);
  check_dev(ret, "ret", at::kFloat);
  check_numel(ret, "ret", K * T * N);
  check_dev(stats_part, "stats_part", at::kFloat);
  check_numel(stats_part, "stats_part", scan_tm_parts(K * N) * 3);
  float* so = fptr_mut(stats_out, "stats_out", 3);
  // device step counters advanced by the same launch (int64 scalars on this device)
  TORCH_CHECK(counters.size() <= 3, "gae_scan_tm: at most 3 counters");
  long long* cnt[3] = {nullptr, nullptr, nullptr};
  long long inc[3] = {0, 0, 0};
  for (size_t q = 0; q < counters.size(); ++q) {
    const Tensor& c = std::get<0>(counters[q]);
    TORCH_CHECK(c.is_cuda() && c.scalar_type() == at::kLong && c.numel() == 1, "gae_scan_tm: counter must be an int64 scalar on the device");
    cnt[q] = reinterpret_cast<long long*>(c.data_ptr<int64_t>());
    inc[q] = (long long)std::get<1>(counters[q]);
  }
  const int rc = rrl_gae_scan_tm(rew.data_ptr<float>(), done.data_ptr<float>(), v, tv, adv.data_ptr<float>(),
                                 ret.data_ptr<float>(), stats_part.data_ptr<float>(), so, (int)K, (int)T, (int)N,
                                 (float)gamma, (float)lam, cnt, inc, (int)counters.size(), cur_stream());
  check_rc(rc, "gae_scan_tm");
}

int64_t scan_flat_blocks(int64_t L) { return rrl_scan_flat_blocks((int)L); }

void scan_flat(const Tensor& rew, const Tensor& done, const OptT& val, const OptT& boot, const Tensor& adv,
               const Tensor& ret, const Tensor& work, const OptT& stats_out, double gamma, double lam) {
  check_dev(rew, "rew", at::kFloat);
  const int64_t L = rew.numel();
  check_dev(done, "done", at::kFloat);
  check_numel(done, "done", L);
  const float* v = fptr(val, "val", L);
  const float* b = fptr(boot, "boot", L);
  check_dev(adv, "adv", at::kFloat);
  check_numel(adv, "adv", L);
  check_dev(ret, "ret", at::kFloat);
  check_numel(ret, "ret", L);
  check_dev(work, "work", at::kFloat);
  check_numel(work, "work", scan_flat_blocks(L) * 9);
  float* so = fptr_mut(stats_out, "stats_out", 3);
  const int rc = rrl_scan_flat(rew.data_ptr<float>(), done.data_ptr<float>(), v, b, adv.data_ptr<float>(),
                               ret.data_ptr<float>(), work.data_ptr<float>(), so, (int)L, (float)gamma, (float)lam,
                               cur_stream());
  check_rc(rc, "scan_flat");
}

void stats_reduce(const Tensor& part, const Tensor& out) {
  check_dev(part, "part", at::kFloat);
  TORCH_CHECK(part.numel() % 3 == 0, "part must be [n, 3]");
  check_dev(out, "out", at::kFloat);
  check_numel(out, "out", 3);
  check_rc(rrl_stats_reduce(part.data_ptr<float>(), (int)(part.numel() / 3), out.data_ptr<float>(), cur_stream()),
           "stats_reduce");
}

void column_sums(const Tensor& part, int64_t cols, const Tensor& out) {
  check_dev(part, "part", at::kFloat);
  TORCH_CHECK(part.dim() == 2 && part.is_contiguous(), "column_sums: part must be a contiguous [rows, ld] tensor");
  TORCH_CHECK(cols >= 1 && cols <= 8 && cols <= part.size(1), "column_sums: 1 <= cols <= min(8, ld)");
  TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kDouble && out.numel() >= cols && out.is_contiguous(),
              "column_sums: out must be a contiguous float64 device tensor of >= cols elements");
  check_rc(rrl_column_sums(part.data_ptr<float>(), (int)part.size(0), (int)part.size(1), (int)cols,
                           out.data_ptr<double>(), cur_stream()),
           "column_sums");
}

void adam(const Tensor& param, const Tensor& m, const Tensor& v, const OptT& grad, const OptT& slab,
          const OptT& grad_out, const Tensor& step, const Tensor& ticket, double lr, double beta1, double beta2,
          double eps, double grad_scale, double weight_decay, int64_t step_add, int64_t step_inc) {
  check_dev(param, "param", at::kFloat);
  const int64_t P = param.numel();
  check_dev(m, "m", at::kFloat);
  check_numel(m, "m", P);
  check_dev(v, "v", at::kFloat);
  check_numel(v, "v", P);
  const float* g = fptr(grad, "grad", P);
  const float* s = nullptr;
  int64_t nslab = 0;
  if (slab.has_value() && slab->defined()) {
    check_dev(*slab, "slab", at::kFloat);
    TORCH_CHECK(slab->dim() == 2 && slab->size(1) == P, "slab must be [nslab, P]");
    nslab = slab->size(0);
    s = slab->data_ptr<float>();
  }
  TORCH_CHECK((g != nullptr) != (s != nullptr), "exactly one of grad / slab must be given");
  float* go = fptr_mut(grad_out, "grad_out", P);
  check_dev(step, "step", at::kInt);
  check_dev(ticket, "ticket", at::kInt);
  const int rc = rrl_adam(param.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), g, s, (int)nslab, go,
                          step.data_ptr<int>(), reinterpret_cast<unsigned*>(ticket.data_ptr<int>()), (int)P, (float)lr,
                          (float)beta1, (float)beta2, (float)eps, (float)grad_scale, (float)weight_decay,
                          (int)step_add, (int)step_inc, cur_stream());
  check_rc(rc, "adam");
}

void reduce_slabs(const Tensor& slab, double scale, const Tensor& out) {
  check_dev(slab, "slab", at::kFloat);
  TORCH_CHECK(slab.dim() == 2, "slab must be [nslab, P]");
  check_dev(out, "out", at::kFloat);
  check_numel(out, "out", slab.size(1));
  check_rc(rrl_reduce_slabs(slab.data_ptr<float>(), (int)slab.size(0), (int)slab.size(1), (float)scale,
                            out.data_ptr<float>(), cur_stream()),
           "reduce_slabs");
}

std::tuple<int64_t, int64_t, int64_t, int64_t> env_dims(int64_t env) {
  int D = 0, A = 0, NS = 0, ms = 0;
  TORCH_CHECK(rrl_env_dims((int)env, &D, &A, &NS, &ms) == 0, "unknown device env id ", env);
  return {D, A, NS, ms};
}

int64_t rollout_grid(int64_t N) { return rrl_rollout_grid((int)N, num_cus()); }

void rollout(int64_t env, const Tensor& params, int64_t H, const Tensor& state, const Tensor& ep_len,
             const Tensor& ep_ret, const Tensor& obs_buf, const Tensor& act_buf, const Tensor& logp_buf,
             const Tensor& rew_buf, const Tensor& done_buf, const OptT& tobs_buf, const Tensor& ep_stats,
             int64_t seed, int64_t step0, bool reset_all, int64_t max_steps) {
  auto [D, A, NS, ms] = env_dims(env);
  (void)ms;
  TORCH_CHECK(H == 64 || H == 128, "hidden size must be 64 or 128");
  check_dev(params, "params", at::kFloat);
  check_numel(params, "params", flat_size(D, H, A, false));
  check_dev(act_buf, "act_buf", at::kInt);
  TORCH_CHECK(act_buf.dim() == 2, "act_buf must be [T, N]");
  const int64_t T = act_buf.size(0), N = act_buf.size(1);
  check_dev(state, "state", at::kFloat);
  check_numel(state, "state", N * NS);
  check_dev(ep_len, "ep_len", at::kInt);
  check_numel(ep_len, "ep_len", N);
  check_dev(ep_ret, "ep_ret", at::kFloat);
  check_numel(ep_ret, "ep_ret", N);
  check_dev(obs_buf, "obs_buf", at::kFloat);
  check_numel(obs_buf, "obs_buf", (T + 1) * N * D);
  check_dev(logp_buf, "logp_buf", at::kFloat);
  check_numel(logp_buf, "logp_buf", T * N);
  check_dev(rew_buf, "rew_buf", at::kFloat);
  check_numel(rew_buf, "rew_buf", T * N);
  check_dev(done_buf, "done_buf", at::kFloat);
  check_numel(done_buf, "done_buf", T * N);
  check_dev(ep_stats, "ep_stats", at::kFloat);
  check_numel(ep_stats, "ep_stats", rollout_grid(N) * 8);
  float* tob = fptr_mut(tobs_buf, "tobs_buf", T * N * D);
  const int rc = rrl_rollout((int)env, params.data_ptr<float>(), (int)N, (int)T, (int)H, state.data_ptr<float>(),
                             ep_len.data_ptr<int>(), ep_ret.data_ptr<float>(), obs_buf.data_ptr<float>(),
                             act_buf.data_ptr<int>(), logp_buf.data_ptr<float>(), rew_buf.data_ptr<float>(),
                             done_buf.data_ptr<float>(), tob, ep_stats.data_ptr<float>(), (uint64_t)seed, (uint64_t)step0,
                             reset_all ? 1 : 0, (int)max_steps, num_cus(), cur_stream());
  check_rc(rc, "rollout");
}

// Continuous-action fused rollout (diagonal Gaussian policy; env id 4 = HalfCheetahSynth).
void rollout_cont(int64_t env, const Tensor& params, const Tensor& env_consts, int64_t H, const Tensor& state,
                  const Tensor& ep_len, const Tensor& ep_ret, const Tensor& obs_buf, const Tensor& act_buf,
                  const Tensor& logp_buf, const Tensor& rew_buf, const Tensor& done_buf, const OptT& tobs_buf,
                  const Tensor& ep_stats, int64_t seed, int64_t step0, bool reset_all, int64_t max_steps) {
  auto [D, A, NS, ms] = env_dims(env);
  (void)ms;
  TORCH_CHECK(env == 4, "rollout_cont supports the continuous device env 4 (HalfCheetahSynth)");
  TORCH_CHECK(H == 64 || H == 128, "hidden size must be 64 or 128");
  check_dev(params, "params", at::kFloat);
  check_numel(params, "params", flat_size(D, H, A, true));
  check_dev(env_consts, "env_consts", at::kFloat);
  check_numel(env_consts, "env_consts", 17 * 17 + 17 * 6);
  check_dev(act_buf, "act_buf", at::kFloat);
  TORCH_CHECK(act_buf.dim() == 3 && act_buf.size(2) == A, "act_buf must be [T, N, A]");
  const int64_t T = act_buf.size(0), N = act_buf.size(1);
  check_dev(state, "state", at::kFloat);
  check_numel(state, "state", N * NS);
  check_dev(ep_len, "ep_len", at::kInt);
  check_numel(ep_len, "ep_len", N);
  check_dev(ep_ret, "ep_ret", at::kFloat);
  check_numel(ep_ret, "ep_ret", N);
  check_dev(obs_buf, "obs_buf", at::kFloat);
  check_numel(obs_buf, "obs_buf", (T + 1) * N * D);
  check_dev(logp_buf, "logp_buf", at::kFloat);
  check_numel(logp_buf, "logp_buf", T * N);
  check_dev(rew_buf, "rew_buf", at::kFloat);
  check_numel(rew_buf, "rew_buf", T * N);
  check_dev(done_buf, "done_buf", at::kFloat);
  check_numel(done_buf, "done_buf", T * N);
  check_dev(ep_stats, "ep_stats", at::kFloat);
  check_numel(ep_stats, "ep_stats", rollout_grid(N) * 8);
  float* tob = fptr_mut(tobs_buf, "tobs_buf", T * N * D);
  check_rc(rrl_rollout_cont((int)env, params.data_ptr<float>(), env_consts.data_ptr<float>(), (int)N, (int)T, (int)H,
                            state.data_ptr<float>(), ep_len.data_ptr<int>(), ep_ret.data_ptr<float>(),
                            obs_buf.data_ptr<float>(), act_buf.data_ptr<float>(), logp_buf.data_ptr<float>(),
                            rew_buf.data_ptr<float>(), done_buf.data_ptr<float>(), tob, ep_stats.data_ptr<float>(),
                            (uint64_t)seed, (uint64_t)step0, reset_all ? 1 : 0, (int)max_steps, num_cus(),
                            cur_stream()),
           "rollout_cont");
}

}  // namespace

void register_cnn_ops(pybind11::module_& m);      // cnn_ops.cpp
void register_rollout_ops(pybind11::module_& m);  // rollout_ops.cpp (host-env rollout driver)

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "relayrl_prototype_amd gfx950 HIP kernels";
  m.def("num_cus", &num_cus);
  m.def("device_cus", &device_cus);
  m.def("relax_thread_capture_mode", []() {
    // hipThreadExchangeStreamCaptureMode(relaxed) for the calling thread, for good: a helper
    // thread's event waits then leave other threads' graph captures alone
    hipStreamCaptureMode m = hipStreamCaptureModeRelaxed;
    return (int)hipThreadExchangeStreamCaptureMode(&m);
  });
  m.def("set_cu_limit", &set_cu_limit, "size grids for n CUs (0 = all); returns the previous limit");
  m.def("cu_masked_stream", &cu_masked_stream);
  m.def("destroy_stream", &destroy_stream);
  m.def("mlp_forward", &mlp_forward);
  m.def("mlp_grad_slabs", &mlp_grad_slabs);
  m.def("mlp_grad", &mlp_grad);
  m.def("set_value_grad_stamps", [](const Tensor& t) { rrl_set_value_grad_stamps(t.numel() ? t.data_ptr() : nullptr); });
  m.def("set_value_grad_tune", [](int64_t t) { return (int64_t)rrl_set_value_grad_tune((int)t); });
  m.def("set_value_grad_mode", [](int64_t mode) { return (int64_t)rrl_set_value_grad_mode((int)mode); },
        "value-MSE gradient kernel: 1 = bf16x6 weight-stationary (H 128, D <= 8), 0 = fp32 MFMA; returns the "
        "previous mode (-1 queries without changing)");
  m.def("set_value_fwd_mode", [](int64_t mode) { return (int64_t)rrl_set_value_fwd_mode((int)mode); },
        "value forward: 1 = bf16x6 weight-stationary split kernel (H 128, D <= 24), 0 = fp32 MFMA; returns "
        "the previous mode (-1 queries)");
  m.def("scan_tm_parts", &scan_tm_parts);
  m.def("gae_scan_tm", &gae_scan_tm, pybind11::arg("rew"), pybind11::arg("done"), pybind11::arg("val"),
        pybind11::arg("tval"), pybind11::arg("adv"), pybind11::arg("ret"), pybind11::arg("stats_part"),
        pybind11::arg("stats_out"), pybind11::arg("gamma"), pybind11::arg("lam"),
        pybind11::arg("counters") = std::vector<std::tuple<Tensor, int64_t>>{});
  m.def("scan_flat_blocks", &scan_flat_blocks);
  m.def("scan_flat", &scan_flat);
  m.def("stats_reduce", &stats_reduce);
  m.def("column_sums", &column_sums, "double column sums of the first cols columns of a [rows, ld] fp32 tensor");
  // step_add / step_inc: t = step + step_add + 1, the counter advances by step_inc (adam.hip)
  m.def("adam", &adam, pybind11::arg("param"), pybind11::arg("m"), pybind11::arg("v"), pybind11::arg("grad"),
        pybind11::arg("slab"), pybind11::arg("grad_out"), pybind11::arg("step"), pybind11::arg("ticket"),
        pybind11::arg("lr"), pybind11::arg("beta1"), pybind11::arg("beta2"), pybind11::arg("eps"),
        pybind11::arg("grad_scale"), pybind11::arg("weight_decay"), pybind11::arg("step_add") = 0,
        pybind11::arg("step_inc") = 1);
  m.def("reduce_slabs", &reduce_slabs);
  m.def("env_dims", &env_dims);
  m.def("rollout_grid", &rollout_grid);
  m.def("rollout", &rollout);
  m.def("rollout_cont", &rollout_cont);
  register_cnn_ops(m);
  register_rollout_ops(m);
}
