// See host_rollout.h.
#include "host_rollout.h"

#include <chrono>
#include <stdexcept>
#include <string>

extern "C" int rrl_mlp_forward(int mode, const float* params, const float* X, int B, int D, int A, int H,
                               const float* mask, const int* act_in, const float* actc_in, int* act_out,
                               float* actc_out, float* out0, float* out1, float* logits_out, uint64_t seed,
                               uint64_t step, uint32_t row_offset, const float* gate, float* x_copy, int* act_host,
                               float* actc_host, int num_cu, void* stream);

namespace rrl {

namespace {

constexpr int kModeCatSample = 1;
constexpr int kModeGaussSample = 4;

using Clock = std::chrono::steady_clock;
double us_since(Clock::time_point t0) {
  return std::chrono::duration<double, std::micro>(Clock::now() - t0).count();
}

// The device address of a pinned host buffer (hipHostMalloc'd: torch's pinned allocator).
template <class T>
T* device_view(T* host, const char* what) {
  if (host == nullptr) return nullptr;
  void* d = nullptr;
  const hipError_t e = hipHostGetDevicePointer(&d, (void*)host, 0);
  if (e != hipSuccess || d == nullptr)
    throw std::runtime_error(std::string("host rollout: ") + what +
                             " is not pinned host memory visible to the GPU (" + hipGetErrorString(e) + ")");
  return static_cast<T*>(d);
}

// Poll a timing-free event: the driver thread owns a core while the GPU samples.  With
// ``backoff`` each query is followed by ~1 us of pause instructions, so the poll does not
// keep the HIP runtime busy while another thread (the overlapped learner) launches kernels.
hipError_t spin(hipEvent_t ev, bool backoff) {
  for (;;) {
    const hipError_t e = hipEventQuery(ev);
    if (e != hipErrorNotReady) return e;
#if defined(__x86_64__)
    for (int i = 0, n = backoff ? 64 : 1; i < n; ++i) __builtin_ia32_pause();
#endif
  }
}

// Scoped hipThreadExchangeStreamCaptureMode(relaxed) for the calling thread.
struct RelaxedCapture {
  hipStreamCaptureMode prev = hipStreamCaptureModeRelaxed;
  RelaxedCapture() { (void)hipThreadExchangeStreamCaptureMode(&prev); }
  ~RelaxedCapture() { (void)hipThreadExchangeStreamCaptureMode(&prev); }
};

}  // namespace

HostRollout::HostRollout(std::vector<VecEnv*> envs, std::vector<int> bounds, int num_cu)
    : envs_(std::move(envs)), bounds_(std::move(bounds)), num_cu_(num_cu) {
  if (envs_.empty() || bounds_.size() != envs_.size() + 1 || bounds_[0] != 0)
    throw std::invalid_argument("host rollout: need bounds [0, ..., N] with one entry per env half");
  D_ = envs_[0]->obs_dim();
  A_ = envs_[0]->act_dim();
  cont_ = envs_[0]->continuous();
  for (size_t h = 0; h < envs_.size(); ++h) {
    VecEnv* e = envs_[h];
    if (e->obs_dim() != D_ || e->act_dim() != A_ || e->continuous() != cont_ ||
        e->num_envs() != bounds_[h + 1] - bounds_[h])
      throw std::invalid_argument("host rollout: env halves disagree with each other or with the bounds");
  }
  ev_.resize(envs_.size());
  for (auto& ev : ev_) {
    const hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    if (e != hipSuccess) throw std::runtime_error(std::string("hipEventCreate: ") + hipGetErrorString(e));
  }
}

HostRollout::~HostRollout() {
  for (auto* e : envs_) e->wait();
  for (auto& ev : ev_) (void)hipEventDestroy(ev);
}

int HostRollout::run(const float* params, int H, int T, const RolloutBuffers& b, uint64_t seed, uint64_t step0,
                     hipStream_t s) {
  const auto t_run = Clock::now();
  // This thread's event polls must not touch another thread's graph capture: the overlapped
  // learner captures its value loop while a rollout runs, and HIP invalidates every active
  // capture when a thread in the default (global) mode calls a synchronising API.
  RelaxedCapture relaxed;
  const int N = bounds_.back(), D = D_, A = A_;
  const int halves = (int)envs_.size();
  const size_t act_w = cont_ ? (size_t)A : 1;  // action elements per env
  float* obs_dev = device_view(b.h_obs, "h_obs");
  void* act_dev = device_view(b.h_act, "h_act");
  int rc = 0;
  int t_done = 0;  // steps whose env halves were submitted
  for (int t = 0; t < T && rc == 0; ++t) {
    const size_t row_t = (size_t)t * N;
    for (int h = 0; h < halves; ++h) {
      const int lo = bounds_[h], nh = bounds_[h + 1] - lo;
      if (t > 0) {
        const auto t0 = Clock::now();
        envs_[h]->wait();  // obs_t of this half (its step t-1 ran on the pool)
        st_.env_wait_us += us_since(t0);
      }
      const auto t1 = Clock::now();
      const size_t r = row_t + lo;
      rc = rrl_mlp_forward(cont_ ? kModeGaussSample : kModeCatSample, params, obs_dev + r * D, nh, D, A, H, nullptr,
                           nullptr, nullptr, cont_ ? nullptr : (int*)b.d_act + r,
                           cont_ ? (float*)b.d_act + r * A : nullptr, b.d_logp + r, nullptr, nullptr, seed,
                           step0 + (uint64_t)t, (uint32_t)lo, nullptr, b.d_obs + r * D,
                           cont_ ? nullptr : (int*)act_dev + r, cont_ ? (float*)act_dev + r * A : nullptr, num_cu_,
                           (void*)s);
      if (rc == 0) rc = (int)hipEventRecord(ev_[h], s);
      st_.launch_us += us_since(t1);
      st_.launches += 1;
      if (rc != 0) break;
    }
    if (rc != 0) break;
    for (int h = 0; h < halves; ++h) {
      const int lo = bounds_[h];
      const auto t0 = Clock::now();
      // this half's actions are in pinned host memory once its event completes
      rc = wait_mode_ == 1 ? (int)hipEventSynchronize(ev_[h]) : (int)spin(ev_[h], wait_mode_ == 2);
      st_.gpu_wait_us += us_since(t0);
      if (rc != 0) break;
      const size_t r = (size_t)t * N + lo;
      envs_[h]->step_async((const char*)b.h_act + r * act_w * 4, b.h_obs + (r + N) * D, b.h_rew + r, b.h_done + r,
                           b.h_tobs ? b.h_tobs + r * D : nullptr);
    }
    t_done = t + 1;
  }
  const auto t2 = Clock::now();
  for (auto* e : envs_) e->wait();
  if (rc == 0 && t_done == T) {
    // last observation + rewards / done codes (+ truncation observations) to HBM, async
    const size_t nT = (size_t)T * N;
    rc = (int)hipMemcpyAsync(b.d_obs + nT * D, b.h_obs + nT * D, (size_t)N * D * 4, hipMemcpyHostToDevice, s);
    if (rc == 0) rc = (int)hipMemcpyAsync(b.d_rew, b.h_rew, nT * 4, hipMemcpyHostToDevice, s);
    if (rc == 0) rc = (int)hipMemcpyAsync(b.d_done, b.h_done, nT * 4, hipMemcpyHostToDevice, s);
    if (rc == 0 && b.h_tobs != nullptr && b.d_tobs != nullptr)
      rc = (int)hipMemcpyAsync(b.d_tobs, b.h_tobs, nT * D * 4, hipMemcpyHostToDevice, s);
  }
  st_.tail_us += us_since(t2);
  st_.steps += T;
  st_.total_us += us_since(t_run);
  return rc;
}

RolloutStats HostRollout::take_stats() {
  RolloutStats s = st_;
  st_ = RolloutStats();
  return s;
}

}  // namespace rrl
