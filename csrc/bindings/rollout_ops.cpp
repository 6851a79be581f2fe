// Bindings of the host-env rollout driver (csrc/runtime/host_rollout.h) and of the env
// pools it steps.  The VecEnv class here is this module's own (module_local): the driver
// calls it from C++, so it must be the same type, not _native's.
#include <ATen/hip/HIPContext.h>
#include <torch/extension.h>

#include "host_rollout.h"
#include "vecenv_bind.h"

namespace {

using at::Tensor;
namespace py = pybind11;

void check(const Tensor& t, const char* name, bool cuda, at::ScalarType dt, int64_t numel) {
  TORCH_CHECK(t.defined(), name, " is required");
  TORCH_CHECK(cuda ? t.is_cuda() : (!t.is_cuda() && t.is_pinned()), name,
              cuda ? " must be a GPU tensor" : " must be a pinned host tensor");
  TORCH_CHECK(t.scalar_type() == dt, name, " has dtype ", t.scalar_type(), ", expected ", dt);
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
  TORCH_CHECK(t.numel() == numel, name, " has ", t.numel(), " elements, expected ", numel);
}

class PyHostRollout {
 public:
  PyHostRollout(py::list envs, std::vector<int> bounds, int num_cu) {
    std::vector<rrl::VecEnv*> e;
    for (auto h : envs) {
      e.push_back(h.cast<rrl::VecEnv*>());
      keep_.push_back(py::reinterpret_borrow<py::object>(h));  // the envs outlive the driver
    }
    if (num_cu <= 0) num_cu = at::cuda::getCurrentDeviceProperties()->multiProcessorCount;
    drv_ = std::make_unique<rrl::HostRollout>(std::move(e), std::move(bounds), num_cu);
  }

  void run(const Tensor& params, int64_t H, const Tensor& h_obs, const Tensor& h_act, const Tensor& h_rew,
           const Tensor& h_done, const std::optional<Tensor>& h_tobs, const Tensor& d_obs, const Tensor& d_act,
           const Tensor& d_logp, const Tensor& d_rew, const Tensor& d_done, const std::optional<Tensor>& d_tobs,
           int64_t seed, int64_t step0) {
    const int64_t N = drv_->num_envs(), D = drv_->obs_dim(), A = drv_->act_dim();
    const bool cont = drv_->continuous();
    TORCH_CHECK(H == 64 || H == 128, "hidden size must be 64 or 128");
    TORCH_CHECK(D <= 32 && A <= 16, "env dims out of the sampling kernel's range");
    TORCH_CHECK(h_rew.dim() == 2 && h_rew.size(1) == N, "h_rew must be [T, N]");
    const int64_t T = h_rew.size(0);
    TORCH_CHECK(T >= 1, "empty rollout");
    TORCH_CHECK((T + 1) * N * std::max(D, A) < (int64_t)INT32_MAX * 4, "rollout too large");
    check(params, "params", true, at::kFloat, H * D + H + H * H + H + A * H + A + (cont ? A : 0));
    check(h_obs, "h_obs", false, at::kFloat, (T + 1) * N * D);
    check(h_act, "h_act", false, cont ? at::kFloat : at::kInt, T * N * (cont ? A : 1));
    check(h_rew, "h_rew", false, at::kFloat, T * N);
    check(h_done, "h_done", false, at::kFloat, T * N);
    check(d_obs, "d_obs", true, at::kFloat, (T + 1) * N * D);
    check(d_act, "d_act", true, cont ? at::kFloat : at::kInt, T * N * (cont ? A : 1));
    check(d_logp, "d_logp", true, at::kFloat, T * N);
    check(d_rew, "d_rew", true, at::kFloat, T * N);
    check(d_done, "d_done", true, at::kFloat, T * N);
    const bool tobs = h_tobs.has_value() && h_tobs->defined();
    TORCH_CHECK(tobs == (d_tobs.has_value() && d_tobs->defined()), "give both or neither of h_tobs / d_tobs");
    if (tobs) {
      check(*h_tobs, "h_tobs", false, at::kFloat, T * N * D);
      check(*d_tobs, "d_tobs", true, at::kFloat, T * N * D);
    }
    rrl::RolloutBuffers b{h_obs.data_ptr<float>(), h_act.data_ptr(), h_rew.data_ptr<float>(),
                          h_done.data_ptr<float>(), tobs ? h_tobs->data_ptr<float>() : nullptr,
                          d_obs.data_ptr<float>(), d_act.data_ptr(), d_logp.data_ptr<float>(),
                          d_rew.data_ptr<float>(), d_done.data_ptr<float>(), tobs ? d_tobs->data_ptr<float>() : nullptr};
    hipStream_t s = at::hip::getCurrentHIPStream().stream();
    int rc;
    {
      py::gil_scoped_release nogil;
      rc = drv_->run(params.data_ptr<float>(), (int)H, (int)T, b, (uint64_t)seed, (uint64_t)step0, s);
    }
    TORCH_CHECK(rc == 0, "host rollout failed with code ", rc,
                rc > 0 ? std::string(" (") + hipGetErrorString((hipError_t)rc) + ")" : std::string(" (bad launch)"));
  }

  void set_wait_mode(int m) { drv_->set_wait_mode(m); }

  py::dict take_stats() {
    const rrl::RolloutStats s = drv_->take_stats();
    py::dict d;
    d["env_wait_us"] = s.env_wait_us;
    d["gpu_wait_us"] = s.gpu_wait_us;
    d["launch_us"] = s.launch_us;
    d["tail_us"] = s.tail_us;
    d["total_us"] = s.total_us;
    d["steps"] = s.steps;
    d["launches"] = s.launches;
    return d;
  }

 private:
  std::vector<py::object> keep_;
  std::unique_ptr<rrl::HostRollout> drv_;
};

}  // namespace

void register_rollout_ops(py::module_& m) {
  rrl::bind_vecenv(m, py::module_local());
  py::class_<PyHostRollout>(m, "HostRollout")
      .def(py::init<py::list, std::vector<int>, int>(), py::arg("envs"), py::arg("bounds"), py::arg("num_cu") = 0)
      .def("run", &PyHostRollout::run, py::arg("params"), py::arg("H"), py::arg("h_obs"), py::arg("h_act"),
           py::arg("h_rew"), py::arg("h_done"), py::arg("h_tobs"), py::arg("d_obs"), py::arg("d_act"),
           py::arg("d_logp"), py::arg("d_rew"), py::arg("d_done"), py::arg("d_tobs"), py::arg("seed"),
           py::arg("step0"))
      .def("take_stats", &PyHostRollout::take_stats)
      .def("set_wait_mode", &PyHostRollout::set_wait_mode);
}
