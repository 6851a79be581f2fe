// pybind11 binding of rrl::VecEnv, shared by the two extensions that own env pools:
// _native (CPU paths, csrc/bindings/native.cpp) and _hip_ops (the GPU host-env rollout
// driver, csrc/bindings/rollout_ops.cpp, which steps these envs from C++).
#pragma once
#include <pybind11/pybind11.h>

#include <cstdint>

#include "vecenv.h"

namespace rrl {

template <class... Extra>
pybind11::class_<VecEnv> bind_vecenv(pybind11::module_& m, const Extra&... extra) {
  namespace py = pybind11;
  py::class_<VecEnv> c(m, "VecEnv", extra...);
  c.def(py::init<const std::string&, int, uint64_t, int>(), py::arg("name"), py::arg("num_envs"), py::arg("seed") = 0,
        py::arg("num_threads") = 1)
      .def_property_readonly("num_envs", &VecEnv::num_envs)
      .def_property_readonly("obs_dim", &VecEnv::obs_dim)
      .def_property_readonly("act_dim", &VecEnv::act_dim)
      .def_property_readonly("continuous", &VecEnv::continuous)
      .def_property_readonly("max_steps", &VecEnv::max_steps)
      // raw-address variants: zero-copy into (pinned) torch / numpy buffers
      .def("reset_ptr",
           [](VecEnv& e, uintptr_t obs) {
             py::gil_scoped_release nogil;
             e.reset((float*)obs);
           })
      .def(
          "step_ptr",
          [](VecEnv& e, uintptr_t act, uintptr_t obs, uintptr_t rew, uintptr_t done, uintptr_t tobs) {
            py::gil_scoped_release nogil;
            e.step((const void*)act, (float*)obs, (float*)rew, (float*)done, (float*)tobs);
          },
          py::arg("act"), py::arg("obs"), py::arg("rew"), py::arg("done"), py::arg("tobs") = 0)
      .def(
          "step_async_ptr",
          [](VecEnv& e, uintptr_t act, uintptr_t obs, uintptr_t rew, uintptr_t done, uintptr_t tobs) {
            py::gil_scoped_release nogil;
            e.step_async((const void*)act, (float*)obs, (float*)rew, (float*)done, (float*)tobs);
          },
          py::arg("act"), py::arg("obs"), py::arg("rew"), py::arg("done"), py::arg("tobs") = 0)
      .def("wait", &VecEnv::wait, py::call_guard<py::gil_scoped_release>())
      .def("take_stats", [](VecEnv& e) {
        EpisodeStats s = e.take_stats();
        py::dict d;
        d["n"] = s.n;
        d["sum"] = s.sum;
        d["sumsq"] = s.sumsq;
        d["max"] = s.n > 0 ? s.max : 0.0;
        d["min"] = s.n > 0 ? s.min : 0.0;
        d["sum_len"] = s.sum_len;
        return d;
      });
  return c;
}

}  // namespace rrl
