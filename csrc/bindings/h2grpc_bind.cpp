// pybind11 module ``_h2grpc``: the native gRPC server (csrc/net/h2grpc.cpp).  A module of its own
// because it links nghttp2; transport/grpc_transport.py falls back to the grpc.aio server
// (and says so) when it cannot be loaded.
#include <pybind11/pybind11.h>

#include "h2grpc.h"

namespace py = pybind11;
using rrl::h2::Item;
using rrl::h2::Server;

PYBIND11_MODULE(_h2grpc, m) {
  m.attr("FRAME") = (int)rrl::h2::kFrame;
  m.attr("ACTIONS") = (int)rrl::h2::kActions;
  m.attr("NEED_TS") = (int)rrl::h2::kNeedTs;
  py::class_<Server>(m, "GrpcServer")
      .def(py::init<const std::string&, int, size_t, size_t, int, size_t>(), py::arg("host"), py::arg("port"),
           py::arg("max_inbox") = 65536, py::arg("max_bytes") = size_t(1) << 30, py::arg("idle_timeout_ms") = 30,
           py::arg("max_request") = size_t(256) << 20)
      .def_property_readonly("port", &Server::port)
      .def(
          "recv",
          [](Server& s, int timeout_ms) -> py::object {
            Item it;
            bool ok;
            {
              py::gil_scoped_release nogil;
              ok = s.recv(it, timeout_ms);
            }
            if (!ok) return py::none();
            return py::make_tuple(it.kind, py::bytes(it.body), it.aux);
          },
          py::arg("timeout_ms") = -1)
      .def(
          "set_model",
          [](Server& s, int64_t version, py::bytes rrlm, py::object ts) {
            std::string r = rrlm, t = ts.is_none() ? std::string() : std::string(ts.cast<py::bytes>());
            py::gil_scoped_release nogil;
            s.set_model(version, std::move(r), std::move(t));
          },
          py::arg("version"), py::arg("rrlm"), py::arg("ts") = py::none())
      .def(
          "set_model_ts",
          [](Server& s, int64_t version, py::bytes ts) {
            std::string t = ts;
            py::gil_scoped_release nogil;
            s.set_model_ts(version, std::move(t));
          },
          py::arg("version"), py::arg("ts"))
      .def("close", &Server::close, py::call_guard<py::gil_scoped_release>())
      .def("inbox_size", &Server::inbox_size)
      .def("stats", [](Server& s) {
        const rrl::h2::Stats st = s.stats();
        py::dict d;
        d["accepted"] = st.accepted;
        d["requests"] = st.requests;
        d["frames"] = st.frames;
        d["actions"] = st.actions;
        d["polls"] = st.polls;
        d["polls_parked"] = st.polls_parked;
        d["polls_timeout"] = st.polls_timeout;
        d["bad_requests"] = st.bad_requests;
        d["bytes_in"] = st.bytes_in;
        d["inbox_waits"] = st.inbox_waits;
        d["dropped_conns"] = st.dropped_conns;
        d["refused_streams"] = st.refused_streams;
        return d;
      });
}
