// pybind11 bindings of the C++ host runtime (csrc/host): codec, ZMTP transport, VecEnv,
// NativePolicy (agent-side CPU inference).
// Replaces the reference's PyO3 layer for the host-side types (rf/src/bindings/python/*).
#include <cstring>
#include <limits>

#include <pybind11/pybind11.h>
#include <pybind11/numpy.h>
#include <pybind11/stl.h>

#include "codec.h"
#include "policy.h"
#include "vecenv.h"
#include "vecenv_bind.h"
#include "zmtp.h"

void bind_pickle(pybind11::module_& m);  // pickle_native.cpp

namespace py = pybind11;
using namespace rrl;

namespace {
struct RowSink {  // see the RowSink binding
  py::array obs, act, mask, logp, val, rew, done;
  py::ssize_t cap = 0;
  int D = 0, AC = 0, M = 0;
  bool act_int = true;
};
}  // namespace

namespace {

py::tuple tensor_to_py(const Tensor& t) {
  return py::make_tuple(std::string(dtype_name(t.dtype)), t.shape, py::bytes(t.raw));
}

Tensor tensor_from_py(const py::handle& h) {
  auto tup = h.cast<py::tuple>();
  if (tup.size() != 3) throw std::invalid_argument("tensor must be (dtype, shape, raw)");
  Tensor t;
  t.dtype = dtype_from_name(tup[0].cast<std::string>());
  t.shape = tup[1].cast<std::vector<int64_t>>();
  t.raw = tup[2].cast<std::string>();
  if ((int64_t)t.raw.size() != t.numel() * (int64_t)dtype_size(t.dtype))
    throw std::invalid_argument("tensor raw size does not match dtype/shape");
  return t;
}

const char* kAuxNames[] = {"Tensor", "Byte", "Short", "Int", "Long", "Float", "Double", "String", "Bool"};

py::object aux_to_py(const AuxValue& v) {
  py::object val;
  switch (v.kind) {
    case AuxValue::TENSOR: val = tensor_to_py(v.tensor); break;
    case AuxValue::BYTE: case AuxValue::SHORT: case AuxValue::INT: case AuxValue::LONG: val = py::int_(v.i); break;
    case AuxValue::FLOAT: case AuxValue::DOUBLE: val = py::float_(v.d); break;
    case AuxValue::STRING: val = py::str(v.s); break;
    case AuxValue::BOOL: val = py::bool_(v.b); break;
  }
  return py::make_tuple(std::string(kAuxNames[(int)v.kind]), val);
}

AuxValue aux_from_py(const py::handle& h) {
  auto tup = h.cast<py::tuple>();
  std::string kind = tup[0].cast<std::string>();
  AuxValue v;
  int k = -1;
  for (int i = 0; i < 9; ++i)
    if (kind == kAuxNames[i]) k = i;
  if (k < 0) throw std::invalid_argument("unknown RelayRLData kind: " + kind);
  v.kind = (AuxValue::Kind)k;
  switch (v.kind) {
    case AuxValue::TENSOR: v.tensor = tensor_from_py(tup[1]); break;
    case AuxValue::BYTE: case AuxValue::SHORT: case AuxValue::INT: case AuxValue::LONG: v.i = tup[1].cast<int64_t>(); break;
    case AuxValue::FLOAT: case AuxValue::DOUBLE: v.d = tup[1].cast<double>(); break;
    case AuxValue::STRING: v.s = tup[1].cast<std::string>(); break;
    case AuxValue::BOOL: v.b = tup[1].cast<bool>(); break;
  }
  return v;
}

py::dict traj_to_py(const Trajectory& t) {
  py::dict d;
  d["server"] = t.server;
  d["max_length"] = t.max_length;
  d["agent_id"] = t.agent_id;
  d["seq"] = t.seq;
  py::list acts;
  for (const Action& a : t.actions) {
    py::dict x;
    x["obs"] = a.has_obs ? py::object(tensor_to_py(a.obs)) : py::none();
    x["act"] = a.has_act ? py::object(tensor_to_py(a.act)) : py::none();
    x["mask"] = a.has_mask ? py::object(tensor_to_py(a.mask)) : py::none();
    x["rew"] = a.rew;
    if (a.has_data) {
      py::dict dd;
      for (const auto& kv : a.data) dd[py::str(kv.first)] = aux_to_py(kv.second);
      x["data"] = dd;
    } else {
      x["data"] = py::none();
    }
    x["done"] = a.done;
    x["reward_updated"] = a.reward_updated;
    acts.append(x);
  }
  d["actions"] = acts;
  return d;
}

Trajectory traj_from_py(const py::dict& d) {
  Trajectory t;
  if (d.contains("server") && !d["server"].is_none()) t.server = d["server"].cast<std::string>();
  if (d.contains("max_length")) t.max_length = d["max_length"].cast<uint32_t>();
  if (d.contains("agent_id") && !d["agent_id"].is_none()) t.agent_id = d["agent_id"].cast<std::string>();
  if (d.contains("seq")) t.seq = d["seq"].cast<uint64_t>();
  for (auto h : d["actions"].cast<py::list>()) {
    py::dict x = h.cast<py::dict>();
    Action a;
    auto opt = [&](const char* k, bool& has, Tensor& dst) {
      if (x.contains(k) && !x[k].is_none()) {
        has = true;
        dst = tensor_from_py(x[k]);
      }
    };
    opt("obs", a.has_obs, a.obs);
    opt("act", a.has_act, a.act);
    opt("mask", a.has_mask, a.mask);
    a.rew = x.contains("rew") ? x["rew"].cast<float>() : 0.f;
    if (x.contains("data") && !x["data"].is_none()) {
      a.has_data = true;
      for (auto kv : x["data"].cast<py::dict>()) a.data.emplace(kv.first.cast<std::string>(), aux_from_py(kv.second));
    }
    a.done = x.contains("done") && x["done"].cast<bool>();
    a.reward_updated = x.contains("reward_updated") && x["reward_updated"].cast<bool>();
    t.actions.push_back(std::move(a));
  }
  return t;
}

}  // namespace

PYBIND11_MODULE(_native, m) {
  m.doc() = "relayrl_prototype_amd host runtime: codec, ZMTP transport, vectorised CPU envs";

  m.def("st_encode", [](const std::string& dtype, std::vector<int64_t> shape, py::bytes raw) {
    Tensor t;
    t.dtype = dtype_from_name(dtype);
    t.shape = std::move(shape);
    t.raw = raw;
    return py::bytes(st_encode(t));
  });
  m.def("st_decode", [](py::bytes data) { return tensor_to_py(st_decode(std::string(data))); });
  m.def("traj_encode", [](const py::dict& d) { return py::bytes(traj_encode(traj_from_py(d))); });
  m.def("traj_decode", [](py::bytes b) {
    std::string s = b;
    Trajectory t;
    {
      py::gil_scoped_release nogil;
      t = traj_decode(s);
    }
    return traj_to_py(t);
  });

  py::enum_<zmtp::SockType>(m, "SockType")
      .value("PUSH", zmtp::SockType::PUSH)
      .value("PULL", zmtp::SockType::PULL)
      .value("DEALER", zmtp::SockType::DEALER)
      .value("ROUTER", zmtp::SockType::ROUTER);

  py::class_<zmtp::Socket>(m, "ZmtpSocket")
      .def(py::init([](zmtp::SockType t, py::bytes identity) { return new zmtp::Socket(t, std::string(identity)); }),
           py::arg("type"), py::arg("identity") = py::bytes(""))
      .def("bind", &zmtp::Socket::bind, py::call_guard<py::gil_scoped_release>())
      .def("connect", &zmtp::Socket::connect, py::call_guard<py::gil_scoped_release>())
      .def(
          "send",
          [](zmtp::Socket& s, const std::vector<py::bytes>& frames, int timeout_ms) {
            std::vector<std::string> f;
            f.reserve(frames.size());
            for (auto& b : frames) f.emplace_back(b);
            py::gil_scoped_release nogil;
            return s.send(f, timeout_ms);
          },
          py::arg("frames"), py::arg("timeout_ms") = -1)
      .def(
          "recv",
          [](zmtp::Socket& s, int timeout_ms) -> py::object {
            zmtp::Message msg;
            bool ok;
            {
              py::gil_scoped_release nogil;
              ok = s.recv(msg, timeout_ms);
            }
            if (!ok) return py::none();
            py::list fr;
            for (auto& f : msg.frames) fr.append(py::bytes(f));
            return py::make_tuple(py::bytes(msg.peer), fr);
          },
          py::arg("timeout_ms") = -1)
      .def("close", &zmtp::Socket::close, py::call_guard<py::gil_scoped_release>())
      .def("closed", &zmtp::Socket::closed)
      .def("peers", [](zmtp::Socket& s) {
        py::list l;
        for (auto& p : s.peers()) l.append(py::bytes(p));
        return l;
      })
      .def("num_connections", &zmtp::Socket::num_connections)
      .def("num_threads", &zmtp::Socket::num_threads)
      .def("set_inbox_limits", &zmtp::Socket::set_inbox_limits, py::arg("max_messages"), py::arg("max_bytes"))
      .def("set_max_message_size", &zmtp::Socket::set_max_message_size, py::arg("max_bytes"))
      .def("max_message_size", &zmtp::Socket::max_message_size)
      .def("inbox_size", &zmtp::Socket::inbox_size)
      .def("inbox_bytes", &zmtp::Socket::inbox_bytes)
      .def("stats", [](zmtp::Socket& s) {
        const zmtp::Stats st = s.stats();
        py::dict d;
        d["accepted"] = st.accepted;
        d["handshakes"] = st.handshakes;
        d["dropped"] = st.dropped;
        d["bad_handshakes"] = st.bad_handshakes;
        d["messages_in"] = st.messages_in;
        d["bytes_in"] = st.bytes_in;
        d["inbox_waits"] = st.inbox_waits;
        d["oversized"] = st.oversized;
        return d;
      });

  bind_pickle(m);
  m.def("env_names", &env_names);
  m.def("env_constants", &env_constants);
  bind_vecenv(m);

  using farr = py::array_t<float, py::array::c_style | py::array::forcecast>;
  // An agent's episode columns (types.EpisodeRecorder), validated once: step_row writes one
  // request_for_action's row into them from C++ (one call per env step instead of ~8 numpy
  // element writes, each ~0.5 us on a busy host).
  py::class_<RowSink>(m, "RowSink")
      .def(py::init([](py::array obs, py::array act, py::array mask, py::array logp, py::array val, py::array rew,
                       py::array done) {
        auto f32 = [](const py::array& a, const char* what) {
          if (!a.dtype().is(py::dtype::of<float>()) || !(a.flags() & py::array::c_style) || !a.writeable())
            throw std::invalid_argument(std::string("RowSink: ") + what + " must be writable C-contiguous float32");
        };
        f32(obs, "obs");
        f32(mask, "mask");
        f32(logp, "logp");
        f32(val, "val");
        f32(rew, "rew");
        if (obs.ndim() != 2 || mask.ndim() != 2 || act.ndim() != 2) throw std::invalid_argument("RowSink: obs / act / mask are [C][.]");
        const bool ai = act.dtype().is(py::dtype::of<int32_t>());
        if (!ai) f32(act, "act");
        if (!(act.flags() & py::array::c_style) || !act.writeable()) throw std::invalid_argument("RowSink: act");
        if (!done.dtype().is(py::dtype::of<uint8_t>()) || !(done.flags() & py::array::c_style) || !done.writeable())
          throw std::invalid_argument("RowSink: done must be writable C-contiguous uint8");
        RowSink k;
        k.cap = obs.shape(0);
        for (const py::array* a : {&act, &mask, &logp, &val, &rew, &done})
          if (a->shape(0) != k.cap) throw std::invalid_argument("RowSink: column lengths differ");
        k.D = static_cast<int>(obs.shape(1));
        k.AC = static_cast<int>(act.shape(1));
        k.M = static_cast<int>(mask.shape(1));
        k.act_int = ai;
        k.obs = obs; k.act = act; k.mask = mask; k.logp = logp; k.val = val; k.rew = rew; k.done = done;
        return k;
      }))
      .def_readonly("capacity", &RowSink::cap);
  py::class_<rrl::NativePolicy>(m, "NativePolicy")
      .def(py::init<int, int, int, bool, uint64_t>(), py::arg("obs_dim"), py::arg("hidden"), py::arg("act_dim"),
           py::arg("discrete"), py::arg("seed") = 0)
      .def("load", [](rrl::NativePolicy& p, farr pi, py::object vf) {
        if (vf.is_none()) {
          p.load(pi.data(), pi.size(), nullptr, 0);
        } else {
          farr v = vf.cast<farr>();
          p.load(pi.data(), pi.size(), v.data(), v.size());
        }
      }, py::arg("pi"), py::arg("vf") = py::none())
      .def_property_readonly("has_value", &rrl::NativePolicy::has_value)
      // -> (act [N] int32 | [N, A] float32, logp [N], v [N] | None)
      .def("step", [](rrl::NativePolicy& p, farr obs, py::object mask) -> py::tuple {
        if (obs.size() % p.D != 0) throw std::invalid_argument("obs size is not a multiple of obs_dim");
        const int N = static_cast<int>(obs.size() / p.D);
        farr m;
        const float* mp = nullptr;
        if (!mask.is_none()) {
          m = mask.cast<farr>();
          if (m.size() != static_cast<py::ssize_t>(N) * p.A) throw std::invalid_argument("mask size != N*act_dim");
          mp = m.data();
        }
        py::array_t<float> logp(N);
        py::object v = py::none();
        float* vp = nullptr;
        if (p.has_value()) {
          py::array_t<float> va(N);
          vp = va.mutable_data();
          v = va;
        }
        if (p.discrete) {
          py::array_t<int32_t> act(N);
          p.step(obs.data(), mp, N, act.mutable_data(), nullptr, logp.mutable_data(), vp);
          return py::make_tuple(act, logp, v);
        }
        py::array_t<float> act({N, p.A});
        p.step(obs.data(), mp, N, nullptr, act.mutable_data(), logp.mutable_data(), vp);
        return py::make_tuple(act, logp, v);
      }, py::arg("obs"), py::arg("mask") = py::none())
      // one observation -> row i of the sink (obs, act, mask, logp, V or NaN, rew = done = 0);
      // -> (a0: 0-d int32 | [A] float32, logp: 0-d float32, v: 0-d float32 | None), the values
      // request_for_action hands back in its RelayRLAction
      .def("step_row", [](rrl::NativePolicy& p, farr obs, farr mask, RowSink& k, py::ssize_t i) -> py::tuple {
        if (obs.size() != p.D || k.D != p.D) throw std::invalid_argument("step_row: obs size != obs_dim");
        if (mask.size() != p.A || k.M != p.A) throw std::invalid_argument("step_row: mask size != act_dim");
        if (i < 0 || i >= k.cap) throw std::out_of_range("step_row: row index outside the episode columns");
        if (p.discrete ? !(k.act_int && k.AC == 1) : (k.act_int || k.AC != p.A))
          throw std::invalid_argument("step_row: action column does not match the policy");
        py::array_t<float> logp(py::array::ShapeContainer{});
        float v = std::numeric_limits<float>::quiet_NaN();
        float* po = static_cast<float*>(k.obs.mutable_data()) + i * k.D;
        std::memcpy(po, obs.data(), sizeof(float) * p.D);
        std::memcpy(static_cast<float*>(k.mask.mutable_data()) + i * k.M, mask.data(), sizeof(float) * p.A);
        py::object a0;
        if (p.discrete) {
          int32_t a = 0;
          p.step(obs.data(), mask.data(), 1, &a, nullptr, logp.mutable_data(), p.has_value() ? &v : nullptr);
          static_cast<int32_t*>(k.act.mutable_data())[i] = a;
          py::array_t<int32_t> aa(py::array::ShapeContainer{});
          *aa.mutable_data() = a;
          a0 = aa;
        } else {
          py::array_t<float> aa(p.A);
          p.step(obs.data(), mask.data(), 1, nullptr, aa.mutable_data(), logp.mutable_data(), p.has_value() ? &v : nullptr);
          std::memcpy(static_cast<float*>(k.act.mutable_data()) + i * k.AC, aa.data(), sizeof(float) * p.A);
          a0 = aa;
        }
        static_cast<float*>(k.logp.mutable_data())[i] = *logp.data();
        static_cast<float*>(k.val.mutable_data())[i] = v;
        static_cast<float*>(k.rew.mutable_data())[i] = 0.f;
        static_cast<uint8_t*>(k.done.mutable_data())[i] = 0;
        py::object vo = py::none();
        if (p.has_value()) {
          py::array_t<float> va(py::array::ShapeContainer{});
          *va.mutable_data() = v;
          vo = va;
        }
        return py::make_tuple(a0, logp, vo);
      }, py::arg("obs"), py::arg("mask"), py::arg("sink"), py::arg("row"))
      .def("logits", [](const rrl::NativePolicy& p, farr obs) {
        const int N = static_cast<int>(obs.size() / p.D);
        py::array_t<float> out({N, p.A});
        p.logits(obs.data(), N, out.mutable_data());
        return out;
      })
      .def("value", [](const rrl::NativePolicy& p, farr obs) {
        const int N = static_cast<int>(obs.size() / p.D);
        py::array_t<float> out(N);
        p.value(obs.data(), N, out.mutable_data());
        return out;
      });
}
