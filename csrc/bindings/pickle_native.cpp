// Native data-only pickle codec for the reference ZMQ trajectory frames
// (serde_pickle(Vec<RelayRLAction>), trajectory.rs:50-90 -> training_zmq.rs:994-1012).
//
// transport/serde_pickle.py holds the reference semantics in Python (``loads`` / ``dumps``).
// Its interpreter runs ~25,000 opcodes per CartPole episode (every safetensors byte of every
// tensor is a BININT1 inside a list), ~19 ms per frame: a server fed by many reference agents
// ingests ~50 uploads/s.  This is the same interpreter in C++:
//
//   * ``pickle_loads(buf, u8_lists_as_bytes)``: the SAME opcode subset (containers, scalars,
//     strings, bytes, memo); every opcode that imports or calls (GLOBAL, REDUCE, BUILD, INST,
//     OBJ, NEWOBJ, EXT*, PERSID, ...) is an error, so a frame can never execute anything.
//     With ``u8_lists_as_bytes`` a list built only from integers 0..255 comes back as a
//     ``bytearray`` (serde's Vec<u8>), not as a list of Python ints.
//   * ``pickle_dumps(obj, bytes_as_u8_list)``: the writer serde_pickle uses (protocol 3, no
//     memo; lists in APPENDS chunks of 1000), byte-identical to serde_pickle.dumps; with
//     ``bytes_as_u8_list`` a bytes object is written as a list of u8 ints (Vec<u8>).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "codec.h"
#include "pickle_vm.h"
#include "ref_columns.h"
#include "st_tensor.h"

namespace py = pybind11;

namespace {

using rrl::pickle::FrameError;
using rrl::pickle::kMaxDepth;

py::object key_of(const py::object& k) {
  if (py::isinstance<py::list>(k) || py::isinstance<py::dict>(k) || py::isinstance<py::set>(k) ||
      py::isinstance<py::bytearray>(k))
    throw FrameError("unhashable key");
  return k;
}

// rrl::pickle::run over Python objects (csrc/host/pickle_vm.h: the opcode loop, shared with the
// sanitizer fuzz harness); with the u8 form an EMPTY_LIST starts as a bytearray (serde's Vec<u8>)
struct PyBuilder {
  using V = py::object;
  V none() { return py::none(); }
  V boolean(bool v) { return py::bool_(v); }
  V small_int(int64_t v) { return py::int_(v); }
  V long_bytes(const uint8_t* p, size_t k) {
    PyObject* v = k ? _PyLong_FromByteArray(p, k, /*little_endian=*/1, /*is_signed=*/1) : PyLong_FromLong(0);
    if (!v) throw py::error_already_set();
    return py::reinterpret_steal<py::object>(v);
  }
  V real(double d) { return py::float_(d); }
  V str(const char* s, size_t k) {
    PyObject* v = PyUnicode_DecodeUTF8(s, (Py_ssize_t)k, "strict");
    if (!v) throw py::error_already_set();
    return py::reinterpret_steal<py::object>(v);
  }
  V bytes(const char* s, size_t k) { return py::bytes(s, k); }
  V empty_list(bool u8) {
    if (u8) return py::reinterpret_steal<py::object>(PyByteArray_FromStringAndSize("", 0));
    return py::list();
  }
  V empty_dict() { return py::dict(); }
  V empty_tuple() { return py::tuple(); }
  V empty_set() { return py::set(); }
  bool is_bytearray(const V& o) { return PyByteArray_Check(o.ptr()); }
  void bytearray_append(V& o, const char* s, size_t k) {
    const Py_ssize_t old = PyByteArray_Size(o.ptr());
    if (PyByteArray_Resize(o.ptr(), old + (Py_ssize_t)k) != 0) throw py::error_already_set();
    if (k) std::memcpy(PyByteArray_AsString(o.ptr()) + old, s, k);
  }
  void bytearray_to_list(V& o) {
    py::list l;
    const char* b = PyByteArray_AsString(o.ptr());
    for (Py_ssize_t i = 0; i < PyByteArray_Size(o.ptr()); ++i) l.append(py::int_((unsigned char)b[i]));
    o = l;
  }
  bool u8_value(const V& o, uint8_t& out) {
    if (!PyLong_CheckExact(o.ptr())) return false;
    int overflow = 0;
    const long v = PyLong_AsLongAndOverflow(o.ptr(), &overflow);
    if (overflow || v < 0 || v > 255) return false;
    out = (uint8_t)v;
    return true;
  }
  bool is_list(const V& o) { return PyList_Check(o.ptr()); }
  void list_extend(V& o, const V* items, size_t k) {
    for (size_t i = 0; i < k; ++i)
      if (PyList_Append(o.ptr(), items[i].ptr()) != 0) throw py::error_already_set();
  }
  bool is_dict(const V& o) { return PyDict_Check(o.ptr()); }
  void dict_set(V& d, const V& k, const V& v) {
    if (PyDict_SetItem(d.ptr(), key_of(k).ptr(), v.ptr()) != 0) throw py::error_already_set();
  }
  bool is_set(const V& o) { return PySet_Check(o.ptr()); }
  void set_add(V& s, const V& k) {
    if (PySet_Add(s.ptr(), key_of(k).ptr()) != 0) throw py::error_already_set();
  }
  V tuple(const V* items, size_t k) {
    py::tuple t(k);
    for (size_t i = 0; i < k; ++i) t[i] = items[i];
    return std::move(t);
  }
  V frozenset(const V* items, size_t k) {
    py::set s;
    for (size_t i = 0; i < k; ++i) set_add(s, items[i]);
    return py::reinterpret_steal<py::object>(PyFrozenSet_New(s.ptr()));
  }
};

py::object loads(const py::bytes& frame, bool u8_as_bytes) {
  char* data = nullptr;
  Py_ssize_t n = 0;
  if (PyBytes_AsStringAndSize(frame.ptr(), &data, &n) != 0) throw py::error_already_set();
  PyBuilder b;
  return rrl::pickle::run(reinterpret_cast<const uint8_t*>(data), (size_t)n, b, u8_as_bytes);
}

void dump(const py::handle& o, std::string& out, int depth, bool bytes_u8) {
  if (depth > kMaxDepth) throw std::invalid_argument("nesting too deep");
  PyObject* p = o.ptr();
  auto put_u32 = [&](uint32_t v) { out.append(reinterpret_cast<const char*>(&v), 4); };
  auto dump_int = [&](long long v) {
    if (v >= 0 && v < 256) {
      out.push_back('K');
      out.push_back((char)v);
    } else if (v >= 0 && v < 65536) {
      out.push_back('M');
      const uint16_t u = (uint16_t)v;
      out.append(reinterpret_cast<const char*>(&u), 2);
    } else {
      out.push_back('J');
      const int32_t s = (int32_t)v;
      out.append(reinterpret_cast<const char*>(&s), 4);
    }
  };
  if (p == Py_None) {
    out.push_back('N');
  } else if (p == Py_True) {
    out.push_back('\x88');
  } else if (p == Py_False) {
    out.push_back('\x89');
  } else if (PyLong_Check(p)) {
    int overflow = 0;
    const long long v = PyLong_AsLongLongAndOverflow(p, &overflow);
    if (!overflow && v >= -2147483648LL && v < 2147483648LL) {
      dump_int(v);
    } else {  // LONG1, as Python's int.to_bytes((bit_length + 8) // 8, "little", signed=True)
      const size_t bits = _PyLong_NumBits(p);
      const size_t k = (bits + 8) / 8;
      std::string raw(k, '\0');
      if (_PyLong_AsByteArray(reinterpret_cast<PyLongObject*>(p), reinterpret_cast<unsigned char*>(&raw[0]), k,
                              /*little_endian=*/1, /*is_signed=*/1) != 0)
        throw py::error_already_set();
      out.push_back('\x8a');
      out.push_back((char)k);
      out += raw;
    }
  } else if (PyFloat_Check(p)) {
    const double d = PyFloat_AsDouble(p);
    uint64_t u;
    std::memcpy(&u, &d, 8);
    out.push_back('G');
    for (int i = 7; i >= 0; --i) out.push_back((char)((u >> (8 * i)) & 0xFF));
  } else if (PyUnicode_Check(p)) {
    Py_ssize_t k = 0;
    const char* s = PyUnicode_AsUTF8AndSize(p, &k);
    if (!s) throw py::error_already_set();
    out.push_back('X');
    put_u32((uint32_t)k);
    out.append(s, (size_t)k);
  } else if (PyBytes_Check(p) || PyByteArray_Check(p)) {
    const char* s = PyBytes_Check(p) ? PyBytes_AS_STRING(p) : PyByteArray_AS_STRING(p);
    const size_t k = (size_t)(PyBytes_Check(p) ? PyBytes_GET_SIZE(p) : PyByteArray_GET_SIZE(p));
    if (bytes_u8) {  // serde's Vec<u8>: a list of ints, APPENDS chunks of 1000
      out.push_back(']');
      for (size_t i = 0; i < k; i += 1000) {
        out.push_back('(');
        for (size_t j = i; j < k && j < i + 1000; ++j) {
          out.push_back('K');
          out.push_back(s[j]);
        }
        out.push_back('e');
      }
    } else if (k < 256) {
      out.push_back('C');
      out.push_back((char)k);
      out.append(s, k);
    } else {
      out.push_back('B');
      put_u32((uint32_t)k);
      out.append(s, k);
    }
  } else if (PyTuple_Check(p)) {
    const Py_ssize_t k = PyTuple_GET_SIZE(p);
    if (k == 0) {
      out.push_back(')');
    } else {
      out.push_back('(');
      for (Py_ssize_t i = 0; i < k; ++i) dump(PyTuple_GET_ITEM(p, i), out, depth + 1, bytes_u8);
      out.push_back('t');
    }
  } else if (PyList_Check(p)) {
    const Py_ssize_t k = PyList_GET_SIZE(p);
    out.push_back(']');
    for (Py_ssize_t i = 0; i < k; i += 1000) {
      out.push_back('(');
      for (Py_ssize_t j = i; j < k && j < i + 1000; ++j) dump(PyList_GET_ITEM(p, j), out, depth + 1, bytes_u8);
      out.push_back('e');
    }
  } else if (PyDict_Check(p)) {
    out.push_back('}');
    if (PyDict_GET_SIZE(p) > 0) {
      out.push_back('(');
      PyObject *k, *v;
      Py_ssize_t pos = 0;
      while (PyDict_Next(p, &pos, &k, &v)) {
        dump(k, out, depth + 1, bytes_u8);
        dump(v, out, depth + 1, bytes_u8);
      }
      out.push_back('u');
    }
  } else {
    throw py::type_error(std::string("cannot serialise ") + Py_TYPE(p)->tp_name);
  }
}

// ------------------------------------------------------------------ reference frame -> columns
template <class T>
py::array_t<T> vec_array(const std::vector<T>& v) {
  py::array_t<T> a((py::ssize_t)v.size());
  if (!v.empty()) std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(T));
  return a;
}

py::object col_array(const rrl::RefCol& c, size_t n, float fill) {
  if (c.width < 0) return py::none();
  py::array_t<float> a({(py::ssize_t)n, (py::ssize_t)c.width});
  float* p = a.mutable_data();
  std::memcpy(p, c.vals.data(), c.vals.size() * sizeof(float));
  for (size_t i = 0; i < n; ++i)
    if (!c.has[i])
      for (long k = 0; k < c.width; ++k) p[i * c.width + k] = fill;
  return std::move(a);
}

// serde_pickle(Vec<RelayRLAction>) (or a RelayRLTrajectory struct) straight to float32 columns,
// decoded by the pure-C++ node-tree path (csrc/host/ref_columns.h) with the GIL RELEASED: the
// per-action objects of serde_pickle.actions_from_reference are never built, and no Python object
// either until the arrays below.
py::dict reference_columns(const py::bytes& frame) {
  char* data = nullptr;
  Py_ssize_t len = 0;
  if (PyBytes_AsStringAndSize(frame.ptr(), &data, &len) != 0) throw py::error_already_set();
  rrl::RefColumns rc;
  {
    py::gil_scoped_release nogil;  // ``frame`` is referenced by the caller for the whole call
    rrl::reference_columns_tree(reinterpret_cast<const uint8_t*>(data), (size_t)len, rc);
  }
  const size_t n = rc.n;
  py::dict out;
  out["n"] = n;
  out["obs"] = col_array(rc.obs, n, 0.f);
  out["has_obs"] = vec_array(rc.obs.has);
  out["act"] = col_array(rc.act, n, 0.f);
  out["has_act"] = vec_array(rc.act.has);
  out["mask"] = col_array(rc.mask, n, 1.f);
  out["has_mask"] = vec_array(rc.mask.has);
  out["rew"] = vec_array(rc.rew);
  out["done"] = vec_array(rc.done);
  out["logp"] = vec_array(rc.logp);
  out["has_logp"] = vec_array(rc.has_logp);
  out["v"] = vec_array(rc.v);
  out["has_v"] = vec_array(rc.has_v);
  return out;
}

// ------------------------------------------------------------------ columns -> reference frame
// The frame a reference agent sends for one episode (agent_zmq.rs:458-610 -> trajectory.rs:50-90),
// written straight from the agent's float32 columns: byte-identical to
// serde_pickle.reference_frame over api.agent's per-action RelayRLAction list, without building
// ~8 Python objects and 4 safetensors byte lists per action.  Row i is
//   {"obs": TD, "act": TD, "mask": TD | None, "rew": rew[i], "data": {"logp_a": {"Tensor": TD},
//    ["v": {"Tensor": TD}]}, "done": False, "reward_updated": reward_updated}
// (TD = {"shape": [w], "dtype": "Float", "data": [u8 of a one-tensor safetensors file]}, "v" only
// where val[i] is not NaN), then the terminal marker {obs, act, mask: None, "rew": last,
// "data": None, "done": True, "reward_updated": False}.
struct RefFrameWriter {
  std::string& o;
  void u32(uint32_t v) { o.append(reinterpret_cast<const char*>(&v), 4); }
  void key(const char* s) {
    const uint32_t k = (uint32_t)std::strlen(s);
    o.push_back('X');
    u32(k);
    o.append(s, k);
  }
  void small(long long v) {  // the ints here: shape entries, u8 values
    if (v >= 0 && v < 256) {
      o.push_back('K');
      o.push_back((char)v);
    } else if (v >= 0 && v < 65536) {
      o.push_back('M');
      const uint16_t u = (uint16_t)v;
      o.append(reinterpret_cast<const char*>(&u), 2);
    } else {
      o.push_back('J');
      const int32_t s = (int32_t)v;
      o.append(reinterpret_cast<const char*>(&s), 4);
    }
  }
  void real(double d) {
    uint64_t u;
    std::memcpy(&u, &d, 8);
    o.push_back('G');
    for (int i = 7; i >= 0; --i) o.push_back((char)((u >> (8 * i)) & 0xFF));
  }
  // the safetensors file of a [width] float32 tensor is a fixed prefix (length + JSON header,
  // which only depend on the width) and the raw bytes: the prefix is built once per width
  std::vector<std::pair<long, std::string>> prefixes;
  const std::string& prefix(long width) {
    for (const auto& pw : prefixes)
      if (pw.first == width) return pw.second;
    rrl::Tensor t;
    t.dtype = rrl::DType::Float;
    t.shape = {width};
    t.raw.assign(sizeof(float) * (size_t)width, '\0');
    std::string f = rrl::st_encode(t);
    f.resize(f.size() - t.raw.size());
    prefixes.emplace_back(width, std::move(f));
    return prefixes.back().second;
  }
  // serde's Vec<u8> of the bytes a[0..na) then b[0..nb): a list of K ints in APPENDS chunks of 1000
  void u8list(const char* a, size_t na, const char* b, size_t nb) {
    const size_t k = na + nb;
    o.push_back(']');
    for (size_t i = 0; i < k; i += 1000) {
      const size_t e = std::min(k, i + 1000);
      const size_t base = o.size();
      o.resize(base + 2 + 2 * (e - i));
      char* d = &o[base];
      *d++ = '(';
      for (size_t j = i; j < e; ++j) {
        *d++ = 'K';
        *d++ = j < na ? a[j] : b[j - na];
      }
      *d = 'e';
    }
  }
  void td(const float* p, long width) {
    const std::string& pre = prefix(width);
    o.push_back('}');
    o.push_back('(');
    key("shape");
    o.push_back(']');
    o.push_back('(');
    small(width);
    o.push_back('e');
    key("dtype");
    key("Float");
    key("data");
    u8list(pre.data(), pre.size(), reinterpret_cast<const char*>(p), sizeof(float) * (size_t)width);
    o.push_back('u');
  }
  void tensor_entry(const char* name, const float* p) {  // "name": {"Tensor": TD of [1]}
    key(name);
    o.push_back('}');
    o.push_back('(');
    key("Tensor");
    td(p, 1);
    o.push_back('u');
  }
};

template <class A>
const float* f32_rows(const A& a, size_t n, long& width, const char* what) {
  if (a.ndim() != 2 || (size_t)a.shape(0) != n) throw std::invalid_argument(std::string(what) + " must be [n][w]");
  width = (long)a.shape(1);
  return a.data();
}

py::bytes reference_frame_columns(py::array_t<float, py::array::c_style | py::array::forcecast> obs,
                                  py::array_t<float, py::array::c_style | py::array::forcecast> act, py::object mask,
                                  py::array_t<float, py::array::c_style | py::array::forcecast> rew,
                                  py::array_t<float, py::array::c_style | py::array::forcecast> logp,
                                  py::array_t<float, py::array::c_style | py::array::forcecast> val, double last,
                                  bool reward_updated) {
  using farr = py::array_t<float, py::array::c_style | py::array::forcecast>;
  const size_t n = (size_t)rew.size();
  if ((size_t)logp.size() != n || (size_t)val.size() != n) throw std::invalid_argument("rew / logp / val lengths differ");
  long wo = 0, wa = 0, wm = 0;
  const float* po = f32_rows(obs, n, wo, "obs");
  const float* pa = f32_rows(act, n, wa, "act");
  farr m;
  const float* pm = nullptr;
  if (!mask.is_none()) {
    m = mask.cast<farr>();
    pm = f32_rows(m, n, wm, "mask");
  }
  const float *pr = rew.data(), *pl = logp.data(), *pv = val.data();
  std::string out = "\x80\x03";
  {
    py::gil_scoped_release nogil;  // the arrays are held by this frame's arguments
    out.reserve(64 + (n + 1) * (size_t)(700 + 240 * (wo + wa + wm)));
    RefFrameWriter w{out, {}};
    const size_t total = n + 1;
    out.push_back(']');
    for (size_t c = 0; c < total; c += 1000) {
      out.push_back('(');
      for (size_t i = c; i < total && i < c + 1000; ++i) {
        out.push_back('}');
        out.push_back('(');
        if (i < n) {
          w.key("obs");
          w.td(po + i * wo, wo);
          w.key("act");
          w.td(pa + i * wa, wa);
          w.key("mask");
          if (pm) w.td(pm + i * wm, wm);
          else out.push_back('N');
          w.key("rew");
          w.real((double)pr[i]);
          w.key("data");
          out.push_back('}');
          out.push_back('(');
          w.tensor_entry("logp_a", pl + i);
          if (!std::isnan(pv[i])) w.tensor_entry("v", pv + i);
          out.push_back('u');
          w.key("done");
          out.push_back('\x89');
          w.key("reward_updated");
          out.push_back(reward_updated ? '\x88' : '\x89');
        } else {
          w.key("obs");
          out.push_back('N');
          w.key("act");
          out.push_back('N');
          w.key("mask");
          out.push_back('N');
          w.key("rew");
          w.real(last);
          w.key("data");
          out.push_back('N');
          w.key("done");
          out.push_back('\x88');
          w.key("reward_updated");
          out.push_back('\x89');
        }
        out.push_back('u');
      }
      out.push_back('e');
    }
    out.push_back('.');
  }
  return py::bytes(out);
}

}  // namespace

void bind_pickle(py::module_& m) {
  static py::exception<FrameError> frame_error(m, "PickleFrameError", PyExc_ValueError);
  m.def(
      "pickle_loads",
      [](const py::bytes& b, bool u8_lists_as_bytes) {
        try {
          return loads(b, u8_lists_as_bytes);
        } catch (const FrameError& e) {
          PyErr_SetString(frame_error.ptr(), e.what());
          throw py::error_already_set();
        }
      },
      py::arg("frame"), py::arg("u8_lists_as_bytes") = false,
      "Data-only pickle interpreter (transport/serde_pickle.py semantics) in C++");
  m.def(
      "pickle_dumps",
      [](const py::handle& o, bool bytes_as_u8_list) {
        std::string out = "\x80\x03";
        dump(o, out, 0, bytes_as_u8_list);
        out.push_back('.');
        return py::bytes(out);
      },
      py::arg("obj"), py::arg("bytes_as_u8_list") = false, "serde_pickle-style writer (protocol 3, no memo)");
  m.def(
      "reference_columns",
      [](const py::bytes& b) {
        try {
          return reference_columns(b);
        } catch (const FrameError& e) {
          PyErr_SetString(frame_error.ptr(), e.what());
          throw py::error_already_set();
        }
      },
      py::arg("frame"),
      "serde_pickle(Vec<RelayRLAction>) -> float32 columns (obs/act/mask, rew, done, logp, v + presence flags)");
  m.def("reference_frame_columns", &reference_frame_columns, py::arg("obs"), py::arg("act"), py::arg("mask"),
        py::arg("rew"), py::arg("logp"), py::arg("val"), py::arg("last"), py::arg("reward_updated"),
        "one episode's float32 columns -> the reference agent's serde_pickle(Vec<RelayRLAction>) frame");
}
