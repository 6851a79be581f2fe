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

#include <cmath>
#include <cstring>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "codec.h"

namespace py = pybind11;

namespace {

constexpr int kMaxDepth = 64;
constexpr size_t kMaxStack = 1u << 20;
constexpr size_t kMaxMemo = 1u << 16;

struct FrameError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

class Reader {
 public:
  Reader(const uint8_t* p, size_t n) : p_(p), n_(n) {}
  // "K b K b ... e" right after a MARK (serde's Vec<u8> chunk: up to 1000 BININT1 + APPENDS):
  // the bytes appended to ``out`` and the run consumed; anything else leaves the position as it was
  bool u8_run(std::string& out) {
    size_t q = pos_;
    const size_t start = out.size();
    while (q + 1 < n_ && p_[q] == 0x4B) {
      out.push_back((char)p_[q + 1]);
      q += 2;
    }
    if (q < n_ && p_[q] == 0x65) {
      pos_ = q + 1;
      return true;
    }
    out.resize(start);
    return false;
  }
  const uint8_t* take(size_t k) {
    if (pos_ + k > n_) throw FrameError("truncated frame");
    const uint8_t* out = p_ + pos_;
    pos_ += k;
    return out;
  }
  uint8_t u8() { return *take(1); }
  template <class T>
  T le() {
    T v;
    std::memcpy(&v, take(sizeof(T)), sizeof(T));
    return v;
  }

 private:
  const uint8_t* p_;
  size_t n_;
  size_t pos_ = 0;
};

py::object key_of(const py::object& k) {
  if (py::isinstance<py::list>(k) || py::isinstance<py::dict>(k) || py::isinstance<py::set>(k) ||
      py::isinstance<py::bytearray>(k))
    throw FrameError("unhashable key");
  return k;
}

bool all_u8(const std::vector<py::object>& items, size_t from) {
  for (size_t i = from; i < items.size(); ++i) {
    PyObject* o = items[i].ptr();
    if (!PyLong_CheckExact(o)) return false;
    int overflow = 0;
    const long v = PyLong_AsLongAndOverflow(o, &overflow);
    if (overflow || v < 0 || v > 255) return false;
  }
  return true;
}

py::object loads(const py::bytes& frame, bool u8_as_bytes) {
  char* data = nullptr;
  Py_ssize_t n = 0;
  if (PyBytes_AsStringAndSize(frame.ptr(), &data, &n) != 0) throw py::error_already_set();
  Reader r(reinterpret_cast<const uint8_t*>(data), (size_t)n);
  std::vector<py::object> stack;
  std::vector<size_t> marks;
  std::unordered_map<uint32_t, py::object> memo;
  std::string run;  // scratch of the u8 fast form
  auto pop_value = [&]() {
    if (stack.empty() || (!marks.empty() && marks.back() == stack.size())) throw FrameError("stack underflow");
    py::object v = std::move(stack.back());
    stack.pop_back();
    return v;
  };
  auto pop_mark = [&]() -> size_t {  // index of the first item above the mark
    if (marks.empty()) throw FrameError("MARK not found");
    const size_t m = marks.back();
    marks.pop_back();
    return m;
  };
  auto top = [&]() -> py::object& {
    if (stack.empty() || (!marks.empty() && marks.back() == stack.size())) throw FrameError("stack underflow");
    return stack.back();
  };
  // the container below the items [from, end): no MARK may sit between them
  auto container_below = [&](size_t from) -> py::object& {
    if (from == 0 || stack.size() < from || (!marks.empty() && marks.back() >= from)) throw FrameError("stack underflow");
    return stack[from - 1];
  };
  auto as_list = [&](py::object& o) {  // a bytearray still being built as a Vec<u8> -> list of ints
    if (u8_as_bytes && py::isinstance<py::bytearray>(o)) {
      py::list l;
      const char* b = PyByteArray_AsString(o.ptr());
      for (Py_ssize_t i = 0; i < PyByteArray_Size(o.ptr()); ++i) l.append(py::int_((unsigned char)b[i]));
      o = l;
    }
  };
  // list APPEND / APPENDS onto the container, with the u8 fast form
  auto extend_top = [&](size_t from) {
    py::object& tgt = container_below(from);
    if (u8_as_bytes && py::isinstance<py::bytearray>(tgt)) {
      if (all_u8(stack, from)) {
        std::string chunk(stack.size() - from, '\0');
        for (size_t i = from; i < stack.size(); ++i) chunk[i - from] = (char)PyLong_AsLong(stack[i].ptr());
        const Py_ssize_t old = PyByteArray_Size(tgt.ptr());
        if (PyByteArray_Resize(tgt.ptr(), old + (Py_ssize_t)chunk.size()) != 0) throw py::error_already_set();
        std::memcpy(PyByteArray_AsString(tgt.ptr()) + old, chunk.data(), chunk.size());
        stack.resize(from);
        return;
      }
      as_list(tgt);  // not a Vec<u8> after all
    }
    if (!py::isinstance<py::list>(tgt)) throw FrameError("expected a list on the stack");
    py::list l = tgt.cast<py::list>();
    for (size_t i = from; i < stack.size(); ++i) l.append(stack[i]);
    stack.resize(from);
  };
  for (;;) {
    if (stack.size() > kMaxStack || memo.size() > kMaxMemo) throw FrameError("frame too large");
    const uint8_t op = r.u8();
    switch (op) {
      case 0x80: r.take(1); break;  // PROTO
      case 0x95: r.take(8); break;  // FRAME
      case 0x2E:                    // STOP
        if (stack.size() != 1 || !marks.empty()) throw FrameError("bad stack at STOP");
        return stack[0];
      case 0x4E: stack.push_back(py::none()); break;
      case 0x88: stack.push_back(py::bool_(true)); break;
      case 0x89: stack.push_back(py::bool_(false)); break;
      case 0x4B: stack.push_back(py::int_(r.u8())); break;                // BININT1
      case 0x4D: stack.push_back(py::int_(r.le<uint16_t>())); break;      // BININT2
      case 0x4A: stack.push_back(py::int_(r.le<int32_t>())); break;       // BININT
      case 0x8A:                                                          // LONG1
      case 0x8B: {                                                        // LONG4
        int64_t k = op == 0x8A ? r.u8() : r.le<int32_t>();
        if (k < 0 || k > 64) throw FrameError("LONG4 too large");
        const uint8_t* b = r.take((size_t)k);
        PyObject* v = k ? _PyLong_FromByteArray(b, (size_t)k, /*little_endian=*/1, /*is_signed=*/1) : PyLong_FromLong(0);
        if (!v) throw py::error_already_set();
        stack.push_back(py::reinterpret_steal<py::object>(v));
        break;
      }
      case 0x47: {  // BINFLOAT (big-endian double)
        const uint8_t* b = r.take(8);
        uint64_t u = 0;
        for (int i = 0; i < 8; ++i) u = (u << 8) | b[i];
        double d;
        std::memcpy(&d, &u, 8);
        stack.push_back(py::float_(d));
        break;
      }
      case 0x58:    // BINUNICODE
      case 0x8C:    // SHORT_BINUNICODE
      case 0x8D: {  // BINUNICODE8
        const uint64_t k = op == 0x58 ? r.le<uint32_t>() : (op == 0x8C ? r.u8() : r.le<uint64_t>());
        if (k > (uint64_t)n) throw FrameError("truncated frame");
        const char* s = reinterpret_cast<const char*>(r.take((size_t)k));
        PyObject* v = PyUnicode_DecodeUTF8(s, (Py_ssize_t)k, "strict");
        if (!v) throw py::error_already_set();
        stack.push_back(py::reinterpret_steal<py::object>(v));
        break;
      }
      case 0x42:    // BINBYTES
      case 0x43:    // SHORT_BINBYTES
      case 0x8E: {  // BINBYTES8
        const uint64_t k = op == 0x42 ? r.le<uint32_t>() : (op == 0x43 ? r.u8() : r.le<uint64_t>());
        if (k > (uint64_t)n) throw FrameError("truncated frame");
        const char* s = reinterpret_cast<const char*>(r.take((size_t)k));
        stack.push_back(py::bytes(s, (size_t)k));
        break;
      }
      case 0x28:  // MARK
        // u8 form: a MARK that opens a pure "K b ... APPENDS" run onto a Vec<u8> being built goes
        // straight into the bytearray, no Python int per byte (~20,000 of them per CartPole frame)
        if (u8_as_bytes && !stack.empty() && (marks.empty() || marks.back() < stack.size()) &&
            PyByteArray_Check(stack.back().ptr())) {
          run.clear();
          if (r.u8_run(run)) {
            PyObject* ba = stack.back().ptr();
            const Py_ssize_t old = PyByteArray_Size(ba);
            if (PyByteArray_Resize(ba, old + (Py_ssize_t)run.size()) != 0) throw py::error_already_set();
            if (!run.empty()) std::memcpy(PyByteArray_AsString(ba) + old, run.data(), run.size());
            break;
          }
        }
        if ((int)marks.size() >= kMaxDepth) throw FrameError("nesting too deep");
        marks.push_back(stack.size());
        break;
      case 0x5D:  // EMPTY_LIST
        if (u8_as_bytes) stack.push_back(py::reinterpret_steal<py::object>(PyByteArray_FromStringAndSize("", 0)));
        else stack.push_back(py::list());
        break;
      case 0x7D: stack.push_back(py::dict()); break;
      case 0x29: stack.push_back(py::tuple()); break;
      case 0x8F: stack.push_back(py::set()); break;
      case 0x61: {  // APPEND
        if (stack.empty() || (!marks.empty() && marks.back() == stack.size())) throw FrameError("stack underflow");
        extend_top(stack.size() - 1);
        break;
      }
      case 0x65: extend_top(pop_mark()); break;  // APPENDS
      case 0x73: {                               // SETITEM
        py::object v = pop_value();
        py::object k = pop_value();
        py::object& d = top();
        if (!py::isinstance<py::dict>(d)) throw FrameError("expected a dict on the stack");
        d.cast<py::dict>()[key_of(k)] = v;
        break;
      }
      case 0x75: {  // SETITEMS
        const size_t m = pop_mark();
        if ((stack.size() - m) % 2) throw FrameError("odd SETITEMS");
        py::object& c = container_below(m);
        if (!py::isinstance<py::dict>(c)) throw FrameError("expected a dict on the stack");
        py::dict d = c.cast<py::dict>();
        for (size_t i = m; i < stack.size(); i += 2) d[key_of(stack[i])] = stack[i + 1];
        stack.resize(m);
        break;
      }
      case 0x90: {  // ADDITEMS
        const size_t m = pop_mark();
        py::object& c = container_below(m);
        if (!py::isinstance<py::set>(c)) throw FrameError("expected a set on the stack");
        py::set s = c.cast<py::set>();
        for (size_t i = m; i < stack.size(); ++i) s.add(key_of(stack[i]));
        stack.resize(m);
        break;
      }
      case 0x91: {  // FROZENSET
        const size_t m = pop_mark();
        py::set s;
        for (size_t i = m; i < stack.size(); ++i) s.add(key_of(stack[i]));
        stack.resize(m);
        stack.push_back(py::reinterpret_steal<py::object>(PyFrozenSet_New(s.ptr())));
        break;
      }
      case 0x74: {  // TUPLE
        const size_t m = pop_mark();
        py::tuple t(stack.size() - m);
        for (size_t i = m; i < stack.size(); ++i) t[i - m] = stack[i];
        stack.resize(m);
        stack.push_back(t);
        break;
      }
      case 0x85:
      case 0x86:
      case 0x87: {  // TUPLE1..3
        const size_t k = op - 0x84;
        if (stack.size() < k || (!marks.empty() && marks.back() > stack.size() - k)) throw FrameError("stack underflow");
        py::tuple t(k);
        for (size_t i = 0; i < k; ++i) t[i] = stack[stack.size() - k + i];
        stack.resize(stack.size() - k);
        stack.push_back(t);
        break;
      }
      // (serde_pickle writes no memo; a memoised list is built as a list, not in the u8 form)
      case 0x71: as_list(top()); memo[r.u8()] = top(); break;                 // BINPUT
      case 0x72: as_list(top()); memo[r.le<uint32_t>()] = top(); break;       // LONG_BINPUT
      case 0x94: as_list(top()); memo[(uint32_t)memo.size()] = top(); break;  // MEMOIZE
      case 0x68:                                            // BINGET
      case 0x6A: {                                          // LONG_BINGET
        const uint32_t k = op == 0x68 ? r.u8() : r.le<uint32_t>();
        auto it = memo.find(k);
        if (it == memo.end()) throw FrameError("memo key not found");
        stack.push_back(it->second);
        break;
      }
      case 0x30:  // POP
        if (!marks.empty() && marks.back() == stack.size()) {
          marks.pop_back();
        } else {
          if (stack.empty()) throw FrameError("stack underflow");
          stack.pop_back();
        }
        break;
      case 0x31: stack.resize(pop_mark()); break;  // POP_MARK
      default: {
        char msg[80];
        snprintf(msg, sizeof(msg), "opcode 0x%02x is not allowed in a trajectory frame", op);
        throw FrameError(msg);
      }
    }
  }
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
// serde enum in any serde_pickle representation -> (variant, payload) (serde_pickle.enum_variant)
std::pair<std::string, py::object> variant(const py::handle& v) {
  if (py::isinstance<py::str>(v)) return {v.cast<std::string>(), py::none()};
  if (py::isinstance<py::dict>(v)) {
    py::dict d = py::reinterpret_borrow<py::dict>(v);
    if (d.size() == 1)
      for (auto kv : d) return {py::str(kv.first).cast<std::string>(), py::reinterpret_borrow<py::object>(kv.second)};
  }
  if (py::isinstance<py::tuple>(v) || py::isinstance<py::list>(v)) {
    py::sequence q = py::reinterpret_borrow<py::sequence>(v);
    if ((q.size() == 1 || q.size() == 2) && py::isinstance<py::str>(q[0]))
      return {q[0].cast<std::string>(), q.size() == 2 ? py::object(q[1]) : py::object(py::none())};
  }
  throw FrameError("not an enum value");
}

std::string byte_payload(const py::handle& data) {
  if (py::isinstance<py::bytearray>(data)) {
    return std::string(PyByteArray_AsString(data.ptr()), (size_t)PyByteArray_Size(data.ptr()));
  }
  if (py::isinstance<py::bytes>(data)) return data.cast<std::string>();
  if (py::isinstance<py::list>(data) || py::isinstance<py::tuple>(data)) {
    py::sequence q = py::reinterpret_borrow<py::sequence>(data);
    std::string out(q.size(), '\0');
    for (size_t i = 0; i < q.size(); ++i) {
      const long v = q[i].cast<long>();
      if (v < 0 || v > 255) throw FrameError("TensorData.data must be bytes or a list of u8");
      out[i] = (char)v;
    }
    return out;
  }
  throw FrameError("TensorData.data must be bytes or a list of u8");
}

// TensorData {shape, dtype, data: one-tensor safetensors file} -> float32 values; false if None.
// Headers are parsed once per distinct header text per frame (every obs of a frame has the same
// one): ``cache`` maps header bytes -> (dtype, shape, data range).
using HeaderCache = std::unordered_map<std::string, rrl::StHeader>;
bool tensor_f32(const py::handle& td, std::vector<float>& out, HeaderCache& cache) {
  if (td.is_none()) return false;
  if (!py::isinstance<py::dict>(td)) throw FrameError("TensorData must be a dict with shape / dtype / data");
  py::dict d = py::reinterpret_borrow<py::dict>(td);
  if (!d.contains("data")) throw FrameError("TensorData must be a dict with shape / dtype / data");
  py::object data = d["data"];
  std::string owned;
  const char* p = nullptr;
  size_t n = 0;
  if (py::isinstance<py::bytearray>(data)) {
    p = PyByteArray_AsString(data.ptr());
    n = (size_t)PyByteArray_Size(data.ptr());
  } else if (py::isinstance<py::bytes>(data)) {
    p = PyBytes_AsString(data.ptr());
    n = (size_t)PyBytes_Size(data.ptr());
  } else {
    owned = byte_payload(data);
    p = owned.data();
    n = owned.size();
  }
  if (n < 8) throw FrameError("TensorData: safetensors: file too short");
  uint64_t hl = 0;
  for (int i = 0; i < 8; ++i) hl |= (uint64_t)(uint8_t)p[i] << (8 * i);
  if (hl > n - 8) throw FrameError("TensorData: safetensors: header length out of range");
  std::string key(p + 8, (size_t)hl);
  auto it = cache.find(key);
  if (it == cache.end()) {
    try {
      it = cache.emplace(std::move(key), rrl::st_header(p + 8, (size_t)hl)).first;
    } catch (const std::exception& e) {
      throw FrameError(std::string("TensorData: ") + e.what());
    }
  }
  const rrl::StHeader& h = it->second;
  const size_t base = 8 + (size_t)hl;
  // st_header guarantees 0 <= off0 <= off1 and off1 - off0 == count * dtype size
  if (h.off0 < 0 || h.off1 < h.off0 || (uint64_t)h.off1 > n - base)
    throw FrameError("TensorData: safetensors: bad data offsets");
  int64_t cnt = 1;
  for (auto s : h.shape) cnt *= s;
  out.resize((size_t)cnt);
  const char* r = p + base + h.off0;
  for (int64_t i = 0; i < cnt; ++i) {
    switch (h.dtype) {
      case rrl::DType::Byte: out[i] = (float)(uint8_t)r[i]; break;
      case rrl::DType::Bool: out[i] = r[i] ? 1.f : 0.f; break;
      case rrl::DType::Short: { int16_t v; std::memcpy(&v, r + 2 * i, 2); out[i] = (float)v; break; }
      case rrl::DType::Int: { int32_t v; std::memcpy(&v, r + 4 * i, 4); out[i] = (float)v; break; }
      case rrl::DType::Long: { int64_t v; std::memcpy(&v, r + 8 * i, 8); out[i] = (float)v; break; }
      case rrl::DType::Float: { float v; std::memcpy(&v, r + 4 * i, 4); out[i] = v; break; }
      case rrl::DType::Double: { double v; std::memcpy(&v, r + 8 * i, 8); out[i] = (float)v; break; }
    }
  }
  return true;
}

// one column of per-action vectors (all present rows must have the same length)
struct Col {
  std::vector<float> vals;
  std::vector<uint8_t> has;
  long width = -1;
  void add(bool present, const std::vector<float>& v) {
    has.push_back(present ? 1 : 0);
    if (present) {
      if (width < 0) {
        width = (long)v.size();
        // earlier absent rows: zero-filled at the new width
        vals.assign((has.size() - 1) * (size_t)width, 0.f);
      } else if ((long)v.size() != width) {
        throw FrameError("ragged tensors in one frame");
      }
      vals.insert(vals.end(), v.begin(), v.end());
    } else if (width >= 0) {
      vals.insert(vals.end(), (size_t)width, 0.f);
    }
  }
  py::object array(size_t n, float fill) const {
    if (width < 0) return py::none();
    py::array_t<float> a({(py::ssize_t)n, (py::ssize_t)width});
    float* p = a.mutable_data();
    std::memcpy(p, vals.data(), vals.size() * sizeof(float));
    for (size_t i = 0; i < n; ++i)
      if (!has[i])
        for (long k = 0; k < width; ++k) p[i * width + k] = fill;
    return std::move(a);
  }
};

template <class T>
py::array_t<T> vec_array(const std::vector<T>& v) {
  py::array_t<T> a((py::ssize_t)v.size());
  if (!v.empty()) std::memcpy(a.mutable_data(), v.data(), v.size() * sizeof(T));
  return a;
}

// serde_pickle(Vec<RelayRLAction>) (or a RelayRLTrajectory struct) straight to float32 columns:
// the per-action objects of serde_pickle.actions_from_reference are never built.
py::dict reference_columns(const py::bytes& frame) {
  py::object root = loads(frame, true);
  if (py::isinstance<py::dict>(root)) {
    py::dict d = root.cast<py::dict>();
    if (d.contains("actions")) root = d["actions"];
  }
  if (py::isinstance<py::bytearray>(root) && PyByteArray_Size(root.ptr()) == 0) root = py::list();
  if (!py::isinstance<py::list>(root) && !py::isinstance<py::tuple>(root)) throw FrameError("expected a list of actions");
  py::sequence acts = py::reinterpret_borrow<py::sequence>(root);
  const size_t n = acts.size();
  Col obs, act, mask;
  HeaderCache hc;
  std::vector<float> rew, logp, v, tmp;
  std::vector<uint8_t> done, has_logp, has_v;
  rew.reserve(n);
  for (size_t i = 0; i < n; ++i) {
    py::handle a = acts[i];
    if (!py::isinstance<py::dict>(a)) throw FrameError("an action must be a dict");
    py::dict ad = py::reinterpret_borrow<py::dict>(a);
    auto field = [&](const char* k) -> py::object { return ad.contains(k) ? py::object(ad[k]) : py::object(py::none()); };
    bool p = tensor_f32(field("obs"), tmp, hc);
    obs.add(p, tmp);
    p = tensor_f32(field("act"), tmp, hc);
    act.add(p, tmp);
    p = tensor_f32(field("mask"), tmp, hc);
    mask.add(p, tmp);
    py::object r = field("rew");
    rew.push_back(r.is_none() ? 0.f : r.cast<float>());
    py::object dn = field("done");
    done.push_back(!dn.is_none() && dn.cast<bool>() ? 1 : 0);
    float lp = NAN, vv = NAN;
    uint8_t hl = 0, hv = 0;
    py::object data = field("data");
    if (!data.is_none()) {
      if (!py::isinstance<py::dict>(data)) throw FrameError("RelayRLAction.data must be a dict");
      for (auto kv : data.cast<py::dict>()) {
        const std::string key = py::str(kv.first).cast<std::string>();
        if (key != "logp_a" && key != "v") continue;
        auto var = variant(kv.second);
        float x = NAN;
        if (var.first == "Tensor") {
          if (!tensor_f32(var.second, tmp, hc) || tmp.empty()) continue;
          x = tmp[0];
        } else if (var.first == "Float" || var.first == "Double" || var.first == "Int" || var.first == "Long" ||
                   var.first == "Short" || var.first == "Byte") {
          x = var.second.cast<float>();
        } else {
          continue;
        }
        if (key == "logp_a") {
          lp = x;
          hl = 1;
        } else {
          vv = x;
          hv = 1;
        }
      }
    }
    logp.push_back(lp);
    has_logp.push_back(hl);
    v.push_back(vv);
    has_v.push_back(hv);
  }
  py::dict out;
  out["n"] = n;
  out["obs"] = obs.array(n, 0.f);
  out["has_obs"] = vec_array(obs.has);
  out["act"] = act.array(n, 0.f);
  out["has_act"] = vec_array(act.has);
  out["mask"] = mask.array(n, 1.f);
  out["has_mask"] = vec_array(mask.has);
  out["rew"] = vec_array(rew);
  out["done"] = vec_array(done);
  out["logp"] = vec_array(logp);
  out["has_logp"] = vec_array(has_logp);
  out["v"] = vec_array(v);
  out["has_v"] = vec_array(has_v);
  return out;
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
}
