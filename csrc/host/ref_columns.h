// A reference agent's upload -- serde_pickle(Vec<RelayRLAction>) (trajectory.rs:50-90), or a
// RelayRLTrajectory struct holding one -- straight to float32 columns, in C++ without Python
// objects: the frame becomes a node tree (pickle_tree.h), every TensorData payload goes through
// st_tensor_f32, and the caller builds numpy arrays once at the end.  The server's decoder
// (bindings/pickle_native.cpp ``reference_columns``) runs this with the GIL released, so the
// ingest of many reference agents no longer serialises on the interpreter lock; the sanitizer
// fuzz harness (selftest/parser_fuzz.cpp) runs it on every accepted mutant.
//
// Semantics of the per-action path (transport/serde_pickle.actions_from_reference): a missing
// field is None; ``rew`` / ``done`` accept numbers and bools; ``data`` keeps the last of
// duplicate keys; ``logp_a`` / ``v`` are read from a Tensor (its first value) or a numeric
// RelayRLData variant; every present obs / act / mask of a frame must have one width.
#pragma once

#include <cmath>
#include <string>
#include <vector>

#include "pickle_tree.h"
#include "st_tensor.h"

namespace rrl {

struct RefCol {
  std::vector<float> vals;
  std::vector<uint8_t> has;
  long width = -1;
  void add(bool present, const std::vector<float>& v) {
    has.push_back(present ? 1 : 0);
    if (present) {
      if (width < 0) {
        width = (long)v.size();
        vals.assign((has.size() - 1) * (size_t)width, 0.f);  // earlier absent rows at the new width
      } else if ((long)v.size() != width) {
        throw pickle::FrameError("ragged tensors in one frame");
      }
      vals.insert(vals.end(), v.begin(), v.end());
    } else if (width >= 0) {
      vals.insert(vals.end(), (size_t)width, 0.f);
    }
  }
};

struct RefColumns {
  size_t n = 0;
  RefCol obs, act, mask;
  std::vector<float> rew, logp, v;
  std::vector<uint8_t> done, has_logp, has_v;
};

namespace refcols {
using pickle::FrameError;
using pickle::Node;

inline bool is_str(const Node* k, const char* s) { return k->k == Node::Str && k->s == s; }

// dict lookup with Python's "last assignment wins"; nullptr = missing
inline const Node* get(const Node* d, const char* key) {
  const Node* out = nullptr;
  for (size_t i = 0; i + 1 < d->items.size(); i += 2)
    if (is_str(d->items[i], key)) out = d->items[i + 1];
  return out;
}

inline double big_value(const std::string& le) {  // LONG1 / LONG4 bytes, little-endian two's complement
  if (le.empty()) return 0.0;
  const bool neg = (uint8_t)le.back() & 0x80;
  double m = 0.0;
  for (size_t i = le.size(); i-- > 0;) m = m * 256.0 + (double)(uint8_t)(neg ? ~(uint8_t)le[i] : (uint8_t)le[i]);
  return neg ? -(m + 1.0) : m;
}

inline float number(const Node* n, const char* what) {
  switch (n->k) {
    case Node::Bool:
    case Node::Int: return (float)n->i;
    case Node::Float: return (float)n->f;
    case Node::Big: return (float)big_value(n->s);
    default: throw FrameError(std::string(what) + " must be a number");
  }
}

inline bool truthy(const Node* n) {
  switch (n->k) {
    case Node::None: return false;
    case Node::Bool:
    case Node::Int: return n->i != 0;
    case Node::Float: return n->f != 0.0;
    case Node::Big: return big_value(n->s) != 0.0;
    default: throw FrameError("done must be a bool");
  }
}

// serde enum in any serde_pickle representation -> (variant, payload) (serde_pickle.enum_variant)
inline std::pair<std::string, const Node*> variant(const Node* v) {
  if (v->k == Node::Str) return {v->s, nullptr};
  if (v->k == Node::Dict) {
    // a one-entry dict (duplicate keys collapse, as in Python)
    const Node* key = nullptr;
    size_t distinct = 0;
    for (size_t i = 0; i + 1 < v->items.size(); i += 2) {
      const Node* k = v->items[i];
      bool seen = false;
      for (size_t j = 0; j < i; j += 2)
        if (v->items[j]->k == Node::Str && k->k == Node::Str && v->items[j]->s == k->s) seen = true;
      if (!seen) {
        ++distinct;
        key = k;
      }
    }
    if (distinct == 1 && key->k == Node::Str) return {key->s, get(v, key->s.c_str())};
  }
  if (v->k == Node::Tuple || v->k == Node::List) {
    if ((v->items.size() == 1 || v->items.size() == 2) && v->items[0]->k == Node::Str)
      return {v->items[0]->s, v->items.size() == 2 ? v->items[1] : nullptr};
  }
  throw FrameError("not an enum value");
}

// TensorData {shape, dtype, data} -> float32 values; false if None / missing
inline bool tensor(const Node* td, std::vector<float>& out, StHeaderCache& hc, std::string& scratch) {
  if (td == nullptr || td->k == Node::None) return false;
  if (td->k != Node::Dict) throw FrameError("TensorData must be a dict with shape / dtype / data");
  const Node* data = get(td, "data");
  if (data == nullptr) throw FrameError("TensorData must be a dict with shape / dtype / data");
  const char* p;
  size_t n;
  if (data->k == Node::Bytes || data->k == Node::ByteArr) {
    p = data->s.data();
    n = data->s.size();
  } else if (data->k == Node::List || data->k == Node::Tuple) {
    scratch.resize(data->items.size());
    for (size_t i = 0; i < data->items.size(); ++i) {
      const Node* b = data->items[i];
      if (!(b->k == Node::Int || b->k == Node::Bool) || b->i < 0 || b->i > 255)
        throw FrameError("TensorData.data must be bytes or a list of u8");
      scratch[i] = (char)b->i;
    }
    p = scratch.data();
    n = scratch.size();
  } else {
    throw FrameError("TensorData.data must be bytes or a list of u8");
  }
  try {
    st_tensor_f32(p, n, out, hc);
  } catch (const FrameError&) {
    throw;
  } catch (const std::exception& e) {
    throw FrameError(std::string("TensorData: ") + e.what());
  }
  return true;
}
}  // namespace refcols

// frame bytes -> columns; throws pickle::FrameError on anything malformed
inline void reference_columns_tree(const uint8_t* frame, size_t len, RefColumns& rc) {
  using namespace refcols;
  pickle::NodeBuilder b;
  const Node* root = pickle::run(frame, len, b, /*u8_form=*/true);
  if (root->k == Node::Dict) {
    if (const Node* a = get(root, "actions")) root = a;
  }
  static const Node kEmptyList = [] {
    Node e;
    e.k = Node::List;
    return e;
  }();
  if (root->k == Node::ByteArr && root->s.empty()) root = &kEmptyList;
  if (root->k != Node::List && root->k != Node::Tuple) throw FrameError("expected a list of actions");
  const size_t n = root->items.size();
  rc = RefColumns();
  rc.n = n;
  rc.rew.reserve(n);
  StHeaderCache hc;
  std::vector<float> tmp;
  std::string scratch;
  for (size_t i = 0; i < n; ++i) {
    const Node* a = root->items[i];
    if (a->k != Node::Dict) throw FrameError("an action must be a dict");
    bool p = tensor(get(a, "obs"), tmp, hc, scratch);
    rc.obs.add(p, tmp);
    p = tensor(get(a, "act"), tmp, hc, scratch);
    rc.act.add(p, tmp);
    p = tensor(get(a, "mask"), tmp, hc, scratch);
    rc.mask.add(p, tmp);
    const Node* r = get(a, "rew");
    rc.rew.push_back(r == nullptr || r->k == Node::None ? 0.f : number(r, "rew"));
    const Node* dn = get(a, "done");
    rc.done.push_back(dn != nullptr && truthy(dn) ? 1 : 0);
    float lp = NAN, vv = NAN;
    uint8_t hl = 0, hv = 0;
    const Node* data = get(a, "data");
    if (data != nullptr && data->k != Node::None) {
      if (data->k != Node::Dict) throw FrameError("RelayRLAction.data must be a dict");
      for (const char* key : {"logp_a", "v"}) {
        const Node* val = get(data, key);
        if (val == nullptr) continue;
        const auto var = variant(val);
        float x = NAN;
        if (var.first == "Tensor") {
          if (!tensor(var.second, tmp, hc, scratch) || tmp.empty()) continue;
          x = tmp[0];
        } else if (var.first == "Float" || var.first == "Double" || var.first == "Int" || var.first == "Long" ||
                   var.first == "Short" || var.first == "Byte") {
          if (var.second == nullptr) throw FrameError("a numeric RelayRLData needs a value");
          x = number(var.second, key);
        } else {
          continue;
        }
        if (key[0] == 'l') {
          lp = x;
          hl = 1;
        } else {
          vv = x;
          hv = 1;
        }
      }
    }
    rc.logp.push_back(lp);
    rc.has_logp.push_back(hl);
    rc.v.push_back(vv);
    rc.has_v.push_back(hv);
  }
}

}  // namespace rrl
