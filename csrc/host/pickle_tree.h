// A pickle frame as a C++ value tree: rrl::pickle::run (pickle_vm.h) instantiated over arena
// nodes, no Python.  Used by the server's reference-frame column decoder with the GIL released
// (ref_columns.h -> bindings/pickle_native.cpp) and by the sanitizer fuzz harness
// (selftest/parser_fuzz.cpp).  Nodes live in the builder's arena: a memo can make a list
// contain itself, so nothing is reference-counted and nothing leaks.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "pickle_vm.h"

namespace rrl {
namespace pickle {

struct Node {
  enum Kind { None, Bool, Int, Big, Float, Str, Bytes, ByteArr, List, Dict, Tuple, Set, Frozen } k = None;
  int64_t i = 0;
  double f = 0;
  std::string s;             // Str / Bytes / ByteArr / Big payload
  std::vector<Node*> items;  // List / Tuple / Set / Frozen; Dict: key, value, key, value, ...
};

inline bool valid_utf8(const char* s, size_t n) {
  size_t i = 0;
  while (i < n) {
    const uint8_t c = (uint8_t)s[i];
    size_t k;
    if (c < 0x80) k = 0;
    else if ((c >> 5) == 6) k = 1;
    else if ((c >> 4) == 14) k = 2;
    else if ((c >> 3) == 30) k = 3;
    else return false;
    if (k > n - i - 1) return false;
    for (size_t j = 1; j <= k; ++j)
      if (((uint8_t)s[i + j] >> 6) != 2) return false;
    i += k + 1;
  }
  return true;
}

// values are arena nodes: a memo can make a list contain itself, so nothing is reference-counted
struct NodeBuilder {
  using V = Node*;
  // nodes are carved from blocks of kBlock (one allocation per 256 values, not one per value)
  static constexpr size_t kBlock = 256;
  std::vector<std::unique_ptr<Node[]>> blocks;
  size_t used = kBlock;
  size_t count = 0;
  Node* make(Node::Kind k) {
    if (used == kBlock) {
      blocks.emplace_back(new Node[kBlock]);
      used = 0;
    }
    Node* n = &blocks.back()[used++];
    n->k = k;
    ++count;
    return n;
  }
  V none() { return make(Node::None); }
  V boolean(bool v) {
    Node* n = make(Node::Bool);
    n->i = v;
    return n;
  }
  V small_int(int64_t v) {
    Node* n = make(Node::Int);
    n->i = v;
    return n;
  }
  V long_bytes(const uint8_t* p, size_t k) {
    Node* n = make(Node::Big);
    n->s.assign(reinterpret_cast<const char*>(p), k);
    return n;
  }
  V real(double d) {
    Node* n = make(Node::Float);
    n->f = d;
    return n;
  }
  V str(const char* s, size_t k) {
    if (!valid_utf8(s, k)) throw FrameError("invalid UTF-8");
    Node* n = make(Node::Str);
    n->s.assign(s, k);
    return n;
  }
  V bytes(const char* s, size_t k) {
    Node* n = make(Node::Bytes);
    n->s.assign(s, k);
    return n;
  }
  V empty_list(bool u8) { return make(u8 ? Node::ByteArr : Node::List); }
  V empty_dict() { return make(Node::Dict); }
  V empty_tuple() { return make(Node::Tuple); }
  V empty_set() { return make(Node::Set); }
  bool is_bytearray(const V& o) { return o->k == Node::ByteArr; }
  void bytearray_append(V& o, const char* s, size_t k) { o->s.append(s, k); }
  void bytearray_to_list(V& o) {
    for (unsigned char c : o->s) o->items.push_back(small_int(c));
    o->s.clear();
    o->k = Node::List;
  }
  bool u8_value(const V& o, uint8_t& out) {
    if (o->k != Node::Int || o->i < 0 || o->i > 255) return false;
    out = (uint8_t)o->i;
    return true;
  }
  bool is_list(const V& o) { return o->k == Node::List; }
  void list_extend(V& o, const V* items, size_t k) {
    o->items.reserve(o->items.size() + k);
    o->items.insert(o->items.end(), items, items + k);
  }
  bool is_dict(const V& o) { return o->k == Node::Dict; }
  static void hashable(const V& k) {
    if (k->k == Node::List || k->k == Node::Dict || k->k == Node::Set || k->k == Node::ByteArr)
      throw FrameError("unhashable key");
  }
  void dict_set(V& d, const V& k, const V& v) {
    hashable(k);
    if (d->items.capacity() == 0) d->items.reserve(8);  // RelayRLAction / TensorData dicts: <= 4 keys
    d->items.push_back(k);
    d->items.push_back(v);
  }
  bool is_set(const V& o) { return o->k == Node::Set; }
  void set_add(V& s, const V& k) {
    hashable(k);
    s->items.push_back(k);
  }
  V tuple(const V* items, size_t k) {
    Node* n = make(Node::Tuple);
    n->items.assign(items, items + k);
    return n;
  }
  V frozenset(const V* items, size_t k) {
    Node* n = make(Node::Frozen);
    for (size_t i = 0; i < k; ++i) hashable(items[i]);
    n->items.assign(items, items + k);
    return n;
  }
};

}  // namespace pickle
}  // namespace rrl
