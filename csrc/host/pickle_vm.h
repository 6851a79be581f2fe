// Data-only pickle interpreter for the reference's ZMQ trajectory frames
// (serde_pickle(Vec<RelayRLAction>), trajectory.rs:50-90), generic over the value representation.
//
// The opcode loop lives here, free of Python, so the SAME code runs in two places:
//   * csrc/bindings/pickle_native.cpp instantiates it with Python objects (the server's decoder);
//   * csrc/host/selftest/parser_fuzz.cpp instantiates it with an arena of C++ nodes and drives it
//     with ~10^5 mutated frames under ASan + UBSan (tools/sanitize_host.sh) -- every input a TCP
//     peer can send reaches this loop first.
// Only containers, scalars, strings, bytes and the memo are understood; every opcode that imports
// or calls (GLOBAL, REDUCE, BUILD, INST, OBJ, NEWOBJ, EXT*, PERSID, ...) is an error, so a frame
// can never execute anything.  Limits: MARK nesting 64, 2^20 stack items, 2^16 memo entries.
//
// Builder interface (B::V is a copyable value handle):
//   V none(); V boolean(bool); V small_int(int64_t); V long_bytes(const uint8_t*, size_t);
//   V real(double); V str(const char*, size_t); V bytes(const char*, size_t);
//   V empty_list(bool u8_form);  // u8_form: a byte buffer (serde's Vec<u8>) until proven otherwise
//   V empty_dict(); V empty_tuple(); V empty_set();
//   bool is_bytearray(const V&); void bytearray_append(V&, const char*, size_t);
//   void bytearray_to_list(V&);  bool u8_value(const V&, uint8_t&);
//   bool is_list(const V&); void list_extend(V&, const V*, size_t);
//   bool is_dict(const V&); void dict_set(V&, const V& key, const V& value);
//   bool is_set(const V&); void set_add(V&, const V&);
//   V tuple(const V*, size_t); V frozenset(const V*, size_t);
// Builders throw FrameError (or any std::exception) for values they reject (bad UTF-8, an
// unhashable key).
#pragma once

#include <cstdint>
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

namespace rrl {
namespace pickle {

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
    while (q + 1 < n_ && p_[q] == 0x4B) q += 2;  // scan first: one resize, no per-byte push
    if (q >= n_ || p_[q] != 0x65) return false;
    const size_t k = (q - pos_) / 2, start = out.size();
    out.resize(start + k);
    char* d = &out[0] + start;
    const uint8_t* src = p_ + pos_ + 1;
    for (size_t i = 0; i < k; ++i) d[i] = (char)src[2 * i];
    pos_ = q + 1;
    return true;
  }
  const uint8_t* take(size_t k) {
    if (k > n_ - pos_) throw FrameError("truncated frame");  // (pos_ <= n_ always)
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
  size_t size() const { return n_; }

 private:
  const uint8_t* p_;
  size_t n_;
  size_t pos_ = 0;
};

template <class B>
typename B::V run(const uint8_t* data, size_t n, B& b, bool u8_form) {
  using V = typename B::V;
  Reader r(data, n);
  std::vector<V> stack;
  std::vector<size_t> marks;
  stack.reserve(64);
  marks.reserve(kMaxDepth);
  std::unordered_map<uint32_t, V> memo;
  std::string run;  // scratch of the u8 fast form
  auto above_mark = [&](size_t k) { return !marks.empty() && marks.back() > stack.size() - k; };
  auto pop_value = [&]() {
    if (stack.empty() || above_mark(1)) throw FrameError("stack underflow");
    V v = std::move(stack.back());
    stack.pop_back();
    return v;
  };
  auto pop_mark = [&]() -> size_t {  // index of the first item above the mark
    if (marks.empty()) throw FrameError("MARK not found");
    const size_t m = marks.back();
    marks.pop_back();
    return m;
  };
  auto top = [&]() -> V& {
    if (stack.empty() || above_mark(1)) throw FrameError("stack underflow");
    return stack.back();
  };
  // the container below the items [from, end): no MARK may sit between them
  auto container_below = [&](size_t from) -> V& {
    if (from == 0 || stack.size() < from || (!marks.empty() && marks.back() >= from))
      throw FrameError("stack underflow");
    return stack[from - 1];
  };
  // list APPEND / APPENDS onto the container, with the u8 fast form
  auto extend_top = [&](size_t from) {
    V& tgt = container_below(from);
    if (u8_form && b.is_bytearray(tgt)) {
      run.clear();
      bool all = true;
      for (size_t i = from; i < stack.size() && all; ++i) {
        uint8_t u = 0;
        all = b.u8_value(stack[i], u);
        run.push_back((char)u);
      }
      if (all) {
        b.bytearray_append(tgt, run.data(), stack.size() - from);
        stack.resize(from);
        return;
      }
      b.bytearray_to_list(tgt);  // not a Vec<u8> after all
    }
    if (!b.is_list(tgt)) throw FrameError("expected a list on the stack");
    b.list_extend(tgt, stack.data() + from, stack.size() - from);
    stack.resize(from);
  };
  auto as_list = [&](V& o) {  // a memoised Vec<u8> in the making is kept as a list of ints
    if (u8_form && b.is_bytearray(o)) b.bytearray_to_list(o);
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
      case 0x4E: stack.push_back(b.none()); break;
      case 0x88: stack.push_back(b.boolean(true)); break;
      case 0x89: stack.push_back(b.boolean(false)); break;
      case 0x4B: stack.push_back(b.small_int(r.u8())); break;             // BININT1
      case 0x4D: stack.push_back(b.small_int(r.le<uint16_t>())); break;   // BININT2
      case 0x4A: stack.push_back(b.small_int(r.le<int32_t>())); break;    // BININT
      case 0x8A:                                                          // LONG1
      case 0x8B: {                                                        // LONG4
        const int64_t k = op == 0x8A ? (int64_t)r.u8() : (int64_t)r.le<int32_t>();
        if (k < 0 || k > 64) throw FrameError("LONG4 too large");
        const uint8_t* p = r.take((size_t)k);
        stack.push_back(b.long_bytes(p, (size_t)k));
        break;
      }
      case 0x47: {  // BINFLOAT (big-endian double)
        const uint8_t* p = r.take(8);
        uint64_t u = 0;
        for (int i = 0; i < 8; ++i) u = (u << 8) | p[i];
        double d;
        std::memcpy(&d, &u, 8);
        stack.push_back(b.real(d));
        break;
      }
      case 0x58:    // BINUNICODE
      case 0x8C:    // SHORT_BINUNICODE
      case 0x8D: {  // BINUNICODE8
        const uint64_t k = op == 0x58 ? r.le<uint32_t>() : (op == 0x8C ? r.u8() : r.le<uint64_t>());
        if (k > (uint64_t)n) throw FrameError("truncated frame");
        const char* s = reinterpret_cast<const char*>(r.take((size_t)k));
        stack.push_back(b.str(s, (size_t)k));
        break;
      }
      case 0x42:    // BINBYTES
      case 0x43:    // SHORT_BINBYTES
      case 0x8E: {  // BINBYTES8
        const uint64_t k = op == 0x42 ? r.le<uint32_t>() : (op == 0x43 ? r.u8() : r.le<uint64_t>());
        if (k > (uint64_t)n) throw FrameError("truncated frame");
        const char* s = reinterpret_cast<const char*>(r.take((size_t)k));
        stack.push_back(b.bytes(s, (size_t)k));
        break;
      }
      case 0x28:  // MARK
        // u8 form: a MARK that opens a pure "K b ... APPENDS" run onto a Vec<u8> being built goes
        // straight into the byte buffer, no value per byte (~20,000 of them per CartPole frame)
        if (u8_form && !stack.empty() && (marks.empty() || marks.back() < stack.size()) &&
            b.is_bytearray(stack.back())) {
          run.clear();
          if (r.u8_run(run)) {
            b.bytearray_append(stack.back(), run.data(), run.size());
            break;
          }
        }
        if ((int)marks.size() >= kMaxDepth) throw FrameError("nesting too deep");
        marks.push_back(stack.size());
        break;
      case 0x5D: stack.push_back(b.empty_list(u8_form)); break;  // EMPTY_LIST
      case 0x7D: stack.push_back(b.empty_dict()); break;
      case 0x29: stack.push_back(b.empty_tuple()); break;
      case 0x8F: stack.push_back(b.empty_set()); break;
      case 0x61:  // APPEND
        if (stack.empty() || above_mark(1)) throw FrameError("stack underflow");
        extend_top(stack.size() - 1);
        break;
      case 0x65: extend_top(pop_mark()); break;  // APPENDS
      case 0x73: {                               // SETITEM
        V v = pop_value();
        V k = pop_value();
        V& d = top();
        if (!b.is_dict(d)) throw FrameError("expected a dict on the stack");
        b.dict_set(d, k, v);
        break;
      }
      case 0x75: {  // SETITEMS
        const size_t m = pop_mark();
        if ((stack.size() - m) % 2) throw FrameError("odd SETITEMS");
        V& c = container_below(m);
        if (!b.is_dict(c)) throw FrameError("expected a dict on the stack");
        for (size_t i = m; i < stack.size(); i += 2) b.dict_set(c, stack[i], stack[i + 1]);
        stack.resize(m);
        break;
      }
      case 0x90: {  // ADDITEMS
        const size_t m = pop_mark();
        V& c = container_below(m);
        if (!b.is_set(c)) throw FrameError("expected a set on the stack");
        for (size_t i = m; i < stack.size(); ++i) b.set_add(c, stack[i]);
        stack.resize(m);
        break;
      }
      case 0x91: {  // FROZENSET
        const size_t m = pop_mark();
        V f = b.frozenset(stack.data() + m, stack.size() - m);
        stack.resize(m);
        stack.push_back(std::move(f));
        break;
      }
      case 0x74: {  // TUPLE
        const size_t m = pop_mark();
        V t = b.tuple(stack.data() + m, stack.size() - m);
        stack.resize(m);
        stack.push_back(std::move(t));
        break;
      }
      case 0x85:
      case 0x86:
      case 0x87: {  // TUPLE1..3
        const size_t k = op - 0x84;
        if (stack.size() < k || above_mark(k)) throw FrameError("stack underflow");
        V t = b.tuple(stack.data() + stack.size() - k, k);
        stack.resize(stack.size() - k);
        stack.push_back(std::move(t));
        break;
      }
      // (serde_pickle writes no memo; a memoised list is built as a list, not in the u8 form)
      case 0x71: {  // BINPUT
        const uint32_t k = r.u8();
        as_list(top());
        memo[k] = top();
        break;
      }
      case 0x72: {  // LONG_BINPUT
        const uint32_t k = r.le<uint32_t>();
        as_list(top());
        memo[k] = top();
        break;
      }
      case 0x94: {  // MEMOIZE
        as_list(top());
        const uint32_t k = (uint32_t)memo.size();
        memo[k] = top();
        break;
      }
      case 0x68:    // BINGET
      case 0x6A: {  // LONG_BINGET
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

}  // namespace pickle
}  // namespace rrl
