// Mutation fuzzer for the network-facing parsers, built WITHOUT Python under ASan + UBSan
// (tools/sanitize_host.sh fuzz, tests/test_sanitizers.py):
//
//   * rrl::pickle::run (csrc/host/pickle_vm.h) -- the opcode loop every reference ZMQ upload
//     reaches first (the server's decoder instantiates the same template over Python objects);
//   * rrl::st_tensor_f32 (csrc/host/st_tensor.h) -- every TensorData payload inside those frames;
//   * rrl::reference_columns_tree (csrc/host/ref_columns.h) -- the server's frame -> columns decoder;
//   * rrl::st_decode / st_header (csrc/host/codec.cpp) -- the gRPC path's safetensors tensors;
//   * rrl::traj_decode (csrc/host/codec.cpp) -- this framework's own RRLT frames, which any peer
//     of the trajectory PULL / the gRPC SendFrame route can send (seeds encoded here).
//
// usage: parser_fuzz ITERATIONS SEED_FILE...   (seeds: real reference frames and safetensors
// files written by the test from transport/serde_pickle.reference_frame).  Each iteration takes
// a seed (or a previous mutant), applies 1-4 mutations -- truncation, byte flips, 4/8-byte length
// fields set to 0xFFFFFFFF / 2^31 / 2^63 / 2^64-1, deep MARK runs, memo misuse (unknown keys,
// self-appending lists), splices, safetensors header numbers made negative / huge -- and runs
// every parser on it.  Rejections are expected; any memory error or UB aborts the process.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <memory>
#include <sstream>
#include <string>
#include <unordered_set>
#include <vector>

#include "codec.h"
#include "pickle_tree.h"
#include "pickle_vm.h"
#include "ref_columns.h"
#include "st_tensor.h"

namespace {

using rrl::pickle::FrameError;
using rrl::pickle::Node;
using rrl::pickle::NodeBuilder;

struct Stats {
  uint64_t runs = 0, accepted = 0, rejected = 0, tensors = 0, tensors_ok = 0, st_ok = 0, st_bad = 0, columns_ok = 0,
           rrlt_ok = 0, rrlt_bad = 0;
};

// valid RRLT frames: episodes with obs / act / mask tensors of several dtypes, tensor and scalar
// aux values, a terminal marker without tensors
std::vector<std::string> rrlt_seeds() {
  std::vector<std::string> out;
  for (int variant = 0; variant < 3; ++variant) {
    rrl::Trajectory t;
    t.server = variant ? "tcp://127.0.0.1:7776" : "";
    t.agent_id = "fuzz-" + std::to_string(variant);
    t.seq = 7 + variant;
    for (int i = 0; i < 3 + 4 * variant; ++i) {
      rrl::Action a;
      a.has_obs = a.has_act = true;
      a.obs.dtype = variant == 2 ? rrl::DType::Double : rrl::DType::Float;
      a.obs.shape = {4};
      a.obs.raw.assign(4 * rrl::dtype_size(a.obs.dtype), (char)(i + 1));
      a.act.dtype = variant == 1 ? rrl::DType::Long : rrl::DType::Int;
      a.act.shape = {1};
      a.act.raw.assign(rrl::dtype_size(a.act.dtype), (char)(i & 1));
      a.has_mask = variant != 1;
      if (a.has_mask) {
        a.mask.dtype = rrl::DType::Float;
        a.mask.shape = {2};
        a.mask.raw.assign(8, '\0');
      }
      a.rew = 0.5f * i;
      a.has_data = true;
      rrl::AuxValue lp;
      lp.kind = rrl::AuxValue::TENSOR;
      lp.tensor.dtype = rrl::DType::Float;
      lp.tensor.shape = {1};
      lp.tensor.raw.assign(4, '\x3f');
      a.data["logp_a"] = lp;
      rrl::AuxValue sv;
      sv.kind = variant == 0 ? rrl::AuxValue::STRING : rrl::AuxValue::DOUBLE;
      sv.s = "note";
      sv.d = 1.5;
      a.data["extra"] = sv;
      t.actions.push_back(a);
    }
    rrl::Action m;  // the terminal marker
    m.done = true;
    m.rew = 1.f;
    t.actions.push_back(m);
    out.push_back(rrl::traj_encode(t));
  }
  return out;
}

// every TensorData-like {.., "data": bytes} below the root goes through the column reader
void walk(Node* n, rrl::StHeaderCache& hc, std::unordered_set<Node*>& seen, Stats& st, int depth) {
  if (!n || depth > 200 || !seen.insert(n).second) return;
  if (n->k == Node::Dict) {
    for (size_t i = 0; i + 1 < n->items.size(); i += 2) {
      Node* key = n->items[i];
      Node* val = n->items[i + 1];
      if (key->k == Node::Str && key->s == "data" && (val->k == Node::Bytes || val->k == Node::ByteArr)) {
        std::vector<float> out;
        ++st.tensors;
        try {
          rrl::st_tensor_f32(val->s.data(), val->s.size(), out, hc);
          ++st.tensors_ok;
          volatile float sink = 0;
          for (float x : out) sink = sink + x;  // touch every value read
        } catch (const std::exception&) {
        }
      }
    }
  }
  for (Node* c : n->items) walk(c, hc, seen, st, depth + 1);
}

struct Rng {
  uint64_t s;
  uint64_t next() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
  }
  size_t below(size_t n) { return n ? (size_t)(next() % n) : 0; }
};

void put_le(std::string& b, size_t at, uint64_t v, int bytes) {
  for (int i = 0; i < bytes && at + i < b.size(); ++i) b[at + i] = (char)((v >> (8 * i)) & 0xFF);
}

std::string mutate(std::string b, const std::vector<std::string>& seeds, Rng& r) {
  static const uint64_t kHuge[] = {0xFFFFFFFFull, 0x7FFFFFFFull, 0x80000000ull, 1ull << 63, ~0ull, 0xFFFFull, 65536};
  static const char* kNums[] = {"-160", "-1", "9223372036854775807", "4611686018427387904", "99999999999999999999",
                                "-9223372036854775808", "0", "2305843009213693952"};
  using namespace std::string_literals;
  static const std::string kSnippets[] = {"]q\x00h\x00" "a"s, "h\x07"s, "j\xff\xff\xff\x7f"s,
                                          std::string(17, '('), "\x8b\xff\xff\xff\x7f"s,
                                          "\x8d\xff\xff\xff\xff\xff\xff\xff\x7f"s,
                                          "\x8e\x00\x00\x00\x00\x00\x00\x00\x80"s, "X\xff\xff\xff\xff"s, "0000"s,
                                          "\x94\x94\x94"s, "}(K\x01]u"s, "\x8f(]\x90"s, "t\x85\x86\x87"s, "1e1e"s,
                                          "]\x94(K\x01h\x00" "e"s};
  const int n_mut = 1 + (int)r.below(4);
  for (int m = 0; m < n_mut; ++m) {
    if (b.empty()) b = seeds[r.below(seeds.size())];
    switch (r.below(9)) {
      case 0:  // truncate
        b.resize(r.below(b.size() + 1));
        break;
      case 1:  // flip bytes
        for (int k = 0, e = 1 + (int)r.below(8); k < e && !b.empty(); ++k) b[r.below(b.size())] ^= (char)(1 + r.below(255));
        break;
      case 2: {  // a length field to a huge value
        if (b.size() < 9) break;
        const int w = r.below(2) ? 4 : 8;
        put_le(b, r.below(b.size() - w), kHuge[r.below(sizeof(kHuge) / sizeof(kHuge[0]))], w);
        break;
      }
      case 3: {  // deep MARK nesting
        const size_t at = r.below(b.size() + 1);
        b.insert(at, std::string(1 + r.below(300), '('));
        break;
      }
      case 4: {  // memo / container misuse snippets
        b.insert(r.below(b.size() + 1), kSnippets[r.below(sizeof(kSnippets) / sizeof(kSnippets[0]))]);
        break;
      }
      case 5: {  // splice another seed's tail in
        const std::string& o = seeds[r.below(seeds.size())];
        const size_t cut = r.below(b.size() + 1), from = r.below(o.size() + 1);
        b = b.substr(0, cut) + o.substr(from, r.below(4096));
        break;
      }
      case 6: {  // safetensors header numbers: negative / huge / overflowing
        std::vector<size_t> digits;
        for (size_t i = 0; i < b.size(); ++i)
          if (b[i] >= '0' && b[i] <= '9' && (i == 0 || b[i - 1] < '0' || b[i - 1] > '9')) digits.push_back(i);
        if (digits.empty()) break;
        size_t at = digits[r.below(digits.size())], end = at;
        while (end < b.size() && b[end] >= '0' && b[end] <= '9') ++end;
        const std::string num = kNums[r.below(sizeof(kNums) / sizeof(kNums[0]))];
        b = b.substr(0, at) + num + b.substr(end);
        break;
      }
      case 7: {  // an embedded safetensors header length (first 8 bytes of a payload)
        if (b.size() < 16) break;
        put_le(b, r.below(b.size() - 8), kHuge[r.below(sizeof(kHuge) / sizeof(kHuge[0]))], 8);
        break;
      }
      default: {  // duplicate a random span (many more items / deeper containers)
        if (b.empty() || b.size() > 60000) break;
        const size_t a = r.below(b.size()), len = 1 + r.below(std::min<size_t>(512, b.size() - a));
        b.insert(r.below(b.size() + 1), b.substr(a, len));
        break;
      }
    }
  }
  if (b.size() > 65536) b.resize(65536);
  return b;
}

// a safetensors payload whose header numbers are replaced, with its 8-byte header length fixed
// up (so the hostile numbers reach st_header instead of failing the length check)
std::string hostile_tensor(const std::string& st_seed, Rng& r) {
  static const char* kNums[] = {"-160", "-8", "-1", "9223372036854775807", "4611686018427387904",
                                "99999999999999999999", "-9223372036854775808", "0", "2305843009213693952", "16",
                                "24", "4294967296"};
  if (st_seed.size() < 8) return st_seed;
  uint64_t hl = 0;
  for (int i = 0; i < 8; ++i) hl |= (uint64_t)(uint8_t)st_seed[i] << (8 * i);
  if (hl > st_seed.size() - 8) return st_seed;
  std::string hdr = st_seed.substr(8, (size_t)hl), data = st_seed.substr(8 + (size_t)hl);
  for (int m = 0, e = 1 + (int)r.below(3); m < e; ++m) {
    std::vector<size_t> digits;
    for (size_t i = 0; i < hdr.size(); ++i)
      if (hdr[i] >= '0' && hdr[i] <= '9' && (i == 0 || hdr[i - 1] < '0' || hdr[i - 1] > '9')) digits.push_back(i);
    if (digits.empty()) break;
    size_t at = digits[r.below(digits.size())], end = at;
    while (end < hdr.size() && hdr[end] >= '0' && hdr[end] <= '9') ++end;
    hdr = hdr.substr(0, at) + kNums[r.below(sizeof(kNums) / sizeof(kNums[0]))] + hdr.substr(end);
  }
  if (r.below(4) == 0) data.resize(r.below(data.size() + 1));
  std::string out(8, '\0');
  put_le(out, 0, hdr.size(), 8);
  return out + hdr + data;
}

// [{"obs": {"data": <payload>}, "rew": 1.0}, ...] as a serde-style frame, the payload either as a
// bytes object or as serde's Vec<u8> (K b ... APPENDS chunks of 1000): frames the VM ACCEPTS, so
// the hostile payload reaches the tensor reader
std::string wrap_frame(const std::vector<std::string>& payloads, bool u8_list) {
  using namespace std::string_literals;  // (the literals hold NUL bytes)
  std::string f = "\x80\x03]("s;
  for (const auto& p : payloads) {
    f += "}(X\x03\x00\x00\x00obs}(X\x04\x00\x00\x00" "data"s;
    if (u8_list) {
      f += "]";
      for (size_t i = 0; i < p.size(); i += 1000) {
        f += "(";
        for (size_t j = i; j < p.size() && j < i + 1000; ++j) {
          f += "K";
          f.push_back(p[j]);
        }
        f += "e";
      }
    } else {
      f += "B";
      std::string len(4, '\0');
      put_le(len, 0, p.size(), 4);
      f += len + p;
    }
    f += "uX\x03\x00\x00\x00rewG?\xf0\x00\x00\x00\x00\x00\x00u"s;
  }
  f += "e.";
  return f;
}

void run_all(const std::string& in, Stats& st) {
  for (int u8 = 0; u8 < 2; ++u8) {
    NodeBuilder b;
    ++st.runs;
    try {
      Node* root = rrl::pickle::run(reinterpret_cast<const uint8_t*>(in.data()), in.size(), b, u8 == 1);
      ++st.accepted;
      rrl::StHeaderCache hc;
      std::unordered_set<Node*> seen;
      walk(root, hc, seen, st, 0);
    } catch (const std::exception&) {
      ++st.rejected;
    }
  }
  // the server's column decoder (ref_columns.h, the GIL-free path every reference upload takes)
  try {
    rrl::RefColumns rc;
    rrl::reference_columns_tree(reinterpret_cast<const uint8_t*>(in.data()), in.size(), rc);
    ++st.columns_ok;
  } catch (const std::exception&) {
  }
  // the same bytes as a safetensors file (gRPC path) and as a bare TensorData payload
  try {
    const rrl::Tensor t = rrl::st_decode(in, "tensor");
    volatile size_t sink = t.raw.size();
    (void)sink;
    ++st.st_ok;
  } catch (const std::exception&) {
    ++st.st_bad;
  }
  try {
    rrl::StHeaderCache hc;
    std::vector<float> out;
    rrl::st_tensor_f32(in.data(), in.size(), out, hc);
  } catch (const std::exception&) {
  }
  // and as this framework's RRLT frame (traj_decode), touching every decoded byte
  try {
    const rrl::Trajectory t = rrl::traj_decode(in);
    size_t sink = t.agent_id.size() + t.server.size();
    for (const auto& a : t.actions) {
      sink += a.obs.raw.size() + a.act.raw.size() + a.mask.raw.size();
      for (const auto& kv : a.data) sink += kv.first.size() + kv.second.tensor.raw.size() + kv.second.s.size();
    }
    volatile size_t v = sink;
    (void)v;
    ++st.rrlt_ok;
  } catch (const std::exception&) {
    ++st.rrlt_bad;
  }
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s ITERATIONS SEED_FILE...\n", argv[0]);
    return 2;
  }
  const long iters = std::atol(argv[1]);
  std::vector<std::string> seeds;
  for (int i = 2; i < argc; ++i) {
    std::ifstream f(argv[i], std::ios::binary);
    std::stringstream ss;
    ss << f.rdbuf();
    if (!ss.str().empty()) seeds.push_back(ss.str());
  }
  if (seeds.empty()) {
    std::fprintf(stderr, "no seeds\n");
    return 2;
  }
  const std::vector<std::string> rrlt = rrlt_seeds();
  seeds.insert(seeds.end(), rrlt.begin(), rrlt.end());
  for (const auto& f : rrlt) rrl::traj_decode(f);  // the encoder's own frames must decode
  std::vector<std::string> st_seeds;  // safetensors files among the seeds (header length + '{')
  for (const auto& s : seeds)
    if (s.size() > 9 && s[8] == '{') st_seeds.push_back(s);
  Stats st;
  for (const auto& s : seeds) run_all(s, st);  // every seed as is must decode
  const uint64_t seed_ok = st.accepted;
  Rng r{0x9E3779B97F4A7C15ull};
  std::string cur;
  for (long it = 0; it < iters; ++it) {
    // mostly fresh mutants of a seed, sometimes a mutant of the previous mutant (deeper damage)
    if (it % 3 == 2 && !st_seeds.empty()) {  // structure-aware: hostile tensors inside valid frames
      std::vector<std::string> ps;
      for (int k = 0, e = 1 + (int)r.below(3); k < e; ++k) ps.push_back(hostile_tensor(st_seeds[r.below(st_seeds.size())], r));
      const std::string f = wrap_frame(ps, r.below(2) == 0);
      run_all(f, st);
      run_all(ps[0], st);
      continue;
    }
    const std::string& base = (it % 4 == 3 && !cur.empty()) ? cur : seeds[r.below(seeds.size())];
    cur = mutate(base, seeds, r);
    run_all(cur, st);
  }
  std::printf("parser fuzz OK: %ld inputs, %llu VM runs (%llu accepted, %llu rejected), %llu tensors read "
              "(%llu valid), st_decode %llu ok / %llu rejected, column frames %llu, RRLT %llu ok / %llu rejected, "
              "seeds decoded %llu\n",
              iters, (unsigned long long)st.runs, (unsigned long long)st.accepted, (unsigned long long)st.rejected,
              (unsigned long long)st.tensors, (unsigned long long)st.tensors_ok, (unsigned long long)st.st_ok,
              (unsigned long long)st.st_bad, (unsigned long long)st.columns_ok, (unsigned long long)st.rrlt_ok,
              (unsigned long long)st.rrlt_bad, (unsigned long long)seed_ok);
  return 0;
}
