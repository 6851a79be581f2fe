#include "codec.h"

#include <cstdint>
#include <cstring>
#include <sstream>

namespace rrl {

static const char* kNames[] = {"Byte", "Short", "Int", "Long", "Float", "Double", "Bool"};
static const char* kTags[] = {"U8", "I16", "I32", "I64", "F32", "F64", "U8"};
static const size_t kSizes[] = {1, 2, 4, 8, 4, 8, 1};

const char* dtype_name(DType d) { return kNames[(int)d]; }
const char* dtype_st_tag(DType d) { return kTags[(int)d]; }
size_t dtype_size(DType d) { return kSizes[(int)d]; }

DType dtype_from_name(const std::string& s) {
  for (int i = 0; i < 7; ++i)
    if (s == kNames[i]) return (DType)i;
  throw std::invalid_argument("unsupported dtype name: " + s);
}

DType dtype_from_st_tag(const std::string& s) {
  if (s == "BOOL") return DType::Bool;
  for (int i = 0; i < 6; ++i)
    if (s == kTags[i]) return (DType)i;
  throw std::invalid_argument("unsupported safetensors dtype: " + s);
}

// --------------------------------------------------------------------- safetensors
std::string st_encode(const Tensor& t, const std::string& name) {
  const size_t nbytes = t.raw.size();
  if ((int64_t)nbytes != t.numel() * (int64_t)dtype_size(t.dtype))
    throw std::invalid_argument("st_encode: byte size does not match shape/dtype");
  std::ostringstream h;
  h << "{\"" << name << "\":{\"dtype\":\"" << dtype_st_tag(t.dtype) << "\",\"shape\":[";
  for (size_t i = 0; i < t.shape.size(); ++i) h << (i ? "," : "") << t.shape[i];
  h << "],\"data_offsets\":[0," << nbytes << "]}}";
  std::string header = h.str();
  while (header.size() % 8 != 0) header.push_back(' ');
  std::string out;
  out.resize(8 + header.size() + nbytes);
  uint64_t hl = header.size();
  for (int i = 0; i < 8; ++i) out[i] = (char)((hl >> (8 * i)) & 0xFF);
  memcpy(&out[8], header.data(), header.size());
  if (nbytes) memcpy(&out[8 + header.size()], t.raw.data(), nbytes);
  return out;
}

// Minimal JSON scanning for the safetensors header (flat, known structure).
static size_t skip_ws(const std::string& s, size_t i) {
  while (i < s.size() && (s[i] == ' ' || s[i] == '\n' || s[i] == '\t' || s[i] == '\r')) ++i;
  return i;
}
static std::string parse_string(const std::string& s, size_t& i) {
  i = skip_ws(s, i);
  if (i >= s.size() || s[i] != '"') throw std::runtime_error("safetensors header: expected string");
  ++i;
  std::string out;
  while (i < s.size() && s[i] != '"') {
    if (s[i] == '\\' && i + 1 < s.size()) ++i;
    out.push_back(s[i++]);
  }
  ++i;
  return out;
}
static int64_t parse_int(const std::string& s, size_t& i) {
  i = skip_ws(s, i);
  size_t j = i;
  if (j < s.size() && s[j] == '-') ++j;
  while (j < s.size() && isdigit((unsigned char)s[j])) ++j;
  if (j == i) throw std::runtime_error("safetensors header: expected integer");
  int64_t v = std::stoll(s.substr(i, j - i));
  i = j;
  return v;
}
static void expect(const std::string& s, size_t& i, char c) {
  i = skip_ws(s, i);
  if (i >= s.size() || s[i] != c) throw std::runtime_error(std::string("safetensors header: expected '") + c + "'");
  ++i;
}
static void skip_value(const std::string& s, size_t& i) {
  i = skip_ws(s, i);
  if (s[i] == '"') {
    parse_string(s, i);
    return;
  }
  if (s[i] == '{' || s[i] == '[') {
    int depth = 0;
    bool instr = false;
    for (; i < s.size(); ++i) {
      char c = s[i];
      if (instr) {
        if (c == '\\') ++i;
        else if (c == '"') instr = false;
        continue;
      }
      if (c == '"') instr = true;
      else if (c == '{' || c == '[') ++depth;
      else if (c == '}' || c == ']') {
        if (--depth == 0) {
          ++i;
          return;
        }
      }
    }
    return;
  }
  while (i < s.size() && s[i] != ',' && s[i] != '}' && s[i] != ']') ++i;
}

StHeader st_header(const char* header_json, size_t len, const std::string& name) {
  const std::string h(header_json, len);
  size_t i = 0;
  expect(h, i, '{');
  bool found = false;
  StHeader t;
  while (true) {
    i = skip_ws(h, i);
    if (i >= h.size()) throw std::runtime_error("safetensors header: unterminated");
    if (h[i] == '}') break;
    std::string key = parse_string(h, i);
    expect(h, i, ':');
    if (key == name) {
      found = true;
      expect(h, i, '{');
      while (true) {
        i = skip_ws(h, i);
        if (i >= h.size()) throw std::runtime_error("safetensors header: unterminated");
        if (h[i] == '}') {
          ++i;
          break;
        }
        std::string k = parse_string(h, i);
        expect(h, i, ':');
        if (k == "dtype") {
          t.dtype = dtype_from_st_tag(parse_string(h, i));
        } else if (k == "shape") {
          expect(h, i, '[');
          i = skip_ws(h, i);
          while (i < h.size() && h[i] != ']') {
            t.shape.push_back(parse_int(h, i));
            i = skip_ws(h, i);
            if (i < h.size() && h[i] == ',') ++i;
            i = skip_ws(h, i);
          }
          ++i;
        } else if (k == "data_offsets") {
          expect(h, i, '[');
          t.off0 = parse_int(h, i);
          expect(h, i, ',');
          t.off1 = parse_int(h, i);
          expect(h, i, ']');
        } else {
          skip_value(h, i);
        }
        i = skip_ws(h, i);
        if (i < h.size() && h[i] == ',') ++i;
      }
    } else {
      skip_value(h, i);
    }
    i = skip_ws(h, i);
    if (i < h.size() && h[i] == ',') ++i;
  }
  if (!found) throw std::runtime_error("safetensors: tensor '" + name + "' not found");
  // untrusted input (any ZMQ / gRPC peer): offsets must be a non-negative ordered range and the
  // element count must not overflow -- callers then only have to check off1 against the buffer
  if (t.off0 < 0 || t.off1 < t.off0) throw std::runtime_error("safetensors: bad data offsets");
  const int64_t esz = (int64_t)dtype_size(t.dtype);
  int64_t n = 1;
  for (auto d : t.shape) {
    if (d < 0) throw std::runtime_error("safetensors: negative shape dimension");
    if (d != 0 && n > (INT64_MAX / esz) / d) throw std::runtime_error("safetensors: shape overflows");
    n *= d;
  }
  if (t.off1 - t.off0 != n * esz) throw std::runtime_error("safetensors: data size does not match shape");
  return t;
}

Tensor st_decode(const std::string& file, const std::string& name) {
  if (file.size() < 8) throw std::runtime_error("safetensors: file too short");
  uint64_t hl = 0;
  for (int i = 0; i < 8; ++i) hl |= (uint64_t)(uint8_t)file[i] << (8 * i);
  if (hl > file.size() - 8) throw std::runtime_error("safetensors: header length out of range");
  const StHeader sh = st_header(file.data() + 8, (size_t)hl, name);
  const size_t base = 8 + hl;
  if ((uint64_t)sh.off1 > file.size() - base) throw std::runtime_error("safetensors: bad data offsets");
  Tensor t;
  t.dtype = sh.dtype;
  t.shape = sh.shape;
  t.raw = file.substr(base + sh.off0, sh.off1 - sh.off0);
  return t;
}

// --------------------------------------------------------------------- RRLT frames
namespace {
struct W {
  std::string b;
  void u8(uint8_t v) { b.push_back((char)v); }
  void u32(uint32_t v) { b.append((const char*)&v, 4); }
  void u64(uint64_t v) { b.append((const char*)&v, 8); }
  void i64(int64_t v) { b.append((const char*)&v, 8); }
  void f32(float v) { b.append((const char*)&v, 4); }
  void f64(double v) { b.append((const char*)&v, 8); }
  void str(const std::string& s) {
    u32((uint32_t)s.size());
    b.append(s);
  }
  void tensor(const Tensor& t) {
    u8((uint8_t)t.dtype);
    u8((uint8_t)t.shape.size());
    for (auto s : t.shape) i64(s);
    u64(t.raw.size());
    b.append(t.raw);
  }
};
struct R {
  const std::string& b;
  size_t i = 0;
  explicit R(const std::string& s) : b(s) {}
  void need(uint64_t n) {  // n may be any 64-bit length field: compared against what is left
    if (n > b.size() - i) throw std::runtime_error("RRLT: truncated frame");
  }
  uint8_t u8() {
    need(1);
    return (uint8_t)b[i++];
  }
  template <class T>
  T pod() {
    need(sizeof(T));
    T v;
    memcpy(&v, b.data() + i, sizeof(T));
    i += sizeof(T);
    return v;
  }
  std::string str() {
    uint32_t n = pod<uint32_t>();
    need(n);
    std::string s = b.substr(i, n);
    i += n;
    return s;
  }
  Tensor tensor() {
    Tensor t;
    uint8_t dt = u8();
    if (dt > 6) throw std::runtime_error("RRLT: bad dtype");
    t.dtype = (DType)dt;
    uint8_t nd = u8();
    for (int k = 0; k < nd; ++k) t.shape.push_back(pod<int64_t>());
    uint64_t n = pod<uint64_t>();
    need(n);
    t.raw = b.substr(i, n);
    i += n;
    // the element count from the (untrusted) shape without overflow: every dim >= 0 and the
    // product bounded by the bytes actually present
    const uint64_t es = dtype_size(t.dtype), cap = t.raw.size() / es;
    uint64_t cnt = 1;
    bool zero = false;
    for (int64_t d : t.shape) {
      if (d < 0) throw std::runtime_error("RRLT: negative dimension");
      if (d == 0) {
        zero = true;
      } else if (!zero) {
        if ((uint64_t)d > cap / cnt) throw std::runtime_error("RRLT: tensor size mismatch");
        cnt *= (uint64_t)d;
      }
    }
    if (zero) cnt = 0;
    if (cnt * es != t.raw.size()) throw std::runtime_error("RRLT: tensor size mismatch");
    return t;
  }
};
constexpr uint32_t kMagic = 0x544C5252u;  // "RRLT"
constexpr uint32_t kVersion = 1;
}  // namespace

std::string traj_encode(const Trajectory& t) {
  W w;
  w.u32(kMagic);
  w.u32(kVersion);
  w.str(t.server);
  w.u32(t.max_length);
  w.str(t.agent_id);
  w.u64(t.seq);
  w.u32((uint32_t)t.actions.size());
  for (const Action& a : t.actions) {
    uint8_t flags = (a.has_obs ? 1 : 0) | (a.has_act ? 2 : 0) | (a.has_mask ? 4 : 0) | (a.has_data ? 8 : 0) |
                    (a.done ? 16 : 0) | (a.reward_updated ? 32 : 0);
    w.u8(flags);
    w.f32(a.rew);
    if (a.has_obs) w.tensor(a.obs);
    if (a.has_act) w.tensor(a.act);
    if (a.has_mask) w.tensor(a.mask);
    if (a.has_data) {
      w.u32((uint32_t)a.data.size());
      for (const auto& kv : a.data) {
        w.str(kv.first);
        const AuxValue& v = kv.second;
        w.u8((uint8_t)v.kind);
        switch (v.kind) {
          case AuxValue::TENSOR: w.tensor(v.tensor); break;
          case AuxValue::BYTE: case AuxValue::SHORT: case AuxValue::INT: case AuxValue::LONG: w.i64(v.i); break;
          case AuxValue::FLOAT: case AuxValue::DOUBLE: w.f64(v.d); break;
          case AuxValue::STRING: w.str(v.s); break;
          case AuxValue::BOOL: w.u8(v.b ? 1 : 0); break;
        }
      }
    }
  }
  return w.b;
}

Trajectory traj_decode(const std::string& buf) {
  R r(buf);
  if (r.pod<uint32_t>() != kMagic) throw std::runtime_error("RRLT: bad magic");
  if (r.pod<uint32_t>() != kVersion) throw std::runtime_error("RRLT: unsupported version");
  Trajectory t;
  t.server = r.str();
  t.max_length = r.pod<uint32_t>();
  t.agent_id = r.str();
  t.seq = r.pod<uint64_t>();
  uint32_t n = r.pod<uint32_t>();
  // every action takes at least 5 bytes (flags + reward): a count the frame cannot hold is refused
  // before anything is allocated for it (a 24-byte frame claiming 2^28 actions used to reserve
  // ~100 GB of Action records)
  if (n > (buf.size() - r.i) / 5) throw std::runtime_error("RRLT: action count exceeds the frame");
  t.actions.resize(n);
  for (uint32_t k = 0; k < n; ++k) {
    Action& a = t.actions[k];
    uint8_t f = r.u8();
    a.has_obs = f & 1;
    a.has_act = f & 2;
    a.has_mask = f & 4;
    a.has_data = f & 8;
    a.done = f & 16;
    a.reward_updated = f & 32;
    a.rew = r.pod<float>();
    if (a.has_obs) a.obs = r.tensor();
    if (a.has_act) a.act = r.tensor();
    if (a.has_mask) a.mask = r.tensor();
    if (a.has_data) {
      uint32_t m = r.pod<uint32_t>();
      for (uint32_t q = 0; q < m; ++q) {
        std::string key = r.str();
        AuxValue v;
        uint8_t kind = r.u8();
        if (kind > AuxValue::BOOL) throw std::runtime_error("RRLT: bad aux kind");
        v.kind = (AuxValue::Kind)kind;
        switch (v.kind) {
          case AuxValue::TENSOR: v.tensor = r.tensor(); break;
          case AuxValue::BYTE: case AuxValue::SHORT: case AuxValue::INT: case AuxValue::LONG: v.i = r.pod<int64_t>(); break;
          case AuxValue::FLOAT: case AuxValue::DOUBLE: v.d = r.pod<double>(); break;
          case AuxValue::STRING: v.s = r.str(); break;
          case AuxValue::BOOL: v.b = r.u8() != 0; break;
        }
        a.data.emplace(std::move(key), std::move(v));
      }
    }
  }
  if (r.i != buf.size()) throw std::runtime_error("RRLT: trailing bytes");
  return t;
}

}  // namespace rrl
