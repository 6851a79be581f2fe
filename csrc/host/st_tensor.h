// One TensorData payload (a one-tensor safetensors file: 8-byte header length, JSON header,
// data) -> float32 values, for the reference-frame column decoder.  Pure C++ so that the
// sanitizer fuzz harness (selftest/parser_fuzz.cpp) runs exactly the code the server runs
// (bindings/pickle_native.cpp).  Every length and offset comes from an untrusted peer.
#pragma once

#include <cstdint>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

#include "codec.h"

namespace rrl {

// header text -> parsed header; every obs of a frame carries the same one, so the last header
// is checked first by a byte compare (no key string built on the hit path)
struct StHeaderCache {
  std::unordered_map<std::string, StHeader> map;
  const std::string* last_key = nullptr;
  const StHeader* last = nullptr;
};

// Throws std::runtime_error on anything malformed; never reads outside [p, p + n).
inline void st_tensor_f32(const char* p, size_t n, std::vector<float>& out, StHeaderCache& cache) {
  if (n < 8) throw std::runtime_error("safetensors: file too short");
  uint64_t hl = 0;
  for (int i = 0; i < 8; ++i) hl |= (uint64_t)(uint8_t)p[i] << (8 * i);
  if (hl > n - 8) throw std::runtime_error("safetensors: header length out of range");
  if (cache.last == nullptr || cache.last_key->size() != hl || std::memcmp(cache.last_key->data(), p + 8, hl) != 0) {
    std::string key(p + 8, (size_t)hl);
    auto it = cache.map.find(key);
    if (it == cache.map.end()) it = cache.map.emplace(std::move(key), st_header(p + 8, (size_t)hl)).first;
    cache.last_key = &it->first;  // (unordered_map nodes are stable)
    cache.last = &it->second;
  }
  const StHeader& h = *cache.last;
  const size_t base = 8 + (size_t)hl;
  // st_header guarantees 0 <= off0 <= off1 and off1 - off0 == count * dtype size
  if (h.off0 < 0 || h.off1 < h.off0 || (uint64_t)h.off1 > n - base)
    throw std::runtime_error("safetensors: bad data offsets");
  int64_t cnt = 1;
  for (auto s : h.shape) cnt *= s;
  out.resize((size_t)cnt);
  const char* r = p + base + h.off0;
  for (int64_t i = 0; i < cnt; ++i) {
    switch (h.dtype) {
      case DType::Byte: out[i] = (float)(uint8_t)r[i]; break;
      case DType::Bool: out[i] = r[i] ? 1.f : 0.f; break;
      case DType::Short: { int16_t v; std::memcpy(&v, r + 2 * i, 2); out[i] = (float)v; break; }
      case DType::Int: { int32_t v; std::memcpy(&v, r + 4 * i, 4); out[i] = (float)v; break; }
      case DType::Long: { int64_t v; std::memcpy(&v, r + 8 * i, 8); out[i] = (float)v; break; }
      case DType::Float: { float v; std::memcpy(&v, r + 4 * i, 4); out[i] = v; break; }
      case DType::Double: { double v; std::memcpy(&v, r + 8 * i, 8); out[i] = (float)v; break; }
    }
  }
}

}  // namespace rrl
