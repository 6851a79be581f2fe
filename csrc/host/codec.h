// Host-side codecs (C++ replacement of relayrl_framework/src/types/{action,trajectory}.rs).
//
//  * safetensors single-tensor files: the reference's TensorData.data is a complete
//    safetensors file holding one tensor named "tensor" (action.rs:342-352).  We emit
//    byte-identical files (header JSON padded with spaces to 8-byte alignment).
//  * RRLT binary trajectory frames: our wire format for trajectory uploads (replaces the
//    serde_pickle(Vec<RelayRLAction>) frame of trajectory.rs:50-55).  Columnar-free,
//    length-prefixed, little-endian; decodes with zero JSON work.
#pragma once
#include <cstdint>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

namespace rrl {

// Reference DType names (action.rs:92-100) <-> safetensors dtype tags.
enum class DType : uint8_t { Byte = 0, Short = 1, Int = 2, Long = 3, Float = 4, Double = 5, Bool = 6 };

const char* dtype_name(DType d);
DType dtype_from_name(const std::string& s);
const char* dtype_st_tag(DType d);  // Bool -> "U8" on write, as the reference does
DType dtype_from_st_tag(const std::string& s);
size_t dtype_size(DType d);

struct Tensor {
  DType dtype = DType::Float;
  std::vector<int64_t> shape;
  std::string raw;  // little-endian element bytes
  int64_t numel() const {
    int64_t n = 1;
    for (auto s : shape) n *= s;
    return n;
  }
};

std::string st_encode(const Tensor& t, const std::string& name = "tensor");
Tensor st_decode(const std::string& file, const std::string& name = "tensor");
// The header of one tensor in a safetensors file: dtype, shape and its byte range within the data
// section (the section starts at 8 + header length).  st_decode = st_header + the range's bytes.
struct StHeader {
  DType dtype = DType::Float;
  std::vector<int64_t> shape;
  int64_t off0 = 0, off1 = 0;
};
StHeader st_header(const char* header_json, size_t len, const std::string& name = "tensor");

// ----------------------------------------------------------------- RelayRLData / action
// Externally tagged aux value (action.rs:207-218): Tensor or a scalar / string.
struct AuxValue {
  enum Kind : uint8_t { TENSOR = 0, BYTE, SHORT, INT, LONG, FLOAT, DOUBLE, STRING, BOOL } kind = DOUBLE;
  Tensor tensor;
  int64_t i = 0;
  double d = 0.0;
  std::string s;
  bool b = false;
};

struct Action {
  bool has_obs = false, has_act = false, has_mask = false;
  Tensor obs, act, mask;
  float rew = 0.f;
  bool has_data = false;
  std::map<std::string, AuxValue> data;
  bool done = false;
  bool reward_updated = false;
};

struct Trajectory {
  std::string server;  // trajectory_server (may be empty)
  uint32_t max_length = 1000;
  std::string agent_id;
  uint64_t seq = 0;  // per-agent sequence number (heartbeat / loss detection)
  std::vector<Action> actions;
};

std::string traj_encode(const Trajectory& t);
Trajectory traj_decode(const std::string& buf);

}  // namespace rrl
