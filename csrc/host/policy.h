// Native CPU policy for off-GPU agents (replaces the reference agent's per-step
// TorchScript interpreter call, agent_wrapper.rs / o3_agent.rs request_for_action).
// Evaluates the framework's 3-layer MLP from the learner's flat fp32 vectors
// (layout: W1[H*D] b1[H] W2[H*H] b2[H] W3[A*H] b3[A] [log_std[A]]) and samples.
#pragma once
#include <cstdint>
#include <vector>

namespace rrl {

class NativePolicy {
 public:
  NativePolicy(int D, int H, int A, bool discrete, uint64_t seed);
  // Loads policy (and optional value) flat vectors; sizes are checked.
  void load(const float* pi, int64_t n_pi, const float* vf, int64_t n_vf);
  bool has_value() const { return has_vf_; }
  // N rows.  obs [N][D]; mask [N][A] or null; act_i [N] (discrete) or act_f [N][A];
  // logp [N]; v [N] or null (written when a value net is loaded).
  void step(const float* obs, const float* mask, int N, int32_t* act_i, float* act_f, float* logp, float* v);
  // Deterministic pieces for tests: logits [N][A] and value [N].
  void logits(const float* obs, int N, float* out) const;
  void value(const float* obs, int N, float* out) const;
  int D, H, A;
  bool discrete;

 private:
  struct Net {
    std::vector<float> w1t, b1, w2t, b2, w3t, b3, log_std;  // w*t: [in][out]
    std::vector<float> w3;  // the head [out][in] as well: dot products for narrow heads
  };
  void trunk(const Net& n, int out_dim, const float* x, float* out, float* h1, float* h2) const;
  static void unpack(Net& n, const float* p, int D, int H, int O, bool gaussian);
  Net pi_, vf_;
  std::vector<float> h1_, h2_, z_;  // step()'s scratch (step is not reentrant: it advances the RNG)
  bool has_vf_ = false;
  uint64_t s_[4];
  double uniform();
  double normal();
  bool have_spare_ = false;
  double spare_ = 0.0;
};

}  // namespace rrl
