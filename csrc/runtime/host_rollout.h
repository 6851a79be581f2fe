// Host-env rollout driver: the T-step "env threads <-> GPU policy" loop of the host-env
// trainer (runtime/host_trainer.py) in C++, with no Python and no allocation per step.
//
// The reference's per-step action path is one agent process doing batch-1 TorchScript
// inference + a gymnasium step + a serialised upload per env step (agent_zmq.rs:458-571,
// cartpole_zmq.ipynb:37-60).  Here N envs are stepped by C++ thread pools (csrc/host/
// vecenv.cpp) in two halves, and each half-step is ONE kernel launch on the caller's HIP
// stream: the sampling kernel (mlp_forward.hip, CAT_SAMPLE / GAUSS_SAMPLE) reads the
// half's observations straight from pinned host memory (zero-copy over PCIe), copies them
// into the HBM rollout buffer for the learner, and writes the sampled actions both to HBM
// and back into pinned host memory for the env threads.  While the GPU samples one half,
// the other half's threads step.  The driver waits on a timing-free HIP event by polling
// (no OS sleep).  After the last step the rewards / done codes / truncation observations
// go to HBM with three async copies on the same stream.
//
// Stream order is the caller's: the first launch of a rollout writes the HBM buffers, so it
// is queued behind whatever the stream already holds (the previous update's reads).
#pragma once
#include <hip/hip_runtime_api.h>

#include <cstdint>
#include <vector>

#include "vecenv.h"

namespace rrl {

struct RolloutBuffers {
  // pinned host staging: obs [T+1][N][D], act [T][N] int32 or [T][N][A] f32, rew / done [T][N],
  // tobs [T][N][D] (null = no truncation bootstrap)
  float* h_obs;
  void* h_act;
  float* h_rew;
  float* h_done;
  float* h_tobs;
  // HBM: obs [T+1][N][D], act, logp [T][N], rew, done, tobs (null when h_tobs is null)
  float* d_obs;
  void* d_act;
  float* d_logp;
  float* d_rew;
  float* d_done;
  float* d_tobs;
};

// Accumulated wall time of the driver thread (microseconds), reset by take_stats().
struct RolloutStats {
  double env_wait_us = 0;   // blocked on an env half's threads (CPU physics not yet done)
  double gpu_wait_us = 0;   // polling a half's sampling event (kernel + PCIe not yet done)
  double launch_us = 0;     // host cost of the launches + event records
  double tail_us = 0;       // final waits + the three H2D copies' enqueue
  double total_us = 0;
  int64_t steps = 0;        // env steps of the whole batch (T per rollout)
  int64_t launches = 0;
};

class HostRollout {
 public:
  HostRollout(std::vector<VecEnv*> envs, std::vector<int> bounds, int num_cu);
  ~HostRollout();
  HostRollout(const HostRollout&) = delete;
  HostRollout& operator=(const HostRollout&) = delete;

  int obs_dim() const { return D_; }
  int act_dim() const { return A_; }
  bool continuous() const { return cont_; }
  int num_envs() const { return bounds_.back(); }

  // One rollout of T steps into ``b`` with the flat policy ``params`` (device pointer).
  // Returns 0 or a HIP / launch error code (the envs are then left waited-for).
  int run(const float* params, int H, int T, const RolloutBuffers& b, uint64_t seed, uint64_t step0,
          hipStream_t stream);
  RolloutStats take_stats();
  // 0: poll the half's event, 1: hipEventSynchronize, 2: poll with ~1 us pause back-off
  void set_wait_mode(int m) { wait_mode_ = m; }

 private:
  int wait_mode_ = 0;
  std::vector<VecEnv*> envs_;
  std::vector<int> bounds_;
  int D_, A_;
  bool cont_;
  int num_cu_;
  std::vector<hipEvent_t> ev_;
  RolloutStats st_;
};

}  // namespace rrl
