// Vectorised CPU environments stepped by a persistent thread pool.
//
// The reference steps one gymnasium env per agent process in Python
// (cartpole_zmq.ipynb:37-60) -- gymnasium is not installed here, so the envs the
// reference examples use are re-implemented natively with gymnasium's dynamics
// (CartPole-v1, MountainCar-v0, Acrobot-v1, Pendulum-v1), plus two synthetic envs with
// the observation/action shapes of the BASELINE configs that need Box2D / MuJoCo
// (LunarLander: 8 obs / 4 actions, HalfCheetah: 17 obs / 6 continuous actions).
//
// step() writes obs/reward/done straight into caller-owned (pinned) buffers so the host
// env path can feed the device through hipMemcpyAsync without extra copies.
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace rrl {

struct Rng {  // xoshiro128+-style small fast generator, seeded with splitmix64
  uint64_t s0, s1;
  explicit Rng(uint64_t seed = 1) {
    auto sm = [&seed]() {
      uint64_t z = (seed += 0x9E3779B97F4A7C15ull);
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      return z ^ (z >> 31);
    };
    s0 = sm();
    s1 = sm();
  }
  uint64_t next() {
    uint64_t a = s0, b = s1;
    const uint64_t r = a + b;
    b ^= a;
    s0 = ((a << 55) | (a >> 9)) ^ b ^ (b << 14);
    s1 = (b << 36) | (b >> 28);
    return r;
  }
  float uniform(float lo, float hi) { return lo + (hi - lo) * (float)((next() >> 40) * (1.0 / 16777216.0)); }
};

class Env {
 public:
  virtual ~Env() = default;
  virtual int obs_dim() const = 0;
  virtual int act_dim() const = 0;  // #actions (discrete) or action dim (continuous)
  virtual bool continuous() const { return false; }
  virtual int max_steps() const = 0;
  virtual void reset(Rng& rng, float* obs) = 0;
  // returns reward; sets terminated
  virtual float step(const float* action, Rng& rng, float* obs, bool& terminated) = 0;
};

std::unique_ptr<Env> make_env(const std::string& name);
std::vector<std::string> env_names();
// Constant tables that define an env (HalfCheetahSynth: A[17x17] then B[17x6]); empty if none.
std::vector<float> env_constants(const std::string& name);

struct EpisodeStats {
  double n = 0, sum = 0, sumsq = 0, max = -1e300, min = 1e300, sum_len = 0;
};

class VecEnv {
 public:
  VecEnv(const std::string& name, int num_envs, uint64_t seed, int num_threads);
  ~VecEnv();
  int num_envs() const { return n_; }
  int obs_dim() const { return obs_dim_; }
  int act_dim() const { return act_dim_; }
  bool continuous() const { return continuous_; }
  int max_steps() const { return max_steps_; }
  void reset(float* obs);
  // actions: int32[N] (discrete) or float[N*act_dim] (continuous).  Finished envs are
  // auto-reset; obs then holds the first observation of the next episode.
  // done codes: 0 running, 1 terminal, 2 time-limit truncation; with ``tobs`` non-null a
  // truncated env's pre-reset observation goes to tobs[i] (its value bootstraps the cut
  // episode), without it truncations are reported as 1.
  void step(const void* actions, float* obs, float* rew, float* done, float* tobs = nullptr);
  // Asynchronous step: the pool starts stepping and the call returns at once; wait() blocks
  // until it finished (the buffers must stay untouched until then).  Two VecEnvs stepped
  // asynchronously keep both thread pools busy at the same time (host_trainer.py pipeline).
  void step_async(const void* actions, float* obs, float* rew, float* done, float* tobs = nullptr);
  void wait();
  EpisodeStats take_stats();

 private:
  void run_parallel(const std::function<void(int, int)>& fn);
  void submit(std::function<void(int, int)> fn);
  void step_range(int tid, int nt, const void* actions, float* obs, float* rew, float* done, float* tobs);
  void worker(int tid);

  std::string name_;
  int n_, obs_dim_, act_dim_, max_steps_;
  bool continuous_;
  bool batch_hc_ = false;  // HalfCheetahSynth: 8 envs per vectorised physics pass
  std::vector<std::unique_ptr<Env>> envs_;
  std::vector<Rng> rngs_;
  std::vector<int> len_;
  std::vector<float> ret_;
  std::vector<EpisodeStats> tstats_;
  // thread pool
  int nthreads_;
  std::vector<std::thread> pool_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  uint64_t gen_ = 0;
  int pending_ = 0;
  bool stop_ = false;
  std::function<void(int, int)> job_;  // owned: an async job outlives the submitting call
  bool busy_ = false;                   // a submitted job has not been waited for
};

}  // namespace rrl
