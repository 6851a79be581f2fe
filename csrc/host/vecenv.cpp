#include "vecenv.h"

#include <algorithm>
#include <emmintrin.h>

#include <cmath>
#include <cstring>
#include <stdexcept>

namespace rrl {

namespace {

constexpr float kPi = 3.14159265358979f;

// ------------------------------------------------------------------ CartPole-v1
class CartPole : public Env {
 public:
  int obs_dim() const override { return 4; }
  int act_dim() const override { return 2; }
  int max_steps() const override { return 500; }
  void reset(Rng& r, float* o) override {
    for (int i = 0; i < 4; ++i) s_[i] = r.uniform(-0.05f, 0.05f);
    std::copy(s_, s_ + 4, o);
  }
  float step(const float* a, Rng&, float* o, bool& term) override {
    const float force = ((int)a[0] == 1) ? 10.f : -10.f;
    const float costh = std::cos(s_[2]), sinth = std::sin(s_[2]);
    const float temp = (force + 0.05f * s_[3] * s_[3] * sinth) / 1.1f;
    const float thacc = (9.8f * sinth - costh * temp) / (0.5f * (4.f / 3.f - 0.1f * costh * costh / 1.1f));
    const float xacc = temp - 0.05f * thacc * costh / 1.1f;
    s_[0] += 0.02f * s_[1];
    s_[1] += 0.02f * xacc;
    s_[2] += 0.02f * s_[3];
    s_[3] += 0.02f * thacc;
    const float lim = 12.f * 2.f * kPi / 360.f;
    term = s_[0] < -2.4f || s_[0] > 2.4f || s_[2] < -lim || s_[2] > lim;
    std::copy(s_, s_ + 4, o);
    return 1.f;
  }

 private:
  float s_[4];
};

// ------------------------------------------------------------------ MountainCar-v0
class MountainCar : public Env {
 public:
  int obs_dim() const override { return 2; }
  int act_dim() const override { return 3; }
  int max_steps() const override { return 200; }
  void reset(Rng& r, float* o) override {
    p_ = r.uniform(-0.6f, -0.4f);
    v_ = 0.f;
    o[0] = p_;
    o[1] = v_;
  }
  float step(const float* a, Rng&, float* o, bool& term) override {
    v_ += ((int)a[0] - 1) * 0.001f + std::cos(3.f * p_) * (-0.0025f);
    v_ = std::min(std::max(v_, -0.07f), 0.07f);
    p_ += v_;
    p_ = std::min(std::max(p_, -1.2f), 0.6f);
    if (p_ == -1.2f && v_ < 0.f) v_ = 0.f;
    term = p_ >= 0.5f;
    o[0] = p_;
    o[1] = v_;
    return -1.f;
  }

 private:
  float p_, v_;
};

// ------------------------------------------------------------------ Acrobot-v1
class Acrobot : public Env {
 public:
  int obs_dim() const override { return 6; }
  int act_dim() const override { return 3; }
  int max_steps() const override { return 500; }
  void reset(Rng& r, float* o) override {
    for (int i = 0; i < 4; ++i) s_[i] = r.uniform(-0.1f, 0.1f);
    obs(o);
  }
  float step(const float* a, Rng&, float* o, bool& term) override {
    const float torque = (float)((int)a[0] - 1);
    const float dt = 0.2f;
    float y0[4] = {s_[0], s_[1], s_[2], s_[3]}, k1[4], k2[4], k3[4], k4[4], y[4];
    dsdt(y0, torque, k1);
    for (int i = 0; i < 4; ++i) y[i] = y0[i] + 0.5f * dt * k1[i];
    dsdt(y, torque, k2);
    for (int i = 0; i < 4; ++i) y[i] = y0[i] + 0.5f * dt * k2[i];
    dsdt(y, torque, k3);
    for (int i = 0; i < 4; ++i) y[i] = y0[i] + dt * k3[i];
    dsdt(y, torque, k4);
    for (int i = 0; i < 4; ++i) s_[i] = y0[i] + dt / 6.f * (k1[i] + 2.f * k2[i] + 2.f * k3[i] + k4[i]);
    s_[0] = wrap(s_[0]);
    s_[1] = wrap(s_[1]);
    s_[2] = std::min(std::max(s_[2], -4.f * kPi), 4.f * kPi);
    s_[3] = std::min(std::max(s_[3], -9.f * kPi), 9.f * kPi);
    term = (-std::cos(s_[0]) - std::cos(s_[1] + s_[0])) > 1.f;
    obs(o);
    return term ? 0.f : -1.f;
  }

 private:
  static float wrap(float x) {
    while (x > kPi) x -= 2 * kPi;
    while (x < -kPi) x += 2 * kPi;
    return x;
  }
  static void dsdt(const float* s, float a, float* d) {
    const float m2 = 1.f, l1 = 1.f, lc1 = 0.5f, lc2 = 0.5f, I1 = 1.f, I2 = 1.f, g = 9.8f, m1 = 1.f;
    const float d1 = m1 * lc1 * lc1 + m2 * (l1 * l1 + lc2 * lc2 + 2 * l1 * lc2 * std::cos(s[1])) + I1 + I2;
    const float d2 = m2 * (lc2 * lc2 + l1 * lc2 * std::cos(s[1])) + I2;
    const float phi2 = m2 * lc2 * g * std::cos(s[0] + s[1] - kPi / 2);
    const float phi1 = -m2 * l1 * lc2 * s[3] * s[3] * std::sin(s[1]) -
                       2 * m2 * l1 * lc2 * s[3] * s[2] * std::sin(s[1]) + (m1 * lc1 + m2 * l1) * g * std::cos(s[0] - kPi / 2) +
                       phi2;
    const float dd2 = (a + d2 / d1 * phi1 - m2 * l1 * lc2 * s[2] * s[2] * std::sin(s[1]) - phi2) /
                      (m2 * lc2 * lc2 + I2 - d2 * d2 / d1);
    const float dd1 = -(d2 * dd2 + phi1) / d1;
    d[0] = s[2];
    d[1] = s[3];
    d[2] = dd1;
    d[3] = dd2;
  }
  void obs(float* o) {
    o[0] = std::cos(s_[0]);
    o[1] = std::sin(s_[0]);
    o[2] = std::cos(s_[1]);
    o[3] = std::sin(s_[1]);
    o[4] = s_[2];
    o[5] = s_[3];
  }
  float s_[4];
};

// ------------------------------------------------------------------ Pendulum-v1 (continuous)
class Pendulum : public Env {
 public:
  int obs_dim() const override { return 3; }
  int act_dim() const override { return 1; }
  bool continuous() const override { return true; }
  int max_steps() const override { return 200; }
  void reset(Rng& r, float* o) override {
    th_ = r.uniform(-kPi, kPi);
    thd_ = r.uniform(-1.f, 1.f);
    obs(o);
  }
  float step(const float* a, Rng&, float* o, bool& term) override {
    const float u = std::min(std::max(a[0], -2.f), 2.f);
    float thn = std::fmod(th_ + kPi, 2 * kPi);
    if (thn < 0) thn += 2 * kPi;
    thn -= kPi;
    const float cost = thn * thn + 0.1f * thd_ * thd_ + 0.001f * u * u;
    thd_ = thd_ + (3.f * 10.f / 2.f * std::sin(th_) + 3.f * u) * 0.05f;
    thd_ = std::min(std::max(thd_, -8.f), 8.f);
    th_ = th_ + thd_ * 0.05f;
    term = false;
    obs(o);
    return -cost;
  }

 private:
  void obs(float* o) {
    o[0] = std::cos(th_);
    o[1] = std::sin(th_);
    o[2] = thd_;
  }
  float th_, thd_;
};

// ------------------------------------------------------------------ LunarLander-shaped (synthetic)
// 8 obs (x, y, vx, vy, angle, angular velocity, leg1, leg2), 4 discrete actions
// (noop, left engine, main engine, right engine).  Point-mass lander with gymnasium's
// potential-based shaping and +-100 terminal bonus.  NOT Box2D: a stand-in with the
// same interface for throughput / plumbing configs (documented in docs/ENVS.md).
class LunarLanderSynth : public Env {
 public:
  int obs_dim() const override { return 8; }
  int act_dim() const override { return 4; }
  int max_steps() const override { return 1000; }
  void reset(Rng& r, float* o) override {
    x_ = r.uniform(-0.3f, 0.3f);
    y_ = 1.4f;
    vx_ = r.uniform(-0.5f, 0.5f);
    vy_ = r.uniform(-0.3f, 0.0f);
    ang_ = r.uniform(-0.1f, 0.1f);
    angv_ = 0.f;
    prev_shaping_ = shaping();
    obs(o);
  }
  float step(const float* a, Rng& r, float* o, bool& term) override {
    const int act = (int)a[0];
    const float dt = 1.f / 50.f;
    float ax = 0.f, ay = -10.f / 6.f, aa = 0.f, fuel = 0.f;
    if (act == 2) {  // main engine along the body axis
      ax += -std::sin(ang_) * 13.f / 6.f;
      ay += std::cos(ang_) * 13.f / 6.f;
      fuel += 0.3f;
    } else if (act == 1 || act == 3) {
      const float dir = act == 1 ? -1.f : 1.f;
      ax += dir * std::cos(ang_) * 0.6f / 6.f;
      aa += -dir * 1.5f;
      fuel += 0.03f;
    }
    ax += r.uniform(-0.05f, 0.05f);
    vx_ += ax * dt * 6.f;
    vy_ += ay * dt * 6.f;
    angv_ += aa * dt;
    x_ += vx_ * dt;
    y_ += vy_ * dt;
    ang_ += angv_ * dt;
    float sh = shaping();
    float rew = sh - prev_shaping_ - fuel;
    prev_shaping_ = sh;
    term = false;
    if (y_ <= 0.f) {
      y_ = 0.f;
      term = true;
      const bool soft = std::fabs(vy_) < 0.5f && std::fabs(vx_) < 0.5f && std::fabs(ang_) < 0.3f && std::fabs(x_) < 0.5f;
      rew += soft ? 100.f : -100.f;
    } else if (std::fabs(x_) >= 1.f) {
      term = true;
      rew -= 100.f;
    }
    obs(o);
    return rew;
  }

 private:
  float shaping() const {
    const float legs = (y_ < 0.05f ? 20.f : 0.f);
    return -100.f * std::sqrt(x_ * x_ + y_ * y_) - 100.f * std::sqrt(vx_ * vx_ + vy_ * vy_) - 100.f * std::fabs(ang_) +
           legs;
  }
  void obs(float* o) {
    o[0] = x_;
    o[1] = y_;
    o[2] = vx_;
    o[3] = vy_;
    o[4] = ang_;
    o[5] = angv_;
    o[6] = y_ < 0.05f ? 1.f : 0.f;
    o[7] = y_ < 0.05f ? 1.f : 0.f;
  }
  float x_, y_, vx_, vy_, ang_, angv_, prev_shaping_;
};

// ------------------------------------------------------------------ HalfCheetah-shaped (synthetic)
// 17 obs / 6 continuous actions in [-1, 1]; a fixed, stable, weakly non-linear
// dynamical system with reward = forward velocity (obs[8]) - 0.1 |a|^2, 1000 steps.
// The system matrices are part of the env definition (also exported to the device env
// through env_constants("HalfCheetahSynth-v0")).
void halfcheetah_matrices(float (&A)[17][17], float (&B)[17][6]) {
  Rng r(12345);
  for (int i = 0; i < 17; ++i)
    for (int j = 0; j < 17; ++j) A[i][j] = (i == j ? 0.9f : 0.f) + r.uniform(-0.03f, 0.03f);
  for (int i = 0; i < 17; ++i)
    for (int j = 0; j < 6; ++j) B[i][j] = r.uniform(-0.2f, 0.2f);
}

struct HalfCheetahConsts {
  float A[17][17], B[17][6];
  float Ap[18][17], Bp[18][6];  // zero-padded to 3 x 6 rows for the branch-free batched pass
  HalfCheetahConsts() {
    halfcheetah_matrices(A, B);
    std::fill(&Ap[0][0], &Ap[0][0] + 18 * 17, 0.f);
    std::fill(&Bp[0][0], &Bp[0][0] + 18 * 6, 0.f);
    std::copy(&A[0][0], &A[0][0] + 17 * 17, &Ap[0][0]);
    std::copy(&B[0][0], &B[0][0] + 17 * 6, &Bp[0][0]);
  }
};

class HalfCheetahSynth : public Env {
 public:
  // one shared copy of the dynamics (a per-env copy was 1.5 KB x N envs of cache traffic per step)
  HalfCheetahSynth() : A_(consts().A), B_(consts().B) {}
  float* state() { return s_; }
  static const HalfCheetahConsts& consts() {
    static const HalfCheetahConsts c;
    return c;
  }
  int obs_dim() const override { return 17; }
  int act_dim() const override { return 6; }
  bool continuous() const override { return true; }
  int max_steps() const override { return 1000; }
  void reset(Rng& r, float* o) override {
    for (int i = 0; i < 17; ++i) s_[i] = r.uniform(-0.1f, 0.1f);
    std::copy(s_, s_ + 17, o);
  }
  float step(const float* a, Rng& r, float* o, bool& term) override {
    float u[6], ctrl = 0.f;
    for (int j = 0; j < 6; ++j) {
      u[j] = std::min(std::max(a[j], -1.f), 1.f);
      ctrl += u[j] * u[j];
    }
    float ns[17];
    for (int i = 0; i < 17; ++i) {
      float v = 0.f;
      for (int j = 0; j < 17; ++j) v += A_[i][j] * s_[j];
      for (int j = 0; j < 6; ++j) v += B_[i][j] * u[j];
      ns[i] = v;
    }
    for (int i = 0; i < 17; ++i) ns[i] = std::tanh(ns[i]) + r.uniform(-0.01f, 0.01f);
    std::copy(ns, ns + 17, s_);
    term = false;
    std::copy(s_, s_ + 17, o);
    return s_[8] - 0.1f * ctrl;
  }

 private:
  const float (&A_)[17][17];
  const float (&B_)[17][6];
  float s_[17];
};

// tanh of 4 floats with SSE2 (any x86-64): tanh(x) = sign(x) (1 - e) / (1 + e), e = exp(-2|x|),
// exp by range reduction to |r| <= ln2 / 2 and a degree-6 polynomial.  Absolute error ~1e-7
// (the env adds U(-0.01, 0.01) noise after it); libm tanhf was ~45 % of the scalar step.
inline __m128 tanh4(__m128 x) {
  const __m128 sign = _mm_and_ps(x, _mm_castsi128_ps(_mm_set1_epi32((int)0x80000000u)));
  __m128 y = _mm_mul_ps(_mm_andnot_ps(_mm_castsi128_ps(_mm_set1_epi32((int)0x80000000u)), x), _mm_set1_ps(-2.f));
  y = _mm_max_ps(y, _mm_set1_ps(-87.f));
  // n = round(y / ln 2) (y <= 0), r = y - n ln 2
  const __m128i ni = _mm_cvttps_epi32(_mm_sub_ps(_mm_mul_ps(y, _mm_set1_ps(1.44269504f)), _mm_set1_ps(0.5f)));
  const __m128 n = _mm_cvtepi32_ps(ni);
  const __m128 r = _mm_sub_ps(_mm_sub_ps(y, _mm_mul_ps(n, _mm_set1_ps(0.693145752f))),
                              _mm_mul_ps(n, _mm_set1_ps(1.42860677e-6f)));
  __m128 p = _mm_set1_ps(1.f / 720.f);
  p = _mm_add_ps(_mm_mul_ps(p, r), _mm_set1_ps(1.f / 120.f));
  p = _mm_add_ps(_mm_mul_ps(p, r), _mm_set1_ps(1.f / 24.f));
  p = _mm_add_ps(_mm_mul_ps(p, r), _mm_set1_ps(1.f / 6.f));
  p = _mm_add_ps(_mm_mul_ps(p, r), _mm_set1_ps(0.5f));
  p = _mm_add_ps(_mm_mul_ps(p, r), _mm_set1_ps(1.f));
  p = _mm_add_ps(_mm_mul_ps(p, r), _mm_set1_ps(1.f));
  const __m128 e = _mm_mul_ps(p, _mm_castsi128_ps(_mm_slli_epi32(_mm_add_epi32(ni, _mm_set1_epi32(127)), 23)));
  const __m128 one = _mm_set1_ps(1.f);
  return _mm_or_ps(_mm_div_ps(_mm_sub_ps(one, e), _mm_add_ps(one, e)), sign);
}

// HalfCheetahSynth physics for envs [i0, i0 + 8): the 17 x 23 matrix-vector products of eight
// envs at once with the env index innermost (vector FMAs across envs) and six output rows per
// pass, so six independent accumulation chains are in flight instead of one 23-deep chain per
// row (the first form was latency-bound: 195 of the scalar path's ~350 ns per env step went to
// the matvec, ~45 % of the rest to libm tanh).  Each env then draws its own noise in the scalar
// path's order.  Writes the new state into the envs and obs, returns the rewards.
void halfcheetah_step8(HalfCheetahSynth* const* e, int nb, const float* act, Rng* rng, float* obs, float* rew) {
  const HalfCheetahConsts& c = HalfCheetahSynth::consts();
  float s[17][8], u[6][8], ns[18][8], ctrl[8];
  for (int k = 0; k < 8; ++k) {
    const bool ok = k < nb;
    const float* st = ok ? e[k]->state() : nullptr;
    for (int j = 0; j < 17; ++j) s[j][k] = ok ? st[j] : 0.f;
    float cs = 0.f;
    for (int j = 0; j < 6; ++j) {
      const float a = ok ? std::min(std::max(act[(size_t)k * 6 + j], -1.f), 1.f) : 0.f;
      u[j][k] = a;
      cs += a * a;
    }
    ctrl[k] = cs;
  }
  for (int i0 = 0; i0 < 18; i0 += 6) {
    float v[6][8] = {};
    for (int j = 0; j < 17; ++j)
      for (int ii = 0; ii < 6; ++ii) {
        const float a = c.Ap[i0 + ii][j];
        for (int k = 0; k < 8; ++k) v[ii][k] += a * s[j][k];
      }
    for (int j = 0; j < 6; ++j)
      for (int ii = 0; ii < 6; ++ii) {
        const float b = c.Bp[i0 + ii][j];
        for (int k = 0; k < 8; ++k) v[ii][k] += b * u[j][k];
      }
    for (int ii = 0; ii < 6; ++ii)
      for (int k = 0; k < 8; ++k) ns[i0 + ii][k] = v[ii][k];
  }
  float* flat = &ns[0][0];
  for (int q = 0; q < 17 * 8; q += 4) _mm_storeu_ps(flat + q, tanh4(_mm_loadu_ps(flat + q)));
  for (int k = 0; k < nb; ++k) {
    float* st = e[k]->state();
    for (int i = 0; i < 17; ++i) st[i] = ns[i][k] + rng[k].uniform(-0.01f, 0.01f);
    std::copy(st, st + 17, obs + (size_t)k * 17);
    rew[k] = st[8] - 0.1f * ctrl[k];
  }
}

}  // namespace

std::vector<float> env_constants(const std::string& name) {
  if (name == "HalfCheetahSynth-v0" || name == "HalfCheetah-v4") {
    float A[17][17], B[17][6];
    halfcheetah_matrices(A, B);
    std::vector<float> out(&A[0][0], &A[0][0] + 17 * 17);
    out.insert(out.end(), &B[0][0], &B[0][0] + 17 * 6);
    return out;
  }
  return {};
}

std::vector<std::string> env_names() {
  return {"CartPole-v1", "MountainCar-v0", "Acrobot-v1", "Pendulum-v1", "LunarLanderSynth-v0", "HalfCheetahSynth-v0"};
}

std::unique_ptr<Env> make_env(const std::string& name) {
  if (name == "CartPole-v1" || name == "CartPole-v0") return std::make_unique<CartPole>();
  if (name == "MountainCar-v0") return std::make_unique<MountainCar>();
  if (name == "Acrobot-v1") return std::make_unique<Acrobot>();
  if (name == "Pendulum-v1") return std::make_unique<Pendulum>();
  if (name == "LunarLanderSynth-v0" || name == "LunarLander-v2" || name == "LunarLander-v3")
    return std::make_unique<LunarLanderSynth>();
  if (name == "HalfCheetahSynth-v0" || name == "HalfCheetah-v4") return std::make_unique<HalfCheetahSynth>();
  throw std::invalid_argument("unknown env: " + name);
}

// ------------------------------------------------------------------ VecEnv
VecEnv::VecEnv(const std::string& name, int num_envs, uint64_t seed, int num_threads) : name_(name), n_(num_envs) {
  if (num_envs <= 0) throw std::invalid_argument("num_envs must be positive");
  for (int i = 0; i < n_; ++i) {
    envs_.push_back(make_env(name));
    rngs_.emplace_back(seed * 0x9E3779B97F4A7C15ull + (uint64_t)i * 0xD1B54A32D192ED03ull + 1);
  }
  obs_dim_ = envs_[0]->obs_dim();
  act_dim_ = envs_[0]->act_dim();
  batch_hc_ = dynamic_cast<HalfCheetahSynth*>(envs_[0].get()) != nullptr;
  continuous_ = envs_[0]->continuous();
  max_steps_ = envs_[0]->max_steps();
  len_.assign(n_, 0);
  ret_.assign(n_, 0.f);
  nthreads_ = std::max(1, std::min(num_threads, n_));
  tstats_.resize(nthreads_);
  // every slice runs on a pool thread (the caller only submits and waits), so a step can
  // also be left running while the caller does other work (step_async)
  for (int t = 0; t < nthreads_; ++t) pool_.emplace_back(&VecEnv::worker, this, t);
}

VecEnv::~VecEnv() {
  wait();
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : pool_) t.join();
}

void VecEnv::worker(int tid) {
  uint64_t seen = 0;
  while (true) {
    {
      std::unique_lock<std::mutex> g(mu_);
      cv_.wait(g, [&] { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen_;
    }
    job_(tid, nthreads_);  // job_ is only replaced after every worker finished (wait())
    {
      std::lock_guard<std::mutex> g(mu_);
      if (--pending_ == 0) done_cv_.notify_all();
    }
  }
}

void VecEnv::submit(std::function<void(int, int)> fn) {
  wait();
  {
    std::lock_guard<std::mutex> g(mu_);
    job_ = std::move(fn);
    pending_ = nthreads_;
    busy_ = true;
    ++gen_;
  }
  cv_.notify_all();
}

void VecEnv::wait() {
  std::unique_lock<std::mutex> g(mu_);
  done_cv_.wait(g, [&] { return pending_ == 0; });
  busy_ = false;
}

void VecEnv::run_parallel(const std::function<void(int, int)>& fn) {
  submit(fn);
  wait();
}

void VecEnv::reset(float* obs) {
  run_parallel([&](int tid, int nt) {
    const int lo = (int)((int64_t)n_ * tid / nt), hi = (int)((int64_t)n_ * (tid + 1) / nt);
    for (int i = lo; i < hi; ++i) {
      envs_[i]->reset(rngs_[i], obs + (size_t)i * obs_dim_);
      len_[i] = 0;
      ret_[i] = 0.f;
    }
  });
}

void VecEnv::step(const void* actions, float* obs, float* rew, float* done, float* tobs) {
  step_async(actions, obs, rew, done, tobs);
  wait();
}

void VecEnv::step_async(const void* actions, float* obs, float* rew, float* done, float* tobs) {
  submit([this, actions, obs, rew, done, tobs](int tid, int nt) { step_range(tid, nt, actions, obs, rew, done, tobs); });
}

void VecEnv::step_range(int tid, int nt, const void* actions, float* obs, float* rew, float* done, float* tobs) {
  {
    const int lo = (int)((int64_t)n_ * tid / nt), hi = (int)((int64_t)n_ * (tid + 1) / nt);
    EpisodeStats& st = tstats_[tid];
    float rb[8];
    for (int i = lo; i < hi; ++i) {
      bool term = false;
      float* o = obs + (size_t)i * obs_dim_;
      float r;
      if (batch_hc_) {
        const int k = (i - lo) & 7;
        if (k == 0) {  // physics of the next 8 envs in one vectorised pass
          HalfCheetahSynth* e8[8];
          const int nb = std::min(8, hi - i);
          for (int q = 0; q < nb; ++q) e8[q] = static_cast<HalfCheetahSynth*>(envs_[i + q].get());
          halfcheetah_step8(e8, nb, (const float*)actions + (size_t)i * 6, &rngs_[i], o, rb);
        }
        r = rb[k];
      } else {
        float a[16];
        const float* ap;
        if (continuous_) {
          ap = (const float*)actions + (size_t)i * act_dim_;
        } else {
          a[0] = (float)((const int32_t*)actions)[i];
          ap = a;
        }
        r = envs_[i]->step(ap, rngs_[i], o, term);
      }
      len_[i] += 1;
      ret_[i] += r;
      const bool d = term || len_[i] >= max_steps_;
      const bool boot = d && !term && tobs != nullptr;
      rew[i] = r;
      done[i] = boot ? 2.f : (d ? 1.f : 0.f);
      if (boot) std::copy(o, o + obs_dim_, tobs + (size_t)i * obs_dim_);
      if (d) {
        st.n += 1;
        st.sum += ret_[i];
        st.sumsq += (double)ret_[i] * ret_[i];
        st.max = std::max(st.max, (double)ret_[i]);
        st.min = std::min(st.min, (double)ret_[i]);
        st.sum_len += len_[i];
        envs_[i]->reset(rngs_[i], o);
        len_[i] = 0;
        ret_[i] = 0.f;
      }
    }
  }
}

EpisodeStats VecEnv::take_stats() {
  wait();  // never read the per-thread sums while an async step is writing them
  EpisodeStats s;
  for (auto& t : tstats_) {
    s.n += t.n;
    s.sum += t.sum;
    s.sumsq += t.sumsq;
    s.max = std::max(s.max, t.max);
    s.min = std::min(s.min, t.min);
    s.sum_len += t.sum_len;
    t = EpisodeStats();
  }
  return s;
}

}  // namespace rrl
