// Device-side vectorised environments for the fused rollout kernel.
//
// The reference steps a single gymnasium env per agent process on the CPU
// (cartpole_zmq.ipynb:37-60).  For the on-device actor every lane of a wave column
// carries one env's state in registers; physics constants follow gymnasium's
// classic-control definitions (CartPole-v1, MountainCar-v0, Acrobot-v1 dims/limits).
#pragma once
#include "common.h"

namespace rrl {

struct CartPoleEnv {
  static constexpr int D = 4, A = 2, NS = 4;
  static constexpr int kMaxSteps = 500;
  RRL_DEV static void reset(float (&s)[NS], uint4 r) {
    s[0] = -0.05f + 0.1f * u01(r.x);
    s[1] = -0.05f + 0.1f * u01(r.y);
    s[2] = -0.05f + 0.1f * u01(r.z);
    s[3] = -0.05f + 0.1f * u01(r.w);
  }
  RRL_DEV static float obs(const float (&s)[NS], int f) {
    return f == 0 ? s[0] : f == 1 ? s[1] : f == 2 ? s[2] : s[3];
  }
  // Euler integration exactly as gymnasium CartPoleEnv.step (kinematics_integrator="euler").
  RRL_DEV static float step(float (&s)[NS], int a, bool& terminated, float /*noise01*/) {
    const float gravity = 9.8f, masspole = 0.1f, total_mass = 1.1f, length = 0.5f;
    const float polemass_length = masspole * length, force_mag = 10.f, tau = 0.02f;
    const float force = a == 1 ? force_mag : -force_mag;
    const float costh = cosf(s[2]), sinth = sinf(s[2]);
    const float temp = (force + polemass_length * s[3] * s[3] * sinth) / total_mass;
    const float thacc = (gravity * sinth - costh * temp) /
                        (length * (4.f / 3.f - masspole * costh * costh / total_mass));
    const float xacc = temp - polemass_length * thacc * costh / total_mass;
    s[0] = s[0] + tau * s[1];
    s[1] = s[1] + tau * xacc;
    s[2] = s[2] + tau * s[3];
    s[3] = s[3] + tau * thacc;
    const float th_lim = 12.f * 2.f * 3.14159265358979f / 360.f;
    terminated = (s[0] < -2.4f) || (s[0] > 2.4f) || (s[2] < -th_lim) || (s[2] > th_lim);
    return 1.f;
  }
};

struct MountainCarEnv {
  static constexpr int D = 2, A = 3, NS = 2;
  static constexpr int kMaxSteps = 200;
  RRL_DEV static void reset(float (&s)[NS], uint4 r) {
    s[0] = -0.6f + 0.2f * u01(r.x);
    s[1] = 0.f;
  }
  RRL_DEV static float obs(const float (&s)[NS], int f) { return f == 0 ? s[0] : s[1]; }
  RRL_DEV static float step(float (&s)[NS], int a, bool& terminated, float /*noise01*/) {
    float pos = s[0], vel = s[1];
    vel += (float)(a - 1) * 0.001f + cosf(3.f * pos) * (-0.0025f);
    vel = fminf(fmaxf(vel, -0.07f), 0.07f);
    pos += vel;
    pos = fminf(fmaxf(pos, -1.2f), 0.6f);
    if (pos == -1.2f && vel < 0.f) vel = 0.f;
    s[0] = pos;
    s[1] = vel;
    terminated = pos >= 0.5f;
    return -1.f;
  }
};

// Acrobot-v1 (RK4 "book" dynamics), 6-dim obs, 3 actions, reward -1 until the tip
// swings above the bar.
struct AcrobotEnv {
  static constexpr int D = 6, A = 3, NS = 4;
  static constexpr int kMaxSteps = 500;
  RRL_DEV static void reset(float (&s)[NS], uint4 r) {
    s[0] = -0.1f + 0.2f * u01(r.x);
    s[1] = -0.1f + 0.2f * u01(r.y);
    s[2] = -0.1f + 0.2f * u01(r.z);
    s[3] = -0.1f + 0.2f * u01(r.w);
  }
  RRL_DEV static float obs(const float (&s)[NS], int f) {
    switch (f) {
      case 0: return cosf(s[0]);
      case 1: return sinf(s[0]);
      case 2: return cosf(s[1]);
      case 3: return sinf(s[1]);
      case 4: return s[2];
      default: return s[3];
    }
  }
  RRL_DEV static void dsdt(const float (&s)[5], float (&d)[4]) {
    const float m1 = 1.f, m2 = 1.f, l1 = 1.f, lc1 = 0.5f, lc2 = 0.5f, I1 = 1.f, I2 = 1.f, g = 9.8f;
    const float a = s[4];
    const float th1 = s[0], th2 = s[1], dth1 = s[2], dth2 = s[3];
    const float d1 = m1 * lc1 * lc1 + m2 * (l1 * l1 + lc2 * lc2 + 2.f * l1 * lc2 * cosf(th2)) + I1 + I2;
    const float d2 = m2 * (lc2 * lc2 + l1 * lc2 * cosf(th2)) + I2;
    const float phi2 = m2 * lc2 * g * cosf(th1 + th2 - 1.5707963267948966f);
    const float phi1 = -m2 * l1 * lc2 * dth2 * dth2 * sinf(th2) - 2.f * m2 * l1 * lc2 * dth2 * dth1 * sinf(th2) +
                       (m1 * lc1 + m2 * l1) * g * cosf(th1 - 1.5707963267948966f) + phi2;
    const float ddth2 = (a + d2 / d1 * phi1 - m2 * l1 * lc2 * dth1 * dth1 * sinf(th2) - phi2) /
                        (m2 * lc2 * lc2 + I2 - d2 * d2 / d1);
    const float ddth1 = -(d2 * ddth2 + phi1) / d1;
    d[0] = dth1; d[1] = dth2; d[2] = ddth1; d[3] = ddth2;
  }
  RRL_DEV static float wrap(float x) {
    const float pi = 3.14159265358979f;
    while (x > pi) x -= 2.f * pi;
    while (x < -pi) x += 2.f * pi;
    return x;
  }
  RRL_DEV static float step(float (&s)[NS], int a, bool& terminated, float /*noise01*/) {
    const float torque = (float)(a - 1);
    const float dt = 0.2f;
    float y0[5] = {s[0], s[1], s[2], s[3], torque}, k1[4], k2[4], k3[4], k4[4], y[5];
    dsdt(y0, k1);
    for (int i = 0; i < 4; ++i) y[i] = y0[i] + 0.5f * dt * k1[i];
    y[4] = torque; dsdt(y, k2);
    for (int i = 0; i < 4; ++i) y[i] = y0[i] + 0.5f * dt * k2[i];
    dsdt(y, k3);
    for (int i = 0; i < 4; ++i) y[i] = y0[i] + dt * k3[i];
    dsdt(y, k4);
    float ns[4];
    for (int i = 0; i < 4; ++i) ns[i] = y0[i] + dt / 6.f * (k1[i] + 2.f * k2[i] + 2.f * k3[i] + k4[i]);
    const float pi = 3.14159265358979f;
    s[0] = wrap(ns[0]);
    s[1] = wrap(ns[1]);
    s[2] = fminf(fmaxf(ns[2], -4.f * pi), 4.f * pi);
    s[3] = fminf(fmaxf(ns[3], -9.f * pi), 9.f * pi);
    terminated = (-cosf(s[0]) - cosf(s[1] + s[0])) > 1.f;
    return terminated ? 0.f : -1.f;
  }
};

// LunarLanderSynth-v0: the same point-mass lander as the host VecEnv (csrc/host/vecenv.cpp
// LunarLanderSynth) -- 8 obs (x, y, vx, vy, angle, angular velocity, leg1, leg2), 4 actions
// (noop, left, main, right), gymnasium-style potential shaping and +-100 terminal bonus.
// The lateral noise draw comes from the kernel's Philox stream instead of the host Rng.
struct LunarLanderSynthEnv {
  static constexpr int D = 8, A = 4, NS = 7;  // x y vx vy ang angv prev_shaping
  static constexpr int kMaxSteps = 1000;
  RRL_DEV static float shaping(const float (&s)[NS]) {
    const float legs = s[1] < 0.05f ? 20.f : 0.f;
    return -100.f * sqrtf(s[0] * s[0] + s[1] * s[1]) - 100.f * sqrtf(s[2] * s[2] + s[3] * s[3]) -
           100.f * fabsf(s[4]) + legs;
  }
  RRL_DEV static void reset(float (&s)[NS], uint4 r) {
    s[0] = -0.3f + 0.6f * u01(r.x);
    s[1] = 1.4f;
    s[2] = -0.5f + 1.0f * u01(r.y);
    s[3] = -0.3f + 0.3f * u01(r.z);
    s[4] = -0.1f + 0.2f * u01(r.w);
    s[5] = 0.f;
    s[6] = shaping(s);
  }
  RRL_DEV static float obs(const float (&s)[NS], int f) {
    if (f < 6) return f == 0 ? s[0] : f == 1 ? s[1] : f == 2 ? s[2] : f == 3 ? s[3] : f == 4 ? s[4] : s[5];
    return s[1] < 0.05f ? 1.f : 0.f;
  }
  RRL_DEV static float step(float (&s)[NS], int a, bool& terminated, float noise01) {
    const float dt = 1.f / 50.f;
    float ax = 0.f, ay = -10.f / 6.f, aa = 0.f, fuel = 0.f;
    if (a == 2) {
      ax += -sinf(s[4]) * 13.f / 6.f;
      ay += cosf(s[4]) * 13.f / 6.f;
      fuel += 0.3f;
    } else if (a == 1 || a == 3) {
      const float dir = a == 1 ? -1.f : 1.f;
      ax += dir * cosf(s[4]) * 0.6f / 6.f;
      aa += -dir * 1.5f;
      fuel += 0.03f;
    }
    ax += -0.05f + 0.1f * noise01;
    s[2] += ax * dt * 6.f;
    s[3] += ay * dt * 6.f;
    s[5] += aa * dt;
    s[0] += s[2] * dt;
    s[1] += s[3] * dt;
    s[4] += s[5] * dt;
    const float sh = shaping(s);
    float rew = sh - s[6] - fuel;
    s[6] = sh;
    terminated = false;
    if (s[1] <= 0.f) {
      s[1] = 0.f;
      terminated = true;
      const bool soft = fabsf(s[3]) < 0.5f && fabsf(s[2]) < 0.5f && fabsf(s[4]) < 0.3f && fabsf(s[0]) < 0.5f;
      rew += soft ? 100.f : -100.f;
    } else if (fabsf(s[0]) >= 1.f) {
      terminated = true;
      rew -= 100.f;
    }
    return rew;
  }
};

// HalfCheetahSynth-v0: the host env's stable weakly non-linear system (csrc/host/vecenv.cpp)
// s' = tanh(A s + B clip(u, -1, 1)) + U(-0.01, 0.01), reward = s'[8] - 0.1 |clip(u)|^2,
// 17 obs, 6 continuous actions, 1000 steps.  A and B come from env_constants() and are
// staged in LDS; the noise comes from the kernel's Philox stream.
struct HalfCheetahSynthEnv {
  static constexpr int D = 17, A = 6, NS = 17;
  static constexpr int kMaxSteps = 1000;
  static constexpr int kConsts = 17 * 17 + 17 * 6;
  RRL_DEV static void reset(float (&s)[NS], uint2 key, uint32_t env, uint64_t step) {
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      const uint4 r = philox4x32(make_uint4(env, (uint32_t)step, (uint32_t)(step >> 32), 16u + q), key);
      const float u[4] = {u01(r.x), u01(r.y), u01(r.z), u01(r.w)};
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (4 * q + k < NS) s[4 * q + k] = -0.1f + 0.2f * u[k];
    }
  }
  RRL_DEV static float step(float (&s)[NS], const float (&a)[kMaxAct], const float* __restrict__ cst, uint2 key,
                            uint32_t env, uint64_t step) {
    float u[A], ctrl = 0.f;
#pragma unroll
    for (int j = 0; j < A; ++j) {
      u[j] = fminf(fmaxf(a[j], -1.f), 1.f);
      ctrl += u[j] * u[j];
    }
    float ns[NS];
#pragma unroll
    for (int i = 0; i < NS; ++i) {
      float v = 0.f;
#pragma unroll
      for (int j = 0; j < NS; ++j) v += cst[i * 17 + j] * s[j];
#pragma unroll
      for (int j = 0; j < A; ++j) v += cst[17 * 17 + i * 6 + j] * u[j];
      ns[i] = tanhf(v);
    }
#pragma unroll
    for (int q = 0; q < 5; ++q) {
      const uint4 r = philox4x32(make_uint4(env, (uint32_t)step, (uint32_t)(step >> 32), 8u + q), key);
      const float n[4] = {u01(r.x), u01(r.y), u01(r.z), u01(r.w)};
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (4 * q + k < NS) s[4 * q + k] = ns[4 * q + k] + (-0.01f + 0.02f * n[k]);
    }
    return s[8] - 0.1f * ctrl;
  }
};

}  // namespace rrl
