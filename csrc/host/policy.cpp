#include "policy.h"

#include <algorithm>
#include <cmath>
#include <stdexcept>

// target_clones dispatches through IFUNC resolvers, which run during relocation --
// before the ThreadSanitizer runtime is up -- so TSan builds use the default clone.
#if defined(__SANITIZE_THREAD__)
#define RRL_TARGET_CLONES
#else
#define RRL_TARGET_CLONES __attribute__((target_clones("avx512f", "avx2", "default")))
#endif

namespace rrl {

namespace {
inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
uint64_t splitmix(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// y[O] = act(b + x[I] @ Wt[I][O]).  Outputs in blocks of 64 whose accumulators stay in
// registers across the whole input loop (4 zmm / 8 ymm), so each weight row is one streamed
// load + FMA; the plain axpy form stored and reloaded y on every input (128 x 128 layer:
// 1.12-1.24 -> 0.73-0.80 us at batch 1).  target_clones picks AVX-512 / AVX2 at load time.
RRL_TARGET_CLONES void dense(const float* __restrict x, int I, const float* __restrict wt,
                             const float* __restrict b, int O, float* __restrict y, bool relu) {
  constexpr int kB = 64;
  int o0 = 0;
  for (; o0 + kB <= O; o0 += kB) {
    float acc[kB];
    for (int k = 0; k < kB; ++k) acc[k] = b[o0 + k];
    for (int i = 0; i < I; ++i) {
      const float xi = x[i];
      const float* w = wt + static_cast<size_t>(i) * O + o0;
#pragma GCC unroll 64
      for (int k = 0; k < kB; ++k) acc[k] += xi * w[k];
    }
    for (int k = 0; k < kB; ++k) y[o0 + k] = relu ? (acc[k] > 0.f ? acc[k] : 0.f) : acc[k];
  }
  if (o0 == O) return;
  for (int o = o0; o < O; ++o) y[o] = b[o];
  for (int i = 0; i < I; ++i) {
    const float xi = x[i];
    const float* w = wt + static_cast<size_t>(i) * O;
    for (int o = o0; o < O; ++o) y[o] += xi * w[o];
  }
  if (relu)
    for (int o = o0; o < O; ++o) y[o] = y[o] > 0.f ? y[o] : 0.f;
}

// y[O] = b + W[O][I] @ x for a narrow head (the action logits, the value): one vectorised dot
// product per output -- through dense()'s tail each output was a serial chain of I FMAs on y[o]
RRL_TARGET_CLONES void dense_dot(const float* __restrict x, int I, const float* __restrict w,
                                 const float* __restrict b, int O, float* __restrict y) {
  for (int o = 0; o < O; ++o) {
    const float* wr = w + static_cast<size_t>(o) * I;
    float part[16] = {};
    int i = 0;
    for (; i + 16 <= I; i += 16)
#pragma GCC unroll 16
      for (int k = 0; k < 16; ++k) part[k] += x[i + k] * wr[i + k];
    float s = 0.f;
    for (; i < I; ++i) s += x[i] * wr[i];
    for (int k = 0; k < 16; ++k) s += part[k];
    y[o] = b[o] + s;
  }
}
}  // namespace

NativePolicy::NativePolicy(int D_, int H_, int A_, bool disc, uint64_t seed) : D(D_), H(H_), A(A_), discrete(disc) {
  if (D <= 0 || H <= 0 || A <= 0) throw std::invalid_argument("NativePolicy: dims must be positive");
  uint64_t s = seed;
  for (auto& w : s_) w = splitmix(s);
  h1_.resize(H);
  h2_.resize(H);
  z_.resize(A);
}

void NativePolicy::unpack(Net& n, const float* p, int D, int H, int O, bool gaussian) {
  auto transpose = [](const float* w, int rows, int cols, std::vector<float>& out) {  // w [rows][cols] -> [cols][rows]
    out.assign(static_cast<size_t>(rows) * cols, 0.f);
    for (int r = 0; r < rows; ++r)
      for (int c = 0; c < cols; ++c) out[static_cast<size_t>(c) * rows + r] = w[static_cast<size_t>(r) * cols + c];
  };
  transpose(p, H, D, n.w1t);
  p += static_cast<size_t>(H) * D;
  n.b1.assign(p, p + H);
  p += H;
  transpose(p, H, H, n.w2t);
  p += static_cast<size_t>(H) * H;
  n.b2.assign(p, p + H);
  p += H;
  transpose(p, O, H, n.w3t);
  n.w3.assign(p, p + static_cast<size_t>(O) * H);
  p += static_cast<size_t>(O) * H;
  n.b3.assign(p, p + O);
  p += O;
  if (gaussian) n.log_std.assign(p, p + O);
  else n.log_std.clear();
}

void NativePolicy::load(const float* pi, int64_t n_pi, const float* vf, int64_t n_vf) {
  const int64_t base = static_cast<int64_t>(H) * D + H + static_cast<int64_t>(H) * H + H;
  const int64_t want_pi = base + static_cast<int64_t>(A) * H + A + (discrete ? 0 : A);
  if (n_pi != want_pi) throw std::invalid_argument("NativePolicy: policy vector has wrong size");
  unpack(pi_, pi, D, H, A, !discrete);
  has_vf_ = vf != nullptr && n_vf > 0;
  if (has_vf_) {
    if (n_vf != base + H + 1) throw std::invalid_argument("NativePolicy: value vector has wrong size");
    unpack(vf_, vf, D, H, 1, false);
  }
}

void NativePolicy::trunk(const Net& n, int O, const float* x, float* out, float* h1, float* h2) const {
  dense(x, D, n.w1t.data(), n.b1.data(), H, h1, true);
  dense(h1, H, n.w2t.data(), n.b2.data(), H, h2, true);
  if (O < 16) dense_dot(h2, H, n.w3.data(), n.b3.data(), O, out);
  else dense(h2, H, n.w3t.data(), n.b3.data(), O, out, false);
}

double NativePolicy::uniform() {  // xoshiro256+ -> [0, 1)
  const uint64_t r = s_[0] + s_[3];
  const uint64_t t = s_[1] << 17;
  s_[2] ^= s_[0];
  s_[3] ^= s_[1];
  s_[1] ^= s_[2];
  s_[0] ^= s_[3];
  s_[2] ^= t;
  s_[3] = rotl(s_[3], 45);
  return static_cast<double>(r >> 11) * 0x1.0p-53;
}

double NativePolicy::normal() {
  if (have_spare_) {
    have_spare_ = false;
    return spare_;
  }
  double u1 = uniform(), u2 = uniform();
  if (u1 < 1e-300) u1 = 1e-300;
  const double r = std::sqrt(-2.0 * std::log(u1)), th = 6.283185307179586 * u2;
  spare_ = r * std::sin(th);
  have_spare_ = true;
  return r * std::cos(th);
}

void NativePolicy::logits(const float* obs, int N, float* out) const {
  std::vector<float> h1(H), h2(H);
  for (int r = 0; r < N; ++r) trunk(pi_, A, obs + static_cast<size_t>(r) * D, out + static_cast<size_t>(r) * A,
                                    h1.data(), h2.data());
}

void NativePolicy::value(const float* obs, int N, float* out) const {
  if (!has_vf_) throw std::runtime_error("NativePolicy: no value network loaded");
  std::vector<float> h1(H), h2(H);
  for (int r = 0; r < N; ++r) trunk(vf_, 1, obs + static_cast<size_t>(r) * D, out + r, h1.data(), h2.data());
}

void NativePolicy::step(const float* obs, const float* mask, int N, int32_t* act_i, float* act_f, float* logp,
                        float* v) {
  std::vector<float>&h1 = h1_, &h2 = h2_, &z = z_;
  constexpr double kHalfLog2Pi = 0.9189385332046727;
  for (int r = 0; r < N; ++r) {
    const float* x = obs + static_cast<size_t>(r) * D;
    trunk(pi_, A, x, z.data(), h1.data(), h2.data());
    if (discrete) {
      if (mask)
        for (int a = 0; a < A; ++a) z[a] += (mask[static_cast<size_t>(r) * A + a] - 1.f) * 1e8f;
      float m = z[0];
      for (int a = 1; a < A; ++a) m = std::max(m, z[a]);
      double se = 0.0;
      for (int a = 0; a < A; ++a) se += std::exp(static_cast<double>(z[a] - m));
      const double lse = std::log(se);
      const double u = uniform();
      double c = 0.0;
      int pick = A - 1;
      for (int a = 0; a < A; ++a) {
        c += std::exp(static_cast<double>(z[a] - m) - lse);
        if (u < c) {
          pick = a;
          break;
        }
      }
      act_i[r] = pick;
      logp[r] = static_cast<float>(static_cast<double>(z[pick] - m) - lse);
    } else {
      double lp = 0.0;
      for (int a = 0; a < A; ++a) {
        const double ls = pi_.log_std[a], e = normal();
        act_f[static_cast<size_t>(r) * A + a] = static_cast<float>(z[a] + std::exp(ls) * e);
        lp += -0.5 * e * e - ls - kHalfLog2Pi;
      }
      logp[r] = static_cast<float>(lp);
    }
    if (v && has_vf_) trunk(vf_, 1, x, v + r, h1.data(), h2.data());
  }
}

}  // namespace rrl
