// PongSynth-v0: a device-resident Pong with Atari-style pixel observations, the env of
// the A2C pixel configuration (BASELINE.json config 4; gymnasium/ALE are absent, so the
// env is synthetic but keeps the Atari interface: 6 actions, frame-skip 4, 84x84
// grayscale, 4 stacked frames, +-1 per point, episode ends at 21 points).
//
// One thread per env steps the physics (pong_step_kernel); a second kernel renders the
// 4-frame stack straight into the uint8 NHWC observation tensor the conv stack reads
// (channel f = frame f, oldest first), so observations never touch the host.
#include "common.h"
#include "pong_render.h"
#include "a2c_head.h"

namespace rrl {

constexpr int kPongState = 32;  // floats per env
// state layout
enum : int {
  P_BX = 0, P_BY, P_VX, P_VY, P_PA, P_PO, P_SA, P_SO, P_T, P_RET,
  P_VALID,     // distinct frames in the stack (1 after a reset .. 4): the frame ring's reset clamp
  P_HIST = 16  // 4 frames x (bx, by, pa, po)
};
constexpr float kPadSpeed = 2.5f, kOppSpeed = 1.6f, kMaxVy = 3.0f, kMaxVx = 3.0f;

RRL_DEV void serve(float* s, uint4 r) {
  s[P_BX] = 41.f;
  s[P_BY] = 30.f + 24.f * u01(r.x);
  s[P_VX] = (r.y & 1) ? 1.5f : -1.5f;
  s[P_VY] = (u01(r.z) - 0.5f) * 3.0f;
}

RRL_DEV void push_hist(float* s) {
#pragma unroll
  for (int f = 0; f < 3; ++f)
#pragma unroll
    for (int j = 0; j < 4; ++j) s[P_HIST + 4 * f + j] = s[P_HIST + 4 * (f + 1) + j];
  s[P_HIST + 12] = s[P_BX];
  s[P_HIST + 13] = s[P_BY];
  s[P_HIST + 14] = s[P_PA];
  s[P_HIST + 15] = s[P_PO];
}

RRL_DEV void reset_env(float* s, uint4 r) {
  for (int i = 0; i < kPongState; ++i) s[i] = 0.f;
  s[P_PA] = 42.f;
  s[P_PO] = 42.f;
  serve(s, r);
  for (int f = 0; f < 4; ++f) push_hist(s);
  s[P_VALID] = 1.f;
}

// One env's step (frame-skip 4); state row written back.  Shared by pong_step_kernel (one
// thread per env) and pong_step_render_kernel (one workgroup per env).
// s: the env's state row, in registers (pong_step_env) or in LDS (pong_step_render_kernel).
RRL_DEV void pong_step_state(int e, float* s, int a, float* __restrict__ rew,
                             float* __restrict__ done, float* __restrict__ fin_ret, float* __restrict__ fin_len,
                             float* __restrict__ ep_acc, uint2 key, uint32_t step_lo, uint32_t step_hi, int max_steps,
                             int reset_all, const unsigned long long* __restrict__ step_base) {
  if (step_base) {  // device step counter (graph replays): the host value is an offset
    const unsigned long long st = (((unsigned long long)step_hi << 32) | step_lo) + *step_base;
    step_lo = (uint32_t)st;
    step_hi = (uint32_t)(st >> 32);
  }
  const uint4 r0 = philox4x32(make_uint4((uint32_t)e, step_lo, step_hi, 0x51u), key);
  if (reset_all) {
    reset_env(s, r0);
  } else {
    const float dir = (a == 2 || a == 4) ? -1.f : ((a == 3 || a == 5) ? 1.f : 0.f);  // RIGHT = up, LEFT = down
    float reward = 0.f;
    bool point = false;
    for (int sub = 0; sub < 4 && !point; ++sub) {
      s[P_PA] = fminf(fmaxf(s[P_PA] + dir * kPadSpeed, kTop + kPadHalf), kBot - kPadHalf);
      // opponent tracks the ball when it approaches, drifts to centre otherwise
      const float target = s[P_VX] < 0.f ? s[P_BY] + 1.f : 42.f;
      const float d = fminf(fmaxf(target - s[P_PO], -kOppSpeed), kOppSpeed);
      s[P_PO] = fminf(fmaxf(s[P_PO] + d, kTop + kPadHalf), kBot - kPadHalf);
      float bx = s[P_BX] + s[P_VX], by = s[P_BY] + s[P_VY];
      if (by < kTop) { by = 2.f * kTop - by; s[P_VY] = -s[P_VY]; }
      if (by + kBall > kBot) { by = 2.f * (kBot - kBall) - by; s[P_VY] = -s[P_VY]; }
      const float cy = by + 0.5f * kBall;
      if (s[P_VX] > 0.f && bx + kBall >= kAgentX && s[P_BX] + kBall <= kAgentX + kPadW &&
          fabsf(cy - s[P_PA]) <= kPadHalf + 1.f) {
        bx = kAgentX - kBall;
        s[P_VX] = -fminf(fabsf(s[P_VX]) * 1.05f, kMaxVx);
        s[P_VY] = fminf(fmaxf(s[P_VY] + 0.35f * (cy - s[P_PA]), -kMaxVy), kMaxVy);
      } else if (s[P_VX] < 0.f && bx <= kOppX + kPadW && s[P_BX] >= kOppX && fabsf(cy - s[P_PO]) <= kPadHalf + 1.f) {
        bx = kOppX + kPadW;
        s[P_VX] = fminf(fabsf(s[P_VX]) * 1.05f, kMaxVx);
        s[P_VY] = fminf(fmaxf(s[P_VY] + 0.35f * (cy - s[P_PO]), -kMaxVy), kMaxVy);
      }
      s[P_BX] = bx;
      s[P_BY] = by;
      if (bx > (float)kPongHW) {  // opponent scores
        reward -= 1.f;
        s[P_SO] += 1.f;
        point = true;
      } else if (bx + kBall < 0.f) {  // agent scores
        reward += 1.f;
        s[P_SA] += 1.f;
        point = true;
      }
    }
    if (point) serve(s, r0);
    s[P_T] += 1.f;
    s[P_RET] += reward;
    push_hist(s);
    s[P_VALID] = fminf(s[P_VALID] + 1.f, 4.f);
    const bool over = s[P_SA] >= 21.f || s[P_SO] >= 21.f || (max_steps > 0 && s[P_T] >= (float)max_steps);
    rew[e] = reward;
    done[e] = over ? 1.f : 0.f;
    fin_ret[e] = over ? s[P_RET] : 0.f;
    fin_len[e] = over ? s[P_T] : 0.f;
    if (over && ep_acc) {  // per-env running episode statistics: count, sum ret, sum len, sum ret^2
      float* acc = ep_acc + 4 * (size_t)e;
      acc[0] += 1.f;
      acc[1] += s[P_RET];
      acc[2] += s[P_T];
      acc[3] += s[P_RET] * s[P_RET];
    }
    if (over) {
      const uint4 r1 = philox4x32(make_uint4((uint32_t)e, step_lo, step_hi, 0x52u), key);
      reset_env(s, r1);
    }
  }
}

RRL_DEV void pong_step_env(int e, float* __restrict__ state, const int32_t* __restrict__ act, float* __restrict__ rew,
                           float* __restrict__ done, float* __restrict__ fin_ret, float* __restrict__ fin_len,
                           float* __restrict__ ep_acc, uint2 key, uint32_t step_lo, uint32_t step_hi, int max_steps,
                           int reset_all, const unsigned long long* __restrict__ step_base, float* __restrict__ hist_out) {
  float s[kPongState];
#pragma unroll
  for (int i = 0; i < kPongState; ++i) s[i] = state[(size_t)e * kPongState + i];
  pong_step_state(e, s, reset_all ? 0 : act[e], rew, done, fin_ret, fin_len, ep_acc, key, step_lo, step_hi, max_steps, reset_all,
                  step_base);
#pragma unroll
  for (int i = 0; i < kPongState; ++i) state[(size_t)e * kPongState + i] = s[i];
  if (hist_out) {  // the new frame history: all a fused-render conv kernel needs to draw the observation
#pragma unroll
    for (int i = 0; i < kPongHist; i += 4)
      *reinterpret_cast<float4*>(hist_out + (size_t)e * kPongHist + i) =
          make_float4(s[P_HIST + i], s[P_HIST + i + 1], s[P_HIST + i + 2], s[P_HIST + i + 3]);
  }
}

__global__ void pong_step_kernel(float* __restrict__ state, const int32_t* __restrict__ act, float* __restrict__ rew,
                                 float* __restrict__ done, float* __restrict__ fin_ret, float* __restrict__ fin_len,
                                 float* __restrict__ ep_acc, int N, uint2 key, uint32_t step_lo, uint32_t step_hi, int max_steps,
                                 int reset_all, const unsigned long long* __restrict__ step_base,
                                 float* __restrict__ hist_out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= N) return;
  pong_step_env(e, state, act, rew, done, fin_ret, fin_len, ep_acc, key, step_lo, step_hi, max_steps, reset_all,
                step_base, hist_out);
}

// The row-only half of pong_render_chunk, once per image row y (84 per env instead of once per
// chunk: 21 chunks share a row): bit f = ball on the row in frame f, 4 + f = agent paddle,
// 8 + f = opponent paddle, 12 = wall.  Same float comparisons, so the render stays bitwise.
RRL_DEV uint32_t pong_row_flags(const float* h, int y) {
  const float fy = (float)y + 0.5f;
  uint32_t m = (fy < kTop || fy >= kBot) ? (1u << 12) : 0u;
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    const float by = h[4 * f + 1], pa = h[4 * f + 2], po = h[4 * f + 3];
    if (fy >= by && fy < by + kBall) m |= 1u << f;
    if (fabsf(fy - pa) < kPadHalf) m |= 1u << (4 + f);
    if (fabsf(fy - po) < kPadHalf) m |= 1u << (8 + f);
  }
  return m;
}

// pong_render_chunk from the per-row flags: an unlit row (most of the screen) is one LDS read
// and a constant; lit rows keep only the per-pixel x tests.
RRL_DEV uint4 pong_render_chunk_rows(const float* h, const uint32_t* rows, int q) {
  const int a = q / 84, rem = q - a * 84, c = rem >> 2, dy = rem & 3;
  const uint32_t m = rows[4 * a + dy];
  const bool wall = (m >> 12) & 1u;
  if ((m & 0xfffu) == 0u) {
    const uint32_t v = wall ? 0x64646464u : 0u;
    return make_uint4(v, v, v, v);
  }
  uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    const float bx = h[4 * f];
    const bool b_on = (m >> f) & 1u, pa_on = (m >> (4 + f)) & 1u, po_on = (m >> (8 + f)) & 1u;
#pragma unroll
    for (int px = 0; px < 4; ++px) {
      const float fx = (float)(4 * c + px) + 0.5f;
      uint32_t v = wall ? 100u : 0u;
      if (pa_on && fx >= kAgentX && fx < kAgentX + kPadW) v = 255u;
      if (po_on && fx >= kOppX && fx < kOppX + kPadW) v = 255u;
      if (b_on && fx >= bx && fx < bx + kBall) v = 255u;
      w[px] |= v << (8 * f);
    }
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

__global__ void pong_render_kernel(const float* __restrict__ state, uint8_t* __restrict__ obs, int N) {
  constexpr int kChunks = kPongHW * kPongHW * 4 / 16;  // 1764 per env
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (t >= (size_t)N * kChunks) return;
  const int e = (int)(t / kChunks), q = (int)(t % kChunks);
  *reinterpret_cast<uint4*>(obs + t * 16) = pong_render_chunk(state + (size_t)e * kPongState + P_HIST, q);
}

// Frame-ring output of a step launch (pong_render.h): frames [R][N][7056] and the frame rows of
// each env's new observation, fidx[N][4] (oldest first); frames == nullptr: no ring
struct RingOut {
  uint8_t* frames;
  int32_t* fidx;
  int R;
};

RRL_DEV long long pong_abs_step(uint32_t lo, uint32_t hi, const unsigned long long* base) {
  unsigned long long st = ((unsigned long long)hi << 32) | lo;
  if (base) st += *base;
  return (long long)st;
}

// Env e's workgroup (grid = N envs, state already stepped in LDS) writes the newest frame of its
// history into slot st and the observation's 4 frame rows: frame f is the one of step st - (3 - f),
// clamped to the env's last reset (P_VALID distinct frames), so a reset needs no re-render of older
// slots -- which the earlier observations of the same rollout still read.
RRL_DEV void pong_ring_write(const RingOut& ro, int e, int N, const float* ss, uint32_t* rows, long long st) {
  const float* h3 = ss + P_HIST + 12;  // the newest frame (bx, by, pa, po)
  const int t = threadIdx.x;
  if (t < kPongHW) rows[t] = pong_frame_row_flags(h3[1], h3[2], h3[3], t);
  if (t < 4) {
    const int valid = (int)ss[P_VALID];
    const int age = min(3 - t, max(valid, 1) - 1);
    ro.fidx[4 * (size_t)e + t] = pong_ring_slot(st - age, ro.R) * N + e;
  }
  __syncthreads();
  uint8_t* fo = ro.frames + ((size_t)pong_ring_slot(st, ro.R) * N + e) * kPongFrameBytes;
  for (int q = t; q < kPongFramePos; q += blockDim.x)
    *reinterpret_cast<uint4*>(fo + 16 * q) = pong_frame_chunk(h3[0], rows, q);
}

// The ring rebuilt from the env state alone (a restored checkpoint / elastic snapshot): the 4-frame
// stack IS a function of the 16-float history, so frames 0..3 of every env are drawn into slots
// st - 3 .. st and the observation points at them.  The slots now hold 4 frames of history each,
// so the env's distinct-frame count becomes 4 (a checkpoint from before the count existed has 0
// there; a recently reset env's older history frames are copies of its reset frame, so pointing at
// them is the same observation).  One workgroup per env.
__global__ void __launch_bounds__(256) pong_ring_fill_kernel(float* __restrict__ state, RingOut ro,
                                                             uint32_t step_lo, uint32_t step_hi,
                                                             const unsigned long long* __restrict__ step_base) {
  __shared__ uint32_t rows[4][kPongHW];
  __shared__ float hv[kPongHist];
  const int e = blockIdx.x, N = gridDim.x, t = threadIdx.x;
  if (t < kPongHist) hv[t] = state[(size_t)e * kPongState + P_HIST + t];
  if (t == 0) state[(size_t)e * kPongState + P_VALID] = 4.f;
  __syncthreads();
  const long long st = pong_abs_step(step_lo, step_hi, step_base);
  for (int q = t; q < 4 * kPongHW; q += 256) {
    const int f = q / kPongHW, y = q - f * kPongHW;
    rows[f][y] = pong_frame_row_flags(hv[4 * f + 1], hv[4 * f + 2], hv[4 * f + 3], y);
  }
  if (t < 4) ro.fidx[4 * (size_t)e + t] = pong_ring_slot(st - 3 + t, ro.R) * N + e;
  __syncthreads();
  for (int q = t; q < 4 * kPongFramePos; q += 256) {
    const int f = q / kPongFramePos, p = q - f * kPongFramePos;
    uint8_t* fo = ro.frames + ((size_t)pong_ring_slot(st - 3 + f, ro.R) * N + e) * kPongFrameBytes;
    *reinterpret_cast<uint4*>(fo + 16 * p) = pong_frame_chunk(hv[4 * f], rows[f], p);
  }
}

// Step + render in one launch: workgroup e steps env e on one thread (the physics is a short
// serial chain) and renders its 1,764 chunks on all 256 threads from the new history in LDS.
// One launch per env step instead of two, and the tiny step kernel's own launch / drain is gone.
template <bool RING>
__global__ void __launch_bounds__(256, 8) pong_step_render_kernel(
    float* __restrict__ state, const int32_t* __restrict__ act, float* __restrict__ rew, float* __restrict__ done,
    float* __restrict__ fin_ret, float* __restrict__ fin_len, float* __restrict__ ep_acc, uint8_t* __restrict__ obs,
    uint2 key, uint32_t step_lo, uint32_t step_hi, int max_steps, int reset_all,
    const unsigned long long* __restrict__ step_base, RingOut ro) {
  constexpr int kChunks = kPongHW * kPongHW * 4 / 16;
  __shared__ float ss[kPongState];
  __shared__ uint32_t rows[kPongHW];
  const int e = blockIdx.x, t = threadIdx.x;
  // the state row moves in and out as one coalesced access and thread 0 steps it in LDS: held
  // in registers it set the kernel at 67 VGPRs = 7 waves per SIMD, so 1/8 of the 2,048
  // workgroups of a step waited for a second round
  if (t < kPongState) ss[t] = state[(size_t)e * kPongState + t];
  __syncthreads();
  if (t == 0)
    pong_step_state(e, ss, reset_all ? 0 : act[e], rew, done, fin_ret, fin_len, ep_acc, key, step_lo, step_hi, max_steps, reset_all,
                    step_base);
  __syncthreads();
  if (t < kPongState) state[(size_t)e * kPongState + t] = ss[t];
  if constexpr (RING) {  // one new frame + the observation's frame rows
    pong_ring_write(ro, e, gridDim.x, ss, rows, pong_abs_step(step_lo, step_hi, step_base));
    return;
  }
  const float* hist = ss + P_HIST;
  // the render is VALU-bound (every chunk re-tested its row against 12 objects): the row tests
  // once per row here, the chunks then read them (21 chunks per row)
  if (t < kPongHW) rows[t] = pong_row_flags(hist, t);
  __syncthreads();
  uint8_t* o = obs + (size_t)e * kChunks * 16;
  for (int q = threadIdx.x; q < kChunks; q += 256)
    *reinterpret_cast<uint4*>(o + (size_t)q * 16) = pong_render_chunk_rows(hist, rows, q);
}


// The rollout step's policy head fused in front of the env step: one workgroup per env, wave 0
// forms the env's hidden row from the fc split-K partials and samples its action
// (a2c_rollout_row_streamed: bitwise the a2c_head_kernel result), thread 0 steps the physics
// with it, and the workgroup renders the new frame stack -- one launch instead of head + step
// (the head launch was ~10 us per rollout step at 2,048 envs, mostly its fixed cost).
template <int AMAX, bool WLDS, bool RING = false>
__global__ void __launch_bounds__(256, 8) pong_head_step_render_kernel(
    HeadArgs ha, float* __restrict__ state, float* __restrict__ rew, float* __restrict__ done,
    float* __restrict__ fin_ret, float* __restrict__ fin_len, float* __restrict__ ep_acc, uint8_t* __restrict__ obs,
    uint2 key, uint32_t step_lo, uint32_t step_hi, int max_steps, const unsigned long long* __restrict__ step_base,
    RingOut ro) {
  constexpr int kChunks = kPongHW * kPongHW * 4 / 16;
  __shared__ float ss[kPongState];
  __shared__ uint32_t rows[kPongHW];
  __shared__ int pick_s;
  const int e = blockIdx.x, t = threadIdx.x;
  if (t < kPongState) ss[t] = state[(size_t)e * kPongState + t];
  if constexpr (WLDS) {
    // waves 1-3 copy the head weights (w_v, then the A policy rows) into LDS while wave 0 sums
    // the fc partials: one L2 round trip instead of one per output row (RRL_PONG_HEAD_WLDS)
    __shared__ __attribute__((aligned(16))) float wl[(AMAX + 1) * kHeadF];
    const int nf4 = (ha.A + 1) * (kHeadF / 4);
    for (int i = t - 64; i >= 0 && i < nf4; i += 192) {
      const float* src = i < kHeadF / 4 ? ha.w_v + 4 * i : ha.w + 4 * (i - kHeadF / 4);
      *reinterpret_cast<float4*>(wl + 4 * i) = *reinterpret_cast<const float4*>(src);
    }
    __syncthreads();
    if (t < 64) {
      const int pick = a2c_rollout_row_streamed<AMAX>(ha, e, t, wl, wl + kHeadF);
      if (t == 0) pick_s = pick;
    }
  } else if (t < 64) {
    const int pick = a2c_rollout_row_streamed<AMAX>(ha, e, t);
    if (t == 0) pick_s = pick;
  }
  __syncthreads();
  if (t == 0)
    pong_step_state(e, ss, pick_s, rew, done, fin_ret, fin_len, ep_acc, key, step_lo, step_hi, max_steps, 0, step_base);
  __syncthreads();
  if (t < kPongState) state[(size_t)e * kPongState + t] = ss[t];
  if constexpr (RING) {
    pong_ring_write(ro, e, gridDim.x, ss, rows, pong_abs_step(step_lo, step_hi, step_base));
    return;
  }
  const float* hist = ss + P_HIST;
  if (t < kPongHW) rows[t] = pong_row_flags(hist, t);
  __syncthreads();
  uint8_t* o = obs + (size_t)e * kChunks * 16;
  for (int q = threadIdx.x; q < kChunks; q += 256)
    *reinterpret_cast<uint4*>(o + (size_t)q * 16) = pong_render_chunk_rows(hist, rows, q);
}
}  // namespace rrl

using namespace rrl;

extern "C" {

int rrl_pong_state_size() { return kPongState; }

int rrl_pong_step(float* state, const int32_t* act, float* rew, float* done, float* fin_ret, float* fin_len,
                  float* ep_acc, int N, unsigned long long seed, unsigned long long step,
                  const unsigned long long* step_base, int max_steps, int reset_all, float* hist_out, void* stream_) {
  hipStream_t st = (hipStream_t)stream_;
  const uint2 key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
  hipLaunchKernelGGL(pong_step_kernel, dim3((N + 255) / 256), dim3(256), 0, st, state, act, rew, done, fin_ret,
                     fin_len, ep_acc, N, key, (uint32_t)step, (uint32_t)(step >> 32), max_steps, reset_all,
                     step_base, hist_out);
  return (int)hipGetLastError();
}

// frames != nullptr: the frame-ring form (frames [R][N][7056], fidx [N][4]; obs unused)
int rrl_pong_step_render(float* state, const int32_t* act, float* rew, float* done, float* fin_ret, float* fin_len,
                         float* ep_acc, uint8_t* obs, int N, unsigned long long seed, unsigned long long step,
                         const unsigned long long* step_base, int max_steps, int reset_all, uint8_t* frames,
                         int32_t* fidx, int R, void* stream_) {
  hipStream_t st = (hipStream_t)stream_;
  if (N < 1) return 0;
  if (frames && (!fidx || R < 5)) return -1;
  const uint2 key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
  const RingOut ro{frames, fidx, R};
  if (frames)
    hipLaunchKernelGGL(pong_step_render_kernel<true>, dim3(N), dim3(256), 0, st, state, act, rew, done, fin_ret, fin_len,
                       ep_acc, obs, key, (uint32_t)step, (uint32_t)(step >> 32), max_steps, reset_all, step_base, ro);
  else
    hipLaunchKernelGGL(pong_step_render_kernel<false>, dim3(N), dim3(256), 0, st, state, act, rew, done, fin_ret, fin_len,
                       ep_acc, obs, key, (uint32_t)step, (uint32_t)(step >> 32), max_steps, reset_all, step_base, ro);
  return (int)hipGetLastError();
}

// the ring rebuilt from the env state (restore): frames of steps st - 3 .. st and fidx [N][4]
int rrl_pong_ring_fill(float* state, uint8_t* frames, int32_t* fidx, int N, int R, unsigned long long step,
                       const unsigned long long* step_base, void* stream_) {
  if (N < 1) return 0;
  if (!frames || !fidx || R < 5) return -1;
  hipLaunchKernelGGL(pong_ring_fill_kernel, dim3(N), dim3(256), 0, (hipStream_t)stream_, state, RingOut{frames, fidx, R},
                     (uint32_t)step, (uint32_t)(step >> 32), step_base);
  return (int)hipGetLastError();
}

// obs[n] drawn from the frame-history rows hist[n][16] (the fused-render path's reference)
__global__ void pong_render_hist_kernel(const float* __restrict__ hist, uint8_t* __restrict__ obs, int N) {
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (t >= (size_t)N * kPongChunks) return;
  const int e = (int)(t / kPongChunks), q = (int)(t % kPongChunks);
  *reinterpret_cast<uint4*>(obs + t * 16) = pong_render_chunk(hist + (size_t)e * kPongHist, q);
}

int rrl_pong_render_hist(const float* hist, uint8_t* obs, int N, void* stream_) {
  const size_t t = (size_t)N * kPongChunks;
  hipLaunchKernelGGL(pong_render_hist_kernel, dim3((unsigned)((t + 255) / 256)), dim3(256), 0, (hipStream_t)stream_,
                     hist, obs, N);
  return (int)hipGetLastError();
}

int rrl_pong_render(const float* state, uint8_t* obs, int N, void* stream_) {
  hipStream_t st = (hipStream_t)stream_;
  const size_t t = (size_t)N * (kPongHW * kPongHW * 4 / 16);
  hipLaunchKernelGGL(pong_render_kernel, dim3((unsigned)((t + 255) / 256)), dim3(256), 0, st, state, obs, N);
  return (int)hipGetLastError();
}


// Fused rollout step: head (from the fc split-K partials part[splits][N][512]) + env step +
// render.  head_params = [A x 512 policy rows | A biases | 512 value row | value bias].
int rrl_pong_head_step_render(const float* part, int splits, const float* fc_b, const float* head_params, int A,
                              uint16_t* h_out, int32_t* act, float* logp, float* value, unsigned long long sample_seed,
                              unsigned long long sample_step, const unsigned long long* sample_base, float* state,
                              float* rew, float* done, float* fin_ret, float* fin_len, float* ep_acc, uint8_t* obs,
                              int N, unsigned long long seed, unsigned long long step,
                              const unsigned long long* step_base, int max_steps, uint8_t* frames, int32_t* fidx,
                              int R, void* stream_) {
  if (N < 1 || A < 1 || A > 8 || splits < 1 || !part || !fc_b || !h_out) return -1;
  if (frames && (!fidx || R < 5)) return -1;
  const RingOut ro{frames, fidx, R};
  HeadArgs a = {};
  a.part = part;
  a.splits = splits;
  a.fc_b = fc_b;
  a.h_out = h_out;
  a.w = head_params;
  a.bias = head_params + A * kHeadF;
  a.w_v = a.bias + A;
  a.b_v = a.w_v + kHeadF;
  a.B = N;
  a.A = A;
  a.act = act;
  a.logp = logp;
  a.value = value;
  a.seed_lo = (uint32_t)sample_seed;
  a.seed_hi = (uint32_t)(sample_seed >> 32);
  a.step_lo = (uint32_t)sample_step;
  a.step_hi = (uint32_t)(sample_step >> 32);
  a.step_base = sample_base;
  const uint2 key = make_uint2((uint32_t)seed, (uint32_t)(seed >> 32));
  const char* wl_env = getenv("RRL_PONG_HEAD_WLDS");
  if (frames) {  // frame ring: one new frame per env
    hipLaunchKernelGGL((pong_head_step_render_kernel<8, false, true>), dim3(N), dim3(256), 0, (hipStream_t)stream_, a, state,
                       rew, done, fin_ret, fin_len, ep_acc, obs, key, (uint32_t)step, (uint32_t)(step >> 32), max_steps,
                       step_base, ro);
  } else if (wl_env && wl_env[0] == '1') {  // the head weights through LDS (A/B)
    hipLaunchKernelGGL((pong_head_step_render_kernel<8, true>), dim3(N), dim3(256), 0, (hipStream_t)stream_, a, state, rew, done,
                       fin_ret, fin_len, ep_acc, obs, key, (uint32_t)step, (uint32_t)(step >> 32), max_steps, step_base, ro);
  } else {
    hipLaunchKernelGGL((pong_head_step_render_kernel<8, false>), dim3(N), dim3(256), 0, (hipStream_t)stream_, a, state, rew, done,
                       fin_ret, fin_len, ep_acc, obs, key, (uint32_t)step, (uint32_t)(step >> 32), max_steps, step_base, ro);
  }
  return (int)hipGetLastError();
}

}  // extern "C"
