// PongSynth-v0 rendering shared by the env kernels (pong.hip) and the conv kernels that draw
// their input frames themselves from the 16-float frame history (cnn_fused.hip, fused render):
// the screen geometry and the renderer of one 16-byte chunk of the space-to-depth frame stack.
#pragma once
#include "common.h"

namespace rrl {

constexpr int kPongHW = 84;
constexpr float kTop = 2.f, kBot = 82.f, kPadHalf = 5.f, kBall = 2.f;
constexpr float kAgentX = 76.f, kOppX = 6.f, kPadW = 2.f;
constexpr int kPongHist = 16;      // floats of the frame history: 4 frames x (bx, by, pa, po), oldest first
constexpr int kPongChunks = 1764;  // 16-byte chunks of one [21][21][64] s2d frame stack

// One thread per (env, row): 84 pixels x 4 frames = 21 x 16 B.  The observation is
// written space-to-depth: obs[n][a][b][dy][dx][f] with y = 4a + dy, x = 4b + dx (i.e.
// [N][21][21][64]), so the first 8x8/4 conv becomes a 2x2/1 conv over 64 contiguous
// channels and its im2col reads 8-byte runs; a 16-byte chunk of 4 pixels x 4 frames of
// one row lands contiguously at (a, b, dy).
// One thread per 16-byte output chunk (4 pixels x 4 frames of one row), chunks in memory
// order, so every wave stores 1 KB contiguously.  Chunk q of an env's [21][21][64] s2d
// frame: a = q / 84 (block row), c = (q % 84) / 4 (block column), dy = q % 4 (row in the
// 4x4 block) -> image row y = 4a + dy, pixels x = 4c .. 4c+3.
// 16-byte chunk q (0 .. 1763) of one env's s2d frame stack from its (bx, by, pa, po) history h.
RRL_DEV uint4 pong_render_chunk(const float* h, int q) {
  const int a = q / 84, rem = q - a * 84, c = rem >> 2, dy = rem & 3;
  const float fy = (float)(4 * a + dy) + 0.5f;
  const bool wall = fy < kTop || fy >= kBot;
  uint32_t w[4] = {0u, 0u, 0u, 0u};
  // rows with nothing lit in any frame (most of the screen): the wall / background pattern
  // only -- whole waves skip the per-pixel tests below
  bool lit = false;
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    const float by = h[4 * f + 1], pa = h[4 * f + 2], po = h[4 * f + 3];
    lit |= (fy >= by && fy < by + kBall) || fabsf(fy - pa) < kPadHalf || fabsf(fy - po) < kPadHalf;
  }
  if (!lit) {
    const uint32_t v = wall ? 0x64646464u : 0u;
    return make_uint4(v, v, v, v);
  }
#pragma unroll
  for (int f = 0; f < 4; ++f) {
    const float bx = h[4 * f], by = h[4 * f + 1], pa = h[4 * f + 2], po = h[4 * f + 3];
    const bool b_on = fy >= by && fy < by + kBall;
    const bool pa_on = fabsf(fy - pa) < kPadHalf;
    const bool po_on = fabsf(fy - po) < kPadHalf;
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

}  // namespace rrl
