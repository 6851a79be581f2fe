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

// ----------------------------------------------------------------------------- frame ring
// The 4-frame stack of consecutive observations shares 3 frames, so the ring path renders ONE
// frame per env step into a frame store and describes an observation by the store rows of its 4
// frames (fidx[n][4], oldest first) -- 7 KB written per env step instead of 28 KB, and the
// frames of a rollout (T + 3 per env) are small enough to stay in the 256 MB MALL between the
// forward and the conv1 weight gradient that re-read them.
//
// A stored frame is one 84 x 84 image in space-to-depth order: frame[a][b][dy][dx] (y = 4a + dy,
// x = 4b + dx), 441 positions x 16 bytes, so the 16-byte chunk of position (a, b) is the 4 x 4
// block the observation's 64 channels interleave across frames (obs[a][b][dy][dx][f]).
constexpr int kPongFrameBytes = 7056;  // 441 x 16
constexpr int kPongFramePos = 441;

// the row-flag bits of one frame (bit 0 ball, 1 agent paddle, 2 opponent paddle, 3 wall):
// the same float comparisons as pong_row_flags / pong_render_chunk, so frames are bitwise the
// corresponding bytes of the 4-frame render
RRL_DEV uint32_t pong_frame_row_flags(float by, float pa, float po, int y) {
  const float fy = (float)y + 0.5f;
  uint32_t m = (fy < kTop || fy >= kBot) ? 8u : 0u;
  if (fy >= by && fy < by + kBall) m |= 1u;
  if (fabsf(fy - pa) < kPadHalf) m |= 2u;
  if (fabsf(fy - po) < kPadHalf) m |= 4u;
  return m;
}

// 16-byte chunk of s2d position pos (0 .. 440) of one frame with ball x bx, from its 84 row flags
RRL_DEV uint4 pong_frame_chunk(float bx, const uint32_t* rows, int pos) {
  const int a = pos / 21, b = pos - 21 * a;
  uint32_t w[4];
#pragma unroll
  for (int dy = 0; dy < 4; ++dy) {
    const uint32_t m = rows[4 * a + dy];
    const bool wall = (m >> 3) & 1u;
    if ((m & 7u) == 0u) {
      w[dy] = wall ? 0x64646464u : 0u;
      continue;
    }
    uint32_t v4 = 0u;
#pragma unroll
    for (int px = 0; px < 4; ++px) {
      const float fx = (float)(4 * b + px) + 0.5f;
      uint32_t v = wall ? 100u : 0u;
      if ((m & 2u) && fx >= kAgentX && fx < kAgentX + kPadW) v = 255u;
      if ((m & 4u) && fx >= kOppX && fx < kOppX + kPadW) v = 255u;
      if ((m & 1u) && fx >= bx && fx < bx + kBall) v = 255u;
      v4 |= v << (8 * px);
    }
    w[dy] = v4;
  }
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// Observation bytes from the frame ring: the 8-byte pieces (rows dy0, dy0 + 1 of one position) of
// frames 0..3 -> the two 16-byte s2d chunks (dy0, dy0 + 1) of the observation, whose byte
// 4 dx + f is frame f's pixel dx: a 4 x 4 byte transpose per row, 8 v_perm_b32 (perm(hi, lo, sel):
// selector bytes 0-3 pick lo's bytes, 4-7 hi's; the shift-and-mask form compiled to ~4x the VALU)
RRL_DEV uint4 pong_interleave_row(uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  const uint32_t ab_lo = __builtin_amdgcn_perm(b, a, 0x05010400u);  // a0 b0 a1 b1
  const uint32_t ab_hi = __builtin_amdgcn_perm(b, a, 0x07030602u);  // a2 b2 a3 b3
  const uint32_t cd_lo = __builtin_amdgcn_perm(d, c, 0x05010400u);  // c0 d0 c1 d1
  const uint32_t cd_hi = __builtin_amdgcn_perm(d, c, 0x07030602u);  // c2 d2 c3 d3
  return make_uint4(__builtin_amdgcn_perm(cd_lo, ab_lo, 0x05040100u), __builtin_amdgcn_perm(cd_lo, ab_lo, 0x07060302u),
                    __builtin_amdgcn_perm(cd_hi, ab_hi, 0x05040100u), __builtin_amdgcn_perm(cd_hi, ab_hi, 0x07060302u));
}

// The frame rows of one image, wave-uniform: moved to SGPRs so the frame addresses need no VGPRs
RRL_DEV int4 uniform_int4(int4 v) {
  return make_int4(__builtin_amdgcn_readfirstlane(v.x), __builtin_amdgcn_readfirstlane(v.y),
                   __builtin_amdgcn_readfirstlane(v.z), __builtin_amdgcn_readfirstlane(v.w));
}

// A persistent conv kernel over images n0, n0 + G, ... stages their frame rows in LDS once (a
// table of up to kRingTab entries): an image's frame loads then wait on an LDS read issued a
// stage earlier, not on a global load in front of them (the first ring forward, with a global fidx
// load ahead of each image's frame loads and shift-and-mask interleaving, ran 57.2 us per 2,048
// frames against 51.3 us on s2d observations).  Images past the table read fidx directly.
constexpr int kRingTab = 1024;
RRL_DEV int ring_images(int N, int n0, int G) { return n0 < N ? (N - n0 + G - 1) / G : 0; }
RRL_DEV void ring_stage_table(int4* tab, const int32_t* __restrict__ fidx, int N, int n0, int G, int tid, int nthreads) {
  const int cnt = min(ring_images(N, n0, G), kRingTab);
  for (int k = tid; k < cnt; k += nthreads) tab[k] = *reinterpret_cast<const int4*>(fidx + 4 * ((size_t)n0 + (size_t)k * G));
}
RRL_DEV int4 ring_row(const int4* tab, const int32_t* __restrict__ fidx, int n0, int G, int j) {
  return uniform_int4(j < kRingTab ? tab[j] : *reinterpret_cast<const int4*>(fidx + 4 * ((size_t)n0 + (size_t)j * G)));
}

// store row of a frame slot: frames are [R slots][N envs][7056 B]
RRL_DEV int pong_ring_slot(long long k, int R) { return (int)(((k % R) + R) % R); }

}  // namespace rrl
