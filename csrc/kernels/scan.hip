// Discounted-return / GAE scans and advantage statistics (K7, K8, K9 of SURVEY §2.6).
//
// Reference: discount_cumsum = scipy.signal.lfilter reversed (BaseReplayBuffer.py:12-27)
// applied per finished path in ReplayBuffer.finish_path (replay_buffer.py:48-79):
//   with baseline   : adv = disc(r + g*V' - V, g*lam), ret = disc(r ++ [last_val], g)[:-1]
//   without baseline: adv = disc(r, g*lam),           ret = disc(r, g)
// Both are reverse linear recurrences y_t = b_t + a_t * y_{t+1} with a_t = 0 at a
// path end.  done codes: 0 = running, 1 = terminal (bootstrap 0), 2 = time-limit
// truncation (bootstrap with V of the pre-reset observation, tval[t]) -- the reference
// bootstraps its cut paths with last_val (replay_buffer.py:48-79, REINFORCE.py:86).
// Two layouts are supported:
//   * time-major [T][N] rollouts from the vectorised actors: one thread per env column,
//     sequential in t (coalesced across envs) -- T is short, N is huge.  A learner shard
//     fed by K actors holds K such blocks back to back ([K][T][N], each received whole
//     over its own link), with the K x N bootstrap values after all of them;
//   * flat [L] buffers of concatenated variable-length paths (the agent/trajectory API):
//     a 3-phase parallel affine scan (thread chunk -> block scan -> block carries).
#include "common.h"

namespace rrl {

struct ScanTM {
  const float* rew;    // [K][T][N]
  const float* done;   // [K][T][N]  (0 running / 1 terminal / 2 truncated)
  const float* val;    // [K*T*N + K*N] or null: V of every step, then V(s_T) of each column
  const float* tval;   // [K][T][N] V(pre-reset obs), read where done == 2, or null
  float* adv;          // [K][T][N]
  float* ret;          // [K][T][N]
  float* stats_part;   // [nblocks][3] adv sum / sumsq / count
  int T, N, K;
  float gamma, lam;
  long long* cnt[3];   // device step counters advanced by block 0 (the Pong update's sampling /
  long long inc[3];    // env / Adam counters: one launch fewer per update), ncnt of them
  int ncnt;
};

__global__ __launch_bounds__(256) void gae_scan_tm_kernel(ScanTM p) {
  if (blockIdx.x == 0 && (int)threadIdx.x < p.ncnt) p.cnt[threadIdx.x][0] += p.inc[threadIdx.x];
  const int col = blockIdx.x * blockDim.x + threadIdx.x;  // column = block k, env n
  float s = 0.f, ss = 0.f, c = 0.f;
  if (col < p.K * p.N) {
    const float gl = p.gamma * p.lam;
    const size_t N = (size_t)p.N;
    const int k = col / p.N;
    const size_t base = (size_t)k * p.T * N + (col - k * p.N);
    if (p.val != nullptr) {
      float v_next = p.val[(size_t)p.K * p.T * N + col];
      float adv_next = 0.f, ret_next = v_next;
      for (int t = p.T - 1; t >= 0; --t) {
        const size_t idx = base + (size_t)t * N;
        const float r = p.rew[idx], d = p.done[idx], v = p.val[idx];
        const float nd = d == 0.f ? 1.f : 0.f;
        const float vb = (d > 1.5f && p.tval != nullptr) ? p.tval[idx] : 0.f;  // truncation bootstrap
        const float delta = r + p.gamma * (v_next * nd + vb) - v;
        const float a = delta + gl * nd * adv_next;
        const float rt = r + p.gamma * (nd * ret_next + vb);
        p.adv[idx] = a;
        p.ret[idx] = rt;
        s += a;
        ss += a * a;
        adv_next = a;
        ret_next = rt;
        v_next = v;
      }
    } else {
      float adv_next = 0.f, ret_next = 0.f;
      for (int t = p.T - 1; t >= 0; --t) {
        const size_t idx = base + (size_t)t * N;
        const float r = p.rew[idx], d = p.done[idx];
        const float nd = d == 0.f ? 1.f : 0.f;  // no value function: truncation cuts like a terminal
        const float a = r + gl * nd * adv_next;
        const float rt = r + p.gamma * nd * ret_next;
        p.adv[idx] = a;
        p.ret[idx] = rt;
        s += a;
        ss += a * a;
        adv_next = a;
        ret_next = rt;
      }
    }
    c = (float)p.T;
  }
  // block reduction of the advantage statistics
  __shared__ float red[3][4];
  s = wave_sum(s);
  ss = wave_sum(ss);
  c = wave_sum(c);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = s;
    red[1][w] = ss;
    red[2][w] = c;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    const int nw = blockDim.x >> 6;
    float v = 0.f;
    for (int k = 0; k < nw; ++k) v += red[threadIdx.x][k];
    p.stats_part[blockIdx.x * 3 + threadIdx.x] = v;
  }
}

// Deterministic final reduction of [nparts][3] partials into out[3] (single block).
__global__ __launch_bounds__(256) void stats_reduce_kernel(const float* part, int nparts, float* out) {
  __shared__ float red[3][4];
  float acc[3] = {0.f, 0.f, 0.f};
  for (int k = threadIdx.x; k < nparts; k += blockDim.x) {
    acc[0] += part[k * 3 + 0];
    acc[1] += part[k * 3 + 1];
    acc[2] += part[k * 3 + 2];
  }
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const float v = wave_sum(acc[q]);
    if ((threadIdx.x & 63) == 0) red[q][w] = v;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    float v = 0.f;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) v += red[threadIdx.x][k];
    out[threadIdx.x] = v;
  }
}

// Column sums, in double, of the first `cols` (<= 8) columns of a [rows][ld] fp32 array (single
// block; the per-epoch episode sums of the threshold check: one launch where a strided torch
// reduction + cast were two at ~14 us).
__global__ __launch_bounds__(256) void column_sums_kernel(const float* part, int rows, int ld, int cols, double* out) {
  __shared__ double red[8][4];
  double acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int k = threadIdx.x; k < rows; k += blockDim.x)
#pragma unroll
    for (int q = 0; q < 8; ++q)
      if (q < cols) acc[q] += (double)part[(size_t)k * ld + q];
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    double v = acc[q];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0) red[q][w] = v;
  }
  __syncthreads();
  if (threadIdx.x < cols) {
    double v = 0;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) v += red[threadIdx.x][k];
    out[threadIdx.x] = v;
  }
}

extern "C" int rrl_column_sums(const float* part, int rows, int ld, int cols, double* out, void* stream) {
  if (rows < 0 || cols < 1 || cols > 8 || ld < cols) return -1;
  hipLaunchKernelGGL(column_sums_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, part, rows, ld, cols, out);
  return (int)hipGetLastError();
}

// ------------------------------------------------------------------ flat segmented scan
// Element t of two coupled recurrences (adv, ret):
//   nd = 1 - done_t ; v_next = done_t ? boot_t : val_{t+1}
//   adv_t = [r_t + g*v_next - v_t]            + (g*lam*nd) * adv_{t+1}      (baseline)
//   adv_t = r_t                               + (g*lam*nd) * adv_{t+1}      (no baseline)
//   ret_t = r_t + g*done_t*boot_t*use_boot    + (g*nd)     * ret_{t+1}
struct ScanFlat {
  const float* rew;
  const float* done;
  const float* val;   // [L] or null
  const float* boot;  // [L] bootstrap at path ends (read where done=1) or null
  float* adv;
  float* ret;
  float* agg;         // [nblocks][4] block aggregates (A_adv, B_adv, A_ret, B_ret)
  float* carry;       // [nblocks][2] values entering each block from the right
  float* stats_part;  // [nblocks][3]
  int L;
  float gamma, lam;
};

constexpr int kFlatPer = 8;   // elements per thread
constexpr int kFlatBlock = 256;
constexpr int kFlatChunk = kFlatPer * kFlatBlock;

RRL_DEV void flat_coeffs(const ScanFlat& p, int t, float& a_adv, float& b_adv, float& a_ret, float& b_ret) {
  const float r = p.rew[t];
  const float d = p.done[t] > 0.f ? 1.f : 0.f;  // flat paths: any nonzero code ends the path
  const float nd = 1.f - d;
  const float boot = (p.boot != nullptr && d > 0.f) ? p.boot[t] : 0.f;
  if (p.val != nullptr) {
    const float v = p.val[t];
    const float v_next = d > 0.f ? boot : (t + 1 < p.L ? p.val[t + 1] : 0.f);
    b_adv = r + p.gamma * v_next - v;
  } else {
    b_adv = r;
  }
  a_adv = p.gamma * p.lam * nd;
  a_ret = p.gamma * nd;
  b_ret = r + ((p.val != nullptr) ? p.gamma * d * boot : 0.f);
}

// phase 1 (apply=false): block aggregates; phase 3 (apply=true): final values.
template <bool APPLY>
__global__ __launch_bounds__(kFlatBlock) void flat_scan_kernel(ScanFlat p) {
  __shared__ float sA[2][kFlatBlock], sB[2][kFlatBlock];
  const int tid = threadIdx.x;
  const int lo = blockIdx.x * kFlatChunk + tid * kFlatPer;
  // thread aggregate over its chunk (reverse)
  float Aa = 1.f, Ba = 0.f, Ar = 1.f, Br = 0.f;
  for (int k = kFlatPer - 1; k >= 0; --k) {
    const int t = lo + k;
    if (t < p.L) {
      float a_adv, b_adv, a_ret, b_ret;
      flat_coeffs(p, t, a_adv, b_adv, a_ret, b_ret);
      Ba = b_adv + a_adv * Ba;
      Aa = a_adv * Aa;
      Br = b_ret + a_ret * Br;
      Ar = a_ret * Ar;
    }
  }
  sA[0][tid] = Aa; sB[0][tid] = Ba; sA[1][tid] = Ar; sB[1][tid] = Br;
  __syncthreads();
  // inclusive suffix scan over threads (Hillis-Steele): S_k = e_k o e_{k+1} o ...
  for (int off = 1; off < kFlatBlock; off <<= 1) {
    float nA0 = sA[0][tid], nB0 = sB[0][tid], nA1 = sA[1][tid], nB1 = sB[1][tid];
    if (tid + off < kFlatBlock) {
      const float A0 = sA[0][tid + off], B0 = sB[0][tid + off];
      const float A1 = sA[1][tid + off], B1 = sB[1][tid + off];
      nB0 = nB0 + nA0 * B0; nA0 = nA0 * A0;
      nB1 = nB1 + nA1 * B1; nA1 = nA1 * A1;
    }
    __syncthreads();
    sA[0][tid] = nA0; sB[0][tid] = nB0; sA[1][tid] = nA1; sB[1][tid] = nB1;
    __syncthreads();
  }
  if (!APPLY) {
    if (tid == 0) {
      p.agg[blockIdx.x * 4 + 0] = sA[0][0];
      p.agg[blockIdx.x * 4 + 1] = sB[0][0];
      p.agg[blockIdx.x * 4 + 2] = sA[1][0];
      p.agg[blockIdx.x * 4 + 3] = sB[1][0];
    }
    return;
  }
  // value entering this thread's chunk from the right
  const float cin_adv = p.carry[blockIdx.x * 2 + 0];
  const float cin_ret = p.carry[blockIdx.x * 2 + 1];
  float ya, yr;
  if (tid + 1 < kFlatBlock) {
    ya = sB[0][tid + 1] + sA[0][tid + 1] * cin_adv;
    yr = sB[1][tid + 1] + sA[1][tid + 1] * cin_ret;
  } else {
    ya = cin_adv;
    yr = cin_ret;
  }
  float s = 0.f, ss = 0.f, c = 0.f;
  for (int k = kFlatPer - 1; k >= 0; --k) {
    const int t = lo + k;
    if (t < p.L) {
      float a_adv, b_adv, a_ret, b_ret;
      flat_coeffs(p, t, a_adv, b_adv, a_ret, b_ret);
      ya = b_adv + a_adv * ya;
      yr = b_ret + a_ret * yr;
      p.adv[t] = ya;
      p.ret[t] = yr;
      s += ya;
      ss += ya * ya;
      c += 1.f;
    }
  }
  __syncthreads();
  s = wave_sum(s);
  ss = wave_sum(ss);
  c = wave_sum(c);
  if ((tid & 63) == 0) {
    sA[0][tid >> 6] = s;
    sB[0][tid >> 6] = ss;
    sA[1][tid >> 6] = c;
  }
  __syncthreads();
  if (tid == 0) {
    float a = 0.f, b = 0.f, cc = 0.f;
    for (int w = 0; w < kFlatBlock / 64; ++w) { a += sA[0][w]; b += sB[0][w]; cc += sA[1][w]; }
    p.stats_part[blockIdx.x * 3 + 0] = a;
    p.stats_part[blockIdx.x * 3 + 1] = b;
    p.stats_part[blockIdx.x * 3 + 2] = cc;
  }
}

// phase 2: sequential suffix over block aggregates (nblocks is L / 2048, small).
__global__ void flat_carry_kernel(const float* agg, float* carry, int nblocks) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  float ya = 0.f, yr = 0.f;
  for (int b = nblocks - 1; b >= 0; --b) {
    carry[b * 2 + 0] = ya;
    carry[b * 2 + 1] = yr;
    ya = agg[b * 4 + 1] + agg[b * 4 + 0] * ya;
    yr = agg[b * 4 + 3] + agg[b * 4 + 2] * yr;
  }
}

}  // namespace rrl

using namespace rrl;

extern "C" int rrl_scan_tm_parts(int N) { return (N + 255) / 256; }

// nparts of rrl_scan_tm_parts(K * N)
extern "C" int rrl_gae_scan_tm(const float* rew, const float* done, const float* val, const float* tval,
                               float* adv, float* ret, float* stats_part, float* stats_out, int K, int T, int N,
                               float gamma, float lam, long long* const* cnt, const long long* inc, int ncnt,
                               void* stream) {
  if (ncnt < 0 || ncnt > 3) return -1;
  hipStream_t s = (hipStream_t)stream;
  const int nb = rrl_scan_tm_parts(K * N);
  ScanTM p{rew, done, val, tval, adv, ret, stats_part, T, N, K, gamma, lam, {}, {}, ncnt};
  for (int i = 0; i < ncnt; ++i) {
    p.cnt[i] = cnt[i];
    p.inc[i] = inc[i];
  }
  hipLaunchKernelGGL(gae_scan_tm_kernel, dim3(nb), dim3(256), 0, s, p);
  if (stats_out) hipLaunchKernelGGL(stats_reduce_kernel, dim3(1), dim3(256), 0, s, stats_part, nb, stats_out);
  return (int)hipGetLastError();
}

extern "C" int rrl_scan_flat_blocks(int L) { return (L + kFlatChunk - 1) / kFlatChunk; }

// work: [nblocks * 9] floats (agg 4 + carry 2 + stats 3 per block)
extern "C" int rrl_scan_flat(const float* rew, const float* done, const float* val, const float* boot,
                             float* adv, float* ret, float* work, float* stats_out, int L, float gamma,
                             float lam, void* stream) {
  if (L <= 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  const int nb = rrl_scan_flat_blocks(L);
  ScanFlat p{rew, done, val, boot, adv, ret, work, work + 4 * nb, work + 6 * nb, L, gamma, lam};
  hipLaunchKernelGGL(flat_scan_kernel<false>, dim3(nb), dim3(kFlatBlock), 0, s, p);
  hipLaunchKernelGGL(flat_carry_kernel, dim3(1), dim3(64), 0, s, (const float*)p.agg, p.carry, nb);
  hipLaunchKernelGGL(flat_scan_kernel<true>, dim3(nb), dim3(kFlatBlock), 0, s, p);
  if (stats_out) hipLaunchKernelGGL(stats_reduce_kernel, dim3(1), dim3(256), 0, s, (const float*)p.stats_part, nb, stats_out);
  return (int)hipGetLastError();
}

extern "C" int rrl_stats_reduce(const float* part, int nparts, float* out, void* stream) {
  hipLaunchKernelGGL(stats_reduce_kernel, dim3(1), dim3(256), 0, (hipStream_t)stream, part, nparts, out);
  return (int)hipGetLastError();
}
