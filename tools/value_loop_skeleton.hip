// Persistent fused value loop vs kernel-per-phase, with the arithmetic taken out.
//
// VERDICT r4 item 5 asks for a persistent value loop (one launch runs all train_vf_iters
// iterations: gradient slabs -> device-wide barrier -> in-kernel reduce + Adam -> barrier) at
// the reference-hyperparameter TTT shape (8,192 rows: 128 workgroups of 64 rows, value net
// P = 17,665 floats), or a MEASURED negative result.  This program times exactly the data
// flow the fused loop adds or removes, with the gradient math replaced by a dependent read:
//
//   per iteration, every workgroup:  read the P parameters (the gradient kernel's prologue)
//                                    write its P-float partial-gradient slab
//   ---- sync 1 ----                 (kernel boundary  |  grid barrier)
//   per iteration, workgroup b:      reduce its P/G share over the G slabs + Adam on it
//   ---- sync 2 ----                 (kernel boundary  |  grid barrier)
//
//   split  : two kernels per iteration, ITERS x 2 launches captured in ONE hipGraph (the
//            shipped learner's structure: value_grad_split_kernel, then the reduce + Adam kernel)
//   fused  : ONE persistent launch, grid barriers between the phases: a flat counter, or
//            XCD-hierarchical (per-group counter, group leaders meet on a top counter)
//
// Every spin is bounded (an error flag instead of a hang), the grid is <= the CU count (one
// 512-thread workgroup per CU is always co-resident), and the barrier uses only vector
// atomics.  Prints one JSON line: us per iteration for each variant.
//
//   hipcc -O3 --offload-arch=gfx950 -o /tmp/vls tools/value_loop_skeleton.hip && /tmp/vls
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                       \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      exit(1);                                                                         \
    }                                                                                  \
  } while (0)

constexpr int kThreads = 512;
constexpr unsigned kSpinLimit = 1u << 26;  // ~seconds of polling: then the error flag, no hang

struct Args {
  float* params;
  float* m;
  float* v;
  float* slab;   // [G][P]
  float* sink;   // [G] keeps the prologue reads alive
  int P, G, iters;
  unsigned* counters;  // [8 groups x 32 (padded)] + top at [8 * 32] + gens at [9 * 32 + g * 32]
  int* err;
  int mode;  // 0 flat barrier, 1 XCD-hierarchical
};

__device__ __forceinline__ unsigned ld_relaxed(unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// epoch-counted barrier (monotonic counters, no reset race): call with epoch = 0, 1, 2, ...
__device__ void grid_barrier(const Args& a, unsigned epoch) {
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // this workgroup's stores before the arrival
    const unsigned G = (unsigned)a.G;
    unsigned spins = 0;
    if (a.mode == 0) {
      unsigned* top = a.counters + 8 * 32;
      __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = (epoch + 1) * G;
      while (ld_relaxed(top) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (++spins > kSpinLimit) {
          atomicOr(a.err, 1);
          break;
        }
      }
    } else {
      const unsigned grp = blockIdx.x & 7u;
      const unsigned members = G / 8 + ((grp < G % 8) ? 1u : 0u);
      const unsigned groups = G < 8 ? G : 8u;
      unsigned* gc = a.counters + grp * 32;
      unsigned* top = a.counters + 8 * 32;
      unsigned* gen = a.counters + 9 * 32 + grp * 32;
      const unsigned old = __hip_atomic_fetch_add(gc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (old + 1 == (epoch + 1) * members) {  // last of its group: the group's leader
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        __hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        while (ld_relaxed(top) < (epoch + 1) * groups) {
          __builtin_amdgcn_s_sleep(1);
          if (++spins > kSpinLimit) {
            atomicOr(a.err, 2);
            break;
          }
        }
        __hip_atomic_store(gen, epoch + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        while (ld_relaxed(gen) < epoch + 1) {
          __builtin_amdgcn_s_sleep(1);
          if (++spins > kSpinLimit) {
            atomicOr(a.err, 4);
            break;
          }
        }
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __syncthreads();
}

// phase 1: read the parameters (prologue), write this workgroup's slab
__device__ void phase_grad(const Args& a, int it) {
  const int b = blockIdx.x;
  float acc = 0.f;
  float* slab = a.slab + (size_t)b * a.P;
  for (int i = threadIdx.x; i < a.P; i += kThreads) {
    const float w = a.params[i];
    acc += w;
    slab[i] = w * 1e-3f + (float)(b + it) * 1e-7f;  // a partial gradient that depends on the weights
  }
  if (acc == 12345.f) a.sink[b] = acc;  // keeps the reads (never true in practice)
}

// phase 2: workgroup b reduces its share of the P columns over the G slabs, then Adam.
// 512 threads = 128 columns x 4 slab quarters (independent loads in flight), LDS combine.
__device__ void phase_adam(const Args& a, int it) {
  __shared__ float part[4][128];
  const int share = (a.P + a.G - 1) / a.G;
  const int lo = blockIdx.x * share;
  const int hi = min(a.P, lo + share);
  const float b1 = 0.9f, b2 = 0.999f, lr = 1e-3f;
  const float bc1 = 1.f - __powf(b1, (float)(it + 1)), bc2 = 1.f - __powf(b2, (float)(it + 1));
  const int c = threadIdx.x & 127, q = threadIdx.x >> 7;
  for (int base = lo; base < hi; base += 128) {
    const int i = base + c;
    float g = 0.f;
    if (i < hi) {
#pragma unroll 8
      for (int k = q; k < a.G; k += 4) g += a.slab[(size_t)k * a.P + i];
    }
    part[q][c] = g;
    __syncthreads();
    if (q == 0 && i < hi) {
      g = (part[0][c] + part[1][c]) + (part[2][c] + part[3][c]);
      const float m = b1 * a.m[i] + (1.f - b1) * g;
      const float v = b2 * a.v[i] + (1.f - b2) * g * g;
      a.m[i] = m;
      a.v[i] = v;
      a.params[i] -= lr * (m / bc1) / (sqrtf(v / bc2) + 1e-8f);
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(kThreads, 1) void k_grad(Args a, int it) { phase_grad(a, it); }
__global__ __launch_bounds__(kThreads, 1) void k_adam(Args a, int it) { phase_adam(a, it); }

__global__ __launch_bounds__(kThreads, 1) void k_fused(Args a) {
  for (int it = 0; it < a.iters; ++it) {
    phase_grad(a, it);
    grid_barrier(a, 2 * it);
    phase_adam(a, it);
    grid_barrier(a, 2 * it + 1);
  }
}

__global__ __launch_bounds__(kThreads, 1) void k_barrier_only(Args a) {
  for (int it = 0; it < 2 * a.iters; ++it) grid_barrier(a, it);
}

int main(int argc, char** argv) {
  const int P = argc > 1 ? atoi(argv[1]) : 17665;  // LunarLander value net: 128x8 + 128 + 128x128 + 128 + 128 + 1
  const int iters = argc > 2 ? atoi(argv[2]) : 80;
  const int reps = 20;
  int dev = 0, cus = 0;
  CHECK(hipGetDevice(&dev));
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  printf("{\"P\": %d, \"iters\": %d, \"cus\": %d", P, iters, cus);
  for (int G : {64, 128, 256}) {
    if (G > cus) continue;
    Args a{};
    a.P = P;
    a.G = G;
    a.iters = iters;
    CHECK(hipMalloc(&a.params, P * 4));
    CHECK(hipMalloc(&a.m, P * 4));
    CHECK(hipMalloc(&a.v, P * 4));
    CHECK(hipMalloc(&a.slab, (size_t)G * P * 4));
    CHECK(hipMalloc(&a.sink, G * 4));
    CHECK(hipMalloc(&a.counters, 20 * 32 * 4));
    CHECK(hipMalloc(&a.err, 4));
    std::vector<float> h(P, 0.01f);
    CHECK(hipMemcpy(a.params, h.data(), P * 4, hipMemcpyHostToDevice));
    CHECK(hipMemset(a.m, 0, P * 4));
    CHECK(hipMemset(a.v, 0, P * 4));
    CHECK(hipMemset(a.err, 0, 4));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    // split: 2 kernels per iteration, captured once
    hipGraph_t g;
    hipGraphExec_t ge;
    CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int it = 0; it < iters; ++it) {
      hipLaunchKernelGGL(k_grad, dim3(G), dim3(kThreads), 0, s, a, it);
      hipLaunchKernelGGL(k_adam, dim3(G), dim3(kThreads), 0, s, a, it);
    }
    CHECK(hipStreamEndCapture(s, &g));
    CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CHECK(hipGraphLaunch(ge, s));
    CHECK(hipStreamSynchronize(s));
    CHECK(hipEventRecord(e0, s));
    for (int r = 0; r < reps; ++r) CHECK(hipGraphLaunch(ge, s));
    CHECK(hipEventRecord(e1, s));
    CHECK(hipEventSynchronize(e1));
    float ms_split = 0.f;
    CHECK(hipEventElapsedTime(&ms_split, e0, e1));
    float ms[2] = {0.f, 0.f}, ms_bar[2] = {0.f, 0.f};
    for (int mode = 0; mode < 2; ++mode) {
      a.mode = mode;
      for (int kind = 0; kind < 2; ++kind) {
        CHECK(hipMemset(a.counters, 0, 20 * 32 * 4));
        CHECK(hipStreamSynchronize(s));
        // warm-up launch, then timed launches; counters reset between launches (epochs restart)
        float tot = 0.f;
        for (int r = 0; r <= reps; ++r) {
          CHECK(hipMemsetAsync(a.counters, 0, 20 * 32 * 4, s));
          CHECK(hipEventRecord(e0, s));
          if (kind == 0) hipLaunchKernelGGL(k_fused, dim3(G), dim3(kThreads), 0, s, a);
          else hipLaunchKernelGGL(k_barrier_only, dim3(G), dim3(kThreads), 0, s, a);
          CHECK(hipEventRecord(e1, s));
          CHECK(hipEventSynchronize(e1));
          float t = 0.f;
          CHECK(hipEventElapsedTime(&t, e0, e1));
          if (r > 0) tot += t;
        }
        (kind == 0 ? ms[mode] : ms_bar[mode]) = tot;
      }
    }
    int err = 0;
    CHECK(hipMemcpy(&err, a.err, 4, hipMemcpyDeviceToHost));
    const double per = 1e3 / ((double)reps * iters);
    printf(", \"G%d\": {\"split_graph_us_per_iter\": %.3f, \"fused_flat_us_per_iter\": %.3f, "
           "\"fused_xcd_us_per_iter\": %.3f, \"barrier_flat_us\": %.3f, \"barrier_xcd_us\": %.3f, \"err\": %d}",
           G, ms_split * per, ms[0] * per, ms[1] * per, ms_bar[0] * per / 2, ms_bar[1] * per / 2, err);
    CHECK(hipGraphExecDestroy(ge));
    CHECK(hipGraphDestroy(g));
    for (void* p : {(void*)a.params, (void*)a.m, (void*)a.v, (void*)a.slab, (void*)a.sink, (void*)a.counters,
                    (void*)a.err})
      CHECK(hipFree(p));
  }
  printf("}\n");
  return 0;
}
