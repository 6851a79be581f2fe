// Issue-budget probe for the value-gradient kernel's MFMA shape question.
//
// Two waves per SIMD (512-thread workgroups, one per CU) run a loop of "units".  A unit is
// the same 16,384 bf16 MACs either as TWO v_mfma_f32_16x16x32_bf16 (the shipped kernel's
// shape) or as ONE v_mfma_f32_32x32x16_bf16, plus NV independent v_fma_f32 and NL
// ds_read_b128 per unit -- the vector work the value-grad kernel issues beside its MFMAs
// (per wave and 64-row slab: 244 16x16x32 MFMAs = 122 units, 566 VALU = 4.6 per unit, 250 LDS
// reads = 2.0 per unit; docs/PERF_NOTES.md).  Output: cycles per unit per wave, from s_memtime
// around the loop (median over waves), for each (shape, NV, NL).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/probes/mfma_shape_probe tools/probes/mfma_shape_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

template <int SHAPE, int NV, int NL>
__global__ __launch_bounds__(512, 1) void probe(unsigned long long* cyc, float* sink, int iters) {
  extern __shared__ __attribute__((aligned(16))) float lds[];
  const int t = threadIdx.x, l = t & 63;
  for (int i = t; i < 8192; i += 512) lds[i] = (float)(i & 127) * 1e-3f;
  __syncthreads();
  bf16x8 a, b;
  for (int i = 0; i < 8; ++i) {
    a[i] = (__bf16)(0.001f * (l + i));
    b[i] = (__bf16)(0.002f * (l - i));
  }
  f32x4 c16[4] = {};
  f32x16 c32[2] = {};
  float v[16];
  for (int i = 0; i < 16; ++i) v[i] = 0.5f + 0.01f * (l + i);
  const float x = 1.0001f, y = 1e-7f;
  f32x4 r[4] = {};
  // LDS byte address of this lane's b128 (conflict-free: consecutive 16-byte chunks)
  const unsigned lbase = (unsigned)(l * 16);
  unsigned long long t0;
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t0)::"memory");
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (SHAPE == 16) {
        c16[u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c16[u], 0, 0, 0);
        c16[(u + 2) & 3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, a, c16[(u + 2) & 3], 0, 0, 0);
      } else {
        c32[u & 1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c32[u & 1], 0, 0, 0);
      }
#pragma unroll
      for (int k = 0; k < NV; ++k) asm volatile("v_fma_f32 %0, %1, %2, %0" : "+v"(v[k & 15]) : "v"(x), "v"(y));
      // the previous unit's reads have landed before their registers are reused (the shipped
      // kernel prefetches one step ahead the same way)
      if (NL > 0) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int k = 0; k < NL; ++k)
        asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r[k & 3]) : "v"(lbase), "i"(1024 * (k + 1)) : "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  unsigned long long t1;
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1)::"memory");
  float s = 0.f;
  for (int i = 0; i < 4; ++i) s += c16[i][0] + r[i][0] + r[i][3];
  for (int i = 0; i < 2; ++i) s += c32[i][0] + c32[i][15];
  for (int i = 0; i < 16; ++i) s += v[i];
  sink[blockIdx.x * 512 + t] = s;
  if (l == 0) cyc[blockIdx.x * 8 + (t >> 6)] = t1 - t0;
}

// cycles per unit per wave (median over waves) and wall ns per unit per wave (HIP events,
// so the clock the chip holds under each shape counts too)
struct Res {
  double cyc, ns;
};

template <int SHAPE, int NV, int NL>
Res run(int iters) {
  const int grid = 256;
  unsigned long long* cyc;
  float* sink;
  (void)hipMalloc(&cyc, grid * 8 * sizeof(unsigned long long));
  (void)hipMalloc(&sink, grid * 512 * sizeof(float));
  const size_t lds = 96 * 1024;  // one workgroup per CU: two waves per SIMD
  (void)hipFuncSetAttribute((const void*)probe<SHAPE, NV, NL>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
  for (int w = 0; w < 20; ++w)  // warm-up: ~0.5 s of back-to-back launches so the clock settles
    hipLaunchKernelGGL((probe<SHAPE, NV, NL>), dim3(grid), dim3(512), lds, 0, cyc, sink, iters);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, 0);
  const int reps = 10;
  for (int w = 0; w < reps; ++w)
    hipLaunchKernelGGL((probe<SHAPE, NV, NL>), dim3(grid), dim3(512), lds, 0, cyc, sink, iters);
  (void)hipEventRecord(e1, 0);
  (void)hipDeviceSynchronize();
  float ms = 0.f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  std::vector<unsigned long long> h(grid * 8);
  (void)hipMemcpy(h.data(), cyc, h.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost);
  std::sort(h.begin(), h.end());
  (void)hipFree(cyc);
  (void)hipFree(sink);
  return Res{(double)h[h.size() / 2] / (4.0 * iters), 1e6 * ms / (reps * 4.0 * iters)};
}

// NL16 / NL32: b128 LDS reads per unit for each shape (a 32x32x16 step consumes one 8-element
// activation fragment per lane where two 16x16x32 steps consume two)
template <int NV, int NL16, int NL32>
void row(int iters) {
  const Res a = run<16, NV, NL16>(iters), b = run<32, NV, NL32>(iters);
  printf("{\"valu_per_unit\": %d, \"lds_b128_per_unit_16\": %d, \"lds_b128_per_unit_32\": %d, "
         "\"cycles_16x16x32\": %.1f, \"cycles_32x32x16\": %.1f, \"cycle_ratio_32_over_16\": %.3f, "
         "\"ns_16x16x32\": %.2f, \"ns_32x32x16\": %.2f, \"wall_ratio_32_over_16\": %.3f}\n",
         NV, NL16, NL32, a.cyc, b.cyc, b.cyc / a.cyc, a.ns, b.ns, b.ns / a.ns);
  fflush(stdout);
}

int main() {
  const int iters = 2000;
  row<0, 0, 0>(iters);
  row<4, 0, 0>(iters);
  row<6, 0, 0>(iters);
  row<8, 0, 0>(iters);
  row<12, 0, 0>(iters);
  row<5, 2, 2>(iters);
  row<5, 2, 1>(iters);  // the value-grad kernel's mix per 16K-MAC unit, with the 32-wide tile's halved reads
  row<6, 2, 1>(iters);
  row<8, 2, 1>(iters);
  row<10, 2, 1>(iters);
  return 0;
}
