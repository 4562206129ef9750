// Issue cost of v_fma_f32 vs v_pk_fma_f32 for ONE wave per SIMD (1,024
// one-wave workgroups on 256 CUs): 8 independent scalar FMA chains vs 4
// independent packed chains (the same FMAs), and a dependent packed chain.
//   hipcc -O3 --offload-arch=gfx950 pk_issue.hip -o pk_issue && ./pk_issue
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));
constexpr int IT = 4096;

__global__ __launch_bounds__(64) void scal(float* out, float s) {
  float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
        a6 = a0 + 6, a7 = a0 + 7;
  for (int i = 0; i < IT; i++) {
#pragma unroll
    for (int u = 0; u < 4; u++) {
      a0 = fmaf(a0, s, 1.f); a1 = fmaf(a1, s, 1.f); a2 = fmaf(a2, s, 1.f); a3 = fmaf(a3, s, 1.f);
      a4 = fmaf(a4, s, 1.f); a5 = fmaf(a5, s, 1.f); a6 = fmaf(a6, s, 1.f); a7 = fmaf(a7, s, 1.f);
    }
  }
  out[blockIdx.x * 64 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}
__global__ __launch_bounds__(64) void pk(float* out, float s) {
  f2 a0 = {(float)threadIdx.x, 1.f}, a1 = a0 + 2.f, a2 = a0 + 4.f, a3 = a0 + 6.f;
  const f2 S = {s, s}, O = {1.f, 1.f};
  for (int i = 0; i < IT; i++) {
#pragma unroll
    for (int u = 0; u < 4; u++) {
      a0 = __builtin_elementwise_fma(a0, S, O); a1 = __builtin_elementwise_fma(a1, S, O);
      a2 = __builtin_elementwise_fma(a2, S, O); a3 = __builtin_elementwise_fma(a3, S, O);
    }
  }
  f2 r = a0 + a1 + a2 + a3;
  out[blockIdx.x * 64 + threadIdx.x] = r.x + r.y;
}
__global__ __launch_bounds__(64) void pkdep(float* out, float s) {
  f2 a0 = {(float)threadIdx.x, 1.f};
  const f2 S = {s, s}, O = {1.f, 1.f};
  for (int i = 0; i < IT; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++) a0 = __builtin_elementwise_fma(a0, S, O);
  }
  out[blockIdx.x * 64 + threadIdx.x] = a0.x + a0.y;
}
__global__ __launch_bounds__(64) void scdep(float* out, float s) {
  float a0 = threadIdx.x;
  for (int i = 0; i < IT; i++) {
#pragma unroll
    for (int u = 0; u < 16; u++) a0 = fmaf(a0, s, 1.f);
  }
  out[blockIdx.x * 64 + threadIdx.x] = a0;
}

template <class K> float run(K k, float* out) {
  hipEvent_t a, b;
  hipEventCreate(&a); hipEventCreate(&b);
  for (int w = 0; w < 3; w++) hipLaunchKernelGGL(k, dim3(1024), dim3(64), 0, 0, out, 0.999f);
  hipEventRecord(a);
  for (int w = 0; w < 10; w++) hipLaunchKernelGGL(k, dim3(1024), dim3(64), 0, 0, out, 0.999f);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  return ms / 10;
}
int main() {
  float* out; hipMalloc(&out, 1024 * 64 * 4);
  // per wave: 32 x IT FMA-instructions (scalar) or 16 x IT (packed)
  float t1 = run(scal, out), t2 = run(pk, out), t3 = run(pkdep, out), t4 = run(scdep, out);
  // cycles per instruction at the measured clock are printed relative: ns per instruction per wave
  printf("{\"scalar_ns_per_inst\": %.4f, \"packed_ns_per_inst\": %.4f, "
         "\"packed_dep_ns_per_inst\": %.4f, \"scalar_dep_ns_per_inst\": %.4f}\n",
         t1 * 1e6 / (32.0 * IT), t2 * 1e6 / (16.0 * IT), t3 * 1e6 / (16.0 * IT), t4 * 1e6 / (16.0 * IT));
  return 0;
}
