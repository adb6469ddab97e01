// Probe: issue cost per wave-instruction of f32 VALU forms on gfx950, one and two waves per SIMD:
// v_fma_f32, v_pk_fma_f32 (float2), v_exp_f32, v_rcp_f32 (independent chains, 8 per lane).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ void probe(float* out, int iters) {
  const int lane = threadIdx.x & 63;
  float r = 0.f;
  if constexpr (MODE == 0) {
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = lane * 1e-3f + k;
    for (int i = 0; i < iters; ++i)
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = __builtin_fmaf(v[k], 0.999f, 1e-3f);
#pragma unroll
    for (int k = 0; k < 8; ++k) r += v[k];
  } else if constexpr (MODE == 1) {
    f2 v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = f2{lane * 1e-3f + k, lane * 2e-3f + k};
    const f2 m = {0.999f, 0.998f}, c = {1e-3f, 2e-3f};
    for (int i = 0; i < iters; ++i)
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = __builtin_elementwise_fma(v[k], m, c);
#pragma unroll
    for (int k = 0; k < 8; ++k) r += v[k][0] + v[k][1];
  } else {
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = lane * 1e-3f + k * 0.1f;
    for (int i = 0; i < iters; ++i)
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = MODE == 2 ? __builtin_amdgcn_exp2f(v[k]) : __builtin_amdgcn_rcpf(v[k]);
#pragma unroll
    for (int k = 0; k < 8; ++k) r += v[k];
  }
  if (r == 12345.678f) out[threadIdx.x] = r;
}

template <int MODE>
float run(float* out, int threads, int iters) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  hipLaunchKernelGGL(probe<MODE>, dim3(256), dim3(threads), 0, 0, out, 100);
  (void)hipEventRecord(e0);
  hipLaunchKernelGGL(probe<MODE>, dim3(256), dim3(threads), 0, 0, out, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  float* out;
  (void)hipMalloc(&out, 1 << 16);
  const int iters = 20000;
  const double clk = 2.4e6;   // cycles per ms at 2.4 GHz (upper bound: the chip may run lower)
  for (int threads : {256, 512}) {
    const int wps = threads / 256;   // waves per SIMD
    float t0 = run<0>(out, threads, iters), t1 = run<1>(out, threads, iters);
    float t2 = run<2>(out, threads, iters), t3 = run<3>(out, threads, iters);
    const double n = (double)iters * 8 * wps;   // wave-instructions per SIMD
    printf("%d wave(s)/SIMD: cycles per wave-instruction  v_fma_f32 %.2f  v_pk_fma_f32 %.2f  v_exp_f32 %.2f  v_rcp_f32 %.2f\n",
           wps, t0 * clk / n, t1 * clk / n, t2 * clk / n, t3 * clk / n);
  }
  return 0;
}
