// Probe: per-SIMD issue throughput of the ordered update's instruction classes on gfx950, by
// s_memtime (shader clock) inside the kernel, at 1, 2 and 4 waves per SIMD (one 4/8/16-wave block
// per CU): cycles per wave64 instruction = elapsed cycles x SIMDs / instructions issued.
// MODE 0 v_fma_f32, 1 v_pk_fma_f32, 2 v_exp_f32, 3 v_rcp_f32, 4 half the waves v_exp_f32 and half
// v_fma_f32 on the same SIMDs (do the transcendental and the plain VALU overlap?), 5 the GRU
// gate mix of one element (3 exp, 3 rcp, ~14 fma-class) as 8 independent chains.
//   hipcc --offload-arch=gfx950 -O3 tools/probes/issue_rates.hip -o tools/probes/issue_rates
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned long long stamp() {
  unsigned long long v;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return v;
}

template <int MODE>
__global__ void probe(float* out, unsigned long long* cyc, int iters) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float r = 0.f;
  float v[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = lane * 1e-4f + k * 0.01f;
  __syncthreads();
  const unsigned long long t0 = stamp();
  const int mode = MODE == 4 ? ((wave & 4) ? 2 : 0) : MODE;   // waves 4..7 of each 4-SIMD group: exp
  if (mode == 0) {
    for (int i = 0; i < iters; ++i)
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = __builtin_fmaf(v[k], 0.999f, 1e-3f);
  } else if (mode == 1) {
    f2 w[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) w[k] = f2{v[k], v[k] + 1.f};
    const f2 m = {0.999f, 0.998f}, c = {1e-3f, 2e-3f};
    for (int i = 0; i < iters; ++i)
#pragma unroll
      for (int k = 0; k < 8; ++k) w[k] = __builtin_elementwise_fma(w[k], m, c);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = w[k][0] + w[k][1];
  } else if (mode == 2) {
    for (int i = 0; i < iters; ++i)
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = __builtin_amdgcn_exp2f(v[k]) - 1.0f;   // +1 fma-class op
  } else if (mode == 3) {
    for (int i = 0; i < iters; ++i)
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = __builtin_amdgcn_rcpf(v[k]) + 0.5f;     // +1 fma-class op
  } else {   // mode 5: one GRU element per chain per iteration
    for (int i = 0; i < iters; ++i)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float a = __builtin_fmaf(v[k], 0.5f, 0.1f);
        const float z = __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(a));
        const float rc = __builtin_amdgcn_rcpf(__builtin_fmaf(__builtin_amdgcn_exp2f(__builtin_fmaf(v[k], 0.3f, 0.2f)), 2.f, 2.f));
        const float g = __builtin_fmaf(rc, v[k], 0.3f);
        const float t = g * 0.34657f, u = t * t;
        float p = __builtin_fmaf(u, -0.00627f, 0.02107f);
        p = __builtin_fmaf(p, u, -0.05385f);
        p = __builtin_fmaf(p, u, 0.13333f);
        p = __builtin_fmaf(p, u, -0.33333f);
        const float small = __builtin_fmaf(t * u, p, t);
        const float big = 1.0f - 2.0f * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(g));
        const float n = __builtin_fabsf(t) < 0.55f ? small : big;
        v[k] = n + z * (v[k] - n);
      }
  }
  const unsigned long long t1 = stamp();
#pragma unroll
  for (int k = 0; k < 8; ++k) r += v[k];
  if (r == 12345.678f) out[threadIdx.x] = r;
  if (lane == 0) cyc[blockIdx.x * 16 + wave] = t1 - t0;
}

template <int MODE>
void run(float* out, unsigned long long* dcyc, int waves_per_simd, int iters, const char* name, double insts_per_iter) {
  const int threads = 64 * 4 * waves_per_simd;
  hipLaunchKernelGGL(probe<MODE>, dim3(256), dim3(threads), 0, 0, out, dcyc, 50);
  hipLaunchKernelGGL(probe<MODE>, dim3(256), dim3(threads), 0, 0, out, dcyc, iters);
  unsigned long long h[256 * 16];
  (void)hipMemcpy(h, dcyc, sizeof(h), hipMemcpyDeviceToHost);
  double mx = 0;
  for (int b = 0; b < 256; ++b)
    for (int w = 0; w < 4 * waves_per_simd; ++w) mx += (double)h[b * 16 + w];
  mx /= 256.0 * 4 * waves_per_simd;   // mean elapsed cycles of a wave
  // per SIMD: waves_per_simd waves each issued iters * insts_per_iter instructions in mx cycles
  printf("%-34s waves/SIMD %d: %.2f cycles per wave-instruction per SIMD (%.0f cycles)\n", name, waves_per_simd,
         mx / (waves_per_simd * (double)iters * insts_per_iter), mx);
}

int main() {
  float* out;
  unsigned long long* cyc;
  (void)hipMalloc(&out, 4096 * sizeof(float));
  (void)hipMalloc(&cyc, 256 * 16 * sizeof(unsigned long long));
  const int it = 4000;
  for (int w : {1, 2, 4}) {
    run<0>(out, cyc, w, it, "v_fma_f32", 8);
    run<1>(out, cyc, w, it, "v_pk_fma_f32", 8);
    run<2>(out, cyc, w, it, "v_exp_f32 (+ v_add)", 8);
    run<3>(out, cyc, w, it, "v_rcp_f32 (+ v_add)", 8);
    if (w >= 2) run<4>(out, cyc, w, it, "half exp+add, half fma (per inst)", 12);
    run<5>(out, cyc, w, it / 10, "GRU element (6 trans, per element)", 1);
  }
  return 0;
}
