// Probe: do f32 MFMA (v_mfma_f32_16x16x4_f32) and plain VALU work from two different waves on
// the same SIMD overlap on gfx950?  Waves 0-3 of a 512-thread block run an MFMA chain, waves 4-7
// a VALU chain (waves w and w+4 share a SIMD).  Time MFMA-only, VALU-only, both.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef short s8 __attribute__((ext_vector_type(8)));

__global__ __launch_bounds__(512) void probe(float* out, int mode, int iters) {
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const bool mf = wave < 4;
  if (mf && !(mode & 1)) return;
  if (!mf && !(mode & 2)) return;
  float r = 0.f;
  if (mf && (mode & 8)) {   // bf16 MFMA chain (16x16x32)
    f4 a0 = {0, 0, 0, 0}, a1 = a0, a2 = a0, a3 = a0;
    s8 x, y;
    for (int k = 0; k < 8; ++k) { x[k] = (short)(0x3f80 + lane + k); y[k] = (short)(0x3f00 + k); }
    for (int i = 0; i < iters; ++i) {
      a0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, y, a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(y, x, a1, 0, 0, 0);
      a2 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(x, x, a2, 0, 0, 0);
      a3 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(y, y, a3, 0, 0, 0);
    }
    r = a0[0] + a1[1] + a2[2] + a3[3];
  } else if (mf) {
    f4 a0 = {0, 0, 0, 0}, a1 = a0, a2 = a0, a3 = a0;
    float x = lane * 1e-3f, y = 1.0f - lane * 1e-4f;
    for (int i = 0; i < iters; ++i) {
      a0 = __builtin_amdgcn_mfma_f32_16x16x4f32(x, y, a0, 0, 0, 0);
      a1 = __builtin_amdgcn_mfma_f32_16x16x4f32(y, x, a1, 0, 0, 0);
      a2 = __builtin_amdgcn_mfma_f32_16x16x4f32(x, x, a2, 0, 0, 0);
      a3 = __builtin_amdgcn_mfma_f32_16x16x4f32(y, y, a3, 0, 0, 0);
    }
    r = a0[0] + a1[1] + a2[2] + a3[3];
  } else if (mode & 4) {   // transcendental chain
    float v0 = lane * 1e-3f, v1 = v0 + 1, v2 = v0 + 2, v3 = v0 + 3;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        v0 = __builtin_amdgcn_exp2f(v0 * -0.5f);
        v1 = __builtin_amdgcn_rcpf(v1 + 1.0f);
        v2 = __builtin_amdgcn_exp2f(v2 * -0.5f);
        v3 = __builtin_amdgcn_rcpf(v3 + 1.0f);
      }
    }
    r = v0 + v1 + v2 + v3;
  } else {
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = lane * 1e-3f + k;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = __builtin_fmaf(v[k], 0.999f, 1e-3f);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = __builtin_fmaf(v[k], 0.999f, 1e-3f);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) r += v[k];
  }
  if (r == 12345.678f) out[threadIdx.x] = r;
}

int main() {
  float* out;
  hipMalloc(&out, 4096);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000;
  const char* names[16] = {"", "mfma only", "valu only", "mfma + valu", "", "", "trans only", "mfma + trans",
                           "", "bf16 mfma only", "", "bf16 mfma + valu", "", "", "", "bf16 mfma + trans"};
  for (int mode : {1, 2, 3, 6, 7, 9, 11, 15}) {
    hipLaunchKernelGGL(probe, dim3(256), dim3(512), 0, 0, out, mode, 100);
    hipEventRecord(e0);
    hipLaunchKernelGGL(probe, dim3(256), dim3(512), 0, 0, out, mode, iters);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    // MFMA waves: 4 MFMA / iter (32 cyc each); VALU waves: 16 fma / iter; trans: 16 trans / iter
    printf("%-14s %8.3f ms\n", names[mode], ms);
  }
  return 0;
}
