// readout_kernels.hip — the readout operations that run before predict (GM:611-655):
// pooling (AUX:1165-1185), element-wise product (AUX:1081-1088), extend_adjacencies
// (AUX:1236-1265).  All HBM-bound row work: coalesced row-major reads, no MFMA.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>

#include "readout_kernels.h"

namespace {

constexpr int kThreads = 256;

__device__ __forceinline__ float pool_init(int mode) { return mode == POOL_MAX ? -INFINITY : 0.f; }
__device__ __forceinline__ float pool_add(int mode, float acc, float v) {
  return mode == POOL_MAX ? (v > acc ? v : acc) : acc + v;
}

// One block per chunk of rows.  R = 256 / F row lanes per column (F <= 256), so a block reads
// R consecutive rows per iteration (R*F*4 contiguous bytes).  Wider rows loop over 256-column
// blocks with R = 1.  The R partials of a column are combined in a fixed order.
__global__ __launch_bounds__(kThreads) void pool_partial_kernel(const float* __restrict__ x, int F,
                                                                 const int64_t* __restrict__ chunk, int mode,
                                                                 float* __restrict__ partial) {
  __shared__ float red[kThreads];
  const int64_t c = blockIdx.x;
  const int64_t r0 = chunk[2 * c], r1 = chunk[2 * c + 1];
  const int t = threadIdx.x;
  for (int c0 = 0; c0 < F; c0 += kThreads) {
    const int Fb = min(F - c0, kThreads);
    const int R = kThreads / Fb;
    const int col = t % Fb, sub = t / Fb;
    float acc = pool_init(mode);
    if (sub < R)
      for (int64_t r = r0 + sub; r < r1; r += R) acc = pool_add(mode, acc, x[r * F + c0 + col]);
    red[t] = acc;
    __syncthreads();
    if (t < Fb) {
      float a = red[t];
      for (int k = 1; k < R; ++k) a = pool_add(mode, a, red[k * Fb + t]);
      partial[c * F + c0 + t] = a;
    }
    __syncthreads();
  }
}

// One block per graph: the graph's chunk partials in chunk order, then the mean's division.
// An empty graph gives 0 (sum), 0/0 = NaN (mean), -inf (max).
__global__ __launch_bounds__(kThreads) void pool_final_kernel(const float* __restrict__ partial, int F,
                                                               const int32_t* __restrict__ chunk_ptr,
                                                               const int64_t* __restrict__ count, int mode,
                                                               float* __restrict__ out) {
  const int g = blockIdx.x;
  for (int col = threadIdx.x; col < F; col += kThreads) {
    float acc = pool_init(mode);
    for (int k = chunk_ptr[g]; k < chunk_ptr[g + 1]; ++k) acc = pool_add(mode, acc, partial[(int64_t)k * F + col]);
    if (mode == POOL_MEAN) acc = acc / (float)count[g];
    out[(int64_t)g * F + col] = acc;
  }
}

__device__ __forceinline__ int64_t graph_of(const int64_t* seg, int G, int64_t r) {
  int lo = 0, hi = G;   // largest g with seg[g] <= r
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (seg[mid] <= r) lo = mid; else hi = mid;
  }
  return lo;
}

// out[r][c] = a[ra][ca] * b[rb][cb]: a per-graph operand (one row per graph) broadcasts over the
// graph's rows, a width-1 operand over the columns (tf.multiply broadcasting).
__global__ __launch_bounds__(kThreads) void product_kernel(ProductArgs p) {
  const int64_t total = p.n * p.F;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < total; i += (int64_t)gridDim.x * kThreads) {
    const int64_t r = i / p.F;
    const int c = (int)(i - r * p.F);
    int64_t g = 0;
    if (p.a_graph || p.b_graph) g = graph_of(p.seg, p.G, r);
    const int64_t ra = p.a_graph ? g : r, rb = p.b_graph ? g : r;
    const float va = p.a[ra * p.Fa + (p.Fa == 1 ? 0 : c)];
    const float vb = p.b[rb * p.Fb + (p.Fb == 1 ? 0 : c)];
    p.out[i] = va * vb;
  }
}

// dst[e][:] = src[idx[e]][:]  (tf.gather on axis 0)
__global__ __launch_bounds__(kThreads) void gather_kernel(const float* __restrict__ src, int F,
                                                           const int32_t* __restrict__ idx, int64_t n,
                                                           float* __restrict__ dst) {
  const int64_t total = n * F;
  for (int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x; i < total; i += (int64_t)gridDim.x * kThreads) {
    const int64_t e = i / F;
    const int c = (int)(i - e * F);
    dst[i] = src[(int64_t)idx[e] * F + c];
  }
}

int grid_of(int64_t total) {
  int64_t b = (total + kThreads - 1) / kThreads;
  if (b < 1) b = 1;
  return (int)(b < 16384 ? b : 16384);
}

// ---- backward (training through the readout operations) --------------------------------------
// tf.reduce_max's gradient splits equally among the rows that equal the maximum: their count
__global__ void pool_ties_kernel(const float* __restrict__ x, const float* __restrict__ y, int F,
                                 const int64_t* __restrict__ off, int G, float* __restrict__ ties) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (int64_t)G * F) return;
  const int g = (int)(i / F), c = (int)(i % F);
  float n = 0.f;
  for (int64_t r = off[g]; r < off[g + 1]; ++r) n += x[r * F + c] == y[i] ? 1.f : 0.f;
  ties[i] = n;
}

// dx[r] += dy[g(r)] (sum), / count (mean), or on the maximal rows / ties (max)
__global__ void pool_bwd_kernel(const float* __restrict__ x, const float* __restrict__ y,
                                const float* __restrict__ dy, const float* __restrict__ ties, int F,
                                const int64_t* __restrict__ off, int G, int mode, int64_t n,
                                float* __restrict__ dx) {
  const int64_t total = n * F;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / F;
    const int c = (int)(e - r * F);
    const int64_t g = graph_of(off, G, r);
    const int64_t gi = g * F + c;
    float v = dy[gi];
    if (mode == POOL_MEAN) v /= (float)(off[g + 1] - off[g]);
    else if (mode == POOL_MAX) v = x[e] == y[gi] ? v / ties[gi] : 0.f;
    dx[e] += v;
  }
}

// out = a * b (widths Fa / Fb, 1 broadcasts; a graph-space operand broadcasts over its graph's
// rows).  da[ra][ca] += sum over the output elements it fed of dout * b.  One thread per element
// of a: deterministic, no atomics.
__global__ void product_bwd_kernel(const float* __restrict__ dout, const float* __restrict__ b, int Fa, int Fb, int F,
                                   int a_graph, int b_graph, const int64_t* __restrict__ seg, int G, int64_t n_a,
                                   float* __restrict__ da) {
  const int64_t total = n_a * Fa;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t ra = e / Fa;
    const int ca = (int)(e - ra * Fa);
    const int64_t r0 = a_graph ? seg[ra] : ra, r1 = a_graph ? seg[ra + 1] : ra + 1;
    const int c0 = (Fa == 1 && F > 1) ? 0 : ca, c1 = (Fa == 1 && F > 1) ? F : ca + 1;
    float s = 0.f;
    for (int64_t r = r0; r < r1; ++r) {
      const int64_t rb = b_graph ? graph_of(seg, G, r) : r;
      for (int c = c0; c < c1; ++c) s += dout[r * F + c] * b[rb * Fb + (Fb == 1 ? 0 : c)];
    }
    da[e] += s;
  }
}

}  // namespace

hipError_t launch_pool(const float* x, int F, int64_t n_chunks, const int64_t* chunk, const int32_t* chunk_ptr,
                       const int64_t* count, int G, int mode, float* partial, float* out, hipStream_t st) {
  if (G == 0) return hipSuccess;
  if (n_chunks > 0) {
    hipLaunchKernelGGL(pool_partial_kernel, dim3((unsigned)n_chunks), dim3(kThreads), 0, st, x, F, chunk, mode,
                       partial);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL(pool_final_kernel, dim3((unsigned)G), dim3(kThreads), 0, st, partial, F, chunk_ptr, count, mode,
                     out);
  return hipGetLastError();
}

hipError_t launch_product(const ProductArgs& a, hipStream_t st) {
  if (a.n == 0) return hipSuccess;
  hipLaunchKernelGGL(product_kernel, dim3(grid_of(a.n * a.F)), dim3(kThreads), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_gather(const float* src, int F, const int32_t* idx, int64_t n, float* dst, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(gather_kernel, dim3(grid_of(n * F)), dim3(kThreads), 0, st, src, F, idx, n, dst);
  return hipGetLastError();
}

hipError_t launch_pool_bwd(const float* x, const float* y, const float* dy, float* ties, int F, const int64_t* off, int G,
                           int mode, int64_t n, float* dx, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (mode == POOL_MAX)
    hipLaunchKernelGGL(pool_ties_kernel, dim3((unsigned)(((int64_t)G * F + kThreads - 1) / kThreads)), dim3(kThreads), 0,
                       st, x, y, F, off, G, ties);
  const int64_t blocks = std::min<int64_t>((n * F + kThreads - 1) / kThreads, 16384);
  hipLaunchKernelGGL(pool_bwd_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, st, x, y, dy, ties, F, off, G, mode, n,
                     dx);
  return hipGetLastError();
}

hipError_t launch_product_bwd(const float* dout, const float* b, int Fa, int Fb, int F, int a_graph, int b_graph,
                              const int64_t* seg, int G, int64_t n_a, float* da, hipStream_t st) {
  if (n_a == 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((n_a * Fa + kThreads - 1) / kThreads, 16384);
  hipLaunchKernelGGL(product_bwd_kernel, dim3((unsigned)blocks), dim3(kThreads), 0, st, dout, b, Fa, Fb, F, a_graph,
                     b_graph, seg, G, n_a, da);
  return hipGetLastError();
}
