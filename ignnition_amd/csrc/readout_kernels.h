// readout_kernels.h — launchers for the readout operations before predict (GM:611-655).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

enum { POOL_SUM = 0, POOL_MEAN = 1, POOL_MAX = 2 };   // = enum ign_pooling
constexpr int64_t POOL_CHUNK = 4096;                 // rows per pooling partial

struct ProductArgs {
  const float* a;
  const float* b;
  int Fa, Fb, F;          // operand widths (1 broadcasts), output width
  int a_graph, b_graph;   // operand has one row per graph (broadcast over the graph's rows)
  const int64_t* seg;     // [G + 1] row offsets of the output space
  int G;
  int64_t n;              // output rows
  float* out;
};

// reduce over each graph's rows (tf.reduce_sum / reduce_mean / reduce_max on axis 0, AUX:1165-1185)
hipError_t launch_pool(const float* x, int F, int64_t n_chunks, const int64_t* chunk, const int32_t* chunk_ptr,
                       const int64_t* count, int G, int mode, float* partial, float* out, hipStream_t st);
// tf.multiply with per-graph / width-1 broadcasting (AUX:1081-1088)
hipError_t launch_product(const ProductArgs& a, hipStream_t st);
// tf.gather on axis 0 (AUX:1236-1265)
hipError_t launch_gather(const float* src, int F, const int32_t* idx, int64_t n, float* dst, hipStream_t st);

// backward (training): pooling over each graph's rows (off: [G + 1] row offsets of the input
// space; ties: [G][F] scratch for max), dx accumulated
hipError_t launch_pool_bwd(const float* x, const float* y, const float* dy, float* ties, int F, const int64_t* off, int G,
                           int mode, int64_t n, float* dx, hipStream_t st);
// d(a) of out = a * b (seg: [G + 1] row offsets of the output space), accumulated
hipError_t launch_product_bwd(const float* dout, const float* b, int Fa, int Fb, int F, int a_graph, int b_graph,
                              const int64_t* seg, int G, int64_t n_a, float* da, hipStream_t st);
