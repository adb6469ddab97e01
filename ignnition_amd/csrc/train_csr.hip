// train_csr.hip — the training tables' transposed CSRs, built on the GPU (round 6).
//
// ign_batch_enable_training's largest host sections on a 512 x synth50 batch were the transposed
// CSRs of the MPs (source row -> the steps / destination rows that read it; csr_gather_add sums a
// row's gradient over them): 14 + 8 ms of one batch builder's ~100 ms, a counting sort whose fill
// pass scatters over 15 MB.  Here the same arrays come from a stable radix sort (hipCUB) of
// (row key, value) pairs on the builder's upload stream, from the step / message tables already on
// the device:
//   ordered MP (no multi rows): step i -> key = its table row (a hole: zero_row, past every row),
//                               value i;
//   sum MP:                     message m of sorted position pos -> key = its code (slot in the
//                               high bits, row below), value order[pos].
// The host built them in the same emission order (steps / messages ascending) and the sort is
// stable, so every row lists its values in the same order: the same arrays, bitwise.  The row
// pointers come from a lower_bound per row over the sorted keys; they index the one sorted value
// array that every source slot shares (csr_gather_add reads idx[ptr[r] .. ptr[r + 1])).
#include <hip/hip_runtime.h>

#include <hipcub/hipcub.hpp>

#include "kernels.h"

namespace {

__global__ void tcsr_seq_keys_kernel(const uint32_t* __restrict__ code, int64_t n, uint32_t zero_row,
                                     uint32_t* __restrict__ keys, int32_t* __restrict__ vals) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t c = code[i];
    keys[i] = c < zero_row ? c : zero_row;
    vals[i] = (int32_t)i;
  }
}

// one thread per sorted position: its messages' codes and its destination row
__global__ void tcsr_sum_keys_kernel(const int32_t* __restrict__ msg_ptr, const int32_t* __restrict__ order,
                                     int64_t n_dst, const uint32_t* __restrict__ msg_src,
                                     uint32_t* __restrict__ keys, int32_t* __restrict__ vals) {
  for (int64_t pos = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; pos < n_dst;
       pos += (int64_t)gridDim.x * blockDim.x) {
    const int32_t d = order[pos];
    for (int32_t m = msg_ptr[pos]; m < msg_ptr[pos + 1]; ++m) {
      keys[m] = msg_src[m];
      vals[m] = d;
    }
  }
}

// ptr[r] = the first sorted position whose key is >= key0 + r, r = 0 .. rows (inclusive)
__global__ void tcsr_ptr_kernel(const uint32_t* __restrict__ sorted, int64_t n, uint32_t key0, int64_t rows,
                                int32_t* __restrict__ ptr) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r <= rows; r += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t key = key0 + (uint32_t)r;
    int64_t lo = 0, hi = n;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (sorted[mid] < key) lo = mid + 1;
      else hi = mid;
    }
    ptr[r] = (int32_t)lo;
  }
}

unsigned grid_of(int64_t n) { return (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 4096)); }

int bits_for(uint64_t max_key) {
  int b = 1;
  while (b < 32 && (max_key >> b)) ++b;
  return b;
}

}  // namespace

size_t tcsr_temp_bytes(int64_t n) {
  size_t bytes = 0;
  hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                     (const int32_t*)nullptr, (int32_t*)nullptr, (int)n, 0, 32);
  return bytes;
}

hipError_t launch_tcsr_keys_seq(const uint32_t* step_code, int64_t n_steps, uint32_t zero_row, uint32_t* keys,
                                int32_t* vals, hipStream_t st) {
  if (n_steps == 0) return hipSuccess;
  hipLaunchKernelGGL(tcsr_seq_keys_kernel, dim3(grid_of(n_steps)), dim3(256), 0, st, step_code, n_steps, zero_row,
                     keys, vals);
  return hipGetLastError();
}

hipError_t launch_tcsr_keys_sum(const int32_t* msg_ptr, const int32_t* order, int64_t n_dst, const uint32_t* msg_src,
                                uint32_t* keys, int32_t* vals, hipStream_t st) {
  if (n_dst == 0) return hipSuccess;
  hipLaunchKernelGGL(tcsr_sum_keys_kernel, dim3(grid_of(n_dst)), dim3(256), 0, st, msg_ptr, order, n_dst, msg_src,
                     keys, vals);
  return hipGetLastError();
}

hipError_t launch_tcsr_sort(void* temp, size_t temp_bytes, const uint32_t* keys_in, uint32_t* keys_out,
                            const int32_t* vals_in, int32_t* vals_out, int64_t n, uint32_t max_key, hipStream_t st) {
  if (n == 0) return hipSuccess;
  return hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, keys_in, keys_out, vals_in, vals_out, (int)n, 0,
                                            bits_for(max_key), st);
}

hipError_t launch_tcsr_ptr(const uint32_t* sorted_keys, int64_t n, uint32_t key0, int64_t rows, int32_t* ptr,
                           hipStream_t st) {
  hipLaunchKernelGGL(tcsr_ptr_kernel, dim3(grid_of(rows + 1)), dim3(256), 0, st, sorted_keys, n, key0, rows, ptr);
  return hipGetLastError();
}
