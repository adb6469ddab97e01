// kernels.hip — gfx950 (CDNA4) kernels of the message-passing engine.
//
// Every kernel works on the CSR tables built by engine.cpp; the layout in HBM is
// documented in DESIGN.md.  The GRU and readout contractions run on fp32-input MFMA
// (v_mfma_f32_16x16x4_f32: exact f32 fma chain, 64 FLOP/clk/SIMD = the chip's fp32 peak).
//
// Transposed formulation used everywhere: D[unit][row] = W^T[unit][k] * X^T[k][row], i.e.
// the MFMA A operand is a weight fragment and the B operand holds 16 graph rows
// (paths / links / nodes) on the lanes.  Lane l holds row j = l & 15 and, in the
// accumulator, units 16t + 4g + r (g = l >> 4, r = register 0..3).  The k order of
// every contraction is permuted as  k(s, g) = 16*(s>>2) + 4*g + (s&3)  so that
//   * the per-row input x is read as float4 chunks [16c + 4g, +4) of the row (one 64-B
//     segment per 4 lanes: a coalesced row gather), and
//   * an accumulator tile is directly the B operand of the next contraction: register
//     (s&3) of tile (s>>2) is exactly x[k(s,g)].  The GRU hidden state therefore never
//     leaves registers across the steps of a sequence (no LDS round trip, no shuffles).
// Weights are pre-packed (pack_* kernels) into that fragment order once per
// ign_plan_set_params, so a wave loads each fragment with one coalesced 256-B read.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include "kernels.h"

#include "device_common.h"

// ---------------------------------------------------------------------------------------------
// Hidden-state init (AUX:128-160): state[n] = [features[n] (F floats) | zeros(H - F)].
__global__ void init_state_kernel(float* __restrict__ state, const float* __restrict__ feats,
                                  int64_t n, int H, int F) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t total = n * (int64_t)H;
  for (; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t row = i / H;
    int c = (int)(i - row * H);
    state[i] = (c < F && feats) ? feats[row * F + c] : 0.0f;
  }
}

// The same with one float4 per thread and the row width a compile-time constant (H = 4 HQ): no
// 64-bit division per element, 16-B stores.
template <int HQ>
__global__ void init_state4_kernel(f4* __restrict__ state, const float* __restrict__ feats, int64_t n, int F) {
  const int64_t total = n * HQ;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = i / HQ;
    const int c = 4 * (int)(i - row * HQ);
    f4 v = f4{0, 0, 0, 0};
    if (c < F && feats) {
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = c + q < F ? feats[row * F + c + q] : 0.0f;
    }
    state[i] = v;
  }
}

// ---------------------------------------------------------------------------------------------
// GRU weight packing.  Keras GRUCell v2 layout: kernel [DIN][3H], recurrent_kernel [H][3H],
// bias [2][3H]; gate column order z, r, h (AUX:748-749).
// Packed fragment (gate, t, s), 64 lanes each, stored float4-grouped over s (see below):
//   lane l -> M[k(s, l>>4)][gate*H + 16t + (l&15)]
__global__ void pack_gru_kernel(const float* __restrict__ W, const float* __restrict__ U,
                                const float* __restrict__ bias, float* __restrict__ Wp,
                                float* __restrict__ Up, float* __restrict__ bp, int DIN, int H) {
  int NT = H / 16;
  int64_t nW = 3LL * NT * (DIN / 4) * 64;
  int64_t nU = 3LL * NT * (H / 4) * 64;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t total = Up ? nW + nU + 4LL * H : nW;   // Up == nullptr: W only (a concat slice)
  for (int64_t e = i; e < total; e += stride) {
    if (e < nW + nU) {
      // float4-grouped fragments: idx = (((gate*NT + t)*KS/4 + s/4)*64 + lane)*4 + s%4, so one
      // 16-B read per lane yields 4 consecutive k-steps (global dwordx4, ds_read_b128, LDS copy)
      bool isU = e >= nW;
      int64_t idx = isU ? e - nW : e;
      int KS = isU ? H / 4 : DIN / 4;
      int lane = (int)((idx >> 2) & 63);
      int64_t f4i = idx >> 8;               // (gate*NT + t)*KS/4 + s/4
      int s = (int)((f4i % (KS / 4)) * 4 + (idx & 3));
      int64_t gt = f4i / (KS / 4);
      int t = (int)(gt % NT);
      int gate = (int)(gt / NT);
      int k = 16 * (s >> 2) + 4 * (lane >> 4) + (s & 3);
      int col = gate * H + 16 * t + (lane & 15);
      const float sc = gate == 2 ? IGN_2LOG2E : IGN_NLOG2E;   // see sig2_/tanh2_
      if (isU) Up[idx] = sc * U[(int64_t)k * 3 * H + col];
      else     Wp[idx] = sc * W[(int64_t)k * 3 * H + col];
    } else {
      // combined, pre-scaled biases: [0] bz_in+bz_rec, [1] br_in+br_rec, [2] bh_in, [3] bh_rec
      int b = (int)(e - nW - nU);
      int which = b / H, u = b % H;
      const float* bin = bias;            // bias[0][:]
      const float* brec = bias + 3 * H;   // bias[1][:]
      float v;
      if (which == 0) v = IGN_NLOG2E * (bin[u] + brec[u]);
      else if (which == 1) v = IGN_NLOG2E * (bin[H + u] + brec[H + u]);
      else if (which == 2) v = IGN_2LOG2E * bin[2 * H + u];
      else v = IGN_2LOG2E * brec[2 * H + u];
      bp[b] = v;
    }
  }
}

// Dense kernel [IN][OUT] -> float4-grouped A fragments: ((u * (IN/16) + c) * 64 + lane) * 4 + q
//   -> W[16c + 4*(lane>>4) + q][16u + (lane&15)]; rows k >= IN_real (input padding) are zero
__global__ void pack_dense_kernel(const float* __restrict__ W, float* __restrict__ Wp, int IN, int OUT,
                                  int IN_real) {
  int64_t total = (int64_t)IN * OUT;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int q = (int)(i & 3);
    int lane = (int)((i >> 2) & 63);
    int64_t f = i >> 8;
    int C = IN / 16;
    int c = (int)(f % C);
    int u = (int)(f / C);
    int k = 16 * c + 4 * (lane >> 4) + q;
    int col = 16 * u + (lane & 15);
    Wp[i] = k < IN_real ? W[(int64_t)k * OUT + col] : 0.f;
  }
}

// ---------------------------------------------------------------------------------------------
// One GRU step for the wave's 16 rows (reset_after=True, AUX:764 / Keras GRUCell v2):
//   z = s(x Wz + h Uz + bz) ; r = s(x Wr + h Ur + br) ; c = tanh(x Wh + bhx + r (h Uh + bhh))
//   h' = z h + (1 - z) c
template <int DIN, int H>
struct GruWeights {
  static constexpr int NT = H / 16, KX = DIN / 4, KH = H / 4;
  float w[3][NT][KX];
  float u[3][NT][KH];
};

template <int DIN, int H>
__device__ __forceinline__ void load_gru_weights(GruWeights<DIN, H>& W, const float* __restrict__ Wp,
                                                 const float* __restrict__ Up, int lane) {
  constexpr int NT = H / 16, KX = DIN / 4, KH = H / 4;
#pragma unroll
  for (int g = 0; g < 3; ++g)
#pragma unroll
    for (int t = 0; t < NT; ++t) {
#pragma unroll
      for (int s = 0; s < KX; ++s) W.w[g][t][s] = Wp[frag_idx(g * NT + t, s, KX, lane)];
#pragma unroll
      for (int s = 0; s < KH; ++s) W.u[g][t][s] = Up[frag_idx(g * NT + t, s, KH, lane)];
    }
}

template <int DIN, int H>
__device__ __forceinline__ void gru_step(const GruWeights<DIN, H>& W, const float* __restrict__ sb,
                                         const f4 (&x)[DIN / 16], f4 (&h)[H / 16], int g) {
  constexpr int NT = H / 16, KX = DIN / 4, KH = H / 4;
  f4 az[NT], ar[NT], ax[NT], ah[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int u0 = 16 * t + 4 * g;
    az[t] = *reinterpret_cast<const f4*>(sb + 0 * H + u0);
    ar[t] = *reinterpret_cast<const f4*>(sb + 1 * H + u0);
    ax[t] = *reinterpret_cast<const f4*>(sb + 2 * H + u0);
    ah[t] = *reinterpret_cast<const f4*>(sb + 3 * H + u0);
  }
#pragma unroll
  for (int s = 0; s < KX; ++s) {
    const float xb = x[s >> 2][s & 3];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      az[t] = MFMA(W.w[0][t][s], xb, az[t]);
      ar[t] = MFMA(W.w[1][t][s], xb, ar[t]);
      ax[t] = MFMA(W.w[2][t][s], xb, ax[t]);
    }
  }
#pragma unroll
  for (int s = 0; s < KH; ++s) {
    const float hb = h[s >> 2][s & 3];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      az[t] = MFMA(W.u[0][t][s], hb, az[t]);
      ar[t] = MFMA(W.u[1][t][s], hb, ar[t]);
      ah[t] = MFMA(W.u[2][t][s], hb, ah[t]);
    }
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float z = sig2_(az[t][r]);
      const float rr = sig2_(ar[t][r]);
      const float c = tanh2_(ax[t][r] + rr * ah[t][r]);
      h[t][r] = c + z * (h[t][r] - c);
    }
  }
}

__device__ __forceinline__ const float* src_ptr(const SrcBases& sb, uint32_t code, int din) {
  uint32_t slot = code >> IGN_SLOT_SHIFT;
  uint32_t row = code & IGN_ROW_MASK;
  const float* b = sb.base[0];
  if (slot == 1) b = sb.base[1];
  if (slot == 2) b = sb.base[2];
  if (slot == 3) b = sb.base[3];
  return b + (int64_t)row * din;
}

// ---------------------------------------------------------------------------------------------
// Input projection of a message table: XW[row] = state[row] . W  (W = the destination cell's input
// kernel [DIN][3H], no bias).  x.W depends only on the source row, so the ordered update below
// gathers projected rows instead of recomputing x.W for every (destination, step): the
// recurrence keeps only h.U on the MFMA pipe.  Exact reassociation of the Keras cell
// (x.W + b_in) + (h.U + b_rec); holes project to 0 and duplicates sum linearly.
// Output row layout [3H]: gate-major z | r | h, same as the Keras kernel columns.
template <int DIN, int H>
__global__ __launch_bounds__(256) void project_kernel(const float* __restrict__ x, int64_t n,
                                                      const float* __restrict__ Wp, const float* __restrict__ bp,
                                                      float* __restrict__ out, float* __restrict__ bias_row) {
  // out points at this source's first row inside the MP's combined projected table.  Rows hold
  // x.W' + b' (pre-scaled, input-side biases [bz, br, bh_in]); bias_row (if set) receives b'
  // alone: the table row of a hole (zero input).
  constexpr int NC = DIN / 16, NT = H / 16, KX = DIN / 4;
  if (bias_row && blockIdx.x == 0)
    for (int i = threadIdx.x; i < 3 * H; i += blockDim.x) bias_row[i] = bp[i];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int j = lane & 15, g = lane >> 4;
  const int64_t r = ((int64_t)blockIdx.x * 4 + wave) * 16 + j;
  const bool valid = r < n;
  f4 xv[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) xv[c] = valid ? ld4(x + r * DIN + 16 * c + 4 * g) : f4{0, 0, 0, 0};
  f4 acc[3][NT];
#pragma unroll
  for (int G = 0; G < 3; ++G)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[G][t] = ld4(bp + G * H + 16 * t + 4 * g);
#pragma unroll
  for (int s = 0; s < KX; ++s) {
    const float xb = xv[s >> 2][s & 3];
#pragma unroll
    for (int G = 0; G < 3; ++G)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[G][t] = MFMA(Wp[frag_idx(G * NT + t, s, KX, lane)], xb, acc[G][t]);
  }
  if (valid) {
#pragma unroll
    for (int G = 0; G < 3; ++G)
#pragma unroll
      for (int t = 0; t < NT; ++t) st4(out + r * 3 * H + G * H + 16 * t + 4 * g, acc[G][t]);
  }
}

// ---------------------------------------------------------------------------------------------
// Positions that receive several messages (scatter_nd adds them, GM:490): row multi_base + k of
// the projected table = sum of the projected rows listed for k.  Rare; one thread per float4.
__global__ void multi_sum_kernel(float* __restrict__ table, int64_t multi_base, int64_t n_multi,
                                 const int32_t* __restrict__ ptr, const uint32_t* __restrict__ rows, int W,
                                 const float* __restrict__ bias_row) {
  // every projected row carries the input bias once; a sum of k rows must carry it once too
  const int64_t q = W / 4;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i < n_multi * q; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = i / q;
    const int c = (int)(i - k * q) * 4;
    f4 acc = f4{0, 0, 0, 0};
    for (int m = ptr[k]; m < ptr[k + 1]; ++m) acc += ld4(table + (int64_t)rows[m] * W + c);
    acc -= (float)(ptr[k + 1] - ptr[k] - 1) * ld4(bias_row + c);
    st4(table + (multi_base + k) * W + c, acc);
  }
}

// ---------------------------------------------------------------------------------------------
// Ordered / interleave / concat(axis 1) update: masked GRU over each destination's message
// sequence (AUX:767-796 with the dense-padding semantics of GM:477-543).  One wave = 16
// destinations of similar length (rows sorted by length, descending).  Step t of destination
// d reads row step_code[step_ptr[d] + t] of the MP's projected table: the projection of its
// message, the zero row for a hole (a padded position below final_len), or a pre-summed row
// where several messages share the position.  Steps t >= final_len[d] leave the state
// unchanged (sequence_mask); their (padded, always valid) codes are still read so the loop
// has no data-dependent branch or select.
// f32-MFMA form (v_mfma_f32_16x16x4_f32; the split-bf16 default is seq_gru_bf in kernels_bf.hip):
// the recurrent-kernel fragments live in LDS (12 KB per block at H=32, shared by its 4 waves).
// LDS image: float4 per lane holding 4 consecutive k-steps, [gate][unit tile][k-step/4][lane] ->
// one ds_read_b128 feeds 4 MFMAs.  Also the training forward's SAVE form at H = 16.
template <int H>
__device__ __forceinline__ void stage_frag_lds(f4* dst, const float* __restrict__ src, int KS) {
  // src is already float4-grouped ([3][NT][KS/4][64] x f4): a straight vector copy
  const int n = 3 * (H / 16) * (KS / 4) * 64;
  const f4* s4 = reinterpret_cast<const f4*>(src);
  for (int e = threadIdx.x; e < n; e += blockDim.x) dst[e] = s4[e];
}

template <int H, bool SAVE>
__global__ __launch_bounds__(256) void seq_gru2_kernel(SeqGruArgs a) {
  constexpr int NT = H / 16, KH = H / 4, K4 = KH / 4;
  __shared__ float sbias[4 * H];
  __shared__ f4 su[3 * NT * K4 * 64];
  for (int i = threadIdx.x; i < 4 * H; i += blockDim.x) sbias[i] = a.bias[i];
  stage_frag_lds<H>(su, a.Up, KH);

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int j = lane & 15, g = lane >> 4;
  const float* tab = a.table + 4 * g;
  __syncthreads();
  // Persistent over tiles: the grid is sized to residency and each wave strides over the
  // length-sorted tiles (so every wave gets a similar mix), paying the block prologue once.
  const int64_t n_tiles = (a.n_dst + 15) / 16;
  for (int64_t tile = xcd_block(a.xcd_remap) * 4 + wave; tile < n_tiles; tile += (int64_t)gridDim.x * 4) {
  const int64_t pos = tile * 16 + j;
  const bool valid = pos < a.n_dst;
  const int row = valid ? a.order[pos] : 0;
  const int L = valid ? a.len[pos] : 0;
  const uint32_t* codes = a.step_code + (valid ? a.step_ptr[pos] : 0);
  f4 h[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) h[t] = valid ? ld4(a.h_in + (int64_t)row * H + 16 * t + 4 * g) : f4{0, 0, 0, 0};
  int Lmax = L;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) Lmax = max(Lmax, __shfl_xor(Lmax, o));
  float* hsv = nullptr;
  if constexpr (SAVE) {          // training: keep h_0 .. h_L of the sequence for the backward
    hsv = a.hs_save + (valid ? (int64_t)a.step_ptr[pos] + pos : 0) * H + 4 * g;
    if (valid) {
#pragma unroll
      for (int t = 0; t < NT; ++t) st4(hsv + 16 * t, h[t]);
    }
  }

  uint32_t code = codes[0];
  for (int t = 0; t < Lmax; ++t) {
    f4 x[3][NT];
    {
      const float* p = tab + (int64_t)code * (3 * H);
#pragma unroll
      for (int G = 0; G < 3; ++G)
#pragma unroll
        for (int i = 0; i < NT; ++i) x[G][i] = ld4(p + G * H + 16 * i);
    }
    const uint32_t next = codes[t + 1];
    __builtin_amdgcn_sched_barrier(0);
    f4 az[NT], ar[NT], ah[NT];
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      az[i] = f4{0, 0, 0, 0};
      ar[i] = f4{0, 0, 0, 0};
      ah[i] = *reinterpret_cast<const f4*>(sbias + 3 * H + 16 * i + 4 * g);
    }
#pragma unroll
    for (int s4 = 0; s4 < K4; ++s4) {
#pragma unroll
      for (int i = 0; i < NT; ++i) {
        const f4 wz = su[((0 * NT + i) * K4 + s4) * 64 + lane];
        const f4 wr = su[((1 * NT + i) * K4 + s4) * 64 + lane];
        const f4 wh = su[((2 * NT + i) * K4 + s4) * 64 + lane];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float hb = h[s4][q];
          az[i] = MFMA(wz[q], hb, az[i]);
          ar[i] = MFMA(wr[q], hb, ar[i]);
          ah[i] = MFMA(wh[q], hb, ah[i]);
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    const bool act = t < L;
#pragma unroll
    for (int i = 0; i < NT; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {   // x rows carry the input-side biases (project_kernel)
        const float z = sig2_(az[i][r] + x[0][i][r]);
        const float rr = sig2_(ar[i][r] + x[1][i][r]);
        const float c = tanh2_(x[2][i][r] + rr * ah[i][r]);
        const float hn = c + z * (h[i][r] - c);
        h[i][r] = act ? hn : h[i][r];
      }
    }
    if constexpr (SAVE) {
      if (act && valid) {
#pragma unroll
        for (int i = 0; i < NT; ++i) st4(hsv + (int64_t)(t + 1) * H + 16 * i, h[i]);
      }
    }
    code = next;
  }
  if (valid) {
#pragma unroll
    for (int t = 0; t < NT; ++t) st4(a.h_out + (int64_t)row * H + 16 * t + 4 * g, h[t]);
  }
  }  // tile loop
}

// ---------------------------------------------------------------------------------------------
// Sum aggregation + single GRU step (AUX:254-262 then AUX:752-765).  Every destination is
// updated, with x = 0 when it receives no message.  One wave = 16 destinations of similar
// in-degree (sorted descending); each lane accumulates its quarter of the row in f32.
// MODE 0 sum (AUX:261); 1 attention: messages weighted by their softmax coefficient (AUX:339-342);
// 2 convolution: x = act((sum_m h_src . K + h) / deg) (AUX:384-401; K.sum = sum.K, exact
// reassociation).  Then one GRU step (AUX:764).
template <int DIN, int H, int MODE>
__global__ __launch_bounds__(256) void sum_gru_kernel(SumGruArgs a) {
  constexpr int NC = DIN / 16, NT = H / 16;
  __shared__ float sbias[4 * H];
  for (int i = threadIdx.x; i < 4 * H; i += blockDim.x) sbias[i] = a.bias[i];

  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int j = lane & 15, g = lane >> 4;
  GruWeights<DIN, H> W;                       // loaded once per wave (persistent over tiles)
  load_gru_weights<DIN, H>(W, a.Wp, a.Up, lane);
  __syncthreads();

  const int64_t n_tiles = (a.n_dst + 15) / 16;
  for (int64_t tile = xcd_block(a.xcd_remap) * 4 + wave; tile < n_tiles; tile += (int64_t)gridDim.x * 4) {
    const int64_t pos = tile * 16 + j;
    const bool valid = pos < a.n_dst;
    const int row = valid ? a.order[pos] : 0;
    const int64_t m0 = valid ? a.msg_ptr[pos] : 0;
    const int64_t m1 = valid ? a.msg_ptr[pos + 1] : 0;

    f4 x[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) x[c] = f4{0, 0, 0, 0};
    int64_t m = m0;
    if constexpr (MODE == 1) {
      for (; m < m1; ++m) {
        const float w = a.msg_w[m];
        const float* p = src_ptr(a.src, a.msg_src[m], DIN);
#pragma unroll
        for (int c = 0; c < NC; ++c) x[c] += ld4(p + 16 * c + 4 * g) * w;
      }
    } else {
      for (; m + 4 <= m1; m += 4) {
        uint32_t c0 = a.msg_src[m], c1 = a.msg_src[m + 1], c2 = a.msg_src[m + 2], c3 = a.msg_src[m + 3];
        const float* p0 = src_ptr(a.src, c0, DIN);
        const float* p1 = src_ptr(a.src, c1, DIN);
        const float* p2 = src_ptr(a.src, c2, DIN);
        const float* p3 = src_ptr(a.src, c3, DIN);
        f4 v0[NC], v1[NC], v2[NC], v3[NC];
#pragma unroll
        for (int c = 0; c < NC; ++c) {
          v0[c] = ld4(p0 + 16 * c + 4 * g);
          v1[c] = ld4(p1 + 16 * c + 4 * g);
          v2[c] = ld4(p2 + 16 * c + 4 * g);
          v3[c] = ld4(p3 + 16 * c + 4 * g);
        }
#pragma unroll
        for (int c = 0; c < NC; ++c) x[c] = (((x[c] + v0[c]) + v1[c]) + v2[c]) + v3[c];
      }
      for (; m < m1; ++m) {
        const float* p = src_ptr(a.src, a.msg_src[m], DIN);
#pragma unroll
        for (int c = 0; c < NC; ++c) x[c] += ld4(p + 16 * c + 4 * g);
      }
    }

    f4 h[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) h[t] = valid ? ld4(a.h_in + (int64_t)row * H + 16 * t + 4 * g) : f4{0, 0, 0, 0};
    if constexpr (MODE == 2) {
      static_assert(MODE != 2 || DIN == H, "convolution needs message dim == destination dim");
      if (a.sum_save && valid) {   // training: the message sum before the convolution kernel
#pragma unroll
        for (int c = 0; c < NC; ++c) st4(a.sum_save + (int64_t)row * DIN + 16 * c + 4 * g, x[c]);
      }
      f4 y[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) y[c] = f4{0, 0, 0, 0};
#pragma unroll
      for (int s = 0; s < DIN / 4; ++s) {
        const float xb = x[s >> 2][s & 3];
#pragma unroll
        for (int t = 0; t < NC; ++t) y[t] = MFMA(a.conv_kp[frag_idx(t, s, DIN / 4, lane)], xb, y[t]);
      }
      const float deg = (float)(m1 - m0);   // no neighbour: 0/0 or h/0, as the reference divides
#pragma unroll
      for (int c = 0; c < NC; ++c)
#pragma unroll
        for (int r = 0; r < 4; ++r) x[c][r] = act_apply((y[c][r] + h[c][r]) / deg, a.conv_act);
    }
    if (a.x_save && valid) {
#pragma unroll
      for (int c = 0; c < NC; ++c) st4(a.x_save + (int64_t)row * DIN + 16 * c + 4 * g, x[c]);
    }
    gru_step<DIN, H>(W, sbias, x, h, g);
    if (valid) {
#pragma unroll
      for (int t = 0; t < NT; ++t) st4(a.h_out + (int64_t)row * H + 16 * t + 4 * g, h[t]);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Windowed sum aggregation (see SumWinArgs).  1024 threads: wave w owns window positions
// 16w .. 16w+15 of its chunk, lanes as in sum_gru (row j, quarter g).  Per window the block
// copies source rows [wb, we) into LDS (coalesced f4 loads), then every lane adds the prefix of
// its ascending source list that falls in the window (8 index loads in flight).
template <int DIN, int WIN_ROWS>
__global__ __launch_bounds__(1024) void sum_win_kernel(SumWinArgs a) {
  constexpr int NC = DIN / 16, F4 = DIN / 4;
  __shared__ f4 win[WIN_ROWS * F4];
  const int64_t* w = a.wg + 4 * (int64_t)blockIdx.x;
  const int64_t pos0 = w[0], pos1 = w[1], s0 = w[2], s1 = w[3];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = lane & 15, g = lane >> 4;
  const int64_t pos = pos0 + 16 * wave + j;
  const bool valid = pos < pos1;
  int32_t m = valid ? a.ptr[pos] : 0;
  const int32_t m1 = valid ? a.ptr[pos + 1] : 0;
  f4 x[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) x[c] = f4{0, 0, 0, 0};
  for (int64_t wb = s0; wb < s1; wb += WIN_ROWS) {
    const int64_t we = wb + WIN_ROWS < s1 ? wb + WIN_ROWS : s1;
    if (wb != s0) __syncthreads();   // the previous window is consumed
    const f4* sv = reinterpret_cast<const f4*>(a.src) + wb * F4;
    const int n = (int)(we - wb) * F4;
    for (int i = threadIdx.x; i < n; i += 1024) win[i] = sv[i];
    __syncthreads();
    while (m < m1) {
      int32_t r[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) r[k] = m + k < m1 ? a.srow[m + k] : 0x7FFFFFFF;
      int k = 0;
#pragma unroll
      for (; k < 8; ++k) {
        if (r[k] >= we) break;
        const f4* row = win + (int64_t)(r[k] - wb) * F4 + g;
#pragma unroll
        for (int c = 0; c < NC; ++c) x[c] += row[4 * c];
      }
      m += k;
      if (k < 8) break;   // the window (or the list) ends inside this batch
    }
  }
  if (valid) {
    const int64_t d = a.dst[pos];
#pragma unroll
    for (int c = 0; c < NC; ++c) st4(a.xsum + d * DIN + 16 * c + 4 * g, x[c]);
  }
}

// High-degree sum (Q-size's path -> node MP: ~140 messages per node over few destinations): one
// wave per destination instead of four lanes, so a destination's messages are gathered RS rows per
// load instruction (RS = 64 / F4, F4 = DIN / 4 lanes per 16-B row piece), U loads in flight per
// lane with the next round's codes prefetched, and the long per-destination chains of the lane
// form become short ones across many waves.  Lane l adds message slots q = l / F4, q + RS, ... in
// CSR order (columns 4 (l % F4) .. + 3); the RS partial sums are then added pairwise across lanes
// (xor RS/2 ... 1 in units of F4 lanes): a fixed summation order, bitwise reproducible.
template <int DIN, int U>
__global__ __launch_bounds__(256) void sum_seg_kernel(SumSegArgs a) {
  constexpr int F4 = DIN / 4, RS = 64 / F4;
  const int lane = threadIdx.x & 63;
  const int64_t pos = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (pos >= a.n_dst) return;   // whole waves: no lane of a live wave leaves early
  const int c = lane % F4, q = lane / F4;
  const int64_t m0 = a.msg_ptr[pos], m1 = a.msg_ptr[pos + 1];
  const int64_t last = m1 > m0 ? m1 - 1 : m0;
  f4 acc = {0, 0, 0, 0};
  uint32_t cc[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t i = m0 + u * RS + q;
    cc[u] = m1 > m0 ? a.msg_src[i < last ? i : last] : 0u;
  }
  for (int64_t m = m0; m < m1; m += U * RS) {
    f4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = ld4(a.src + (int64_t)(cc[u] & IGN_ROW_MASK) * DIN + 4 * c);
#pragma unroll
    for (int u = 0; u < U; ++u) {   // the next round's codes, clamped into the range: no branch
      const int64_t i = m + (U + u) * RS + q;
      cc[u] = a.msg_src[i < last ? i : last];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool on = m + u * RS + q < m1;
      const f4 s = acc + v[u];
#pragma unroll
      for (int k = 0; k < 4; ++k) acc[k] = on ? s[k] : acc[k];
    }
  }
#pragma unroll
  for (int o = 32; o >= F4; o >>= 1)
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[k] += __shfl_xor(acc[k], o);
  if (q == 0) st4(a.xsum + (int64_t)a.order[pos] * DIN + 4 * c, acc);
}

hipError_t launch_sum_seg(const SumSegArgs& args, int din, hipStream_t st) {
  if (args.n_dst == 0) return hipSuccess;
  const dim3 grid((unsigned)((args.n_dst + 3) / 4)), block(256);
  if (din == 32) hipLaunchKernelGGL((sum_seg_kernel<32, 4>), grid, block, 0, st, args);
  else if (din == 16) hipLaunchKernelGGL((sum_seg_kernel<16, 4>), grid, block, 0, st, args);
  else if (din == 64) hipLaunchKernelGGL((sum_seg_kernel<64, 4>), grid, block, 0, st, args);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

// Attention softmax weights: one wave per (graph, position) group.
__global__ __launch_bounds__(256) void attn_softmax_kernel(AttnArgs a) {
  const int lane = threadIdx.x & 63;
  const int64_t grp = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (grp >= a.n_groups) return;
  const int c0 = a.group_ptr[grp], c1 = a.group_ptr[grp + 1];
  if (c0 == c1) return;   // only empty cells: no message reads this group
  float mx = a.group_empty[grp] > 0 ? 0.f : -INFINITY;
  for (int c = c0 + lane; c < c1; c += 64) {
    const float sd = a.s_dst[a.cell_dst[c]];
    float e = 0.f;
    for (int q = a.cell_ptr[c]; q < a.cell_ptr[c + 1]; ++q) {
      const uint32_t code = a.msg_src[a.cell_msgs[q]];
      const float v = a.s_src[code >> IGN_SLOT_SHIFT][code & IGN_ROW_MASK] + sd;
      e += v > 0.f ? v : 0.2f * v;                       // LeakyReLU(alpha=0.2), scatter_nd adds
    }
    a.ecell[c] = e;
    mx = fmaxf(mx, e);
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  float z = 0.f;
  for (int c = c0 + lane; c < c1; c += 64) z += __expf(a.ecell[c] - mx);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) z += __shfl_xor(z, o);
  z += (float)a.group_empty[grp] * __expf(-mx);         // empty cells hold 0
  const float inv = 1.0f / z;
  for (int c = c0 + lane; c < c1; c += 64) {
    const float w = __expf(a.ecell[c] - mx) * inv;
    for (int q = a.cell_ptr[c]; q < a.cell_ptr[c + 1]; ++q) a.msg_w[a.cell_msgs[q]] = w;
  }
}

__global__ void attn_vectors_kernel(const float* __restrict__ K1, const float* __restrict__ K2,
                                    const float* __restrict__ av, int F, float* __restrict__ w12) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= 2 * F) return;
  const float* K = i < F ? K1 : K2;
  const int r = i < F ? i : i - F;
  const float* aa = i < F ? av : av + F;
  float s = 0.f;
  for (int jj = 0; jj < F; ++jj) s += K[r * F + jj] * aa[jj];
  w12[i] = s;
}

// ---------------------------------------------------------------------------------------------
// Sum update for wide cells with the weights in LDS: W and U fragments (96 KB at 64/64) are
// staged once per block, so the per-tile weight stream (96 KB per 16 rows) comes from LDS
// instead of L2.  One 12-wave block per CU (3 waves per SIMD), persistent over the
// in-degree-sorted tiles.
template <int DIN, int H, int WAVES, int GU>
__global__ __launch_bounds__(64 * WAVES) void sum_gru_lds_kernel(SumGruArgs a) {
  constexpr int NC = DIN / 16, NT = H / 16, X4 = DIN / 16, H4 = H / 16;
  constexpr int WF = 3 * NT * X4 * 64, UF = 3 * NT * H4 * 64;   // float4 fragments
  __shared__ f4 sW[WF];
  __shared__ f4 sU[UF];
  __shared__ float sbias[4 * H];
  {
    const f4* gW = reinterpret_cast<const f4*>(a.Wp);
    const f4* gU = reinterpret_cast<const f4*>(a.Up);
    for (int i = threadIdx.x; i < WF; i += 64 * WAVES) sW[i] = gW[i];
    for (int i = threadIdx.x; i < UF; i += 64 * WAVES) sU[i] = gU[i];
    for (int i = threadIdx.x; i < 4 * H; i += 64 * WAVES) sbias[i] = a.bias[i];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int j = lane & 15, g = lane >> 4;
  const int64_t n_tiles = (a.n_dst + 15) / 16;
  for (int64_t tile = xcd_block(a.xcd_remap) * WAVES + wave; tile < n_tiles; tile += (int64_t)gridDim.x * WAVES) {
    const int64_t pos = tile * 16 + j;
    const bool valid = pos < a.n_dst;
    const int row = valid ? a.order[pos] : 0;
    const int64_t m0 = valid ? a.msg_ptr[pos] : 0;
    const int64_t m1 = valid ? a.msg_ptr[pos + 1] : 0;
    f4 h[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) h[t] = valid ? ld4(a.h_in + (int64_t)row * H + 16 * t + 4 * g) : f4{0, 0, 0, 0};
    f4 x[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) x[c] = f4{0, 0, 0, 0};
    int64_t m = m0;
    for (; m + GU <= m1; m += GU) {       // GU messages in flight per lane
      f4 v[GU][NC];
#pragma unroll
      for (int u = 0; u < GU; ++u) {
        const float* p = src_ptr(a.src, a.msg_src[m + u], DIN);
#pragma unroll
        for (int c = 0; c < NC; ++c) v[u][c] = ld4(p + 16 * c + 4 * g);
      }
#pragma unroll
      for (int u = 0; u < GU; ++u)
#pragma unroll
        for (int c = 0; c < NC; ++c) x[c] += v[u][c];
    }
    for (; m + 2 <= m1; m += 2) {
      const float* p0 = src_ptr(a.src, a.msg_src[m], DIN);
      const float* p1 = src_ptr(a.src, a.msg_src[m + 1], DIN);
      f4 v0[NC], v1[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        v0[c] = ld4(p0 + 16 * c + 4 * g);
        v1[c] = ld4(p1 + 16 * c + 4 * g);
      }
#pragma unroll
      for (int c = 0; c < NC; ++c) x[c] = (x[c] + v0[c]) + v1[c];
    }
    for (; m < m1; ++m) {
      const float* p = src_ptr(a.src, a.msg_src[m], DIN);
#pragma unroll
      for (int c = 0; c < NC; ++c) x[c] += ld4(p + 16 * c + 4 * g);
    }
    if (a.x_save && valid) {
#pragma unroll
      for (int c = 0; c < NC; ++c) st4(a.x_save + (int64_t)row * DIN + 16 * c + 4 * g, x[c]);
    }
    // the weight reads are loop-invariant: an opaque offset keeps the compiler from hoisting
    // all 96 KB of them out of the tile loop into (spilled) registers
    int wofs = lane;
    asm volatile("" : "+v"(wofs));
    f4 hn[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const int u0 = 16 * t + 4 * g;
      f4 az = *reinterpret_cast<const f4*>(sbias + 0 * H + u0);
      f4 ar = *reinterpret_cast<const f4*>(sbias + 1 * H + u0);
      f4 ax = *reinterpret_cast<const f4*>(sbias + 2 * H + u0);
      f4 ah = *reinterpret_cast<const f4*>(sbias + 3 * H + u0);
#pragma unroll
      for (int s4 = 0; s4 < X4; ++s4) {
        const f4 wz = sW[((0 * NT + t) * X4 + s4) * 64 + wofs];
        const f4 wr = sW[((1 * NT + t) * X4 + s4) * 64 + wofs];
        const f4 wh = sW[((2 * NT + t) * X4 + s4) * 64 + wofs];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float xb = x[s4][q];
          az = MFMA(wz[q], xb, az);
          ar = MFMA(wr[q], xb, ar);
          ax = MFMA(wh[q], xb, ax);
        }
      }
#pragma unroll
      for (int s4 = 0; s4 < H4; ++s4) {
        const f4 wz = sU[((0 * NT + t) * H4 + s4) * 64 + wofs];
        const f4 wr = sU[((1 * NT + t) * H4 + s4) * 64 + wofs];
        const f4 wh = sU[((2 * NT + t) * H4 + s4) * 64 + wofs];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float hb = h[s4][q];
          az = MFMA(wz[q], hb, az);
          ar = MFMA(wr[q], hb, ar);
          ah = MFMA(wh[q], hb, ah);
        }
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float z = sig2_(az[r]);
        const float rr = sig2_(ar[r]);
        const float c = tanh2_(ax[r] + rr * ah[r]);
        hn[t][r] = c + z * (h[t][r] - c);
      }
    }
    if (valid) {
#pragma unroll
      for (int t = 0; t < NT; ++t) st4(a.h_out + (int64_t)row * H + 16 * t + 4 * g, hn[t]);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Fused readout MLP (GM:611-629, RNJ:113-142): y = act2(act1(X W1 + b1) W2 + b2) . w3 + b3.
// One wave = 32 rows (two 16-row B tiles).  Layer-1 activations stay in registers in the
// accumulator layout (N1/16 tiles x 2) and feed layer 2 as B operands; layer 2 is produced
// 16 units at a time and immediately contracted with the 1-unit output layer, so the second
// hidden layer is never materialised.  W1/W2 fragments stream from L2 as float4 per lane.
template <int DIN, int N1, int N2, int ACT>
__global__ __launch_bounds__(256) void readout3_kernel(Readout3Args a) {
  constexpr int C0 = DIN / 16, U1 = N1 / 16, U2 = N2 / 16;
  __shared__ f4 sw2[2][U1 * 64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int j = lane & 15, g = lane >> 4;
  const int64_t base = ((int64_t)blockIdx.x * 4 + wave) * 32;

  // x B fragments for the two row tiles
  f4 xb[2][C0];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    int64_t r = base + 16 * p + j;
    bool ok = r < a.n_rows;
    const float* xr = a.x + (ok ? r : 0) * (int64_t)a.x_stride;
#pragma unroll
    for (int c = 0; c < C0; ++c) xb[p][c] = ok ? ld4(xr + 16 * c + 4 * g) : f4{0, 0, 0, 0};
  }

  f4 h1[U1][2];
#pragma unroll
  for (int u = 0; u < U1; ++u) {
    f4 b = ld4(a.b1 + 16 * u + 4 * g);
    f4 acc0 = b, acc1 = b;
#pragma unroll
    for (int c = 0; c < C0; ++c) {
      f4 w = ld4(a.W1p + ((((int64_t)u * C0 + c) << 6) + lane) * 4);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc0 = MFMA(w[q], xb[0][c][q], acc0);
        acc1 = MFMA(w[q], xb[1][c][q], acc1);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      acc0[r] = act_t<ACT>(acc0[r]);
      acc1[r] = act_t<ACT>(acc1[r]);
    }
    h1[u][0] = acc0;
    h1[u][1] = acc1;
  }

  // Layer 2, 16 output units (one 16 KB chunk of packed W2 fragments) at a time.  The chunk is
  // staged in LDS once per workgroup (4 waves share it) and double-buffered: the next chunk is
  // loaded into registers while this one feeds the MFMAs, then stored behind one barrier.
  constexpr int CH = U1 * 64;   // float4 per chunk
  static_assert(CH % 256 == 0, "chunk must split evenly over the block");
  constexpr int PER = CH / 256;
  const f4* W2v = reinterpret_cast<const f4*>(a.W2p);
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < PER; ++k) sw2[0][tid + 256 * k] = W2v[tid + 256 * k];
  __syncthreads();

  float y0 = 0.f, y1 = 0.f;
#pragma unroll 1
  for (int v = 0; v < U2; ++v) {
    const int cur = v & 1;
    // small per-chunk vectors first: vmcnt retires loads in issue order, so loading them after
    // the stage loads would make their first use wait for the whole next chunk
    const f4 b = ld4(a.b2 + 16 * v + 4 * g);
    const f4 w3 = ld4(a.w3 + 16 * v + 4 * g);
    // unconditional (wraps to chunk 0 on the last pass): a branch here would make the compiler
    // wait for these loads at the join before the first use of b
    const int nv = (v + 1) % U2;
    f4 stage[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) stage[k] = W2v[(int64_t)nv * CH + tid + 256 * k];
    __builtin_amdgcn_sched_barrier(0);   // keep the stage loads ahead of this chunk's MFMAs
    f4 acc0 = b, acc1 = b;
#pragma unroll
    for (int c = 0; c < U1; ++c) {
      const f4 w = sw2[cur][c * 64 + lane];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        acc0 = MFMA(w[q], h1[c][0][q], acc0);
        acc1 = MFMA(w[q], h1[c][1][q], acc1);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      y0 += w3[r] * act_t<ACT>(acc0[r]);
      y1 += w3[r] * act_t<ACT>(acc1[r]);
    }
#pragma unroll
    for (int k = 0; k < PER; ++k) sw2[cur ^ 1][tid + 256 * k] = stage[k];
    __syncthreads();
  }
  // reduce the four unit groups (lanes j, j+16, j+32, j+48)
  y0 += __shfl_xor(y0, 16);
  y1 += __shfl_xor(y1, 16);
  y0 += __shfl_xor(y0, 32);
  y1 += __shfl_xor(y1, 32);
  if (g == 0) {
    const float b3 = a.b3 ? a.b3[0] : 0.f;
    int64_t r0 = base + j, r1 = base + 16 + j;
    if (r0 < a.n_rows) a.y[r0] = act_apply(y0 + b3, a.act3);
    if (r1 < a.n_rows) a.y[r1] = act_apply(y1 + b3, a.act3);
  }
}

// Generic Dense layer (any shape): y[n][o] = act(sum_k x[n][k] W[k][o] + b[o]).  Used for
// readout stacks that do not match the fused 3-layer kernel.
__global__ void dense_generic_kernel(const float* __restrict__ x, int64_t n, int in, int x_stride,
                                     const float* __restrict__ W, const float* __restrict__ b, int out,
                                     int act, float* __restrict__ y) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t total = n * (int64_t)out;
  for (; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = i / out;
    int o = (int)(i - r * out);
    float acc = b ? b[o] : 0.f;
    const float* xr = x + r * x_stride;
    for (int k = 0; k < in; ++k) acc = fmaf(xr[k], W[(int64_t)k * out + o], acc);
    y[i] = act_apply(acc, act);
  }
}

// Column copy used to concatenate several readout inputs (GM:615-621).
__global__ void concat_cols_kernel(float* __restrict__ dst, int64_t n, int dst_stride, int col0,
                                   const float* __restrict__ src, int width) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  int64_t total = n * (int64_t)width;
  for (; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    int64_t r = i / width;
    int c = (int)(i - r * width);
    dst[r * dst_stride + col0 + c] = src[i];
  }
}

// Halo pack: dst[i] = src[idx[i]] for rows of `cols` floats.  One float4 per lane,
// consecutive lanes walk one row, so each gathered row is a coalesced 16*cols/4-byte read.
__global__ void gather_rows_kernel(const float* __restrict__ src, int64_t ld, const int32_t* __restrict__ idx,
                                   int64_t n, int cols, float* __restrict__ dst) {
  const int q = cols >> 2;                      // float4 per row
  const int64_t total = n * q;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / q;
    const int c = (int)(i - r * q);
    const float4 v = reinterpret_cast<const float4*>(src + (int64_t)idx[r] * ld)[c];
    reinterpret_cast<float4*>(dst + r * cols)[c] = v;
  }
}

// ---------------------------------------------------------------------------------------------
// Host-side launchers
static inline int grid_for(int64_t n, int per_block) { return (int)((n + per_block - 1) / per_block); }

hipError_t launch_init_state(float* state, const float* feats, int64_t n, int H, int F, hipStream_t st) {
  int64_t total = n * (int64_t)H;
  if ((H == 16 || H == 32 || H == 64) && (reinterpret_cast<uintptr_t>(state) & 15) == 0) {
    const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((total / 4 + 255) / 256, 16384));
    f4* s4 = reinterpret_cast<f4*>(state);
    if (H == 16) hipLaunchKernelGGL(init_state4_kernel<4>, dim3(blocks), dim3(256), 0, st, s4, feats, n, F);
    else if (H == 32) hipLaunchKernelGGL(init_state4_kernel<8>, dim3(blocks), dim3(256), 0, st, s4, feats, n, F);
    else hipLaunchKernelGGL(init_state4_kernel<16>, dim3(blocks), dim3(256), 0, st, s4, feats, n, F);
    return hipGetLastError();
  }
  int blocks = (int)std::min<int64_t>((total + 255) / 256, 8192);
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(init_state_kernel, dim3(blocks), dim3(256), 0, st, state, feats, n, H, F);
  return hipGetLastError();
}

hipError_t launch_pack_gru(const float* W, const float* U, const float* bias, float* Wp, float* Up, float* bp,
                           int DIN, int H, hipStream_t st) {
  hipLaunchKernelGGL(pack_gru_kernel, dim3(64), dim3(256), 0, st, W, U, bias, Wp, Up, bp, DIN, H);
  return hipGetLastError();
}

hipError_t launch_pack_dense(const float* W, float* Wp, int IN, int OUT, hipStream_t st) {
  return launch_pack_dense_pad(W, Wp, IN, IN, OUT, st);
}

hipError_t launch_pack_dense_pad(const float* W, float* Wp, int IN, int IN_pad, int OUT, hipStream_t st) {
  const int64_t total = (int64_t)IN_pad * OUT;
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((total + 255) / 256, 4096));
  hipLaunchKernelGGL(pack_dense_kernel, dim3(blocks), dim3(256), 0, st, W, Wp, IN_pad, OUT, IN);
  return hipGetLastError();
}

#define GRU_DISPATCH(KERNEL, DIN_, H_, ARGS, N)                                                      \
  if (din == DIN_ && h == H_) {                                                                   \
    hipLaunchKernelGGL((KERNEL<DIN_, H_>), dim3(grid_for(N, 64)), dim3(256), 0, st, ARGS);         \
    return hipGetLastError();                                                                     \
  }

bool gru_shape_supported(int din, int h) {
  return ((din == 16 || din == 32) && (h == 16 || h == 32)) || (din == 64 && h == 64);
}

hipError_t launch_project(const float* x, int64_t n, const float* Wp, const float* bp, float* out, float* bias_row,
                          int din, int h, hipStream_t st) {
  dim3 grid(std::max(1, grid_for(n, 64))), block(256);
  if (din == 32 && h == 32) hipLaunchKernelGGL((project_kernel<32, 32>), grid, block, 0, st, x, n, Wp, bp, out, bias_row);
  else if (din == 16 && h == 16) hipLaunchKernelGGL((project_kernel<16, 16>), grid, block, 0, st, x, n, Wp, bp, out, bias_row);
  else if (din == 16 && h == 32) hipLaunchKernelGGL((project_kernel<16, 32>), grid, block, 0, st, x, n, Wp, bp, out, bias_row);
  else if (din == 32 && h == 16) hipLaunchKernelGGL((project_kernel<32, 16>), grid, block, 0, st, x, n, Wp, bp, out, bias_row);
  else if (din == 64 && h == 64) hipLaunchKernelGGL((project_kernel<64, 64>), grid, block, 0, st, x, n, Wp, bp, out, bias_row);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_multi_sum(float* table, int64_t multi_base, int64_t n_multi, const int32_t* ptr,
                            const uint32_t* rows, int W, const float* bias_row, hipStream_t st) {
  if (n_multi == 0) return hipSuccess;
  int64_t total = n_multi * (W / 4);
  int blocks = (int)std::min<int64_t>((total + 255) / 256, 4096);
  hipLaunchKernelGGL(multi_sum_kernel, dim3(blocks), dim3(256), 0, st, table, multi_base, n_multi, ptr, rows, W,
                     bias_row);
  return hipGetLastError();
}

// Grid for a persistent kernel: resident blocks per CU (occupancy API) x CUs, at most the work.
template <typename K>
static int persistent_grid(K kernel, int64_t n_blocks_of_work, int block = 256) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, 0) != hipSuccess || per_cu <= 0) per_cu = 1;
  int64_t g = (int64_t)per_cu * cus;
  return (int)std::max<int64_t>(1, std::min<int64_t>(g, n_blocks_of_work));
}

hipError_t launch_seq_gru(const SeqGruArgs& args, int h, int variant, hipStream_t st) {
  if (args.n_dst == 0) return hipSuccess;
  // 6: split-fp16 h.U, 3 piece products; 4: split-bf16 h.U, 6 piece products (kernels_bf.hip;
  // H = 32, 64); 2: f32 MFMA.  (Round 3 dropped the 4-product fp16 and 9-product bf16 forms: no
  // caller after the full-batch precision study)
  if (variant == 6 && (h == 32 || h == 64) && args.Uh && args.hdr) return launch_seq_gru_h16(args, h, 3, st);
  if (variant >= 4 && (h == 32 || h == 64)) return launch_seq_gru_bf(args, h, 6, st);
  const int64_t work = grid_for(args.n_dst, 64);
  if (h == 32) {
    auto k = args.hs_save ? seq_gru2_kernel<32, true> : seq_gru2_kernel<32, false>;
    hipLaunchKernelGGL(k, dim3(persistent_grid(k, work)), dim3(256), 0, st, args);
  } else if (h == 16) {
    auto k = args.hs_save ? seq_gru2_kernel<16, true> : seq_gru2_kernel<16, false>;
    hipLaunchKernelGGL(k, dim3(persistent_grid(k, work)), dim3(256), 0, st, args);
  } else if (h == 64) {
    auto k = args.hs_save ? seq_gru2_kernel<64, true> : seq_gru2_kernel<64, false>;
    hipLaunchKernelGGL(k, dim3(persistent_grid(k, work)), dim3(256), 0, st, args);
  } else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_sum_win(const SumWinArgs& args, int din, hipStream_t st) {
  if (args.n_wg == 0) return hipSuccess;
  const dim3 grid((unsigned)args.n_wg), block(1024);
  if (din == 32) hipLaunchKernelGGL((sum_win_kernel<32, 1200>), grid, block, 0, st, args);
  else if (din == 16) hipLaunchKernelGGL((sum_win_kernel<16, 2400>), grid, block, 0, st, args);
  else if (din == 64) hipLaunchKernelGGL((sum_win_kernel<64, 600>), grid, block, 0, st, args);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

hipError_t launch_sum_gru(const SumGruArgs& args, int din, int h, int variant, hipStream_t st) {
  if (args.n_dst == 0) return hipSuccess;
  // one tile per wave: measured faster than a persistent grid for this latency-bound gather
  // (0.109 vs 0.141 ms on 512 x synth50): more independent waves queue behind the resident ones
  dim3 grid(grid_for(args.n_dst, 64));
  const int mode = args.conv_kp ? 2 : args.msg_w ? 1 : 0;
  // variant 7 (default): split-bf16 GRU step where its kernels exist (plain sums at DIN = H = 32
  // or 64); otherwise the f32-MFMA kernels
  if (din == 32 && h == 32 && mode == 0 && variant == 7 && args.Wbf && args.Ubf)
    return launch_sum_gru_g32(args, 6, st);   // 6 rows in flight: 0.100 ms vs 0.105 (8), 0.108 (4)
  if (args.proj_out) return hipErrorInvalidValue;   // the fused projection exists in sum_gru_g32 only
#define SUM_CASE(D, HH)                                                                    \
  if (din == D && h == HH) {                                                               \
    if (mode == 1) hipLaunchKernelGGL((sum_gru_kernel<D, HH, 1>), grid, dim3(256), 0, st, args); \
    else if (mode == 2 && D == HH) hipLaunchKernelGGL((sum_gru_kernel<D, (D == HH ? HH : D), (D == HH ? 2 : 0)>), grid, dim3(256), 0, st, args); \
    else if (mode == 2) return hipErrorInvalidValue;                                       \
    else hipLaunchKernelGGL((sum_gru_kernel<D, HH, 0>), grid, dim3(256), 0, st, args);    \
    return hipGetLastError();                                                              \
  }
  SUM_CASE(32, 32)
  SUM_CASE(16, 16)
  SUM_CASE(16, 32)
  SUM_CASE(32, 16)
#undef SUM_CASE
  if (din == 64 && h == 64) {
    if (mode != 0) return hipErrorInvalidValue;
    if (variant == 8 && args.Wbf && args.Ubf) return launch_sum_gru_h16(args, din, h, st);
    if (variant == 7 && args.Wbf && args.Ubf) return launch_sum_gru_bf(args, din, h, st);
    constexpr int WV = 12;   // f32 MFMA, W / U in LDS, 4 rows in flight per lane
    auto kern = sum_gru_lds_kernel<64, 64, WV, 4>;
    const int64_t work = (args.n_dst + 16 * WV - 1) / (16 * WV);
    hipLaunchKernelGGL(kern, dim3(persistent_grid(kern, work, 64 * WV)), dim3(64 * WV), 0, st, args);
    return hipGetLastError();
  }
  return hipErrorInvalidValue;
}

bool readout3_supported(int din, int n1, int n2, int act1, int act2) {
  return (din == 16 || din == 32 || din == 64) && n1 == 256 && n2 == 256 && act1 == act2;
}

template <int DIN>
static hipError_t readout3_din(const Readout3Args& args, int act, dim3 grid, hipStream_t st) {
  switch (act) {
    case IGN_K_ACT_SELU: hipLaunchKernelGGL((readout3_kernel<DIN, 256, 256, IGN_K_ACT_SELU>), grid, dim3(256), 0, st, args); break;
    case IGN_K_ACT_RELU: hipLaunchKernelGGL((readout3_kernel<DIN, 256, 256, IGN_K_ACT_RELU>), grid, dim3(256), 0, st, args); break;
    case IGN_K_ACT_TANH: hipLaunchKernelGGL((readout3_kernel<DIN, 256, 256, IGN_K_ACT_TANH>), grid, dim3(256), 0, st, args); break;
    case IGN_K_ACT_SIGMOID: hipLaunchKernelGGL((readout3_kernel<DIN, 256, 256, IGN_K_ACT_SIGMOID>), grid, dim3(256), 0, st, args); break;
    default: hipLaunchKernelGGL((readout3_kernel<DIN, 256, 256, IGN_K_ACT_LINEAR>), grid, dim3(256), 0, st, args); break;
  }
  return hipGetLastError();
}

hipError_t launch_readout3(const Readout3Args& args, int din, int n1, int n2, hipStream_t st) {
  if (args.n_rows == 0) return hipSuccess;
  if (!readout3_supported(din, n1, n2, args.act1, args.act2)) return hipErrorInvalidValue;
  dim3 grid(grid_for(args.n_rows, 128));
  if (din == 32) return readout3_din<32>(args, args.act1, grid, st);
  if (din == 16) return readout3_din<16>(args, args.act1, grid, st);
  return readout3_din<64>(args, args.act1, grid, st);
}

hipError_t launch_dense_generic(const float* x, int64_t n, int in, int x_stride, const float* W, const float* b,
                                int out, int act, float* y, hipStream_t st) {
  int64_t total = n * (int64_t)out;
  int blocks = (int)std::min<int64_t>((total + 255) / 256, 16384);
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(dense_generic_kernel, dim3(blocks), dim3(256), 0, st, x, n, in, x_stride, W, b, out, act, y);
  return hipGetLastError();
}

hipError_t launch_concat_cols(float* dst, int64_t n, int dst_stride, int col0, const float* src, int width,
                              hipStream_t st) {
  int64_t total = n * (int64_t)width;
  int blocks = (int)std::min<int64_t>((total + 255) / 256, 8192);
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(concat_cols_kernel, dim3(blocks), dim3(256), 0, st, dst, n, dst_stride, col0, src, width);
  return hipGetLastError();
}

hipError_t launch_gather_rows(const float* src, int64_t ld, const int32_t* idx, int64_t n, int cols, float* dst,
                              hipStream_t st) {
  if (n <= 0) return hipSuccess;
  const int64_t total = n * (cols / 4);
  int blocks = (int)std::min<int64_t>((total + 255) / 256, 16384);
  hipLaunchKernelGGL(gather_rows_kernel, dim3(blocks), dim3(256), 0, st, src, ld, idx, n, cols, dst);
  return hipGetLastError();
}

hipError_t launch_attn_softmax(const AttnArgs& a, hipStream_t st) {
  if (a.n_groups == 0) return hipSuccess;
  hipLaunchKernelGGL(attn_softmax_kernel, dim3((unsigned)((a.n_groups + 3) / 4)), dim3(256), 0, st, a);
  return hipGetLastError();
}

hipError_t launch_attn_vectors(const float* K1, const float* K2, const float* a, int F, float* w12, hipStream_t st) {
  hipLaunchKernelGGL(attn_vectors_kernel, dim3((2 * F + 63) / 64), dim3(64), 0, st, K1, K2, a, F, w12);
  return hipGetLastError();
}

__global__ void msg_gather_kernel(MsgGatherArgs a) {
  const int64_t total = a.n * a.ld;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t e = i / a.ld;
    const int c = (int)(i - e * a.ld);
    float v = 0.f;
    for (int q = 0; q < a.nparts; ++q)
      if (c >= a.col[q] && c < a.col[q] + a.width[q]) {
        const int64_t r = a.rows[q] ? a.rows[q][e] : e;
        v = a.base[q][r * a.width[q] + (c - a.col[q])];
      }
    a.out[i] = v;
  }
}

hipError_t launch_msg_gather(const MsgGatherArgs& a, hipStream_t st) {
  if (a.n == 0) return hipSuccess;
  const int64_t total = a.n * a.ld;
  const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((total + 255) / 256, 65536));
  hipLaunchKernelGGL(msg_gather_kernel, dim3(blocks), dim3(256), 0, st, a);
  return hipGetLastError();
}
