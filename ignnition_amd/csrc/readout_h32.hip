// readout_h32.hip — the fused readout Dense(256) -> Dense(256) -> Dense(1) (GM:611-629) on
// v_mfma_f32_32x32x16_f16: readout variant 5 (IGN_READOUT_VARIANT=5; round 6, measured slower than
// variant 4 and kept as the record of that experiment, DESIGN.md §3b'''').
//
// The same arithmetic class as readout_h16 (kernels_bf.hip, variant 4): both layers on scaled
// two-piece fp16 operands (device_common.h split2h), three piece products per fp32 product, fp32
// accumulation; the same power-of-two scales per row tile (W1 by sigma1, W2 by sigma2 at pack time,
// the layer-1 input of a tile by S1 = 2^(15 - E(max |x|)), max floored at 1, the layer-2 input by S
// from the a-priori bound on the layer-1 activations).  What changes is the matrix instruction and
// the loop order.  The premise (MI355X_MICROARCH.md, row 'vector-instruction ISSUE cost'): a 16x16x32
// MFMA holds the SIMD's vector issue for 8 of its 16 cycles, a 32x32x16 one for 8 of its 32, so the
// 32x32 form leaves three times the issue slots beside the same matrix work to the activations, the
// fp16 splits and the w3 dot product.  Measured (512 x synth50 rows, one launch): 0.64-0.71 ms against
// readout_h16's 0.54; timing-only ablations put 19 % in the W2 DMA issue, 15 % in layer 2's
// activation and 16 % in layer 1's -- with one wave per SIMD (the 128 accumulator registers of a
// 32-row tile plus its fragments need more than the 256 of two waves per SIMD) the VALU issues at
// one wave's rate (4 cycles) and does not fit the MFMA shadow.  So variant 4 stays the default.
//
// Layout.  Rows on the B side (32 rows per wave tile, one row per lane pair: lane l holds row
// l & 31, half h = l >> 5), units on the A side, D[unit][row].  A 32x32 accumulator holds units
// (q & 3) + 8 (q >> 2) + 4 h of its 32-unit tile in register q, so registers 8s .. 8s+7 are the
// B fragment of the next layer's k-step s with the k order permuted (cdna_hip_programming.md
// §Fragment layout): layer 2's k-step 2u + s reads layer-1 unit 32u + 16s + 8(j >> 2) + 4h + (j & 3)
// in element j, and W2's pieces are packed in that order.  Layer 1 reads its input rows from memory
// in natural k order (8 consecutive floats per lane and k-step).
// Loop order: k-outer for layer 2.  Layer-1 tile u (32 units) is formed, activated and split, then
// contracted into all eight layer-2 accumulators (256 units x 32 rows = 128 registers) as their
// k-steps 2u, 2u + 1; the next tile's layer-1 MFMAs and VALU sit between these MFMAs (hand-placed
// slices).  W2 is streamed through LDS by chunks of 32 input units (32 KB: every output tile's two
// k-steps, both pieces) by LDS-DMA, double-buffered, one barrier per chunk; W1's pieces stay in LDS.
// SAVE (the training forward): the layer-1 and layer-2 activations are written out unscaled, as
// readout_h16<SAVE> does.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <cstdlib>

#include "kernels.h"
#include "device_common.h"

namespace {

typedef float f16v __attribute__((ext_vector_type(16)));
#define MFMA32(a, b, c) __builtin_amdgcn_mfma_f32_32x32x16_f16((a), (b), (c), 0, 0, 0)

constexpr int kN1 = 256, kN2 = 256;
constexpr int kWaves = 4;                       // 1 per SIMD: 512 registers (the layer-2 accumulators in AGPRs)
constexpr int kChunkFrags = 8 * 2 * 2 * 64;     // 16-B fragments per W2 chunk: 8 out tiles x 2 k-steps x 2 pieces
constexpr float kLam = 1.0507009873554805f, kLa = kLam * 1.6732632423543772f, kLog2e = 1.4426950408889634f;

int num_cus() {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  return cus;
}

// So act(zs c) for zs = z / c (c, So powers of two) -- readout_h16's act_scaled (kernels_bf.hip)
template <int ACT>
__device__ __forceinline__ float act_sc(float zs, float c, float k, float cl, float laS, float So) {
  if constexpr (ACT == IGN_K_ACT_RELU) return zs > 0.f ? zs * k : 0.f;
  else if constexpr (ACT == IGN_K_ACT_SELU) {
    const float e = __builtin_amdgcn_exp2f(__builtin_amdgcn_fmed3f(zs, -3.0e38f, 0.f) * cl);
    return fmaf(k, __builtin_amdgcn_fmed3f(zs, 0.f, 3.0e38f), fmaf(laS, e, -laS));
  } else if constexpr (ACT == IGN_K_ACT_LINEAR) return zs * k;
  else return So * act_t<ACT>(zs * c);
}

}  // namespace

// Pieces of the variant-5 packed buffer (same size and header positions as variant 4's):
// [W2 pieces | 64-float header: e(sigma2), A, B | W1 pieces | 64-float header: e(sigma1)]
// W2: chunk u (layer-1 units 32u .. 32u + 31), out tile v, k-step s, piece p, lane, j (fp16):
//     piece p of sigma2 W2[32u + 16s + 8(j >> 2) + 4(lane >> 5) + (j & 3)][32v + (lane & 31)]
// W1: tile u, k-step s (DIN / 16 of them), piece p, lane, j:
//     piece p of sigma1 W1[16s + 8(lane >> 5) + j][32u + (lane & 31)]
// The headers are pack_readout_h16_kernel's (launch_pack_readout_h16 writes them).
__global__ __launch_bounds__(256) void pack_readout_h32_frag_kernel(const float* __restrict__ W1,
                                                                    const float* __restrict__ W2,
                                                                    uint16_t* __restrict__ out, int IN1) {
  const int64_t total2 = (int64_t)kN1 * kN2 * 2, total1 = (int64_t)IN1 * kN1 * 2;
  uint16_t* o1 = out + total2 + 128;
  const float sigma2 = __int_as_float((127 + reinterpret_cast<const int*>(out + total2)[0]) << 23);
  const float sigma1 = __int_as_float((127 + reinterpret_cast<const int*>(o1 + total1)[0]) << 23);
  const int KS1 = IN1 / 16;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total2 + total1;
       e += (int64_t)gridDim.x * blockDim.x) {
    const bool l2 = e < total2;
    const int64_t ee = l2 ? e : e - total2;
    const int j = (int)(ee & 7), lane = (int)((ee >> 3) & 63);
    const int r = lane & 31, h = lane >> 5;
    int64_t f = ee >> 9;
    const int piece = (int)(f & 1);
    f >>= 1;
    float v;
    if (l2) {   // f = (u * 8 + vt) * 2 + s
      const int s = (int)(f & 1), vt = (int)((f >> 1) & 7), u = (int)(f >> 4);
      const int k = 32 * u + 16 * s + 8 * (j >> 2) + 4 * h + (j & 3);
      v = sigma2 * W2[(int64_t)k * kN2 + 32 * vt + r];
    } else {    // f = u * KS1 + s
      const int s = (int)(f % KS1), u = (int)(f / KS1);
      v = sigma1 * W1[(int64_t)(16 * s + 8 * h + j) * kN1 + 32 * u + r];
    }
    const _Float16 hi = (_Float16)v;
    const _Float16 pc = piece == 0 ? hi : (_Float16)(v - (float)hi);
    (l2 ? out : o1)[ee] = __builtin_bit_cast(uint16_t, pc);
  }
}

template <int DIN, int ACT, bool SAVE>
__global__ __launch_bounds__(64 * kWaves) __attribute__((amdgpu_waves_per_eu(1, 1)))
void readout_h32_kernel(Readout3Args a, const h8* __restrict__ Wp) {
  constexpr int KS1 = DIN / 16;                  // layer-1 k-steps of 16
#ifndef IGN_RO32_RT
#define IGN_RO32_RT 1
#endif
  // 32-row tiles per wave (each W2 fragment read feeds 3 RT MFMAs).  RT = 2 (-DIGN_RO32_RT=2, DIN 32)
  // needs the 256 accumulators of both tiles in AGPRs and spills ~340 VGPRs: not built by default
  constexpr int RT = DIN == 32 ? IGN_RO32_RT : 1;
  constexpr int W1F = 8 * KS1 * 2 * 64;          // W1 fragments (16 B)
  constexpr int NTH = 64 * kWaves;
  constexpr int PER = kChunkFrags / NTH;         // LDS-DMA pieces (1 KB per wave-instruction) per wave and chunk
  constexpr int ROWS = 32 * RT * kWaves;         // rows per block and W2 pass
  static_assert(kChunkFrags % NTH == 0, "whole DMA pieces per wave");
  __shared__ h8 sw2[2][kChunkFrags];             // the W2 ring: 2 x 32 KB (chunk u in slot u & 1)
  __shared__ h8 sw1[W1F];                        // 32 KB (DIN 32) / 64 KB (DIN 64)
  __shared__ float sb[3][kN1];                   // b1 | b2 | w3
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const u4v* W2v = reinterpret_cast<const u4v*>(Wp);
  const h8* W1f = reinterpret_cast<const h8*>(reinterpret_cast<const float*>(Wp) + kN1 * kN2 + 64);
  {
    const u4v* src = reinterpret_cast<const u4v*>(W1f);
    for (int i = tid; i < W1F; i += NTH) reinterpret_cast<u4v*>(sw1)[i] = src[i];
  }
  for (int i = tid; i < kN1; i += NTH) {
    sb[0][i] = a.b1[i];
    sb[1][i] = a.b2[i];
    sb[2][i] = a.w3[i];
  }
  const int es1 = reinterpret_cast<const int*>(W1f + W1F)[0];
  const int* hdr = reinterpret_cast<const int*>(reinterpret_cast<const float*>(Wp) + kN1 * kN2);
  const int es2 = hdr[0];
  const float A1 = __int_as_float(hdr[1]), B1 = __int_as_float(hdr[2]);
  const float b3 = a.b3 ? a.b3[0] : 0.f;
  const int64_t n_groups = (a.n_rows + ROWS - 1) / ROWS;
  // W2 chunk c into ring slot `slot` (compile-time after unrolling) by LDS-DMA (readout_bf_kernel:
  // why asm, and M0); this wave's pieces wave, wave + 4, ...: M0 = its first piece's LDS address + a
  // constant, one scalar add per piece
  const uint32_t m0w = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)(sw2[0] + wave * 64));
  const u4v* srcw = W2v + wave * 64 + lane;
  auto dma_chunk = [&](int c, int slot) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const uint32_t m0 = m0w + (uint32_t)((slot * kChunkFrags + kWaves * k * 64) * 16);
      const u4v* src = srcw + (int64_t)c * kChunkFrags + kWaves * k * 64;
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
#ifndef IGN_RO32_ABL_NODMA   // timing ablation (wrong results): the ring keeps its first chunk
      asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(m0) : "memory", "m0");
#else
      if (c == 0) asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src), "s"(m0) : "memory", "m0");
#endif
#pragma clang diagnostic pop
    }
  };
  if ((int64_t)blockIdx.x < n_groups) dma_chunk(0, 0);
  // the input rows of a group: lane (r, h) of tile t holds x[row][16 s + 8 h .. + 7] for each k-step s
  f4 xl[RT][KS1][2];
  auto load_x = [&](int64_t grp) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      const int64_t row = grp * ROWS + (wave * RT + t) * 32 + r;
      const bool ok = row < a.n_rows;
      const float* xr = a.x + (ok ? row : 0) * (int64_t)a.x_stride + 8 * h;
#pragma unroll
      for (int s = 0; s < KS1; ++s) {
        xl[t][s][0] = ok ? ld4(xr + 16 * s) : f4{0, 0, 0, 0};
        xl[t][s][1] = ok ? ld4(xr + 16 * s + 4) : f4{0, 0, 0, 0};
      }
    }
  };
  load_x(blockIdx.x);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  f16v acc2[RT][8];   // layer 2: 256 units x 32 rows per tile (accumulation registers)
  for (int64_t grp = blockIdx.x; grp < n_groups; grp += gridDim.x) {
    const bool more = grp + (int64_t)gridDim.x < n_groups;
    int64_t row[RT];
    float S[RT], SS[RT], cSS[RT], S1S[RT], c1[RT], k1[RT];
    h8 xf[RT][KS1][2];
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      row[t] = grp * ROWS + (wave * RT + t) * 32 + r;
      // the tile's scales (readout_h16: the max over its rows of |x|, floored at 1)
      float mx = 1.f;
#pragma unroll
      for (int s = 0; s < KS1; ++s)
#pragma unroll
        for (int q = 0; q < 4; ++q) mx = fmaxf(mx, fmaxf(fabsf(xl[t][s][0][q]), fabsf(xl[t][s][1][q])));
      mx = wave_max_nonneg(mx);
      const float bnd = fmaf(fmaf(A1, mx, B1), 1.0508f, 1.7582f);
      const int E = (__builtin_amdgcn_readfirstlane(__float_as_int(bnd)) >> 23) - 126;   // bnd < 2^E
      const int eS = 15 - E;
      S[t] = __int_as_float((127 + eS) << 23);
      SS[t] = __int_as_float((127 + eS + es2) << 23);
      cSS[t] = __int_as_float((127 - eS - es2) << 23);
      const int E1 = (__builtin_amdgcn_readfirstlane(__float_as_int(fmaxf(mx, 1e-18f))) >> 23) - 126;
      const int eS1 = min(60, max(-60, 15 - E1));
      const float S1 = __int_as_float((127 + eS1) << 23);
      S1S[t] = __int_as_float((127 + eS1 + es1) << 23);
      c1[t] = __int_as_float((127 - eS1 - es1) << 23);
      k1[t] = (ACT == IGN_K_ACT_SELU ? kLam : 1.0f) * S[t] * c1[t];
#pragma unroll
      for (int s = 0; s < KS1; ++s) {
        const f4 lo = xl[t][s][0] * S1, hi = xl[t][s][1] * S1;
        const hpair p0 = split2h(lo[0], lo[1]), p1 = split2h(lo[2], lo[3]);
        const hpair p2 = split2h(hi[0], hi[1]), p3 = split2h(hi[2], hi[3]);
        const u4v w0 = {p0.hi, p1.hi, p2.hi, p3.hi}, w1 = {p0.lo, p1.lo, p2.lo, p3.lo};
        xf[t][s][0] = __builtin_bit_cast(h8, w0);
        xf[t][s][1] = __builtin_bit_cast(h8, w1);
      }
#pragma unroll
      for (int v = 0; v < 8; ++v)
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const f4 b = *reinterpret_cast<const f4*>(&sb[1][32 * v + 8 * m + 4 * h]) * SS[t];
#pragma unroll
          for (int e = 0; e < 4; ++e) acc2[t][v][4 * m + e] = b[e];
        }
    }
    // the next group's input rows load during this group (xl is dead from here on)
    if (more) load_x(grp + gridDim.x);
    // Layer-1 tile u of row tile t: x3 fp16 products from W1's pieces in LDS (l1_mfma), the activation
    // on the layer-2 scale (l1_act, four values at a time), the two fp16 pieces of layer 2's k-steps
    // 2u, 2u + 1 (l1_split: registers 8s .. 8s + 7).  The chunk loop places these pieces between its
    // MFMAs by hand (sched_barrier fences), so their VALU runs beside the matrix pipe.
    auto l1_mfma = [&](int u, int t, f16v& acc) __attribute__((always_inline)) {
#pragma unroll
      for (int m = 0; m < 4; ++m) {
        const f4 b = *reinterpret_cast<const f4*>(&sb[0][32 * u + 8 * m + 4 * h]) * S1S[t];
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[4 * m + e] = b[e];
      }
      int lofs = lane;   // opaque: the fragment addresses stay inside the loop
      asm volatile("" : "+v"(lofs));
#pragma unroll
      for (int s = 0; s < KS1; ++s) {
        const h8 w0 = sw1[((u * KS1 + s) * 2 + 0) * 64 + lofs];
        const h8 w1 = sw1[((u * KS1 + s) * 2 + 1) * 64 + lofs];
        acc = MFMA32(w1, xf[t][s][0], acc);
        acc = MFMA32(w0, xf[t][s][1], acc);
        acc = MFMA32(w0, xf[t][s][0], acc);
      }
    };
    auto l1_act = [&](int u, int t, f16v& acc, int m) __attribute__((always_inline)) {   // registers 4m .. 4m + 3
#ifndef IGN_RO32_ABL_NOL1V   // timing ablation (wrong results): no layer-1 activation
#pragma unroll
      for (int e = 0; e < 4; ++e)
        acc[4 * m + e] = act_sc<ACT>(acc[4 * m + e], c1[t], k1[t], c1[t] * kLog2e, kLa * S[t], S[t]);
#endif
      if constexpr (SAVE) {
        if (row[t] < a.n_rows) {
          const float iS = __int_as_float((254 - ((__float_as_int(S[t]) >> 23) & 255)) << 23);   // 1 / S, exact
          st4(a.save1 + row[t] * kN1 + 32 * u + 8 * m + 4 * h,
              f4{acc[4 * m], acc[4 * m + 1], acc[4 * m + 2], acc[4 * m + 3]} * iS);
        }
      }
    };
    auto l1_split = [&](const f16v& v, h8 (&hf)[2][2], int s) __attribute__((always_inline)) {
      u4v w0, w1;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const hpair p = split2h(v[8 * s + 2 * q], v[8 * s + 2 * q + 1]);
        w0[q] = p.hi;
        w1[q] = p.lo;
      }
      hf[s][0] = __builtin_bit_cast(h8, w0);
      hf[s][1] = __builtin_bit_cast(h8, w1);
    };
    h8 hfb[2][RT][2][2];   // [chunk parity][row tile][k-step][piece]
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      f16v a1;
      l1_mfma(0, t, a1);
#pragma unroll
      for (int m = 0; m < 4; ++m) l1_act(0, t, a1, m);
      l1_split(a1, hfb[0][t], 0);
      l1_split(a1, hfb[0][t], 1);
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int slot = u & 1;
      // the next chunk's DMA into the other slot (its previous chunk was released by the barrier)
      if (u < 7) dma_chunk(u + 1, slot ^ 1);
      else if (more) dma_chunk(0, slot ^ 1);
      int lofs = lane;
      asm volatile("" : "+v"(lofs));
      const h8* wb = sw2[slot] + lofs;
      // the chunk's 16 fragment pairs (out tile v = i / 2, k-step s = i % 2), each read one step
      // ahead and used by 3 RT MFMAs; beside them the next layer-1 tile: its MFMAs (i = 0), its
      // activation (i = 2 .. 9, one row tile's four values at a time), its split (i = 12 .. 15)
      h8 wc0 = wb[0], wc1 = wb[64];
      f16v a1[RT];
      if (u < 7)
#pragma unroll
        for (int t = 0; t < RT; ++t) l1_mfma(u + 1, t, a1[t]);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int v = i >> 1, sk = i & 1;
        h8 wn0 = wc0, wn1 = wc1;
        if (i < 15) {
          wn0 = wb[((i + 1) * 2 + 0) * 64];
          wn1 = wb[((i + 1) * 2 + 1) * 64];
        }
        // W2 lo x a hi, W2 hi x {a lo, a hi}
#pragma unroll
        for (int t = 0; t < RT; ++t) acc2[t][v] = MFMA32(wc1, hfb[u & 1][t][sk][0], acc2[t][v]);
#pragma unroll
        for (int t = 0; t < RT; ++t) acc2[t][v] = MFMA32(wc0, hfb[u & 1][t][sk][1], acc2[t][v]);
#pragma unroll
        for (int t = 0; t < RT; ++t) acc2[t][v] = MFMA32(wc0, hfb[u & 1][t][sk][0], acc2[t][v]);
        if (u < 7) {
          constexpr int A0 = 2, SPL = 12;   // act slices i = A0 .. A0 + 4 RT - 1; split slices SPL ..
          if (i >= A0 && i < A0 + 4 * RT) l1_act(u + 1, (i - A0) >> 2, a1[(i - A0) >> 2], (i - A0) & 3);
          if (i >= SPL && i < SPL + 2 * RT) l1_split(a1[(i - SPL) >> 1], hfb[(u & 1) ^ 1][(i - SPL) >> 1], (i - SPL) & 1);
        }
        __builtin_amdgcn_sched_barrier(0);
        wc0 = wn0;
        wc1 = wn1;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the DMA has landed (for every wave: barrier)
      __syncthreads();
    }
    // layer 2's activation on its scale and the 1-unit output layer, per lane over its 128 units,
    // then the two lane halves of the row
#pragma unroll
    for (int t = 0; t < RT; ++t) {
      float y = 0.f;
#pragma unroll
      for (int v = 0; v < 8; ++v)
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          const f4 w3 = *reinterpret_cast<const f4*>(&sb[2][32 * v + 8 * m + 4 * h]);
          f4 av;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
#ifndef IGN_RO32_ABL_NOEPI   // timing ablation (wrong results): no layer-2 activation
            av[e] = act_sc<ACT>(acc2[t][v][4 * m + e], cSS[t], ACT == IGN_K_ACT_SELU ? kLam : 1.0f, cSS[t] * kLog2e,
                                kLa * SS[t], SS[t]);
#else
            av[e] = acc2[t][v][4 * m + e];
#endif
            y = fmaf(w3[e], av[e], y);
          }
          if constexpr (SAVE)
            if (row[t] < a.n_rows) st4(a.save2 + row[t] * kN2 + 32 * v + 8 * m + 4 * h, av * cSS[t]);
        }
      y += __shfl_xor(y, 32);
      if (h == 0 && row[t] < a.n_rows) a.y[row[t]] = act_apply(fmaf(y, cSS[t], b3), a.act3);
    }
  }
}

template <int DIN, int ACT>
static void readout_h32_launch(const Readout3Args& args, const h8* w, hipStream_t st) {
  auto k = args.save1 ? readout_h32_kernel<DIN, ACT, true> : readout_h32_kernel<DIN, ACT, false>;
  constexpr int rows = 32 * (DIN == 32 ? IGN_RO32_RT : 1) * kWaves;
  const int64_t groups = (args.n_rows + rows - 1) / rows;
  const int64_t grid = std::max<int64_t>(1, std::min<int64_t>(groups, num_cus()));
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(64 * kWaves), 0, st, args, w);
}

template <int DIN>
static void readout_h32_din(const Readout3Args& args, const h8* w, hipStream_t st) {
  switch (args.act1) {
    case IGN_K_ACT_SELU: readout_h32_launch<DIN, IGN_K_ACT_SELU>(args, w, st); break;
    case IGN_K_ACT_RELU: readout_h32_launch<DIN, IGN_K_ACT_RELU>(args, w, st); break;
    case IGN_K_ACT_TANH: readout_h32_launch<DIN, IGN_K_ACT_TANH>(args, w, st); break;
    case IGN_K_ACT_SIGMOID: readout_h32_launch<DIN, IGN_K_ACT_SIGMOID>(args, w, st); break;
    default: readout_h32_launch<DIN, IGN_K_ACT_LINEAR>(args, w, st); break;
  }
}

hipError_t launch_readout_h32(const Readout3Args& args, const void* Wh, int din, hipStream_t st) {
  if (args.n_rows == 0) return hipSuccess;
  if ((din != 32 && din != 64) || !Wh || !args.b1 || !args.b2 || !args.w3 || args.act1 != args.act2 ||
      (args.save1 != nullptr) != (args.save2 != nullptr))
    return hipErrorInvalidValue;
  const h8* w = static_cast<const h8*>(Wh);
  if (din == 32) readout_h32_din<32>(args, w, st);
  else readout_h32_din<64>(args, w, st);
  return hipGetLastError();
}

// the headers by pack_readout_h16_kernel (the same positions), then the variant-5 pieces
hipError_t launch_pack_readout_h32(const float* W1, const float* b1, const float* W2, void* out, int in1, int n1,
                                   int n2, hipStream_t st) {
  if (n1 != kN1 || n2 != kN2 || (in1 != 32 && in1 != 64)) return hipErrorInvalidValue;
  hipError_t e = launch_pack_readout_h16_header(W1, b1, W2, out, in1, n1, n2, st);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(pack_readout_h32_frag_kernel, dim3(128), dim3(256), 0, st, W1, W2, static_cast<uint16_t*>(out), in1);
  return hipGetLastError();
}
