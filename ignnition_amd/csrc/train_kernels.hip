// train_kernels.hip — gfx950 kernels of the training step (backward + optimizer).
//
// Same MFMA conventions as kernels.hip (transposed formulation D[unit][row], k order
// k(s, g) = 16(s>>2) + 4g + (s&3), so an accumulator tile is the next contraction's B operand).
// The backward contractions that run along a row (dh = gu.U^T, dx = ga.W^T, readout dX = dz.W^T)
// use "A" fragments of the matrix itself (pack_a: tiles over its rows, k over its columns).
// Weight gradients are contractions over rows (sum_r A[r]^T B[r]): tsgemm_kernel puts the rows
// on the MFMA k axis and writes one partial tile per row chunk; reduce_add sums the chunks in a
// fixed order, so every gradient is deterministic.
//
// Gate math of the backward (Keras GRUCell v2, reset_after=True; u = h.U + b_rec, a = x.W + b_in):
//   z = s(a_z + u_z), r = s(a_r + u_r), c = tanh(a_h + r u_h), h' = z h + (1 - z) c
//   dz = dh' (h - c) z (1 - z);  dc = dh' (1 - z)(1 - c^2);  dr = dc u_h r (1 - r)
//   da = (dz, dr, dc);  du = (dz, dr, dc r);  dh = dh' z + du.U^T;  dx = da.W^T
// z, r, c are recomputed exactly as the forward computed them (pre-scaled pre-activations,
// sig2_/tanh2_), u_h is unscaled from the pre-scaled accumulator.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>
#include <stdlib.h>

#include "device_common.h"
#include "kernels.h"
#include "train_kernels.h"

namespace {

constexpr float kInv2Log2e = 0.34657359027997264f;   // 1 / (2 log2 e)

__device__ __forceinline__ float act_grad(float a, int act) {
  // derivative of the activation expressed through its output a
  switch (act) {
    case IGN_K_ACT_RELU: return a > 0.f ? 1.f : 0.f;
    case IGN_K_ACT_SELU: {
      const float lam = 1.0507009873554805f, la = 1.0507009873554805f * 1.6732632423543772f;
      return a > 0.f ? lam : a + la;
    }
    case IGN_K_ACT_SIGMOID: return a * (1.f - a);
    case IGN_K_ACT_TANH: return 1.f - a * a;
    default: return 1.f;
  }
}

// pack_a: Mat [rows][cols] row-major -> float4-grouped A fragments, tiles over rows, k over cols:
//   element ((t * KS/4 + s/4) * 64 + lane) * 4 + s%4 = Mat[16t + (lane&15)][k(s, lane>>4)], KS = cols/4
__global__ void pack_a_kernel(const float* __restrict__ M, int rows, int cols, float* __restrict__ out) {
  const int64_t total = (int64_t)rows * cols;
  const int KS = cols / 4;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int q = (int)(i & 3);
    const int lane = (int)((i >> 2) & 63);
    const int64_t f = i >> 8;
    const int s = (int)((f % (KS / 4)) * 4 + q);
    const int t = (int)(f / (KS / 4));
    const int k = 16 * (s >> 2) + 4 * (lane >> 4) + (s & 3);
    out[i] = M[(int64_t)(16 * t + (lane & 15)) * cols + k];
  }
}

// ---------------------------------------------------------------------------------------------
// Ordered update backward.  One wave = the forward's 16-row tile (same order), steps in reverse.
// Lanes whose sequence is shorter skip the step (mask): their gradient passes through.
// H <= 32: the U and U^T fragments (2 x 12 KB at H = 32) are staged in LDS per block; read from L2
// per MFMA they cost 24 KB of L2 reads per wave-step (measured 1.34 ms per launch at 512 x synth50).
// FUSE (H 16 / 32): persistent waves also form the recurrent-kernel gradient dU = sum h_prev^T du
// on the MFMA instead of writing du per step for a separate row contraction: each step, h_prev and
// du are transposed through a per-wave LDS tile ([unit][row], 4-row groups XOR-swizzled by unit so
// a lane reads its 4 rows as one b128), rows on the MFMA k axis (row 4kk + ks for lane group kk,
// k-step ks).  Each wave writes one (H + 2) x 3H partial (row H: the column sums of da = b_in's
// gradient, row H + 1: those of du = b_rec's; they differ in the h gate only, dc vs dc r), so no
// separate column-sum pass over ga is needed; launch_seq_gru_bwd reduces the partials in a fixed order.
// RC, the gate recompute of h.U (H = 32), on the forward's own path so that the recomputed gates
// are bitwise the forward's (the same pieces, scales, MFMA order and bias seeding):
// 0: f32 MFMA (seq_gru2); 1: split-bf16 x6 (seq_gru_bf); 2: scaled split-fp16 x3 (seq_gru_h16<SAVE>,
// the tile's state scale recomputed from its saved first states exactly as the forward formed it).
template <int H, bool FUSE, int RC = 0>
__global__ __launch_bounds__(256, 2) void seq_gru_bwd_kernel(SeqBwdArgs a) {
  constexpr int NT = H / 16, KH = H / 4, K3 = 3 * H / 4, KS = H / 32;
  constexpr bool BF = RC == 1, H16 = RC == 2;
  constexpr bool LDSU = H <= 32;
  static_assert(!FUSE || LDSU, "fused dU: H 16 / 32");
  static_assert(RC == 0 || H == 32, "split recompute: H 32");
  constexpr int KS3 = 3 * H / 32;                  // H16: k-steps of dh = du . U^T on 16x16x32
  constexpr int NUP = LDSU && RC == 0 ? 3 * NT * KH * 64 : 1, NUT = LDSU && !H16 ? NT * K3 * 64 : 1;
  constexpr int NUB = BF ? 9 * NT * KS * 64 : 1;   // bf8 fragments of U's pieces
  constexpr int NUH = H16 ? 6 * NT * KS * 64 : 1;  // h8 fragments of sigma U's fp16 pieces
  constexpr int NUTH = H16 ? 2 * NT * KS3 * 64 : 1;   // h8 fragments of sigma_t U (dh's A operand)
  constexpr int NTR = FUSE ? 4 * 3 * H * 16 : 1;   // per-wave transpose tiles
  __shared__ float sUp[NUP];
  __shared__ bf8 sUb[NUB];
  __shared__ h8 sUh[NUH];
  __shared__ h8 sUth[NUTH];
  __shared__ float sUt[NUT];
  __shared__ float sT[NTR];
  int es = 0, est = 0;   // H16: sigma's and sigma_t's exponents (pack_u_f16_kernel, pack_ut_f16_kernel)
  if constexpr (LDSU) {
    if constexpr (BF) {
      for (int e = threadIdx.x; e < NUB; e += blockDim.x)
        reinterpret_cast<u4v*>(sUb)[e] = static_cast<const u4v*>(a.Ubf)[e];
    } else if constexpr (H16) {
      for (int e = threadIdx.x; e < NUH; e += blockDim.x)
        reinterpret_cast<u4v*>(sUh)[e] = static_cast<const u4v*>(a.Uh)[e];
      es = __float_as_int(static_cast<const float*>(a.Uh)[(int64_t)NUH * 4]);
      for (int e = threadIdx.x; e < NUTH; e += blockDim.x)
        reinterpret_cast<u4v*>(sUth)[e] = static_cast<const u4v*>(a.Uth)[e];
      est = __float_as_int(static_cast<const float*>(a.Uth)[(int64_t)NUTH * 4]);
    } else {
      for (int e = threadIdx.x; e < NUP / 4; e += blockDim.x)
        reinterpret_cast<f4*>(sUp)[e] = reinterpret_cast<const f4*>(a.Up)[e];
    }
    if constexpr (!H16)
      for (int e = threadIdx.x; e < NUT / 4; e += blockDim.x)
        reinterpret_cast<f4*>(sUt)[e] = reinterpret_cast<const f4*>(a.Ut)[e];
    __syncthreads();
  }
  const float* Up = LDSU ? sUp : a.Up;
  const float* Ut = LDSU ? sUt : a.Ut;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int j = lane & 15, g = lane >> 4;
  f4 dU[NT][3 * NT], bsum[NT], bz[NT], br[NT], bc[NT];
#pragma unroll
  for (int mt = 0; mt < NT; ++mt) {
    bsum[mt] = f4{0, 0, 0, 0};
    bz[mt] = f4{0, 0, 0, 0};
    br[mt] = f4{0, 0, 0, 0};
    bc[mt] = f4{0, 0, 0, 0};
#pragma unroll
    for (int nt = 0; nt < 3 * NT; ++nt) dU[mt][nt] = f4{0, 0, 0, 0};
  }
  float* R = sT + (FUSE ? wave * (3 * H * 16) : 0);
  // transpose-tile offsets: write (unit 16t + 4g + q, row j); read (unit 16x + j, rows 4g .. 4g+3)
  const int wofs = j ^ (4 * g), rofs = j * 16 + 4 * (g ^ ((j >> 2) & 3));
  const int64_t n_tiles = (a.n_dst + 15) / 16;
  f4 bh0[NT];   // the candidate's recurrent bias (the accumulator seed; H16: times the tile's SS)
#pragma unroll
  for (int t = 0; t < NT; ++t) bh0[t] = ld4(a.bias + 3 * H + 16 * t + 4 * g);
  const int64_t tile_stride = FUSE ? (int64_t)gridDim.x * 4 : n_tiles;
  // hdr (seq_bwd_hdr_kernel, padded to whole tiles): per position {row, len, step_ptr, the code of
  // its last step}.  The wave loads its next tile's headers while the current tile runs, so a tile
  // starts by issuing its dh rows, first states and last step's rows together (one round trip).
  int64_t tile = (int64_t)blockIdx.x * 4 + wave;
  i4v hd = *reinterpret_cast<const i4v*>(a.hdr + 4 * (min(tile, n_tiles - 1) * 16 + j));
  // FUSE: persistent waves (static tile order: deterministic partials); otherwise one tile per wave
  for (; tile < n_tiles; tile += tile_stride) {
    const int64_t pos = tile * 16 + j;
    const bool valid = pos < a.n_dst;
    const int row = hd[0];
    const int L = hd[1];
    const int64_t sp = valid ? hd[2] : 0;
    // where this lane's ga stores go once past its sequence (seq_gru_bwd's FUSE store rule below):
    // its own step 0 row, or for a padding position the pad slot (its step_ptr, row n_steps)
    const int gpast = hd[2];
    const uint32_t code_last = (uint32_t)hd[3];
    const int64_t hbase = valid ? sp + pos : 0;
    f4 dh[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) dh[t] = valid ? ld4(a.dh_in + (int64_t)row * H + 16 * t + 4 * g) : f4{0, 0, 0, 0};
    f4 h0[NT];   // H16: the tile's first states, for the forward's tile scale
    if constexpr (H16) {
#pragma unroll
      for (int t = 0; t < NT; ++t) h0[t] = ld4(a.h_in + (int64_t)row * H + 16 * t + 4 * g);
    }
    // positions are sorted by length, descending: lane 0 (position tile * 16) is the longest
    const int Lmax = __builtin_amdgcn_readfirstlane(L);
    // A step's state row and projected rows are loaded during the step before it (in the reverse
    // order), before that step's stores: gfx9's vmcnt counts stores too, in issue order, so a load
    // issued after a store would be waited for with it.  A lane past its sequence reads step 0 (the
    // first loaded step, Lmax - 1: its own last step; masked either way).  Step codes are loaded
    // two steps ahead, so a step's row loads never wait for its code.
    f4 hp[NT], x[3][NT];
    // a step's h_prev; step 0's is the state before the MP, read from that state version (h_in): the
    // resident training forward does not save it as hs row hbase (the batched one does; same bits)
    auto load_rows = [&](int64_t hr, uint32_t code) __attribute__((always_inline)) {
      const float* hsrc = hr == hbase ? a.h_in + (int64_t)row * H : a.hs + hr * H;
#pragma unroll
      for (int t = 0; t < NT; ++t) hp[t] = ld4(hsrc + 16 * t + 4 * g);
#pragma unroll
      for (int G = 0; G < 3; ++G)
#pragma unroll
        for (int t = 0; t < NT; ++t) x[G][t] = ld4(a.table + (int64_t)code * (3 * H) + G * H + 16 * t + 4 * g);
    };
    auto code_of = [&](int st) { return a.step_code[sp + (st < L ? st : 0)]; };
    load_rows(hbase + (L > 0 ? L - 1 : 0), code_last);
    uint32_t code_n1 = Lmax >= 2 ? code_of(Lmax - 2) : 0u;   // the code of step `step - 1`
    hd = *reinterpret_cast<const i4v*>(a.hdr + 4 * (min(tile + tile_stride, n_tiles - 1) * 16 + j));
    f4 bh[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) bh[t] = bh0[t];
    // H16: the forward's tile scale, from the tile's first states (saved as read): S = 2^(15 - E),
    // m = max(1, max |h_0|) = f 2^E; SS = S sigma, cS = 1 / SS.  After the first iteration every
    // |h| <= 1, so a ballot settles m and the cross-lane reduction runs only for a larger state
    float S = 1.f, SS = 1.f, cS = 1.f;
    if constexpr (H16) {
      float m = 1.0f;
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) m = fmaxf(m, valid ? fabsf(h0[t][r]) : 0.f);
      if (__ballot(m > 1.0f) != 0) {
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
      }
      const int E = (__builtin_amdgcn_readfirstlane(__float_as_int(m)) >> 23) - 126;
      const int eS = 15 - E;
      S = __int_as_float((127 + eS) << 23);
      SS = __int_as_float((127 + eS + es) << 23);
      cS = __int_as_float((127 - eS - es) << 23);
#pragma unroll
      for (int t = 0; t < NT; ++t) bh[t] *= SS;   // the candidate accumulator's seed, as sbn
    }

    for (int step = Lmax - 1; step >= 0; --step) {
      const bool act = step < L;
      const int64_t tt = act ? step : 0;
      const int64_t i = sp + tt;
      const int64_t hr = hbase + tt;
      const uint32_t code_next = code_n1;
      if (step >= 2) code_n1 = code_of(step - 2);
      // opaque lane offset: keeps the loop-invariant fragment reads inside the step loop (registers)
      int lofs = lane;
      asm volatile("" : "+v"(lofs));
      f4 az[NT], ar[NT], ah[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        az[t] = f4{0, 0, 0, 0};
        ar[t] = f4{0, 0, 0, 0};
        ah[t] = bh[t];
      }
      if constexpr (H16) {
        h8 hf[2][KS];
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          u4v w0, w1;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int e0 = 2 * q, e1 = 2 * q + 1;
            const hpair p = split2h(S * hp[2 * s + (e0 >> 2)][e0 & 3], S * hp[2 * s + (e1 >> 2)][e1 & 3]);
            w0[q] = p.hi;
            w1[q] = p.lo;
          }
          hf[0][s] = __builtin_bit_cast(h8, w0);
          hf[1][s] = __builtin_bit_cast(h8, w1);
        }
        // seq_gru_h16's order: U lo x h hi, then U hi x {h lo, h hi}
#pragma unroll
        for (int pu = 1; pu >= 0; --pu)
#pragma unroll
          for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int t = 0; t < NT; ++t) {
              const h8 wz = sUh[(((pu * 3 + 0) * NT + t) * KS + s) * 64 + lofs];
              const h8 wr = sUh[(((pu * 3 + 1) * NT + t) * KS + s) * 64 + lofs];
              const h8 wh = sUh[(((pu * 3 + 2) * NT + t) * KS + s) * 64 + lofs];
#pragma unroll
              for (int ph = 1; ph >= 0; --ph) {
                if (pu + ph > 1) continue;
                az[t] = MFMA_H(wz, hf[ph][s], az[t]);
                ar[t] = MFMA_H(wr, hf[ph][s], ar[t]);
                ah[t] = MFMA_H(wh, hf[ph][s], ah[t]);
              }
            }
      } else if constexpr (BF) {
        bf8 hf[3][KS];
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          u4v w0, w1, w2;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int e0 = 2 * q, e1 = 2 * q + 1;
            float a0, a1, a2, b0, b1, b2;
            split3(hp[2 * s + (e0 >> 2)][e0 & 3], a0, a1, a2);
            split3(hp[2 * s + (e1 >> 2)][e1 & 3], b0, b1, b2);
            w0[q] = pack_hi16(a0, b0);
            w1[q] = pack_hi16(a1, b1);
            w2[q] = pack_hi16(a2, b2);
          }
          hf[0][s] = __builtin_bit_cast(bf8, w0);
          hf[1][s] = __builtin_bit_cast(bf8, w1);
          hf[2][s] = __builtin_bit_cast(bf8, w2);
        }
#pragma unroll
        for (int pu = 2; pu >= 0; --pu)
#pragma unroll
          for (int s = 0; s < KS; ++s)
#pragma unroll
            for (int t = 0; t < NT; ++t) {
              const bf8 wz = sUb[(((pu * 3 + 0) * NT + t) * KS + s) * 64 + lofs];
              const bf8 wr = sUb[(((pu * 3 + 1) * NT + t) * KS + s) * 64 + lofs];
              const bf8 wh = sUb[(((pu * 3 + 2) * NT + t) * KS + s) * 64 + lofs];
#pragma unroll
              for (int ph = 2 - pu; ph >= 0; --ph) {
                az[t] = MFMA_BF(wz, hf[ph][s], az[t]);
                ar[t] = MFMA_BF(wr, hf[ph][s], ar[t]);
                ah[t] = MFMA_BF(wh, hf[ph][s], ah[t]);
              }
            }
      } else {
#pragma unroll
        for (int s = 0; s < KH; ++s) {
          const float hb = hp[s >> 2][s & 3];
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            az[t] = MFMA(Up[frag_idx(0 * NT + t, s, KH, lofs)], hb, az[t]);
            ar[t] = MFMA(Up[frag_idx(1 * NT + t, s, KH, lofs)], hb, ar[t]);
            ah[t] = MFMA(Up[frag_idx(2 * NT + t, s, KH, lofs)], hb, ah[t]);
          }
        }
      }
      f4 gz[NT], gr[NT], gh[NT], guh[NT], acc[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float z, rr, c, uh;
#ifdef IGN_BWD_ABL_NOGATE   // timing-only ablation (wrong gradients): no transcendental gate recompute
          if constexpr (H16) {
            z = fmaf(az[t][r], cS, x[0][t][r]);
            rr = fmaf(ar[t][r], cS, x[1][t][r]);
            c = fmaf(rr, ah[t][r], x[2][t][r]);
            uh = ah[t][r] * cS * kInv2Log2e;
          } else
#endif
          if constexpr (H16) {   // seq_gru_h16's gate arithmetic on the scaled accumulators
            z = rcpf_(1.0f + __builtin_amdgcn_exp2f(fmaf(az[t][r], cS, x[0][t][r])));
            const float rc = rcpf_(fmaf(__builtin_amdgcn_exp2f(fmaf(ar[t][r], cS, x[1][t][r])), SS, SS));
            c = tanh2_(fmaf(rc, ah[t][r], x[2][t][r]));
            rr = rc * SS;
            uh = ah[t][r] * cS * kInv2Log2e;
          } else {
            z = sig2_(az[t][r] + x[0][t][r]);
            rr = sig2_(ar[t][r] + x[1][t][r]);
            c = tanh2_(x[2][t][r] + rr * ah[t][r]);
            uh = ah[t][r] * kInv2Log2e;
          }
          const float d = act ? dh[t][r] : 0.f;
          const float dzp = d * (hp[t][r] - c) * z * (1.f - z);
          const float dcp = d * (1.f - z) * (1.f - c * c);
          const float drp = dcp * uh * rr * (1.f - rr);
          gz[t][r] = dzp;
          gr[t][r] = drp;
          gh[t][r] = dcp;
          guh[t][r] = dcp * rr;
          acc[t][r] = dh[t][r] * z;
        }
      }
      f4 af[NT];
      if constexpr (FUSE) {   // h_prev through the transpose tile, before hp is reloaded
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int q = 0; q < 4; ++q) R[(16 * t + 4 * g + q) * 16 + wofs] = hp[t][q];
#pragma unroll
        for (int mt = 0; mt < NT; ++mt) af[mt] = ld4(R + mt * 256 + rofs);
      }
#ifndef IGN_BWD_ABL_NOLOAD   // timing-only ablation (wrong gradients): every step reuses the first step's rows
      if (step > 0) load_rows(hbase + (step - 1 < L ? step - 1 : 0), code_next);
#endif
      // FUSE: every lane stores, so no branch skips the stores and the step's closing wait for the
      // prefetched rows can leave them in flight (a conditional store block made the compiler merge
      // its two paths into vmcnt(0): each step waited for its ga stores to reach memory).  A lane past
      // its sequence stores its zeros to its own step 0 row (its real step 0, stored later by the
      // same lane, wins); a padding lane to the pad slot, row n_steps (hdr; ga has one more row)
      const int gi = act ? (int)i : gpast;
#ifdef IGN_BWD_ABL_NOGA
      if (act && !FUSE) {   // timing-only ablation: no ga stores (wrong gradients)
#else
      if (FUSE || act) {
#endif
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          float* pa = a.ga + (int64_t)gi * (3 * H) + 16 * t + 4 * g;
          st4(pa, gz[t]);
          st4(pa + H, gr[t]);
          st4(pa + 2 * H, gh[t]);
          if constexpr (!FUSE) {
            float* pu = a.gu + hr * (3 * H) + 16 * t + 4 * g;
            st4(pu, gz[t]);
            st4(pu + H, gr[t]);
            st4(pu + 2 * H, guh[t]);
          }
        }
      }
      if constexpr (FUSE) {   // dU += h_prev^T du over the tile's 16 rows (inactive rows: du = 0)
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            R[(16 * t + 4 * g + q) * 16 + wofs] = gz[t][q];
            R[(H + 16 * t + 4 * g + q) * 16 + wofs] = gr[t][q];
            R[(2 * H + 16 * t + 4 * g + q) * 16 + wofs] = guh[t][q];
          }
#ifndef IGN_BWD_ABL_NODU   // timing-only ablation: no dU contraction (wrong gradients)
#pragma unroll
        for (int nt = 0; nt < 3 * NT; ++nt) {
          const f4 bf = ld4(R + nt * 256 + rofs);
#pragma unroll
          for (int ks = 0; ks < 4; ++ks)
#pragma unroll
            for (int mt = 0; mt < NT; ++mt) dU[mt][nt] = MFMA(af[mt][ks], bf[ks], dU[mt][nt]);
        }
#endif
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          bsum[t] += guh[t];
          bz[t] += gz[t];
          br[t] += gr[t];
          bc[t] += gh[t];
        }
      }
      // dh_prev = dh' z + du . U^T   (k over the 3H gate units, gate-major)
      if constexpr (H16) {
        // scaled split-fp16 x3 on 16x16x32: du is already the chained B operand (k-step s = gate
        // tiles 2s, 2s+1 = z, r, h for H = 32).  B's column n is the tile's row j, so each row
        // gets a scale of its own, Sd = 2^(15 - E(max |du| over the row's 3H values: lanes j,
        // j + 16, j + 32, j + 48)): its fp16 pieces neither overflow nor lose bits however the
        // rows' gradients differ in size; the seed dh' z and the result carry Sd sigma_t per lane
        uint32_t mb = 0;   // max |du| as the bit pattern (non-negative floats order as integers)
#pragma unroll
        for (int t = 0; t < NT; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            mb = max(mb, max(__float_as_uint(fabsf(gz[t][r])),
                             max(__float_as_uint(fabsf(gr[t][r])), __float_as_uint(fabsf(guh[t][r])))));
        {
          const auto s32 = __builtin_amdgcn_permlane32_swap(mb, mb, false, false);   // lanes l, l ^ 32
          mb = max(s32[0], s32[1]);
          const auto s16 = __builtin_amdgcn_permlane16_swap(mb, mb, false, false);   // lanes l, l ^ 16
          mb = max(s16[0], s16[1]);
        }
        // Sd's exponent, clamped so that the seed and unseed exponents (eSd + est, -(eSd + est))
        // stay inside [-126, 126]: normal powers of two whatever du and sigma_t are
        const int eSd = mb ? min(min(60, 126 - est), max(max(-100, -126 - est), 15 - ((int)(mb >> 23) - 126)))
                           : min(max(0, -126 - est), 126 - est);
        const float Sd = __int_as_float((127 + eSd) << 23);
        const float seed = __int_as_float((127 + eSd + est) << 23);
        const float unseed = __int_as_float((127 - eSd - est) << 23);
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] *= seed;
        // one k-step at a time (its two B pieces live only for its 3 x NT products: registers)
#pragma unroll
        for (int s = 0; s < KS3; ++s) {
          const f4* src = s == 0 ? gz : s == 1 ? gr : guh;
          u4v w0, w1;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int e0 = 2 * q, e1 = 2 * q + 1;
            const hpair p = split2h(Sd * src[e0 >> 2][e0 & 3], Sd * src[e1 >> 2][e1 & 3]);
            w0[q] = p.hi;
            w1[q] = p.lo;
          }
          const h8 bf[2] = {__builtin_bit_cast(h8, w0), __builtin_bit_cast(h8, w1)};
#pragma unroll
          for (int pu = 1; pu >= 0; --pu)
#pragma unroll
            for (int t = 0; t < NT; ++t) {
              const h8 w = sUth[((pu * NT + t) * KS3 + s) * 64 + lofs];
#pragma unroll
              for (int ph = 1; ph >= 0; --ph) {
                if (pu + ph > 1) continue;
                acc[t] = MFMA_H(w, bf[ph], acc[t]);
              }
            }
        }
#pragma unroll
        for (int t = 0; t < NT; ++t) acc[t] *= unseed;
      } else {
#pragma unroll
        for (int s = 0; s < K3; ++s) {
          const int gt = s >> 2, G = gt / NT, t2 = gt % NT;
          const float b = G == 0 ? gz[t2][s & 3] : G == 1 ? gr[t2][s & 3] : guh[t2][s & 3];
#pragma unroll
          for (int t = 0; t < NT; ++t) acc[t] = MFMA(Ut[frag_idx(t, s, K3, lofs)], b, acc[t]);
        }
      }
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) dh[t][r] = act ? acc[t][r] : dh[t][r];
    }
    if (valid) {
#pragma unroll
      for (int t = 0; t < NT; ++t) st4(a.dh_out + (int64_t)row * H + 16 * t + 4 * g, dh[t]);
      if constexpr (!FUSE) {
        // the final state's row of gu has no step (no memset of the whole buffer needed)
        float* pz = a.gu + (hbase + L) * (3 * H) + 4 * g;
#pragma unroll
        for (int t = 0; t < 3 * NT; ++t) st4(pz + 16 * t, f4{0, 0, 0, 0});
      }
    }
  }  // tile loop
  if constexpr (FUSE) {
    // this wave's partial: rows 0..H-1 = dU (lane: D[16mt + 4g + q][16nt + j]),
    // row H = [sum da_z, sum da_r, sum da_h], row H + 1 = [sum du_z, sum du_r, sum du_h]
    float* P = a.part + ((int64_t)blockIdx.x * 4 + wave) * (H + 2) * (3 * H);
#pragma unroll
    for (int mt = 0; mt < NT; ++mt)
#pragma unroll
      for (int nt = 0; nt < 3 * NT; ++nt)
#pragma unroll
        for (int q = 0; q < 4; ++q) P[(16 * mt + 4 * g + q) * (3 * H) + 16 * nt + j] = dU[mt][nt][q];
#pragma unroll
    for (int t = 0; t < NT; ++t)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float s = bsum[t][q], sz = bz[t][q], sr = br[t][q], sc = bc[t][q];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {   // over the 16 rows j of group g
          s += __shfl_xor(s, o);
          sz += __shfl_xor(sz, o);
          sr += __shfl_xor(sr, o);
          sc += __shfl_xor(sc, o);
        }
        bsum[t][q] = s;
        bz[t][q] = sz;
        br[t][q] = sr;
        bc[t][q] = sc;
      }
    if (j == 0) {
      float* Pa = P + H * (3 * H);
      float* Pu = Pa + 3 * H;
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const int u = 16 * t + 4 * g;
        st4(Pa + u, bz[t]);
        st4(Pa + H + u, br[t]);
        st4(Pa + 2 * H + u, bc[t]);
        st4(Pu + u, bz[t]);
        st4(Pu + H + u, br[t]);
        st4(Pu + 2 * H + u, bsum[t]);
      }
    }
  }
}

__global__ void seq_bwd_hdr_kernel(const int32_t* __restrict__ hdr, const uint32_t* __restrict__ step_code,
                                   int64_t n, int32_t* __restrict__ out) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    i4v h = *reinterpret_cast<const i4v*>(hdr + 4 * i);
    h[3] = (int32_t)step_code[(int64_t)h[2] + max(h[1], 1) - 1];   // padding: len 0, step_ptr = the pad slot
    *reinterpret_cast<i4v*>(out + 4 * i) = h;
  }
}

// ---------------------------------------------------------------------------------------------
// Sum update backward: one wave = 16 destination rows (identity order).
template <int DIN, int H>
__global__ __launch_bounds__(256) void sum_gru_bwd_kernel(SumBwdArgs a) {
  constexpr int NC = DIN / 16, NT = H / 16, KX = DIN / 4, KH = H / 4, K3 = 3 * H / 4;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int j = lane & 15, g = lane >> 4;
  const int64_t row = ((int64_t)blockIdx.x * 4 + wave) * 16 + j;
  const bool valid = row < a.n_dst;
  const int64_t rr0 = valid ? row : 0;
  f4 x[NC], h[NT], dh[NT];
#pragma unroll
  for (int c = 0; c < NC; ++c) x[c] = ld4(a.x + rr0 * DIN + 16 * c + 4 * g);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    h[t] = ld4(a.h + rr0 * H + 16 * t + 4 * g);
    dh[t] = valid ? ld4(a.dh_in + rr0 * H + 16 * t + 4 * g) : f4{0, 0, 0, 0};
  }
  f4 az[NT], ar[NT], ax[NT], ah[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    az[t] = ld4(a.bias + 0 * H + 16 * t + 4 * g);
    ar[t] = ld4(a.bias + 1 * H + 16 * t + 4 * g);
    ax[t] = ld4(a.bias + 2 * H + 16 * t + 4 * g);
    ah[t] = ld4(a.bias + 3 * H + 16 * t + 4 * g);
  }
#pragma unroll
  for (int s = 0; s < KX; ++s) {
    const float xb = x[s >> 2][s & 3];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      az[t] = MFMA(a.Wp[frag_idx(0 * NT + t, s, KX, lane)], xb, az[t]);
      ar[t] = MFMA(a.Wp[frag_idx(1 * NT + t, s, KX, lane)], xb, ar[t]);
      ax[t] = MFMA(a.Wp[frag_idx(2 * NT + t, s, KX, lane)], xb, ax[t]);
    }
  }
#pragma unroll
  for (int s = 0; s < KH; ++s) {
    const float hb = h[s >> 2][s & 3];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      az[t] = MFMA(a.Up[frag_idx(0 * NT + t, s, KH, lane)], hb, az[t]);
      ar[t] = MFMA(a.Up[frag_idx(1 * NT + t, s, KH, lane)], hb, ar[t]);
      ah[t] = MFMA(a.Up[frag_idx(2 * NT + t, s, KH, lane)], hb, ah[t]);
    }
  }
  f4 gz[NT], gr[NT], gh[NT], guh[NT], acc[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float z = sig2_(az[t][r]);
      const float rr = sig2_(ar[t][r]);
      const float c = tanh2_(ax[t][r] + rr * ah[t][r]);
      const float uh = ah[t][r] * kInv2Log2e;
      const float d = dh[t][r];
      const float dzp = d * (h[t][r] - c) * z * (1.f - z);
      const float dcp = d * (1.f - z) * (1.f - c * c);
      const float drp = dcp * uh * rr * (1.f - rr);
      gz[t][r] = dzp;
      gr[t][r] = drp;
      gh[t][r] = dcp;
      guh[t][r] = dcp * rr;
      acc[t][r] = d * z;
    }
  }
  f4 dxa[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) dxa[c] = f4{0, 0, 0, 0};
#pragma unroll
  for (int s = 0; s < K3; ++s) {
    const int gt = s >> 2, G = gt / NT, t2 = gt % NT;
    const float ba = G == 0 ? gz[t2][s & 3] : G == 1 ? gr[t2][s & 3] : gh[t2][s & 3];
    const float bu = G == 0 ? gz[t2][s & 3] : G == 1 ? gr[t2][s & 3] : guh[t2][s & 3];
#pragma unroll
    for (int c = 0; c < NC; ++c) dxa[c] = MFMA(a.Wt[frag_idx(c, s, K3, lane)], ba, dxa[c]);
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[t] = MFMA(a.Ut[frag_idx(t, s, K3, lane)], bu, acc[t]);
  }
  if (valid) {
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      st4(a.dh_out + row * H + 16 * t + 4 * g, acc[t]);
      float* pa = a.ga + row * (3 * H) + 16 * t + 4 * g;
      st4(pa, gz[t]);
      st4(pa + H, gr[t]);
      st4(pa + 2 * H, gh[t]);
      float* pu = a.gu + row * (3 * H) + 16 * t + 4 * g;
      st4(pu, gz[t]);
      st4(pu + H, gr[t]);
      st4(pu + 2 * H, guh[t]);
    }
#pragma unroll
    for (int c = 0; c < NC; ++c) st4(a.dx + row * DIN + 16 * c + 4 * g, dxa[c]);
  }
}

// ---------------------------------------------------------------------------------------------
// V: 4-float vectors per thread (cols % (4 V) == 0); each thread walks its row's list in batches
// of eight entries, the last (< 8) batch with indices clamped to the list's last entry (a cached
// re-read) and masked additions; the additions keep the CSR order (bitwise one at a time).  The
// batched tail: a RouteNet path (~3 links) was a 4-batch and single rows, each a dependent
// idx -> row round trip; the link-update backward's gather 114 -> 98 us, 16.60 -> 16.43 ms per
// training step (same box, tools/gpu_calls/r05_c54.sh)
#ifndef IGN_GATHER_BATCH   // rows per batch in flight; 16 measured slower: 16.06-16.16 against
#define IGN_GATHER_BATCH 8   // 15.65-15.72 ms per training step, same box (r06_c29.sh), the same bits
#endif
template <int V, bool NT = false, int GB = IGN_GATHER_BATCH>
__global__ void csr_gather_add_kernel(float* __restrict__ out, int64_t n_rows, const int32_t* __restrict__ ptr,
                                      const int32_t* __restrict__ idx, const float* __restrict__ in, int cols,
                                      int accumulate) {
  const int q = cols / (4 * V);
  const int64_t total = n_rows * q;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / q;
    const int c = (int)(e - r * q) * 4 * V;
    f4 acc[V];
#pragma unroll
    for (int w = 0; w < V; ++w) acc[w] = accumulate ? ld4(out + r * cols + c + 4 * w) : f4{0, 0, 0, 0};
    const int k1 = ptr[r + 1];
    for (int k = ptr[r]; k < k1; k += GB) {
      int i8[GB];
#pragma unroll
      for (int u = 0; u < GB; ++u) i8[u] = idx[min(k + u, k1 - 1)];
      f4 v8[GB][V];
#pragma unroll
      for (int u = 0; u < GB; ++u)
#pragma unroll
        for (int w = 0; w < V; ++w) {
          const float* pv = in + (int64_t)i8[u] * cols + c + 4 * w;
          v8[u][w] = NT ? __builtin_nontemporal_load(reinterpret_cast<const f4*>(pv)) : ld4(pv);
        }
#pragma unroll
      for (int u = 0; u < GB; ++u)
        if (k + u < k1) {
#pragma unroll
          for (int w = 0; w < V; ++w) acc[w] += v8[u][w];
        }
    }
#pragma unroll
    for (int w = 0; w < V; ++w) st4(out + r * cols + c + 4 * w, acc[w]);
  }
}

// ---------------------------------------------------------------------------------------------
// Attention aggregation backward (AUX:287-343).  Forward: v_m = s_src(src_m) + s_dst(d_m),
// e_c = sum_{m in cell c} LeakyReLU_0.2(v_m), w = softmax over each (graph, position) group of
// cells (empty cells count as 0), x_d = sum_m w_{c(m)} h_src(src_m).
//   dw_m  = dx_d . h_src(src_m)                               attn_dcoef
//   de_c  = w_c (sum_{m in c} dw_m - S_g), S_g = sum_c w_c dw_c  attn_softmax_bwd (one wave per group)
//   dv_m  = de_c LeakyReLU'(v_m)
//   dh_src += sum_m w_m dx_{d_m} + (sum_m dv_m) w1             attn_src_bwd (also ds_src per row)
//   dh_dst += (sum_{m -> d} dv_m) w2                           attn_dst_bwd (also ds_dst per row)
__device__ __forceinline__ const float* attn_row(const SrcBases& sb, uint32_t code, int F) {
  return sb.base[code >> IGN_SLOT_SHIFT] + (int64_t)(code & IGN_ROW_MASK) * F;
}

__global__ void attn_dcoef_kernel(const float* __restrict__ dx, const int32_t* __restrict__ mdst,
                                  const uint32_t* __restrict__ msg_src, SrcBases src, int F, int64_t n,
                                  float* __restrict__ dw) {
  for (int64_t m = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; m < n; m += (int64_t)gridDim.x * blockDim.x) {
    const float* h = attn_row(src, msg_src[m], F);
    const float* g = dx + (int64_t)mdst[m] * F;
    float s = 0.f;
    for (int k = 0; k < F; ++k) s += g[k] * h[k];
    dw[m] = s;
  }
}

__global__ __launch_bounds__(256) void attn_softmax_bwd_kernel(AttnArgs a, const float* __restrict__ dw,
                                                               float* __restrict__ dv) {
  const int lane = threadIdx.x & 63;
  const int64_t grp = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (grp >= a.n_groups) return;
  const int c0 = a.group_ptr[grp], c1 = a.group_ptr[grp + 1];
  float S = 0.f;
  for (int c = c0 + lane; c < c1; c += 64) {
    float dc = 0.f;
    for (int q = a.cell_ptr[c]; q < a.cell_ptr[c + 1]; ++q) dc += dw[a.cell_msgs[q]];
    S += a.msg_w[a.cell_msgs[a.cell_ptr[c]]] * dc;
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) S += __shfl_xor(S, o);
  for (int c = c0 + lane; c < c1; c += 64) {
    float dc = 0.f;
    for (int q = a.cell_ptr[c]; q < a.cell_ptr[c + 1]; ++q) dc += dw[a.cell_msgs[q]];
    const float de = a.msg_w[a.cell_msgs[a.cell_ptr[c]]] * (dc - S);
    const float sd = a.s_dst[a.cell_dst[c]];
    for (int q = a.cell_ptr[c]; q < a.cell_ptr[c + 1]; ++q) {
      const int m = a.cell_msgs[q];
      const uint32_t code = a.msg_src[m];
      const float v = a.s_src[code >> IGN_SLOT_SHIFT][code & IGN_ROW_MASK] + sd;
      dv[m] = v > 0.f ? de : 0.2f * de;
    }
  }
}

// one thread per (source row, column): rows of one source slot; sptr / sidx: row -> CSR messages
__global__ void attn_src_bwd_kernel(int64_t rows, const int32_t* __restrict__ sptr, const int32_t* __restrict__ sidx,
                                    const float* __restrict__ msg_w, const float* __restrict__ dv,
                                    const int32_t* __restrict__ mdst, const float* __restrict__ dx,
                                    const float* __restrict__ w1, int F, float* __restrict__ dh,
                                    float* __restrict__ ds) {
  const int64_t total = rows * F;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / F;
    const int c = (int)(e - r * F);
    float acc = 0.f, sv = 0.f;
    for (int k = sptr[r]; k < sptr[r + 1]; ++k) {
      const int m = sidx[k];
      acc += msg_w[m] * dx[(int64_t)mdst[m] * F + c];
      sv += dv[m];
    }
    dh[e] += acc + sv * w1[c];
    if (c == 0) ds[r] = sv;
  }
}

// one thread per (order position, column): the destination's messages are CSR range ptr[pos] ..
__global__ void attn_dst_bwd_kernel(int64_t n_pos, const int32_t* __restrict__ order, const int32_t* __restrict__ ptr,
                                    const float* __restrict__ dv, const float* __restrict__ w2, int F,
                                    float* __restrict__ dh, float* __restrict__ ds) {
  const int64_t total = n_pos * F;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t pos = e / F;
    const int c = (int)(e - pos * F);
    float sv = 0.f;
    for (int m = ptr[pos]; m < ptr[pos + 1]; ++m) sv += dv[m];
    const int64_t d = order[pos];
    dh[d * F + c] += sv * w2[c];
    if (c == 0) ds[d] = sv;
  }
}

// w1 = K1 a1, w2 = K2 a2 (attn_vectors): dK1 += dw1 a1^T, da1 += K1^T dw1 (same for K2, a2)
__global__ void attn_param_bwd_kernel(const float* __restrict__ dw12, const float* __restrict__ K1,
                                      const float* __restrict__ K2, const float* __restrict__ av, int F,
                                      float* __restrict__ dK1, float* __restrict__ dK2, float* __restrict__ dav) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < 2 * F * F) {
    const int which = i / (F * F), r = (i % (F * F)) / F, c = i % F;
    if (which == 0) dK1[r * F + c] += dw12[r] * av[c];
    else dK2[r * F + c] += dw12[F + r] * av[F + c];
  }
  if (i < 2 * F) {
    const int which = i / F, c = i % F;
    const float* K = which ? K2 : K1;
    const float* d = dw12 + which * F;
    float s = 0.f;
    for (int r = 0; r < F; ++r) s += K[r * F + c] * d[r];
    dav[which * F + c] += s;
  }
}

// Convolution aggregation backward, elementwise part (AUX:384-401): x = act((s.K + h) / deg), so
// du = dx act'(x) / deg (act' through the output x), and the destination's own state gets du.
__global__ void conv_bwd_kernel(const float* __restrict__ dx, const float* __restrict__ x,
                                const float* __restrict__ deg, int64_t n, int F, int act, float* __restrict__ du,
                                float* __restrict__ dh) {
  const int64_t total = n * F;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const float v = dx[i] * act_grad(x[i], act) / deg[i / F];
    du[i] = v;
    dh[i] += v;
  }
}

// out[r][c] (+)= sum over k in ptr[r] .. ptr[r+1] of in[idx[k]][col0 + c], c < width: a column slice
// of a per-edge gradient gathered back to the rows it came from (any width / offset).
__global__ void csr_gather_cols_add_kernel(float* __restrict__ out, int64_t n_rows, const int32_t* __restrict__ ptr,
                                           const int32_t* __restrict__ idx, const float* __restrict__ in,
                                           int in_stride, int col0, int width, int accumulate) {
  const int64_t total = n_rows * width;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / width;
    const int c = (int)(e - r * width);
    float acc = accumulate ? out[e] : 0.f;
    for (int k = ptr[r]; k < ptr[r + 1]; ++k) acc += in[(int64_t)idx[k] * in_stride + col0 + c];
    out[e] = acc;
  }
}

// out[r][m] (+)= sum_k in[r][k] Mat[m][k]; optional *= act'(aprev[r][m]).  One wave = 16 rows.
template <int K, int M>
__global__ __launch_bounds__(256) void row_gemm_t_kernel(const float* __restrict__ in, int64_t n,
                                                         const float* __restrict__ Ap, float* __restrict__ out,
                                                         int accumulate, int act, const float* __restrict__ aprev) {
  constexpr int KS = K / 4, NM = M / 16, NCH = K / 16;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int j = lane & 15, g = lane >> 4;
  const int64_t r = ((int64_t)blockIdx.x * 4 + wave) * 16 + j;
  const bool valid = r < n;
  const int64_t rr = valid ? r : 0;
  f4 acc[NM];
#pragma unroll
  for (int t = 0; t < NM; ++t) acc[t] = f4{0, 0, 0, 0};
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const f4 b = valid ? ld4(in + rr * K + 16 * c + 4 * g) : f4{0, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int s = 4 * c + q;
#pragma unroll
      for (int t = 0; t < NM; ++t) acc[t] = MFMA(Ap[frag_idx(t, s, KS, lane)], b[q], acc[t]);
    }
  }
  if (!valid) return;
#pragma unroll
  for (int t = 0; t < NM; ++t) {
    float* po = out + r * M + 16 * t + 4 * g;
    f4 v = acc[t];
    if (act >= 0) {
      const f4 av = ld4(aprev + r * M + 16 * t + 4 * g);
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] *= act_grad(av[q], act);
    }
    if (accumulate) v += ld4(po);
    st4(po, v);
  }
}

__global__ void row_gemm_t_generic_kernel(const float* __restrict__ in, int64_t n, int K, const float* __restrict__ Mat,
                                          int M, float* __restrict__ out, int accumulate, int act,
                                          const float* __restrict__ aprev) {
  const int64_t total = n * M;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / M;
    const int m = (int)(e - r * M);
    float s = 0.f;
    for (int k = 0; k < K; ++k) s += in[r * K + k] * Mat[(int64_t)m * K + k];
    if (act >= 0) s *= act_grad(aprev[e], act);
    out[e] = accumulate ? out[e] + s : s;
  }
}

// K = 1 (the backward of a 1-unit output layer): out[r][m] (+)= in[r] Mat[m] act'(aprev[r][m]),
// four columns per thread (16-B accesses); the same per-element arithmetic as the generic kernel
__global__ void row_outer_t_kernel(const float* __restrict__ in, int64_t n, const float* __restrict__ Mat, int M,
                                   float* __restrict__ out, int accumulate, int act, const float* __restrict__ aprev) {
  const int M4 = M >> 2;
  const int64_t total = n * M4;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = e / M4;
    const int m = (int)(e - r * M4) * 4;
    const float x = in[r];
    const f4 w = ld4(Mat + m);
    const f4 av = act >= 0 ? ld4(aprev + r * M + m) : f4{0, 0, 0, 0};
    f4 o = accumulate ? ld4(out + r * M + m) : f4{0, 0, 0, 0};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float s = 0.f;
      s += x * w[q];
      if (act >= 0) s *= act_grad(av[q], act);
      o[q] = accumulate ? o[q] + s : s;
    }
    st4(out + r * M + m, o);
  }
}

__global__ void split_cols_add_kernel(float* __restrict__ dst, int64_t n, int width, const float* __restrict__ src,
                                      int src_stride, int col0) {
  const int64_t total = n * width;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = i / width;
    const int c = (int)(i - r * width);
    dst[i] += src[r * src_stride + col0 + c];
  }
}

__global__ void act_bwd_kernel(const float* __restrict__ da, const float* __restrict__ a, int64_t n, int act,
                               float* __restrict__ dz) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    dz[i] = da[i] * act_grad(a[i], act);
}

// ---------------------------------------------------------------------------------------------
// Row contractions C[M][N] = sum_r A[r][:M]^T B[r][:N] (weight gradients), optionally with a
// virtual all-ones column appended to A: C row M = sum_r B[r] (the bias gradient).  Rows are the
// MFMA k axis (4 per MFMA); a wave owns a 64 x 64 output tile and a chunk of rows, 16 rows per
// iteration (32 loads in flight), and writes its partial tile.  Chunks are sized so the grid
// holds ~8k waves; two reduction passes (segments, then final) sum the partials in a fixed order.
constexpr int kTsWaves = 8192;
constexpr int kBwdMaxWaves = kBwdPartialWaves;   // fused ordered backward: partial slots
constexpr int kTsSegs = kTsReduceSegs;

struct TsPlan {
  int Mx, tiles;
  int64_t chunks, chunk;
};

TsPlan ts_plan(int64_t n_rows, int M, int N, int ones) {
  TsPlan p;
  p.Mx = M + ones;
  p.tiles = ((p.Mx + 63) / 64) * ((N + 63) / 64);
  // at least 128 rows per chunk (IGN_TS_MIN_ROWS): the MP weight gradients (32-33 x 96 over ~10^5
  // rows) had one wave per SIMD at 256 (416 chunks x 2 tiles); at 128 the step is 0.18 ms shorter, at
  // 64 the larger reduction eats the gain (r05_c40.sh)
  static const int64_t min_rows = [] {
    const char* v = getenv("IGN_TS_MIN_ROWS");
    return v && atoi(v) >= 32 ? (int64_t)atoi(v) : (int64_t)128;
  }();
  const int64_t max_chunks = std::max<int64_t>(1, (n_rows + min_rows - 1) / min_rows);
  p.chunks = std::max<int64_t>(1, std::min<int64_t>((kTsWaves + p.tiles - 1) / p.tiles, max_chunks));
  p.chunk = ((n_rows + p.chunks - 1) / p.chunks + 15) / 16 * 16;
  p.chunks = std::max<int64_t>(1, (n_rows + p.chunk - 1) / p.chunk);
  return p;
}

// The N = 1 contraction (a 1-unit output layer's weight gradient, attention's score vectors):
// part[chunk][m][0] = sum_r A[r][m] B[r], part[chunk][M][0] = sum_r B[r] (ones).  One wave per row
// in turn, lane l holding columns 4l .. 4l + 3 (M <= 256): each row is one contiguous read, where
// the MFMA kernel's lanes read 4-B column pieces of 8 rows (2.9 TB/s on the readout's 256-wide
// activations); the block's four waves add in a fixed order (deterministic).
__global__ __launch_bounds__(256) void tsgemv_kernel(const float* __restrict__ A, int lda, const float* __restrict__ B,
                                                     int ldb, int64_t n_rows, int M, int ones, int64_t chunk,
                                                     float* __restrict__ part) {
  __shared__ f4 sp[4][64];
  __shared__ float sb[4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * chunk, r1 = min<int64_t>(n_rows, r0 + chunk);
  const bool on = 4 * lane < M;
  f4 acc = {0, 0, 0, 0};
  float bs = 0.f;
  int64_t r = r0 + wave;
  for (; r + 12 < r1; r += 16) {   // four rows of this wave in flight
    f4 a[4];
    float b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a[u] = on ? ld4(A + (r + 4 * u) * lda + 4 * lane) : f4{0, 0, 0, 0};
      b[u] = B[(r + 4 * u) * ldb];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int q = 0; q < 4; ++q) acc[q] = fmaf(a[u][q], b[u], acc[q]);
      bs += b[u];
    }
  }
  for (; r < r1; r += 4) {
    const f4 a = on ? ld4(A + r * lda + 4 * lane) : f4{0, 0, 0, 0};
    const float b = B[r * ldb];
#pragma unroll
    for (int q = 0; q < 4; ++q) acc[q] = fmaf(a[q], b, acc[q]);
    bs += b;
  }
  sp[wave][lane] = acc;
  if (lane == 0) sb[wave] = bs;
  __syncthreads();
  if (wave == 0) {
    f4 t = sp[0][lane];
#pragma unroll
    for (int w = 1; w < 4; ++w) t = t + sp[w][lane];
    float* P = part + (int64_t)blockIdx.x * (M + ones);
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (4 * lane + q < M) P[4 * lane + q] = t[q];
    if (ones && lane == 0) P[M] = ((sb[0] + sb[1]) + sb[2]) + sb[3];
  }
}

__global__ __launch_bounds__(256) void tsgemm_kernel(const float* __restrict__ A, int lda, const float* __restrict__ B,
                                                     int ldb, int64_t n_rows, int M, int N, int ones, int64_t chunk,
                                                     float* __restrict__ part) {
  // The ones column (bias gradient) is not an MFMA row: the tile whose m range would hold it
  // accumulates plain column sums of B on the VALU (lanes of one kk own 4 rows each).
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int Mx = M + ones;
  const int tiles_m = (Mx + 63) / 64, tiles_n = (N + 63) / 64;
  const int tile = blockIdx.y * (blockDim.x >> 6) + wave;   // blocks of min(4, tiles) waves
  if (tile >= tiles_m * tiles_n) return;
  const int m0 = (tile / tiles_n) * 64, n0 = (tile % tiles_n) * 64;
  const int na = max(0, min(4, (M - m0 + 15) / 16)), nb = min(4, (N - n0 + 15) / 16);
  const bool has_ones = ones && M >= m0 && M < m0 + 64;
  const int64_t r0 = (int64_t)blockIdx.x * chunk;
  const int64_t r1 = std::min<int64_t>(n_rows, r0 + chunk);
  const int kk = lane >> 4, c = lane & 15;
  f4 acc[4][4];
  float csum[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) acc[x][y] = f4{0, 0, 0, 0};
  for (int64_t r = r0; r < r1; r += 16) {
    float av[4][4], bv[4][4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t rr = r + 4 * q + kk;
      const bool ok = rr < r1;
#pragma unroll
      for (int x = 0; x < 4; ++x) {
        const int m = m0 + 16 * x + c;
        av[q][x] = (x < na && ok && m < M) ? A[rr * lda + m] : 0.f;
        const int n = n0 + 16 * x + c;
        bv[q][x] = (x < nb && ok && n < N) ? B[rr * ldb + n] : 0.f;
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int y = 0; y < 4; ++y) csum[y] += bv[q][y];
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y)
          if (x < na && y < nb) acc[x][y] = MFMA(av[q][x], bv[q][y], acc[x][y]);
    }
  }
  float* P = part + (int64_t)blockIdx.x * Mx * N;
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) {
      const int n = n0 + 16 * y + c;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int m = m0 + 16 * x + 4 * kk + q;
        if (x < na && y < nb && m < M && n < N) P[(int64_t)m * N + n] = acc[x][y][q];
      }
    }
  if (has_ones) {
#pragma unroll
    for (int y = 0; y < 4; ++y) {      // sum over the 4 row phases kk (lanes c, c+16, c+32, c+48)
      float s = csum[y];
      s += __shfl_xor(s, 16);
      s += __shfl_xor(s, 32);
      const int n = n0 + 16 * y + c;
      if (kk == 0 && n < N) P[(int64_t)M * N + n] = s;
    }
  }
}

// pass 1: seg[s][i] = sum of part[c][i] over chunks c = s, s + S, ...   (grid: elements x S)
__global__ void reduce_seg_kernel(const float* __restrict__ part, int64_t nchunks, int64_t size, int S,
                                  float* __restrict__ seg) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int s = blockIdx.y;
  if (i >= size) return;
  float acc = 0.f;
  // unrolled: the loads of 8 chunks are in flight at once (the adds keep the chunk order)
#pragma unroll 8
  for (int64_t c = s; c < nchunks; c += S) acc += part[c * size + i];
  seg[(int64_t)s * size + i] = acc;
}

// pass 2: C[m][n] += sum_s seg[s][m][n] for m < M; row M (ones column) goes to Cb[n]
__global__ void reduce_final_kernel(const float* __restrict__ seg, int S, int M, int N, int ones,
                                    float* __restrict__ C, float* __restrict__ Cb) {
  const int64_t size = (int64_t)(M + ones) * N;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < size; i += (int64_t)gridDim.x * blockDim.x) {
    float acc = 0.f;
#pragma unroll 16
    for (int s = 0; s < S; ++s) acc += seg[(int64_t)s * size + i];
    if (i < (int64_t)M * N) C[i] += acc;
    else Cb[i - (int64_t)M * N] += acc;
  }
}

// y[r][m] = act(sum_k x[r][k] W[k][m] + b[m]); W given as pack_dense fragments (A[m][k] = W[k][m]).
template <int K, int M>
__global__ __launch_bounds__(256) void dense_fwd_kernel(const float* __restrict__ x, int64_t n, int x_stride,
                                                        const float* __restrict__ Wp, const float* __restrict__ bias,
                                                        int act, float* __restrict__ y) {
  constexpr int KS = K / 4, NM = M / 16, NCH = K / 16;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  const int j = lane & 15, g = lane >> 4;
  const int64_t r = ((int64_t)blockIdx.x * 4 + wave) * 16 + j;
  const bool valid = r < n;
  const int64_t rr = valid ? r : 0;
  f4 acc[NM];
#pragma unroll
  for (int t = 0; t < NM; ++t) acc[t] = bias ? ld4(bias + 16 * t + 4 * g) : f4{0, 0, 0, 0};
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    const f4 b = ld4(x + rr * x_stride + 16 * c + 4 * g);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int s = 4 * c + q;
#pragma unroll
      for (int t = 0; t < NM; ++t) acc[t] = MFMA(Wp[frag_idx(t, s, KS, lane)], b[q], acc[t]);
    }
  }
  if (!valid) return;
#pragma unroll
  for (int t = 0; t < NM; ++t) {
    f4 v = acc[t];
#pragma unroll
    for (int q = 0; q < 4; ++q) v[q] = act_apply(v[q], act);
    st4(y + r * M + 16 * t + 4 * g, v);
  }
}

// y[r] = act(x[r] . w + b) for a 1-unit layer: 16 lanes per row, float4 loads, shuffle reduce
__global__ void dense_dot_kernel(const float* __restrict__ x, int64_t n, int K, int x_stride,
                                 const float* __restrict__ w, const float* __restrict__ bias, int act,
                                 float* __restrict__ y) {
  const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 4;
  const int l = threadIdx.x & 15;
  float s = 0.f;
  if (r < n)
    for (int k = 4 * l; k < K; k += 64) {
      const f4 a = ld4(x + r * x_stride + k);
      const f4 b = ld4(w + k);
      s += a[0] * b[0] + a[1] * b[1] + a[2] * b[2] + a[3] * b[3];
    }
#pragma unroll
  for (int o = 8; o >= 1; o >>= 1) s += __shfl_xor(s, o, 16);
  if (r < n && l == 0) y[r] = act_apply(s + (bias ? bias[0] : 0.f), act);
}

__global__ void axpy_kernel(float* __restrict__ y, const float* __restrict__ x, float alpha, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] += alpha * x[i];
}

__global__ void mse_kernel(const float* __restrict__ pred, const float* __restrict__ label, int64_t n,
                           float* __restrict__ dpred, double* __restrict__ part) {
  __shared__ double red[256];
  double s = 0.0;
  const float sc = 2.0f / (float)n;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float d = pred[i] - label[i];
    dpred[i] = sc * d;
    s += (double)d * (double)d;
  }
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

__global__ void sumsq_kernel(const float* __restrict__ x, int64_t n, double* __restrict__ part) {
  __shared__ double red[256];
  double s = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    s += (double)x[i] * (double)x[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

// Keras Adam (training_ops.ApplyAdam): m = b1 m + (1-b1) g; v = b2 v + (1-b2) g^2;
// w -= lr_t m / (sqrt(v) + eps), lr_t = lr sqrt(1 - b2^t) / (1 - b1^t) computed by the host
__global__ void adam_kernel(float* __restrict__ w, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, int64_t n, float lr_t, float b1, float b2, float eps) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const float gi = g[i];
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    w[i] -= lr_t * mi / (sqrtf(vi) + eps);
  }
}

int blocks_for(int64_t n, int per = 256, int cap = 16384) {
  return (int)std::max<int64_t>(1, std::min<int64_t>((n + per - 1) / per, cap));
}

}  // namespace

// =============================================================================================
hipError_t launch_pack_a(const float* M, int rows, int cols, float* out, hipStream_t st) {
  if (rows % 16 || cols % 16) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pack_a_kernel, dim3(blocks_for((int64_t)rows * cols)), dim3(256), 0, st, M, rows, cols, out);
  return hipGetLastError();
}

bool bwd_shape_supported(int din, int h) {
  return (din == 16 || din == 32 || din == 64) && (h == 16 || h == 32 || h == 64) && (h != 64 || din == 64) &&
         (din != 64 || h == 64);
}

bool seq_bwd_fused_supported(int h) { return h == 16 || h == 32; }

int64_t seq_bwd_partial_floats(int h) { return (int64_t)(kBwdMaxWaves + kTsSegs) * (h + 2) * 3 * h; }

template <int H, int RC>
static int64_t seq_bwd_fused_blocks(int64_t n_dst) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, seq_gru_bwd_kernel<H, true, RC>, 256, 0) != hipSuccess ||
      per_cu <= 0)
    per_cu = 1;
  const int64_t tiles = (n_dst + 15) / 16;
  return std::max<int64_t>(1, std::min<int64_t>({(tiles + 3) / 4, (int64_t)per_cu * cus, kBwdMaxWaves / 4}));
}

template <int H, int RC>
static hipError_t seq_bwd_fused(const SeqBwdArgs& a, hipStream_t st) {
  const int64_t blocks = seq_bwd_fused_blocks<H, RC>(a.n_dst);
  hipLaunchKernelGGL((seq_gru_bwd_kernel<H, true, RC>), dim3((unsigned)blocks), dim3(256), 0, st, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || a.defer_reduce) return e;   // (deferred: launch_seq_bwd_reduce later)
  return launch_seq_bwd_reduce(a, blocks * 4, H, st);
}

int64_t seq_bwd_fused_waves(const SeqBwdArgs& a, int h) {
  if (h == 16) return 4 * seq_bwd_fused_blocks<16, 0>(a.n_dst);
  if (h == 32)
    return 4 * (a.Uh ? seq_bwd_fused_blocks<32, 2>(a.n_dst) : a.Ubf ? seq_bwd_fused_blocks<32, 1>(a.n_dst)
                                                                   : seq_bwd_fused_blocks<32, 0>(a.n_dst));
  return 0;
}

hipError_t launch_seq_bwd_reduce(const SeqBwdArgs& a, int64_t waves, int H, hipStream_t st) {
  // rows 0..H (dU, da sums) into scratch, row H + 1 (du sums) straight into db_rec
  hipError_t e = hipMemsetAsync(a.scratch, 0, (size_t)(H + 1) * 3 * H * sizeof(float), st);
  if (e != hipSuccess) return e;
  if ((e = launch_partials_reduce_add(a.part, waves, H + 1, 3 * H, 1, a.scratch, a.db_rec, st)) != hipSuccess)
    return e;
  if ((e = launch_axpy(a.dU, a.scratch, 1.f, (int64_t)H * 3 * H, st)) != hipSuccess) return e;
  return launch_axpy(a.db_in, a.scratch + (int64_t)H * 3 * H, 1.f, 3 * H, st);
}

hipError_t launch_seq_bwd_hdr(const int32_t* fwd_hdr, const uint32_t* step_code, int64_t n_pos, int32_t* out,
                              hipStream_t st) {
  if (n_pos <= 0) return hipSuccess;
  const int64_t blocks = std::min<int64_t>((n_pos + 255) / 256, 4096);
  hipLaunchKernelGGL(seq_bwd_hdr_kernel, dim3((unsigned)blocks), dim3(256), 0, st, fwd_hdr, step_code, n_pos, out);
  return hipGetLastError();
}

hipError_t launch_seq_gru_bwd(const SeqBwdArgs& a, int h, hipStream_t st) {
  if (a.n_dst == 0) return hipSuccess;
  if (!a.h_in) return hipErrorInvalidValue;
  if (a.part) {   // fused dU / b_rec(h) gradients
    if (!a.dU || !a.db_rec || !a.db_in || !a.scratch) return hipErrorInvalidValue;
    if (h == 16) return seq_bwd_fused<16, 0>(a, st);
    if (h == 32) return a.Uh ? seq_bwd_fused<32, 2>(a, st) : a.Ubf ? seq_bwd_fused<32, 1>(a, st) : seq_bwd_fused<32, 0>(a, st);
    return hipErrorInvalidValue;
  }
  if (!a.gu) return hipErrorInvalidValue;
  dim3 grid((unsigned)((a.n_dst + 63) / 64));
  if (h == 16) hipLaunchKernelGGL((seq_gru_bwd_kernel<16, false, 0>), grid, dim3(256), 0, st, a);
  else if (h == 32) hipLaunchKernelGGL((seq_gru_bwd_kernel<32, false, 0>), grid, dim3(256), 0, st, a);
  else if (h == 64) hipLaunchKernelGGL((seq_gru_bwd_kernel<64, false, 0>), grid, dim3(256), 0, st, a);
  else return hipErrorInvalidValue;
  return hipGetLastError();
}

// Sum update backward with its weight gradients formed in the kernel (DIN = H = 32: the RouteNet /
// Q-size sum MPs).  Persistent waves take 16-row tiles in a static order and, besides dh and dx
// (sum_gru_bwd_kernel's arithmetic), accumulate dW = sum x^T da and dU = sum h^T du on the f32 MFMA
// through a per-wave transpose tile (seq_gru_bwd_kernel's FUSE scheme: rows on the k axis) and the
// bias sums on the VALU.  Each wave writes one partial of dW plus the db_in row and one of dU plus
// the db_rec row, in launch_partials_reduce_add's layout, so da and du never go to memory and the
// two row contractions over them (tsgemm) are gone.  Rows past n_dst have dh = 0, so da = du = 0.
template <int DIN, int H>
__global__ __launch_bounds__(256, 2) void sum_gru_bwd_fused_kernel(SumBwdArgs a, float* __restrict__ part_w,
                                                                float* __restrict__ part_u) {
  constexpr int NC = DIN / 16, NT = H / 16, KX = DIN / 4, KH = H / 4, K3 = 3 * H / 4;
  constexpr int UNITS = DIN + 5 * H;   // transposed: x, h, dz, dr, dc (= da_h), dc r (= du_h)
  __shared__ float sT[4][UNITS * 16];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int j = lane & 15, g = lane >> 4;
  float* R = sT[wave];
  // transpose-tile offsets (seq_gru_bwd_kernel): write (unit 16t + 4g + q, row j); read (unit 16x + j,
  // rows 4g .. 4g + 3)
  const int wofs = j ^ (4 * g), rofs = j * 16 + 4 * (g ^ ((j >> 2) & 3));
  f4 dW[NC][3 * NT], dU[NT][3 * NT], bz[NT], br[NT], bc[NT], bu[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    bz[t] = br[t] = bc[t] = bu[t] = f4{0, 0, 0, 0};
#pragma unroll
    for (int nt = 0; nt < 3 * NT; ++nt) dU[t][nt] = f4{0, 0, 0, 0};
  }
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int nt = 0; nt < 3 * NT; ++nt) dW[c][nt] = f4{0, 0, 0, 0};
  const int64_t n_tiles = (a.n_dst + 15) / 16;
  for (int64_t tile = (int64_t)blockIdx.x * 4 + wave; tile < n_tiles; tile += (int64_t)gridDim.x * 4) {
    const int64_t row = tile * 16 + j;
    const bool valid = row < a.n_dst;
    const int64_t rr0 = valid ? row : 0;
    f4 x[NC], h[NT], dh[NT];
#pragma unroll
    for (int c = 0; c < NC; ++c) x[c] = ld4(a.x + rr0 * DIN + 16 * c + 4 * g);
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      h[t] = ld4(a.h + rr0 * H + 16 * t + 4 * g);
      dh[t] = valid ? ld4(a.dh_in + rr0 * H + 16 * t + 4 * g) : f4{0, 0, 0, 0};
    }
    f4 az[NT], ar[NT], ax[NT], ah[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      az[t] = ld4(a.bias + 0 * H + 16 * t + 4 * g);
      ar[t] = ld4(a.bias + 1 * H + 16 * t + 4 * g);
      ax[t] = ld4(a.bias + 2 * H + 16 * t + 4 * g);
      ah[t] = ld4(a.bias + 3 * H + 16 * t + 4 * g);
    }
    int lofs = lane;   // opaque: the fragment reads stay inside the tile loop (registers)
    asm volatile("" : "+v"(lofs));
#pragma unroll
    for (int s = 0; s < KX; ++s) {
      const float xb = x[s >> 2][s & 3];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        az[t] = MFMA(a.Wp[frag_idx(0 * NT + t, s, KX, lofs)], xb, az[t]);
        ar[t] = MFMA(a.Wp[frag_idx(1 * NT + t, s, KX, lofs)], xb, ar[t]);
        ax[t] = MFMA(a.Wp[frag_idx(2 * NT + t, s, KX, lofs)], xb, ax[t]);
      }
    }
#pragma unroll
    for (int s = 0; s < KH; ++s) {
      const float hb = h[s >> 2][s & 3];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        az[t] = MFMA(a.Up[frag_idx(0 * NT + t, s, KH, lofs)], hb, az[t]);
        ar[t] = MFMA(a.Up[frag_idx(1 * NT + t, s, KH, lofs)], hb, ar[t]);
        ah[t] = MFMA(a.Up[frag_idx(2 * NT + t, s, KH, lofs)], hb, ah[t]);
      }
    }
    f4 gz[NT], gr[NT], gh[NT], guh[NT], acc[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float z = sig2_(az[t][r]);
        const float rr = sig2_(ar[t][r]);
        const float c = tanh2_(ax[t][r] + rr * ah[t][r]);
        const float uh = ah[t][r] * kInv2Log2e;
        const float d = dh[t][r];
        const float dzp = d * (h[t][r] - c) * z * (1.f - z);
        const float dcp = d * (1.f - z) * (1.f - c * c);
        const float drp = dcp * uh * rr * (1.f - rr);
        gz[t][r] = dzp;
        gr[t][r] = drp;
        gh[t][r] = dcp;
        guh[t][r] = dcp * rr;
        acc[t][r] = d * z;
      }
    }
    f4 dxa[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) dxa[c] = f4{0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < K3; ++s) {
      const int gt = s >> 2, G = gt / NT, t2 = gt % NT;
      const float ba = G == 0 ? gz[t2][s & 3] : G == 1 ? gr[t2][s & 3] : gh[t2][s & 3];
      const float bv = G == 0 ? gz[t2][s & 3] : G == 1 ? gr[t2][s & 3] : guh[t2][s & 3];
#pragma unroll
      for (int c = 0; c < NC; ++c) dxa[c] = MFMA(a.Wt[frag_idx(c, s, K3, lofs)], ba, dxa[c]);
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[t] = MFMA(a.Ut[frag_idx(t, s, K3, lofs)], bv, acc[t]);
    }
    if (valid) {
#pragma unroll
      for (int t = 0; t < NT; ++t) st4(a.dh_out + row * H + 16 * t + 4 * g, acc[t]);
#pragma unroll
      for (int c = 0; c < NC; ++c) st4(a.dx + row * DIN + 16 * c + 4 * g, dxa[c]);
    }
    // the tile's x, h, da and du through the transpose tile, rows on the MFMA k axis
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int c = 0; c < NC; ++c) R[(16 * c + 4 * g + q) * 16 + wofs] = x[c][q];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        R[(DIN + 16 * t + 4 * g + q) * 16 + wofs] = h[t][q];
        R[(DIN + H + 16 * t + 4 * g + q) * 16 + wofs] = gz[t][q];
        R[(DIN + 2 * H + 16 * t + 4 * g + q) * 16 + wofs] = gr[t][q];
        R[(DIN + 3 * H + 16 * t + 4 * g + q) * 16 + wofs] = gh[t][q];
        R[(DIN + 4 * H + 16 * t + 4 * g + q) * 16 + wofs] = guh[t][q];
      }
    }
    f4 axT[NC], ahT[NT];
#pragma unroll
    for (int c = 0; c < NC; ++c) axT[c] = ld4(R + c * 256 + rofs);
#pragma unroll
    for (int t = 0; t < NT; ++t) ahT[t] = ld4(R + (DIN / 16 + t) * 256 + rofs);
#pragma unroll
    for (int nt = 0; nt < 3 * NT; ++nt) {
      const int gate = nt / NT, t2 = nt % NT;
      const f4 bda = ld4(R + ((DIN + H) / 16 + nt) * 256 + rofs);   // dz, dr, dc
      const f4 bdu = gate < 2 ? bda : ld4(R + ((DIN + 4 * H) / 16 + t2) * 256 + rofs);   // dz, dr, dc r
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
#pragma unroll
        for (int c = 0; c < NC; ++c) dW[c][nt] = MFMA(axT[c][ks], bda[ks], dW[c][nt]);
#pragma unroll
        for (int t = 0; t < NT; ++t) dU[t][nt] = MFMA(ahT[t][ks], bdu[ks], dU[t][nt]);
      }
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      bz[t] += gz[t];
      br[t] += gr[t];
      bc[t] += gh[t];
      bu[t] += guh[t];
    }
  }
  // this wave's partials: rows 0..DIN-1 / 0..H-1 = dW / dU (lane: D[16m + 4g + q][16nt + j]), then the
  // bias row [sum dz, sum dr, sum dc] (db_in) / [sum dz, sum dr, sum dc r] (db_rec)
  const int64_t wv = (int64_t)blockIdx.x * 4 + wave;
  float* Pw = part_w + wv * (DIN + 1) * (3 * H);
  float* Pu = part_u + wv * (H + 1) * (3 * H);
#pragma unroll
  for (int nt = 0; nt < 3 * NT; ++nt)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
#pragma unroll
      for (int c = 0; c < NC; ++c) Pw[(16 * c + 4 * g + q) * (3 * H) + 16 * nt + j] = dW[c][nt][q];
#pragma unroll
      for (int t = 0; t < NT; ++t) Pu[(16 * t + 4 * g + q) * (3 * H) + 16 * nt + j] = dU[t][nt][q];
    }
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      float sz = bz[t][q], sr = br[t][q], sc = bc[t][q], su = bu[t][q];
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {   // over the 16 rows j of group g
        sz += __shfl_xor(sz, o);
        sr += __shfl_xor(sr, o);
        sc += __shfl_xor(sc, o);
        su += __shfl_xor(su, o);
      }
      if (j == 0) {
        const int u = 16 * t + 4 * g + q;
        Pw[DIN * (3 * H) + u] = sz;
        Pw[DIN * (3 * H) + H + u] = sr;
        Pw[DIN * (3 * H) + 2 * H + u] = sc;
        Pu[H * (3 * H) + u] = sz;
        Pu[H * (3 * H) + H + u] = sr;
        Pu[H * (3 * H) + 2 * H + u] = su;
      }
    }
}

static int64_t sum_bwd_fused_blocks(int64_t n_dst) {
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (cus <= 0) cus = 256;
  }
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, sum_gru_bwd_fused_kernel<32, 32>, 256, 0) != hipSuccess ||
      per_cu <= 0)
    per_cu = 1;
  const int64_t tiles = (n_dst + 15) / 16;
  return std::max<int64_t>(1, std::min<int64_t>((tiles + 3) / 4, (int64_t)per_cu * cus));
}

int64_t sum_bwd_fused_waves(int64_t n_dst, int din, int h) {
  return (din == 32 && h == 32 && n_dst > 0) ? 4 * sum_bwd_fused_blocks(n_dst) : 0;
}

hipError_t launch_sum_gru_bwd_fused(const SumBwdArgs& a, int din, int h, float* part_w, float* part_u,
                                    hipStream_t st) {
  if (a.n_dst == 0) return hipSuccess;
  if (din != 32 || h != 32 || !part_w || !part_u) return hipErrorInvalidValue;
  hipLaunchKernelGGL((sum_gru_bwd_fused_kernel<32, 32>), dim3((unsigned)sum_bwd_fused_blocks(a.n_dst)), dim3(256), 0,
                     st, a, part_w, part_u);
  return hipGetLastError();
}

hipError_t launch_sum_gru_bwd(const SumBwdArgs& a, int din, int h, hipStream_t st) {
  if (a.n_dst == 0) return hipSuccess;
  dim3 grid((unsigned)((a.n_dst + 63) / 64));
#define SB_CASE(D, HH)                                                                   \
  if (din == D && h == HH) {                                                             \
    hipLaunchKernelGGL((sum_gru_bwd_kernel<D, HH>), grid, dim3(256), 0, st, a);          \
    return hipGetLastError();                                                            \
  }
  SB_CASE(16, 16)
  SB_CASE(16, 32)
  SB_CASE(32, 16)
  SB_CASE(32, 32)
  SB_CASE(64, 64)
#undef SB_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_attn_bwd_parts(const AttnArgs& a, const float* dx, const int32_t* mdst, SrcBases src, int F,
                                  int64_t n_msgs, float* dw, float* dv, hipStream_t st) {
  if (n_msgs == 0) return hipSuccess;
  hipLaunchKernelGGL(attn_dcoef_kernel, dim3(blocks_for(n_msgs)), dim3(256), 0, st, dx, mdst, a.msg_src, src, F, n_msgs, dw);
  if (a.n_groups)
    hipLaunchKernelGGL(attn_softmax_bwd_kernel, dim3((unsigned)((a.n_groups + 3) / 4)), dim3(256), 0, st, a, dw, dv);
  return hipGetLastError();
}

hipError_t launch_attn_src_bwd(int64_t rows, const int32_t* sptr, const int32_t* sidx, const float* msg_w,
                               const float* dv, const int32_t* mdst, const float* dx, const float* w1, int F, float* dh,
                               float* ds, hipStream_t st) {
  if (rows == 0) return hipSuccess;
  hipLaunchKernelGGL(attn_src_bwd_kernel, dim3(blocks_for(rows * F)), dim3(256), 0, st, rows, sptr, sidx, msg_w, dv, mdst,
                     dx, w1, F, dh, ds);
  return hipGetLastError();
}

hipError_t launch_attn_dst_bwd(int64_t n_pos, const int32_t* order, const int32_t* ptr, const float* dv, const float* w2,
                               int F, float* dh, float* ds, hipStream_t st) {
  if (n_pos == 0) return hipSuccess;
  hipLaunchKernelGGL(attn_dst_bwd_kernel, dim3(blocks_for(n_pos * F)), dim3(256), 0, st, n_pos, order, ptr, dv, w2, F,
                     dh, ds);
  return hipGetLastError();
}

hipError_t launch_attn_param_bwd(const float* dw12, const float* K1, const float* K2, const float* av, int F, float* dK1,
                                 float* dK2, float* dav, hipStream_t st) {
  hipLaunchKernelGGL(attn_param_bwd_kernel, dim3((2 * F * F + 255) / 256), dim3(256), 0, st, dw12, K1, K2, av, F, dK1,
                     dK2, dav);
  return hipGetLastError();
}

hipError_t launch_conv_bwd(const float* dx, const float* x, const float* deg, int64_t n, int F, int act, float* du,
                           float* dh, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(conv_bwd_kernel, dim3(blocks_for(n * F)), dim3(256), 0, st, dx, x, deg, n, F, act, du, dh);
  return hipGetLastError();
}

hipError_t launch_csr_gather_cols_add(float* out, int64_t n_rows, const int32_t* ptr, const int32_t* idx,
                                      const float* in, int in_stride, int col0, int width, int accumulate,
                                      hipStream_t st) {
  if (n_rows == 0 || width == 0) return hipSuccess;
  hipLaunchKernelGGL(csr_gather_cols_add_kernel, dim3(blocks_for(n_rows * width)), dim3(256), 0, st, out, n_rows, ptr,
                     idx, in, in_stride, col0, width, accumulate);
  return hipGetLastError();
}

hipError_t launch_csr_gather_add(float* out, int64_t n_rows, const int32_t* ptr, const int32_t* idx, const float* in,
                                 int cols, int accumulate, hipStream_t st) {
  if (n_rows == 0) return hipSuccess;
  if (cols % 4) return hipErrorInvalidValue;
  // V = 2 (8 columns per thread) for the ordered update's 96-column table gradient measured slower:
  // 305 -> 330 us per launch, 16.41 -> 16.58 ms per training step (tools/gpu_calls/r05_c57.sh)
#ifndef IGN_GATHER_TEMPORAL
  // the wide gather (the ordered update's ga rows, 1.4 GB read once per MP instance) loads its rows
  // non-temporally, so they do not push the other kernels' data out of L2 / MALL: 16.49 -> 16.20 ms
  // per training step, same box (tools/gpu_calls/r05_c59.sh); the same bits
  if (cols >= 64) {
    hipLaunchKernelGGL((csr_gather_add_kernel<1, true>), dim3(blocks_for(n_rows * (cols / 4))), dim3(256), 0, st, out,
                       n_rows, ptr, idx, in, cols, accumulate);
    return hipGetLastError();
  }
#endif
  hipLaunchKernelGGL(csr_gather_add_kernel<1>, dim3(blocks_for(n_rows * (cols / 4))), dim3(256), 0, st, out, n_rows,
                     ptr, idx, in, cols, accumulate);
  return hipGetLastError();
}

bool row_gemm_supported(int K, int M) {
  return (K == 48 || K == 96 || K == 192 || K == 256) && (M == 16 || M == 32 || M == 64 || M == 256);
}

hipError_t launch_row_gemm_t(const float* in, int64_t n, int K, const float* Ap, int M, float* out, int accumulate,
                             int act, const float* aprev, hipStream_t st) {
  if (n == 0) return hipSuccess;
  dim3 grid((unsigned)((n + 63) / 64));
#define RG_CASE(KK, MM)                                                                                  \
  if (K == KK && M == MM) {                                                                              \
    hipLaunchKernelGGL((row_gemm_t_kernel<KK, MM>), grid, dim3(256), 0, st, in, n, Ap, out, accumulate, act, aprev); \
    return hipGetLastError();                                                                            \
  }
  RG_CASE(48, 16)
  RG_CASE(96, 16)
  RG_CASE(48, 32)
  RG_CASE(96, 32)
  RG_CASE(192, 64)
  RG_CASE(256, 16)
  RG_CASE(256, 32)
  RG_CASE(256, 64)
  RG_CASE(256, 256)
#undef RG_CASE
  return hipErrorInvalidValue;
}

hipError_t launch_row_gemm_t_generic(const float* in, int64_t n, int K, const float* Mat, int M, float* out,
                                     int accumulate, int act, const float* aprev, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (K == 1 && M % 4 == 0) {
    hipLaunchKernelGGL(row_outer_t_kernel, dim3(blocks_for(n * (M / 4))), dim3(256), 0, st, in, n, Mat, M, out,
                       accumulate, act, aprev);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(row_gemm_t_generic_kernel, dim3(blocks_for(n * M)), dim3(256), 0, st, in, n, K, Mat, M, out,
                     accumulate, act, aprev);
  return hipGetLastError();
}

hipError_t launch_split_cols_add(float* dst, int64_t n, int width, const float* src, int src_stride, int col0,
                                 hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(split_cols_add_kernel, dim3(blocks_for(n * width)), dim3(256), 0, st, dst, n, width, src,
                     src_stride, col0);
  return hipGetLastError();
}

hipError_t launch_act_bwd(const float* da, const float* a, int64_t n, int act, float* dz, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(act_bwd_kernel, dim3(blocks_for(n)), dim3(256), 0, st, da, a, n, act, dz);
  return hipGetLastError();
}

static int g_tsgemm_bf = 1;   // set per backward from the plan (ign_backward: set_tsgemm_bf)
void set_tsgemm_bf(bool on) { g_tsgemm_bf = on ? 1 : 0; }

int64_t tsgemm_partial_floats(int64_t n_rows, int M, int N) {
  const TsPlan p = ts_plan(n_rows, M, N, 1);
  return (p.chunks + kTsSegs) * (int64_t)p.Mx * N;
}

int64_t tsgemm_chunks(int64_t n_rows, int M, int N, int ones) { return n_rows ? ts_plan(n_rows, M, N, ones).chunks : 0; }

hipError_t launch_tsgemm_add(const float* A, int lda, const float* B, int ldb, int64_t n_rows, int M, int N,
                             float* part, float* C, float* Cb, hipStream_t st) {
  if (n_rows == 0) return hipSuccess;
  const int ones = Cb != nullptr;
  const hipError_t e = launch_tsgemm_partials(A, lda, B, ldb, n_rows, M, N, ones, part, st);
  if (e != hipSuccess) return e;
  return launch_partials_reduce_add(part, tsgemm_chunks(n_rows, M, N, ones), M, N, ones, C, Cb, st);
}

hipError_t launch_tsgemm_partials(const float* A, int lda, const float* B, int ldb, int64_t n_rows, int M, int N,
                                  int ones, float* part, hipStream_t st) {
  if (n_rows == 0) return hipSuccess;
  const TsPlan p = ts_plan(n_rows, M, N, ones);
  // one wave per 64x64 tile: a 1- or 2-tile contraction gets 1- or 2-wave blocks, no idle waves
  const int wpb = std::min(4, p.tiles);
  dim3 grid((unsigned)p.chunks, (unsigned)((p.tiles + wpb - 1) / wpb));
  // split-bf16 contraction (kernels_bf.hip) when A is present; the plan's IGN_TSGEMM_BF=0 keeps f32 MFMA
  hipError_t e;
  if (A && N == 1 && M % 4 == 0 && M <= 256 && lda % 4 == 0 && ((uintptr_t)A & 15) == 0) {   // exact f32 fma
    hipLaunchKernelGGL(tsgemv_kernel, dim3((unsigned)p.chunks), dim3(256), 0, st, A, lda, B, ldb, n_rows, M, ones,
                       p.chunk, part);
    e = hipGetLastError();
  } else if (g_tsgemm_bf && A) {
    e = launch_tsgemm_bf(A, lda, B, ldb, n_rows, M, N, ones, p.chunk, p.chunks, p.tiles, wpb, part, st);
  } else {
    hipLaunchKernelGGL(tsgemm_kernel, grid, dim3(64 * wpb), 0, st, A, lda, B, ldb, n_rows, M, N, ones, p.chunk, part);
    e = hipGetLastError();
  }
  return e;
}

// C[m][n] (+ Cb[n] for the ones row m = M) += sum over chunks c of part[c][m][n], in chunk order
// (segment sums, then the segments in order); part holds kTsSegs more chunk slots as scratch
hipError_t launch_partials_reduce_add(float* part, int64_t nchunks, int M, int N, int ones, float* C, float* Cb,
                                      hipStream_t st) {
  const int64_t size = (int64_t)(M + ones) * N;
  float* seg = part + nchunks * size;
  const int S = (int)std::min<int64_t>(kTsSegs, nchunks);
  hipLaunchKernelGGL(reduce_seg_kernel, dim3((unsigned)((size + 255) / 256), (unsigned)S), dim3(256), 0, st, part,
                     nchunks, size, S, seg);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(reduce_final_kernel, dim3(blocks_for(size)), dim3(256), 0, st, seg, S, M, N, ones, C, Cb);
  return hipGetLastError();
}

hipError_t launch_colsum_add(const float* B, int ldb, int64_t n_rows, int N, float* part, float* C, hipStream_t st) {
  return launch_tsgemm_add(nullptr, 0, B, ldb, n_rows, 0, N, part, nullptr, C, st);
}

bool dense_fwd_supported(int K, int M) {
  return (K == 16 || K == 32 || K == 48 || K == 64 || K == 96 || K == 128 || K == 256) &&
         (M == 16 || M == 32 || M == 64 || M == 128 || M == 256);
}

hipError_t launch_dense_fwd(const float* x, int64_t n, int K, int x_stride, const float* Wp, const float* W,
                            const float* bias, int M, int act, float* y, hipStream_t st) {
  if (n == 0) return hipSuccess;
  if (M == 1 && K % 4 == 0 && x_stride % 4 == 0) {
    hipLaunchKernelGGL(dense_dot_kernel, dim3((unsigned)((n * 16 + 255) / 256)), dim3(256), 0, st, x, n, K, x_stride,
                       W, bias, act, y);
    return hipGetLastError();
  }
  dim3 grid((unsigned)((n + 63) / 64));
#define DF_CASE(KK, MM)                                                                                        \
  if (K == KK && M == MM && Wp) {                                                                              \
    hipLaunchKernelGGL((dense_fwd_kernel<KK, MM>), grid, dim3(256), 0, st, x, n, x_stride, Wp, bias, act, y);  \
    return hipGetLastError();                                                                                  \
  }
  DF_CASE(16, 16)
  DF_CASE(16, 32)
  DF_CASE(16, 64)
  DF_CASE(16, 128)
  DF_CASE(16, 256)
  DF_CASE(32, 16)
  DF_CASE(32, 32)
  DF_CASE(32, 64)
  DF_CASE(32, 128)
  DF_CASE(32, 256)
  DF_CASE(48, 16)
  DF_CASE(48, 32)
  DF_CASE(48, 64)
  DF_CASE(48, 128)
  DF_CASE(48, 256)
  DF_CASE(64, 16)
  DF_CASE(64, 32)
  DF_CASE(64, 64)
  DF_CASE(64, 128)
  DF_CASE(64, 256)
  DF_CASE(96, 16)
  DF_CASE(96, 32)
  DF_CASE(96, 64)
  DF_CASE(96, 128)
  DF_CASE(96, 256)
  DF_CASE(128, 16)
  DF_CASE(128, 32)
  DF_CASE(128, 64)
  DF_CASE(128, 128)
  DF_CASE(128, 256)
  DF_CASE(256, 16)
  DF_CASE(256, 32)
  DF_CASE(256, 64)
  DF_CASE(256, 128)
  DF_CASE(256, 256)
#undef DF_CASE
  return launch_dense_generic(x, n, K, x_stride, W, bias, M, act, y, st);
}

hipError_t launch_axpy(float* y, const float* x, float alpha, int64_t n, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(axpy_kernel, dim3(blocks_for(n)), dim3(256), 0, st, y, x, alpha, n);
  return hipGetLastError();
}

hipError_t launch_mse(const float* pred, const float* label, int64_t n, float* dpred, double* part, int nblk,
                      hipStream_t st) {
  hipLaunchKernelGGL(mse_kernel, dim3(nblk), dim3(256), 0, st, pred, label, n, dpred, part);
  return hipGetLastError();
}

hipError_t launch_sumsq(const float* x, int64_t n, double* part, int nblk, hipStream_t st) {
  hipLaunchKernelGGL(sumsq_kernel, dim3(nblk), dim3(256), 0, st, x, n, part);
  return hipGetLastError();
}

hipError_t launch_adam(float* w, const float* g, float* m, float* v, int64_t n, float lr_t, float b1, float b2,
                       float eps, hipStream_t st) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(adam_kernel, dim3(blocks_for(n)), dim3(256), 0, st, w, g, m, v, n, lr_t, b1, b2, eps);
  return hipGetLastError();
}
