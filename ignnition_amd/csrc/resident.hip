// resident.hip — the graph-resident forward for small graphs (RouteNet-shaped models).
//
// The batched kernels (seq_gru_h16, sum_gru_g32) run every MP over the whole batch: one launch per MP
// and iteration, states and projected tables in HBM / Infinity Cache between launches.  For graphs
// whose states fit in LDS (GEANT2: 552 paths, 74 links; NSFNET) the sum update is the slow part:
// 2.4 k link tiles per 512-graph batch leave ~2 waves per SIMD, each walking chains of up to 90
// dependent row loads (DESIGN.md §3b''').  Here one workgroup owns one graph for all T iterations:
//   LDS: path states [P][36], link states [L][36], the ordered MP's projected table [L + 1][100]
//        (the hole row last), U's fp16 pieces;
//   per iteration: phase A, the ordered update (link -> path, seq_gru_h16's tile loop over the
//        graph's paths sorted by length; the projected rows and states come from LDS), barrier,
//        phase B, the sum update (path -> link) in three passes over all 16 waves: B1 the message
//        sums (sum_gru_g32's adds in message order, one lane per (link, float4 column), the local
//        CSR in LDS), B2 its split-bf16 GRU step (one wave per (link tile, column half)), B3 the
//        next iteration's projection of the new link states (sum_gru_g32's fused projection, one
//        wave per (link tile, gate)), barriers between.
// The arithmetic per row is that of the batched kernels: the same message order, pieces, products
// and gate formulas (iteration 0 projects with project_kernel's f32 MFMA, later iterations with
// sum_gru_g32's fused split-bf16 projection), so the predictions are the batched forward's bits and
// a graph's predictions do not depend on which path its batch took.  (The ordered update's tiles
// hold one graph's paths here; a tile's power-of-two scale only moves bits when a state lies
// outside [-1, 1] and its low fp16 piece goes subnormal -- tests/test_gpu_parity.py checks equality.)
// Only the final states leave the workgroup; the batched readout then runs on the path states.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "kernels.h"
#include "device_common.h"

#ifdef IGN_RES_STAMP
// Diagnostic build only (tools/build_ab.sh NAME -DIGN_RES_STAMP; tools/probes/res_stamps.py): per
// wave of the first 256 workgroups, s_memtime sums of the phases (cdna_hip_programming.md §7).
__device__ unsigned long long ign_res_stamps[256 * kResidentWaves * 8];
#define IGN_STAMP(v)                                                          \
  do {                                                                        \
    __builtin_amdgcn_sched_barrier(0);                                        \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(v)::"memory"); \
    __builtin_amdgcn_sched_barrier(0);                                        \
  } while (0)
extern "C" int ign_debug_res_stamps(unsigned long long* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(ign_res_stamps), (size_t)n * 8, 0, hipMemcpyDeviceToHost);
}
#endif

namespace {

constexpr int kW = kResidentWaves;
constexpr int SP = kResidentStateStride;   // LDS row stride of a 32-wide state row (floats)
constexpr int ST = kResidentTableStride;   // LDS row stride of a 96-wide projected row (floats)

__device__ __forceinline__ f4 lds4(const float* p) { return *reinterpret_cast<const f4*>(p); }
__device__ __forceinline__ void lds4w(float* p, f4 v) { *reinterpret_cast<f4*>(p) = v; }

// the three exact bf16 pieces of a lane's 8 values in the chained B layout (kernels_bf.hip)
__device__ __forceinline__ void split_frags1(const f4* v, bf8 (&f)[3][1]) {
  u4v w0, w1, w2;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int e0 = 2 * q, e1 = 2 * q + 1;
    float a0, a1, a2, b0, b1, b2;
    split3(v[e0 >> 2][e0 & 3], a0, a1, a2);
    split3(v[e1 >> 2][e1 & 3], b0, b1, b2);
    w0[q] = pack_hi16(a0, b0);
    w1[q] = pack_hi16(a1, b1);
    w2[q] = pack_hi16(a2, b2);
  }
  f[0][0] = __builtin_bit_cast(bf8, w0);
  f[1][0] = __builtin_bit_cast(bf8, w1);
  f[2][0] = __builtin_bit_cast(bf8, w2);
}

// the ordered MP's projected row of a link state in the B layout (sum_gru_g32's fused projection:
// split-bf16 x6, the pieces of W' from L2), written to the LDS table row ll
__device__ __forceinline__ void project_row(const ResidentArgs& a, const f4 (&hn)[2], float* tab, int ll, bool valid,
                                            int lane, int g) {
  // an opaque lane offset: keeps the loop-invariant fragment addresses from being hoisted out of the
  // tile loops into (spilled) registers
  int lofs = lane;
  asm volatile("" : "+v"(lofs));
  constexpr int H = 32, NT = 2;
  bf8 pf[3][1];
  split_frags1(hn, pf);
  const bf8* pw = static_cast<const bf8*>(a.proj_W);
#pragma unroll
  for (int G = 0; G < 3; ++G)
#pragma unroll
    for (int i = 0; i < NT; ++i) {
      f4 acc = ld4(a.proj_b + G * H + 16 * i + 4 * g);
#pragma unroll
      for (int pu = 2; pu >= 0; --pu) {
        const bf8 w = pw[((pu * 3 + G) * NT + i) * 64 + lofs];
#pragma unroll
        for (int ph = 2 - pu; ph >= 0; --ph) acc = MFMA_BF(w, pf[ph][0], acc);
      }
      if (valid) lds4w(tab + (int64_t)ll * ST + G * H + 16 * i + 4 * g, acc);
    }
}

// the iteration-0 projected row as project_kernel computes it (f32 MFMA, x.W' over k-steps of 1 on
// the bias) so the resident forward reproduces the batched forward's bits
__device__ __forceinline__ void project_row_f32(const ResidentArgs& a, const f4 (&xv)[2], float* tab, int ll,
                                                bool valid, int lane, int g) {
  int lofs = lane;
  asm volatile("" : "+v"(lofs));
  constexpr int H = 32, NT = 2, KX = 32 / 4;
  f4 acc[3][NT];
#pragma unroll
  for (int G = 0; G < 3; ++G)
#pragma unroll
    for (int t = 0; t < NT; ++t) acc[G][t] = ld4(a.proj_b + G * H + 16 * t + 4 * g);
#pragma unroll
  for (int s = 0; s < KX; ++s) {
    const float xb = xv[s >> 2][s & 3];
#pragma unroll
    for (int G = 0; G < 3; ++G)
#pragma unroll
      for (int t = 0; t < NT; ++t) acc[G][t] = MFMA(a.proj_Wf[frag_idx(G * NT + t, s, KX, lofs)], xb, acc[G][t]);
  }
  if (valid) {
#pragma unroll
    for (int G = 0; G < 3; ++G)
#pragma unroll
      for (int t = 0; t < NT; ++t) lds4w(tab + (int64_t)ll * ST + G * H + 16 * t + 4 * g, acc[G][t]);
  }
}

}  // namespace

// PG: the path states stay in the batch's state buffer in HBM / L2 (rows of 32 floats) and the
// ordered MP's step codes are read from global memory: the form for graphs whose path states do
// not fit (synth50: 2 450 paths); LDS then holds the link states, the projected table and the
// sum MP's CSR
template <bool PG>
__global__ __launch_bounds__(64 * kW) void resident_forward_kernel(ResidentArgs a) {
  constexpr int H = 32, NT = 2, KS = 1, NF = 6 * NT * KS;   // U's fp16 pieces: 2 pieces x 3 gates x NT
  constexpr int NFB = 18;                                     // bf16 pieces of W / U per matrix (g32)
  __shared__ h8 su[NF * 64];
  __shared__ float sbn[kW][H];
  __shared__ float sbias[H];
  __shared__ int sctr[2];   // phase A's tile counters (alternate iterations)
  extern __shared__ float dyn[];
  const int gph = blockIdx.x;
  const int64_t p0 = a.path_off[gph], P = a.path_off[gph + 1] - p0;
  const int64_t l0 = a.link_off[gph], L = a.link_off[gph + 1] - l0;
  constexpr int SPP = PG ? H : SP;   // row stride of the path states
  float* hP = PG ? a.path_state + p0 * H : dyn;
  float* hL = PG ? dyn : hP + P * SP;
  float* tab = hL + L * SP;
  int* smp = reinterpret_cast<int*>(tab + (L + 1) * ST);   // the sum MP's CSR by local link row
  uint16_t* slo = reinterpret_cast<uint16_t*>(smp + L + 1);   // link order for the message sums
  uint16_t* sms_l = slo + ((L + 1) & ~1);
  const int64_t ms0 = a.lmsg_off[gph], M = a.lmsg_off[gph + 1] - ms0;
  uint16_t* scd_l = sms_l + M;   // the ordered MP's local step codes
  const int64_t cd0 = a.lcode_off[gph], NC = a.lcode_off[gph + 1] - cd0;
  const uint16_t* sms = sms_l;                      // in LDS in both forms
  const uint16_t* scd = PG ? a.lcode + cd0 : scd_l;   // PG: read from global memory
  float* xs = tab;   // phase B's message sums [L][SP] alias the (consumed) projected table
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j = lane & 15, g = lane >> 4;
#ifdef IGN_RES_STAMP
  unsigned long long t_0, t_a, t_b, s_init = 0, s_aw = 0, s_ab = 0, s_bw = 0, s_bb = 0, n_at = 0, n_bt = 0;
  IGN_STAMP(t_0);
#endif
  for (int i = tid; i < H; i += 64 * kW) sbias[i] = a.seq_bias[3 * H + i];
  if (tid < 2) sctr[tid] = 0;
  {
    const u4v* src = reinterpret_cast<const u4v*>(a.Uh);
    u4v* dst = reinterpret_cast<u4v*>(su);
    for (int e = tid; e < NF * 64; e += 64 * kW) dst[e] = src[e];
  }
  const int es = __float_as_int(reinterpret_cast<const float*>(a.Uh)[(int64_t)NF * 64 * 4]);
  // GM:396-400: state_0 = [features | zeros]
  for (int64_t i = tid; i < P * H; i += 64 * kW) {
    const int64_t r = i / H;
    const int c = (int)(i - r * H);
    hP[r * SPP + c] = c < a.path_F ? a.path_feat[(p0 + r) * a.path_F + c] : 0.f;
  }
  for (int64_t i = tid; i < L * H; i += 64 * kW) {
    const int64_t r = i / H;
    const int c = (int)(i - r * H);
    hL[r * SP + c] = c < a.link_F ? a.link_feat[(l0 + r) * a.link_F + c] : 0.f;
  }
  for (int i = tid; i < 3 * H; i += 64 * kW) tab[L * ST + i] = a.proj_b[i];   // the hole row: b' alone
  {
    const int* gp = a.lmsg_ptr + l0 + gph;
    for (int64_t i = tid; i <= L; i += 64 * kW) smp[i] = gp[i];
    for (int64_t i = tid; i < M; i += 64 * kW) sms_l[i] = a.lmsg_src[ms0 + i];
    for (int64_t i = tid; i < L; i += 64 * kW) slo[i] = a.lorder[l0 + i];
    if constexpr (!PG)
      for (int64_t i = tid; i < NC; i += 64 * kW) scd_l[i] = a.lcode[cd0 + i];
  }
  __syncthreads();
  const int64_t nlt = (L + 15) / 16;   // link tiles
  // the first iteration's projected table
  for (int64_t k = wave; k < nlt; k += kW) {
    const int64_t idx = 16 * k + j;
    const bool valid = idx < L;
    const int ll = valid ? (int)idx : 0;
    f4 h[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) h[t] = valid ? lds4(hL + (int64_t)ll * SP + 16 * t + 4 * g) : f4{0, 0, 0, 0};
    project_row_f32(a, h, tab, ll, valid, lane, g);
  }
  __syncthreads();
#ifdef IGN_RES_STAMP
  IGN_STAMP(t_a);
  s_init = t_a - t_0;
#endif

  const int64_t pt0 = a.ptile_off[gph], npt = (a.ptile_off[gph + 1] - pt0) / 16;
  for (int it = 0; it < a.T; ++it) {
    // ---- phase A: the ordered update (seq_gru_h16's tile loop over the graph's path tiles) ----
#ifdef IGN_RES_STATIC
    auto claim = [&](int k) -> int { return k < 0 ? wave : k + kW; };   // A/B: wave w takes tiles w, w + 16, ...
#else
    // the waves claim tiles from an LDS counter, longest tiles first (a greedy longest-first schedule:
    // the SIMDs' arbitration decides which wave gets more of them; results do not depend on it)
    int* ctr = &sctr[it & 1];
    if (tid == 0) sctr[(it + 1) & 1] = 0;   // the next iteration's counter (its last user finished)
    auto claim = [&](int) -> int {
      int v = 0;
      if (lane == 0) v = atomicAdd(ctr, 1);
      return __builtin_amdgcn_readfirstlane(v);
    };
#endif
    int k = claim(-1);
    i4v hd_next = k < npt ? *reinterpret_cast<const i4v*>(a.hdr + 4 * (pt0 + 16 * k + j)) : i4v{0, 0, 0, 0};
    while (k < npt) {
      const i4v hd = hd_next;   // the next tile's header loads under this tile's steps
      const int kn = claim(k);
      if (kn < npt) hd_next = *reinterpret_cast<const i4v*>(a.hdr + 4 * (pt0 + 16 * kn + j));
      const int Lr = hd[1];
      const bool valid = Lr > 0;   // tile padding: length 0
      const int64_t rl = valid ? hd[0] : 0;
      const int cbase = hd[2];   // (an index, not a pointer: one VGPR live through the tile)
      f4 h[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const f4 v = lds4(hP + rl * SPP + 16 * t + 4 * g);
        h[t] = valid ? v : f4{0, 0, 0, 0};
      }
      f4 x[3][NT];
      auto load_x = [&](uint32_t code, f4 (&xx)[3][NT]) __attribute__((always_inline)) {
        const float* p = tab + (int64_t)code * ST + 4 * g;
#pragma unroll
        for (int G = 0; G < 3; ++G)
#pragma unroll
          for (int i = 0; i < NT; ++i) xx[G][i] = lds4(p + G * H + 16 * i);
      };
      load_x((uint32_t)hd[3], x);
      uint32_t code = scd[cbase + 1];
      // positions are sorted by length, descending, within the graph: lane 0 is the longest
      const int Lmax = __builtin_amdgcn_readfirstlane(Lr);
      float m = 1.0f;
#pragma unroll
      for (int t = 0; t < NT; ++t)
#pragma unroll
        for (int r = 0; r < 4; ++r) m = fmaxf(m, fabsf(h[t][r]));
      if (__ballot(m > 1.0f) != 0) {
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
      }
      const int E = (__builtin_amdgcn_readfirstlane(__float_as_int(m)) >> 23) - 126;
      const int eS = 15 - E;
      const float S = __int_as_float((127 + eS) << 23);
      const float SS = __int_as_float((127 + eS + es) << 23);
      const float c = __int_as_float((127 - eS - es) << 23);
      const float iS = __int_as_float((127 - eS) << 23);
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        h[t] *= S;
        *reinterpret_cast<f4*>(&sbn[wave][16 * t + 4 * g]) = *reinterpret_cast<const f4*>(sbias + 16 * t + 4 * g) * SS;
      }
      auto step = [&](int t, const f4 (&xx)[3][NT], auto masked) __attribute__((always_inline)) {
        h8 hf[2][KS];
        {
          u4v w0, w1;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const int e0 = 2 * q, e1 = 2 * q + 1;
            const hpair pr = split2h(h[e0 >> 2][e0 & 3], h[e1 >> 2][e1 & 3]);
            w0[q] = pr.hi;
            w1[q] = pr.lo;
          }
          hf[0][0] = __builtin_bit_cast(h8, w0);
          hf[1][0] = __builtin_bit_cast(h8, w1);
        }
        f4 acc[3][NT];
#pragma unroll
        for (int i = 0; i < NT; ++i) {
          acc[0][i] = f4{0, 0, 0, 0};
          acc[1][i] = f4{0, 0, 0, 0};
          acc[2][i] = *reinterpret_cast<const f4*>(&sbn[wave][16 * i + 4 * g]);
        }
        int lofs = lane;
        asm volatile("" : "+v"(lofs));
#pragma unroll
        for (int pu = 1; pu >= 0; --pu)
#pragma unroll
          for (int i = 0; i < NT; ++i) {
            h8 w[3];
#pragma unroll
            for (int G = 0; G < 3; ++G) w[G] = su[((pu * 3 + G) * NT + i) * KS * 64 + lofs];
#pragma unroll
            for (int ph = 1; ph >= 0; --ph) {
              if (pu + ph > 1) continue;
#pragma unroll
              for (int G = 0; G < 3; ++G) acc[G][i] = MFMA_H(w[G], hf[ph][0], acc[G][i]);
            }
          }
        const bool act = t < Lr;
#pragma unroll
        for (int i = 0; i < NT; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float z = rcpf_(1.0f + __builtin_amdgcn_exp2f(fmaf(acc[0][i][r], c, xx[0][i][r])));
            const float rc = rcpf_(fmaf(__builtin_amdgcn_exp2f(fmaf(acc[1][i][r], c, xx[1][i][r])), SS, SS));
            const float n = S * tanh2_(fmaf(rc, acc[2][i][r], xx[2][i][r]));
            const float hn = n + z * (h[i][r] - n);
            if constexpr (decltype(masked)::value) h[i][r] = act ? hn : h[i][r];
            else h[i][r] = hn;
          }
      };
      // the tile's shortest sequence: its last real path's (tiles are padded at the graph's end)
      const int Lmin = __builtin_amdgcn_readlane(Lr, (int)min<int64_t>(15, P - 1 - 16 * k));
      for (int t = 0;;) {
        if (t < Lmin) step(t, x, std::false_type{});
        else step(t, x, std::true_type{});
        if (++t >= Lmax) break;
        load_x(code, x);
        code = scd[cbase + t + 1];
      }
      if (valid) {
#pragma unroll
        for (int t = 0; t < NT; ++t) lds4w(hP + rl * SPP + 16 * t + 4 * g, h[t] * iS);
      }
      k = kn;
    }
#ifdef IGN_RES_STAMP
    IGN_STAMP(t_b);
    s_aw += t_b - t_a;
#endif
    __syncthreads();
#ifdef IGN_RES_STAMP
    IGN_STAMP(t_a);
    s_ab += t_a - t_b;
#endif
    // ---- phase B: the sum update, in three passes over all 16 waves ----
    // B1: the message sums, one lane per (link, float4 column): the adds of sum_gru_g32's lane walk
    // (message order from zero, per column), the codes from LDS
    for (int64_t i = tid; i < L * (H / 4); i += 64 * kW) {
      const int64_t ll = slo[i >> 3];   // links by message count, descending: the long chains first
      const int c4 = (int)(i & 7);
      const int m0 = smp[ll], m1 = smp[ll + 1];
      const float* hp = hP + 4 * c4;
      f4 x = {0, 0, 0, 0};
      int m = m0;
      if constexpr (PG) {   // rows from L2: sixteen in flight (two groups of eight double-buffered
                            // spilled 276 B per lane and ran 40 % slower)
        for (; m + 16 <= m1; m += 16) {
          int rr[16];
#pragma unroll
          for (int u = 0; u < 16; ++u) rr[u] = sms[m + u];
          f4 v[16];
#pragma unroll
          for (int u = 0; u < 16; ++u) v[u] = lds4(hp + rr[u] * SPP);
#pragma unroll
          for (int u = 0; u < 16; ++u) x = x + v[u];
        }
      }
      for (; m + 8 <= m1; m += 8) {
        int rr[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) rr[u] = sms[m + u];
        f4 v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = lds4(hp + rr[u] * SPP);
#pragma unroll
        for (int u = 0; u < 8; ++u) x = x + v[u];
      }
      for (; m < m1; ++m) x = x + lds4(hp + sms[m] * SPP);
      lds4w(xs + ll * SP + 4 * c4, x);
    }
    __syncthreads();
#ifdef IGN_RES_STAMP
    {   // B1's end (after its barrier): n_at accumulates B1, n_bt B1 + B2 (diagnostic fields)
      unsigned long long t_c;
      IGN_STAMP(t_c);
      n_at += t_c - t_a;
    }
#endif
    // B2: the split-bf16 GRU step (sum_gru_g32's): one output half (16 columns) of a link tile
    const bool last = it + 1 == a.T;
    const bf8* sW = static_cast<const bf8*>(a.sWbf);
    const bf8* sU = static_cast<const bf8*>(a.sUbf);
    auto gru_half = [&](const bf8 (&xf)[3][1], const bf8 (&hf)[3][1], const f4 ho, int t) __attribute__((always_inline)) {
      int lofs = lane + 64 * t;   // opaque: the fragment addresses stay inside the loop (as project_row)
      asm volatile("" : "+v"(lofs));
      const int u0 = 16 * t + 4 * g;
      f4 az = ld4(a.sum_bias + 0 * H + u0), ar = ld4(a.sum_bias + 1 * H + u0);
      f4 ax = ld4(a.sum_bias + 2 * H + u0), ah = ld4(a.sum_bias + 3 * H + u0);
#pragma unroll
      for (int pu = 2; pu >= 0; --pu) {
        const bf8 wz = sW[((pu * 3 + 0) * NT) * 64 + lofs];
        const bf8 wr = sW[((pu * 3 + 1) * NT) * 64 + lofs];
        const bf8 wh = sW[((pu * 3 + 2) * NT) * 64 + lofs];
#pragma unroll
        for (int ph = 2 - pu; ph >= 0; --ph) {
          az = MFMA_BF(wz, xf[ph][0], az);
          ar = MFMA_BF(wr, xf[ph][0], ar);
          ax = MFMA_BF(wh, xf[ph][0], ax);
        }
        const bf8 uz = sU[((pu * 3 + 0) * NT) * 64 + lofs];
        const bf8 ur = sU[((pu * 3 + 1) * NT) * 64 + lofs];
        const bf8 uh = sU[((pu * 3 + 2) * NT) * 64 + lofs];
#pragma unroll
        for (int ph = 2 - pu; ph >= 0; --ph) {
          az = MFMA_BF(uz, hf[ph][0], az);
          ar = MFMA_BF(ur, hf[ph][0], ar);
          ah = MFMA_BF(uh, hf[ph][0], ah);
        }
      }
      f4 hn;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float z = sig2_(az[r]);
        const float rg = sig2_(ar[r]);
        const float cnd = tanh2_(ax[r] + rg * ah[r]);
        hn[r] = cnd + z * (ho[r] - cnd);
      }
      return hn;
    };
#ifdef IGN_RES_B23_SPLIT   // A/B: B2 and B3 as separate passes whatever the link count
    const bool fused23 = false;
#else
    const bool fused23 = nlt <= kW;   // block-uniform
#endif
    if (fused23) {
      // B2 + B3 in one pass, one wave per link tile: the GRU step of both halves, the new states,
      // then the next iteration's projected rows of the tile.  The message sums are read into
      // registers before a barrier: they alias table rows that other waves' projections overwrite
      const int64_t k = wave;
      const bool act = k < nlt;   // wave-uniform
      const int64_t idx = 16 * k + j;
      const bool valid = act && idx < L;
      const int ll = valid ? (int)idx : 0;
      f4 x[2], h[2];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        x[c] = act ? lds4(xs + (int64_t)ll * SP + 16 * c + 4 * g) : f4{0, 0, 0, 0};
        h[c] = act ? lds4(hL + (int64_t)ll * SP + 16 * c + 4 * g) : f4{0, 0, 0, 0};
      }
      __syncthreads();
      if (act) {
        bf8 xf[3][1], hf[3][1];
        split_frags1(x, xf);
        split_frags1(h, hf);
        f4 hn[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) hn[t] = gru_half(xf, hf, h[t], t);
        if (valid) {
#pragma unroll
          for (int t = 0; t < NT; ++t) lds4w(hL + (int64_t)ll * SP + 16 * t + 4 * g, hn[t]);
        }
        if (!last) project_row(a, hn, tab, ll, valid, lane, g);
      }
    } else {
    // B2 as its own pass: one wave per (link tile, half); the new states are written after a
    // barrier (the other half's wave still reads the old ones)
    const int64_t nb2 = 2 * nlt, rounds2 = (nb2 + kW - 1) / kW;
    for (int64_t rr = 0; rr < rounds2; ++rr) {
      const int64_t item = rr * kW + wave;
      const bool act = item < nb2;   // wave-uniform
      const int64_t k = act ? item >> 1 : 0;
      const int t = (int)(item & 1);
      const int64_t idx = 16 * k + j;
      const bool valid = act && idx < L;
      const int ll = valid ? (int)idx : 0;
      f4 hn = {0, 0, 0, 0};
      if (act) {
        f4 x[2], h[2];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          x[c] = lds4(xs + (int64_t)ll * SP + 16 * c + 4 * g);
          h[c] = lds4(hL + (int64_t)ll * SP + 16 * c + 4 * g);
        }
        bf8 xf[3][1], hf[3][1];
        split_frags1(x, xf);
        split_frags1(h, hf);
        hn = gru_half(xf, hf, t ? h[1] : h[0], t);
      }
      __syncthreads();
      if (valid) lds4w(hL + (int64_t)ll * SP + 16 * t + 4 * g, hn);
    }
    static_assert(NFB == 18, "g32 piece layout");
#ifdef IGN_RES_STAMP
    {
      unsigned long long t_c;
      IGN_STAMP(t_c);
      n_bt += t_c - t_a;
    }
#endif
    // B3: the next iteration's projected table (sum_gru_g32's fused projection), one wave per
    // (link tile, gate)
    if (!last) {
      __syncthreads();
      const bf8* pw = static_cast<const bf8*>(a.proj_W);
      for (int64_t item = wave; item < 3 * nlt; item += kW) {
        const int64_t k = item / 3;
        const int G = (int)(item - 3 * k);
        const int64_t idx = 16 * k + j;
        const bool valid = idx < L;
        const int ll = valid ? (int)idx : 0;
        f4 h[2];
#pragma unroll
        for (int c = 0; c < 2; ++c) h[c] = lds4(hL + (int64_t)ll * SP + 16 * c + 4 * g);
        bf8 pf[3][1];
        split_frags1(h, pf);
        int lofs = lane + 64 * NT * G;
        asm volatile("" : "+v"(lofs));
#pragma unroll
        for (int i = 0; i < NT; ++i) {
          f4 acc = ld4(a.proj_b + G * H + 16 * i + 4 * g);
#pragma unroll
          for (int pu = 2; pu >= 0; --pu) {
            const bf8 w = pw[(pu * 3 * NT + i) * 64 + lofs];
#pragma unroll
            for (int ph = 2 - pu; ph >= 0; --ph) acc = MFMA_BF(w, pf[ph][0], acc);
          }
          if (valid) lds4w(tab + (int64_t)ll * ST + G * H + 16 * i + 4 * g, acc);
        }
      }
    }
    }   // B2, B3 as separate passes
#ifdef IGN_RES_STAMP
    IGN_STAMP(t_b);
    s_bw += t_b - t_a;
#endif
    __syncthreads();
#ifdef IGN_RES_STAMP
    IGN_STAMP(t_a);
    s_bb += t_a - t_b;
#endif
  }
#ifdef IGN_RES_STAMP
  if (lane == 0 && gph < 256) {
    unsigned long long* o = ign_res_stamps + 8 * (gph * kW + wave);
    o[0] = s_init; o[1] = s_aw; o[2] = s_ab; o[3] = s_bw; o[4] = s_bb; o[5] = n_at; o[6] = n_bt;
    o[7] = t_a - t_0;
  }
#endif
  // the final states leave the workgroup (the readout and ign_batch_state read them)
  if constexpr (!PG)   // PG: the path states are already there
    for (int64_t i = tid; i < P * (H / 4); i += 64 * kW) {
      const int64_t r = i / (H / 4);
      const int c4 = (int)(i - r * (H / 4));
      st4(a.path_state + (p0 + r) * H + 4 * c4, lds4(hP + r * SP + 4 * c4));
    }
  for (int64_t i = tid; i < L * (H / 4); i += 64 * kW) {
    const int64_t r = i / (H / 4);
    const int c4 = (int)(i - r * (H / 4));
    st4(a.link_state + (l0 + r) * H + 4 * c4, lds4(hL + r * SP + 4 * c4));
  }
}

hipError_t launch_resident_forward(const ResidentArgs& a, int n_graphs, size_t lds_bytes, bool path_global,
                                   hipStream_t st) {
  if (n_graphs == 0) return hipSuccess;
  static bool attr = false;
  if (!attr) {
    for (const void* k : {reinterpret_cast<const void*>(resident_forward_kernel<false>),
                          reinterpret_cast<const void*>(resident_forward_kernel<true>)}) {
      hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kResidentMaxDynLds);
      if (e != hipSuccess) return e;
    }
    attr = true;
  }
  if (lds_bytes > kResidentMaxDynLds) return hipErrorInvalidValue;
  if (path_global)
    hipLaunchKernelGGL(resident_forward_kernel<true>, dim3((unsigned)n_graphs), dim3(64 * kW), lds_bytes, st, a);
  else
    hipLaunchKernelGGL(resident_forward_kernel<false>, dim3((unsigned)n_graphs), dim3(64 * kW), lds_bytes, st, a);
  return hipGetLastError();
}
