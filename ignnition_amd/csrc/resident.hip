// resident.hip — the graph-resident forward for small graphs (RouteNet-shaped models).
//
// The batched kernels (seq_gru_h16, sum_gru_g32, sum_seg) run every MP over the whole batch: one
// launch per MP and iteration, states and projected tables in HBM / Infinity Cache between launches.
// Here one workgroup owns one graph for all T iterations of a model of this shape: one ordered MP
// into the "path" entity from S <= 2 source entities (RouteNet: links; Q-size: links and nodes,
// interleaved), and for each source entity a sum MP from the paths back to it.  The source entities'
// rows of the graph form one "union" row range (entity 0's rows, then entity 1's); the ordered MP's
// projected table has one row per union row plus the hole row.
//   LDS: path states [P][36] (or, for graphs whose paths do not fit, the batch's state buffer in
//        HBM / L2), union-row states [U][36], the projected table [U + 1][100] (the hole row last),
//        the sum MPs' CSR by union row (or, when it does not fit, read from L2), U's fp16 pieces;
//   per iteration: phase A, the ordered update (seq_gru_h16's tile loop over the graph's paths
//        sorted by length; projected rows and states from LDS), barrier, phase B, the sum updates
//        over all 16 waves: B1 the message sums (high in-degree rows: sum_seg_kernel's wave per
//        row; the others: sum_gru_g32's adds in message order, one lane per (row, float4 column)),
//        barrier, B2+B3 per union-row tile (at most two per wave): the split-bf16 GRU step with the
//        tile's own sum MP's weights, then the next iteration's projection of the new states.
// The arithmetic per row is that of the batched kernels: the same message order, pieces, products
// and gate formulas (iteration 0 projects with project_kernel's f32 MFMA, later iterations with
// sum_gru_g32's fused split-bf16 projection), so the predictions are the batched forward's bits and
// a graph's predictions do not depend on which path its batch took.  (The ordered update's tiles
// hold one graph's paths here; a tile's power-of-two scale only moves bits when a state lies
// outside [-1, 1] and its low fp16 piece goes subnormal -- tests/test_gpu_parity.py checks equality.)
// Only the final states leave the workgroup; the batched readout then runs on the path states.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>
#include <vector>

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
// a pointer read from a pointer array (the training form's versions and saves) is generic: its loads
// and stores would be flat_*, which count in both vmcnt and lgkmcnt and complete out of order, so
// the compiler waits for both counters to drain (every LDS read waits for the step's hs stores).  A
// round trip through the global address space lets the compiler issue them as global_*
__device__ __forceinline__ float* in_global(float* p) {
  return (float*)(__attribute__((address_space(1))) float*)p;
}
// the batched table row of local union row ll (source entity 0's rows, then entity 1's)
__device__ __forceinline__ int64_t tab_row(const ResidentArgs& a, int64_t ll, int64_t L0, int64_t s00, int64_t s10) {
  return ll >= L0 ? a.tab_off[1] + s10 + (ll - L0) : a.tab_off[0] + s00 + ll;
}
__device__ __forceinline__ void gst4(float* p, f4 v) { *(__attribute__((address_space(1))) f4*)p = v; }
// the path states: global memory (PG) or LDS
template <bool G> __device__ __forceinline__ f4 ldp4(const float* p) {
  if constexpr (G) return *(const __attribute__((address_space(1))) f4*)p;
  else return lds4(p);
}
template <bool G> __device__ __forceinline__ void stp4(float* p, f4 v) {
  if constexpr (G) *(__attribute__((address_space(1))) f4*)p = v;
  else lds4w(p, v);
}

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

// the ordered MP's projected row of a union-row state in the B layout (sum_gru_g32's fused
// projection: split-bf16 x6, the pieces of W' from L2), written to the LDS table row ll
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
                                                bool valid, int lane, int g, float* gsave = nullptr) {
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
      for (int t = 0; t < NT; ++t) {
        lds4w(tab + (int64_t)ll * ST + G * H + 16 * t + 4 * g, acc[G][t]);
        if (gsave) gst4(gsave + G * H + 16 * t + 4 * g, acc[G][t]);   // (the training form's saved table)
      }
  }
}

// one output half (16 columns, t) of sum_gru_g32's split-bf16 GRU step for a tile of 16 union rows:
// x.W and h.U piece products (x6) from the sum MP's pieces in L2, then the gates
__device__ __forceinline__ f4 gru_half(const void* Wbf, const void* Ubf, const float* bias, const bf8 (&xf)[3][1],
                                       const bf8 (&hf)[3][1], const f4 ho, int t, int lane, int g) {
  constexpr int H = 32, NT = 2;
  int lofs = lane + 64 * t;   // opaque: the fragment addresses stay inside the loop (as project_row)
  asm volatile("" : "+v"(lofs));
  const bf8* sW = static_cast<const bf8*>(Wbf);
  const bf8* sU = static_cast<const bf8*>(Ubf);
  const int u0 = 16 * t + 4 * g;
  f4 az = ld4(bias + 0 * H + u0), ar = ld4(bias + 1 * H + u0);
  f4 ax = ld4(bias + 2 * H + u0), ah = ld4(bias + 3 * H + u0);
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
}

}  // namespace

// PG: the path states stay in the batch's state buffer in HBM / L2 (rows of 32 floats) and the
// ordered MP's step codes are read from global memory: the form for graphs whose path states do
// not fit (synth50: 2 450 paths).  CL: the sum MPs' CSR (message rows) in LDS; else read from L2
// (Q-size synth50: its two sum MPs' 14 k messages do not fit beside the 250 union rows' table)
template <bool PG, bool CL, bool SAVE>
#ifdef IGN_RES_MIN_WAVES   // A/B: at least this many waves per SIMD (VGPR budget 512 / that)
__global__ __launch_bounds__(64 * kW, IGN_RES_MIN_WAVES) void resident_forward_kernel(ResidentArgs a) {
#else
__global__ __launch_bounds__(64 * kW) void resident_forward_kernel(ResidentArgs a) {
#endif
  static_assert(PG || !SAVE, "the training form keeps the path states in global memory (versions)");
  constexpr int H = 32, NT = 2, KS = 1, NF = 6 * NT * KS;   // U's fp16 pieces: 2 pieces x 3 gates x NT
  __shared__ h8 su[NF * 64];
  __shared__ float sbn[kW][H];
  __shared__ float sbias[H];
  __shared__ int sctr[2];   // phase A's tile counters (alternate iterations)
  extern __shared__ float dyn[];
  const int gph = a.gorder ? a.gorder[blockIdx.x] : (int)blockIdx.x;   // longest graphs first (LPT)
  const int64_t p0 = a.path_off[gph], P = a.path_off[gph + 1] - p0;
  const int64_t s00 = a.src_off[0][gph], L0 = a.src_off[0][gph + 1] - s00;
  const int64_t s10 = a.n_src > 1 ? a.src_off[1][gph] : 0;
  const int64_t L1 = a.n_src > 1 ? a.src_off[1][gph + 1] - s10 : 0;
  const int64_t U = L0 + L1;   // union rows: entity 0's, then entity 1's
  constexpr int SPP = PG ? H : SP;   // row stride of the path states
  float* hP = PG ? (SAVE ? in_global(a.path_ver[0]) : a.path_state) + p0 * H : dyn;   // (SAVE: per iteration below)
  float* hL = PG ? dyn : hP + P * SP;
  float* tab = hL + U * SP;
  int* smp = reinterpret_cast<int*>(tab + (U + 1) * ST);   // the sum MPs' CSR by local union row
  uint16_t* slo = reinterpret_cast<uint16_t*>(smp + U + 1);   // union-row order for the message sums
  uint16_t* sms_l = slo + ((U + 1) & ~1);
  const int64_t ms0 = a.lmsg_off[gph], M = a.lmsg_off[gph + 1] - ms0;
  uint16_t* scd_l = sms_l + (CL ? M : 0);   // the ordered MP's local step codes
  const int64_t cd0 = a.lcode_off[gph], NC = a.lcode_off[gph + 1] - cd0;
  const uint16_t* sms = CL ? sms_l : a.lmsg_src + ms0;   // LDS, or L2 (!CL)
  const uint16_t* scd = PG ? a.lcode + cd0 : scd_l;      // PG: read from global memory
  float* xs = tab;   // phase B's message sums [U][SP] alias the (consumed) projected table
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
  // GM:396-400: state_0 = [features | zeros] (SAVE: path_ver[0] holds it already)
  for (int64_t i = SAVE ? P * H : tid; i < P * H; i += 64 * kW) {
    const int64_t r = i / H;
    const int c = (int)(i - r * H);
    hP[r * SPP + c] = c < a.path_F ? a.path_feat[(p0 + r) * a.path_F + c] : 0.f;
  }
  for (int64_t i = tid; i < U * H; i += 64 * kW) {
    const int64_t r = i / H;
    const int c = (int)(i - r * H);
    const bool e1 = r >= L0;
    const int F = e1 ? a.src_F[1] : a.src_F[0];
    const float* f = e1 ? a.src_feat[1] + (s10 + r - L0) * F : a.src_feat[0] + (s00 + r) * F;
    hL[r * SP + c] = c < F ? f[c] : 0.f;
  }
  for (int i = tid; i < 3 * H; i += 64 * kW) tab[U * ST + i] = a.proj_b[i];   // the hole row: b' alone
  {
    const int64_t u0 = a.urow_off[gph];
    const int* gp = a.lmsg_ptr + u0 + gph;
    for (int64_t i = tid; i <= U; i += 64 * kW) smp[i] = gp[i];
    if constexpr (CL)
      for (int64_t i = tid; i < M; i += 64 * kW) sms_l[i] = a.lmsg_src[ms0 + i];
    for (int64_t i = tid; i < U; i += 64 * kW) slo[i] = a.lorder[u0 + i];
    if constexpr (!PG)
      for (int64_t i = tid; i < NC; i += 64 * kW) scd_l[i] = a.lcode[cd0 + i];
  }
  __syncthreads();
  const int64_t nut = (U + 15) / 16;   // union-row tiles of the projection
  // the first iteration's projected table
  for (int64_t k = wave; k < nut; k += kW) {
    const int64_t idx = 16 * k + j;
    const bool valid = idx < U;
    const int ll = valid ? (int)idx : 0;
    f4 h[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) h[t] = valid ? lds4(hL + (int64_t)ll * SP + 16 * t + 4 * g) : f4{0, 0, 0, 0};
    float* gs = nullptr;   // SAVE: the table of iteration 0, row of this union row
    if constexpr (SAVE)
      if (a.tab_save) gs = in_global(a.tab_save[0]) + tab_row(a, ll, L0, s00, s10) * 96;
    project_row_f32(a, h, tab, ll, valid, lane, g, gs);
  }
  if constexpr (SAVE)   // every saved table's hole row: the bias alone (one workgroup writes them)
    if (a.tab_save && gph == 0)
      for (int i = tid; i < a.T * 96; i += 64 * kW) in_global(a.tab_save[i / 96])[a.tab_hole * 96 + i % 96] = a.proj_b[i % 96];
  __syncthreads();
#ifdef IGN_RES_STAMP
  IGN_STAMP(t_a);
  s_init = t_a - t_0;
#endif

  const int64_t pt0 = a.ptile_off[gph], npt = (a.ptile_off[gph + 1] - pt0) / 16;
#ifdef IGN_RES_PRIO   // A/B: static priority for the second-dispatched half (MI355X_MICROARCH.md, item 4)
  if (wave >= kW / 2) __builtin_amdgcn_s_setprio(1);
#endif
  for (int it = 0; it < a.T; ++it) {
    // the path states this iteration reads (hPi) and writes (hPo): one buffer, or the versions
    const float* hPi = SAVE ? in_global(a.path_ver[it]) + p0 * H : hP;
    float* hPo = SAVE ? in_global(a.path_ver[it + 1]) + p0 * H : hP;
    float* hsv = SAVE ? in_global(a.hs_save[it]) : nullptr;
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
      const bool valid = hd[0] >= 0;   // tile padding: row -1 (a real path may have length 0)
      const int64_t rl = valid ? hd[0] : 0;
      const int cbase = hd[2];   // (an index, not a pointer: one VGPR live through the tile)
      f4 h[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) {
        const f4 v = ldp4<PG>(hPi + rl * SPP + 16 * t + 4 * g);
        h[t] = valid ? v : f4{0, 0, 0, 0};
      }
      // SAVE: the position's first hs_save row, the state before the sequence -- not saved: it is the
      // path version this iteration read, and the backward reads it there (as the final row, below)
      int hb = 0;
      if constexpr (SAVE) hb = a.hsb[pt0 + 16 * k + j];
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
#ifndef IGN_RES_ABL_MFMA
#pragma unroll
            for (int ph = 1; ph >= 0; --ph) {
              if (pu + ph > 1) continue;
#pragma unroll
              for (int G = 0; G < 3; ++G) acc[G][i] = MFMA_H(w[G], hf[ph][0], acc[G][i]);
            }
#else   // timing ablation (wrong results): no MFMAs, the state still flows into the gates
#pragma unroll
            for (int G = 0; G < 3; ++G) acc[G][i] += h[i] + __builtin_bit_cast(f4, w[G]);
#endif
          }
        const bool act = t < Lr;
#ifdef IGN_RES_ABL_GATE   // timing ablation (wrong results): one fma per element instead of the gates
#pragma unroll
        for (int i = 0; i < NT; ++i)
#pragma unroll
          for (int r = 0; r < 4; ++r)
            h[i][r] = fmaf(fmaf(acc[0][i][r], c, xx[0][i][r]), 1e-3f, fmaf(acc[2][i][r], c, xx[2][i][r]) * 1e-3f);
        (void)masked; (void)act;
        return;
#endif
        // the gates stage by stage across the lane's 8 elements (the same arithmetic as seq_gru_h16, so the
        // same bits): the exponentials of all 8, then the reciprocals, then the candidates; the compiler
        // otherwise chains each element's exp -> rcp through one register (phase A -2.4 %, stamps)
        float ez[8], er[8], zz[8], gg[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          ez[e] = __builtin_amdgcn_exp2f(fmaf(acc[0][e >> 2][e & 3], c, xx[0][e >> 2][e & 3]));
          er[e] = __builtin_amdgcn_exp2f(fmaf(acc[1][e >> 2][e & 3], c, xx[1][e >> 2][e & 3]));
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          zz[e] = rcpf_(1.0f + ez[e]);
          gg[e] = fmaf(rcpf_(fmaf(er[e], SS, SS)), acc[2][e >> 2][e & 3], xx[2][e >> 2][e & 3]);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int i = e >> 2, r = e & 3;
          const float n = S * tanh2_(gg[e]);
          const float hn = n + zz[e] * (h[i][r] - n);
          if constexpr (decltype(masked)::value) h[i][r] = act ? hn : h[i][r];
          else h[i][r] = hn;
        }

      };
      // the tile's shortest sequence: its last real path's (tiles are padded at the graph's end)
      const int Lmin = __builtin_amdgcn_readlane(Lr, (int)min<int64_t>(15, P - 1 - 16 * k));
      for (int t = 0;;) {
        if (t < Lmin) step(t, x, std::false_type{});
        else step(t, x, std::true_type{});
        if constexpr (SAVE) {   // the state after step t, but the last (seq_gru_h16<SAVE>'s save less
                                // its final row: the next path version, which the backward never reads)
          if (t + 1 < Lr) {
#pragma unroll
            for (int i = 0; i < NT; ++i) gst4(hsv + (int64_t)(hb + t + 1) * H + 16 * i + 4 * g, h[i] * iS);
          }
        }
        if (++t >= Lmax) break;
        load_x(code, x);
        code = scd[cbase + t + 1];
      }
      if (valid) {
#pragma unroll
        for (int t = 0; t < NT; ++t) stp4<PG>(hPo + rl * SPP + 16 * t + 4 * g, h[t] * iS);
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
    // ---- phase B: the sum updates ----
    // B1: the message sums.  Rows with >= 64 messages (lorder's first nseg, per destination as the
    // batched forward decides): sum_seg_kernel<32, 4>'s order, one wave per row -- lane (c, q) adds
    // messages q, q + 8, ... of the row (columns 4c .. 4c + 3), four rows in flight, then the eight
    // partial sums pairwise across lanes (xor 32, 16, 8).  The others: sum_gru_g32's lane walk, one
    // lane per (row, float4 column) adding in message order from zero, long chains first.
    const int nseg = a.seg_on ? a.lnseg[gph] : 0;
    for (int k = wave; k < nseg; k += kW) {
      const int ll = slo[k];
      int lo = lane;   // opaque: the lane's column pointer stays inside the loop (no spill, as project_row)
      asm volatile("" : "+v"(lo));
      const int c = lo & 7, q = lo >> 3;
      const int m0 = smp[ll], m1 = smp[ll + 1];
      const int last = m1 > m0 ? m1 - 1 : m0;
      const float* hp = hPo + 4 * c;
      f4 acc = {0, 0, 0, 0};
      int cc[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = m0 + 8 * u + q;
        cc[u] = m1 > m0 ? sms[i < last ? i : last] : 0;
      }
      for (int m = m0; m < m1; m += 32) {
        f4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = ldp4<PG>(hp + cc[u] * SPP);
#pragma unroll
        for (int u = 0; u < 4; ++u) {   // the next round's rows, clamped into the range
          const int i = m + 8 * (4 + u) + q;
          cc[u] = sms[i < last ? i : last];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const bool on = m + 8 * u + q < m1;
          const f4 s = acc + v[u];
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[e] = on ? s[e] : acc[e];
        }
      }
#pragma unroll
      for (int o = 32; o >= 8; o >>= 1)
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] += __shfl_xor(acc[e], o);
      if (q == 0) lds4w(xs + ll * SP + 4 * c, acc);
    }
    int tlw = tid;   // opaque (as above)
    asm volatile("" : "+v"(tlw));
    for (int64_t i = (int64_t)nseg * 8 + tlw; i < U * (H / 4); i += 64 * kW) {
      const int64_t ll = slo[i >> 3];   // rows by message count, descending: the long chains first
      const int c4 = (int)(i & 7);
      const int m0 = smp[ll], m1 = smp[ll + 1];
      const float* hp = hPo + 4 * c4;
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
          for (int u = 0; u < 16; ++u) v[u] = ldp4<PG>(hp + rr[u] * SPP);
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
        for (int u = 0; u < 8; ++u) v[u] = ldp4<PG>(hp + rr[u] * SPP);
#pragma unroll
        for (int u = 0; u < 8; ++u) x = x + v[u];
      }
      for (; m < m1; ++m) x = x + ldp4<PG>(hp + sms[m] * SPP);
      lds4w(xs + ll * SP + 4 * c4, x);
      if constexpr (SAVE) {   // sum_gru_g32's x_save, by the entity's global row
        const bool e1 = ll >= L0;
        gst4((e1 ? a.x_save[1][it] + (s10 + ll - L0) * H : a.x_save[0][it] + (s00 + ll) * H) + 4 * c4, x);
      }
    }
    __syncthreads();
#ifdef IGN_RES_STAMP
    {   // B1's end (after its barrier): n_at accumulates B1
      unsigned long long t_c;
      IGN_STAMP(t_c);
      n_at += t_c - t_a;
    }
#endif
    // B2 + B3, one wave per union-row tile (tiles w and w + 16; a tile holds one entity's rows):
    // the GRU step of both column halves with the tile's own sum MP's weights, the new states, then
    // the next iteration's projected rows of the tile.  Each wave reads its tiles' message sums into
    // registers before a barrier: they alias table rows that other waves' projections overwrite (a
    // tile's states are only written by its own wave: read after the barrier)
    const bool last = it + 1 == a.T;
    const int nt0 = (int)((L0 + 15) / 16);
    const int ntt = nt0 + (int)((L1 + 15) / 16);
    f4 xr[2][2];
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int k = wave + kW * q;
      const bool act = k < ntt;   // wave-uniform
      const bool e1 = k >= nt0;
      const int64_t idx = e1 ? L0 + 16 * (k - nt0) + j : 16 * k + j;
      const bool valid = act && idx < (e1 ? U : L0);
      const int ll = valid ? (int)idx : 0;
#pragma unroll
      for (int c = 0; c < 2; ++c) xr[q][c] = act ? lds4(xs + (int64_t)ll * SP + 16 * c + 4 * g) : f4{0, 0, 0, 0};
    }
    __syncthreads();
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const int k = wave + kW * q;
      if (k >= ntt) break;   // wave-uniform
      const int e1 = k >= nt0;
      const int64_t idx = e1 ? L0 + 16 * (k - nt0) + j : 16 * k + j;
      const bool valid = idx < (e1 ? U : L0);
      const int ll = valid ? (int)idx : 0;
      f4 hr[2];
#pragma unroll
      for (int c = 0; c < 2; ++c) hr[c] = lds4(hL + (int64_t)ll * SP + 16 * c + 4 * g);
      bf8 xf[3][1], hf[3][1];
      split_frags1(xr[q], xf);
      split_frags1(hr, hf);
      const void* W = e1 ? a.sWbf[1] : a.sWbf[0];
      const void* Ub = e1 ? a.sUbf[1] : a.sUbf[0];
      const float* bias = e1 ? a.sum_bias[1] : a.sum_bias[0];
      f4 hn[NT];
#pragma unroll
      for (int t = 0; t < NT; ++t) hn[t] = gru_half(W, Ub, bias, xf, hf, hr[t], t, lane, g);
      if (valid) {
#pragma unroll
        for (int t = 0; t < NT; ++t) lds4w(hL + (int64_t)ll * SP + 16 * t + 4 * g, hn[t]);
        if constexpr (SAVE) {   // the entity's next version
          float* o = in_global(e1 ? a.src_ver[1][it + 1] + (s10 + ll - L0) * H : a.src_ver[0][it + 1] + (s00 + ll) * H);
#pragma unroll
          for (int t = 0; t < NT; ++t) gst4(o + 16 * t + 4 * g, hn[t]);
        }
      }
      if (!last) {
        if constexpr (SAVE) {   // build_table's projection (and the next iteration's saved table)
          float* gs = nullptr;
          if (a.tab_save && it + 1 < a.T) gs = in_global(a.tab_save[it + 1]) + tab_row(a, ll, L0, s00, s10) * 96;
          project_row_f32(a, hn, tab, ll, valid, lane, g, gs);
        }
        else project_row(a, hn, tab, ll, valid, lane, g);
      }
    }
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
  // the final states leave the workgroup (the readout and ign_batch_state read them; SAVE: the
  // versions hold every state already)
  if constexpr (SAVE) return;
  if constexpr (!PG)   // PG: the path states are already there
    for (int64_t i = tid; i < P * (H / 4); i += 64 * kW) {
      const int64_t r = i / (H / 4);
      const int c4 = (int)(i - r * (H / 4));
      st4(a.path_state + (p0 + r) * H + 4 * c4, lds4(hP + r * SP + 4 * c4));
    }
  for (int64_t i = tid; i < U * (H / 4); i += 64 * kW) {
    const int64_t r = i / (H / 4);
    const int c4 = (int)(i - r * (H / 4));
    float* o = r >= L0 ? a.src_state[1] + (s10 + r - L0) * H : a.src_state[0] + (s00 + r) * H;
    st4(o + 4 * c4, lds4(hL + r * SP + 4 * c4));
  }
}

// once per device, before any launch or capture (resident_batch calls it)
hipError_t resident_prepare_device() {
  static std::mutex mu;
  static std::vector<char> done;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  std::lock_guard<std::mutex> lk(mu);
  if ((int)done.size() <= dev) done.resize(dev + 1, 0);
  if (done[dev]) return hipSuccess;
  for (const void* k : {reinterpret_cast<const void*>(resident_forward_kernel<false, true, false>),
                        reinterpret_cast<const void*>(resident_forward_kernel<true, true, false>),
                        reinterpret_cast<const void*>(resident_forward_kernel<true, false, false>),
                        reinterpret_cast<const void*>(resident_forward_kernel<true, true, true>),
                        reinterpret_cast<const void*>(resident_forward_kernel<true, false, true>)}) {
    e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kResidentMaxDynLds);
    if (e != hipSuccess) return e;
  }
  done[dev] = 1;
  return hipSuccess;
}

hipError_t launch_resident_forward(const ResidentArgs& a, int n_graphs, size_t lds_bytes, int form, bool save,
                                   hipStream_t st) {
  if (n_graphs == 0) return hipSuccess;
  if (lds_bytes > kResidentMaxDynLds || a.n_src < 1 || a.n_src > kResidentMaxSrc) return hipErrorInvalidValue;
  if (save && (form == IGN_RES_ALL_LDS || !a.path_ver || !a.hs_save || !a.hsb)) return hipErrorInvalidValue;
  const dim3 grid((unsigned)n_graphs), block(64 * kW);
  if (save && form == IGN_RES_PATH_CSR_GLOBAL)
    hipLaunchKernelGGL((resident_forward_kernel<true, false, true>), grid, block, lds_bytes, st, a);
  else if (save)
    hipLaunchKernelGGL((resident_forward_kernel<true, true, true>), grid, block, lds_bytes, st, a);
  else if (form == IGN_RES_PATH_CSR_GLOBAL)
    hipLaunchKernelGGL((resident_forward_kernel<true, false, false>), grid, block, lds_bytes, st, a);
  else if (form == IGN_RES_PATH_GLOBAL)
    hipLaunchKernelGGL((resident_forward_kernel<true, true, false>), grid, block, lds_bytes, st, a);
  else if (form == IGN_RES_ALL_LDS)
    hipLaunchKernelGGL((resident_forward_kernel<false, true, false>), grid, block, lds_bytes, st, a);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}
