// ORACLE (test infrastructure and bench.py's second CPU line only) — C++/OpenMP restatement of
// ComnetModel.call (code/utils/generate_model.py:384-658, "GM") for the models the benchmark
// configurations use: sum / ordered / interleave / concat (axis 1 and 2) aggregation, the
// Keras GRU update and the predict Dense stack.  Nothing under ignnition_amd/ links or loads it;
// the product path has no CPU execution.
//
// It reads the engine's own input structures (include/ignmp.h: the lowered plan and one batch
// of graphs) and the parameters in Keras layout, and computes graph by graph exactly what the
// TF op sequence computes, in float32 like TF on the CPU (the bench line) or in float64 (the
// checker of the engine's full-size outputs):
//   hidden states   AUX:146-159  [features | zeros]
//   per MP          GM:423-543   messages = source states gathered per edge (GM:432); position of
//                                a message = the previous sources' per-graph max(seq)+1 plus seq
//                                (GM:533), or the interleave index of that slot (AUX:432-439), or
//                                seq for the axis-2 concat (AUX:443-456); duplicates add
//                                (scatter_nd, GM:490); final_len = the per-destination count
//                                (GM:481, 505/519/543; axis 2: the first source's)
//   sum             AUX:254-262  x = sum of the destination's messages; one GRU step (AUX:752-765)
//   sorted          AUX:767-796  x_t = the sum at position t, t < final_len, GRU over t; a mask
//                                narrower than the padded length raises like K.rnn
//   GRU             Keras GRUCell v2: z, r, h column blocks, reset_after=True:
//                                z = sig(xWz + bz + hUz + b'z), r = sig(...),
//                                hh = tanh(xWh + bh + r (hUh + b'h)), h' = z h + (1 - z) hh
//   readout         GM:611-629   concat of the predict inputs (entity states), Dense stack
// Parallel over graphs (each graph is independent, GM:712-724) or, for one large graph, over
// the destinations of each MP.
#include <omp.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../include/ignmp.h"

namespace {

thread_local char g_err[512];

int err(int code, const char* msg) {
  snprintf(g_err, sizeof g_err, "%s", msg);
  return code;
}

template <typename T>
inline T act(T x, int a) {
  const T lam = T(1.0507009873554805), alpha = T(1.6732632423543772);
  switch (a) {
    case IGN_ACT_RELU: return x > T(0) ? x : T(0);
    case IGN_ACT_SELU:   // exp of min(x, 0): both arms stay finite (-ffast-math)
      return x > T(0) ? lam * x : lam * alpha * (std::exp(std::min(x, T(0))) - T(1));
    case IGN_ACT_SIGMOID: return T(1) / (T(1) + std::exp(-std::min(T(80), std::max(T(-80), x))));
    case IGN_ACT_TANH: return std::tanh(x);
    default: return x;
  }
}

// act over a row, the switch hoisted so that each arm vectorises (libmvec expf under -ffast-math)
template <typename T>
void act_row(T* __restrict__ x, int n, int a) {
  switch (a) {
    case IGN_ACT_RELU:
      for (int j = 0; j < n; ++j) x[j] = act(x[j], IGN_ACT_RELU);
      break;
    case IGN_ACT_SELU:
      for (int j = 0; j < n; ++j) x[j] = act(x[j], IGN_ACT_SELU);
      break;
    case IGN_ACT_SIGMOID:
      for (int j = 0; j < n; ++j) x[j] = act(x[j], IGN_ACT_SIGMOID);
      break;
    case IGN_ACT_TANH:
      for (int j = 0; j < n; ++j) x[j] = act(x[j], IGN_ACT_TANH);
      break;
    default:
      break;
  }
}

struct Cell {
  int din, H;
  const float *W, *U, *b;   // [din][3H], [H][3H], [2][3H]
};

// R Keras GRU steps of independent rows: out[r] = GRU(x[r], h[r]), for the compile-time widths of
// the example models.
template <int DIN, int H, typename T, int R>
void gru_rows_t(const Cell& c, const T* const* x, const T* const* h, T* const* out) {
  constexpr int H3 = 3 * H, VL = 32 / sizeof(T), NV = 3, JB = NV * VL;
  static_assert(H3 % JB == 0, "column blocks");
  typedef T V __attribute__((vector_size(32)));
  T mx[R][H3], mh[R][H3];
  // R rows x NV vectors of accumulators (12 AVX2 registers at R = 4): each weight vector loaded
  // from L1/L2 feeds R FMAs (the 2 x 64 x 192 weights of H = 64 do not fit L1)
  auto block = [&](const T* const* in, const float* __restrict__ M, const float* bias, int K, T (*dst)[H3],
                   int j0) __attribute__((always_inline)) {
    V a[R][NV];
    for (int v = 0; v < NV; ++v) {
      V bv;
      for (int l = 0; l < VL; ++l) bv[l] = bias[j0 + v * VL + l];
      for (int r = 0; r < R; ++r) a[r][v] = bv;
    }
    for (int k = 0; k < K; ++k) {
      const float* w = M + (int64_t)k * H3 + j0;
      V wv[NV];
      for (int v = 0; v < NV; ++v)
        for (int l = 0; l < VL; ++l) wv[v][l] = w[v * VL + l];
      for (int r = 0; r < R; ++r) {
        const T xv = in[r][k];
        for (int v = 0; v < NV; ++v) a[r][v] += xv * wv[v];
      }
    }
    for (int r = 0; r < R; ++r) memcpy(&dst[r][j0], a[r], sizeof a[r]);
  };
  for (int j0 = 0; j0 < H3; j0 += JB) {
    block(x, c.W, c.b, DIN, mx, j0);
    block(h, c.U, c.b + H3, H, mh, j0);
  }
  for (int r = 0; r < R; ++r) {
    T* __restrict__ zx = mx[r];
    T* __restrict__ zh = mh[r];
    // z | r; the argument is clamped to +-80 so that no exp overflows (-ffast-math assumes finite
    // values; sigmoid is saturated there: exp(-80) is below float32's resolution of 1)
    for (int j = 0; j < 2 * H; ++j) zx[j] = T(1) / (T(1) + std::exp(-std::min(T(80), std::max(T(-80), zx[j] + zh[j]))));
    for (int j = 0; j < H; ++j) zh[j] = std::tanh(zx[2 * H + j] + zx[H + j] * zh[2 * H + j]);
    for (int j = 0; j < H; ++j) out[r][j] = zx[j] * h[r][j] + (T(1) - zx[j]) * zh[j];
  }
}

// one Keras GRU step for one row: out = GRU(x, h).  The loops are written so that the compiler
// vectorises them (libmvec expf / tanhf under -ffast-math); this is the timed CPU line.
template <int DIN, int H, typename T>
void gru_step_t(const Cell& c, const T* x, const T* h, T* out) {
  gru_rows_t<DIN, H, T, 1>(c, &x, &h, &out);
}

template <typename T>
void gru_step_any(const Cell& c, const T* __restrict__ x, const T* __restrict__ h, T* __restrict__ out,
                  T* __restrict__ mx, T* __restrict__ mh) {
  const int H3 = 3 * c.H, H = c.H;
  for (int j = 0; j < H3; ++j) {
    mx[j] = c.b[j];
    mh[j] = c.b[H3 + j];
  }
  for (int k = 0; k < c.din; ++k) {
    const T xv = x[k];
    const float* __restrict__ w = c.W + (int64_t)k * H3;
    for (int j = 0; j < H3; ++j) mx[j] += xv * w[j];
  }
  for (int k = 0; k < H; ++k) {
    const T hv = h[k];
    const float* __restrict__ u = c.U + (int64_t)k * H3;
    for (int j = 0; j < H3; ++j) mh[j] += hv * u[j];
  }
  // z | r; the argument is clamped to +-80 so that no exp overflows (-ffast-math assumes finite
  // values; sigmoid is saturated there: exp(-80) is below float32's resolution of 1)
  for (int j = 0; j < 2 * H; ++j) mx[j] = T(1) / (T(1) + std::exp(-std::min(T(80), std::max(T(-80), mx[j] + mh[j]))));
  for (int j = 0; j < H; ++j) mh[j] = std::tanh(mx[2 * H + j] + mx[H + j] * mh[2 * H + j]);
  for (int j = 0; j < H; ++j) out[j] = mx[j] * h[j] + (T(1) - mx[j]) * mh[j];
}

template <typename T>
inline void gru_step(const Cell& c, const T* x, const T* h, T* out, T* mx, T* mh) {
  if (c.din == 32 && c.H == 32) return gru_step_t<32, 32, T>(c, x, h, out);
  if (c.din == 64 && c.H == 64) return gru_step_t<64, 64, T>(c, x, h, out);
  if (c.din == 16 && c.H == 16) return gru_step_t<16, 16, T>(c, x, h, out);
  gru_step_any<T>(c, x, h, out, mx, mh);
}

// four rows at once where a compile-time width exists (false: the caller steps them one by one)
template <typename T>
inline bool gru_rows4(const Cell& c, const T* const* x, const T* const* h, T* const* out) {
  if (c.din == 32 && c.H == 32) return gru_rows_t<32, 32, T, 4>(c, x, h, out), true;
  if (c.din == 64 && c.H == 64) return gru_rows_t<64, 64, T, 4>(c, x, h, out), true;
  if (c.din == 16 && c.H == 16) return gru_rows_t<16, 16, T, 4>(c, x, h, out), true;
  return false;
}

struct Graph {            // graph-local views of one graph of the batch
  std::vector<int64_t> n;                 // rows per entity
  std::vector<const float*> feat;         // per entity
  std::vector<const int64_t*> src, dst, seq;
  std::vector<int64_t> ne;                // edges per adjacency
  std::vector<const int64_t*> il;
  std::vector<int64_t> nil;
};

struct Model {
  const ign_plan_desc* p;
  std::vector<Cell> cells;
  struct Layer {
    int in, out, act;
    const float *W, *b;
  };
  std::vector<Layer> dense;
};

// The forward of one graph; par: parallelise over the destinations of each MP (one big graph)
template <typename T>
int graph_forward(const Model& m, const Graph& g, float* out, bool par, std::string& msg) {
  const ign_plan_desc* p = m.p;
  const int E = p->num_entities;
  std::vector<std::vector<T>> S(E), S2(E);
  for (int e = 0; e < E; ++e) {
    const int H = p->entities[e].hidden_dim, F = p->entities[e].feature_total;
    S[e].assign(g.n[e] * H, 0.f);
    for (int64_t r = 0; r < g.n[e]; ++r)
      for (int f = 0; f < F; ++f) S[e][r * H + f] = g.feat[e][r * F + f];
  }
  // Per MP, the messages of each destination (CSR, message order within a destination) and the
  // sequence lengths: they depend on the graph only, so they are built once, not per iteration
  // (serial work that dominated one large graph's time under OpenMP).
  struct Msg { int64_t pos; int s; int64_t row; };
  struct Prep {
    std::vector<int64_t> ptr, flen;
    std::vector<Msg> msgs;
  };
  std::vector<Prep> preps(p->num_mps);
  for (int mi = 0; mi < p->num_mps; ++mi) {
    const ign_mp_desc& mp = p->mps[mi];
    const int dst = mp.dst_entity, NS = mp.num_sources;
    const int64_t ND = g.n[dst];
    const bool sorted = mp.aggregation != IGN_AGGR_SUM;
    const bool axis2 = mp.aggregation == IGN_AGGR_CONCAT && mp.concat_axis == 2;
    std::vector<int64_t> lmax(NS, 0);
    std::vector<int64_t>& flen = preps[mi].flen;
    flen.assign(ND, 0);
    int64_t total = 0;
    std::vector<int64_t> ilflat;
    for (int s = 0; s < NS; ++s) {
      const int a = mp.sources[s].adjacency;
      int64_t mx = -1;
      for (int64_t k = 0; k < g.ne[a]; ++k) mx = std::max(mx, g.seq[a][k]);
      if (mx < 0) { msg = "adjacency with no edges (reduce_max of an empty seq, GM:484)"; return IGN_ERR_INVALID; }
      lmax[s] = mx + 1;
      total += lmax[s];
      if (mp.aggregation == IGN_AGGR_INTERLEAVE) {
        const int il = mp.sources[s].interleave;
        ilflat.insert(ilflat.end(), g.il[il], g.il[il] + g.nil[il]);
      }
    }
    if (axis2) total = lmax[0];
    // messages by destination (CSR, message order within a destination)
    std::vector<int64_t>& ptr = preps[mi].ptr;
    ptr.assign(ND + 1, 0);
    for (int s = 0; s < NS; ++s) {
      const int a = mp.sources[s].adjacency, se = mp.sources[s].entity;
      for (int64_t k = 0; k < g.ne[a]; ++k) {
        const int64_t si = g.src[a][k], di = g.dst[a][k];
        if (si < 0 || si >= g.n[se] || di < 0 || di >= ND) { msg = "index out of range (gather, GM:432)"; return IGN_ERR_INVALID; }
        ptr[di + 1]++;
      }
    }
    for (int64_t r = 0; r < ND; ++r) ptr[r + 1] += ptr[r];
    std::vector<Msg>& msgs = preps[mi].msgs;
    msgs.resize(ptr[ND]);
    std::vector<int64_t> fill(ptr.begin(), ptr.end() - 1);
    int64_t off = 0;
    if (mp.aggregation == IGN_AGGR_INTERLEAVE && (int64_t)ilflat.size() != total) {
      msg = "interleave indices do not cover the slots (AUX:435)";
      return IGN_ERR_INVALID;
    }
    for (int s = 0; s < NS; ++s) {
      const int a = mp.sources[s].adjacency;
      for (int64_t k = 0; k < g.ne[a]; ++k) {
        const int64_t si = g.src[a][k], di = g.dst[a][k];
        int64_t pos = axis2 ? g.seq[a][k] : off + g.seq[a][k];
        if (mp.aggregation == IGN_AGGR_INTERLEAVE) {
          pos = ilflat[pos];
          if (pos < 0 || pos >= total) { msg = "interleave index out of range (AUX:435)"; return IGN_ERR_INVALID; }
        }
        msgs[fill[di]++] = {pos, s, si};
        if (!axis2 || s == 0) flen[di]++;
      }
      off += lmax[s];
    }
    if (sorted && ND) {
      int64_t mxl = 0;
      for (int64_t d = 0; d < ND; ++d) {
        if (flen[d] == 0) { msg = "a destination receives no message (gather_nd -1, AUX:793-795)"; return IGN_ERR_INVALID; }
        if (flen[d] > total) { msg = "final_len beyond the padded length (AUX:793-795)"; return IGN_ERR_INVALID; }
        mxl = std::max(mxl, flen[d]);
      }
      if (mxl < total) { msg = "sequence_mask(final_len) narrower than the padded sequence (AUX:785-790)"; return IGN_ERR_INVALID; }
    }
  }
  for (int it = 0; it < p->num_iterations; ++it) {
    for (int mi = 0; mi < p->num_mps; ++mi) {
      const ign_mp_desc& mp = p->mps[mi];
      const Cell& c = m.cells[mp.cell];
      const int dst = mp.dst_entity, H = c.H;
      const int64_t ND = g.n[dst];
      const bool sorted = mp.aggregation != IGN_AGGR_SUM;
      const bool axis2 = mp.aggregation == IGN_AGGR_CONCAT && mp.concat_axis == 2;
      const std::vector<int64_t>& ptr = preps[mi].ptr;
      const std::vector<int64_t>& flen = preps[mi].flen;
      const std::vector<Msg>& msgs = preps[mi].msgs;
      std::vector<T>& out_s = S2[dst];
      out_s.assign(ND * H, T(0));
      const int DIN = c.din;
      auto run = [&](int64_t d, std::vector<T>& x, std::vector<T>& h, std::vector<T>& hn,
                     std::vector<T>& mx, std::vector<T>& mh) {
        const T* h0 = S[dst].data() + d * H;
        if (!sorted) {
          std::fill(x.begin(), x.end(), T(0));
          for (int64_t i = ptr[d]; i < ptr[d + 1]; ++i) {
            const Msg& q = msgs[i];
            const int se = mp.sources[q.s].entity;
            const T* v = S[se].data() + q.row * p->entities[se].hidden_dim;
            for (int k = 0; k < DIN; ++k) x[k] += v[k];
          }
          gru_step(c, x.data(), h0, out_s.data() + d * H, mx.data(), mh.data());
          return;
        }
        std::copy(h0, h0 + H, h.begin());
        for (int64_t t = 0; t < flen[d]; ++t) {
          std::fill(x.begin(), x.end(), T(0));
          for (int64_t i = ptr[d]; i < ptr[d + 1]; ++i) {
            const Msg& q = msgs[i];
            if (q.pos != t) continue;
            const int se = mp.sources[q.s].entity;
            const int w = p->entities[se].hidden_dim;
            int col = 0;
            if (axis2)
              for (int s2 = 0; s2 < q.s; ++s2) col += p->entities[mp.sources[s2].entity].hidden_dim;
            const T* v = S[se].data() + q.row * w;
            for (int k = 0; k < w; ++k) x[col + k] += v[k];
          }
          gru_step(c, x.data(), h.data(), hn.data(), mx.data(), mh.data());
          std::swap(h, hn);
        }
        std::copy(h.begin(), h.end(), out_s.begin() + d * H);
      };
      // sum MPs: four destinations per GRU call where a compile-time width exists (gru_rows4)
      auto run4 = [&](int64_t d0, std::vector<T>& x4, std::vector<T>& h, std::vector<T>& hn,
                      std::vector<T>& mx, std::vector<T>& mh) {
        if (sorted || d0 + 4 > ND) {
          for (int64_t d = d0; d < std::min(d0 + 4, ND); ++d) run(d, x4, h, hn, mx, mh);
          return;
        }
        std::fill(x4.begin(), x4.end(), T(0));
        const T* xs[4];
        const T* hs[4];
        T* os[4];
        for (int r = 0; r < 4; ++r) {
          const int64_t d = d0 + r;
          T* x = x4.data() + (size_t)r * DIN;
          for (int64_t i = ptr[d]; i < ptr[d + 1]; ++i) {
            const Msg& q = msgs[i];
            const int se = mp.sources[q.s].entity;
            const T* v = S[se].data() + q.row * p->entities[se].hidden_dim;
            for (int k = 0; k < DIN; ++k) x[k] += v[k];
          }
          xs[r] = x;
          hs[r] = S[dst].data() + d * H;
          os[r] = out_s.data() + d * H;
        }
        if (!gru_rows4(c, xs, hs, os))
          for (int r = 0; r < 4; ++r) gru_step(c, xs[r], hs[r], os[r], mx.data(), mh.data());
      };
      const int64_t nblk = (ND + 3) / 4;
      if (par) {
#pragma omp parallel
        {
          std::vector<T> x4(4 * DIN), h(H), hn(H), mx(3 * H), mh(3 * H);
#pragma omp for schedule(dynamic, 16)
          for (int64_t b = 0; b < nblk; ++b) run4(4 * b, x4, h, hn, mx, mh);
        }
      } else {
        std::vector<T> x4(4 * DIN), h(H), hn(H), mx(3 * H), mh(3 * H);
        for (int64_t b = 0; b < nblk; ++b) run4(4 * b, x4, h, hn, mx, mh);
      }
      std::swap(S[dst], S2[dst]);   // GM:602: the destination's state is overwritten
    }
  }
  // readout: the predict inputs concatenated on axis 1, then the Dense stack (GM:611-629)
  const int64_t R = g.n[p->readout_inputs[0]];
  int width = 0;
  for (int i = 0; i < p->num_readout_inputs; ++i) width += p->entities[p->readout_inputs[i]].hidden_dim;
  // RB rows of the readout at a time (rows are independent; a block reuses each weight row it
  // loads RB times, where one row at a time streamed the 256x256 layer from L2 per row); one large
  // graph splits the blocks over the threads in static chunks
  constexpr int RB = 3, CB = 32;   // 12 AVX2 accumulators (float)
  int maxw = width;
  for (const auto& L : m.dense) maxw = std::max(maxw, L.out);
  auto readout_rows = [&](int64_t r0, std::vector<T>& a, std::vector<T>& b2) {
    const int nr = (int)std::min<int64_t>(RB, R - r0);
    a.assign((size_t)RB * maxw, T(0));
    b2.assign((size_t)RB * maxw, T(0));
    for (int i = 0; i < nr; ++i) {
      int col = 0;
      for (int q = 0; q < p->num_readout_inputs; ++q) {
        const int e = p->readout_inputs[q], H = p->entities[e].hidden_dim;
        std::copy(S[e].begin() + (r0 + i) * H, S[e].begin() + (r0 + i + 1) * H, a.begin() + (size_t)i * maxw + col);
        col += H;
      }
    }
    T* cur = a.data();
    T* nxt = b2.data();
    int width_out = width;
    for (const auto& L : m.dense) {
      for (int j0 = 0; j0 < L.out; j0 += CB) {   // CB output columns of RB rows (register-resident)
        const int nj = std::min(CB, L.out - j0);
        T acc[RB][CB];
        for (int i = 0; i < RB; ++i)
          for (int j = 0; j < CB; ++j) acc[i][j] = j < nj && L.b ? T(L.b[j0 + j]) : T(0);
        if (nj == CB) {
          for (int k = 0; k < L.in; ++k) {
            const float* __restrict__ w = L.W + (int64_t)k * L.out + j0;
            for (int i = 0; i < RB; ++i) {
              const T v = cur[(size_t)i * maxw + k];
              for (int j = 0; j < CB; ++j) acc[i][j] += v * w[j];
            }
          }
        } else {
          for (int k = 0; k < L.in; ++k) {
            const float* w = L.W + (int64_t)k * L.out + j0;
            for (int i = 0; i < RB; ++i) {
              const T v = cur[(size_t)i * maxw + k];
              for (int j = 0; j < nj; ++j) acc[i][j] += v * w[j];
            }
          }
        }
        for (int i = 0; i < RB; ++i)
          for (int j = 0; j < nj; ++j) nxt[(size_t)i * maxw + j0 + j] = acc[i][j];
      }
      for (int i = 0; i < RB; ++i) act_row(nxt + (size_t)i * maxw, L.out, L.act);
      std::swap(cur, nxt);
      width_out = L.out;
    }
    for (int i = 0; i < nr; ++i)
      for (int j = 0; j < width_out; ++j) out[(r0 + i) * (int64_t)width_out + j] = (float)cur[(size_t)i * maxw + j];
  };
  const int64_t nblk = (R + RB - 1) / RB;
  if (par) {
#pragma omp parallel
    {
      std::vector<T> a, b2;
#pragma omp for schedule(static)
      for (int64_t bI = 0; bI < nblk; ++bI) readout_rows(bI * RB, a, b2);
    }
  } else {
    std::vector<T> a, b2;
    for (int64_t bI = 0; bI < nblk; ++bI) readout_rows(bI * RB, a, b2);
  }
  return IGN_OK;
}

}  // namespace

extern "C" {

const char* ign_oracle_last_error(void) { return g_err; }

// params: the parameter tensors in MPPlan.param_specs order (Keras layout), n_params of them.
// out: the predictions of every graph, concatenated (model_fn's flattened order, GM:712-724).
// precision: 0 = float32 (TF's arithmetic on the CPU; the bench line), 1 = float64 (the checker)
int ign_oracle_forward(const ign_plan_desc* p, const ign_batch_desc* d, const float* const* params, int32_t n_params,
                       float* out, int32_t threads, int32_t precision) {
  if (!p || !d || !params || !out) return err(IGN_ERR_INVALID, "null argument");
  if (d->index_bytes == 4) return err(IGN_ERR_UNSUPPORTED, "oracle: int32 index arrays (ABI 13) are not read here");
  if (p->num_readout_ops) return err(IGN_ERR_UNSUPPORTED, "oracle: readout operations before predict are not restated in C++");
  if (p->num_readout_inputs < 1) return err(IGN_ERR_INVALID, "no predict inputs");
  Model m;
  m.p = p;
  int k = 0;
  for (int c = 0; c < p->num_cells; ++c) {
    if (k + 3 > n_params) return err(IGN_ERR_INVALID, "too few parameter tensors");
    m.cells.push_back({p->cells[c].input_dim, p->cells[c].units, params[k], params[k + 1], params[k + 2]});
    k += 3;
  }
  for (int i = 0; i < p->num_mps; ++i) {
    const ign_mp_desc& mp = p->mps[i];
    if (mp.aggregation == IGN_AGGR_ATTENTION || mp.aggregation == IGN_AGGR_CONVOLUTION)
      return err(IGN_ERR_UNSUPPORTED, "oracle: attention / convolution are not restated in C++");
    for (int s = 0; s < mp.num_sources; ++s)
      if (mp.sources[s].msg_num_layers) return err(IGN_ERR_UNSUPPORTED, "oracle: message networks are not restated in C++");
  }
  int in = 0;
  for (int i = 0; i < p->num_readout_inputs; ++i) in += p->entities[p->readout_inputs[i]].hidden_dim;
  for (int l = 0; l < p->num_dense; ++l) {
    if (k + 2 > n_params) return err(IGN_ERR_INVALID, "too few parameter tensors");
    m.dense.push_back({in, p->dense[l].units, p->dense[l].activation, params[k], params[k + 1]});
    in = p->dense[l].units;
    k += 2;
  }
  if (k != n_params) return err(IGN_ERR_INVALID, "parameter tensor count does not match the plan");
  const int G = d->num_graphs, E = p->num_entities, A = p->num_adjacencies, I = p->num_interleave;
  std::vector<Graph> gs(G);
  std::vector<int64_t> foff(E, 0), eoff(A, 0), ioff(I, 0);
  int64_t ooff = 0;
  std::vector<int64_t> out_off(G + 1, 0);
  const int out_units = p->dense[p->num_dense - 1].units;
  for (int g = 0; g < G; ++g) {
    Graph& x = gs[g];
    for (int e = 0; e < E; ++e) {
      x.n.push_back(d->num_nodes[(int64_t)g * E + e]);
      const int F = p->entities[e].feature_total;
      x.feat.push_back(F ? d->features[e] + foff[e] * F : nullptr);
      foff[e] += x.n[e];
    }
    for (int a = 0; a < A; ++a) {
      const int64_t n = d->adj_edges[(int64_t)g * A + a];
      x.src.push_back(d->adj_src[a] + eoff[a]);
      x.dst.push_back(d->adj_dst[a] + eoff[a]);
      x.seq.push_back(d->adj_seq[a] + eoff[a]);
      x.ne.push_back(n);
      eoff[a] += n;
    }
    for (int i = 0; i < I; ++i) {
      const int64_t n = d->interleave_len[(int64_t)g * I + i];
      x.il.push_back(d->interleave_idx[i] + ioff[i]);
      x.nil.push_back(n);
      ioff[i] += n;
    }
    ooff += x.n[p->readout_inputs[0]] * out_units;
    out_off[g + 1] = ooff;
  }
  if (threads > 0) omp_set_num_threads(threads);
  const int nt = threads > 0 ? threads : omp_get_max_threads();
  int rc = IGN_OK;
  std::string msg;
  if (G >= 2 * nt) {   // graphs in parallel
#pragma omp parallel for schedule(dynamic, 1)
    for (int g = 0; g < G; ++g) {
      std::string m2;
      const int r = precision ? graph_forward<double>(m, gs[g], out + out_off[g], false, m2)
                              : graph_forward<float>(m, gs[g], out + out_off[g], false, m2);
      if (r) {
#pragma omp critical
        {
          rc = r;
          msg = m2;
        }
      }
    }
  } else {
    for (int g = 0; g < G && !rc; ++g)
      rc = precision ? graph_forward<double>(m, gs[g], out + out_off[g], true, msg)
                     : graph_forward<float>(m, gs[g], out + out_off[g], true, msg);
  }
  if (rc) return err(rc, ("oracle: " + msg).c_str());
  return IGN_OK;
}

}  // extern "C"
