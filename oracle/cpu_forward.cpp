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

struct Cell {
  int din, H;
  const float *W, *U, *b;   // [din][3H], [H][3H], [2][3H]
};

// one Keras GRU step for one row: out = GRU(x, h).  The loops are written so that the compiler
// vectorises them (libmvec expf / tanhf under -ffast-math) and, for the compile-time widths of
// the example models, keeps the 3H accumulators in registers across the k loop: this is the
// timed CPU line.
template <int DIN, int H, typename T>
void gru_step_t(const Cell& c, const T* __restrict__ x, const T* __restrict__ h, T* __restrict__ out) {
  constexpr int H3 = 3 * H;
  T mx[H3], mh[H3];
  for (int j = 0; j < H3; ++j) {
    mx[j] = c.b[j];
    mh[j] = c.b[H3 + j];
  }
  for (int k = 0; k < DIN; ++k) {
    const T xv = x[k];
    const float* __restrict__ w = c.W + k * H3;
#pragma GCC unroll 16
    for (int j = 0; j < H3; ++j) mx[j] += xv * w[j];
  }
  for (int k = 0; k < H; ++k) {
    const T hv = h[k];
    const float* __restrict__ u = c.U + k * H3;
#pragma GCC unroll 16
    for (int j = 0; j < H3; ++j) mh[j] += hv * u[j];
  }
  // z | r; the argument is clamped to +-80 so that no exp overflows (-ffast-math assumes finite
  // values; sigmoid is saturated there: exp(-80) is below float32's resolution of 1)
  for (int j = 0; j < 2 * H; ++j) mx[j] = T(1) / (T(1) + std::exp(-std::min(T(80), std::max(T(-80), mx[j] + mh[j]))));
  for (int j = 0; j < H; ++j) mh[j] = std::tanh(mx[2 * H + j] + mx[H + j] * mh[2 * H + j]);
  for (int j = 0; j < H; ++j) out[j] = mx[j] * h[j] + (T(1) - mx[j]) * mh[j];
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
  for (int it = 0; it < p->num_iterations; ++it) {
    for (int mi = 0; mi < p->num_mps; ++mi) {
      const ign_mp_desc& mp = p->mps[mi];
      const Cell& c = m.cells[mp.cell];
      const int dst = mp.dst_entity, H = c.H, NS = mp.num_sources;
      const int64_t ND = g.n[dst];
      const bool sorted = mp.aggregation != IGN_AGGR_SUM;
      const bool axis2 = mp.aggregation == IGN_AGGR_CONCAT && mp.concat_axis == 2;
      // per destination: (position, source slot, source row), in source then edge order
      std::vector<int64_t> lmax(NS, 0), flen(ND, 0);
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
      struct Msg { int64_t pos; int s; int64_t row; };
      std::vector<int64_t> ptr(ND + 1, 0);
      for (int s = 0; s < NS; ++s) {
        const int a = mp.sources[s].adjacency, se = mp.sources[s].entity;
        for (int64_t k = 0; k < g.ne[a]; ++k) {
          const int64_t si = g.src[a][k], di = g.dst[a][k];
          if (si < 0 || si >= g.n[se] || di < 0 || di >= ND) { msg = "index out of range (gather, GM:432)"; return IGN_ERR_INVALID; }
          ptr[di + 1]++;
        }
      }
      for (int64_t r = 0; r < ND; ++r) ptr[r + 1] += ptr[r];
      std::vector<Msg> msgs(ptr[ND]);
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
      if (par) {
#pragma omp parallel
        {
          std::vector<T> x(DIN), h(H), hn(H), mx(3 * H), mh(3 * H);
#pragma omp for schedule(dynamic, 64)
          for (int64_t d = 0; d < ND; ++d) run(d, x, h, hn, mx, mh);
        }
      } else {
        std::vector<T> x(DIN), h(H), hn(H), mx(3 * H), mh(3 * H);
        for (int64_t d = 0; d < ND; ++d) run(d, x, h, hn, mx, mh);
      }
      std::swap(S[dst], S2[dst]);   // GM:602: the destination's state is overwritten
    }
  }
  // readout: the predict inputs concatenated on axis 1, then the Dense stack (GM:611-629)
  const int64_t R = g.n[p->readout_inputs[0]];
  int width = 0;
  for (int i = 0; i < p->num_readout_inputs; ++i) width += p->entities[p->readout_inputs[i]].hidden_dim;
  // one row of the readout; rows are independent, so one large graph splits them over the
  // threads in static chunks (the serial loop was most of the 25k-node graph's CPU time)
  auto readout_row = [&](int64_t r, std::vector<T>& a, std::vector<T>& b2) {
    int col = 0;
    for (int i = 0; i < p->num_readout_inputs; ++i) {
      const int e = p->readout_inputs[i], H = p->entities[e].hidden_dim;
      std::copy(S[e].begin() + r * H, S[e].begin() + (r + 1) * H, a.begin() + col);
      col += H;
    }
    std::vector<T>& cur = a;
    for (const auto& L : m.dense) {
      b2.assign(L.out, T(0));
      for (int j0 = 0; j0 < L.out; j0 += 64) {   // 64 output columns at a time (register-resident)
        const int nj = std::min(64, L.out - j0);
        T acc[64];
        for (int j = 0; j < 64; ++j) acc[j] = j < nj && L.b ? T(L.b[j0 + j]) : T(0);
        if (nj == 64) {
          for (int k = 0; k < L.in; ++k) {
            const T v = cur[k];
            const float* __restrict__ w = L.W + (int64_t)k * L.out + j0;

            for (int j = 0; j < 64; ++j) acc[j] += v * w[j];
          }
        } else {
          for (int k = 0; k < L.in; ++k) {
            const T v = cur[k];
            const float* w = L.W + (int64_t)k * L.out + j0;
            for (int j = 0; j < nj; ++j) acc[j] += v * w[j];
          }
        }
        for (int j = 0; j < nj; ++j) b2[j0 + j] = act(acc[j], L.act);
      }
      cur.swap(b2);
    }
    for (size_t j = 0; j < cur.size(); ++j) out[r * (int64_t)cur.size() + j] = (float)cur[j];
  };
  if (par) {
#pragma omp parallel
    {
      std::vector<T> a(width), b2;
#pragma omp for schedule(static)
      for (int64_t r = 0; r < R; ++r) {
        a.resize(width);
        readout_row(r, a, b2);
      }
    }
  } else {
    std::vector<T> a(width), b2;
    for (int64_t r = 0; r < R; ++r) {
      a.resize(width);
      readout_row(r, a, b2);
    }
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
