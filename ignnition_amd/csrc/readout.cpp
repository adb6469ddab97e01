// readout.cpp — the readout program of ComnetModel.call (GM:605-655): the operations that run
// before predict, each writing a named tensor the later operations read (get_global_var_or_input,
// GM:660-675).
//
//   neural_network       Readout_nn (AUX:1188-1211): Dense stack on the axis-1 concatenation of
//                        its inputs; weights readout_model_<op index> (GM:352-358)
//   pooling              Pooling_operation (AUX:1136-1185): sum / mean / max over axis 0 of one
//                        graph's rows -> [1, F]
//   product              Product_operation element_wise (AUX:1054-1094): tf.multiply
//   extend_adjacencies   Extend_adjacencies (AUX:1214-1265): gather the adjacency's source and
//                        destination rows per edge
//
// The reference runs them once per graph (model_fn's loop, GM:712-724).  In the batch every
// tensor lives on a row space whose rows are graph-contiguous: an entity's rows, one row per
// graph, or an adjacency's edges.  Pooling reduces per graph and a per-graph operand broadcasts
// over its own graph's rows, so the batch equals the per-graph loop.
//
// Not lowered: product dot_product (tf.tensordot axes=0 is an outer product of rank 4, while the
// reference records its width as 1, GM:374-375), products or concatenations across different
// entity row spaces (TF accepts them only when the row counts happen to agree), raw input
// features as readout inputs.
#include <algorithm>
#include <cstring>

#include "engine_internal.h"
#include "readout_kernels.h"
#include "train_kernels.h"

namespace ign {

int act_ok(int a);

namespace {

int parse_dense(const ign_dense_desc* d, int n, int in, std::vector<DenseP>& out, const char* what, int idx) {
  for (int l = 0; l < n; ++l) {
    DenseP dp;
    dp.in = in;
    dp.out = d[l].units;
    dp.act = d[l].activation;
    dp.use_bias = d[l].use_bias;
    dp.l2 = d[l].l2;
    if (dp.out <= 0) return fail(IGN_ERR_INVALID, "%s %d, dense layer %d: units must be > 0", what, idx, l);
    if (!act_ok(dp.act)) return fail(IGN_ERR_UNSUPPORTED, "%s %d, dense layer %d: activation %d", what, idx, l, dp.act);
    out.push_back(dp);
    in = dp.out;
  }
  return IGN_OK;
}

const char* space_name(int s) { return s == RS_ENTITY ? "entity" : s == RS_GRAPH ? "graph" : "adjacency"; }

}  // namespace

int readout_plan(ign_plan* p, const ign_plan_desc* d) {
  const int NE = (int)p->ents.size();
  p->adj_src_ent.assign(p->n_adj, -1);
  p->adj_dst_ent.assign(p->n_adj, -1);
  for (const MPP& mp : p->mps)
    for (const auto& s : mp.src) {
      p->adj_src_ent[s.adjacency] = s.entity;
      p->adj_dst_ent[s.adjacency] = mp.dst;
    }
  p->ro_t.clear();
  p->ro_ops.clear();
  for (int e = 0; e < NE; ++e) p->ro_t.push_back({RS_ENTITY, e, p->ents[e].hidden_dim});
  if (d->num_readout_ops < 0 || (d->num_readout_ops > 0 && !d->readout_ops))
    return fail(IGN_ERR_INVALID, "bad readout operation list");
  for (int k = 0; k < d->num_readout_ops; ++k) {
    const ign_readout_op_desc& od = d->readout_ops[k];
    RoOp op;
    op.type = od.type;
    op.mode = od.mode;
    op.adj = od.adjacency;
    if (od.num_inputs <= 0 || !od.inputs) return fail(IGN_ERR_INVALID, "readout op %d: no input", k);
    for (int i = 0; i < od.num_inputs; ++i) {
      const int id = od.inputs[i];
      if (id < 0 || id >= (int)p->ro_t.size()) return fail(IGN_ERR_INVALID, "readout op %d: input tensor %d", k, id);
      op.in.push_back(id);
    }
    const RoTensor t0 = p->ro_t[op.in[0]];   // copies: ro_t grows below
    op.out = (int)p->ro_t.size();
    int rc;
    switch (op.type) {
      case IGN_RO_NEURAL_NETWORK: {
        for (int id : op.in) {
          if (!p->ro_t[id].same_space(t0))
            return fail(IGN_ERR_UNSUPPORTED, "readout op %d: inputs on different row spaces (concat axis 1)", k);
          op.in_width += p->ro_t[id].width;
        }
        if (od.num_dense <= 0 || !od.dense) return fail(IGN_ERR_INVALID, "readout op %d: no Dense layer", k);
        if ((rc = parse_dense(od.dense, od.num_dense, op.in_width, op.layers, "readout op", k))) return rc;
        p->ro_t.push_back({t0.space, t0.sid, op.layers.back().out});
        break;
      }
      case IGN_RO_POOLING:   // Pooling_operation reads input[0] only (GM:634)
        if (op.mode < IGN_POOL_SUM || op.mode > IGN_POOL_MAX)
          return fail(IGN_ERR_INVALID, "readout op %d: pooling type %d", k, op.mode);
        p->ro_t.push_back({RS_GRAPH, 0, t0.width});
        break;
      case IGN_RO_PRODUCT: {  // input[0] * input[1] (GM:641-642)
        if (op.mode != 0)
          return fail(IGN_ERR_UNSUPPORTED, "readout op %d: dot_product (tf.tensordot axes=0) is a rank-4 outer "
                      "product the reference records as width 1 (GM:374-375); only element_wise is lowered", k);
        if (op.in.size() < 2) return fail(IGN_ERR_INVALID, "readout op %d: product needs two inputs", k);
        const RoTensor t1 = p->ro_t[op.in[1]];
        if (t1.width != t0.width && t1.width != 1)
          return fail(t0.width == 1 ? IGN_ERR_UNSUPPORTED : IGN_ERR_INVALID,
                      "readout op %d: product of widths %d and %d (the result keeps input 0's width, GM:372-373)",
                      k, t0.width, t1.width);
        RoTensor o = t0;
        if (!t0.same_space(t1)) {
          if (t0.space == RS_GRAPH) o = {t1.space, t1.sid, t0.width};
          else if (t1.space != RS_GRAPH)
            return fail(IGN_ERR_UNSUPPORTED, "readout op %d: product of tensors on different row spaces (%s %d, %s %d)",
                        k, space_name(t0.space), t0.sid, space_name(t1.space), t1.sid);
        }
        p->ro_t.push_back(o);
        break;
      }
      case IGN_RO_EXTEND: {
        if (op.in.size() < 2) return fail(IGN_ERR_INVALID, "readout op %d: extend_adjacencies needs two inputs", k);
        if (op.adj < 0 || op.adj >= p->n_adj || p->adj_src_ent[op.adj] < 0)
          return fail(IGN_ERR_INVALID, "readout op %d: adjacency slot %d is not read by any message passing", k, op.adj);
        const RoTensor t1 = p->ro_t[op.in[1]];
        if (t0.space != RS_ENTITY || t0.sid != p->adj_src_ent[op.adj] || t1.space != RS_ENTITY ||
            t1.sid != p->adj_dst_ent[op.adj])
          return fail(IGN_ERR_INVALID, "readout op %d: extend_adjacencies inputs must live on the adjacency's source "
                      "and destination entities", k);
        p->ro_t.push_back({RS_ADJ, op.adj, t0.width});
        p->ro_t.push_back({RS_ADJ, op.adj, t1.width});
        break;
      }
      default:
        return fail(IGN_ERR_UNSUPPORTED, "readout op %d: type %d", k, op.type);
    }
    p->ro_ops.push_back(std::move(op));
  }

  // predict (GM:612-629)
  p->ro_in.assign(d->readout_inputs, d->readout_inputs + d->num_readout_inputs);
  if (p->ro_in.empty()) return fail(IGN_ERR_INVALID, "readout has no input");
  int width = 0;
  for (int id : p->ro_in) {
    if (id < 0 || id >= (int)p->ro_t.size()) return fail(IGN_ERR_INVALID, "readout input tensor %d", id);
    if (!p->ro_t[id].same_space(p->ro_t[p->ro_in[0]]))
      return fail(IGN_ERR_UNSUPPORTED, "predict inputs on different row spaces (concat axis 1)");
    width += p->ro_t[id].width;
  }
  p->ro_width = width;
  int rc = parse_dense(d->dense, d->num_dense, width, p->dense, "predict", 0);
  if (rc) return rc;
  if (p->dense.empty()) return fail(IGN_ERR_INVALID, "readout has no Dense layer");
  p->fused_readout = p->dense.size() == 3 &&
                     readout3_supported(width, p->dense[0].out, p->dense[1].out, p->dense[0].act, p->dense[1].act) &&
                     p->dense[2].out == 1 && p->dense[0].use_bias && p->dense[1].use_bias;
  return IGN_OK;
}

static int64_t align64(int64_t x) { return (x + 63) & ~int64_t(63); }

int64_t readout_layout(ign_plan* p, int64_t off) {
  for (size_t k = 0; k < p->ro_ops.size(); ++k)
    for (size_t l = 0; l < p->ro_ops[k].layers.size(); ++l) {
      DenseP& dp = p->ro_ops[k].layers[l];
      const int owner = (int)(k * 64 + l);
      dp.off_w = off; p->tensors.push_back({11, owner, off, dp.in, dp.out}); off = align64(off + (int64_t)dp.in * dp.out);
      if (dp.use_bias) { dp.off_b = off; p->tensors.push_back({12, owner, off, 1, dp.out}); off = align64(off + dp.out); }
    }
  return off;
}

int64_t readout_packed(ign_plan* p, int64_t pk) {
  for (auto& op : p->ro_ops)
    for (auto& dp : op.layers)
      if (dense_fwd_supported(dp.in, dp.out)) { dp.pk_w = pk; pk = align64(pk + (int64_t)dp.in * dp.out); }
  return pk;
}

int readout_repack(ign_plan* p) {
  for (auto& op : p->ro_ops)
    for (auto& dp : op.layers)
      if (dp.pk_w >= 0) HIP_TRY(launch_pack_dense(p->d_params + dp.off_w, p->d_packed + dp.pk_w, dp.in, dp.out, p->stream));
  return IGN_OK;
}

int64_t space_rows(const ign_plan* p, const ign_batch* b, const RoTensor& t) {
  (void)p;
  if (t.space == RS_ENTITY) return b->rows[t.sid];
  if (t.space == RS_GRAPH) return b->G;
  return b->adj_rows[t.sid];
}

// graph offsets of a row space ([G + 1])
static std::vector<int64_t> space_offsets(const ign_batch* b, const RoTensor& t) {
  std::vector<int64_t> off(b->G + 1);
  for (int g = 0; g <= b->G; ++g) {
    if (t.space == RS_GRAPH) off[g] = g;
    else if (t.space == RS_ADJ) off[g] = b->adj_off[t.sid][g];
    else off[g] = g < b->G ? b->row_off[t.sid][g] : b->rows[t.sid];
  }
  return off;
}

const float* readout_tensor(const ign_plan* p, const ign_batch* b, int id) {
  const int NE = (int)p->ents.size();
  if (id < NE) return b->d_state[b->cur[id]][id];
  return b->ro_buf[id];
}

int readout_batch(ign_plan* p, ign_batch* b, const ign_batch_desc* d) {
  const int G = b->G, NA = p->n_adj;
  b->adj_rows.assign(NA, 0);
  b->adj_off.assign(NA, std::vector<int64_t>(G + 1, 0));
  for (int a = 0; a < NA; ++a) {
    for (int g = 0; g < G; ++g) b->adj_off[a][g + 1] = b->adj_off[a][g] + d->adj_edges[(int64_t)g * NA + a];
    b->adj_rows[a] = b->adj_off[a][G];
  }
  b->ro_buf.assign(p->ro_t.size(), nullptr);
  b->ro.clear();
  b->ro.resize(p->ro_ops.size());
  if (!p->ro_ops.empty() && d->halo_rows)
    for (size_t e = 0; e < p->ents.size(); ++e)
      if (d->halo_rows[e] > 0) return fail(IGN_ERR_UNSUPPORTED, "readout operations on an edge-cut partition");
  int rc;
  for (size_t k = 0; k < p->ro_ops.size(); ++k) {
    const RoOp& op = p->ro_ops[k];
    RoBatchOp& bo = b->ro[k];
    const int nout = op.type == IGN_RO_EXTEND ? 2 : 1;
    for (int j = 0; j < nout; ++j) {
      const RoTensor& t = p->ro_t[op.out + j];
      if ((rc = dev_alloc(b, &bo.out[j], std::max<int64_t>(1, space_rows(p, b, t) * t.width)))) return rc;
      b->ro_buf[op.out + j] = bo.out[j];
    }
    const RoTensor& t0 = p->ro_t[op.in[0]];
    const int64_t n_in = space_rows(p, b, t0);
    switch (op.type) {
      case IGN_RO_NEURAL_NETWORK:
        if (op.in.size() > 1 && (rc = dev_alloc(b, &bo.cat, std::max<int64_t>(1, n_in * op.in_width)))) return rc;
        for (size_t l = 0; l + 1 < op.layers.size(); ++l) {
          float* t = nullptr;
          if ((rc = dev_alloc(b, &t, std::max<int64_t>(1, n_in * op.layers[l].out)))) return rc;
          bo.tmp.push_back(t);
        }
        break;
      case IGN_RO_POOLING: {
        const std::vector<int64_t> off = space_offsets(b, t0);
        std::vector<int64_t> chunk, count(G);
        std::vector<int32_t> cptr(G + 1, 0);
        for (int g = 0; g < G; ++g) {
          count[g] = off[g + 1] - off[g];
          for (int64_t r = off[g]; r < off[g + 1]; r += POOL_CHUNK) {
            chunk.push_back(r);
            chunk.push_back(std::min(off[g + 1], r + POOL_CHUNK));
          }
          cptr[g + 1] = (int32_t)(chunk.size() / 2);
        }
        bo.n_chunks = (int64_t)chunk.size() / 2;
        if ((rc = dev_upload(b, &bo.d_chunk, chunk)) || (rc = dev_upload(b, &bo.d_chunk_ptr, cptr)) ||
            (rc = dev_upload(b, &bo.d_count, count)) || (rc = dev_upload(b, &bo.d_inoff, off)))
          return rc;
        if ((rc = dev_alloc(b, &bo.d_partial, std::max<int64_t>(1, bo.n_chunks * t0.width)))) return rc;
        break;
      }
      case IGN_RO_PRODUCT:
        if ((rc = dev_upload(b, &bo.d_seg, space_offsets(b, p->ro_t[op.out])))) return rc;
        break;
      case IGN_RO_EXTEND: {
        const int a = op.adj;
        const int se = p->adj_src_ent[a], de = p->adj_dst_ent[a];
        std::vector<int32_t> is(b->adj_rows[a]), id(b->adj_rows[a]);
        for (int g = 0; g < G; ++g)
          for (int64_t e = b->adj_off[a][g]; e < b->adj_off[a][g + 1]; ++e) {
            const int64_t s = IdxArr(d->adj_src[a], d->index_bytes)[e], t = IdxArr(d->adj_dst[a], d->index_bytes)[e];
            const int64_t ns = d->num_nodes[(int64_t)g * p->ents.size() + se];
            const int64_t nd = d->num_nodes[(int64_t)g * p->ents.size() + de];
            if (s < 0 || s >= ns || t < 0 || t >= nd)   // the reference logs and exits (AUX:1253-1263)
              return fail(IGN_ERR_INVALID, "extend_adjacencies: graph %d edge %lld of adjacency %d indexes outside "
                          "its entities", g, (long long)(e - b->adj_off[a][g]), a);
            is[e] = (int32_t)(b->row_off[se][g] + s);
            id[e] = (int32_t)(b->row_off[de][g] + t);
          }
        if ((rc = dev_upload(b, &bo.idx[0], is)) || (rc = dev_upload(b, &bo.idx[1], id))) return rc;
        bo.h_idx[0] = std::move(is);
        bo.h_idx[1] = std::move(id);
        break;
      }
    }
  }
  return IGN_OK;
}

int readout_ops_run(ign_plan* p, ign_batch* b, hipStream_t st, const float* const* ent) {
  const float* prm = p->d_params;
  const int NE = (int)p->ents.size();
  auto readout_tensor = [&](const ign_plan* pp, const ign_batch* bb, int id) -> const float* {
    return ent && id < NE ? ent[id] : ign::readout_tensor(pp, bb, id);
  };
  for (size_t k = 0; k < p->ro_ops.size(); ++k) {
    const RoOp& op = p->ro_ops[k];
    RoBatchOp& bo = b->ro[k];
    const RoTensor& t0 = p->ro_t[op.in[0]];
    const int64_t n = space_rows(p, b, t0);
    switch (op.type) {
      case IGN_RO_NEURAL_NETWORK: {   // GM:612-628
        const float* x = readout_tensor(p, b, op.in[0]);
        if (op.in.size() > 1) {
          int col = 0;
          for (int id : op.in) {
            HIP_TRY(launch_concat_cols(bo.cat, n, op.in_width, col, readout_tensor(p, b, id), p->ro_t[id].width, st));
            col += p->ro_t[id].width;
          }
          x = bo.cat;
        }
        int stride = op.in_width;
        for (size_t l = 0; l < op.layers.size(); ++l) {
          const DenseP& dl = op.layers[l];
          float* y = l + 1 == op.layers.size() ? bo.out[0] : bo.tmp[l];
          HIP_TRY(launch_dense_fwd(x, n, dl.in, stride, dl.pk_w >= 0 ? p->d_packed + dl.pk_w : nullptr,
                                   prm + dl.off_w, dl.use_bias ? prm + dl.off_b : nullptr, dl.out, dl.act, y, st));
          x = y;
          stride = dl.out;
        }
        break;
      }
      case IGN_RO_POOLING:            // GM:632-637
        HIP_TRY(launch_pool(readout_tensor(p, b, op.in[0]), t0.width, bo.n_chunks, bo.d_chunk, bo.d_chunk_ptr,
                            bo.d_count, b->G, op.mode, bo.d_partial, bo.out[0], st));
        break;
      case IGN_RO_PRODUCT: {          // GM:640-645
        const RoTensor& t1 = p->ro_t[op.in[1]];
        const RoTensor& to = p->ro_t[op.out];
        ProductArgs a{readout_tensor(p, b, op.in[0]), readout_tensor(p, b, op.in[1]), t0.width, t1.width, to.width,
                      t0.space == RS_GRAPH && to.space != RS_GRAPH, t1.space == RS_GRAPH && to.space != RS_GRAPH,
                      bo.d_seg, b->G, space_rows(p, b, to), bo.out[0]};
        HIP_TRY(launch_product(a, st));
        break;
      }
      case IGN_RO_EXTEND: {           // GM:647-655
        const int64_t e = b->adj_rows[op.adj];
        HIP_TRY(launch_gather(readout_tensor(p, b, op.in[0]), t0.width, bo.idx[0], e, bo.out[0], st));
        HIP_TRY(launch_gather(readout_tensor(p, b, op.in[1]), p->ro_t[op.in[1]].width, bo.idx[1], e, bo.out[1], st));
        break;
      }
    }
  }
  return IGN_OK;
}

}  // namespace ign
