// train.cpp — the training step behind the C ABI: model_fn's TRAIN branch
// (code/utils/generate_model.py:697-830 = GM).
//
//   ign_forward_train   the forward of ComnetModel.call (GM:384-658), keeping what the backward
//                       needs: every hidden-state version (no ping-pong), the per-step states of
//                       each ordered update, the aggregated messages of each sum update, and
//                       the readout activations
//   ign_backward        tf.gradients(total_loss, trainable_variables) (GM:790) for a given
//                       dLoss/dpredictions, plus the Dense l2 regularizer terms (AUX:833-834)
//   ign_mse_loss        MeanSquaredError over the batch's flat predictions (GM:716-753)
//   ign_adam_step       Keras Adam with the host-evaluated ExponentialDecay rate (GM:797-818)
//
// Backward schedule: readout Dense stack in reverse, then the MP instances of the forward in
// reverse order.  Per entity one gradient buffer tracks dLoss/d(current version); an MP turns
// the gradient of its output version into that of its input version (GRU backward) and adds
// the message gradients to its sources.  Weight gradients are row-contractions
// (tsgemm_add) reduced in a fixed order: the result is deterministic.

#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>
#include <memory>
#include <vector>

#include "engine_internal.h"
#include "readout_kernels.h"
#include "train_kernels.h"

struct MPTrain {
  std::vector<float*> hs;     // sorted MPs: per iteration [(n_steps + n_dst)][H]
  std::vector<float*> xs;     // sum MPs: per iteration [rows][DIN]
  std::vector<float*> ss;     // convolution MPs: per iteration, message sums before K [rows][DIN]
  float* deg = nullptr;       // convolution MPs: messages per destination row (float)
  int32_t* amdst = nullptr;   // attention MPs: destination row of every CSR message
  std::vector<int32_t*> asptr, asidx;   // attention MPs, per slot: source row -> CSR messages
  int64_t hs_rows = 0;
  int32_t* hdrb = nullptr;    // sorted MPs: the ordered backward's tile headers (launch_seq_bwd_hdr)
  std::vector<int32_t*> tptr, tidx;   // per source slot: source row -> steps (sorted) / dst rows (sum)
  hvec<int64_t> trows;         // (a source with a message network: its rows are the edges)
  // message networks, per source slot: state row -> its edges (ascending), for the hs_source /
  // hs_dest columns of the network's input gradient
  int32_t* nsrc_ptr[IGN_MAX_SLOTS] = {nullptr, nullptr, nullptr, nullptr};
  int32_t* nsrc_idx[IGN_MAX_SLOTS] = {nullptr, nullptr, nullptr, nullptr};
  int32_t* ndst_ptr[IGN_MAX_SLOTS] = {nullptr, nullptr, nullptr, nullptr};
  int32_t* ndst_idx[IGN_MAX_SLOTS] = {nullptr, nullptr, nullptr, nullptr};
};

struct MPRec {
  int mi, it, v_in;
  int src_v[IGN_MAX_SLOTS];
};

struct TrainState {
  std::vector<std::vector<float*>> ver;   // [entity][version] hidden states
  hvec<int> cur;                   // current version per entity (after the forward)
  std::vector<MPTrain> mp;
  std::vector<MPRec> recs;
  float* ga = nullptr;
  float* gu = nullptr;
  float* dx = nullptr;
  float* dtab = nullptr;
  std::vector<float*> dS[2];
  std::vector<float*> act;                // readout activations of layers 0 .. L-2
  float* dz[2] = {nullptr, nullptr};
  float* part = nullptr;
  float* bsum = nullptr;                  // [(H + 1) 3H], H <= 32: fused ordered backward's reduction
  float* ro_x = nullptr;                  // concatenated readout input (several input entities)
  float* dro = nullptr;
  float* dmsg = nullptr;                  // message networks: d(messages) [edges][out]
  float* mz[2] = {nullptr, nullptr};      // ... layer gradients (ping-pong) [edges][widest]
  float* mdin = nullptr;                  // ... d(network input) [edges][din]
  float* adw = nullptr;                   // attention: d(weight) and d(score input) per message,
  float* adv = nullptr;                   //   d(score) per source / destination row, d(w1 | w2)
  float* ads_src = nullptr;
  float* ads_dst = nullptr;
  float* adw12 = nullptr;
  // readout operations before predict (GM:605-655): d(tensor) per op output, Dense scratch
  std::vector<float*> dT;                 // per readout tensor id (null for entity states)
  float* rz[2] = {nullptr, nullptr};
  float* rcat = nullptr;
  float* rties = nullptr;
  std::vector<int32_t*> rx_ptr, rx_idx;   // extend ops: per op 2 transposed CSRs (input row -> edges)
  bool forward_done = false;
  // stepped forward / backward (ign_forward_train_begin .. _end, ign_backward_begin .. _end): the
  // edge-cut driver exchanges halo rows between the steps
  int f_it = 0, f_mi = 0;
  bool f_open = false;
  float** res_ptrs = nullptr;   // the graph-resident training forward's version / save pointer arrays
  std::vector<float*> tsave;    // its saved projected tables of the ordered MP, per iteration
  bool tab_saved = false;       // this forward saved them (the backward skips build_table)
  // weight gradients formed once per MP instance (T of them per backward) keep their partial tiles
  // here and are reduced once, at ign_backward_end, in instance order (IGN_DEFER_WGRAD=0: per instance)
  struct DeferredGrad {
    int64_t off_c, off_cb;   // gradient offsets in the parameter layout (off_cb -1: no bias column)
    int M, N, ones;
    float* part;
    int64_t cap, used;   // chunk slots (plus the reduction's scratch after cap)
  };
  std::vector<DeferredGrad> defer;
  struct DeferredSeq {   // the fused ordered backward's per-wave dU / bias partials, per cell
    int cell, H;
    float* part;
    int64_t cap, used;   // partial slots (plus the reduction's scratch after cap)
  };
  std::vector<DeferredSeq> defer_seq;
  int b_ri = -1;
  bool b_open = false;
  hvec<int> dcur;                          // backward: current gradient buffer per entity
  float* grads = nullptr;                  // backward: the caller's gradient vector
  float l2_scale = 1.f;                    // backward: weight of the l2 terms (1/ranks under edge-cut)
  std::vector<void*> allocs;               // blocks of pool
  DevPool* pool = nullptr;                 // the batch's (outlives this state)
  hipStream_t stream = nullptr;            // the plan stream, for the release fence
};

void train_state_destroy(TrainState* t) {
  if (!t) return;
  if (t->pool) pool_release(t->pool, t->allocs, t->stream);
  delete t;
}

namespace {

int talloc(TrainState* t, float** out, int64_t n) {
  void* p = nullptr;
  hipError_t e = pool_alloc(t->pool, &p, (std::max<int64_t>(n, 0) + 256) * sizeof(float), true);
  if (e != hipSuccess) return fail(IGN_ERR_OOM, "training buffers: device alloc (%lld floats): %s", (long long)n,
                                   hipGetErrorString(e));
  t->allocs.push_back(p);
  *out = static_cast<float*>(p);
  return IGN_OK;
}

// The transposed CSRs of MP mb on the GPU (train_csr.hip; IGN_TRAIN_CSR_GPU=0: build_csrs on the
// host): a stable radix sort of the step (seq) or message keys on the upload stream, the same
// arrays as the host's.  ptr[s]: row pointers of source slot s into idx, the sorted values every
// slot shares.  The keys and the sort's scratch go back to the pool behind a fence.
int tcsr_gpu(TrainState* t, const MPB& mb, int S, const int64_t* tkeys, bool seq, std::vector<int32_t*>& ptr,
             int32_t*& idx) {
  hipStream_t st = upload_stream();
  const int64_t n = seq ? mb.n_steps : mb.n_msgs;
  int rc;
  float* f = nullptr;
  if ((rc = talloc(t, &f, std::max<int64_t>(n, 1)))) return rc;
  idx = reinterpret_cast<int32_t*>(f);
  ptr.assign(S, nullptr);
  for (int s = 0; s < S; ++s) {
    if ((rc = talloc(t, &f, tkeys[s] + 1))) return rc;
    ptr[s] = reinterpret_cast<int32_t*>(f);
  }
  const size_t nb = (size_t)std::max<int64_t>(n, 1) * 4, tb = tcsr_temp_bytes(std::max<int64_t>(n, 1));
  std::vector<void*> scratch(4, nullptr);
  for (int k = 0; k < 4; ++k) {
    const hipError_t e = pool_alloc(t->pool, &scratch[k], k < 3 ? nb : std::max<size_t>(tb, 256), false);
    if (e != hipSuccess) {
      scratch.resize(k);
      pool_release(t->pool, scratch, st);
      return fail(IGN_ERR_OOM, "training CSR scratch: device alloc: %s", hipGetErrorString(e));
    }
  }
  uint32_t* keys_in = static_cast<uint32_t*>(scratch[0]);
  uint32_t* keys_out = static_cast<uint32_t*>(scratch[1]);
  int32_t* vals_in = static_cast<int32_t*>(scratch[2]);
  uint32_t max_key = 0;
  hipError_t e;
  if (seq) {
    e = launch_tcsr_keys_seq(mb.d_step_code, n, (uint32_t)mb.zero_row, keys_in, vals_in, st);
    max_key = (uint32_t)mb.zero_row;
  } else {
    e = launch_tcsr_keys_sum(mb.d_msg_ptr, mb.d_order, mb.n_dst, mb.d_msg_src, keys_in, vals_in, st);
    // one slot: the codes are the rows (radix passes over the row bits only); else slot bits above
    max_key = S == 1 ? (uint32_t)std::max<int64_t>(tkeys[0], 1) : ((uint32_t)(S - 1) << IGN_SLOT_SHIFT) | IGN_ROW_MASK;
  }
  if (e == hipSuccess) e = launch_tcsr_sort(scratch[3], tb, keys_in, keys_out, vals_in, idx, n, max_key, st);
  for (int s = 0; s < S && e == hipSuccess; ++s) {
    const uint32_t key0 = seq ? (uint32_t)mb.src_off[s] : (uint32_t)s << IGN_SLOT_SHIFT;
    e = launch_tcsr_ptr(keys_out, n, key0, tkeys[s], ptr[s], st);
  }
  pool_release(t->pool, scratch, st);
  if (e != hipSuccess) return fail(IGN_ERR_DEVICE, "training CSR sort: %s", hipGetErrorString(e));
  return IGN_OK;
}

template <typename T, typename A>
int tupload(TrainState* t, T** out, const std::vector<T, A>& h) {
  void* p = nullptr;
  size_t n = std::max<size_t>(h.size(), 1);
  hipError_t e = pool_alloc(t->pool, &p, n * sizeof(T), h.empty());
  if (e != hipSuccess) return fail(IGN_ERR_OOM, "training buffers: device alloc: %s", hipGetErrorString(e));
  t->allocs.push_back(p);
  if (!h.empty()) HIP_TRY(upload_bytes(p, h.data(), h.size() * sizeof(T)));
  *out = static_cast<T*>(p);
  return IGN_OK;
}

// C (+ Cb) += A^T B over n_rows rows, its partial tiles parked for ign_backward_end's reduction
// when C has a deferred slot with room (else reduced now, as launch_tsgemm_add)
int tsgemm_deferred(TrainState* t, const float* A, int lda, const float* B, int ldb, int64_t n_rows, int M, int N,
                    float* C, float* Cb, hipStream_t st) {
  const int ones = Cb != nullptr;
  const int64_t ch = tsgemm_chunks(n_rows, M, N, ones);
  for (auto& d : t->defer)
    if (t->grads + d.off_c == C && (d.off_cb < 0 ? Cb == nullptr : Cb == t->grads + d.off_cb) && d.M == M &&
        d.N == N && d.used + ch <= d.cap) {
      HIP_TRY(launch_tsgemm_partials(A, lda, B, ldb, n_rows, M, N, ones, d.part + d.used * (int64_t)(M + ones) * N, st));
      d.used += ch;
      return IGN_OK;
    }
  HIP_TRY(launch_tsgemm_add(A, lda, B, ldb, n_rows, M, N, t->part, C, Cb, st));
  return IGN_OK;
}

int tsgemm_deferred_flush(const ign_plan* p, TrainState* t, hipStream_t st) {
  for (auto& d : t->defer_seq)
    if (d.used) {
      const CellP& cp = p->cells[d.cell];
      SeqBwdArgs a{};
      a.part = d.part;
      a.scratch = t->bsum;
      a.dU = t->grads + cp.off_rk;
      a.db_rec = t->grads + cp.off_b + 3 * cp.H;
      a.db_in = t->grads + cp.off_b;
      HIP_TRY(launch_seq_bwd_reduce(a, d.used, d.H, st));
      d.used = 0;
    }
  for (auto& d : t->defer)
    if (d.used) {
      HIP_TRY(launch_partials_reduce_add(d.part, d.used, d.M, d.N, d.ones, t->grads + d.off_c,
                                         d.off_cb < 0 ? nullptr : t->grads + d.off_cb, st));
      d.used = 0;
    }
  return IGN_OK;
}

// CSR of (key, value) pairs over n_keys keys, values kept in insertion order per key
void build_csr(int64_t n_keys, const hvec<std::pair<int64_t, int32_t>>& kv, hvec<int32_t>& ptr,
               hvec<int32_t>& idx) {
  ptr.assign(n_keys + 1, 0);
  for (auto& p : kv) ptr[p.first + 1]++;
  for (int64_t k = 0; k < n_keys; ++k) ptr[k + 1] += ptr[k];
  idx.resize(kv.size());
  hvec<int32_t> fill(ptr.begin(), ptr.end() - 1);
  for (auto& p : kv) idx[fill[p.first]++] = p.second;
}

// Per source slot s, the CSR of the (row, value) pairs visit() emits, values in emission order
// per row: one counting pass and one filling pass over the same visit, no pair list.
template <class Visit>
void build_csrs(int S, const int64_t* n_keys, Visit visit, std::vector<hvec<int32_t>>& ptr,
                std::vector<hvec<int32_t>>& idx) {
  ptr.assign(S, hvec<int32_t>());
  idx.assign(S, hvec<int32_t>());
  for (int s = 0; s < S; ++s) ptr[s].assign(n_keys[s] + 1, 0);
  visit([&](int s, int64_t key, int32_t) { ptr[s][key + 1]++; });
  std::vector<hvec<int32_t>> fill(S);
  for (int s = 0; s < S; ++s) {
    for (int64_t k = 0; k < n_keys[s]; ++k) ptr[s][k + 1] += ptr[s][k];
    idx[s].resize(ptr[s][n_keys[s]]);
    fill[s].assign(ptr[s].begin(), ptr[s].end() - 1);
  }
  visit([&](int s, int64_t key, int32_t v) { idx[s][fill[s][key]++] = v; });
}

int check_train(ign_plan* p, ign_batch* b) {
  if (!p || !b) return fail(IGN_ERR_INVALID, "null argument");
  if (b->plan != p) return fail(IGN_ERR_INVALID, "batch was created for another plan");
  if (!b->train) return fail(IGN_ERR_INVALID, "training not enabled on this batch (ign_batch_enable_training)");
  if (!p->params_set) return fail(IGN_ERR_INVALID, "parameters not set (ign_plan_set_params)");
  return set_device(p->device);
}

// project every source of sorted MP mb into its table, from the given source states
int build_table(ign_plan* p, const MPP& mp, const MPB& mb, const CellP& cp, const float* const* src) {
  const int W3 = 3 * cp.H;
  for (size_t s = 0; s < mp.src.size(); ++s) {
    // axis-2 concat (AUX:443-456): each source through its own row slice of the input kernel
    const int sdin = mp.feature_concat ? p->ents[mp.src[s].entity].hidden_dim : mp.din;
    const float* wp = p->d_packed + (mp.feature_concat ? mp.pk_slice[s] : cp.pk_w);
    HIP_TRY(launch_project(src[s], mb.src_rows[s], wp, p->d_packed + cp.pk_b, mb.d_table + mb.src_off[s] * W3,
                           s == 0 ? mb.d_table + mb.zero_row * W3 : nullptr, sdin, cp.H, p->stream));
  }
  if (mb.n_multi)
    HIP_TRY(launch_multi_sum(mb.d_table, mb.zero_row + 1, mb.n_multi, mb.d_multi_ptr, mb.d_multi_rows, W3,
                             mb.d_table + mb.zero_row * W3, p->stream));
  return IGN_OK;
}

// Backward of MP source s's message-creation network (GM:440-475), given d(messages) in t->dmsg:
// Dense stack in reverse (weight / bias gradients; the l2 terms are added once per step by
// ign_backward, not per MP instance), then the hs_source / hs_dest column
// slices of d(input) gathered back to the state rows they were read from.  The layer activations
// are the ones run_message_net left in mb (recomputed for this MP instance by the caller).
int msg_net_backward(ign_plan* p, ign_batch* b, TrainState* t, const MPP& mp, const MPB& mb, const MPTrain& mt,
                     int s, float* dsrc, float* ddst, float* grads, hipStream_t st) {
  const MsgNN& nn = mp.nn[s];
  const int64_t ne = mb.n_edges[s];
  const int L = (int)nn.layers.size();
  int zi = 0;
  HIP_TRY(launch_act_bwd(t->dmsg, mb.d_msg_layer[s][L - 1], ne * nn.layers[L - 1].out, nn.layers[L - 1].act,
                         t->mz[0], st));
  for (int l = L - 1; l >= 0; --l) {
    const DenseP& d = nn.layers[l];
    const int K = l == 0 ? nn.din : nn.layers[l - 1].out;
    const float* A = l == 0 ? mb.d_msg_in[s] : mb.d_msg_layer[s][l - 1];
    const int lda = l == 0 ? nn.din_pad : nn.layers[l - 1].out;
    HIP_TRY(launch_tsgemm_add(A, lda, t->mz[zi], d.out, ne, K, d.out, t->part, grads + d.off_w,
                              d.use_bias ? grads + d.off_b : nullptr, st));
    if (l > 0)
      HIP_TRY(launch_row_gemm_t_generic(t->mz[zi], ne, d.out, p->d_params + d.off_w, K, t->mz[1 - zi], 0,
                                        nn.layers[l - 1].act, mb.d_msg_layer[s][l - 1], st));
    else
      HIP_TRY(launch_row_gemm_t_generic(t->mz[zi], ne, d.out, p->d_params + d.off_w, K, t->mdin, 0, -1, nullptr, st));
    zi = 1 - zi;
  }
  int col = 0;
  for (size_t q = 0; q < nn.inputs.size(); ++q) {
    const int w = nn.widths[q];
    if (nn.inputs[q] == IGN_MSG_HS_SOURCE)
      HIP_TRY(launch_csr_gather_cols_add(dsrc, b->rows[mp.src[s].entity] + b->halo[mp.src[s].entity], mt.nsrc_ptr[s],
                                         mt.nsrc_idx[s], t->mdin,
                                         nn.din, col, w, 1, st));
    else if (nn.inputs[q] == IGN_MSG_HS_DEST)
      HIP_TRY(launch_csr_gather_cols_add(ddst, b->rows[mp.dst], mt.ndst_ptr[s], mt.ndst_idx[s], t->mdin, nn.din,
                                         col, w, 1, st));
    col += w;   // edge_params: input data, no gradient
  }
  return IGN_OK;
}

}  // namespace

extern "C" {

int ign_batch_enable_training(ign_plan* p, ign_batch* b) {
  if (!p || !b) return fail(IGN_ERR_INVALID, "null argument");
  if (b->plan != p) return fail(IGN_ERR_INVALID, "batch was created for another plan");
  if (b->train) return IGN_OK;
  int rc = ensure_device(p);
  if (rc) return rc;
  UploadScope scope("ign_batch_enable_training");
  const char* tcsr_env = getenv("IGN_TRAIN_CSR_GPU");
  const bool tcsr_on = !tcsr_env || atoi(tcsr_env) != 0;   // the transposed CSRs on the GPU (train_csr.hip)
  const char* fine = getenv("IGN_BUILD_PROF_FINE");
  BuildMarks bm(fine && atoi(fine) != 0);   // IGN_BUILD_PROF_FINE=1: host sections of this build
  const int E = (int)p->ents.size();
  for (size_t c = 0; c < p->cells.size(); ++c) {
    const CellP& cp = p->cells[c];
    if (!cp.used) continue;
    bool concat_only = true;   // W^T is not needed by a cell fed only by axis-2 concat MPs
    for (auto& mp : p->mps)
      if (mp.cell == (int)c && !mp.feature_concat) concat_only = false;
    if (cp.pk_ut < 0 || (cp.pk_wt < 0 && !concat_only))
      return fail(IGN_ERR_UNSUPPORTED, "no backward kernel for GRU shape (input %d, units %d)", cp.din, cp.H);
  }
  std::unique_ptr<TrainState, void (*)(TrainState*)> t(new TrainState(), train_state_destroy);
  t->pool = b->pool.get();
  t->stream = p->stream;
  const int64_t P = b->n_pred;
  // hidden-state versions: 1 + T x (MPs updating the entity)
  hvec<int> nver(E, 1);
  for (auto& mp : p->mps) nver[mp.dst] += p->T;
  t->ver.resize(E);
  t->cur.assign(E, 0);
  for (int e = 0; e < E; ++e) {
    const int64_t n = (b->rows[e] + b->halo[e]) * p->ents[e].hidden_dim;   // owned rows, then halo rows
    for (int v = 0; v < nver[e]; ++v) {
      float* f = nullptr;
      if ((rc = talloc(t.get(), &f, n))) return rc;
      t->ver[e].push_back(f);
    }
    for (int k = 0; k < 2; ++k) {
      float* f = nullptr;
      if ((rc = talloc(t.get(), &f, n))) return rc;
      t->dS[k].push_back(f);
    }
  }
  int64_t ga_n = 0, gu_n = 0, dx_n = 0, dtab_n = 0, part_n = 0, dmsg_n = 0, mz_n = 0, mdin_n = 0;
  int64_t amsg_n = 0, arows_n = 0;
  auto need_part = [&](int64_t rows, int M, int N) {
    part_n = std::max(part_n, tsgemm_partial_floats(rows, M, N));
  };
  for (size_t mi = 0; mi < p->mps.size(); ++mi) {
    const MPP& mp = p->mps[mi];
    const MPB& mb = b->mp[mi];
    const CellP& cp = p->cells[mp.cell];
    const int H = cp.H, DIN = mp.din, S = (int)mp.src.size();
    MPTrain mt;
    // transposed CSRs (source row -> steps / destinations reading it), built below: on the GPU
    // (mt.tptr, gidx) or on the host (tptr, tidx, uploaded with the slots below)
    std::vector<hvec<int32_t>> tptr, tidx;
    int32_t* gidx = nullptr;
    int64_t tkeys[IGN_MAX_SLOTS] = {0, 0, 0, 0};
    for (int s = 0; s < S; ++s)
      tkeys[s] = mp.nn[s].layers.empty() ? b->rows[mp.src[s].entity] + b->halo[mp.src[s].entity] : mb.n_edges[s];
    if (mb.sorted) {
      mt.hs_rows = mb.n_steps + mb.n_dst;
      for (int it = 0; it < p->T; ++it) {
        float* f = nullptr;
        // + one pad row: the resident training forward's tile headers point padding positions there
        // (resident.hip, hsb; its stores skip them, so the row stays unwritten)
        if ((rc = talloc(t.get(), &f, (mt.hs_rows + 1) * H))) return rc;
        mt.hs.push_back(f);
      }
      {
        const int64_t n_pos = (mb.n_dst + 15) / 16 * 16;
        float* f = nullptr;
        if ((rc = talloc(t.get(), &f, 4 * n_pos))) return rc;
        mt.hdrb = reinterpret_cast<int32_t*>(f);
        // on the upload stream, behind the block's IGN_POOL_POISON fill (pool_alloc) and before the
        // synchronisation at the end of this call: a launch on the plan stream could land first
        HIP_TRY(launch_seq_bwd_hdr(mb.d_seq_hdr, mb.d_step_code, n_pos, mt.hdrb, upload_stream()));
      }
      // source row -> steps whose input contains it (directly or through a pre-summed row)
      if (tcsr_on && mb.n_multi == 0) {
        if ((rc = tcsr_gpu(t.get(), mb, S, tkeys, true, mt.tptr, gidx))) return rc;
      } else build_csrs(S, tkeys, [&](auto&& emit) {
        auto add_row = [&](uint32_t trow, int32_t step) {
          for (int s = S - 1; s >= 0; --s)
            if ((int64_t)trow >= mb.src_off[s]) {
              emit(s, (int64_t)trow - mb.src_off[s], step);
              return;
            }
        };
        for (int64_t pos = 0; pos < mb.n_dst; ++pos)
          for (int32_t tt = 0; tt < mb.h_len[pos]; ++tt) {
            const int32_t i = mb.h_step_ptr[pos] + tt;
            const uint32_t code = mb.h_step_code[i];
            if ((int64_t)code < mb.zero_row) {
              add_row(code, i);
            } else if ((int64_t)code > mb.zero_row) {
              const int64_t k = code - mb.zero_row - 1;
              for (int32_t m = mb.h_multi_ptr[k]; m < mb.h_multi_ptr[k + 1]; ++m) add_row(mb.h_multi_rows[m], i);
            }
          }
      }, tptr, tidx);
      ga_n = std::max(ga_n, (mb.n_steps + 1) * 3 * H);   // + the pad slot row (seq_gru_bwd_kernel)
      gu_n = std::max(gu_n, mt.hs_rows * 3 * H);
      need_part(mt.hs_rows, H, 3 * H);
      if (p->bwd_fuse && seq_bwd_fused_supported(H)) part_n = std::max(part_n, seq_bwd_partial_floats(H));
      for (int s = 0; s < S; ++s) {
        dtab_n = std::max(dtab_n, mb.src_rows[s] * 3 * H);
        need_part(mb.src_rows[s], mp.feature_concat ? p->ents[mp.src[s].entity].hidden_dim : DIN, 3 * H);
      }
    } else {
      for (int it = 0; it < p->T; ++it) {
        float* f = nullptr;
        if ((rc = talloc(t.get(), &f, mb.n_dst * DIN))) return rc;
        mt.xs.push_back(f);
        if (mp.aggr == IGN_AGGR_CONVOLUTION) {
          if ((rc = talloc(t.get(), &f, mb.n_dst * DIN))) return rc;
          mt.ss.push_back(f);
        }
      }
      if (mp.aggr == IGN_AGGR_ATTENTION) {   // AUX:287-343: message -> destination row, row -> messages
        hvec<int32_t> mdst(mb.n_msgs);
        for (int64_t pos = 0; pos < mb.n_dst; ++pos)
          for (int32_t m = mb.h_msg_ptr[pos]; m < mb.h_msg_ptr[pos + 1]; ++m) mdst[m] = mb.h_order[pos];
        if ((rc = tupload(t.get(), &mt.amdst, mdst))) return rc;
        std::vector<hvec<std::pair<int64_t, int32_t>>> am(S);
        for (int64_t m = 0; m < mb.n_msgs; ++m)
          am[mb.h_msg_src[m] >> IGN_SLOT_SHIFT].push_back({(int64_t)(mb.h_msg_src[m] & IGN_ROW_MASK), (int32_t)m});
        for (int s = 0; s < S; ++s) {
          // a message network's codes address its edges (the per-edge message rows)
          const int64_t rows_s = mp.nn[s].layers.empty() ? b->rows[mp.src[s].entity] : mb.n_edges[s];
          hvec<int32_t> ptr, idx;
          build_csr(rows_s, am[s], ptr, idx);
          int32_t *dp = nullptr, *di = nullptr;
          if ((rc = tupload(t.get(), &dp, ptr)) || (rc = tupload(t.get(), &di, idx))) return rc;
          mt.asptr.push_back(dp);
          mt.asidx.push_back(di);
          arows_n = std::max(arows_n, rows_s);
          need_part(rows_s, DIN, 1);
        }
        amsg_n = std::max(amsg_n, mb.n_msgs);
        arows_n = std::max(arows_n, mb.n_dst);
        need_part(mb.n_dst, H, 1);
      }
      if (mp.aggr == IGN_AGGR_CONVOLUTION) {
        hvec<float> deg(mb.n_dst, 0.f);
        for (int64_t pos = 0; pos < mb.n_dst; ++pos)
          deg[mb.h_order[pos]] = (float)(mb.h_msg_ptr[pos + 1] - mb.h_msg_ptr[pos]);
        if ((rc = tupload(t.get(), &mt.deg, deg))) return rc;
        dtab_n = std::max(dtab_n, 2 * mb.n_dst * DIN);   // du and d(sum) of the convolution
        need_part(mb.n_dst, DIN, DIN);
      }
      if (tcsr_on) {
        if ((rc = tcsr_gpu(t.get(), mb, S, tkeys, false, mt.tptr, gidx))) return rc;
      } else build_csrs(S, tkeys, [&](auto&& emit) {
        for (int64_t pos = 0; pos < mb.n_dst; ++pos)
          for (int32_t m = mb.h_msg_ptr[pos]; m < mb.h_msg_ptr[pos + 1]; ++m) {
            const uint32_t code = mb.h_msg_src[m];
            emit((int)(code >> IGN_SLOT_SHIFT), (int64_t)(code & IGN_ROW_MASK), mb.h_order[pos]);
          }
      }, tptr, tidx);
      ga_n = std::max(ga_n, mb.n_dst * 3 * H);
      gu_n = std::max(gu_n, mb.n_dst * 3 * H);
      dx_n = std::max(dx_n, mb.n_dst * DIN);
      need_part(mb.n_dst, std::max(DIN, H), 3 * H);
    }
    need_part(std::max<int64_t>(mb.n_steps, mb.n_dst), 1, 3 * H);   // colsum
    for (int s = 0; s < S; ++s) {
      const int se = mp.src[s].entity;
      const MsgNN& nn = mp.nn[s];
      const int64_t rows_s = tkeys[s];
      if (gidx) {
        mt.tidx.push_back(gidx);   // (mt.tptr[s] set by tcsr_gpu)
      } else {
        int32_t *dp = nullptr, *di = nullptr;
        if ((rc = tupload(t.get(), &dp, tptr[s])) || (rc = tupload(t.get(), &di, tidx[s]))) return rc;
        mt.tptr.push_back(dp);
        mt.tidx.push_back(di);
      }
      mt.trows.push_back(rows_s);
      if (nn.layers.empty()) continue;
      // message network (GM:440-475): buffers for its backward, and the state row -> edge CSRs
      const int64_t ne = mb.n_edges[s];
      int widest = nn.din_pad;
      for (size_t l = 0; l < nn.layers.size(); ++l) {
        widest = std::max(widest, nn.layers[l].out);
        need_part(ne, l == 0 ? nn.din : nn.layers[l].in, nn.layers[l].out);
      }
      dmsg_n = std::max(dmsg_n, ne * nn.dout());
      mz_n = std::max(mz_n, ne * widest);
      mdin_n = std::max(mdin_n, ne * nn.din);
      hvec<int32_t> es(ne), ed(ne);
      HIP_TRY(hipMemcpyAsync(es.data(), mb.d_edge_src[s], ne * sizeof(int32_t), hipMemcpyDeviceToHost, upload_stream()));
      HIP_TRY(hipMemcpyAsync(ed.data(), mb.d_edge_dst[s], ne * sizeof(int32_t), hipMemcpyDeviceToHost, upload_stream()));
      HIP_TRY(hipStreamSynchronize(upload_stream()));
      HIP_TRY(upload_flush());
      hvec<std::pair<int64_t, int32_t>> ks(ne), kd(ne);
      for (int64_t e = 0; e < ne; ++e) {
        ks[e] = {es[e], (int32_t)e};
        kd[e] = {ed[e], (int32_t)e};
      }
      hvec<int32_t> p1, i1, p2, i2;
      build_csr(b->rows[se] + b->halo[se], ks, p1, i1);   // sources may be halo rows (edge-cut)
      build_csr(b->rows[mp.dst], kd, p2, i2);
      if ((rc = tupload(t.get(), &mt.nsrc_ptr[s], p1)) || (rc = tupload(t.get(), &mt.nsrc_idx[s], i1)) ||
          (rc = tupload(t.get(), &mt.ndst_ptr[s], p2)) || (rc = tupload(t.get(), &mt.ndst_idx[s], i2)))
        return rc;
    }
    t->mp.push_back(std::move(mt));
    bm.mark(mi == 0 ? "mp0" : mi == 1 ? "mp1" : "mp2+");
  }
  if ((rc = talloc(t.get(), &t->ga, ga_n)) || (rc = talloc(t.get(), &t->gu, gu_n)) ||
      (rc = talloc(t.get(), &t->dx, dx_n)) || (rc = talloc(t.get(), &t->dtab, dtab_n)))
    return rc;
  if (amsg_n && ((rc = talloc(t.get(), &t->adw, amsg_n)) || (rc = talloc(t.get(), &t->adv, amsg_n)) ||
                 (rc = talloc(t.get(), &t->ads_src, arows_n)) || (rc = talloc(t.get(), &t->ads_dst, arows_n)) ||
                 (rc = talloc(t.get(), &t->adw12, 2 * p->attn_F))))
    return rc;
  if (dmsg_n && ((rc = talloc(t.get(), &t->dmsg, dmsg_n)) || (rc = talloc(t.get(), &t->mz[0], mz_n)) ||
                 (rc = talloc(t.get(), &t->mz[1], mz_n)) || (rc = talloc(t.get(), &t->mdin, mdin_n))))
    return rc;
  // readout
  int64_t widest = p->ro_width;
  for (size_t l = 0; l < p->dense.size(); ++l) {
    const DenseP& d = p->dense[l];
    widest = std::max<int64_t>(widest, d.out);
    need_part(P, d.in, d.out);
    if (l + 1 < p->dense.size()) {
      float* f = nullptr;
      if ((rc = talloc(t.get(), &f, P * d.out))) return rc;
      t->act.push_back(f);
    }
  }
  if ((rc = talloc(t.get(), &t->dz[0], P * widest)) || (rc = talloc(t.get(), &t->dz[1], P * widest))) return rc;
  if (p->ro_in.size() > 1 &&
      ((rc = talloc(t.get(), &t->ro_x, P * p->ro_width)) || (rc = talloc(t.get(), &t->dro, P * p->ro_width))))
    return rc;
  // readout operations (GM:605-655)
  t->dT.assign(p->ro_t.size(), nullptr);
  {
    int64_t rz_n = 0, rcat_n = 0, ties_n = 0;
    for (size_t k = 0; k < p->ro_ops.size(); ++k) {
      const RoOp& op = p->ro_ops[k];
      const RoBatchOp& bo = b->ro[k];
      const int nout = op.type == IGN_RO_EXTEND ? 2 : 1;
      for (int j = 0; j < nout; ++j) {
        const RoTensor& to = p->ro_t[op.out + j];
        if ((rc = talloc(t.get(), &t->dT[op.out + j], space_rows(p, b, to) * to.width))) return rc;
      }
      const int64_t n = space_rows(p, b, p->ro_t[op.in[0]]);
      if (op.type == IGN_RO_NEURAL_NETWORK) {
        int widest = op.in_width, K = op.in_width;
        for (auto& d : op.layers) {
          widest = std::max(widest, d.out);
          need_part(n, K, d.out);
          K = d.out;
        }
        rz_n = std::max(rz_n, n * widest);
        if (op.in.size() > 1) rcat_n = std::max(rcat_n, n * op.in_width);
      } else if (op.type == IGN_RO_POOLING) {
        ties_n = std::max(ties_n, (int64_t)b->G * p->ro_t[op.in[0]].width);
      } else if (op.type == IGN_RO_EXTEND) {
        for (int j = 0; j < 2; ++j) {
          const std::vector<int32_t>& ix = bo.h_idx[j];
          hvec<std::pair<int64_t, int32_t>> kv(ix.size());
          for (size_t e2 = 0; e2 < ix.size(); ++e2) kv[e2] = {ix[e2], (int32_t)e2};
          hvec<int32_t> ptr, idx;
          build_csr(space_rows(p, b, p->ro_t[op.in[j]]), kv, ptr, idx);
          int32_t *dp = nullptr, *di = nullptr;
          if ((rc = tupload(t.get(), &dp, ptr)) || (rc = tupload(t.get(), &di, idx))) return rc;
          t->rx_ptr.push_back(dp);
          t->rx_idx.push_back(di);
        }
      }
    }
    if ((rz_n && ((rc = talloc(t.get(), &t->rz[0], rz_n)) || (rc = talloc(t.get(), &t->rz[1], rz_n)))) ||
        (rcat_n && (rc = talloc(t.get(), &t->rcat, rcat_n))) || (ties_n && (rc = talloc(t.get(), &t->rties, ties_n))))
      return rc;
  }
  if ((rc = talloc(t.get(), &t->part, part_n)) || (rc = talloc(t.get(), &t->bsum, (32 + 1) * 3 * 32))) return rc;
  if (const char* v = getenv("IGN_DEFER_WGRAD"); !v || atoi(v) != 0) {
    // the per-instance weight gradients of the plain sum and ordered MPs (ign_backward_mp): one slot
    // per (gradient tensor, shape), room for every instance of a backward
    struct Want { int64_t c, cb; int M, N, ones; int64_t chunks; };
    std::vector<Want> want;
    auto add = [&](int64_t c, int64_t cb, int M, int N, int64_t rows, int64_t min_slots = 0) {
      const int ones = cb >= 0;
      const int64_t ch = std::max(tsgemm_chunks(rows, M, N, ones), min_slots) * p->T;
      for (auto& w : want)
        if (w.c == c && w.cb == cb && w.M == M && w.N == N) { w.chunks += ch; return; }
      want.push_back({c, cb, M, N, ones, ch});
    };
    for (size_t mi = 0; mi < p->mps.size(); ++mi) {
      const MPP& mp = p->mps[mi];
      const MPB& mb = b->mp[mi];
      const CellP& cp = p->cells[mp.cell];
      bool nets = false;
      for (auto& nn : mp.nn) nets = nets || !nn.layers.empty();
      if (nets || mp.feature_concat) continue;
      const int H = cp.H, H3 = 3 * cp.H, DIN = mp.din;
      if (mp.sorted) {
        for (size_t s2 = 0; s2 < mp.src.size(); ++s2) add(cp.off_k, -1, DIN, H3, t->mp[mi].trows[s2]);
      } else if (mp.aggr == IGN_AGGR_SUM) {
        const int64_t fw = sum_bwd_fused_waves(mb.n_dst, DIN, H);   // the fused sum backward's partials
        add(cp.off_k, cp.off_b, DIN, H3, mb.n_dst, fw);
        add(cp.off_rk, cp.off_b + H3, H, H3, mb.n_dst, fw);
      }
    }
    for (size_t mi = 0; mi < p->mps.size(); ++mi) {   // the fused ordered backward's partials
      const MPP& mp = p->mps[mi];
      const CellP& cp = p->cells[mp.cell];
      if (!mp.sorted || !p->bwd_fuse || !seq_bwd_fused_supported(cp.H)) continue;
      const int64_t tiles = (b->mp[mi].n_dst + 15) / 16;
      const int64_t waves = std::min<int64_t>((tiles + 3) / 4 * 4, kBwdPartialWaves) * p->T;   // upper bound
      bool found = false;
      for (auto& d : t->defer_seq)
        if (d.cell == mp.cell) { d.cap += waves; found = true; }
      if (!found) t->defer_seq.push_back({mp.cell, cp.H, nullptr, waves, 0});
    }
    for (auto& d : t->defer_seq)
      if ((rc = talloc(t.get(), &d.part, (d.cap + kTsReduceSegs) * (int64_t)(d.H + 2) * 3 * d.H))) return rc;
    for (auto& w : want) {
      TrainState::DeferredGrad d{w.c, w.cb, w.M, w.N, w.ones, nullptr, w.chunks, 0};
      if ((rc = talloc(t.get(), &d.part, (w.chunks + kTsReduceSegs) * (int64_t)(w.M + w.ones) * w.N))) return rc;
      t->defer.push_back(d);
    }
  }
  bm.mark("rest");
  HIP_TRY(hipStreamSynchronize(upload_stream()));   // IGN_POOL_POISON fills have landed
  HIP_TRY(upload_flush());                           // (and every staged copy)
  bm.mark("wait");
  bm.print("ign_batch_enable_training fine");
  b->train = t.release();
  return IGN_OK;
}

int ign_forward_train_begin(ign_plan* p, ign_batch* b) {
  int rc = check_train(p, b);
  if (rc) return rc;
  TrainState* t = b->train;
  hipStream_t st = p->stream;
  const int E = (int)p->ents.size();
  for (int e = 0; e < E; ++e) {   // GM:396-400 (owned rows; an edge-cut driver fills the halo rows)
    HIP_TRY(launch_init_state(t->ver[e][0], b->d_feat[e], b->rows[e], p->ents[e].hidden_dim,
                              p->ents[e].feature_total, st));
    t->cur[e] = 0;
  }
  t->recs.clear();
  t->tab_saved = false;
  t->f_it = t->f_mi = 0;
  t->f_open = true;
  t->forward_done = false;
  return IGN_OK;
}

int ign_forward_train_mp(ign_plan* p, ign_batch* b) {
  int rc = check_train(p, b);
  if (rc) return rc;
  TrainState* t = b->train;
  if (!t->f_open || t->f_it >= p->T) return fail(IGN_ERR_INVALID, "ign_forward_train_mp outside begin .. end");
  hipStream_t st = p->stream;
  const int it = t->f_it, mi = t->f_mi;
  {
      const MPP& mp = p->mps[mi];
      const MPB& mb = b->mp[mi];
      const CellP& cp = p->cells[mp.cell];
      MPTrain& mt = t->mp[mi];
      MPRec rec{mi, it, t->cur[mp.dst], {0, 0, 0, 0}};
      SrcBases sb{};
      const float* srcs[IGN_MAX_SLOTS] = {nullptr, nullptr, nullptr, nullptr};
      for (size_t s = 0; s < mp.src.size(); ++s) {
        const int se = mp.src[s].entity;
        rec.src_v[s] = t->cur[se];
        srcs[s] = sb.base[s] = t->ver[se][t->cur[se]];
      }
      const float* hin = t->ver[mp.dst][rec.v_in];
      float* hout = t->ver[mp.dst][rec.v_in + 1];
      for (size_t s = 0; s < mp.src.size(); ++s) {   // message-creation networks (GM:440-475)
        if (mp.nn[s].layers.empty()) continue;
        if ((rc = run_message_net(p, mp.nn[s], mb, (int)s, srcs[s], hin, st))) return rc;
        srcs[s] = sb.base[s] = mb.d_msg_layer[s].back();
      }
      if (mp.sorted) {
        if ((rc = build_table(p, mp, mb, cp, srcs))) return rc;
        SeqGruArgs a{hin, hout, mb.d_table, mb.d_order, mb.d_len, mb.d_step_ptr, mb.d_step_code,
                     p->d_packed + cp.pk_u, p->d_packed + cp.pk_b, mb.n_dst, p->xcd_remap};
        a.hs_save = mt.hs[it];
        if (cp.pk_ubf >= 0) a.Ubf = p->d_packed + cp.pk_ubf;
        if (cp.pk_uh >= 0) a.Uh = p->d_packed + cp.pk_uh;
        a.hdr = mb.d_seq_hdr;
        HIP_TRY(launch_seq_gru(a, cp.H, train_seq_variant(p, cp.H), st));
      } else {
        SumGruArgs a{hin, hout, sb, mb.d_order, mb.d_msg_ptr, mb.d_msg_src, p->d_packed + cp.pk_w,
                     p->d_packed + cp.pk_u, p->d_packed + cp.pk_b, mb.n_dst, p->xcd_remap};
        a.x_save = mt.xs[it];
        if (mp.aggr == IGN_AGGR_ATTENTION) {     // AUX:287-343
          if ((rc = attention_weights(p, b, mp, mb, srcs, hin, st))) return rc;
          a.msg_w = mb.d_msg_w;
        }
        if (mp.aggr == IGN_AGGR_CONVOLUTION) {   // AUX:384-401
          a.conv_kp = p->d_packed + p->pk_conv;
          a.conv_act = mp.act;
          a.sum_save = mt.ss[it];
        }
        // 64-wide plain sums on the forward's default split-bf16 kernel (x_save supported); else f32
        if (p->sum_variant >= 7 && mp.aggr == IGN_AGGR_SUM && cp.pk_wbf >= 0 && cp.pk_ubf >= 0 && mp.din == cp.din &&
            !mp.feature_concat) {
          a.Wbf = p->d_packed + cp.pk_wbf;
          a.Ubf = p->d_packed + cp.pk_ubf;
        }
        HIP_TRY(launch_sum_gru(a, mp.din, cp.H, cp.H == 64 ? (a.Wbf ? 7 : 3) : std::min(p->sum_variant, 7), st));
      }
      t->cur[mp.dst] = rec.v_in + 1;
      t->recs.push_back(rec);
  }
  if (++t->f_mi == (int)p->mps.size()) {
    t->f_mi = 0;
    ++t->f_it;
  }
  return IGN_OK;
}

int ign_forward_train_end(ign_plan* p, ign_batch* b, float* pred_out) {
  int rc = check_train(p, b);
  if (rc) return rc;
  TrainState* t = b->train;
  if (!t->f_open || t->f_it != p->T) return fail(IGN_ERR_INVALID, "ign_forward_train_end before every MP ran");
  t->f_open = false;
  hipStream_t st = p->stream;
  const int E = (int)p->ents.size();
  // readout operations, then the predict stack with every activation kept (GM:605-629)
  std::vector<const float*> ent(E);
  for (int e = 0; e < E; ++e) ent[e] = t->ver[e][t->cur[e]];
  if (!p->ro_ops.empty() && (rc = readout_ops_run(p, b, st, ent.data()))) return rc;
  auto tensor = [&](int id) -> const float* { return id < E ? ent[id] : b->ro_buf[id]; };
  const int64_t P = b->n_pred;
  const float* x = tensor(p->ro_in[0]);
  if (p->ro_in.size() > 1) {
    int col = 0;
    for (int id : p->ro_in) {
      HIP_TRY(launch_concat_cols(t->ro_x, P, p->ro_width, col, tensor(id), p->ro_t[id].width, st));
      col += p->ro_t[id].width;
    }
    x = t->ro_x;
  }
  const float* in = x;
  int in_stride = p->ro_width;
  // the inference readout kernel (readout_h16) with its activations written out: one launch, no
  // re-read of layer 1's output (readout.cpp's fused-readout conditions, variant 4)
  const bool fused = p->train_fused_readout && p->fused_readout && p->readout_variant >= 4 && p->dense.size() == 3 &&
                     p->dense[1].pk_h >= 0 && p->dense[0].pk_bf >= 0 && p->dense[1].pk_bf >= 0 &&
                     p->dense[0].use_bias && p->dense[1].use_bias;
  if (fused) {
    const DenseP &l1 = p->dense[0], &l2 = p->dense[1], &l3 = p->dense[2];
    Readout3Args a{x, P, in_stride,
                   nullptr, p->d_params + l1.off_b,   // readout_h16 reads its pieces from pk_h only
                   nullptr, p->d_params + l2.off_b,
                   p->d_params + l3.off_w, l3.use_bias ? p->d_params + l3.off_b : nullptr,
                   l1.act, l2.act, l3.act, b->d_pred, t->act[0], t->act[1]};
    if (p->readout_variant == 5 && l2.pk_h32 >= 0)   // the inference kernel's variant (same predictions)
      HIP_TRY(launch_readout_h32(a, p->d_packed + l2.pk_h32, l1.in, st));
    else
      HIP_TRY(launch_readout_h16(a, p->d_packed + l2.pk_h, l1.in, st));
  }
  for (size_t l = 0; !fused && l < p->dense.size(); ++l) {
    const DenseP& d = p->dense[l];
    float* o = l + 1 == p->dense.size() ? b->d_pred : t->act[l];
    if (p->train_dense_bf && p->train_dense_h16 && d.pk_hn >= 0 && in_stride % 4 == 0)   // split-fp16 (x3)
      HIP_TRY(launch_dense_h16(in, P, d.in, in_stride, p->d_packed + d.pk_hn, d.use_bias ? p->d_params + d.off_b : nullptr,
                               d.out, d.act, o, st));
    else if (p->train_dense_bf && d.pk_bfn >= 0 && in_stride % 4 == 0)   // split-bf16, fp32-exact operands
      HIP_TRY(launch_dense_bf(in, P, d.in, in_stride, p->d_packed + d.pk_bfn, d.use_bias ? p->d_params + d.off_b : nullptr,
                              d.out, d.act, o, st));
    else
      HIP_TRY(launch_dense_fwd(in, P, d.in, in_stride, d.pk_w >= 0 ? p->d_packed + d.pk_w : nullptr,
                               p->d_params + d.off_w, d.use_bias ? p->d_params + d.off_b : nullptr, d.out, d.act, o, st));
    in = o;
    in_stride = d.out;
  }
  if (pred_out) {
    HIP_TRY(hipMemcpyAsync(pred_out, b->d_pred, P * b->out_units * sizeof(float), hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
  }
  t->forward_done = true;
  return IGN_OK;
}

// The training forward's whole MP loop as one graph-resident launch (resident.hip's SAVE form,
// DESIGN.md §3d) where the plan and batch allow it: the same states, per-step saves, message sums and
// versions as ign_forward_train_mp's launches, and the same MP-instance records for the backward
static int resident_train_forward(ign_plan* p, ign_batch* b, bool* done) {
  *done = false;
  int sum_mp[kResidentMaxSrc] = {-1, -1}, S = 0;
  // the resident form computes the ordered update with seq_gru_h16's arithmetic and leaves each
  // sequence's first and final state rows unsaved (the path versions hold them): only under the
  // backward that recomputes those gates and reads neither row (the fused split-fp16 one; the unfused
  // one contracts every hs row)
  // (the training form keeps its path states in global memory: IGN_RESIDENT_PG=0 turns it off too)
  if (!p->resident_train || !p->resident_pg || !resident_sum_mps(p, sum_mp, &S) || train_seq_variant(p, 32) != 6)
    return IGN_OK;
  int rc = resident_tables(p, b);
  if (rc || !b->resident) return rc;
  TrainState* t = b->train;
  const int path = p->mps[0].dst, T = p->T;
  int src_ent[kResidentMaxSrc] = {-1, -1};
  for (int s = 0; s < S; ++s) src_ent[s] = p->mps[0].src[s].entity;
  if ((int)t->ver[path].size() != T + 1) return IGN_OK;
  for (int s = 0; s < S; ++s)
    if ((int)t->ver[src_ent[s]].size() != T + 1) return IGN_OK;
  // pointer arrays: path versions [T + 1] | per source: versions [T + 1] | hs_save [T] | per source:
  // x_save [T] | the ordered MP's projected tables [T] (saved for the backward: no recompute)
  const int64_t n_ptr = (T + 1) * (1 + S) + T * (1 + S) + T;
  const MPB& m0 = b->mp[0];
  const bool save_tab = p->resident_save_table && m0.n_multi == 0;
  if (!t->res_ptrs) {
    for (int k = 0; k < T && save_tab; ++k) {
      float* f = nullptr;
      if ((rc = talloc(t, &f, (m0.zero_row + 1) * 3 * p->cells[p->mps[0].cell].H))) return rc;
      t->tsave.push_back(f);
    }
    hvec<float*> v;
    for (int k = 0; k <= T; ++k) v.push_back(t->ver[path][k]);
    for (int s = 0; s < S; ++s)
      for (int k = 0; k <= T; ++k) v.push_back(t->ver[src_ent[s]][k]);
    for (int k = 0; k < T; ++k) v.push_back(t->mp[0].hs[k]);
    for (int s = 0; s < S; ++s)
      for (int k = 0; k < T; ++k) v.push_back(t->mp[sum_mp[s]].xs[k]);
    for (int k = 0; k < T; ++k) v.push_back(save_tab ? t->tsave[k] : nullptr);
    if ((int64_t)v.size() != n_ptr) return fail(IGN_ERR_RUNTIME, "resident training pointers");
    if ((rc = tupload(t, &t->res_ptrs, v))) return rc;
  }
  ResidentSave sv{};
  sv.path_ver = t->res_ptrs;
  for (int s = 0; s < S; ++s) sv.src_ver[s] = t->res_ptrs + (T + 1) * (1 + s);
  sv.hs_save = t->res_ptrs + (T + 1) * (1 + S);
  for (int s = 0; s < S; ++s) sv.x_save[s] = t->res_ptrs + (T + 1) * (1 + S) + T * (1 + s);
  if (!t->tsave.empty()) sv.tab_save = t->res_ptrs + (T + 1) * (1 + S) + T * (1 + S);
  if ((rc = resident_launch(p, b, &sv))) return rc;
  t->tab_saved = !t->tsave.empty();
  // the records ign_forward_train_mp would have left (GM:404-603 order)
  for (int it = 0; it < T; ++it)
    for (int mi = 0; mi < (int)p->mps.size(); ++mi) {
      const MPP& mp = p->mps[mi];
      MPRec rec{mi, it, t->cur[mp.dst], {0, 0, 0, 0}};
      for (size_t s = 0; s < mp.src.size(); ++s) rec.src_v[s] = t->cur[mp.src[s].entity];
      t->cur[mp.dst] = rec.v_in + 1;
      t->recs.push_back(rec);
    }
  t->f_it = T;
  t->f_mi = 0;
  *done = true;
  return IGN_OK;
}

int ign_forward_train(ign_plan* p, ign_batch* b, float* pred_out) {
  int rc = ign_forward_train_begin(p, b);
  bool done = false;
  if (!rc) rc = resident_train_forward(p, b, &done);
  for (int k = 0; !rc && !done && k < p->T * (int)p->mps.size(); ++k) rc = ign_forward_train_mp(p, b);
  return rc ? rc : ign_forward_train_end(p, b, pred_out);
}

int ign_backward_begin(ign_plan* p, ign_batch* b, const float* dpred, float* grads, float l2_scale) {
  int rc = check_train(p, b);
  if (rc) return rc;
  if (!dpred || !grads) return fail(IGN_ERR_INVALID, "null argument");
  TrainState* t = b->train;
  if (!t->forward_done)
    return fail(IGN_ERR_INVALID, "ign_backward needs a preceding ign_forward_train (a backward consumes the "
                "forward's saved activations: one backward per forward)");
  // the readout backward below may write gradient rows over the saved activations (fuse_outer_bwd):
  // a second backward of the same forward would read them as activations
  t->forward_done = false;
  hipStream_t st = p->stream;
  const int E = (int)p->ents.size();
  const int64_t P = b->n_pred;
  set_tsgemm_bf(p->tsgemm_bf);
  HIP_TRY(hipMemsetAsync(grads, 0, p->n_params * sizeof(float), st));
  t->grads = grads;
  t->l2_scale = l2_scale;
  for (auto& d : t->defer) d.used = 0;   // (a backward that failed part-way leaves no stale partials)
  for (auto& d : t->defer_seq) d.used = 0;
  t->dcur.assign(E, 0);
  for (int e = 0; e < E; ++e)   // owned and halo rows (edge-cut: peers' gradients arrive in the owned rows)
    HIP_TRY(hipMemsetAsync(t->dS[0][e], 0, (b->rows[e] + b->halo[e]) * p->ents[e].hidden_dim * sizeof(float), st));

  // ---- readout (GM:605-629) in reverse: predict, then the operations before it
  for (size_t id = 0; id < t->dT.size(); ++id)
    if (t->dT[id])
      HIP_TRY(hipMemsetAsync(t->dT[id], 0, space_rows(p, b, p->ro_t[id]) * p->ro_t[id].width * sizeof(float), st));
  auto tensor = [&](int id) -> const float* { return id < E ? t->ver[id][t->cur[id]] : b->ro_buf[id]; };
  auto grad_of = [&](int id) -> float* { return id < E ? t->dS[0][id] : t->dT[id]; };
  const int L = (int)p->dense.size();
  const float* X = p->ro_in.size() > 1 ? t->ro_x : tensor(p->ro_in[0]);
  int zi = 0;
  HIP_TRY(launch_act_bwd(dpred, b->d_pred, P * p->dense[L - 1].out, p->dense[L - 1].act, t->dz[0], st));
  // a 1-unit output layer's backward rows, dz[r][k] = dz_out[r] w[k] act'(a[r][k]), are formed by
  // the layer below's input-gradient kernel (dense_bf) as it loads a, and written over a in place
  // for that layer's weight gradient: row_outer_t's separate read of a is gone
  OuterRows xo{};
  auto dense_t_bf = [&](const DenseP& d) { return p->train_dense_bf && (p->train_dense_h16 ? d.pk_ht >= 0 : d.pk_bft >= 0); };
  for (int l = L - 1; l >= 0; --l) {
    const DenseP& d = p->dense[l];
    const float* A = l == 0 ? X : t->act[l - 1];
    const bool outer = xo.s != nullptr;   // this layer's dz is formed by its dense_t from act[l]
    if (!outer)
      HIP_TRY(launch_tsgemm_add(A, d.in, t->dz[zi], d.out, P, d.in, d.out, t->part, grads + d.off_w,
                                d.use_bias ? grads + d.off_b : nullptr, st));
    if (l > 0 && d.out == 1 && d.in % 4 == 0 && p->fuse_outer_bwd && dense_t_bf(p->dense[l - 1])) {
      if (d.l2 != 0.f) HIP_TRY(launch_axpy(grads + d.off_w, p->d_params + d.off_w, 2.f * d.l2 * l2_scale, (int64_t)d.in * d.out, st));
      xo = OuterRows{t->dz[zi], p->d_params + d.off_w, p->dense[l - 1].act, t->act[l - 1]};
      continue;   // zi stays: dz[zi] holds dz_out for the layer below
    }
    if (!outer && d.l2 != 0.f)
      HIP_TRY(launch_axpy(grads + d.off_w, p->d_params + d.off_w, 2.f * d.l2 * l2_scale, (int64_t)d.in * d.out, st));
    float* out;
    int act = -1, acc = 0;
    const float* aprev = nullptr;
    if (l > 0) {
      out = t->dz[1 - zi];
      act = p->dense[l - 1].act;
      aprev = t->act[l - 1];
    } else if (p->ro_in.size() > 1) {
      out = t->dro;
    } else {
      out = grad_of(p->ro_in[0]);
      acc = 1;
    }
    const float* dzin = outer ? xo.out : t->dz[zi];
    if (p->train_dense_bf && p->train_dense_h16 && d.pk_ht >= 0)   // split-fp16 (x3)
      HIP_TRY(launch_dense_h16_t(dzin, P, d.out, p->d_packed + d.pk_ht, d.in, out, acc, act, aprev, st, xo));
    else if (p->train_dense_bf && d.pk_bft >= 0)   // split-bf16, fp32-exact operands
      HIP_TRY(launch_dense_bf_t(dzin, P, d.out, p->d_packed + d.pk_bft, d.in, out, acc, act, aprev, st, xo));
    else if (outer)
      return fail(IGN_ERR_RUNTIME, "on-the-fly output-layer gradient without a dense_bf backward");
    else if (d.pk_wt >= 0)
      HIP_TRY(launch_row_gemm_t(t->dz[zi], P, d.out, p->d_packed + d.pk_wt, d.in, out, acc, act, aprev, st));
    else
      HIP_TRY(launch_row_gemm_t_generic(t->dz[zi], P, d.out, p->d_params + d.off_w, d.in, out, acc, act, aprev, st));
    if (outer) {   // the weight gradient on the rows dense_t just wrote over act[l], then its l2 term
      HIP_TRY(launch_tsgemm_add(A, d.in, xo.out, d.out, P, d.in, d.out, t->part, grads + d.off_w,
                                d.use_bias ? grads + d.off_b : nullptr, st));
      if (d.l2 != 0.f)
        HIP_TRY(launch_axpy(grads + d.off_w, p->d_params + d.off_w, 2.f * d.l2 * l2_scale, (int64_t)d.in * d.out, st));
    }
    xo = OuterRows{};
    zi = 1 - zi;
  }
  if (p->ro_in.size() > 1) {   // split dX by columns into the input tensors (concat axis 1)
    int col = 0;
    for (int id : p->ro_in) {
      const int w = p->ro_t[id].width;
      HIP_TRY(launch_split_cols_add(grad_of(id), P, w, t->dro, p->ro_width, col, st));
      col += w;
    }
  }
  int xi = (int)t->rx_ptr.size();   // extend CSRs are stored in op order, two per op
  for (int k = (int)p->ro_ops.size() - 1; k >= 0; --k) {
    const RoOp& op = p->ro_ops[k];
    const RoBatchOp& bo = b->ro[k];
    const RoTensor& t0 = p->ro_t[op.in[0]];
    const int64_t n = space_rows(p, b, t0);
    switch (op.type) {
      case IGN_RO_NEURAL_NETWORK: {   // Readout_nn (AUX:1188-1211): Dense stack on concat(inputs)
        const int NL = (int)op.layers.size();
        int rz = 0;
        HIP_TRY(launch_act_bwd(t->dT[op.out], bo.out[0], n * op.layers[NL - 1].out, op.layers[NL - 1].act, t->rz[0], st));
        for (int l = NL - 1; l >= 0; --l) {
          const DenseP& d = op.layers[l];
          const int K = l == 0 ? op.in_width : op.layers[l - 1].out;
          const float* A = l > 0 ? bo.tmp[l - 1] : op.in.size() > 1 ? bo.cat : tensor(op.in[0]);
          HIP_TRY(launch_tsgemm_add(A, K, t->rz[rz], d.out, n, K, d.out, t->part, grads + d.off_w,
                                    d.use_bias ? grads + d.off_b : nullptr, st));
          if (d.l2 != 0.f) HIP_TRY(launch_axpy(grads + d.off_w, p->d_params + d.off_w, 2.f * d.l2 * l2_scale, (int64_t)K * d.out, st));
          if (l > 0) {
            HIP_TRY(launch_row_gemm_t_generic(t->rz[rz], n, d.out, p->d_params + d.off_w, K, t->rz[1 - rz], 0,
                                              op.layers[l - 1].act, bo.tmp[l - 1], st));
            rz = 1 - rz;
          } else if (op.in.size() > 1) {
            HIP_TRY(launch_row_gemm_t_generic(t->rz[rz], n, d.out, p->d_params + d.off_w, K, t->rcat, 0, -1, nullptr, st));
            int col = 0;
            for (int id : op.in) {
              const int w = p->ro_t[id].width;
              HIP_TRY(launch_split_cols_add(grad_of(id), n, w, t->rcat, op.in_width, col, st));
              col += w;
            }
          } else {
            HIP_TRY(launch_row_gemm_t_generic(t->rz[rz], n, d.out, p->d_params + d.off_w, K, grad_of(op.in[0]), 1, -1,
                                              nullptr, st));
          }
        }
        break;
      }
      case IGN_RO_POOLING:   // Pooling_operation (AUX:1165-1185)
        HIP_TRY(launch_pool_bwd(tensor(op.in[0]), bo.out[0], t->dT[op.out], t->rties, t0.width, bo.d_inoff, b->G, op.mode,
                                n, grad_of(op.in[0]), st));
        break;
      case IGN_RO_PRODUCT: {   // element_wise (AUX:1081-1088)
        const RoTensor& t1 = p->ro_t[op.in[1]];
        const RoTensor& to = p->ro_t[op.out];
        const int ag = t0.space == RS_GRAPH && to.space != RS_GRAPH, bg = t1.space == RS_GRAPH && to.space != RS_GRAPH;
        HIP_TRY(launch_product_bwd(t->dT[op.out], tensor(op.in[1]), t0.width, t1.width, to.width, ag, bg, bo.d_seg, b->G,
                                   n, grad_of(op.in[0]), st));
        HIP_TRY(launch_product_bwd(t->dT[op.out], tensor(op.in[0]), t1.width, t0.width, to.width, bg, ag, bo.d_seg, b->G,
                                   space_rows(p, b, t1), grad_of(op.in[1]), st));
        break;
      }
      case IGN_RO_EXTEND: {   // Extend_adjacencies (AUX:1236-1265): gathers, so scatter back per row
        xi -= 2;
        for (int j = 0; j < 2; ++j) {
          const RoTensor& tj = p->ro_t[op.in[j]];
          HIP_TRY(launch_csr_gather_cols_add(grad_of(op.in[j]), space_rows(p, b, tj), t->rx_ptr[xi + j], t->rx_idx[xi + j],
                                             t->dT[op.out + j], tj.width, 0, tj.width, 1, st));
        }
        break;
      }
    }
  }
  t->b_ri = (int)t->recs.size() - 1;
  t->b_open = true;
  return IGN_OK;
}

int ign_backward_mp(ign_plan* p, ign_batch* b) {
  int rc = check_train(p, b);
  if (rc) return rc;
  TrainState* t = b->train;
  if (!t->b_open || t->b_ri < 0) return fail(IGN_ERR_INVALID, "ign_backward_mp outside begin .. end");
  hipStream_t st = p->stream;
  hvec<int>& dcur = t->dcur;
  float* grads = t->grads;
  const int ri = t->b_ri--;
  {
    const MPRec& rec = t->recs[ri];
    const MPP& mp = p->mps[rec.mi];
    const MPB& mb = b->mp[rec.mi];
    const CellP& cp = p->cells[mp.cell];
    const MPTrain& mt = t->mp[rec.mi];
    const int dst = mp.dst, H = cp.H, DIN = mp.din, H3 = 3 * cp.H;
    float* dh_in = t->dS[dcur[dst]][dst];
    float* dh_out = t->dS[1 - dcur[dst]][dst];
    if (b->halo[dst])   // a self-loop MP's source gradient lands in dh_out's halo rows too
      HIP_TRY(hipMemsetAsync(dh_out + b->rows[dst] * H, 0, b->halo[dst] * H * sizeof(float), st));
    const float* srcs[IGN_MAX_SLOTS] = {nullptr, nullptr, nullptr, nullptr};
    for (size_t s = 0; s < mp.src.size(); ++s) srcs[s] = t->ver[mp.src[s].entity][rec.src_v[s]];
    for (size_t s = 0; s < mp.src.size(); ++s) {   // recompute this instance's message networks
      if (mp.nn[s].layers.empty()) continue;
      if ((rc = run_message_net(p, mp.nn[s], mb, (int)s, srcs[s], t->ver[dst][rec.v_in], st))) return rc;
      srcs[s] = mb.d_msg_layer[s].back();
    }
    auto src_grad = [&](size_t s) -> float* {      // where d(state of source s) accumulates
      const int se = mp.src[s].entity;
      return se == dst ? dh_out : t->dS[dcur[se]][se];
    };
    float* gk = grads + cp.off_k;
    float* grk = grads + cp.off_rk;
    float* gb = grads + cp.off_b;
    if (mp.sorted) {
      // the forward's table of this instance: saved by the resident training forward, else recomputed
      const bool saved = t->tab_saved && rec.mi == 0 && rec.it < (int)t->tsave.size();
      if (!saved && (rc = build_table(p, mp, mb, cp, srcs))) return rc;
      SeqBwdArgs a{mt.hs[rec.it], saved ? t->tsave[rec.it] : mb.d_table, mb.d_order, mb.d_len, mb.d_step_ptr, mb.d_step_code,
                   p->d_packed + cp.pk_u, p->d_packed + cp.pk_b, p->d_packed + cp.pk_ut, dh_in, dh_out,
                   t->ga, t->gu, mb.n_dst};
      a.h_in = t->ver[dst][rec.v_in];
      a.hdr = mt.hdrb;
      if (p->bwd_fuse && seq_bwd_fused_supported(H)) {
        // dU and both bias gradients (column sums of da and du) inside the kernel
        a.gu = nullptr;
        a.part = t->part;
        a.dU = grk;
        a.db_rec = gb + H3;
        a.db_in = gb;
        a.scratch = t->bsum;
        // gate recompute on the forward's path (bitwise the forward's gates): split-fp16 x3 after
        // seq_gru_h16<SAVE>, split-bf16 x6 after seq_gru_bf x6; IGN_BWD_BF=0 keeps the f32 MFMA recompute
        if (p->bwd_bf && H == 32 && cp.pk_uh >= 0 && cp.pk_uth >= 0 && train_seq_variant(p, H) == 6) {
          a.Uh = p->d_packed + cp.pk_uh;
          a.Uth = p->d_packed + cp.pk_uth;
        }
        else if (p->bwd_bf && H == 32 && cp.pk_ubf >= 0 && train_seq_variant(p, H) == 4) a.Ubf = p->d_packed + cp.pk_ubf;
        // the partials stay for one reduction per backward (ign_backward_end) where the cell has room
        const int64_t waves = seq_bwd_fused_waves(a, H);
        for (auto& d : t->defer_seq)
          if (d.cell == mp.cell && d.used + waves <= d.cap) {
            a.part = d.part + d.used * (int64_t)(H + 2) * H3;
            a.defer_reduce = true;
            d.used += waves;
            break;
          }
        HIP_TRY(launch_seq_gru_bwd(a, H, st));
      } else {
        HIP_TRY(launch_seq_gru_bwd(a, H, st));
        HIP_TRY(launch_tsgemm_add(mt.hs[rec.it], H, t->gu, H3, mt.hs_rows, H, H3, t->part, grk, gb + H3, st));
        HIP_TRY(launch_colsum_add(t->ga, H3, mb.n_steps, H3, t->part, gb, st));
      }
      for (size_t s = 0; s < mp.src.size(); ++s) {
        const int se = mp.src[s].entity;
        HIP_TRY(launch_csr_gather_add(t->dtab, mt.trows[s], mt.tptr[s], mt.tidx[s], t->ga, H3, 0, st));
        const bool net = !mp.nn[s].layers.empty();
        float* target = net ? t->dmsg : se == dst ? dh_out : t->dS[dcur[se]][se];
        if (mp.feature_concat) {   // AUX:443-456: the source's slice of the input kernel
          const int sdin = p->ents[se].hidden_dim;
          const int64_t koff = (int64_t)mp.slice_off[s] * H3;
          HIP_TRY(launch_tsgemm_add(srcs[s], sdin, t->dtab, H3, mt.trows[s], sdin, H3, t->part, gk + koff, nullptr, st));
          HIP_TRY(launch_row_gemm_t_generic(t->dtab, mt.trows[s], H3, p->d_params + cp.off_k + koff, sdin, target,
                                            net ? 0 : 1, -1, nullptr, st));
        } else {
          if ((rc = tsgemm_deferred(t, srcs[s], DIN, t->dtab, H3, mt.trows[s], DIN, H3, gk, nullptr, st))) return rc;
          HIP_TRY(launch_row_gemm_t(t->dtab, mt.trows[s], H3, p->d_packed + cp.pk_wt, DIN, target, net ? 0 : 1, -1,
                                    nullptr, st));
        }
        if (net && (rc = msg_net_backward(p, b, t, mp, mb, mt, (int)s, src_grad(s), dh_out, grads, st))) return rc;
      }
    } else {
      const float* hin = t->ver[dst][rec.v_in];
      SumBwdArgs a{mt.xs[rec.it], hin, p->d_packed + cp.pk_w, p->d_packed + cp.pk_u, p->d_packed + cp.pk_b,
                   p->d_packed + cp.pk_wt, p->d_packed + cp.pk_ut, dh_in, dh_out, t->dx, t->ga, t->gu, mb.n_dst};
      // plain sums at DIN = H = 32: dW / dU formed in the backward kernel, its partials into the
      // deferred slots (IGN_SUM_BWD_FUSE=0: da / du written, then the two row contractions; with no
      // deferred slot, IGN_DEFER_WGRAD=0, the unfused path runs whatever IGN_SUM_BWD_FUSE says)
      TrainState::DeferredGrad* dw = nullptr;
      TrainState::DeferredGrad* du = nullptr;
      const int64_t fw = mp.aggr == IGN_AGGR_SUM && p->sum_bwd_fuse ? sum_bwd_fused_waves(mb.n_dst, DIN, H) : 0;
      for (auto& d : t->defer) {
        if (fw && d.off_c == cp.off_k && d.off_cb == cp.off_b && d.M == DIN && d.N == H3 && d.used + fw <= d.cap) dw = &d;
        if (fw && d.off_c == cp.off_rk && d.off_cb == cp.off_b + H3 && d.M == H && d.N == H3 && d.used + fw <= d.cap) du = &d;
      }
      if (dw && du) {
        HIP_TRY(launch_sum_gru_bwd_fused(a, DIN, H, dw->part + dw->used * (int64_t)(DIN + 1) * H3,
                                         du->part + du->used * (int64_t)(H + 1) * H3, st));
        dw->used += fw;
        du->used += fw;
      } else {
        HIP_TRY(launch_sum_gru_bwd(a, DIN, H, st));
        if ((rc = tsgemm_deferred(t, mt.xs[rec.it], DIN, t->ga, H3, mb.n_dst, DIN, H3, gk, gb, st)) ||
            (rc = tsgemm_deferred(t, hin, H, t->gu, H3, mb.n_dst, H, H3, grk, gb + H3, st)))
          return rc;
      }
      if (mp.aggr == IGN_AGGR_ATTENTION) {   // AUX:287-343 (see train_kernels.hip)
        if ((rc = attention_weights(p, b, mp, mb, srcs, hin, st))) return rc;   // this instance's weights
        const int F = DIN;
        SrcBases sb{};
        for (size_t s = 0; s < mp.src.size(); ++s) sb.base[s] = srcs[s];
        AttnArgs aa{mb.d_group_ptr, mb.d_group_empty, mb.d_cell_dst, mb.d_cell_ptr, mb.d_cell_msgs, mb.d_msg_src,
                    {mb.d_s_src[0], mb.d_s_src[1], mb.d_s_src[2], mb.d_s_src[3]}, mb.d_s_dst, mb.d_ecell, mb.d_msg_w,
                    mb.n_groups};
        const float* w12 = p->d_packed + p->pk_w12;
        HIP_TRY(hipMemsetAsync(t->adw12, 0, 2 * p->attn_F * sizeof(float), st));
        HIP_TRY(launch_attn_bwd_parts(aa, t->dx, mt.amdst, sb, F, mb.n_msgs, t->adw, t->adv, st));
        for (size_t s = 0; s < mp.src.size(); ++s) {
          // over a message network the source rows are its per-edge messages: their gradient goes
          // through the network's backward to the states it read (GM:440-475)
          const bool net = !mp.nn[s].layers.empty();
          const int64_t rows_s = net ? mb.n_edges[s] : b->rows[mp.src[s].entity];
          if (net) HIP_TRY(hipMemsetAsync(t->dmsg, 0, rows_s * F * sizeof(float), st));
          HIP_TRY(launch_attn_src_bwd(rows_s, mt.asptr[s], mt.asidx[s], mb.d_msg_w, t->adv, mt.amdst, t->dx, w12, F,
                                      net ? t->dmsg : src_grad(s), t->ads_src, st));
          HIP_TRY(launch_tsgemm_add(srcs[s], F, t->ads_src, 1, rows_s, F, 1, t->part, t->adw12, nullptr, st));
          if (net && (rc = msg_net_backward(p, b, t, mp, mb, mt, (int)s, src_grad(s), dh_out, grads, st))) return rc;
        }
        HIP_TRY(launch_attn_dst_bwd(mb.n_dst, mb.d_order, mb.d_msg_ptr, t->adv, w12 + p->attn_F, H, dh_out, t->ads_dst,
                                    st));
        HIP_TRY(launch_tsgemm_add(hin, H, t->ads_dst, 1, mb.n_dst, H, 1, t->part, t->adw12 + p->attn_F, nullptr, st));
        HIP_TRY(launch_attn_param_bwd(t->adw12, p->d_params + p->off_k1, p->d_params + p->off_k2,
                                      p->d_params + p->off_att, p->attn_F, grads + p->off_k1, grads + p->off_k2,
                                      grads + p->off_att, st));
        dcur[dst] = 1 - dcur[dst];
        return IGN_OK;
      }
      const float* dmsgs = t->dx;   // gradient of the aggregated messages, by destination row
      if (mp.aggr == IGN_AGGR_CONVOLUTION) {
        // x = act((s.K + h) / deg): du = dx act'(x) / deg, dh += du, dK += s^T du, ds = du K^T
        float* du = t->dtab;
        float* ds = t->dtab + mb.n_dst * DIN;
        HIP_TRY(launch_conv_bwd(t->dx, mt.xs[rec.it], mt.deg, mb.n_dst, DIN, mp.act, du, dh_out, st));
        HIP_TRY(launch_tsgemm_add(mt.ss[rec.it], DIN, du, DIN, mb.n_dst, DIN, DIN, t->part, grads + p->off_conv, nullptr, st));
        HIP_TRY(launch_row_gemm_t_generic(du, mb.n_dst, DIN, p->d_params + p->off_conv, DIN, ds, 0, -1, nullptr, st));
        dmsgs = ds;
      }
      for (size_t s = 0; s < mp.src.size(); ++s) {
        const bool net = !mp.nn[s].layers.empty();
        float* target = net ? t->dmsg : src_grad(s);
        HIP_TRY(launch_csr_gather_add(target, mt.trows[s], mt.tptr[s], mt.tidx[s], dmsgs, DIN, net ? 0 : 1, st));
        if (net && (rc = msg_net_backward(p, b, t, mp, mb, mt, (int)s, src_grad(s), dh_out, grads, st))) return rc;
      }
    }
    dcur[dst] = 1 - dcur[dst];
  }
  return IGN_OK;
}

int ign_backward_end(ign_plan* p, ign_batch* b) {
  int rc = check_train(p, b);
  if (rc) return rc;
  TrainState* t = b->train;
  if (!t->b_open || t->b_ri >= 0) return fail(IGN_ERR_INVALID, "ign_backward_end before every MP instance ran");
  t->b_open = false;
  hipStream_t st = p->stream;
  float* grads = t->grads;
  if ((rc = tsgemm_deferred_flush(p, t, st))) return rc;
  for (auto& mp : p->mps)   // message-network l2 terms (AUX:833-834), once per step
    for (auto& nn : mp.nn)
      for (size_t l = 0; l < nn.layers.size(); ++l) {
        const DenseP& d = nn.layers[l];
        const int K = l == 0 ? nn.din : nn.layers[l - 1].out;
        if (d.l2 != 0.f) HIP_TRY(launch_axpy(grads + d.off_w, p->d_params + d.off_w, 2.f * d.l2 * t->l2_scale, (int64_t)K * d.out, st));
      }
  return IGN_OK;
}

int ign_batch_train_buffers(const ign_batch* b, int32_t e, float** state, float** grad) {
  if (!b || !b->train) return fail(IGN_ERR_INVALID, "training not enabled on this batch");
  const TrainState* t = b->train;
  if (e < 0 || e >= (int)t->ver.size()) return fail(IGN_ERR_INVALID, "entity %d out of range", e);
  if (state) *state = t->ver[e][t->cur[e]];
  if (grad) *grad = t->dS[t->dcur.empty() ? 0 : t->dcur[e]][e];
  return IGN_OK;
}

int ign_backward(ign_plan* p, ign_batch* b, const float* dpred, float* grads) {
  int rc = ign_backward_begin(p, b, dpred, grads, 1.f);
  while (!rc && b->train->b_ri >= 0) rc = ign_backward_mp(p, b);
  return rc ? rc : ign_backward_end(p, b);
}

int ign_mse_loss(ign_plan* p, const float* pred, const float* labels, int64_t n, float* dpred, double* loss) {
  if (!p || !pred || !labels || !dpred) return fail(IGN_ERR_INVALID, "null argument");
  if (n <= 0) return fail(IGN_ERR_INVALID, "empty prediction vector");
  int rc = ensure_device(p);
  if (rc) return rc;
  constexpr int NB = 256;
  if (!p->d_red) HIP_TRY(hipMalloc(&p->d_red, 1024 * sizeof(double)));
  HIP_TRY(launch_mse(pred, labels, n, dpred, p->d_red, NB, p->stream));
  if (loss) {
    double h[NB];
    HIP_TRY(hipMemcpyAsync(h, p->d_red, NB * sizeof(double), hipMemcpyDeviceToHost, p->stream));
    HIP_TRY(hipStreamSynchronize(p->stream));
    double s = 0;
    for (int i = 0; i < NB; ++i) s += h[i];
    *loss = s / (double)n;
  }
  return IGN_OK;
}

int ign_l2_loss(ign_plan* p, double* loss) {
  if (!p || !loss) return fail(IGN_ERR_INVALID, "null argument");
  if (!p->params_set) return fail(IGN_ERR_INVALID, "parameters not set (ign_plan_set_params)");
  int rc = ensure_device(p);
  if (rc) return rc;
  constexpr int NB = 64;
  if (!p->d_red) HIP_TRY(hipMalloc(&p->d_red, 1024 * sizeof(double)));
  double total = 0;
  std::vector<const DenseP*> layers;   // readout and message-network Dense layers (model.losses)
  for (auto& d : p->dense) layers.push_back(&d);
  for (auto& mp : p->mps)
    for (auto& nn : mp.nn)
      for (auto& d : nn.layers) layers.push_back(&d);
  for (const DenseP* dl : layers) {
    const DenseP& d = *dl;
    if (d.l2 == 0.f) continue;
    HIP_TRY(launch_sumsq(p->d_params + d.off_w, (int64_t)d.in * d.out, p->d_red, NB, p->stream));
    double h[NB];
    HIP_TRY(hipMemcpyAsync(h, p->d_red, NB * sizeof(double), hipMemcpyDeviceToHost, p->stream));
    HIP_TRY(hipStreamSynchronize(p->stream));
    double s = 0;
    for (int i = 0; i < NB; ++i) s += h[i];
    total += (double)d.l2 * s;
  }
  *loss = total;
  return IGN_OK;
}

int ign_adam_step(ign_plan* p, const float* grads, float* m, float* v, int64_t iteration, float lr, float beta1,
                  float beta2, float epsilon) {
  if (!p || !grads || !m || !v) return fail(IGN_ERR_INVALID, "null argument");
  if (!p->params_set) return fail(IGN_ERR_INVALID, "parameters not set (ign_plan_set_params)");
  if (iteration < 0) return fail(IGN_ERR_INVALID, "negative iteration");
  int rc = ensure_device(p);
  if (rc) return rc;
  const double tstep = (double)iteration + 1.0;
  const double lr_t = (double)lr * std::sqrt(1.0 - std::pow((double)beta2, tstep)) / (1.0 - std::pow((double)beta1, tstep));
  HIP_TRY(launch_adam(p->d_params, grads, m, v, p->n_params, (float)lr_t, beta1, beta2, epsilon, p->stream));
  return repack(p);
}

int ign_plan_get_params(ign_plan* p, float* host_out) {
  if (!p || !host_out) return fail(IGN_ERR_INVALID, "null argument");
  if (!p->params_set) return fail(IGN_ERR_INVALID, "parameters not set (ign_plan_set_params)");
  int rc = ensure_device(p);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(host_out, p->d_params, p->n_params * sizeof(float), hipMemcpyDeviceToHost, p->stream));
  HIP_TRY(hipStreamSynchronize(p->stream));
  return IGN_OK;
}

}  // extern "C"
