// engine_internal.h — plan / batch structures shared by engine.cpp (inference) and train.cpp
// (training).  Not part of the C ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstdarg>
#include <cstdint>
#include <memory>
#include <new>
#include <string>
#include <vector>

#include "../../include/ignmp.h"
#include "kernels.h"

struct TrainState;                 // train.cpp
void train_state_destroy(TrainState* t);

namespace ign {

int fail(int code, const char* fmt, ...);

// devpool.cpp: the plan's device-memory cache (batch and training buffers).  Blocks handed back by
// pool_release are reused once an event recorded on `after` has completed.  scratch: a block the
// caller does not fill on allocation (IGN_POOL_POISON=1 fills it with NaN, via the upload stream).
struct DevPool;
std::shared_ptr<DevPool> pool_create(int device);
hipError_t pool_alloc(DevPool* pool, void** out, size_t bytes, bool scratch);
void pool_release(DevPool* pool, const std::vector<void*>& blocks, hipStream_t after);
void pool_stats(DevPool* pool, int64_t* live_bytes, int64_t* idle_bytes);
bool pool_enabled(const DevPool* pool);
void pool_trim_idle(DevPool* pool);   // every idle block, waiting for its fence
void host_cache_trim();               // every idle host block

// devpool.cpp: process-wide cache of large host blocks (>= kHostBlockMin bytes) for the batch
// builders' index tables.  A batch touches ~10^8 bytes of fresh host memory; straight from malloc
// that is mmap + page faults on every batch and munmap on destroy, serialised on the process's
// address-space lock across the input workers.  Cached blocks keep their pages (transparent huge
// pages where the kernel allows) and are pinned for DMA uploads where the runtime allows.
constexpr size_t kHostBlockMin = (size_t)1 << 20;
void* host_block_alloc(size_t bytes);
void host_block_free(void* p, size_t bytes);
template <class T>
struct HostAlloc {
  using value_type = T;
  HostAlloc() = default;
  template <class U>
  HostAlloc(const HostAlloc<U>&) {}
  T* allocate(size_t n) {
    const size_t bytes = n * sizeof(T);
    void* p = bytes >= kHostBlockMin ? host_block_alloc(bytes) : std::malloc(std::max<size_t>(bytes, 1));
    if (!p) throw std::bad_alloc();
    return static_cast<T*>(p);
  }
  void deallocate(T* p, size_t n) {
    const size_t bytes = n * sizeof(T);
    if (bytes >= kHostBlockMin) host_block_free(p, bytes);
    else std::free(p);
  }
  template <class U>
  bool operator==(const HostAlloc<U>&) const { return true; }
  template <class U>
  bool operator!=(const HostAlloc<U>&) const { return false; }
};
template <class T>
using hvec = std::vector<T, HostAlloc<T>>;
#define HIP_TRY(expr)                                                                             \
  do {                                                                                            \
    hipError_t _e = (expr);                                                                       \
    if (_e != hipSuccess) return fail(IGN_ERR_DEVICE, "%s: %s", #expr, hipGetErrorString(_e));    \
  } while (0)

enum { K_INIT = 0, K_SEQ = 1, K_SUM = 2, K_READOUT = 3, K_PROJECT = 4, K_OTHER = 5, K_RESIDENT = 6, K_KINDS = 7 };

// per timed launch: algorithmic FLOPs / bytes and the FLOPs its MFMAs execute (bf16 / f32 pipe)
struct EvCost {
  double flops = 0, bytes = 0, mfma_bf16 = 0, mfma_f32 = 0;
};
constexpr double kMfmaBf16Flops = 2.0 * 16 * 16 * 32;   // v_mfma_f32_16x16x32_bf16
constexpr double kMfmaF32Flops = 2.0 * 16 * 16 * 4;     // v_mfma_f32_16x16x4_f32

struct Tensor {
  int kind, owner;
  int64_t offset;
  int rows, cols;
};

struct CellP {
  int din, H;
  int64_t off_k, off_rk, off_b;   // raw Keras-layout params
  int64_t pk_w, pk_u, pk_b;       // packed fragments (in d_packed)
  int64_t pk_wt = -1, pk_ut = -1; // backward: unscaled W^T / U^T fragments (pack_a)
  int64_t pk_wbf = -1;            // split-bf16 input-kernel fragments (sum variant 7, DIN = H = 64)
  int64_t pk_ubf = -1;            // split-bf16 recurrent-kernel fragments (seq variants 4/5)
  int64_t pk_wh = -1;             // split-fp16 input-kernel fragments + scale (sum variant 8, DIN = H = 64)
  int64_t pk_uh = -1;             // split-fp16 recurrent-kernel fragments + scale (seq variants 6/7)
  int64_t pk_uth = -1;            // backward: split-fp16 U fragments for dh = du . U^T (H = 32)
  bool used = false;
};

struct DenseP {
  int in, out, act, use_bias;
  float l2 = 0.f;
  int64_t off_w, off_b, pk_w = -1;   // pk_w: forward fragments (fused readout, training readout)
  int64_t pk_wt = -1;             // backward: A fragments of W [in][out] (row_gemm_t), if supported
  int64_t pk_bf = -1;             // fused readout: split-bf16 A fragments (readout variants 2/3)
  int64_t pk_h = -1;              // fused readout, layer 2: scaled split-fp16 fragments (readout variant 4)
  int64_t pk_h32 = -1;            // ... the same pieces in variant 5's order (readout_h32.hip)
  int64_t pk_bfn = -1;            // training forward: split-bf16 pieces, natural k (dense_bf)
  int64_t pk_bft = -1;            // training backward: split-bf16 pieces of W^T (dense_bf_t)
  int64_t pk_hn = -1, pk_ht = -1;  // training: scaled split-fp16 pieces of W / W^T (dense_h16)
};

struct MsgNN {                    // message-creation network of one MP source (GM:440-475)
  std::vector<int> inputs;        // enum ign_message_input, in order
  std::vector<int> widths;        // floats per edge of each input part
  int param_dim = 0;
  int din = 0, din_pad = 0;       // concatenated input width, padded to 16 for the MFMA layers
  std::vector<DenseP> layers;
  int dout() const { return layers.empty() ? 0 : layers.back().out; }
};

struct MPP {
  int dst, aggr, concat_axis, cell;
  std::vector<ign_source_desc> src;
  bool sorted;                    // sorted (sequence) update vs single-step update
  int din;
  int act = 0;                    // convolution activation (AUX:370-374)
  bool feature_concat = false;    // concat on axis 2 (AUX:443-456): step input = [src_1 | src_2 | ...]
  std::vector<int> slice_off;     // feature_concat: first kernel row of each source's slice
  std::vector<int64_t> pk_slice;  // feature_concat: packed W-slice fragments per source
  std::vector<MsgNN> nn;          // per source; no layers = direct_assignation
};


struct MPB {
  bool sorted = false;
  int64_t n_dst = 0, n_steps = 0, n_msgs = 0, edges = 0;
  int64_t wave_steps = 0;          // sorted MPs: sum over 16-row tiles of the tile's longest sequence
  int32_t* d_order = nullptr;
  int32_t* d_len = nullptr;
  int32_t* d_step_ptr = nullptr;
  int32_t* d_msg_ptr = nullptr;
  uint32_t* d_msg_src = nullptr;
  uint32_t* d_step_code = nullptr;
  int32_t* d_seq_hdr = nullptr;   // sorted MPs: per order position {order, len, step_ptr, first code} (SeqGruArgs::hdr)
  float* d_table = nullptr;       // sorted MPs: [sources' rows | zero row | multi rows][3H]
  std::vector<int64_t> src_off;   // first table row of each source
  std::vector<int64_t> src_rows;
  int64_t zero_row = 0, n_multi = 0;
  int64_t n_interior = 0;         // sum MPs: order[0, n_interior) reads no halo row
  int32_t* d_multi_ptr = nullptr;
  uint32_t* d_multi_rows = nullptr;
  // attention (AUX:264-343): per-message softmax weights over dense (destination, position)
  // cells, grouped per (graph, position) for the axis-0 softmax
  int64_t n_cells = 0, n_groups = 0;
  float* d_msg_w = nullptr;       // [n_msgs] in CSR order
  int32_t* d_group_ptr = nullptr; // [n_groups + 1] cell ranges
  int32_t* d_group_empty = nullptr;
  int32_t* d_cell_dst = nullptr;
  int32_t* d_cell_ptr = nullptr;  // [n_cells + 1] ranges of d_cell_msgs
  int32_t* d_cell_msgs = nullptr; // CSR message positions
  float* d_ecell = nullptr;
  float* d_s_src[IGN_MAX_SLOTS] = {nullptr, nullptr, nullptr, nullptr};
  float* d_s_dst = nullptr;
  // message networks: per source, the per-edge input, the layer outputs (last = the messages)
  int64_t n_edges[IGN_MAX_SLOTS] = {0, 0, 0, 0};
  int32_t* d_edge_src[IGN_MAX_SLOTS] = {nullptr, nullptr, nullptr, nullptr};
  int32_t* d_edge_dst[IGN_MAX_SLOTS] = {nullptr, nullptr, nullptr, nullptr};
  float* d_edge_params[IGN_MAX_SLOTS] = {nullptr, nullptr, nullptr, nullptr};
  float* d_msg_in[IGN_MAX_SLOTS] = {nullptr, nullptr, nullptr, nullptr};
  std::vector<float*> d_msg_layer[IGN_MAX_SLOTS];
  // windowed sum (SumWinArgs; single-source sums over graph-local rows): the aggregation runs per
  // (graph, destination chunk) from LDS windows, then the GRU step reads x through an identity CSR
  int64_t n_win_wg = 0;
  bool sum_seg = false;        // segmented sum (sum_seg_kernel) into d_xsum, then the GRU step
  int64_t n_seg = 0;           // ... for order positions [0, n_seg): destinations with >= 64 messages
                               // (seg_min_messages); the GRU step reads their x from d_xsum (slot 1)
  int64_t* d_win_wg = nullptr;
  int32_t* d_win_dst = nullptr;
  int32_t* d_win_ptr = nullptr;
  int32_t* d_win_src = nullptr;
  float* d_xsum = nullptr;
  int32_t* d_id_ptr = nullptr;
  uint32_t* d_id_src = nullptr;
  double flops = 0, bytes = 0;    // algorithmic, per launch
  // host copies of the index tables (the training path builds their transposes)
  hvec<int32_t> h_order, h_len, h_step_ptr, h_msg_ptr, h_multi_ptr;
  hvec<uint32_t> h_step_code, h_msg_src, h_multi_rows;
};

// readout program (GM:611-655): tensors on row spaces, operations before predict
enum { RS_ENTITY = 0, RS_GRAPH = 1, RS_ADJ = 2 };
struct RoTensor {
  int space = RS_ENTITY, sid = 0;   // sid: entity or adjacency slot
  int width = 0;
  bool same_space(const RoTensor& o) const { return space == o.space && (space == RS_GRAPH || sid == o.sid); }
};
struct RoOp {
  int type = 0, mode = 0, adj = -1;
  std::vector<int> in;            // tensor ids
  std::vector<DenseP> layers;     // IGN_RO_NEURAL_NETWORK
  int in_width = 0;               // neural_network: concatenated input width
  int out = -1;                   // first output tensor id
};
struct RoBatchOp {
  float* out[2] = {nullptr, nullptr};
  float* cat = nullptr;           // neural_network: concatenated input
  std::vector<float*> tmp;        // neural_network: hidden layer outputs
  int32_t* idx[2] = {nullptr, nullptr};   // extend: global source / destination rows per edge
  // pooling: chunks of <= POOL_CHUNK rows, per-graph chunk ranges, partial results
  int64_t n_chunks = 0;
  int64_t* d_chunk = nullptr;     // [n_chunks][2] global row ranges
  int32_t* d_chunk_ptr = nullptr; // [G + 1]
  int64_t* d_count = nullptr;     // [G] rows per graph
  float* d_partial = nullptr;     // [n_chunks][F]
  int64_t* d_seg = nullptr;       // product: [G + 1] row offsets of the output space
  int64_t* d_inoff = nullptr;     // pooling: [G + 1] row offsets of the input space (backward)
  std::vector<int32_t> h_idx[2];  // extend: host copies of idx (the backward's transposed CSRs)
};

}  // namespace ign

using namespace ign;

struct ign_plan {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  bool external_stream = false;   // set by ign_plan_set_stream (may be the null stream)
  int T = 0;
  std::vector<ign_entity_desc> ents;
  int n_adj = 0, n_il = 0;
  std::vector<MPP> mps;
  std::vector<CellP> cells;
  std::vector<int> ro_in;         // predict inputs: readout tensor ids
  std::vector<DenseP> dense;
  std::vector<RoTensor> ro_t;     // readout tensors: entity states, then the op outputs
  std::vector<RoOp> ro_ops;
  std::vector<int> adj_src_ent, adj_dst_ent;   // per adjacency slot (from the MPs that read it)
  // one convolution / attention weight set per plan (GM:288-300: the last MP's weights serve all)
  int conv_F = 0, attn_F = 0;
  int64_t off_conv = -1, off_k1 = -1, off_k2 = -1, off_att = -1;
  int64_t pk_conv = -1, pk_w12 = -1;
  std::vector<Tensor> tensors;
  int64_t n_params = 0, n_packed = 0;
  float* d_params = nullptr;
  float* d_packed = nullptr;
  bool params_set = false;
  bool fused_readout = false;
  int readout_variant = 4;        // fused readout: 4 = both layers on split-fp16 (3 products) on 16x16x32 MFMAs
                                  // (readout_h16), 5 = the same on 32x32x16 (readout_h32.hip, slower: DESIGN
                                  // §3b), 1 = f32
                                  // MFMA (readout3), 2 = split-bf16 x6 (readout_bf); IGN_READOUT_VARIANT
  int ro_width = 0;
  int seq_variant = 6;            // ordered update: 6 = split-fp16 h.U with 3 piece products (H = 32,
                                  // 64), 4 = split-bf16 x6, 2 = f32 MFMA; IGN_SEQ_VARIANT
  int xcd_remap = 0;              // XCD-aware tile order in the GRU kernels (placement only; off:
                                  // measured slower, profiles/r02/seq_experiments)
  bool fuse_proj = true;          // sum_gru_g32 projects for the next ordered MP (IGN_FUSE_PROJ=0: off)
  int sum_variant = 8;            // sum update: 8 = split-fp16 GRU step at DIN = H = 64 and split-bf16
                                  // at 32, 7 = split-bf16 at both, 3 = f32 MFMA; IGN_SUM_VARIANT
  bool train_dense_bf = true;     // training forward's Dense layers on dense_bf (IGN_TRAIN_DENSE_BF=0: f32)
  bool train_dense_h16 = true;    // ... on the split-fp16 form of dense_bf (IGN_TRAIN_DENSE_H16=0: split-bf16)
  bool tsgemm_bf = true;          // weight-gradient row contractions on tsgemm_bf (IGN_TSGEMM_BF=0: f32 MFMA)
  bool train_fused_readout = true;   // training forward's readout on readout_h16 with saves (IGN_TRAIN_FUSED_READOUT=0: per layer)
  bool fuse_outer_bwd = true;     // 1-unit output layer's backward formed on the fly (IGN_FUSE_OUTER_BWD=0: row_outer_t)
  bool bwd_bf = true;             // ordered backward's gate recompute on split-bf16 (IGN_BWD_BF=0: f32 MFMA)
  bool train_seq_h16 = true;      // training forward's ordered update on split-fp16 (IGN_TRAIN_SEQ_H16=0: bf16)
  bool bwd_fuse = true;           // ordered backward forms dU in the kernel (IGN_BWD_FUSE=0: tsgemm)
  bool sum_bwd_fuse = true;       // sum backward forms dW / dU in the kernel (IGN_SUM_BWD_FUSE=0: tsgemm)
  bool resident = true;           // graph-resident forward for small RouteNet-shaped graphs (IGN_RESIDENT=0: off)
  bool resident_pg = true;        // ... with the path states in global memory where they do not fit LDS (IGN_RESIDENT_PG)
  bool resident_path_global = false;   // IGN_RESIDENT=2: that form for every eligible batch (tests)
  bool resident_train = true;     // the training forward on the resident form's SAVE variant (IGN_RESIDENT_TRAIN=0: off)
  bool res_lpt = true;            // resident workgroups take their graphs longest first (IGN_RES_LPT=0: batch order)
  int res_group = 0;              // consecutive graphs per resident workgroup (IGN_RES_GROUP; 0: auto, 1 or 2)
  bool resident_save_table = true;   // ... which also saves the ordered MP's tables (IGN_RESIDENT_SAVE_TABLE=0: recompute)
  int sum_window = -1;            // IGN_SUM_WINDOW: 1 windowed sum aggregation where eligible; -1 (default)
                                  // segmented for destinations of >= 64 messages, 0 of >= 128, 2 for all.
                                  // (The windowed form:)
                                  // Measured 0.120 vs 0.112 ms (RouteNet link update, 37 messages per link);
                                  // Q-size x512 7.33 -> 6.44 ms/step with both sum MPs windowed
  // timing
  bool timing = false;
  uint32_t timing_kinds = ~0u;    // kernel kinds that get event pairs (ign_plan_set_timing_kinds)
  std::vector<hipEvent_t> ev;     // pairs
  std::vector<int> ev_kind;
  std::vector<EvCost> ev_cost;
  int ev_slot = 0;                // events recorded since ign_forward_begin
  double* d_red = nullptr;        // loss reductions (training)
  bool use_graph = true;          // replay ign_forward as one captured hipGraph; IGN_HIP_GRAPH=0 disables
  ign_stats_t stats{};
  std::shared_ptr<DevPool> pool;  // batch / training buffers (created with the stream, ensure_device)
  std::string describe;           // ign_plan_create_json: ign_plan_describe_json's document
};

// the ordered update of the training forward saves every step's state, which the split-fp16 kernels
// (variant 6 at H = 64) do not: training runs the x6 split-bf16 form there
// the training forward's ordered update: split-fp16 x3 with state saving (seq_gru_h16<SAVE>) where
// the backward can recompute its gates bitwise (fused seq_gru_bwd, H = 32; IGN_TRAIN_SEQ_H16=0: the
// split-bf16 x6 form), else split-bf16 x6 / f32
inline int train_seq_variant(const ign_plan* p, int H) {
  if (p->seq_variant == 6 && H == 32 && p->train_seq_h16 && p->bwd_bf && p->bwd_fuse) return 6;
  return p->seq_variant >= 6 ? 4 : std::max(2, p->seq_variant);
}


struct ign_batch {
  ign_plan* plan = nullptr;
  int G = 0;
  std::vector<int64_t> rows;                    // per entity (owned rows)
  std::vector<int64_t> halo;                    // per entity: peer rows after the owned ones (§8e)
  std::vector<std::vector<int64_t>> row_off;    // [entity][graph]
  std::vector<float*> d_feat;                   // per entity [rows][F] or null
  std::vector<float*> d_state[2];               // per entity ping-pong
  std::vector<int> cur;
  std::vector<MPB> mp;
  // forward_body only: a sum update may project its new states for the next ordered MP that reads
  // them (fused_proj_target); proj_ready[m'] tells m' that its table is already filled
  bool fuse_ok = false, fuse_last_iter = false;
  // the graph-resident forward (resident.hip, plan->resident): per-graph offsets, the ordered MP's
  // per-graph tile headers, the sum MP's per-graph CSR (local rows); dynamic LDS of the largest graph
  bool resident = false;
  bool res_tried = false;         // resident_batch ran (lazily, at the first ign_forward)
  size_t res_lds = 0;
  int res_form = 0;               // IGN_RES_ALL_LDS / IGN_RES_PATH_GLOBAL / IGN_RES_PATH_CSR_GLOBAL
  int res_graphs = 0;             // resident workgroups per launch (graphs / IGN_RES_GROUP)
  ign_resident_info_t res_info{}; // per launch: bytes (compulsory, round trips, SURVEY B_stage), FLOPs,
                                  // MFMA FLOPs, tile-steps (ign_batch_resident_info)
  int64_t* d_res_path_off = nullptr;
  int64_t* d_res_src_off[kResidentMaxSrc] = {nullptr, nullptr};
  int64_t* d_res_urow_off = nullptr;
  int32_t* d_res_ptile_off = nullptr;
  int32_t* d_res_hdr = nullptr;
  int32_t* d_res_lmsg_off = nullptr;
  int32_t* d_res_lmsg_ptr = nullptr;
  uint16_t* d_res_lmsg_src = nullptr;
  uint16_t* d_res_lorder = nullptr;
  int32_t* d_res_lnseg = nullptr;
  int32_t* d_res_gorder = nullptr;   // workgroup -> graph, by estimated cost, descending (IGN_RES_LPT)
  int32_t* d_res_lcode_off = nullptr;
  uint16_t* d_res_lcode = nullptr;
  int32_t* d_res_hsb = nullptr;   // per header: the training forward's hs_save row of the position
  int res_train_form = 0;         // the training forward's form (path states in global memory) ...
  size_t res_train_lds = 0;       // ... and its dynamic LDS
  std::vector<char> proj_ready;
  float* d_ro_in = nullptr;                     // concat scratch (multi-input readout)
  std::vector<float*> d_ro_tmp;                 // generic readout intermediates
  std::vector<RoBatchOp> ro;                    // readout ops
  std::vector<float*> ro_buf;                   // per readout tensor: op output buffer (null for states)
  std::vector<int64_t> adj_rows;                // per adjacency: edges in the batch
  std::vector<std::vector<int64_t>> adj_off;    // [adjacency][graph + 1] edge offsets
  float* d_pred = nullptr;
  int64_t n_pred = 0, out_units = 1;
  int64_t edges_per_forward = 0, gru_steps = 0;
  std::vector<void*> allocs;                    // blocks of pool (returned on destroy)
  std::shared_ptr<DevPool> pool;                // the plan's (outlives the plan if need be)
  TrainState* train = nullptr;                  // ign_batch_enable_training
  // captured ign_forward (init .. readout) for replay; the event slots it records
  hipGraphExec_t graph = nullptr;
  bool graph_timing = false;
  std::vector<int> graph_kind;
  std::vector<EvCost> graph_cost;
};

namespace ign {
// the graph-resident forward (engine.cpp, resident.hip): save = the training forward's state versions
struct ResidentSave {
  float* const* path_ver;                    // [T + 1] the path entity's versions
  float* const* src_ver[kResidentMaxSrc];    // [T + 1] per source entity of the ordered MP
  float* const* hs_save;                     // [T] the ordered MP's per-step states
  float* const* x_save[kResidentMaxSrc];     // [T] per source entity: its sum MP's message sums
  float* const* tab_save = nullptr;          // [T] optional: the ordered MP's projected table per iteration
};
int resident_tables(ign_plan* p, ign_batch* b);   // once per batch; leaves b->resident false if not eligible
int resident_launch(ign_plan* p, ign_batch* b, const ResidentSave* save);
int resident_sum_mps(const ign_plan* p, int* sum_mp, int* n_src);   // 0: not a resident plan shape
int set_device(int dev);
int ensure_device(ign_plan* p);
int dev_alloc(ign_batch* b, float** out, int64_t n);
int repack(ign_plan* p);                      // fragments from d_params (set_params, optimizer)
// message-creation network of MP source s (GM:440-475): per-edge inputs, then the Dense stack into
// mb.d_msg_layer[s] (the last layer's rows are the messages)
int run_message_net(ign_plan* p, const MsgNN& nn, const MPB& mb, int s, const float* src_state,
                    const float* dst_state, hipStream_t st);
// attention weights of one MP instance (AUX:287-343) into mb.d_msg_w (scores in mb.d_s_src / d_s_dst)
int attention_weights(ign_plan* p, ign_batch* b, const MPP& mp, const MPB& mb, const float* const* srcs,
                      const float* hin, hipStream_t st);
// readout.cpp: the readout program (operations before predict, GM:611-655)
int readout_plan(ign_plan* p, const ign_plan_desc* d);          // parse + row spaces + widths
int64_t readout_layout(ign_plan* p, int64_t off);              // raw parameter tensors (kinds 11/12)
int64_t readout_packed(ign_plan* p, int64_t pk);               // packed Dense fragments
int readout_repack(ign_plan* p);
int readout_batch(ign_plan* p, ign_batch* b, const ign_batch_desc* d);
// ent: entity-state tensors to read (training keeps every version); null = the batch's current states
int readout_ops_run(ign_plan* p, ign_batch* b, hipStream_t st, const float* const* ent = nullptr);
const float* readout_tensor(const ign_plan* p, const ign_batch* b, int id);
int64_t space_rows(const ign_plan* p, const ign_batch* b, const RoTensor& t);
// Batch construction (ign_batch_create, ign_batch_enable_training) copies and clears on a
// non-blocking stream of the calling host thread, never the legacy null stream: a batch built on a
// worker thread does not wait for, or serialise with, the GPU step running on the engine's stream
// (the training input pipeline overlaps them, ignnition_amd/training.py BatchPrefetcher).
hipStream_t upload_stream();
// Host -> device copies of the batch builders.  Inside an UploadScope (ign_batch_create,
// ign_batch_enable_training) a copy of up to 4 MiB goes through the thread's pinned staging arena
// and is not waited for: the scope waits once, at its end, for all of them (a builder used to wait
// for every one of ~10^2 small copies, and eight builders waiting on the runtime at once stretched
// each stage 2-4x).  Larger copies, and every copy outside a scope, are waited for at once (their
// source may die after the call).  IGN_UPLOAD_DEFER=0 waits for every copy.  IGN_BUILD_PROF=1
// prints each scope's copy count, bytes and time spent enqueueing and waiting to stderr.
hipError_t upload_bytes(void* dst, const void* src, size_t bytes);
void host_cache_stats(int64_t* live, int64_t* idle, int64_t* maps, int64_t* unmaps);
hipError_t upload_flush();   // wait for this thread's pending copies
// one index array of an ign_batch_desc (adj_src / adj_dst / adj_seq / interleave_idx): int32
// elements when the desc's index_bytes is 4 (ABI 13), else int64
struct IdxArr {
  const void* p = nullptr;
  bool w32 = false;
  IdxArr() = default;
  IdxArr(const int64_t* q, int32_t index_bytes) : p(q), w32(index_bytes == 4) {}
  int64_t operator[](int64_t k) const {
    return w32 ? (int64_t) static_cast<const int32_t*>(p)[k] : static_cast<const int64_t*>(p)[k];
  }
};

// IGN_BUILD_PROF=1: named host sections of one batch build (the time since the previous mark),
// printed as one line at the end of the build
struct BuildMarks {
  bool on;
  double last = 0;
  std::string line;
  static double now() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
  }
  explicit BuildMarks(bool enabled) : on(enabled), last(enabled ? now() : 0.0) {}
  void mark(const char* what) {
    if (!on) return;
    const double t = now();
    char buf[96];
    snprintf(buf, sizeof buf, " %s %.2f", what, t - last);
    line += buf;
    last = t;
  }
  void print(const char* head) const {
    if (on) fprintf(stderr, "[ign-build] %s sections:%s\n", head, line.c_str());
  }
};
struct UploadScope {
  explicit UploadScope(const char* what);
  ~UploadScope();
  const char* what;
  double t0;
};
template <typename T, typename A>
int dev_upload(ign_batch* b, T** out, const std::vector<T, A>& host) {
  size_t n = std::max<size_t>(host.size(), 1);
  void* p = nullptr;
  hipError_t e = pool_alloc(b->pool.get(), &p, n * sizeof(T), false);
  if (e != hipSuccess) return fail(IGN_ERR_OOM, "device alloc (%zu bytes): %s", n * sizeof(T), hipGetErrorString(e));
  b->allocs.push_back(p);
  if (!host.empty()) HIP_TRY(upload_bytes(p, host.data(), host.size() * sizeof(T)));
  else HIP_TRY(hipMemsetAsync(p, 0, sizeof(T), upload_stream()));
  *out = static_cast<T*>(p);
  return IGN_OK;
}
}  // namespace ign
