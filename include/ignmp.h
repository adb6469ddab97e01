/*
 * ignmp.h — C ABI of the MI355X message-passing engine (libignmp.so).
 *
 * This is the drop-in boundary for IGNNITION's hot path: the multi-stage
 * message-passing loop + readout that the reference lowers to TensorFlow ops in
 * ComnetModel.call (code/utils/generate_model.py:384-658).  The reference's own
 * boundary is a Python/Keras operator:
 *
 *   ComnetModel()                       generate_model.py:235-382  (plan from Model_information)
 *   ComnetModel.call(input, training)   generate_model.py:384      (feature dict -> [P,1] predictions)
 *
 * whose input dict is fixed by input_fn (generate_model.py:127-158): per feature a
 * float vector, per adjacency src_<adj>/dst_<adj> int64 [E], seq_<srcEnt>_<dstEnt>
 * int64 [E], num_<entity> int64 scalar, indices_<src>_to_<dst> int64 [L].
 *
 *   ign_plan_create     <-> ComnetModel.__init__  (GM:235-382): entities, MP stages,
 *                           GRU cells (one per destination entity, GM:309-313),
 *                           readout Dense stack (GM:350-358, AUX:918-975).
 *   ign_plan_set_params <-> the Keras variables (kernel / recurrent_kernel / bias,
 *                           Dense kernel / bias) — layout from ign_plan_param_tensor.
 *   ign_batch_create    <-> the feature dict of input_fn (GM:127-158) for a batch of
 *                           graphs (model_fn's per-graph loop, GM:712-724, becomes
 *                           one disjoint-union batch; exact for sum/ordered/interleave
 *                           + predict).
 *   ign_forward         <-> model(f) for every graph + concat of the flattened
 *                           predictions in batch order (GM:716-724).
 *
 * Conventions: plain C types only.  Status 0 = OK, negative = error class; the
 * message of the last error on the calling thread is ign_last_error().  The caller
 * owns every host array passed in (borrowed for the call); plans and batches own
 * their device memory.  Calls on one plan are not reentrant; one plan per thread.
 * There is no CPU execution path: every compute entry point runs HIP kernels on
 * the plan's device and fails with IGN_ERR_DEVICE when no GPU is present.
 */
#ifndef IGNMP_H
#define IGNMP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IGN_ABI_VERSION 13

enum ign_status {
  IGN_OK = 0,
  IGN_ERR_INVALID = -1,      /* malformed plan/batch (reference: ValueError / InvalidArgument) */
  IGN_ERR_UNSUPPORTED = -2,  /* schema-legal but not (yet) lowered: FF update, attention, ... */
  IGN_ERR_DEVICE = -3,       /* no GPU / HIP runtime error */
  IGN_ERR_OOM = -4,
  IGN_ERR_RUNTIME = -5
};

enum ign_aggregation {        /* AUX:229-456, dispatch GM:547-569 */
  IGN_AGGR_SUM = 0,
  IGN_AGGR_ORDERED = 1,
  IGN_AGGR_INTERLEAVE = 2,
  IGN_AGGR_CONCAT = 3,
  IGN_AGGR_ATTENTION = 4,
  IGN_AGGR_CONVOLUTION = 5
};

enum ign_activation {         /* Dense activations accepted by the readout (AUX:836-837) */
  IGN_ACT_LINEAR = 0,          /* "None" / "linear" */
  IGN_ACT_RELU = 1,
  IGN_ACT_SELU = 2,
  IGN_ACT_SIGMOID = 3,
  IGN_ACT_TANH = 4
};

typedef struct ign_plan ign_plan;
typedef struct ign_batch ign_batch;

typedef struct {
  int32_t hidden_dim;              /* hidden_state_dimension (AUX:101) */
  int32_t feature_total;           /* sum of feature sizes, features concatenated in listed order (AUX:140-153) */
} ign_entity_desc;

enum ign_message_input {        /* message-creation network inputs (GM:446-462) */
  IGN_MSG_HS_SOURCE = 0,
  IGN_MSG_HS_DEST = 1,
  IGN_MSG_EDGE_PARAMS = 2
};

typedef struct ign_dense_desc_s ign_dense_desc;

typedef struct {
  int32_t entity;                  /* source entity index */
  int32_t adjacency;               /* adjacency slot: index into ign_batch_desc.adj_* */
  int32_t interleave;              /* interleave slot (indices_<src>_to_<dst>) or -1 */
  /* Message creation (GM:440-475): 0 layers = direct_assignation (message = source state);
   * otherwise a Dense stack on the per-edge concatenation of msg_inputs (enum
   * ign_message_input, in order).  edge_params has msg_param_dim floats per edge. */
  int32_t msg_num_inputs;
  const int32_t* msg_inputs;
  int32_t msg_param_dim;
  int32_t msg_num_layers;
  const ign_dense_desc* msg_layers;
} ign_source_desc;

typedef struct {
  int32_t dst_entity;              /* GM:415 */
  int32_t aggregation;             /* enum ign_aggregation */
  int32_t concat_axis;             /* for IGN_AGGR_CONCAT (AUX:456) */
  int32_t cell;                    /* GRU cell index (one per destination entity name, GM:313) */
  int32_t num_sources;
  const ign_source_desc* sources;  /* in model_description order (GM:423) */
  int32_t activation;              /* IGN_AGGR_CONVOLUTION: activation_function (AUX:370-374) */
} ign_mp_desc;

typedef struct {
  int32_t input_dim;               /* message dimension fed to the cell */
  int32_t units;                   /* = hidden_dim of the destination (AUX:747) */
} ign_cell_desc;

struct ign_dense_desc_s {
  int32_t units;
  int32_t activation;              /* enum ign_activation */
  int32_t use_bias;
  float l2;                        /* kernel_regularizer coefficient c: loss += c * sum(W^2) (AUX:833-834) */
};

enum ign_readout_op_type {     /* readout operations before predict (GM:611-655, AUX:1033-1234) */
  IGN_RO_NEURAL_NETWORK = 0,     /* Readout_nn: Dense stack on the axis-1 concat of its inputs (GM:612-628) */
  IGN_RO_POOLING = 1,            /* Pooling_operation: reduce over the graph's rows -> [1, F] (AUX:1163-1185) */
  IGN_RO_PRODUCT = 2,            /* Product_operation element_wise: tf.multiply with broadcasting (AUX:1081-1088) */
  IGN_RO_EXTEND = 3              /* Extend_adjacencies: gather both ends of an adjacency (AUX:1236-1265) */
};

enum ign_pooling { IGN_POOL_SUM = 0, IGN_POOL_MEAN = 1, IGN_POOL_MAX = 2 };

/* Readout tensors are numbered: [0, num_entities) the entity hidden states, then the outputs
 * of the readout ops in order (one each; extend_adjacencies has two: src then dst).  Every
 * tensor lives on one row space: an entity's rows, one row per graph (pooling), or an
 * adjacency's edges (extend_adjacencies); the predict op's inputs share one space, whose
 * rows are the predictions. */
typedef struct {
  int32_t type;                    /* enum ign_readout_op_type */
  int32_t num_inputs;
  const int32_t* inputs;           /* readout tensor ids (GM:660-675 resolves names to states) */
  int32_t mode;                    /* IGN_RO_POOLING: enum ign_pooling; IGN_RO_PRODUCT: 0 = element_wise */
  int32_t adjacency;               /* IGN_RO_EXTEND: adjacency slot (one that some MP reads) */
  int32_t num_dense;               /* IGN_RO_NEURAL_NETWORK: its Dense stack */
  const ign_dense_desc* dense;
} ign_readout_op_desc;

typedef struct {
  int32_t num_iterations;          /* GM:406 */
  int32_t num_entities;
  const ign_entity_desc* entities;
  int32_t num_adjacencies;
  int32_t num_interleave;
  int32_t num_mps;                 /* stages flattened in execution order (GM:410-414) */
  const ign_mp_desc* mps;
  int32_t num_cells;
  const ign_cell_desc* cells;
  int32_t num_readout_inputs;      /* predict op inputs, concatenated on axis 1 (GM:615-621) */
  const int32_t* readout_inputs;   /* readout tensor ids (entity indices when there are no readout ops) */
  int32_t num_dense;
  const ign_dense_desc* dense;     /* readout Dense stack (RNJ:113-142) */
  int32_t num_readout_ops;         /* operations run before predict, in model_description order */
  const ign_readout_op_desc* readout_ops;
} ign_plan_desc;

typedef struct {
  int32_t num_graphs;
  const int64_t* num_nodes;        /* [num_graphs][num_entities]  num_<entity> per graph */
  const float* const* features;    /* [num_entities] -> [sum_g N_e(g)][feature_total] (NULL if no features) */
  const int64_t* adj_edges;        /* [num_graphs][num_adjacencies] edges per graph */
  const int64_t* const* adj_src;   /* [num_adjacencies] -> graph-concatenated, graph-local src_<adj> */
  const int64_t* const* adj_dst;   /* graph-local dst_<adj> */
  const int64_t* const* adj_seq;   /* seq_<srcEnt>_<dstEnt> */
  const int64_t* interleave_len;   /* [num_graphs][num_interleave] */
  const int64_t* const* interleave_idx; /* [num_interleave] -> graph-concatenated indices_<src>_to_<dst> */
  /* Edge-cut partitions (num_graphs must be 1 when used): per entity, extra state rows
   * after the owned num_<entity> rows that hold peers' hidden states.  Sources may address them
   * (src index in [num, num + halo)); destinations, features and the readout cover owned rows only.
   * The caller fills them (ign_batch_bind_state + its own collective) before an MP reads them.
   * NULL = no halo. */
  const int64_t* halo_rows;        /* [num_entities] or NULL */
  /* per adjacency: graph-concatenated params_<adj> [edges][param dim] (cast to float, GM:454-456),
   * needed by message networks that read edge_params; NULL entries / NULL array when absent */
  const float* const* adj_params;
  /* ABI 13: the width of adj_src, adj_dst, adj_seq and interleave_idx's elements: 0 or 8 = int64_t
   * (the pointer types above), 4 = int32_t (the pointers then point at int32_t arrays; the native
   * reader's narrow gather, ign_dataset_batch_get_narrow, hands them over without a widening copy) */
  int32_t index_bytes;
}  ign_batch_desc;

typedef struct {
  int64_t num_graphs;
  int64_t predictions;             /* rows of the predict input space (outputs = predictions * last units) */
  int64_t output_units;
  int64_t edges_per_forward;       /* T * sum over MPs and sources of |adj| */
  int64_t gru_steps_per_forward;   /* GRU cell applications (per destination row / sequence step) */
  int64_t rows[8];                 /* total rows per entity (first 8 entities) */
} ign_batch_info_t;

/* Per-kernel timing (HIP events on the plan stream, enabled by ign_plan_set_timing), accumulated
 * over every timed launch since the last ign_plan_set_timing / ign_plan_set_timing_kinds.  The
 * event pairs are resolved lazily: ign_stats waits for the plan's stream and then reads them, so
 * it blocks, and like every call on a plan it must come from the plan's one host thread.
 * kind: 0 init_state, 1 seq_gru, 2 sum_gru, 3 readout, 4 project, 5 other, 6 mp_resident (round 4:
 * the graph-resident forward, every MP of every iteration in one launch) */
typedef struct {
  int32_t kinds;
  int64_t launches[8];
  double  ms[8];
  double  flops[8];                /* algorithmic FLOPs of those launches */
  double  bytes[8];                /* algorithmic HBM bytes of those launches */
  double  mfma_bf16[8];            /* FLOPs the matrix pipe executed as bf16 MFMAs (the split-bf16
                                      kernels' piece products; dense peak 2.5 PFLOP/s) */
  double  mfma_f32[8];             /* FLOPs executed as f32 MFMAs (v_mfma_f32_16x16x4_f32) */
} ign_stats_t;

int  ign_abi_version(void);
const char* ign_last_error(void);
int  ign_device_count(int32_t* n);

int  ign_plan_create(const ign_plan_desc* desc, int32_t device, ign_plan** out);
/* The same plan from the files the reference reads (ComnetModel.__init__ over Model_information,
 * GM:235-382 / JO:128-149): model_description.json text and the dataset dimensions as a JSON
 * object {feature or adjacency name: size} (JO:162-180).  Lowered in C++ (csrc/plan_json.cpp)
 * exactly as ignnition_amd/engine.py MPPlan.from_model_info + to_desc; IGN_ERR_UNSUPPORTED for a
 * model the engine does not lower (same messages), IGN_ERR_INVALID for one the reference rejects. */
int  ign_plan_create_json(const char* model_json, const char* dims_json, int32_t device, ign_plan** out);
/* For a plan from ign_plan_create_json: a JSON document with the entity / feature order, every
 * adjacency slot's input keys (src_<adj>, dst_<adj>, seq_<src>_<dst>, GM:127-158), the interleave
 * keys (indices_<src>_to_<dst>), the label and the parameter tensors' Keras-style names and shapes
 * in ign_plan_param_tensor order.  *needed = bytes incl. the terminating NUL; buf may be NULL. */
int  ign_plan_describe_json(const ign_plan* plan, char* buf, int64_t size, int64_t* needed);
void ign_plan_destroy(ign_plan* plan);
int  ign_plan_num_params(const ign_plan* plan, int64_t* n_floats);
int  ign_plan_num_param_tensors(const ign_plan* plan, int32_t* n);
/* tensor i: kind 0 gru kernel [in,3H], 1 gru recurrent_kernel [H,3H], 2 gru bias [2,3H],
 *           3 dense kernel [in,out], 4 dense bias [1,out]; owner = cell or dense index;
 *           5 convolution kernel [F,F], 6 attention kernel1 [F,F], 7 attention kernel2 [F,F],
 *           8 attention attn_kernel [2F,1] (one set per plan, GM:288-300; owner -1);
 *           9 message-network Dense kernel [in,out], 10 its bias [1,out] (owner = mp * 4 + source);
 *           11 readout neural_network op Dense kernel [in,out], 12 its bias [1,out] (owner = op * 64 + layer).
 * Order: cells, message networks (MP order, source order, layer order), convolution, attention,
 * readout neural_network ops (op order, layer order), predict Dense layers. */
int  ign_plan_param_tensor(const ign_plan* plan, int32_t i, int32_t* kind, int32_t* owner,
                           int64_t* offset, int32_t* rows, int32_t* cols);
int  ign_plan_set_params(ign_plan* plan, const float* params, int32_t on_device);
int  ign_plan_set_timing(ign_plan* plan, int32_t enabled);   /* also resets the statistics */
/* Restrict the event pairs to kernel kinds in the bit mask (bit k = kind k of ign_stats_t);
 * default all.  Each event pair costs a few microseconds of queue time. */
int  ign_plan_set_timing_kinds(ign_plan* plan, uint32_t kinds);
/* Run the plan on an external stream from now on.  Waits for the plan's previous stream (its own
 * or an earlier external one) first, so buffers of destroyed batches are never reused early. */
int  ign_plan_set_stream(ign_plan* plan, void* hip_stream);
/* Give the plan's idle cached device blocks (kept for the next batches, IGN_POOL_CACHE_GB) and the
 * process's idle pinned host blocks (IGN_HOST_CACHE_GB) back to the runtime, waiting for the
 * in-flight work that still reads them: call when another allocator (torch, RCCL) runs short.
 * No reference counterpart (TF owns its allocator). */
int  ign_plan_trim_cache(ign_plan* plan);

int  ign_batch_create(ign_plan* plan, const ign_batch_desc* desc, ign_batch** out);
void ign_batch_destroy(ign_batch* batch);
int  ign_batch_info(const ign_batch* batch, ign_batch_info_t* out);

/* The graph-resident forward of a batch (ABI 11, 12): decided by ign_batch_create (with
 * IGN_RESIDENT_EAGER=0 at the batch's first ign_forward or ign_forward_train, active = 0 before it),
 * with the per-launch cost model of its one launch.  The training forward (ign_forward_train) runs
 * the same form, saving what the backward reads (IGN_RESIDENT_TRAIN=0: per-MP launches). */
typedef struct {
  int32_t active;                  /* 1: ign_forward runs the whole MP loop as one launch */
  int32_t form;                    /* 0: every state in LDS; 1: path states in HBM / L2; 2: ... and the
                                      sum MPs' CSR read from L2 */
  int64_t lds_bytes;               /* dynamic LDS per workgroup (the batch's largest graph) */
  int64_t tile_steps;              /* phase A: 16-path tile-steps per launch (T x per tile its longest
                                      sequence) */
  int64_t union_tiles;             /* phase B: 16-row tiles of the source entities' rows, per iteration */
  int64_t seg_rows;                /* rows whose message sum takes sum_seg's wave-per-row order */
  int64_t messages;                /* sum-MP messages per iteration */
  double  bytes_compulsory;        /* features, index tables read once, final states written once */
  double  bytes_roundtrip;         /* global-path forms: the path states' (and CSR's) L2 round trips */
  double  bytes_stage;             /* sum over the T iterations' MPs of
                                      B_stage = E (4 + 4H) + 2 N_d 4H + 4 (N_d + 1) */
  double  flops;                   /* executed FLOPs (fp32-equivalent) */
  double  mfma_bf16;               /* FLOPs issued on the 16-bit matrix pipe */
  double  mfma_f32;                /* ... on the f32 matrix pipe */
  int32_t workgroups;              /* ABI 12: workgroups per launch (graphs / graphs_per_workgroup) */
  int32_t graphs_per_workgroup;    /* ABI 12: consecutive graphs one workgroup runs as one disjoint union
                                      (IGN_RES_GROUP; auto: 2 where a graph's all-LDS form fits twice) */
} ign_resident_info_t;
int  ign_batch_resident_info(const ign_batch* batch, ign_resident_info_t* out);

/* Full forward (hidden-state init, T x stages x MPs, readout) on the plan stream.
 * pred_out: host pointer (copied + synchronised) or NULL (stays on device, async).
 * Untimed forwards on a non-null stream replay one hipGraph captured per batch on first use
 * (IGN_HIP_GRAPH=0 disables it).  */
int  ign_forward(ign_plan* plan, ign_batch* batch, float* pred_out);
int  ign_synchronize(ign_plan* plan);
/* Device pointer of the batch's prediction buffer (valid until ign_batch_destroy). */
int  ign_batch_predictions(ign_batch* batch, const float** dev_ptr);
/* Copy the batch's predictions [n_pred][units] to host after the forwards enqueued on the plan's
 * stream (waits for that stream only): the host side of a forward launched with pred_out NULL,
 * e.g. one of several sub-batches on several plans launched before any wait (ABI 10). */
int  ign_batch_read_predictions(ign_plan* plan, ign_batch* batch, float* host_out);
/* Copy the current hidden state of an entity (after ign_forward) to host [rows][H]. */
int  ign_batch_state(ign_plan* plan, ign_batch* batch, int32_t entity, float* host_out);
int  ign_stats(const ign_plan* plan, ign_stats_t* out);

/* ---- Stepped forward, for edge-cut partitions exchanging halo rows between MPs ----
 * ign_forward == ign_forward_begin; for it < T: for mp: ign_forward_mp(mp, IGN_PART_ALL);
 * ign_forward_end.  A sum MP can run as two launches, IGN_PART_INTERIOR (destinations none of
 * whose messages come from halo rows; may overlap the halo exchange) then IGN_PART_BOUNDARY;
 * the destination state flips to the new buffer after IGN_PART_ALL or IGN_PART_BOUNDARY.  */
enum ign_part { IGN_PART_ALL = 0, IGN_PART_INTERIOR = 1, IGN_PART_BOUNDARY = 2 };
int  ign_forward_begin(ign_plan* plan, ign_batch* batch);
int  ign_forward_mp(ign_plan* plan, ign_batch* batch, int32_t mp, int32_t part);
int  ign_forward_end(ign_plan* plan, ign_batch* batch, float* pred_out);
/* Destinations of MP `mp` in the interior / boundary launch (all destinations are interior
 * without halo rows). */
int  ign_batch_mp_split(const ign_batch* batch, int32_t mp, int64_t* interior, int64_t* boundary);
/* Replace an entity's two state buffers by caller-owned device memory, each at least
 * (rows + halo) * hidden_dim + 256 floats, 16-byte aligned.  State contents are not copied. */
int  ign_batch_bind_state(ign_plan* plan, ign_batch* batch, int32_t entity, float* dev0, float* dev1,
                          int64_t capacity_floats);
/* Which of the two state buffers (0/1) holds the entity's current state. */
int  ign_batch_state_slot(const ign_batch* batch, int32_t entity, int32_t* slot);
/* dst[i][:] = src[idx[i]][:] on the plan stream (halo pack); cols % 4 == 0, device pointers. */
int  ign_gather_rows(ign_plan* plan, const float* src, int64_t ld, const int32_t* idx, int64_t n, int32_t cols,
                     float* dst);

/* ---- Training step (model_fn's TRAIN branch, GM:697-830) -------------------------
 * ign_batch_enable_training allocates what the backward keeps (every hidden-state version, the
 * per-step states of ordered updates, the aggregated messages of sum updates, the readout
 * activations) and the transposed index tables.  Device pointers throughout; gradients come in
 * the flat parameter layout of ign_plan_param_tensor and include the Dense l2 terms. */
int  ign_batch_enable_training(ign_plan* plan, ign_batch* batch);
/* forward of ComnetModel.call keeping the activations; pred_out: host or NULL (see ign_forward) */
int  ign_forward_train(ign_plan* plan, ign_batch* batch, float* pred_out);
/* grads[n_params] = dLoss/dparams for dLoss/dpredictions = dpred[predictions * output_units].
 * A backward consumes its forward: the readout backward writes gradient rows over the saved
 * activations, so a second ign_backward / ign_backward_begin returns IGN_ERR_INVALID until the
 * next ign_forward_train. */
int  ign_backward(ign_plan* plan, ign_batch* batch, const float* dpred, float* grads);
/* The same two calls in steps, for a training step on an edge-cut partition (ABI 9): the caller
 * exchanges halo rows between the steps (ignnition_amd/partition.py EdgeCutTraining).
 *   ign_forward_train_begin; then T x num_mps times ign_forward_train_mp (MP instances in order:
 *   before one, the current version of each source entity must hold its peers' halo rows);
 *   ign_forward_train_end (readout, predictions).
 *   ign_backward_begin (readout backward; l2_scale weights the kernel_regularizer terms, e.g.
 *   1/ranks when the ranks' gradients are summed); then ign_backward_mp once per MP instance
 *   (reverse order: after one, the halo rows of each source entity's current gradient hold
 *   gradient for peers' rows: send them to their owners, add, zero them); ign_backward_end.
 * ign_batch_train_buffers: the current state version and gradient buffer of an entity,
 * [owned rows | halo rows][hidden] each. */
int  ign_forward_train_begin(ign_plan* plan, ign_batch* batch);
int  ign_forward_train_mp(ign_plan* plan, ign_batch* batch);
int  ign_forward_train_end(ign_plan* plan, ign_batch* batch, float* pred_out);
int  ign_backward_begin(ign_plan* plan, ign_batch* batch, const float* dpred, float* grads, float l2_scale);
int  ign_backward_mp(ign_plan* plan, ign_batch* batch);
int  ign_backward_end(ign_plan* plan, ign_batch* batch);
int  ign_batch_train_buffers(const ign_batch* batch, int32_t entity, float** state, float** grad);
/* MeanSquaredError: loss = mean((pred - labels)^2) (host, may be NULL), dpred = 2 (pred - labels) / n */
int  ign_mse_loss(ign_plan* plan, const float* pred, const float* labels, int64_t n, float* dpred, double* loss);
/* sum over Dense layers of l2 * sum(W^2) for the current parameters (the regularization loss) */
int  ign_l2_loss(ign_plan* plan, double* loss);
/* Keras Adam on the plan's parameters (in place) with lr = the schedule at `iteration`:
 * lr_t = lr sqrt(1 - beta2^(it+1)) / (1 - beta1^(it+1)); m, v: caller-owned device state. */
int  ign_adam_step(ign_plan* plan, const float* grads, float* m, float* v, int64_t iteration, float lr,
                   float beta1, float beta2, float epsilon);
/* Copy the current parameters (flat layout) to host. */
int  ign_plan_get_params(ign_plan* plan, float* host_out);

/* ---- Native dataset reader (GEN:32-230 = the reference's generator) -----
 * Reads the *.tar.gz files of <dir> (sorted by name; data.json inside, a list of samples) on `threads`
 * host threads and builds the generator's index contract per sample.  A sample that fails
 * abandons the rest of its file and is reported through ign_dataset_error (GEN:229-230); a file
 * without data.json fails the open.  Batches are gathered by sample id; ign_dataset_get returns
 * the batch's graph-concatenated array of one generator key (feature names, src_/dst_<adj>,
 * seq_<src>_<dst>, params_<adj>, num_<entity>, indices_<src>_to_<dst>, or "__label__") with its
 * per-graph lengths; pointers stay valid until the next gather. */
typedef struct ign_dataset ign_dataset;
typedef struct {
  int32_t num_features;
  const char* const* features;      /* feature names (model order) */
  const char* output_name;          /* label key; NULL when reading without labels (predict) */
  int32_t num_adjacencies;          /* model_info.get_adjecency_info() order (GEN:134) */
  const char* const* adj_name;
  const char* const* adj_src;       /* source entity type */
  const char* const* adj_dst;       /* destination entity type */
  const int32_t* adj_params;        /* 1: keep [node, params] parameters ("True") */
  int32_t num_interleave;           /* get_interleave_tensors(): (definition key, destination) */
  const char* const* il_name;
  const char* const* il_dst;
  int32_t num_additional;
  const char* const* additional;
} ign_dataset_desc;
int  ign_dataset_open(const char* dir, const ign_dataset_desc* desc, int32_t threads, ign_dataset** out);
void ign_dataset_close(ign_dataset* ds);
int  ign_dataset_size(const ign_dataset* ds, int64_t* n_samples, int32_t* n_errors);
const char* ign_dataset_error(const ign_dataset* ds, int32_t i);
int  ign_dataset_gather(ign_dataset* ds, const int64_t* ids, int32_t count);
/* dtype: 0 float32, 1 int64 (2 int32: ign_dataset_batch_get_narrow only) */
int  ign_dataset_get(ign_dataset* ds, const char* key, int32_t* dtype, const void** ptr, int64_t* total,
                     const int64_t** per_graph);
/* The same gather as a batch object with its own buffers (pointers valid until it is destroyed):
 * any number may exist, and threads may create and read them concurrently on one dataset (the
 * training input pipeline builds several batches in parallel; tf.data's map/prefetch, GM:181-192). */
typedef struct ign_dataset_batch ign_dataset_batch;
int  ign_dataset_batch_create(const ign_dataset* ds, const int64_t* ids, int32_t count, ign_dataset_batch** out);
int  ign_dataset_batch_get(ign_dataset_batch* batch, const char* key, int32_t* dtype, const void** ptr,
                           int64_t* total, const int64_t** per_graph);
/* ABI 13: the same, with an integer key's values as int32 (dtype 2) when every sample's fit (the
 * reader stores them so), else as int64 (dtype 1): half the bytes of the int64 concatenation, for
 * ign_batch_desc.index_bytes = 4 */
int  ign_dataset_batch_get_narrow(ign_dataset_batch* batch, const char* key, int32_t* dtype, const void** ptr,
                                  int64_t* total, const int64_t** per_graph);
void ign_dataset_batch_destroy(ign_dataset_batch* batch);

#ifdef __cplusplus
}
#endif
#endif /* IGNMP_H */
