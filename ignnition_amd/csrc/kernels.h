// kernels.h — kernel argument blocks and launchers shared by engine.cpp and kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define IGN_SLOT_SHIFT 29u
#define IGN_ROW_MASK ((1u << IGN_SLOT_SHIFT) - 1u)
#define IGN_MAX_SLOTS 4

enum { IGN_K_ACT_LINEAR = 0, IGN_K_ACT_RELU = 1, IGN_K_ACT_SELU = 2, IGN_K_ACT_SIGMOID = 3, IGN_K_ACT_TANH = 4 };

// Base pointer of each source slot's current hidden-state table (message code = slot<<29 | row).
struct SrcBases {
  const float* base[IGN_MAX_SLOTS];
};

struct SeqGruArgs {
  const float* h_in;         // [rows][H] destination state before the update
  float* h_out;              // [rows][H] destination state after the update
  const float* table;        // projected message table [sources' rows | bias row | multi rows][3H]
  const int32_t* order;      // [n_dst] destination rows, sorted by final_len (descending)
  const int32_t* len;        // [n_dst] final_len per order position
  const int32_t* step_ptr;   // [n_dst] first step of each order position
  const uint32_t* step_code; // [n_steps + pad] table row of every step (padded with the zero row)
  const float* Up;           // packed recurrent-kernel fragments
  const float* bias;         // [4][H] combined biases
  int64_t n_dst;
  int xcd_remap;             // XCD-aware tile order (speed only)
  float* hs_save = nullptr;  // training: [n_steps + n_dst][H], order position p writes rows
                             // step_ptr[p] + p (state before) .. + len[p] (after each step)
  const void* Ubf = nullptr;  // variants 4/5: recurrent kernel as exact 3-piece bf16 A fragments
  const void* Uh = nullptr;   // variants 6/7: scaled 2-piece fp16 A fragments + scale (pack_u_f16)
  // variants 6/7: [ceil(n_dst / 16) * 16][4] per order position {order, len, step_ptr,
  // step_code[step_ptr]}; the padding positions are {0, 0, n_steps, zero row}
  const int32_t* hdr = nullptr;
};

struct SumGruArgs {
  const float* h_in;
  float* h_out;
  SrcBases src;
  const int32_t* order;    // [n_dst] destination rows, sorted by in-degree (descending)
  const int32_t* msg_ptr;  // [n_dst + 1] message range per order position
  const uint32_t* msg_src;
  const float* Wp;
  const float* Up;
  const float* bias;
  int64_t n_dst;
  int xcd_remap;
  float* x_save = nullptr;   // training: [rows][DIN] aggregated messages, by destination row
  const float* msg_w = nullptr;    // attention: per-message weight (CSR order), x = sum w_m h_src
  const float* conv_kp = nullptr;  // convolution: packed kernel; x = act((sum h_src . K + h) / deg)
  int conv_act = 0;
  float* sum_save = nullptr;       // training, convolution: [rows][DIN] message sums before K
  const void* Wbf = nullptr;       // split-bf16 pieces of W / U (pack_w_bf16 / pack_u_bf16): variant 7
  const void* Ubf = nullptr;
  // sum_gru_g32 only: also project the new states for the next ordered MP that reads them
  // (table row r = h_new[r] . W' + b', as project_kernel; split-bf16 x6): its projected table,
  // its input kernel's pack_w_bf16 pieces and its combined pre-scaled biases
  float* proj_out = nullptr;
  const void* proj_W = nullptr;
  const float* proj_b = nullptr;
  float* proj_bias_row = nullptr;  // the table's hole row: receives proj_b alone (as project_kernel)
};

// Attention weights (AUX:287-343): per (graph, position) group of dense cells, the axis-0 softmax
// of e = LeakyReLU_0.2(s_src + s_dst) summed per cell, written to every message of the cell.
struct AttnArgs {
  const int32_t* group_ptr;
  const int32_t* group_empty;      // empty cells of the group (they score 0 in the softmax)
  const int32_t* cell_dst;
  const int32_t* cell_ptr;
  const int32_t* cell_msgs;        // CSR message positions
  const uint32_t* msg_src;         // message codes (slot << 29 | row)
  const float* s_src[IGN_MAX_SLOTS];   // h_src . (K1 a1) per source row
  const float* s_dst;              // h_dst . (K2 a2) per destination row
  float* ecell;
  float* msg_w;
  int64_t n_groups;
};

struct Readout3Args {
  const float* x;          // [n_rows][x_stride]
  int64_t n_rows;
  int x_stride;
  const float* W1p; const float* b1;
  const float* W2p; const float* b2;
  const float* w3;  const float* b3;  // [N2] (output units == 1), [1]
  int act1, act2, act3;
  float* y;                // [n_rows]
  float* save1 = nullptr;  // readout_h16 only: [n_rows][N1] layer-1 activations (training forward)
  float* save2 = nullptr;  //   [n_rows][N2] layer-2 activations
};

hipError_t launch_init_state(float* state, const float* feats, int64_t n, int H, int F, hipStream_t st);
hipError_t launch_pack_gru(const float* W, const float* U, const float* bias, float* Wp, float* Up, float* bp,
                           int DIN, int H, hipStream_t st);
hipError_t launch_pack_dense(const float* W, float* Wp, int IN, int OUT, hipStream_t st);
bool gru_shape_supported(int din, int h);
hipError_t launch_project(const float* x, int64_t n, const float* Wp, const float* bp, float* out, float* bias_row,
                          int din, int h, hipStream_t st);
hipError_t launch_multi_sum(float* table, int64_t multi_base, int64_t n_multi, const int32_t* ptr,
                            const uint32_t* rows, int W, const float* bias_row, hipStream_t st);
hipError_t launch_seq_gru(const SeqGruArgs& args, int h, int variant, hipStream_t st);
// split-bf16 ordered update (kernels_bf.hip), passes 6 or 9
hipError_t launch_seq_gru_bf(const SeqGruArgs& args, int h, int passes, hipStream_t st);
// recurrent kernel -> split-bf16 A fragments for seq variants 4/5 (H = 32 or 64); floats used: 9 H^2 / 2
hipError_t launch_pack_u_bf16(const float* U, void* out, int H, hipStream_t st);
inline int64_t pack_u_bf16_floats(int H) { return (H == 32 || H == 64) ? 9LL * H * H / 2 : 0; }
// split-fp16 ordered update (kernels_bf.hip, inference only), passes 3 or 4
hipError_t launch_seq_gru_h16(const SeqGruArgs& args, int h, int passes, hipStream_t st);
// recurrent kernel -> scaled 2-piece fp16 A fragments for seq variants 6/7 (H = 32 or 64), then the
// scale's exponent; floats used: 3 H^2 + 64
hipError_t launch_pack_u_f16(const float* U, void* out, int H, hipStream_t st);
inline int64_t pack_u_f16_floats(int H) { return (H == 32 || H == 64) ? 3LL * H * H + 64 : 0; }
// U (unscaled, [H][3H]) as the A operand of dh = du . U^T in the ordered backward (rows: the H state
// units, k: the 3H gate units in the chained order), scaled fp16 pieces + scale exponent; H = 32
hipError_t launch_pack_ut_f16(const float* U, void* out, int H, hipStream_t st);
inline int64_t pack_ut_f16_floats(int H) { return H == 32 ? 3LL * H * H + 64 : 0; }
// [K][3H] input kernel -> the same scaled fp16 layout (K % 32 == 0) for sum variant 8
hipError_t launch_pack_w_f16(const float* W, void* out, int K, int H, hipStream_t st);
inline int64_t pack_w_f16_floats(int K, int H) { return ((H == 32 || H == 64) && K % 32 == 0) ? 3LL * K * H + 64 : 0; }
// sum variant 8: the split-fp16 sum update (DIN = H = 64; Wbf / Ubf carry pack_w_f16 / pack_u_f16)
hipError_t launch_sum_gru_h16(const SumGruArgs& args, int din, int h, hipStream_t st);
// pieces of a [K][3H] input kernel (K % 32 == 0) for the split-bf16 sum update
hipError_t launch_pack_w_bf16(const float* W, void* out, int K, int H, hipStream_t st);
inline int64_t pack_w_bf16_floats(int K, int H) { return ((H == 32 || H == 64) && K % 32 == 0) ? 9LL * K * H / 2 : 0; }
// split-bf16 sum update (DIN = H = 64, no message weights / convolution); hipErrorInvalidValue otherwise
hipError_t launch_sum_gru_bf(const SumGruArgs& args, int din, int h, hipStream_t st);
// sum update at DIN = H = 32: code-prefetched gather (gu rows in flight per lane), split-bf16 GRU step
hipError_t launch_sum_gru_g32(const SumGruArgs& args, int gu, hipStream_t st);
// Rows formed on the fly from the backward of a 1-unit output layer: row[r][k] = (0 + s[r] w[k]) *
// act'(raw[r][k]), raw = the layer's input activations (row_outer_t's arithmetic); s == nullptr: off
struct OuterRows {
  const float* s = nullptr;   // [rows] the output layer's pre-activation gradient
  const float* w = nullptr;   // [K] its weights
  int act = 0;                // the activation of raw
  float* out = nullptr;       // where the formed rows are also written (may be raw: in place)
};
// split-bf16 form of the training row contraction (train_kernels.hip tsgemm; same grid and partials)
hipError_t launch_tsgemm_bf(const float* A, int lda, const float* B, int ldb, int64_t n_rows, int M, int N, int ones,
                            int64_t chunk, int64_t chunks, int tiles, int wpb, float* part, hipStream_t st);
hipError_t launch_sum_gru(const SumGruArgs& args, int din, int h, int variant, hipStream_t st);

// Windowed sum (AUX:254-262 for single-source sum MPs of graph-local batches): one workgroup per
// (graph, destination chunk) stages the graph's source rows through LDS in windows with coalesced
// loads, so each source row leaves HBM once per chunk instead of once per message; x[dst] = sum of
// the destination's source rows (ascending source order) is written for the GRU step.
struct SumWinArgs {
  const float* src;        // source states [rows][DIN]
  const int64_t* wg;       // [n_wg][4]: first / end window position, first / end source row
  const int32_t* dst;      // [positions] destination row
  const int32_t* ptr;      // [positions + 1] message range
  const int32_t* srow;     // [messages] source rows, ascending per destination
  float* xsum;             // [rows][DIN]
  int64_t n_wg;
};
hipError_t launch_sum_win(const SumWinArgs& args, int din, hipStream_t st);
// High-degree sum (IGN_SUM_WINDOW=2 / auto): one wave per destination, xsum[order[p]] = sum of its
// messages (single-source MP, slot 0), RS = 64 / (DIN / 4) message rows per load instruction
struct SumSegArgs {
  const float* src;        // source states [rows][DIN]
  const int32_t* order;    // [n_dst] destination rows
  const int32_t* msg_ptr;  // [n_dst + 1] message range per order position (the sum MP's CSR)
  const uint32_t* msg_src; // [messages] source codes (slot 0)
  float* xsum;             // [rows][DIN]
  int64_t n_dst;
};
hipError_t launch_sum_seg(const SumSegArgs& args, int din, hipStream_t st);

// Graph-resident forward (resident.hip): one workgroup per graph runs the T iterations of one ordered
// MP into the "path" entity from S <= 2 source entities ("links"; Q-size: links and nodes, the
// interleave) and, for each source entity, one sum MP from the paths back to it (RouteNet: S = 1),
// H = DIN = 32, with the graph's source-entity states and the projected table in LDS; writes the
// final states of every entity.  The source entities' rows of a graph form one "union" row range:
// entity 0's rows, then entity 1's.
#ifndef IGN_RES_WAVES   // A/B builds only (the host's eligibility assumes the default)
#define IGN_RES_WAVES 16
#endif
constexpr int kResidentWaves = IGN_RES_WAVES;
constexpr int kResidentMaxSrc = 2;
constexpr int kResidentMaxTiles = 2 * kResidentWaves;   // union-row tiles of a graph (B2/B3: two per wave)
constexpr int kResidentStateStride = 36;    // LDS floats per 32-wide state row
constexpr int kResidentTableStride = 100;   // LDS floats per 96-wide projected row
constexpr size_t kResidentMaxDynLds = 144 * 1024;   // + ~14.5 KB static (U pieces, biases)
enum { IGN_RES_ALL_LDS = 0, IGN_RES_PATH_GLOBAL = 1, IGN_RES_PATH_CSR_GLOBAL = 2 };   // kernel forms
struct ResidentArgs {
  const int32_t* gorder;      // [G] the graph of workgroup b (longest first; nullptr: b), round 6
  const int64_t* path_off;    // [G + 1] rows of the ordered MP's destination entity ("paths") per graph
  const int64_t* src_off[kResidentMaxSrc];   // [G + 1] rows of each source entity per graph
  const int64_t* urow_off;    // [G + 1] graph g's union rows start here (lmsg_ptr, lorder)
  const int32_t* ptile_off;   // [G + 1] first header of graph g (multiples of 16)
  const int32_t* hdr;         // [headers][4] per graph, its paths by length descending, padded to whole
                              // tiles: {local path row (-1: padding), final_len, local step offset,
                              // first step's local code}
  const int32_t* lcode_off;   // [G + 1] graph g's ordered-MP step codes start here in lcode
  const uint16_t* lcode;      //   local union rows (U_g = the hole), then max_len + 8 hole codes
  const int32_t* lmsg_off;    // [G + 1] graph g's sum-MP messages start here in lmsg_src; its CSR
  const int32_t* lmsg_ptr;    //   [urow_off[g] + g ...][U_g + 1] local offsets, by local union row
  const uint16_t* lmsg_src;   //   local path rows, each union row's messages in its sum MP's order
  const uint16_t* lorder;     // [union rows] per graph, its local union rows by message count, descending
  const int32_t* lnseg;       // [G] the first lnseg[g] rows of lorder (>= 64 messages) take
                              // sum_seg_kernel's summation order, the others the lane walk
  const float* path_feat; int path_F;
  const float* src_feat[kResidentMaxSrc]; int src_F[kResidentMaxSrc];
  float* path_state;          // [rows][32] final states
  float* src_state[kResidentMaxSrc];
  const void* Uh;             // the ordered MP's U, scaled fp16 pieces (pack_u_f16) + exponent
  const float* seq_bias;      // the ordered MP's combined biases [4][H]
  const void* sWbf[kResidentMaxSrc];   // each sum MP's W / U split-bf16 pieces, combined biases
  const void* sUbf[kResidentMaxSrc];
  const float* sum_bias[kResidentMaxSrc];
  const void* proj_W;         // the ordered MP's input kernel as split-bf16 pieces, its biases
  const float* proj_b;
  const float* proj_Wf;       // ... and as project_kernel's f32 fragments (the iteration-0 projection)
  int T;
  int n_src;
  int seg_on;                 // 0: every message sum as the lane walk (the training forward's sums)
  // SAVE (the training forward, global-path forms): iteration it's ordered MP reads the path states
  // path_ver[it] and writes path_ver[it + 1] and every step's state into hs_save[it] from row hsb of
  // each position (seq_gru_h16<SAVE>'s layout); the sum MPs write their message sums into
  // x_save[s][it] and their new states into src_ver[s][it + 1]; every iteration projects with f32
  // MFMA (build_table's project_kernel).  ver[.][0] hold the initial states (init_state).
  float* const* path_ver;
  float* const* src_ver[kResidentMaxSrc];
  float* const* hs_save;
  float* const* x_save[kResidentMaxSrc];
  const int32_t* hsb;         // [headers] the position's first hs_save row (step_ptr + order position)
  float* const* tab_save;     // SAVE, optional: [T] the ordered MP's projected table per iteration, in
                              // the batched layout (the backward's table; build_table is skipped)
  int64_t tab_off[kResidentMaxSrc];   // table row of each source entity's row 0 (MPB::src_off)
  int64_t tab_hole;           // the table's zero row (a hole: the bias alone)
};
// the kernels' dynamic-LDS limit, once per device: call before any launch or stream capture
hipError_t resident_prepare_device();
hipError_t launch_resident_forward(const ResidentArgs& a, int n_graphs, size_t lds_bytes, int form, bool save,
                                   hipStream_t st);
bool readout3_supported(int din, int n1, int n2, int act1, int act2);
hipError_t launch_readout3(const Readout3Args& args, int din, int n1, int n2, hipStream_t st);
// readout on split-bf16 contractions (fp32-exact operands; passes 6 or 9), weights from
// launch_pack_dense_bf16 (W1 natural k order, W2 chained); floats used: 3 IN OUT / 2
bool readout_bf_supported(int din, int n1, int n2, int act1, int act2);
// readout variant 4: both layers on scaled 2-piece fp16 pieces (pack_readout_h16: W2, header, W1,
// header; floats 256 * 256 + 64 + IN1 * 256 + 64)
hipError_t launch_readout_h16(const Readout3Args& args, const void* Wh, int din, hipStream_t st);
hipError_t launch_pack_readout_h16(const float* W1, const float* b1, const float* W2, void* out, int in1, int n1,
                                   int n2, hipStream_t st);
hipError_t launch_pack_readout_h16_header(const float* W1, const float* b1, const float* W2, void* out, int in1, int n1,
                                          int n2, hipStream_t st);
// readout variant 5 (readout_h32.hip): variant 4's arithmetic class on v_mfma_f32_32x32x16_f16, k-outer
// layer 2 (pack_readout_h32: the same buffer size and header positions as variant 4's)
hipError_t launch_readout_h32(const Readout3Args& args, const void* Wh, int din, hipStream_t st);
hipError_t launch_pack_readout_h32(const float* W1, const float* b1, const float* W2, void* out, int in1, int n1,
                                   int n2, hipStream_t st);
hipError_t launch_readout_bf(const Readout3Args& args, const void* W1f, const void* W2f, int din, int passes,
                             hipStream_t st);
hipError_t launch_pack_dense_bf16(const float* W, void* out, int IN, int OUT, int chained, hipStream_t st);
// y[r][0..M) = act(x[r] . W + b), split-bf16 (x6) with fp32 accumulation; W packed by
// launch_pack_dense_bf16 with chained = 0.  K in {32, 64, 128, 256}, M a multiple of 128.
bool dense_bf_supported(int K, int M);
hipError_t launch_dense_bf(const float* x, int64_t n, int K, int x_stride, const void* Wbf, const float* bias, int M,
                           int act, float* y, hipStream_t st);
// the backward row GEMM out[r][0..M) (+)= (dz[r] . W^T) * act'(aprev[r]) (act < 0: no act'), dz [n][K]
// dense; W^T packed by launch_pack_dense_bf16_t(W [M][K])
hipError_t launch_dense_bf_t(const float* dz, int64_t n, int K, const void* Wtbf, int M, float* out, int accumulate,
                             int act, const float* aprev, hipStream_t st, OuterRows xo = OuterRows{});
hipError_t launch_pack_dense_bf16_t(const float* W, void* out, int IN, int OUT, hipStream_t st);
// the same two row GEMMs on scaled split-fp16 (x3; DESIGN.md §3b'): W pieces from
// launch_pack_dense_f16 (IN x OUT natural k, trans = 1 for W^T: IN = OUT_orig, OUT = IN_orig);
// floats used: IN * OUT + 64
hipError_t launch_dense_h16(const float* x, int64_t n, int K, int x_stride, const void* Wh, const float* bias, int M,
                            int act, float* y, hipStream_t st);
hipError_t launch_dense_h16_t(const float* dz, int64_t n, int K, const void* Wth, int M, float* out, int accumulate,
                              int act, const float* aprev, hipStream_t st, OuterRows xo = OuterRows{});
hipError_t launch_pack_dense_f16(const float* W, void* out, int IN, int OUT, int trans, hipStream_t st);
hipError_t launch_dense_generic(const float* x, int64_t n, int in, int x_stride, const float* W, const float* b,
                                int out, int act, float* y, hipStream_t st);
hipError_t launch_concat_cols(float* dst, int64_t n, int dst_stride, int col0, const float* src, int width,
                              hipStream_t st);
hipError_t launch_gather_rows(const float* src, int64_t ld, const int32_t* idx, int64_t n, int cols, float* dst,
                              hipStream_t st);
hipError_t launch_attn_softmax(const AttnArgs& a, hipStream_t st);
// w12[0:F] = K1 . a[0:F], w12[F:2F] = K2 . a[F:2F]  (attention score vectors)
hipError_t launch_attn_vectors(const float* K1, const float* K2, const float* a, int F, float* w12, hipStream_t st);

// Message-network input (GM:446-462): out[e][col_q .. col_q + width_q) = part q of edge e, where a
// part is a state row (rows[q][e]) or the edge's parameters (rows[q] == nullptr: row e).
struct MsgGatherArgs {
  float* out;
  int64_t n;
  int ld;
  int nparts;
  int col[4], width[4];
  const float* base[4];
  const int32_t* rows[4];
};
hipError_t launch_msg_gather(const MsgGatherArgs& a, hipStream_t st);
hipError_t launch_pack_dense_pad(const float* W, float* Wp, int IN, int IN_pad, int OUT, hipStream_t st);

// train_csr.hip: the training tables' transposed CSRs by a stable radix sort on the device
size_t tcsr_temp_bytes(int64_t n);
hipError_t launch_tcsr_keys_seq(const uint32_t* step_code, int64_t n_steps, uint32_t zero_row, uint32_t* keys,
                                int32_t* vals, hipStream_t st);
hipError_t launch_tcsr_keys_sum(const int32_t* msg_ptr, const int32_t* order, int64_t n_dst, const uint32_t* msg_src,
                                uint32_t* keys, int32_t* vals, hipStream_t st);
hipError_t launch_tcsr_sort(void* temp, size_t temp_bytes, const uint32_t* keys_in, uint32_t* keys_out,
                            const int32_t* vals_in, int32_t* vals_out, int64_t n, uint32_t max_key, hipStream_t st);
hipError_t launch_tcsr_ptr(const uint32_t* sorted_keys, int64_t n, uint32_t key0, int64_t rows, int32_t* ptr,
                           hipStream_t st);
