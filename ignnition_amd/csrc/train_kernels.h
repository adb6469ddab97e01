// train_kernels.h — argument blocks and launchers of the backward / optimizer kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Backward of the ordered update (reverse-time GRU, AUX:767-796).
struct SeqBwdArgs {
  const float* hs;           // [n_steps + n_dst][H]: order position p owns rows step_ptr[p]+p .. +len[p]
                             // (h_0 = state before the MP, then the state after every step)
  const float* table;        // the MP's projected table (pre-scaled, as the forward built it)
  const int32_t* order;
  const int32_t* len;
  const int32_t* step_ptr;
  const uint32_t* step_code;
  const float* Up;           // forward recurrent fragments (pre-scaled)
  const float* bias;         // forward combined biases [4][H] (pre-scaled)
  const float* Ut;           // U^T fragments (unscaled): tiles over H, k over 3H
  const float* dh_in;        // [rows][H] dLoss/d(state after the MP)
  float* dh_out;             // [rows][H] dLoss/d(state before the MP), GRU part
  float* ga;                 // [n_steps][3H]  dLoss/d(x.W + b_in) per step
  float* gu;                 // [n_steps + n_dst][3H] dLoss/d(h.U + b_rec), rows aligned with hs
                             // (the kernel zeroes each sequence's final-state row); unused when fused
  int64_t n_dst;
  const float* h_in = nullptr;   // [rows][H] the state before the MP (h_prev of every sequence's step 0)
  // fused form (part != nullptr, H 16 / 32): dU += sum h_prev^T du, db_rec += sum du and
  // db_in += sum da are formed in the kernel (per-wave partials in part, reduced in a fixed order);
  // gu is not written
  float* part = nullptr;     // seq_bwd_partial_floats(H)
  float* dU = nullptr;       // [H][3H] recurrent-kernel gradient (accumulated)
  float* db_rec = nullptr;   // [3H] recurrent-bias gradient (accumulated)
  float* db_in = nullptr;    // [3H] input-bias gradient (accumulated)
  float* scratch = nullptr;  // [(H + 1) * 3H] reduction target
  const void* Ubf = nullptr; // fused, H = 32: U's split-bf16 pieces (pack_u_bf16) -> gate recompute as seq_gru_bf x6
  const void* Uh = nullptr;  // fused, H = 32: U's scaled fp16 pieces (pack_u_f16) -> gate recompute as seq_gru_h16 x3
  const void* Uth = nullptr; // with Uh: U's scaled fp16 pieces as dh = du . U^T's A operand (pack_ut_f16)
  const int32_t* hdr = nullptr;   // per order position, padded to whole tiles: {row, len, step_ptr,
                                  // the code of the last step} (launch_seq_bwd_hdr)
  bool defer_reduce = false;   // fused: leave the per-wave partials in part (launch_seq_bwd_reduce later)
};

// Backward of the sum update (AUX:752-765): one GRU step per destination row.
struct SumBwdArgs {
  const float* x;            // [rows][DIN] aggregated messages saved by the forward
  const float* h;            // [rows][H] state before the MP
  const float* Wp;           // forward fragments (pre-scaled)
  const float* Up;
  const float* bias;
  const float* Wt;           // W^T fragments (unscaled): tiles over DIN, k over 3H
  const float* Ut;           // U^T fragments (unscaled): tiles over H, k over 3H
  const float* dh_in;
  float* dh_out;
  float* dx;                 // [rows][DIN] dLoss/dx
  float* ga;                 // [rows][3H]
  float* gu;                 // [rows][3H]
  int64_t n_dst;
};

hipError_t launch_pack_a(const float* M, int rows, int cols, float* out, hipStream_t st);
bool bwd_shape_supported(int din, int h);
hipError_t launch_seq_gru_bwd(const SeqBwdArgs& a, int h, hipStream_t st);
// the ordered backward's tile headers from the forward's (SeqGruArgs::hdr: {row, len, step_ptr,
// first code}): the same with the code of each position's last step; n_pos padded to whole tiles
hipError_t launch_seq_bwd_hdr(const int32_t* fwd_hdr, const uint32_t* step_code, int64_t n_pos, int32_t* out,
                              hipStream_t st);
bool seq_bwd_fused_supported(int h);
// fused form: the per-wave partial slots one launch writes, and their reduction into dU / db_rec /
// db_in (part may hold the partials of several launches, waves = their total)
int64_t seq_bwd_fused_waves(const SeqBwdArgs& a, int h);
hipError_t launch_seq_bwd_reduce(const SeqBwdArgs& a, int64_t waves, int h, hipStream_t st);
int64_t seq_bwd_partial_floats(int h);
hipError_t launch_sum_gru_bwd(const SumBwdArgs& a, int din, int h, hipStream_t st);
// the same with the weight gradients formed in the kernel (din = h = 32; ga / gu unused): per-wave
// partials of dW (+ db_in row) at part_w and of dU (+ db_rec row) at part_u, sum_bwd_fused_waves of
// each, in launch_partials_reduce_add's layout (M = din / h, N = 3h, ones)
int64_t sum_bwd_fused_waves(int64_t n_dst, int din, int h);
hipError_t launch_sum_gru_bwd_fused(const SumBwdArgs& a, int din, int h, float* part_w, float* part_u,
                                    hipStream_t st);
// out[r][:cols] (+)= sum over k in [ptr[r], ptr[r+1]) of in[idx[k]][:cols]   (cols % 4 == 0)
// attention backward (AUX:287-343; see train_kernels.hip): per-message dw / dv, then per source row
// and per destination the state gradients and the score-vector gradients ds; then the weights
hipError_t launch_attn_bwd_parts(const AttnArgs& a, const float* dx, const int32_t* mdst, SrcBases src, int F,
                                  int64_t n_msgs, float* dw, float* dv, hipStream_t st);
hipError_t launch_attn_src_bwd(int64_t rows, const int32_t* sptr, const int32_t* sidx, const float* msg_w,
                               const float* dv, const int32_t* mdst, const float* dx, const float* w1, int F, float* dh,
                               float* ds, hipStream_t st);
hipError_t launch_attn_dst_bwd(int64_t n_pos, const int32_t* order, const int32_t* ptr, const float* dv, const float* w2,
                               int F, float* dh, float* ds, hipStream_t st);
hipError_t launch_attn_param_bwd(const float* dw12, const float* K1, const float* K2, const float* av, int F, float* dK1,
                                 float* dK2, float* dav, hipStream_t st);
// convolution backward, elementwise: du = dx act'(x) / deg[row]; dh += du  ([n][F], rows by dst row)
hipError_t launch_conv_bwd(const float* dx, const float* x, const float* deg, int64_t n, int F, int act, float* du,
                           float* dh, hipStream_t st);
// out[r][0:width] (+)= sum over the CSR list of r of in[idx][col0 : col0 + width] (row stride in_stride)
hipError_t launch_csr_gather_cols_add(float* out, int64_t n_rows, const int32_t* ptr, const int32_t* idx,
                                      const float* in, int in_stride, int col0, int width, int accumulate,
                                      hipStream_t st);
hipError_t launch_csr_gather_add(float* out, int64_t n_rows, const int32_t* ptr, const int32_t* idx,
                                 const float* in, int cols, int accumulate, hipStream_t st);
// out[r][m] (+)= sum_k in[r][k] * Mat[m][k] (Mat packed by launch_pack_a, K % 16 == 0, M % 16 == 0),
// then (act >= 0) multiplied by act'(aprev[r][m]) given the activation values aprev.
bool row_gemm_supported(int K, int M);
hipError_t launch_row_gemm_t(const float* in, int64_t n, int K, const float* Ap, int M, float* out, int accumulate,
                             int act, const float* aprev, hipStream_t st);
// generic VALU version (any K, M): out[r][m] (+)= sum_k in[r][k] * Mat[m][k] (Mat row-major [M][K])
hipError_t launch_row_gemm_t_generic(const float* in, int64_t n, int K, const float* Mat, int M, float* out,
                                     int accumulate, int act, const float* aprev, hipStream_t st);
// dst[r][:width] += src[r][col0 : col0 + width]
hipError_t launch_split_cols_add(float* dst, int64_t n, int width, const float* src, int src_stride, int col0,
                                 hipStream_t st);
// dz[r][c] = da[r][c] * act'(a[r][c])
hipError_t launch_act_bwd(const float* da, const float* a, int64_t n, int act, float* dz, hipStream_t st);
// C[M][N] += sum_r A[r][:M]^T B[r][:N] and, if Cb, Cb[N] += sum_r B[r][:N] (a virtual ones column);
// partial sums per row chunk, reduced in a fixed order (deterministic)
int64_t tsgemm_partial_floats(int64_t n_rows, int M, int N);
// weight-gradient contractions on the split-bf16 kernel (default) or f32 MFMA; the plan sets it per backward
void set_tsgemm_bf(bool on);
// C[m][n] (row m = M: Cb[n]) += sum of nchunks partial tiles part[c][M + ones][N], in chunk order
hipError_t launch_partials_reduce_add(float* part, int64_t nchunks, int M, int N, int ones, float* C, float* Cb,
                                      hipStream_t st);
// the reduction of partial tiles uses this many chunk slots after the partials as scratch
constexpr int kTsReduceSegs = 64;
constexpr int kBwdPartialWaves = 4096;   // the fused ordered backward's partial slots per launch (at most)
// the contraction's partial tiles only (tsgemm_chunks of them at part), for a reduction later
int64_t tsgemm_chunks(int64_t n_rows, int M, int N, int ones);
hipError_t launch_tsgemm_partials(const float* A, int lda, const float* B, int ldb, int64_t n_rows, int M, int N,
                                  int ones, float* part, hipStream_t st);
hipError_t launch_tsgemm_add(const float* A, int lda, const float* B, int ldb, int64_t n_rows, int M, int N,
                             float* part, float* C, float* Cb, hipStream_t st);
// forward Dense layer for the training readout: y = act(x W + b), MFMA when packed fragments exist
bool dense_fwd_supported(int K, int M);
hipError_t launch_dense_fwd(const float* x, int64_t n, int K, int x_stride, const float* Wp, const float* W,
                            const float* bias, int M, int act, float* y, hipStream_t st);
// C[N] += sum_r B[r][:N]
hipError_t launch_colsum_add(const float* B, int ldb, int64_t n_rows, int N, float* part, float* C, hipStream_t st);
// y[i] += alpha * x[i]
hipError_t launch_axpy(float* y, const float* x, float alpha, int64_t n, hipStream_t st);
// dpred = 2 (pred - label) / n ; part[b] = partial sums of (pred - label)^2
hipError_t launch_mse(const float* pred, const float* label, int64_t n, float* dpred, double* part, int nblk,
                      hipStream_t st);
// part[b] = partial sums of x^2
hipError_t launch_sumsq(const float* x, int64_t n, double* part, int nblk, hipStream_t st);
hipError_t launch_adam(float* w, const float* g, float* m, float* v, int64_t n, float lr_t, float b1, float b2,
                       float eps, hipStream_t st);
