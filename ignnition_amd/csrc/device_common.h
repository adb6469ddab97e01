// device_common.h — device helpers shared by kernels.hip (inference) and train_kernels.hip.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "kernels.h"

typedef float f4 __attribute__((ext_vector_type(4)));

#define MFMA(a, b, c) __builtin_amdgcn_mfma_f32_16x16x4f32((a), (b), (c), 0, 0, 0)

// ---- split-bf16 contraction (fp32-exact operands on the bf16 matrix path) ------------------------
// An fp32 value has 24 significand bits; truncating it to its top 16 bits (a bf16) and repeating on
// the exact remainders gives x = hi + mid + lo EXACTLY (each piece <= 8 significant bits; the two
// subtractions are exact, Sterbenz).  Products of bf16 pieces are exact in fp32, so a contraction
// built from the piece products and accumulated in fp32 is an fp32 computation: all 9 products
// (x9) differ from an fp32 fma chain only in summation order; x6 also drops mid*lo, lo*mid and
// lo*lo.  The pieces are truncations (|mid| < 2^-8 |x|, |lo| < 2^-16 |x|), so one dropped term is
// below 2^-22 |a b| (2^-22.1 measured over 2M random pairs) and the three together below 2^-21
// (2^-21.2 measured): a few half-ulps of the product, not below one.  The measured end-to-end
// errors stay at the f32-MFMA kernels' level.
// The f32 MFMA (v_mfma_f32_16x16x4_f32) issues at the fp32 vector rate and does not overlap with
// VALU work on its SIMD (tools/probes: MFMA + VALU time = sum); v_mfma_f32_16x16x32_bf16 does 16x
// the MACs per cycle, so even 6-9 piece products cost less than one f32 pass.
typedef short bf8 __attribute__((ext_vector_type(8)));      // 8 bf16: A/B fragment of 16x16x32
typedef uint32_t u4v __attribute__((ext_vector_type(4)));
typedef int32_t i4v __attribute__((ext_vector_type(4)));
#define MFMA_BF(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_bf16((a), (b), (c), 0, 0, 0)

// ---- split-fp16 contraction (scaled two-piece fp16 operands, 3 products) --------------------------
// fp16 carries 11 significand bits: x' = s x (s a power of two putting max |x'| below 2^15) is
// rounded to hi = fp16(x') (RNE), the exact remainder to lo = fp16(x' - hi), so
// |x' - hi - lo| <= 2^-22 |x'| (plus 2^-25 absolute where lo falls below the fp16 normal range,
// i.e. for values 2^-18 below the operand's scale).  Three products hi*hi + hi*lo + lo*hi drop
// lo*lo (< 2^-22 |ab|): per product about 3 * 2^-22, the same class as the x6 bf16 split
// (2^-21.2 measured), from half the MFMAs and two pieces instead of three.
typedef _Float16 h8 __attribute__((ext_vector_type(8)));    // 8 fp16: A/B fragment of 16x16x32
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef float f2 __attribute__((ext_vector_type(2)));
#define MFMA_H(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_f16((a), (b), (c), 0, 0, 0)

// (hi, lo) fp16 pieces of the pair (a, b), each packed [a | b << 16] (v_cvt_pk_f16_f32, RNE).
// lo = fp16(a - hi): a - hi is exact in fp32 (hi is a's nearest fp16), so one mixed-precision fma
// per value, v_fma_mix{lo,hi}_f16 (a * 1 - hi, rounded once to fp16), gives the same bits as
// converting hi back to fp32, subtracting and converting again: 3 instructions per pair, not 5.
struct hpair { uint32_t hi, lo; };
__device__ __forceinline__ hpair split2h(float a, float b) {
  const h2 p = __builtin_convertvector((f2){a, b}, h2);
  const uint32_t hi = __builtin_bit_cast(uint32_t, p);
  uint32_t lo;   // mixlo leaves bits 31:16 alone and mixhi overwrites them: no initial value
  asm("v_fma_mixlo_f16 %0, %1, 1.0, -%3 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %0, %2, 1.0, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(lo) : "v"(a), "v"(b), "v"(hi));
  return {hi, lo};
}

__device__ __forceinline__ void split3(float x, float& hi, float& mid, float& lo) {
  hi = __uint_as_float(__float_as_uint(x) & 0xFFFF0000u);
  const float r1 = x - hi;
  mid = __uint_as_float(__float_as_uint(r1) & 0xFFFF0000u);
  lo = r1 - mid;
}
// [bf16(a) | bf16(b) << 16] of values whose low 16 bits are dropped (exact for split3 pieces)
__device__ __forceinline__ uint32_t pack_hi16(float a, float b) {
  return __builtin_amdgcn_perm(__float_as_uint(b), __float_as_uint(a), 0x07060302u);
}

// Gate nonlinearities on v_exp_f32 + v_rcp_f32 (1 ulp each; an IEEE divide would expand to
// ~10 VALU instructions and dominate the recurrence's VALU stream).  Both saturate cleanly:
// exp overflow gives rcp(inf) = 0.
__device__ __forceinline__ float rcpf_(float x) { return __builtin_amdgcn_rcpf(x); }

__device__ __forceinline__ float sigmoidf_(float x) { return rcpf_(1.0f + __expf(-x)); }

// tanh(t), given t and c = 2 log2(e) t.  Away from 0: 1 - 2 / (1 + 2^c).  Near 0 that form
// cancels: its absolute error stays ~2 ulp(1) while tanh -> 0, and the GRU recurrence amplifies
// it over the iterations (over the 512 x synth50 batch it doubled the worst-case error against a
// float32 evaluation with libm's tanhf).  |t| < 0.55: t + t^3 p(t^2), p a degree-4
// weighted least-squares fit of (tanh(t)/t - 1)/t^2 (<= 1.2 ulp relative in fp32).
__device__ __forceinline__ float tanh_tc_(float t, float c) {
  const float u = t * t;
  float p = fmaf(u, -0.0062725638953669005f, 0.021070224531615167f);
  p = fmaf(p, u, -0.0538518588145328f);
  p = fmaf(p, u, 0.13332580319582182f);
  p = fmaf(p, u, -0.3333331730407817f);
  const float small = fmaf(t * u, p, t);
  const float big = 1.0f - 2.0f * rcpf_(1.0f + __builtin_amdgcn_exp2f(c));
  return fabsf(t) < 0.55f ? small : big;
}

__device__ __forceinline__ float tanhf_(float x) { return tanh_tc_(x, x * 2.8853900817779268f); }

// GRU gates on pre-scaled pre-activations.  pack_gru scales the z/r columns (and their biases)
// by -log2(e) and the candidate columns by 2*log2(e), so
//   sigmoid(a) = 1 / (1 + 2^(a'))      with a' = -log2(e) a
//   tanh(c)    = 1 - 2 / (1 + 2^(c'))  with c' = 2 log2(e) c   (c' is linear in x, h, biases)
// i.e. one v_exp_f32 + one v_rcp_f32 per gate and no scaling multiply.
#define IGN_NLOG2E (-1.4426950408889634f)
#define IGN_2LOG2E (2.8853900817779268f)
__device__ __forceinline__ float sig2_(float a) { return rcpf_(1.0f + __builtin_amdgcn_exp2f(a)); }
// tanh of the pre-scaled candidate argument c' = 2 log2(e) c (ln2 / 2 = 1 / (2 log2 e))
__device__ __forceinline__ float tanh2_(float c) { return tanh_tc_(c * 0.34657359027997264f, c); }

__device__ __forceinline__ float act_apply(float x, int act) {
  switch (act) {
    case IGN_K_ACT_RELU: return x > 0.f ? x : 0.f;
    case IGN_K_ACT_SELU: {
      const float lam = 1.0507009873554805f, alpha = 1.6732632423543772f;
      return x > 0.f ? lam * x : lam * alpha * (__expf(x) - 1.0f);
    }
    case IGN_K_ACT_SIGMOID: return sigmoidf_(x);
    case IGN_K_ACT_TANH: return tanhf_(x);
    default: return x;
  }
}

template <int ACT>
__device__ __forceinline__ float act_t(float x) {
  if constexpr (ACT == IGN_K_ACT_RELU) return x > 0.f ? x : 0.f;
  else if constexpr (ACT == IGN_K_ACT_SELU) {   // branch-free: exp of min(x, 0), then select
    const float lam = 1.0507009873554805f, la = 1.0507009873554805f * 1.6732632423543772f;
    const float e = __expf(__builtin_amdgcn_fmed3f(x, -3.0e38f, 0.f));   // min(x, 0), no canonicalise
    return x > 0.f ? lam * x : la * (e - 1.0f);
  } else if constexpr (ACT == IGN_K_ACT_SIGMOID) return sigmoidf_(x);
  else if constexpr (ACT == IGN_K_ACT_TANH) return tanhf_(x);
  else return x;
}

// max over the wave of a value >= 0 in every lane, in every lane: DPP row shifts (lane 15 of each
// row of 16 ends with the row's max), two row broadcasts (lane 63 ends with the wave's), readlane.
// No LDS round trip, unlike a __shfl_xor butterfly.
// (The comparisons run on the bit patterns: non-negative floats order as unsigned integers, and an
// integer max needs no canonicalising v_max_f32 x, x, x first.)
__device__ __forceinline__ float wave_max_nonneg(float x) {
  uint32_t v = __float_as_uint(x);
#define IGN_DPP_MAX(ctrl, rmask) \
  v = max(v, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, ctrl, rmask, 0xf, true))
  IGN_DPP_MAX(0x111, 0xf);   // row_shr:1
  IGN_DPP_MAX(0x112, 0xf);   // row_shr:2
  IGN_DPP_MAX(0x114, 0xf);   // row_shr:4
  IGN_DPP_MAX(0x118, 0xf);   // row_shr:8
  IGN_DPP_MAX(0x142, 0xa);   // row_bcast:15 into rows 1 and 3
  IGN_DPP_MAX(0x143, 0xc);   // row_bcast:31 into rows 2 and 3
#undef IGN_DPP_MAX
  return __uint_as_float((uint32_t)__builtin_amdgcn_readlane((int)v, 63));
}

// XCD-aware block order: the dispatcher deals blocks round-robin over the 8 XCDs (b, b+8, ...
// share one), so remap so that XCD x runs a contiguous range of tiles (bijective for any grid,
// cdna_hip_programming.md §5.5).  Consecutive tiles are the same graph -> that graph's source
// rows stay in one XCD's L2.  Placement only affects speed, never results.
__device__ __forceinline__ int64_t xcd_block(int enabled) {
  const int64_t b = blockIdx.x, nb = gridDim.x;
  if (!enabled) return b;
  const int64_t xcd = b & 7, q = nb >> 3, r = nb & 7;
  const int64_t base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (b >> 3);
}

__device__ __forceinline__ f4 ld4(const float* p) { return *reinterpret_cast<const f4*>(p); }
__device__ __forceinline__ void st4(float* p, f4 v) { *reinterpret_cast<f4*>(p) = v; }

// element (gate-tile gt, k-step s, lane) of a float4-grouped fragment array with KS k-steps
__device__ __forceinline__ int64_t frag_idx(int gt, int s, int KS, int lane) {
  return ((((int64_t)gt * (KS / 4) + (s >> 2)) * 64 + lane) << 2) + (s & 3);
}

