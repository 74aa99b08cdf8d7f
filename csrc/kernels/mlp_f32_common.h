// Helpers shared by the fp32 persistent epoch kernels (mlp_persistent_f32.hip: owners + heads,
// mlp_persistent_f32v2.hip: owners only): shapes, exact three-term bf16 split of fp32 operands,
// f32-input MFMA, the register-resident optimizer update and sc1 (L1-bypassing) accessors.
#pragma once
#include "mlp_fused.h"
#include "persist_common.h"

namespace f32k {

using persist::gu32;

constexpr int NT = 512;  // threads per workgroup (8 waves)
constexpr int PD1 = 256, PD2 = 128;
// K steps of the W1 GEMMs: D0 columns plus at least one padding column, column D0, which carries
// b1: the X tile holds 1 there for valid rows, so the forward MFMAs add b1 and the dW1 MFMAs
// produce db1 in the register slot that holds b1 (no separate bias add, sum or update).
__host__ __device__ inline int ks1_of(int D0) { return D0 / 32 + 1; }
constexpr int LDD = PD2 + 4;   // fp32 row stride of the owner's dH2 tile [B][128]
constexpr int LDH1 = PD1 + 4;  // fp32 row stride of the head's H1 tile [B][256]
constexpr int LD16 = 20;       // fp32 row stride of [*][16] tiles
constexpr int F32_FPP = 304;   // hand-off flag lines per peer (every gang layout shares the flag block)
constexpr unsigned DONE_MARK = 1u << 23;   // commit flag value (above every step's t + 1)
constexpr unsigned RETRY_BASE = 1u << 24;  // hand-off flag base of the retry attempt
constexpr int ERR_RETRY = 64;              // err layout: [0, 64) first attempt, [64, 128) retry, per peer

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x4 mfma_f32(float a, float b, const f32x4& c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }
__device__ __forceinline__ int kappa(int h, int j) { return j < 4 ? 4 * h + j : 16 + 4 * h + (j - 4); }
__device__ __forceinline__ bf16x8 cat8(const bf16x4& lo, const bf16x4& hi) { return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7); }
__device__ __forceinline__ float ld_wt32(const float* p) {  // 4-byte L1-bypassing (sc1) load
  return __builtin_bit_cast(float, __hip_atomic_load((gu32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ float4 as_f4(const u32x4& v) { return __builtin_bit_cast(float4, v); }
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* base, int bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, bytes, 0x00020000);
}
// 16-byte sc1 load (L1 bypass) of a handed-off tile
__device__ __forceinline__ float4 ld_sc1_16(__amdgpu_buffer_rsrc_t r, int byte_off) { return as_f4(__builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 16)); }

// frag_b_tr (common.h) with the lane index passed in (a per-step laundered copy)
__device__ __forceinline__ bf16x8 frag_b_tr_l(const bf16* base, int ld, int k0, int n0, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const bf16* p0 = base + (k0 + 8 * g + q) * ld + n0 + 4 * pp;
  const mlp_s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((mlp_lds_s16x4*)(p0));
  const mlp_s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((mlp_lds_s16x4*)(p0 + 4 * ld));
  return __builtin_bit_cast(bf16x8, (mlp_s16x8)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

// Exact split of fp32 values into three bf16 terms: x == hi + mid + lo. hi = RNE(x) leaves a
// remainder that is a multiple of x's 24-bit ulp below 2^16 ulps, mid takes its top 8 bits and lo
// the last <= 8 (both subtractions are exact), so the three terms carry all 24 significand bits.
__device__ __forceinline__ void split3(const float (&x)[8], bf16x8& hi, bf16x8& mid, bf16x8& lo) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const bf16 a = (bf16)x[j];
    const float r = x[j] - (float)a;
    const bf16 b = (bf16)r;
    hi[j] = a;
    mid[j] = b;
    lo[j] = (bf16)(r - (float)b);
  }
}
// acc += A · (hi + mid + lo), smallest terms first
__device__ __forceinline__ f32x4 mfma3(const bf16x8& a, const bf16x8& hi, const bf16x8& mid, const bf16x8& lo, f32x4 acc) {
  acc = mfma_bf16(a, lo, acc);
  acc = mfma_bf16(a, mid, acc);
  return mfma_bf16(a, hi, acc);
}

// Per-element constant of the FedProx / SCAFFOLD terms. FedProx: g += mu·(w − anchor) is
// g += mu·w + e with e = −mu·anchor (the mu·w part is folded into weight decay). SCAFFOLD
// (o.scaf_upd; never together with FedProx on this path): e = c − c_i, applied after the step as
// w −= lr·e (update space, see opt_update in common.h).
__device__ __forceinline__ float extra_at(const MLPArgs& a, int64_t idx) {
  float e = 0.f;
  if (a.cg != nullptr) e = a.cg[idx] - a.cl[idx];
  if (a.anchor != nullptr) e = fmaf(-a.opt.mu, a.anchor[idx], e);
  return e;
}

// torch.optim.Adam / SGD(+momentum, nesterov) update of one register-resident element. The same
// code updates the head's W2 rows and the owners' W2 replica: identical inputs give identical bits.
template <bool ADAM, bool EXTRA>
__device__ __forceinline__ void upd32(const OptParams& o, float g, float& w, float& m, float& v, float e, float lr_t, float inv, float wdmu) {
  g = fmaf(wdmu, w, g);  // weight decay (+ FedProx mu); 0: exact no-op
  if (EXTRA && !o.scaf_upd) g += e;
  if (ADAM) {
    m = fmaf(o.beta1, m, (1.f - o.beta1) * g);
    v = fmaf(o.beta2, v, (1.f - o.beta2) * (g * g));
    const float denom = fmaf(__builtin_amdgcn_sqrtf(v), inv, o.eps);
    w = fmaf(-lr_t, m * __builtin_amdgcn_rcpf(denom), w);
  } else {
    if (o.momentum != 0.f) {
      m = fmaf(o.momentum, m, g);
      g = o.nesterov ? fmaf(o.momentum, m, g) : m;
    }
    w = fmaf(-o.lr, g, w);
  }
  if (EXTRA && o.scaf_upd) w = fmaf(-o.lr, e, w);
}

__device__ __forceinline__ int rows_at(const MLPArgs& a, int n, int t) {
  const int r = n - t * a.B;
  return r < 0 ? 0 : (r > a.B ? a.B : r);
}

}  // namespace f32k
