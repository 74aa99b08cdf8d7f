// Shared device helpers for the gfx950 (MI355X, CDNA4) kernels of myfyp_amd.
//
// MFMA used everywhere: v_mfma_f32_16x16x32_bf16 (wave64).
//   A fragment: lane l holds A[row = l&15][k = 8*(l>>4) + j], j = 0..7
//   B fragment: lane l holds B[k = 8*(l>>4) + j][col = l&15]
//   C/D:        lane l holds C[row = 4*(l>>4) + i][col = l&15], i = 0..3
// (cdna_hip_programming.md §3). Operands are bf16, accumulation fp32.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define WAVE 64

__device__ __forceinline__ f32x4 mfma_bf16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x4 zero4() { return f32x4{0.f, 0.f, 0.f, 0.f}; }

__device__ __forceinline__ bf16x8 zero_bf16x8() {
  bf16x8 z;
#pragma unroll
  for (int j = 0; j < 8; ++j) z[j] = (bf16)0.f;
  return z;
}

// 16-byte aligned load of 8 bf16
__device__ __forceinline__ bf16x8 ld8(const bf16* p) { return *reinterpret_cast<const bf16x8*>(p); }

// 8 uint8 (8-byte aligned) -> 8 bf16 (exact for 0..255)
__device__ __forceinline__ bf16x8 ld8_u8(const uint8_t* p) {
  uint2 v = *reinterpret_cast<const uint2*>(p);
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) r[j] = (bf16)(float)((v.x >> (8 * j)) & 0xffu);
#pragma unroll
  for (int j = 0; j < 4; ++j) r[4 + j] = (bf16)(float)((v.y >> (8 * j)) & 0xffu);
  return r;
}

typedef short mlp_s16x4 __attribute__((ext_vector_type(4)));
typedef short mlp_s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) mlp_s16x4 mlp_lds_s16x4;

// B fragment B[k0 + 8 (lane>>4) + j][n0 + (lane & 15)] from a row-major [k][n] bf16 LDS image
// (two 4-row transposed reads; EXEC must be full — call from wave-uniform control flow only)
__device__ __forceinline__ bf16x8 frag_b_tr(const bf16* base, int ld, int k0, int n0) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
  const bf16* p0 = base + (k0 + 8 * g + q) * ld + n0 + 4 * pp;
  const mlp_s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((mlp_lds_s16x4*)(p0));
  const mlp_s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((mlp_lds_s16x4*)(p0 + 4 * ld));
  return __builtin_bit_cast(bf16x8, (mlp_s16x8)__builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations and meets the
// other waves, but leaves global loads in flight (``__syncthreads()`` also drains vmcnt, which
// stalls every wave on prefetches it does not need yet). Single asm with a memory clobber so the
// compiler moves no memory access across it. Never use it to publish global-memory data.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

__device__ __forceinline__ float warp_sum16(float v) {
  // reduce across the 16 lanes of a lane-group (lanes sharing l>>4)
  v += __shfl_xor(v, 1);
  v += __shfl_xor(v, 2);
  v += __shfl_xor(v, 4);
  v += __shfl_xor(v, 8);
  return v;
}

__device__ __forceinline__ float warp_max16(float v) {
  v = fmaxf(v, __shfl_xor(v, 1));
  v = fmaxf(v, __shfl_xor(v, 2));
  v = fmaxf(v, __shfl_xor(v, 4));
  v = fmaxf(v, __shfl_xor(v, 8));
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// Optimizer epilogue shared by every fused wgrad kernel and by the flat optimizer kernels.
// g is the raw gradient; extras (FedProx anchor, SCAFFOLD control variates) are optional.
//
// SCAFFOLD's correction is applied in the UPDATE space: w <- step(w, g) - lr·(c - c_i). For plain
// SGD that is the paper's g + c - c_i; for Adam / momentum it keeps the correction in the units of
// the local step, which is what the control variate update c_i+ = c_i - c + (x - y)/(K·lr) measures
// (the reference's option II, scaffold_callback.py:129). Fed into Adam's gradient instead, the
// correction is a difference of normalised steps read as a gradient (no learning).
struct OptParams {
  int kind;            // 0 = Adam, 1 = SGD (+momentum)
  float lr, beta1, beta2, eps, weight_decay, momentum;
  int nesterov;
  float mu;            // FedProx proximal coefficient (0 = off)
  int scaf_upd;        // fused MLP epochs: the per-element extra term is a SCAFFOLD update-space correction
};

__device__ __forceinline__ void opt_update(const OptParams& o, float g, float& w, float& m, float& v, float bc1, float bc2_sqrt,
                                           const float* anchor, const float* cg, const float* cl, int64_t idx) {
  if (anchor != nullptr && o.mu != 0.f) g += o.mu * (w - anchor[idx]);
  const float corr = cg != nullptr ? cg[idx] - cl[idx] : 0.f;
  if (o.weight_decay != 0.f) g += o.weight_decay * w;
  if (o.kind == 0) {
    m = fmaf(o.beta1, m, (1.f - o.beta1) * g);
    v = fmaf(o.beta2, v, (1.f - o.beta2) * g * g);
    // torch.optim.Adam: w -= (lr / bc1) * m / (sqrt(v) / sqrt(bc2) + eps)
    const float denom = sqrtf(v) * (1.f / bc2_sqrt) + o.eps;
    w -= (o.lr / bc1) * __fdiv_rn(m, denom);
  } else {
    if (o.momentum != 0.f) {
      m = o.momentum * m + g;
      g = o.nesterov ? g + o.momentum * m : m;
    }
    w -= o.lr * g;
  }
  if (cg != nullptr) w -= o.lr * corr;
}
