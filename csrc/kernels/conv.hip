// Implicit-GEMM convolutions on MFMA (gfx950, wave64), grouped over co-located peers.
//
// k_conv_gemm<MODE, BN, PRO>: C[M][Ncol] = A[M][K] · B[K][Ncol]
//   MODE 0 (forward) : rows = output pixels, A = im2col(X) gathered on the fly, K = (r, s, ci),
//                      B = Wf[co][r][s][ci] rows (K-contiguous), staged [n][k] XOR-swizzled
//   MODE 1 (dgrad)   : rows = input pixels,  A = dY gathered at ((h+pad-r)/st, (w+pad-s)/st) when
//                      divisible (zero otherwise), K = (r, s, co); B[k][ci] = Wf[co][r][s][ci] is
//                      N-contiguous, staged [k][n] and read as MFMA fragments with the gfx950 LDS
//                      transpose read (ds_read_b64_tr_b16) — no transposed weight copy exists
//   128 x BN tiles (2 x 2 waves, each 64 rows), BK = 64, 256 threads, 16x16x32 bf16 MFMA, fp32
//   accumulate.
//   A is register-staged into a double-buffered LDS image whose 16-byte chunks are XOR-swizzled
//   (chunk ^ ((row >> 1) & 7)) so every ds_read_b128 fragment read is conflict-free; one barrier
//   per K-step (the next tile's global loads are in flight during the MFMAs).
//   Fused epilogue: + bias, + residual, ReLU, zeroed channel padding, BatchNorm sums (atomics).
//   XCD-aware bijective block remap so tiles sharing an operand panel land on one L2.
//
// k_conv_wgrad<BM, BN, PRO>: dW[co][(r,s,ci)] = sum_m dY[m][co] · im2col(X)[m][(r,s,ci)]
//   K = pixels (split over workgroups), both operands staged [m][channels] as loaded and read
//   as MFMA fragments with the transposed LDS read. The gradient is written in the GEMM's own
//   (Wf) layout [cp_out][R][S][cp_in] fp32: 16 lanes of a row write 64 contiguous bytes (plain
//   stores when the pixel dimension is not split, fp32 atomics otherwise). The optimizer kernel
//   maps it to torch order through LDS (a torch-order scatter here cost ~0.45 ms per layer).
#include <hip/hip_runtime.h>

#include <cstddef>

#include "conv.h"

#include <cstdlib>

struct bf8 { bf16 v[8]; };

#define CG_BK 64

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int xcd = orig & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (orig >> 3);
}

// x / d for 0 <= x < 2^22 with a float reciprocal and one correction step (the gathers divide
// by runtime geometry — Wo, Ho*Wo, S, channel chunks — in their inner loops; integer division is
// a long VALU sequence on CDNA)
__device__ __forceinline__ int fdiv(int x, int d, float inv) {
  int q = (int)((float)x * inv);
  q -= (q * d > x) ? 1 : 0;
  q += ((q + 1) * d <= x) ? 1 : 0;
  return q;
}

// relu(v*sc + sh) on one 16-byte chunk of 8 bf16 channels (the k_bn_act arithmetic: fmaf, relu,
// round to bf16 — bit-identical to the materialised activation)
__device__ __forceinline__ uint4 bn_relu8(uint4 u, const float* sc, const float* sh) {
  bf16 v[8];
  __builtin_memcpy(v, &u, 16);
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (bf16)fmaxf(fmaf((float)v[j], sc[j], sh[j]), 0.f);
  uint4 r;
  __builtin_memcpy(&r, v, 16);
  return r;
}

// Operand gathers as raw buffer loads (CONV_BUFLOAD, default on): a 32-bit byte offset against a
// per-peer resource, and an out-of-range offset for padding / masked chunks, which the buffer unit
// returns as zeros — no 64-bit address arithmetic and no 4-way select per 16-byte chunk.
#ifndef CONV_BUFLOAD
#define CONV_BUFLOAD 1
#endif
typedef unsigned conv_u32x4 __attribute__((ext_vector_type(4)));
constexpr int CONV_OOB = (int)0x80000000u;  // >= num_records: the load returns zeros
__device__ __forceinline__ __amdgpu_buffer_rsrc_t conv_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ uint4 conv_ld16(__amdgpu_buffer_rsrc_t r, int byte_off) {
  return __builtin_bit_cast(uint4, (conv_u32x4)__builtin_amdgcn_raw_buffer_load_b128(r, byte_off, 0, 0));
}

__device__ __forceinline__ int swz(int row, int chunk) { return row * CG_BK + ((chunk ^ ((row >> 1) & 7)) << 3); }
// Patch rows (the halo kernels' staged 64-channel patch): the MFMA A reads of a tap start at ANY
// patch row, and a ds_read_b128 lane group ({0-3,12-15,20-27}, ...) takes 8 rows at chunk c and the
// other 8 of the 16 at chunk c + 1; with swz's key (row >> 1) & 7 that was 2-way conflicted for
// half the start rows (1.41 conflicts per LDS instruction, profiles/r4n_*). Key row & 6 is
// conflict-free for every start row (exhaustive check over the lane groups and 16-byte bank units).
#ifndef HALO_SWZP
#define HALO_SWZP 1
#endif
__device__ __forceinline__ int swzp(int row, int chunk) { return HALO_SWZP ? row * CG_BK + ((chunk ^ (row & 6)) << 3) : swz(row, chunk); }

// [k][W] images read with ds_read_b64_tr_b16 (W = 64 or 128 bf16, unpadded rows): 8-byte granules
// XOR-permuted by a row function so that the 32 lanes of a half-wave (rows 8g+q, g = 0/1, q = 0..3,
// four granules each) hit 32 distinct bank granules; the permutation is a multiple of 4 granules,
// so a lane's 4 elements and a writer's 16-byte chunk stay contiguous (measured: ~1-1.6 bank
// conflicts per LDS instruction with a +8-element row pad instead).
template <int W>
__device__ __forceinline__ int trf(int row) {
  if (W == 128) return ((row & 3) | (((row >> 3) & 1) << 2)) << 2;
  return (((row >> 1) & 1) | (((row >> 3) & 1) << 1)) << 2;
}
template <int W>
__device__ __forceinline__ int tr_off(int row, int col) {  // col multiple of 4
  return row * W + ((((col >> 2) ^ trf<W>(row))) << 2);
}
// transposed MFMA fragment from a [k][W] image: lane i of group g gets column (col0 + i), rows k0 + 8g + 0..7
template <int W>
__device__ __forceinline__ bf16x8 frag_tr(const bf16* base, int col0, int k0, int lane) {
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  const int r0 = k0 + 8 * g + q;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + tr_off<W>(r0, col0 + 4 * p)));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + tr_off<W>(r0 + 4, col0 + 4 * p)));
  // whole-vector bit cast (an element-wise short->bf16 cast miscompiles into lane-duplicating perms)
  const s16x8 both = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, both);
}

// Epilogue shared by the conv GEMM kernels (BM x BN tile, NT threads, NT / 64 waves as
// (BM / 64) x 2, each 64 x BN/2): the accumulator tile goes through LDS (fp32) so that every thread
// then owns one 16-byte chunk (8 channels) of a row: bias, residual, mask and y operands are 16-byte
// loads and the output a 16-byte store. Straight from the MFMA layout a lane holds 1 column x 16 rows,
// i.e. 2-byte accesses (and 3-4x as many VMEM instructions again for the BN-backward operands).
// Staging layout: [BM][BN] fp32, column XOR-swizzled by bits 2-3 of the row — the four row groups of
// one MFMA write (rows 4q + e) land in four distinct 16-bank groups — and by bit 0 of the row into
// the other 16-byte half of each 32-byte chunk, so that at BN = 64 the two rows of a 16-lane read
// phase (8 chunks each) hit disjoint banks. The caller's operand buffers
// must be idle (a barrier after the last K step's LDS reads).
// per-thread column sums of the epilogue (8 channels): BN statistics (q0 = sum x, q1 = sum x^2) or
// BN-backward sums (q0 = sum g, q1 / q2 = sum g * xhat of the one / two BatchNorms)
struct EpiSums {
  float q0[8], q1[8], q2[8];
  __device__ void zero() {
#pragma unroll
    for (int j = 0; j < 8; ++j) q0[j] = q1[j] = q2[j] = 0.f;
  }
};

// One tile: stage, apply, store, and add this thread's rows into q (no reduction: see conv_epilogue_sums).
// PARTS > 1: the tile goes through a staging area of BM / PARTS rows (`stg`, fp32) in PARTS rounds,
// row slab by row slab (the waves of a slab stage, everyone applies), so that the rest of LDS can
// take the next tile's first operand stage meanwhile (k_conv_fwd_dma).
// SPEC >= 0: the epilogue's operand set fixed at compile time (bit 0 residual, 1 BN-backward sums,
// 2 a second BN, 3 ReLU mask from a materialised activation, 4 ReLU mask from y0 and the BN's
// scale / shift, 5 forward BN statistics; no bias, no ReLU, every column valid) — the runtime-flag epilogue keeps every
// variant's registers and branches live in the persistent halo dgrad (11.7 VALU per MFMA); -1: flags
// from the arguments.
// one tile's epilogue operand chunks (residual, ReLU mask, y0, y1), loaded ahead of the apply
template <int NP>
struct EpiPre {
  uint4 r[NP], m[NP], y0[NP], y1[NP];
};
template <int BM, int BN, int NT, int PARTS>
constexpr int epi_np() { return PARTS * ((BM / PARTS) / (NT / (BN / 8))); }

// output row of GEMM row m (MODE 2: back from the class sub-grid to the dX pixel)
template <int MODE>
__device__ __forceinline__ int conv_out_row(const ConvGemmArgs& a, int m, int hw, int rw, int ph, int pw) {
  if (MODE != 2) return m;
  const int img = m / hw, rem = m - img * hw;
  const int hh = rem / rw, ww = rem - hh * rw;
  return (img * a.out_h + 2 * hh + ph) * a.out_w + 2 * ww + pw;
}

// the loads of conv_epilogue_tile's operand chunks for a compile-time operand set (SPEC >= 0), in the
// order its passes consume them; rows past the batch (and a column chunk past ncol) load zeros
// through the buffer range check
template <int MODE, int BM, int BN, int NT, int PARTS, int SPEC>
__device__ __forceinline__ void conv_epilogue_prefetch(const ConvGemmArgs& a, int peer, int m0, int n0, int M, int hw, int rw, int ph, int pw,
                                                       EpiPre<epi_np<BM, BN, NT, PARTS>()>& pre) {
  static_assert(SPEC >= 0, "compile-time operand sets only");
  constexpr int CH = BN / 8, RP = NT / CH, SR = BM / PARTS, PASSES = SR / RP, NP = PARTS * PASSES;
  constexpr bool resid_on = (SPEC & 1) != 0, bnb = MODE != 0 && (SPEC & 2) != 0;
  constexpr bool bnb2 = bnb && (SPEC & 4) != 0, bmask_on = bnb && (SPEC & 8) != 0;
  const int tid = threadIdx.x, ch = tid % CH, rr = tid / CH;
  const int col0 = n0 + ch * 8;
  const bool chok = col0 < a.ncol;
  const uint4 z = make_uint4(0, 0, 0, 0);
  const __amdgpu_buffer_rsrc_t rr_ = conv_rsrc(resid_on ? a.resid + peer * a.resid_ps : a.out);
  const __amdgpu_buffer_rsrc_t rm_ = conv_rsrc(bmask_on ? a.bnb_mask + peer * a.bnb_mask_ps : a.out);
  const __amdgpu_buffer_rsrc_t r0_ = conv_rsrc(bnb ? a.bnb_y0 + peer * a.bnb_y0_ps : a.out);
  const __amdgpu_buffer_rsrc_t r1_ = conv_rsrc(bnb2 ? a.bnb_y1 + peer * a.bnb_y1_ps : a.out);
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    const int m = m0 + (k / PASSES) * SR + rr + (k % PASSES) * RP;
    const int off = (chok && m < M) ? (int)(((int64_t)conv_out_row<MODE>(a, m, hw, rw, ph, pw) * a.ncol + col0) * 2) : CONV_OOB;
    pre.r[k] = resid_on ? conv_ld16(rr_, off) : z;
    pre.m[k] = bmask_on ? conv_ld16(rm_, off) : z;
    pre.y0[k] = bnb ? conv_ld16(r0_, off) : z;
    pre.y1[k] = bnb2 ? conv_ld16(r1_, off) : z;
  }
}

// EPI_PF: with a compile-time operand set that reads residual / mask / y operands (the dgrads), all of
// this thread's operand chunks of the tile (every slab and pass) are loaded before the staging, in
// one round trip — the pass loop used to issue them two rows at a time, exposing one HBM round trip
// per two rows (four per 128 x 128 tile) while every wave of the workgroup waited in the epilogue.
#ifndef EPI_PF
#define EPI_PF 1
#endif
// ext: the operand chunks already loaded by the caller (conv_epilogue_prefetch, issued before the
// tile's MFMAs), or null
template <int MODE, int BM, int BN, int NT, int PARTS = 1, int SPEC = -1>
__device__ __forceinline__ void conv_epilogue_tile(const ConvGemmArgs& a, const f32x4 (&acc)[4][BN / 32], float* stg, int peer, int m0, int n0, int M,
                                                   int hw, int rw, int ph, int pw, EpiSums& q,
                                                   const EpiPre<epi_np<BM, BN, NT, PARTS>()>* ext = nullptr) {
  constexpr bool SP = SPEC >= 0;
  constexpr int NF = BN / 32;
  constexpr int SR = BM / PARTS;  // staged rows per round (a multiple of the 64 rows of a wave)
  static_assert(SR % 64 == 0, "staging rounds hold whole wave rows");
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  float* cst = stg;

  constexpr int CH = BN / 8, RP = NT / CH, PASSES = SR / RP, NW = NT / 64;
  const int ch = tid % CH, rr = tid / CH;
  const int col0 = n0 + ch * 8;
  const bool chok = col0 < a.ncol;  // ncol is a multiple of 8
  bf16* out = a.out + peer * a.out_ps;
  const bool resid_on = SP ? (SPEC & 1) != 0 : a.resid != nullptr;
  const bf16* resid = resid_on ? a.resid + peer * a.resid_ps : nullptr;
  // BN-backward epilogue (dgrad only)
  const bool bnb = MODE != 0 && (SP ? (SPEC & 2) != 0 : a.bnb_part0 != nullptr);
  const bool bnb2 = bnb && (SP ? (SPEC & 4) != 0 : a.bnb_part1 != nullptr);
  const bool bmask_on = bnb && (SP ? (SPEC & 8) != 0 : a.bnb_mask != nullptr);
  const bf16* bmask = bmask_on ? a.bnb_mask + peer * a.bnb_mask_ps : nullptr;
  const bool ymask = bnb && !bmask_on && (SP ? (SPEC & 16) != 0 : a.bnb_mask_ss != nullptr);  // mask = relu(BN(y0)) > 0
  const bool bias_on = !SP && a.bias != nullptr;
  const bool relu_on = !SP && a.relu;
  const bf16* by0 = bnb ? a.bnb_y0 + peer * a.bnb_y0_ps : nullptr;
  const bf16* by1 = bnb2 ? a.bnb_y1 + peer * a.bnb_y1_ps : nullptr;
  const bool fstats = !bnb && (SP ? (SPEC & 32) != 0 : a.stats != nullptr);
  // the per-column constants are re-read for every tile (pointers laundered through an empty asm):
  // hoisted out of a persistent kernel's tile loop they would hold 56 VGPRs across the MFMAs
  auto fresh = [](const float* p) {
    asm volatile("" : "+s"(p));
    return p;
  };
  float bv[8], mean0[8], inv0[8], mean1[8], inv1[8], msc[8], msh[8];
  float(&q0)[8] = q.q0;
  float(&q1)[8] = q.q1;
  float(&q2)[8] = q.q2;
  bool cval[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int col = col0 + j;
    cval[j] = SP || col < a.ncol_valid;
    bv[j] = (bias_on && cval[j]) ? fresh(a.bias + peer * a.bias_ps)[col] : 0.f;
    mean0[j] = inv0[j] = mean1[j] = inv1[j] = msc[j] = msh[j] = 0.f;
    if (ymask && chok) {
      const float* ssp = fresh(a.bnb_mask_ss + peer * a.bnb_mask_ss_ps);
      msc[j] = ssp[col];
      msh[j] = ssp[a.ncol + col];
    }
    if (bnb && chok) {
      const float* m0p = fresh(a.bnb_ms0 + peer * 2 * a.ncol);
      mean0[j] = m0p[col];
      inv0[j] = m0p[a.ncol + col];
      if (bnb2) {
        const float* m1p = fresh(a.bnb_ms1 + peer * 2 * a.ncol);
        mean1[j] = m1p[col];
        inv1[j] = m1p[a.ncol + col];
      }
    }
  }
  auto out_row = [&](int m) -> int { return conv_out_row<MODE>(a, m, hw, rw, ph, pw); };
  constexpr bool PF = EPI_PF && SP && (SPEC & 3) != 0;  // prefetch the operand chunks (see EPI_PF)
  EpiPre<epi_np<BM, BN, NT, PARTS>()> own;
  if (PF && ext == nullptr) conv_epilogue_prefetch<MODE, BM, BN, NT, PARTS, SP ? SPEC : 0>(a, peer, m0, n0, M, hw, rw, ph, pw, own);
  const EpiPre<epi_np<BM, BN, NT, PARTS>()>& pre = ext != nullptr ? *ext : own;
#pragma unroll
  for (int part = 0; part < PARTS; ++part) {
  if (wr * 64 / SR == part) {  // this wave's rows are in the slab: stage them
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < NF; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int row = wr * 64 - part * SR + i * 16 + 4 * (lane >> 4) + e;
          const int col = wc * (BN / 2) + j * 16 + (lane & 15);
          cst[row * BN + (col ^ (((row >> 2) & 3) << 4) ^ ((row & 1) << 2))] = acc[i][j][e];
        }
  }
  __syncthreads();
  if (chok) {
#pragma unroll PF ? PASSES : 2
    for (int p = 0; p < PASSES; ++p) {
      const int row = rr + p * RP;  // row within the slab
      const int m = m0 + part * SR + row;
      if (m >= M) break;
      const int64_t o = (int64_t)out_row(m) * a.ncol + col0;
      uint4 ur = make_uint4(0, 0, 0, 0), um = ur, uy0 = ur, uy1 = ur;
      if (PF) {
        ur = pre.r[part * PASSES + p];
        um = pre.m[part * PASSES + p];
        uy0 = pre.y0[part * PASSES + p];
        uy1 = pre.y1[part * PASSES + p];
      } else {
        if (resid_on) ur = *reinterpret_cast<const uint4*>(resid + o);
        if (bmask_on) um = *reinterpret_cast<const uint4*>(bmask + o);
        if (bnb) uy0 = *reinterpret_cast<const uint4*>(by0 + o);
        if (bnb2) uy1 = *reinterpret_cast<const uint4*>(by1 + o);
      }
      const int sw = (((row >> 2) & 3) << 4) ^ ((row & 1) << 2);
      const float4 lo = *reinterpret_cast<const float4*>(cst + row * BN + ((ch * 8) ^ sw));
      const float4 hi = *reinterpret_cast<const float4*>(cst + row * BN + ((ch * 8 + 4) ^ sw));
      float v[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
      const bf8 br = __builtin_bit_cast(bf8, ur), bm = __builtin_bit_cast(bf8, um);
      const bf8 b0 = __builtin_bit_cast(bf8, uy0), b1 = __builtin_bit_cast(bf8, uy1);
      bf8 ob;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float x = bias_on ? v[j] + bv[j] : v[j];
        if (resid_on) x += (float)br.v[j];
        if (relu_on) x = fmaxf(x, 0.f);
        if (!cval[j]) x = 0.f;
        if (bnb) {
          if (bmask_on && !((float)bm.v[j] > 0.f)) x = 0.f;
          // the bf16 activation relu(y*sc + sh) (bn_relu8) is > 0 exactly when y*sc + sh > 0
          if (ymask && !(fmaf((float)b0.v[j], msc[j], msh[j]) > 0.f)) x = 0.f;
          ob.v[j] = (bf16)x;
          const float g = (float)ob.v[j];  // the sums see exactly the g the BN apply reads back
          q0[j] += g;
          q1[j] += g * ((float)b0.v[j] - mean0[j]) * inv0[j];
          if (bnb2) q2[j] += g * ((float)b1.v[j] - mean1[j]) * inv1[j];
        } else {
          ob.v[j] = (bf16)x;
          q0[j] += x;
          q1[j] += x * x;
        }
      }
      *reinterpret_cast<uint4*>(out + o) = __builtin_bit_cast(uint4, ob);
    }
  }
  if (PARTS > 1) __syncthreads();  // the slab is read: the next round may restage
  }
}

// The column sums of one or more tiles (q) -> one atomic per column and statistic into accumulator
// row `srow` of the peer (rows spread the atomics of many workgroups over several addresses). Over
// the wave's rows (lanes of one chunk) by shuffles, over the waves in LDS (the staging tile must no
// longer be read: this starts with a barrier).
template <int MODE, int BN, int NT, int SPEC = -1>
__device__ __forceinline__ void conv_epilogue_sums(const ConvGemmArgs& a, bf16* lds, int peer, int n0, int srow, EpiSums& q) {
  constexpr int CH = BN / 8, NW = NT / 64;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ch = tid % CH;
  const bool bnb = MODE != 0 && (SPEC >= 0 ? (SPEC & 2) != 0 : a.bnb_part0 != nullptr);
  const bool bnb2 = bnb && (SPEC >= 0 ? (SPEC & 4) != 0 : a.bnb_part1 != nullptr);
  const bool fstats = !bnb && (SPEC >= 0 ? (SPEC & 32) != 0 : a.stats != nullptr);
  if (!bnb && !fstats) return;
  float(&q0)[8] = q.q0;
  float(&q1)[8] = q.q1;
  float(&q2)[8] = q.q2;
  float* cst = reinterpret_cast<float*>(lds);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
#pragma unroll
    for (int off = CH; off < 64; off <<= 1) {
      q0[j] += __shfl_xor(q0[j], off);
      q1[j] += __shfl_xor(q1[j], off);
      if (bnb2) q2[j] += __shfl_xor(q2[j], off);
    }
  }
  __syncthreads();  // staging tile no longer read
  float* red = cst;  // [NW waves][3][BN]
  if (lane < CH) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[(wave * 3 + 0) * BN + ch * 8 + j] = q0[j];
      red[(wave * 3 + 1) * BN + ch * 8 + j] = q1[j];
      red[(wave * 3 + 2) * BN + ch * 8 + j] = q2[j];
    }
  }
  __syncthreads();
  if (tid < BN) {
    const int col = n0 + tid;
    if (col < a.ncol) {
      float t0 = 0.f, t1 = 0.f, t2 = 0.f;
#pragma unroll
      for (int w = 0; w < NW; ++w) {
        t0 += red[(w * 3 + 0) * BN + tid];
        t1 += red[(w * 3 + 1) * BN + tid];
        t2 += red[(w * 3 + 2) * BN + tid];
      }
      if (bnb) {
        const int prow = srow % (a.bnb_rows > 1 ? a.bnb_rows : 1);
        float* p0 = a.bnb_part0 + peer * a.bnb_part_ps + prow * 2 * a.ncol;
        atomicAdd(p0 + col, t0);
        atomicAdd(p0 + a.ncol + col, t1);
        if (bnb2) {
          float* p1 = a.bnb_part1 + peer * a.bnb_part_ps + prow * 2 * a.ncol;
          atomicAdd(p1 + col, t0);
          atomicAdd(p1 + a.ncol + col, t2);
        }
      } else {
        // BatchNorm batch statistics straight into the peer's [2][ncol] accumulator (bn_finalize
        // reads and re-zeroes it)
        float* st = a.stats + peer * a.stats_ps + (srow % (a.stats_rows > 1 ? a.stats_rows : 1)) * 2 * a.ncol;
        atomicAdd(st + col, t0);
        atomicAdd(st + a.ncol + col, t1);
      }
    }
  }
}

// one tile's whole epilogue (its sums into accumulator row m0 / 128)
template <int MODE, int BM, int BN, int NT, int SPEC = -1>
__device__ __forceinline__ void conv_epilogue(const ConvGemmArgs& a, const f32x4 (&acc)[4][BN / 32], bf16* lds, int peer, int m0, int n0, int M,
                                              int hw, int rw, int ph, int pw) {
  EpiSums q;
  q.zero();
  conv_epilogue_tile<MODE, BM, BN, NT, 1, SPEC>(a, acc, reinterpret_cast<float*>(lds), peer, m0, n0, M, hw, rw, ph, pw, q);
  conv_epilogue_sums<MODE, BN, NT, SPEC>(a, lds, peer, n0, m0 >> 7, q);
}

// ------------------------------------------------------------------------------------------------
// Fused BatchNorm finalize (ConvGemmArgs::fin_cnt): the work of k_bn_finalize / k_bn_bwd_finalize
// (cnn_ops.hip) done by the peer's last workgroup to finish, instead of a launch of its own after
// every BN-producing conv (~40 launches of ~5 us plus their gaps per ResNet-18 step). The epilogue
// sums are float atomics, which execute at the memory side and leave no L2 copy; every wave waits
// for its own (vmcnt 0), the workgroup barrier joins them, one lane draws an arrival ticket from
// the peer's counter (agent-scope atomic) and the workgroup with the last ticket reads the rows
// back with sc1 loads and re-arms them with sc1 stores (conv_fin_gather): arrival-ticket hand-off,
// MI355X_MICROARCH.md inter-workgroup visibility, valid-forms row 1. No workgroup waits for another.
// ------------------------------------------------------------------------------------------------
// red[j] = sum over the `rows` accumulator rows of base[r * E2 + j] (j < E2, E2 % 4 == 0), every
// element re-armed to 0. The rows were written only by memory-side float atomics of this launch
// (no L2 copy anywhere), so 16-byte sc1 loads (L1 bypassed, aux 16) read their final values, and
// sc1 zero stores (write-through: the line leaves this XCD's L2 as well) re-arm them for the next
// launch. Each thread sums its chunk column over a row subset in registers (all its loads in
// flight), the subsets are added in a fixed order. Measured slower forms (profiles/r4u_bn_fin_tail):
// reading the rows back by atomic exchange (+13-31 us per conv: one CU issuing 16 x 2 x Cp
// returning atomics), LDS float atomicAdd of the loaded chunks (+12-45 us).
__device__ __forceinline__ void conv_fin_gather(float* base, int rows, int E2, float* red) {
  const int NT = (int)blockDim.x, tid = (int)threadIdx.x;
  const int Q = E2 >> 2;                  // 16-byte chunks per row
  const int TPC = Q <= NT ? NT / Q : 1;   // threads per chunk column (each sums a row subset)
  const __amdgpu_buffer_rsrc_t rs = conv_rsrc(base);
  float* part = red + E2;                 // [TPC][E2] partial column sums, reduced in fixed order
  constexpr int U = 16;
  for (int q0 = 0; q0 < Q; q0 += (Q <= NT ? Q : NT)) {
    const int q = q0 + (Q <= NT ? tid % Q : tid), rr = Q <= NT ? tid / Q : 0;
    if (q < Q && rr < TPC) {
      float acc[4] = {0.f, 0.f, 0.f, 0.f};
      for (int r = rr; r < rows; r += U * TPC) {
        conv_u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int ri = r + u * TPC;
          v[u] = (conv_u32x4)__builtin_amdgcn_raw_buffer_load_b128(rs, ri < rows ? (ri * Q + q) * 16 : CONV_OOB, 0, 16);
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {  // out-of-range rows loaded zeros
          acc[0] += __uint_as_float(v[u].x);
          acc[1] += __uint_as_float(v[u].y);
          acc[2] += __uint_as_float(v[u].z);
          acc[3] += __uint_as_float(v[u].w);
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) part[rr * E2 + q * 4 + k] = acc[k];
    }
  }
  __syncthreads();
  for (int j = tid; j < E2; j += NT) {
    float t = 0.f;
    for (int k = 0; k < TPC; ++k) t += part[k * E2 + j];
    red[j] = t;
  }
  const conv_u32x4 z = {0u, 0u, 0u, 0u};
  for (int e = tid; e < rows * Q; e += NT) __builtin_amdgcn_raw_buffer_store_b128(z, rs, e * 16, 0, 16);
  __syncthreads();
}

// The per-channel operands are loaded before the gather (channels tid + k * blockDim.x, k < 4:
// ncol <= 4 * blockDim.x, checked by conv_gemm_launch), so their latency overlaps it.
constexpr int FIN_CPT = 4;
__device__ __forceinline__ void conv_fin_fwd(const ConvGemmArgs& a, int peer, float* red) {
  const int Cp = a.ncol, NT = (int)blockDim.x, tid = (int)threadIdx.x;
  const bool train = a.fin_train != 0 && a.stats != nullptr;
  const int n = (a.nbatch ? a.nbatch[peer] : a.max_batch) * a.out_h * a.out_w;
  const float cnt = (float)max(1, n);
  float* ssp = a.fin_ss + peer * 2 * Cp;
  float* msp = a.fin_ms + peer * 2 * Cp;
  float* rm = a.fin_rmean + peer * a.fin_run_ps;
  float* rv = a.fin_rvar + peer * a.fin_run_ps;
  float g[FIN_CPT], b[FIN_CPT], m0[FIN_CPT], v0[FIN_CPT];
#pragma unroll
  for (int k = 0; k < FIN_CPT; ++k) {
    const int c = tid + k * NT;
    const bool on = c < a.fin_C0;
    g[k] = on ? a.fin_gamma0[peer * a.fin_param_ps + c] : 0.f;
    b[k] = on ? a.fin_beta[peer * a.fin_param_ps + c] : 0.f;
    m0[k] = on ? rm[c] : 0.f;
    v0[k] = on ? rv[c] : 1.f;
  }
  if (train) conv_fin_gather(a.stats + peer * a.stats_ps, a.stats_rows > 1 ? a.stats_rows : 1, 2 * Cp, red);
#pragma unroll
  for (int k = 0; k < FIN_CPT; ++k) {
    const int c = tid + k * NT;
    if (c >= Cp) break;
    if (c >= a.fin_C0) {
      ssp[c] = 0.f; ssp[Cp + c] = 0.f; msp[c] = 0.f; msp[Cp + c] = 0.f;
      continue;
    }
    float mean = m0[k], var = v0[k];
    if (train) {
      mean = red[c] / cnt;
      var = fmaxf(red[Cp + c] / cnt - mean * mean, 0.f);
      if (n > 0) {  // a peer without samples this step keeps its running statistics
        const float unbiased = cnt > 1.f ? var * cnt / (cnt - 1.f) : var;
        rm[c] = (1.f - a.fin_momentum) * m0[k] + a.fin_momentum * mean;
        rv[c] = (1.f - a.fin_momentum) * v0[k] + a.fin_momentum * unbiased;
      }
    }
    const float inv = rsqrtf(var + a.fin_eps);
    ssp[c] = g[k] * inv;
    ssp[Cp + c] = b[k] - mean * g[k] * inv;
    msp[c] = mean;
    msp[Cp + c] = inv;
  }
}

__device__ __forceinline__ void conv_fin_bwd(const ConvGemmArgs& a, int peer, float* part, const float* ms, const float* gamma, float* dgamma,
                                             float* dbeta, float* coef, int C, float* red) {
  const int Cp = a.ncol, NT = (int)blockDim.x, tid = (int)threadIdx.x;
  const float cnt = (float)max(1, (a.nbatch ? a.nbatch[peer] : a.max_batch) * a.out_h * a.out_w);
  float* cp = coef + peer * 3 * Cp;
  float k1[FIN_CPT], dg[FIN_CPT], db[FIN_CPT];
#pragma unroll
  for (int k = 0; k < FIN_CPT; ++k) {
    const int c = tid + k * NT;
    const bool on = c < C;
    k1[k] = on ? gamma[peer * a.fin_param_ps + c] * ms[peer * 2 * Cp + Cp + c] : 0.f;
    dg[k] = on ? dgamma[peer * a.fin_param_ps + c] : 0.f;
    db[k] = on ? dbeta[peer * a.fin_param_ps + c] : 0.f;
  }
  conv_fin_gather(part + peer * a.bnb_part_ps, a.bnb_rows > 1 ? a.bnb_rows : 1, 2 * Cp, red);
#pragma unroll
  for (int k = 0; k < FIN_CPT; ++k) {
    const int c = tid + k * NT;
    if (c >= Cp) break;
    if (c >= C) {
      cp[c] = 0.f; cp[Cp + c] = 0.f; cp[2 * Cp + c] = 0.f;
      continue;
    }
    const float sg = red[c], sgx = red[Cp + c];
    dgamma[peer * a.fin_param_ps + c] = dg[k] + sgx;
    dbeta[peer * a.fin_param_ps + c] = db[k] + sg;
    cp[c] = k1[k];
    cp[Cp + c] = sg / cnt;
    cp[2 * Cp + c] = sgx / cnt;
  }
}

// Arrival counters, per peer: one top word and FIN_SHARDS shard words, each on its own 128-byte
// line. A workgroup draws its ticket from shard (block index % FIN_SHARDS), the last of a shard from
// the top word. One counter per peer that every workgroup hit cost ~30 us per conv: returning
// atomics on one line serialize at the memory side (~256 workgroups x 8 peers on one line,
// profiles/r4u_bn_fin_tail); a shard sees ~1/8 of the arrivals, the top word at most 8.
constexpr int FIN_LINE = 32, FIN_SHARDS = 8, FIN_WORDS = (FIN_SHARDS + 1) * FIN_LINE;

// every workgroup calls this exactly once, as its last action (early exits included); flag: LDS the
// workgroup no longer uses (one word + 2 * ncol floats from word 4)
__device__ __forceinline__ void conv_fin_tail(const ConvGemmArgs& a, int peer, int* flag) {
  if (a.fin_cnt == nullptr) return;
  if (!(a.fin_dbg & 1)) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's epilogue atomics performed
  __syncthreads();
  if (a.fin_dbg & 2) return;
  if (threadIdx.x == 0) {
    int* cnt = a.fin_cnt + peer * FIN_WORDS;
    const int nwg = (int)(gridDim.x * gridDim.y), b = (int)(blockIdx.y * gridDim.x + blockIdx.x);
    const int sh = b % FIN_SHARDS;
    const int members = nwg / FIN_SHARDS + (sh < nwg % FIN_SHARDS ? 1 : 0);
    int* sc = cnt + (1 + sh) * FIN_LINE;
    bool last = false;
    // release: this workgroup's epilogue sums (every wave drained, then the barrier above) are
    // visible before its ticket; the shard's last arriver acquires its members' and releases them on
    // with the top ticket; the last workgroup acquires everything before it gathers
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    if (__hip_atomic_fetch_add(sc, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == members - 1) {
      __hip_atomic_store(sc, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == min(FIN_SHARDS, nwg) - 1;
      if (last) {
        __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      }
    }
    *flag = last ? 1 : 0;
  }
  __syncthreads();
  if (*flag == 0 || (a.fin_dbg & 4)) return;
  float* red = reinterpret_cast<float*>(flag) + 4;  // [2 * ncol] column sums
  if (a.fin_ss != nullptr) {
    conv_fin_fwd(a, peer, red);
  } else {
    if (a.bnb_part0 != nullptr) conv_fin_bwd(a, peer, a.bnb_part0, a.bnb_ms0, a.fin_gamma0, a.fin_dgamma0, a.fin_dbeta0, a.fin_coef0, a.fin_C0, red);
    __syncthreads();  // red reused
    if (a.bnb_part1 != nullptr) conv_fin_bwd(a, peer, a.bnb_part1, a.bnb_ms1, a.fin_gamma1, a.fin_dgamma1, a.fin_dbeta1, a.fin_coef1, a.fin_C1, red);
  }
}

template <int MODE, int BN, bool PRO, int SPEC = -1>
__global__ __launch_bounds__(256, 2) void k_conv_gemm(ConvGemmArgs a, int tiles_m, int tiles_n) {
  // MODE 0 forward, MODE 1 dgrad (all taps; MODE 3 = MODE 1 at stride 1), MODE 2 strided dgrad by output parity class,
  // MODE 4 stride-1 dgrad run as a forward conv over dY (pad R-1-pad) with the flipped, transposed
  // weights Wt[ci][R-1-r][S-1-s][co] (k_conv_wt_flip): the forward's K-contiguous B panel and tap
  // walk (measured 15-25 % faster than MODE 3 per layer), with the dgrad epilogue (BN-backward sums)
  // (blockIdx.y = class (ph, pw): rows are the dX pixels (2hh+ph, 2ww+pw), K walks only the taps
  // r = r0 + 2i, s = s0 + 2j that reach them — a plain stride-2 dgrad multiplies zeros for 3 of
  // every 4 (pixel, tap) pairs)
  constexpr int BM = 128;
  constexpr int AR = BM / 32;          // A rows (16-byte chunks) per thread
  constexpr int NB = BN / 32;          // B 16-byte chunks per thread
  constexpr int NF = BN / 32;          // n-fragments per wave (2 x 2 waves, each 64 x BN/2)
  constexpr bool FWD = MODE == 0 || MODE == 4;  // forward gathers (MODE 4: stride-1 dgrad as a forward conv)
  constexpr bool BT = !FWD;            // B staged [k][n] (N-contiguous source)
  constexpr int BUF = BM * CG_BK + BN * CG_BK;
  __shared__ __attribute__((aligned(16))) bf16 lds[2 * BUF];

  const int peer = blockIdx.z;
  const int nb = a.nbatch ? a.nbatch[peer] : a.max_batch;
  // row geometry (MODE 2: the parity class's sub-grid of dX)
  const int ph = MODE == 2 ? (int)(blockIdx.y >> 1) : 0, pw = MODE == 2 ? (int)(blockIdx.y & 1) : 0;
  const int rh = MODE == 2 ? (a.out_h - ph + 1) >> 1 : a.out_h;
  const int rw = MODE == 2 ? (a.out_w - pw + 1) >> 1 : a.out_w;
  const int r0 = MODE == 2 ? (ph + a.pad) & 1 : 0, s0 = MODE == 2 ? (pw + a.pad) & 1 : 0;
  const int tR = MODE == 2 ? (a.R - r0 + 1) >> 1 : a.R;  // taps walked along r / s
  const int tS = MODE == 2 ? (a.S - s0 + 1) >> 1 : a.S;
  const int hw = rh * rw;
  const int M = nb * hw;
  const int wgid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tn = wgid % tiles_n, tm = wgid / tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;

  if (m0 >= M) {  // tile past this peer's batch
    conv_fin_tail(a, peer, reinterpret_cast<int*>(lds));
    return;
  }

  const bf16* src = a.src + peer * a.src_ps;
  const bf16* wt = a.wt + peer * a.wt_ps;
  const __amdgpu_buffer_rsrc_t rs_src = conv_rsrc(src), rs_wt = conv_rsrc(wt);
  (void)rs_src;
  (void)rs_wt;
  // PRO (MODE 0): the source is a BN output y; the A operand is relu(y*sc + sh) of the previous
  // BatchNorm, applied when the staged registers go to LDS (after this K-step's MFMAs, so the
  // loads stay in flight across them; transforming at load time put a vmcnt(0) before the MFMAs)
  const float* pro = PRO ? a.pro_ss + peer * a.pro_ss_ps : nullptr;
  const int Ktot = (tR > 0 && tS > 0) ? tR * tS * a.src_c : 0;  // 0: a parity class no tap reaches (zeros + resid)
  const int nk = (Ktot + CG_BK - 1) / CG_BK;
  const int cc = tid & 7;            // this thread's 16-byte chunk within a K-step
  const int cpp = a.src_c >> 3;      // chunks per pixel

  // per-thread A rows (fixed for the whole K loop): a_bh/a_bw = source coordinate of tap (0, 0)
  int a_img[AR], a_bh[AR], a_bw[AR];
  bool a_ok[AR];
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    const int m = m0 + (tid >> 3) + 32 * i;
    a_ok[i] = m < M;
    const int mm = a_ok[i] ? m : 0;
    const int img = mm / hw, rem = mm - img * hw;
    const int oh = rem / rw, ow = rem - oh * rw;
    a_img[i] = img * a.src_h * a.src_w;
    if (FWD) {
      a_bh[i] = oh * a.stride - a.pad;
      a_bw[i] = ow * a.stride - a.pad;
    } else if (MODE == 1 || MODE == 3) {
      a_bh[i] = oh + a.pad;
      a_bw[i] = ow + a.pad;
    } else {  // dY row of tap (r0, s0) for dX pixel (2oh+ph, 2ow+pw); tap i steps back one dY row
      a_bh[i] = oh + ((ph + a.pad - r0) >> 1);
      a_bw[i] = ow + ((pw + a.pad - s0) >> 1);
    }
  }

  // K-walk state, advanced incrementally (the im2col index math was ~6-22 VALU per MFMA with a
  // division-based decomposition per K-step): this thread's A chunk is q8 = kt * 8 + cc of
  // (tap r, tap s, c8); B rows (MODE 1/2) are (tap, co) pairs
  const float inv_st = 1.f / (float)a.stride;
  int ar = 0, as_ = 0, ac8 = cc;
  while (ac8 >= cpp) {
    ac8 -= cpp;
    if (++as_ == tS) { as_ = 0; ++ar; }
  }
  int a_pix[AR];  // MODE 0: pixel index of tap (0, 0)
#pragma unroll
  for (int i = 0; i < AR; ++i) a_pix[i] = a_img[i] + a_bh[i] * a.src_w + a_bw[i];
  // element offset of each row's tap-(0, 0) pixel: a K step adds (MODE 0) or subtracts (MODE 2 / 3)
  // one per-thread tap offset, so the rows need no multiply in the K loop
  int a_pixc[AR];
#pragma unroll
  for (int i = 0; i < AR; ++i) a_pixc[i] = a_pix[i] * a.src_c;
  constexpr int BCH = BN / 8;          // BT: 16-byte chunks per staged k row
  const int bt_c = tid % BCH, bt_r = tid / BCH;
  int b_t[NB], b_co[NB];
  if (BT) {
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int kk = bt_r + (256 / BCH) * i;
      b_t[i] = kk / a.src_c;
      b_co[i] = kk - b_t[i] * a.src_c;
    }
  }
  const int RS = a.R * a.S, TT = tR * tS;
  const float inv_tS = 1.f / (float)(tS > 0 ? tS : 1);  // MODE 2: tap index -> (ti, tj) without an integer division
  uint4 ra[AR], rb[NB];
  float4 psc[2], psh[2];  // PRO: scale / shift of the staged chunk's 8 channels
  unsigned aok = 0;       // PRO: staged A rows that are real pixels (padding stays 0, not relu(sh))
  auto load = [&](int kt) {
    const int k = kt * CG_BK + cc * 8;
    const bool kok = ar < tR;
    const int r = ar, s = as_, c8 = ac8;
    const int tapc = (r * a.src_w + s) * a.src_c;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      bool ok = kok && a_ok[i];
      int pix;
      int eoff = 0;  // element offset for the strength-reduced modes (0, 2, 3)
      if (FWD) {
        ok = ok && (unsigned)(a_bh[i] + r) < (unsigned)a.src_h && (unsigned)(a_bw[i] + s) < (unsigned)a.src_w;
        pix = a_pix[i] + r * a.src_w + s;
        eoff = a_pixc[i] + tapc + c8 * 8;
      } else if (MODE == 2) {
        const int h = a_bh[i] - r, w = a_bw[i] - s;
        ok = ok && (unsigned)h < (unsigned)a.src_h && (unsigned)w < (unsigned)a.src_w;
        pix = a_img[i] + h * a.src_w + w;
        eoff = a_pixc[i] - tapc + c8 * 8;
      } else {
        const int th = a_bh[i] - r, tw = a_bw[i] - s;
        int h, w;
        if (MODE == 3 || a.stride == 1) {
          h = th;
          w = tw;
        } else {
          h = th >= 0 ? fdiv(th, a.stride, inv_st) : -1;
          w = tw >= 0 ? fdiv(tw, a.stride, inv_st) : -1;
          ok = ok && h * a.stride == th && w * a.stride == tw;
        }
        ok = ok && th >= 0 && tw >= 0 && (unsigned)h < (unsigned)a.src_h && (unsigned)w < (unsigned)a.src_w;
        pix = a_img[i] + h * a.src_w + w;
        eoff = MODE == 3 ? a_pixc[i] - tapc + c8 * 8 : pix * a.src_c + c8 * 8;
      }
      if (CONV_BUFLOAD)
        ra[i] = conv_ld16(rs_src, ok ? eoff * 2 : CONV_OOB);
      else
        ra[i] = ok ? *reinterpret_cast<const uint4*>(src + pix * a.src_c + c8 * 8) : make_uint4(0, 0, 0, 0);
      if (PRO) aok = ok ? (aok | (1u << i)) : (aok & ~(1u << i));
    }
    if (PRO) {
      const float4* p4 = reinterpret_cast<const float4*>(pro + c8 * 8);
      const float4* q4 = reinterpret_cast<const float4*>(pro + a.src_c + c8 * 8);
      psc[0] = p4[0]; psc[1] = p4[1];
      psh[0] = q4[0]; psh[1] = q4[1];
    }
    // advance the A chunk by one K-step (8 chunks)
    ac8 += 8;
    while (ac8 >= cpp) {
      ac8 -= cpp;
      if (++as_ == tS) { as_ = 0; ++ar; }
    }
    if (!BT) {
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int n = n0 + (tid >> 3) + 32 * i;
        if (CONV_BUFLOAD)
          rb[i] = conv_ld16(rs_wt, (k < Ktot && n < a.ncol) ? (n * Ktot + k) * 2 : CONV_OOB);
        else
          rb[i] = (k < Ktot && n < a.ncol) ? *reinterpret_cast<const uint4*>(wt + (int64_t)n * Ktot + k) : make_uint4(0, 0, 0, 0);
      }
    } else {
      // k row = (tap, co): Wf[co][r][s][n0 + 8 * chunk ..] (ncol = Wf row length = cp_in)
      const int n = n0 + bt_c * 8;
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const bool ok = b_t[i] < TT && n < a.ncol;
        int rs = b_t[i];
        if (MODE == 2) {
          const int ti = tS == 1 ? b_t[i] : fdiv(b_t[i], tS, inv_tS), tj = b_t[i] - ti * tS;
          rs = (r0 + 2 * ti) * a.S + s0 + 2 * tj;
        }
        if (CONV_BUFLOAD)
          rb[i] = conv_ld16(rs_wt, ok ? ((b_co[i] * RS + rs) * a.ncol + n) * 2 : CONV_OOB);
        else
          rb[i] = ok ? *reinterpret_cast<const uint4*>(wt + (b_co[i] * RS + rs) * a.ncol + n) : make_uint4(0, 0, 0, 0);
        b_co[i] += CG_BK;
        while (b_co[i] >= a.src_c) {
          b_co[i] -= a.src_c;
          ++b_t[i];
        }
      }
    }
  };
  auto store = [&](int buf) {
    bf16* As = lds + buf * BUF;
    bf16* Bs = As + BM * CG_BK;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      uint4 v = ra[i];
      if (PRO && ((aok >> i) & 1u)) v = bn_relu8(v, reinterpret_cast<const float*>(psc), reinterpret_cast<const float*>(psh));
      *reinterpret_cast<uint4*>(As + swz((tid >> 3) + 32 * i, cc)) = v;
    }
    if (!BT) {
#pragma unroll
      for (int i = 0; i < NB; ++i) *reinterpret_cast<uint4*>(Bs + swz((tid >> 3) + 32 * i, cc)) = rb[i];
    } else {
#pragma unroll
      for (int i = 0; i < NB; ++i) *reinterpret_cast<uint4*>(Bs + tr_off<BN>(bt_r + (256 / BCH) * i, bt_c * 8)) = rb[i];
    }
  };
  f32x4 acc[4][NF];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[i][j] = zero4();

  static_assert(BM * BN * 4 <= 2 * BUF * 2, "staging tile must fit the operand buffers");
  // one register stage (loads of K-step kt+1 in flight during kt's MFMAs); measured: a second
  // register stage with LDS-only barriers is 20-60 % slower here (VGPR pressure, occupancy)
  if (nk > 0) {
    load(0);
    store(0);
  }
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) load(kt + 1);
    const bf16* As = lds + cur * BUF;
    const bf16* Bs = As + BM * CG_BK;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int ch = h * 4 + (lane >> 4);
      bf16x8 af[4], bfr[NF];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = ld8(As + swz(wr * 64 + i * 16 + (lane & 15), ch));
#pragma unroll
      for (int j = 0; j < NF; ++j)
        bfr[j] = BT ? frag_tr<BN>(Bs, wc * (BN / 2) + j * 16, h * 32, lane) : ld8(Bs + swz(wc * (BN / 2) + j * 16 + (lane & 15), ch));
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < NF; ++j) acc[i][j] = mfma_bf16(af[i], bfr[j], acc[i][j]);
    }
    if (kt + 1 < nk) store(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  // ---------------------------------------------------------------- epilogue
  conv_epilogue<MODE, BM, BN, 256, SPEC>(a, acc, lds, peer, m0, n0, M, hw, rw, ph, pw);
  conv_fin_tail(a, peer, reinterpret_cast<int*>(lds));
}

// ------------------------------------------------------------------------------------------------
// forward-shaped convs (MODE 0 without the BN prologue, MODE 4) through an LDS-DMA stage ring
// ------------------------------------------------------------------------------------------------
// k_conv_fwd_dma<MODE, BM, BN, NS, MINB>: the same implicit GEMM as k_conv_gemm's forward gathers,
// restructured around gfx950 direct-to-LDS loads (buffer_load_dwordx4 ... lds):
//   BM x BN tiles, 2 BM threads (BM / 32 waves as (BM / 64) x 2, each 64 x BN/2 — the same per-wave
//   MFMA block as k_conv_gemm), NS LDS stages of [BM][64] A + [BN][64] B, MINB workgroups per CU.
//   Every operand chunk goes HBM/L2 -> LDS with no VGPR destination: the K loop keeps NS - 1 stages
//   in flight across its barriers (counted vmcnt, raw s_barrier — __syncthreads() would drain them),
//   instead of the register stage of k_conv_gemm, which covers one K step of MFMAs (the convs were
//   latency-bound: 43-58 % of wave cycles waiting, profiles/r2l_cnn_pmc).
//   LDS-DMA writes lane l of a wave instruction at base + 16 l, so a wave instruction fills 8
//   contiguous 128-byte rows; the XOR chunk swizzle of swz() is applied on the SOURCE side: lane l
//   loads logical chunk (l & 7) ^ ((row >> 1) & 7), which for rows 8 (w + NW i) + (l >> 3) (NW waves,
//   even) is the same chunk cc for all of a thread's rows — so one incremental (r, s, c8) tap walk
//   per thread serves every A row, and the B rows (K-contiguous weight rows) use the same chunk.
//   Padding taps, rows past the batch and K past R*S*C load through an out-of-range offset: the
//   buffer unit writes zeros.
// Configurations (conv_gemm_launch, measured on the ResNet-18 shapes, profiles/r3z_conv_dma): two
// stages and more workgroups per CU beat a deeper ring — 128 x 128 / 2 stages / 2 per CU for the wide
// layers and 128 x 64 / 2 stages / 3 per CU for the 64-channel ones are 10-15 % faster than the
// register stage on every forward and MODE 4 shape (layer-4 forward 90.0 -> 76.1 us, 1016 TF/s;
// layer-1 forward 159.1 -> 135.5 us); 256 x 128 / 3 stages / 1 per CU is 12 % faster on layers 3-4
// only, and 3-stage 64-channel tiles are slower than the register stage (short K: 9 K steps).
// The epilogue (bias, residual, ReLU, BN sums / BN-backward sums) is conv_epilogue.
#ifndef CONV_XT
// k_conv_fwd_dma forward: the next tile's first stage under the epilogue. Measured neutral (layer-1
// forward with statistics 161 vs 158 us, ResNet-18 2.199 / 2.199 vs 2.211 / 2.195 rounds/s,
// profiles/r3z_conv_dma/xtab): the slab-staged epilogue's extra barriers eat the overlap. Off.
#define CONV_XT 0
#endif
typedef __attribute__((address_space(3))) void lds_void;
// stride-2 dgrad parity classes (ph, pw) = (c >> 1, c & 1): taps of the classes before class c
// (their weights come first in the parity-flipped layout)
__host__ __device__ __forceinline__ int conv_parity_taps(int R, int S, int pad, int c) {
  const int r0 = ((c >> 1) + pad) & 1, s0 = ((c & 1) + pad) & 1;
  return ((R - r0 + 1) >> 1) * ((S - s0 + 1) >> 1);
}
__host__ __device__ __forceinline__ int conv_parity_taps_before(int R, int S, int pad, int c) {
  int t = 0;
  for (int k = 0; k < c; ++k) t += conv_parity_taps(R, S, pad, k);
  return t;
}
__device__ __forceinline__ void conv_dma16(__amdgpu_buffer_rsrc_t r, bf16* lds_wave_base, int byte_off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)lds_wave_base, 16, byte_off, 0, 0, 0);
}
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

template <int MODE, int BM, int BN, int NS, int MINB, int SPEC = -1>
__global__ __launch_bounds__(2 * BM, MINB) void k_conv_fwd_dma(ConvGemmArgs a, int tiles_m, int tiles_n) {
  static_assert(MODE == 0 || MODE == 4 || MODE == 5, "forward-shaped gathers only");
  constexpr int EMODE = MODE == 5 ? 2 : MODE;  // epilogue: MODE 5 writes MODE 2's class rows
  constexpr int NT = 2 * BM, NW = NT / 64;
  constexpr int AR = BM * 8 / NT;  // A 16-byte chunks per thread per K step (4)
  constexpr int NB = BN * 8 / NT;  // B chunks per thread per K step
  static_assert(NB >= 1 && NW % 2 == 0, "tile shape");
  constexpr int G_ = AR + NB;      // LDS-DMA instructions per thread per stage
  constexpr int NF = BN / 32;
  constexpr int STAGE = (BM + BN) * CG_BK;
  constexpr int OPER = NS * STAGE, EPI = BM * BN * 2;  // bf16 units (the epilogue stages fp32)
  static_assert(NS >= 2 && NS <= 4, "stage ring depth");
  // one LDS object only: a second one makes hipcc wait vmcnt(0) before the K loop's LDS reads
  __shared__ __attribute__((aligned(16))) bf16 lds[OPER > EPI ? OPER : EPI];

  // Persistent over M tiles: gridDim.x = G * tiles_n workgroups per peer; workgroup (g, tn) runs
  // the tiles tm = g, g + G, ... of column tile tn and keeps the epilogue's column sums (BN
  // statistics / BN-backward sums) in registers across them, so a conv issues one set of atomics
  // per workgroup instead of per tile (the 64-channel layers have 1024 tiles per peer adding into
  // the same columns).
  //
  // MODE 5: the stride-2 dgrad of parity class blockIdx.y = (ph, pw) — rows are the dX pixels
  // (2hh + ph, 2ww + pw), reached by the taps r = r0 + 2i, s = s0 + 2j only — run as a stride-1
  // forward conv over dY with the class's tR x tS taps flipped (tap i' = tR-1-i reads dY row
  // hh - pad' + i', pad' = tR - 1 - (ph + pad - r0) / 2) and the class weights written by
  // k_conv_wt_flip (parity layout: classes in order, each [ci][tR][tS][co]).
  const int peer = blockIdx.z;
  const int nb = a.nbatch ? a.nbatch[peer] : a.max_batch;
  int gh = a.out_h, gw = a.out_w, kR = a.R, kS = a.S, kst = a.stride, pad_h = a.pad, pad_w = a.pad, ph = 0, pw = 0;
  int woff = 0;  // element offset of the class's weights
  if (MODE == 5) {
    ph = (int)blockIdx.y >> 1;
    pw = (int)blockIdx.y & 1;
    const int r0 = (ph + a.pad) & 1, s0 = (pw + a.pad) & 1;
    kR = (a.R - r0 + 1) >> 1;
    kS = (a.S - s0 + 1) >> 1;
    gh = (a.out_h - ph + 1) >> 1;
    gw = (a.out_w - pw + 1) >> 1;
    pad_h = kR - 1 - ((ph + a.pad - r0) >> 1);
    pad_w = kS - 1 - ((pw + a.pad - s0) >> 1);
    kst = 1;
    woff = conv_parity_taps_before(a.R, a.S, a.pad, (int)blockIdx.y) * a.src_c * a.ncol;
  }
  const int hw = gh * gw;
  const int M = nb * hw;
  const int wgid = xcd_remap(blockIdx.x, gridDim.x);
  const int G = gridDim.x / tiles_n;
  const int tn = wgid % tiles_n, g0 = wgid / tiles_n;
  const int n0 = tn * BN;
  const int tiles_mp = (M + BM - 1) / BM;  // this peer's M tiles
  if (g0 >= tiles_mp) {  // uniform: no tile for this workgroup
    conv_fin_tail(a, peer, reinterpret_cast<int*>(lds));
    return;
  }
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const __amdgpu_buffer_rsrc_t rs_src = conv_rsrc(a.src + peer * a.src_ps), rs_wt = conv_rsrc(a.wt + peer * a.wt_ps + woff);
  const int Ktot = kR * kS * a.src_c;  // 0: a parity class no tap reaches (zeros + the epilogue's residual)
  const int nk = (Ktot + CG_BK - 1) / CG_BK;
  const int cc = (lane & 7) ^ (((wave & 1) << 2) | (lane >> 4));  // this thread's logical 16-byte chunk
  const int cpp = a.src_c >> 3;
  int b_off[NB];  // element offset of this thread's weight rows (K-contiguous), -1: past ncol
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int n = n0 + 8 * (wave + NW * i) + (lane >> 3);
    b_off[i] = n < a.ncol ? n * Ktot : -1;
  }
  // the K walk's start (chunk cc of K step 0)
  int ar0 = 0, as0 = 0, ac80 = cc;
  while (ac80 >= cpp) {
    ac80 -= cpp;
    if (++as0 == kS) { as0 = 0; ++ar0; }
  }
  EpiSums q;
  q.zero();
  // Two-stage rings overlap tiles: once a tile's K loop is done, the next tile's first operand
  // stage is issued into stage 0 and the epilogue stages the accumulators in two 64-row slabs
  // through stage 1, so that DMA (and the next tile's row setup) runs under the epilogue instead of
  // after it (the persistent loop otherwise serialises every tile's pipeline fill; separate
  // workgroups per tile overlapped it across the CU's slots).
  // (The dgrad modes spill or lose occupancy with it: forward only, and off by default — CONV_XT.)
  constexpr bool XT = CONV_XT && MODE == 0 && NS == 2 && BM == 128 && BM / 2 * BN * 4 <= STAGE * 2;
  if constexpr (XT) {
    // A rows 8 (wave + NW i) + (lane >> 3): source coordinate of tap (0, 0) and its element offset
    int a_bh[AR], a_bw[AR], a_pixc[AR];
    bool a_ok[AR];
    int ar = ar0, as_ = as0, ac8 = ac80, kk = cc * 8;  // K walk of this thread's chunk: k = 64 kt + 8 cc = (r, s, c8)
    auto setup = [&](int tm_) {
      const int mb = tm_ * BM;
  #pragma unroll
      for (int i = 0; i < AR; ++i) {
        const int m = mb + 8 * (wave + NW * i) + (lane >> 3);
        a_ok[i] = m < M;
        const int mm = a_ok[i] ? m : 0;
        const int img = mm / hw, rem = mm - img * hw;
        const int oh = rem / gw, ow = rem - oh * gw;
        a_bh[i] = oh * kst - pad_h;
        a_bw[i] = ow * kst - pad_w;
        a_pixc[i] = ((img * a.src_h + a_bh[i]) * a.src_w + a_bw[i]) * a.src_c;
      }
      ar = ar0;
      as_ = as0;
      ac8 = ac80;
      kk = cc * 8;
    };
    auto issue = [&](int buf) {
      bf16* As = lds + buf * STAGE;
      bf16* Bs = As + BM * CG_BK;
      const bool kok = ar < kR;
      const int tapc = (ar * a.src_w + as_) * a.src_c + ac8 * 8;
  #pragma unroll
      for (int i = 0; i < AR; ++i) {
        const bool ok = kok && a_ok[i] && (unsigned)(a_bh[i] + ar) < (unsigned)a.src_h && (unsigned)(a_bw[i] + as_) < (unsigned)a.src_w;
        conv_dma16(rs_src, As + 8 * (wave + NW * i) * CG_BK, ok ? (a_pixc[i] + tapc) * 2 : CONV_OOB);
      }
  #pragma unroll
      for (int i = 0; i < NB; ++i) conv_dma16(rs_wt, Bs + 8 * (wave + NW * i) * CG_BK, (kk < Ktot && b_off[i] >= 0) ? (b_off[i] + kk) * 2 : CONV_OOB);
      ac8 += 8;
      kk += CG_BK;
      while (ac8 >= cpp) {
        ac8 -= cpp;
        if (++as_ == kS) { as_ = 0; ++ar; }
      }
    };
    setup(g0);
  #pragma unroll
    for (int st = 0; st < NS - 1; ++st)
      if (st < nk) issue(st);
    for (int tm = g0; tm < tiles_mp; tm += G) {
      const int m0 = tm * BM;
      f32x4 acc[4][NF];
  #pragma unroll
      for (int i = 0; i < 4; ++i)
  #pragma unroll
        for (int j = 0; j < NF; ++j) acc[i][j] = zero4();

      int rd = 0, wb = NS - 1;  // stage read this K step, stage the next issue writes
      for (int kt = 0; kt < nk; ++kt) {
        // this thread's DMA of stage kt has landed; the stages issued after it stay in flight
        const int ahead = nk - 1 - kt;
        if (NS >= 4 && ahead >= 2) wait_vmcnt<2 * G_>();
        else if (NS >= 3 && ahead >= 1) wait_vmcnt<G_>();
        else wait_vmcnt<0>();
        lds_barrier();  // every wave's DMA of stage kt landed; every wave is done reading stage kt - 1
        if (kt + NS - 1 < nk) issue(wb);
        const bf16* As = lds + rd * STAGE;
        const bf16* Bs = As + BM * CG_BK;
  #pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int ch = h * 4 + (lane >> 4);
          bf16x8 af[4], bfr[NF];
  #pragma unroll
          for (int i = 0; i < 4; ++i) af[i] = ld8(As + swz(wr * 64 + i * 16 + (lane & 15), ch));
  #pragma unroll
          for (int j = 0; j < NF; ++j) bfr[j] = ld8(Bs + swz(wc * (BN / 2) + j * 16 + (lane & 15), ch));
  #pragma unroll
          for (int i = 0; i < 4; ++i)
  #pragma unroll
            for (int j = 0; j < NF; ++j) acc[i][j] = mfma_bf16(af[i], bfr[j], acc[i][j]);
        }
        rd = rd + 1 == NS ? 0 : rd + 1;
        wb = wb + 1 == NS ? 0 : wb + 1;
      }
      __syncthreads();  // operand stages idle
      const bool more = tm + G < tiles_mp;
      if (more) {
        setup(tm + G);
        if (nk > 0) issue(0);  // the next tile's first stage lands under this epilogue
      }
      conv_epilogue_tile<EMODE, BM, BN, NT, 2, SPEC>(a, acc, reinterpret_cast<float*>(lds + STAGE), peer, m0, n0, M, hw, gw, ph, pw, q);
    }
  } else {
    for (int tm = g0; tm < tiles_mp; tm += G) {
      const int m0 = tm * BM;
      // A rows 8 (wave + NW i) + (lane >> 3): source coordinate of tap (0, 0) and its element offset
      int a_bh[AR], a_bw[AR], a_pixc[AR];
      bool a_ok[AR];
  #pragma unroll
      for (int i = 0; i < AR; ++i) {
        const int m = m0 + 8 * (wave + NW * i) + (lane >> 3);
        a_ok[i] = m < M;
        const int mm = a_ok[i] ? m : 0;
        const int img = mm / hw, rem = mm - img * hw;
        const int oh = rem / gw, ow = rem - oh * gw;
        a_bh[i] = oh * kst - pad_h;
        a_bw[i] = ow * kst - pad_w;
        a_pixc[i] = ((img * a.src_h + a_bh[i]) * a.src_w + a_bw[i]) * a.src_c;
      }
      // K walk of this thread's chunk: K step kt covers k = 64 kt + 8 cc = (tap r, tap s, channel chunk c8)
      int ar = ar0, as_ = as0, ac8 = ac80, kk = cc * 8;
      auto issue = [&](int buf) {
        bf16* As = lds + buf * STAGE;
        bf16* Bs = As + BM * CG_BK;
        const bool kok = ar < kR;
        const int tapc = (ar * a.src_w + as_) * a.src_c + ac8 * 8;
  #pragma unroll
        for (int i = 0; i < AR; ++i) {
          const bool ok = kok && a_ok[i] && (unsigned)(a_bh[i] + ar) < (unsigned)a.src_h && (unsigned)(a_bw[i] + as_) < (unsigned)a.src_w;
          conv_dma16(rs_src, As + 8 * (wave + NW * i) * CG_BK, ok ? (a_pixc[i] + tapc) * 2 : CONV_OOB);
        }
  #pragma unroll
        for (int i = 0; i < NB; ++i) conv_dma16(rs_wt, Bs + 8 * (wave + NW * i) * CG_BK, (kk < Ktot && b_off[i] >= 0) ? (b_off[i] + kk) * 2 : CONV_OOB);
        ac8 += 8;
        kk += CG_BK;
        while (ac8 >= cpp) {
          ac8 -= cpp;
          if (++as_ == kS) { as_ = 0; ++ar; }
        }
      };
      f32x4 acc[4][NF];
  #pragma unroll
      for (int i = 0; i < 4; ++i)
  #pragma unroll
        for (int j = 0; j < NF; ++j) acc[i][j] = zero4();

  #pragma unroll
      for (int st = 0; st < NS - 1; ++st)
        if (st < nk) issue(st);
      int rd = 0, wb = NS - 1;  // stage read this K step, stage the next issue writes
      for (int kt = 0; kt < nk; ++kt) {
        // this thread's DMA of stage kt has landed; the stages issued after it stay in flight
        const int ahead = nk - 1 - kt;
        if (NS >= 4 && ahead >= 2) wait_vmcnt<2 * G_>();
        else if (NS >= 3 && ahead >= 1) wait_vmcnt<G_>();
        else wait_vmcnt<0>();
        lds_barrier();  // every wave's DMA of stage kt landed; every wave is done reading stage kt - 1
        if (kt + NS - 1 < nk) issue(wb);
        const bf16* As = lds + rd * STAGE;
        const bf16* Bs = As + BM * CG_BK;
  #pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int ch = h * 4 + (lane >> 4);
          bf16x8 af[4], bfr[NF];
  #pragma unroll
          for (int i = 0; i < 4; ++i) af[i] = ld8(As + swz(wr * 64 + i * 16 + (lane & 15), ch));
  #pragma unroll
          for (int j = 0; j < NF; ++j) bfr[j] = ld8(Bs + swz(wc * (BN / 2) + j * 16 + (lane & 15), ch));
  #pragma unroll
          for (int i = 0; i < 4; ++i)
  #pragma unroll
            for (int j = 0; j < NF; ++j) acc[i][j] = mfma_bf16(af[i], bfr[j], acc[i][j]);
        }
        rd = rd + 1 == NS ? 0 : rd + 1;
        wb = wb + 1 == NS ? 0 : wb + 1;
      }
      __syncthreads();  // operand stages idle: the epilogue stages the tile over them
      conv_epilogue_tile<EMODE, BM, BN, NT, 1, SPEC>(a, acc, reinterpret_cast<float*>(lds), peer, m0, n0, M, hw, gw, ph, pw, q);
      __syncthreads();  // staging tile read: the next tile's DMA may overwrite it
    }
  }
  conv_epilogue_sums<EMODE, BN, NT, SPEC>(a, lds, peer, n0, MODE == 5 ? g0 * 4 + (int)blockIdx.y : g0, q);
  conv_fin_tail(a, peer, reinterpret_cast<int*>(lds));
}


// ------------------------------------------------------------------------------------------------
// k_conv_fwd_halo<MODE>: forward-shaped 3x3 / stride-1 / pad-1 conv with 64 input and 64 output
// channels on 32-wide images (ResNet-18 layer 1: forward, MODE 0, and the stride-1 dgrad as a
// forward conv, MODE 4), with the im2col operand read out of ONE staged patch per tile.
//   A 256-pixel M tile is 8 image rows; its nine taps are shifted windows of the 10 x 34 x 64 patch
//   around them (43.5 KB, zero padding outside the image) — the LDS-DMA kernel fetches 9 x 32 KB of
//   im2col rows per tile instead. A fragments are plain 16-byte LDS reads at per-lane patch rows.
//   The 64 x 576 weights stay in LDS for the whole (persistent) workgroup: nine [64 co][64 k]
//   tap blocks. 8 waves as 4 x 2 (64 rows x 32 columns each), the shared epilogue
//   (conv_epilogue_tile / conv_epilogue_sums) with column sums carried across the workgroup's tiles.
//   The forward prefetches the next tile's patch into registers while the current one is multiplied.
// ------------------------------------------------------------------------------------------------
// MODE 4 (and MODE 0 without the BN prologue when HALO_DMA0 is set) stage the patch by LDS DMA
// (buffer_load ... lds) into two patch buffers: the next tile's patch lands under this tile's MFMAs
// and epilogue without a register round trip. MODE 4's BN-backward epilogue left no registers for
// the register prefetch, so it used to load each patch after the previous epilogue, exposed
// (237 us per layer-1 dgrad vs 110 us for the same-shape forward, profiles/r4i_resnet_window).
// Two 344-row patch buffers + the weights fill 158 KB of the 160 KB; the epilogue stages in two
// 128-row slabs over the patch just read.
#ifndef HALO_DMA0
#define HALO_DMA0 0
#endif
#ifndef HALO_DMA4
#define HALO_DMA4 1
#endif
// EPI_PF_HALO=1: the halo dgrads load their epilogue operands before the tile's MFMAs instead of at
// the start of the epilogue. The kernels get faster (177 / 174 -> 168 / 163 us) but ResNet-18 does
// not (2.594 / 2.585 vs 2.607 / 2.608 rounds/s, same box, profiles/r4x_halo_prefetch): off
#ifndef EPI_PF_HALO
#define EPI_PF_HALO 0
#endif
#ifndef HALO_SPEC  // the layer-1 dgrads with compile-time epilogue operand sets (conv_epilogue_tile SPEC)
#define HALO_SPEC 1
#endif
template <int MODE, bool PRO, int SPEC = -1>
__global__ __launch_bounds__(512, 1) void k_conv_fwd_halo(ConvGemmArgs a, int tiles_m) {
  static_assert(MODE == 0 || MODE == 4, "forward-shaped convs");
  static_assert(!PRO || MODE == 0, "BN prologue on the forward only");
  constexpr int W = 32, C = 64, BM = 256, BN = 64, NT = 512;
  constexpr int TR = BM / W, PW = W + 2, PROWS = (TR + 2) * PW;  // tile rows, patch width / rows
  constexpr int PCH = PROWS * 8, PPT = (PCH + NT - 1) / NT;       // 16-byte patch chunks (per thread)
  constexpr int WE = 9 * C * BN;                                  // weight elements (bf16)
  constexpr int PE = PROWS * C;
  constexpr int EPI = BM * BN * 2;                                // fp32 staging, in bf16 units
  constexpr bool DMA = (MODE == 4 && HALO_DMA4) || (MODE == 0 && HALO_DMA0 && !PRO);
  constexpr int PROWS8 = (PROWS + 7) / 8 * 8;  // DMA writes whole 8-row blocks (the tail gets zeros)
  constexpr int PEP = PROWS8 * C;
  static_assert(!DMA || (PEP >= BM / 2 * BN * 2 && PEP >= 8 * 3 * BN * 2), "a patch buffer holds a staging slab / the sums");
  static_assert(!DMA || (WE + 2 * PEP) * 2 <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) bf16 lds[DMA ? WE + 2 * PEP : WE + (PE > EPI ? PE : EPI)];
  bf16* wl = lds;       // [tap][64 n][64 k] (swz rows)
  bf16* pat = lds + WE;  // [patch row][64 ci] (swz rows); the epilogue stages over it
  const int peer = blockIdx.z;
  const int nb = a.nbatch ? a.nbatch[peer] : a.max_batch;
  const int HW = a.src_h * W;
  const int M = nb * HW;
  const int tiles_mp = (M + BM - 1) / BM;
  const int G = gridDim.x;
  const int g0 = xcd_remap(blockIdx.x, G);
  if (g0 >= tiles_mp) {
    conv_fin_tail(a, peer, reinterpret_cast<int*>(lds));
    return;
  }
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const __amdgpu_buffer_rsrc_t rs_src = conv_rsrc(a.src + peer * a.src_ps), rs_wt = conv_rsrc(a.wt + peer * a.wt_ps);
  // weights once: 9 taps x 64 rows x 8 chunks = 4608 chunks, 9 per thread
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int e = tid + NT * i;
    const int t = e >> 9, n = (e >> 3) & 63, ch = e & 7;
    const uint4 v = conv_ld16(rs_wt, n < a.ncol ? (n * 9 * C + t * C + ch * 8) * 2 : CONV_OOB);
    *reinterpret_cast<uint4*>(wl + t * C * BN + swz(n, ch)) = v;
  }
  uint4 rp[PPT];
  // PRO: src is a BatchNorm input y and the operand is relu(y*sc + sh) (bn_relu8, bit-identical to
  // k_bn_act), applied once per staged pixel as the patch goes to LDS — the patch holds each pixel
  // once for all nine taps, so the fold costs one transform per element, not nine (the register
  // stage's prologue fold, MYFYP_CNN_FUSE_BN, repeats it per tap). This thread's chunks are always
  // channels 8 (tid & 7) .. +7 (NT is a multiple of 8): 16 scale / shift registers. Padding taps
  // stay 0 (not relu(sh)): `pok` marks the chunks that are real pixels.
  float psc[8], psh[8];
  unsigned pok = 0;
  if (PRO) {
    const float* pro = a.pro_ss + peer * a.pro_ss_ps;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      psc[j] = pro[(tid & 7) * 8 + j];
      psh[j] = pro[a.src_c + (tid & 7) * 8 + j];
    }
  }
  auto load_patch = [&](int tm) {
    const int m0 = tm * BM;
    const int img = m0 / HW, h0 = (m0 - img * HW) / W;
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int e = tid + NT * i;
      const int kp = e >> 3, ch = e & 7;
      const int pr = kp / PW, pc = kp - pr * PW;
      const int h = h0 - 1 + pr, w = pc - 1;
      const bool ok = e < PCH && (unsigned)h < (unsigned)a.src_h && (unsigned)w < (unsigned)W && img < nb;
      rp[i] = conv_ld16(rs_src, ok ? (((img * a.src_h + h) * W + w) * C + ch * 8) * 2 : CONV_OOB);
      if (PRO) pok = ok ? (pok | (1u << i)) : (pok & ~(1u << i));
    }
  };
  auto store_patch = [&]() {
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int e = tid + NT * i;
      uint4 v = rp[i];
      if (PRO && ((pok >> i) & 1u)) v = bn_relu8(v, psc, psh);
      if (e < PCH) *reinterpret_cast<uint4*>(pat + swzp(e >> 3, e & 7)) = v;
    }
  };
  // patch row of tap (0, 0) for this lane's A rows (row = wr * 64 + i * 16 + (lane & 15) of the tile)
  int prow0[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int p = wr * 64 + i * 16 + (lane & 15);
    prow0[i] = (p / W) * PW + (p % W);
  }
  EpiSums q;
  q.zero();
  if constexpr (DMA) {
    const int wv = __builtin_amdgcn_readfirstlane(wave);
    // physical 8-row block blk of the patch: lane L writes row 8 blk + L / 8, physical chunk L % 8,
    // i.e. logical chunk (L % 8) ^ (row & 6) of swzp's layout; rows past the patch, padding
    // pixels and rows of a missing image read the zero page (CONV_OOB)
    auto dma_patch = [&](int tm, bf16* dst) {
      const int m0 = tm * BM;
      const int img = m0 / HW, h0 = (m0 - img * HW) / W;
#pragma unroll
      for (int i = 0; i < (PROWS8 / 8 + 7) / 8; ++i) {
        const int blk = wv + 8 * i;
        if (blk * 8 >= PROWS) break;
        const int R = blk * 8 + (lane >> 3);
        const int chl = (lane & 7) ^ (HALO_SWZP ? (R & 6) : ((R >> 1) & 7));
        const int pr = R / PW, pc = R - pr * PW;
        const int h = h0 - 1 + pr, w = pc - 1;
        const bool ok = R < PROWS && (unsigned)h < (unsigned)a.src_h && (unsigned)w < (unsigned)W && img < nb;
        conv_dma16(rs_src, dst + blk * 8 * C, ok ? (((img * a.src_h + h) * W + w) * C + chl * 8) * 2 : CONV_OOB);
      }
    };
    int cur = 0;
    dma_patch(g0, pat);
    for (int tm = g0; tm < tiles_mp; tm += G) {
      bf16* pc = pat + cur * PEP;
      wait_vmcnt<0>();
      __syncthreads();  // every wave's patch DMA landed (and the weights, the first time); the other buffer is free
      // the dgrad epilogue's operand chunks of this tile, in flight under its MFMAs (issued before the
      // next patch's DMA, so the epilogue's wait for them does not wait for that DMA)
      EpiPre<epi_np<BM, BN, NT, 2>()> epre;
      constexpr bool HPF = EPI_PF_HALO && EPI_PF && SPEC >= 0 && (SPEC & 3) != 0;
      if (HPF) conv_epilogue_prefetch<MODE, BM, BN, NT, 2, HPF ? SPEC : 0>(a, peer, tm * BM, 0, M, HW, W, 0, 0, epre);
      if (tm + G < tiles_mp) dma_patch(tm + G, pat + (cur ^ 1) * PEP);  // lands under this tile's MFMAs + epilogue
      f32x4 acc[4][2];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = zero4();
      // the 72 A / 36 B LDS addresses of the nine taps are recomputed per tile (laundered rows):
      // hoisted out of the tile loop they held ~100 VGPRs and spilled
      int pr0[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        pr0[i] = prow0[i];
        asm volatile("" : "+v"(pr0[i]));
      }
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int toff = (t / 3) * PW + (t % 3);
        const bf16* wt_t = wl + t * C * BN;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int ch = h * 4 + (lane >> 4);
          bf16x8 af[4], bfr[2];
#pragma unroll
          for (int i = 0; i < 4; ++i) af[i] = ld8(pc + swzp(pr0[i] + toff, ch));
#pragma unroll
          for (int j = 0; j < 2; ++j) bfr[j] = ld8(wt_t + swz(wc * 32 + j * 16 + (lane & 15), ch));
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = mfma_bf16(af[i], bfr[j], acc[i][j]);
        }
      }
      __syncthreads();  // patch reads done: the epilogue stages over it, two 128-row slabs
      conv_epilogue_tile<MODE, BM, BN, NT, 2, SPEC>(a, acc, reinterpret_cast<float*>(pc), peer, tm * BM, 0, M, HW, W, 0, 0, q, HPF ? &epre : nullptr);
      cur ^= 1;
    }
    conv_epilogue_sums<MODE, BN, NT, SPEC>(a, pat, peer, 0, g0, q);
    conv_fin_tail(a, peer, reinterpret_cast<int*>(lds));
    return;
  }
  // MODE 0 prefetches the next tile's patch into registers under the MFMAs
  constexpr bool PREF = MODE == 0;
  if (PREF) load_patch(g0);
  for (int tm = g0; tm < tiles_mp; tm += G) {
    if (!PREF) load_patch(tm);
    store_patch();
    __syncthreads();  // patch (and, the first time, the weights) staged
    if (PREF && tm + G < tiles_mp) load_patch(tm + G);  // next tile's patch in flight under the MFMAs
    f32x4 acc[4][2];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = zero4();
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int toff = (t / 3) * PW + (t % 3);
      const bf16* wt_t = wl + t * C * BN;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int ch = h * 4 + (lane >> 4);
        bf16x8 af[4], bfr[2];
#pragma unroll
        for (int i = 0; i < 4; ++i) af[i] = ld8(pat + swzp(prow0[i] + toff, ch));
#pragma unroll
        for (int j = 0; j < 2; ++j) bfr[j] = ld8(wt_t + swz(wc * 32 + j * 16 + (lane & 15), ch));
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = mfma_bf16(af[i], bfr[j], acc[i][j]);
      }
    }
    __syncthreads();  // patch reads done: the epilogue stages over it
    conv_epilogue_tile<MODE, BM, BN, NT, 1, SPEC>(a, acc, reinterpret_cast<float*>(pat), peer, tm * BM, 0, M, HW, W, 0, 0, q);
    __syncthreads();  // staging read: the next patch may be stored
  }
  conv_epilogue_sums<MODE, BN, NT, SPEC>(a, pat, peer, 0, g0, q);
  conv_fin_tail(a, peer, reinterpret_cast<int*>(lds));
}

// ------------------------------------------------------------------------------------------------
// weight gradient
// ------------------------------------------------------------------------------------------------
// Wf-layout gradient [dy_c][ncol_tot] of one wgrad tile: lanes 0..15 of a row group write 16
// consecutive floats (fp32 atomics when the pixel dimension is split)
template <int BM, int BN>
__device__ __forceinline__ void wgrad_store(const WgradArgs& a, const f32x4 (&acc)[BM / 32][BN / 32], int peer, int co0, int n0, int ncol_tot) {
  constexpr int FM = BM / 32, FN = BN / 32;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  float* grad = a.grad + peer * a.grad_ps;
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = n0 + wc * (BN / 2) + j * 16 + (lane & 15);
    if (n >= ncol_tot) continue;
#pragma unroll
    for (int i = 0; i < FM; ++i) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int co = co0 + wr * (BM / 2) + i * 16 + 4 * (lane >> 4) + e;
        if (co < a.dy_c) {
          float* dst = grad + (int64_t)co * ncol_tot + n;
          if (a.accumulate) atomicAdd(dst, acc[i][j][e]);
          else *dst = acc[i][j][e];
        }
      }
    }
  }
}

template <int BM, int BN, bool PRO>
__global__ __launch_bounds__(256) void k_conv_wgrad(WgradArgs a, int tiles_m, int tiles_n, int splits) {
  constexpr int FM = BM / 32, FN = BN / 32;       // fragments per wave
  constexpr int CA = BM / 8, CB = BN / 8;         // 16-byte chunks per staged row
  constexpr int NA = 64 * CA / 256, NBr = 64 * CB / 256;
  __shared__ __attribute__((aligned(16))) bf16 lds[2 * 64 * (BM + BN)];

  const int peer = blockIdx.z;
  const int nb = a.nbatch ? a.nbatch[peer] : a.max_batch;
  const int M = nb * a.Ho * a.Wo;
  // grid.x = splits x tiles: consecutive remapped ids (one XCD) share a split, i.e. the same dY / X
  // rows, so the tiles of one pixel range hit one L2 (the split index in grid.y spread them over all
  // eight: 2.5 % L2 hits measured on the 64-channel layers)
  const int ntile = tiles_m * tiles_n;
  const int wgid = xcd_remap(blockIdx.x, ntile * splits);
  const int split = wgid / ntile, tile = wgid - split * ntile;
  const int kbeg = split * a.k_per_split;
  const int kend = min(M, kbeg + a.k_per_split);
  if (kbeg >= kend) return;
  const int tn = tile % tiles_n, tm = tile / tiles_n;
  const int co0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const bf16* dy = a.dy + peer * a.dy_ps;
  const bf16* x = a.x + peer * a.x_ps;
  const __amdgpu_buffer_rsrc_t rs_dy = conv_rsrc(dy), rs_x = conv_rsrc(x);
  (void)rs_dy;
  (void)rs_x;
  const int hwo = a.Ho * a.Wo;
  const int ncol_tot = a.R * a.S * a.x_c;

  // B chunk of this thread: fixed (r, s, ci) for the whole loop
  const int ccb = tid % CB;
  const int nb0 = n0 + ccb * 8;
  const bool bcol_ok = nb0 < ncol_tot;
  int br = 0, bs = 0, bci = 0;
  if (bcol_ok) {
    const int rs = nb0 / a.x_c;
    bci = nb0 - rs * a.x_c;
    br = rs / a.S;
    bs = rs - br * a.S;
  }
  const int cca = tid % CA;
  const bool acol_ok = co0 + cca * 8 < a.dy_c;
  // PRO: x is a BN output y and the B operand is relu(y*sc + sh); constants of this thread's fixed
  // channel chunk (bci .. bci + 7), applied at the LDS store (the loads stay in flight across the MFMAs)
  float psc[8], psh[8];
  unsigned bok = 0;
  if (PRO) {
    const float* pro = a.pro_ss + peer * a.pro_ss_ps;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      psc[j] = bcol_ok ? pro[bci + j] : 1.f;
      psh[j] = bcol_ok ? pro[a.x_c + bci + j] : 0.f;
    }
  }

  // per-row output coordinates (img, oh, ow) of this thread's B rows, advanced by +64 pixels per
  // K-step with carries (no per-step division)
  int b_img[NBr], b_oh[NBr], b_ow[NBr];
#pragma unroll
  for (int i = 0; i < NBr; ++i) {
    const int m = kbeg + tid / CB + (256 / CB) * i;
    b_img[i] = m / hwo;
    const int rem = m - b_img[i] * hwo;
    b_oh[i] = rem / a.Wo;
    b_ow[i] = rem - b_oh[i] * a.Wo;
  }
  const int d_img = 64 / hwo, d_rem = 64 - d_img * hwo, d_oh = d_rem / a.Wo, d_ow = d_rem - d_oh * a.Wo;
  const int hb = br - a.pad, wb = bs - a.pad;
  uint4 ra[NA], rb[NBr];
  auto load = [&](int m_base) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int m = m_base + tid / CA + (256 / CA) * i;
      if (CONV_BUFLOAD)
        ra[i] = conv_ld16(rs_dy, (acol_ok && m < kend) ? (m * a.dy_c + co0 + cca * 8) * 2 : CONV_OOB);
      else
        ra[i] = (acol_ok && m < kend) ? *reinterpret_cast<const uint4*>(dy + (int64_t)m * a.dy_c + co0 + cca * 8) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < NBr; ++i) {
      const int m = m_base + tid / CB + (256 / CB) * i;
      const int h = b_oh[i] * a.stride + hb, w = b_ow[i] * a.stride + wb;
      const bool ok = bcol_ok && m < kend && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
      if (CONV_BUFLOAD)
        rb[i] = conv_ld16(rs_x, ok ? (((b_img[i] * a.H + h) * a.W + w) * a.x_c + bci) * 2 : CONV_OOB);
      else
        rb[i] = ok ? *reinterpret_cast<const uint4*>(x + ((b_img[i] * a.H + h) * a.W + w) * a.x_c + bci) : make_uint4(0, 0, 0, 0);
      if (PRO) bok = ok ? (bok | (1u << i)) : (bok & ~(1u << i));
      b_ow[i] += d_ow;
      if (b_ow[i] >= a.Wo) { b_ow[i] -= a.Wo; ++b_oh[i]; }
      b_oh[i] += d_oh;
      if (b_oh[i] >= a.Ho) { b_oh[i] -= a.Ho; ++b_img[i]; }
      b_img[i] += d_img;
    }
  };
  auto store = [&](int buf) {
    bf16* As = lds + buf * 64 * (BM + BN);
    bf16* Bs = As + 64 * BM;
#pragma unroll
    for (int i = 0; i < NA; ++i) *reinterpret_cast<uint4*>(As + tr_off<BM>(tid / CA + (256 / CA) * i, cca * 8)) = ra[i];
#pragma unroll
    for (int i = 0; i < NBr; ++i) {
      uint4 v = rb[i];
      if (PRO && ((bok >> i) & 1u)) v = bn_relu8(v, psc, psh);
      *reinterpret_cast<uint4*>(Bs + tr_off<BN>(tid / CB + (256 / CB) * i, ccb * 8)) = v;
    }
  };
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = zero4();

  const int nk = (kend - kbeg + 63) / 64;
  load(kbeg);
  store(0);
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) load(kbeg + (kt + 1) * 64);
    const bf16* As = lds + cur * 64 * (BM + BN);
    const bf16* Bs = As + 64 * BM;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = frag_tr<BM>(As, wr * (BM / 2) + i * 16, h * 32, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = frag_tr<BN>(Bs, wc * (BN / 2) + j * 16, h * 32, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma_bf16(af[i], bfr[j], acc[i][j]);
    }
    if (kt + 1 < nk) store(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  wgrad_store<BM, BN>(a, acc, peer, co0, n0, ncol_tot);
}

// k_conv_wgrad_dma<BM, BN, NS, MINB>: k_conv_wgrad with its operands staged by LDS-DMA into an
// NS-stage ring (no register stage, counted vmcnt + raw barriers; see k_conv_fwd_dma). A thread
// keeps the rows of the register-staged kernel (a wave instruction fills 64 / CW consecutive rows of
// the [64][W] image, W / 8 = CW chunks per row); the transposed-read layout tr_off<W> permutes 16-byte
// chunks by trf<W>(row) / 2, which is the same for all of a thread's rows, so the thread loads the
// fixed logical chunk (lane % CW) ^ (trf(row) / 2) — one (r, s, ci) column per thread as before.
// No BN prologue (PRO launches take k_conv_wgrad).
template <int BM, int BN, int NS, int MINB>
__global__ __launch_bounds__(256, MINB) void k_conv_wgrad_dma(WgradArgs a, int tiles_m, int tiles_n, int splits) {
  constexpr int FM = BM / 32, FN = BN / 32;
  constexpr int CA = BM / 8, CB = BN / 8;
  constexpr int NA = 64 * CA / 256, NBr = 64 * CB / 256;
  constexpr int G = NA + NBr;  // LDS-DMA instructions per thread per stage
  constexpr int STAGE = 64 * (BM + BN);
  static_assert(NS >= 2 && NS <= 3, "stage ring depth");
  __shared__ __attribute__((aligned(16))) bf16 lds[NS * STAGE];  // the only LDS object (see k_conv_fwd_dma)

  const int peer = blockIdx.z;
  const int nb = a.nbatch ? a.nbatch[peer] : a.max_batch;
  const int M = nb * a.Ho * a.Wo;
  const int ntile = tiles_m * tiles_n;
  const int wgid = xcd_remap(blockIdx.x, ntile * splits);
  const int split = wgid / ntile, tile = wgid - split * ntile;
  const int kbeg = split * a.k_per_split;
  const int kend = min(M, kbeg + a.k_per_split);
  if (kbeg >= kend) return;
  const int tn = tile % tiles_n, tm = tile / tiles_n;
  const int co0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave >> 1, wc = wave & 1;
  const __amdgpu_buffer_rsrc_t rs_dy = conv_rsrc(a.dy + peer * a.dy_ps), rs_x = conv_rsrc(a.x + peer * a.x_ps);
  const int hwo = a.Ho * a.Wo;
  const int ncol_tot = a.R * a.S * a.x_c;

  // logical chunks of this thread (source-side swizzle), fixed for the whole loop
  const int cca = (lane % CA) ^ (trf<BM>(tid / CA) >> 1);
  const int ccb = (lane % CB) ^ (trf<BN>(tid / CB) >> 1);
  const int nb0 = n0 + ccb * 8;
  const bool bcol_ok = nb0 < ncol_tot;
  int br = 0, bs = 0, bci = 0;
  if (bcol_ok) {
    const int rs = nb0 / a.x_c;
    bci = nb0 - rs * a.x_c;
    br = rs / a.S;
    bs = rs - br * a.S;
  }
  const bool acol_ok = co0 + cca * 8 < a.dy_c;
  int b_img[NBr], b_oh[NBr], b_ow[NBr];
#pragma unroll
  for (int i = 0; i < NBr; ++i) {
    const int m = kbeg + tid / CB + (256 / CB) * i;
    b_img[i] = m / hwo;
    const int rem = m - b_img[i] * hwo;
    b_oh[i] = rem / a.Wo;
    b_ow[i] = rem - b_oh[i] * a.Wo;
  }
  const int d_img = 64 / hwo, d_rem = 64 - d_img * hwo, d_oh = d_rem / a.Wo, d_ow = d_rem - d_oh * a.Wo;
  const int hb = br - a.pad, wb0 = bs - a.pad;
  int m_next = kbeg;  // first pixel of the next K step to issue
  auto issue = [&](int buf) {
    bf16* As = lds + buf * STAGE;
    bf16* Bs = As + 64 * BM;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int m = m_next + tid / CA + (256 / CA) * i;
      conv_dma16(rs_dy, As + ((64 / CA) * wave + (256 / CA) * i) * BM, (acol_ok && m < kend) ? (m * a.dy_c + co0 + cca * 8) * 2 : CONV_OOB);
    }
#pragma unroll
    for (int i = 0; i < NBr; ++i) {
      const int m = m_next + tid / CB + (256 / CB) * i;
      const int h = b_oh[i] * a.stride + hb, w = b_ow[i] * a.stride + wb0;
      const bool ok = bcol_ok && m < kend && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)a.W;
      conv_dma16(rs_x, Bs + ((64 / CB) * wave + (256 / CB) * i) * BN, ok ? (((b_img[i] * a.H + h) * a.W + w) * a.x_c + bci) * 2 : CONV_OOB);
      b_ow[i] += d_ow;
      if (b_ow[i] >= a.Wo) { b_ow[i] -= a.Wo; ++b_oh[i]; }
      b_oh[i] += d_oh;
      if (b_oh[i] >= a.Ho) { b_oh[i] -= a.Ho; ++b_img[i]; }
      b_img[i] += d_img;
    }
    m_next += 64;
  };
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = zero4();

  const int nk = (kend - kbeg + 63) / 64;
#pragma unroll
  for (int st = 0; st < NS - 1; ++st)
    if (st < nk) issue(st);
  int rd = 0, wbuf = NS - 1;
  for (int kt = 0; kt < nk; ++kt) {
    const int ahead = nk - 1 - kt;
    if (NS >= 3 && ahead >= 1) wait_vmcnt<G>();
    else wait_vmcnt<0>();
    lds_barrier();  // every wave's DMA of stage kt landed; every wave is done reading stage kt - 1
    if (kt + NS - 1 < nk) issue(wbuf);
    const bf16* As = lds + rd * STAGE;
    const bf16* Bs = As + 64 * BM;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = frag_tr<BM>(As, wr * (BM / 2) + i * 16, h * 32, lane);
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = frag_tr<BN>(Bs, wc * (BN / 2) + j * 16, h * 32, lane);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma_bf16(af[i], bfr[j], acc[i][j]);
    }
    rd = rd + 1 == NS ? 0 : rd + 1;
    wbuf = wbuf + 1 == NS ? 0 : wbuf + 1;
  }
  wgrad_store<BM, BN>(a, acc, peer, co0, n0, ncol_tot);
}


// ------------------------------------------------------------------------------------------------
// k_conv_wgrad_halo<W>: weight gradient of a 3x3 / stride-1 / pad-1 conv (channel counts multiples
// of 64; ResNet-18 layers 1-3), from ONE staged X patch per K step instead of nine gathers. A
// workgroup owns a 64-output x 64-input channel block (all nine taps: 64 x 576 gradient columns).
//   A K step is 64 pixels = 64 / W complete image rows (H * W % 64 == 0). Its nine im2col taps are
//   shifted windows of the (64 / W + 2) x (W + 2) x 64 patch around those rows (zero padding
//   outside the image), so the patch is staged once (17 KB at W = 32) where the generic wgrad
//   gathers 9 x 8 KB. Each B fragment reads its tap's window through the transposed LDS read with
//   per-lane patch rows: the 8 pixels of a lane group are consecutive within one image row, so
//   they are 8 consecutive patch rows.
//   One workgroup computes the whole 64 x 576 gradient of its pixel range: 8 waves as 2 (co halves)
//   x 4 (column quarters of 144 = 9 fragments), fp32 accumulators, split-K over pixel ranges with
//   fp32 atomics (as k_conv_wgrad). Register-staged, double-buffered.
// ------------------------------------------------------------------------------------------------
// transposed MFMA B fragment whose 8 k rows of lane group g are patch rows rlo + 0..3 and rhi + 0..3
// (per lane: the two 4-pixel halves of the group, each within one image row)
__device__ __forceinline__ bf16x8 frag_tr_rows(const bf16* base, int col0, int rlo, int rhi, int lane) {
  const int q = (lane & 15) >> 2, p = lane & 3;
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + tr_off<64>(rlo + q, col0 + 4 * p)));
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + tr_off<64>(rhi + q, col0 + 4 * p)));
  const s16x8 both = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
  return __builtin_bit_cast(bf16x8, both);
}

// W: image width; HI: image height when a K step spans several whole images (H * W < 64: one
// padded patch per image, NI images per step), 0 when it is 64 / W rows of one image
// PF: global loads in flight ahead of the K step being computed. PF = 1: the next K step's loads are
// issued at the start of this one (one register stage). PF = 2: two register stages alternate, the
// loads two K steps ahead — a K step's 36 MFMAs per wave (~1150 cycles per SIMD) are shorter than a
// loaded HBM round trip, so at PF = 1 every K step waited for its own operands
// (scripts/probes/wgrad_atomic_share.py, profiles/r6d_wgrad).
template <int W, int HI, bool PRO, int PF = 1>
__global__ __launch_bounds__(512, 1) void k_conv_wgrad_halo(WgradArgs a, int splits, int tiles_co, int tiles_ci) {
  constexpr int C = 64;
  constexpr int NI = HI ? 64 / (HI * W) : 1;    // images per K step
  constexpr int RR = HI ? HI : 64 / W;          // image rows per K step and image
  constexpr int PW = W + 2, PIMG = (RR + 2) * PW, PROWS = NI * PIMG;
  constexpr int DYE = 64 * C, PE = PROWS * C, STG = DYE + PE;  // bf16 elements per stage
  constexpr int PCH = PROWS * 8;                                // 16-byte patch chunks per K step
  constexpr int PPT = (PCH + 511) / 512;                        // patch chunks per thread
  static_assert(W >= 4 && W <= 64 && (HI ? 64 % (HI * W) == 0 : 64 % W == 0), "image shape");
  // (C: the 64-channel blocks of dY and X this workgroup stages)
  __shared__ __attribute__((aligned(16))) bf16 lds[2 * STG];

  const int peer = blockIdx.z;
  const int nb = a.nbatch ? a.nbatch[peer] : a.max_batch;
  const int HW = a.H * W;
  const int M = nb * HW;
  // consecutive remapped ids (one XCD) share a split, i.e. the same pixels (dY rows and X patch)
  const int ntile = tiles_co * tiles_ci;
  const int wgid = xcd_remap(blockIdx.x, ntile * splits);
  const int split = wgid / ntile, tile = wgid - split * ntile;
  const int co0 = (tile / tiles_ci) * 64, ci0 = (tile % tiles_ci) * 64;
  const int ncol = 9 * a.x_c;
  const int kbeg = split * a.k_per_split;
  const int kend = min(M, kbeg + a.k_per_split);
  if (kbeg >= kend) return;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wco = wave & 1, wn = wave >> 1;
  const __amdgpu_buffer_rsrc_t rs_dy = conv_rsrc(a.dy + peer * a.dy_ps), rs_x = conv_rsrc(a.x + peer * a.x_ps);

  struct Stage {  // one K step's operand chunks of this thread, in registers
    uint4 dy, p[PPT];
    unsigned pok;
  };
  Stage st0, st1;
  // PRO: x is a BatchNorm input y and the B operand is relu(y*sc + sh), applied once per staged X
  // pixel (as k_conv_fwd_halo); this thread's chunks are channels ci0 + 8 (tid & 7) .. +7
  float psc[8], psh[8];
  if (PRO) {
    const float* pro = a.pro_ss + peer * a.pro_ss_ps;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      psc[j] = pro[ci0 + (tid & 7) * 8 + j];
      psh[j] = pro[a.x_c + ci0 + (tid & 7) * 8 + j];
    }
  }
  auto load = [&](Stage& S, int m0) {  // K step starting at pixel m0 (a multiple of 64: whole image rows / images)
    {
      const int row = tid >> 3, ch = tid & 7;
      S.dy = conv_ld16(rs_dy, m0 + row < kend ? ((m0 + row) * a.dy_c + co0 + ch * 8) * 2 : CONV_OOB);
    }
    S.pok = 0;
    const int img0 = m0 / HW, h0 = HI ? 0 : (m0 - img0 * HW) / W;
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int e = tid + 512 * i;
      const int kp = e >> 3, ch = e & 7;
      const int il = kp / PIMG, rem = kp - il * PIMG;
      const int pr = rem / PW, pc = rem - pr * PW;
      const int h = h0 - 1 + pr, w = pc - 1, img = img0 + il;
      // images past the peer's batch (the last step of a multi-image K loop) load zeros
      const bool ok = e < PCH && (unsigned)h < (unsigned)a.H && (unsigned)w < (unsigned)W && img < nb;
      S.p[i] = conv_ld16(rs_x, ok ? (((img * a.H + h) * W + w) * a.x_c + ci0 + ch * 8) * 2 : CONV_OOB);
      if (PRO && ok) S.pok |= 1u << i;
    }
  };
  auto store = [&](const Stage& S, int buf) {
    bf16* dys = lds + buf * STG;
    bf16* pat = dys + DYE;
    *reinterpret_cast<uint4*>(dys + tr_off<64>(tid >> 3, (tid & 7) * 8)) = S.dy;
#pragma unroll
    for (int i = 0; i < PPT; ++i) {
      const int e = tid + 512 * i;
      uint4 v = S.p[i];
      if (PRO && ((S.pok >> i) & 1u)) v = bn_relu8(v, psc, psh);
      if (e < PCH) *reinterpret_cast<uint4*>(pat + tr_off<64>(e >> 3, (e & 7) * 8)) = v;
    }
  };
  // patch row of tap (0, 0) for pixel p of a K step
  auto prow = [](int p) { return (p / (RR * W)) * PIMG + ((p % (RR * W)) / W) * PW + (p % W); };
  f32x4 acc[2][9];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int f = 0; f < 9; ++f) acc[i][f] = zero4();

  const int nk = (kend - kbeg + 63) / 64;
  const int g = lane >> 4;
  auto compute = [&](int cur) {
    const bf16* dys = lds + cur * STG;
    const bf16* pat = dys + DYE;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      bf16x8 af[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = frag_tr<64>(dys, wco * 32 + i * 16, hh * 32, lane);
      // this lane group's 8 pixels 32 hh + 8 g .. +7, as two 4-pixel halves within one image row
      const int k8 = hh * 32 + 8 * g;
      const int plo = prow(k8), phi = prow(k8 + 4);
#pragma unroll
      for (int f = 0; f < 9; ++f) {
        const int col = wn * 144 + f * 16;  // gradient column (tap, ci): 16 columns within one tap
        const int tap = col >> 6, ci0 = col & 63;
        const int r = tap / 3, s_ = tap - 3 * r;
        const bf16x8 b = frag_tr_rows(pat, ci0, plo + r * PW + s_, phi + r * PW + s_, lane);
#pragma unroll
        for (int i = 0; i < 2; ++i) acc[i][f] = mfma_bf16(af[i], b, acc[i][f]);
      }
    }
  };
  load(st0, kbeg);
  store(st0, 0);
  if (PF == 1) {
    __syncthreads();
    int cur = 0;
    for (int kt = 0; kt < nk; ++kt) {
      if (kt + 1 < nk) load(st0, kbeg + (kt + 1) * 64);
      compute(cur);
      if (kt + 1 < nk) store(st0, cur ^ 1);
      __syncthreads();
      cur ^= 1;
    }
  } else {
    // buf[kt & 1] holds K step kt; the register stage of K step kt + 1 is in flight. Two register
    // stages alternate (unrolled by two: register arrays need static indices)
    if (nk > 1) load(st1, kbeg + 64);
    __syncthreads();
    auto step = [&](int kt, Stage& free_st, const Stage& next_st) {
      if (kt + 2 < nk) load(free_st, kbeg + (kt + 2) * 64);  // free_st's K step kt is already in LDS
      compute(kt & 1);
      if (kt + 1 < nk) store(next_st, (kt + 1) & 1);
      __syncthreads();
    };
    for (int kt = 0; kt < nk; kt += 2) {
      step(kt, st0, st1);
      if (kt + 1 < nk) step(kt + 1, st1, st0);
    }
  }
  // Wf-layout gradient [co][tap][ci]: block column n = tap * 64 + local ci
  float* grad = a.grad + peer * a.grad_ps;
#pragma unroll
  for (int f = 0; f < 9; ++f) {
    const int nl = wn * 144 + f * 16 + (lane & 15);
    const int n = (nl >> 6) * a.x_c + ci0 + (nl & 63);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int co = co0 + wco * 32 + i * 16 + 4 * (lane >> 4) + e;
        float* dst = grad + (int64_t)co * ncol + n;
        if (a.accumulate) atomicAdd(dst, acc[i][f][e]);
        else *dst = acc[i][f][e];
      }
  }
}

// ------------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------------
// workgroups of a persistent DMA conv launch over all column tiles and peers (0 = one resident wave;
// tests set a small count so that every workgroup runs many M tiles)
static int g_conv_dma_wgs = 0;
extern "C" int conv_set_dma_wgs(int n) {
  const int old = g_conv_dma_wgs;
  g_conv_dma_wgs = n > 0 ? n : 0;
  return old;
}
// 64-channel 3x3 convs on 32-wide images through k_conv_fwd_halo (MYFYP_FWD_HALO=0: the DMA kernel)
static int g_fwd_halo = [] {
  const char* e = getenv("MYFYP_FWD_HALO");
  return (e != nullptr && atoi(e) == 0) ? 0 : 1;
}();
extern "C" int conv_set_fwd_halo(int on) {
  const int old = g_fwd_halo;
  if (on >= 0) g_fwd_halo = on ? 1 : 0;
  return old;
}
// 64-channel 3x3 weight gradients through k_conv_wgrad_halo (MYFYP_WGRAD_HALO=0: the generic kernel)
static int g_wgrad_halo = [] {
  const char* e = getenv("MYFYP_WGRAD_HALO");
  return (e != nullptr && atoi(e) == 0) ? 0 : 1;
}();
extern "C" int conv_set_wgrad_halo(int on) {
  const int old = g_wgrad_halo;
  if (on >= 0) g_wgrad_halo = on ? 1 : 0;
  return old;
}
// halo wgrad prefetch depth (k_conv_wgrad_halo PF): MYFYP_WGRAD_PF=1|2, conv_set_wgrad_pf (tests / A-B)
static int g_wgrad_halo_pf = [] {
  const char* e = getenv("MYFYP_WGRAD_PF");
  return (e != nullptr && atoi(e) == 1) ? 1 : 2;
}();
extern "C" int conv_set_wgrad_pf(int pf) {
  const int old = g_wgrad_halo_pf;
  if (pf == 1 || pf == 2) g_wgrad_halo_pf = pf;
  return old;
}
// widest channel count the halo wgrad takes (0 = any multiple of 64; MYFYP_WGRAD_HALO_MAXC, the A/B knob)
static int g_wgrad_halo_max_c = [] {
  const char* e = getenv("MYFYP_WGRAD_HALO_MAXC");
  return e != nullptr ? atoi(e) : 0;
}();
static int conv_num_cus() {
  static int cus = 0;
  if (cus == 0) {
    int dev = 0;
    hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  }
  return cus;
}

// forward-shaped convs through k_conv_fwd_dma (default) or k_conv_gemm's register stage
// (MYFYP_CONV_DMA=0, or conv_set_dma(0): the A/B switch)
static int g_conv_dma = -1;
static bool conv_dma_enabled() {
  if (g_conv_dma < 0) {
    const char* e = getenv("MYFYP_CONV_DMA");
    g_conv_dma = e != nullptr ? atoi(e) : 1;
  }
  return g_conv_dma != 0;
}
extern "C" int conv_set_dma(int v) {
  conv_dma_enabled();
  const int old = g_conv_dma;
  if (v >= 0) g_conv_dma = v;
  return old;
}

// compile-time epilogue operand set of a launch (conv_epilogue_tile SPEC), -1 = runtime flags
static int conv_spec(const ConvGemmArgs& a, int mode) {
  if (!HALO_SPEC || a.bias != nullptr || a.relu || a.ncol_valid != a.ncol) return -1;
  if (mode == 0) return (a.resid == nullptr && a.pro_ss == nullptr) ? (a.stats != nullptr ? 32 : 0) : -1;
  if (a.bnb_part0 == nullptr) return (a.resid == nullptr && a.stats == nullptr) ? 0 : -1;  // a plain dgrad
  return (a.resid ? 1 : 0) | 2 | (a.bnb_part1 ? 4 : 0) | (a.bnb_mask ? 8 : (a.bnb_mask_ss ? 16 : 0));
}

static int g_fin_dbg = 0;
extern "C" int conv_set_fin_debug(int bits) {
  const int old = g_fin_dbg;
  if (bits >= 0) g_fin_dbg = bits;
  return old;
}

extern "C" int conv_gemm_launch(int mode, const ConvGemmArgs* pa, int peers, void* stream) {
  ConvGemmArgs a_ = *pa;
  a_.fin_dbg = g_fin_dbg;
  const ConvGemmArgs& a = a_;
  if (a.fin_cnt != nullptr && a.ncol > FIN_CPT * 256) return 1;  // conv_fin_fwd / _bwd: channels per thread
  // mode 0 forward, 1 dgrad, 4 stride-1 dgrad as a forward conv over dY with k_conv_wt_flip weights
  // (the caller passes the forward-shaped arguments: src = dY, pad = R-1-pad, ncol = cin)
  // mode 5: stride-2 dgrad by parity class as forward convs over dY with conv_wt_flip_parity_launch's
  // weights (dgrad-shaped arguments: src = dY, out = dX, the conv's R, S, pad; LDS-DMA kernel only)
  if ((a.src_c & 7) || (a.ncol & 7) || peers < 1 || !(mode == 0 || mode == 1 || mode == 4 || mode == 5)) return 1;
  if ((mode == 4 || mode == 5) && a.pro_ss != nullptr) return 1;
  if ((mode == 4 && a.stride != 1) || (mode == 5 && (a.stride != 2 || !conv_dma_enabled()))) return 1;
  // the buffer-load gathers form 32-bit byte offsets within one peer's source and weights
  if (CONV_BUFLOAD && ((int64_t)a.max_batch * a.src_h * a.src_w * a.src_c * 2 >= INT32_MAX ||
                       (int64_t)a.ncol * a.R * a.S * a.src_c * 2 >= INT32_MAX))
    return 3;
  const bool wide = a.ncol > 64;
  hipStream_t s = (hipStream_t)stream;
  // 64 -> 64 channel 3x3 convs on 32-wide images (ResNet-18 layer 1): im2col from one staged patch.
  // The two-BN dgrad epilogue spilled in the register-staged version (252 vs 238 us on the DMA
  // kernel); the DMA-staged one (HALO_DMA4) has 0 spills with it
  if (((mode == 4 && (HALO_DMA4 || a.bnb_y1 == nullptr)) || mode == 0) && g_fwd_halo && a.src_c == 64 && a.ncol == 64 && a.R == 3 && a.S == 3 && a.stride == 1 &&
      a.pad == 1 && a.src_w == 32 && a.out_w == 32 && a.out_h == a.src_h && (a.src_h * 32) % 256 == 0) {
    const int tiles_m = (a.max_batch * a.out_h * 32 + 255) / 256;
    int G = g_conv_dma_wgs > 0 ? g_conv_dma_wgs : (conv_num_cus() + peers - 1) / peers;  // one workgroup per CU
    G = G < 1 ? 1 : (G > tiles_m ? tiles_m : G);
    // the layer-1 dgrads' two epilogue operand sets, compiled specialised (conv_epilogue_tile SPEC):
    // conv2 (BN1-backward sums, ReLU mask from y1) and conv1 (skip gradient, BN-backward sums of the
    // previous block's BN2, mask from the block input)
    // (the forward with the BN1 prologue counts as stats-only: the prologue is on the operand side)
    const int spec = mode == 4 ? (HALO_DMA4 ? conv_spec(a, 4) : -1) : (a.pro_ss ? [&] {
      ConvGemmArgs b = a;
      b.pro_ss = nullptr;
      return conv_spec(b, 0);
    }() : conv_spec(a, 0));
    if (mode == 4 && spec == 11) hipLaunchKernelGGL((k_conv_fwd_halo<4, false, 11>), dim3(G, 1, peers), dim3(512), 0, s, a, tiles_m);
    else if (mode == 4 && spec == 18) hipLaunchKernelGGL((k_conv_fwd_halo<4, false, 18>), dim3(G, 1, peers), dim3(512), 0, s, a, tiles_m);
    else if (mode == 4) hipLaunchKernelGGL((k_conv_fwd_halo<4, false>), dim3(G, 1, peers), dim3(512), 0, s, a, tiles_m);
    else if (a.pro_ss != nullptr && spec == 32) hipLaunchKernelGGL((k_conv_fwd_halo<0, true, 32>), dim3(G, 1, peers), dim3(512), 0, s, a, tiles_m);
    else if (a.pro_ss != nullptr && spec == 0) hipLaunchKernelGGL((k_conv_fwd_halo<0, true, 0>), dim3(G, 1, peers), dim3(512), 0, s, a, tiles_m);
    else if (a.pro_ss != nullptr) hipLaunchKernelGGL((k_conv_fwd_halo<0, true>), dim3(G, 1, peers), dim3(512), 0, s, a, tiles_m);
    else if (spec == 32) hipLaunchKernelGGL((k_conv_fwd_halo<0, false, 32>), dim3(G, 1, peers), dim3(512), 0, s, a, tiles_m);
    else if (spec == 0) hipLaunchKernelGGL((k_conv_fwd_halo<0, false, 0>), dim3(G, 1, peers), dim3(512), 0, s, a, tiles_m);
    else hipLaunchKernelGGL((k_conv_fwd_halo<0, false>), dim3(G, 1, peers), dim3(512), 0, s, a, tiles_m);
    return hipGetLastError() == hipSuccess ? 0 : 2;
  }
  if ((mode == 4 || mode == 5 || (mode == 0 && a.pro_ss == nullptr)) && conv_dma_enabled()) {
    // variant code (conv_set_dma / MYFYP_CONV_DMA): 1 = the measured defaults below; otherwise bits
    // 1-2 pick the 64-channel tile (0 register stage, 1 128x64/3 stages/2 per CU, 2 128x64/2/3,
    // 3 256x64/3/1), bits 3-4 the wide one (0 register stage, 1 256x128/3/1, 2 128x128/2/2) and
    // bits 5-6 the weight gradient's (conv_wgrad_launch)
    int v = g_conv_dma;
    if (v == 1) v = (2 << 1) | (2 << 3);  // measured best for every ResNet-18 shape (profiles/r3z_conv_dma)
    int var = wide ? (v >> 3) & 3 : (v >> 1) & 3;
    if (mode == 5 && var == 0) var = 2;  // no register-staged MODE 5
    if (var != 0) {
      const int bm = (wide ? var == 1 : var == 3) ? 256 : 128, bn = wide ? 128 : 64;
      const int rows = mode == 5 ? ((a.out_h + 1) >> 1) * ((a.out_w + 1) >> 1) : a.out_h * a.out_w;  // largest class
      const int tiles_m = (a.max_batch * rows + bm - 1) / bm;
      const int tiles_n = (a.ncol + bn - 1) / bn;
      // persistent over M tiles: about one resident wave of workgroups (occupancy x CUs) in all
      const int per_cu = (wide ? var == 1 : var == 3) ? 1 : (wide ? 2 : (var == 1 ? 2 : 3));
      const int want = g_conv_dma_wgs > 0 ? g_conv_dma_wgs : conv_num_cus() * per_cu;
      int G = (want + tiles_n * peers - 1) / (tiles_n * peers);
      G = G < 1 ? 1 : (G > tiles_m ? tiles_m : G);
      if (mode == 5) G = (G + 3) / 4;  // four classes share the resident wave
      dim3 grid(G * tiles_n, mode == 5 ? 4 : 1, peers), block(2 * bm);
#define DMA_LAUNCH(BM_, BN_, NS_, MB_)                                                                                   \
  do {                                                                                                                   \
    if (mode == 4) hipLaunchKernelGGL((k_conv_fwd_dma<4, BM_, BN_, NS_, MB_>), grid, block, 0, s, a, tiles_m, tiles_n); \
    else if (mode == 5) hipLaunchKernelGGL((k_conv_fwd_dma<5, BM_, BN_, NS_, MB_>), grid, block, 0, s, a, tiles_m, tiles_n); \
    else hipLaunchKernelGGL((k_conv_fwd_dma<0, BM_, BN_, NS_, MB_>), grid, block, 0, s, a, tiles_m, tiles_n);          \
  } while (0)
      // the default wide tile with the layers 2-4 operand sets compiled in (conv_epilogue_tile SPEC):
      // forward (BN statistics only; the evaluation's: nothing) and the stride-1 dgrads (conv2: BN1-backward, mask from a1;
      // conv1: skip gradient, previous BN2, mask from the block input; with a projection BN too it
      // spilled 22 VGPRs, so that one keeps the runtime flags)
      const int spec = conv_spec(a, mode);
      // MODE 5 (stride-2 dgrad by parity class): the projection's plain dgrad and the block conv1's
      // (skip gradient, previous BN2, mask from the block input), both tile widths
      if (mode == 5 && wide && var != 1 && spec == 0) hipLaunchKernelGGL((k_conv_fwd_dma<5, 128, 128, 2, 2, 0>), grid, block, 0, s, a, tiles_m, tiles_n);
      else if (mode == 5 && wide && var != 1 && spec == 11) hipLaunchKernelGGL((k_conv_fwd_dma<5, 128, 128, 2, 2, 11>), grid, block, 0, s, a, tiles_m, tiles_n);
      else if (mode == 5 && !wide && var == 2 && spec == 0) hipLaunchKernelGGL((k_conv_fwd_dma<5, 128, 64, 2, 3, 0>), grid, block, 0, s, a, tiles_m, tiles_n);
      else if (mode == 5 && !wide && var == 2 && spec == 11) hipLaunchKernelGGL((k_conv_fwd_dma<5, 128, 64, 2, 3, 11>), grid, block, 0, s, a, tiles_m, tiles_n);
      // the 64-column tile (the stem: K = 72, so the epilogue is most of the kernel) likewise
      else if (!wide && var == 2 && mode == 0 && spec == 32) hipLaunchKernelGGL((k_conv_fwd_dma<0, 128, 64, 2, 3, 32>), grid, block, 0, s, a, tiles_m, tiles_n);
      else if (!wide && var == 2 && mode == 0 && spec == 0) hipLaunchKernelGGL((k_conv_fwd_dma<0, 128, 64, 2, 3, 0>), grid, block, 0, s, a, tiles_m, tiles_n);
      else if (wide && var != 1 && mode == 0 && spec == 32) hipLaunchKernelGGL((k_conv_fwd_dma<0, 128, 128, 2, 2, 32>), grid, block, 0, s, a, tiles_m, tiles_n);
      else if (wide && var != 1 && mode == 0 && spec == 0) hipLaunchKernelGGL((k_conv_fwd_dma<0, 128, 128, 2, 2, 0>), grid, block, 0, s, a, tiles_m, tiles_n);
      else if (wide && var != 1 && mode == 4 && spec == 10) hipLaunchKernelGGL((k_conv_fwd_dma<4, 128, 128, 2, 2, 10>), grid, block, 0, s, a, tiles_m, tiles_n);
      else if (wide && var != 1 && mode == 4 && spec == 11) hipLaunchKernelGGL((k_conv_fwd_dma<4, 128, 128, 2, 2, 11>), grid, block, 0, s, a, tiles_m, tiles_n);
      else if (wide) {
        if (var == 1) DMA_LAUNCH(256, 128, 3, 1);
        else DMA_LAUNCH(128, 128, 2, 2);
      } else {
        if (var == 1) DMA_LAUNCH(128, 64, 3, 2);
        else if (var == 2) DMA_LAUNCH(128, 64, 2, 3);
        else DMA_LAUNCH(256, 64, 3, 1);
      }
#undef DMA_LAUNCH
      return hipGetLastError() == hipSuccess ? 0 : 2;
    }
  }
  const bool parity = mode == 1 && a.stride == 2;  // strided dgrad: one launch row per parity class
  const int rows = parity ? ((a.out_h + 1) >> 1) * ((a.out_w + 1) >> 1) : a.out_h * a.out_w;
  const int tiles_m = (a.max_batch * rows + 127) / 128;
  const int tiles_n = (a.ncol + (wide ? 127 : 63)) / (wide ? 128 : 64);
  dim3 grid(tiles_m * tiles_n, parity ? 4 : 1, peers), block(256);
#define CG_LAUNCH(M_, BN_, P_, ...) hipLaunchKernelGGL((k_conv_gemm<M_, BN_, P_, ##__VA_ARGS__>), grid, block, 0, s, a, tiles_m, tiles_n)
  if (mode == 4) {
    if (wide) CG_LAUNCH(4, 128, false);
    else CG_LAUNCH(4, 64, false);
  } else if (mode == 0 && a.pro_ss != nullptr) {
    if (wide) CG_LAUNCH(0, 128, true);
    else CG_LAUNCH(0, 64, true);
  } else if (mode == 0) {
    if (wide) CG_LAUNCH(0, 128, false);
    else CG_LAUNCH(0, 64, false);
  } else if (parity) {
    // stride-2 dgrads with their operand sets compiled in: the projection's (plain) and the block
    // conv1's (skip gradient, previous BN2, mask from the block input); 1-4-tap K loops leave the
    // epilogue the largest part of these kernels
    const int spec = conv_spec(a, 2);
    if (wide && spec == 0) CG_LAUNCH(2, 128, false, 0);
    else if (wide && spec == 11) CG_LAUNCH(2, 128, false, 11);
    else if (!wide && spec == 0) CG_LAUNCH(2, 64, false, 0);
    else if (!wide && spec == 11) CG_LAUNCH(2, 64, false, 11);
    else if (wide) CG_LAUNCH(2, 128, false);
    else CG_LAUNCH(2, 64, false);
  } else if (a.stride == 1) {  // MODE 3: MODE 1 specialised to stride 1 (no divisibility test, no division)
    if (wide) CG_LAUNCH(3, 128, false);
    else CG_LAUNCH(3, 64, false);
  } else {
    if (wide) CG_LAUNCH(1, 128, false);
    else CG_LAUNCH(1, 64, false);
  }
#undef CG_LAUNCH
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// Flipped, transposed weights for MODE 4: Wt[ci][r][s][co] = Wf[co][R-1-r][S-1-s][ci] per peer (both
// channel counts padded to multiples of 8). Per tap it is a [co][ci] -> [ci][co] transpose: 64 x 64
// tiles through LDS, 16-byte coalesced loads along ci and stores along co.
// parity_pad >= 0 (MODE 5, stride-2 dgrad with that padding): the four parity classes' weights in
// class order, class c = (ph, pw) as [ci][i'][j'][co] over its tR x tS taps r = r0 + 2 (tR-1-i'),
// s = s0 + 2 (tS-1-j') (flipped, so the class runs as a forward conv over dY).
// grid = (ceil(ci / 64) * ceil(co / 64), R * S, peers), block 256.
// One 64 x 64 tile (index `tile`) of destination tap `tap` of one peer's weights.
__device__ __forceinline__ void wt_flip_tile(const bf16* __restrict__ src, bf16* __restrict__ dst0, int cout, int cin, int R, int S, int parity_pad,
                                             int tile, int tap) {
  // row pad 2: the transposed reads (column of 8 rows per 8-lane group, 8 groups) hit 32 distinct
  // banks; a +8 pad put the groups 32 banks apart (12.4 conflicts per LDS instruction, profiles/r3z_pmc)
  __shared__ bf16 tile_l[64][64 + 2];
  auto& tl = tile_l;
  const int tci = (cin + 63) / 64;
  const int ci0 = (tile % tci) * 64, co0 = (tile / tci) * 64;
  const int RS = R * S;
  int rs_src, taps, dtap, base_taps;  // source tap, taps of the destination block, tap within it, taps before it
  if (parity_pad < 0) {
    rs_src = (R - 1 - tap / S) * S + (S - 1 - tap % S);
    taps = RS;
    dtap = tap;
    base_taps = 0;
  } else {
    int c = 0, t = tap;
    while (c < 3 && t >= conv_parity_taps(R, S, parity_pad, c)) t -= conv_parity_taps(R, S, parity_pad, c++);
    const int r0 = ((c >> 1) + parity_pad) & 1, s0 = ((c & 1) + parity_pad) & 1;
    const int tR = (R - r0 + 1) >> 1, tS = (S - s0 + 1) >> 1;
    const int ip = t / tS, jp = t - ip * tS;
    rs_src = (r0 + 2 * (tR - 1 - ip)) * S + s0 + 2 * (tS - 1 - jp);
    taps = tR * tS;
    dtap = t;
    base_taps = tap - t;
  }
  bf16* dst = dst0 + (int64_t)base_taps * cin * cout;
#pragma unroll
  for (int k = 0; k < 2; ++k) {  // 64 co rows x 8 chunks of 8 ci
    const int q = threadIdx.x + 256 * k, row = q >> 3, ch = q & 7;
    const int co = co0 + row, ci = ci0 + ch * 8;
    bf8 v{};
    if (co < cout && ci < cin) v = *reinterpret_cast<const bf8*>(src + ((int64_t)co * RS + rs_src) * cin + ci);
#pragma unroll
    for (int j = 0; j < 8; ++j) tl[row][ch * 8 + j] = v.v[j];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 2; ++k) {  // 64 ci rows x 8 chunks of 8 co
    const int q = threadIdx.x + 256 * k, row = q >> 3, ch = q & 7;
    const int ci = ci0 + row, co = co0 + ch * 8;
    if (ci >= cin || co >= cout) continue;
    bf8 v;
#pragma unroll
    for (int j = 0; j < 8; ++j) v.v[j] = tl[ch * 8 + j][row];
    *reinterpret_cast<bf8*>(dst + ((int64_t)ci * taps + dtap) * cout + co) = v;
  }
}

__global__ __launch_bounds__(256) void k_conv_wt_flip(const bf16* __restrict__ wf, int64_t wf_ps, bf16* __restrict__ wt, int64_t wt_ps, int cout,
                                                      int cin, int R, int S, int parity_pad) {
  const int peer = blockIdx.z;
  wt_flip_tile(wf + peer * wf_ps, wt + peer * wt_ps, cout, cin, R, S, parity_pad, blockIdx.x, blockIdx.y);
}

// Every MODE-4 layer's flip of a backward pass in ONE launch (instead of one launch before each
// layer's dgrad): block b of grid.x is tile (b - start[l]) / RS, tap (b - start[l]) % RS of layer l.
#define WT_FLIP_MAX 32
struct WtFlipBatch {
  int n;
  int start[WT_FLIP_MAX + 1];
  int64_t off[WT_FLIP_MAX];  // element offset of the layer's weights in both the Wf and the Wt buffer
  int cout[WT_FLIP_MAX], cin[WT_FLIP_MAX], R[WT_FLIP_MAX], S[WT_FLIP_MAX];
};
__global__ __launch_bounds__(256) void k_conv_wt_flip_multi(const bf16* __restrict__ wf, int64_t wf_ps, bf16* __restrict__ wt, int64_t wt_ps,
                                                            WtFlipBatch fb) {
  const int b = blockIdx.x, peer = blockIdx.y;
  int l = 0;
  while (l + 1 < fb.n && b >= fb.start[l + 1]) ++l;
  const int local = b - fb.start[l], RS = fb.R[l] * fb.S[l];
  wt_flip_tile(wf + peer * wf_ps + fb.off[l], wt + peer * wt_ps + fb.off[l], fb.cout[l], fb.cin[l], fb.R[l], fb.S[l], -1, local / RS, local % RS);
}

extern "C" int conv_wt_flip_launch(const void* wf, long long wf_ps, void* wt, long long wt_ps, int cout, int cin, int R, int S, int peers, void* stream) {
  if ((cout & 7) || (cin & 7) || peers < 1) return 1;
  const unsigned tiles = (unsigned)(((cin + 63) / 64) * ((cout + 63) / 64));
  hipLaunchKernelGGL(k_conv_wt_flip, dim3(tiles, (unsigned)(R * S), (unsigned)peers), dim3(256), 0, (hipStream_t)stream, (const bf16*)wf, (int64_t)wf_ps,
                     (bf16*)wt, (int64_t)wt_ps, cout, cin, R, S, -1);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
// n layers: offs[l] element offsets (same in wf and wt), dims[4 l ..] = cout, cin, R, S
extern "C" int conv_wt_flip_multi_launch(const void* wf, long long wf_ps, void* wt, long long wt_ps, int n, const long long* offs, const int* dims,
                                         int peers, void* stream) {
  if (n < 1 || n > WT_FLIP_MAX || peers < 1) return 1;
  WtFlipBatch fb{};
  fb.n = n;
  int blocks = 0;
  for (int l = 0; l < n; ++l) {
    const int cout = dims[4 * l], cin = dims[4 * l + 1], R = dims[4 * l + 2], S = dims[4 * l + 3];
    if ((cout & 7) || (cin & 7) || R < 1 || S < 1) return 1;
    fb.start[l] = blocks;
    fb.off[l] = offs[l];
    fb.cout[l] = cout;
    fb.cin[l] = cin;
    fb.R[l] = R;
    fb.S[l] = S;
    blocks += ((cin + 63) / 64) * ((cout + 63) / 64) * R * S;
  }
  fb.start[n] = blocks;
  hipLaunchKernelGGL(k_conv_wt_flip_multi, dim3((unsigned)blocks, (unsigned)peers), dim3(256), 0, (hipStream_t)stream, (const bf16*)wf, (int64_t)wf_ps,
                     (bf16*)wt, (int64_t)wt_ps, fb);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
// MODE 5's parity-class weights (stride-2 dgrad with padding `pad`)
extern "C" int conv_wt_flip_parity_launch(const void* wf, long long wf_ps, void* wt, long long wt_ps, int cout, int cin, int R, int S, int pad, int peers,
                                          void* stream) {
  if ((cout & 7) || (cin & 7) || peers < 1 || pad < 0) return 1;
  const unsigned tiles = (unsigned)(((cin + 63) / 64) * ((cout + 63) / 64));
  hipLaunchKernelGGL(k_conv_wt_flip, dim3(tiles, (unsigned)(R * S), (unsigned)peers), dim3(256), 0, (hipStream_t)stream, (const bf16*)wf, (int64_t)wf_ps,
                     (bf16*)wt, (int64_t)wt_ps, cout, cin, R, S, pad);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// rows of the BN statistics buffer a conv epilogue writes: one (sum, sumsq) accumulator row
// (MYFYP_BN_STAT_ROWS). Round 3 set 16: the 64-channel forward convs were then bound by 1024
// workgroups per peer adding into the same 128 addresses (144 -> 122 us per conv with 16 rows,
// profiles/r3z_conv_dma). The persistent convs now add once per workgroup, and a sweep of the
// row counts of both buffers on the round-4 tree put 4 ahead: ResNet-18 2.689 (4) / 2.681 (8) /
// 2.675 (16) / 2.684 (2) / 2.683 (1) rounds/s, 3 alternations each (profiles/r4sw_bn_rows)
extern "C" int conv_gemm_stats_rows(int max_batch, int out_h, int out_w) {
  static int rows = -1;
  if (rows < 0) {
    const char* e = getenv("MYFYP_BN_STAT_ROWS");
    rows = e != nullptr && atoi(e) >= 1 ? atoi(e) : 4;
  }
  const int tiles = (max_batch * out_h * out_w + 127) / 128;
  return rows < tiles ? rows : (tiles > 0 ? tiles : 1);
}
// rows of the BN-backward partial-sum buffers (MYFYP_BNB_ROWS, default 4 — see above; conv epilogues and
// k_bn_bwd_reduce accumulate into them, k_bn_bwd_finalize sums and re-zeroes every row)
extern "C" int conv_fin_words() { return FIN_WORDS; }
// layout of the argument structs the Python side mirrors with ctypes (checked when it loads the
// library): size and offset of the last field of ConvGemmArgs, then of WgradArgs
extern "C" int conv_args_abi(long long* out) {
  out[0] = (long long)sizeof(ConvGemmArgs);
  out[1] = (long long)offsetof(ConvGemmArgs, fin_dbg);
  out[2] = (long long)sizeof(WgradArgs);
  out[3] = (long long)offsetof(WgradArgs, pro_ss_ps);
  return 4;
}  // ints per peer of a ConvGemmArgs::fin_cnt buffer

extern "C" int conv_bnb_rows() {
  static int rows = -1;
  if (rows < 0) {
    const char* e = getenv("MYFYP_BNB_ROWS");
    rows = e != nullptr && atoi(e) >= 1 ? atoi(e) : 4;
  }
  return rows;
}

extern "C" int conv_wgrad_launch(const WgradArgs* pa, int peers, int splits, void* stream) {
  const WgradArgs& a = *pa;
  if ((a.x_c & 7) || (a.dy_c & 7) || (a.k_per_split & 63) || peers < 1 || splits < 1) return 1;
  if (splits > 1 && !a.accumulate) return 1;  // split-K partial sums must be added
  if (CONV_BUFLOAD && ((int64_t)a.max_batch * a.H * a.W * a.x_c * 2 >= INT32_MAX ||
                       (int64_t)a.max_batch * a.Ho * a.Wo * a.dy_c * 2 >= INT32_MAX))
    return 3;  // 32-bit byte offsets of the buffer-load gathers
  const int ncol = a.R * a.S * a.x_c;
  const bool wm = a.dy_c > 64, wn = ncol > 64;
  const int BM = wm ? 128 : 64, BN = wn ? 128 : 64;
  const int tiles_m = (a.dy_c + BM - 1) / BM, tiles_n = (ncol + BN - 1) / BN;
  dim3 grid(tiles_m * tiles_n * splits, 1, peers), block(256);
  hipStream_t s = (hipStream_t)stream;
  // 64 -> 64 channel 3x3 stride-1 convs (ResNet-18 layer 1): all nine taps from one staged X patch
  const bool halo_shape = ((a.H * a.W) % 64 == 0 && (a.W == 8 || a.W == 16 || a.W == 32 || a.W == 64)) || (a.H == 4 && a.W == 4);
  if (g_wgrad_halo && a.x_c % 64 == 0 && a.dy_c % 64 == 0 && a.R == 3 && a.S == 3 && a.stride == 1 && a.pad == 1 &&
      a.Ho == a.H && a.Wo == a.W && halo_shape && (g_wgrad_halo_max_c == 0 || (a.x_c <= g_wgrad_halo_max_c && a.dy_c <= g_wgrad_halo_max_c))) {
    const int tco = a.dy_c / 64, tci = a.x_c / 64;
    dim3 hg(splits * tco * tci, 1, peers), hb(512);
#define WH_LAUNCH(W_, HI_)                                                                                                  \
  do {                                                                                                                       \
    if (g_wgrad_halo_pf == 2) {                                                                                              \
      if (a.pro_ss != nullptr) hipLaunchKernelGGL((k_conv_wgrad_halo<W_, HI_, true, 2>), hg, hb, 0, s, a, splits, tco, tci);  \
      else hipLaunchKernelGGL((k_conv_wgrad_halo<W_, HI_, false, 2>), hg, hb, 0, s, a, splits, tco, tci);                    \
    } else {                                                                                                                 \
      if (a.pro_ss != nullptr) hipLaunchKernelGGL((k_conv_wgrad_halo<W_, HI_, true, 1>), hg, hb, 0, s, a, splits, tco, tci);  \
      else hipLaunchKernelGGL((k_conv_wgrad_halo<W_, HI_, false, 1>), hg, hb, 0, s, a, splits, tco, tci);                    \
    }                                                                                                                        \
  } while (0)
    if (a.W == 4) WH_LAUNCH(4, 4);  // 4 images per K step
    else if (a.W == 8) WH_LAUNCH(8, 0);
    else if (a.W == 16) WH_LAUNCH(16, 0);
    else if (a.W == 32) WH_LAUNCH(32, 0);
    else WH_LAUNCH(64, 0);
#undef WH_LAUNCH
    return hipGetLastError() == hipSuccess ? 0 : 2;
  }
  // LDS-DMA stage ring (conv_set_dma variant bits 5-6: 0 register stage, 1 two stages, 2 three
  // stages). The default code 1 keeps the register stage: in the engine the two-stage ring measured
  // 3-10 % slower per wgrad shape (same-box kernel traces, profiles/r3z_conv_dma), although the
  // isolated probe put it within 3 % either way.
  const int wv = conv_dma_enabled() && g_conv_dma != 1 ? (g_conv_dma >> 5) & 3 : 0;
  if (a.pro_ss == nullptr && wv != 0) {
#define WGD_LAUNCH(BM_, BN_, NS_, MB_) hipLaunchKernelGGL((k_conv_wgrad_dma<BM_, BN_, NS_, MB_>), grid, block, 0, s, a, tiles_m, tiles_n, splits)
    if (wv == 1) {
      if (wm && wn) WGD_LAUNCH(128, 128, 2, 2);
      else if (wm) WGD_LAUNCH(128, 64, 2, 3);
      else if (wn) WGD_LAUNCH(64, 128, 2, 3);
      else WGD_LAUNCH(64, 64, 2, 4);
    } else {
      if (wm && wn) WGD_LAUNCH(128, 128, 3, 1);
      else if (wm) WGD_LAUNCH(128, 64, 3, 2);
      else if (wn) WGD_LAUNCH(64, 128, 3, 2);
      else WGD_LAUNCH(64, 64, 3, 3);
    }
#undef WGD_LAUNCH
    return hipGetLastError() == hipSuccess ? 0 : 2;
  }
#define WG_LAUNCH(BM_, BN_)                                                                                      \
  do {                                                                                                           \
    if (a.pro_ss != nullptr) hipLaunchKernelGGL((k_conv_wgrad<BM_, BN_, true>), grid, block, 0, s, a, tiles_m, tiles_n, splits); \
    else hipLaunchKernelGGL((k_conv_wgrad<BM_, BN_, false>), grid, block, 0, s, a, tiles_m, tiles_n, splits);  \
  } while (0)
  if (wm && wn) WG_LAUNCH(128, 128);
  else if (wm) WG_LAUNCH(128, 64);
  else if (wn) WG_LAUNCH(64, 128);
  else WG_LAUNCH(64, 64);
#undef WG_LAUNCH
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// Resolve one kernel of this translation unit on the current device: loads the unit's code object
// now (myfyp_warm_all, at engine prewarm) instead of at its first launch, which waited for the
// kernels in flight (the first FedAvg launch blocked the host until the running epoch ended)
extern "C" int myfyp_warm_conv() {
  hipFuncAttributes attr;
  return hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(&k_conv_wt_flip)) == hipSuccess ? 0 : 1;
}
