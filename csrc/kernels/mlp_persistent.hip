// Weight-stationary persistent epoch kernel for the reference MLP (784-256-128-10) on gfx950.
//
// Why: the 3-launch step (mlp_fused.hip) re-reads and re-writes every peer's fp32 master weights and
// Adam moments each step (~49 MB/step for 8 peers) and pays three kernel boundaries per step. Here a
// whole local epoch is ONE launch and the optimizer state never leaves the chip: every peer is a
// gang of 17 workgroups (512 threads, one per CU) that live for the epoch —
//
//   owner g (g = 0..15) keeps W1 rows 16g..16g+15 (+ b1 slice) and W2 columns 16g..16g+15 as fp32
//            {w, m, v} IN REGISTERS, laid out exactly as the MFMA operand/result fragments that use
//            them, and the step's input batch in LDS. It computes H1[:, 16g:16g+16] (forward),
//            dH1 slice = dH2 · W2[:, slice] ⊙ [H1>0], dW1 rows, dW2 columns, and applies Adam/SGD to
//            its own registers.
//   head     keeps W3, b2, b3; computes H2 = relu(H1·W2ᵀ+b2), logits, log-softmax + NLL, dlogits,
//            dH2 = dlogits·W3 ⊙ [H2>0], dW3, db2, db3.
//
// Per step the gang exchanges three small tiles through L2 (H1 2 KB per owner → head; dH2 16 KB head →
// owners; the updated bf16 W2 slice 4 KB per owner → head), with write-through (sc1) stores, a drained
// sc1 flag per producer and sc1 loads on the consumer (cdna_hip_programming.md §6 Guideline 16, valid
// form row 1 of MI355X_MICROARCH.md's hand-off table). Flags carry the step number, so no flag is ever
// reset inside a launch; the launch's memset node zeroes them. Every spin is bounded (1 s) and sets a
// sticky error word the host checks with the step statistics.
//
// Fragment bookkeeping. MFMA v_mfma_f32_16x16x32_bf16: lane (h = l>>4, c = l&15) holds
// A[c][8h+j], B[8h+j][c], C[4h+i][c]. A weight-gradient tile computed as C[m = input index][n = c]
// puts 4h+i of the input dimension in lane (h, c); a 32-wide K step split into two such tiles gives
// lane h the inputs {4h..4h+3, 16+4h..16+4h+3}. The forward (and dH1) MFMAs therefore use the
// K-slot permutation κ(h, j) = j < 4 ? 4h + j : 16 + 4h + (j − 4) on BOTH operands, so the gradient
// of a weight lands in the very lane and register slot that holds the weight: the optimizer is an
// in-register epilogue with no data movement.
//
// Placement: block b serves XCD slot b % 8, so the 17 workgroups of a gang share one XCD's L2 under
// round-robin dispatch (speed only — the protocol does not depend on placement).
#include "mlp_persistent.h"
#include "persist_common.h"

// Optional phase timestamps (build with -DMLP_STAMPS): peer 0's owner 0 and head, steps < 32,
// read with mlp_debug_persistent_stamps (wall_clock64 ticks, 100 MHz).
#ifdef MLP_STAMPS
__device__ unsigned long long g_pe_stamps[2][32][8];
#define PE_STAMP(role, t, i)                                                               \
  do {                                                                                     \
    if (p == 0 && threadIdx.x == 0 && (t) < 32) g_pe_stamps[role][t][i] = wall_clock64(); \
  } while (0)
extern "C" int mlp_debug_persistent_stamps(void* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pe_stamps), sizeof(g_pe_stamps)) == hipSuccess ? 0 : 1;
}
#else
#define PE_STAMP(role, t, i) \
  do {                       \
  } while (0)
#endif

namespace {

using persist::gu32;
using persist::gu64;
using persist::ld_wt;
using persist::row_max16;
using persist::row_min16;
using persist::row_sum16;
using persist::st_wt;
using persist::al16;

constexpr int NT = 512;  // threads per workgroup (8 waves)
constexpr int NG = 16;   // owners per peer (D1 / 16)
constexpr int PD1 = 256, PD2 = 128;
constexpr int ROLES = NG + 1;
constexpr int FLAGS_PER_PEER = 2 * NG + 3;
constexpr int F_XCC = 2 * NG + 1;  // two lines: the roles' XCC reports (persist::gang_same_xcd)
constexpr int F_H1 = 0, F_W2 = NG, F_DH2 = 2 * NG;
constexpr int KS1_MAX = 32;                              // D0 <= 1024
constexpr int LD2 = PD2 + 8;                             // bf16 row stride of [*][128] LDS tiles
constexpr int LDH = PD1 + 8;                             // bf16 row stride of [*][256] LDS tiles
constexpr int LDL = 40;                                  // dlogits [b][32 (classes, K-padded)] + 8
constexpr int LDW3 = PD2 + 8;                            // W3 bf16 [32][128] + 8

__device__ __forceinline__ int kappa(int h, int j) { return j < 4 ? 4 * h + j : 16 + 4 * h + (j - 4); }

typedef short pe_s16x4 __attribute__((ext_vector_type(4)));
// v_mfma_f32_16x16x16_bf16: A lane (h, c) = A[c][4h..4h+3], B = B[4h..4h+3][c], C as 16x16x32
__device__ __forceinline__ f32x4 mfma16_bf16(const bf16x4& a, const bf16x4& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(pe_s16x4, a), __builtin_bit_cast(pe_s16x4, b), c, 0, 0, 0);
}

__device__ __forceinline__ bf16x8 cat8(const bf16x4& lo, const bf16x4& hi) {
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

__device__ __forceinline__ void publish(unsigned* flags, int p, int idx, unsigned value, int plain) {
  persist::publish_p(flags, FLAGS_PER_PEER, p, idx, value, plain);
}
// 8-byte hand-off payload store: plain in a single-XCD gang (the line stays in that XCD's L2),
// write-through otherwise (persist::pub32, mlp_persistent_f32.hip)
__device__ __forceinline__ void pub64(int plain, void* ptr, unsigned long long v) {
  if (plain)
    __hip_atomic_store((persist::gu64*)ptr, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  else
    persist::st_wt(ptr, v);
}
__device__ __forceinline__ bool wg_wait(unsigned* flags, int p, int idx0, int n, unsigned target, int* err, int* sOk) {
  return persist::wg_wait(flags, FLAGS_PER_PEER, p, idx0, n, target, err, sOk);
}

__device__ __forceinline__ int rows_at(const MLPArgs& a, int n, int t) {
  const int r = n - t * a.B;
  return r < 0 ? 0 : (r > a.B ? a.B : r);
}

__device__ __forceinline__ void bias_corr(const MLPArgs& a, int t0, int t, float& lr_t, float& inv) {
  persist::bias_corr(a.opt, t0, t, lr_t, inv);
}

// torch.optim.Adam / SGD(no momentum) update in registers. The register-resident epilogue runs on
// the step's critical path (~15 k parameters per owner workgroup), so it uses the hardware
// v_sqrt_f32 / v_rcp_f32 (1 ulp) instead of the IEEE-exact division sequence of opt_update.
template <bool ADAM>
__device__ __forceinline__ void upd(const MLPArgs& a, float g, float& w, float& m, float& v, float lr_t, float inv) {
  const OptParams& o = a.opt;
  g = fmaf(o.weight_decay, w, g);  // weight_decay = 0: exact no-op, and no branch
  if (ADAM) {
    m = fmaf(o.beta1, m, (1.f - o.beta1) * g);
    v = fmaf(o.beta2, v, (1.f - o.beta2) * (g * g));
    const float denom = fmaf(__builtin_amdgcn_sqrtf(v), inv, o.eps);
    w = fmaf(-lr_t, m * __builtin_amdgcn_rcpf(denom), w);
  } else {
    w = fmaf(-o.lr, g, w);
  }
}

// ---- LDS carving (all offsets multiples of 16 bytes; dynamic region only: Guideline 17)
struct OwnerLds {
  int ldx;  // bf16 row stride of the X tile
  size_t x, red, dh2, h1, dh1, w2g, b1, db1, ok, total;
};
__host__ __device__ inline OwnerLds owner_lds(int Bpad, int D0) {
  OwnerLds L;
  const int ks1 = (D0 + 31) / 32;
  L.ldx = ks1 * 32 + 8;
  const int MT = Bpad / 16;
  size_t o = 0;
  L.x = o;   o += al16((size_t)Bpad * L.ldx * 2);
  L.red = o; o += al16((size_t)8 * MT * 64 * 16);
  L.dh2 = o; o += al16((size_t)Bpad * LD2 * 2);
  L.h1 = o;  o += al16((size_t)Bpad * 16 * 2);
  L.dh1 = o; o += al16((size_t)Bpad * 16 * 2);
  L.w2g = o; o += al16((size_t)PD2 * 16 * 2);
  L.b1 = o;  o += al16(3 * 16 * 4);
  L.db1 = o; o += al16(16 * 4);
  L.ok = o;  o += 16;
  L.total = o;
  return L;
}
struct HeadLds {
  size_t h1, h2, dlog, w3, b2, b3, ok, total;
};
__host__ __device__ inline HeadLds head_lds(int Bpad) {
  HeadLds L;
  const int MT = Bpad / 16;
  size_t o = 0;
  L.h1 = o;   o += al16((size_t)Bpad * LDH * 2);  // also the dH2 staging tile (disjoint lifetimes)
  L.h2 = o;   o += al16((size_t)Bpad * LD2 * 2);
  L.dlog = o; o += al16((size_t)Bpad * LDL * 2);
  L.w3 = o;   o += al16((size_t)32 * LDW3 * 2);
  L.b2 = o;   o += al16(3 * PD2 * 4);
  L.b3 = o;   o += al16(3 * 16 * 4);
  L.ok = o;   o += 16;
  L.total = o;
  return L;
}

// =============================================================================================
// owner workgroup
// =============================================================================================
template <int BP, bool ADAM>
__device__ void owner(const MLPArgs& a, const MLPPersistBufs& pb, int p, int g, char* smem) {
  constexpr int MT = BP / 16;
  constexpr int XPT = BP / 4;  // 8-byte X chunks per lane: 4 K steps x BP rows x 4 chunks / 64 lanes
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 4, c = lane & 15;
  const int D0 = a.D0, KS1 = (D0 + 31) / 32;
  const OwnerLds L = owner_lds(BP, D0);
  const int LDX = L.ldx;
  bf16* sX = reinterpret_cast<bf16*>(smem + L.x);
  f32x4* sRed = reinterpret_cast<f32x4*>(smem + L.red);
  bf16* sDH2 = reinterpret_cast<bf16*>(smem + L.dh2);
  bf16* sH1 = reinterpret_cast<bf16*>(smem + L.h1);
  bf16* sDH1 = reinterpret_cast<bf16*>(smem + L.dh1);
  bf16* sW2g = reinterpret_cast<bf16*>(smem + L.w2g);
  float* sB1 = reinterpret_cast<float*>(smem + L.b1);  // [3][16] w, m, v
  float* sDb1 = reinterpret_cast<float*>(smem + L.db1);
  int* sOk = reinterpret_cast<int*>(smem + L.ok);

  const int4 ctl = a.ctl[p];
  const bool fresh = (ctl.x & 2) != 0;  // fresh optimizer state this fit: moments start at 0
  const int n = ctl.y;
  const int nsteps = (n + a.B - 1) / a.B;
  const int64_t pS = (int64_t)p * a.S;
  constexpr bool adam = ADAM;

  // ---- resident state: W1 rows (all waves; wave w owns K steps w, w+8, w+16, w+24) and the W2
  //      column slice (waves 4..7; wave 4+k owns o2 32k..32k+31)
  float w1[4][8], m1[4][8], v1[4][8];
  float w2[4], m2[4], v2[4];
  const int orow = NG * g + c;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int s = wave + 8 * q;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int k = 32 * s + 16 * half + 4 * h;
      float4 wv = {0.f, 0.f, 0.f, 0.f}, mv = wv, vv = wv;
      if (s < KS1 && k < D0) {
        const int64_t idx = pS + a.off_w1 + (int64_t)orow * D0 + k;
        wv = *reinterpret_cast<const float4*>(a.params + idx);
        if (!fresh) {
          mv = *reinterpret_cast<const float4*>(a.m + idx);
          if (adam) vv = *reinterpret_cast<const float4*>(a.v + idx);
        }
      }
      const float wa[4] = {wv.x, wv.y, wv.z, wv.w}, ma[4] = {mv.x, mv.y, mv.z, mv.w}, va[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        w1[q][4 * half + i] = wa[i];
        m1[q][4 * half + i] = ma[i];
        v1[q][4 * half + i] = va[i];
      }
    }
  }
  // W2 slice: wave w holds W2[16w + 4h + j][16g + c], j < 4 — the B fragment of a 16x16x16 MFMA
  // over its 16 o2 rows and, identically, the lane layout of the dW2 tile C[o2][o] it computes
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int64_t idx = pS + a.off_w2 + (int64_t)(16 * wave + 4 * h + j) * PD1 + NG * g + c;
    w2[j] = a.params[idx];
    m2[j] = fresh ? 0.f : a.m[idx];
    v2[j] = (adam && !fresh) ? a.v[idx] : 0.f;
  }
  if (tid < 16) {
    const int64_t idx = pS + a.off_b1 + NG * g + tid;
    sB1[tid] = a.params[idx];
    sB1[16 + tid] = fresh ? 0.f : a.m[idx];
    sB1[32 + tid] = (adam && !fresh) ? a.v[idx] : 0.f;
  }

  // ---- X staging. Every wave only ever reads its OWN K-step columns of the batch tile (the
  //      forward A fragments and the dW1 Xᵀ fragments of K steps w, w+8, w+16, w+24), so each
  //      wave stages exactly those columns itself, with no workgroup barrier: bf16 in LDS, rows
  //      beyond the valid batch zero; the K padding columns D0..KS1*32 are zeroed once.
  //      Chunk k of lane l: K step wave + 8 (k / (BP/16)), row ((k % (BP/16)) * 64 + l) / 4,
  //      8 columns at 8 * (l % 4).
  auto xw_addr = [&](int t, int k, int lv, bool& ok, int& r, int& col) {
    const int q = k / (BP / 16), kk = k % (BP / 16);
    const int s = wave + 8 * q;
    const int idx = kk * 64 + lv;
    r = idx >> 2;
    col = 32 * s + 8 * (idx & 3);
    ok = s < KS1 && col < D0;
    return a.Xb16 + ((int64_t)p * a.xb_rows + (int64_t)t * a.B + r) * D0 + col;
  };
  auto xw_stage = [&](int t, int lv) {  // batch t -> LDS (16-byte bf16 chunks, no conversion)
    const int rows = rows_at(a, n, t);
#pragma unroll
    for (int k = 0; k < XPT; ++k) {
      bool ok;
      int r, col;
      const bf16* src = xw_addr(t, k, lv, ok, r, col);
      if (ok) *reinterpret_cast<uint4*>(sX + r * LDX + col) = r < rows ? *reinterpret_cast<const uint4*>(src) : uint4{0u, 0u, 0u, 0u};
    }
  };
  for (int e = tid; e < BP * (KS1 * 32 - D0); e += NT) {
    const int r = e / (KS1 * 32 - D0), q = e % (KS1 * 32 - D0);
    sX[r * LDX + D0 + q] = (bf16)0.f;
  }
  if (nsteps > 0) xw_stage(0, lane);

  // ---- the bf16 W2 slice goes to the head in ITS B-fragment order: chunk (wave w, K step ks,
  //      lane l) = 8 bf16 W2[16w + (l & 15)][32ks + 8(l >> 4) .. +8] at w2x[p][w][ks][l], so each
  //      head wave reads 1 KB contiguous per load instruction. This owner's 16 columns are K step
  //      g/2, lane groups 2(g&1) and 2(g&1)+1. One 8-byte write-through store per thread.
  auto w2_store = [&](int tv) {
    const int o2 = tv >> 2, part = tv & 3, half = part >> 1, sub = part & 1;
    const int lane_h = 2 * (g & 1) + half;
    const int64_t chunk = (((int64_t)p * 8 + (o2 >> 4)) * (PD1 / 32) + (g >> 1)) * 64 + lane_h * 16 + (o2 & 15);
    pub64(pb.plain, pb.w2x + chunk * 8 + 4 * sub, *reinterpret_cast<const unsigned long long*>(sW2g + o2 * 16 + 4 * part));
  };
  // ---- initial W2 publish (version 1)
  auto publish_w2 = [&](unsigned version) {
#pragma unroll
    for (int j = 0; j < 4; ++j) sW2g[(16 * wave + 4 * h + j) * 16 + c] = (bf16)w2[j];
    __syncthreads();
    w2_store(tid);
    publish(pb.flags, p, F_W2 + g, version, pb.plain);
  };
  publish_w2(1u);

  for (int t = 0; t < nsteps; ++t) {
    // per-iteration copy of the thread index, opaque to the compiler: every address below is
    // re-derived each step instead of being hoisted out of the loop and kept live (VGPR pressure)
    int tv = tid;
    asm volatile("" : "+v"(tv));
    const int rows = rows_at(a, n, t);
    float lr_t, inv_bc2;
    bias_corr(a, ctl.z, t, lr_t, inv_bc2);
    if (tid < 16) sDb1[tid] = 0.f;
    if (g == 0) PE_STAMP(0, t, 0);

    // ================= A: H1 slice = relu(X · W1sliceᵀ + b1), split-K over the 8 waves
    {
      f32x4 acc[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt] = zero4();
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int s = wave + 8 * q;
        if (s < KS1) {
          bf16x8 bw;
#pragma unroll
          for (int j = 0; j < 8; ++j) bw[j] = (bf16)w1[q][j];
#pragma unroll
          for (int mt = 0; mt < MT; ++mt) {
            const bf16* xp = sX + (16 * mt + c) * LDX + 32 * s + 4 * h;
            const bf16x8 af = cat8(*reinterpret_cast<const bf16x4*>(xp), *reinterpret_cast<const bf16x4*>(xp + 16));
            acc[mt] = mfma_bf16(af, bw, acc[mt]);
          }
        }
        __builtin_amdgcn_sched_barrier(0);  // bound the live fragment set (register pressure)
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) sRed[(wave * MT + mt) * 64 + lane] = acc[mt];
    }
    lds_barrier();
    if (tid < MT * 64) {
      const int mt = tid >> 6, hh = (tid & 63) >> 4, cc = tid & 15;
      f32x4 s = sRed[mt * 64 + (tid & 63)];
#pragma unroll
      for (int w = 1; w < 8; ++w) s += sRed[(w * MT + mt) * 64 + (tid & 63)];
      const float bias = sB1[cc];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int b = 16 * mt + 4 * hh + i;
        const float v = b < rows ? fmaxf(s[i] + bias, 0.f) : 0.f;
        sH1[b * 16 + cc] = (bf16)v;
      }
    }
    lds_barrier();
    if (tid < BP * 4) {
      const int b = tv >> 2, part = tv & 3;
      pub64(pb.plain, pb.h1x + ((int64_t)p * BP + b) * PD1 + NG * g + 4 * part, *reinterpret_cast<const unsigned long long*>(sH1 + b * 16 + 4 * part));
    }
    publish(pb.flags, p, F_H1 + g, (unsigned)(t + 1), pb.plain);
    if (g == 0) PE_STAMP(0, t, 1);

    // next step's batch: pull this wave's columns into the XCD's L2 while the head works (the
    // loads are consumed right away, so no registers stay live across the backward phase); they
    // are re-read from L2 and staged after this wave's dW1 update
    const bool more = t + 1 < nsteps;
    if (more) {  // one 4-byte load per 64-byte row segment pulls the line into L2
      const int rows_n = rows_at(a, n, t + 1);
      unsigned sink = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int s = wave + 8 * q;
        const int r = lane;  // rows 0..63 (BP <= 64)
        if (s < KS1 && r < rows_n && r < BP)
          sink ^= *reinterpret_cast<const unsigned*>(a.Xb16 + ((int64_t)p * a.xb_rows + (int64_t)(t + 1) * a.B + r) * D0 + 32 * s);
      }
      asm volatile("" ::"v"(sink));
    }

    // ================= C: backward of this slice
    if (!wg_wait(pb.flags, p, F_DH2, 1, (unsigned)(t + 1), pb.err, sOk)) return;
    if (g == 0) PE_STAMP(0, t, 2);
#pragma unroll
    for (int k = 0; k < BP / 16; ++k) {  // BP x 128 bf16 = BP*32 chunks of 8 B
      const int e = tv + NT * k;
      const int b = e >> 5, q = e & 31;
      const unsigned long long v = ld_wt(pb.dh2x + ((int64_t)p * BP + b) * PD2 + 4 * q);
      *reinterpret_cast<unsigned long long*>(sDH2 + b * LD2 + 4 * q) = v;
    }
    lds_barrier();
    // C1: dH1 partials — every wave its 16 o2 rows (K = 16), W2 before this step's update
    {
      bf16x4 bw;
#pragma unroll
      for (int j = 0; j < 4; ++j) bw[j] = (bf16)w2[j];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
        sRed[(wave * MT + mt) * 64 + lane] = mfma16_bf16(*reinterpret_cast<const bf16x4*>(sDH2 + (16 * mt + c) * LD2 + 16 * wave + 4 * h), bw, zero4());
    }
    lds_barrier();
    if (tid < MT * 64) {
      const int mt = tid >> 6, hh = (tid & 63) >> 4, cc = tid & 15;
      f32x4 s = sRed[mt * 64 + (tid & 63)];
#pragma unroll
      for (int w = 1; w < 8; ++w) s += sRed[(w * MT + mt) * 64 + (tid & 63)];
      float db = 0.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int b = 16 * mt + 4 * hh + i;
        const bf16 d = (bf16)((float)sH1[b * 16 + cc] > 0.f ? s[i] : 0.f);
        sDH1[b * 16 + cc] = d;
        db += (float)d;
      }
      db += __shfl_xor(db, 16);
      db += __shfl_xor(db, 32);
      if (hh == 0) atomicAdd(&sDb1[cc], db);
    }
    lds_barrier();
    if (g == 0) PE_STAMP(0, t, 3);
    // C3 (every wave, its 16 o2 rows): dW2 tile + update, bf16 slice staged in LDS for the publish
    // below; then C2 (every wave, its own K steps): dW1 rows + update
    {
      f32x4 acc = zero4();
#pragma unroll
      for (int kb = 0; kb < BP / 32; ++kb) acc = mfma_bf16(frag_b_tr(sDH2, LD2, 32 * kb, 16 * wave), frag_b_tr(sH1, 16, 32 * kb, 0), acc);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        upd<ADAM>(a, acc[j], w2[j], m2[j], v2[j], lr_t, inv_bc2);
        sW2g[(16 * wave + 4 * h + j) * 16 + c] = (bf16)w2[j];
      }
    }
    {
      bf16x8 bd[BP / 32];
#pragma unroll
      for (int kb = 0; kb < BP / 32; ++kb) bd[kb] = frag_b_tr(sDH1, 16, 32 * kb, 0);
      int lv = lane;
      asm volatile("" : "+v"(lv));
      const int rows_next = more ? rows_at(a, n, t + 1) : 0;
      const bf16* xnext = a.Xb16 + ((int64_t)p * a.xb_rows + (int64_t)(t + 1) * a.B) * D0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int s = wave + 8 * q;
        __builtin_amdgcn_sched_barrier(0);
        if (s < KS1) {
          // the next batch's columns of this K step (L2-resident since the touch above): issued
          // first, landed in LDS right after this K step's dW1 MFMAs have read the current ones
          constexpr int XQ = BP / 16;
          uint4 xq[XQ];
#pragma unroll
          for (int kk = 0; kk < XQ; ++kk) {
            const int idx = kk * 64 + lv;
            const int r = idx >> 2, col = 32 * s + 8 * (idx & 3);
            xq[kk] = (more && col < D0 && r < rows_next) ? *reinterpret_cast<const uint4*>(xnext + (unsigned)(r * D0 + col)) : uint4{0u, 0u, 0u, 0u};
          }
          float gr[8];
#pragma unroll
          for (int tt = 0; tt < 2; ++tt) {
            f32x4 acc = zero4();
#pragma unroll
            for (int kb = 0; kb < BP / 32; ++kb) acc = mfma_bf16(frag_b_tr(sX, LDX, 32 * kb, 32 * s + 16 * tt), bd[kb], acc);
#pragma unroll
            for (int i = 0; i < 4; ++i) gr[4 * tt + i] = acc[i];
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) upd<ADAM>(a, gr[j], w1[q][j], m1[q][j], v1[q][j], lr_t, inv_bc2);
          if (more) {
#pragma unroll
            for (int kk = 0; kk < XQ; ++kk) {
              const int idx = kk * 64 + lv;
              const int r = idx >> 2, col = 32 * s + 8 * (idx & 3);
              if (col < D0) *reinterpret_cast<uint4*>(sX + r * LDX + col) = xq[kk];
            }
          }
        }
      }
    }
    if (tid < 16) upd<ADAM>(a, sDb1[tid], sB1[tid], sB1[16 + tid], sB1[32 + tid], lr_t, inv_bc2);
    __syncthreads();  // sDH1 / sB1 reads done; sW2g complete
    if (g == 0) PE_STAMP(0, t, 4);
    // updated W2 slice to the head (write-through) and the next batch into LDS; one drain + flag
    w2_store(tv);
    publish(pb.flags, p, F_W2 + g, (unsigned)(t + 2), pb.plain);
    if (g == 0) PE_STAMP(0, t, 5);
  }

  // ---- write the state back (fp32 master, moments, bf16 shadow). The row / peer offsets are
  //      laundered through empty asm so the compiler re-derives these addresses here instead of
  //      keeping the prologue's ~70 VGPRs of 64-bit addresses alive across the whole step loop.
  int orow_w = orow;
  int64_t pS_w = pS;
  asm volatile("" : "+v"(orow_w), "+s"(pS_w));
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int s = wave + 8 * q;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int k = 32 * s + 16 * half + 4 * h;
      if (s < KS1 && k < D0) {
        const int64_t idx = pS_w + a.off_w1 + (int64_t)orow_w * D0 + k;
        const int j0 = 4 * half;
        *reinterpret_cast<float4*>(a.params + idx) = float4{w1[q][j0], w1[q][j0 + 1], w1[q][j0 + 2], w1[q][j0 + 3]};
        *reinterpret_cast<float4*>(a.m + idx) = float4{m1[q][j0], m1[q][j0 + 1], m1[q][j0 + 2], m1[q][j0 + 3]};
        if (adam) *reinterpret_cast<float4*>(a.v + idx) = float4{v1[q][j0], v1[q][j0 + 1], v1[q][j0 + 2], v1[q][j0 + 3]};
        bf16x4 sh;
#pragma unroll
        for (int i = 0; i < 4; ++i) sh[i] = (bf16)w1[q][j0 + i];
        *reinterpret_cast<bf16x4*>(a.shadow + idx) = sh;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int o2 = 16 * wave + 4 * h + j;
    const int64_t idx = pS_w + a.off_w2 + (int64_t)o2 * PD1 + orow_w;
    a.params[idx] = w2[j];
    a.m[idx] = m2[j];
    if (adam) a.v[idx] = v2[j];
    a.shadow[idx] = (bf16)w2[j];
    a.w2t[(int64_t)p * PD1 * PD2 + (int64_t)orow_w * PD2 + o2] = (bf16)w2[j];
  }
  if (tid < 16) {
    const int64_t idx = pS_w + a.off_b1 + NG * g + tid;
    a.params[idx] = sB1[tid];
    a.m[idx] = sB1[16 + tid];
    if (adam) a.v[idx] = sB1[32 + tid];
    a.shadow[idx] = (bf16)sB1[tid];
  }
}

// =============================================================================================
// head workgroup
// =============================================================================================
template <int BP, bool ADAM>
__device__ void head(const MLPArgs& a, const MLPPersistBufs& pb, int p, char* smem) {
  constexpr int MT = BP / 16;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 4, c = lane & 15;
  const int D3 = a.D3;
  const HeadLds L = head_lds(BP);
  bf16* sH1 = reinterpret_cast<bf16*>(smem + L.h1);
  bf16* sDH2 = sH1;  // dH2 staging reuses the H1 tile (H1 is dead after the H2 GEMM)
  bf16* sH2 = reinterpret_cast<bf16*>(smem + L.h2);
  bf16* sDlog = reinterpret_cast<bf16*>(smem + L.dlog);
  bf16* sW3 = reinterpret_cast<bf16*>(smem + L.w3);
  float* sB2 = reinterpret_cast<float*>(smem + L.b2);  // [3][128]
  float* sB3 = reinterpret_cast<float*>(smem + L.b3);  // [3][16]
  int* sOk = reinterpret_cast<int*>(smem + L.ok);

  const int4 ctl = a.ctl[p];
  const bool fresh = (ctl.x & 2) != 0;  // fresh optimizer state this fit: moments start at 0
  const int n = ctl.y;
  const int nsteps = (n + a.B - 1) / a.B;
  const int64_t pS = (int64_t)p * a.S;
  constexpr bool adam = ADAM;
  const bool cin = c < D3;

  // resident W3 (waves 0..3, wave w owns o2 32w..32w+31), biases in LDS
  float w3[8], m3[8], v3[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    w3[j] = m3[j] = v3[j] = 0.f;
    if (wave < 4 && cin) {
      const int64_t idx = pS + a.off_w3 + (int64_t)c * PD2 + 32 * wave + kappa(h, j);
      w3[j] = a.params[idx];
      m3[j] = fresh ? 0.f : a.m[idx];
      if (adam) v3[j] = fresh ? 0.f : a.v[idx];
    }
  }
  for (int e = tid; e < 32 * LDW3; e += NT) sW3[e] = (bf16)0.f;
  for (int e = tid; e < BP * LDL; e += NT) sDlog[e] = (bf16)0.f;
  if (tid < PD2) {
    const int64_t idx = pS + a.off_b2 + tid;
    sB2[tid] = a.params[idx];
    sB2[PD2 + tid] = fresh ? 0.f : a.m[idx];
    sB2[2 * PD2 + tid] = (adam && !fresh) ? a.v[idx] : 0.f;
  } else if (tid < PD2 + 16) {
    const int k = tid - PD2;
    const int64_t idx = pS + a.off_b3 + k;
    sB3[k] = k < D3 ? a.params[idx] : 0.f;
    sB3[16 + k] = (k < D3 && !fresh) ? a.m[idx] : 0.f;
    sB3[32 + k] = (k < D3 && adam && !fresh) ? a.v[idx] : 0.f;
  }
  __syncthreads();
  if (wave < 4 && cin) {
#pragma unroll
    for (int j = 0; j < 8; ++j) sW3[c * LDW3 + 32 * wave + kappa(h, j)] = (bf16)w3[j];
  }
  float loss_acc = 0.f, correct_acc = 0.f;

  for (int t = 0; t < nsteps; ++t) {
    int tv = tid;  // opaque per-iteration thread index (see owner)
    asm volatile("" : "+v"(tv));
    const int rows = rows_at(a, n, t);
    float lr_t, inv_bc2;
    bias_corr(a, ctl.z, t, lr_t, inv_bc2);

    // ---- W2 (bf16, version t+1) and H1 (step t) from the owners
    PE_STAMP(1, t, 0);
    if (!wg_wait(pb.flags, p, F_W2, NG, (unsigned)(t + 1), pb.err, sOk)) return;
    PE_STAMP(1, t, 1);
    // W2 (bf16) goes straight into this wave's B fragments — rows 16w..16w+15 of W2, all 256
    // inputs (32 VGPRs): it lands well before H1 (the owners publish it ahead of their forward)
    // and never touches LDS
    bf16x8 w2f[PD1 / 32];
    {
      const bf16* wfrag = pb.w2x + (((int64_t)p * 8 + wave) * (PD1 / 32) * 64 + lane) * 8;
#pragma unroll
      for (int ks = 0; ks < PD1 / 32; ++ks) {
        const unsigned long long lo = ld_wt(wfrag + ks * 64 * 8), hi = ld_wt(wfrag + ks * 64 * 8 + 4);
        w2f[ks] = __builtin_bit_cast(bf16x8, (unsigned long long __attribute__((ext_vector_type(2)))){lo, hi});
      }
    }
    if (!wg_wait(pb.flags, p, F_H1, NG, (unsigned)(t + 1), pb.err, sOk)) return;
    PE_STAMP(1, t, 2);
    {
      unsigned long long h1r[BP / 8];
#pragma unroll
      for (int k = 0; k < BP / 8; ++k) {  // BP x 256 bf16 = BP*64 chunks
        const int e = tv + NT * k;
        h1r[k] = ld_wt(pb.h1x + (int64_t)p * BP * PD1 + (int64_t)e * 4);
      }
#pragma unroll
      for (int k = 0; k < BP / 8; ++k) {
        const int e = tv + NT * k;
        *reinterpret_cast<unsigned long long*>(sH1 + (e >> 6) * LDH + 4 * (e & 63)) = h1r[k];
      }
    }
    lds_barrier();

    // ---- H2 = relu(H1 · W2ᵀ + b2): wave w owns output columns 16w..16w+15
    {
      f32x4 acc[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt] = zero4();
#pragma unroll
      for (int ks = 0; ks < PD1 / 32; ++ks) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[mt] = mfma_bf16(ld8(sH1 + (16 * mt + c) * LDH + 32 * ks + 8 * h), w2f[ks], acc[mt]);
      }
      const int o2 = 16 * wave + c;
      const float bias = sB2[o2];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int b = 16 * mt + 4 * h + i;
          sH2[b * LD2 + o2] = (bf16)(b < rows ? fmaxf(acc[mt][i] + bias, 0.f) : 0.f);
        }
    }
    lds_barrier();
    PE_STAMP(1, t, 3);
    // ---- logits + log-softmax + NLL + argmax + dlogits: wave w < MT owns batch rows 16w..16w+15
    //      and all 128 inputs (4 chained MFMAs, W3 bf16 from LDS, before this step's update), so
    //      the row statistics need no cross-wave reduction
    if (wave < MT) {
      f32x4 lg = zero4();
#pragma unroll
      for (int ks = 0; ks < PD2 / 32; ++ks)
        lg = mfma_bf16(ld8(sH2 + (16 * wave + c) * LD2 + 32 * ks + 8 * h), ld8(sW3 + c * LDW3 + 32 * ks + 8 * h), lg);
      const float b3 = sB3[c];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int b = 16 * wave + 4 * h + i;
        const bool rvalid = b < rows;
        const int y = rvalid ? a.Yb[(int64_t)p * a.xb_rows + (int64_t)t * a.B + b] : -1;
        const float logit = cin ? lg[i] + b3 : -INFINITY;
        const float mx = row_max16(logit);
        const float se = row_sum16(cin ? __expf(logit - mx) : 0.f);
        const float logp = logit - (mx + __logf(se));
        const int cand = row_min16((cin && logit == mx) ? c : 16);
        if (rvalid && c == y) loss_acc -= logp;
        if (rvalid && c == 0) correct_acc += (cand == y) ? 1.f : 0.f;
        const float d = (rvalid && cin) ? (__expf(logp) - (c == y ? 1.f : 0.f)) / (float)rows : 0.f;
        sDlog[b * LDL + c] = (bf16)d;
      }
    }
    lds_barrier();
    PE_STAMP(1, t, 4);
    // ---- dH2 = dlogits · W3 ⊙ [H2 > 0] (wave w: columns 16w..16w+15; K = classes padded to 32)
    {
      const bf16x8 bw = frag_b_tr(sW3, LDW3, 0, 16 * wave);
      const int o2 = 16 * wave + c;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const f32x4 acc = mfma_bf16(ld8(sDlog + (16 * mt + c) * LDL + 8 * h), bw, zero4());
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int b = 16 * mt + 4 * h + i;
          sDH2[b * LD2 + o2] = (bf16)((float)sH2[b * LD2 + o2] > 0.f ? acc[i] : 0.f);
        }
      }
    }
    lds_barrier();
#pragma unroll
    for (int k = 0; k < BP / 16; ++k) {  // row-wise 8-byte chunks: whole 256-byte rows per wave
      const int e = tv + NT * k;
      const int b = e >> 5, q = e & 31;
      pub64(pb.plain, pb.dh2x + ((int64_t)p * BP + b) * PD2 + 4 * q, *reinterpret_cast<const unsigned long long*>(sDH2 + b * LD2 + 4 * q));
    }
    publish(pb.flags, p, F_DH2, (unsigned)(t + 1), pb.plain);
    PE_STAMP(1, t, 5);

    // ---- off the critical path: dW3 (waves 0..3), db2 (waves 4,5), db3 (wave 6)
    if (wave < 4) {
      float gr[8];
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        f32x4 acc = zero4();
#pragma unroll
        for (int kb = 0; kb < BP / 32; ++kb)
          acc = mfma_bf16(frag_b_tr(sH2, LD2, 32 * kb, 32 * wave + 16 * tt), frag_b_tr(sDlog, LDL, 32 * kb, 0), acc);
#pragma unroll
        for (int i = 0; i < 4; ++i) gr[4 * tt + i] = acc[i];
      }
      if (cin) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          upd<ADAM>(a, gr[j], w3[j], m3[j], v3[j], lr_t, inv_bc2);
          sW3[c * LDW3 + 32 * wave + kappa(h, j)] = (bf16)w3[j];
        }
      }
    } else if (wave < 6) {
      const int o2 = tid - 256;
      float db = 0.f;
      for (int b = 0; b < BP; ++b) db += (float)sDH2[b * LD2 + o2];
      upd<ADAM>(a, db, sB2[o2], sB2[PD2 + o2], sB2[2 * PD2 + o2], lr_t, inv_bc2);
    } else if (wave == 6 && lane < D3) {
      float db = 0.f;
      for (int b = 0; b < BP; ++b) db += (float)sDlog[b * LDL + lane];
      upd<ADAM>(a, db, sB3[lane], sB3[16 + lane], sB3[32 + lane], lr_t, inv_bc2);
    }
    __syncthreads();
    PE_STAMP(1, t, 6);
  }

  // ---- write back W3 / b2 / b3 and the epoch's loss / accuracy sums
  if (wave < 4 && cin) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int64_t idx = pS + a.off_w3 + (int64_t)c * PD2 + 32 * wave + kappa(h, j);
      a.params[idx] = w3[j];
      a.m[idx] = m3[j];
      if (adam) a.v[idx] = v3[j];
      a.shadow[idx] = (bf16)w3[j];
    }
  }
  if (tid < PD2) {
    const int64_t idx = pS + a.off_b2 + tid;
    a.params[idx] = sB2[tid];
    a.m[idx] = sB2[PD2 + tid];
    if (adam) a.v[idx] = sB2[2 * PD2 + tid];
    a.shadow[idx] = (bf16)sB2[tid];
  } else if (tid < PD2 + 16 && tid - PD2 < D3) {
    const int k = tid - PD2;
    const int64_t idx = pS + a.off_b3 + k;
    a.params[idx] = sB3[k];
    a.m[idx] = sB3[16 + k];
    if (adam) a.v[idx] = sB3[32 + k];
    a.shadow[idx] = (bf16)sB3[k];
  }
  if (wave < MT) {
    const float l = wave_sum(loss_acc), cr = wave_sum(correct_acc);
    if (lane == 0) {
      atomicAdd(&a.loss_acc[p], l);
      atomicAdd(&a.correct_acc[p], (int)(cr + 0.5f));
    }
  }
}

template <int BP, bool ADAM>
__global__ __launch_bounds__(NT) void mlp_persistent_epoch(MLPArgs a, MLPPersistBufs pb) {
  extern __shared__ __attribute__((aligned(16))) char smem_pe[];
  const int b = blockIdx.x;
  const int slot = b & 7, idx = b >> 3;
  const int p = (idx / ROLES) * 8 + slot;
  const int role = idx % ROLES;
  if (p >= a.P) return;
  const int4 ctl = a.ctl[p];
  if (!ctl.x || ctl.y <= 0) return;
  // a peer's blocks share b & 7: one XCD under round-robin dispatch, checked here (speed only)
  pb.plain = pb.plain_ok && persist::gang_same_xcd(persist::flag_at(pb.flags, FLAGS_PER_PEER, p, F_XCC), role, ROLES, 0x100u,
                                                   reinterpret_cast<int*>(smem_pe), 10000ull);
  if (role < NG)
    owner<BP, ADAM>(a, pb, p, role, smem_pe);
  else
    head<BP, ADAM>(a, pb, p, smem_pe);
}

}  // namespace

bool mlp_persistent_supported(const MLPArgs& a) {
  if (a.D1 != PD1 || a.D2 != PD2 || a.D3 < 1 || a.D3 > 16) return false;
  if (a.D0 % 8 != 0 || (a.D0 + 31) / 32 > KS1_MAX) return false;
  if (a.Bpad != 32 && a.Bpad != 64) return false;
  if (a.anchor != nullptr || a.cg != nullptr || a.cl != nullptr) return false;
  if (a.opt.kind == 1 && a.opt.momentum != 0.f) return false;  // SGD momentum buffer: 3-launch path
  const size_t lds = owner_lds(a.Bpad, a.D0).total > head_lds(a.Bpad).total ? owner_lds(a.Bpad, a.D0).total : head_lds(a.Bpad).total;
  return lds <= 160 * 1024;
}

size_t mlp_persistent_bytes(int P, int Bpad) { return (size_t)P * ((size_t)Bpad * PD1 + (size_t)PD2 * PD1 + (size_t)Bpad * PD2) * sizeof(bf16); }
size_t mlp_persistent_flag_bytes(int P) { return (size_t)P * FLAGS_PER_PEER * persist::FLAG_LINE * sizeof(unsigned); }
int mlp_persistent_blocks(int P) { return 8 * ROLES * ((P + 7) / 8); }

static size_t persistent_lds(const MLPArgs& a) {
  const size_t lo = owner_lds(a.Bpad, a.D0).total, lh = head_lds(a.Bpad).total;
  return lo > lh ? lo : lh;
}

template <int BP, bool ADAM>
static hipError_t prepare_one(int lds) {
  return hipFuncSetAttribute((const void*)mlp_persistent_epoch<BP, ADAM>, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
}

hipError_t mlp_persistent_prepare(const MLPArgs& a) {
  const int lds = (int)persistent_lds(a);
  hipError_t e = a.Bpad == 64 ? prepare_one<64, true>(lds) : prepare_one<32, true>(lds);
  if (e != hipSuccess) return e;
  return a.Bpad == 64 ? prepare_one<64, false>(lds) : prepare_one<32, false>(lds);
}

hipError_t mlp_launch_persistent_epoch(const MLPArgs& a, const MLPPersistBufs& pb_in, hipStream_t s, bool zero_flags) {
  MLPPersistBufs pb = pb_in;
  pb.plain_ok = mlp_plain_pub_mode() != 0 ? 1 : 0;  // as the fp32 kernels (MYFYP_F32_PLAIN_PUB)
  pb.plain = 0;
  if (zero_flags) {
    hipError_t e = hipMemsetAsync(pb.flags, 0, pb.flag_bytes, s);
    if (e != hipSuccess) return e;
  }
  const size_t lds = persistent_lds(a);
  const dim3 grid(mlp_persistent_blocks(a.P)), block(NT);
  const bool adam = a.opt.kind == 0;
  if (a.Bpad == 64) {
    if (adam)
      hipLaunchKernelGGL((mlp_persistent_epoch<64, true>), grid, block, lds, s, a, pb);
    else
      hipLaunchKernelGGL((mlp_persistent_epoch<64, false>), grid, block, lds, s, a, pb);
  } else {
    if (adam)
      hipLaunchKernelGGL((mlp_persistent_epoch<32, true>), grid, block, lds, s, a, pb);
    else
      hipLaunchKernelGGL((mlp_persistent_epoch<32, false>), grid, block, lds, s, a, pb);
  }
  return hipGetLastError();
}
