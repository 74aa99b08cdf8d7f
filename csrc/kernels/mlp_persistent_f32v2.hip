// fp32 weight-stationary persistent epoch kernel for the reference MLP (784-256-128-10), gang
// layout 2: OWNERS ONLY, two hand-offs per step (mlp_persistent_f32.hip, layout 1, has three).
// Same arithmetic contract as layout 1: exact fp32 products (three-term bf16 split against the
// exact-bf16 uint8 inputs for the two W1 GEMMs, f32-input MFMA everywhere else), fp32
// accumulation, fp32 master weights and optimizer state resident for the whole epoch. It trains
// the reference's step (/root/reference/p2pfl/learning/frameworks/pytorch/lightning_model.py:169-191:
// Linear+ReLU x2, Linear, log_softmax, cross_entropy, torch.optim.Adam at :181-183).
//
// Gang of one peer: NG = 16 workgroups of 512 threads, one per CU. Owner g holds
//   * W1 rows 16g..16g+15 (+ the b1 slice in the bias column) in registers (+ one K step in LDS),
//   * W2 COLUMNS 16g..16g+15 (all 128 rows): the master copy, in the lane layout of its dW2 tile,
//     plus a transposed copy (the B fragments of the H2 partial),
//   * W3 columns 8g..8g+7 (all classes) in LDS; b2 and b3 replicated in every owner (updated from
//     the same full-batch sums in every owner: the copies stay bit-identical).
// Step t (the chain every owner walks):
//   A  H1 slice = relu(X · W1sliceᵀ + b1)                            [as layout 1]
//   B  H2 partial over the slice: P_g = H1slice · W2[:, slice]ᵀ      (64 x 128, K = 16)
//      -> publish P_g (write-through, fragment order) + the owner's W3 columns            HAND-OFF 1
//   R  reducer for batch rows 4g..4g+3: H2 rows = relu(Σ_g' P_g' + b2) in a fixed order, logits
//      with the gathered W3, log-softmax + NLL + argmax, dlogits, dH2 rows = dlogits·W3 ⊙ [H2>0]
//      -> publish dH2 rows, H2 rows, dlogits rows                                           HAND-OFF 2
//   C  full dH2 -> dH1 slice (old W2), dW2 columns + update, db2 / db3 (replicated), the owner's
//      dW3 columns + update, then dW1 rows + update + next batch staged          [C2 as layout 1]
// Layout 1 moves H1 to 8 head workgroups (hand-off 1), exchanges partial logits between the heads
// (hand-off 2) and returns dH2 (hand-off 3). Here the only cross-CU traffic is the H2 partial
// all-to-all (32 KB out, 32 KB in per owner) and the row all-gather (2-4 KB out, 38 KB in).
//
// Hand-offs as layout 1 (persist_common.h): write-through (sc1) stores, drain, workgroup meet, one
// relaxed flag store; the consumer polls from one wave and reads with sc1 loads. Buffers are
// double-buffered by step parity: an owner writes parity (t & 1) of step t + 2 only after every
// owner published step t + 1's F2, i.e. after every reader of step t finished with it.
#include "mlp_f32_common.h"
#include "mlp_persistent.h"

#ifdef MLP_STAMPS
__device__ unsigned long long g_p32v2_stamps[32][16];
#define V2_STAMP(t, i)                                                                         \
  do {                                                                                         \
    if (p == 0 && g == 0 && threadIdx.x == 0 && (t) < 32) g_p32v2_stamps[t][i] = wall_clock64(); \
  } while (0)
extern "C" int mlp_debug_persistent_f32v2_stamps(void* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_p32v2_stamps), sizeof(g_p32v2_stamps)) == hipSuccess ? 0 : 1;
}
#else
#define V2_STAMP(t, i) \
  do {                 \
  } while (0)
#endif

namespace {

using namespace f32k;
using persist::al16;
using persist::row_max16;
using persist::row_min16;
using persist::row_sum16;

constexpr int NG = 16;  // owners per peer = the gang
constexpr int PPL = 8;  // peers per launch (8 x 16 workgroups)
constexpr int F1 = 0, F2 = NG, FDONE = 2 * NG;  // flag lines of a peer (within the shared F32_FPP block)
constexpr int RQ = 3;                           // register-resident W1 K steps per wave (K step 24 in LDS)
constexpr int W3LD = PD2 + 4;                   // fp32 row stride of the gathered W3 [16][128]
constexpr int DW3P = (PD2 + 1) * 16;            // floats of one reducer's dW3 partial: [o2][class] + the db3 row

// ---- exchange buffer (floats, from pb.h1x), region-major over peers
struct V2Layout {
  int64_t h2p, w3s, dh2r, dw3p, lossp, total;
};
__host__ __device__ inline V2Layout v2_layout(int P, int BP) {
  V2Layout L;
  int64_t o = 0;
  L.h2p = o;   o += (int64_t)P * 2 * NG * BP * PD2;  // [P][2][g][mt][w][lane][4]: H2 partials in MFMA C order
  L.w3s = o;   o += (int64_t)P * 2 * NG * 16 * 8;    // [P][2][g][class][8]: W3 columns 8g..8g+7
  L.dh2r = o;  o += (int64_t)P * 2 * BP * PD2;       // [P][2][BP][128]: dH2 rows
  L.dw3p = o;  o += (int64_t)P * 2 * NG * DW3P;      // [P][2][reducer][129][16]: dW3ᵀ partial over its rows + db3 partial
  L.lossp = o; o += (int64_t)P * NG * 8;             // [P][g][reducer row][2]: epoch loss / correct partials
  L.total = o;
  return L;
}

struct OwnerLdsV2 {
  int ldx, ldt;
  size_t x, red, h1, dh1s, w1x, w3st, b2st, b3st, ok, total;
  // reducer scratch, inside red (free between B and C)
  size_t r_part, r_w3, r_h2, r_dl;
};
__host__ __device__ inline OwnerLdsV2 owner_lds_v2(int BP, int D0) {
  OwnerLdsV2 L;
  L.ldx = ks1_of(D0) * 32 + 8;
  L.ldt = BP + 8;
  const int MT = BP / 16;
  const size_t red = (size_t)8 * MT * 64 * 16, dh2 = (size_t)BP * LDD * 4;
  L.r_part = 0;
  L.r_w3 = L.r_part + (size_t)4 * 128 * 16;
  L.r_h2 = L.r_w3 + (size_t)16 * W3LD * 4;
  L.r_dl = L.r_h2 + (size_t)(BP / NG) * PD2 * 4;
  const size_t rsc = L.r_dl + (size_t)(BP / NG) * 16 * 4;
  size_t o = 0, rr = red > dh2 ? red : dh2;
  rr = rr > rsc ? rr : rsc;
  L.x = o;    o += al16((size_t)BP * L.ldx * 2);
  L.red = o;  o += al16(rr);                          // cross-wave partials / dH2 tile / reducer scratch
  L.h1 = o;   o += al16((size_t)BP * LD16 * 4);        // own H1 slice [BP][16] (stride LD16)
  L.dh1s = o; o += al16((size_t)3 * 16 * L.ldt * 2);  // dH1ᵀ as hi / mid / lo bf16 (exact split)
  L.w1x = o;  o += al16((size_t)4 * 16 * 32 * 4);     // W1 state of K step 24 (w, m, v, e)
  L.w3st = o; o += al16((size_t)4 * 16 * 8 * 4);      // W3 columns 8g..8g+7: w, m, v, e [4][class][8]
  L.b2st = o; o += al16((size_t)4 * PD2 * 4);         // b2 (replicated): w, m, v, e
  L.b3st = o; o += al16((size_t)4 * 16 * 4);          // b3 (replicated): w, m, v, e
  L.ok = o;   o += 16;
  L.total = o;
  return L;
}

// Gang commit (as layout 1): no owner stores state before every owner finished every step.
__device__ __forceinline__ bool gang_commit_v2(const MLPArgs& a, const MLPPersistF32Bufs& pb, int p, int g, int* sOk) {
  if (pb.fbase == 0 && g == 0 && a.debug_giveup == p + 1 + 256) {
    if (threadIdx.x == 0) __hip_atomic_store(pb.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return false;
  }
  persist::publish(pb.flags, F32_FPP, p, FDONE + g, pb.fbase + DONE_MARK);
  return persist::wg_wait(pb.flags, F32_FPP, p, FDONE, NG, pb.fbase + DONE_MARK, pb.err, sOk);
}

// Transposed copy of the W2 columns: from the master layout w2c[i] = W2[16w + 4h + i][16g + c]
// (lane (h, c)) to the B fragments of the H2 partial, w2f[ks] = W2[16w + c][16g + 4h + ks].
// Lane (h, c) takes register (c & 3) of lane 16 (c >> 2) + 4h + ks: four cross-lane reads per ks.
__device__ __forceinline__ void w2_transpose(const float (&w2c)[4], float (&w2f)[4], int lane) {
  const int h = lane >> 4, c = lane & 15;
  const int sel = c & 3;
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const int src = (16 * (c >> 2) + 4 * h + ks) * 4;
    const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src, __builtin_bit_cast(int, w2c[0])));
    const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src, __builtin_bit_cast(int, w2c[1])));
    const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src, __builtin_bit_cast(int, w2c[2])));
    const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src, __builtin_bit_cast(int, w2c[3])));
    w2f[ks] = sel == 0 ? r0 : (sel == 1 ? r1 : (sel == 2 ? r2 : r3));
  }
}

template <int BP, bool ADAM, bool EXTRA>
__device__ void owner_v2(const MLPArgs& a, const MLPPersistF32Bufs& pb, int p, int g, char* smem) {
  constexpr int MT = BP / 16;
  constexpr int RPO = BP / NG;  // batch rows this owner reduces (4 at BP = 64, 2 at BP = 32)
  constexpr int XPT = BP / 4;   // 16-byte X chunks per lane: 4 K steps x BP rows x 4 chunks / 64 lanes
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int h = lane >> 4, c = lane & 15;
  const int D0 = a.D0, D3 = a.D3;
  const int KS1 = ks1_of(D0);
  const OwnerLdsV2 L = owner_lds_v2(BP, D0);
  const int LDX = L.ldx, LDT = L.ldt;
  bf16* sX = reinterpret_cast<bf16*>(smem + L.x);
  f32x4* sRed = reinterpret_cast<f32x4*>(smem + L.red);
  float* sDH2 = reinterpret_cast<float*>(smem + L.red);
  f32x4* sPart = reinterpret_cast<f32x4*>(smem + L.red + L.r_part);
  float* sW3 = reinterpret_cast<float*>(smem + L.red + L.r_w3);
  float* sH2r = reinterpret_cast<float*>(smem + L.red + L.r_h2);
  float* sDl = reinterpret_cast<float*>(smem + L.red + L.r_dl);
  float* sH1 = reinterpret_cast<float*>(smem + L.h1);
  bf16* sD3 = reinterpret_cast<bf16*>(smem + L.dh1s);
  float* sW1x = reinterpret_cast<float*>(smem + L.w1x);
  float* sW3s = reinterpret_cast<float*>(smem + L.w3st);  // [w, m, v, e][class][8]
  float* sB2 = reinterpret_cast<float*>(smem + L.b2st);   // [w, m, v, e][128]
  float* sB3 = reinterpret_cast<float*>(smem + L.b3st);   // [w, m, v, e][16]
  int* sOk = reinterpret_cast<int*>(smem + L.ok);

  const OptParams& o = a.opt;
  const int4 ctl = a.ctl[p];
  const bool fresh = (ctl.x & 2) != 0;
  const int n = ctl.y;
  const int nsteps = (n + a.B - 1) / a.B;
  const int64_t pS = (int64_t)p * a.S;
  const float wdmu = o.weight_decay + (a.anchor != nullptr ? o.mu : 0.f);
  const V2Layout XL = v2_layout(a.P, BP);
  float* const xbase = pb.h1x;
  const int R0 = RPO * g;  // first batch row reduced by this owner
  const int mt_r = R0 >> 4, h_r = (R0 & 15) >> 2, i0_r = R0 & 3;

  // ---- resident W1 rows (as layout 1, KS = 1): wave w owns K steps w, w+8, w+16 (registers) and
  //      24 (LDS, wave 0), κ slot order; the slot of column D0 holds b1
  float w1[RQ][8], m1[RQ][8], v1[RQ][8], e1[RQ][8];
  const int orow = 16 * g + c;
#pragma unroll
  for (int q = 0; q < RQ + 1; ++q) {
    const int s = wave + 8 * q;
    if (q == RQ && s >= KS1) break;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int k = 32 * s + 16 * half + 4 * h;
      float4 wv = {0.f, 0.f, 0.f, 0.f}, mv = wv, vv = wv, ev = wv;
      if (s < KS1 && k < D0) {
        const int64_t idx = pS + a.off_w1 + (int64_t)orow * D0 + k;
        wv = *reinterpret_cast<const float4*>(a.params + idx);
        if (!fresh) {
          mv = *reinterpret_cast<const float4*>(a.m + idx);
          if (ADAM) vv = *reinterpret_cast<const float4*>(a.v + idx);
        }
        if (EXTRA) ev = float4{extra_at(a, idx), extra_at(a, idx + 1), extra_at(a, idx + 2), extra_at(a, idx + 3)};
      } else if (s < KS1 && k == D0) {
        const int64_t idx = pS + a.off_b1 + orow;
        wv.x = a.params[idx];
        if (!fresh) {
          mv.x = a.m[idx];
          if (ADAM) vv.x = a.v[idx];
        }
        if (EXTRA) ev.x = extra_at(a, idx);
      }
      if (q < RQ) {
        const float wa[4] = {wv.x, wv.y, wv.z, wv.w}, ma[4] = {mv.x, mv.y, mv.z, mv.w}, va[4] = {vv.x, vv.y, vv.z, vv.w},
                    ea[4] = {ev.x, ev.y, ev.z, ev.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          w1[q][4 * half + i] = wa[i];
          m1[q][4 * half + i] = ma[i];
          v1[q][4 * half + i] = va[i];
          e1[q][4 * half + i] = ea[i];
        }
      } else {
        const int off = c * 32 + 16 * half + 4 * h;
        *reinterpret_cast<float4*>(sW1x + off) = wv;
        *reinterpret_cast<float4*>(sW1x + 512 + off) = mv;
        *reinterpret_cast<float4*>(sW1x + 1024 + off) = vv;
        *reinterpret_cast<float4*>(sW1x + 1536 + off) = ev;
      }
    }
  }
  // ---- W2 columns 16g..16g+15 (master): wave w holds W2[16w + 4h + i][16g + c]
  float w2c[4], m2c[4], v2c[4], e2c[4], w2f[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t idx = pS + a.off_w2 + (int64_t)(16 * wave + 4 * h + i) * PD1 + 16 * g + c;
    w2c[i] = a.params[idx];
    m2c[i] = fresh ? 0.f : a.m[idx];
    v2c[i] = (ADAM && !fresh) ? a.v[idx] : 0.f;
    e2c[i] = EXTRA ? extra_at(a, idx) : 0.f;
  }
  w2_transpose(w2c, w2f, lane);
  // ---- W3 columns 8g..8g+7, b2, b3 -> LDS state
  if (tid < 128) {
    const int cls = tid >> 3, j = tid & 7;
    const bool in = cls < D3;
    const int64_t idx = pS + a.off_w3 + (int64_t)cls * PD2 + 8 * g + j;
    sW3s[tid] = in ? a.params[idx] : 0.f;
    sW3s[128 + tid] = (in && !fresh) ? a.m[idx] : 0.f;
    sW3s[256 + tid] = (in && ADAM && !fresh) ? a.v[idx] : 0.f;
    sW3s[384 + tid] = (in && EXTRA) ? extra_at(a, idx) : 0.f;
  } else if (tid < 256) {
    const int k = tid - 128;
    const int64_t idx = pS + a.off_b2 + k;
    sB2[k] = a.params[idx];
    sB2[128 + k] = fresh ? 0.f : a.m[idx];
    sB2[256 + k] = (ADAM && !fresh) ? a.v[idx] : 0.f;
    sB2[384 + k] = EXTRA ? extra_at(a, idx) : 0.f;
  } else if (tid < 272) {
    const int k = tid - 256;
    const bool in = k < D3;
    const int64_t idx = pS + a.off_b3 + k;
    sB3[k] = in ? a.params[idx] : 0.f;
    sB3[16 + k] = (in && !fresh) ? a.m[idx] : 0.f;
    sB3[32 + k] = (in && ADAM && !fresh) ? a.v[idx] : 0.f;
    sB3[48 + k] = (in && EXTRA) ? extra_at(a, idx) : 0.f;
  }

  // ---- X staging (as layout 1): each wave stages its own K-step columns; the chunk at column D0
  //      carries the bias input (1 for valid rows)
  auto bias_chunk = [](bool valid) { return uint4{valid ? 0x3F80u : 0u, 0u, 0u, 0u}; };  // bf16 1.0
  auto xw_stage = [&](int t, int lv) {
    const int rows = rows_at(a, n, t);
#pragma unroll
    for (int k = 0; k < XPT; ++k) {
      const int q = k / (BP / 16), kk = k % (BP / 16);
      if (q > RQ) break;
      const int s = wave + 8 * q;
      const int idx = kk * 64 + lv;
      const int r = idx >> 2, col = 32 * s + 8 * (idx & 3);
      if (s < KS1 && col < D0) {
        const bf16* src = a.Xb16 + ((int64_t)p * a.xb_rows + (int64_t)t * a.B + r) * D0 + col;
        *reinterpret_cast<uint4*>(sX + r * LDX + col) = r < rows ? *reinterpret_cast<const uint4*>(src) : uint4{0u, 0u, 0u, 0u};
      } else if (s < KS1 && col == D0) {
        *reinterpret_cast<uint4*>(sX + r * LDX + col) = bias_chunk(r < rows);
      }
    }
  };
  {  // columns past D0 (the bias column's K step) are zero for the whole epoch
    const int z0 = D0, z1 = KS1 * 32;
    for (int e = tid; e < BP * (z1 - z0); e += NT) {
      const int r = e / (z1 - z0), q = e % (z1 - z0);
      sX[r * LDX + z0 + q] = (bf16)0.f;
    }
  }
  if (nsteps > 0) xw_stage(0, lane);

  auto fwd_kstep = [&](int q, f32x4(&acc)[MT]) {
    const int s = wave + 8 * q;
    if (s >= KS1) return;
    int lq = lane;
    asm volatile("" : "+v"(lq));
    const int hq = lq >> 4, cq = lq & 15;
    float wq[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) wq[j] = q < RQ ? w1[q < RQ ? q : 0][j] : sW1x[cq * 32 + kappa(hq, j)];
    bf16x8 bh, bm, bl;
    split3(wq, bh, bm, bl);
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      const bf16* xp = sX + (16 * mt + cq) * LDX + 32 * s + 4 * hq;
      const bf16x8 af = cat8(*reinterpret_cast<const bf16x4*>(xp), *reinterpret_cast<const bf16x4*>(xp + 16));
      acc[mt] = mfma3(af, bh, bm, bl, acc[mt]);
    }
  };
  if (tid == 0) sOk[1] = 1;
  __syncthreads();  // LDS state written

  persist::BiasCorr bc;
  bc.init(o, ctl.z);
  float lr_t = 0.f, inv_bc2 = 0.f;
  float loss_acc = 0.f, correct_acc = 0.f;
  for (int t = 0; t < nsteps; ++t) {
    int tv = tid;
    asm volatile("" : "+v"(tv));
    const int rows = rows_at(a, n, t);
    const int par = t & 1;
    const unsigned target = pb.fbase + (unsigned)(t + 1);
    bc.next(o, lr_t, inv_bc2);
    V2_STAMP(t, 0);
    // labels of the reducer rows (wave i < RPO: row R0 + i), loaded early
    int yv = -1;
    if (wave < RPO && R0 + wave < rows) yv = a.Yb[(int64_t)p * a.xb_rows + (int64_t)t * a.B + R0 + wave];

    // ================= A: H1 slice = relu(X · W1sliceᵀ + b1), split-K over the 8 waves
    {
      f32x4 acc[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) acc[mt] = zero4();
#pragma unroll
      for (int q = 0; q < RQ + 1; ++q) {
        fwd_kstep(q, acc);
        __builtin_amdgcn_sched_barrier(0);
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
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int b = 16 * mt + 4 * hh + i;
        sH1[b * LD16 + cc] = b < rows ? fmaxf(s[i], 0.f) : 0.f;
      }
    }
    lds_barrier();
    V2_STAMP(t, 1);

    // ================= B: H2 partial of this slice, P_g[b][o2 = 16w + c] (K = the 16 slice columns,
    //                  k order 4h + ks), stored in MFMA C order: [mt][w][lane][4 rows]
    {
      float* dst = xbase + XL.h2p + (((int64_t)p * 2 + par) * NG + g) * BP * PD2;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const float4 av = *reinterpret_cast<const float4*>(sH1 + (16 * mt + c) * LD16 + 4 * h);
        f32x4 acc = mfma_f32(av.x, w2f[0], zero4());
        acc = mfma_f32(av.y, w2f[1], acc);
        acc = mfma_f32(av.z, w2f[2], acc);
        acc = mfma_f32(av.w, w2f[3], acc);
        persist::pub128(pb.plain, dst, BP * PD2 * 4, ((mt * 8 + wave) * 64 + lane) * 16, __builtin_bit_cast(u32x4, acc));
      }
      if (tid < 32) {  // this owner's W3 columns (current weights) for every reducer's logits
        float* w3d = xbase + XL.w3s + (((int64_t)p * 2 + par) * NG + g) * 128;
        persist::pub128(pb.plain, w3d, 128 * 4, tid * 16, __builtin_bit_cast(u32x4, *reinterpret_cast<const float4*>(sW3s + 4 * tid)));
      }
    }
    persist::publish_p(pb.flags, F32_FPP, p, F1 + g, target, pb.plain);
    V2_STAMP(t, 2);

    // next step's batch: pull this wave's columns into the XCD's L2 (staged during C2)
    const bool more = t + 1 < nsteps;
    if (more) {
      const int rows_n = rows_at(a, n, t + 1);
      unsigned sink = 0;
#pragma unroll
      for (int q = 0; q < RQ + 1; ++q) {
        const int s = wave + 8 * q;
        if (s < KS1 && 32 * s < D0 && lane < rows_n && lane < BP)
          sink ^= *reinterpret_cast<const unsigned*>(a.Xb16 + ((int64_t)p * a.xb_rows + (int64_t)(t + 1) * a.B + lane) * D0 + 32 * s);
      }
      asm volatile("" ::"v"(sink));
    }

    // ================= R: reducer of rows R0..R0+RPO-1
    if (!persist::wg_wait(pb.flags, F32_FPP, p, F1, NG, target, pb.err, sOk)) return;
    V2_STAMP(t, 3);
    {
      const int q = tv & 127, pg = tv >> 7;  // chunk (w = q >> 4, cc = q & 15), producer group
      const int64_t pbase = XL.h2p + ((int64_t)p * 2 + par) * NG * BP * PD2;
      const __amdgpu_buffer_rsrc_t rp = rsrc_of(xbase + pbase, NG * BP * PD2 * 4);
      const int coff = ((mt_r * 8 + (q >> 4)) * 64 + 16 * h_r + (q & 15)) * 16;
      float4 v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = ld_sc1_16(rp, (4 * pg + j) * BP * PD2 * 4 + coff);
      const __amdgpu_buffer_rsrc_t rw = rsrc_of(xbase + XL.w3s + ((int64_t)p * 2 + par) * NG * 128, NG * 128 * 4);
      const float4 wv = ld_sc1_16(rw, tv * 16);  // producer tv >> 5, class (tv & 31) >> 1, columns 4 (tv & 1)..
      float4 s4 = v[0];
#pragma unroll
      for (int j = 1; j < 4; ++j) {
        s4.x += v[j].x;
        s4.y += v[j].y;
        s4.z += v[j].z;
        s4.w += v[j].w;
      }
      sPart[pg * 128 + q] = f32x4{s4.x, s4.y, s4.z, s4.w};
      *reinterpret_cast<float4*>(sW3 + ((tv & 31) >> 1) * W3LD + 8 * (tv >> 5) + 4 * (tv & 1)) = wv;
    }
    lds_barrier();
    V2_STAMP(t, 11);
    if (tv < 128) {  // fixed-order sum of the four producer groups, + b2, relu
      f32x4 s = sPart[tv];
#pragma unroll
      for (int pg = 1; pg < 4; ++pg) s += sPart[pg * 128 + tv];
      const float b2v = sB2[tv];
#pragma unroll
      for (int i = 0; i < RPO; ++i) sH2r[i * PD2 + tv] = R0 + i < rows ? fmaxf(s[i0_r + i] + b2v, 0.f) : 0.f;
    }
    lds_barrier();
    V2_STAMP(t, 12);
    if (wave < RPO) {  // row R0 + wave: logits (lane: class c, part h of 32 o2), softmax, NLL, dlogits
      const int i = wave, b = R0 + i;
      const bool cin = c < D3;
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float4 hv = *reinterpret_cast<const float4*>(sH2r + i * PD2 + 32 * h + 4 * k);
        const float4 wv = *reinterpret_cast<const float4*>(sW3 + c * W3LD + 32 * h + 4 * k);
        acc = fmaf(hv.x, wv.x, acc);
        acc = fmaf(hv.y, wv.y, acc);
        acc = fmaf(hv.z, wv.z, acc);
        acc = fmaf(hv.w, wv.w, acc);
      }
      acc += __shfl_xor(acc, 16);
      acc += __shfl_xor(acc, 32);
      const bool rvalid = b < rows;
      const int y = yv;
      const float logit = cin ? acc + sB3[c] : -INFINITY;
      const float mx = row_max16(logit);
      const float se = row_sum16(cin ? expf(logit - mx) : 0.f);
      const float logp = logit - (mx + logf(se));
      const int cand = row_min16((cin && logit == mx) ? c : 16);
      if (h == 0) {
        if (rvalid && c == y) loss_acc -= logp;
        if (rvalid && c == 0) correct_acc += (cand == y) ? 1.f : 0.f;
      }
      // dlogits: p_c / rows, and −Σ_{c≠y} p_c / rows for the true class (layout 1's stable form)
      const float pc = cin ? expf(logp) : 0.f;
      const float others = row_sum16(c != y ? pc : 0.f);
      if (h == 0) sDl[i * 16 + c] = (rvalid && cin) ? (c == y ? -others : pc) / (float)rows : 0.f;
    }
    lds_barrier();
    V2_STAMP(t, 13);
    {  // dH2 rows = dlogits · W3 ⊙ [H2 > 0], and this reducer's share of dW3 / db3; publish both
      const int i = tv >> 7, o2 = tv & 127;
      const int64_t rbase = ((int64_t)p * 2 + par) * BP;
      if (i < RPO) {
        float acc = 0.f;
        for (int k = 0; k < D3; ++k) acc = fmaf(sDl[i * 16 + k], sW3[k * W3LD + o2], acc);
        const float hv = sH2r[i * PD2 + o2];
        persist::pub32(pb.plain, xbase + XL.dh2r + (rbase + R0 + i) * PD2 + o2, hv > 0.f ? acc : 0.f);
      }
      // dW3ᵀ partial over the reducer rows: one MFMA per wave, A = dlogᵀ[class = c][row = h],
      // B = H2[row = h][o2 = 16w + c] -> C[class 4h + i][o2 16w + c], stored [o2][class]
      float* dst = xbase + XL.dw3p + (((int64_t)p * 2 + par) * NG + g) * DW3P;
      const float av = h < RPO ? sDl[h * 16 + c] : 0.f;
      const float bv = h < RPO ? sH2r[h * PD2 + 16 * wave + c] : 0.f;
      const f32x4 pw = mfma_f32(av, bv, zero4());
      persist::pub128(pb.plain, dst, DW3P * 4, ((16 * wave + c) * 16 + 4 * h) * 4, __builtin_bit_cast(u32x4, pw));
      if (tv < 16) {  // db3 partial: Σ over the reducer rows of dlogits
        float d = 0.f;
#pragma unroll
        for (int r = 0; r < RPO; ++r) d += sDl[r * 16 + tv];
        persist::pub32(pb.plain, dst + PD2 * 16 + tv, d);
      }
    }
    persist::publish_p(pb.flags, F32_FPP, p, F2 + g, target, pb.plain);
    V2_STAMP(t, 4);

    // ================= C: backward of this slice
    if (!persist::wg_wait(pb.flags, F32_FPP, p, F2, NG, target, pb.err, sOk)) return;
    V2_STAMP(t, 5);
    // dW3 columns 8g..8g+7 and db3 from the reducers' partials: lane (row r = tv & 15 of a DPP row)
    // loads reducer r's chunk e = tv >> 4 (o2 = 8g + (e >> 2), classes 4 (e & 3)..+3), the 16 lanes of
    // a row add their chunks (a fixed butterfly: the same bits in every run); tv < 64 do the same
    // for db3 (row 128 of every partial; replicated in every owner)
    float4 w3g, b3g;
    {
      const __amdgpu_buffer_rsrc_t rw = rsrc_of(xbase + XL.dw3p + ((int64_t)p * 2 + par) * NG * DW3P, NG * DW3P * 4);
      const int r = tv & 15, e = tv >> 4;
      w3g = ld_sc1_16(rw, (r * DW3P + (8 * g + (e >> 2)) * 16 + 4 * (e & 3)) * 4);
      b3g = ld_sc1_16(rw, (r * DW3P + PD2 * 16 + 4 * (e & 3)) * 4);
    }
    {
      const __amdgpu_buffer_rsrc_t rd = rsrc_of(xbase + XL.dh2r + ((int64_t)p * 2 + par) * BP * PD2, BP * PD2 * 4);
      float4 v[BP / 16];
#pragma unroll
      for (int k = 0; k < BP / 16; ++k) v[k] = ld_sc1_16(rd, (tv + NT * k) * 16);  // BP x 128 fp32 = BP*32 chunks
#pragma unroll
      for (int k = 0; k < BP / 16; ++k) {
        const int e = tv + NT * k;
        *reinterpret_cast<float4*>(sDH2 + (e >> 5) * LDD + 4 * (e & 31)) = v[k];
      }
    }
    {
      // after the butterfly every lane of the row holds the four sums: lane r < 4 updates class
      // 4 (e & 3) + r (one optimizer update per lane, not four in a row)
      const int r = tv & 15, e = tv >> 4;
      const float s0 = row_sum16(w3g.x), s1 = row_sum16(w3g.y), s2 = row_sum16(w3g.z), s3 = row_sum16(w3g.w);
      const float sv = r == 0 ? s0 : (r == 1 ? s1 : (r == 2 ? s2 : s3));
      const int cls = 4 * (e & 3) + r;
      if (r < 4 && cls < D3) {
        const int k = cls * 8 + (e >> 2);
        upd32<ADAM, EXTRA>(o, sv, sW3s[k], sW3s[128 + k], sW3s[256 + k], sW3s[384 + k], lr_t, inv_bc2, wdmu);
      }
      if (tv < 64) {  // wave 0's four rows: classes 4e + r (e = 0..3)
        const float t0 = row_sum16(b3g.x), t1 = row_sum16(b3g.y), t2 = row_sum16(b3g.z), t3 = row_sum16(b3g.w);
        const float tsv = r == 0 ? t0 : (r == 1 ? t1 : (r == 2 ? t2 : t3));
        const int cb = 4 * e + r;
        if (r < 4 && cb < D3) upd32<ADAM, EXTRA>(o, tsv, sB3[cb], sB3[16 + cb], sB3[32 + cb], sB3[48 + cb], lr_t, inv_bc2, wdmu);
      }
    }
    lds_barrier();
    V2_STAMP(t, 6);
    // dH2 fragments of this wave's 16 W2 rows, read before the C1 partials overwrite the tile:
    //   C1 (dH1):  A = dH2[16mt + c][16w + 4h + ks]
    //   dW2:       A = dH2ᵀ[o2 = 16w + c][b = 4kb + h]
    float4 av1[MT];
    f32x4 gw2;      // dW2[o2 = 16w + 4h + i][k = c] over the batch (two interleaved MFMA chains)
    float db2s;     // db2[16w + c] partial over rows 4kb + h
    {
      int lq = lane;
      asm volatile("" : "+v"(lq));
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) av1[mt] = *reinterpret_cast<const float4*>(sDH2 + (16 * mt + (lq & 15)) * LDD + 16 * wave + 4 * (lq >> 4));
      float dv[BP / 4];
#pragma unroll
      for (int kb = 0; kb < BP / 4; ++kb) dv[kb] = sDH2[(4 * kb + (lq >> 4)) * LDD + 16 * wave + (lq & 15)];
      f32x4 g0 = zero4(), g1 = zero4();
#pragma unroll
      for (int kb = 0; kb < BP / 4; kb += 2) {
        g0 = mfma_f32(dv[kb], sH1[(4 * kb + (lq >> 4)) * LD16 + (lq & 15)], g0);
        g1 = mfma_f32(dv[kb + 1], sH1[(4 * kb + 4 + (lq >> 4)) * LD16 + (lq & 15)], g1);
      }
      gw2 = g0 + g1;
      db2s = 0.f;
#pragma unroll
      for (int kb = 0; kb < BP / 4; ++kb) db2s += dv[kb];
    }
    lds_barrier();  // every wave holds its fragments: the tile region is free for the partials
    V2_STAMP(t, 7);
    // C1: dH1 partials — wave w sums its 16 o2 rows (k order o2 = 16w + 4h + ks) with the OLD W2
    {
      f32x4 acc1[MT];
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        f32x4 acc = mfma_f32(av1[mt].x, w2c[0], zero4());
        acc = mfma_f32(av1[mt].y, w2c[1], acc);
        acc = mfma_f32(av1[mt].z, w2c[2], acc);
        acc1[mt] = mfma_f32(av1[mt].w, w2c[3], acc);
      }
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) sRed[(wave * MT + mt) * 64 + lane] = acc1[mt];
    }
    lds_barrier();
    V2_STAMP(t, 8);
    if (tv < MT * 64) {
      const int mt = tv >> 6, hh = (tv & 63) >> 4, cc = tv & 15;
      f32x4 s = sRed[mt * 64 + (tv & 63)];
#pragma unroll
      for (int w = 1; w < 8; ++w) s += sRed[(w * MT + mt) * 64 + (tv & 63)];
      bf16x4 dh, dm, dl;  // exact three-term split of dH1 (the B operand of the dW1 MFMAs)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float d = sH1[(16 * mt + 4 * hh + i) * LD16 + cc] > 0.f ? s[i] : 0.f;
        const bf16 x0 = (bf16)d;
        const float r = d - (float)x0;
        const bf16 x1 = (bf16)r;
        dh[i] = x0;
        dm[i] = x1;
        dl[i] = (bf16)(r - (float)x1);
      }
      const int off = cc * LDT + 16 * mt + 4 * hh;
      *reinterpret_cast<bf16x4*>(sD3 + off) = dh;
      *reinterpret_cast<bf16x4*>(sD3 + 16 * LDT + off) = dm;
      *reinterpret_cast<bf16x4*>(sD3 + 32 * LDT + off) = dl;
    }
    // W2 columns: update from dW2, transposed copy; db2 (rows 4kb + h summed above, then across h)
    {
      int lq = lane;
      asm volatile("" : "+v"(lq));
#pragma unroll
      for (int i = 0; i < 4; ++i) upd32<ADAM, EXTRA>(o, gw2[i], w2c[i], m2c[i], v2c[i], e2c[i], lr_t, inv_bc2, wdmu);
      w2_transpose(w2c, w2f, lq);
      float s = db2s;
      s += __shfl_xor(s, 16);
      s += __shfl_xor(s, 32);
      if (lq < 16) {
        const int k = 16 * wave + lq;
        upd32<ADAM, EXTRA>(o, s, sB2[k], sB2[128 + k], sB2[256 + k], sB2[384 + k], lr_t, inv_bc2, wdmu);
      }
    }
    lds_barrier();
    V2_STAMP(t, 9);
    // C2 (every wave, its own K steps): dW1 rows (and db1, in the bias slot) against the exact
    // three-term split of dH1, W1 update, the next batch's columns staged right after this K step's
    // reads (as layout 1, KS = 1)
    {
      int lv = lane;
      asm volatile("" : "+v"(lv));
      const int rows_next = more ? rows_at(a, n, t + 1) : 0;
      const bf16* xnext = a.Xb16 + ((int64_t)p * a.xb_rows + (int64_t)(t + 1) * a.B) * D0;
#pragma unroll
      for (int q = 0; q < RQ + 1; ++q) {
        const int s = wave + 8 * q;
        if (s < KS1) {
          int lq = lane;
          asm volatile("" : "+v"(lq));
          const bf16* dfrag = sD3 + (lq & 15) * LDT + 8 * (lq >> 4);
          constexpr int XQ = BP / 16;
          uint4 xq[XQ];
#pragma unroll
          for (int kk = 0; kk < XQ; ++kk) {
            const int idx = kk * 64 + lv;
            const int r = idx >> 2, col = 32 * s + 8 * (idx & 3);
            xq[kk] = (more && col < D0 && r < rows_next) ? *reinterpret_cast<const uint4*>(xnext + (unsigned)(r * D0 + col)) : uint4{0u, 0u, 0u, 0u};
          }
#pragma unroll
          for (int tt = 0; tt < 2; ++tt) {
            f32x4 acc = zero4();  // C[k = 32s + 16tt + 4h + i][o1 = c]
#pragma unroll
            for (int kb = 0; kb < BP / 32; ++kb)
              acc = mfma3(frag_b_tr_l(sX, LDX, 32 * kb, 32 * s + 16 * tt, lq), ld8(dfrag + 32 * kb), ld8(dfrag + 16 * LDT + 32 * kb),
                          ld8(dfrag + 32 * LDT + 32 * kb), acc);
            if (q < RQ) {
              const int qq = q < RQ ? q : 0;
#pragma unroll
              for (int i = 0; i < 4; ++i)
                upd32<ADAM, EXTRA>(o, acc[i], w1[qq][4 * tt + i], m1[qq][4 * tt + i], v1[qq][4 * tt + i], e1[qq][4 * tt + i], lr_t, inv_bc2, wdmu);
            } else {  // the LDS-resident K step
              const int off = (lq & 15) * 32 + 16 * tt + 4 * (lq >> 4);
              float4 w = *reinterpret_cast<float4*>(sW1x + off), m = *reinterpret_cast<float4*>(sW1x + 512 + off),
                     v = *reinterpret_cast<float4*>(sW1x + 1024 + off), e = *reinterpret_cast<float4*>(sW1x + 1536 + off);
              upd32<ADAM, EXTRA>(o, acc[0], w.x, m.x, v.x, e.x, lr_t, inv_bc2, wdmu);
              upd32<ADAM, EXTRA>(o, acc[1], w.y, m.y, v.y, e.y, lr_t, inv_bc2, wdmu);
              upd32<ADAM, EXTRA>(o, acc[2], w.z, m.z, v.z, e.z, lr_t, inv_bc2, wdmu);
              upd32<ADAM, EXTRA>(o, acc[3], w.w, m.w, v.w, e.w, lr_t, inv_bc2, wdmu);
              *reinterpret_cast<float4*>(sW1x + off) = w;
              *reinterpret_cast<float4*>(sW1x + 512 + off) = m;
              *reinterpret_cast<float4*>(sW1x + 1024 + off) = v;
            }
          }
          if (more) {
#pragma unroll
            for (int kk = 0; kk < XQ; ++kk) {
              const int idx = kk * 64 + lv;
              const int r = idx >> 2, col = 32 * s + 8 * (idx & 3);
              if (col < D0)
                *reinterpret_cast<uint4*>(sX + r * LDX + col) = xq[kk];
              else if (col == D0)
                *reinterpret_cast<uint4*>(sX + r * LDX + col) = bias_chunk(r < rows_next);
            }
          }
        }
      }
    }
    __syncthreads();
    V2_STAMP(t, 10);
  }

  // ---- epoch loss / correct partials of this owner's reducer rows (published before the commit)
  {
    const float l = wave_sum(loss_acc), cr = wave_sum(correct_acc);
    if (wave < (RPO < 2 ? 2 : RPO) && lane == 0) {  // waves >= RPO store zeros (whole float4 slots)
      persist::pub32(pb.plain, xbase + XL.lossp + ((int64_t)p * NG + g) * 8 + 2 * wave, l);
      persist::pub32(pb.plain, xbase + XL.lossp + ((int64_t)p * NG + g) * 8 + 2 * wave + 1, cr);
    }
  }
  if (!gang_commit_v2(a, pb, p, g, sOk)) return;
  // ---- write the state back (addresses re-derived from laundered indices, as layout 1)
  int lw = lane;
  int64_t pS_w = pS;
  asm volatile("" : "+v"(lw), "+s"(pS_w));
  const int hw = lw >> 4, cw = lw & 15;
  const int orow_w = 16 * g + cw;
#pragma unroll
  for (int q = 0; q < RQ + 1; ++q) {
    const int s = wave + 8 * q;
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      const int k = 32 * s + 16 * half + 4 * hw;
      if (s >= KS1 || k > D0) continue;
      float4 w, m, v;
      if (q < RQ) {
        const int qq = q < RQ ? q : 0;
        const int j0 = 4 * half;
        w = float4{w1[qq][j0], w1[qq][j0 + 1], w1[qq][j0 + 2], w1[qq][j0 + 3]};
        m = float4{m1[qq][j0], m1[qq][j0 + 1], m1[qq][j0 + 2], m1[qq][j0 + 3]};
        v = float4{v1[qq][j0], v1[qq][j0 + 1], v1[qq][j0 + 2], v1[qq][j0 + 3]};
      } else {
        const int off = cw * 32 + 16 * half + 4 * hw;
        w = *reinterpret_cast<float4*>(sW1x + off);
        m = *reinterpret_cast<float4*>(sW1x + 512 + off);
        v = *reinterpret_cast<float4*>(sW1x + 1024 + off);
      }
      if (k < D0) {
        const int64_t idx = pS_w + a.off_w1 + (int64_t)orow_w * D0 + k;
        *reinterpret_cast<float4*>(a.params + idx) = w;
        *reinterpret_cast<float4*>(a.m + idx) = m;
        if (ADAM) *reinterpret_cast<float4*>(a.v + idx) = v;
      } else {  // k == D0: b1 from the bias slot
        const int64_t idx = pS_w + a.off_b1 + orow_w;
        a.params[idx] = w.x;
        a.m[idx] = m.x;
        if (ADAM) a.v[idx] = v.x;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t idx = pS_w + a.off_w2 + (int64_t)(16 * wave + 4 * hw + i) * PD1 + 16 * g + cw;
    a.params[idx] = w2c[i];
    a.m[idx] = m2c[i];
    if (ADAM) a.v[idx] = v2c[i];
    if (pb.w2chk != nullptr) pb.w2chk[(int64_t)p * PD2 * PD1 + (int64_t)(16 * wave + 4 * hw + i) * PD1 + 16 * g + cw] = w2c[i];
  }
  if (tid < 128) {
    const int cls = tid >> 3, j = tid & 7;
    if (cls < D3) {
      const int64_t idx = pS_w + a.off_w3 + (int64_t)cls * PD2 + 8 * g + j;
      a.params[idx] = sW3s[tid];
      a.m[idx] = sW3s[128 + tid];
      if (ADAM) a.v[idx] = sW3s[256 + tid];
    }
  }
  if (g == 0) {
    if (tid >= 128 && tid < 256) {
      const int k = tid - 128;
      const int64_t idx = pS_w + a.off_b2 + k;
      a.params[idx] = sB2[k];
      a.m[idx] = sB2[128 + k];
      if (ADAM) a.v[idx] = sB2[256 + k];
    } else if (tid >= 256 && tid < 256 + D3) {
      const int k = tid - 256;
      const int64_t idx = pS_w + a.off_b3 + k;
      a.params[idx] = sB3[k];
      a.m[idx] = sB3[16 + k];
      if (ADAM) a.v[idx] = sB3[32 + k];
    } else if (tid == 320) {  // the gang's epoch loss / correct: every owner's partials, fixed order
      const __amdgpu_buffer_rsrc_t r = rsrc_of(xbase + XL.lossp + (int64_t)p * NG * 8, NG * 32);
      float l = 0.f, cr = 0.f;
      for (int k = 0; k < NG; ++k) {
        for (int j = 0; j < RPO; j += 2) {  // slots of rows j, j + 1 (zero-filled above RPO)
          const float4 v = ld_sc1_16(r, k * 32 + j * 8);
          l += v.x + v.z;
          cr += v.y + v.w;
        }
      }
      atomicAdd(&a.loss_acc[p], l);
      atomicAdd(&a.correct_acc[p], (int)(cr + 0.5f));
    }
  }
}

template <int BP, bool ADAM, bool EXTRA>
__global__ __launch_bounds__(NT) void mlp_persistent_f32v2_epoch(MLPArgs a, MLPPersistF32Bufs pb, int p_base, int attempt) {
  extern __shared__ __attribute__((aligned(16))) char smem_v2[];
  const int b = blockIdx.x;
  const int p = p_base + b % PPL;
  const int g = b / PPL;
  if (p >= a.P) return;
  const int4 ctl = a.ctl[p];
  if (!(ctl.x & 1) || ctl.y <= 0) return;
  int* err_first = pb.err + p;
  if (attempt) {
    if (__hip_atomic_load(err_first, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) return;
    pb.err = pb.err + ERR_RETRY + p;
    pb.fbase = RETRY_BASE;
  } else {
    if (a.debug_giveup == p + 1) {  // test hook: this peer's first attempt gives up at once
      if (g == 0 && threadIdx.x == 0) __hip_atomic_store(err_first, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    pb.err = err_first;
    pb.fbase = 0;
  }
  // single-XCD gang (blocks b = p mod 8): hand-offs kept in that XCD's L2 (persist::gang_same_xcd,
  // mlp_persistent_f32.hip); the last two lines of the shared flag block hold the XCC reports
  static_assert(FDONE + NG <= F32_FPP - 2, "v2 flags leave the XCC lines free");
  pb.plain = pb.plain_ok && persist::gang_same_xcd(persist::flag_at(pb.flags, F32_FPP, p, F32_FPP - 2), g, NG, pb.fbase ? 0x200u : 0x100u,
                                                   reinterpret_cast<int*>(smem_v2), 10000ull)
                 ? pb.plain_ok
                 : 0;
  owner_v2<BP, ADAM, EXTRA>(a, pb, p, g, smem_v2);
  if (g == 0) {
    __syncthreads();
    if (threadIdx.x == 0 && __hip_atomic_load(pb.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) {
      __hip_atomic_store(pb.gen + p, __hip_atomic_load(pb.gen + p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
      if (attempt) __hip_atomic_store(err_first, 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // the gang recovered
    }
  }
}

template <int BP, bool ADAM, bool EXTRA>
const void* v2_fn() {
  return (const void*)mlp_persistent_f32v2_epoch<BP, ADAM, EXTRA>;
}
template <int BP>
void launch_v2_bp(const MLPArgs& a, const MLPPersistF32Bufs& pb, hipStream_t s, int p_base, size_t lds, int attempt) {
  const dim3 grid(PPL * NG), block(NT);
  const bool adam = a.opt.kind == 0;
  const bool extra = a.anchor != nullptr || a.cg != nullptr;
  if (adam && !extra) hipLaunchKernelGGL((mlp_persistent_f32v2_epoch<BP, true, false>), grid, block, lds, s, a, pb, p_base, attempt);
  else if (adam) hipLaunchKernelGGL((mlp_persistent_f32v2_epoch<BP, true, true>), grid, block, lds, s, a, pb, p_base, attempt);
  else if (!extra) hipLaunchKernelGGL((mlp_persistent_f32v2_epoch<BP, false, false>), grid, block, lds, s, a, pb, p_base, attempt);
  else hipLaunchKernelGGL((mlp_persistent_f32v2_epoch<BP, false, true>), grid, block, lds, s, a, pb, p_base, attempt);
}

}  // namespace

// ---- host interface (dispatched from mlp_persistent_f32.hip)
bool mlp_f32v2_supported(const MLPArgs& a) {
  if (a.D1 != PD1 || a.D2 != PD2 || a.D3 < 1 || a.D3 > 16) return false;
  if (a.D0 % 8 != 0 || ks1_of(a.D0) > 1 + 8 * RQ) return false;  // at most 25 K steps (three per wave + one in LDS)
  if (a.Bpad != 32 && a.Bpad != 64) return false;
  if ((a.cg == nullptr) != (a.cl == nullptr)) return false;
  if (a.cg != nullptr && a.anchor != nullptr) return false;  // one extra term per element (mlp_f32_common.h)
  return owner_lds_v2(a.Bpad, a.D0).total <= 160 * 1024;
}
size_t mlp_f32v2_lds(const MLPArgs& a) { return owner_lds_v2(a.Bpad, a.D0).total; }
size_t mlp_f32v2_bytes(int P, int Bpad) { return (size_t)v2_layout(P, Bpad).total * sizeof(float); }
int mlp_f32v2_launch_wgs() { return PPL * NG; }
int mlp_f32v2_resident_capacity(const MLPArgs& a, int num_cus) {
  int per_cu = 0;
  const void* fn = a.Bpad == 64 ? v2_fn<64, true, false>() : v2_fn<32, true, false>();
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, NT, mlp_f32v2_lds(a)) != hipSuccess) return 0;
  return per_cu * num_cus;
}
hipError_t mlp_f32v2_prepare(const MLPArgs& a) {
  const int lds = (int)mlp_f32v2_lds(a);
  const void* fns[8] = {v2_fn<64, true, false>(), v2_fn<64, true, true>(), v2_fn<64, false, false>(), v2_fn<64, false, true>(),
                        v2_fn<32, true, false>(), v2_fn<32, true, true>(), v2_fn<32, false, false>(), v2_fn<32, false, true>()};
  for (const void* fn : fns) {
    const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}
// One epoch of every active peer: groups of PPL peers (a launch's gangs must all be co-resident),
// then the recovery launches (attempt 1): a no-op exit for every gang that did not give up.
void mlp_f32v2_launch(const MLPArgs& a, const MLPPersistF32Bufs& pb, hipStream_t s) {
  const size_t lds = mlp_f32v2_lds(a);
  for (int attempt = 0; attempt < 2; ++attempt)
    for (int p0 = 0; p0 < a.P; p0 += PPL) {
      if (a.Bpad == 64) launch_v2_bp<64>(a, pb, s, p0, lds, attempt);
      else launch_v2_bp<32>(a, pb, s, p0, lds, attempt);
    }
}
