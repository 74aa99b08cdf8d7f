// Grouped fused MLP engine kernels (gfx950 / MI355X).
//
// One federated "round" of local training for P co-located peers is a sequence of steps; each
// step is three launches that each cover ALL peers (grid.z = peer):
//
//   K1 mlp_fc1_fwd   : H1 = relu(gather(X)·W1ᵀ + b1)          uint8→bf16 convert fused into the
//                      A-fragment load; also writes H1ᵀ and Xᵀ for the weight gradients.
//   K2 mlp_head      : H2 = relu(H1·W2ᵀ + b2) → logits → log_softmax + NLL (+argmax) →
//                      dlogits → dH2 = dlogits·W3 ⊙ [H2>0] → dH1 = dH2·W2 ⊙ [H1>0]
//                      (one workgroup per 16 batch rows; H2/dlogits/dH2 stay in LDS).
//   K3 mlp_wgrad_opt : dW1 = dH1ᵀ·X, dW2 = dH2ᵀ·H1, dW3, db1..3 — each 16×16 MFMA tile applies
//                      the optimizer (Adam/SGD, + FedProx/SCAFFOLD terms) in its epilogue and
//                      refreshes the bf16 shadow copies. No gradient buffer ever hits HBM.
//
// All GEMMs are v_mfma_f32_16x16x32_bf16 with fp32 accumulation; master weights, Adam moments
// and the loss are fp32. Whole epochs are captured into one hipGraph by the engine (mlp_engine.hip).
#include "common.h"
#include "mlp_fused.h"

// Optional per-block phase timestamps (build with -DMLP_STAMPS; read with mlp_debug_stamps).
#ifdef MLP_STAMPS
__device__ unsigned long long g_mlp_stamps[3][4096][4];
#define MLP_STAMP(k, i)                                                                                         \
  do {                                                                                                          \
    const unsigned _b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);                        \
    if (threadIdx.x == 0 && _b < 4096) g_mlp_stamps[k][_b][i] = wall_clock64();                                \
  } while (0)
extern "C" int mlp_debug_stamps(void* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_mlp_stamps), sizeof(g_mlp_stamps)) == hipSuccess ? 0 : 1;
}
#else
#define MLP_STAMP(k, i) \
  do {                  \
  } while (0)
#endif

namespace {

__device__ __forceinline__ int rows_valid_train(const MLPArgs& a, const int4& ctl, int step) {
  int r = ctl.y - step * a.B;
  return r < 0 ? 0 : (r > a.B ? a.B : r);
}

__device__ __forceinline__ int rows_valid_eval(const MLPArgs& a, const int4& ctl, int base) {
  int r = ctl.w - base;
  return r < 0 ? 0 : (r > MLP_EVAL_CHUNK ? MLP_EVAL_CHUNK : r);
}

// rows of this peer in this step (0 = inactive peer or exhausted data)
template <bool TRAIN>
__device__ __forceinline__ int peer_rows(const MLPArgs& a, const int4& ctl, int step, int base) {
  if (!ctl.x) return 0;
  return TRAIN ? rows_valid_train(a, ctl, step) : rows_valid_eval(a, ctl, base);
}

// training row r of step `step` in the epoch-gathered batch buffer
__device__ __forceinline__ int64_t batch_row(const MLPArgs& a, int p, int step, int r) { return (int64_t)p * a.xb_rows + (int64_t)step * a.B + r; }

}  // namespace

// ---------------------------------------------------------------------------------------------
// K1: fc1 forward. grid = (D1/32, rows/32, P), block = 256.
//   Block tile = 32 rows × 32 cols (2×2 MFMA tiles); the 4 waves split K (= D0) four ways so
//   each wave's dependent load chain is ≤ 8 k-steps, with all fragment loads of a chunk hoisted
//   ahead of its MFMAs (the kernel is load-latency bound: 0.2 GFLOP/step for 8 peers). Partial
//   accumulators are reduced through LDS; wave 0 runs the epilogue.
// ---------------------------------------------------------------------------------------------
template <bool TRAIN>
__global__ __launch_bounds__(256) void mlp_fc1_fwd(MLPArgs a, int step, int base) {
  if (TRAIN) MLP_STAMP(0, 0);
  constexpr int MT = 2, NT = 2, KCH = 8;
  __shared__ __attribute__((aligned(16))) float sRed[3][64][MT * NT * 4];
  const int p = blockIdx.z;
  const int4 ctl = a.ctl[p];
  const int rows = peer_rows<TRAIN>(a, ctl, step, base);
  if (rows == 0) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 4, c = lane & 15;
  const int row0 = blockIdx.y * 32;
  const int col0 = blockIdx.x * 32;
  const int D0 = a.D0, D1 = a.D1;
  float bias[2];
#pragma unroll
  for (int nt = 0; nt < 2; ++nt) bias[nt] = a.params[(int64_t)p * a.S + a.off_b1 + col0 + nt * 16 + c];
  const uint8_t* X = TRAIN ? a.Xb : a.Xtp[p];

  const uint8_t* arow[MT];
  bool avalid[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int r = row0 + mt * 16 + c;
    avalid[mt] = r < rows;
    arow[mt] = avalid[mt] ? X + (TRAIN ? batch_row(a, p, step, r) : (int64_t)(base + r)) * (int64_t)D0 : X;
  }
  const bf16* wrow[NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) wrow[nt] = a.shadow + (int64_t)p * a.S + a.off_w1 + (int64_t)(col0 + nt * 16 + c) * D0;

  // this wave's k-step range
  const int ksteps = (D0 + 31) / 32;
  const int per = (ksteps + 3) / 4;
  const int ks_begin = wave * per;
  const int ks_end = min(ksteps, ks_begin + per);

  f32x4 acc[MT][NT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = zero4();

  for (int ks0 = ks_begin; ks0 < ks_end; ks0 += KCH) {
    bf16x8 af[KCH][MT], bfr[KCH][NT];
#pragma unroll
    for (int j = 0; j < KCH; ++j) {
      const int k = (ks0 + j) * 32 + 8 * h;
      const bool kin = (ks0 + j) < ks_end && k < D0;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) af[j][mt] = (kin && avalid[mt]) ? ld8_u8(arow[mt] + k) : zero_bf16x8();
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) bfr[j][nt] = kin ? ld8(wrow[nt] + k) : zero_bf16x8();
    }
#pragma unroll
    for (int j = 0; j < KCH; ++j)
#pragma unroll
      for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = mfma_bf16(af[j][mt], bfr[j][nt], acc[mt][nt]);
  }

  if (TRAIN) MLP_STAMP(0, 1);
  // cross-wave K reduction
  if (wave > 0) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int i = 0; i < 4; ++i) sRed[wave - 1][lane][(mt * NT + nt) * 4 + i] = acc[mt][nt][i];
  }
  lds_barrier();
  if (wave != 0) return;
  if (TRAIN) MLP_STAMP(0, 2);
#pragma unroll
  for (int w = 0; w < 3; ++w)
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[mt][nt][i] += sRed[w][lane][(mt * NT + nt) * 4 + i];

  // epilogue: + b1, ReLU, zero invalid rows; H1 row-major (+ H1ᵀ when training)
  bf16* H1 = a.H1 + (int64_t)p * a.h1_rows * D1;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int col = col0 + nt * 16 + c;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      bf16x4 packed;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = row0 + mt * 16 + 4 * h + i;
        float v = fmaxf(acc[mt][nt][i] + bias[nt], 0.f);
        if (r >= rows) v = 0.f;
        packed[i] = (bf16)v;
        H1[(int64_t)r * D1 + col] = packed[i];
      }
      if (TRAIN) {
        bf16* H1T = a.H1T + (int64_t)p * D1 * a.Bpad;
        *reinterpret_cast<bf16x4*>(H1T + (int64_t)col * a.Bpad + row0 + mt * 16 + 4 * h) = packed;
      }
    }
  }
  if (TRAIN) MLP_STAMP(0, 3);
}

// ---------------------------------------------------------------------------------------------
// K2: head. grid = (rows/16, 1, P), block = 256. TP2 = D2/64, TP1 = D1/64 column tiles per wave.
// ---------------------------------------------------------------------------------------------
template <int TP1, int TP2, bool TRAIN>
__global__ __launch_bounds__(256) void mlp_head(MLPArgs a, int step, int base) {
  if (TRAIN) MLP_STAMP(1, 0);
  constexpr int D1 = TP1 * 64, D2 = TP2 * 64;
  constexpr int LD1 = D1 + 8, LD2 = D2 + 8;  // padded LDS rows (bf16) to spread banks
  constexpr int LDD = 32 + 8;
  constexpr int KS1 = D1 / 32, KS2 = D2 / 32;
  __shared__ __attribute__((aligned(16))) bf16 sH1[16 * LD1];
  __shared__ __attribute__((aligned(16))) bf16 sH2[16 * LD2];
  __shared__ __attribute__((aligned(16))) bf16 sDH2[16 * LD2];
  __shared__ __attribute__((aligned(16))) bf16 sDlog[16 * LDD];
  __shared__ __attribute__((aligned(16))) bf16 sW3[16 * LD2];

  const int p = blockIdx.z;
  const int4 ctl = a.ctl[p];
  const int rows = peer_rows<TRAIN>(a, ctl, step, base);
  if (rows == 0) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 4, c = lane & 15;
  const int row0 = blockIdx.x * 16;
  const int D3 = a.D3;
  const int64_t pS = (int64_t)p * a.S;
  const bf16* H1 = a.H1 + (int64_t)p * a.h1_rows * D1;
  const bool cin = c < D3;
  // W3 (≤16 × D2 bf16) staged once in LDS with vector loads; rows ≥ D3 are zero
  for (int e = threadIdx.x; e < 16 * (D2 / 8); e += 256) {
    const int r = e / (D2 / 8), q = e % (D2 / 8);
    *reinterpret_cast<bf16x8*>(&sW3[r * LD2 + q * 8]) = r < D3 ? ld8(a.shadow + pS + a.off_w3 + (int64_t)r * D2 + q * 8) : zero_bf16x8();
  }

  // ---- issue every independent global load up front (the kernel is latency bound)
  bf16x8 a1[KS1];
  const bf16* arow = H1 + (int64_t)(row0 + c) * D1;
#pragma unroll
  for (int k = 0; k < KS1; ++k) a1[k] = ld8(arow + k * 32 + 8 * h);
  bf16x8 w2f[KS1][TP2];
#pragma unroll
  for (int k = 0; k < KS1; ++k)
#pragma unroll
    for (int t = 0; t < TP2; ++t) w2f[k][t] = ld8(a.shadow + pS + a.off_w2 + (int64_t)((wave + 4 * t) * 16 + c) * D1 + k * 32 + 8 * h);
  float b2v[TP2];
#pragma unroll
  for (int t = 0; t < TP2; ++t) b2v[t] = a.params[pS + a.off_b2 + (wave + 4 * t) * 16 + c];
  // wave 0: logits operands + labels
  bf16x8 w3f[KS2];
  float b3 = 0.f;
  int ylab[4] = {-1, -1, -1, -1};
  if (wave == 0) {
    b3 = cin ? a.params[pS + a.off_b3 + c] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int grow = row0 + 4 * h + i;
      if (grow < rows) {
        ylab[i] = TRAIN ? a.Yb[batch_row(a, p, step, grow)] : a.Ytp[p][base + grow];
      }
    }
  }
  bf16x8 w3c[TP2];

  // stage H1 rows in LDS (mask for dH1) and zero the dlogits tile (k 16..31 = K padding)
  if (TRAIN && wave == 0) {
#pragma unroll
    for (int k = 0; k < KS1; ++k) *reinterpret_cast<bf16x8*>(&sH1[c * LD1 + k * 32 + 8 * h]) = a1[k];
  }
  for (int i = threadIdx.x; i < 16 * LDD; i += 256) sDlog[i] = (bf16)0.f;

  lds_barrier();  // sW3 / sH1 / sDlog ready; H1 and W2 loads may still be in flight
  if (TRAIN) MLP_STAMP(1, 1);
  // training: W2ᵀ fragments for dH1, only needed in the last phase — issued here so their
  // latency hides under the H2 / logits / softmax phases instead of delaying the first barrier
  bf16x8 w2tf[TRAIN ? TP1 : 1][TRAIN ? KS2 : 1];
  if (TRAIN) {
    const bf16* w2t = a.w2t + (int64_t)p * D1 * D2;
#pragma unroll
    for (int t = 0; t < (TRAIN ? TP1 : 1); ++t)
#pragma unroll
      for (int k = 0; k < (TRAIN ? KS2 : 1); ++k) w2tf[t][k] = ld8(w2t + (int64_t)((wave + 4 * t) * 16 + c) * D2 + k * 32 + 8 * h);
  }
  if (wave == 0) {
#pragma unroll
    for (int k = 0; k < KS2; ++k) w3f[k] = *reinterpret_cast<const bf16x8*>(&sW3[c * LD2 + k * 32 + 8 * h]);
  }
  if (TRAIN) {
#pragma unroll
    for (int t = 0; t < TP2; ++t) {
      const int n = (wave + 4 * t) * 16 + c;
#pragma unroll
      for (int j = 0; j < 8; ++j) w3c[t][j] = (8 * h + j) < 16 ? sW3[(8 * h + j) * LD2 + n] : (bf16)0.f;
    }
  }

  // ---- H2 = relu(H1 · W2ᵀ + b2): wave owns column tiles {wave + 4*t}
  f32x4 h2[TP2];
#pragma unroll
  for (int t = 0; t < TP2; ++t) h2[t] = zero4();
#pragma unroll
  for (int k = 0; k < KS1; ++k)
#pragma unroll
    for (int t = 0; t < TP2; ++t) h2[t] = mfma_bf16(a1[k], w2f[k][t], h2[t]);
#pragma unroll
  for (int t = 0; t < TP2; ++t) {
    const int col = (wave + 4 * t) * 16 + c;
    bf16x4 packed;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 4 * h + i;
      float v = fmaxf(h2[t][i] + b2v[t], 0.f);
      if (row0 + r >= rows) v = 0.f;
      h2[t][i] = v;
      packed[i] = (bf16)v;
      sH2[r * LD2 + col] = packed[i];
    }
    if (TRAIN) *reinterpret_cast<bf16x4*>(a.H2T + (int64_t)p * D2 * a.Bpad + (int64_t)col * a.Bpad + row0 + 4 * h) = packed;
  }
  lds_barrier();

  // ---- logits, log-softmax, NLL, argmax, dlogits (wave 0)
  if (wave == 0) {
    f32x4 lg = zero4();
#pragma unroll
    for (int k = 0; k < KS2; ++k) lg = mfma_bf16(*reinterpret_cast<const bf16x8*>(&sH2[c * LD2 + k * 32 + 8 * h]), w3f[k], lg);
    float loss_part = 0.f;
    int correct_part = 0;
    bf16x4 dpack;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 4 * h + i;
      const int y = ylab[i];
      const bool rvalid = y >= 0;
      const float logit = cin ? lg[i] + b3 : -INFINITY;
      const float mx = warp_max16(logit);
      const float se = warp_sum16(cin ? __expf(logit - mx) : 0.f);
      const float logp = logit - (mx + __logf(se));
      int cand = (cin && logit == mx) ? c : 16;
      cand = min(cand, __shfl_xor(cand, 1));
      cand = min(cand, __shfl_xor(cand, 2));
      cand = min(cand, __shfl_xor(cand, 4));
      cand = min(cand, __shfl_xor(cand, 8));
      if (rvalid && c == y) loss_part -= logp;
      if (rvalid && c == 0) {
        correct_part += (cand == y);
        if (!TRAIN && a.conf != nullptr && y < 16 && cand < 16) atomicAdd(&a.conf[(p * 16 + y) * 16 + cand], 1);
      }
      float d = 0.f;
      if (TRAIN && rvalid && cin) d = (__expf(logp) - (c == y ? 1.f : 0.f)) / (float)rows;
      dpack[i] = (bf16)d;
      if (TRAIN) sDlog[r * LDD + c] = dpack[i];
    }
    if (TRAIN) *reinterpret_cast<bf16x4*>(a.dlogT + (int64_t)p * 16 * a.Bpad + (int64_t)c * a.Bpad + row0 + 4 * h) = dpack;
    loss_part = wave_sum(loss_part);
    const float cp = wave_sum((float)correct_part);
    if (lane == 0) {
      atomicAdd(&a.loss_acc[p], loss_part);
      atomicAdd(&a.correct_acc[p], (int)(cp + 0.5f));
    }
  }
  if (!TRAIN) return;
  lds_barrier();
  MLP_STAMP(1, 2);

  // ---- dH2 = dlogits · W3 ⊙ [H2 > 0]   (K = 16 classes, padded to 32)
  {
    const bf16x8 av = *reinterpret_cast<const bf16x8*>(&sDlog[c * LDD + 8 * h]);
#pragma unroll
    for (int t = 0; t < TP2; ++t) {
      const int n = (wave + 4 * t) * 16 + c;
      const f32x4 acc = mfma_bf16(av, w3c[t], zero4());
      bf16x4 packed;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        packed[i] = (bf16)(h2[t][i] > 0.f ? acc[i] : 0.f);
        sDH2[(4 * h + i) * LD2 + n] = packed[i];
      }
      *reinterpret_cast<bf16x4*>(a.dH2T + (int64_t)p * D2 * a.Bpad + (int64_t)n * a.Bpad + row0 + 4 * h) = packed;
    }
  }
  lds_barrier();

  // ---- dH1 = dH2 · W2 ⊙ [H1 > 0]   (B operand = W2ᵀ shadow, prefetched)
  bf16x8 adh[KS2];
#pragma unroll
  for (int k = 0; k < KS2; ++k) adh[k] = *reinterpret_cast<const bf16x8*>(&sDH2[c * LD2 + k * 32 + 8 * h]);
#pragma unroll
  for (int t = 0; t < TP1; ++t) {
    const int n = (wave + 4 * t) * 16 + c;
    f32x4 acc = zero4();
#pragma unroll
    for (int k = 0; k < KS2; ++k) acc = mfma_bf16(adh[k], w2tf[TRAIN ? t : 0][TRAIN ? k : 0], acc);
    bf16x4 packed;
#pragma unroll
    for (int i = 0; i < 4; ++i) packed[i] = (bf16)((float)sH1[(4 * h + i) * LD1 + n] > 0.f ? acc[i] : 0.f);
    *reinterpret_cast<bf16x4*>(a.dH1T + (int64_t)p * D1 * a.Bpad + (int64_t)n * a.Bpad + row0 + 4 * h) = packed;
  }
  MLP_STAMP(1, 3);
}

// ---------------------------------------------------------------------------------------------
// K3: weight gradients + optimizer. grid = (nb_w1 + nb_w2 + 1, 1, P), block = 256.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void step_bias_corr(const MLPArgs& a, const int4& ctl, int step, float& bc1, float& bc2s) {
  const int t = ctl.z + step + 1;
  bc1 = 1.f - __powf(a.opt.beta1, (float)t);
  bc2s = sqrtf(1.f - __powf(a.opt.beta2, (float)t));
}

__device__ __forceinline__ void update_elem(const MLPArgs& a, int64_t idx, float g, float bc1, float bc2s) {
  float w = a.params[idx], m = a.m[idx];
  float v = a.opt.kind == 0 ? a.v[idx] : 0.f;
  opt_update(a.opt, g, w, m, v, bc1, bc2s, a.anchor, a.cg, a.cl, idx);
  a.params[idx] = w;
  a.m[idx] = m;
  if (a.opt.kind == 0) a.v[idx] = v;
  a.shadow[idx] = (bf16)w;
}

// Block decomposition (grid.x): [0, nb1) W1 blocks — a 16-row × 64-column tile of W1 (4 waves ×
// 16 columns) whose X slab (64 columns × batch) is staged once, transposed to bf16, in LDS;
// [nb1, nb1+nb2) W2 blocks — 16 × 64 tiles; [nb1+nb2, +nb3) W3 blocks. After the MFMAs every block
// re-lays its fp32 gradient tile out through LDS so that each thread updates 4 consecutive
// elements (float4): a wave instruction then covers 4 rows × 256 contiguous bytes of params/m/v
// (coalesced optimizer traffic — the dominant HBM/MALL stream of a step). Bias gradients are row
// sums of A fragments, produced by the blocks whose column group is 0.
__device__ __forceinline__ float frag_sum(const bf16x8& v) {
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += (float)v[j];
  return s;
}

// Block-wide vectorised optimizer update of a 16 × WG_COLS tile by 256 threads: float4 chunk q of
// the row-major tile (q = tid + 256 k) is row q / (WG_COLS/4) — every wave instruction covers
// contiguous row segments of params/m/v. The optimizer state is prefetched at block entry
// (independent of the gradient) so its latency hides under the staging and the MFMAs; the
// gradient tile arrives through LDS (sG, fp32, row stride WG_LDG).
//
// Tile choice, measured with the -DMLP_STAMPS build (8 peers, B = 64): 16 × 64 tiles / 4 waves
// finish the kernel first (≈12.7 µs). Fatter tiles dispatch faster (the grid is launched at
// ≈1 wave/ns: 1664 × 4 waves start over 5.9 µs, 576 × 4 over 0.3 µs) but each block's optimizer
// chunk grows and the kernel — ≈49 MB of fp32 w/m/v traffic per step — ends later (16 × 256:
// 14.3 µs; 16 × 128 with 8 waves: 13.7 µs).
#define WG_WAVES 4                       // waves per wgrad block
#define WG_NT 1                          // 16-column MFMA tiles per wave
#define WG_COLS (16 * WG_WAVES * WG_NT)  // columns of a gradient tile (16 rows x 64)
#define WG_LDG (WG_COLS + 4)             // fp32 row stride of the LDS gradient tile
#define WG_Q (16 * WG_COLS / 4 / 256)    // float4 chunks per thread

struct TileState {
  float4 w[WG_Q], m[WG_Q], v[WG_Q];
  int64_t base;
  int row0, col0, ncols, ld;
};

__device__ __forceinline__ void chunk_pos(int k, int& r, int& c4) {
  const int q = threadIdx.x + 256 * k;
  r = q / (WG_COLS / 4);
  c4 = (q % (WG_COLS / 4)) * 4;
}

__device__ __forceinline__ TileState tile_prefetch(const MLPArgs& a, int64_t base, int ld, int row0, int col0, int ncols) {
  TileState st;
  st.base = base;
  st.row0 = row0;
  st.col0 = col0;
  st.ncols = ncols;
  st.ld = ld;
#pragma unroll
  for (int k = 0; k < WG_Q; ++k) {
    int r, c4;
    chunk_pos(k, r, c4);
    const int col = col0 + c4;
    if (col + 4 <= ncols && (ld & 3) == 0) {
      const int64_t idx = base + (int64_t)(row0 + r) * ld + col;
      st.w[k] = *reinterpret_cast<const float4*>(a.params + idx);
      st.m[k] = *reinterpret_cast<const float4*>(a.m + idx);
      st.v[k] = a.opt.kind == 0 ? *reinterpret_cast<const float4*>(a.v + idx) : float4{0.f, 0.f, 0.f, 0.f};
    }
  }
  return st;
}

__device__ __forceinline__ void tile_apply(const MLPArgs& a, const TileState& st, const float* sG, float bc1, float bc2s, bool w2t_refresh, int p) {
#pragma unroll
  for (int k = 0; k < WG_Q; ++k) {
    int r, c4;
    chunk_pos(k, r, c4);
    const int col = st.col0 + c4;
    if (col >= st.ncols) continue;
    const float* g = sG + r * WG_LDG + c4;
    const int64_t idx = st.base + (int64_t)(st.row0 + r) * st.ld + col;
    if (col + 4 <= st.ncols && (st.ld & 3) == 0) {
      float wv[4] = {st.w[k].x, st.w[k].y, st.w[k].z, st.w[k].w}, mv[4] = {st.m[k].x, st.m[k].y, st.m[k].z, st.m[k].w},
            vv[4] = {st.v[k].x, st.v[k].y, st.v[k].z, st.v[k].w};
      bf16x4 sh;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        opt_update(a.opt, g[j], wv[j], mv[j], vv[j], bc1, bc2s, a.anchor, a.cg, a.cl, idx + j);
        sh[j] = (bf16)wv[j];
      }
      *reinterpret_cast<float4*>(a.params + idx) = float4{wv[0], wv[1], wv[2], wv[3]};
      *reinterpret_cast<float4*>(a.m + idx) = float4{mv[0], mv[1], mv[2], mv[3]};
      if (a.opt.kind == 0) *reinterpret_cast<float4*>(a.v + idx) = float4{vv[0], vv[1], vv[2], vv[3]};
      *reinterpret_cast<bf16x4*>(a.shadow + idx) = sh;
      if (w2t_refresh) {
#pragma unroll
        for (int j = 0; j < 4; ++j) a.w2t[(int64_t)p * a.D1 * a.D2 + (int64_t)(col + j) * a.D2 + st.row0 + r] = sh[j];
      }
    } else {
      for (int j = 0; j < 4 && col + j < st.ncols; ++j) {
        float w = a.params[idx + j], m = a.m[idx + j], v = a.opt.kind == 0 ? a.v[idx + j] : 0.f;
        opt_update(a.opt, g[j], w, m, v, bc1, bc2s, a.anchor, a.cg, a.cl, idx + j);
        a.params[idx + j] = w;
        a.m[idx + j] = m;
        if (a.opt.kind == 0) a.v[idx + j] = v;
        a.shadow[idx + j] = (bf16)w;
        if (w2t_refresh) a.w2t[(int64_t)p * a.D1 * a.D2 + (int64_t)(col + j) * a.D2 + st.row0 + r] = (bf16)w;
      }
    }
  }
}

// LDS is sized at launch for the real padded batch: sG 16 x (WG_COLS + 4) fp32 + the X slab, Bpad
// rows x (WG_COLS + 8) bf16, staged ROW-major (coalesced 8-byte global loads along a sample row, one
// ds_write_b128 per 8 pixels) and read as MFMA B fragments with the gfx950 transposed LDS read
// (ds_read_b64_tr_b16) — no per-element transposing LDS writes (50 KB at Bpad = 64).
#define WG_LDXR (WG_COLS + 8)
static inline size_t wgrad_lds_bytes(int Bpad) { return 16 * WG_LDG * sizeof(float) + (size_t)Bpad * WG_LDXR * sizeof(bf16); }

__global__ __launch_bounds__(256) void mlp_wgrad_opt(MLPArgs a, int step) {
  extern __shared__ __attribute__((aligned(16))) char smem_wg[];
  float* sG = reinterpret_cast<float*>(smem_wg);
  bf16* sX = reinterpret_cast<bf16*>(smem_wg + 16 * WG_LDG * sizeof(float));
  MLP_STAMP(2, 0);
  const int p = blockIdx.z;
  const int4 ctl = a.ctl[p];
  const int rows = peer_rows<true>(a, ctl, step, 0);
  if (rows == 0) return;
  float bc1, bc2s;
  step_bias_corr(a, ctl, step, bc1, bc2s);
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // provably wave-uniform
  const int h = lane >> 4, c = lane & 15;
  const int D0 = a.D0, D1 = a.D1, D2 = a.D2, D3 = a.D3, Bp = a.Bpad;
  const int64_t pS = (int64_t)p * a.S;
  const int cg1 = (D0 + WG_COLS - 1) / WG_COLS;  // 256-column groups of W1
  const int cg2 = (D1 + WG_COLS - 1) / WG_COLS;  // 256-column groups of W2
  const int nb1 = (D1 / 16) * cg1;
  const int nb2 = (D2 / 16) * cg2;
  const int b = blockIdx.x;

  if (b < nb1 + nb2) {
    const bool w1 = b < nb1;
    const int bb = w1 ? b : b - nb1;
    const int cg = w1 ? cg1 : cg2;
    const int ob = bb / cg, ig = bb % cg;
    const int i0 = ig * WG_COLS;
    const int ncols = w1 ? D0 : D1;
    const TileState st = tile_prefetch(a, pS + (w1 ? a.off_w1 : a.off_w2), ncols, ob * 16, i0, ncols);
    if (w1) {
      // ---- stage the X slab row-major: sX[r][j] = Xb[step row r][i0 + j] as bf16 (0 outside);
      //      a wave covers 2 rows x 256 contiguous bytes per load instruction.
      for (int e = threadIdx.x; e < Bp * (WG_COLS / 8); e += 256) {
        const int r = e / (WG_COLS / 8), q = e % (WG_COLS / 8);
        uint2 v = {0u, 0u};
        const int col = i0 + q * 8;
        if (r < rows && col < D0) v = *reinterpret_cast<const uint2*>(a.Xb + batch_row(a, p, step, r) * (int64_t)D0 + col);
        bf16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (bf16)(float)(((j < 4 ? v.x : v.y) >> (8 * (j & 3))) & 0xffu);
        *reinterpret_cast<bf16x8*>(&sX[r * WG_LDXR + q * 8]) = o;
      }
      lds_barrier();
    }
    MLP_STAMP(2, 1);
    // dW[o][i] = Σ_b A[o][b] · B[i][b]:  A = dH1ᵀ (W1) or dH2ᵀ (W2); B = Xᵀ slab in LDS (W1) or H1ᵀ (W2)
    const bf16* A = (w1 ? a.dH1T + (int64_t)p * D1 * Bp : a.dH2T + (int64_t)p * D2 * Bp) + (int64_t)(ob * 16 + c) * Bp;
    f32x4 acc[WG_NT];
#pragma unroll
    for (int t = 0; t < WG_NT; ++t) acc[t] = zero4();
    float bsum = 0.f;
    for (int k0 = 0; k0 < Bp; k0 += 32) {
      const bf16x8 av = ld8(A + k0 + 8 * h);
      if (ig == 0 && wave == 0) bsum += frag_sum(av);
#pragma unroll
      for (int t = 0; t < WG_NT; ++t) {
        const int i = i0 + (wave * WG_NT + t) * 16;  // first column of this n-tile
        if (i >= ncols) continue;
        const bf16x8 bv = w1 ? frag_b_tr(sX, WG_LDXR, k0, (wave * WG_NT + t) * 16)
                             : ld8(a.H1T + (int64_t)p * D1 * Bp + (int64_t)(i + c) * Bp + k0 + 8 * h);
        acc[t] = mfma_bf16(av, bv, acc[t]);
      }
    }
#pragma unroll
    for (int t = 0; t < WG_NT; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) sG[(4 * h + r) * WG_LDG + (wave * WG_NT + t) * 16 + c] = acc[t][r];
    if (ig == 0 && wave == 0) {
      bsum += __shfl_xor(bsum, 16);
      bsum += __shfl_xor(bsum, 32);
      if (h == 0) update_elem(a, pS + (w1 ? a.off_b1 : a.off_b2) + ob * 16 + c, bsum, bc1, bc2s);
    }
    lds_barrier();
    MLP_STAMP(2, 2);
    tile_apply(a, st, sG, bc1, bc2s, !w1, p);
    MLP_STAMP(2, 3);
    return;
  }
  // ---- W3 tiles: dW3[cls][o2] = Σ_b dlogitsᵀ[cls][b] · H2ᵀ[o2][b]  (classes padded to 16)
  const int t = (b - nb1 - nb2) * WG_WAVES + wave;
  if (t >= D2 / 16) return;
  const bf16* A = a.dlogT + (int64_t)p * 16 * Bp + (int64_t)c * Bp;
  const bf16* Bm = a.H2T + (int64_t)p * D2 * Bp + (int64_t)(t * 16 + c) * Bp;
  f32x4 acc = zero4();
  float bsum = 0.f;
  for (int k0 = 0; k0 < Bp; k0 += 32) {
    const bf16x8 av = ld8(A + k0 + 8 * h);
    if (t == 0) bsum += frag_sum(av);
    acc = mfma_bf16(av, ld8(Bm + k0 + 8 * h), acc);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int cls = 4 * h + r;
    if (cls < D3) update_elem(a, pS + a.off_w3 + (int64_t)cls * D2 + t * 16 + c, acc[r], bc1, bc2s);
  }
  if (t == 0) {
    bsum += __shfl_xor(bsum, 16);
    bsum += __shfl_xor(bsum, 32);
    if (h == 0 && c < D3) update_elem(a, pS + a.off_b3 + c, bsum, bc1, bc2s);
  }
}

// Keyed pseudo-random permutation of [0, n): 4-round balanced Feistel network on the smallest even
// bit width covering n, cycle-walked back into range (expected < 4 rounds of walking). Used to draw
// each peer's epoch order without a host-side sort.
__device__ __forceinline__ unsigned mix32(unsigned x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
__device__ unsigned feistel_perm(unsigned x, unsigned n, unsigned long long key) {
  if (n <= 1) return 0;
  int bits = 32 - __clz(n - 1);
  if (bits < 2) bits = 2;
  if (bits & 1) ++bits;
  const int half = bits / 2;
  const unsigned mask = (1u << half) - 1u;
  const unsigned k0 = (unsigned)key, k1 = (unsigned)(key >> 32);
  unsigned y = x;
  do {
    unsigned L = y >> half, R = y & mask;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const unsigned f = mix32(R ^ ((r & 1) ? k1 : k0) ^ (0x9e3779b9u * (unsigned)(r + 1))) & mask;
      const unsigned t = L ^ f;
      L = R;
      R = t;
    }
    y = (L << half) | R;
  } while (y >= n);
  return y;
}

// ---------------------------------------------------------------------------------------------
// epoch gather: Xb[p][i] = X_p[perm_p[i]], Yb[p][i] = Y_p[perm_p[i]] for i < n_p (first node of
// every epoch graph). grid = (ceil(xb_rows / 4), 1, P), block = 256 = 4 rows x 64 lanes (8 B each).
// ---------------------------------------------------------------------------------------------
constexpr int GATHER_RPW = 4;  // rows per wave: their loads are in flight together
__global__ __launch_bounds__(256) void mlp_gather_epoch(MLPArgs a) {
  const int p = blockIdx.z;
  const int n = a.ctl[p].y;
  const int lane = threadIdx.x & 63;
  if (a.flags_zero != nullptr && blockIdx.x == 0)  // the persistent epoch's flags start at 0 (replaces a memset node)
    for (int q = threadIdx.x; q < a.flags_per_peer; q += 256) a.flags_zero[(int64_t)p * a.flags_per_peer + q] = 0u;
  if (!a.ctl[p].x) return;
  const int nblk = (a.xb_rows + 4 * GATHER_RPW - 1) / (4 * GATHER_RPW);
  // grid-stride over the row blocks: a capped grid (the gather ahead of an epoch) leaves the CUs
  // the running epoch's gangs hold alone
  for (int blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
  const int i0 = (blk * 4 + (threadIdx.x >> 6)) * GATHER_RPW;
  const uint8_t* xp = a.Xp[p];
  const int* yp = a.Yp[p];
  constexpr int QPL = 4;  // uint2 pieces per lane per row (D0 <= 2048)
  int64_t src[GATHER_RPW];
#pragma unroll
  for (int r = 0; r < GATHER_RPW; ++r) {
    const int i = i0 + r;
    const bool ok = i < n && i < a.xb_rows;
    src[r] = !ok ? -1
                 : (a.shuffle_native ? (int64_t)feistel_perm((unsigned)i, (unsigned)n, *a.seed ^ (0x9e3779b97f4a7c15ull * (unsigned long long)(p + 1)))
                                     : (int64_t)a.perm[(int64_t)p * a.perm_stride + i]);
  }
  uint2 v[GATHER_RPW][QPL];
#pragma unroll
  for (int r = 0; r < GATHER_RPW; ++r)
#pragma unroll
    for (int k = 0; k < QPL; ++k) {
      const int q = lane + 64 * k;
      v[r][k] = (src[r] >= 0 && q < a.D0 / 8) ? reinterpret_cast<const uint2*>(xp + src[r] * (int64_t)a.D0)[q] : uint2{0u, 0u};
    }
#pragma unroll
  for (int r = 0; r < GATHER_RPW; ++r) {
    if (src[r] < 0) continue;
    const int64_t row = (int64_t)p * a.xb_rows + i0 + r;
#pragma unroll
    for (int k = 0; k < QPL; ++k) {
      const int q = lane + 64 * k;
      if (q >= a.D0 / 8) continue;
      if (a.Xb16 == nullptr) {  // uint8 rows for the step path
        reinterpret_cast<uint2*>(a.Xb + row * a.D0)[q] = v[r][k];
      } else {  // bf16 rows for the persistent epoch kernel (converted once per epoch; it never reads Xb)
        bf16x8 h;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          h[j] = (bf16)(float)((v[r][k].x >> (8 * j)) & 0xffu);
          h[4 + j] = (bf16)(float)((v[r][k].y >> (8 * j)) & 0xffu);
        }
        reinterpret_cast<bf16x8*>(a.Xb16 + row * a.D0)[q] = h;
      }
    }
    if (lane == 0) a.Yb[row] = yp[src[r]];
  }
  }
}

// direct-X epochs: xidx[p][i] = perm_p(i) and Yb[p][i] = Y_p[perm_p(i)] (no image rows move: the
// fp32 epoch kernel reads them from the static bf16 copy through xidx). grid = (ceil(xb_rows / 256),
// 1, P), block 256.
__global__ __launch_bounds__(256) void mlp_index_epoch(MLPArgs a) {
  const int p = blockIdx.z;
  const int n = a.ctl[p].y;
  if (a.flags_zero != nullptr && blockIdx.x == 0)
    for (int q = threadIdx.x; q < a.flags_per_peer; q += 256) a.flags_zero[(int64_t)p * a.flags_per_peer + q] = 0u;
  if (!a.ctl[p].x) return;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n || i >= a.xb_rows) return;
  const int src = a.shuffle_native ? (int)feistel_perm((unsigned)i, (unsigned)n, *a.seed ^ (0x9e3779b97f4a7c15ull * (unsigned long long)(p + 1)))
                                   : a.perm[(int64_t)p * a.perm_stride + i];
  a.xidx[(int64_t)p * a.xb_rows + i] = src;
  a.Yb[(int64_t)p * a.xb_rows + i] = a.Yp[p][src];
}

void mlp_launch_index_epoch(const MLPArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(mlp_index_epoch, dim3((unsigned)((a.xb_rows + 255) / 256), 1, a.P), dim3(256), 0, s, a);
}

void mlp_launch_gather_epoch(const MLPArgs& a, hipStream_t s, int max_wgs) {
  const int64_t waves = (a.xb_rows + GATHER_RPW - 1) / GATHER_RPW;
  int64_t gx = (waves + 3) / 4;
  if (max_wgs > 0) {
    const int64_t cap = max_wgs / a.P > 0 ? max_wgs / a.P : 1;
    if (gx > cap) gx = cap;
  }
  hipLaunchKernelGGL(mlp_gather_epoch, dim3((unsigned)gx, 1, a.P), dim3(256), 0, s, a);
}

// ---------------------------------------------------------------------------------------------
// shadow refresh: bf16 copy of every parameter + W2ᵀ (after params change outside the engine)
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void mlp_sync_shadow(MLPArgs a) {
  const int p = blockIdx.y;
  const int64_t pS = (int64_t)p * a.S;
  const int64_t n = a.numel;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const bf16 v = (bf16)a.params[pS + i];
    a.shadow[pS + i] = v;
    const int64_t j = i - a.off_w2;
    if (j >= 0 && j < (int64_t)a.D1 * a.D2) {
      const int o2 = (int)(j / a.D1), o1 = (int)(j % a.D1);
      a.w2t[(int64_t)p * a.D1 * a.D2 + (int64_t)o1 * a.D2 + o2] = v;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// host-side launchers
// ---------------------------------------------------------------------------------------------
template <int TP1, int TP2>
static void launch_head(const MLPArgs& a, int step, int base, bool train, int rows, hipStream_t s) {
  dim3 grid(rows / 16, 1, a.P);
  if (train)
    hipLaunchKernelGGL((mlp_head<TP1, TP2, true>), grid, dim3(256), 0, s, a, step, base);
  else
    hipLaunchKernelGGL((mlp_head<TP1, TP2, false>), grid, dim3(256), 0, s, a, step, base);
}

bool mlp_shape_supported(int D0, int D1, int D2, int D3) {
  if (D0 <= 0 || D0 % 8 != 0 || D0 > 2048 || D3 < 1 || D3 > 16) return false;
  const int t1 = D1 / 64, t2 = D2 / 64;
  if (D1 % 64 || D2 % 64) return false;
  return (t1 == 4 && t2 == 2) || (t1 == 2 && t2 == 1) || (t1 == 4 && t2 == 4) || (t1 == 8 && t2 == 4) || (t1 == 2 && t2 == 2) ||
         (t1 == 1 && t2 == 1) || (t1 == 8 && t2 == 2);
}

static void launch_head_dispatch(const MLPArgs& a, int step, int base, bool train, int rows, hipStream_t s) {
  const int t1 = a.D1 / 64, t2 = a.D2 / 64;
  if (t1 == 4 && t2 == 2) launch_head<4, 2>(a, step, base, train, rows, s);
  else if (t1 == 2 && t2 == 1) launch_head<2, 1>(a, step, base, train, rows, s);
  else if (t1 == 4 && t2 == 4) launch_head<4, 4>(a, step, base, train, rows, s);
  else if (t1 == 8 && t2 == 4) launch_head<8, 4>(a, step, base, train, rows, s);
  else if (t1 == 2 && t2 == 2) launch_head<2, 2>(a, step, base, train, rows, s);
  else if (t1 == 1 && t2 == 1) launch_head<1, 1>(a, step, base, train, rows, s);
  else if (t1 == 8 && t2 == 2) launch_head<8, 2>(a, step, base, train, rows, s);
}

void mlp_launch_train_step(const MLPArgs& a, int step, hipStream_t s) {
  hipLaunchKernelGGL((mlp_fc1_fwd<true>), dim3(a.D1 / 32, a.Bpad / 32, a.P), dim3(256), 0, s, a, step, 0);
  launch_head_dispatch(a, step, 0, true, a.Bpad, s);
  const int nb1 = (a.D1 / 16) * ((a.D0 + WG_COLS - 1) / WG_COLS);
  const int nb2 = (a.D2 / 16) * ((a.D1 + WG_COLS - 1) / WG_COLS);
  const int nb3 = (a.D2 / 16 + WG_WAVES - 1) / WG_WAVES;
  hipLaunchKernelGGL(mlp_wgrad_opt, dim3(nb1 + nb2 + nb3, 1, a.P), dim3(256), wgrad_lds_bytes(a.Bpad), s, a, step);
}

void mlp_launch_eval_chunk(const MLPArgs& a, int base, hipStream_t s) {
  hipLaunchKernelGGL((mlp_fc1_fwd<false>), dim3(a.D1 / 32, MLP_EVAL_CHUNK / 32, a.P), dim3(256), 0, s, a, 0, base);
  launch_head_dispatch(a, 0, base, false, MLP_EVAL_CHUNK, s);
}

void mlp_launch_sync_shadow(const MLPArgs& a, hipStream_t s) {
  const int64_t blocks = (a.numel + 255) / 256;
  hipLaunchKernelGGL(mlp_sync_shadow, dim3((unsigned)(blocks < 1024 ? blocks : 1024), a.P), dim3(256), 0, s, a);
}

// Resolve one kernel of this translation unit on the current device: loads the unit's code object
// now (myfyp_warm_all, at engine prewarm) instead of at its first launch, which waited for the
// kernels in flight (the first FedAvg launch blocked the host until the running epoch ended)
extern "C" int myfyp_warm_mlp_fused() {
  hipFuncAttributes attr;
  return hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(&mlp_wgrad_opt)) == hipSuccess ? 0 : 1;
}
