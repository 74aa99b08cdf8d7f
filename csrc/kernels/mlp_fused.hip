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

namespace {

__device__ __forceinline__ int rows_valid_train(const MLPArgs& a, int p, int step) {
  int r = a.n[p] - step * a.B;
  return r < 0 ? 0 : (r > a.B ? a.B : r);
}

__device__ __forceinline__ int rows_valid_eval(const MLPArgs& a, int p, int base) {
  int r = a.n_t[p] - base;
  return r < 0 ? 0 : (r > MLP_EVAL_CHUNK ? MLP_EVAL_CHUNK : r);
}

// local sample index of batch row r
__device__ __forceinline__ int64_t sample_index(const MLPArgs& a, bool train, int p, int step, int base, int r) {
  if (train) return a.perm[(int64_t)p * a.perm_stride + (int64_t)step * a.B + r];
  return base + r;
}

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
  constexpr int MT = 2, NT = 2, KCH = 8;
  __shared__ __attribute__((aligned(16))) float sRed[3][64][MT * NT * 4];
  const int p = blockIdx.z;
  if (!a.active[p]) return;
  const int rows = TRAIN ? rows_valid_train(a, p, step) : rows_valid_eval(a, p, base);
  if (rows == 0) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 4, c = lane & 15;
  const int row0 = blockIdx.y * 32;
  const int col0 = blockIdx.x * 32;
  const int D0 = a.D0, D1 = a.D1;
  const uint8_t* X = TRAIN ? a.Xp[p] : a.Xtp[p];

  const uint8_t* arow[MT];
  bool avalid[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) {
    const int r = row0 + mt * 16 + c;
    avalid[mt] = r < rows;
    arow[mt] = avalid[mt] ? X + sample_index(a, TRAIN, p, step, base, r) * (int64_t)D0 : X;
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

  // cross-wave K reduction
  if (wave > 0) {
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int i = 0; i < 4; ++i) sRed[wave - 1][lane][(mt * NT + nt) * 4 + i] = acc[mt][nt][i];
  }
  __syncthreads();
  if (wave != 0) return;
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
    const float bias = a.params[(int64_t)p * a.S + a.off_b1 + col];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
      bf16x4 packed;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = row0 + mt * 16 + 4 * h + i;
        float v = fmaxf(acc[mt][nt][i] + bias, 0.f);
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
}

// ---------------------------------------------------------------------------------------------
// K2: head. grid = (rows/16, 1, P), block = 256. TP2 = D2/64, TP1 = D1/64 column tiles per wave.
// ---------------------------------------------------------------------------------------------
template <int TP1, int TP2, bool TRAIN>
__global__ __launch_bounds__(256) void mlp_head(MLPArgs a, int step, int base) {
  constexpr int D1 = TP1 * 64, D2 = TP2 * 64;
  constexpr int LD2 = D2 + 8;  // padded LDS row (bf16) to spread banks
  constexpr int LDD = 32 + 8;
  __shared__ __attribute__((aligned(16))) bf16 sH2[16 * LD2];
  __shared__ __attribute__((aligned(16))) bf16 sDH2[16 * LD2];
  __shared__ __attribute__((aligned(16))) bf16 sDlog[16 * LDD];

  const int p = blockIdx.z;
  if (!a.active[p]) return;
  const int rows = TRAIN ? rows_valid_train(a, p, step) : rows_valid_eval(a, p, base);
  if (rows == 0) return;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 4, c = lane & 15;
  const int row0 = blockIdx.x * 16;
  const int D3 = a.D3;
  const int64_t pS = (int64_t)p * a.S;
  const bf16* H1 = a.H1 + (int64_t)p * a.h1_rows * D1;

  // zero the dlogits tile (k columns 16..31 stay zero = K padding)
  for (int i = threadIdx.x; i < 16 * LDD; i += 256) sDlog[i] = (bf16)0.f;

  // ---- H2 = relu(H1 · W2ᵀ + b2): wave owns column tiles {wave + 4*t}
  f32x4 h2[TP2];
#pragma unroll
  for (int t = 0; t < TP2; ++t) h2[t] = zero4();
  const bf16* arow = H1 + (int64_t)(row0 + c) * D1;
#pragma unroll
  for (int k0 = 0; k0 < D1; k0 += 32) {
    const bf16x8 av = ld8(arow + k0 + 8 * h);
#pragma unroll
    for (int t = 0; t < TP2; ++t) {
      const int n = (wave + 4 * t) * 16 + c;
      const bf16x8 bv = ld8(a.shadow + pS + a.off_w2 + (int64_t)n * D1 + k0 + 8 * h);
      h2[t] = mfma_bf16(av, bv, h2[t]);
    }
  }
#pragma unroll
  for (int t = 0; t < TP2; ++t) {
    const int col = (wave + 4 * t) * 16 + c;
    const float bias = a.params[pS + a.off_b2 + col];
    bf16x4 packed;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 4 * h + i;
      float v = fmaxf(h2[t][i] + bias, 0.f);
      if (row0 + r >= rows) v = 0.f;
      h2[t][i] = v;
      packed[i] = (bf16)v;
      sH2[r * LD2 + col] = packed[i];
    }
    if (TRAIN) *reinterpret_cast<bf16x4*>(a.H2T + (int64_t)p * D2 * a.Bpad + (int64_t)col * a.Bpad + row0 + 4 * h) = packed;
  }
  __syncthreads();

  // ---- logits, log-softmax, NLL, argmax, dlogits (wave 0)
  if (wave == 0) {
    f32x4 lg = zero4();
    const bool cin = c < D3;
#pragma unroll
    for (int k0 = 0; k0 < D2; k0 += 32) {
      const bf16x8 av = *reinterpret_cast<const bf16x8*>(&sH2[c * LD2 + k0 + 8 * h]);
      const bf16x8 bv = cin ? ld8(a.shadow + pS + a.off_w3 + (int64_t)c * D2 + k0 + 8 * h) : zero_bf16x8();
      lg = mfma_bf16(av, bv, lg);
    }
    const float b3 = cin ? a.params[pS + a.off_b3 + c] : 0.f;
    float loss_part = 0.f;
    int correct_part = 0;
    bf16x4 dpack;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = 4 * h + i;
      const int grow = row0 + r;
      const bool rvalid = grow < rows;
      const float logit = cin ? lg[i] + b3 : -INFINITY;
      const float mx = warp_max16(logit);
      const float se = warp_sum16(cin ? __expf(logit - mx) : 0.f);
      const float lse = mx + __logf(se);
      const float logp = logit - lse;
      int y = -1;
      if (rvalid) {
        const int64_t idx = sample_index(a, TRAIN, p, step, base, grow);
        y = TRAIN ? a.Yp[p][idx] : a.Ytp[p][idx];
      }
      // argmax (first max), reduced over the 16 lanes of this row
      int cand = (cin && logit == mx) ? c : 16;
      cand = min(cand, __shfl_xor(cand, 1));
      cand = min(cand, __shfl_xor(cand, 2));
      cand = min(cand, __shfl_xor(cand, 4));
      cand = min(cand, __shfl_xor(cand, 8));
      if (rvalid && c == y) loss_part -= logp;
      if (rvalid && c == 0) {
        correct_part += (cand == y);
        if (!TRAIN && a.conf != nullptr && y >= 0 && y < 16 && cand < 16) atomicAdd(&a.conf[(p * 16 + y) * 16 + cand], 1);
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
  __syncthreads();

  // ---- dH2 = dlogits · W3 ⊙ [H2 > 0]   (K = 16 classes, padded to 32)
  {
    bf16x8 av = *reinterpret_cast<const bf16x8*>(&sDlog[c * LDD + 8 * h]);
#pragma unroll
    for (int t = 0; t < TP2; ++t) {
      const int n = (wave + 4 * t) * 16 + c;
      bf16x8 bv;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int k = 8 * h + j;
        bv[j] = k < D3 ? a.shadow[pS + a.off_w3 + (int64_t)k * D2 + n] : (bf16)0.f;
      }
      f32x4 acc = mfma_bf16(av, bv, zero4());
      bf16x4 packed;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v = h2[t][i] > 0.f ? acc[i] : 0.f;
        packed[i] = (bf16)v;
        sDH2[(4 * h + i) * LD2 + n] = packed[i];
      }
      *reinterpret_cast<bf16x4*>(a.dH2T + (int64_t)p * D2 * a.Bpad + (int64_t)n * a.Bpad + row0 + 4 * h) = packed;
    }
  }
  __syncthreads();

  // ---- dH1 = dH2 · W2 ⊙ [H1 > 0]   (B operand from the transposed shadow W2ᵀ [D1][D2])
  const bf16* w2t = a.w2t + (int64_t)p * D1 * D2;
#pragma unroll
  for (int t = 0; t < TP1; ++t) {
    const int n = (wave + 4 * t) * 16 + c;
    f32x4 acc = zero4();
#pragma unroll
    for (int k0 = 0; k0 < D2; k0 += 32) {
      const bf16x8 av = *reinterpret_cast<const bf16x8*>(&sDH2[c * LD2 + k0 + 8 * h]);
      const bf16x8 bv = ld8(w2t + (int64_t)n * D2 + k0 + 8 * h);
      acc = mfma_bf16(av, bv, acc);
    }
    bf16x4 packed;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float h1 = (float)H1[(int64_t)(row0 + 4 * h + i) * D1 + n];
      packed[i] = (bf16)(h1 > 0.f ? acc[i] : 0.f);
    }
    *reinterpret_cast<bf16x4*>(a.dH1T + (int64_t)p * D1 * a.Bpad + (int64_t)n * a.Bpad + row0 + 4 * h) = packed;
  }
}

// ---------------------------------------------------------------------------------------------
// K3: weight gradients + optimizer. grid = (nb_w1 + nb_w2 + 1, 1, P), block = 256.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void step_bias_corr(const MLPArgs& a, int p, int step, float& bc1, float& bc2s) {
  const int t = a.t0[p] + step + 1;
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

// Block decomposition (grid.x): [0, nb1) W1 blocks — 4 tiles sharing one 16-column slab of X
// (staged once, transposed to bf16 in LDS) and 4 different 16-row blocks of W1; [nb1, nb1+nb2)
// W2 blocks — 4 tiles each; [nb1+nb2, +nb3) W3 blocks. Bias gradients are row sums of the A
// fragments and are produced by the waves whose column slab is 0.
__device__ __forceinline__ float frag_sum(const bf16x8& v) {
  float s = 0.f;
#pragma unroll
  for (int j = 0; j < 8; ++j) s += (float)v[j];
  return s;
}

__global__ __launch_bounds__(256) void mlp_wgrad_opt(MLPArgs a, int step) {
  constexpr int LDX = MLP_MAX_BPAD + 8;
  __shared__ __attribute__((aligned(16))) bf16 sX[16 * LDX];
  const int p = blockIdx.z;
  if (!a.active[p]) return;
  const int rows = rows_valid_train(a, p, step);
  if (rows == 0) return;
  float bc1, bc2s;
  step_bias_corr(a, p, step, bc1, bc2s);
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int h = lane >> 4, c = lane & 15;
  const int D0 = a.D0, D1 = a.D1, D2 = a.D2, D3 = a.D3, Bp = a.Bpad;
  const int64_t pS = (int64_t)p * a.S;
  const int tiles_i = (D0 + 15) / 16;
  const int obg = D1 / 64;  // groups of 4 row-blocks of W1
  const int nb1 = tiles_i * obg;
  const int nb2 = (D2 / 16) * (D1 / 16) / 4;
  const int b = blockIdx.x;

  if (b < nb1) {
    const int ib = b / obg, og = b % obg;
    const int ob = og * 4 + wave;
    // stage Xᵀ slab: sX[j][r] = X[sample(r)][ib*16 + j] (bf16), zero for invalid rows / cols ≥ D0
    for (int r = threadIdx.x; r < Bp; r += 256) {
      uint4 v = {0u, 0u, 0u, 0u};
      const int i0 = ib * 16;
      if (r < rows) {
        const uint8_t* src = a.Xp[p] + sample_index(a, true, p, step, 0, r) * (int64_t)D0 + i0;
        if (i0 + 16 <= D0) {
          const uint2 lo = *reinterpret_cast<const uint2*>(src), hi = *reinterpret_cast<const uint2*>(src + 8);
          v = uint4{lo.x, lo.y, hi.x, hi.y};
        } else {
          uint8_t tmp[16] = {0};
          for (int j = 0; j < 16 && i0 + j < D0; ++j) tmp[j] = src[j];
          v = *reinterpret_cast<const uint4*>(tmp);
        }
      }
      const uint32_t w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 16; ++j) sX[j * LDX + r] = (bf16)(float)((w4[j >> 2] >> (8 * (j & 3))) & 0xffu);
    }
    __syncthreads();
    const bf16* A = a.dH1T + (int64_t)p * D1 * Bp + (int64_t)(ob * 16 + c) * Bp;
    f32x4 acc = zero4();
    float bsum = 0.f;
    for (int k0 = 0; k0 < Bp; k0 += 32) {
      const bf16x8 av = ld8(A + k0 + 8 * h);
      const bf16x8 bv = *reinterpret_cast<const bf16x8*>(&sX[c * LDX + k0 + 8 * h]);
      if (ib == 0) bsum += frag_sum(av);
      acc = mfma_bf16(av, bv, acc);
    }
    const int i = ib * 16 + c;
    if (i < D0) {
#pragma unroll
      for (int r = 0; r < 4; ++r) update_elem(a, pS + a.off_w1 + (int64_t)(ob * 16 + 4 * h + r) * D0 + i, acc[r], bc1, bc2s);
    }
    if (ib == 0) {
      bsum += __shfl_xor(bsum, 16);
      bsum += __shfl_xor(bsum, 32);
      if (h == 0) update_elem(a, pS + a.off_b1 + ob * 16 + c, bsum, bc1, bc2s);
    }
    return;
  }
  if (b < nb1 + nb2) {
    // ---- W2 tile: dW2[o2][o1] = Σ_b dH2ᵀ[o2][b] · H1ᵀ[o1][b]; also refresh the W2ᵀ shadow
    const int tile = (b - nb1) * 4 + wave;
    const int ob = tile / (D1 / 16), ib = tile % (D1 / 16);
    const bf16* A = a.dH2T + (int64_t)p * D2 * Bp + (int64_t)(ob * 16 + c) * Bp;
    const bf16* Bm = a.H1T + (int64_t)p * D1 * Bp + (int64_t)(ib * 16 + c) * Bp;
    f32x4 acc = zero4();
    float bsum = 0.f;
    for (int k0 = 0; k0 < Bp; k0 += 32) {
      const bf16x8 av = ld8(A + k0 + 8 * h);
      if (ib == 0) bsum += frag_sum(av);
      acc = mfma_bf16(av, ld8(Bm + k0 + 8 * h), acc);
    }
    const int o1 = ib * 16 + c;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int o2 = ob * 16 + 4 * h + r;
      const int64_t idx = pS + a.off_w2 + (int64_t)o2 * D1 + o1;
      update_elem(a, idx, acc[r], bc1, bc2s);
      a.w2t[(int64_t)p * D1 * D2 + (int64_t)o1 * D2 + o2] = a.shadow[idx];
    }
    if (ib == 0) {
      bsum += __shfl_xor(bsum, 16);
      bsum += __shfl_xor(bsum, 32);
      if (h == 0) update_elem(a, pS + a.off_b2 + ob * 16 + c, bsum, bc1, bc2s);
    }
    return;
  }
  // ---- W3 tiles: dW3[cls][o2] = Σ_b dlogitsᵀ[cls][b] · H2ᵀ[o2][b]  (classes padded to 16)
  const int t = (b - nb1 - nb2) * 4 + wave;
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
  if (D0 <= 0 || D0 % 8 != 0 || D3 < 1 || D3 > 16) return false;
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
  const int nb1 = ((a.D0 + 15) / 16) * (a.D1 / 64);
  const int nb2 = (a.D2 / 16) * (a.D1 / 16) / 4;
  const int nb3 = (a.D2 / 16 + 3) / 4;
  hipLaunchKernelGGL(mlp_wgrad_opt, dim3(nb1 + nb2 + nb3, 1, a.P), dim3(256), 0, s, a, step);
}

void mlp_launch_eval_chunk(const MLPArgs& a, int base, hipStream_t s) {
  hipLaunchKernelGGL((mlp_fc1_fwd<false>), dim3(a.D1 / 32, MLP_EVAL_CHUNK / 32, a.P), dim3(256), 0, s, a, 0, base);
  launch_head_dispatch(a, 0, base, false, MLP_EVAL_CHUNK, s);
}

void mlp_launch_sync_shadow(const MLPArgs& a, hipStream_t s) {
  const int64_t blocks = (a.numel + 255) / 256;
  hipLaunchKernelGGL(mlp_sync_shadow, dim3((unsigned)(blocks < 1024 ? blocks : 1024), a.P), dim3(256), 0, s, a);
}
