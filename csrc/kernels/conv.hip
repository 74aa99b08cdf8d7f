// Implicit-GEMM convolutions on MFMA (gfx950, wave64), grouped over co-located peers.
//
// k_conv_gemm<MODE, BN>: C[M][Ncol] = A[M][K] · B[K][Ncol]
//   MODE 0 (forward) : rows = output pixels, A = im2col(X) gathered on the fly, K = (r, s, ci),
//                      B = Wf[co][r][s][ci] rows (K-contiguous), staged [n][k] XOR-swizzled
//   MODE 1 (dgrad)   : rows = input pixels,  A = dY gathered at ((h+pad-r)/st, (w+pad-s)/st) when
//                      divisible (zero otherwise), K = (r, s, co); B[k][ci] = Wf[co][r][s][ci] is
//                      N-contiguous, staged [k][n] and read as MFMA fragments with the gfx950 LDS
//                      transpose read (ds_read_b64_tr_b16) — no transposed weight copy exists
//   128 x BN tile, BK = 64, 256 threads = 4 waves (2 x 2), 16x16x32 bf16 MFMA, fp32 accumulate.
//   A is register-staged into a double-buffered LDS image whose 16-byte chunks are XOR-swizzled
//   (chunk ^ ((row >> 1) & 7)) so every ds_read_b128 fragment read is conflict-free; one barrier
//   per K-step (the next tile's global loads are in flight during the MFMAs).
//   Fused epilogue: + bias, + residual, ReLU, zeroed channel padding, BatchNorm sums (atomics).
//   XCD-aware bijective block remap so tiles sharing an operand panel land on one L2.
//
// k_conv_wgrad<BM, BN>: dW[co][(r,s,ci)] = sum_m dY[m][co] · im2col(X)[m][(r,s,ci)]
//   K = pixels (split over blockIdx.y), both operands staged [m][channels] as loaded and read
//   as MFMA fragments with the transposed LDS read. The gradient is written in the GEMM's own
//   (Wf) layout [cp_out][R][S][cp_in] fp32: 16 lanes of a row write 64 contiguous bytes (plain
//   stores when the pixel dimension is not split, fp32 atomics otherwise). The optimizer kernel
//   maps it to torch order through LDS (a torch-order scatter here cost ~0.45 ms per layer).
#include <hip/hip_runtime.h>

#include "conv.h"

#define CG_BM 128
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

__device__ __forceinline__ int swz(int row, int chunk) { return row * CG_BK + ((chunk ^ ((row >> 1) & 7)) << 3); }

template <int MODE, int BN>
__global__ __launch_bounds__(256) void k_conv_gemm(ConvGemmArgs a, int tiles_m, int tiles_n) {
  constexpr int NB = BN / 32;          // B 16-byte chunks per thread
  constexpr int NF = BN / 32;          // n-fragments per wave (wave covers BN/2 columns)
  constexpr bool BT = MODE == 1;       // B staged [k][n] (N-contiguous source)
  constexpr int LBT = BN + 8;          // padded row stride of the [k][n] image
  constexpr int BSZ = BT ? CG_BK * LBT : BN * CG_BK;
  constexpr int BUF = CG_BM * CG_BK + BSZ;
  __shared__ __attribute__((aligned(16))) bf16 lds[2 * BUF];

  const int peer = blockIdx.z;
  const int nb = a.nbatch ? a.nbatch[peer] : a.max_batch;
  const int hw = a.out_h * a.out_w;
  const int M = nb * hw;
  const int wgid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tn = wgid % tiles_n, tm = wgid / tiles_n;
  const int m0 = tm * CG_BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;

  if (m0 >= M) return;  // tile past this peer's batch

  const bf16* src = a.src + peer * a.src_ps;
  const bf16* wt = a.wt + peer * a.wt_ps;
  const int Ktot = a.R * a.S * a.src_c;
  const int nk = (Ktot + CG_BK - 1) / CG_BK;
  const int cc = tid & 7;            // this thread's 16-byte chunk within a K-step
  const int cpp = a.src_c >> 3;      // chunks per pixel

  // per-thread A rows (fixed for the whole K loop)
  int a_img[4], a_bh[4], a_bw[4];
  bool a_ok[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = m0 + (tid >> 3) + 32 * i;
    a_ok[i] = m < M;
    const int mm = a_ok[i] ? m : 0;
    const int img = mm / hw, rem = mm - img * hw;
    const int oh = rem / a.out_w, ow = rem - oh * a.out_w;
    a_img[i] = img * a.src_h * a.src_w;
    if (MODE == 0) {
      a_bh[i] = oh * a.stride - a.pad;
      a_bw[i] = ow * a.stride - a.pad;
    } else {
      a_bh[i] = oh + a.pad;
      a_bw[i] = ow + a.pad;
    }
  }

  const float inv_cpp = 1.f / (float)cpp, inv_S = 1.f / (float)a.S, inv_st = 1.f / (float)a.stride;
  const float inv_srcc = 1.f / (float)a.src_c;
  constexpr int BCH = BN / 8;          // MODE 1: 16-byte chunks per staged k row
  const int bt_c = tid % BCH, bt_r = tid / BCH;
  uint4 ra[4], rb[NB];
  auto load = [&](int kt) {
    const int k = kt * CG_BK + cc * 8;
    const bool kok = k < Ktot;
    int r = 0, s = 0, c8 = 0;
    if (kok) {
      const int q8 = k >> 3;
      const int rs = fdiv(q8, cpp, inv_cpp);
      c8 = q8 - rs * cpp;
      r = fdiv(rs, a.S, inv_S);
      s = rs - r * a.S;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      bool ok = kok && a_ok[i];
      int h, w;
      if (MODE == 0) {
        h = a_bh[i] + r;
        w = a_bw[i] + s;
      } else {
        const int th = a_bh[i] - r, tw = a_bw[i] - s;
        h = th >= 0 ? fdiv(th, a.stride, inv_st) : -1;
        w = tw >= 0 ? fdiv(tw, a.stride, inv_st) : -1;
        ok = ok && th >= 0 && tw >= 0 && h * a.stride == th && w * a.stride == tw;
      }
      ok = ok && h >= 0 && w >= 0 && h < a.src_h && w < a.src_w;
      ra[i] = ok ? *reinterpret_cast<const uint4*>(src + (int64_t)(a_img[i] + h * a.src_w + w) * a.src_c + c8 * 8) : make_uint4(0, 0, 0, 0);
    }
    if (!BT) {
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int n = n0 + (tid >> 3) + 32 * i;
        rb[i] = (kok && n < a.ncol) ? *reinterpret_cast<const uint4*>(wt + (int64_t)n * Ktot + k) : make_uint4(0, 0, 0, 0);
      }
    } else {
      // k row = (r, s, co): Wf[co][rs][n0 + 8 * chunk ..] (ncol = Wf row length = cp_in)
      const int n = n0 + bt_c * 8;
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int kk = kt * CG_BK + bt_r + (256 / BCH) * i;
        bool ok = kk < Ktot && n < a.ncol;
        int64_t off = 0;
        if (ok) {
          const int rs = fdiv(kk, a.src_c, inv_srcc), co = kk - rs * a.src_c;
          off = ((int64_t)co * (a.R * a.S) + rs) * a.ncol + n;
        }
        rb[i] = ok ? *reinterpret_cast<const uint4*>(wt + off) : make_uint4(0, 0, 0, 0);
      }
    }
  };
  auto store = [&](int buf) {
    bf16* As = lds + buf * BUF;
    bf16* Bs = As + CG_BM * CG_BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<uint4*>(As + swz((tid >> 3) + 32 * i, cc)) = ra[i];
    if (!BT) {
#pragma unroll
      for (int i = 0; i < NB; ++i) *reinterpret_cast<uint4*>(Bs + swz((tid >> 3) + 32 * i, cc)) = rb[i];
    } else {
#pragma unroll
      for (int i = 0; i < NB; ++i) *reinterpret_cast<uint4*>(Bs + (bt_r + (256 / BCH) * i) * LBT + bt_c * 8) = rb[i];
    }
  };
  // transposed fragment (MODE 1 B): lane i of group g gets column (col0 + i), rows k0 + 8g + 0..7
  const int tg = lane >> 4, tq = (lane & 15) >> 2, tp = lane & 3;
  auto frag_t = [&](const bf16* base, int col0, int k0) -> bf16x8 {
    const bf16* p0 = base + (k0 + 8 * tg + tq) * LBT + col0 + 4 * tp;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0 + 4 * LBT));
    const s16x8 both = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, both);
  };

  f32x4 acc[4][NF];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < NF; ++j) acc[i][j] = zero4();

  load(0);
  store(0);
  __syncthreads();
  int cur = 0;
  for (int kt = 0; kt < nk; ++kt) {
    if (kt + 1 < nk) load(kt + 1);
    const bf16* As = lds + cur * BUF;
    const bf16* Bs = As + CG_BM * CG_BK;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int ch = h * 4 + (lane >> 4);
      bf16x8 af[4], bfr[NF];
#pragma unroll
      for (int i = 0; i < 4; ++i) af[i] = ld8(As + swz(wr * 64 + i * 16 + (lane & 15), ch));
#pragma unroll
      for (int j = 0; j < NF; ++j)
        bfr[j] = BT ? frag_t(Bs, wc * (BN / 2) + j * 16, h * 32) : ld8(Bs + swz(wc * (BN / 2) + j * 16 + (lane & 15), ch));
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
  bf16* out = a.out + peer * a.out_ps;
  const bf16* resid = a.resid ? a.resid + peer * a.resid_ps : nullptr;
  const float* bias = a.bias ? a.bias + peer * a.bias_ps : nullptr;
#pragma unroll
  for (int j = 0; j < NF; ++j) {
    const int col = n0 + wc * (BN / 2) + j * 16 + (lane & 15);
    const bool cok = col < a.ncol;
    const bool cvalid = col < a.ncol_valid;
    const float bv = (bias != nullptr && cvalid) ? bias[col] : 0.f;
    float s = 0.f, ss = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = m0 + wr * 64 + i * 16 + 4 * (lane >> 4) + e;
        if (row < M && cok) {
          float v = acc[i][j][e] + bv;
          if (resid != nullptr) v += (float)resid[(int64_t)row * a.ncol + col];
          if (a.relu) v = fmaxf(v, 0.f);
          if (!cvalid) v = 0.f;
          out[(int64_t)row * a.ncol + col] = (bf16)v;
          s += v;
          ss += v * v;
        }
      }
    }
    if (a.stats != nullptr) {
      // BatchNorm batch statistics: the wave's column sums go straight into the peer's [2][ncol]
      // accumulator (no partial-row slab, no serial reduction kernel; bn_finalize reads and re-zeroes it)
      s += __shfl_xor(s, 16);
      s += __shfl_xor(s, 32);
      ss += __shfl_xor(ss, 16);
      ss += __shfl_xor(ss, 32);
      if ((lane >> 4) == 0 && cok) {
        float* st = a.stats + peer * a.stats_ps;
        atomicAdd(st + col, s);
        atomicAdd(st + a.ncol + col, ss);
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------
// weight gradient
// ------------------------------------------------------------------------------------------------
template <int BM, int BN>
__global__ __launch_bounds__(256) void k_conv_wgrad(WgradArgs a, int tiles_m, int tiles_n) {
  constexpr int LA = BM + 8, LB = BN + 8;        // padded LDS row strides (elements)
  constexpr int FM = BM / 32, FN = BN / 32;       // fragments per wave
  constexpr int CA = BM / 8, CB = BN / 8;         // 16-byte chunks per staged row
  constexpr int NA = 64 * CA / 256, NBr = 64 * CB / 256;
  __shared__ __attribute__((aligned(16))) bf16 lds[2 * 64 * (LA + LB)];

  const int peer = blockIdx.z;
  const int nb = a.nbatch ? a.nbatch[peer] : a.max_batch;
  const int M = nb * a.Ho * a.Wo;
  const int kbeg = blockIdx.y * a.k_per_split;
  const int kend = min(M, kbeg + a.k_per_split);
  if (kbeg >= kend) return;
  const int wgid = xcd_remap(blockIdx.x, tiles_m * tiles_n);
  const int tn = wgid % tiles_n, tm = wgid / tiles_n;
  const int co0 = tm * BM, n0 = tn * BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;
  const bf16* dy = a.dy + peer * a.dy_ps;
  const bf16* x = a.x + peer * a.x_ps;
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

  const float inv_hwo = 1.f / (float)hwo, inv_wo = 1.f / (float)a.Wo;
  uint4 ra[NA], rb[NBr];
  auto load = [&](int m_base) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int m = m_base + tid / CA + (256 / CA) * i;
      ra[i] = (acol_ok && m < kend) ? *reinterpret_cast<const uint4*>(dy + (int64_t)m * a.dy_c + co0 + cca * 8) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < NBr; ++i) {
      const int m = m_base + tid / CB + (256 / CB) * i;
      bool ok = bcol_ok && m < kend;
      int64_t off = 0;
      if (ok) {
        const int img = fdiv(m, hwo, inv_hwo), rem = m - img * hwo;
        const int oh = fdiv(rem, a.Wo, inv_wo), ow = rem - oh * a.Wo;
        const int h = oh * a.stride - a.pad + br, w = ow * a.stride - a.pad + bs;
        ok = h >= 0 && w >= 0 && h < a.H && w < a.W;
        off = ((int64_t)(img * a.H + h) * a.W + w) * a.x_c + bci;
      }
      rb[i] = ok ? *reinterpret_cast<const uint4*>(x + off) : make_uint4(0, 0, 0, 0);
    }
  };
  auto store = [&](int buf) {
    bf16* As = lds + buf * 64 * (LA + LB);
    bf16* Bs = As + 64 * LA;
#pragma unroll
    for (int i = 0; i < NA; ++i) *reinterpret_cast<uint4*>(As + (tid / CA + (256 / CA) * i) * LA + cca * 8) = ra[i];
#pragma unroll
    for (int i = 0; i < NBr; ++i) *reinterpret_cast<uint4*>(Bs + (tid / CB + (256 / CB) * i) * LB + ccb * 8) = rb[i];
  };
  // transposed fragment: lane i of group g gets column (col0 + i), rows k0 + 8g + 0..7
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  auto frag_t = [&](const bf16* base, int ld, int col0, int k0) -> bf16x8 {
    const bf16* p0 = base + (k0 + 8 * g + q) * ld + col0 + 4 * p;
    const bf16* p1 = p0 + 4 * ld;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p0));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(p1));
    // whole-vector bit cast (an element-wise short->bf16 cast miscompiles into lane-duplicating perms)
    const s16x8 both = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(bf16x8, both);
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
    const bf16* As = lds + cur * 64 * (LA + LB);
    const bf16* Bs = As + 64 * LA;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) af[i] = frag_t(As, LA, wr * (BM / 2) + i * 16, h * 32);
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[j] = frag_t(Bs, LB, wc * (BN / 2) + j * 16, h * 32);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) acc[i][j] = mfma_bf16(af[i], bfr[j], acc[i][j]);
    }
    if (kt + 1 < nk) store(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  // Wf-layout gradient [dy_c][ncol_tot]: lanes 0..15 of a row group write 16 consecutive floats
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

// ------------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------------
extern "C" int conv_gemm_launch(int mode, const ConvGemmArgs* pa, int peers, void* stream) {
  const ConvGemmArgs& a = *pa;
  if ((a.src_c & 7) || (a.ncol & 7) || peers < 1) return 1;
  const int M = a.max_batch * a.out_h * a.out_w;
  const int tiles_m = (M + CG_BM - 1) / CG_BM;
  const bool wide = a.ncol > 64;
  const int BN = wide ? 128 : 64;
  const int tiles_n = (a.ncol + BN - 1) / BN;
  dim3 grid(tiles_m * tiles_n, 1, peers), block(256);
  hipStream_t s = (hipStream_t)stream;
  if (mode == 0) {
    if (wide) hipLaunchKernelGGL((k_conv_gemm<0, 128>), grid, block, 0, s, a, tiles_m, tiles_n);
    else hipLaunchKernelGGL((k_conv_gemm<0, 64>), grid, block, 0, s, a, tiles_m, tiles_n);
  } else {
    if (wide) hipLaunchKernelGGL((k_conv_gemm<1, 128>), grid, block, 0, s, a, tiles_m, tiles_n);
    else hipLaunchKernelGGL((k_conv_gemm<1, 64>), grid, block, 0, s, a, tiles_m, tiles_n);
  }
  return hipGetLastError() == hipSuccess ? 0 : 2;
}

// rows of the BN statistics buffer a conv epilogue writes: one (sum, sumsq) accumulator row
extern "C" int conv_gemm_stats_rows(int max_batch, int out_h, int out_w) { return 1; }

extern "C" int conv_wgrad_launch(const WgradArgs* pa, int peers, int splits, void* stream) {
  const WgradArgs& a = *pa;
  if ((a.x_c & 7) || (a.dy_c & 7) || (a.k_per_split & 63) || peers < 1 || splits < 1) return 1;
  if (splits > 1 && !a.accumulate) return 1;  // split-K partial sums must be added
  const int ncol = a.R * a.S * a.x_c;
  const bool wm = a.dy_c > 64, wn = ncol > 64;
  const int BM = wm ? 128 : 64, BN = wn ? 128 : 64;
  const int tiles_m = (a.dy_c + BM - 1) / BM, tiles_n = (ncol + BN - 1) / BN;
  dim3 grid(tiles_m * tiles_n, splits, peers), block(256);
  hipStream_t s = (hipStream_t)stream;
  if (wm && wn) hipLaunchKernelGGL((k_conv_wgrad<128, 128>), grid, block, 0, s, a, tiles_m, tiles_n);
  else if (wm) hipLaunchKernelGGL((k_conv_wgrad<128, 64>), grid, block, 0, s, a, tiles_m, tiles_n);
  else if (wn) hipLaunchKernelGGL((k_conv_wgrad<64, 128>), grid, block, 0, s, a, tiles_m, tiles_n);
  else hipLaunchKernelGGL((k_conv_wgrad<64, 64>), grid, block, 0, s, a, tiles_m, tiles_n);
  return hipGetLastError() == hipSuccess ? 0 : 2;
}
