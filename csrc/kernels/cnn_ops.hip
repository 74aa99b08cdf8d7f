// Memory-bound companions of the implicit-GEMM convolutions (grouped over peers, grid.y/z = peer):
// input gather + u8->bf16 NHWC conversion, BatchNorm (finalize / apply+residual+ReLU / backward
// reduce / finalize / apply), 2x2 max-pool and global average pool (fwd + bwd), log-softmax + NLL
// head (loss, correct, confusion, dlogits), and the fused SGD(+momentum/wd, FedProx, SCAFFOLD)
// update that also refreshes both bf16 weight shadows of every conv/fc layer in the same pass.
// All activation kernels move 16 bytes (8 bf16 channels) per lane.
#include <hip/hip_runtime.h>

#include "common.h"

struct bf8 { bf16 v[8]; };

__device__ __forceinline__ void unpack8(const uint4& u, float* f) {
  const bf8 b = __builtin_bit_cast(bf8, u);
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (float)b.v[j];
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  bf8 b;
#pragma unroll
  for (int j = 0; j < 8; ++j) b.v[j] = (bf16)f[j];
  return __builtin_bit_cast(uint4, b);
}

// ------------------------------------------------------------------------------------------------
// input: x_p[perm_p[offset + b]] (u8 HWC) -> bf16 [B][H][W][Cp] * scale ; labels -> int32; nb[p]
// ------------------------------------------------------------------------------------------------
// stop / fit_id (nullable): an interrupted fit (reference: a Lightning fit stopped mid-epoch,
// lightning_learner.py:110-114). stop is host-pinned memory the host writes while the epoch runs;
// a peer whose stop word equals its current fit id gets an empty batch from this step on, so every
// later kernel of the step (optimizer included: it skips peers with nb = 0) leaves it alone.
__global__ void k_input_prep(const uint8_t* const* xs, const int64_t* const* ys, const int* n_samples, const int* perm, int64_t perm_ps,
                             int offset, int B, int H, int W, int C, int Cp, float scale, bf16* out, int64_t out_ps, int* labels, int* nb,
                             const int* stop, const int* fit_id) {
  const int peer = blockIdx.y;
  const int n = n_samples[peer];
  const int valid = max(0, min(B, n - offset));
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    // one host-memory read per peer and step: the batch this block stages below is then simply unused
    const int fid = stop != nullptr ? fit_id[peer] : 0;
    const bool stopped = fid != 0 && __hip_atomic_load(stop + peer, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == fid;
    nb[peer] = stopped ? 0 : valid;
  }
  const int64_t pix = (int64_t)B * H * W;
  const int cpp = Cp / 8;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < pix * cpp; i += (int64_t)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % cpp);
    const int64_t px = i / cpp;
    const int b = (int)(px / (H * W));
    const int hw = (int)(px - (int64_t)b * H * W);
    float f[8];
    if (b < valid) {
      const int idx = perm ? perm[peer * perm_ps + offset + b] : offset + b;
      const uint8_t* s = xs[peer] + ((int64_t)idx * H * W + hw) * C;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int c = c8 * 8 + j;
        f[j] = c < C ? scale * (float)s[c] : 0.f;
      }
      if (c8 == 0 && hw == 0) labels[peer * B + b] = (int)ys[peer][idx];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = 0.f;
    }
    *reinterpret_cast<uint4*>(out + peer * out_ps + px * Cp + c8 * 8) = pack8(f);
  }
}

// ------------------------------------------------------------------------------------------------
// BatchNorm forward finalize: partial (sum, sumsq) rows -> scale/shift (+ running stats) or eval
// ------------------------------------------------------------------------------------------------
__global__ void k_bn_finalize(const float* stats, int64_t stats_ps, int rows, const int* nb, int hw, const float* gamma, const float* beta,
                              int64_t param_ps, float* rmean, float* rvar, int64_t run_ps, int C, int Cp, float eps, float momentum, int train,
                              float* ss, float* ms) {
  const int peer = blockIdx.y;
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;
  __shared__ float red[2][4][64];
  float s = 0.f, sq = 0.f;
  if (train && c < Cp) {
    const float* st = stats + peer * stats_ps;
    for (int r = rg; r < rows; r += 4) {
      s += st[(r * 2 + 0) * Cp + c];
      sq += st[(r * 2 + 1) * Cp + c];
    }
  }
  red[0][rg][threadIdx.x & 63] = s;
  red[1][rg][threadIdx.x & 63] = sq;
  __syncthreads();
  if (train && c < Cp) {  // re-arm the accumulator rows for the next step's conv epilogue
    float* st = (float*)stats + peer * stats_ps;
    for (int r = rg; r < rows; r += 4) {
      st[(r * 2 + 0) * Cp + c] = 0.f;
      st[(r * 2 + 1) * Cp + c] = 0.f;
    }
  }
  if (rg != 0 || c >= Cp) return;
  float* ssp = ss + peer * 2 * Cp;
  float* msp = ms + peer * 2 * Cp;
  if (c >= C) {
    ssp[c] = 0.f; ssp[Cp + c] = 0.f; msp[c] = 0.f; msp[Cp + c] = 0.f;
    return;
  }
  float mean, var;
  float* rm = rmean + peer * run_ps;
  float* rv = rvar + peer * run_ps;
  if (train) {
    s = red[0][0][c & 63] + red[0][1][c & 63] + red[0][2][c & 63] + red[0][3][c & 63];
    sq = red[1][0][c & 63] + red[1][1][c & 63] + red[1][2][c & 63] + red[1][3][c & 63];
    const int n = nb[peer] * hw;
    const float cnt = (float)max(1, n);
    mean = s / cnt;
    var = fmaxf(sq / cnt - mean * mean, 0.f);
    if (n > 0) {  // a peer without samples this step keeps its running statistics
      const float unbiased = cnt > 1.f ? var * cnt / (cnt - 1.f) : var;
      rm[c] = (1.f - momentum) * rm[c] + momentum * mean;
      rv[c] = (1.f - momentum) * rv[c] + momentum * unbiased;
    }
  } else {
    mean = rm[c];
    var = rv[c];
  }
  const float inv = rsqrtf(var + eps);
  const float g = gamma[peer * param_ps + c], b = beta[peer * param_ps + c];
  ssp[c] = g * inv;
  ssp[Cp + c] = b - mean * g * inv;
  msp[c] = mean;
  msp[Cp + c] = inv;
}

// Element-wise BN kernels: thread t of a block always handles the same 8-channel chunk
// (t % cpp) of rows (t / cpp) + k * rpb, rpb = 256 / cpp rows per block pass, so the per-channel
// constants sit in registers and the loop has no 64-bit division (the flat index i / cpp, i % cpp
// of the first version was a ~40-instruction software division per 16-byte chunk); RU rows are
// loaded before any is used, so each thread keeps several loads in flight.
constexpr int EW_RU = 4;
struct EwMap {
  int cpp, rpb, c8, r;  // chunks per row, rows per block pass, this thread's chunk / first row
  bool active;
  __device__ EwMap(int Cp) {
    cpp = Cp >> 3;
    rpb = 256 / cpp;
    c8 = threadIdx.x % cpp;
    r = threadIdx.x / cpp;
    active = r < rpb;
  }
};

// out = act(y*sc + sh [+ res] [+ y2*sc2 + sh2]) ; rows = nb[p]*hw (flat chunk index: measured faster
// here than the EwMap form above, 18.2 vs 28.2 ms per profiled run)
__global__ void k_bn_act(const bf16* y, int64_t y_ps, const float* ss, const bf16* res, int64_t res_ps, const bf16* y2, int64_t y2_ps,
                         const float* ss2, int relu, const int* nb, int hw, int Cp, bf16* out, int64_t out_ps) {
  const int peer = blockIdx.y;
  const int64_t rows = (int64_t)nb[peer] * hw;
  const int cpp = Cp / 8;
  const float* sp = ss + peer * 2 * Cp;
  const float* sp2 = ss2 ? ss2 + peer * 2 * Cp : nullptr;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < rows * cpp; i += (int64_t)gridDim.x * blockDim.x) {
    const int c0 = (int)(i % cpp) * 8;
    const int64_t off = (i / cpp) * Cp + c0;
    float f[8], t[8];
    unpack8(*reinterpret_cast<const uint4*>(y + peer * y_ps + off), f);
#pragma unroll
    for (int j = 0; j < 8; ++j) f[j] = fmaf(f[j], sp[c0 + j], sp[Cp + c0 + j]);
    if (res != nullptr) {
      unpack8(*reinterpret_cast<const uint4*>(res + peer * res_ps + off), t);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] += t[j];
    }
    if (y2 != nullptr) {
      unpack8(*reinterpret_cast<const uint4*>(y2 + peer * y2_ps + off), t);
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] += fmaf(t[j], sp2[c0 + j], sp2[Cp + c0 + j]);
    }
    if (relu) {
#pragma unroll
      for (int j = 0; j < 8; ++j) f[j] = fmaxf(f[j], 0.f);
    }
    *reinterpret_cast<uint4*>(out + peer * out_ps + off) = pack8(f);
  }
}

// ------------------------------------------------------------------------------------------------
// BatchNorm backward: g = dz * [mask > 0]; partial (sum g, sum g*xhat) per block; optional g out
// ------------------------------------------------------------------------------------------------
// mss (optional, instead of mask): the ReLU mask is recomputed as y*sc + sh > 0 from this BN's
// forward scale/shift — the activation relu(y*sc + sh) was never materialised
template <bool MSS>
__global__ __launch_bounds__(256) void k_bn_bwd_reduce(const bf16* dz, int64_t dz_ps, const bf16* mask, int64_t mask_ps, const bf16* y, int64_t y_ps,
                                                       const float* ms, const int* nb, int hw, int Cp, float* part, int64_t part_ps, bf16* gout,
                                                       int64_t gout_ps, const float* mss) {
  const int peer = blockIdx.y;
  const int64_t rows = (int64_t)nb[peer] * hw;
  const int cpp = Cp / 8;
  const int rpp = 256 / cpp;  // rows per pass
  const int tid = threadIdx.x;
  const int c8 = tid % cpp, rr = tid / cpp;
  const float* mp = ms + peer * 2 * Cp;
  float mean[8], inv[8], sg[8], sgx[8], msc[8], msh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    mean[j] = mp[c8 * 8 + j];
    inv[j] = mp[Cp + c8 * 8 + j];
    sg[j] = 0.f;
    sgx[j] = 0.f;
    msc[j] = MSS ? mss[peer * 2 * Cp + c8 * 8 + j] : 0.f;
    msh[j] = MSS ? mss[peer * 2 * Cp + Cp + c8 * 8 + j] : 0.f;
  }
  if (rr < rpp) {
    const int64_t per_blk = (rows + gridDim.x - 1) / gridDim.x;
    const int64_t r0 = blockIdx.x * per_blk, r1 = min(rows, r0 + per_blk);
    const bf16* dzp = dz + peer * dz_ps + c8 * 8;
    const bf16* mkp = (!MSS && mask) ? mask + peer * mask_ps + c8 * 8 : nullptr;
    const bf16* yp = y + peer * y_ps + c8 * 8;
    bf16* gop = gout ? gout + peer * gout_ps + c8 * 8 : nullptr;
    for (int64_t rb = r0 + rr; rb < r1; rb += EW_RU * rpp) {
      uint4 vd[EW_RU], vm[EW_RU], vy[EW_RU];  // all loads of EW_RU rows first (latency hiding)
#pragma unroll
      for (int u = 0; u < EW_RU; ++u) {
        const int64_t r = rb + u * rpp;
        const bool ok = r < r1;
        const int64_t off = r * Cp;
        vd[u] = ok ? *reinterpret_cast<const uint4*>(dzp + off) : uint4{0u, 0u, 0u, 0u};
        vm[u] = (ok && mkp) ? *reinterpret_cast<const uint4*>(mkp + off) : uint4{0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u};
        vy[u] = ok ? *reinterpret_cast<const uint4*>(yp + off) : uint4{0u, 0u, 0u, 0u};
      }
#pragma unroll
      for (int u = 0; u < EW_RU; ++u) {
        const int64_t r = rb + u * rpp;
        if (r >= r1) break;
        float g[8], t[8];
        unpack8(vd[u], g);
        if (MSS) {
          unpack8(vy[u], t);
#pragma unroll
          for (int j = 0; j < 8; ++j) g[j] = fmaf(t[j], msc[j], msh[j]) > 0.f ? g[j] : 0.f;
        } else {
          unpack8(vm[u], t);
#pragma unroll
          for (int j = 0; j < 8; ++j) g[j] = t[j] > 0.f ? g[j] : 0.f;
        }
        if (gop != nullptr) *reinterpret_cast<uint4*>(gop + r * Cp) = pack8(g);
        unpack8(vy[u], t);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          sg[j] += g[j];
          sgx[j] += g[j] * (t[j] - mean[j]) * inv[j];
        }
      }
    }
  }
  __shared__ float red[256][17];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[tid][j] = sg[j];
    red[tid][8 + j] = sgx[j];
  }
  __syncthreads();
  if (tid < cpp) {
    float a[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) a[j] = 0.f;
    for (int k = 0; k < rpp; ++k)
#pragma unroll
      for (int j = 0; j < 16; ++j) a[j] += red[k * cpp + tid][j];
    // straight into the peer's [2][Cp] accumulator (the finalize kernel reads and re-zeroes it;
    // a partial-row slab made the finalize a serial 128-row walk, ~22 us per BatchNorm)
    float* pp = part + peer * part_ps;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      atomicAdd(pp + tid * 8 + j, a[j]);
      atomicAdd(pp + Cp + tid * 8 + j, a[8 + j]);
    }
  }
}

// sum partials -> dgamma/dbeta (accumulated into the flat grad) + apply coefficients; the nblk
// accumulator rows [nblk][2][Cp] (spread atomics) are summed by 4 row groups of 64 channels per
// block (as k_bn_finalize) and re-armed
__global__ void k_bn_bwd_finalize(const float* part, int64_t part_ps, int nblk, const int* nb, int hw, const float* gamma, int64_t param_ps,
                                  const float* ms, float* dgamma, float* dbeta, int C, int Cp, float* coef) {
  const int peer = blockIdx.y;
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;
  __shared__ float red[2][4][64];
  float sg = 0.f, sgx = 0.f;
  float* pp = const_cast<float*>(part) + peer * part_ps;
  if (c < Cp) {
    for (int r = rg; r < nblk; r += 4) {
      sg += pp[r * 2 * Cp + c];
      sgx += pp[r * 2 * Cp + Cp + c];
    }
    for (int r = rg; r < nblk; r += 4) {
      pp[r * 2 * Cp + c] = 0.f;
      pp[r * 2 * Cp + Cp + c] = 0.f;
    }
  }
  red[0][rg][threadIdx.x & 63] = sg;
  red[1][rg][threadIdx.x & 63] = sgx;
  __syncthreads();
  if (rg != 0 || c >= Cp) return;
  sg = red[0][0][c & 63] + red[0][1][c & 63] + red[0][2][c & 63] + red[0][3][c & 63];
  sgx = red[1][0][c & 63] + red[1][1][c & 63] + red[1][2][c & 63] + red[1][3][c & 63];
  float* cp = coef + peer * 3 * Cp;
  if (c >= C) {
    cp[c] = 0.f; cp[Cp + c] = 0.f; cp[2 * Cp + c] = 0.f;
    return;
  }
  dgamma[peer * param_ps + c] += sgx;
  dbeta[peer * param_ps + c] += sg;
  const float cnt = (float)max(1, nb[peer] * hw);
  const float inv = ms[peer * 2 * Cp + Cp + c];
  cp[c] = gamma[peer * param_ps + c] * inv;
  cp[Cp + c] = sg / cnt;
  cp[2 * Cp + c] = sgx / cnt;
}

// dy = k1 * (g - mean_g - xhat * mean_gxhat), g recomputed from dz and mask
template <bool MSS>
__global__ __launch_bounds__(256) void k_bn_bwd_apply(const bf16* dz, int64_t dz_ps, const bf16* mask, int64_t mask_ps, const bf16* y, int64_t y_ps,
                                                      const float* ms, const float* coef, const int* nb, int hw, int Cp, bf16* dy, int64_t dy_ps,
                                                      const float* mss) {
  const int peer = blockIdx.y;
  const int rows = nb[peer] * hw;
  const EwMap m(Cp);
  if (!m.active) return;
  const int c0 = m.c8 * 8;
  const float* mp = ms + peer * 2 * Cp;
  const float* cp = coef + peer * 3 * Cp;
  float mean[8], inv[8], k1[8], mg[8], mgx[8], msc[8], msh[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    msc[j] = MSS ? mss[peer * 2 * Cp + c0 + j] : 0.f;
    msh[j] = MSS ? mss[peer * 2 * Cp + Cp + c0 + j] : 0.f;
    mean[j] = mp[c0 + j];
    inv[j] = mp[Cp + c0 + j];
    k1[j] = cp[c0 + j];
    mg[j] = cp[Cp + c0 + j];
    mgx[j] = cp[2 * Cp + c0 + j];
  }
  dz += peer * dz_ps + c0;
  y += peer * y_ps + c0;
  dy += peer * dy_ps + c0;
  if (MSS) mask = nullptr;
  if (mask) mask += peer * mask_ps + c0;
  const int step = gridDim.x * m.rpb;
  for (int r0 = blockIdx.x * m.rpb + m.r; r0 < rows; r0 += EW_RU * step) {
    uint4 vd[EW_RU], vm[EW_RU], vy[EW_RU];
#pragma unroll
    for (int u = 0; u < EW_RU; ++u) {
      const int r = r0 + u * step;
      const bool ok = r < rows;
      const int64_t off = (int64_t)r * Cp;
      vd[u] = ok ? *reinterpret_cast<const uint4*>(dz + off) : uint4{0u, 0u, 0u, 0u};
      vm[u] = (ok && mask) ? *reinterpret_cast<const uint4*>(mask + off) : uint4{0x3F803F80u, 0x3F803F80u, 0x3F803F80u, 0x3F803F80u};
      vy[u] = ok ? *reinterpret_cast<const uint4*>(y + off) : uint4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int u = 0; u < EW_RU; ++u) {
      const int r = r0 + u * step;
      if (r >= rows) break;
      float g[8], t[8], q[8];
      unpack8(vd[u], g);
      unpack8(vm[u], t);
      unpack8(vy[u], q);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const bool live = MSS ? fmaf(q[j], msc[j], msh[j]) > 0.f : t[j] > 0.f;
        const float gg = live ? g[j] : 0.f;
        const float xh = (q[j] - mean[j]) * inv[j];
        g[j] = k1[j] * (gg - mg[j] - xh * mgx[j]);
      }
      *reinterpret_cast<uint4*>(dy + (int64_t)r * Cp) = pack8(g);
    }
  }
}

// dz * [mask > 0] (ReLU backward without BN, e.g. LeNet / fc layers) and optional bias-grad
__global__ __launch_bounds__(256) void k_relu_bwd(const bf16* dz, int64_t dz_ps, const bf16* mask, int64_t mask_ps, const int* nb, int hw, int Cp,
                                                  bf16* out, int64_t out_ps) {
  const int peer = blockIdx.y;
  const int rows = nb[peer] * hw;
  const EwMap m(Cp);
  if (!m.active) return;
  const int c0 = m.c8 * 8;
  dz += peer * dz_ps + c0;
  mask += peer * mask_ps + c0;
  out += peer * out_ps + c0;
  const int step = gridDim.x * m.rpb;
  for (int r0 = blockIdx.x * m.rpb + m.r; r0 < rows; r0 += EW_RU * step) {
    uint4 vd[EW_RU], vm[EW_RU];
#pragma unroll
    for (int u = 0; u < EW_RU; ++u) {
      const int r = r0 + u * step;
      const bool ok = r < rows;
      vd[u] = ok ? *reinterpret_cast<const uint4*>(dz + (int64_t)r * Cp) : uint4{0u, 0u, 0u, 0u};
      vm[u] = ok ? *reinterpret_cast<const uint4*>(mask + (int64_t)r * Cp) : uint4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int u = 0; u < EW_RU; ++u) {
      const int r = r0 + u * step;
      if (r >= rows) break;
      float g[8], t[8];
      unpack8(vd[u], g);
      unpack8(vm[u], t);
#pragma unroll
      for (int j = 0; j < 8; ++j) g[j] = t[j] > 0.f ? g[j] : 0.f;
      *reinterpret_cast<uint4*>(out + (int64_t)r * Cp) = pack8(g);
    }
  }
}

// column sums of a [rows][Cp] bf16 tensor accumulated into fp32 (bias gradients): one block per
// 8-channel chunk group, atomics only once per block and channel
__global__ __launch_bounds__(256) void k_colsum(const bf16* x, int64_t x_ps, const int* nb, int hw, int Cp, int C, float* out, int64_t out_ps) {
  const int peer = blockIdx.y;
  const int64_t rows = (int64_t)nb[peer] * hw;
  const int cpp = Cp / 8;
  const int rpp = max(1, 256 / cpp);
  const int tid = threadIdx.x;
  const int c8 = tid % cpp, rr = tid / cpp;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (rr < rpp && tid < rpp * cpp) {
    const int64_t per_blk = (rows + gridDim.x - 1) / gridDim.x;
    const int64_t r0 = blockIdx.x * per_blk, r1 = min(rows, r0 + per_blk);
    for (int64_t r = r0 + rr; r < r1; r += rpp) {
      float t[8];
      unpack8(*reinterpret_cast<const uint4*>(x + peer * x_ps + r * Cp + c8 * 8), t);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += t[j];
    }
  }
  __shared__ float red[256][9];
#pragma unroll
  for (int j = 0; j < 8; ++j) red[tid][j] = (rr < rpp && tid < rpp * cpp) ? acc[j] : 0.f;
  __syncthreads();
  if (tid < cpp) {
    for (int k = 1; k < rpp; ++k)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += red[k * cpp + tid][j];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = tid * 8 + j;
      if (c < C) atomicAdd(out + peer * out_ps + c, acc[j]);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// pooling
// ------------------------------------------------------------------------------------------------
__global__ void k_maxpool2_fwd(const bf16* x, int64_t x_ps, const int* nb, int H, int W, int Cp, bf16* out, int64_t out_ps) {
  const int peer = blockIdx.y;
  const int Ho = H / 2, Wo = W / 2, cpp = Cp / 8;
  const int64_t n = (int64_t)nb[peer] * Ho * Wo * cpp;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % cpp);
    const int64_t px = i / cpp;
    const int b = (int)(px / (Ho * Wo)), rem = (int)(px % (Ho * Wo)), oh = rem / Wo, ow = rem % Wo;
    float m[8], t[8];
    for (int j = 0; j < 8; ++j) m[j] = -INFINITY;
    for (int dh = 0; dh < 2; ++dh)
      for (int dw = 0; dw < 2; ++dw) {
        unpack8(*reinterpret_cast<const uint4*>(x + peer * x_ps + (((int64_t)b * H + 2 * oh + dh) * W + 2 * ow + dw) * Cp + c8 * 8), t);
#pragma unroll
        for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], t[j]);
      }
    *reinterpret_cast<uint4*>(out + peer * out_ps + px * Cp + c8 * 8) = pack8(m);
  }
}

// gradient to the first maximal element of each window (torch semantics)
__global__ void k_maxpool2_bwd(const bf16* x, int64_t x_ps, const bf16* dy, int64_t dy_ps, const int* nb, int H, int W, int Cp, bf16* dx, int64_t dx_ps) {
  const int peer = blockIdx.y;
  const int Ho = H / 2, Wo = W / 2, cpp = Cp / 8;
  const int64_t n = (int64_t)nb[peer] * Ho * Wo * cpp;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % cpp);
    const int64_t px = i / cpp;
    const int b = (int)(px / (Ho * Wo)), rem = (int)(px % (Ho * Wo)), oh = rem / Wo, ow = rem % Wo;
    float v[4][8], g[8], m[8];
    unpack8(*reinterpret_cast<const uint4*>(dy + peer * dy_ps + px * Cp + c8 * 8), g);
    for (int j = 0; j < 8; ++j) m[j] = -INFINITY;
    for (int k = 0; k < 4; ++k) {
      unpack8(*reinterpret_cast<const uint4*>(x + peer * x_ps + (((int64_t)b * H + 2 * oh + k / 2) * W + 2 * ow + k % 2) * Cp + c8 * 8), v[k]);
#pragma unroll
      for (int j = 0; j < 8; ++j) m[j] = fmaxf(m[j], v[k][j]);
    }
    bool taken[8] = {false, false, false, false, false, false, false, false};
    for (int k = 0; k < 4; ++k) {
      float o[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const bool hit = !taken[j] && v[k][j] == m[j];
        o[j] = hit ? g[j] : 0.f;
        taken[j] = taken[j] || hit;
      }
      *reinterpret_cast<uint4*>(dx + peer * dx_ps + (((int64_t)b * H + 2 * oh + k / 2) * W + 2 * ow + k % 2) * Cp + c8 * 8) = pack8(o);
    }
  }
}

__global__ void k_avgpool_fwd(const bf16* x, int64_t x_ps, const int* nb, int hw, int Cp, bf16* out, int64_t out_ps) {
  const int peer = blockIdx.y;
  const int cpp = Cp / 8;
  const int64_t n = (int64_t)nb[peer] * cpp;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % cpp);
    const int64_t b = i / cpp;
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, t[8];
    for (int k = 0; k < hw; ++k) {
      unpack8(*reinterpret_cast<const uint4*>(x + peer * x_ps + (b * hw + k) * Cp + c8 * 8), t);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += t[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s[j] *= 1.f / hw;
    *reinterpret_cast<uint4*>(out + peer * out_ps + b * Cp + c8 * 8) = pack8(s);
  }
}

__global__ void k_avgpool_bwd(const bf16* dy, int64_t dy_ps, const int* nb, int hw, int Cp, bf16* dx, int64_t dx_ps) {
  const int peer = blockIdx.y;
  const int cpp = Cp / 8;
  const int64_t n = (int64_t)nb[peer] * hw * cpp;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int c8 = (int)(i % cpp);
    const int64_t px = i / cpp, b = px / hw;
    float t[8];
    unpack8(*reinterpret_cast<const uint4*>(dy + peer * dy_ps + b * Cp + c8 * 8), t);
#pragma unroll
    for (int j = 0; j < 8; ++j) t[j] *= 1.f / hw;
    *reinterpret_cast<uint4*>(dx + peer * dx_ps + px * Cp + c8 * 8) = pack8(t);
  }
}

// ------------------------------------------------------------------------------------------------
// log-softmax + NLL: loss/correct sums, confusion, dlogits = (softmax - onehot) / nb
// ------------------------------------------------------------------------------------------------
__global__ void k_xent(const bf16* logits, int64_t lg_ps, int Lp, int K, const int* labels, int B, const int* nb, float* stats, int* confusion,
                       bf16* dlogits, int64_t dl_ps) {
  const int peer = blockIdx.y;
  const int n = nb[peer];
  float loss = 0.f, correct = 0.f;
  for (int b = threadIdx.x; b < B; b += blockDim.x) {
    const bf16* row = logits + peer * lg_ps + (int64_t)b * Lp;
    if (b >= n) {
      if (dlogits != nullptr)
        for (int k = 0; k < Lp; ++k) dlogits[peer * dl_ps + (int64_t)b * Lp + k] = (bf16)0.f;
      continue;
    }
    float z[32];
    float mx = -INFINITY;
    int am = 0;
    for (int k = 0; k < K; ++k) {
      z[k] = (float)row[k];
      if (z[k] > mx) { mx = z[k]; am = k; }
    }
    float se = 0.f;
    for (int k = 0; k < K; ++k) se += __expf(z[k] - mx);
    const float lse = mx + __logf(se);
    const int y = labels[peer * B + b];
    loss += lse - z[y];
    correct += (am == y) ? 1.f : 0.f;
    if (confusion != nullptr) atomicAdd(confusion + (peer * 16 + y) * 16 + am, 1);
    if (dlogits != nullptr) {
      const float invn = 1.f / (float)n;
      for (int k = 0; k < Lp; ++k) {
        const float pk = k < K ? __expf(z[k] - lse) : 0.f;
        dlogits[peer * dl_ps + (int64_t)b * Lp + k] = (bf16)((pk - (k == y ? 1.f : 0.f)) * invn);
      }
    }
  }
  loss = wave_sum(loss);
  correct = wave_sum(correct);
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(stats + peer * 4 + 0, loss);
    atomicAdd(stats + peer * 4 + 1, correct);
  }
}

// ------------------------------------------------------------------------------------------------
// fused optimizer + bf16 weight shadow refresh
//
// One block per work item (grid.x) and peer (grid.y); the work table lists (segment, row) pairs so
// no block is launched empty (a (max_cout x n_segments) grid dispatched ~250k idle blocks per step).
//   conv/fc weight row co (kind 1): the Wf-layout gradient row [R*S][cp_in] is staged into LDS
//     (coalesced, padded rows: conflict-free column reads), the torch-order master row
//     W[co][cin][R][S] and its momentum are updated in one coalesced pass (FedProx / SCAFFOLD /
//     weight decay / Nesterov via opt_update), the new row is kept in LDS and written out as the
//     bf16 shadow row Wf[co][R][S][cp_in] (engine channel order; colmaps for fc after a flatten).
//   plain vector chunk (kind 0: biases, BN affine): elementwise update of 256 elements.
// Consumed gradients that are accumulated with atomics are re-zeroed here (no per-step memset).
// ------------------------------------------------------------------------------------------------
struct Segment {
  int64_t off;          // element offset in the flat parameter vector (torch order)
  int n;                // elements
  int kind;             // 0 plain, 1 conv/fc weight with a Wf shadow
  int cout, cin, R, S, cp_in, cp_out;
  int zero_after;       // re-zero the consumed gradient (atomically accumulated ones)
  int pad_;
  int64_t wf_off;       // offset of the layer's Wf shadow (bf16) and Wf-layout gradient (fp32)
  const int* e2t;       // engine input channel -> torch input column (fc after flatten) or null
  const int* t2e;       // torch input column -> engine input channel, or null
};

#define SHADOW_MAX_ROW (4608 + 64)  // cin * R * S floats of one output channel (512 * 3 * 3) + cin / 8 pad
#define GRAD_MAX_ROW (9 * (512 + 4))     // R * S rows of cp_in + 4 floats

__global__ __launch_bounds__(256) void k_opt_step(float* w, float* g, float* mbuf, int64_t ps, const float* gf, int64_t gf_ps,
                                                  const Segment* segs, const int2* work, OptParams o, const float* anchor, const float* cg,
                                                  const float* cl, int update, bf16* shadow, int64_t shadow_ps, const int* active) {
  const int peer = blockIdx.y;
  if (active != nullptr && !active[peer]) return;
  const int2 wk = work[blockIdx.x];
  const Segment sg = segs[wk.x];
  const int tid = threadIdx.x;
  float* wp = w + peer * ps;
  float* mp = mbuf + peer * ps;
  const float* ap = anchor ? anchor + peer * ps : nullptr;
  const float* cgp = cg ? cg + peer * ps : nullptr;
  const float* clp = cl ? cl + peer * ps : nullptr;
  float vdummy = 0.f;
  if (sg.kind == 0) {
    const int i = wk.y * 256 + tid;
    if (!update || i >= sg.n) return;
    const int64_t idx = sg.off + i;
    float* gp = g + peer * ps + idx;
    float wv = wp[idx], mv = mp[idx];
    opt_update(o, *gp, wv, mv, vdummy, 1.f, 1.f, ap, cgp, clp, idx);
    wp[idx] = wv;
    mp[idx] = mv;
    if (sg.zero_after) *gp = 0.f;
    return;
  }
  __shared__ float gl[GRAD_MAX_ROW];
  __shared__ float wl[SHADOW_MAX_ROW];
  const int co = wk.y;
  // LDS layouts (bank conflicts modelled per access pattern; the former +1 row pad gave 8-9-way
  // conflicts on the column reads): gradient rows padded to cp_in + 4 (16-byte aligned, column reads
  // <= 2-way), the torch-order master row padded by one float per 8 input channels (the shadow
  // pass's 8-channel-per-lane reads become conflict-free)
  const int rsz = sg.R * sg.S, n = sg.cin * rsz, nf = rsz * sg.cp_in, ldg = sg.cp_in + 4;
  auto wli = [&](int ct, int rs) { return ct * rsz + rs + (ct >> 3); };
  const int64_t row = sg.off + (int64_t)co * n;
  // i / rsz and j / cp_in without integer division (exact: i, j < 2^22)
  const float inv_rsz = 1.f / (float)rsz, inv_cp = 1.f / (float)sg.cp_in;
  auto qdiv = [](int x, int d, float inv) {
    int q = (int)((float)x * inv);
    q -= (q * d > x) ? 1 : 0;
    q += ((q + 1) * d <= x) ? 1 : 0;
    return q;
  };
  float* grow = const_cast<float*>(gf) + peer * gf_ps + sg.wf_off + (int64_t)co * nf;
  bf16* dst = shadow + peer * shadow_ps + sg.wf_off + (int64_t)co * nf;
  // 16-byte passes when the row's addresses allow it (cp_in is a multiple of 8, so a 4- or
  // 8-element group never straddles two taps); uniform per block
  const bool vg = ((reinterpret_cast<uintptr_t>(grow) & 15) == 0);
  const bool vw = ((reinterpret_cast<uintptr_t>(wp + row) & 15) == 0) && ((reinterpret_cast<uintptr_t>(mp + row) & 15) == 0) && (n & 3) == 0;
  const bool vs = ((reinterpret_cast<uintptr_t>(dst) & 15) == 0);
  if (update) {
    if (vg) {
      for (int j = tid * 4; j < nf; j += 1024) {
        const float4 v = *reinterpret_cast<const float4*>(grow + j);
        const int rs = qdiv(j, sg.cp_in, inv_cp), ci = j - rs * sg.cp_in;
        *reinterpret_cast<float4*>(gl + rs * ldg + ci) = v;
        if (sg.zero_after) *reinterpret_cast<float4*>(grow + j) = float4{0.f, 0.f, 0.f, 0.f};
      }
    } else {
      for (int j = tid; j < nf; j += 256) {
        const int rs = qdiv(j, sg.cp_in, inv_cp), ci = j - rs * sg.cp_in;
        gl[rs * ldg + ci] = grow[j];
        if (sg.zero_after) grow[j] = 0.f;
      }
    }
    __syncthreads();
    if (vw) {
      for (int i0 = tid * 4; i0 < n; i0 += 1024) {
        float4 w4 = *reinterpret_cast<const float4*>(wp + row + i0), m4 = *reinterpret_cast<const float4*>(mp + row + i0);
        float wv[4] = {w4.x, w4.y, w4.z, w4.w}, mv[4] = {m4.x, m4.y, m4.z, m4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int i = i0 + e;
          const int ct = qdiv(i, rsz, inv_rsz), rs = i - ct * rsz;
          const int ce = sg.t2e ? sg.t2e[ct] : ct;
          opt_update(o, gl[rs * ldg + ce], wv[e], mv[e], vdummy, 1.f, 1.f, ap, cgp, clp, row + i);
          wl[wli(ct, rs)] = wv[e];
        }
        *reinterpret_cast<float4*>(wp + row + i0) = float4{wv[0], wv[1], wv[2], wv[3]};
        *reinterpret_cast<float4*>(mp + row + i0) = float4{mv[0], mv[1], mv[2], mv[3]};
      }
    } else {
      for (int i = tid; i < n; i += 256) {
        const int ct = qdiv(i, rsz, inv_rsz), rs = i - ct * rsz;
        const int ce = sg.t2e ? sg.t2e[ct] : ct;
        const int64_t idx = row + i;
        float wv = wp[idx], mv = mp[idx];
        opt_update(o, gl[rs * ldg + ce], wv, mv, vdummy, 1.f, 1.f, ap, cgp, clp, idx);
        wp[idx] = wv;
        mp[idx] = mv;
        wl[wli(ct, rs)] = wv;
      }
    }
  } else {
    for (int i = tid; i < n; i += 256) {
      const int ct = qdiv(i, rsz, inv_rsz);
      wl[wli(ct, i - ct * rsz)] = wp[row + i];
    }
  }
  __syncthreads();
  if (vs) {
    for (int j = tid * 8; j < nf; j += 2048) {
      const int rs = qdiv(j, sg.cp_in, inv_cp), ci0 = j - rs * sg.cp_in;
      float v[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int ci = ci0 + e;
        const int tc = sg.e2t ? sg.e2t[ci] : (ci < sg.cin ? ci : -1);
        v[e] = tc >= 0 ? wl[wli(tc, rs)] : 0.f;
      }
      *reinterpret_cast<uint4*>(dst + j) = pack8(v);
    }
  } else {
    for (int j = tid; j < nf; j += 256) {
      const int rs = qdiv(j, sg.cp_in, inv_cp), ci = j - rs * sg.cp_in;
      const int tc = sg.e2t ? sg.e2t[ci] : (ci < sg.cin ? ci : -1);
      dst[j] = (bf16)(tc >= 0 ? wl[wli(tc, rs)] : 0.f);
    }
  }
}

// ------------------------------------------------------------------------------------------------
// C API
// ------------------------------------------------------------------------------------------------
static inline int ew_blocks(int64_t work) {
  const int64_t b = (work + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 4096 ? 4096 : b));
}
static inline int ok() { return hipGetLastError() == hipSuccess ? 0 : 2; }
// blocks per peer for the EwMap kernels: each block pass covers 256 / (Cp / 8) rows, EW_RU passes
// per loop iteration
static inline int ew_row_blocks(int max_rows, int Cp) {
  const int rpb = 256 / (Cp / 8 > 0 ? Cp / 8 : 1);
  const int64_t b = ((int64_t)max_rows + (int64_t)rpb * EW_RU - 1) / ((int64_t)rpb * EW_RU);
  return (int)(b < 1 ? 1 : (b > 2048 ? 2048 : b));
}

extern "C" {
int cnn_input_prep(const uint8_t* const* xs, const int64_t* const* ys, const int* n_samples, const int* perm, int64_t perm_ps, int offset, int B,
                   int H, int W, int C, int Cp, float scale, bf16* out, int64_t out_ps, int* labels, int* nb, int peers, void* s, const int* stop,
                   const int* fit_id) {
  hipLaunchKernelGGL(k_input_prep, dim3(ew_blocks((int64_t)B * H * W * (Cp / 8)), peers), dim3(256), 0, (hipStream_t)s, xs, ys, n_samples, perm,
                     perm_ps, offset, B, H, W, C, Cp, scale, out, out_ps, labels, nb, stop, fit_id);
  return ok();
}
int cnn_bn_finalize(const float* stats, int64_t stats_ps, int rows, const int* nb, int hw, const float* gamma, const float* beta, int64_t param_ps,
                    float* rmean, float* rvar, int64_t run_ps, int C, int Cp, float eps, float momentum, int train, float* ss, float* ms, int peers,
                    void* s) {
  hipLaunchKernelGGL(k_bn_finalize, dim3((Cp + 63) / 64, peers), dim3(256), 0, (hipStream_t)s, stats, stats_ps, rows, nb, hw, gamma, beta, param_ps,
                     rmean, rvar, run_ps, C, Cp, eps, momentum, train, ss, ms);
  return ok();
}
int cnn_bn_act(const bf16* y, int64_t y_ps, const float* ss, const bf16* res, int64_t res_ps, const bf16* y2, int64_t y2_ps, const float* ss2,
               int relu, const int* nb, int max_rows, int hw, int Cp, bf16* out, int64_t out_ps, int peers, void* s) {
  if ((Cp & 7) || Cp / 8 > 256) return 1;
  hipLaunchKernelGGL(k_bn_act, dim3(ew_blocks((int64_t)max_rows * (Cp / 8)), peers), dim3(256), 0, (hipStream_t)s, y, y_ps, ss, res, res_ps, y2,
                     y2_ps, ss2, relu, nb, hw, Cp, out, out_ps);
  return ok();
}
int cnn_bn_bwd_reduce(const bf16* dz, int64_t dz_ps, const bf16* mask, int64_t mask_ps, const bf16* y, int64_t y_ps, const float* ms, const int* nb,
                      int hw, int Cp, float* part, int64_t part_ps, int nblk, bf16* gout, int64_t gout_ps, int peers, void* s, const float* mss) {
  if (Cp / 8 > 256 || (Cp & 7)) return 1;
  if (mss != nullptr)
    hipLaunchKernelGGL(k_bn_bwd_reduce<true>, dim3(nblk, peers), dim3(256), 0, (hipStream_t)s, dz, dz_ps, mask, mask_ps, y, y_ps, ms, nb, hw, Cp,
                       part, part_ps, gout, gout_ps, mss);
  else
    hipLaunchKernelGGL(k_bn_bwd_reduce<false>, dim3(nblk, peers), dim3(256), 0, (hipStream_t)s, dz, dz_ps, mask, mask_ps, y, y_ps, ms, nb, hw, Cp,
                       part, part_ps, gout, gout_ps, mss);
  return ok();
}
int cnn_bn_bwd_finalize(const float* part, int64_t part_ps, int nblk, const int* nb, int hw, const float* gamma, int64_t param_ps, const float* ms,
                        float* dgamma, float* dbeta, int C, int Cp, float* coef, int peers, void* s) {
  hipLaunchKernelGGL(k_bn_bwd_finalize, dim3((Cp + 63) / 64, peers), dim3(256), 0, (hipStream_t)s, part, part_ps, nblk, nb, hw, gamma, param_ps,
                     ms, dgamma, dbeta, C, Cp, coef);
  return ok();
}
int cnn_bn_bwd_apply(const bf16* dz, int64_t dz_ps, const bf16* mask, int64_t mask_ps, const bf16* y, int64_t y_ps, const float* ms,
                     const float* coef, const int* nb, int max_rows, int hw, int Cp, bf16* dy, int64_t dy_ps, int peers, void* s, const float* mss) {
  if ((Cp & 7) || Cp / 8 > 256) return 1;
  if (mss != nullptr)
    hipLaunchKernelGGL(k_bn_bwd_apply<true>, dim3(ew_row_blocks(max_rows, Cp), peers), dim3(256), 0, (hipStream_t)s, dz, dz_ps, mask, mask_ps,
                       y, y_ps, ms, coef, nb, hw, Cp, dy, dy_ps, mss);
  else
    hipLaunchKernelGGL(k_bn_bwd_apply<false>, dim3(ew_row_blocks(max_rows, Cp), peers), dim3(256), 0, (hipStream_t)s, dz, dz_ps, mask, mask_ps,
                       y, y_ps, ms, coef, nb, hw, Cp, dy, dy_ps, mss);
  return ok();
}
int cnn_relu_bwd(const bf16* dz, int64_t dz_ps, const bf16* mask, int64_t mask_ps, const int* nb, int max_rows, int hw, int Cp, bf16* out,
                 int64_t out_ps, int peers, void* s) {
  if ((Cp & 7) || Cp / 8 > 256) return 1;
  hipLaunchKernelGGL(k_relu_bwd, dim3(ew_row_blocks(max_rows, Cp), peers), dim3(256), 0, (hipStream_t)s, dz, dz_ps, mask, mask_ps, nb,
                     hw, Cp, out, out_ps);
  return ok();
}
int cnn_colsum(const bf16* x, int64_t x_ps, const int* nb, int hw, int Cp, int C, float* out, int64_t out_ps, int nblk, int peers, void* s) {
  if (Cp / 8 > 256 || (Cp & 7)) return 1;
  hipLaunchKernelGGL(k_colsum, dim3(nblk, peers), dim3(256), 0, (hipStream_t)s, x, x_ps, nb, hw, Cp, C, out, out_ps);
  return ok();
}
int cnn_maxpool2(int bwd, const bf16* x, int64_t x_ps, const bf16* dy, int64_t dy_ps, const int* nb, int max_batch, int H, int W, int Cp, bf16* out,
                 int64_t out_ps, int peers, void* s) {
  const int64_t work = (int64_t)max_batch * (H / 2) * (W / 2) * (Cp / 8);
  if (bwd)
    hipLaunchKernelGGL(k_maxpool2_bwd, dim3(ew_blocks(work), peers), dim3(256), 0, (hipStream_t)s, x, x_ps, dy, dy_ps, nb, H, W, Cp, out, out_ps);
  else
    hipLaunchKernelGGL(k_maxpool2_fwd, dim3(ew_blocks(work), peers), dim3(256), 0, (hipStream_t)s, x, x_ps, nb, H, W, Cp, out, out_ps);
  return ok();
}
int cnn_avgpool(int bwd, const bf16* x, int64_t x_ps, const int* nb, int max_batch, int hw, int Cp, bf16* out, int64_t out_ps, int peers, void* s) {
  if (bwd)
    hipLaunchKernelGGL(k_avgpool_bwd, dim3(ew_blocks((int64_t)max_batch * hw * (Cp / 8)), peers), dim3(256), 0, (hipStream_t)s, x, x_ps, nb, hw, Cp,
                       out, out_ps);
  else
    hipLaunchKernelGGL(k_avgpool_fwd, dim3(ew_blocks((int64_t)max_batch * (Cp / 8)), peers), dim3(256), 0, (hipStream_t)s, x, x_ps, nb, hw, Cp, out,
                       out_ps);
  return ok();
}
int cnn_xent(const bf16* logits, int64_t lg_ps, int Lp, int K, const int* labels, int B, const int* nb, float* stats, int* confusion, bf16* dlogits,
             int64_t dl_ps, int peers, void* s) {
  if (K > 16 || Lp < K) return 1;
  hipLaunchKernelGGL(k_xent, dim3(1, peers), dim3(256), 0, (hipStream_t)s, logits, lg_ps, Lp, K, labels, B, nb, stats, confusion, dlogits, dl_ps);
  return ok();
}
// one fused optimizer + shadow pass (update = 0: shadow refresh only)
int cnn_opt_step(float* w, float* g, float* m, int64_t ps, const float* gf, int64_t gf_ps, const void* segs, const void* work, int nwork, int kind,
                 float lr, float momentum, float weight_decay, int nesterov, float mu, const float* anchor, const float* cg, const float* cl, int update,
                 bf16* shadow, int64_t shadow_ps, const int* active, int peers, void* s) {
  OptParams o;
  o.kind = kind;
  o.lr = lr;
  o.beta1 = 0.9f;
  o.beta2 = 0.999f;
  o.eps = 1e-8f;
  o.weight_decay = weight_decay;
  o.momentum = momentum;
  o.nesterov = nesterov;
  o.mu = mu;
  o.scaf_upd = 0;  // opt_update applies SCAFFOLD through the cg / cl pointers
  if (nwork < 1) return 1;
  hipLaunchKernelGGL(k_opt_step, dim3(nwork, peers), dim3(256), 0, (hipStream_t)s, w, g, m, ps, gf, gf_ps, (const Segment*)segs, (const int2*)work, o,
                     anchor, cg, cl, update, shadow, shadow_ps, active);
  return ok();
}
int cnn_segment_size() { return (int)sizeof(Segment); }
}

// Resolve one kernel of this translation unit on the current device: loads the unit's code object
// now (myfyp_warm_all, at engine prewarm) instead of at its first launch, which waited for the
// kernels in flight (the first FedAvg launch blocked the host until the running epoch ended)
extern "C" int myfyp_warm_cnn_ops() {
  hipFuncAttributes attr;
  return hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(&k_input_prep)) == hipSuccess ? 0 : 1;
}
