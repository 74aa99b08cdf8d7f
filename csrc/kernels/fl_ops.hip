// Federated-learning elementwise/reduction kernels (gfx950): FedAvg reductions, fused optimizers,
// coordinate median, attack injection. All memory-bound: 16-byte vector accesses, grid-stride,
// grid capped at 2048 blocks (cdna_hip_programming.md Guideline 11/13).
#include "common.h"
#include "fl_ops.h"

#define FL_BLOCK 256

static inline unsigned grid_for(int64_t n_vec) {
  int64_t g = (n_vec + FL_BLOCK - 1) / FL_BLOCK;
  if (g > 2048) g = 2048;
  if (g < 1) g = 1;
  return (unsigned)g;
}

// out[i] = Σ_k w[k] · src_k[i]   (src pointers in a device array)
__global__ __launch_bounds__(FL_BLOCK) void k_weighted_sum(float* __restrict__ out, const uint64_t* __restrict__ srcs, const float* __restrict__ w, int K,
                                                            int64_t n) {
  const int64_t n4 = n / 4;
  const int64_t stride = (int64_t)gridDim.x * FL_BLOCK;
  for (int64_t i = blockIdx.x * FL_BLOCK + threadIdx.x; i < n4; i += stride) {
    float4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < K; ++k) {
      const float4 v = reinterpret_cast<const float4*>(srcs[k])[i];
      const float wk = w[k];
      acc.x += wk * v.x; acc.y += wk * v.y; acc.z += wk * v.z; acc.w += wk * v.w;
    }
    reinterpret_cast<float4*>(out)[i] = acc;
  }
  for (int64_t i = n4 * 4 + blockIdx.x * FL_BLOCK + threadIdx.x; i < n; i += stride) {
    float acc = 0.f;
    for (int k = 0; k < K; ++k) acc += w[k] * reinterpret_cast<const float*>(srcs[k])[i];
    out[i] = acc;
  }
}

// out[i] = scale · Σ_p w[p] · stacked[p*ld + i]   (co-located peers, [P][ld] buffer)
__global__ __launch_bounds__(FL_BLOCK) void k_stacked_weighted_sum(float* __restrict__ out, const float* __restrict__ stacked, int P, int64_t n, int64_t ld,
                                                                    const float* __restrict__ w, float scale) {
  const int64_t n4 = n / 4;
  const int64_t stride = (int64_t)gridDim.x * FL_BLOCK;
  const bool vec = (ld % 4) == 0;
  if (vec) {
    for (int64_t i = blockIdx.x * FL_BLOCK + threadIdx.x; i < n4; i += stride) {
      float4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int p = 0; p < P; ++p) {
        const float wp = w[p];
        if (wp == 0.f) continue;
        const float4 v = reinterpret_cast<const float4*>(stacked + p * ld)[i];
        acc.x += wp * v.x; acc.y += wp * v.y; acc.z += wp * v.z; acc.w += wp * v.w;
      }
      acc.x *= scale; acc.y *= scale; acc.z *= scale; acc.w *= scale;
      reinterpret_cast<float4*>(out)[i] = acc;
    }
  }
  for (int64_t i = (vec ? n4 * 4 : 0) + blockIdx.x * FL_BLOCK + threadIdx.x; i < n; i += stride) {
    float acc = 0.f;
    for (int p = 0; p < P; ++p) acc += w[p] * stacked[p * ld + i];
    out[i] = acc * scale;
  }
}

// stacked[p*ld + i] = src[i] for rows with mask[p] != 0 (mask null = all rows)
__global__ __launch_bounds__(FL_BLOCK) void k_broadcast_rows(float* __restrict__ stacked, const float* __restrict__ src, int P, int64_t n, int64_t ld,
                                                              const float* __restrict__ mask) {
  const int p = blockIdx.y;
  if (mask != nullptr && mask[p] == 0.f) return;
  const int64_t stride = (int64_t)gridDim.x * FL_BLOCK;
  float* dst = stacked + p * ld;
  if ((ld % 4) == 0) {
    const int64_t n4 = n / 4;
    for (int64_t i = blockIdx.x * FL_BLOCK + threadIdx.x; i < n4; i += stride)
      reinterpret_cast<float4*>(dst)[i] = reinterpret_cast<const float4*>(src)[i];
    for (int64_t i = n4 * 4 + blockIdx.x * FL_BLOCK + threadIdx.x; i < n; i += stride) dst[i] = src[i];
  } else {
    for (int64_t i = blockIdx.x * FL_BLOCK + threadIdx.x; i < n; i += stride) dst[i] = src[i];
  }
}

// FedAvg over a stacked [P][ld] group with the per-peer weights / mask passed BY VALUE (kernel
// arguments): no host→device copy, nothing for the host to wait on.
//   reduce: out[i] = Σ_p w[p] · stacked[p*ld + i] (i < n), *wsum_slot = wsum (when non-null)
//   apply:  stacked[p*ld + i] = out[i] / max(*wsum_slot, 1e-12) for rows with mask bit p set
// A bucketed all-reduce calls them per bucket (sub-ranges of out / stacked, bucket 0 carries the
// weight sum in a slot in front of the data, so bucket k's apply only waits for buckets 0 and k).
// out2 / wsum2 (nullable): a second copy of the partial sums (the failover's retained input), written
// by the same pass instead of a separate device copy behind it
__global__ __launch_bounds__(FL_BLOCK) void k_fedavg_reduce(float* __restrict__ out, float* __restrict__ wsum_slot, const float* __restrict__ stacked,
                                                             int P, int64_t n, int64_t ld, FedAvgWeights w, float* __restrict__ out2,
                                                             float* __restrict__ wsum2) {
  const int64_t stride = (int64_t)gridDim.x * FL_BLOCK;
  const int64_t t0 = blockIdx.x * FL_BLOCK + threadIdx.x;
  if (t0 == 0 && wsum_slot != nullptr) *wsum_slot = w.wsum;
  if (t0 == 0 && wsum2 != nullptr) *wsum2 = w.wsum;
  if ((ld % 4) == 0) {
    const int64_t n4 = n / 4;
    for (int64_t i = t0; i < n4; i += stride) {
      float4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int p = 0; p < P; ++p) {
        const float wp = w.w[p];
        if (wp == 0.f) continue;
        const float4 v = reinterpret_cast<const float4*>(stacked + p * ld)[i];
        acc.x += wp * v.x; acc.y += wp * v.y; acc.z += wp * v.z; acc.w += wp * v.w;
      }
      reinterpret_cast<float4*>(out)[i] = acc;
      if (out2 != nullptr) reinterpret_cast<float4*>(out2)[i] = acc;
    }
    for (int64_t i = n4 * 4 + t0; i < n; i += stride) {
      float acc = 0.f;
      for (int p = 0; p < P; ++p)
        if (w.w[p] != 0.f) acc += w.w[p] * stacked[p * ld + i];  // rows of weight 0 are never read (may be uninitialised)
      out[i] = acc;
      if (out2 != nullptr) out2[i] = acc;
    }
  } else {
    for (int64_t i = t0; i < n; i += stride) {
      float acc = 0.f;
      for (int p = 0; p < P; ++p)
        if (w.w[p] != 0.f) acc += w.w[p] * stacked[p * ld + i];  // rows of weight 0 are never read (may be uninitialised)
      out[i] = acc;
      if (out2 != nullptr) out2[i] = acc;
    }
  }
}

__global__ __launch_bounds__(FL_BLOCK) void k_fedavg_apply(float* __restrict__ stacked, const float* __restrict__ out, const float* __restrict__ wsum_slot,
                                                            int P, int64_t n, int64_t ld, unsigned long long mask) {
  const int p = blockIdx.y;
  if (!((mask >> p) & 1ull)) return;
  const float inv = 1.f / fmaxf(*wsum_slot, 1e-12f);
  const int64_t stride = (int64_t)gridDim.x * FL_BLOCK;
  float* dst = stacked + p * ld;
  if ((ld % 4) == 0) {
    const int64_t n4 = n / 4;
    for (int64_t i = blockIdx.x * FL_BLOCK + threadIdx.x; i < n4; i += stride) {
      float4 v = reinterpret_cast<const float4*>(out)[i];
      v.x *= inv; v.y *= inv; v.z *= inv; v.w *= inv;
      reinterpret_cast<float4*>(dst)[i] = v;
    }
    for (int64_t i = n4 * 4 + blockIdx.x * FL_BLOCK + threadIdx.x; i < n; i += stride) dst[i] = out[i] * inv;
  } else {
    for (int64_t i = blockIdx.x * FL_BLOCK + threadIdx.x; i < n; i += stride) dst[i] = out[i] * inv;
  }
}

// Single-rank FedAvg (no all-reduce between reduce and apply): each thread forms the weighted mean
// of its coordinates over the rows and writes it into every masked row — one launch instead of two.
__global__ __launch_bounds__(FL_BLOCK) void k_fedavg_local(float* __restrict__ stacked, int P, int64_t n, int64_t ld, FedAvgWeights w,
                                                           unsigned long long mask) {
  const int64_t stride = (int64_t)gridDim.x * FL_BLOCK;
  const float inv = 1.f / fmaxf(w.wsum, 1e-12f);
  if ((ld % 4) == 0) {
    const int64_t n4 = n / 4;
    for (int64_t i = blockIdx.x * FL_BLOCK + threadIdx.x; i < n4; i += stride) {
      float4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int p = 0; p < P; ++p) {
        const float wp = w.w[p];
        if (wp == 0.f) continue;
        const float4 v = reinterpret_cast<const float4*>(stacked + p * ld)[i];
        acc.x += wp * v.x; acc.y += wp * v.y; acc.z += wp * v.z; acc.w += wp * v.w;
      }
      acc.x *= inv; acc.y *= inv; acc.z *= inv; acc.w *= inv;
      for (int p = 0; p < P; ++p)
        if ((mask >> p) & 1ull) reinterpret_cast<float4*>(stacked + p * ld)[i] = acc;
    }
    for (int64_t i = n4 * 4 + blockIdx.x * FL_BLOCK + threadIdx.x; i < n; i += stride) {
      float acc = 0.f;
      for (int p = 0; p < P; ++p)
        if (w.w[p] != 0.f) acc += w.w[p] * stacked[p * ld + i];  // rows of weight 0 are never read (may be uninitialised)
      for (int p = 0; p < P; ++p)
        if ((mask >> p) & 1ull) stacked[p * ld + i] = acc * inv;
    }
  } else {
    for (int64_t i = blockIdx.x * FL_BLOCK + threadIdx.x; i < n; i += stride) {
      float acc = 0.f;
      for (int p = 0; p < P; ++p)
        if (w.w[p] != 0.f) acc += w.w[p] * stacked[p * ld + i];  // rows of weight 0 are never read (may be uninitialised)
      for (int p = 0; p < P; ++p)
        if ((mask >> p) & 1ull) stacked[p * ld + i] = acc * inv;
    }
  }
}

void fl_fedavg_local(float* stacked, int P, int64_t n, int64_t ld, const FedAvgWeights& w, unsigned long long mask, hipStream_t s) {
  hipLaunchKernelGGL(k_fedavg_local, dim3(grid_for((n + 3) / 4)), dim3(FL_BLOCK), 0, s, stacked, P, n, ld, w, mask);
}

void fl_fedavg_reduce(float* out, float* wsum_slot, const float* stacked, int P, int64_t n, int64_t ld, const FedAvgWeights& w, hipStream_t s,
                      float* out2, float* wsum2) {
  hipLaunchKernelGGL(k_fedavg_reduce, dim3(grid_for((n + 3) / 4)), dim3(FL_BLOCK), 0, s, out, wsum_slot, stacked, P, n, ld, w, out2, wsum2);
}

void fl_fedavg_apply(float* stacked, const float* out, const float* wsum_slot, int P, int64_t n, int64_t ld, unsigned long long mask, hipStream_t s) {
  unsigned gx = grid_for((n + 3) / 4);
  if (gx > 256) gx = 256;
  hipLaunchKernelGGL(k_fedavg_apply, dim3(gx, P), dim3(FL_BLOCK), 0, s, stacked, out, wsum_slot, P, n, ld, mask);
}

// Delayed averaging (opt-in): land the previous round's average as a correction and take the new
// snapshot in one pass, for every row with mask bit p set:
//   x = stacked[p][i] + avg[i] / wsum - snap[p][i];  stacked[p][i] = x;  snap[p][i] = x
// With avg == nullptr (nothing pending) it only snapshots.
__global__ __launch_bounds__(FL_BLOCK) void k_fedavg_delayed_land(float* __restrict__ stacked, float* __restrict__ snap, int64_t ld_snap,
                                                                   const float* __restrict__ avg, const float* __restrict__ wsum_slot, int P, int64_t n,
                                                                   int64_t ld, unsigned long long mask) {
  const int p = blockIdx.y;
  if (!((mask >> p) & 1ull)) return;
  const float inv = avg != nullptr ? 1.f / fmaxf(*wsum_slot, 1e-12f) : 0.f;
  float* x = stacked + p * ld;
  float* sp = snap + p * ld_snap;
  const int64_t stride = (int64_t)gridDim.x * FL_BLOCK;
  for (int64_t i = blockIdx.x * FL_BLOCK + threadIdx.x; i < n; i += stride) {
    float v = x[i];
    if (avg != nullptr) {
      v = v + (avg[i] * inv - sp[i]);
      x[i] = v;
    }
    sp[i] = v;
  }
}

void fl_fedavg_delayed_land(float* stacked, float* snap, int64_t ld_snap, const float* avg, const float* wsum_slot, int P, int64_t n, int64_t ld,
                            unsigned long long mask, hipStream_t s) {
  unsigned gx = grid_for(n);
  if (gx > 512) gx = 512;
  hipLaunchKernelGGL(k_fedavg_delayed_land, dim3(gx, P), dim3(FL_BLOCK), 0, s, stacked, snap, ld_snap, avg, wsum_slot, P, n, ld, mask);
}

// Gossip neighbour averaging of co-located peers (reference: aggregator over the neighbours'
// models, p2pfl/learning/aggregators/fedavg.py driven by gossip_weights). One thread owns a float4
// column of every row: it loads all P rows into registers, then writes each row's mixture back, so
// the in-place update never reads a row another thread has already written.
template <int P>
__global__ __launch_bounds__(FL_BLOCK) void k_neighbor_mix(float* __restrict__ stacked, int64_t n4, int64_t ld, MixPlan m) {
  const int64_t stride = (int64_t)gridDim.x * FL_BLOCK;
  for (int64_t i = blockIdx.x * FL_BLOCK + threadIdx.x; i < n4; i += stride) {
    float4 v[P];
#pragma unroll
    for (int p = 0; p < P; ++p) v[p] = reinterpret_cast<const float4*>(stacked + p * ld)[i];
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const int ns = m.nsrc[p];
      if (ns == 0) continue;
      float4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int k = 0; k < MIX_MAX_SRC; ++k) {
        if (k >= ns) break;
        const float wk = m.w[p][k];
        float4 s = v[0];
        // register-array select (a dynamic index would spill v to scratch)
#pragma unroll
        for (int q = 0; q < P; ++q)
          if (q == m.idx[p][k]) s = v[q];
        acc.x += wk * s.x; acc.y += wk * s.y; acc.z += wk * s.z; acc.w += wk * s.w;
      }
      reinterpret_cast<float4*>(stacked + p * ld)[i] = acc;
    }
  }
}

void fl_neighbor_mix(float* stacked, int P, int64_t n, int64_t ld, const MixPlan& m, hipStream_t s) {
  // rows are padded to ld (a multiple of 4); mixing the padding too keeps every access a float4
  const int64_t n4 = (n + 3) / 4;
  const dim3 g(grid_for(n4)), b(FL_BLOCK);
  switch (P) {
#define MIX_CASE(K) \
  case K: hipLaunchKernelGGL(k_neighbor_mix<K>, g, b, 0, s, stacked, n4, ld, m); break;
    MIX_CASE(1) MIX_CASE(2) MIX_CASE(3) MIX_CASE(4) MIX_CASE(5) MIX_CASE(6) MIX_CASE(7) MIX_CASE(8)
    MIX_CASE(9) MIX_CASE(10) MIX_CASE(11) MIX_CASE(12) MIX_CASE(13) MIX_CASE(14) MIX_CASE(15) MIX_CASE(16)
#undef MIX_CASE
    default: break;
  }
}

// per-coordinate median of K ≤ 16 models: branch-free compare-exchange network over K registers,
// the result stored into P destination rows (every peer that takes the aggregate). Row pointers
// travel as kernel arguments (no pointer table on the device, no H2D copy); each thread loads its
// coordinate from every row before storing, so destinations may alias sources.
template <int K>
__global__ __launch_bounds__(FL_BLOCK) void k_coordinate_median(OutPtrs outs, int P, RowPtrs rows, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * FL_BLOCK;
  for (int64_t i = blockIdx.x * FL_BLOCK + threadIdx.x; i < n; i += stride) {
    float v[K];
#pragma unroll
    for (int k = 0; k < K; ++k) v[k] = rows.p[k][i];
#pragma unroll
    for (int a = 0; a < K; ++a) {
#pragma unroll
      for (int b = 0; b < K - 1 - a; ++b) {
        const float lo = fminf(v[b], v[b + 1]);
        v[b + 1] = fmaxf(v[b], v[b + 1]);
        v[b] = lo;
      }
    }
    const float med = (K & 1) ? v[(K - 1) / 2] : 0.5f * (v[K / 2 - 1] + v[K / 2]);
    for (int p = 0; p < P; ++p) outs.p[p][i] = med;
  }
}

// SCAFFOLD (Karimireddy et al.) server step in two launches around one all-reduce; float4 body,
// scalar tail. Sums run in the same k order as the host reference.
__global__ __launch_bounds__(FL_BLOCK) void k_scaffold_reduce(float* __restrict__ buf, RowPtrs dy, RowPtrs dc, RowW w, int K, int64_t n) {
  const int64_t gid = (int64_t)blockIdx.x * FL_BLOCK + threadIdx.x;
  const int64_t stride = (int64_t)gridDim.x * FL_BLOCK;
  for (int64_t i = gid; i < n; i += stride) {
    float sy = 0.f, sc = 0.f;
    for (int k = 0; k < K; ++k) {
      sy = fmaf(w.w[k], dy.p[k][i], sy);
      sc += dc.p[k][i];
    }
    buf[i] = sy;
    buf[n + 1 + i] = sc;
  }
  if (gid == 0) {
    float ws = 0.f;
    for (int k = 0; k < K; ++k) ws += w.w[k];
    buf[n] = ws;
    buf[2 * n + 1] = (float)K;
  }
}

__global__ __launch_bounds__(FL_BLOCK) void k_scaffold_apply(OutPtrs outs, int P, const float* __restrict__ x_start, const float* __restrict__ buf,
                                                             float* __restrict__ c, int c_init, float glr, int64_t n) {
  const float scale = glr / fmaxf(buf[n], 1e-12f);
  const float inv_cnt = 1.f / fmaxf(buf[2 * n + 1], 1.f);
  const int64_t stride = (int64_t)gridDim.x * FL_BLOCK;
  for (int64_t i = (int64_t)blockIdx.x * FL_BLOCK + threadIdx.x; i < n; i += stride) {
    const float x = fmaf(buf[i], scale, x_start[i]);
    for (int p = 0; p < P; ++p) outs.p[p][i] = x;
    c[i] = (c_init ? 0.f : c[i]) + buf[n + 1 + i] * inv_cnt;
  }
}

// Fused Adam / SGD over a flat fp32 buffer (torch.optim semantics) + optional FedProx/SCAFFOLD terms
__global__ __launch_bounds__(FL_BLOCK) void k_opt_step(float* __restrict__ param, const float* __restrict__ grad, float* __restrict__ m,
                                                        float* __restrict__ v, bf16* __restrict__ shadow, int64_t n, OptParams o, float bc1, float bc2s,
                                                        const float* __restrict__ anchor, const float* __restrict__ cg, const float* __restrict__ cl) {
  const int64_t stride = (int64_t)gridDim.x * FL_BLOCK;
  for (int64_t i = blockIdx.x * FL_BLOCK + threadIdx.x; i < n; i += stride) {
    float w = param[i];
    float mm = m != nullptr ? m[i] : 0.f;
    float vv = v != nullptr ? v[i] : 0.f;
    opt_update(o, grad[i], w, mm, vv, bc1, bc2s, anchor, cg, cl, i);
    param[i] = w;
    if (m != nullptr) m[i] = mm;
    if (v != nullptr) v[i] = vv;
    if (shadow != nullptr) shadow[i] = (bf16)w;
  }
}

// t = scale·t + σ·N(0,1), counter-based RNG (splitmix64 + Box-Muller)
__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

__global__ __launch_bounds__(FL_BLOCK) void k_scale_add_noise(float* __restrict__ t, int64_t n, float scale, float sigma, uint64_t seed) {
  const int64_t stride = (int64_t)gridDim.x * FL_BLOCK;
  for (int64_t i = blockIdx.x * FL_BLOCK + threadIdx.x; i < n; i += stride) {
    float val = t[i] * scale;
    if (sigma != 0.f) {
      const uint64_t r = splitmix64(seed * 0x100000001B3ull + (uint64_t)i);
      const float u1 = ((r >> 40) + 1) * (1.0f / 16777217.0f);
      const float u2 = ((r & 0xFFFFFFull)) * (1.0f / 16777216.0f);
      val += sigma * sqrtf(-2.f * __logf(u1)) * __cosf(6.2831853f * u2);
    }
    t[i] = val;
  }
}

// ------------------------------------------------------------------------------------------------
void fl_weighted_sum(float* out, const uint64_t* srcs, const float* w, int K, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_weighted_sum, dim3(grid_for(n / 4 + 1)), dim3(FL_BLOCK), 0, s, out, srcs, w, K, n);
}
void fl_stacked_weighted_sum(float* out, const float* stacked, int P, int64_t n, int64_t ld, const float* w, float scale, hipStream_t s) {
  hipLaunchKernelGGL(k_stacked_weighted_sum, dim3(grid_for(n / 4 + 1)), dim3(FL_BLOCK), 0, s, out, stacked, P, n, ld, w, scale);
}
void fl_broadcast_rows(float* stacked, const float* src, int P, int64_t n, int64_t ld, const float* mask, hipStream_t s) {
  unsigned gx = grid_for(n / 4 + 1);
  if (gx > 256) gx = 256;
  hipLaunchKernelGGL(k_broadcast_rows, dim3(gx, P), dim3(FL_BLOCK), 0, s, stacked, src, P, n, ld, mask);
}
void fl_coordinate_median(const OutPtrs& outs, int P, const RowPtrs& rows, int K, int64_t n, hipStream_t s) {
  const dim3 g(grid_for(n)), b(FL_BLOCK);
  switch (K) {
#define MED_CASE(KK) \
  case KK: hipLaunchKernelGGL(k_coordinate_median<KK>, g, b, 0, s, outs, P, rows, n); break;
    MED_CASE(1) MED_CASE(2) MED_CASE(3) MED_CASE(4) MED_CASE(5) MED_CASE(6) MED_CASE(7) MED_CASE(8)
    MED_CASE(9) MED_CASE(10) MED_CASE(11) MED_CASE(12) MED_CASE(13) MED_CASE(14) MED_CASE(15) MED_CASE(16)
#undef MED_CASE
    default: break;
  }
}
void fl_scaffold_reduce(float* buf, const RowPtrs& dy, const RowPtrs& dc, const RowW& w, int K, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_scaffold_reduce, dim3(grid_for(n)), dim3(FL_BLOCK), 0, s, buf, dy, dc, w, K, n);
}
void fl_scaffold_apply(const OutPtrs& outs, int P, const float* x_start, const float* buf, float* c, int c_init, float glr, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(k_scaffold_apply, dim3(grid_for(n)), dim3(FL_BLOCK), 0, s, outs, P, x_start, buf, c, c_init, glr, n);
}
void fl_opt_step(float* param, const float* grad, float* m, float* v, bf16* shadow, int64_t n, const OptParams& o, int step, const float* anchor,
                 const float* cg, const float* cl, hipStream_t s) {
  const float bc1 = 1.f - powf(o.beta1, (float)step);
  const float bc2s = sqrtf(1.f - powf(o.beta2, (float)step));
  hipLaunchKernelGGL(k_opt_step, dim3(grid_for(n)), dim3(FL_BLOCK), 0, s, param, grad, m, v, shadow, n, o, bc1, bc2s, anchor, cg, cl);
}
void fl_scale_add_noise(float* t, int64_t n, float scale, float sigma, uint64_t seed, hipStream_t s) {
  hipLaunchKernelGGL(k_scale_add_noise, dim3(grid_for(n)), dim3(FL_BLOCK), 0, s, t, n, scale, sigma, seed);
}

// Resolve one kernel of this translation unit on the current device: loads the unit's code object
// now (myfyp_warm_all, at engine prewarm) instead of at its first launch, which waited for the
// kernels in flight (the first FedAvg launch blocked the host until the running epoch ended)
extern "C" int myfyp_warm_fl_ops() {
  hipFuncAttributes attr;
  return hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(&k_weighted_sum)) == hipSuccess ? 0 : 1;
}
