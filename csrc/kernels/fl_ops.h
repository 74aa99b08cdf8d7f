#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "common.h"

void fl_weighted_sum(float* out, const uint64_t* srcs, const float* w, int K, int64_t n, hipStream_t s);
void fl_stacked_weighted_sum(float* out, const float* stacked, int P, int64_t n, int64_t ld, const float* w, float scale, hipStream_t s);
void fl_broadcast_rows(float* stacked, const float* src, int P, int64_t n, int64_t ld, const float* mask, hipStream_t s);
#define FEDAVG_MAX_PEERS 64
struct FedAvgWeights {
  float w[FEDAVG_MAX_PEERS];
  float wsum;
};
void fl_fedavg_reduce(float* out, float* wsum_slot, const float* stacked, int P, int64_t n, int64_t ld, const FedAvgWeights& w, hipStream_t s,
                      float* out2 = nullptr, float* wsum2 = nullptr);
void fl_fedavg_apply(float* stacked, const float* out, const float* wsum_slot, int P, int64_t n, int64_t ld, unsigned long long mask, hipStream_t s);
void fl_fedavg_delayed_land(float* stacked, float* snap, int64_t ld_snap, const float* avg, const float* wsum_slot, int P, int64_t n, int64_t ld,
                            unsigned long long mask, hipStream_t s);
void fl_fedavg_local(float* stacked, int P, int64_t n, int64_t ld, const FedAvgWeights& w, unsigned long long mask, hipStream_t s);
// Topology mixing of a stacked group in place: row p <- sum_k w[p][k] * row idx[p][k] (P <= 16 rows,
// up to P sources per row; rows with nsrc == 0 are left alone).
#define MIX_MAX_PEERS 16
#define MIX_MAX_SRC MIX_MAX_PEERS  // a row may mix every local peer (full / star topologies)
struct MixPlan {
  float w[MIX_MAX_PEERS][MIX_MAX_SRC];
  unsigned char idx[MIX_MAX_PEERS][MIX_MAX_SRC];
  unsigned char nsrc[MIX_MAX_PEERS];
};
void fl_neighbor_mix(float* stacked, int P, int64_t n, int64_t ld, const MixPlan& m, hipStream_t s);
struct RowPtrs {  // up to 16 row base pointers passed by value
  const float* p[16];
};
struct OutPtrs {  // up to 16 destination rows passed by value
  float* p[16];
};
struct RowW {
  float w[16];
};
// out rows 0..P-1 <- per-coordinate median of rows 0..K-1 (outputs may alias inputs)
void fl_coordinate_median(const OutPtrs& outs, int P, const RowPtrs& rows, int K, int64_t n, hipStream_t s);
// SCAFFOLD server step, packed buffer [Σ w_k dy_k | Σ w_k | Σ dc_k | K] (2n + 2 floats):
//   reduce: buf <- the local contributions (before the cross-rank all-reduce)
//   apply : out rows <- x_start + glr · buf[0:n] / buf[n];  c <- (c_init ? 0 : c) + buf[n+1:2n+1] / buf[2n+1]
void fl_scaffold_reduce(float* buf, const RowPtrs& dy, const RowPtrs& dc, const RowW& w, int K, int64_t n, hipStream_t s);
void fl_scaffold_apply(const OutPtrs& outs, int P, const float* x_start, const float* buf, float* c, int c_init, float glr, int64_t n, hipStream_t s);
void fl_opt_step(float* param, const float* grad, float* m, float* v, bf16* shadow, int64_t n, const OptParams& o, int step, const float* anchor,
                 const float* cg, const float* cl, hipStream_t s);
void fl_scale_add_noise(float* t, int64_t n, float scale, float sigma, uint64_t seed, hipStream_t s);
