// Argument block shared by the grouped fused-MLP kernels and the engine.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "common.h"

#define MLP_EVAL_CHUNK 512
#define MLP_MAX_BPAD 256  // largest padded local batch the fused engine supports

struct MLPArgs {
  int P, D0, D1, D2, D3, D0pad;
  int64_t S;       // per-peer stride (elements) of params/shadow/m/v
  int64_t numel;   // trainable elements per peer
  int64_t off_w1, off_b1, off_w2, off_b2, off_w3, off_b3;
  // parameters and optimizer state, [P][S]
  float* params;
  bf16* shadow;
  bf16* w2t;       // [P][D1][D2] transposed bf16 copy of W2
  float* m;
  float* v;
  const float* anchor;  // FedProx anchor [P][S] or null
  const float* cg;      // SCAFFOLD global control variate [P][S] or null
  const float* cl;      // SCAFFOLD local control variate  [P][S] or null
  // training data: per-peer device pointers (uint8 [n][D0] images, int32 labels) + counts
  const uint8_t* const* Xp;
  const int* const* Yp;
  const int* n;
  const int* perm;  // [P][perm_stride] local indices (epoch permutation)
  int64_t perm_stride;
  int shuffle_native;                // 1: permutation drawn in the gather kernel from *seed
  const unsigned long long* seed;    // epoch shuffle key (device word, uploaded per epoch)
  // the epoch's batches, gathered once in permutation order at the start of the epoch so that the
  // per-step kernels read contiguous rows instead of chasing perm -> pointer table -> row
  uint8_t* Xb;      // [P][xb_rows][D0]
  bf16* Xb16;       // same batches as bf16 (persistent path; null otherwise)
  int* Yb;          // [P][xb_rows]
  int64_t xb_rows;  // max_steps * B
  // direct-X epochs (fp32 layout 1): the kernel reads each batch row from a static exact-bf16 copy of
  // the peer's images through the epoch's sample index (xidx), so no per-epoch image gather runs;
  // the epoch's index / label kernel (mlp_index_epoch) writes xidx and Yb
  const bf16* const* Xp16;  // [P] device pointers to [n_p][D0] bf16 images (or null)
  int* xidx;                // [P][xb_rows] sample index of each epoch position
  int x_direct;             // 1: the fp32 layout-1 epoch reads X through xidx / Xp16
  unsigned* flags_zero;  // persistent epoch: hand-off flag lines zeroed by the gather kernel (or null)
  int flags_per_peer;    // u32 words per peer
  // test data
  const uint8_t* const* Xtp;
  const int* const* Ytp;
  const int* n_t;
  // control
  const int4* ctl;    // [P] {active (bit 0; bit 1 = fresh optimizer state), n_train, optimizer steps already
                      //      taken (t0), n_test} — one scalar load
  const int* active;  // [P]
  const int* t0;      // [P] optimizer steps each peer already took in this fit
  // workspace
  bf16* H1;   // [P][h1_rows][D1]
  int h1_rows;
  bf16* H1T;  // [P][D1][Bpad]
  bf16* XT;   // unused (Xᵀ slabs are staged in LDS by the wgrad kernel)
  bf16* H2T;  // [P][D2][Bpad]
  bf16* dH2T; // [P][D2][Bpad]
  bf16* dH1T; // [P][D1][Bpad]
  bf16* dlogT;// [P][16][Bpad]
  int B, Bpad;
  // accumulators
  float* loss_acc;   // [P]
  int* correct_acc;  // [P]
  int* conf;         // [P][16][16] (eval) or null
  OptParams opt;
  int debug_giveup;  // fp32 persistent epoch test hook: peer + 1 whose first attempt gives up (0 = none)
  int f32_ks;        // fp32 persistent epoch owner K split: 1, 2, or 0 = by P
  int f32_variant;   // fp32 persistent epoch gang layout: 1 owners + heads, 2 owners only, 0 = default
};

bool mlp_shape_supported(int D0, int D1, int D2, int D3);
void mlp_launch_train_step(const MLPArgs& a, int step, hipStream_t s);
void mlp_launch_eval_chunk(const MLPArgs& a, int base, hipStream_t s);
void mlp_launch_sync_shadow(const MLPArgs& a, hipStream_t s);
// the epoch's sample index and labels (direct-X epochs); zeroes the hand-off flags like the gather
void mlp_launch_index_epoch(const MLPArgs& a, hipStream_t s);
// max_wgs > 0 caps the grid (at least one workgroup per peer); rows are grid-strided
void mlp_launch_gather_epoch(const MLPArgs& a, hipStream_t s, int max_wgs = 0);
