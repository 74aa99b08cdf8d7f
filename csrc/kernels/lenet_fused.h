// Fused LeNet-5 train / eval step for the grouped CNN engine (BASELINE config 3).
#pragma once
#include <cstdint>

#include "common.h"

struct LenetArgs {
  // data: per-peer uint8 HWC images and int64 labels (device pointer tables), sample counts, epoch permutation
  const uint8_t* const* xs;
  const int64_t* const* ys;
  const int* n_samples;
  const int* perm;  // [P][perm_ps] or null (evaluation: identity)
  int64_t perm_ps;
  int offset;  // first sample of this step
  int B;       // batch (per peer)
  float scale;
  // parameters: bf16 Wf shadows [cp_out][R][S][cp_in] and fp32 biases (torch order), per-peer rows
  const bf16* shadow;
  int64_t shadow_ps;
  int64_t w_c1, w_c2, w_f1, w_f2, w_f3;
  const float* params;
  int64_t params_ps;
  int64_t b_c1, b_c2, b_f1, b_f2, b_f3;
  // gradients: Wf-layout fp32 and torch-order biases, written by the second kernel (no atomics)
  float* gf;
  int64_t gf_ps;
  float* g;
  int64_t g_ps;
  // fc activations handed from the step kernel to the fc weight-gradient kernel: [P][act_ps] bf16
  bf16* act;
  int64_t act_ps;
  // per-workgroup conv gradient records [P][B / ipw][4832] fp32 (reduced by the second kernel)
  float* part;
  int64_t part_ps;
  // fused optimizer (SGD + momentum / weight decay / Nesterov / FedProx / SCAFFOLD) applied by the
  // second kernel where each gradient is produced: master rows, momentum and bf16 shadow updated in
  // place (no k_opt_step launch). mom == null: gradients only (into gf / g).
  float* wmaster;  // the params rows (writable view)
  float* mom;
  bf16* shadow_rw;
  const float* anchor;
  const float* cg;
  const float* cl;
  OptParams opt;
  int64_t t_c1, t_c2, t_f1, t_f2, t_f3;  // torch-order offsets of the weight tensors
  const int* f1_e2t;                     // fc1: engine input column -> torch column
  // outputs
  float* stats;    // [P][4]: loss sum, correct
  int* confusion;  // [P][16][16] or null
  int* nb;         // [P] valid samples of this step (read by the optimizer)
  int train;
};

extern "C" {
// Shapes the fused path implements: 3x32x32 input, conv 5x5 (3->6, 6->16), fc 400-120-84-10, B % ipw == 0.
int lenet_fused_supported(int in_c, int in_h, int c1, int c2, int f1, int f2, int f3, int B);
// One step for every peer: the fused forward/backward kernel and (train) the fc weight-gradient kernel.
int lenet_fused_step(const LenetArgs* a, int peers, int ipw, void* stream);
int lenet_args_size();
}
