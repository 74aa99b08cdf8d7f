// Grouped NHWC bf16 convolution / BatchNorm / pooling / loss kernels for the CNN engine
// (LeNet-5, ResNet-18; BASELINE configs 3-5). Every kernel handles P co-located peers in one
// launch (grid.z = peer): a peer's tensors live at base + peer * peer_stride.
//
// Layouts
//   activations : [rows = n*H*W][Cp] bf16, Cp = round_up(C, 8) (padding channels are kept zero)
//   conv weights: fp32 master in the flat parameter buffer, torch order [Cout][Cin][R][S];
//                 one bf16 shadow Wf[Cp_out][R][S][Cp_in] (forward B operand K-contiguous; the
//                 dgrad reads it N-contiguous through the LDS transpose read);
//                 gradient in the same Wf layout, fp32
//   fc layers   : 1x1 convolutions on a 1x1 image (H = W = 1)
#pragma once
#include <stdint.h>

#include "common.h"

struct ConvGemmArgs {
  // A operand gather source: FWD = input activations X, DGRAD = output gradient dY
  const bf16* src; int64_t src_ps;      // peer stride (elements)
  int src_h, src_w, src_c;              // spatial dims + channel stride of src
  // geometry of the rows (M) this GEMM produces: FWD = output pixels, DGRAD = input pixels
  int out_h, out_w;
  int R, S, stride, pad;
  // B operand: the Wf shadow (FWD: [Ncol][K], K = R*S*src_c; DGRAD: [co][R*S][Ncol])
  const bf16* wt; int64_t wt_ps;
  int ncol;          // output channel stride (Cp_out for FWD, Cp_in for DGRAD = Wf row length)
  int ncol_valid;    // logical channels (columns >= ncol_valid are written as 0)
  // epilogue
  bf16* out; int64_t out_ps;
  const float* bias; int64_t bias_ps;   // optional, per column
  const bf16* resid; int64_t resid_ps;  // optional, same layout as out (added before relu)
  int relu;
  float* stats; int64_t stats_ps;       // optional BN partial sums [2*tiles_m][2][ncol]
  // per-peer valid batch (rows = nb * out_h * out_w); nullptr = all max_batch rows
  const int* nbatch;
  int max_batch;
  // MODE 0 prologue (optional): src holds a BatchNorm INPUT y; the A operand is relu(y*sc + sh)
  // per channel ([sc | sh], 2*src_c floats per peer), padding taps stay 0 — the BN-apply + ReLU
  // pass that would materialise it is skipped
  const float* pro_ss; int64_t pro_ss_ps;
  // dgrad epilogue (optional, MODE 1/2): the output is the gradient dz of a ReLU(BatchNorm) output.
  // out = g = bf16(acc + resid) * [mask > 0], and the BN-backward column sums (sum g, sum g*xhat)
  // accumulate into bnb_part0/1 ([sum g | sum g*xhat] per channel, 2*ncol floats per peer) for up to
  // two BatchNorms whose inputs y0/y1 share that gradient (a block's BN2 and its projection BN);
  // xhat = (y - mean) * inv from bnb_ms0/1 ([mean | inv], 2*ncol per peer). Replaces the separate
  // k_bn_bwd_reduce pass over (dz, mask, y).
  const bf16* bnb_mask; int64_t bnb_mask_ps;
  const bf16* bnb_y0; int64_t bnb_y0_ps;
  const bf16* bnb_y1; int64_t bnb_y1_ps;
  const float* bnb_ms0; const float* bnb_ms1;
  float* bnb_part0; float* bnb_part1; int64_t bnb_part_ps;
  // accumulator rows of `stats` ([rows][2][ncol] per peer; 0 = 1): the epilogue of M tile t adds
  // into row t % rows, so the tiles' fp32 atomics spread over `rows` addresses per column
  int stats_rows;
  int bnb_rows;  // same for the BN-backward partials bnb_part0/1 ([rows][2][ncol] per peer)
  // dgrad epilogue: the ReLU mask of the output comes from y0 itself, mask = (y0*sc + sh > 0) with
  // this [sc | sh] (2*ncol floats per peer) — the activation relu(BN(y0)) was never materialised
  // (its consumers read y0 through a BN prologue). Used when bnb_mask is null.
  const float* bnb_mask_ss; int64_t bnb_mask_ss_ps;
  // fused BatchNorm finalize (optional, fin_cnt != nullptr; conv_fin_tail): the last workgroup of a
  // peer to finish turns that peer's accumulator rows into the BN constants, in place of a
  // k_bn_finalize (fin_ss set: `stats` rows, or the running statistics when fin_train is 0) or
  // k_bn_bwd_finalize (fin_ss null: bnb_part0/1 -> fin_coef0/1 and dgamma/dbeta) launch.
  // fin_cnt: conv_fin_words() arrival-counter ints per peer, 0 between launches (re-armed in-kernel)
  int* fin_cnt;
  const float* fin_gamma0; const float* fin_gamma1; const float* fin_beta;  // [peer * fin_param_ps + c]
  int64_t fin_param_ps;
  float* fin_rmean; float* fin_rvar; int64_t fin_run_ps;  // forward: running statistics
  float* fin_ss; float* fin_ms;                            // forward: [sc | sh], [mean | inv] (2*ncol per peer)
  float* fin_dgamma0; float* fin_dbeta0; float* fin_dgamma1; float* fin_dbeta1;  // dgrad: flat gradient
  float* fin_coef0; float* fin_coef1;                      // dgrad: apply coefficients (3*ncol per peer)
  int fin_C0, fin_C1;                                      // logical channels of BN 0 / 1
  int fin_train;
  float fin_eps, fin_momentum;
  int fin_dbg;  // set by conv_gemm_launch from conv_set_fin_debug (timing probe only; 0 in use)
};

struct WgradArgs {
  const bf16* dy; int64_t dy_ps;        // [rows][dy_c] (rows = n*Ho*Wo)
  const bf16* x; int64_t x_ps;          // [n*H*W][x_c]
  int H, W, x_c, Ho, Wo, dy_c;
  int R, S, stride, pad;
  float* grad; int64_t grad_ps;         // Wf layout [dy_c][R][S][x_c] fp32
  int accumulate;                       // 1: atomic add (required when splits > 1), 0: store
  int k_per_split;                      // rows of M per split (multiple of 64)
  const int* nbatch;
  int max_batch;
  // optional prologue on x: relu(x*sc + sh) per channel (see ConvGemmArgs::pro_ss)
  const float* pro_ss; int64_t pro_ss_ps;
};

extern "C" {
int conv_gemm_launch(int mode, const ConvGemmArgs* a, int peers, void* stream);
int conv_fin_words(void);
int conv_args_abi(long long* out);
int conv_set_fin_debug(int bits);
int conv_set_dma(int on);
int conv_set_dma_wgs(int n);
int conv_set_wgrad_halo(int on);
int conv_set_fwd_halo(int on);  // layer-1 forward / stride-1 dgrad from one staged patch per tile (1, default)  // 64-channel 3x3 wgrads from one staged X patch (1, default) or the generic kernel  // persistent DMA conv: workgroups per launch (0 = auto)  // forward-shaped convs via the LDS-DMA kernel (1, default) or the register stage (0); -1 queries
int conv_wgrad_launch(const WgradArgs* a, int peers, int splits, void* stream);
int conv_wt_flip_launch(const void* wf, long long wf_ps, void* wt, long long wt_ps, int cout, int cin, int R, int S, int peers, void* stream);
int conv_wt_flip_multi_launch(const void* wf, long long wf_ps, void* wt, long long wt_ps, int n, const long long* offs, const int* dims, int peers,
                              void* stream);
int conv_wt_flip_parity_launch(const void* wf, long long wf_ps, void* wt, long long wt_ps, int cout, int cin, int R, int S, int pad, int peers,
                               void* stream);
}
