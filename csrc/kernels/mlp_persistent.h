// Weight-stationary persistent epoch kernel for the reference MLP family (D1 = 256, D2 = 128).
#pragma once
#include "mlp_fused.h"

// Exchange buffers of one engine (allocated when the persistent path is eligible).
struct MLPPersistBufs {
  bf16* h1x;        // [P][Bpad][256]   owner g -> head: H1 columns 16g..16g+15
  bf16* w2x;        // [P][8][8][64][8]  owner g -> head: updated bf16 W2 in the head's B-fragment order
  bf16* dh2x;       // [P][Bpad][128]   head -> owners: dH2
  unsigned* flags;  // [P][35][32] one 128-B line per flag (16 H1, 16 W2, 1 dH2, 2 XCC reports); zeroed per launch
  size_t flag_bytes;
  int* err;         // sticky give-up word (bounded spins); zeroed per fit
  int plain_ok;     // hand-offs may be stored plain when a gang sits on one XCD (set at launch)
  int plain;        // ... and this gang does (set in the kernel)
};

// Shape / resource check for the persistent path (device-independent part).
bool mlp_persistent_supported(const MLPArgs& a);
size_t mlp_persistent_bytes(int P, int Bpad);  // exchange-buffer bytes (h1x + w2x + dh2x)
size_t mlp_persistent_flag_bytes(int P);
int mlp_persistent_blocks(int P);
hipError_t mlp_persistent_prepare(const MLPArgs& a);  // kernel attributes (once per engine)
// Zero the flags (memset node) and launch one whole epoch for every active peer.
// zero_flags = false: the epoch's gather kernel already zeroed them (MLPArgs::flags_zero).
hipError_t mlp_launch_persistent_epoch(const MLPArgs& a, const MLPPersistBufs& pb, hipStream_t s, bool zero_flags = true);

// ---- fp32 variant (mlp_persistent_f32.hip): exact fp32 products, fp32 accumulation and state;
//      gangs of 16 owners + 8 heads, one launch per group of 8 peers.
struct MLPPersistF32Bufs {
  float* h1x;       // [P][Bpad][256]      owner g -> heads: H1 columns 16g..16g+15
  float* plx;       // [P][8][Bpad*16][2]  head hd -> heads: partial logits over its H2 slice, LL (value, tag) pairs
  float* dh2x;      // [P][2][Bpad][128][2] head hd -> owners: dH2 columns 16hd..16hd+15 (step parity), LL pairs
  unsigned* gen;    // [P] epoch generation of the LL tags (advanced by every completed epoch)
  unsigned* flags;  // [P][32][32] one 128-B line per flag (16 H1, 8 PL, 8 dH2); zeroed per launch
  size_t flag_bytes;
  int* err;         // give-up words: [0,64) per peer first attempt (1 gave up, 2 recovered), [64,128) retry
  unsigned fbase;   // hand-off flag base of the running attempt (set in the kernel)
  float* w2chk;     // debug: owners' W2 replica after the epoch [P][128][256], or null
  int plain_ok;     // fp32 layouts 1 / 3: hand-offs may be stored plain when a gang sits on one XCD (set at launch;
                    // 1 payloads and flags, 2 payloads only, 0 never)
  int plain;        // plain_ok if this gang does, else 0 (set in the kernel); cross-XCD K split: within a group
  int plain_x;      // hand-offs between the groups of a gang (set in the kernel: plain, or 0 for a cross-XCD K split)
};

int mlp_plain_pub_mode();  // single-XCD hand-off mode of the persistent kernels (MYFYP_F32_PLAIN_PUB / mlp_set_plain_pub)
bool mlp_persistent_f32_supported(const MLPArgs& a);
size_t mlp_persistent_f32_h1x_floats(int P, int Bpad);  // H1-partial exchange region at the start of the buffer
size_t mlp_persistent_f32_bytes(int P, int Bpad);
size_t mlp_persistent_f32_flag_bytes(int P);
int mlp_persistent_f32_gang();
int mlp_persistent_f32_resident_capacity(const MLPArgs& a, int num_cus);
int mlp_persistent_f32_launch_wgs(const MLPArgs& a);  // workgroups of one epoch launch
int mlp_persistent_f32_ks(const MLPArgs& a);
int mlp_persistent_f32_variant(const MLPArgs& a);
// 1: this build's fp32 epoch for `a` reads X directly (needs a.Xp16 and the index kernel's xidx / Yb)
int mlp_persistent_f32_x_direct(const MLPArgs& a);
int mlp_persistent_f32_x_direct_build();  // the build's P32_XDIRECT  // gang layout: 1 owners + heads, 2 owners only          // K split of the owners (1 or 2)             // workgroups (CUs) per peer
int mlp_persistent_f32_flags_per_peer();   // u32 words per peer in the flag block
// flag block layout: u32 per flag line, flag lines per peer, and how many of each peer's last lines
// use every word (the gang placement slots); every other line's flag is its word 0
void mlp_persistent_f32_flag_layout(int* line, int* lines_per_peer, int* full_lines);
hipError_t mlp_persistent_f32_prepare(const MLPArgs& a);
// active (nullable, a.P host flags): launches (and retry launches) are enqueued only for the
// groups of ppl peers with an active peer; null: every group (graph capture: any later active set)
hipError_t mlp_launch_persistent_f32_epoch(const MLPArgs& a, const MLPPersistF32Bufs& pb, hipStream_t s, bool zero_flags = true,
                                           const int* active = nullptr);
// fp32 forward of every active peer's whole test split (loss sum, correct, confusion) in one launch
void mlp_launch_eval_f32(const MLPArgs& a, int max_rows, hipStream_t s);
