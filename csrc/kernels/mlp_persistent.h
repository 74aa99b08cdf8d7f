// Weight-stationary persistent epoch kernel for the reference MLP family (D1 = 256, D2 = 128).
#pragma once
#include "mlp_fused.h"

// Exchange buffers of one engine (allocated when the persistent path is eligible).
struct MLPPersistBufs {
  bf16* h1x;        // [P][Bpad][256]   owner g -> head: H1 columns 16g..16g+15
  bf16* w2x;        // [P][8][8][64][8]  owner g -> head: updated bf16 W2 in the head's B-fragment order
  bf16* dh2x;       // [P][Bpad][128]   head -> owners: dH2
  unsigned* flags;  // [P][33][32] one 128-B line per flag (16 H1, 16 W2, 1 dH2); zeroed per launch
  size_t flag_bytes;
  int* err;         // sticky give-up word (bounded spins); zeroed per fit
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
