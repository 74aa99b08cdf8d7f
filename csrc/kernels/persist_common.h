// Device helpers shared by the weight-stationary persistent epoch kernels (mlp_persistent.hip,
// mlp_persistent_f32.hip): in-launch hand-offs between the workgroups of a peer's gang, Adam bias
// correction, and 16-lane DPP row reductions.
//
// Hand-off protocol (cdna_hip_programming.md §6 Guideline 16, valid form row 1 of
// MI355X_MICROARCH.md's hand-off table): payload stored write-through (sc1), every storing wave
// drains its stores, the workgroup meets, ONE lane stores a relaxed agent-scope flag = step + 1;
// the consumer polls relaxed from one wave, meets its workgroup, and reads every payload byte with
// sc1 loads (no acquire fence needed). Flags are monotone within a launch and zeroed per launch.
#pragma once
#include "common.h"

namespace persist {

typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;

constexpr int FLAG_LINE = 32;                            // u32 per flag: one 128-byte line each
constexpr unsigned long long SPIN_TICKS = 100000000ull;  // wall_clock64 runs at 100 MHz: 1 s

// Poll loops: the hand-off's own load is the only memory round trip of an iteration. The gang's
// error word (another L2 round trip) and the clock (s_memrealtime, a scalar-memory round trip)
// are read on every PERSIST_POLL_EVERY-th iteration only: before, each iteration serialised three
// round trips, so a flag that flipped was seen on average 1.5 of them late, on every hand-off of
// every step. Timeouts and give-ups are still seen within PERSIST_POLL_EVERY iterations.
// No s_sleep between polls (PERSIST_POLL_SLEEP 0): a polling wave has one load in flight at a time
// either way. Measured on the 8-peer headline (profiles/r6v_poll, 3 runs each): every poll 627.0 /
// 622.8 / 625.6 rounds/s, every 32nd + s_sleep 1 628.5 / 631.1 / 630.7, every 32nd without the
// sleep 637.8 / 637.5 / 635.7
#ifndef PERSIST_POLL_EVERY
#define PERSIST_POLL_EVERY 32
#endif
#ifndef PERSIST_POLL_SLEEP
#define PERSIST_POLL_SLEEP 0
#endif
static_assert((PERSIST_POLL_EVERY & (PERSIST_POLL_EVERY - 1)) == 0, "PERSIST_POLL_EVERY: a power of two");
__device__ __forceinline__ bool poll_check(unsigned it) { return (it & (PERSIST_POLL_EVERY - 1)) == 0; }
__device__ __forceinline__ void poll_sleep() {
  if (PERSIST_POLL_SLEEP > 0) __builtin_amdgcn_s_sleep(PERSIST_POLL_SLEEP);
}

__device__ __forceinline__ unsigned* flag_at(unsigned* flags, int flags_per_peer, int p, int idx) {
  return flags + ((size_t)p * flags_per_peer + idx) * FLAG_LINE;
}
__device__ __forceinline__ void st_wt(void* ptr, unsigned long long v) {  // 8-byte write-through store
  __hip_atomic_store((gu64*)ptr, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt32(float* ptr, float v) {  // 4-byte write-through store
  __hip_atomic_store((gu32*)ptr, __builtin_bit_cast(unsigned, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
typedef unsigned u32x4_t __attribute__((ext_vector_type(4)));
// 16-byte write-through (sc1) store at byte offset `off` (per lane) of a UNIFORM base: the buffer
// resource must be wave-uniform (a per-lane base would be read from the first lane only)
__device__ __forceinline__ void st_wt128(float* base, int bytes, int off, u32x4_t v) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, bytes, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16);
}
// Hand-off payload stores by gang placement: write-through (sc1) in general; plain when every
// workgroup of the gang was seen on ONE XCD (the line then stays in that XCD's L2, which is where
// the consumers' L1-bypassing loads look; sc1 stores drop it, and a same-XCD reader then reads at
// the cross-XCD rate: MI355X_MICROARCH.md). Placement is checked at run time (gang_same_xcd), never
// assumed: round-robin dispatch is observed behaviour, not a HIP guarantee.
__device__ __forceinline__ void pub32(int plain, float* ptr, float v) {
  if (plain)
    *ptr = v;
  else
    __hip_atomic_store((gu32*)ptr, __builtin_bit_cast(unsigned, v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void pub128(int plain, float* base, int bytes, int off, u32x4_t v) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, bytes, 0x00020000);
  if (plain)
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 0);
  else
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16);
}

// Gang placement check at kernel entry: role `role` of `nr` (nr <= 64) stores mark | its XCC id into
// slots[role] (zeroed per launch; `mark` differs per attempt, 0x100 or 0x200), wave 0 polls all nr
// slots (bounded by `ticks`), and the workgroup learns whether every role reported the same XCC.
// Any timeout answers false (write-through stays, always correct). `word` is an LDS int.
__device__ __forceinline__ int gang_same_xcd(unsigned* slots, int role, int nr, unsigned mark, int* word, unsigned long long ticks) {
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  xcc &= 0xFFu;
  if (threadIdx.x == 0) __hip_atomic_store((gu32*)(slots + role), mark | xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const unsigned long long t0 = wall_clock64();
    int same = 1;
    unsigned v = mark | xcc;
    for (;;) {
      if (lane < nr) v = __hip_atomic_load((gu32*)(slots + lane), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__all((v & ~0xFFu) == mark)) break;
      if (wall_clock64() - t0 > ticks) {
        same = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (same) same = __all((v & 0xFFu) == xcc) ? 1 : 0;
    if (lane == 0) *(volatile int*)word = same;
  }
  __syncthreads();
  const int r = *(volatile int*)word;
  __syncthreads();  // the word may be reused by the caller's LDS carving
  return r;
}

// The same check for a GROUP of roles (first + k·stride, k < n <= 64) that hands off among itself:
// role `role` reports into slots[role] and learns whether every member of its group reported its own
// XCC. Members of different groups may sit on different XCDs (the cross-XCD K split).
__device__ __forceinline__ int group_same_xcd(unsigned* slots, int role, int first, int stride, int n, unsigned mark, int* word,
                                              unsigned long long ticks) {
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  xcc &= 0xFFu;
  if (threadIdx.x == 0) __hip_atomic_store((gu32*)(slots + role), mark | xcc, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const unsigned long long t0 = wall_clock64();
    int same = 1;
    unsigned v = mark | xcc;
    for (;;) {
      if (lane < n) v = __hip_atomic_load((gu32*)(slots + first + lane * stride), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__all((v & ~0xFFu) == mark)) break;
      if (wall_clock64() - t0 > ticks) {
        same = 0;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (same) same = __all((v & 0xFFu) == xcc) ? 1 : 0;
    if (lane == 0) *(volatile int*)word = same;
  }
  __syncthreads();
  const int r = *(volatile int*)word;
  __syncthreads();
  return r;
}

__device__ __forceinline__ unsigned long long ld_wt(const void* ptr) {  // 8-byte L1-bypassing load
  return __hip_atomic_load((gu64*)ptr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Producer side: every storing wave drains its write-through stores, the workgroup meets, ONE lane
// stores the flag (sc1).
__device__ __forceinline__ void publish(unsigned* flags, int fpp, int p, int idx, unsigned value) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_store((gu32*)flag_at(flags, fpp, p, idx), value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// publish() for a gang found on one XCD (plain != 0): the flag is stored without sc1 as well, so its
// line stays in that XCD's L2, where the consumers' sc1 polls read it (a workgroup-scope atomic store
// is a plain store the compiler keeps; the empty asm keeps it ahead of the caller's wait loop)
__device__ __forceinline__ void publish_p(unsigned* flags, int fpp, int p, int idx, unsigned value, int plain) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    if (plain == 1) {  // (2: payloads plain, flags written through — A/B)
      __hip_atomic_store((gu32*)flag_at(flags, fpp, p, idx), value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      asm volatile("" ::: "memory");
    } else {
      __hip_atomic_store((gu32*)flag_at(flags, fpp, p, idx), value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// Consumer side: wave 0 polls flags idx0..idx0+n-1 (one lane each, relaxed sc1 loads + s_sleep)
// until all reach `target`, then the workgroup meets; every later load of the handed-off bytes is
// an sc1 load. Bounded: gives up after `ticks` or when another workgroup gave up.
//
// PERSIST_WAVE_POLL (A/B build): every wave polls the flags itself and goes on to its payload loads
// when it sees them, without the workgroup meet (flags are monotone within a launch: a wave that
// saw them set cannot disagree with another; a wave that times out or sees the error word returns
// false and the caller's wave leaves the kernel, which a later barrier of the others tolerates).
// Measured within noise of the meet (profiles/r6z_wavepoll: 641.7 / 616.9 / 637.3 vs 641.1 / 610.3 /
// 639.8 rounds/s): off.
__device__ __forceinline__ bool wg_wait(unsigned* flags, int fpp, int p, int idx0, int n, unsigned target, int* err, int* sOk,
                                        unsigned long long ticks = SPIN_TICKS) {
#ifdef PERSIST_WAVE_POLL
  {
    const int lane = threadIdx.x & 63;
    const unsigned* f = flag_at(flags, fpp, p, idx0 + (lane < n ? lane : 0));
    const unsigned long long t0 = wall_clock64();
    for (unsigned it = 1;; ++it) {
      const unsigned v = lane < n ? __hip_atomic_load((gu32*)f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : target;
      if (__all(v >= target)) break;
      if (poll_check(it)) {
        if (__hip_atomic_load((gu32*)err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return false;
        if (wall_clock64() - t0 > ticks) {
          if (lane == 0) __hip_atomic_store((gu32*)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          return false;
        }
      }
      poll_sleep();
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    return true;
  }
#endif
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const unsigned* f = flag_at(flags, fpp, p, idx0 + (lane < n ? lane : 0));
    const unsigned long long t0 = wall_clock64();
    int ok = 1;
    for (unsigned it = 1;; ++it) {
      const unsigned v = lane < n ? __hip_atomic_load((gu32*)f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : target;
      if (__all(v >= target)) break;
      if (poll_check(it)) {
        if (__hip_atomic_load((gu32*)err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
          ok = 0;
          break;
        }
        if (wall_clock64() - t0 > ticks) {
          if (lane == 0) __hip_atomic_store((gu32*)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok = 0;
          break;
        }
      }
      poll_sleep();
    }
    if (lane == 0) *sOk = ok;
  }
  __syncthreads();
  const int ok = *sOk;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // keeps the payload loads below the poll
  return ok != 0;
}

// ---- LL hand-off (the "low latency" protocol of RCCL): every 4-byte payload word travels with a
// 4-byte tag in ONE naturally aligned 8-byte store, so the consumer's load of the data is its own
// readiness check — no drain of the producer's stores, no workgroup meet and no flag store on the
// producer side (the flag protocol above costs two L2 round trips more per hand-off). The tag is
// unique per (epoch generation, attempt, step): stale pairs of an earlier step or launch never match.
__device__ __forceinline__ unsigned ll_tag(unsigned gen, unsigned fbase, int t) {
  return ((gen & 0xFFFu) << 20) | (fbase ? (1u << 19) : 0u) | (unsigned)(t + 1);
}
typedef unsigned ll_u32x4 __attribute__((ext_vector_type(4)));
// 16-byte write-through store of two LL pairs {v0, tag, v1, tag} at byte offset `off` of a uniform base
__device__ __forceinline__ void ll_st2(float* base, int bytes, int off, float v0, float v1, unsigned tag) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, bytes, 0x00020000);
  const ll_u32x4 v = {__builtin_bit_cast(unsigned, v0), tag, __builtin_bit_cast(unsigned, v1), tag};
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16);
}
// 8-byte write-through store of one LL pair
__device__ __forceinline__ void ll_st1(float* pair, float v, unsigned tag) {
  st_wt(pair, ((unsigned long long)tag << 32) | __builtin_bit_cast(unsigned, v));
}
// LL stores for a gang found on one XCD (plain: the pair stays in that XCD's L2; one 8- or 16-byte
// store instruction each, as for the write-through form)
__device__ __forceinline__ void ll_st1p(int plain, float* pair, float v, unsigned tag) {
  const unsigned long long w = ((unsigned long long)tag << 32) | __builtin_bit_cast(unsigned, v);
  if (plain)
    __hip_atomic_store((gu64*)pair, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  else
    st_wt(pair, w);
}
__device__ __forceinline__ void ll_st2p(int plain, float* base, int bytes, int off, float v0, float v1, unsigned tag) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, (short)0, bytes, 0x00020000);
  const ll_u32x4 v = {__builtin_bit_cast(unsigned, v0), tag, __builtin_bit_cast(unsigned, v1), tag};
  if (plain)
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 0);
  else
    __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, 16);
}
// 16-byte L1-bypassing load of two LL pairs
__device__ __forceinline__ ll_u32x4 ll_ld2(__amdgpu_buffer_rsrc_t r, int off) { return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16); }
__device__ __forceinline__ bool ll_ok2(const ll_u32x4& v, unsigned tag) { return v[1] == tag && v[3] == tag; }
// Payload words of a received chunk: read them with __uint_as_float(v[i]). amdclang 22 (ROCm 7.2)
// miscompiles __builtin_bit_cast(float, v[i]) on an ext-vector ELEMENT lvalue: it reads element 0
// whatever i is (tests/test_kernel_lint.py rejects the pattern).

// Consumer side of an LL hand-off with N 16-byte chunks per lane: `load(k)` issues chunk k's load;
// spins (s_sleep between polls, chunks that already matched are not reloaded) until every chunk of
// every lane of the wave carries `tag`. Bounded like wg_wait: false when the gang gave up (err set by
// any workgroup) or after `ticks`.
template <int N, class Load>
__device__ __forceinline__ bool ll_wait(ll_u32x4 (&v)[N], Load load, unsigned tag, int* err, unsigned long long ticks = SPIN_TICKS) {
#pragma unroll
  for (int k = 0; k < N; ++k) v[k] = load(k);
  unsigned long long t0 = 0;
  for (unsigned it = 1;; ++it) {
    bool ready = true;
#pragma unroll
    for (int k = 0; k < N; ++k) ready = ready && ll_ok2(v[k], tag);
    if (__all(ready)) return true;
    if (it == 1 || poll_check(it)) {
      if (__hip_atomic_load((gu32*)err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return false;
      const unsigned long long now = wall_clock64();
      if (t0 == 0) {
        t0 = now;
      } else if (now - t0 > ticks) {
        if ((threadIdx.x & 63) == 0) __hip_atomic_store((gu32*)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return false;
      }
    }
    poll_sleep();
#pragma unroll
    for (int k = 0; k < N; ++k)
      if (!ll_ok2(v[k], tag)) v[k] = load(k);
  }
}

// Representative wait of an LL hand-off with n <= 64 producers (long waits: the consumer workgroup
// must not hammer L2 with bulk polls): wave 0, lane k < n, polls one 16-byte chunk of producer k
// (`probe(k)` issues its load) until its tags match, then the workgroup meets; the bulk loads that
// follow still verify every tag (ll_wait), since a producer's other chunks may land later.
template <class Probe>
__device__ __forceinline__ bool ll_wg_wait(Probe probe, int n, unsigned tag, int* err, int* sOk, unsigned long long ticks = SPIN_TICKS) {
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    const int k = lane < n ? lane : 0;
    const unsigned long long t0 = wall_clock64();
    int ok = 1;
    for (unsigned it = 1;; ++it) {
      const bool ready = lane >= n || ll_ok2(probe(k), tag);
      if (__all(ready)) break;
      if (poll_check(it)) {
        if (__hip_atomic_load((gu32*)err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
          ok = 0;
          break;
        }
        if (wall_clock64() - t0 > ticks) {
          if (lane == 0) __hip_atomic_store((gu32*)err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok = 0;
          break;
        }
      }
      poll_sleep();
    }
    if (lane == 0) *sOk = ok;
  }
  __syncthreads();
  const int ok = *sOk;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  return ok != 0;
}

// Per-step optimizer constants: lr_t = lr / (1 - β1^k), inv = 1 / sqrt(1 - β2^k), k = t0 + t + 1.
__device__ __forceinline__ void bias_corr(const OptParams& o, int t0, int t, float& lr_t, float& inv) {
  const int k = t0 + t + 1;
  lr_t = o.lr / (1.f - __powf(o.beta1, (float)k));
  inv = 1.f / sqrtf(1.f - __powf(o.beta2, (float)k));
}

// Running Adam bias corrections for the fp32 epoch: torch computes 1 - β^k in double on the host
// every step; here the powers advance by one f64 multiply per step (exact to ~1e-16 relative)
// instead of two fp32 pow() calls per step, ~150 VALU instructions at the head of every step.
// The powers are wave-uniform: they live in SGPRs (readfirstlane), not in the VGPR budget.
__device__ __forceinline__ double uniform_f64(double v) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)u), hi = __builtin_amdgcn_readfirstlane((unsigned)(u >> 32));
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
__device__ __forceinline__ float uniform_f32(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(unsigned, v)));
}
struct BiasCorr {
  double b1k, b2k;  // β1^k, β2^k of the last step produced
  __device__ __forceinline__ void init(const OptParams& o, int t0) {
    b1k = uniform_f64(pow((double)o.beta1, (double)t0));
    b2k = uniform_f64(pow((double)o.beta2, (double)t0));
  }
  // advance to the next optimizer step k and return lr / (1 - β1^k), 1 / sqrt(1 - β2^k)
  __device__ __forceinline__ void next(const OptParams& o, float& lr_t, float& inv) {
    b1k = uniform_f64(b1k * (double)o.beta1);
    b2k = uniform_f64(b2k * (double)o.beta2);
    lr_t = uniform_f32((float)((double)o.lr / (1.0 - b1k)));
    inv = uniform_f32((float)(1.0 / sqrt(1.0 - b2k)));
  }
};

// 16-lane (one MFMA row group) butterfly reductions on DPP: quad_perm xor1, xor2, then
// row_half_mirror and row_mirror — VALU-latency instead of ds_bpermute round trips.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
template <int CTRL>
__device__ __forceinline__ int dpp_i(int v) {
  return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xf, 0xf, false);
}
__device__ __forceinline__ float row_max16(float v) {
  v = fmaxf(v, dpp_f<0xB1>(v));
  v = fmaxf(v, dpp_f<0x4E>(v));
  v = fmaxf(v, dpp_f<0x141>(v));
  return fmaxf(v, dpp_f<0x140>(v));
}
__device__ __forceinline__ float row_sum16(float v) {
  v += dpp_f<0xB1>(v);
  v += dpp_f<0x4E>(v);
  v += dpp_f<0x141>(v);
  return v + dpp_f<0x140>(v);
}
__device__ __forceinline__ int row_min16(int v) {
  v = min(v, dpp_i<0xB1>(v));
  v = min(v, dpp_i<0x4E>(v));
  v = min(v, dpp_i<0x141>(v));
  return min(v, dpp_i<0x140>(v));
}

__host__ __device__ inline size_t al16(size_t v) { return (v + 15) / 16 * 16; }

}  // namespace persist
