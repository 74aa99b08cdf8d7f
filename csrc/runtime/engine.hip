// C++ runtime for the grouped fused-MLP engine + the C ABI of libmyfyp_hip.so.
//
// MLPEngine owns the per-step workspace of P co-located peers and a hipGraph holding one whole
// local epoch (steps × {fc1_fwd, head, wgrad_opt}). A round's local training is then a single
// hipGraphLaunch per epoch from the calling thread — Python (and the GIL) is off the per-step
// path, and launch overhead is amortised by the graph (cdna_hip_programming.md §5.6 verdict:
// launch-bound chains of small kernels belong in hipGraphs, not in a grid-barrier megakernel).
//
// Every entry point returns 0 on success, non-zero on failure (message via myfyp_last_error()).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <chrono>
#include <atomic>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "../kernels/fl_ops.h"
#include "../kernels/mlp_fused.h"
#include "../kernels/mlp_persistent.h"
#include <cstdlib>

static thread_local std::string g_last_error;

#define CHECK_HIP(expr)                                                                   \
  do {                                                                                    \
    hipError_t _e = (expr);                                                               \
    if (_e != hipSuccess) {                                                               \
      g_last_error = std::string(#expr) + ": " + hipGetErrorString(_e);                   \
      return 1;                                                                           \
    }                                                                                     \
  } while (0)

namespace {

// Control words / active mask travel as kernel arguments (captured at launch), so the host never
// enqueues a copy from pageable memory: nothing on the round's path blocks the host on the GPU.
#define MLP_CTL_MAX 64
// give-up words of a fit: [0, 64) per-peer first attempt (1 gave up, 2 recovered by the retry
// launch), [64, 128) per-peer retry; the bf16 epoch uses word 0 for the whole launch
#define MLP_ERR_WORDS 128
struct CtlUpload {
  int4 ctl[MLP_CTL_MAX];
  int active[MLP_CTL_MAX];
  unsigned long long seed;  // epoch shuffle key (in-kernel permutation)
  int P;
  int with_active;
  // accumulators zeroed by the same launch (null = leave): the fit's loss / correct / give-up word,
  // or the evaluation's loss / correct / confusion
  float* zero_loss;
  int* zero_correct;
  int* zero_err;
  int* zero_conf;
  unsigned* zero_flags;  // the persistent epoch's hand-off flags (prep-stream gather mode)
  int n_flags;
  // fp32 flag block: only word 0 of each flag line is a flag, except the last `flag_full` lines of
  // every peer (the gang placement slots, every word used); 0 = zero all n_flags words
  int flag_line, flag_lpp, flag_full;
  // where the epoch graph's last node publishes the fit's results (null loss: nowhere — an earlier
  // epoch of a multi-epoch fit, or stats published by a separate launch)
  struct PubDst {
    float* loss;
    int* correct;
    int* err;
    unsigned* seq;
    unsigned gen;
  } pub;
};
using PubDst = CtlUpload::PubDst;
__global__ void k_upload_ctl(CtlUpload u, int4* ctl, int* active, unsigned long long* seed, PubDst* pub) {
  const int p = threadIdx.x;
  if (pub != nullptr && p == 0) *pub = u.pub;
  if (p < u.P) {
    ctl[p] = u.ctl[p];
    if (u.with_active) active[p] = u.active[p];
    if (u.zero_loss) u.zero_loss[p] = 0.f;
    if (u.zero_correct) u.zero_correct[p] = 0;
  }
  if (u.zero_conf)
    for (int q = p; q < u.P * 256; q += blockDim.x) u.zero_conf[q] = 0;
  if (u.zero_err)
    for (int q = p; q < MLP_ERR_WORDS; q += blockDim.x) u.zero_err[q] = 0;
  if (u.zero_flags) {
    if (u.flag_line > 0) {
      // one store per flag line (was every word of every line: 8 peers x 304 lines x 32 words,
      // ~12 us of one workgroup between two epochs, profiles/r6w_bnd), whole lines for the slots
      const int lines = u.n_flags / u.flag_line;
#ifndef ENGINE_FLAGS_BROKEN_TEST  // (negative control of test_f32_flag_block_sparse_zeroing only)
      for (int q = p; q < lines; q += blockDim.x) u.zero_flags[(int64_t)q * u.flag_line] = 0u;
#endif
      const int per_peer = u.flag_full * u.flag_line / 4;  // 16-byte chunks of one peer's slot lines
      for (int q = p; q < (lines / u.flag_lpp) * per_peer; q += blockDim.x) {
        const int pp = q / per_peer, k = q - pp * per_peer;
        uint4* base = reinterpret_cast<uint4*>(u.zero_flags + ((int64_t)pp * u.flag_lpp + u.flag_lpp - u.flag_full) * u.flag_line);
        base[k] = uint4{0u, 0u, 0u, 0u};
      }
    } else {
      for (int q = p; q < u.n_flags; q += blockDim.x) u.zero_flags[q] = 0u;
    }
  }
  if (p == 0) *seed = u.seed;
}

// Evaluation snapshot for the overlapped evaluation, in one launch: fp32 copy + bf16 shadow + W2T of
// every peer's parameters (the epoch rewrites the live rows while the evaluation reads these), plus
// the evaluation's control words and zeroed accumulators (block 0).
__global__ __launch_bounds__(256) void k_eval_snapshot(MLPArgs a, float* params_out, bf16* shadow_out, bf16* w2t_out, CtlUpload u, int4* ctl,
                                                       int* active) {
  const int p = blockIdx.y;
  if (blockIdx.x == 0 && p == 0) {
    const int t = threadIdx.x;
    if (t < u.P) {
      ctl[t] = u.ctl[t];
      active[t] = u.active[t];
      u.zero_loss[t] = 0.f;
      u.zero_correct[t] = 0;
    }
    for (int q = t; q < u.P * 256; q += blockDim.x) u.zero_conf[q] = 0;
  }
  const int64_t pS = (int64_t)p * a.S;
  const int64_t n = a.numel;
  for (int64_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float f = a.params[pS + i];
    params_out[pS + i] = f;
    const bf16 v = (bf16)f;
    shadow_out[pS + i] = v;
    const int64_t j = i - a.off_w2;
    if (j >= 0 && j < (int64_t)a.D1 * a.D2) {
      const int o2 = (int)(j / a.D1), o1 = (int)(j % a.D1);
      w2t_out[(int64_t)p * a.D1 * a.D2 + (int64_t)o1 * a.D2 + o2] = v;
    }
  }
}

// Results -> pinned, host-mapped ring slot in ONE launch (instead of one copy per buffer). The slot's
// sequence word is stored last, with system-scope release: the host polls it (mlp_engine_fetch)
// instead of waiting on an event recorded behind this launch — an event record on the main stream
// costs the GPU a 6-14 us idle gap before the next kernel (profiles/r4i_*/timeline_prep0.txt).
__device__ __forceinline__ void publish_body(const float* loss, const int* correct, const int* err, const int* conf, int P, float* o_loss,
                                             int* o_correct, int* o_err, int* o_conf, unsigned* o_seq, unsigned seq) {
  const int t = threadIdx.x;
  if (t < P) {
    o_loss[t] = loss[t];
    o_correct[t] = correct[t];
  }
  // give-up status, bit 0: a give-up that was not recovered, bit 1: one recovered by the retry
  __shared__ int st;
  if (t == 0) st = 0;
  __syncthreads();
  if (err && t < MLP_ERR_WORDS) {
    const int v = err[t];
    if (v != 0) atomicOr(&st, (v == 2 && t < 64) ? 2 : 1);
  }
  __syncthreads();
  if (t == 0) *o_err = st;
  if (conf && o_conf)
    for (int q = t; q < P * 256; q += blockDim.x) o_conf[q] = conf[q];
  if (o_seq) {
    __threadfence_system();
    __syncthreads();
    if (t == 0) __hip_atomic_store(o_seq, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
__global__ void k_publish(const float* loss, const int* correct, const int* err, const int* conf, int P, float* o_loss, int* o_correct,
                          int* o_err, int* o_conf, unsigned* o_seq, unsigned seq) {
  publish_body(loss, correct, err, conf, P, o_loss, o_correct, o_err, o_conf, o_seq, seq);
}
// The epoch graph's last node: the fit's results to the ring slot the epoch's control upload named
// (the graph is fixed, the slot is not); a separate publish launch after the graph left the main
// stream idle ~10 us behind the graph (profiles/r4j_*/timeline.txt).
__global__ void k_publish_dev(const float* loss, const int* correct, const int* err, int P, const PubDst* pd) {
  const PubDst d = *pd;
  if (d.loss == nullptr) return;
  publish_body(loss, correct, err, nullptr, P, d.loss, d.correct, d.err, nullptr, d.seq, d.gen);
}

#define MLP_RING 16
struct ResultSlot {
  float* loss = nullptr;  // pinned host memory, mapped: the same pointers are written by k_publish
  int* correct = nullptr;
  int* conf = nullptr;
  int* err = nullptr;
  unsigned* seq = nullptr;  // k_publish stores `gen` here last
  std::atomic<unsigned> gen{0};
  hipStream_t stream = nullptr;  // where the publish was enqueued (fault check while polling)
  hipEvent_t ev = nullptr;       // MYFYP_RING_EVENTS=1: completion event instead of the sequence word
};
// MYFYP_GRAPH_PUBLISH=0: the fit's results by a separate launch after the epoch graph
static bool graph_publish() {
  static const int v = [] {
    const char* e = getenv("MYFYP_GRAPH_PUBLISH");
    return e != nullptr ? atoi(e) : 1;
  }();
  return v != 0;
}
// MYFYP_EVAL_GATHER_ORDER=0: the gather ahead always waits on an event recorded before the epoch (A/B)
static bool eval_gather_order() {
  static const int v = [] {
    const char* e = getenv("MYFYP_EVAL_GATHER_ORDER");
    return e != nullptr ? atoi(e) : 1;
  }();
  return v != 0;
}
static bool ring_events() {
  static const int v = [] {
    const char* e = getenv("MYFYP_RING_EVENTS");
    return e != nullptr ? atoi(e) : 0;
  }();
  return v != 0;
}

struct MLPEngine {
  MLPArgs a{};
  int max_steps = 0;
  hipGraph_t graph = nullptr;
  hipGraph_t graph_alt = nullptr;  // prep mode: the second executable's graph (other batch buffers)
  // Prep-stream gather (persistent path with the in-kernel shuffle): the epoch's batch gather runs on
  // its own stream into one of two batch buffers while the previous round's epoch still runs on the
  // main stream (the gangs leave CUs free), so it is off the round's critical path. Executable i
  // reads buffer i; the gather into buffer i waits only for the last epoch that read it.
  // Opt-in (MYFYP_PREP_GATHER=1): measured round-rate neutral on the fp32 headline (488.2 / 500.7
  // vs 498.0 / 501.7 rounds/s in-graph, profiles/r3_host_timeline) — the 28 us gather overlapped with
  // the epoch costs the epoch about as much as it saves. Bit-identical to the in-graph gather (test).
  // MYFYP_PREP_GATHER=2 (ahead, the default; 0 = the gather as the first node of the epoch graph):
  // the gather of epoch r waits for the START of epoch r-1 (an event
  // recorded on the main stream right before its graph launch; epoch r-2, the last reader of the
  // buffer, is then done) and runs on a capped grid (MYFYP_PREP_GATHER_WGS, default 64) beside it,
  // instead of at the round boundary (its earliest start in mode 1), where it slowed the FedAvg.
  // direct-X fp32 epochs (mlp_persistent_f32_x_direct): the graph's first node is the index / label
  // kernel (8 x 7.5k indices) instead of the image gather, and no prep stream is used
  bool x_direct = false;
  bool prep_mode = false;
  int prep_level = 0;
  int prep_wgs = 64;
  hipEvent_t ev_start = nullptr;
  bool start_rec = false;
  bf16* xb16_buf[2] = {nullptr, nullptr};
  int* yb_buf[2] = {nullptr, nullptr};
  hipStream_t prep_stream = nullptr;
  hipEvent_t ev_gath[2] = {nullptr, nullptr}, ev_done[2] = {nullptr, nullptr};
  bool done_rec[2] = {false, false};
  int4* d_ctl_prep = nullptr;
  int* d_active_prep = nullptr;
  unsigned long long* d_seed_prep = nullptr;
  // Two executables of the same epoch graph, launched alternately, so a launch never reuses the
  // launch state of an execution still on the GPU. Measured (profiles/r3_host_timeline): with one or
  // two, hipGraphLaunch holds the host 4-8 us and the round rate is the same within noise (485-491
  // rounds/s): the host already runs rounds ahead (it waits on the result ring, not on the GPU).
  // Kept for the launch-time counters below; MYFYP_GRAPH_EXECS=1 selects one.
  hipGraphExec_t execs[2] = {nullptr, nullptr};
  hipGraphExec_t exec = nullptr;  // execs[0]: non-null once captured
  int n_execs = 2;
  unsigned long long launches = 0, launch_ns = 0, launch_max_ns = 0;
  int graph_steps = -1;
  // gather ahead (prep mode): right after epoch r is launched, the gather of epoch r + 1 (seed given
  // beforehand with mlp_engine_set_next_epoch_seed) is enqueued on the prep stream into the other
  // batch buffer. In steady state the GPU does the same as before (the gather runs beside epoch r);
  // the difference is that it is already enqueued when the host reaches epoch r + 1 — after a host
  // synchronisation (the bench's clock start) or a late host, the gather is not exposed.
  bool next_seed_valid = false;
  unsigned long long next_seed = 0;
  bool ahead_valid[2] = {false, false};
  unsigned long long ahead_seed[2] = {0, 0};
  // The prep and evaluation streams are created on a helper thread started with the engine: each
  // is a new hardware queue (5.5 ms to create, profiles/r5_start), and the data binding and code
  // object loading of node start run meanwhile. take_stream joins it.
  std::thread stream_maker;
  bool making = false;
  hipStream_t made[2] = {nullptr, nullptr};
  void make_streams_async() {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return;
    making = true;
    stream_maker = std::thread([this, dev] {
      if (hipSetDevice(dev) != hipSuccess) return;
      for (auto& st : made)
        if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) st = nullptr;
    });
  }
  hipStream_t take_stream(int i) {
    if (making) {
      stream_maker.join();
      making = false;
    }
    hipStream_t st = made[i];
    made[i] = nullptr;
    if (st == nullptr && hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) st = nullptr;
    return st;
  }
  hipStream_t cap_stream = nullptr;  // capture stream when there is no prep stream to capture on
  hipStream_t cs = nullptr;          // the stream the current capture runs on
  // engine-owned device buffers
  void* ws = nullptr;
  int* d_active = nullptr;
  int* d_t0 = nullptr;
  int4* d_ctl = nullptr;
  unsigned long long* d_seed = nullptr;
  unsigned long long seed_host = 0;
  PubDst* d_pub = nullptr;      // the graph's publish destination (written by the control upload)
  int graph_pub_slot = -1;      // ring slot the last epoch graph published into (stats_async skips it)
  bool graph_has_pub = false;   // the captured graph ends with k_publish_dev
  std::vector<int4> ctl_host;
  float* d_loss = nullptr;
  int* d_correct = nullptr;
  int* d_conf = nullptr;
  std::vector<void*> owned;
  std::mutex mu;
  int max_test_rows = 0;
  ResultSlot ring[MLP_RING];  // pinned host result buffers + completion events
  // weight-stationary persistent epoch (mlp_persistent.hip): exchange buffers + mode
  MLPPersistBufs pb{};
  MLPPersistF32Bufs pb32{};
  int persist_mode = -1;  // -1 auto (eligible configs), 0 off
  // 1 = fp32 (the reference's precision: fp32 persistent epoch + fp32 evaluation; no bf16 fallback),
  // 0 = bf16 MFMA operands with fp32 master weights (persistent or 3-launch step path)
  int precision = 1;
  int num_cus = 0;
  // CUs left to a concurrently running RCCL kernel (side-stream all-reduce / delayed averaging)
  // when sizing the co-resident gangs: the persistent epoch needs every workgroup of a gang resident
  int reserved_cus = 0;
  bool graph_persistent = false;
  // deferred to the epoch's control upload on the persistent path (fewer tiny launches per round)
  bool pending_zero_acc = false;  // zero loss / correct / give-up word
  bool pending_fresh = false;     // fresh optimizer state: the kernel starts the moments at 0
  std::vector<int> active_host_cache;
  // evaluation overlapped with the epoch (persistent path): it reads a snapshot of the parameters
  // taken on the main stream and runs on its own stream on the CUs the epoch's gangs leave free
  // Two evaluation sides, used alternately: the snapshot for evaluation r overwrites the side that
  // evaluation r-2 read, and the host (not the main stream) waits for that one — a stream wait on
  // the previous evaluation cost the main stream a 6-7 us idle gap every round
  // (profiles/r4j_*/timeline.txt); evaluation r-2 ends about a round before the host gets here.
  hipStream_t eval_stream = nullptr;
  bool eval_stream_owned = false;  // false: it is the prep stream
  hipEvent_t ev_snap = nullptr;
  // The gather ahead is ordered after this round's overlapped evaluation (its done event is recorded
  // on the evaluation stream anyway) when one was enqueued on the epoch's stream with no epoch
  // launched since: no ordering event on the main stream, and the gather's workgroups start after
  // the evaluation's instead of competing with the epoch's dispatch (profiles/r5_evalorder)
  hipStream_t snap_rec_stream = nullptr;
  unsigned long long snap_rec_launches = ~0ull;
  hipEvent_t last_eval_done = nullptr;
  struct EvalSide {
    float* params = nullptr;
    bf16* shadow = nullptr;
    bf16* w2t = nullptr;
    int4* ctl = nullptr;
    int* active = nullptr;
    float* loss = nullptr;
    int* correct = nullptr;
    int* conf = nullptr;
    hipEvent_t done = nullptr;
    bool rec = false;
  } eside[2];
  int eval_idx = 0;
  int64_t snap_S = 0;

  bool use_persistent() const {
    if (precision == 1) return fp32_ready();
    if (persist_mode == 0 || pb.h1x == nullptr || a.Xb16 == nullptr) return false;
    if (a.P * 17 > num_cus) return false;  // every gang must be co-resident (one workgroup per CU)
    return mlp_persistent_supported(a);
  }
  // the fp32 path: every gang of a launch (8 peers x 24 workgroups) co-resident, one per CU
  // Co-residency: the occupancy calculator (registers, LDS, 512 threads) must place the whole launch
  // at once; epochs of every engine of the process run one after another (gang_order below), and
  // the concurrent evaluation kernels are finite, so a launch is never starved for good — and a gang
  // that still times out is re-run by the retry launch.
  mutable int f32_cap_bpad = -1, f32_cap = 0;
  bool fp32_ready() const {
    if (pb32.h1x == nullptr || a.Xb16 == nullptr) return false;
    if (!mlp_persistent_f32_supported(a)) return false;
    if (f32_cap_bpad != a.Bpad) {
      f32_cap = mlp_persistent_f32_resident_capacity(a, num_cus - reserved_cus > 0 ? num_cus - reserved_cus : 1);
      f32_cap_bpad = a.Bpad;
    }
    return mlp_persistent_f32_launch_wgs(a) <= f32_cap;
  }
  int recoveries = 0;
  // direct epoch launches: the active flags of this epoch (skip groups without an active peer);
  // null while capturing the epoch graph (it must serve any later active set)
  const int* launch_active = nullptr;
  int launch_active_buf[MLP_CTL_MAX];
  int launch_epoch_kernel(hipStream_t s, bool zero_flags) {
    const hipError_t le = precision == 1 ? mlp_launch_persistent_f32_epoch(a, pb32, s, zero_flags, launch_active) : mlp_launch_persistent_epoch(a, pb, s, zero_flags);
    if (le != hipSuccess) {
      g_last_error = std::string("persistent epoch launch: ") + hipGetErrorString(le);
      return 1;
    }
    return 0;
  }
  void set_flag_zeroing(MLPArgs& ga) const {
    if (precision == 1) {
      ga.flags_zero = pb32.flags;
      ga.flags_per_peer = mlp_persistent_f32_flags_per_peer();
    } else {
      ga.flags_zero = pb.flags;
      ga.flags_per_peer = (int)(pb.flag_bytes / sizeof(unsigned) / a.P);
    }
  }
  void launch_eval(const MLPArgs& ea, hipStream_t s) const {
    if (precision == 1)
      mlp_launch_eval_f32(ea, max_test_rows, s);
    else
      for (int base = 0; base < max_test_rows; base += MLP_EVAL_CHUNK) mlp_launch_eval_chunk(ea, base, s);
  }

  ~MLPEngine() {
    if (making) stream_maker.join();
    for (auto& st : made)
      if (st) hipStreamDestroy(st);
    if (prep_stream) {
      hipStreamSynchronize(prep_stream);
      hipStreamDestroy(prep_stream);
    }
    for (int i = 0; i < 2; ++i) {
      if (ev_gath[i]) hipEventDestroy(ev_gath[i]);
      if (ev_done[i]) hipEventDestroy(ev_done[i]);
    }
    if (xb16_buf[1]) hipFree(xb16_buf[1]);
    if (yb_buf[1]) hipFree(yb_buf[1]);
    if (eval_stream && eval_stream_owned) {
      hipStreamSynchronize(eval_stream);
      hipStreamDestroy(eval_stream);
    }
    if (ev_snap) hipEventDestroy(ev_snap);
    for (auto& es : eside) {
      if (es.done) hipEventDestroy(es.done);
      if (es.params) hipFree(es.params);
      if (es.shadow) hipFree(es.shadow);
      if (es.w2t) hipFree(es.w2t);
    }
    for (auto& x : execs)
      if (x) hipGraphExecDestroy(x);
    if (graph) hipGraphDestroy(graph);
    if (graph_alt) hipGraphDestroy(graph_alt);
    if (cap_stream) hipStreamDestroy(cap_stream);
    for (void* p : owned) hipFree(p);
    if (a.Xb) hipFree(a.Xb);
    if (a.Xb16) hipFree(a.Xb16);
    if (a.Yb) hipFree(a.Yb);
    if (a.xidx) hipFree(a.xidx);
    for (auto& r : ring) {
      if (r.ev) hipEventDestroy(r.ev);
      if (r.loss) hipHostFree(r.loss);
      if (r.correct) hipHostFree(r.correct);
      if (r.conf) hipHostFree(r.conf);
      if (r.err) hipHostFree(r.err);
      if (r.seq) hipHostFree(r.seq);
    }
  }

  int alloc_ring() {
    for (auto& r : ring) {
      const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;  // written by k_publish
      CHECK_HIP(hipHostMalloc((void**)&r.loss, sizeof(float) * a.P, fl));
      CHECK_HIP(hipHostMalloc((void**)&r.correct, sizeof(int) * a.P, fl));
      CHECK_HIP(hipHostMalloc((void**)&r.conf, sizeof(int) * a.P * 256, fl));
      CHECK_HIP(hipHostMalloc((void**)&r.err, sizeof(int), fl));
      *r.err = 0;
      CHECK_HIP(hipHostMalloc((void**)&r.seq, sizeof(unsigned), fl));
      *r.seq = 0;
      r.gen = 0;
      CHECK_HIP(hipEventCreateWithFlags(&r.ev, hipEventDisableTiming));
    }
    return 0;
  }

  void flag_words(unsigned** ptr, int* n) const {
    if (precision == 1) {
      *ptr = pb32.flags;
      *n = a.P * mlp_persistent_f32_flags_per_peer();
    } else {
      *ptr = pb.flags;
      *n = (int)(pb.flag_bytes / sizeof(unsigned));
    }
  }
  bool debug_poison_flags = false;  // test hook: every word of the flag block set to ~0 before its zeroing
  int poisoned = 0;                 // uploads that poisoned the block (the hook reports it)
  int upload(hipStream_t s, const int* active_host, bool zero_fit = false, bool fresh = false, bool zero_flags = false, const PubDst* pub = nullptr) {
    CtlUpload u{};
    if (pub) u.pub = *pub;  // else null: the graph's publish node does nothing
    if (zero_flags) {
      flag_words(&u.zero_flags, &u.n_flags);
#ifndef ENGINE_FLAGS_DENSE  // (A/B build: -DENGINE_FLAGS_DENSE zeroes every word, as before)
      if (precision == 1) mlp_persistent_f32_flag_layout(&u.flag_line, &u.flag_lpp, &u.flag_full);
#endif
      // (the words the sparse zeroing skips must never be read: a stale ~0 there would release a
      // consumer before its hand-off is written; tests/test_mlp_f32_gpu.py poisons them)
      if (debug_poison_flags) {
        CHECK_HIP(hipMemsetAsync(u.zero_flags, 0xFF, (size_t)u.n_flags * sizeof(unsigned), s));
        ++poisoned;
      }
    }
    u.P = a.P;
    u.with_active = active_host != nullptr;
    u.seed = seed_host;
    for (int p = 0; p < a.P; ++p) {
      u.ctl[p] = ctl_host[p];
      if (fresh && u.ctl[p].x) u.ctl[p].x |= 2;
      u.active[p] = active_host ? active_host[p] : 0;
    }
    if (zero_fit) {
      u.zero_loss = d_loss;
      u.zero_correct = d_correct;
      u.zero_err = pb.err;
    }
    hipLaunchKernelGGL(k_upload_ctl, dim3(1), dim3(256), 0, s, u, d_ctl, d_active, d_seed, d_pub);
    CHECK_HIP(hipGetLastError());
    return 0;
  }
  // Prep mode: the gather into batch buffer i on the prep stream, after the last epoch that read it;
  // it gets its own copy of the control words and the shuffle key (nothing on the main stream).
  // ahead: the gather of the NEXT epoch (seed ``seed``), for every peer with data (the next round's
  // active set is not known yet), ordered after the start of the epoch just launched (which reads
  // the other buffer; the one that last read buffer i has then finished)
  int prep_gather(int i, hipStream_t main, unsigned long long seed, bool ahead = false, bool after_eval = false) {
    if (after_eval) {  // this round's overlapped evaluation: it follows epoch r - 1, the last reader of buffer i
      CHECK_HIP(hipStreamWaitEvent(prep_stream, last_eval_done, 0));
    } else if (prep_level == 2 && start_rec) {
      CHECK_HIP(hipStreamWaitEvent(prep_stream, ev_start, 0));
    } else if (done_rec[i]) {
      CHECK_HIP(hipStreamWaitEvent(prep_stream, ev_done[i], 0));
    } else {  // first gather after a (re)capture: behind everything already on the main stream
      CHECK_HIP(hipEventRecord(ev_start, main));
      CHECK_HIP(hipStreamWaitEvent(prep_stream, ev_start, 0));
    }
    CtlUpload u{};
    u.P = a.P;
    u.seed = seed;
    for (int p = 0; p < a.P; ++p) {
      u.ctl[p] = ctl_host[p];
      if (ahead) u.ctl[p].x = ctl_host[p].y > 0 ? 1 : 0;
    }
    hipLaunchKernelGGL(k_upload_ctl, dim3(1), dim3(256), 0, prep_stream, u, d_ctl_prep, d_active_prep, d_seed_prep, (PubDst*)nullptr);
    MLPArgs ga = a;
    ga.ctl = d_ctl_prep;
    ga.seed = d_seed_prep;
    ga.Xb16 = xb16_buf[i];
    ga.Yb = yb_buf[i];
    ga.flags_zero = nullptr;
    // debug (MYFYP_DEBUG_NO_GATHER=1, timing experiments only): once both batch buffers hold a real
    // epoch, later epochs re-read them and no gather runs beside the epoch (prices its interference)
    static const bool no_gather = [] {
      const char* e = getenv("MYFYP_DEBUG_NO_GATHER");
      return e != nullptr && atoi(e) != 0;
    }();
    if (!(no_gather && ++prep_gathers > 2)) mlp_launch_gather_epoch(ga, prep_stream, prep_level == 2 ? prep_wgs : 0);
    CHECK_HIP(hipGetLastError());
    CHECK_HIP(hipEventRecord(ev_gath[i], prep_stream));
    return 0;
  }
  long long prep_gathers = 0;

  // publish into ring slot r; completion: the slot's sequence word (or its event, MYFYP_RING_EVENTS=1)
  int publish(hipStream_t s, ResultSlot& r, const float* loss, const int* correct, const int* err, const int* conf) {
    const unsigned g = r.gen.load() + 1;
    r.stream = s;
    hipLaunchKernelGGL(k_publish, dim3(1), dim3(256), 0, s, loss, correct, err, conf, a.P, r.loss, r.correct, r.err, conf ? r.conf : nullptr,
                       ring_events() ? nullptr : r.seq, g);
    CHECK_HIP(hipGetLastError());
    if (ring_events()) CHECK_HIP(hipEventRecord(r.ev, s));
    r.gen.store(g);
    return 0;
  }

  // evaluation resources for the overlapped path (allocated on first use)
  int ensure_eval_side() {
    if (!eval_stream) {
      // a stream of its own: sharing the prep stream saved 5.5 ms of node start (one hardware
      // queue fewer) but cost 15 % of the round rate (452-456 vs 527-539 rounds/s,
      // profiles/r5_start): the evaluation's wait for the snapshot held the next-epoch gather
      eval_stream = take_stream(1);
      if (eval_stream == nullptr) {
        g_last_error = "evaluation stream creation failed";
        return 1;
      }
      eval_stream_owned = true;
      CHECK_HIP(hipEventCreateWithFlags(&ev_snap, hipEventDisableTiming));
      for (auto& es : eside) {
        CHECK_HIP(hipEventCreateWithFlags(&es.done, hipEventDisableTiming));
        void* p;
        if (alloc(&p, (size_t)a.P * 16)) return 1;
        es.ctl = (int4*)p;
        if (alloc(&p, (size_t)a.P * 4)) return 1;
        es.active = (int*)p;
        if (alloc(&p, (size_t)a.P * 4)) return 1;
        es.loss = (float*)p;
        if (alloc(&p, (size_t)a.P * 4)) return 1;
        es.correct = (int*)p;
        if (alloc(&p, (size_t)a.P * 256 * 4)) return 1;
        es.conf = (int*)p;
      }
    }
    if (snap_S != a.S) {
      for (auto& es : eside) {
        if (es.params) hipFree(es.params);
        if (es.shadow) hipFree(es.shadow);
        if (es.w2t) hipFree(es.w2t);
        CHECK_HIP(hipMalloc((void**)&es.params, (size_t)a.P * a.S * sizeof(float)));
        CHECK_HIP(hipMalloc((void**)&es.shadow, (size_t)a.P * a.S * sizeof(bf16)));
        CHECK_HIP(hipMalloc((void**)&es.w2t, (size_t)a.P * a.D1 * a.D2 * sizeof(bf16)));
      }
      snap_S = a.S;
    }
    return 0;
  }
  // the main stream must not run ahead of an overlapped evaluation that reads what it is about to
  // change (a non-persistent evaluation on the main stream, a re-snapshot of the same side)
  int wait_evals(hipStream_t s) {
    for (auto& es : eside)
      if (es.rec) CHECK_HIP(hipStreamWaitEvent(s, es.done, 0));
    return 0;
  }

  void invalidate() {
    ahead_valid[0] = ahead_valid[1] = false;
    for (auto& x : execs) {
      if (x) hipGraphExecDestroy(x);
      x = nullptr;
    }
    if (graph) hipGraphDestroy(graph);
    if (graph_alt) hipGraphDestroy(graph_alt);
    graph_alt = nullptr;
    exec = nullptr;
    graph = nullptr;
    graph_steps = -1;
  }

  // Zeroed device buffer owned by the engine. Small ones (control words, accumulators, flags) are
  // carved out of 2 MiB arena chunks that are allocated and zeroed once: an engine makes ~30 of
  // them, and a hipMalloc + synchronous hipMemset each cost node start several ms
  // (profiles/r5_start). 256-byte alignment (every consumer wants at most 16).
  static constexpr size_t kArenaChunk = 2u << 20, kArenaMax = 256u << 10, kArenaAlign = 256;
  char* arena = nullptr;
  size_t arena_used = kArenaChunk;
  int alloc(void** p, size_t bytes) {
    bytes = bytes < 16 ? 16 : bytes;
    if (bytes <= kArenaMax) {
      const size_t need = (bytes + kArenaAlign - 1) / kArenaAlign * kArenaAlign;
      if (arena_used + need > kArenaChunk) {
        void* c = nullptr;
        CHECK_HIP(hipMalloc(&c, kArenaChunk));
        CHECK_HIP(hipMemset(c, 0, kArenaChunk));
        owned.push_back(c);
        arena = (char*)c;
        arena_used = 0;
      }
      *p = arena + arena_used;
      arena_used += need;
      return 0;
    }
    CHECK_HIP(hipMalloc(p, bytes));
    CHECK_HIP(hipMemset(*p, 0, bytes));
    owned.push_back(*p);
    return 0;
  }

  int launch_graph(hipStream_t s) {
    hipGraphExec_t x = execs[n_execs > 1 ? (int)(launches & 1) : 0];
    const auto t0 = std::chrono::steady_clock::now();
    CHECK_HIP(hipGraphLaunch(x, s));
    const unsigned long long ns = (unsigned long long)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    ++launches;
    launch_ns += ns;
    if (ns > launch_max_ns) launch_max_ns = ns;
    return 0;
  }

  // One epoch: [gather (unless prep mode), epoch kernel + retry launch] or the step chain, then the
  // fit's publish; buf selects the batch buffers the epoch reads in prep mode. Captured into the
  // epoch graph, or enqueued directly (direct_epoch_launch()).
  int enqueue_epoch(hipStream_t st, int steps, int buf) {
    const MLPArgs saved = a;
    if (prep_mode) {
      a.Xb16 = xb16_buf[buf];
      a.Yb = yb_buf[buf];
    }
    if (x_direct) {
      MLPArgs ga = a;
      set_flag_zeroing(ga);  // the index kernel zeroes the hand-off flags (no memset node)
      mlp_launch_index_epoch(ga, st);
    } else if (!prep_mode) {
      MLPArgs ga = a;  // the bf16 batch copy is only produced for the persistent kernel
      if (!graph_persistent) ga.Xb16 = nullptr;
      if (graph_persistent) set_flag_zeroing(ga);  // ... which also zeroes the hand-off flags (no memset node)
      mlp_launch_gather_epoch(ga, st);
    }
    int rc = 0;
    if (graph_persistent) {
      rc = launch_epoch_kernel(st, false);
    } else {
      for (int s = 0; s < steps; ++s) mlp_launch_train_step(a, s, st);
    }
    if (graph_has_pub) hipLaunchKernelGGL(k_publish_dev, dim3(1), dim3(256), 0, st, d_loss, d_correct, pb.err, a.P, (const PubDst*)d_pub);
    a = saved;
    return rc;
  }

  // The persistent epoch's launches (epoch, retry, publish) are enqueued directly instead of as a
  // graph launch (MYFYP_EPOCH_GRAPH=1: the graph). A graph launch costs the device ~6.5 us before its
  // first kernel and ~2.7 us after its last, a plain kernel boundary ~1.3 us
  // (scripts/probes/gap_probe.hip, profiles/r5_gap): +0.4 % rounds/s, 4 of 4 alternations
  // (602.8 vs 600.6 mean, profiles/r5_direct); the host, rounds ahead, absorbs the two extra launch
  // calls. The graphs are still captured (the step-chain path and MYFYP_EPOCH_GRAPH=1 use them).
  bool direct_epoch_launch() const {
    static const int v = [] {
      const char* e = getenv("MYFYP_EPOCH_GRAPH");
      return e != nullptr ? atoi(e) : 0;
    }();
    return v == 0 && graph_persistent;
  }
  int launch_epoch(hipStream_t s) {
    if (!direct_epoch_launch()) return launch_graph(s);
    const int buf = n_execs > 1 ? (int)(launches & 1) : 0;
    const auto t0 = std::chrono::steady_clock::now();
    for (int p = 0; p < a.P && p < MLP_CTL_MAX; ++p) launch_active_buf[p] = ctl_host[p].x & 1;
    launch_active = launch_active_buf;
    const int rc_e = enqueue_epoch(s, graph_steps, buf);
    launch_active = nullptr;
    if (rc_e) return 1;
    CHECK_HIP(hipGetLastError());
    const unsigned long long ns = (unsigned long long)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    ++launches;
    launch_ns += ns;
    if (ns > launch_max_ns) launch_max_ns = ns;
    return 0;
  }

  int capture_one(int steps, int buf, hipGraph_t* out) {
    graph_has_pub = graph_publish() && !ring_events() && d_pub != nullptr;
    CHECK_HIP(hipStreamBeginCapture(cs, hipStreamCaptureModeRelaxed));
    const int rc = enqueue_epoch(cs, steps, buf);
    hipGraph_t g = nullptr;
    const hipError_t e = hipStreamEndCapture(cs, &g);
    if (rc || e != hipSuccess) {
      if (g) hipGraphDestroy(g);
      if (!rc) g_last_error = std::string("hipStreamEndCapture: ") + hipGetErrorString(e);
      return 1;
    }
    *out = g;
    return 0;
  }

  int ensure_prep() {
    if (!prep_stream) {
      prep_stream = take_stream(0);
      if (prep_stream == nullptr) {
        g_last_error = "prep stream creation failed";
        return 1;
      }
      CHECK_HIP(hipEventCreateWithFlags(&ev_start, hipEventDisableTiming));
      for (int i = 0; i < 2; ++i) {
        CHECK_HIP(hipEventCreateWithFlags(&ev_gath[i], hipEventDisableTiming));
        CHECK_HIP(hipEventCreateWithFlags(&ev_done[i], hipEventDisableTiming));
      }
      void* p;
      if (alloc(&p, (size_t)a.P * 16)) return 1;
      d_ctl_prep = (int4*)p;
      if (alloc(&p, (size_t)a.P * 4)) return 1;
      d_active_prep = (int*)p;
      if (alloc(&p, 8)) return 1;
      d_seed_prep = (unsigned long long*)p;
    }
    return 0;
  }

  int capture(int steps) {
    const auto q0 = std::chrono::steady_clock::now();
    invalidate();
    const auto q1 = std::chrono::steady_clock::now();
    graph_persistent = use_persistent();
    const auto q2 = std::chrono::steady_clock::now();
    x_direct = graph_persistent && precision == 1 && mlp_persistent_f32_x_direct(a);
    if (x_direct && (a.Xp16 == nullptr || a.xidx == nullptr)) {
      g_last_error = "fp32 direct-X epoch: no bf16 image table bound (mlp_engine_set_train_x16)";
      return 1;
    }
    a.x_direct = x_direct ? 1 : 0;
    {
      const char* env = getenv("MYFYP_PREP_GATHER");
      prep_level = env != nullptr ? atoi(env) : 2;  // default: ahead (+0.5-1 %, profiles/r4h_*, r4j_*)
      prep_mode = !x_direct && graph_persistent && a.shuffle_native && xb16_buf[1] != nullptr && (prep_level == 1 || prep_level == 2);
      if (const char* w = getenv("MYFYP_PREP_GATHER_WGS")) prep_wgs = atoi(w);
      if (prep_mode && ensure_prep()) return 1;
      if (prep_mode) {
        // the batch buffers were (re)allocated or the graph changed: nothing in flight reads them
        done_rec[0] = done_rec[1] = false;
        start_rec = false;
        xb16_buf[0] = a.Xb16;
        yb_buf[0] = a.Yb;
      }
      const char* e2 = getenv("MYFYP_GRAPH_EXECS");
      n_execs = (!prep_mode && e2 != nullptr && atoi(e2) == 1) ? 1 : 2;
    }
    // capture on the prep stream when there is one (the engine's launches are serialised by its
    // mutex, so nothing else enqueues there meanwhile): each stream beyond the first few costs a
    // hardware queue, 5.5 ms to create (profiles/r5_start)
    if (prep_mode) {
      CHECK_HIP(hipStreamSynchronize(prep_stream));  // a re-capture: the previous graph's gather is done
      cs = prep_stream;
    } else {
      if (!cap_stream) CHECK_HIP(hipStreamCreateWithFlags(&cap_stream, hipStreamNonBlocking));
      cs = cap_stream;
    }
    const auto c0 = std::chrono::steady_clock::now();
    if (const char* tv = getenv("MYFYP_TIME_PREPARE"); tv != nullptr && atoi(tv) != 0) {
      auto d = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
        return (long long)std::chrono::duration_cast<std::chrono::microseconds>(b - a).count();
      };
      fprintf(stderr, "[prepare] invalidate+stream %lld us, use_persistent %lld us, prep setup %lld us\n", d(q0, q1), d(q1, q2), d(q2, c0));
    }
    if (capture_one(steps, 0, &graph)) return 1;
    if (prep_mode && capture_one(steps, 1, &graph_alt)) return 1;
    const auto c1 = std::chrono::steady_clock::now();
    for (int i = 0; i < n_execs; ++i) CHECK_HIP(hipGraphInstantiate(&execs[i], (prep_mode && i == 1) ? graph_alt : graph, nullptr, nullptr, 0));
    if (const char* tv = getenv("MYFYP_TIME_PREPARE"); tv != nullptr && atoi(tv) != 0)
      fprintf(stderr, "[prepare] capture_one x%d %lld us, instantiate x%d %lld us\n", prep_mode ? 2 : 1,
              (long long)std::chrono::duration_cast<std::chrono::microseconds>(c1 - c0).count(), n_execs,
              (long long)std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - c1).count());
    exec = execs[0];
    graph_steps = steps;
    return 0;
  }
};

// Persistent epochs of all engines in this process run in launch order (stream-ordered through
// one event; the host never waits): two gangs' launches never compete for the same CUs. One
// process per GPU is the deployment; ranks sharing a GPU are rehearsals.
// The event is recorded lazily, only when an epoch is launched on a stream other than the last one
// (recorded then on that stream: a superset of its last epoch, so still a safe order); an engine
// that stays on one stream never records it — an event record behind every epoch cost a 14 us idle
// gap before the next kernel (profiles/r4i_*/timeline_prep0.txt). MYFYP_GANG_EVENT=1: the old
// record-after-every-epoch.
struct GangOrder {
  std::mutex mu;
  hipEvent_t ev = nullptr;
  bool ev_ready = false;
  bool has_last = false;
  hipStream_t last = nullptr;
};
static bool gang_event_always() {
  static const int v = [] {
    const char* e = getenv("MYFYP_GANG_EVENT");
    return e != nullptr ? atoi(e) : 0;
  }();
  return v != 0;
}
// One order per DEVICE: persistent epochs only compete for the CUs of their own GPU. A device mesh
// (one process driving several GPUs, csrc/runtime/rccl_mesh.hip) must not chain device d's epoch
// behind device d-1's (that would serialise the GPUs), and an event may only be recorded on a stream
// of the device it was created on.
#define GANG_ORDER_MAX_DEVICES 64
GangOrder& gang_order(hipStream_t s) {
  static GangOrder g[GANG_ORDER_MAX_DEVICES];
  int dev = 0;
  if (hipStreamGetDevice(s, &dev) != hipSuccess || dev < 0 || dev >= GANG_ORDER_MAX_DEVICES) dev = 0;
  return g[dev];
}

}  // namespace

extern "C" {

int myfyp_version() { return 1; }
const char* myfyp_last_error() { return g_last_error.c_str(); }

// ------------------------------------------------------------------------------ generic FL ops
int myfyp_weighted_sum(float* out, const uint64_t* srcs, const float* w, int K, int64_t n, void* stream) {
  fl_weighted_sum(out, srcs, w, K, n, (hipStream_t)stream);
  CHECK_HIP(hipGetLastError());
  return 0;
}
int myfyp_stacked_weighted_sum(float* out, const float* stacked, int P, int64_t n, int64_t ld, const float* w, float scale, void* stream) {
  fl_stacked_weighted_sum(out, stacked, P, n, ld, w, scale, (hipStream_t)stream);
  CHECK_HIP(hipGetLastError());
  return 0;
}
int myfyp_broadcast_rows(float* stacked, const float* src, int P, int64_t n, int64_t ld, const float* mask, void* stream) {
  fl_broadcast_rows(stacked, src, P, n, ld, mask, (hipStream_t)stream);
  CHECK_HIP(hipGetLastError());
  return 0;
}
// FedAvg of a stacked [P][ld] group: weights / mask by value (P <= 64); out has n + 1 floats.
static bool fedavg_rows_ok(int P) {
  if (P >= 1 && P <= FEDAVG_MAX_PEERS) return true;
  g_last_error = "fedavg_stacked: 1..64 rows";
  return false;
}
static unsigned long long mask_bits(const float* mask_host, int P) {
  unsigned long long mask = 0;
  for (int p = 0; p < P; ++p)
    if (mask_host[p] != 0.f) mask |= 1ull << p;
  return mask;
}
// wsum_slot: where the weight sum goes (nullptr: not written, e.g. buckets after the first)
int myfyp_fedavg_bucket_reduce(float* out, float* wsum_slot, const float* stacked, int P, int64_t n, int64_t ld, const float* w_host, void* stream) {
  if (!fedavg_rows_ok(P)) return 2;
  FedAvgWeights w{};
  double sum = 0.0;
  for (int p = 0; p < P; ++p) {
    w.w[p] = w_host[p];
    sum += w_host[p];
  }
  w.wsum = (float)sum;
  fl_fedavg_reduce(out, wsum_slot, stacked, P, n, ld, w, (hipStream_t)stream);
  CHECK_HIP(hipGetLastError());
  return 0;
}
// the same, with a second copy of the partial sums (the failover's retained input) from the same pass
int myfyp_fedavg_bucket_reduce2(float* out, float* wsum_slot, float* out2, float* wsum2, const float* stacked, int P, int64_t n, int64_t ld,
                                const float* w_host, void* stream) {
  if (!fedavg_rows_ok(P)) return 2;
  FedAvgWeights w{};
  double sum = 0.0;
  for (int p = 0; p < P; ++p) {
    w.w[p] = w_host[p];
    sum += w_host[p];
  }
  w.wsum = (float)sum;
  fl_fedavg_reduce(out, wsum_slot, stacked, P, n, ld, w, (hipStream_t)stream, out2, wsum2);
  CHECK_HIP(hipGetLastError());
  return 0;
}
int myfyp_fedavg_bucket_apply(float* stacked, const float* out, const float* wsum_slot, int P, int64_t n, int64_t ld, const float* mask_host, void* stream) {
  if (!fedavg_rows_ok(P)) return 2;
  fl_fedavg_apply(stacked, out, wsum_slot, P, n, ld, mask_bits(mask_host, P), (hipStream_t)stream);
  CHECK_HIP(hipGetLastError());
  return 0;
}
// Unbucketed layout: out[0:n] | out[n] = weight sum.
int myfyp_fedavg_stacked_reduce(float* out, const float* stacked, int P, int64_t n, int64_t ld, const float* w_host, void* stream) {
  return myfyp_fedavg_bucket_reduce(out, out + n, stacked, P, n, ld, w_host, stream);
}
int myfyp_fedavg_stacked_apply(float* stacked, const float* out, int P, int64_t n, int64_t ld, const float* mask_host, void* stream) {
  return myfyp_fedavg_bucket_apply(stacked, out, out + n, P, n, ld, mask_host, stream);
}
// Delayed averaging: rows in mask <- row + avg / *wsum_slot - snap, snap <- row (avg null: snapshot only)
int myfyp_fedavg_delayed_land(float* stacked, float* snap, int64_t ld_snap, const float* avg, const float* wsum_slot, int P, int64_t n, int64_t ld,
                              const float* mask_host, void* stream) {
  if (!fedavg_rows_ok(P)) return 2;
  fl_fedavg_delayed_land(stacked, snap, ld_snap, avg, wsum_slot, P, n, ld, mask_bits(mask_host, P), (hipStream_t)stream);
  CHECK_HIP(hipGetLastError());
  return 0;
}
// Single-rank FedAvg of a stacked group in one launch (weights and mask by value).
int myfyp_fedavg_stacked_local(float* stacked, int P, int64_t n, int64_t ld, const float* w_host, const float* mask_host, void* stream) {
  if (P < 1 || P > FEDAVG_MAX_PEERS) {
    g_last_error = "fedavg_stacked: 1..64 rows";
    return 2;
  }
  FedAvgWeights w{};
  double sum = 0.0;
  unsigned long long mask = 0;
  for (int p = 0; p < P; ++p) {
    w.w[p] = w_host[p];
    sum += w_host[p];
    if (mask_host[p] != 0.f) mask |= 1ull << p;
  }
  w.wsum = (float)sum;
  fl_fedavg_local(stacked, P, n, ld, w, mask, (hipStream_t)stream);
  CHECK_HIP(hipGetLastError());
  return 0;
}
// Topology mixing of a stacked group in one launch. w_host is the dense [P][P] mixing matrix
// (row p: the weights of the sources of row p, already renormalised); rows of an all-zero matrix
// row are left untouched. ld must be a multiple of 4 (stacked rows are padded to 64 floats).
int myfyp_neighbor_mix_stacked(float* stacked, int P, int64_t n, int64_t ld, const float* w_host, void* stream) {
  if (P < 1 || P > MIX_MAX_PEERS || (ld % 4) != 0 || ld < ((n + 3) / 4) * 4) {
    g_last_error = "neighbor_mix_stacked: 1..16 rows, ld a multiple of 4 covering n";
    return 2;
  }
  MixPlan m{};
  for (int p = 0; p < P; ++p) {
    int k = 0;
    for (int q = 0; q < P; ++q) {
      const float wq = w_host[p * P + q];
      if (wq == 0.f) continue;
      if (k == MIX_MAX_SRC) {
        g_last_error = "neighbor_mix_stacked: more sources in a row than MIX_MAX_SRC";
        return 2;
      }
      m.w[p][k] = wq;
      m.idx[p][k] = (unsigned char)q;
      ++k;
    }
    m.nsrc[p] = (unsigned char)k;
  }
  fl_neighbor_mix(stacked, P, n, ld, m, (hipStream_t)stream);
  CHECK_HIP(hipGetLastError());
  return 0;
}
// Row-pointer arguments below are HOST arrays of device pointers; they travel as kernel arguments.
static bool rows_ok(int k, const char* what) {
  if (k >= 1 && k <= 16) return true;
  g_last_error = std::string(what) + " supports 1..16 rows";
  return false;
}
int myfyp_coordinate_median_multi(const uint64_t* outs, int P, const uint64_t* srcs, int K, int64_t n, void* stream) {
  if (!rows_ok(K, "coordinate_median") || !rows_ok(P, "coordinate_median outputs")) return 2;
  RowPtrs rows{};
  OutPtrs o{};
  for (int k = 0; k < K; ++k) rows.p[k] = reinterpret_cast<const float*>(srcs[k]);
  for (int p = 0; p < P; ++p) o.p[p] = reinterpret_cast<float*>(outs[p]);
  fl_coordinate_median(o, P, rows, K, n, (hipStream_t)stream);
  CHECK_HIP(hipGetLastError());
  return 0;
}
int myfyp_coordinate_median(float* out, const uint64_t* srcs, int K, int64_t n, void* stream) {
  return myfyp_coordinate_median_multi((const uint64_t*)&out, 1, srcs, K, n, stream);
}
int myfyp_scaffold_reduce(float* buf, const uint64_t* dy, const uint64_t* dc, const float* w, int K, int64_t n, void* stream) {
  if (K < 0 || K > 16) {
    g_last_error = "scaffold_reduce supports 0..16 rows";
    return 2;
  }
  RowPtrs y{}, c{};
  RowW ww{};
  for (int k = 0; k < K; ++k) {
    y.p[k] = reinterpret_cast<const float*>(dy[k]);
    c.p[k] = reinterpret_cast<const float*>(dc[k]);
    ww.w[k] = w[k];
  }
  fl_scaffold_reduce(buf, y, c, ww, K, n, (hipStream_t)stream);
  CHECK_HIP(hipGetLastError());
  return 0;
}
int myfyp_scaffold_apply(const uint64_t* outs, int P, const float* x_start, const float* buf, float* c, int c_init, float glr, int64_t n, void* stream) {
  if (!rows_ok(P, "scaffold_apply outputs")) return 2;
  OutPtrs o{};
  for (int p = 0; p < P; ++p) o.p[p] = reinterpret_cast<float*>(outs[p]);
  fl_scaffold_apply(o, P, x_start, buf, c, c_init, glr, n, (hipStream_t)stream);
  CHECK_HIP(hipGetLastError());
  return 0;
}
int myfyp_adam_step(float* param, const float* grad, float* m, float* v, bf16* shadow, int64_t n, float lr, float b1, float b2, float eps, float wd,
                    int step, const float* anchor, const float* cg, const float* cl, float mu, void* stream) {
  OptParams o{0, lr, b1, b2, eps, wd, 0.f, 0, mu};
  fl_opt_step(param, grad, m, v, shadow, n, o, step < 1 ? 1 : step, anchor, cg, cl, (hipStream_t)stream);
  CHECK_HIP(hipGetLastError());
  return 0;
}
int myfyp_sgd_step(float* param, const float* grad, float* mom, int64_t n, float lr, float momentum, float wd, int nesterov, const float* anchor,
                   const float* cg, const float* cl, float mu, void* stream) {
  OptParams o{1, lr, 0.9f, 0.999f, 1e-8f, wd, momentum, nesterov, mu};
  fl_opt_step(param, grad, momentum != 0.f ? mom : nullptr, nullptr, nullptr, n, o, 1, anchor, cg, cl, (hipStream_t)stream);
  CHECK_HIP(hipGetLastError());
  return 0;
}
int myfyp_scale_add_noise(float* t, int64_t n, float scale, float sigma, uint64_t seed, void* stream) {
  fl_scale_add_noise(t, n, scale, sigma, seed, (hipStream_t)stream);
  CHECK_HIP(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------------------ MLP engine
int mlp_shape_ok(int D0, int D1, int D2, int D3) { return mlp_shape_supported(D0, D1, D2, D3) ? 1 : 0; }

void* mlp_engine_create(int P, int D0, int D1, int D2, int D3, int B) {
  if (!mlp_shape_supported(D0, D1, D2, D3) || P < 1 || P > MLP_CTL_MAX || B < 1 || (B + 31) / 32 * 32 > MLP_MAX_BPAD) {
    g_last_error = "unsupported MLP shape";
    return nullptr;
  }
  auto* e = new MLPEngine();
  e->make_streams_async();
  MLPArgs& a = e->a;
  a.P = P;
  a.D0 = D0; a.D1 = D1; a.D2 = D2; a.D3 = D3;
  a.D0pad = (D0 + 15) / 16 * 16;
  a.B = B;
  a.Bpad = (B + 31) / 32 * 32;
  a.h1_rows = a.Bpad > MLP_EVAL_CHUNK ? a.Bpad : MLP_EVAL_CHUNK;
  a.off_w1 = 0;
  a.off_b1 = (int64_t)D1 * D0;
  a.off_w2 = a.off_b1 + D1;
  a.off_b2 = a.off_w2 + (int64_t)D2 * D1;
  a.off_w3 = a.off_b2 + D2;
  a.off_b3 = a.off_w3 + (int64_t)D3 * D2;
  a.numel = a.off_b3 + D3;
  const size_t bp = (size_t)a.Bpad;
  void* p;
  int rc = 0;
  rc |= e->alloc(&p, (size_t)P * a.h1_rows * D1 * 2); a.H1 = (bf16*)p;
  rc |= e->alloc(&p, (size_t)P * D1 * bp * 2); a.H1T = (bf16*)p;
  a.XT = nullptr;
  rc |= e->alloc(&p, (size_t)P * D2 * bp * 2); a.H2T = (bf16*)p;
  rc |= e->alloc(&p, (size_t)P * D2 * bp * 2); a.dH2T = (bf16*)p;
  rc |= e->alloc(&p, (size_t)P * D1 * bp * 2); a.dH1T = (bf16*)p;
  rc |= e->alloc(&p, (size_t)P * 16 * bp * 2); a.dlogT = (bf16*)p;
  rc |= e->alloc(&p, (size_t)P * 4); e->d_active = (int*)p; a.active = e->d_active;
  rc |= e->alloc(&p, (size_t)P * 4); e->d_t0 = (int*)p; a.t0 = e->d_t0;
  rc |= e->alloc(&p, (size_t)P * 16); e->d_ctl = (int4*)p; a.ctl = e->d_ctl;
  rc |= e->alloc(&p, 16); e->d_seed = (unsigned long long*)p; a.seed = e->d_seed;
  rc |= e->alloc(&p, sizeof(PubDst)); e->d_pub = (PubDst*)p;
  e->ctl_host.assign(P, int4{0, 0, 0, 0});
  rc |= e->alloc(&p, (size_t)P * 4); e->d_loss = (float*)p; a.loss_acc = e->d_loss;
  rc |= e->alloc(&p, (size_t)P * 4); e->d_correct = (int*)p; a.correct_acc = e->d_correct;
  rc |= e->alloc(&p, (size_t)P * 256 * 4); e->d_conf = (int*)p; a.conf = e->d_conf;
  rc |= e->alloc_ring();
  {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&e->num_cus, hipDeviceAttributeMultiprocessorCount, dev);
    const char* env = getenv("MYFYP_MLP_PERSISTENT");
    if (env && env[0] == '0') e->persist_mode = 0;
    if (D1 == 256 && D2 == 128 && (a.Bpad == 32 || a.Bpad == 64)) {
      const size_t xb = mlp_persistent_bytes(P, a.Bpad);
      rc |= e->alloc(&p, xb);
      e->pb.h1x = (bf16*)p;
      e->pb.w2x = e->pb.h1x + (size_t)P * a.Bpad * 256;
      e->pb.dh2x = e->pb.w2x + (size_t)P * 128 * 256;
      e->pb.flag_bytes = mlp_persistent_flag_bytes(P);
      rc |= e->alloc(&p, e->pb.flag_bytes);
      e->pb.flags = (unsigned*)p;
      rc |= e->alloc(&p, MLP_ERR_WORDS * sizeof(int));
      e->pb.err = (int*)p;
      if (mlp_persistent_prepare(a) != hipSuccess) e->persist_mode = 0;
      // fp32 exchange buffers + flags (err word shared)
      rc |= e->alloc(&p, mlp_persistent_f32_bytes(P, a.Bpad));
      e->pb32.h1x = (float*)p;
      e->pb32.plx = e->pb32.h1x + mlp_persistent_f32_h1x_floats(P, a.Bpad);  // H1 partials: [P][KSMAX][parity]
      e->pb32.dh2x = e->pb32.plx + (size_t)P * 8 * a.Bpad * 16 * 2;           // LL pairs
      rc |= e->alloc(&p, (size_t)P * sizeof(unsigned));
      e->pb32.gen = (unsigned*)p;
      e->pb32.flag_bytes = mlp_persistent_f32_flag_bytes(P);
      rc |= e->alloc(&p, e->pb32.flag_bytes);
      e->pb32.flags = (unsigned*)p;
      e->pb32.err = e->pb.err;
      if (mlp_persistent_f32_prepare(a) != hipSuccess) e->pb32.h1x = nullptr;
    }
  }
  if (rc) {
    delete e;
    return nullptr;
  }
  a.opt = OptParams{0, 1e-3f, 0.9f, 0.999f, 1e-8f, 0.f, 0.f, 0, 0.f};
  return e;
}

void mlp_engine_destroy(void* h) { delete (MLPEngine*)h; }

int64_t mlp_engine_numel(void* h) { return ((MLPEngine*)h)->a.numel; }

int mlp_engine_bind_params(void* h, float* params, bf16* shadow, bf16* w2t, float* m, float* v, int64_t S) {
  auto* e = (MLPEngine*)h;
  std::lock_guard<std::mutex> g(e->mu);
  e->a.params = params; e->a.shadow = shadow; e->a.w2t = w2t; e->a.m = m; e->a.v = v; e->a.S = S;
  e->invalidate();
  return 0;
}

int mlp_engine_set_train_data(void* h, const uint64_t* Xp, const uint64_t* Yp, const int* n, const int* perm, int64_t perm_stride, int max_steps) {
  auto* e = (MLPEngine*)h;
  std::lock_guard<std::mutex> g(e->mu);
  e->a.Xp = (const uint8_t* const*)Xp; e->a.Yp = (const int* const*)Yp; e->a.n = n; e->a.perm = perm; e->a.perm_stride = perm_stride;
  e->max_steps = max_steps;
  const int64_t rows = (int64_t)(max_steps > 0 ? max_steps : 1) * e->a.B;
  if (rows != e->a.xb_rows) {  // epoch batch buffers
    if (e->a.Xb) hipFree(e->a.Xb);
    if (e->a.Xb16) hipFree(e->a.Xb16);
    if (e->a.Yb) hipFree(e->a.Yb);
    e->a.Xb = nullptr;
    e->a.Xb16 = nullptr;
    e->a.Yb = nullptr;
    CHECK_HIP(hipMalloc((void**)&e->a.Xb, (size_t)e->a.P * rows * e->a.D0));
    CHECK_HIP(hipMalloc((void**)&e->a.Yb, (size_t)e->a.P * rows * sizeof(int)));
    CHECK_HIP(hipMemset(e->a.Xb, 0, (size_t)e->a.P * rows * e->a.D0));
    CHECK_HIP(hipMemset(e->a.Yb, 0, (size_t)e->a.P * rows * sizeof(int)));
    if (e->a.xidx) hipFree(e->a.xidx);
    CHECK_HIP(hipMalloc((void**)&e->a.xidx, (size_t)e->a.P * rows * sizeof(int)));
    CHECK_HIP(hipMemset(e->a.xidx, 0, (size_t)e->a.P * rows * sizeof(int)));
    if (e->xb16_buf[1]) hipFree(e->xb16_buf[1]);
    if (e->yb_buf[1]) hipFree(e->yb_buf[1]);
    e->xb16_buf[0] = e->xb16_buf[1] = nullptr;
    e->yb_buf[0] = e->yb_buf[1] = nullptr;
    if (e->pb.h1x != nullptr) {
      CHECK_HIP(hipMalloc((void**)&e->a.Xb16, (size_t)e->a.P * rows * e->a.D0 * sizeof(bf16)));
      CHECK_HIP(hipMemset(e->a.Xb16, 0, (size_t)e->a.P * rows * e->a.D0 * sizeof(bf16)));
      // second batch buffers for the prep-stream gather (288 GB of HBM: ~95 MB each is nothing)
      CHECK_HIP(hipMalloc((void**)&e->xb16_buf[1], (size_t)e->a.P * rows * e->a.D0 * sizeof(bf16)));
      CHECK_HIP(hipMemset(e->xb16_buf[1], 0, (size_t)e->a.P * rows * e->a.D0 * sizeof(bf16)));
      CHECK_HIP(hipMalloc((void**)&e->yb_buf[1], (size_t)e->a.P * rows * sizeof(int)));
      CHECK_HIP(hipMemset(e->yb_buf[1], 0, (size_t)e->a.P * rows * sizeof(int)));
    }
    e->a.xb_rows = rows;
  }
  e->invalidate();
  return 0;
}

// Direct-X fp32 epochs: per-peer device pointers to exact-bf16 copies of the training images ([n_p][D0],
// the caller keeps them alive and rebinds when the data changes). Re-captures.
// Drain the prep stream (the next epoch's gather, enqueued ahead, reads the bound data tensors)
// and forget the gathers ahead: called before the caller drops its references to the data it
// bound, since the torch allocator does not know this stream.
int mlp_engine_drain_prep(void* h) {
  auto* e = (MLPEngine*)h;
  std::lock_guard<std::mutex> g(e->mu);
  if (e->prep_stream) CHECK_HIP(hipStreamSynchronize(e->prep_stream));
  e->ahead_valid[0] = e->ahead_valid[1] = false;
  return 0;
}

int mlp_engine_set_train_x16(void* h, const uint64_t* Xp16) {
  auto* e = (MLPEngine*)h;
  std::lock_guard<std::mutex> g(e->mu);
  e->a.Xp16 = (const bf16* const*)Xp16;
  e->invalidate();
  return 0;
}
// 1 if this build's fp32 layout-1 epoch reads X directly (the caller then binds the bf16 images)
int mlp_engine_x_direct_build() { return mlp_persistent_f32_x_direct_build(); }
// 1 if the fp32 epoch of this engine's current configuration reads X directly (needs set_train_x16)
int mlp_engine_x_direct(void* h) {
  auto* e = (MLPEngine*)h;
  return e->precision == 1 && mlp_persistent_f32_x_direct(e->a) ? 1 : 0;
}

// host copies of the per-peer sample counts (packed into the control words)
int mlp_engine_set_counts(void* h, const int* n_host, const int* nt_host) {
  auto* e = (MLPEngine*)h;
  for (int p = 0; p < e->a.P; ++p) {
    if (e->ctl_host[p].y != n_host[p]) e->ahead_valid[0] = e->ahead_valid[1] = false;
    e->ctl_host[p].y = n_host[p];
    e->ctl_host[p].w = nt_host[p];
  }
  return 0;
}

int mlp_engine_set_test_data(void* h, const uint64_t* Xtp, const uint64_t* Ytp, const int* n_t, int max_rows) {
  auto* e = (MLPEngine*)h;
  std::lock_guard<std::mutex> g(e->mu);
  e->a.Xtp = (const uint8_t* const*)Xtp; e->a.Ytp = (const int* const*)Ytp; e->a.n_t = n_t;
  e->max_test_rows = max_rows;
  return 0;
}

int mlp_engine_set_optimizer(void* h, int kind, float lr, float b1, float b2, float eps, float wd, float momentum, int nesterov, float mu) {
  auto* e = (MLPEngine*)h;
  std::lock_guard<std::mutex> g(e->mu);
  OptParams o{kind, lr, b1, b2, eps, wd, momentum, nesterov, mu, e->a.cg != nullptr ? 1 : 0};
  if (memcmp(&o, &e->a.opt, sizeof(o)) != 0) {
    e->a.opt = o;
    e->invalidate();
  }
  return 0;
}

int mlp_engine_set_extras(void* h, const float* anchor, const float* cg, const float* cl) {
  auto* e = (MLPEngine*)h;
  std::lock_guard<std::mutex> g(e->mu);
  if (anchor != e->a.anchor || cg != e->a.cg || cl != e->a.cl) {
    e->a.anchor = anchor; e->a.cg = cg; e->a.cl = cl;
    e->a.opt.scaf_upd = cg != nullptr ? 1 : 0;
    e->invalidate();
  }
  return 0;
}

// Upload the active mask, zero the accumulators and refresh the bf16 shadows (stream-ordered,
// never blocks the host).
int mlp_engine_begin(void* h, const int* active_host, void* stream) {
  auto* e = (MLPEngine*)h;
  hipStream_t s = (hipStream_t)stream;
  for (int p = 0; p < e->a.P; ++p) e->ctl_host[p].x = active_host[p];
  if (e->use_persistent()) {
    // the persistent epoch reads the fp32 master rows (no shadow refresh needed) and the next
    // epoch upload carries the mask and zeroes the accumulators: nothing to launch here
    e->active_host_cache.assign(active_host, active_host + e->a.P);
    e->pending_zero_acc = true;
    return 0;
  }
  if (e->upload(s, active_host)) return 1;
  CHECK_HIP(hipMemsetAsync(e->d_loss, 0, sizeof(float) * e->a.P, s));
  CHECK_HIP(hipMemsetAsync(e->d_correct, 0, sizeof(int) * e->a.P, s));
  if (e->pb.err) CHECK_HIP(hipMemsetAsync(e->pb.err, 0, MLP_ERR_WORDS * sizeof(int), s));
  mlp_launch_sync_shadow(e->a, s);
  CHECK_HIP(hipGetLastError());
  return 0;
}

// Zero the Adam moments of every slot (fresh optimizer state per fit; one memset node each).
int mlp_engine_zero_state(void* h, void* stream) {
  auto* e = (MLPEngine*)h;
  hipStream_t s = (hipStream_t)stream;
  if (e->use_persistent()) {  // the next persistent epoch starts its moments at 0 in registers
    e->pending_fresh = true;
    return 0;
  }
  const size_t bytes = (size_t)e->a.P * e->a.S * sizeof(float);
  CHECK_HIP(hipMemsetAsync(e->a.m, 0, bytes, s));
  if (e->a.v) CHECK_HIP(hipMemsetAsync(e->a.v, 0, bytes, s));
  return 0;
}

// Epoch shuffle: native = 1 draws every peer's permutation inside the gather kernel (keyed
// Feistel permutation, key uploaded per epoch with the control words); 0 reads `perm`.
int mlp_engine_set_shuffle(void* h, int native) {
  auto* e = (MLPEngine*)h;
  std::lock_guard<std::mutex> g(e->mu);
  if (native != e->a.shuffle_native) {
    e->a.shuffle_native = native;
    e->invalidate();
  }
  return 0;
}
int mlp_engine_set_epoch_seed(void* h, unsigned long long seed) {
  ((MLPEngine*)h)->seed_host = seed;
  return 0;
}

// Shuffle key of the epoch after the next one launched: that launch then enqueues its gather ahead
// (prep mode; see MLPEngine::next_seed). The caller passes the same key to set_epoch_seed later.
int mlp_engine_set_next_epoch_seed(void* h, unsigned long long seed) {
  auto* e = (MLPEngine*)h;
  e->next_seed = seed;
  e->next_seed_valid = true;
  return 0;
}

// Persistent-epoch mode: -1 auto (default; MYFYP_MLP_PERSISTENT=0 turns it off), 0 off.
int mlp_engine_set_persistent(void* h, int mode) {
  auto* e = (MLPEngine*)h;
  std::lock_guard<std::mutex> g(e->mu);
  if (mode != e->persist_mode) {
    e->persist_mode = mode;
    e->invalidate();
  }
  return 0;
}

// Precision of the engine: 1 = fp32 (default), 0 = bf16 operands / fp32 master weights.
int mlp_engine_set_precision(void* h, int precision) {
  auto* e = (MLPEngine*)h;
  std::lock_guard<std::mutex> g(e->mu);
  if (precision != e->precision) {
    e->precision = precision;
    e->invalidate();
  }
  return 0;
}
// 1 if the fp32 persistent epoch supports this shape and local batch on this device.
int mlp_f32_ok(int D0, int D1, int D2, int D3, int B) {
  if (!mlp_shape_supported(D0, D1, D2, D3) || B < 1) return 0;
  MLPArgs a{};
  a.D0 = D0; a.D1 = D1; a.D2 = D2; a.D3 = D3;
  a.B = B;
  a.Bpad = (B + 31) / 32 * 32;
  int dev = 0, cus = 0;
  hipGetDevice(&dev);
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (!mlp_persistent_f32_supported(a) || mlp_persistent_f32_prepare(a) != hipSuccess) return 0;
  return mlp_persistent_f32_launch_wgs(a) <= mlp_persistent_f32_resident_capacity(a, cus) ? 1 : 0;
}
// Debug: the owners of the fp32 epoch write their W2 replica to `buf` ([P][D2][D1] fp32) after the
// epoch (null = off), for the bitwise check against the heads' rows.
int mlp_engine_set_w2chk(void* h, float* buf) {
  auto* e = (MLPEngine*)h;
  std::lock_guard<std::mutex> g(e->mu);
  if (buf != e->pb32.w2chk) {
    e->pb32.w2chk = buf;
    e->invalidate();
  }
  return 0;
}

// 1 if the next epoch runs as the persistent kernel.
int mlp_engine_uses_persistent(void* h) { return ((MLPEngine*)h)->use_persistent() ? 1 : 0; }

// One local epoch for every active peer: a single graph replay (captured on first use). slot >= 0:
// the graph's last node publishes the fit's results into that ring slot (mlp_engine_stats_async
// for the slot is then a no-op); -1: nothing (earlier epochs of a multi-epoch fit, or the caller
// publishes with mlp_engine_stats_async).
static int run_epoch_impl(MLPEngine* e, const int* t0_host, int slot, hipStream_t s);
int mlp_engine_run_epoch(void* h, const int* t0_host, void* stream) { return run_epoch_impl((MLPEngine*)h, t0_host, -1, (hipStream_t)stream); }
int mlp_engine_run_epoch_pub(void* h, const int* t0_host, int slot, void* stream) {
  return run_epoch_impl((MLPEngine*)h, t0_host, slot, (hipStream_t)stream);
}
static int run_epoch_impl(MLPEngine* e, const int* t0_host, int slot, hipStream_t s) {
  std::lock_guard<std::mutex> g(e->mu);
  if (e->max_steps <= 0) return 0;
  if (e->precision == 1 && !e->use_persistent()) {
    g_last_error = "fp32 MLP engine: shape / batch / CU count not supported by the fp32 persistent epoch (no silent bf16 fallback)";
    return 2;
  }
  if (!e->exec || e->graph_steps != e->max_steps) {
    if (e->capture(e->max_steps)) return 1;
  }
  for (int p = 0; p < e->a.P; ++p) e->ctl_host[p].z = t0_host[p];
  const bool pa = e->graph_persistent && e->pending_zero_acc;
  PubDst pd{};
  ResultSlot* pr = nullptr;
  if (slot >= 0 && e->graph_has_pub) {
    pr = &e->ring[slot % MLP_RING];
    pd = PubDst{pr->loss, pr->correct, pr->err, pr->seq, pr->gen.load() + 1};
  }
  if (e->upload(s, pa ? e->active_host_cache.data() : nullptr, pa, e->graph_persistent && e->pending_fresh, e->prep_mode, &pd)) return 1;
  if (e->graph_persistent) e->pending_zero_acc = e->pending_fresh = false;
  const int buf = e->n_execs > 1 ? (int)(e->launches & 1) : 0;  // the executable launch_graph takes
  if (e->prep_mode) {
    const bool have = e->ahead_valid[buf] && e->ahead_seed[buf] == e->seed_host;
    e->ahead_valid[buf] = false;
    if (!have && e->prep_gather(buf, s, e->seed_host)) return 1;
    CHECK_HIP(hipStreamWaitEvent(s, e->ev_gath[buf], 0));
  }
  if (e->graph_persistent) {
    GangOrder& go = gang_order(s);
    std::lock_guard<std::mutex> og(go.mu);
    if (!go.ev) CHECK_HIP(hipEventCreateWithFlags(&go.ev, hipEventDisableTiming));
    if (gang_event_always()) {
      if (go.ev_ready) CHECK_HIP(hipStreamWaitEvent(s, go.ev, 0));
    } else if (go.has_last && go.last != s) {
      CHECK_HIP(hipEventRecord(go.ev, go.last));
      CHECK_HIP(hipStreamWaitEvent(s, go.ev, 0));
    }
    const bool after_eval = e->prep_mode && e->prep_level == 2 && e->n_execs > 1 && e->next_seed_valid && e->last_eval_done != nullptr &&
                            e->snap_rec_stream == s && e->snap_rec_launches == e->launches && eval_gather_order();
    if (e->prep_mode && e->prep_level == 2) {
      if (after_eval) {
        e->start_rec = false;  // a later gather that is not ahead records its own ordering event
      } else {
        CHECK_HIP(hipEventRecord(e->ev_start, s));
        e->start_rec = true;
      }
    }
    if (e->launch_epoch(s)) return 1;
    if (e->prep_mode && e->prep_level == 1) {  // (mode 2 orders its gathers by ev_start)
      CHECK_HIP(hipEventRecord(e->ev_done[buf], s));
      e->done_rec[buf] = true;
    }
    if (e->prep_mode && e->prep_level == 2 && e->n_execs > 1 && e->next_seed_valid) {
      const int nb = buf ^ 1;  // the buffer the next launch's executable reads
      if (e->prep_gather(nb, s, e->next_seed, true, after_eval)) return 1;
      e->ahead_valid[nb] = true;
      e->ahead_seed[nb] = e->next_seed;
    }
    e->next_seed_valid = false;
    if (gang_event_always()) {
      CHECK_HIP(hipEventRecord(go.ev, s));
      go.ev_ready = true;
    }
    go.has_last = true;
    go.last = s;
  } else {
    if (e->launch_epoch(s)) return 1;
  }
  if (pr != nullptr) {
    pr->stream = s;
    pr->gen.store(pd.gen);
    e->graph_pub_slot = slot;
  }
  return 0;
}

// One-time setup ahead of the first epoch (node start, Settings.ENGINE_PREWARM): capture and
// instantiate the epoch graph for the bound data and optimizer, upload its executables, allocate
// the overlapped-evaluation resources, and load this library's code object with a no-op launch.
// No training work runs: the first real epoch then starts from a ready graph instead of paying
// these in round 0 (which time-to-accuracy counts).
int mlp_engine_prepare(void* h, void* stream) {
  auto* e = (MLPEngine*)h;
  std::lock_guard<std::mutex> g(e->mu);
  hipStream_t s = (hipStream_t)stream;
  if (e->max_steps <= 0) return 0;
  if (e->precision == 1 && !e->use_persistent()) return 0;  // run_epoch reports it
  // MYFYP_TIME_PREPARE=1: host µs of each part on stderr (node-start breakdown, profiles/r5_start)
  static const bool timed = [] {
    const char* v = getenv("MYFYP_TIME_PREPARE");
    return v != nullptr && atoi(v) != 0;
  }();
  auto now = [] { return std::chrono::steady_clock::now(); };
  auto us = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
    return (long long)std::chrono::duration_cast<std::chrono::microseconds>(b - a).count();
  };
  const auto t0 = now();
  if (!e->exec || e->graph_steps != e->max_steps) {
    if (e->capture(e->max_steps)) return 1;
  }
  const auto t1 = now();
  for (int i = 0; i < e->n_execs; ++i)
    if (e->execs[i]) CHECK_HIP(hipGraphUpload(e->execs[i], s));
  const auto t2 = now();
  if (e->use_persistent() && e->ensure_eval_side()) return 1;
  const auto t3 = now();
  // code-object load: a publish of zero peers (its only store zeroes d_correct[0], which every fit
  // re-zeroes before accumulating; no ring slot is touched)
  hipLaunchKernelGGL(k_publish, dim3(1), dim3(256), 0, s, e->d_loss, e->d_correct, (const int*)nullptr, (const int*)nullptr, 0, e->d_loss,
                     e->d_correct, e->d_correct, (int*)nullptr, (unsigned*)nullptr, 0u);
  CHECK_HIP(hipGetLastError());
  if (timed)
    fprintf(stderr, "[prepare] capture %lld us, upload %lld us, eval side %lld us, publish launch %lld us\n", us(t0, t1), us(t1, t2), us(t2, t3),
            us(t3, now()));
  return 0;
}

// Host time spent inside hipGraphLaunch: out[0] launches, out[1] total ns, out[2] max ns.
int mlp_engine_graph_launch_stats(void* h, unsigned long long* out) {
  auto* e = (MLPEngine*)h;
  std::lock_guard<std::mutex> g(e->mu);
  out[0] = e->launches;
  out[1] = e->launch_ns;
  out[2] = e->launch_max_ns;
  return e->n_execs;
}

// Same epoch without the graph (debug / profiling A-B).
int mlp_engine_run_epoch_eager(void* h, const int* t0_host, void* stream) {
  auto* e = (MLPEngine*)h;
  hipStream_t s = (hipStream_t)stream;
  for (int p = 0; p < e->a.P; ++p) e->ctl_host[p].z = t0_host[p];
  const bool pers = e->use_persistent();
  const bool pa = pers && e->pending_zero_acc;
  if (e->upload(s, pa ? e->active_host_cache.data() : nullptr, pa, pers && e->pending_fresh)) return 1;
  if (pers) e->pending_zero_acc = e->pending_fresh = false;
  if (e->precision == 1 && !pers) {
    g_last_error = "fp32 MLP engine: shape / batch / CU count not supported by the fp32 persistent epoch";
    return 2;
  }
  if (pers && e->precision == 1 && mlp_persistent_f32_x_direct(e->a)) {
    if (e->a.Xp16 == nullptr || e->a.xidx == nullptr) {
      g_last_error = "fp32 direct-X epoch: no bf16 image table bound (mlp_engine_set_train_x16)";
      return 1;
    }
    e->a.x_direct = 1;
    mlp_launch_index_epoch(e->a, s);
  } else {
    MLPArgs ga = e->a;
    if (!pers) ga.Xb16 = nullptr;
    mlp_launch_gather_epoch(ga, s);
  }
  if (pers) {
    if (e->launch_epoch_kernel(s, true)) return 1;
  } else {
    for (int st = 0; st < e->max_steps; ++st) mlp_launch_train_step(e->a, st, s);
  }
  CHECK_HIP(hipGetLastError());
  return 0;
}

// ---- asynchronous results: enqueue D2H into pinned ring slot `slot`, fetch later
int mlp_engine_stats_async(void* h, int slot, void* stream) {
  auto* e = (MLPEngine*)h;
  hipStream_t s = (hipStream_t)stream;
  ResultSlot& r = e->ring[slot % MLP_RING];
  if (e->graph_pub_slot == slot) {  // the epoch graph already published into this slot
    e->graph_pub_slot = -1;
    return 0;
  }
  e->graph_pub_slot = -1;
  if (e->pending_zero_acc) {  // a fit with no epoch launched: zero what it would have zeroed
    if (e->upload(s, e->active_host_cache.data(), true, false)) return 1;
    e->pending_zero_acc = false;
  }
  if (e->publish(s, r, e->d_loss, e->d_correct, e->pb.err, nullptr)) return 1;
  return 0;
}

// Forward the whole test split of every active peer (loss sum, correct, confusion [P][16][16]) into slot.
int mlp_engine_eval_async(void* h, const int* active_host, int slot, void* stream) {
  auto* e = (MLPEngine*)h;
  hipStream_t s = (hipStream_t)stream;
  ResultSlot& r = e->ring[slot % MLP_RING];
  for (int p = 0; p < e->a.P; ++p) e->ctl_host[p].x = active_host[p];
  if (e->use_persistent()) {
    // Overlapped evaluation: snapshot the parameters on the main stream (one launch: control words,
    // accumulators, fp32 + bf16 + W2T copies), then evaluate the snapshot on the side stream while
    // the main stream goes on to the epoch, whose gangs leave ~half of the CUs free. The evaluation
    // that last used this side (two evaluations back) must be done with it before it is overwritten.
    std::lock_guard<std::mutex> g(e->mu);
    if (e->ensure_eval_side()) return 1;
    auto& es = e->eside[e->eval_idx];
    e->eval_idx ^= 1;
    // evaluation r-2 (a host wait, not a stream wait), polled: a blocking hipEventSynchronize
    // sleeps until an interrupt and stalled the round driver up to 11 ms (profiles/r4l_*)
    if (es.rec) {
      for (long it = 0;; ++it) {
        const hipError_t q = hipEventQuery(es.done);
        if (q == hipSuccess) break;
        if (q != hipErrorNotReady) CHECK_HIP(q);
        if (it >= 64) std::this_thread::sleep_for(std::chrono::microseconds(20));
      }
    }
    CtlUpload u{};
    u.P = e->a.P;
    u.with_active = 1;
    u.seed = e->seed_host;
    for (int p = 0; p < e->a.P; ++p) {
      u.ctl[p] = e->ctl_host[p];
      u.active[p] = active_host[p];
    }
    u.zero_loss = es.loss;
    u.zero_correct = es.correct;
    u.zero_conf = es.conf;
    MLPArgs ea = e->a;
    ea.params = es.params;
    ea.shadow = es.shadow;
    ea.w2t = es.w2t;
    ea.ctl = es.ctl;
    ea.active = es.active;
    ea.loss_acc = es.loss;
    ea.correct_acc = es.correct;
    ea.conf = es.conf;
    {
      const int64_t blocks = (e->a.numel + 255) / 256;
      hipLaunchKernelGGL(k_eval_snapshot, dim3((unsigned)(blocks < 1024 ? blocks : 1024), e->a.P), dim3(256), 0, s, e->a, es.params,
                         es.shadow, es.w2t, u, es.ctl, es.active);
      CHECK_HIP(hipGetLastError());
    }
    CHECK_HIP(hipEventRecord(e->ev_snap, s));
    hipStream_t xs = e->eval_stream;
    CHECK_HIP(hipStreamWaitEvent(xs, e->ev_snap, 0));
    // debug (MYFYP_DEBUG_NO_EVAL=1, timing experiments only): no evaluation kernel beside the epoch
    // (results read as zero loss / accuracy; prices the evaluation's interference)
    static const bool no_eval = [] {
      const char* v = getenv("MYFYP_DEBUG_NO_EVAL");
      return v != nullptr && atoi(v) != 0;
    }();
    if (!no_eval) e->launch_eval(ea, xs);
    CHECK_HIP(hipGetLastError());
    if (e->publish(xs, r, es.loss, es.correct, nullptr, es.conf)) return 1;
    CHECK_HIP(hipEventRecord(es.done, xs));
    es.rec = true;
    e->snap_rec_stream = s;
    e->snap_rec_launches = e->launches;
    e->last_eval_done = es.done;
    return 0;
  }
  if (e->wait_evals(s)) return 1;
  if (e->upload(s, active_host)) return 1;
  CHECK_HIP(hipMemsetAsync(e->d_loss, 0, sizeof(float) * e->a.P, s));
  CHECK_HIP(hipMemsetAsync(e->d_correct, 0, sizeof(int) * e->a.P, s));
  CHECK_HIP(hipMemsetAsync(e->d_conf, 0, sizeof(int) * e->a.P * 256, s));
  if (e->precision != 1) mlp_launch_sync_shadow(e->a, s);
  e->launch_eval(e->a, s);
  CHECK_HIP(hipGetLastError());
  if (e->publish(s, r, e->d_loss, e->d_correct, nullptr, e->d_conf)) return 1;
  return 0;
}

// Wait for slot's event, copy its pinned results out (conf may be null).
int mlp_engine_fetch(void* h, int slot, float* loss_host, int* correct_host, int* conf_host) {
  auto* e = (MLPEngine*)h;
  ResultSlot& r = e->ring[slot % MLP_RING];
  if (ring_events()) {
    CHECK_HIP(hipEventSynchronize(r.ev));
  } else {
    // poll the slot's sequence word: spin briefly, then sleep in 20 us steps; every ~0.5 s ask the
    // publishing stream for a fault (a faulted stream reports it; an idle one must have published)
    const unsigned want = r.gen.load();
    for (long it = 0;; ++it) {
      if (__atomic_load_n(r.seq, __ATOMIC_ACQUIRE) == want) break;
      if (it < 256) continue;
      std::this_thread::sleep_for(std::chrono::microseconds(20));
      if ((it & 16383) == 0) {
        const hipError_t q = hipStreamQuery(r.stream);
        if (q != hipSuccess && q != hipErrorNotReady) {
          g_last_error = std::string("result publish: ") + hipGetErrorString(q);
          return 1;
        }
        if (q == hipSuccess && __atomic_load_n(r.seq, __ATOMIC_ACQUIRE) != want) {
          g_last_error = "result publish: stream idle but the slot's sequence word was not written";
          return 1;
        }
      }
    }
  }
  memcpy(loss_host, r.loss, sizeof(float) * e->a.P);
  memcpy(correct_host, r.correct, sizeof(int) * e->a.P);
  if (conf_host) memcpy(conf_host, r.conf, sizeof(int) * e->a.P * 256);
  const int st = *r.err;
  if (st & 2) e->recoveries++;
  if (st & 1) {
    g_last_error = "persistent MLP epoch gave up (a gang workgroup was not resident or a hand-off timed out) and its retry did not recover";
    return 3;
  }
  return 0;
}

// Give-ups recovered by the retry launch so far (fetched results only).
int mlp_engine_recoveries(void* h) { return ((MLPEngine*)h)->recoveries; }

// fp32 persistent epoch: owner K split (1 or 2; 0 = by engine capacity). Re-captures on change.
int mlp_engine_set_f32_ks(void* h, int ks) {
  auto* e = (MLPEngine*)h;
  std::lock_guard<std::mutex> g(e->mu);
  if (ks != e->a.f32_ks) {
    e->a.f32_ks = ks;
    e->f32_cap_bpad = -1;  // the co-resident capacity depends on the instantiation
    e->invalidate();
  }
  return 0;
}
// CUs reserved for a concurrent RCCL kernel in the co-residency capacity (0 = none). Re-captures.
int mlp_engine_set_reserved_cus(void* h, int cus) {
  auto* e = (MLPEngine*)h;
  std::lock_guard<std::mutex> g(e->mu);
  if (cus < 0) cus = 0;
  if (cus != e->reserved_cus) {
    e->reserved_cus = cus;
    e->f32_cap_bpad = -1;
    e->invalidate();
  }
  return 0;
}
int mlp_engine_f32_ks(void* h) { return mlp_persistent_f32_ks(((MLPEngine*)h)->a); }
// fp32 persistent epoch gang layout (1 owners + heads, 2 owners only; 0 = default). Re-captures.
int mlp_engine_set_f32_variant(void* h, int v) {
  auto* e = (MLPEngine*)h;
  std::lock_guard<std::mutex> g(e->mu);
  if (v != e->a.f32_variant) {
    e->a.f32_variant = v;
    e->f32_cap_bpad = -1;
    e->invalidate();
  }
  return 0;
}
int mlp_engine_f32_variant(void* h) { return mlp_persistent_f32_variant(((MLPEngine*)h)->a); }

// Test hook: peer p's next fp32 epochs give up on their first attempt (p < 0: off), at launch or
// (at_end) at the gang commit after the last step. Re-captures.
int mlp_engine_debug_giveup(void* h, int peer, int at_end) {
  auto* e = (MLPEngine*)h;
  std::lock_guard<std::mutex> g(e->mu);
  e->a.debug_giveup = peer < 0 ? 0 : peer + 1 + (at_end ? 256 : 0);
  e->invalidate();
  return 0;
}

// Test hook: fill the whole hand-off flag block with ~0 before each epoch's (sparse) flag zeroing
// (on = 1 / 0; -1 leaves the setting). Returns how many uploads have poisoned it so far.
int mlp_engine_debug_poison_flags(void* h, int on) {
  auto* e = (MLPEngine*)h;
  std::lock_guard<std::mutex> g(e->mu);
  if (on >= 0) e->debug_poison_flags = on != 0;
  return e->poisoned;
}

int mlp_engine_ring_size() { return MLP_RING; }

// synchronous conveniences (tests / tools)
int mlp_engine_read_stats(void* h, float* loss_host, int* correct_host, void* stream) {
  if (mlp_engine_stats_async(h, MLP_RING - 1, stream)) return 1;
  return mlp_engine_fetch(h, MLP_RING - 1, loss_host, correct_host, nullptr);
}

int mlp_engine_eval(void* h, const int* active_host, float* loss_host, int* correct_host, int* conf_host, void* stream) {
  if (mlp_engine_eval_async(h, active_host, MLP_RING - 1, stream)) return 1;
  return mlp_engine_fetch(h, MLP_RING - 1, loss_host, correct_host, conf_host);
}

}  // extern "C"

// Load every kernel translation unit's code object on the current device (engine prewarm, once per
// device): a unit's first launch otherwise loads it then, and that load waited for the kernels in
// flight — the first FedAvg of a run blocked the host for the whole running epoch (1.7 ms,
// profiles/r5_start). Returns the number of units that failed to resolve.
extern "C" int myfyp_warm_fl_ops();
extern "C" int myfyp_warm_cnn_ops();
extern "C" int myfyp_warm_conv();
extern "C" int myfyp_warm_lenet();
extern "C" int myfyp_warm_mlp_fused();
extern "C" int myfyp_warm_mlp_f32();
// families: bit 0 = the MLP engine's units, bit 1 = the CNN engine's (FedAvg kernels in both)
extern "C" int myfyp_warm_all(int families) {
  hipFuncAttributes attr;
  int bad = myfyp_warm_fl_ops();
  if (families & 1)
    bad += (hipFuncGetAttributes(&attr, reinterpret_cast<const void*>(&k_publish)) == hipSuccess ? 0 : 1) + myfyp_warm_mlp_fused() + myfyp_warm_mlp_f32();
  if (families & 2) bad += myfyp_warm_cnn_ops() + myfyp_warm_conv() + myfyp_warm_lenet();
  return bad;
}
