// In-process RCCL device mesh: one process drives G MI355X devices.
//
// The reference keeps every peer of a simulation in ONE process and moves models between them with
// direct method calls (p2pfl/communication/protocols/memory/server_singleton.py:22-43,
// memory_client.py:139). The MI355X equivalent keeps that process model: peers are placed
// round-robin over the G devices, and the weights plane is a set of G RCCL communicators created
// together by ncclCommInitAll. Every collective is issued from ONE host thread for all G devices
// inside ncclGroupStart/End (the single-thread multi-device pattern RCCL requires), on each
// device's compute stream, so the round's device work stays stream-ordered and the host never
// waits:
//
//   rmesh_allreduce / rmesh_broadcast / rmesh_allgather / rmesh_p2p — grouped collectives over
//   the mesh (p2p = the NeighborAvg topology exchange);
//   rmesh_fedavg — the whole FedAvg of G stacked engine groups: per device the weighted partial
//   sum of its rows (k_fedavg_reduce, weights as kernel arguments) → ONE grouped all-reduce of
//   [Σ w x | Σ w] over xGMI → per device the apply kernel writing the mean into its live rows;
//   rmesh_fedavg_bucketed — the same FedAvg bucketed and overlapped: per device the reduce and
//   the per-bucket grouped all-reduces on a side (comm) stream, the compute stream waiting per
//   bucket for its apply (or not at all: delayed averaging, landed by rmesh_delayed_land);
//   rmesh_check / rmesh_abort / rmesh_shrink — failure handling: poll ncclCommGetAsyncError,
//   ncclCommAbort every communicator (local: ends kernels stuck on a dead peer), and rebuild the
//   mesh over the surviving devices with a fresh ncclCommInitAll;
//   rmesh_rebuild — the same rebuild for a HEALTHY mesh (a device whose last peer left): the
//   caller has drained every device, so the communicators are destroyed, not aborted (an abort
//   would end collectives still queued on a device);
//   rmesh_debug_inject — fault hook: rmesh_check reports an asynchronous error on one rank.
// The round-level policy around these (deadline per collective, retained partial sums, aggregate
// what arrived) is parallel/mesh_guard.py.
//
// Every entry point returns 0 on success, non-zero on failure (message via rmesh_last_error()).
// The current HIP device of the calling thread is restored on return.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "../kernels/fl_ops.h"

namespace {

thread_local std::string g_err;

struct DevEvents {  // reusable events of one device (bucketed FedAvg)
  hipEvent_t ready = nullptr;       // compute stream -> comm stream: the rows are final
  std::vector<hipEvent_t> bucket;   // comm stream -> compute stream: bucket k is all-reduced
};

struct Mesh {
  std::vector<int> devs;          // HIP device ordinal per mesh rank
  std::vector<ncclComm_t> comms;  // one communicator per device (rank i <-> devs[i])
  bool aborted = false;
  int injected = -1;  // fault hook (rmesh_debug_inject): rmesh_check reports an error on this rank
  std::map<int, DevEvents> ev;  // by HIP device ordinal (survives a rebuild over fewer devices)
  int last_nb = 0;              // buckets of the last bucketed FedAvg (its last event = "landed")
};

struct DeviceGuard {  // restores the caller's current device
  int prev = -1;
  DeviceGuard() { (void)hipGetDevice(&prev); }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

bool nccl_ok(ncclResult_t r, const char* what) {
  if (r == ncclSuccess || r == ncclInProgress) return true;
  g_err = std::string(what) + ": " + ncclGetErrorString(r);
  return false;
}

bool hip_ok(hipError_t e, const char* what) {
  if (e == hipSuccess) return true;
  g_err = std::string(what) + ": " + hipGetErrorString(e);
  return false;
}

bool dtype_of(int code, ncclDataType_t* t, size_t* size) {
  switch (code) {
    case 0: *t = ncclFloat32; *size = 4; return true;
    case 1: *t = ncclBfloat16; *size = 2; return true;
    case 2: *t = ncclFloat16; *size = 2; return true;
    case 3: *t = ncclInt32; *size = 4; return true;
    case 4: *t = ncclInt64; *size = 8; return true;
    case 5: *t = ncclFloat64; *size = 8; return true;
    case 6: *t = ncclUint8; *size = 1; return true;
    default: g_err = "rmesh: unknown dtype code " + std::to_string(code); return false;
  }
}

bool usable(Mesh* m) {
  if (m == nullptr) {
    g_err = "rmesh: null mesh";
    return false;
  }
  if (m->aborted) {
    g_err = "rmesh: mesh was aborted (rebuild it with rmesh_shrink)";
    return false;
  }
  return true;
}

// Closes a ncclGroupStart opened by the caller whatever happened inside it (an unbalanced group
// would poison every later RCCL call of this thread).
bool group_end(bool ok) {
  ncclResult_t r = ncclGroupEnd();
  return nccl_ok(r, "ncclGroupEnd") && ok;
}

int fedavg_apply_all(Mesh* m, void** params, void** res, const int* P, int64_t n, const int64_t* ld, const float* mask, void** streams);

// the current device's events, with at least nb bucket events (created on first use)
DevEvents* events_for(Mesh* m, int dev, int nb) {
  DevEvents& e = m->ev[dev];
  if (e.ready == nullptr && !hip_ok(hipEventCreateWithFlags(&e.ready, hipEventDisableTiming), "hipEventCreate")) return nullptr;
  while ((int)e.bucket.size() < nb) {
    hipEvent_t x = nullptr;
    if (!hip_ok(hipEventCreateWithFlags(&x, hipEventDisableTiming), "hipEventCreate")) return nullptr;
    e.bucket.push_back(x);
  }
  return &e;
}

// [b0, b1) bucket bounds over n floats; every b0 a multiple of 4 (float4 kernels stay aligned)
int64_t bucket_step(int64_t bucket) {
  int64_t step = bucket / 4 * 4;
  return step < 4 ? 4 : step;
}

unsigned long long mask_bits(const float* mask, int off, int P) {
  unsigned long long bits = 0;
  for (int p = 0; p < P; ++p)
    if (mask[off + p] != 0.f) bits |= 1ull << p;
  return bits;
}

}  // namespace

extern "C" {

const char* rmesh_last_error() { return g_err.c_str(); }

int rmesh_version() {
  int v = 0;
  ncclGetVersion(&v);
  return v;
}

// One communicator per device of devs[0..ndev) (a device may appear only once: RCCL refuses two
// ranks on one device). Returns an opaque handle, or null (rmesh_last_error()).
void* rmesh_create(int ndev, const int* devs) {
  DeviceGuard g;
  if (ndev < 1 || devs == nullptr) {
    g_err = "rmesh_create: ndev must be >= 1";
    return nullptr;
  }
  int count = 0;
  if (!hip_ok(hipGetDeviceCount(&count), "hipGetDeviceCount")) return nullptr;
  for (int i = 0; i < ndev; ++i) {
    if (devs[i] < 0 || devs[i] >= count) {
      g_err = "rmesh_create: device " + std::to_string(devs[i]) + " not visible (" + std::to_string(count) + " devices)";
      return nullptr;
    }
    for (int j = 0; j < i; ++j)
      if (devs[j] == devs[i]) {
        g_err = "rmesh_create: device " + std::to_string(devs[i]) + " listed twice";
        return nullptr;
      }
  }
  auto* m = new Mesh();
  m->devs.assign(devs, devs + ndev);
  m->comms.assign(ndev, nullptr);
  if (!nccl_ok(ncclCommInitAll(m->comms.data(), ndev, m->devs.data()), "ncclCommInitAll")) {
    delete m;
    return nullptr;
  }
  return m;
}

int rmesh_size(void* h) { return h ? (int)static_cast<Mesh*>(h)->devs.size() : 0; }

int rmesh_device(void* h, int rank) {
  auto* m = static_cast<Mesh*>(h);
  return (m && rank >= 0 && rank < (int)m->devs.size()) ? m->devs[rank] : -1;
}

// In-place all-reduce of bufs[i] (count elements on device devs[i]) on streams[i]. op: 0 sum,
// 1 max, 2 min, 3 avg.
int rmesh_allreduce(void* h, void** bufs, int64_t count, int dtype, int op, void** streams) {
  auto* m = static_cast<Mesh*>(h);
  if (!usable(m)) return 1;
  ncclDataType_t t;
  size_t es;
  if (!dtype_of(dtype, &t, &es)) return 2;
  ncclRedOp_t rop = op == 1 ? ncclMax : op == 2 ? ncclMin : op == 3 ? ncclAvg : ncclSum;
  DeviceGuard g;
  bool ok = nccl_ok(ncclGroupStart(), "ncclGroupStart");
  if (!ok) return 1;
  for (size_t i = 0; i < m->devs.size() && ok; ++i)
    ok = nccl_ok(ncclAllReduce(bufs[i], bufs[i], (size_t)count, t, rop, m->comms[i], (hipStream_t)streams[i]), "ncclAllReduce");
  return group_end(ok) ? 0 : 1;
}

// bufs[root] is copied into every other device's buffer.
int rmesh_broadcast(void* h, void** bufs, int64_t count, int dtype, int root, void** streams) {
  auto* m = static_cast<Mesh*>(h);
  if (!usable(m)) return 1;
  if (root < 0 || root >= (int)m->devs.size()) {
    g_err = "rmesh_broadcast: root out of range";
    return 2;
  }
  ncclDataType_t t;
  size_t es;
  if (!dtype_of(dtype, &t, &es)) return 2;
  DeviceGuard g;
  if (!nccl_ok(ncclGroupStart(), "ncclGroupStart")) return 1;
  bool ok = true;
  for (size_t i = 0; i < m->devs.size() && ok; ++i)
    ok = nccl_ok(ncclBroadcast(bufs[i], bufs[i], (size_t)count, t, root, m->comms[i], (hipStream_t)streams[i]), "ncclBroadcast");
  return group_end(ok) ? 0 : 1;
}

// recv[i] (G * count elements) <- concat over ranks of send[r] (count elements each).
int rmesh_allgather(void* h, void** send, void** recv, int64_t count, int dtype, void** streams) {
  auto* m = static_cast<Mesh*>(h);
  if (!usable(m)) return 1;
  ncclDataType_t t;
  size_t es;
  if (!dtype_of(dtype, &t, &es)) return 2;
  DeviceGuard g;
  if (!nccl_ok(ncclGroupStart(), "ncclGroupStart")) return 1;
  bool ok = true;
  for (size_t i = 0; i < m->devs.size() && ok; ++i)
    ok = nccl_ok(ncclAllGather(send[i], recv[i], (size_t)count, t, m->comms[i], (hipStream_t)streams[i]), "ncclAllGather");
  return group_end(ok) ? 0 : 1;
}

// Grouped point-to-point exchange: op k is issued by mesh rank rank[k]; kind[k] 0 = send to
// peer[k], 1 = receive from peer[k]; bufs[k] holds counts[k] elements on rank[k]'s device,
// streams[k] is a stream of that device. All ops go in ONE group (no ordering deadlock).
int rmesh_p2p(void* h, int nops, const int* kind, const int* rank, const int* peer, void** bufs, const int64_t* counts, int dtype, void** streams) {
  auto* m = static_cast<Mesh*>(h);
  if (!usable(m)) return 1;
  ncclDataType_t t;
  size_t es;
  if (!dtype_of(dtype, &t, &es)) return 2;
  int G = (int)m->devs.size();
  for (int k = 0; k < nops; ++k)
    if (rank[k] < 0 || rank[k] >= G || peer[k] < 0 || peer[k] >= G || peer[k] == rank[k]) {
      g_err = "rmesh_p2p: op " + std::to_string(k) + " has a bad rank/peer";
      return 2;
    }
  DeviceGuard g;
  if (!nccl_ok(ncclGroupStart(), "ncclGroupStart")) return 1;
  bool ok = true;
  for (int k = 0; k < nops && ok; ++k) {
    ncclComm_t c = m->comms[rank[k]];
    hipStream_t s = (hipStream_t)streams[k];
    ok = kind[k] == 0 ? nccl_ok(ncclSend(bufs[k], (size_t)counts[k], t, peer[k], c, s), "ncclSend")
                      : nccl_ok(ncclRecv(bufs[k], (size_t)counts[k], t, peer[k], c, s), "ncclRecv");
  }
  return group_end(ok) ? 0 : 1;
}

// FedAvg of G stacked engine groups (group i on mesh rank i): params[i] is a [P_i][ld] fp32 row
// block, bufs[i] a scratch of n + 1 floats on that device, w[off_i .. off_i + P_i) the rows'
// sample weights (0 = not a trainer) and mask[...] the rows that receive the mean (every live
// local peer), with off_i = sum_{j<i} P_j. Per device: reduce (weights as kernel arguments) →
// one grouped all-reduce of [Σ w x | Σ w] → apply. Three launches per device, host never waits.
//
// outs (nullable): out-of-place all-reduce into outs[i] (n + 1 floats), the apply reads outs. bufs
// then keep each device's local partial sum after the call, so a failed or aborted all-reduce can
// be re-run over the surviving devices from them (rmesh_fedavg_retry) without re-reading rows the
// failed round's apply may already have overwritten.
int rmesh_fedavg(void* h, void** params, void** bufs, const int* P, int64_t n, const int64_t* ld, const float* w, const float* mask, void** streams,
                 void** outs) {
  auto* m = static_cast<Mesh*>(h);
  if (!usable(m)) return 1;
  const int G = (int)m->devs.size();
  DeviceGuard g;
  int off = 0;
  for (int i = 0; i < G; ++i) {
    if (P[i] < 0 || P[i] > FEDAVG_MAX_PEERS) {
      g_err = "rmesh_fedavg: 0..64 rows per device";
      return 2;
    }
    float* out = static_cast<float*>(bufs[i]);
    hipStream_t s = (hipStream_t)streams[i];
    if (!hip_ok(hipSetDevice(m->devs[i]), "hipSetDevice")) return 1;
    if (P[i] == 0) {  // a device without live rows still takes part: it contributes zero
      if (!hip_ok(hipMemsetAsync(out, 0, (size_t)(n + 1) * sizeof(float), s), "hipMemsetAsync")) return 1;
    } else {
      FedAvgWeights fw{};
      double sum = 0.0;
      for (int p = 0; p < P[i]; ++p) {
        fw.w[p] = w[off + p];
        sum += w[off + p];
      }
      fw.wsum = (float)sum;
      fl_fedavg_reduce(out, out + n, static_cast<const float*>(params[i]), P[i], n, ld[i], fw, s);
      if (!hip_ok(hipGetLastError(), "fl_fedavg_reduce")) return 1;
    }
    off += P[i];
  }
  if (!nccl_ok(ncclGroupStart(), "ncclGroupStart")) return 1;
  bool ok = true;
  for (int i = 0; i < G && ok; ++i)
    ok = nccl_ok(ncclAllReduce(bufs[i], outs ? outs[i] : bufs[i], (size_t)(n + 1), ncclFloat32, ncclSum, m->comms[i], (hipStream_t)streams[i]),
                 "ncclAllReduce");
  if (!group_end(ok)) return 1;
  return fedavg_apply_all(m, params, outs ? outs : bufs, P, n, ld, mask, streams);
}

// Second half of a FedAvg whose all-reduce failed: the retained partial sums bufs[i] (from
// rmesh_fedavg with outs) are all-reduced again over the CURRENT (rebuilt) mesh into outs[i] and
// applied to the rows in mask. Arrays are indexed by the current mesh ranks.
int rmesh_fedavg_retry(void* h, void** params, void** bufs, void** outs, const int* P, int64_t n, const int64_t* ld, const float* mask, void** streams) {
  auto* m = static_cast<Mesh*>(h);
  if (!usable(m)) return 1;
  const int G = (int)m->devs.size();
  DeviceGuard g;
  if (!nccl_ok(ncclGroupStart(), "ncclGroupStart")) return 1;
  bool ok = true;
  for (int i = 0; i < G && ok; ++i)
    ok = nccl_ok(ncclAllReduce(bufs[i], outs[i], (size_t)(n + 1), ncclFloat32, ncclSum, m->comms[i], (hipStream_t)streams[i]), "ncclAllReduce");
  if (!group_end(ok)) return 1;
  return fedavg_apply_all(m, params, outs, P, n, ld, mask, streams);
}

// Bucketed, overlapped FedAvg: the weight exchange runs on a side stream of
// every device. Buffers use the layout [Σw, pad x3 | Σ w x (n floats)] (n + 4 floats, the data
// float4-aligned); keep[i] receives device i's local partial sums and is never overwritten by the
// all-reduce (out of place into outs[i]), so a failed exchange can be re-run from it.
//
//   per device: event on the compute stream (the rows are final) -> the comm stream waits on it ->
//   the weighted partial sums of every bucket on the comm stream;
//   per bucket k: ONE grouped all-reduce over the mesh (bucket 0 also carries Σw), then an event
//   per device on its comm stream;
//   apply = 1: per device the compute stream waits on bucket k's event and applies bucket k, so
//   bucket k's apply overlaps bucket k + 1's all-reduce and the compute stream never waits on the
//   exchange as a whole; apply = 0 (delayed averaging): nothing is applied and the compute stream
//   does not wait — the next local epoch runs beside the exchange (rmesh_delayed_land lands it).
// Per device rows params[i] ([P_i][ld_i] fp32), weights w / mask as in rmesh_fedavg. A device with
// P_i = 0 contributes zeros.
int rmesh_fedavg_bucketed(void* h, void** params, void** keep, void** outs, const int* P, int64_t n, const int64_t* ld, const float* w,
                          const float* mask, void** streams, void** comm_streams, int64_t bucket, int apply) {
  auto* m = static_cast<Mesh*>(h);
  if (!usable(m)) return 1;
  const int G = (int)m->devs.size();
  const int64_t step = bucket_step(bucket);
  const int nb = n > 0 ? (int)((n + step - 1) / step) : 1;
  DeviceGuard g;
  int off = 0;
  for (int i = 0; i < G; ++i) {
    if (P[i] < 0 || P[i] > FEDAVG_MAX_PEERS) {
      g_err = "rmesh_fedavg_bucketed: 0..64 rows per device";
      return 2;
    }
    if (!hip_ok(hipSetDevice(m->devs[i]), "hipSetDevice")) return 1;
    DevEvents* e = events_for(m, m->devs[i], nb);
    if (e == nullptr) return 1;
    hipStream_t cs = (hipStream_t)comm_streams[i];
    if (!hip_ok(hipEventRecord(e->ready, (hipStream_t)streams[i]), "hipEventRecord") || !hip_ok(hipStreamWaitEvent(cs, e->ready, 0), "hipStreamWaitEvent"))
      return 1;
    float* kb = static_cast<float*>(keep[i]);
    if (P[i] == 0) {
      if (!hip_ok(hipMemsetAsync(kb, 0, (size_t)(n + 4) * sizeof(float), cs), "hipMemsetAsync")) return 1;
    } else {
      FedAvgWeights fw{};
      double sum = 0.0;
      for (int p = 0; p < P[i]; ++p) {
        fw.w[p] = w[off + p];
        sum += w[off + p];
      }
      fw.wsum = (float)sum;
      const float* src = static_cast<const float*>(params[i]);
      for (int k = 0; k < nb; ++k) {
        const int64_t b0 = k * step, b1 = b0 + step < n ? b0 + step : n;
        fl_fedavg_reduce(kb + 4 + b0, k == 0 ? kb : nullptr, src + b0, P[i], b1 - b0, ld[i], fw, cs);
      }
      if (!hip_ok(hipGetLastError(), "fl_fedavg_reduce")) return 1;
    }
    off += P[i];
  }
  for (int k = 0; k < nb; ++k) {
    const int64_t b0 = k * step, b1 = b0 + step < n ? b0 + step : n;
    const int64_t lo = k == 0 ? 0 : 4 + b0, hi = 4 + b1;
    if (!nccl_ok(ncclGroupStart(), "ncclGroupStart")) return 1;
    bool ok = true;
    for (int i = 0; i < G && ok; ++i)
      ok = nccl_ok(ncclAllReduce(static_cast<float*>(keep[i]) + lo, static_cast<float*>(outs[i]) + lo, (size_t)(hi - lo), ncclFloat32, ncclSum, m->comms[i],
                                 (hipStream_t)comm_streams[i]),
                   "ncclAllReduce");
    if (!group_end(ok)) return 1;
    for (int i = 0; i < G; ++i) {
      if (!hip_ok(hipSetDevice(m->devs[i]), "hipSetDevice")) return 1;
      if (!hip_ok(hipEventRecord(m->ev[m->devs[i]].bucket[k], (hipStream_t)comm_streams[i]), "hipEventRecord")) return 1;
    }
  }
  m->last_nb = nb;
  if (!apply) return 0;
  off = 0;
  for (int i = 0; i < G; ++i) {
    const unsigned long long bits = P[i] > 0 ? mask_bits(mask, off, P[i]) : 0ull;
    off += P[i];
    if (!bits) continue;
    if (!hip_ok(hipSetDevice(m->devs[i]), "hipSetDevice")) return 1;
    hipStream_t s = (hipStream_t)streams[i];
    const float* ob = static_cast<const float*>(outs[i]);
    float* dst = static_cast<float*>(params[i]);
    for (int k = 0; k < nb; ++k) {
      const int64_t b0 = k * step, b1 = b0 + step < n ? b0 + step : n;
      if (!hip_ok(hipStreamWaitEvent(s, m->ev[m->devs[i]].bucket[k], 0), "hipStreamWaitEvent")) return 1;
      fl_fedavg_apply(dst + b0, ob + 4 + b0, ob, P[i], b1 - b0, ld[i], bits, s);
    }
    if (!hip_ok(hipGetLastError(), "fl_fedavg_apply")) return 1;
  }
  return 0;
}

// Delayed averaging on the mesh: per device the compute stream waits on the last bucketed
// exchange (if have_avg) and, for every masked row, lands it as x += avg / Σw - snap and takes the
// new snapshot snap = x (one pass); without have_avg it only snapshots. snaps[i] is [P_i][ld_snap].
int rmesh_delayed_land(void* h, void** params, void** snaps, void** outs, const int* P, int64_t n, const int64_t* ld, int64_t ld_snap, const float* mask,
                       void** streams, int have_avg) {
  auto* m = static_cast<Mesh*>(h);
  if (!usable(m)) return 1;
  const int G = (int)m->devs.size();
  DeviceGuard g;
  int off = 0;
  for (int i = 0; i < G; ++i) {
    const unsigned long long bits = P[i] > 0 ? mask_bits(mask, off, P[i]) : 0ull;
    off += P[i];
    if (!bits) continue;
    if (!hip_ok(hipSetDevice(m->devs[i]), "hipSetDevice")) return 1;
    hipStream_t s = (hipStream_t)streams[i];
    const float* ob = static_cast<const float*>(outs[i]);
    if (have_avg) {
      auto it = m->ev.find(m->devs[i]);
      if (it == m->ev.end() || m->last_nb < 1) {
        g_err = "rmesh_delayed_land: no bucketed exchange pending on device " + std::to_string(m->devs[i]);
        return 2;
      }
      if (!hip_ok(hipStreamWaitEvent(s, it->second.bucket[m->last_nb - 1], 0), "hipStreamWaitEvent")) return 1;
    }
    fl_fedavg_delayed_land(static_cast<float*>(params[i]), static_cast<float*>(snaps[i]), ld_snap, have_avg ? ob + 4 : nullptr, ob, P[i], n, ld[i], bits, s);
    if (!hip_ok(hipGetLastError(), "fl_fedavg_delayed_land")) return 1;
  }
  return 0;
}

// Retry of a bucketed FedAvg after a failure: the retained partial sums keep[i] ([Σw, pad | data])
// are all-reduced again over the CURRENT (rebuilt) mesh into outs[i] on the compute streams and,
// if apply, applied to the masked rows. Arrays are indexed by the current mesh ranks.
int rmesh_fedavg_bucketed_retry(void* h, void** params, void** keep, void** outs, const int* P, int64_t n, const int64_t* ld, const float* mask,
                                void** streams, int apply) {
  auto* m = static_cast<Mesh*>(h);
  if (!usable(m)) return 1;
  const int G = (int)m->devs.size();
  DeviceGuard g;
  if (!nccl_ok(ncclGroupStart(), "ncclGroupStart")) return 1;
  bool ok = true;
  for (int i = 0; i < G && ok; ++i)
    ok = nccl_ok(ncclAllReduce(keep[i], outs[i], (size_t)(n + 4), ncclFloat32, ncclSum, m->comms[i], (hipStream_t)streams[i]), "ncclAllReduce");
  if (!group_end(ok)) return 1;
  if (!apply) return 0;
  int off = 0;
  for (int i = 0; i < G; ++i) {
    const unsigned long long bits = P[i] > 0 ? mask_bits(mask, off, P[i]) : 0ull;
    off += P[i];
    if (!bits) continue;
    if (!hip_ok(hipSetDevice(m->devs[i]), "hipSetDevice")) return 1;
    const float* ob = static_cast<const float*>(outs[i]);
    fl_fedavg_apply(static_cast<float*>(params[i]), ob + 4, ob, P[i], n, ld[i], bits, (hipStream_t)streams[i]);
    if (!hip_ok(hipGetLastError(), "fl_fedavg_apply")) return 1;
  }
  return 0;
}

}  // extern "C"

namespace {
// per device: the apply kernel over the rows in mask (the mean in res[i][0..n), Σw in res[i][n])
int fedavg_apply_all(Mesh* m, void** params, void** res, const int* P, int64_t n, const int64_t* ld, const float* mask, void** streams) {
  const int G = (int)m->devs.size();
  int off = 0;
  for (int i = 0; i < G; ++i) {
    if (P[i] > 0) {
      unsigned long long bits = 0;
      for (int p = 0; p < P[i]; ++p)
        if (mask[off + p] != 0.f) bits |= 1ull << p;
      if (bits) {
        if (!hip_ok(hipSetDevice(m->devs[i]), "hipSetDevice")) return 1;
        const float* out = static_cast<const float*>(res[i]);
        fl_fedavg_apply(static_cast<float*>(params[i]), out, out + n, P[i], n, ld[i], bits, (hipStream_t)streams[i]);
        if (!hip_ok(hipGetLastError(), "fl_fedavg_apply")) return 1;
      }
    }
    off += P[i];
  }
  return 0;
}
}  // namespace

extern "C" {

// 0: every communicator healthy; otherwise the first asynchronous error (message set).
int rmesh_check(void* h) {
  auto* m = static_cast<Mesh*>(h);
  if (!usable(m)) return 1;
  if (m->injected >= 0 && m->injected < (int)m->devs.size()) {
    g_err = "rank " + std::to_string(m->injected) + " (device " + std::to_string(m->devs[m->injected]) + "): injected asynchronous error (rmesh_debug_inject)";
    return 1;
  }
  for (size_t i = 0; i < m->comms.size(); ++i) {
    ncclResult_t e = ncclSuccess;
    if (!nccl_ok(ncclCommGetAsyncError(m->comms[i], &e), "ncclCommGetAsyncError")) return 1;
    if (e != ncclSuccess && e != ncclInProgress) {
      g_err = "rank " + std::to_string(i) + " (device " + std::to_string(m->devs[i]) + "): " + ncclGetErrorString(e);
      return 1;
    }
  }
  return 0;
}

// Abort every communicator (local; never waits for a dead peer; ends kernels stuck in the mesh).
int rmesh_abort(void* h) {
  auto* m = static_cast<Mesh*>(h);
  if (m == nullptr) return 1;
  if (m->aborted) return 0;
  DeviceGuard g;
  int rc = 0;
  for (size_t i = 0; i < m->comms.size(); ++i) {
    if (m->comms[i] == nullptr) continue;
    if (!nccl_ok(ncclCommAbort(m->comms[i]), "ncclCommAbort")) rc = 1;
    m->comms[i] = nullptr;
  }
  m->aborted = true;
  return rc;
}

// Rebuild the mesh over the listed surviving ranks (indices into the current device list): the
// old communicators are aborted, a fresh ncclCommInitAll runs over the survivors' devices, and
// the survivors are renumbered 0..nkeep-1 in the given order.
int rmesh_shrink(void* h, const int* keep, int nkeep) {
  auto* m = static_cast<Mesh*>(h);
  if (m == nullptr || nkeep < 1) {
    g_err = "rmesh_shrink: need a mesh and at least one survivor";
    return 2;
  }
  std::vector<int> devs;
  for (int k = 0; k < nkeep; ++k) {
    if (keep[k] < 0 || keep[k] >= (int)m->devs.size()) {
      g_err = "rmesh_shrink: survivor index out of range";
      return 2;
    }
    devs.push_back(m->devs[keep[k]]);
  }
  if (!m->aborted && rmesh_abort(m) != 0) return 1;
  DeviceGuard g;
  std::vector<ncclComm_t> comms(devs.size(), nullptr);
  if (!nccl_ok(ncclCommInitAll(comms.data(), (int)devs.size(), devs.data()), "ncclCommInitAll")) return 1;
  m->devs = devs;
  m->comms = comms;
  m->aborted = false;
  m->injected = -1;
  return 0;
}

// Rebuild a healthy mesh over the listed ranks. The caller has drained every device of the mesh
// (hipDeviceSynchronize / stream syncs), so no collective is queued: the communicators are
// destroyed (a clean teardown) and a fresh ncclCommInitAll runs over the kept devices. An aborted
// mesh takes rmesh_shrink's path.
int rmesh_rebuild(void* h, const int* keep, int nkeep) {
  auto* m = static_cast<Mesh*>(h);
  if (m == nullptr || nkeep < 1) {
    g_err = "rmesh_rebuild: need a mesh and at least one member";
    return 2;
  }
  if (m->aborted) return rmesh_shrink(h, keep, nkeep);
  std::vector<int> devs;
  for (int k = 0; k < nkeep; ++k) {
    if (keep[k] < 0 || keep[k] >= (int)m->devs.size()) {
      g_err = "rmesh_rebuild: member index out of range";
      return 2;
    }
    devs.push_back(m->devs[keep[k]]);
  }
  DeviceGuard g;
  int rc = 0;
  for (auto& c : m->comms) {
    if (c != nullptr && !nccl_ok(ncclCommDestroy(c), "ncclCommDestroy")) rc = 1;
    c = nullptr;
  }
  m->aborted = true;  // no usable communicator until the init below succeeds
  if (rc != 0) return 1;
  std::vector<ncclComm_t> comms(devs.size(), nullptr);
  if (!nccl_ok(ncclCommInitAll(comms.data(), (int)devs.size(), devs.data()), "ncclCommInitAll")) return 1;
  m->devs = devs;
  m->comms = comms;
  m->aborted = false;
  m->injected = -1;
  return 0;
}

// Fault hook for tests: rmesh_check reports an asynchronous error on mesh rank `rank` until the
// mesh is rebuilt (-1 clears it).
int rmesh_debug_inject(void* h, int rank) {
  auto* m = static_cast<Mesh*>(h);
  if (m == nullptr) return 1;
  m->injected = rank;
  return 0;
}

void rmesh_destroy(void* h) {
  auto* m = static_cast<Mesh*>(h);
  if (m == nullptr) return;
  DeviceGuard g;
  if (!m->aborted)
    for (auto c : m->comms)
      if (c != nullptr) ncclCommDestroy(c);
  for (auto& kv : m->ev) {
    (void)hipSetDevice(kv.first);
    if (kv.second.ready != nullptr) (void)hipEventDestroy(kv.second.ready);
    for (auto e : kv.second.bucket) (void)hipEventDestroy(e);
  }
  delete m;
}

}  // extern "C"
