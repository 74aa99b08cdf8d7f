// Node-local control-plane collectives over POSIX shared memory.
//
// The collective workflow exchanges a few hundred bytes per round between ranks (train-set votes,
// live-peer lists).  The reference does this with TTL-relayed gRPC broadcasts
// (p2pfl/stages/base_node/vote_train_set_stage.py:101-107 + grpc_server.py:211-215); a gloo
// all_gather_object costs two TCP collectives plus pickling (~1-5 ms for 8 ranks), which is the
// same order as a whole MLP round on MI355X.  All ranks of a single-node job share one mapping:
//
//   [Header 256 B][RankCtl x world (128 B each)][data: world x 2 parity slots x slot_bytes]
//
// allgather(gen): write own payload into parity slot (gen & 1), publish `arrived = gen` with a
// release store, spin (pause -> yield) until every rank published >= gen, then copy all slots out.
// Two parity slots suffice: a rank can only write generation g+2 into parity (g & 1) after every
// rank arrived at g+1, i.e. after every rank finished reading generation g.
//
// Payloads larger than the slot publish an overflow marker; every rank then sees the overflow and
// the caller falls back to the gloo path collectively (no rank can diverge).
//
// Membership (fault tolerance). Each rank's `status` word is either the last generation it
// published or kGone | g, "gone from generation g on" (it published g - 1 and never joins g or
// later). Both transitions are compare-and-swaps on that one word, so a rank that is evicted can
// no longer publish, and every survivor computes the same participant set for a generation:
// r participates in g  <=>  status_r >= g (not gone)  or  status_r == kGone | h with h > g.
// A rank leaves on purpose (shmc_leave: its last local peer died, or the job ends) or is evicted
// by a waiter once its heartbeat (shmc_heartbeat, CLOCK_MONOTONIC ns) is older than `fail_s`.
// This replaces the reference's heartbeat eviction + "aggregate whatever arrived"
// (p2pfl/communication/protocols/heartbeater.py:94-103, learning/aggregators/aggregator.py:190-208)
// for the collective weights plane: the caller rebuilds its process groups over the survivors.
//
// Plain C ABI (ctypes), host-only: no GPU state is touched.
#include <atomic>
#include <cerrno>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <fcntl.h>
#include <sched.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

namespace {

constexpr uint64_t kMagic = 0x6d79667970736d63ull;  // "myfypsmc"
constexpr uint64_t kOverflow = ~0ull;
constexpr uint64_t kGone = 1ull << 63;
constexpr uint64_t kLeft = 1ull << 62;  // with kGone: the rank left on purpose (shmc_leave), not evicted
constexpr uint64_t kGenMask = kLeft - 1;

struct Header {
  std::atomic<uint64_t> magic;
  int32_t world;
  int32_t pad;
  uint64_t slot_bytes;
  std::atomic<int32_t> attached;
  char reserved[256 - 32];
};
static_assert(sizeof(Header) == 256, "header layout");

struct alignas(128) RankCtl {
  std::atomic<uint64_t> status;   // last published generation, or kGone | first generation not joined
  uint64_t len[2];                // payload length per parity slot (kOverflow = too large)
  std::atomic<uint64_t> beat_ns;  // heartbeat, CLOCK_MONOTONIC ns (0 = no heartbeat thread)
  std::atomic<int32_t> pid;       // the rank's process (single host): a vanished pid is a crash
};
static_assert(sizeof(RankCtl) == 128, "rank ctl layout");

struct Handle {
  void* base;
  size_t bytes;
  int rank;
  int world;
  uint64_t slot_bytes;
  uint64_t gen;
  bool owns_map = true;  // false for shmc_view handles (same mapping, another rank)
  Header* hdr() const { return reinterpret_cast<Header*>(base); }
  RankCtl* ctl(int r) const { return reinterpret_cast<RankCtl*>(static_cast<char*>(base) + sizeof(Header)) + r; }
  char* slot(int r, int parity) const {
    char* d = static_cast<char*>(base) + sizeof(Header) + sizeof(RankCtl) * world;
    return d + (static_cast<size_t>(r) * 2 + parity) * slot_bytes;
  }
};

size_t total_bytes(int world, uint64_t slot_bytes) {
  return sizeof(Header) + sizeof(RankCtl) * world + static_cast<size_t>(world) * 2 * slot_bytes;
}

double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}
uint64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return static_cast<uint64_t>(ts.tv_sec) * 1000000000ull + static_cast<uint64_t>(ts.tv_nsec);
}

// 1: r took part in generation gen; 0: r never will (gone before it); -1: not decided yet
int joined(uint64_t s, uint64_t gen) {
  if (s & kGone) return (s & kGenMask) > gen ? 1 : 0;
  return s >= gen ? 1 : -1;
}

// The rank's process no longer exists (killed / crashed): no need to wait for its heartbeat to go
// stale. All ranks of a job share the host (and the pid namespace) by construction of the segment.
bool process_gone(const RankCtl* c) {
  const int32_t pid = c->pid.load(std::memory_order_acquire);
  if (pid <= 0) return false;
  if (kill(pid, 0) != 0) return errno == ESRCH;
  // exited but not yet reaped by its launcher (torchrun polls its workers): a zombie
  char path[64], buf[256];
  snprintf(path, sizeof(path), "/proc/%d/stat", pid);
  const int fd = open(path, O_RDONLY);
  if (fd < 0) return false;
  const ssize_t n = read(fd, buf, sizeof(buf) - 1);
  close(fd);
  if (n <= 0) return false;
  buf[n] = 0;
  const char* rp = strrchr(buf, ')');
  return rp && rp[1] == ' ' && (rp[2] == 'Z' || rp[2] == 'X');
}

// r is still a member but unresponsive: its process is gone, or its heartbeat is older than fail_ns
bool unresponsive(const RankCtl* c, uint64_t fail_ns) {
  if (process_gone(c)) return true;
  if (!fail_ns) return false;
  const uint64_t beat = c->beat_ns.load(std::memory_order_acquire);
  return beat && now_ns() - beat > fail_ns;
}

inline void cpu_relax() {
#if defined(__x86_64__)
  __builtin_ia32_pause();
#endif
}

// spin briefly, then yield; returns false on timeout
template <class Pred>
bool wait_until(Pred ready, double timeout_s) {
  for (int i = 0; i < 4096; ++i) {
    if (ready()) return true;
    cpu_relax();
  }
  const double t0 = now_s();
  for (uint64_t i = 0;; ++i) {
    if (ready()) return true;
    sched_yield();
    if ((i & 255) == 0 && timeout_s > 0 && now_s() - t0 > timeout_s) return ready();
  }
}

}  // namespace

extern "C" {

int shmc_version() { return 1; }

// Rank 0 creates (`create`=1) the segment, the others attach. Returns nullptr on failure (errno set).
void* shmc_open(const char* name, int rank, int world, uint64_t slot_bytes, int create, double timeout_s) {
  if (world < 1 || world > 64 || rank < 0 || rank >= world || slot_bytes < 64) {
    errno = EINVAL;
    return nullptr;
  }
  slot_bytes = (slot_bytes + 127) & ~uint64_t(127);
  const size_t bytes = total_bytes(world, slot_bytes);
  int fd = -1;
  if (create) {
    fd = shm_open(name, O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) return nullptr;
    if (ftruncate(fd, static_cast<off_t>(bytes)) != 0) {
      close(fd);
      shm_unlink(name);
      return nullptr;
    }
  } else {
    const double t0 = now_s();
    for (;;) {
      fd = shm_open(name, O_RDWR, 0600);
      if (fd >= 0) {
        struct stat st;
        if (fstat(fd, &st) == 0 && static_cast<size_t>(st.st_size) >= bytes) break;
        close(fd);
        fd = -1;
      }
      if (now_s() - t0 > timeout_s) {
        errno = ETIMEDOUT;
        return nullptr;
      }
      usleep(1000);
    }
  }
  void* base = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (base == MAP_FAILED) return nullptr;
  Handle* h = new Handle{base, bytes, rank, world, slot_bytes, 0, true};
  Header* hd = h->hdr();
  if (create) {
    std::memset(base, 0, sizeof(Header) + sizeof(RankCtl) * world);
    hd->world = world;
    hd->slot_bytes = slot_bytes;
    hd->magic.store(kMagic, std::memory_order_release);
  } else {
    if (!wait_until([&] { return hd->magic.load(std::memory_order_acquire) == kMagic; }, timeout_s) || hd->world != world ||
        hd->slot_bytes != slot_bytes) {
      munmap(base, bytes);
      delete h;
      errno = EPROTO;
      return nullptr;
    }
  }
  h->ctl(rank)->pid.store(static_cast<int32_t>(getpid()), std::memory_order_release);
  hd->attached.fetch_add(1, std::memory_order_acq_rel);
  return h;
}

// Block until all `world` ranks attached (then the creator may unlink the name). 0 ok, -1 timeout.
int shmc_wait_attached(void* handle, double timeout_s) {
  Handle* h = static_cast<Handle*>(handle);
  return wait_until([&] { return h->hdr()->attached.load(std::memory_order_acquire) >= h->world; }, timeout_s) ? 0 : -1;
}

int shmc_unlink(const char* name) { return shm_unlink(name); }

uint64_t shmc_slot_bytes(void* handle) { return static_cast<Handle*>(handle)->slot_bytes; }

// Membership-aware all-gather of variable-length byte payloads. `out` has room for
// world * slot_bytes; rank r's payload lands at out + r * slot_bytes with its length in lens[r]
// (0 for a rank that did not take part). *members gets the participant bitmask (world <= 64).
// A rank that has not arrived is evicted once its heartbeat is older than fail_s (fail_s <= 0:
// never). Returns 0 ok, 1 if some participant's payload overflowed its slot (all participants
// return 1 for the same generation), -1 timeout, -3 this rank was evicted (or left) already.
int shmc_allgather_m(void* handle, const void* in, uint64_t n, void* out, uint64_t* lens, uint64_t* members, double timeout_s,
                     double fail_s) {
  Handle* h = static_cast<Handle*>(handle);
  const uint64_t gen = ++h->gen;
  const int par = static_cast<int>(gen & 1);
  RankCtl* me = h->ctl(h->rank);
  if (in != nullptr && n <= h->slot_bytes) {
    std::memcpy(h->slot(h->rank, par), in, n);
    me->len[par] = n;
  } else {
    me->len[par] = in == nullptr ? 0 : kOverflow;
  }
  uint64_t expect = gen - 1;
  if (!me->status.compare_exchange_strong(expect, gen, std::memory_order_acq_rel, std::memory_order_acquire)) return -3;
  int rc = 0;
  uint64_t mask = 0;
  const uint64_t fail_ns = fail_s > 0 ? static_cast<uint64_t>(fail_s * 1e9) : 0;
  for (int r = 0; r < h->world; ++r) {
    RankCtl* c = h->ctl(r);
    int j = -1;
    const double t0 = now_s();
    bool ok = wait_until(
        [&] {
          uint64_t s = c->status.load(std::memory_order_acquire);
          j = joined(s, gen);
          if (j >= 0) return true;
          if (fail_ns) {  // evict a crashed rank: process gone, or heartbeat stale
            const uint64_t beat = c->beat_ns.load(std::memory_order_acquire);
            const bool stale = process_gone(c) || (beat ? now_ns() - beat > fail_ns : now_s() - t0 > fail_s);
            if (stale && c->status.compare_exchange_strong(s, kGone | gen, std::memory_order_acq_rel, std::memory_order_acquire)) {
              j = 0;
              return true;
            }
          }
          return false;
        },
        timeout_s);
    if (!ok) return -1;
    if (j == 0) {
      if (lens) lens[r] = 0;
      continue;
    }
    mask |= 1ull << r;
    const uint64_t len = c->len[par];
    if (len == kOverflow) {
      rc = 1;
      if (lens) lens[r] = 0;
      continue;
    }
    if (lens) lens[r] = len;
    if (out != nullptr && len) std::memcpy(static_cast<char*>(out) + static_cast<size_t>(r) * h->slot_bytes, h->slot(r, par), len);
  }
  if (members) *members = mask;
  return rc;
}

// Diagnostics: out[0] = this handle's generation, out[1 + r] = rank r's status word.
int shmc_state(void* handle, uint64_t* out) {
  Handle* h = static_cast<Handle*>(handle);
  out[0] = h->gen;
  for (int r = 0; r < h->world; ++r) out[1 + r] = h->ctl(r)->status.load(std::memory_order_acquire);
  return h->world;
}

// All-gather over every rank (no eviction). Returns 0 / 1 (overflow) / -1 (timeout or a rank left).
int shmc_allgather(void* handle, const void* in, uint64_t n, void* out, uint64_t* lens, double timeout_s) {
  Handle* h = static_cast<Handle*>(handle);
  uint64_t mask = 0;
  const int rc = shmc_allgather_m(handle, in, n, out, lens, &mask, timeout_s, 0.0);
  if (rc < 0) return -1;
  const uint64_t all = h->world >= 64 ? ~0ull : ((1ull << h->world) - 1);
  return mask == all ? rc : -1;
}

// Barrier = all-gather of nothing (over the current participants).
int shmc_barrier(void* handle, double timeout_s) {
  Handle* h = static_cast<Handle*>(handle);
  uint64_t mask = 0;
  const int rc = shmc_allgather_m(handle, nullptr, 0, nullptr, nullptr, &mask, timeout_s, 0.0);
  (void)h;
  return rc < 0 ? -1 : 0;
}

// This rank leaves: it never joins a later generation. 0 ok, 1 already gone. The kLeft bit tells
// the others it left on purpose (after completing every collective it had joined), as opposed to
// an eviction of an unresponsive rank (shmc_left_clean).
// shmc_leave_ex(clean = 0): leave WITHOUT the kLeft bit — a rank that could not confirm every
// collective it joined (timeout, error) must look like an eviction, so the survivors recover.
int shmc_leave_ex(void* handle, int clean) {
  Handle* h = static_cast<Handle*>(handle);
  RankCtl* me = h->ctl(h->rank);
  const uint64_t bits = kGone | (clean ? kLeft : 0);
  uint64_t s = me->status.load(std::memory_order_acquire);
  while (!(s & kGone)) {
    if (me->status.compare_exchange_weak(s, bits | ((s + 1) & kGenMask), std::memory_order_acq_rel, std::memory_order_acquire)) return 0;
  }
  return 1;
}
int shmc_leave(void* handle) { return shmc_leave_ex(handle, 1); }

// Bitmask of the ranks that left on purpose (shmc_leave), not by eviction.
uint64_t shmc_left_clean(void* handle) {
  Handle* h = static_cast<Handle*>(handle);
  uint64_t mask = 0;
  for (int r = 0; r < h->world; ++r) {
    const uint64_t s = h->ctl(r)->status.load(std::memory_order_acquire);
    if ((s & kGone) && (s & kLeft)) mask |= 1ull << r;
  }
  return mask;
}

void shmc_heartbeat(void* handle) {
  Handle* h = static_cast<Handle*>(handle);
  h->ctl(h->rank)->beat_ns.store(now_ns(), std::memory_order_release);
}

// Bitmask of the ranks that have not left (and were not evicted).
uint64_t shmc_alive(void* handle) {
  Handle* h = static_cast<Handle*>(handle);
  uint64_t mask = 0;
  for (int r = 0; r < h->world; ++r)
    if (!(h->ctl(r)->status.load(std::memory_order_acquire) & kGone)) mask |= 1ull << r;
  return mask;
}

// Bitmask of the member ranks that are unresponsive right now (process gone, or heartbeat older
// than fail_s; fail_s <= 0: process check only). Read-only: the collective watchdog uses it to
// abort an in-flight weight collective; eviction itself stays with the all-gathers.
uint64_t shmc_unresponsive(void* handle, double fail_s) {
  Handle* h = static_cast<Handle*>(handle);
  const uint64_t fail_ns = fail_s > 0 ? static_cast<uint64_t>(fail_s * 1e9) : 0;
  uint64_t mask = 0;
  for (int r = 0; r < h->world; ++r) {
    const RankCtl* c = h->ctl(r);
    if (r == h->rank || (c->status.load(std::memory_order_acquire) & kGone)) continue;
    if (unresponsive(c, fail_ns)) mask |= 1ull << r;
  }
  return mask;
}

// Wait until every rank left (job end: keeps the rendezvous host alive until the last rank is
// done). A rank that crashed after its last gather never leaves by itself: it is evicted once it
// is unresponsive (process gone, or heartbeat older than fail_s). 0 ok, -1 timeout.
int shmc_wait_all_gone(void* handle, double timeout_s, double fail_s) {
  Handle* h = static_cast<Handle*>(handle);
  const uint64_t fail_ns = fail_s > 0 ? static_cast<uint64_t>(fail_s * 1e9) : 0;
  return wait_until(
             [&] {
               for (int r = 0; r < h->world; ++r) {
                 RankCtl* c = h->ctl(r);
                 uint64_t s = c->status.load(std::memory_order_acquire);
                 if (!(s & kGone) && unresponsive(c, fail_ns)) c->status.compare_exchange_strong(s, kGone | (s + 1), std::memory_order_acq_rel);
               }
               return shmc_alive(handle) == 0;
             },
             timeout_s)
             ? 0
             : -1;
}

// A second rank's handle onto the SAME mapping as `handle` (threads as ranks inside one process:
// the ThreadSanitizer driver csrc/host/tests/shm_collective_tsan.cpp uses it so that every rank's
// accesses hit the same addresses and the publish/acquire protocol is checked, not just run).
void* shmc_view(void* handle, int rank) {
  Handle* h = static_cast<Handle*>(handle);
  if (!h || rank < 0 || rank >= h->world) {
    errno = EINVAL;
    return nullptr;
  }
  Handle* v = new Handle{h->base, h->bytes, rank, h->world, h->slot_bytes, 0, false};
  v->hdr()->attached.fetch_add(1, std::memory_order_acq_rel);
  return v;
}

void shmc_close(void* handle) {
  Handle* h = static_cast<Handle*>(handle);
  if (!h) return;
  if (h->owns_map) munmap(h->base, h->bytes);
  delete h;
}

}  // extern "C"
