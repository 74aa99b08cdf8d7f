// Sanitizer driver for the shared-memory control-plane collectives (csrc/host/shm_collective.cpp).
//
// Ranks are threads of this process that share ONE mapping (shmc_view), so ThreadSanitizer sees
// every rank's payload writes, length words and `arrived` publications on the same addresses and
// checks the two-parity-slot protocol's happens-before edges — not only that it returns the right
// bytes. Built and run by myfyp_amd/ops/build.py::build_sanitized ("thread" and
// "address,undefined"), tests/test_sanitizers.py. Exit 0 and "OK" on success.
//
//   shm_collective_stress <world> <iterations>
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include <unistd.h>

extern "C" {
void* shmc_open(const char* name, int rank, int world, uint64_t slot_bytes, int create, double timeout_s);
void* shmc_view(void* handle, int rank);
int shmc_wait_attached(void* handle, double timeout_s);
int shmc_unlink(const char* name);
uint64_t shmc_slot_bytes(void* handle);
int shmc_allgather(void* handle, const void* in, uint64_t n, void* out, uint64_t* lens, double timeout_s);
int shmc_barrier(void* handle, double timeout_s);
int shmc_allgather_m(void* handle, const void* in, uint64_t n, void* out, uint64_t* lens, uint64_t* members, double timeout_s, double fail_s);
int shmc_leave(void* handle);
uint64_t shmc_alive(void* handle);
int shmc_wait_all_gone(void* handle, double timeout_s, double fail_s);
void shmc_close(void* handle);
}

namespace {

// payload of rank r at iteration i: length and bytes are a function of (r, i); every 97th
// iteration rank (i % world) overflows its slot, which every rank must see as rc = 1
uint64_t payload_len(int r, int i, uint64_t slot) { return (static_cast<uint64_t>(r) * 131 + static_cast<uint64_t>(i) * 17) % (slot + 1); }
unsigned char payload_byte(int r, int i, uint64_t k) { return static_cast<unsigned char>((r * 37 + i * 11 + k * 7) & 0xff); }

}  // namespace

int main(int argc, char** argv) {
  const int world = argc > 1 ? std::atoi(argv[1]) : 4;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 2000;
  const std::string name = "/myfyp_stress_" + std::to_string(getpid());
  void* root = shmc_open(name.c_str(), 0, world, 256, 1, 10.0);
  if (!root) {
    std::perror("shmc_open");
    return 2;
  }
  const uint64_t slot = shmc_slot_bytes(root);
  std::vector<void*> views(world, nullptr);
  views[0] = root;
  for (int r = 1; r < world; ++r) views[r] = shmc_view(root, r);
  if (shmc_wait_attached(root, 10.0) != 0) return 3;
  shmc_unlink(name.c_str());

  std::atomic<int> errors{0};
  auto rank_main = [&](int r) {
    void* h = views[r];
    std::vector<unsigned char> in(slot + 64), out(static_cast<size_t>(world) * slot);
    std::vector<uint64_t> lens(world);
    for (int i = 0; i < iters; ++i) {
      const bool overflow = i % 97 == 0 && r == i % world;
      const uint64_t n = overflow ? slot + 1 : payload_len(r, i, slot);
      for (uint64_t k = 0; k < n; ++k) in[k] = payload_byte(r, i, k);
      const int rc = shmc_allgather(h, in.data(), n, out.data(), lens.data(), 30.0);
      const bool any_overflow = i % 97 == 0;
      if (rc != (any_overflow ? 1 : 0)) {
        errors.fetch_add(1);
        continue;
      }
      for (int q = 0; q < world; ++q) {
        if (any_overflow && q == i % world) continue;
        const uint64_t m = payload_len(q, i, slot);
        if (lens[q] != m) {
          errors.fetch_add(1);
          break;
        }
        for (uint64_t k = 0; k < m; ++k)
          if (out[static_cast<size_t>(q) * slot + k] != payload_byte(q, i, k)) {
            errors.fetch_add(1);
            break;
          }
      }
      if (i % 50 == 0 && shmc_barrier(h, 30.0) != 0) errors.fetch_add(1);
    }
  };
  std::vector<std::thread> threads;
  for (int r = 0; r < world; ++r) threads.emplace_back(rank_main, r);
  for (auto& t : threads) t.join();

  // membership phase: the last rank leaves after `leave_at` rounds; every survivor must see it in
  // the participant mask until then and never after, with the same payloads; finally every rank
  // leaves and waits for the others (the job-end protocol of Federation.shutdown)
  const int rounds = 200, leave_at = 37;
  const uint64_t all = (world >= 64) ? ~0ull : ((1ull << world) - 1), survivors = all & ~(1ull << (world - 1));
  auto member_main = [&](int r) {
    void* h = views[r];
    std::vector<unsigned char> in(slot), out(static_cast<size_t>(world) * slot);
    std::vector<uint64_t> lens(world);
    for (int i = 0; i < rounds; ++i) {
      if (r == world - 1 && i == leave_at) {
        if (shmc_leave(h) != 0) errors.fetch_add(1);
        break;
      }
      const uint64_t n = payload_len(r, i, slot - 1);
      for (uint64_t k = 0; k < n; ++k) in[k] = payload_byte(r, i, k);
      uint64_t mask = 0;
      if (shmc_allgather_m(h, in.data(), n, out.data(), lens.data(), &mask, 30.0, 0.0) != 0) {
        errors.fetch_add(1);
        continue;
      }
      if (mask != (i < leave_at ? all : survivors)) errors.fetch_add(1);
      for (int q = 0; q < world; ++q) {
        if (!(mask >> q & 1)) continue;
        const uint64_t m = payload_len(q, i, slot - 1);
        if (lens[q] != m || (m && out[static_cast<size_t>(q) * slot + m - 1] != payload_byte(q, i, m - 1))) errors.fetch_add(1);
      }
    }
    shmc_leave(h);
    if (shmc_wait_all_gone(h, 30.0, 0.0) != 0 || shmc_alive(h) != 0) errors.fetch_add(1);
  };
  threads.clear();
  for (int r = 0; r < world; ++r) threads.emplace_back(member_main, r);
  for (auto& t : threads) t.join();
  for (int r = world - 1; r >= 0; --r) shmc_close(views[r]);  // views first, the owner unmaps last
  if (errors.load() != 0) {
    std::printf("FAILED errors=%d\n", errors.load());
    return 1;
  }
  std::printf("OK world=%d iters=%d slot=%llu\n", world, iters, static_cast<unsigned long long>(slot));
  return 0;
}
