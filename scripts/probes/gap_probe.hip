// Device-side cost of stream operations between two kernels on one MI355X stream (round-boundary
// cost model for the headline engine). Each pattern is enqueued behind a 2 ms spin kernel, so the
// host is far ahead and every gap is device time. A probe kernel stamps wall_clock64 (100 MHz) at
// its start and end; the gap is next start - previous end.
//
//   hipcc --offload-arch=gfx950 -O2 -o build/gap_probe scripts/probes/gap_probe.hip
//   ./build/gap_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 1;                                                                            \
    }                                                                                      \
  } while (0)

struct Big {  // kernel-argument block of the engine's control upload size (~1.4 KB)
  int4 a[64];
  int b[64];
  unsigned long long c;
  int d[16];
};

__global__ void k_spin(unsigned long long ticks) {
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
}

__global__ void k_probe(unsigned long long* t, int i, unsigned* flag, unsigned v) {
  if (blockIdx.x == 0 && threadIdx.x == 0) t[2 * i] = wall_clock64();
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (flag) __hip_atomic_store(flag, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    t[2 * i + 1] = wall_clock64();
  }
}

__global__ void k_write(unsigned long long* t, int i, float* buf, int n) {
  if (blockIdx.x == 0 && threadIdx.x == 0) t[2 * i] = wall_clock64();
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < n; k += gridDim.x * blockDim.x) buf[k] = (float)k;
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0) t[2 * i + 1] = wall_clock64();
}

__global__ __launch_bounds__(512) void k_fat(unsigned long long* t, int i) {  // retry-launch shape: exits at once
  extern __shared__ char lds[];
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    t[2 * i] = wall_clock64();
    lds[0] = 1;
    t[2 * i + 1] = wall_clock64() + (lds[0] & 0);
  }
}

__global__ void k_probe_big(unsigned long long* t, int i, Big b) {
  if (blockIdx.x == 0 && threadIdx.x == 0) t[2 * i] = wall_clock64() + (b.c & 0);
  __syncthreads();
  if (blockIdx.x == 0 && threadIdx.x == 0) t[2 * i + 1] = wall_clock64();
}

int main() {
  const int R = 60;
  unsigned long long* t;
  CK(hipMalloc(&t, sizeof(unsigned long long) * 2 * (R * 4 + 8)));
  unsigned* flag;
  CK(hipMalloc(&flag, 64));
  CK(hipMemset(flag, 0, 64));
  hipStream_t s, s2;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t ev, ev_old;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  CK(hipEventCreateWithFlags(&ev_old, hipEventDisableTiming));
  CK(hipEventRecord(ev_old, s2));
  CK(hipStreamSynchronize(s2));
  int wv = 0;
  (void)hipDeviceGetAttribute(&wv, hipDeviceAttributeCanUseStreamWaitValue, 0);
  printf("stream wait value supported: %d\n", wv);

  // a graph of one probe kernel (its stamp index is fixed: slot 2R+4)
  hipGraph_t g;
  hipGraphExec_t gx;
  CK(hipStreamBeginCapture(s2, hipStreamCaptureModeRelaxed));
  hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, s2, t, 2 * R + 4, (unsigned*)nullptr, 0u);
  CK(hipStreamEndCapture(s2, &g));
  CK(hipGraphInstantiate(&gx, g, nullptr, nullptr, 0));

  const char* names[] = {"back-to-back",
                         "event record (no waiter)",
                         "event record + other stream waits on it",
                         "wait on a completed event of another stream",
                         "big kernel arguments (1.4 KB) for the 2nd kernel",
                         "256-workgroup 2nd kernel",
                         "graph launch of one kernel between",
                         "other stream waits on a value the kernel wrote (hipStreamWaitValue32)",
                         "memset 64 B between",
                         "1st kernel writes 8 MB",
                         "2nd kernel: 192 x 512-thread workgroups, 96 KB LDS (retry shape)"};
  const int NP = 11;
  float* wbuf;
  CK(hipMalloc(&wbuf, 8 << 20));
  CK(hipFuncSetAttribute((const void*)k_fat, hipFuncAttributeMaxDynamicSharedMemorySize, 96 << 10));
  for (int pat = 0; pat < NP; ++pat) {
    if (pat == 7 && !wv) continue;
    CK(hipMemset(flag, 0, 64));
    hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, s, 200000ull);  // 2 ms
    Big big{};
    for (int r = 0; r < R; ++r) {
      const int i0 = 2 * r, i1 = 2 * r + 1;
      if (pat == 9)
        hipLaunchKernelGGL(k_write, dim3(256), dim3(256), 0, s, t, i0, wbuf, (8 << 20) / 4);
      else
        hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, s, t, i0, pat == 7 ? flag : (unsigned*)nullptr, (unsigned)(r + 1));
      switch (pat) {
        case 1: CK(hipEventRecord(ev, s)); break;
        case 2: CK(hipEventRecord(ev, s)); CK(hipStreamWaitEvent(s2, ev, 0)); break;
        case 3: CK(hipStreamWaitEvent(s, ev_old, 0)); break;
        case 6: CK(hipGraphLaunch(gx, s)); break;
        case 7: CK(hipStreamWaitValue32(s2, flag, (unsigned)(r + 1), hipStreamWaitValueGte, 0xffffffffu)); break;
        case 8: CK(hipMemsetAsync(flag + 8, 0, 64 - 32, s)); break;
        default: break;
      }
      if (pat == 4)
        hipLaunchKernelGGL(k_probe_big, dim3(1), dim3(64), 0, s, t, i1, big);
      else if (pat == 10)
        hipLaunchKernelGGL(k_fat, dim3(192), dim3(512), 96 << 10, s, t, i1);
      else
        hipLaunchKernelGGL(k_probe, dim3(pat == 5 ? 256 : 1), dim3(64), 0, s, t, i1, (unsigned*)nullptr, 0u);
    }
    CK(hipStreamSynchronize(s));
    CK(hipStreamSynchronize(s2));
    std::vector<unsigned long long> h(2 * (R * 4 + 8));
    CK(hipMemcpy(h.data(), t, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost));
    std::vector<double> gap, next, dur;
    for (int r = 1; r < R; ++r) {
      const int i0 = 2 * r, i1 = 2 * r + 1;
      gap.push_back((h[2 * i1] - h[2 * i0 + 1]) * 0.01);      // end of 1st -> start of 2nd (us)
      dur.push_back((h[2 * i1 + 1] - h[2 * i1]) * 0.01);
      next.push_back((h[2 * (i0 + 2)] - h[2 * i1 + 1]) * 0.01);  // end of 2nd -> start of the next pair
    }
    auto med = [](std::vector<double> v) {
      std::sort(v.begin(), v.end());
      return v[v.size() / 2];
    };
    printf("%-72s gap %6.2f us   (2nd kernel %5.2f us, then -> next pair %6.2f us)\n", names[pat], med(gap), med(dur), med(next));
  }
  CK(hipGraphExecDestroy(gx));
  CK(hipGraphDestroy(g));
  return 0;
}
