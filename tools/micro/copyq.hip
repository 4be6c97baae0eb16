// Latency of the run's small host round trips (8-byte H2D / D2H, pageable and pinned, an empty kernel +
// stream sync) on one stream while the input's large H2D streams on another -- whether a small copy
// queues behind the bulk transfer on the copy engine (the clustering's read-backs and h2d() calls).
// usage: copyq  (GPU box)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_nop(uint64_t *p) { if (threadIdx.x == 0 && blockIdx.x == 0 && p[0] == 12345) p[1] = 1; }

static double now() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main() {
  const size_t n = 1ull << 30;
  void *d, *h;
  uint64_t *hsmall, *dsmall;
  CK(hipMalloc(&d, n));
  CK(hipMemset(d, 1, n));
  CK(hipHostMalloc(&h, n, hipHostMallocDefault));
  memset(h, 2, n);
  CK(hipHostMalloc((void **)&hsmall, 64, hipHostMallocDefault));
  CK(hipMalloc((void **)&dsmall, 64));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // kind: 0 D2H pageable, 1 D2H pinned, 2 H2D pageable, 3 H2D pinned, 4 kernel + sync
  auto small = [&](int kind, int reps, double &mx) {
    double s = 0;
    mx = 0;
    uint64_t v = 7;
    for (int r = 0; r < reps; ++r) {
      const double a = now();
      switch (kind) {
        case 0: (void)hipMemcpyAsync(&v, dsmall, 8, hipMemcpyDeviceToHost, s2); break;
        case 1: (void)hipMemcpyAsync(hsmall, dsmall, 8, hipMemcpyDeviceToHost, s2); break;
        case 2: (void)hipMemcpyAsync(dsmall, &v, 8, hipMemcpyHostToDevice, s2); break;
        case 3: (void)hipMemcpyAsync(dsmall, hsmall, 8, hipMemcpyHostToDevice, s2); break;
        default: hipLaunchKernelGGL(k_nop, dim3(1), dim3(64), 0, s2, dsmall); break;
      }
      (void)hipStreamSynchronize(s2);
      const double t = now() - a;
      s += t;
      mx = std::max(mx, t);
    }
    return s / reps;
  };
  const char *names[5] = {"D2H pageable", "D2H pinned  ", "H2D pageable", "H2D pinned  ", "kernel+sync "};
  for (int k = 0; k < 5; ++k) {
    double mx;
    const double av = small(k, 20, mx);
    printf("idle       %s: avg %.3f ms max %.3f ms\n", names[k], av, mx);
  }
  for (int dir = 0; dir < 2; ++dir)
    for (int k = 0; k < 5; ++k) {
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0, s1));
      for (size_t o = 0; o < n; o += 32ull << 20) {
        if (dir == 0) CK(hipMemcpyAsync((char *)d + o, (char *)h + o, 32ull << 20, hipMemcpyHostToDevice, s1));
        else CK(hipMemcpyAsync((char *)h + o, (char *)d + o, 32ull << 20, hipMemcpyDeviceToHost, s1));
      }
      CK(hipEventRecord(e1, s1));
      const double t0 = now();
      double mx;
      const double av = small(k, 10, mx);
      const double t1 = now();
      CK(hipEventSynchronize(e1));
      const double t2 = now();
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      printf("bulk %s 1 GiB (%.1f GB/s, %.2f ms): %s avg %.3f ms max %.3f ms; the 10 probes took %.2f ms, bulk done %.2f ms later\n",
             dir ? "D2H" : "H2D", n / ms / 1e6, ms, names[k], av, mx, t1 - t0, t2 - t1);
    }
  return 0;
}
