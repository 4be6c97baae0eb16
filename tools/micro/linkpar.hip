// PCIe link rate of 32 MiB chunk copies between HBM and pinned host memory spread over 1, 2 or 4 streams
// (one copy engine each?), per direction, and both directions at once (full duplex) -- how the result
// stream and the input upload should be issued.
// usage: linkpar  (GPU box)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

static double now() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main() {
  const size_t n = 1ull << 30, chunk = 32ull << 20;
  void *d, *d2, *h, *h2;
  CK(hipMalloc(&d, n));
  CK(hipMalloc(&d2, n));
  CK(hipHostMalloc(&h, n, hipHostMallocDefault));
  CK(hipHostMalloc(&h2, n, hipHostMallocDefault));
  memset(h, 1, n);
  memset(h2, 2, n);
  CK(hipMemset(d, 3, n));
  CK(hipDeviceSynchronize());
  hipStream_t s[8];
  for (auto &x : s) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
  auto run = [&](int dir, int ns, bool duplex) {  // dir 0: H2D, 1: D2H; duplex: the other direction on streams 4..
    double best = 1e30;
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipDeviceSynchronize();
      const double t0 = now();
      for (size_t o = 0, k = 0; o < n; o += chunk, ++k) {
        hipStream_t q = s[k % ns];
        if (dir == 0) (void)hipMemcpyAsync((char *)d + o, (char *)h + o, chunk, hipMemcpyHostToDevice, q);
        else (void)hipMemcpyAsync((char *)h + o, (char *)d + o, chunk, hipMemcpyDeviceToHost, q);
        if (duplex) {
          hipStream_t q2 = s[4 + k % ns];
          if (dir == 0) (void)hipMemcpyAsync((char *)h2 + o, (char *)d2 + o, chunk, hipMemcpyDeviceToHost, q2);
          else (void)hipMemcpyAsync((char *)d2 + o, (char *)h2 + o, chunk, hipMemcpyHostToDevice, q2);
        }
      }
      (void)hipDeviceSynchronize();
      const double t = now() - t0;
      if (t < best) best = t;
    }
    printf("%s %d stream(s)%s: %.1f GB/s per direction (%.2f ms for 1 GiB)\n", dir ? "D2H" : "H2D", ns,
           duplex ? " + the other direction at once" : "", n / best / 1e6, best);
  };
  for (int dir = 0; dir < 2; ++dir)
    for (int ns : {1, 2, 4}) run(dir, ns, false);
  for (int ns : {1, 2}) run(1, ns, true);
  return 0;
}
