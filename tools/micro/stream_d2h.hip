// The result stream's copy pattern against the link: 1 GiB device -> pinned host in chunks of 8 / 32 /
// 64 MiB, with at most K chunks in flight and the host waiting on each chunk's event before issuing
// chunk k + K (the snap thread's loop), against everything queued at once.
// usage: stream_d2h  (GPU box)
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

static double now() { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main() {
  const size_t n = 1ull << 30;
  void *d, *h;
  CK(hipMalloc(&d, n));
  CK(hipMemset(d, 3, n));
  CK(hipHostMalloc(&h, n, hipHostMallocDefault));
  memset(h, 1, n);
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  std::vector<hipEvent_t> ev(8);
  for (size_t i = 0; i < ev.size(); ++i) CK(hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
  CK(hipDeviceSynchronize());
  for (size_t chunk : {8ull << 20, 32ull << 20, 64ull << 20})
    for (int K : {1, 2, 3, 4, 0}) {  // 0: all queued, one sync at the end
      double best = 1e30;
      for (int rep = 0; rep < 3; ++rep) {
        CK(hipDeviceSynchronize());
        const double t0 = now();
        size_t k = 0;
        for (size_t o = 0; o < n; o += chunk, ++k) {
          if (K && k >= (size_t)K) CK(hipEventSynchronize(ev[k % K]));
          CK(hipMemcpyAsync((char *)h + o, (char *)d + o, chunk, hipMemcpyDeviceToHost, s));
          if (K) CK(hipEventRecord(ev[k % K], s));
        }
        CK(hipStreamSynchronize(s));
        const double t = now() - t0;
        if (t < best) best = t;
      }
      printf("D2H 1 GiB in %3zu MiB chunks, %s: %.1f GB/s\n", chunk >> 20, K ? (K == 1 ? "1 in flight" : K == 2 ? "2 in flight" : K == 3 ? "3 in flight" : "4 in flight") : "all queued",
             n / best / 1e6);
    }
  return 0;
}
