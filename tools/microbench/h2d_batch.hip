// Microbenchmark (not product code): hipMemcpyBatchAsync (SDMA) of the
// present rows of 4 KiB-row payloads (random 1/3 erased, runs of consecutive
// present rows merged) from pinned host memory, against one contiguous DMA and
// the gather kernel's rate (h2d_gather.hip).  Also with a concurrent D2H.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#define CK(x)                                                               \
  do {                                                                      \
    hipError_t e_ = (x);                                                    \
    if (e_ != hipSuccess) {                                                 \
      std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                         \
    }                                                                       \
  } while (0)

int main() {
  const size_t row = 4096, n = 1024, payloads = 64;
  const size_t bytes = payloads * n * row;  // 256 MiB
  uint8_t *h, *d, *hout;
  CK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
  CK(hipHostMalloc(&hout, bytes / 4, hipHostMallocDefault));
  CK(hipMalloc(&d, bytes + bytes / 4));
  std::mt19937 rng(1);
  std::vector<void*> dsts, srcs;
  std::vector<size_t> sizes;
  size_t moved = 0;
  for (size_t b = 0; b < payloads; ++b) {
    std::vector<uint8_t> pres(n, 1);
    for (size_t e = 0; e < 342;) {
      const size_t v = rng() % n;
      if (pres[v]) pres[v] = 0, ++e;
    }
    for (size_t v = 0; v < n;) {
      if (!pres[v]) { ++v; continue; }
      size_t w = v;
      while (w < n && pres[w]) ++w;
      srcs.push_back(h + (b * n + v) * row);
      dsts.push_back(d + (b * n + v) * row);
      sizes.push_back((w - v) * row);
      moved += (w - v) * row;
      v = w;
    }
  }
  std::printf("%zu copies, %.1f MB present of %.1f MB\n", sizes.size(), moved / 1e6, bytes / 1e6);
  hipStream_t s, s2;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  float ms;
  for (size_t chunk : {size_t(256), size_t(4096), sizes.size()}) {
    for (int rep = 0; rep < 2; ++rep) {
      auto t0 = std::chrono::steady_clock::now();
      CK(hipEventRecord(a, s));
      for (size_t i = 0; i < sizes.size(); i += chunk) {
        size_t cnt = std::min(chunk, sizes.size() - i), fail = 0;
        CK(hipMemcpyBatchAsync(dsts.data() + i, srcs.data() + i, sizes.data() + i, cnt, nullptr, nullptr, 0, &fail, s));
      }
      CK(hipEventRecord(b, s));
      auto t1 = std::chrono::steady_clock::now();
      CK(hipEventSynchronize(b));
      CK(hipEventElapsedTime(&ms, a, b));
      std::printf("batch of %zu: %.1f GB/s present bytes (%.2f ms GPU, host enqueue %.2f ms)\n", chunk,
                  moved / (ms * 1e-3) / 1e9, ms, std::chrono::duration<double, std::milli>(t1 - t0).count());
    }
  }
  CK(hipEventRecord(a, s));
  CK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s));
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  CK(hipEventElapsedTime(&ms, a, b));
  std::printf("contiguous DMA: %.1f GB/s\n", bytes / (ms * 1e-3) / 1e9);
  // with a concurrent D2H of a quarter of the bytes, 3 times
  hipEvent_t c0, c1;
  CK(hipEventCreate(&c0));
  CK(hipEventCreate(&c1));
  CK(hipEventRecord(c0, s2));
  for (int i = 0; i < 3; ++i) CK(hipMemcpyAsync(hout, d + bytes, bytes / 4, hipMemcpyDeviceToHost, s2));
  CK(hipEventRecord(c1, s2));
  CK(hipEventRecord(a, s));
  size_t fail = 0;
  CK(hipMemcpyBatchAsync(dsts.data(), srcs.data(), sizes.data(), sizes.size(), nullptr, nullptr, 0, &fail, s));
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  CK(hipEventSynchronize(c1));
  float mc;
  CK(hipEventElapsedTime(&ms, a, b));
  CK(hipEventElapsedTime(&mc, c0, c1));
  std::printf("batch + D2H: batch %.1f GB/s (%.2f ms), D2H %.1f GB/s (%.2f ms)\n", moved / (ms * 1e-3) / 1e9, ms,
              3.0 * bytes / 4 / (mc * 1e-3) / 1e9, mc);
  return 0;
}
