// Microbenchmark for the pageable host reconstruct (engine.cpp host_gather):
// host memcpy rate from pageable into pinned memory on 1-16 threads, the cost
// of pinning a pageable range in place (hipHostRegister / Unregister), and
// the runtime's own pageable H2D / D2H copies.  Not product code.
#include <hip/hip_runtime.h>

#include <immintrin.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);         \
      return 1;                                                               \
    }                                                                         \
  } while (0)

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void stream_copy(uint8_t* dst, const uint8_t* src, size_t len) {  // as engine.cpp
  for (size_t i = 0; i + 64 <= len; i += 64) {
    const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i));
    const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 16));
    const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 32));
    const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 48));
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i), a);
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 16), b);
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 32), c);
    _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 48), d);
  }
  _mm_sfence();
}

int main() {
  const size_t bytes = size_t(256) << 20;
  uint8_t* pg = static_cast<uint8_t*>(std::aligned_alloc(4096, bytes));
  uint8_t* pg2 = static_cast<uint8_t*>(std::aligned_alloc(4096, bytes));
  memset(pg, 1, bytes);
  memset(pg2, 2, bytes);
  uint8_t* pin = nullptr;
  CK(hipHostMalloc(reinterpret_cast<void**>(&pin), bytes, 0));
  memset(pin, 3, bytes);
  void* dev = nullptr;
  CK(hipMalloc(&dev, bytes));
  printf("host copy pageable -> pinned, 256 MiB, 4 KiB rows (memcpy / streaming stores):\n");
  for (unsigned t : {1u, 2u, 4u, 8u, 16u, 32u}) {
    printf("  %2u threads:", t);
    for (int mode = 0; mode < 2; ++mode) {
      double best = 1e9;
      for (int r = 0; r < 3; ++r) {
        const double t0 = now();
        std::vector<std::thread> th;
        for (unsigned w = 0; w < t; ++w)
          th.emplace_back([&, w] {
            for (size_t off = size_t(w) * 4096; off < bytes; off += size_t(t) * 4096) {
              if (mode == 0)
                memcpy(pin + off, pg + off, 4096);
              else
                stream_copy(pin + off, pg + off, 4096);
            }
          });
        for (auto& x : th) x.join();
        best = std::min(best, now() - t0);
      }
      printf(" %6.1f GB/s", bytes / best / 1e9);
    }
    printf("\n");
  }
  printf("pin in place (hipHostRegister + hipHostUnregister):\n");
  for (size_t mb : {64, 256}) {
    double reg = 1e9, unreg = 1e9;
    for (int r = 0; r < 3; ++r) {
      const double t0 = now();
      CK(hipHostRegister(pg2, mb << 20, hipHostRegisterDefault));
      const double t1 = now();
      CK(hipHostUnregister(pg2));
      const double t2 = now();
      reg = std::min(reg, t1 - t0);
      unreg = std::min(unreg, t2 - t1);
    }
    printf("  %3zu MiB: register %.2f ms (%.1f GB/s), unregister %.2f ms\n", mb, reg * 1e3, (mb << 20) / reg / 1e9,
           unreg * 1e3);
  }
  printf("runtime copies, 256 MiB:\n");
  for (int dir = 0; dir < 4; ++dir) {
    double best = 1e9;
    for (int r = 0; r < 3; ++r) {
      const double t0 = now();
      if (dir == 0) CK(hipMemcpy(dev, pg, bytes, hipMemcpyHostToDevice));
      if (dir == 1) CK(hipMemcpy(pg, dev, bytes, hipMemcpyDeviceToHost));
      if (dir == 2) CK(hipMemcpy(dev, pin, bytes, hipMemcpyHostToDevice));
      if (dir == 3) CK(hipMemcpy(pin, dev, bytes, hipMemcpyDeviceToHost));
      best = std::min(best, now() - t0);
    }
    const char* nm[] = {"pageable H2D", "pageable D2H", "pinned H2D", "pinned D2H"};
    printf("  %-13s %6.1f GB/s\n", nm[dir], bytes / best / 1e9);
  }
  CK(hipFree(dev));
  CK(hipHostFree(pin));
  free(pg);
  free(pg2);
  return 0;
}
