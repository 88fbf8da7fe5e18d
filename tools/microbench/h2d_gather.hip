// Microbenchmark (not product code): how fast can a kernel read pinned host
// memory over PCIe, against the DMA engine (hipMemcpyAsync H2D)?  Drives the
// design of np_reconstruct_batch_host's present-row gather (engine.cpp).
//   allocations: hipHostMalloc default (coherent), hipHostMallocNonCoherent,
//                malloc + hipHostRegister
//   kernels: one wave per 4 KiB row, 16 / 8 / 4-byte loads, nontemporal loads,
//            1 / 2 / 4 waves per row, and every other row (a 1/2 present mask)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::printf("%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));            \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

constexpr size_t kRow = 4096;
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef unsigned int v2u __attribute__((ext_vector_type(2)));

template <typename T, bool NT>
__global__ __launch_bounds__(256) void k_rows(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst, size_t rows,
                                              uint32_t step, uint32_t wpr) {
  const uint32_t lane = threadIdx.x & 63;
  const size_t waves = static_cast<size_t>(gridDim.x) * 4;
  const size_t per = kRow / sizeof(T) / wpr;
  for (size_t w = static_cast<size_t>(blockIdx.x) * 4 + (threadIdx.x >> 6); w < rows * wpr; w += waves) {
    const size_t r = (w / wpr) * step, part = w % wpr;
    if (r >= rows) continue;
    const T* s = reinterpret_cast<const T*>(src + r * kRow) + part * per;
    T* d = reinterpret_cast<T*>(dst + r * kRow) + part * per;
    T x[16];
    const uint32_t cnt = static_cast<uint32_t>(per / 64);
#pragma unroll
    for (uint32_t i = 0; i < 16; ++i)
      if (i < cnt) x[i] = NT ? __builtin_nontemporal_load(s + lane + 64 * i) : s[lane + 64 * i];
#pragma unroll
    for (uint32_t i = 0; i < 16; ++i)
      if (i < cnt) d[lane + 64 * i] = x[i];
  }
}

template <typename T, bool NT>
float run(const uint8_t* src, uint8_t* dst, size_t rows, uint32_t step, uint32_t wpr, hipStream_t s,
          uint32_t blocks = 8192) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  k_rows<T, NT><<<blocks, 256, 0, s>>>(src, dst, rows, step, wpr);
  CK(hipEventRecord(a, s));
  for (int it = 0; it < 3; ++it) k_rows<T, NT><<<blocks, 256, 0, s>>>(src, dst, rows, step, wpr);
  CK(hipEventRecord(b, s));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  const double bytes = 3.0 * ((rows + step - 1) / step) * kRow;
  return static_cast<float>(bytes / (ms * 1e-3) / 1e9);
}

int main() {
  const size_t rows = (size_t(1) << 30) / kRow;  // 1 GiB
  const size_t bytes = rows * kRow;
  hipStream_t s;
  CK(hipStreamCreate(&s));
  uint8_t* dst;
  CK(hipMalloc(&dst, bytes));
  struct Alloc {
    const char* name;
    uint8_t* h;
    uint8_t* d;
  };
  std::vector<Alloc> al;
  {
    uint8_t* h;
    CK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
    al.push_back({"hipHostMalloc(default)", h, nullptr});
    CK(hipHostMalloc(&h, bytes, hipHostMallocNonCoherent));
    al.push_back({"hipHostMalloc(NonCoherent)", h, nullptr});
    h = static_cast<uint8_t*>(std::aligned_alloc(4096, bytes));
    CK(hipHostRegister(h, bytes, hipHostRegisterMapped));
    al.push_back({"malloc+hipHostRegister", h, nullptr});
  }
  for (auto& x : al) {
    for (size_t i = 0; i < bytes; i += 4096) x.h[i] = static_cast<uint8_t>(i >> 12);
    void* d = nullptr;
    CK(hipHostGetDevicePointer(&d, x.h, 0));
    x.d = static_cast<uint8_t*>(d);
    // DMA reference
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipMemcpyAsync(dst, x.h, bytes, hipMemcpyHostToDevice, s));
    CK(hipEventRecord(a, s));
    for (int it = 0; it < 3; ++it) CK(hipMemcpyAsync(dst, x.h, bytes, hipMemcpyHostToDevice, s));
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    std::printf("%-28s dev==host %d  DMA H2D %.1f GB/s\n", x.name, x.d == x.h, 3.0 * bytes / (ms * 1e-3) / 1e9);
    for (uint32_t wpr : {1u, 2u, 4u}) {
      std::printf("  wpr %u: x16 %.1f  x8 %.1f  x4 %.1f  x16nt %.1f  x16 half-rows %.1f GB/s\n", wpr,
                  run<v4u, false>(x.d, dst, rows, 1, wpr, s), run<v2u, false>(x.d, dst, rows, 1, wpr, s),
                  run<uint32_t, false>(x.d, dst, rows, 1, wpr, s), run<v4u, true>(x.d, dst, rows, 1, wpr, s),
                  run<v4u, false>(x.d, dst, rows, 2, wpr, s));
    }
    {  // a D2H DMA while the kernel reads host memory (the upstream link carries the read requests)
      hipStream_t s2;
      CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
      const size_t ob = size_t(256) << 20;
      uint8_t* hout;
      CK(hipHostMalloc(&hout, ob, hipHostMallocDefault));
      hipEvent_t c0, c1, g0, g1;
      CK(hipEventCreate(&c0));
      CK(hipEventCreate(&c1));
      CK(hipEventCreate(&g0));
      CK(hipEventCreate(&g1));
      CK(hipMemcpyAsync(hout, dst, ob, hipMemcpyDeviceToHost, s2));
      CK(hipStreamSynchronize(s2));
      CK(hipEventRecord(c0, s2));
      CK(hipMemcpyAsync(hout, dst, ob, hipMemcpyDeviceToHost, s2));
      CK(hipEventRecord(c1, s2));
      CK(hipEventSynchronize(c1));
      float ma, mb;
      CK(hipEventElapsedTime(&ma, c0, c1));
      for (uint32_t bl : {32u, 64u, 256u}) {
        CK(hipEventRecord(g0, s));
        k_rows<v4u, false><<<bl, 256, 0, s>>>(x.d, dst + ob, rows - ob / kRow, 1, 1);
        CK(hipEventRecord(g1, s));
        CK(hipEventRecord(c0, s2));
        for (int it = 0; it < 3; ++it) CK(hipMemcpyAsync(hout, dst, ob, hipMemcpyDeviceToHost, s2));
        CK(hipEventRecord(c1, s2));
        CK(hipEventSynchronize(c1));
        CK(hipEventSynchronize(g1));
        CK(hipEventElapsedTime(&mb, c0, c1));
        float mg;
        CK(hipEventElapsedTime(&mg, g0, g1));
        std::printf("  D2H alone %.1f GB/s; with gather (%u blocks): D2H %.1f (%.1f ms), gather %.1f GB/s (%.1f ms)\n",
                    ob / (ma * 1e-3) / 1e9, bl, 3.0 * ob / (mb * 1e-3) / 1e9, mb, (bytes - ob) / (mg * 1e-3) / 1e9, mg);
      }
      // the same D2H by a kernel storing to the mapped host buffer
      uint8_t* dout = nullptr;
      CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dout), hout, 0));
      for (uint32_t wb : {32u, 64u, 256u}) {
        CK(hipEventRecord(c0, s2));
        for (int it = 0; it < 3; ++it) k_rows<v4u, false><<<wb, 256, 0, s2>>>(dst, dout, ob / kRow, 1, 1);
        CK(hipEventRecord(c1, s2));
        CK(hipEventSynchronize(c1));
        CK(hipEventElapsedTime(&ma, c0, c1));
        CK(hipEventRecord(g0, s));
        k_rows<v4u, false><<<32, 256, 0, s>>>(x.d, dst + ob, rows - ob / kRow, 1, 1);
        CK(hipEventRecord(g1, s));
        CK(hipEventRecord(c0, s2));
        for (int it = 0; it < 3; ++it) k_rows<v4u, false><<<wb, 256, 0, s2>>>(dst, dout, ob / kRow, 1, 1);
        CK(hipEventRecord(c1, s2));
        CK(hipEventSynchronize(c1));
        CK(hipEventSynchronize(g1));
        CK(hipEventElapsedTime(&mb, c0, c1));
        float mg;
        CK(hipEventElapsedTime(&mg, g0, g1));
        std::printf("  kernel D2H (%u blocks) alone %.1f GB/s; with gather (32 blocks): D2H %.1f (%.1f ms), gather %.1f GB/s (%.1f ms)\n",
                    wb, 3.0 * ob / (ma * 1e-3) / 1e9, 3.0 * ob / (mb * 1e-3) / 1e9, mb, (bytes - ob) / (mg * 1e-3) / 1e9, mg);
      }
      CK(hipHostFree(hout));
    }
    std::printf("  grid sweep (x16, wpr 1):");
    for (uint32_t bl : {8u, 16u, 32u, 64u, 128u, 256u, 1024u})
      std::printf("  %u blocks %.1f", bl, run<v4u, false>(x.d, dst, rows, 1, 1, s, bl));
    std::printf(" GB/s\n");
  }
  return 0;
}
