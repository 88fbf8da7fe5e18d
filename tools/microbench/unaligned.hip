// Checks that 8- and 16-byte global loads and stores at 2-byte (and 1-byte)
// aligned addresses move the right bytes on this platform (the KFD runs gfx9
// queues in unaligned-access mode), and times them against aligned ones.  Not
// product code: it pins the assumption behind the resident kernels' vector
// row accesses for odd chunk counts (kernels_res.hip rows_vec_ok).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

#define CK(x)                                                        \
  do {                                                               \
    hipError_t e = (x);                                              \
    if (e != hipSuccess) {                                           \
      printf("HIP error %s line %d\n", hipGetErrorString(e), __LINE__); \
      return 1;                                                      \
    }                                                                \
  } while (0)

__global__ void k_copy8(const uint8_t* src, uint8_t* dst, size_t n8) {
  const size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x;
  if (i < n8) *reinterpret_cast<uint2*>(dst + 8 * i) = *reinterpret_cast<const uint2*>(src + 8 * i);
}
__global__ void k_copy16(const uint8_t* src, uint8_t* dst, size_t n16) {
  const size_t i = blockIdx.x * static_cast<size_t>(blockDim.x) + threadIdx.x;
  if (i < n16) *reinterpret_cast<uint4*>(dst + 16 * i) = *reinterpret_cast<const uint4*>(src + 16 * i);
}

int main() {
  const size_t bytes = size_t(1) << 28;
  uint8_t *a, *b;
  CK(hipMalloc(&a, bytes + 64));
  CK(hipMalloc(&b, bytes + 64));
  std::vector<uint8_t> h(bytes + 64), g(bytes + 64);
  for (size_t i = 0; i < h.size(); ++i) h[i] = static_cast<uint8_t>(i * 2654435761u >> 13);
  CK(hipMemcpy(a, h.data(), h.size(), hipMemcpyHostToDevice));
  int bad = 0;
  for (int width : {8, 16}) {
    for (int off : {0, 2, 4, 1}) {
      CK(hipMemset(b, 0, bytes + 64));
      const size_t n = (bytes - 32) / width;
      const unsigned blocks = static_cast<unsigned>((n + 255) / 256);
      auto launch = [&]() {
        if (width == 8)
          k_copy8<<<blocks, 256>>>(a + off, b + off, n);
        else
          k_copy16<<<blocks, 256>>>(a + off, b + off, n);
      };
      launch();
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(g.data(), b, g.size(), hipMemcpyDeviceToHost));
      size_t wrong = 0;
      for (size_t i = 0; i < n * width; ++i) wrong += g[off + i] != h[off + i];
      hipEvent_t e0, e1;
      CK(hipEventCreate(&e0));
      CK(hipEventCreate(&e1));
      float best = 1e9f;
      for (int r = 0; r < 5; ++r) {
        CK(hipEventRecord(e0));
        launch();
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
      }
      printf("width %2d offset %d: %zu wrong bytes, copy %.0f GB/s\n", width, off, wrong, 2.0 * n * width / best / 1e6);
      bad += wrong != 0;
    }
  }
  printf(bad ? "UNALIGNED ACCESS BROKEN\n" : "unaligned access ok\n");
  return bad;
}
