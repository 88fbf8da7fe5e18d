// Calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE for the access widths the
// codec kernels use (8 B per lane, coalesced rows), on buffers far larger
// than the 256 MiB Infinity Cache.  Run under rocprofv3 --pmc FETCH_SIZE (and
// separately WRITE_SIZE); known bytes per dispatch are printed.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

__global__ void copy8(const uint2* __restrict__ in, uint2* __restrict__ out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = in[i];
}

__global__ void copy16(const uint4* __restrict__ in, uint4* __restrict__ out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = in[i];
}

__global__ void read8(const uint2* __restrict__ in, uint32_t* __restrict__ sink, size_t n) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    acc ^= in[i].x ^ in[i].y;
  if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
  const size_t bytes = size_t(1) << 30;  // 1 GiB each
  const size_t n = bytes / 8;
  uint2 *a, *b;
  uint32_t* sink;
  if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess)
    return 1;
  hipMemset(a, 1, bytes);
  hipDeviceSynchronize();
  for (int it = 0; it < 3; ++it) {
    hipLaunchKernelGGL(read8, dim3(8192), dim3(256), 0, 0, a, sink, n);
    hipLaunchKernelGGL(copy8, dim3(8192), dim3(256), 0, 0, a, b, n);
  }
  hipDeviceSynchronize();
  printf("read8: %zu bytes read per dispatch; copy8: %zu read + %zu written per dispatch\n", bytes, bytes, bytes);
  // achievable HBM bandwidth: timed copies of 1 GiB (read + write)
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int w = 8; w <= 16; w += 8) {
    float best = 1e30f;
    for (int it = 0; it < 5; ++it) {
      hipEventRecord(e0, 0);
      if (w == 8)
        hipLaunchKernelGGL(copy8, dim3(8192), dim3(256), 0, 0, a, b, n);
      else
        hipLaunchKernelGGL(copy16, dim3(8192), dim3(256), 0, 0, (const uint4*)a, (uint4*)b, bytes / 16);
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    printf("copy%d: %.3f ms for 1 GiB read + 1 GiB written -> %.0f GB/s\n", w, best, 2.0 * bytes / (best * 1e-3) / 1e9);
  }
  hipFree(a);
  hipFree(b);
  hipFree(sink);
  return 0;
}
