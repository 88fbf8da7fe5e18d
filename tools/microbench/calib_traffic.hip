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


typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__device__ inline uint4 nt_ld(const uint4* p) { const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p)); return make_uint4(v.x, v.y, v.z, v.w); }
__device__ inline void nt_st(uint4 v, uint4* p) { __builtin_nontemporal_store(v4u{v.x, v.y, v.z, v.w}, reinterpret_cast<v4u*>(p)); }
// 4 independent 16-byte loads in flight per lane before their stores
__global__ __launch_bounds__(256) void copy16x4(const uint4* __restrict__ in, uint4* __restrict__ out, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += 4 * stride) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = (i + u * stride < n) ? in[i + u * stride] : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < 4; ++u) if (i + u * stride < n) out[i + u * stride] = v[u];
  }
}
__global__ __launch_bounds__(256) void copy16x4nt(const uint4* __restrict__ in, uint4* __restrict__ out, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += 4 * stride) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = (i + u * stride < n) ? nt_ld(in + i + u * stride) : make_uint4(0, 0, 0, 0);
#pragma unroll
    for (int u = 0; u < 4; ++u) if (i + u * stride < n) nt_st(v[u], out + i + u * stride);
  }
}
__global__ __launch_bounds__(256) void copy8x8(const uint2* __restrict__ in, uint2* __restrict__ out, size_t n) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += 8 * stride) {
    uint2 v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = (i + u * stride < n) ? in[i + u * stride] : make_uint2(0, 0);
#pragma unroll
    for (int u = 0; u < 8; ++u) if (i + u * stride < n) out[i + u * stride] = v[u];
  }
}
__global__ __launch_bounds__(256) void write16(uint4* __restrict__ out, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = make_uint4(i, i, i, i);
}
__global__ __launch_bounds__(256) void read16(const uint4* __restrict__ in, uint32_t* __restrict__ sink, size_t n) {
  uint32_t acc = 0;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += 4 * stride) {
#pragma unroll
    for (int u = 0; u < 4; ++u) if (i + u * stride < n) { const uint4 v = in[i + u * stride]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
  }
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
  auto timed = [&](const char* name, double moved, auto launch) {
    float best = 1e30f;
    for (int it = 0; it < 5; ++it) {
      hipEventRecord(e0, 0);
      launch();
      hipEventRecord(e1, 0);
      hipEventSynchronize(e1);
      float ms = 0;
      hipEventElapsedTime(&ms, e0, e1);
      if (ms < best) best = ms;
    }
    printf("%-34s %.3f ms -> %.0f GB/s\n", name, best, moved / (best * 1e-3) / 1e9);
  };
  const double two = 2.0 * bytes;
  for (int grid : {8192, 2048, 1024}) {
    printf("grid %d x 256 threads:\n", grid);
    timed("  copy8 (1 GiB r + 1 GiB w)", two, [&] { hipLaunchKernelGGL(copy8, dim3(grid), dim3(256), 0, 0, a, b, n); });
    timed("  copy16", two, [&] { hipLaunchKernelGGL(copy16, dim3(grid), dim3(256), 0, 0, (const uint4*)a, (uint4*)b, bytes / 16); });
    timed("  copy16x4 (4 loads in flight)", two, [&] { hipLaunchKernelGGL(copy16x4, dim3(grid), dim3(256), 0, 0, (const uint4*)a, (uint4*)b, bytes / 16); });
    timed("  copy16x4nt", two, [&] { hipLaunchKernelGGL(copy16x4nt, dim3(grid), dim3(256), 0, 0, (const uint4*)a, (uint4*)b, bytes / 16); });
    timed("  copy8x8 (8 loads in flight)", two, [&] { hipLaunchKernelGGL(copy8x8, dim3(grid), dim3(256), 0, 0, a, b, n); });
    timed("  write16 (1 GiB w)", bytes, [&] { hipLaunchKernelGGL(write16, dim3(grid), dim3(256), 0, 0, (uint4*)b, bytes / 16); });
    timed("  read16x4 (1 GiB r)", bytes, [&] { hipLaunchKernelGGL(read16, dim3(grid), dim3(256), 0, 0, (const uint4*)a, sink, bytes / 16); });
  }
  hipFree(a);
  hipFree(b);
  hipFree(sink);
  return 0;
}
