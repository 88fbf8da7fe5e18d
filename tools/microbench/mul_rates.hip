// Microbenchmark: throughput of GF(2^16) multiply-by-uniform-constant strategies on gfx950.
// Used to choose the hot-path multiplier design. Not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int ITERS = 256;
constexpr int CH = 8;  // independent chains per thread

// (a) LDS split tables: 64+32+32 u16 entries per constant, uniform across the wave.
__global__ __launch_bounds__(256) void k_lds(uint32_t* out, const uint16_t* tabs, int ntab) {
  __shared__ uint16_t t[128 * 16];
  for (int i = threadIdx.x; i < 128 * 16; i += 256) t[i] = tabs[i];
  __syncthreads();
  uint32_t y[CH];
  for (int c = 0; c < CH; ++c) y[c] = (blockIdx.x * 256 + threadIdx.x) * 2654435761u + c;
  for (int it = 0; it < ITERS; ++it) {
    const uint16_t* tb = t + (it & 15) * 128;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      uint32_t v = y[c] & 0xffff;
      uint32_t r = tb[v & 63] ^ tb[64 + ((v >> 6) & 31)] ^ tb[96 + (v >> 11)];
      y[c] = (y[c] ^ r) + 0x9e37;
    }
  }
  uint32_t acc = 0;
  for (int c = 0; c < CH; ++c) acc ^= y[c];
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// (b) same tables in global memory (all lanes of a wave index one constant's table).
__global__ __launch_bounds__(256) void k_gmem(uint32_t* out, const uint16_t* __restrict__ tabs, int ntab) {
  uint32_t y[CH];
  for (int c = 0; c < CH; ++c) y[c] = (blockIdx.x * 256 + threadIdx.x) * 2654435761u + c;
  for (int it = 0; it < ITERS; ++it) {
    const uint16_t* tb = tabs + ((it + blockIdx.x) % ntab) * 128;
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      uint32_t v = y[c] & 0xffff;
      uint32_t r = tb[v & 63] ^ tb[64 + ((v >> 6) & 31)] ^ tb[96 + (v >> 11)];
      y[c] = (y[c] ^ r) + 0x9e37;
    }
  }
  uint32_t acc = 0;
  for (int c = 0; c < CH; ++c) acc ^= y[c];
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// (c) v_perm byte-planar quad multiply: 4 symbols per (L,H) register pair, 12 byte-table lookups.
__device__ __forceinline__ uint32_t x3(uint32_t a, uint32_t b, uint32_t c) { return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96); }
__global__ __launch_bounds__(256) void k_perm(uint32_t* out, const uint32_t* __restrict__ ptab, int ntab) {
  uint32_t L[CH], H[CH];
  for (int c = 0; c < CH; ++c) { L[c] = (blockIdx.x * 256 + threadIdx.x) * 2654435761u + c; H[c] = L[c] * 747796405u; }
  for (int it = 0; it < ITERS; ++it) {
    const uint32_t* tb = ptab + ((it + blockIdx.x) % ntab) * 20;   // uniform -> s_load
    uint32_t t[20];
#pragma unroll
    for (int i = 0; i < 20; ++i) t[i] = tb[i];
#pragma unroll
    for (int c = 0; c < CH; ++c) {
      uint32_t l = L[c], h = H[c];
      uint32_t s0 = l & 0x07070707u, s1 = (l >> 3) & 0x07070707u, s2 = (l >> 6) & 0x03030303u;
      uint32_t s3 = h & 0x07070707u, s4 = (h >> 3) & 0x07070707u, s5 = (h >> 6) & 0x03030303u;
      uint32_t ol = x3(__builtin_amdgcn_perm(t[0], t[1], s0), __builtin_amdgcn_perm(t[2], t[3], s1), __builtin_amdgcn_perm(t[4], t[4], s2));
      ol = x3(ol, __builtin_amdgcn_perm(t[5], t[6], s3), __builtin_amdgcn_perm(t[7], t[8], s4));
      ol ^= __builtin_amdgcn_perm(t[9], t[9], s5);
      uint32_t oh = x3(__builtin_amdgcn_perm(t[10], t[11], s0), __builtin_amdgcn_perm(t[12], t[13], s1), __builtin_amdgcn_perm(t[14], t[14], s2));
      oh = x3(oh, __builtin_amdgcn_perm(t[15], t[16], s3), __builtin_amdgcn_perm(t[17], t[18], s4));
      oh ^= __builtin_amdgcn_perm(t[19], t[19], s5);
      L[c] = (l ^ ol) + 0x9e37; H[c] = h ^ oh;
    }
  }
  uint32_t acc = 0;
  for (int c = 0; c < CH; ++c) acc ^= L[c] ^ H[c];
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

int main() {
  const int blocks = 256 * 16, threads = 256;
  const int ntab = 1024;
  std::vector<uint16_t> h(ntab * 128);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (uint16_t)(i * 40503u);
  std::vector<uint32_t> hp(ntab * 20);
  for (size_t i = 0; i < hp.size(); ++i) hp[i] = (uint32_t)(i * 2246822519u);
  uint16_t* dt; uint32_t* dp; uint32_t* dout;
  CK(hipMalloc(&dt, h.size() * 2)); CK(hipMalloc(&dp, hp.size() * 4)); CK(hipMalloc(&dout, blocks * threads * 4));
  CK(hipMemcpy(dt, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(dp, hp.data(), hp.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int which = 0; which < 3; ++which) {
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      CK(hipEventRecord(a));
      if (which == 0) k_lds<<<blocks, threads>>>(dout, dt, ntab);
      if (which == 1) k_gmem<<<blocks, threads>>>(dout, dt, ntab);
      if (which == 2) k_perm<<<blocks, threads>>>(dout, dp, ntab);
      CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
      float ms; CK(hipEventElapsedTime(&ms, a, b)); if (ms < best) best = ms;
    }
    double muls = (double)blocks * threads * ITERS * CH * (which == 2 ? 4 : 1);
    printf("%s: %.3f ms  %.2f T mul/s\n", which == 0 ? "lds_split_tables" : which == 1 ? "gmem_split_tables" : "vperm_quads", best, muls / best / 1e9);
  }
  return 0;
}
