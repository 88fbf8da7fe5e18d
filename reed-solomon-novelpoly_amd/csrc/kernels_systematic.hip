// reconstruct_from_systematic (mod.rs:247-285) on the device: the message is
// the first k shards read column-wise -- out byte pair 2(c*k + j) is symbol c
// of shard j -- so this is a transpose of a k x syms matrix of 16-bit symbols,
// no field arithmetic.  HBM-bound: a workgroup moves a 64 x 64 symbol tile
// through LDS so that both the row reads (shard j, 64 symbols = 128 B) and the
// column writes (message column c, 64 symbols = 128 B) are contiguous.
#include <algorithm>

#include "device_common.hpp"
#include "launchers.hpp"

namespace np {
namespace {

constexpr int kSysTile = 64;

__global__ __launch_bounds__(256) void k_systematic(const uint8_t* shards, size_t shard_len, size_t bstride,
                                                    uint32_t k, uint32_t syms, uint8_t* out, size_t ostride,
                                                    uint32_t ctiles, uint32_t jtiles) {
  __shared__ uint16_t t[kSysTile][kSysTile + 1];
  const uint32_t per_b = ctiles * jtiles;
  const uint32_t b = blockIdx.x / per_b, rest = blockIdx.x % per_b;
  const uint32_t j0 = (rest / ctiles) * kSysTile, c0 = (rest % ctiles) * kSysTile;
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  const uint8_t* src = shards + static_cast<size_t>(b) * bstride;
  // rows j0 + w + 4i, symbols c0 + lane (big-endian pairs copied as they are)
  for (uint32_t i = 0; i < kSysTile / 4; ++i) {
    const uint32_t j = j0 + w + 4 * i, c = c0 + lane;
    uint16_t v = 0;
    if (j < k && c < syms) {
      const uint8_t* p = src + static_cast<size_t>(j) * shard_len + 2 * static_cast<size_t>(c);
      v = static_cast<uint16_t>(p[0] | (p[1] << 8));
    }
    t[w + 4 * i][lane] = v;
  }
  __syncthreads();
  uint8_t* dst = out + static_cast<size_t>(b) * ostride;
  // message columns c0 + w + 4i, symbols j0 + lane
  for (uint32_t i = 0; i < kSysTile / 4; ++i) {
    const uint32_t c = c0 + w + 4 * i, j = j0 + lane;
    if (j < k && c < syms) {
      const uint16_t v = t[lane][w + 4 * i];
      uint8_t* p = dst + (static_cast<size_t>(c) * k + j) * 2;
      p[0] = static_cast<uint8_t>(v);
      p[1] = static_cast<uint8_t>(v >> 8);
    }
  }
}


// Row copies between device memory and host memory mapped into the device
// address space (pinned: hipHostMalloc, torch's pin_memory, hipHostRegister);
// np_reconstruct_batch_host's gather of the present rows: dst[b][v] =
// src[b][v] (row_bytes each) for b < count, v < rows, skipping rows whose
// present flag (present[b * n + v], when given) is 0.  Absent rows of dst are
// left as they are: the reconstruct kernels never read them (the reference
// replaces them by zeros, inc_reconstruct.rs:61-85).  One wave per 4 KiB chunk
// of a row, a few persistent workgroups: 32 of them already read host memory
// at the PCIe rate (tools/microbench/h2d_gather.hip), and a small grid stays
// resident next to the decode kernels of the other pipeline streams instead
// of queueing behind them.
constexpr uint32_t kXferWaves = 4;
constexpr size_t kXferChunk = 4096;

__global__ __launch_bounds__(64 * kXferWaves) void k_copy_rows(const uint8_t* __restrict__ src, size_t sstride,
                                                              uint8_t* __restrict__ dst, size_t dstride,
                                                              size_t row_bytes, const uint8_t* __restrict__ present,
                                                              uint32_t n, uint32_t rows, size_t chunks, size_t total) {
  const uint32_t lane = threadIdx.x & 63;
  const size_t waves = static_cast<size_t>(gridDim.x) * kXferWaves;
  const uintptr_t al = reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst) | sstride | dstride | row_bytes;
  const bool vec = (al & 15) == 0, vec4 = (al & 3) == 0;
  for (size_t u = static_cast<size_t>(blockIdx.x) * kXferWaves + (threadIdx.x >> 6); u < total; u += waves) {
    const size_t r = u / chunks, ch = u - r * chunks;
    const size_t b = r / rows, v = r - b * rows;
    if (present && !present[b * n + v]) continue;
    const size_t off = ch * kXferChunk, len = row_bytes - off < kXferChunk ? row_bytes - off : kXferChunk;
    const uint8_t* s = src + b * sstride + v * row_bytes + off;
    uint8_t* d = dst + b * dstride + v * row_bytes + off;
    if (vec) {
      const uint4* s4 = reinterpret_cast<const uint4*>(s);
      uint4* d4 = reinterpret_cast<uint4*>(d);
      const size_t q = len / 16;
      if (q == 256) {  // a whole chunk: four 1 KiB loads in flight per wave
        const uint4 x0 = s4[lane], x1 = s4[lane + 64], x2 = s4[lane + 128], x3 = s4[lane + 192];
        d4[lane] = x0;
        d4[lane + 64] = x1;
        d4[lane + 128] = x2;
        d4[lane + 192] = x3;
      } else {
        for (size_t i = lane; i < q; i += 64) d4[i] = s4[i];
      }
    } else if (vec4) {  // e.g. rows of 19,532 bytes (the reference bench's 10 MB at k = 512)
      const uint32_t* s1 = reinterpret_cast<const uint32_t*>(s);
      uint32_t* d1 = reinterpret_cast<uint32_t*>(d);
      const size_t q = len / 4;
      size_t i = lane;
      for (; i + 192 < q; i += 256) {  // four 256-byte loads in flight per wave
        const uint32_t x0 = s1[i], x1 = s1[i + 64], x2 = s1[i + 128], x3 = s1[i + 192];
        d1[i] = x0;
        d1[i + 64] = x1;
        d1[i + 128] = x2;
        d1[i + 192] = x3;
      }
      for (; i < q; i += 64) d1[i] = s1[i];
    } else {
      for (size_t i = lane; i < len; i += 64) d[i] = s[i];
    }
  }
}

// np_reconstruct_batch_host's packed present rows (engine.cpp, host-memory
// pipeline): host threads pack the present rows of a sub-batch one after the
// other into pinned staging (row j at src + j * row_bytes) with the device
// offset of each (dst_off[j] = b * dstride + v * row_bytes), one DMA brings
// both over, and this kernel puts every row in its place of the n-row device
// layout (HBM to HBM).  One wave per 4 KiB piece of a row.
__global__ __launch_bounds__(64 * kXferWaves) void k_expand_rows(const uint8_t* __restrict__ src,
                                                                const uint64_t* __restrict__ dst_off,
                                                                uint8_t* __restrict__ dst, size_t row_bytes,
                                                                size_t chunks, size_t total) {
  const uint32_t lane = threadIdx.x & 63;
  const size_t waves = static_cast<size_t>(gridDim.x) * kXferWaves;
  for (size_t u = static_cast<size_t>(blockIdx.x) * kXferWaves + (threadIdx.x >> 6); u < total; u += waves) {
    const size_t j = u / chunks, ch = u - j * chunks;
    const size_t off = ch * kXferChunk, len = row_bytes - off < kXferChunk ? row_bytes - off : kXferChunk;
    const uint8_t* s = src + j * row_bytes + off;
    uint8_t* d = dst + dst_off[j] + off;
    const uintptr_t al = reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d) | len;
    if ((al & 15) == 0) {
      const uint4* s4 = reinterpret_cast<const uint4*>(s);
      uint4* d4 = reinterpret_cast<uint4*>(d);
      const size_t q = len / 16;
      if (q == 256) {
        const uint4 x0 = s4[lane], x1 = s4[lane + 64], x2 = s4[lane + 128], x3 = s4[lane + 192];
        d4[lane] = x0;
        d4[lane + 64] = x1;
        d4[lane + 128] = x2;
        d4[lane + 192] = x3;
      } else {
        for (size_t i = lane; i < q; i += 64) d4[i] = s4[i];
      }
    } else if ((al & 3) == 0) {
      const uint32_t* s1 = reinterpret_cast<const uint32_t*>(s);
      uint32_t* d1 = reinterpret_cast<uint32_t*>(d);
      for (size_t i = lane; i < len / 4; i += 64) d1[i] = s1[i];
    } else {  // rows are whole symbols: 2-byte pieces
      const uint16_t* s1 = reinterpret_cast<const uint16_t*>(s);
      uint16_t* d1 = reinterpret_cast<uint16_t*>(d);
      for (size_t i = lane; i < len / 2; i += 64) d1[i] = s1[i];
    }
  }
}

}  // namespace

hipError_t launch_expand_rows(const uint8_t* src, const uint64_t* dst_off, uint8_t* dst, size_t row_bytes,
                              size_t nrows, hipStream_t s) {
  const size_t chunks = (row_bytes + kXferChunk - 1) / kXferChunk, total = nrows * chunks;
  if (total == 0) return hipSuccess;
  if (row_bytes & 1) return hipErrorInvalidValue;
  const size_t grid = std::min<size_t>((total + kXferWaves - 1) / kXferWaves, 4096);
  k_expand_rows<<<static_cast<uint32_t>(grid), 64 * kXferWaves, 0, s>>>(src, dst_off, dst, row_bytes, chunks, total);
  return hipGetLastError();
}

hipError_t launch_systematic(const uint8_t* shards, size_t shard_len, size_t bstride, uint32_t k, size_t batch,
                             uint8_t* out, size_t ostride, hipStream_t s) {
  const size_t syms = shard_len / 2;
  if (syms == 0 || batch == 0 || k == 0) return hipSuccess;
  const size_t ctiles = (syms + kSysTile - 1) / kSysTile, jtiles = (k + kSysTile - 1) / kSysTile;
  const size_t blocks = batch * ctiles * jtiles;
  if (blocks > 0x7fffffffu || syms > 0xffffffffu) return hipErrorInvalidValue;
  k_systematic<<<static_cast<uint32_t>(blocks), 256, 0, s>>>(shards, shard_len, bstride, k,
                                                              static_cast<uint32_t>(syms), out, ostride,
                                                              static_cast<uint32_t>(ctiles),
                                                              static_cast<uint32_t>(jtiles));
  return hipGetLastError();
}

hipError_t launch_copy_rows(const uint8_t* src, size_t sstride, uint8_t* dst, size_t dstride, size_t row_bytes,
                            const uint8_t* present, uint32_t n, uint32_t rows, size_t count, uint32_t blocks,
                            hipStream_t s) {
  const size_t chunks = (row_bytes + kXferChunk - 1) / kXferChunk, total = count * rows * chunks;
  if (total == 0) return hipSuccess;
  const size_t grid = std::min<size_t>((total + kXferWaves - 1) / kXferWaves, blocks);
  k_copy_rows<<<static_cast<uint32_t>(grid), 64 * kXferWaves, 0, s>>>(src, sstride, dst, dstride, row_bytes, present,
                                                                     n, rows, chunks, total);
  return hipGetLastError();
}

}  // namespace np
