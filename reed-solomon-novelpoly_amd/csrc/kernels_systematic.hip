// reconstruct_from_systematic (mod.rs:247-285) on the device: the message is
// the first k shards read column-wise -- out byte pair 2(c*k + j) is symbol c
// of shard j -- so this is a transpose of a k x syms matrix of 16-bit symbols,
// no field arithmetic.  HBM-bound: a workgroup moves a 64 x 64 symbol tile
// through LDS so that both the row reads (shard j, 64 symbols = 128 B) and the
// column writes (message column c, 64 symbols = 128 B) are contiguous.
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

}  // namespace

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

}  // namespace np
