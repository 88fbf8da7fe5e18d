// Device-side shared definitions for the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "dev_tables.hpp"

namespace np {

constexpr uint32_t kQ = 65535u;

// a * g^m, inc_log_mul.rs:42-49 (table gathers; generic path only).
__device__ __forceinline__ uint16_t gf_mul_log(const DevTables& T, uint32_t a, uint32_t m) {
  if (a == 0) return 0;
  const uint32_t s = static_cast<uint32_t>(T.log[a]) + m;
  return T.exp[(s & 0xffffu) + (s >> 16)];
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Big-endian symbol from bytes (inc_encode.rs:193-196: odd tail -> low byte 0).
__device__ __forceinline__ uint16_t be_sym(const uint8_t* p, size_t off, size_t len) {
  const uint32_t hi = off < len ? p[off] : 0u;
  const uint32_t lo = off + 1 < len ? p[off + 1] : 0u;
  return static_cast<uint16_t>((hi << 8) | lo);
}

}  // namespace np
