// Device-side shared definitions for the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "dev_tables.hpp"
#include "launchers.hpp"

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

// ------------------------------------------------------- checked builds ----
// -DNP_BOUNDS_CHECK=1 (`make -C reed-solomon-novelpoly_amd chk` ->
// lib/libnovelpoly_hip_chk.so; never the product library) checks the global
// accesses of the kernels in the window of round 5's probe p11 (DESIGN.md §6:
// k_error_locator, k_prefix_locator / k_locator_records, k_reconstruct_res)
// against the extents their arguments imply.  Each such kernel arms this
// translation unit's extent set at entry (bounds_arm: every workgroup writes
// the same values, computed from its arguments; the checked tests run one
// launch at a time), and every instrumented access goes through bchk: an
// address outside its buffer is counted, the first one recorded (kind, line,
// workgroup, thread, offset, bytes), and redirected to a sink, so that the
// kernel finishes and the host reads the record (np_debug_bounds_check).
// The record is one per code object and device, so checked runs launch one
// kernel at a time (tests/test_gpu_bounds.py: one pipeline stream, no
// concurrent contexts).  Kinds whose extent is empty pass unchecked.  Every kernel of an instrumented
// translation unit arms (or clears) the set at entry, so that no kernel is
// checked against the extents of an earlier launch (round 6: k_big_records
// was, and flagged its own present flags against another launch's batch).
enum BoundsKind : uint32_t {
  kBkShards, kBkPresent, kBkLocators, kBkRecords, kBkOut, kBkStatus, kBkZeros, kBkPayloads, kBkCount
};
struct BoundsSet {
  uint64_t lo[kBkCount], hi[kBkCount];
};
constexpr int kBoundsRecordWords = 8;  // count, kind, line, workgroup, thread, offset lo, offset hi, bytes

}  // namespace np

#ifndef NP_BOUNDS_CHECK
#define NP_BOUNDS_CHECK 0
#endif

namespace np {
namespace {

#if NP_BOUNDS_CHECK
__device__ BoundsSet g_bounds;
__device__ uint32_t g_bounds_viol[kBoundsRecordWords];
__device__ __attribute__((aligned(256))) uint8_t g_bounds_sink[4096];

__device__ __forceinline__ void bounds_arm(const BoundsSet& b) {
  if (threadIdx.x == 0) {
    for (int i = 0; i < kBkCount; ++i) {
      g_bounds.lo[i] = b.lo[i];
      g_bounds.hi[i] = b.hi[i];
    }
  }
  __syncthreads();
}

__device__ __forceinline__ bool bounds_in(uint64_t a, uint64_t bytes, uint32_t kind) {
  const uint64_t lo = g_bounds.lo[kind], hi = g_bounds.hi[kind];
  return hi == 0 || (a >= lo && a + bytes <= hi);
}

// Records the wave's violating lanes (`bad`), the first one in detail.  Called
// behind a wave-uniform branch (a ballot) and straight-line inside: divergent
// control flow next to the kernels' scalar-operand asm made the compiler copy
// VGPRs into SGPRs it cannot.
__device__ __forceinline__ void bounds_record(uint64_t a, uint64_t bytes, uint32_t kind, uint32_t line, bool bad) {
  const uint32_t old = atomicAdd(&g_bounds_viol[0], bad ? 1u : 0u);
  const bool first = bad && old == 0;
  uint32_t* d = first ? g_bounds_viol : reinterpret_cast<uint32_t*>(g_bounds_sink) + 64u * (threadIdx.x & 15u);
  const uint64_t off = a - g_bounds.lo[kind];
  d[1] = kind;
  d[2] = line;
  d[3] = blockIdx.x;
  d[4] = threadIdx.x;
  d[5] = static_cast<uint32_t>(off);
  d[6] = static_cast<uint32_t>(off >> 32);
  d[7] = static_cast<uint32_t>(bytes);
}
#endif

// p if [p, p + bytes) lies in the armed buffer of `kind` (or `alt`, e.g. the
// zero page that stands in for absent rows), else the sink (checked builds).
template <class T>
__device__ __forceinline__ T* bchk(T* p, uint64_t bytes, uint32_t kind, uint32_t line, uint32_t alt = kBkCount) {
#if NP_BOUNDS_CHECK
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const bool bad = bytes != 0 && !bounds_in(a, bytes, kind) && !(alt < kBkCount && bounds_in(a, bytes, alt));
  if (__builtin_amdgcn_ballot_w64(bad)) bounds_record(a, bytes, kind, line, bad);  // wave-uniform branch
  return bad ? reinterpret_cast<T*>(g_bounds_sink) : p;
#else
  (void)bytes, (void)kind, (void)line, (void)alt;
  return p;
#endif
}
// A table index below `size` (checked builds: counted as a records-kind
// violation at offset idx and clamped to 0).
__device__ __forceinline__ uint32_t ichk(uint32_t idx, uint32_t size, uint32_t line) {
#if NP_BOUNDS_CHECK
  const bool bad = idx >= size;
  if (__builtin_amdgcn_ballot_w64(bad)) bounds_record(g_bounds.lo[kBkRecords] + idx, size, kBkRecords, line, bad);
  return bad ? 0u : idx;
#else
  (void)size, (void)line;
  return idx;
#endif
}
// NP_BNOTE: check and record only, for accesses that cannot be redirected
// (buffer loads and stores, which the descriptor bounds anyway, and scalar
// table loads).
#if NP_BOUNDS_CHECK
#define NP_BCHK(p, bytes, kind) ::np::bchk((p), (bytes), (kind), __LINE__)
#define NP_BCHK2(p, bytes, kind, alt) ::np::bchk((p), (bytes), (kind), __LINE__, (alt))
#define NP_ICHK(i, size) ::np::ichk((i), (size), __LINE__)
#define NP_BNOTE(p, bytes, kind) ((void)::np::bchk((p), (bytes), (kind), __LINE__))
#else  // the product: the expressions themselves (code objects unchanged, tools/isa_same.sh)
#define NP_BCHK(p, bytes, kind) (p)
#define NP_BCHK2(p, bytes, kind, alt) (p)
#define NP_ICHK(i, size) (i)
#define NP_BNOTE(p, bytes, kind) ((void)0)
#endif

// The extents a ReconstructArgs implies (launchers.hpp), plus the zero page.
__device__ __forceinline__ BoundsSet bounds_of(const ReconstructArgs& a, const DevTables& T, size_t rec_stride) {
  BoundsSet b{};
  auto set = [&](uint32_t k, const void* p, uint64_t bytes) {
    if (!p || bytes == 0) return;
    b.lo[k] = reinterpret_cast<uint64_t>(p);
    b.hi[k] = b.lo[k] + bytes;
  };
  const uint64_t n = a.n, nb = a.batch;
  if (nb) {
    set(kBkShards, a.shards, (nb - 1) * a.batch_stride + n * a.shard_len);
    set(kBkPresent, a.present, nb * n);
    set(kBkLocators, a.locators, nb * n * 2);
    set(kBkRecords, a.prefix, nb * rec_stride);
    set(kBkOut, a.out, (nb - 1) * a.out_stride + (a.shard_len / 2) * 2 * static_cast<uint64_t>(a.k));
#if NP_BOUNDS_CHECK
    if (b.hi[kBkOut]) b.hi[kBkOut] -= a.chk_shrink_out;
#endif
    set(kBkStatus, a.status, nb * 8);
  }
  set(kBkZeros, T.zeros, kZeroPageBytes);
  return b;
}

// The extents an EncodeArgs implies: the payloads read, the shard rows below
// wanted_n written.
__device__ __forceinline__ BoundsSet bounds_of_enc(const EncodeArgs& a) {
  BoundsSet b{};
  if (a.batch) {
    b.lo[kBkPayloads] = reinterpret_cast<uint64_t>(a.payloads);
    b.hi[kBkPayloads] = b.lo[kBkPayloads] + (a.batch - 1) * a.payload_stride + a.payload_len;
    b.lo[kBkShards] = reinterpret_cast<uint64_t>(a.shards);
    b.hi[kBkShards] = b.lo[kBkShards] + (a.batch - 1) * a.batch_stride + static_cast<uint64_t>(a.wanted_n) * a.shard_len;
  }
  return b;
}

__device__ __forceinline__ BoundsSet bounds_for(const EncodeArgs& a, const DevTables&) { return bounds_of_enc(a); }
__device__ __forceinline__ BoundsSet bounds_for(const ReconstructArgs& a, const DevTables& T) {
  return bounds_of(a, T, 0);  // (records of other layouts: unchecked)
}

// Host side of a translation unit: its first violation record since the last
// call (out[0] = count), then cleared.  hipErrorNotSupported in the product.
inline hipError_t bounds_take_tu(uint32_t out[kBoundsRecordWords]) {
#if NP_BOUNDS_CHECK
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_bounds_viol), sizeof(uint32_t) * kBoundsRecordWords);
  static const uint32_t zero[kBoundsRecordWords] = {};
  if (e == hipSuccess) e = hipMemcpyToSymbol(HIP_SYMBOL(g_bounds_viol), zero, sizeof zero);
  return e;
#else
  for (int i = 0; i < kBoundsRecordWords; ++i) out[i] = 0;
  return hipErrorNotSupported;
#endif
}

}  // namespace
}  // namespace np
