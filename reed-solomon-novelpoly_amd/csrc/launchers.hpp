// Internal launch API between the host engine (engine.cpp) and the kernels.
// All functions enqueue on `s` and return hipSuccess or the launch error.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "dev_tables.hpp"

namespace np {

struct EncodeArgs {
  const uint8_t* payloads;
  size_t payload_len, payload_stride, batch;
  uint32_t n, k, wanted_n;
  size_t shard_len;  // bytes per shard = 2 * chunks
  uint8_t* shards;
  size_t batch_stride;
};

struct ReconstructArgs {
  const uint8_t* shards;
  size_t shard_len, batch_stride;
  const uint8_t* present;    // device, batch x n
  const uint16_t* locators;  // device, batch x n (log form)
  // fast path: per-payload decode prefix, row multipliers and their tables
  // from launch_prefix_locator (stride prefix_stride(n) bytes); big path: the
  // records of launch_big_records (stride big_record_stride(n))
  const uint8_t* prefix;
  size_t batch;
  uint32_t n, k;
  uint8_t* out;
  size_t out_stride;
  // device, batch x {status, have}: NP_ERR_NEED_MORE_SHARDS (mod.rs:178-180)
  // and the present-row count of a payload with fewer than k present rows
  // (its output is left untouched), {0, have} otherwise.  Written by
  // launch_payload_status or, on the fast path, by launch_prefix_locator;
  // the decode kernels skip the payloads it marks.
  uint32_t* status;
  // Codeword-only callers (np_reconstruct_codewords_batch_dev): the fast path
  // may decode from the shortest row prefix holding k present rows, which
  // equals the reference's output only when the received shards form a
  // codeword.  Never set by the crate-equivalent entry points.
  bool trusted;
#if NP_BOUNDS_CHECK
  // Checked builds only: bytes taken off the end of the out extent the
  // kernels check against (NP_BOUNDS_SELFTEST, the checker's own test).
  uint32_t chk_shrink_out;
#endif
};

// Status code of a payload with fewer than k present rows (include/novelpoly.h).
constexpr uint32_t kStatusNeedMoreShards = 5;

// ---- generic path: any power-of-two n <= 65536, k <= n/2 (kernels_generic.hip) ----
hipError_t launch_encode_generic(const DevTables& T, const EncodeArgs& a, hipStream_t s);
hipError_t launch_reconstruct_generic(const DevTables& T, const ReconstructArgs& a, hipStream_t s);
hipError_t launch_error_locator(const DevTables& T, uint32_t n, const uint8_t* present, size_t batch,
                                uint16_t* locators, hipStream_t s);
// a.status of every payload from its present rows (generic and k = 1024 paths).
hipError_t launch_payload_status(const ReconstructArgs& a, hipStream_t s);
// parity hooks
hipError_t launch_afft(const DevTables& T, uint16_t* data, uint32_t size, uint32_t index, size_t cols,
                       bool inverse, hipStream_t s);
hipError_t launch_walsh(uint16_t* data, uint32_t size, hipStream_t s);
hipError_t launch_mul(const DevTables& T, const uint16_t* a, const uint16_t* m, uint16_t* out, size_t count,
                      hipStream_t s);
hipError_t launch_encode_low(const DevTables& T, const uint16_t* data, uint32_t k, uint16_t* codeword,
                             uint32_t n, size_t cols, hipStream_t s);
hipError_t launch_decode_main(const DevTables& T, uint16_t* codeword, uint32_t upto, const uint8_t* present,
                              const uint16_t* locator, uint32_t n, size_t cols, hipStream_t s);

// ---- reconstruct_from_systematic (kernels_systematic.hip) ----
// out[b][2(c*k + j) .. +2) = shards[b][j][2c .. +2) for j < k, c < shard_len / 2.
hipError_t launch_systematic(const uint8_t* shards, size_t shard_len, size_t bstride, uint32_t k, size_t batch,
                             uint8_t* out, size_t ostride, hipStream_t s);
// dst[b][v] = src[b][v] (row_bytes each) for b < count, v < rows, skipping rows
// with present[b * n + v] == 0 when present is given; src or dst may be host
// memory mapped into the device address space.  `blocks` caps the grid.
hipError_t launch_copy_rows(const uint8_t* src, size_t sstride, uint8_t* dst, size_t dstride, size_t row_bytes,
                            const uint8_t* present, uint32_t n, uint32_t rows, size_t count, uint32_t blocks,
                            hipStream_t s);

// dst + dst_off[j] = row j of src (row_bytes each, rows packed one after the
// other), for j < nrows: the packed present rows of a staged host reconstruct
// put in their n-row device layout.  row_bytes even.
hipError_t launch_expand_rows(const uint8_t* src, const uint64_t* dst_off, uint8_t* dst, size_t row_bytes,
                              size_t nrows, hipStream_t s);

// ---- fast path (kernels_fast.hip) ----
// Returns true if a specialised kernel serves (n, k).
bool fast_encode_supported(uint32_t n, uint32_t k);
bool fast_reconstruct_supported(uint32_t n, uint32_t k);
hipError_t launch_encode_fast(const DevTables& T, const EncodeArgs& a, hipStream_t s);
hipError_t launch_reconstruct_fast(const DevTables& T, const ReconstructArgs& a, hipStream_t s);
// Per payload: the rows to decode from (k rows when all k systematic rows are
// present -- a copy --, otherwise all n; with a.trusted also the 2k-row
// prefix when it holds k present rows), the folded erasure locator over them
// as row multipliers with their v_perm tables for the fast reconstruct kernel
// (a.prefix), and a.status; with a.locators set, the caller's locators over
// all n rows instead.  `out` holds batch * prefix_stride(n, k) bytes.
size_t prefix_stride(uint32_t n, uint32_t k);
hipError_t launch_prefix_locator(const DevTables& T, const ReconstructArgs& a, uint8_t* out, hipStream_t s);

// ---- k in {8, 16, 32} (kernels_small.hip), served through the fast-path entry
// points above (the same per-payload records from launch_prefix_locator) ----
bool small_encode_supported(uint32_t n, uint32_t k);       // 2k <= n <= 8k
bool small_reconstruct_supported(uint32_t n, uint32_t k);  // n / k in {2, 4, 8}
hipError_t launch_encode_small(const DevTables& T, const EncodeArgs& a, hipStream_t s);
hipError_t launch_reconstruct_small(const DevTables& T, const ReconstructArgs& a, hipStream_t s);

// ---- k = 512, 1024 (kernels_big.hip): per-workgroup scratch, launches split to fit it ----
bool big_encode_supported(uint32_t n, uint32_t k);
bool big_reconstruct_supported(uint32_t n, uint32_t k);  // n / k in {2, 4, 8}
size_t big_encode_scratch_per_tile(uint32_t k);
// scratch slots a launch of the (n, k) encode / reconstruct instance uses at most (multiple of 8)
size_t big_resident_slots(int device, uint32_t n, uint32_t k, bool reconstruct);
size_t big_reconstruct_scratch_per_tile(uint32_t n, uint32_t k);
// Per-payload records (status, mode, row multipliers, present flags) of the
// big reconstruct, big_record_stride(n) bytes each, into `records`; the
// reconstruct launch reads them through a.prefix.
size_t big_record_stride(uint32_t n);
hipError_t launch_big_records(const DevTables& T, const ReconstructArgs& a, uint8_t* records, hipStream_t s);
hipError_t launch_encode_big(const DevTables& T, const EncodeArgs& a, uint8_t* scratch, size_t scratch_bytes,
                             hipStream_t s);
hipError_t launch_reconstruct_big(const DevTables& T, const ReconstructArgs& a, uint8_t* scratch,
                                  size_t scratch_bytes, hipStream_t s);

}  // namespace np

namespace np {
// Checked builds (device_common.hpp, -DNP_BOUNDS_CHECK=1): the first bounds
// violation record of each instrumented translation unit since the last call
// (out[0] = count), then cleared; hipErrorNotSupported in the product build.
hipError_t bounds_take_generic(uint32_t out[8]);
hipError_t bounds_take_fast(uint32_t out[8]);
hipError_t bounds_take_res(uint32_t out[8]);
hipError_t bounds_take_small(uint32_t out[8]);
hipError_t bounds_take_big(uint32_t out[8]);
hipError_t bounds_take_huge(uint32_t out[8]);

// Raises the dynamic-LDS limit of the kernels that need > 64 KiB (call once per device).
hipError_t configure_generic_kernels();
hipError_t configure_fast_kernels();
hipError_t configure_big_kernels();

// ---- k = 1024 with the whole transform of a 64-column tile resident in the
// workgroup (kernels_res.hip); the decode reads the records of
// launch_prefix_locator.  NP_RES=0 in the environment falls back to the
// scratch kernels (kernels_big.hip) for A/B measurements. ----
bool res_enabled();
bool res_encode_supported(uint32_t n, uint32_t k);
bool res_reconstruct_supported(uint32_t n, uint32_t k);
hipError_t launch_encode_res(const DevTables& T, const EncodeArgs& a, hipStream_t s);
hipError_t launch_reconstruct_res(const DevTables& T, const ReconstructArgs& a, hipStream_t s);
// NP_REC_RES256=1: k = 256 (n = 2k, 4k, 8k) decodes on the resident kernels
// (a 64-column tile, four workgroups per CU) instead of the fast ones.
bool res256_reconstruct(uint32_t n, uint32_t k);
hipError_t configure_res_kernels();

// ---- k = 2048 .. 16384 (kernels_huge.hip): M = k / 1024 resident size-1024
// sub-transforms plus the top levels, through per-tile scratch slots of
// 128 KiB (scratch_per_payload bytes per payload of the slice). ----
bool huge_encode_supported(uint32_t n, uint32_t k);       // n >= 2k, n <= 65536
bool huge_reconstruct_supported(uint32_t n, uint32_t k);  // n / k in {2, 4, 8}
size_t huge_encode_scratch_per_payload(size_t shard_len, uint32_t n, uint32_t k);
size_t huge_reconstruct_scratch_per_payload(size_t shard_len, uint32_t n, uint32_t k);
// Slots of a slice of `batch` payloads, two payloads per tile where the launch
// pairs them (32 columns or fewer): multiples of 128 KiB.
size_t huge_encode_scratch(size_t batch, size_t payload_len, uint32_t n, uint32_t k);
size_t huge_reconstruct_scratch(size_t batch, size_t shard_len, uint32_t n, uint32_t k);
hipError_t launch_encode_huge(const DevTables& T, const EncodeArgs& a, uint8_t* scratch, hipStream_t s);
// side: huge_side_bytes(batch) (per-payload mode bytes, then the 1024-row
// block occupancy words); locators: batch x n u16 (unused when a.locators is set)
constexpr size_t huge_side_bytes(size_t batch) { return (batch + 15) / 16 * 16 + 8 * batch; }
hipError_t launch_reconstruct_huge(const DevTables& T, const ReconstructArgs& a, uint8_t* scratch, uint8_t* mode,
                                   uint16_t* locators, hipStream_t s);
hipError_t configure_huge_kernels();
}  // namespace np
