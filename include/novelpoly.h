/*
 * novelpoly.h -- C ABI of the MI355X-native novel-polynomial-basis
 * Reed-Solomon engine (drop-in for the encode/reconstruct hot path of
 * paritytech/reed-solomon-novelpoly v2.0.0).
 *
 * Paths cited below are relative to the reference crate
 * /root/reference/reed-solomon-novelpoly/.  Every entry point names the
 * reference interface it replaces.  The reference's own FFI slot for an
 * alternative implementation is src/cxx.rs:23-31 (encode/reconstruct are
 * `unimplemented!()` there); INTEGRATION.md shows the Rust-side binding.
 *
 * Conventions
 *  - plain pointers and sizes only; every buffer is caller-owned;
 *  - host entry points take host memory; `_dev` entry points take device
 *    pointers (hipMalloc'd on the context's device) and a hipStream_t passed
 *    as `void*` and are asynchronous on that stream; NULL is HIP's legacy
 *    null stream (the caller's default stream, e.g. torch's), so work queued
 *    there before the call is ordered before it;
 *  - a context is bound to one GPU; host-API calls on one context are
 *    serialised on its own stream; distinct contexts may be used from
 *    distinct threads;
 *  - status 0 is success, 1..8 mirror `Error` in src/errors.rs:4-28 in
 *    declaration order, >= 100 are engine failures.
 */
#ifndef NOVELPOLY_H
#define NOVELPOLY_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes: src/errors.rs:4-28 ------------------------------------ */
typedef enum np_status {
  NP_OK = 0,
  NP_ERR_WANTED_SHARD_COUNT_TOO_HIGH = 1,        /* Error::WantedShardCountTooHigh(n)          */
  NP_ERR_WANTED_SHARD_COUNT_TOO_LOW = 2,         /* Error::WantedShardCountTooLow(n)           */
  NP_ERR_WANTED_PAYLOAD_SHARD_COUNT_TOO_LOW = 3, /* Error::WantedPayloadShardCountTooLow(k)    */
  NP_ERR_PAYLOAD_SIZE_IS_ZERO = 4,               /* Error::PayloadSizeIsZero                   */
  NP_ERR_NEED_MORE_SHARDS = 5,                   /* Error::NeedMoreShards{have,min,all}        */
  NP_ERR_PARAMETER_MUST_BE_POWER_OF_2 = 6,       /* Error::ParamterMustBePowerOf2{n,k}         */
  NP_ERR_INCONSISTENT_SHARD_LENGTHS = 7,         /* Error::InconsistentShardLengths{first,other}*/
  NP_ERR_EMPTY_SHARD = 8,                        /* Error::EmptyShard                          */
  NP_ERR_INVALID_ARGUMENT = 100, /* NULL pointer, too-small buffer, or a case the reference asserts on */
  NP_ERR_DEVICE = 101,           /* HIP runtime / kernel launch failure                           */
  NP_ERR_ALLOC = 102,            /* device or pinned allocation failed                            */
  NP_ERR_NO_DEVICE = 103         /* no usable gfx950 device                                       */
} np_status;

/* Error payload of the last failing call on this thread (fields as in
 * errors.rs: NeedMoreShards -> {have,min,all}; InconsistentShardLengths ->
 * {first,other,0}; WantedShardCountTooHigh/Low -> {n,0,0};
 * WantedPayloadShardCountTooLow -> {k,0,0}; ParamterMustBePowerOf2 -> {n,k,0};
 * NP_ERR_DEVICE / NP_ERR_ALLOC -> {hipError_t, call-site id, 0}: the id is the
 * engine line of the HIP call that returned the error, 0 if not recorded). */
void np_last_error_detail(size_t out[3]);
/* The HIP call behind the last NP_ERR_DEVICE / NP_ERR_ALLOC on this thread, as
 * text ("engine.cpp:<line> <call>: <hipError name>"; "" before any).  An
 * asynchronous kernel or copy fault is reported by the synchronisation that saw
 * it; with NP_SYNC_EACH set in the environment the host batch calls synchronise
 * after every step, so that the step itself is named. */
const char* np_last_error_site(void);
/* Human readable message mirroring the thiserror strings of errors.rs. */
const char* np_status_message(int status);

/* ---- parameters: src/novel_poly_basis/mod.rs:24-115, src/util.rs:1-42 ---- */
typedef struct np_code_params {
  size_t n;        /* power of two, total symbols per codeword   (CodeParams::n, mod.rs:80) */
  size_t k;        /* power of two, data symbols per codeword    (CodeParams::k, mod.rs:85) */
  size_t wanted_n; /* shards actually produced                   (CodeParams.wanted_n)      */
} np_code_params;

/* util.rs:40 recoverablity_subset_size */
size_t np_recoverability_subset_size(size_t n_wanted_shards);
/* mod.rs:43-61 CodeParams::derive_parameters */
int np_derive_parameters(size_t n_wanted, size_t k_wanted, np_code_params* out);
/* mod.rs:109-115 ReedSolomon::new validation (fails only if neither n nor k is a power of 2) */
int np_params_new(size_t n, size_t k, size_t wanted_n, np_code_params* out);
/* mod.rs:102-107 ReedSolomon::shard_len */
size_t np_shard_len(const np_code_params* params, size_t payload_size);
/* mod.rs:64-71 CodeParams::is_faster8 analogue: 1 if specialised GPU kernels serve both
   directions of (n,k) for 1 MiB payloads (fast, small, resident, huge or big kernels) */
int np_is_fast_path(const np_code_params* params);

/* ---- context ------------------------------------------------------------- */
typedef struct np_ctx np_ctx;
/* Creates a context on HIP device `device` (-1 = current), uploads the field
 * tables (inc_gen_field_tables.rs:29-72) and skew factors (inc_afft.rs:386-445). */
int np_ctx_create(int device, np_ctx** out);
void np_ctx_destroy(np_ctx* ctx);
/* Checked builds only (lib/libnovelpoly_hip_chk.so, -DNP_BOUNDS_CHECK=1;
 * DESIGN.md §6): waits for the device, then returns in out[0] the number of
 * global accesses since the last call that fell outside the buffers the
 * kernels' arguments imply (error locator, prefix locator / locator records,
 * the encode and reconstruct kernels' payload, row and output accesses), and
 * in out[1..7] the first one (buffer kind, kernel
 * source line, workgroup, thread, byte offset lo/hi, width); clears them.
 * NP_ERR_INVALID_ARGUMENT in the product build. */
int np_debug_bounds_check(np_ctx* ctx, uint32_t out[8]);

/* The in-place pin registry of the host batch calls (NP_PAGEABLE=pin):
 * out[0] = page ranges registered now (0 between calls), out[1] =
 * hipHostUnregister calls the runtime refused since the process started. */
void np_pin_registry_stats(size_t out[2]);

/* The context's stream (hipStream_t as void*). */
void* np_ctx_stream(np_ctx* ctx);
int np_ctx_device(np_ctx* ctx);
/* Waits for all work queued on the context's stream and on the device's
 * legacy null stream (the `_dev` calls given a NULL stream). */
int np_ctx_synchronize(np_ctx* ctx);

/* ---- host-memory API (the crate's surface) -------------------------------- */
/* encode.rs:6-11 `encode(bytes, n_min)`: derives (n,k) from n_min like the crate.
 * shards_out: wanted_n rows of `shard_len` bytes each, row-major; shard_len must
 * equal np_shard_len(params, payload_len). */
int np_encode(np_ctx* ctx, const uint8_t* payload, size_t payload_len, size_t n_min, uint8_t* shards_out,
              size_t shard_len);
/* mod.rs:117-157 ReedSolomon::encode with explicit parameters. */
int np_rs_encode(np_ctx* ctx, const np_code_params* params, const uint8_t* payload, size_t payload_len,
                 uint8_t* shards_out, size_t shard_len);
/* reconstruct.rs:4-9 `reconstruct(received, validator_count)`.
 * shards[i] == NULL marks a missing shard; shard_lens[i] in bytes (odd lengths
 * are zero padded like WrappedShard::new, wrapped_shard.rs:33-39).
 * out receives shard_symbols*2*k bytes (payload zero padded; the caller
 * truncates, as with the crate).  *out_len is set on success. */
int np_reconstruct(np_ctx* ctx, const uint8_t* const* shards, const size_t* shard_lens, size_t n_received,
                   size_t validator_count, uint8_t* out, size_t out_capacity, size_t* out_len);
/* mod.rs:162-239 ReedSolomon::reconstruct with explicit parameters. */
int np_rs_reconstruct(np_ctx* ctx, const np_code_params* params, const uint8_t* const* shards,
                      const size_t* shard_lens, size_t n_received, uint8_t* out, size_t out_capacity,
                      size_t* out_len);
/* mod.rs:247-285 ReedSolomon::reconstruct_from_systematic (first k shards, all present). */
int np_rs_reconstruct_from_systematic(np_ctx* ctx, const np_code_params* params, const uint8_t* const* chunks,
                                      const size_t* chunk_lens, size_t n_chunks, uint8_t* out,
                                      size_t out_capacity, size_t* out_len);

/* ---- device-resident batch API (what bench.py measures) ------------------- */
/* Encodes `batch` independent payloads of equal length.
 *   d_payloads: payload b at d_payloads + b*payload_stride (bytes)
 *   d_shards  : shard v of payload b at d_shards + b*batch_stride + v*shard_len
 *               (batch_stride >= wanted_n*shard_len)
 * Equivalent to calling ReedSolomon::encode (mod.rs:117-157) per payload. */
int np_encode_batch_dev(np_ctx* ctx, const np_code_params* params, const uint8_t* d_payloads,
                        size_t payload_len, size_t payload_stride, size_t batch, uint8_t* d_shards,
                        size_t batch_stride, void* stream);
/* Reconstructs `batch` payloads; every payload has its own erasure pattern.
 *   d_shards : shard v of payload b at d_shards + b*batch_stride + v*shard_len (n rows;
 *              rows of missing shards are never read)
 *   present  : HOST array, present[b*n + v] != 0 if shard v of payload b was received
 *   d_out    : payload b at d_out + b*out_stride, (shard_len/2)*2k bytes
 * Fails with NP_ERR_NEED_MORE_SHARDS (host-side check) like mod.rs:178-180. */
int np_reconstruct_batch_dev(np_ctx* ctx, const np_code_params* params, const uint8_t* d_shards,
                             size_t shard_len, size_t batch_stride, const uint8_t* present, size_t batch,
                             uint8_t* d_out, size_t out_stride, void* stream);
/* Per-payload outcome of a device batch reconstruct (device memory, one entry
 * per payload): status = NP_OK, or NP_ERR_NEED_MORE_SHARDS when the payload
 * has fewer than k present shards (mod.rs:178-180; the error's fields are
 * {have, min = k, all = n}); have = its present-shard count.  A payload marked
 * NeedMoreShards is not decoded: its output bytes are left untouched. */
typedef struct np_payload_status {
  int32_t status;
  uint32_t have;
} np_payload_status;

/* Same as np_reconstruct_batch_dev with the present mask on the device
 * (d_present: batch rows of n bytes) and optionally the erasure locators already
 * computed (d_locators: batch rows of n uint16, see np_error_locator_dev).
 * d_locators == NULL: the locators are computed on the device by a per-payload
 * kernel.  Every payload is decoded from all its present shards, as the
 * reference (inc_reconstruct.rs:61-85), or copied when its k systematic shards
 * are all present (inc_reconstruct.rs:46-50) -- bit-exact for any received
 * bytes.  d_status (device, batch entries, may be NULL) receives each
 * payload's np_payload_status; the NeedMoreShards check runs on the device. */
int np_reconstruct_batch_dev3(np_ctx* ctx, const np_code_params* params, const uint8_t* d_shards,
                              size_t shard_len, size_t batch_stride, const uint8_t* d_present,
                              const uint16_t* d_locators, size_t batch, uint8_t* d_out, size_t out_stride,
                              np_payload_status* d_status, void* stream);
/* The 0.1.0 entry: np_reconstruct_batch_dev3 with d_status = NULL (kept with
 * its original argument list, so callers built against 0.1.0 stay correct). */
int np_reconstruct_batch_dev2(np_ctx* ctx, const np_code_params* params, const uint8_t* d_shards,
                              size_t shard_len, size_t batch_stride, const uint8_t* d_present,
                              const uint16_t* d_locators, size_t batch, uint8_t* d_out, size_t out_stride,
                              void* stream);
/* OPT-IN, not crate-equivalent: for callers whose received shards are known
 * to be an unmodified codeword (e.g. verified by a Merkle proof upstream).
 * Like np_reconstruct_batch_dev3 with d_locators = NULL, but a payload whose
 * first 2k shards hold k present ones may be decoded from those 2k rows only
 * (n = 4k shapes of the fast path).  That equals the reference's output only
 * when the shards form a codeword; for other bytes the reference's decode
 * (a linear map of every present shard) differs. */
int np_reconstruct_codewords_batch_dev(np_ctx* ctx, const np_code_params* params, const uint8_t* d_shards,
                                       size_t shard_len, size_t batch_stride, const uint8_t* d_present,
                                       size_t batch, uint8_t* d_out, size_t out_stride,
                                       np_payload_status* d_status, void* stream);
/* mod.rs:247-285 ReedSolomon::reconstruct_from_systematic for `batch` payloads
 * whose first k shards are all present: d_shards as for np_encode_batch_dev
 * (batch_stride >= k*shard_len, only rows 0..k-1 are read), d_out as for
 * np_reconstruct_batch_dev.  A transpose-gather, no field arithmetic. */
int np_reconstruct_from_systematic_batch_dev(np_ctx* ctx, const np_code_params* params, const uint8_t* d_shards,
                                             size_t shard_len, size_t batch_stride, size_t batch, uint8_t* d_out,
                                             size_t out_stride, void* stream);
/* inc_reconstruct.rs:90-113 eval_error_polynomial for `batch` erasure patterns
 * (d_present: batch rows of n bytes, nonzero = present).  Writes the first n
 * entries of each 65536-entry locator (log form) to d_locators (batch x n). */
int np_error_locator_dev(np_ctx* ctx, size_t n, const uint8_t* d_present, size_t batch, uint16_t* d_locators,
                         void* stream);

/* ---- host-memory batch API: the caller's buffers in host memory ----------
 * Same layouts as the device batch API, host pointers.  The batch is
 * pipelined over several streams in sub-batches (H2D, kernel, D2H overlap);
 * pinned host memory (hipHostMalloc / hipHostRegister) gives full overlap.
 * Reconstruct copies only the shard rows the kernels read (the k systematic
 * rows when every payload of the batch has them all, else all n rows).  Both
 * calls return when the outputs are in host memory. */
int np_encode_batch_host(np_ctx* ctx, const np_code_params* params, const uint8_t* payloads, size_t payload_len,
                         size_t payload_stride, size_t batch, uint8_t* shards, size_t batch_stride);
int np_reconstruct_batch_host(np_ctx* ctx, const np_code_params* params, const uint8_t* shards, size_t shard_len,
                              size_t batch_stride, const uint8_t* present, size_t batch, uint8_t* out,
                              size_t out_stride);

/* ---- multi-GPU: one batch over several devices ------------------------------
 * payloads are independent, so `batch` splits into contiguous
 * ranges, one per context (np_batch_split: the first batch % nctx ranges hold
 * one payload more), with no exchange between devices and no collective.  One
 * host thread per context drives its range on that context's stream; every
 * call returns when all ranges are done (the first failing status is
 * returned, its detail in np_last_error_detail).  Replaces the caller-side
 * loop over payloads (mod.rs:117-239) across GPUs. */
void np_batch_split(size_t batch, size_t ndev, size_t i, size_t* begin, size_t* count);
/* Device memory: d_payloads[i] / d_shards[i] / d_present[i] / d_out[i] /
 * d_status[i] (d_status may be NULL) are device i's buffers holding its range,
 * laid out as in np_encode_batch_dev / np_reconstruct_batch_dev3 (payload
 * np_batch_split(...).begin of the batch at index 0). */
int np_encode_batch_multi(np_ctx* const* ctxs, size_t nctx, const np_code_params* params,
                          const uint8_t* const* d_payloads, size_t payload_len, size_t payload_stride, size_t batch,
                          uint8_t* const* d_shards, size_t batch_stride);
int np_reconstruct_batch_multi(np_ctx* const* ctxs, size_t nctx, const np_code_params* params,
                               const uint8_t* const* d_shards, size_t shard_len, size_t batch_stride,
                               const uint8_t* const* d_present, size_t batch, uint8_t* const* d_out,
                               size_t out_stride, np_payload_status* const* d_status);
/* Host memory: one whole batch as in np_encode_batch_host / np_reconstruct_batch_host,
 * each device copying and computing its range. */
int np_encode_batch_host_multi(np_ctx* const* ctxs, size_t nctx, const np_code_params* params,
                               const uint8_t* payloads, size_t payload_len, size_t payload_stride, size_t batch,
                               uint8_t* shards, size_t batch_stride);
int np_reconstruct_batch_host_multi(np_ctx* const* ctxs, size_t nctx, const np_code_params* params,
                                    const uint8_t* shards, size_t shard_len, size_t batch_stride,
                                    const uint8_t* present, size_t batch, uint8_t* out, size_t out_stride);

/* ---- low-level parity hooks (device pointers, `cols` independent columns) ----
 * data layout: column c, position i at d_data[c*size + i] (uint16, plain values). */
/* inc_afft.rs:267-332 afft */
int np_afft_dev(np_ctx* ctx, uint16_t* d_data, size_t size, size_t index, size_t cols, void* stream);
/* inc_afft.rs:139-214 inverse_afft */
int np_inverse_afft_dev(np_ctx* ctx, uint16_t* d_data, size_t size, size_t index, size_t cols, void* stream);
/* inc_log_mul.rs:92-114 walsh, in place, one transform of `size` values */
int np_walsh_dev(np_ctx* ctx, uint16_t* d_data, size_t size, void* stream);
/* inc_log_mul.rs:42-49 mul: d_out[i] = d_a[i] * EXP[d_m[i]] (log-form multiplier) */
int np_mul_dev(np_ctx* ctx, const uint16_t* d_a, const uint16_t* d_m, uint16_t* d_out, size_t count,
               void* stream);
/* inc_encode.rs:15-48 encode_low on `cols` codewords: d_data cols x k, d_codeword cols x n */
int np_encode_low_dev(np_ctx* ctx, const uint16_t* d_data, size_t k, uint16_t* d_codeword, size_t n,
                      size_t cols, void* stream);
/* inc_reconstruct.rs:61-85 decode_main on `cols` codewords sharing one erasure pattern:
 * d_codeword cols x n (in/out), d_present n bytes, d_locator n uint16 */
int np_decode_main_dev(np_ctx* ctx, uint16_t* d_codeword, size_t recover_up_to, const uint8_t* d_present,
                       const uint16_t* d_locator, size_t n, size_t cols, void* stream);

/* Engine build/version string. */
const char* np_version(void);

#ifdef __cplusplus
}
#endif
#endif /* NOVELPOLY_H */
