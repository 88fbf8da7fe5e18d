// Host engine behind the C ABI (include/novelpoly.h): parameter derivation,
// validation with the crate's error behaviour, per-device contexts, staging
// and kernel dispatch.  Mirrors src/novel_poly_basis/mod.rs:24-285 of the
// reference crate; the per-chunk / per-column loops of mod.rs:144-154 and
// :221-236 are replaced by batched GPU kernels.
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/novelpoly.h"
#include "field_tables.hpp"
#include "launchers.hpp"

namespace {

thread_local size_t g_detail[3] = {0, 0, 0};

int fail(int st, size_t a = 0, size_t b = 0, size_t c = 0) {
  g_detail[0] = a;
  g_detail[1] = b;
  g_detail[2] = c;
  return st;
}

bool is_pow2(size_t x) { return x && !(x & (x - 1)); }
size_t next_pow2(size_t x) {
  size_t p = 1;
  while (p < x) p <<= 1;
  return p;
}
size_t prev_pow2(size_t x) {
  size_t p = 1;
  while ((p << 1) <= x) p <<= 1;
  return p;
}

// Device buffer that only grows.
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    // exactly the size asked for (the context scratch is capped by its callers:
    // engine.cpp big_scratch, kBigScratchCap)
    hipError_t e = hipMalloc(&p, bytes);
    if (e == hipSuccess) cap = bytes;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

struct HostBuf {  // pinned staging that only grows
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocDefault);
    if (e == hipSuccess) cap = bytes;
    return e;
  }
  void release() {
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

std::mutex g_cfg_mu;
std::vector<int> g_configured_devices;

}  // namespace

struct np_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  np::DevTables T{};
  std::vector<void*> table_allocs;
  std::mutex mu;  // serialises host-API calls (they share the scratch buffers)
  DevBuf d_in, d_out, d_present;
  HostBuf h_in, h_out;
  // Per-workgroup scratch of the k = 1024 kernels (kernels_big.hip).  Launches
  // on different streams are ordered through big_done so they never share it.
  DevBuf d_big;
  hipEvent_t big_done = nullptr;
  bool big_used = false;
  // Host-memory batch pipeline (np_*_batch_host): per slot a stream and
  // device buffers for one sub-batch; created on first use.
  static constexpr int kPipe = 3;
  hipStream_t pipe_s[kPipe] = {};
  DevBuf pipe_in[kPipe], pipe_out[kPipe];
  DevBuf pipe_pres;  // the present mask of a whole host reconstruct call
  // Pageable host reconstruct: pinned staging per slot for the present rows
  // (gathered by host threads) and for the outputs, and the slot's last event.
  HostBuf pipe_hin[kPipe], pipe_hout[kPipe];
  hipEvent_t pipe_ev[kPipe] = {};
};

namespace {

int dev_err(hipError_t e) {
  if (e == hipSuccess) return NP_OK;
  if (e == hipErrorOutOfMemory) return fail(NP_ERR_ALLOC);
  return fail(NP_ERR_DEVICE, static_cast<size_t>(e));
}

template <class T>
hipError_t upload(np_ctx* c, const std::vector<T>& v, const T** dst) {
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, v.size() * sizeof(T));
  if (e != hipSuccess) return e;
  c->table_allocs.push_back(p);
  e = hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice);
  *dst = static_cast<const T*>(p);
  return e;
}

int check_params(const np_code_params* p) {
  if (!p) return fail(NP_ERR_INVALID_ARGUMENT);
  if (!is_pow2(p->n) && !is_pow2(p->k)) return fail(NP_ERR_PARAMETER_MUST_BE_POWER_OF_2, p->n, p->k);
  // The crate asserts these (inc_encode.rs:166-169, inc_reconstruct.rs:8-11).
  if (!is_pow2(p->n) || !is_pow2(p->k) || 2 * p->k > p->n || p->n > np::kFieldSize || p->wanted_n > p->n)
    return fail(NP_ERR_INVALID_ARGUMENT, p->n, p->k, p->wanted_n);
  return NP_OK;
}

np::EncodeArgs enc_args(const np_code_params* p, const uint8_t* payloads, size_t len, size_t pstride, size_t batch,
                        uint8_t* shards, size_t bstride) {
  np::EncodeArgs a{};
  a.payloads = payloads;
  a.payload_len = len;
  a.payload_stride = pstride;
  a.batch = batch;
  a.n = static_cast<uint32_t>(p->n);
  a.k = static_cast<uint32_t>(p->k);
  a.wanted_n = static_cast<uint32_t>(p->wanted_n);
  a.shard_len = np_shard_len(p, len);
  a.shards = shards;
  a.batch_stride = bstride;
  return a;
}

constexpr size_t kBigScratchCap = size_t(2) << 30;  // bytes of big-kernel scratch per context (k = 2048 decode: 256 slots of 4.9 MiB)

// Big-kernel scratch of `want` bytes (capped), ordered after every earlier
// big launch of this context on any stream.  Caller holds the context lock.
hipError_t big_scratch(np_ctx* c, size_t want, hipStream_t s, uint8_t** out, size_t* bytes) {
  want = std::min(want, kBigScratchCap);
  hipError_t e = hipSuccess;
  if (!c->big_done) e = hipEventCreateWithFlags(&c->big_done, hipEventDisableTiming);
  if (e == hipSuccess && c->big_used) {
    if (want > c->d_big.cap) e = hipEventSynchronize(c->big_done);  // about to free the old buffer
    if (e == hipSuccess) e = hipStreamWaitEvent(s, c->big_done, 0);
  }
  if (e == hipSuccess) e = c->d_big.ensure(want);
  *out = c->d_big.as<uint8_t>();
  *bytes = c->d_big.cap;
  return e;
}

hipError_t big_done(np_ctx* c, hipStream_t s, hipError_t e) {
  if (e != hipSuccess) return e;
  c->big_used = true;
  return hipEventRecord(c->big_done, s);
}

// Scratch slots of a k = 512 / 1024 launch over `tiles` tiles: one per resident workgroup.
size_t big_slots(const np_ctx* c, size_t tiles, uint32_t n, uint32_t k, bool reconstruct) {
  return std::min((tiles + 7) / 8 * 8, np::big_resident_slots(c->device, n, k, reconstruct));
}

// k >= 4096 (and k = 2048 with NP_HUGE=1) on the sub-transform path of
// kernels_huge.hip; NP_HUGE=0 keeps the big / generic kernels (A/B runs).
bool huge_on(uint32_t k) {
  static const int mode = [] {
    const char* e = std::getenv("NP_HUGE");
    return e ? (e[0] == '0' ? 0 : 2) : 1;
  }();
  return mode == 2 || (mode == 1 && k >= 4096);
}

// The kernel family a reconstruct of (n, k, shard_len) runs on, chosen once for
// launch_reconstruct and for rows_needed (which rows the host pipeline ships):
// every family but the generic one has a copy mode that reads only the k
// systematic rows when all of them are present.
enum class RecPath { FastRes, Huge, Big, Generic };

RecPath rec_path(uint32_t n, uint32_t k, size_t shard_len) {
  if (np::fast_reconstruct_supported(n, k) || (np::res_reconstruct_supported(n, k) && np::res_enabled()))
    return RecPath::FastRes;
  if (np::huge_reconstruct_supported(n, k) && huge_on(k) &&
      np::huge_reconstruct_scratch_per_payload(shard_len, n, k) <= kBigScratchCap / 2)
    return RecPath::Huge;
  if (np::big_reconstruct_supported(n, k)) return RecPath::Big;
  return RecPath::Generic;
}

// Caller holds the context lock.
hipError_t launch_encode(np_ctx* c, const np::EncodeArgs& a, hipStream_t s) {
  if (np::fast_encode_supported(a.n, a.k)) return np::launch_encode_fast(c->T, a, s);
  if (np::res_encode_supported(a.n, a.k) && np::res_enabled()) return np::launch_encode_res(c->T, a, s);
  const size_t huge_per = np::huge_encode_scratch_per_payload(a.shard_len, a.n, a.k);
  if (np::huge_encode_supported(a.n, a.k) && huge_on(a.k) && huge_per <= kBigScratchCap) {
    // slices of the batch whose tile slots fit the context scratch
    const size_t per = std::max<size_t>(1, kBigScratchCap / std::max<size_t>(1, huge_per));
    for (size_t b0 = 0; b0 < a.batch; b0 += per) {
      np::EncodeArgs sub = a;
      sub.batch = std::min(per, a.batch - b0);
      sub.payloads = a.payloads + b0 * a.payload_stride;
      sub.shards = a.shards + b0 * a.batch_stride;
      uint8_t* scr = nullptr;
      size_t bytes = 0;
      hipError_t e = big_scratch(c, sub.batch * huge_per, s, &scr, &bytes);
      if (e == hipSuccess) e = np::launch_encode_huge(c->T, sub, scr, s);
      e = big_done(c, s, e);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  if (np::big_encode_supported(a.n, a.k)) {
    const size_t tiles = ((a.payload_len + 2 * a.k - 1) / (2 * a.k) + 255) / 256;
    uint8_t* scr = nullptr;
    size_t bytes = 0;
    hipError_t e = big_scratch(c, big_slots(c, a.batch * tiles, a.n, a.k, false) * np::big_encode_scratch_per_tile(a.k), s, &scr, &bytes);
    if (e == hipSuccess) e = np::launch_encode_big(c->T, a, scr, bytes, s);
    return big_done(c, s, e);
  }
  return np::launch_encode_generic(c->T, a, s);
}

// Payload `b0` onward of a (a slice of the batch; status follows when set).
np::ReconstructArgs slice(const np::ReconstructArgs& a, size_t b0, size_t cnt) {
  np::ReconstructArgs sub = a;
  sub.batch = cnt;
  sub.shards = a.shards + b0 * a.batch_stride;
  sub.present = a.present + b0 * a.n;
  if (a.locators) sub.locators = a.locators + b0 * a.n;
  if (a.status) sub.status = a.status + 2 * b0;
  sub.out = a.out + b0 * a.out_stride;
  return sub;
}

constexpr size_t kStatusBytes = 2 * sizeof(uint32_t);  // per payload (launchers.hpp ReconstructArgs::status)

// a.locators == nullptr: the locators are computed on the device, into the
// ordered context scratch (prefix locators on the fast path, full locators on
// the generic path; fused into the k = 1024 kernels).  a.status == nullptr:
// the per-payload status goes to the context scratch too (payloads with fewer
// than k present rows are still skipped).  Batches larger than the scratch cap
// go in slices.  Caller holds the context lock.
hipError_t launch_reconstruct(np_ctx* c, const np::ReconstructArgs& a, hipStream_t s) {
  const size_t own_status = a.status ? 0 : kStatusBytes;  // scratch bytes per payload for the status
  const RecPath path = rec_path(a.n, a.k, a.shard_len);
  const bool res = !np::fast_reconstruct_supported(a.n, a.k);
  if (path == RecPath::FastRes) {
    // per-payload decode rows + row multipliers and their tables (from the
    // caller's locators when given) and the status, then the decode
    const size_t stride = np::prefix_stride(a.n, a.k);
    const size_t per = std::max<size_t>(1, kBigScratchCap / (stride + own_status));
    for (size_t b0 = 0; b0 < a.batch; b0 += per) {
      np::ReconstructArgs sub = slice(a, b0, std::min(per, a.batch - b0));
      uint8_t* scr = nullptr;
      size_t bytes = 0;
      hipError_t e = big_scratch(c, sub.batch * (stride + own_status), s, &scr, &bytes);
      if (!a.status) sub.status = reinterpret_cast<uint32_t*>(scr + sub.batch * stride);
      if (e == hipSuccess) e = np::launch_prefix_locator(c->T, sub, scr, s);
      sub.prefix = scr;
      if (e == hipSuccess) e = res ? np::launch_reconstruct_res(c->T, sub, s) : np::launch_reconstruct_fast(c->T, sub, s);
      e = big_done(c, s, e);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  const size_t huge_per = np::huge_reconstruct_scratch_per_payload(a.shard_len, a.n, a.k);
  if (path == RecPath::Huge) {
    // per payload: tile slots, mode byte, locators (unless the caller's), status
    const size_t side = 16 + (a.locators ? 0 : 2 * static_cast<size_t>(a.n)) + own_status;
    const size_t per = std::max<size_t>(1, kBigScratchCap / (huge_per + side));
    for (size_t b0 = 0; b0 < a.batch; b0 += per) {
      np::ReconstructArgs sub = slice(a, b0, std::min(per, a.batch - b0));
      uint8_t* scr = nullptr;
      size_t bytes = 0;
      hipError_t e = big_scratch(c, sub.batch * (huge_per + side), s, &scr, &bytes);
      uint8_t* side0 = scr + sub.batch * huge_per;  // huge_per is a multiple of 128 KiB
      uint16_t* loc = reinterpret_cast<uint16_t*>(side0);
      uint8_t* mode = side0 + (a.locators ? 0 : 2 * static_cast<size_t>(a.n) * sub.batch);
      if (!a.status) sub.status = reinterpret_cast<uint32_t*>(mode + (sub.batch + 15) / 16 * 16);
      if (e == hipSuccess) e = np::launch_reconstruct_huge(c->T, sub, scr, mode, loc, s);
      e = big_done(c, s, e);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  if (path == RecPath::Big) {
    // per-payload records (status, locator as row multipliers) for a slice of
    // the batch, then the decode over the resident workgroups' tile scratch
    const size_t tiles = (a.shard_len / 2 + 255) / 256;
    const size_t per_tile = np::big_reconstruct_scratch_per_tile(a.n, a.k);
    const size_t rstride = np::big_record_stride(a.n) + own_status;
    const size_t per = std::max<size_t>(1, kBigScratchCap / 4 / rstride);
    for (size_t b0 = 0; b0 < a.batch; b0 += per) {
      np::ReconstructArgs sub = slice(a, b0, std::min(per, a.batch - b0));
      const size_t rec_bytes = (sub.batch * rstride + 255) / 256 * 256;
      uint8_t* scr = nullptr;
      size_t bytes = 0;
      hipError_t e = big_scratch(c, rec_bytes + big_slots(c, sub.batch * tiles, sub.n, sub.k, true) * per_tile, s, &scr, &bytes);
      if (e == hipSuccess && bytes < rec_bytes + 8 * per_tile) e = hipErrorInvalidValue;
      if (!a.status) sub.status = reinterpret_cast<uint32_t*>(scr + sub.batch * np::big_record_stride(a.n));
      sub.prefix = scr;
      if (e == hipSuccess) e = np::launch_big_records(c->T, sub, scr, s);
      if (e == hipSuccess) e = np::launch_reconstruct_big(c->T, sub, scr + rec_bytes, bytes - rec_bytes, s);
      e = big_done(c, s, e);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  // generic path: the status, and the locators unless the caller gave them,
  // into the ordered context scratch
  const size_t loc_bytes = a.locators ? 0 : a.n * sizeof(uint16_t);
  const size_t per = std::max<size_t>(1, kBigScratchCap / (loc_bytes + own_status + 1));
  for (size_t b0 = 0; b0 < a.batch; b0 += per) {
    np::ReconstructArgs b = slice(a, b0, std::min(per, a.batch - b0));
    uint8_t* scr = nullptr;
    size_t bytes = 0;
    hipError_t e = big_scratch(c, std::max<size_t>(1, b.batch * (loc_bytes + own_status)), s, &scr, &bytes);
    if (!a.status) b.status = reinterpret_cast<uint32_t*>(scr + b.batch * loc_bytes);
    if (e == hipSuccess) e = np::launch_payload_status(b, s);
    if (!a.locators) {
      b.locators = reinterpret_cast<uint16_t*>(scr);
      if (e == hipSuccess) e = np::launch_error_locator(c->T, a.n, b.present, b.batch, reinterpret_cast<uint16_t*>(scr), s);
    }
    if (e == hipSuccess) e = np::launch_reconstruct_generic(c->T, b, s);
    e = big_done(c, s, e);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipStream_t pick(np_ctx* c, void* s) { return s ? static_cast<hipStream_t>(s) : c->stream; }

// Host copy with streaming (non-temporal) stores where the destination allows
// it: the pageable gather and copy-out move tens of MB per call that no CPU
// core reads again, and streaming stores skip the read-for-ownership of every
// destination line (one memory pass fewer per byte).  The caller fences
// (stream_fence) before the copied bytes are handed on.
void stream_copy(uint8_t* dst, const uint8_t* src, size_t len) {
  size_t i = 0;
  if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
    for (; i + 64 <= len; i += 64) {
      const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i));
      const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 16));
      const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 32));
      const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i*>(src + i + 48));
      _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i), a);
      _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 16), b);
      _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 32), c);
      _mm_stream_si128(reinterpret_cast<__m128i*>(dst + i + 48), d);
    }
  }
  if (i < len) std::memcpy(dst + i, src + i, len - i);
}
void stream_fence() { _mm_sfence(); }

// f(i) for i in [0, count) on up to kHostThreads host threads (the calling
// thread is one of them): the host side of the pageable reconstruct's gather
// and copy-out, which move memcpy-sized row pieces.
constexpr unsigned kHostThreads = 16;

template <class F>
void parallel_for(size_t count, F f) {
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const size_t t = std::min<size_t>({count, kHostThreads, hw});
  if (t <= 1) {
    for (size_t i = 0; i < count; ++i) f(i);
    stream_fence();
    return;
  }
  std::vector<std::thread> pool;
  pool.reserve(t - 1);
  for (size_t w = 1; w < t; ++w)
    pool.emplace_back([&, w] {
      for (size_t i = w; i < count; i += t) f(i);
      stream_fence();
    });
  for (size_t i = 0; i < count; i += t) f(i);
  stream_fence();
  for (auto& th : pool) th.join();
}

}  // namespace

extern "C" {

void np_last_error_detail(size_t out[3]) {
  if (!out) return;
  out[0] = g_detail[0];
  out[1] = g_detail[1];
  out[2] = g_detail[2];
}

const char* np_status_message(int st) {
  switch (st) {  // errors.rs:4-28
    case NP_OK: return "ok";
    case NP_ERR_WANTED_SHARD_COUNT_TOO_HIGH: return "Number of wanted shards exceeds max of 2^16";
    case NP_ERR_WANTED_SHARD_COUNT_TOO_LOW: return "Number of wanted shards must be at least 2";
    case NP_ERR_WANTED_PAYLOAD_SHARD_COUNT_TOO_LOW: return "Number of wanted payload shards must be at least 1";
    case NP_ERR_PAYLOAD_SIZE_IS_ZERO: return "Size of the payload is zero";
    case NP_ERR_NEED_MORE_SHARDS: return "Needs more shards to recover";
    case NP_ERR_PARAMETER_MUST_BE_POWER_OF_2: return "Parameters: n and k both must be a power of 2";
    case NP_ERR_INCONSISTENT_SHARD_LENGTHS: return "Shards do have inconsistent lengths";
    case NP_ERR_EMPTY_SHARD: return "Shard is empty";
    case NP_ERR_INVALID_ARGUMENT: return "invalid argument (a case the reference asserts on)";
    case NP_ERR_DEVICE: return "HIP runtime failure";
    case NP_ERR_ALLOC: return "allocation failure";
    case NP_ERR_NO_DEVICE: return "no gfx950 device available";
    default: return "unknown status";
  }
}

const char* np_version(void) { return "novelpoly-mi355x 0.3.0 (gfx950)"; }

size_t np_recoverability_subset_size(size_t n) { return (n ? (n - 1) / 3 : 0) + 1; }

int np_derive_parameters(size_t n_wanted, size_t k_wanted, np_code_params* out) {
  if (!out) return fail(NP_ERR_INVALID_ARGUMENT);
  if (n_wanted < 2) return fail(NP_ERR_WANTED_SHARD_COUNT_TOO_LOW, n_wanted);
  if (k_wanted < 1) return fail(NP_ERR_WANTED_PAYLOAD_SHARD_COUNT_TOO_LOW, k_wanted);
  const size_t k = prev_pow2(k_wanted), n = next_pow2(n_wanted);
  if (n > np::kFieldSize) return fail(NP_ERR_WANTED_SHARD_COUNT_TOO_HIGH, n_wanted);
  out->n = n;
  out->k = k;
  out->wanted_n = n_wanted;
  return NP_OK;
}

int np_params_new(size_t n, size_t k, size_t wanted_n, np_code_params* out) {
  if (!out) return fail(NP_ERR_INVALID_ARGUMENT);
  if (!is_pow2(n) && !is_pow2(k)) return fail(NP_ERR_PARAMETER_MUST_BE_POWER_OF_2, n, k);
  out->n = n;
  out->k = k;
  out->wanted_n = wanted_n;
  return NP_OK;
}

size_t np_shard_len(const np_code_params* p, size_t payload_size) {
  if (!p || p->k == 0) return 0;
  const size_t syms = (payload_size + 1) / 2;
  return ((syms + p->k - 1) / p->k) * 2;
}

// 1 when both directions of (n, k) run specialised kernels (fast / small,
// resident, sub-transform or big), 0 when either falls to the generic
// LOG/EXP-gather kernels.  The sub-transform decode also needs its per-payload
// scratch to fit (very long shards fall back); this answers for shards of
// up to 64 KiB.
int np_is_fast_path(const np_code_params* p) {
  if (!p) return 0;
  const uint32_t n = static_cast<uint32_t>(p->n), k = static_cast<uint32_t>(p->k);
  const bool enc = np::fast_encode_supported(n, k) || (np::res_encode_supported(n, k) && np::res_enabled()) ||
                   (np::huge_encode_supported(n, k) && huge_on(k)) || np::big_encode_supported(n, k);
  // the reconstruct family for a 1 MiB payload (the huge kernels' tile slots
  // depend on the shard length: far longer shards fall to the generic decode)
  return (enc && rec_path(n, k, np_shard_len(p, size_t(1) << 20)) != RecPath::Generic) ? 1 : 0;
}

int np_ctx_create(int device, np_ctx** out) {
  if (!out) return fail(NP_ERR_INVALID_ARGUMENT);
  *out = nullptr;
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess || count == 0) return fail(NP_ERR_NO_DEVICE);
  if (device < 0) {
    if (hipGetDevice(&device) != hipSuccess) return fail(NP_ERR_NO_DEVICE);
  }
  if (device >= count) return fail(NP_ERR_NO_DEVICE, static_cast<size_t>(device));
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess) return fail(NP_ERR_NO_DEVICE);
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) return fail(NP_ERR_NO_DEVICE, static_cast<size_t>(device));
  if (hipSetDevice(device) != hipSuccess) return fail(NP_ERR_DEVICE);
  np_ctx* c = new (std::nothrow) np_ctx();
  if (!c) return fail(NP_ERR_ALLOC);
  c->device = device;
  hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  const np::HostTables& t = np::host_tables();
  if (e == hipSuccess) e = upload(c, t.log, &c->T.log);
  if (e == hipSuccess) e = upload(c, t.exp, &c->T.exp);
  if (e == hipSuccess) e = upload(c, t.skew, &c->T.skew);
  if (e == hipSuccess) e = upload(c, t.skew_add, &c->T.skew_add);
  if (e == hipSuccess) e = upload(c, t.log_walsh, &c->T.log_walsh);
  if (e == hipSuccess) e = upload(c, t.lw_fold, &c->T.lw_fold);
  if (e == hipSuccess) e = upload(c, t.perm_pools, &c->T.perm_pools);
  if (e == hipSuccess) e = upload(c, t.tower_pools, &c->T.tower_pools);
  if (e == hipSuccess) e = upload(c, t.in_pools, &c->T.in_pools);
  if (e == hipSuccess) e = upload(c, t.out_pools, &c->T.out_pools);
  if (e == hipSuccess) e = upload(c, t.tower_full_sub, &c->T.tower_full_sub);
  if (e == hipSuccess) e = upload(c, std::vector<uint8_t>(np::kZeroPageBytes, 0), &c->T.zeros);
  if (e == hipSuccess) {
    std::lock_guard<std::mutex> g(g_cfg_mu);
    if (std::find(g_configured_devices.begin(), g_configured_devices.end(), device) == g_configured_devices.end()) {
      e = np::configure_generic_kernels();
      if (e == hipSuccess) e = np::configure_fast_kernels();
      if (e == hipSuccess) e = np::configure_big_kernels();
      if (e == hipSuccess) e = np::configure_res_kernels();
      if (e == hipSuccess) e = np::configure_huge_kernels();
      if (e == hipSuccess) g_configured_devices.push_back(device);
    }
  }
  if (e != hipSuccess) {
    np_ctx_destroy(c);
    return dev_err(e);
  }
  *out = c;
  return NP_OK;
}

void np_ctx_destroy(np_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  for (void* p : c->table_allocs) (void)hipFree(p);
  c->d_in.release();
  c->d_out.release();
  c->d_present.release();
  c->d_big.release();
  if (c->big_done) (void)hipEventDestroy(c->big_done);
  for (int i = 0; i < np_ctx::kPipe; ++i) {
    if (c->pipe_s[i]) (void)hipStreamSynchronize(c->pipe_s[i]);
    c->pipe_in[i].release();
    c->pipe_out[i].release();
    c->pipe_hin[i].release();
    c->pipe_hout[i].release();
    if (c->pipe_ev[i]) (void)hipEventDestroy(c->pipe_ev[i]);
    if (c->pipe_s[i]) (void)hipStreamDestroy(c->pipe_s[i]);
  }
  c->pipe_pres.release();
  c->h_in.release();
  c->h_out.release();
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

void* np_ctx_stream(np_ctx* c) { return c ? static_cast<void*>(c->stream) : nullptr; }
int np_ctx_device(np_ctx* c) { return c ? c->device : -1; }

int np_ctx_synchronize(np_ctx* c) {
  if (!c) return fail(NP_ERR_INVALID_ARGUMENT);
  (void)hipSetDevice(c->device);
  return dev_err(hipStreamSynchronize(c->stream));
}

// --------------------------------------------------------------- encode ----
int np_rs_encode(np_ctx* c, const np_code_params* p, const uint8_t* payload, size_t len, uint8_t* shards_out,
                 size_t shard_len) {
  if (!c) return fail(NP_ERR_INVALID_ARGUMENT);
  int st = check_params(p);
  if (st) return st;
  if (len == 0) return fail(NP_ERR_PAYLOAD_SIZE_IS_ZERO);  // mod.rs:118-120
  if (!payload || !shards_out || shard_len != np_shard_len(p, len)) return fail(NP_ERR_INVALID_ARGUMENT);
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipSetDevice(c->device);
  const size_t out_bytes = p->wanted_n * shard_len;
  hipError_t e = c->d_in.ensure(len);
  if (e == hipSuccess) e = c->d_out.ensure(std::max<size_t>(out_bytes, 1));
  if (e == hipSuccess) e = c->h_in.ensure(len);
  if (e == hipSuccess) e = c->h_out.ensure(std::max<size_t>(out_bytes, 1));
  if (e != hipSuccess) return dev_err(e);
  std::memcpy(c->h_in.p, payload, len);
  e = hipMemcpyAsync(c->d_in.p, c->h_in.p, len, hipMemcpyHostToDevice, c->stream);
  np::EncodeArgs a = enc_args(p, c->d_in.as<uint8_t>(), len, len, 1, c->d_out.as<uint8_t>(), out_bytes);
  if (e == hipSuccess) e = launch_encode(c, a, c->stream);
  if (e == hipSuccess) e = hipMemcpyAsync(c->h_out.p, c->d_out.p, out_bytes, hipMemcpyDeviceToHost, c->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) return dev_err(e);
  std::memcpy(shards_out, c->h_out.p, out_bytes);
  return NP_OK;
}

int np_encode(np_ctx* c, const uint8_t* payload, size_t len, size_t n_min, uint8_t* shards_out, size_t shard_len) {
  // encode.rs:6-11
  np_code_params p;
  int st = np_derive_parameters(n_min, np_recoverability_subset_size(n_min), &p);
  if (st) return st;
  return np_rs_encode(c, &p, payload, len, shards_out, shard_len);
}

int np_encode_batch_dev(np_ctx* c, const np_code_params* p, const uint8_t* d_payloads, size_t len, size_t pstride,
                        size_t batch, uint8_t* d_shards, size_t bstride, void* stream) {
  if (!c) return fail(NP_ERR_INVALID_ARGUMENT);
  int st = check_params(p);
  if (st) return st;
  if (len == 0) return fail(NP_ERR_PAYLOAD_SIZE_IS_ZERO);
  const size_t sl = np_shard_len(p, len);
  if (!d_payloads || !d_shards || pstride < len || bstride < p->wanted_n * sl) return fail(NP_ERR_INVALID_ARGUMENT);
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipSetDevice(c->device);
  np::EncodeArgs a = enc_args(p, d_payloads, len, pstride, batch, d_shards, bstride);
  return dev_err(launch_encode(c, a, pick(c, stream)));
}

// ------------------------------------------------- host-memory pipeline ----
// the caller's view of encode / reconstruct, buffers in host
// memory.  The batch goes in sub-batches of about kPipeSlotBytes over
// np_ctx::kPipe streams; each sub-batch is H2D -> kernel -> D2H on its
// stream, so the copies of one overlap the kernels and the opposite-direction
// copies of the others (PCIe is full duplex).  Host buffers allocated with
// hipHostMalloc / registered with hipHostRegister are copied by DMA directly;
// pageable ones are staged by the runtime and overlap less.
namespace {

constexpr size_t kPipeSlotBytes = size_t(64) << 20;

hipError_t pipe_init(np_ctx* c) {
  for (int i = 0; i < np_ctx::kPipe; ++i)
    if (!c->pipe_s[i]) {
      hipError_t e = hipStreamCreateWithFlags(&c->pipe_s[i], hipStreamNonBlocking);
      if (e != hipSuccess) return e;
    }
  return hipSuccess;
}

hipError_t pipe_sync(np_ctx* c, hipError_t e) {
  for (int i = 0; i < np_ctx::kPipe; ++i) {
    const hipError_t r = hipStreamSynchronize(c->pipe_s[i]);
    if (e == hipSuccess) e = r;
  }
  return e;
}

// Rows of each payload the reconstruct kernels read: on the fast, resident,
// huge and big paths only the k systematic rows when all of them are present
// (the output is those rows: kernels_fast.hip k_prefix_locator, kernels_huge.hip
// k_huge_records, kernels_big.hip kBigCopy), otherwise -- and on the generic
// path -- all n rows: the reference decodes from every present row
// (inc_reconstruct.rs:61-85).  The path is the one launch_reconstruct takes
// (rec_path), so a generic decode never reads rows that were not shipped.
size_t rows_needed(const np_code_params* p, size_t shard_len, const uint8_t* present, size_t batch) {
  const uint32_t n = static_cast<uint32_t>(p->n), k = static_cast<uint32_t>(p->k);
  if (rec_path(n, k, shard_len) == RecPath::Generic) return p->n;
  for (size_t b = 0; b < batch; ++b) {
    const uint8_t* pr = present + b * p->n;
    for (size_t v = 0; v < p->k; ++v)
      if (!pr[v]) return p->n;
  }
  return p->k;
}

// Workgroups of the present-row gather (launch_copy_rows): 32 read host
// memory at the PCIe rate (tools/microbench/h2d_gather.hip).
constexpr uint32_t kGatherBlocks = 32;

// Device address of [p, p + bytes) when the whole range lies in one pinned host
// allocation mapped into the device address space (hipHostMalloc, torch's
// pin_memory, hipHostRegister), else nullptr (pageable memory).
const uint8_t* mapped_host_range(const uint8_t* p, size_t bytes) {
  if (bytes == 0 || std::getenv("NP_NO_GATHER")) return nullptr;
  hipPointerAttribute_t a0{}, a1{};
  if (hipPointerGetAttributes(&a0, p) != hipSuccess || hipPointerGetAttributes(&a1, p + bytes - 1) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  if (a0.type != hipMemoryTypeHost || a1.type != hipMemoryTypeHost || !a0.devicePointer || !a1.devicePointer)
    return nullptr;
  const uint8_t* d0 = static_cast<const uint8_t*>(a0.devicePointer);
  if (static_cast<const uint8_t*>(a1.devicePointer) != d0 + (bytes - 1)) return nullptr;
  return d0;
}

// Pins the pages of [p, p + bytes) in place and maps them for the device
// (hipHostRegister); returns the registered base for unpin, or nullptr when the
// runtime refuses (the range overlaps a registered one, ...).
void* pin_range(const void* p, size_t bytes) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p) & ~uintptr_t(4095);
  const uintptr_t z = (reinterpret_cast<uintptr_t>(p) + bytes + 4095) & ~uintptr_t(4095);
  if (hipHostRegister(reinterpret_cast<void*>(a), z - a, hipHostRegisterMapped) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return reinterpret_cast<void*>(a);
}

// How pageable buffers of the host reconstruct go: "pin" (default) registers
// them for the call, "gather" copies the present rows into pinned staging on
// host threads (NP_PAGEABLE).
bool pageable_pin() {
  const char* m = std::getenv("NP_PAGEABLE");
  return !m || std::strcmp(m, "gather") != 0;
}

}  // namespace

int np_encode_batch_host(np_ctx* c, const np_code_params* p, const uint8_t* payloads, size_t len, size_t pstride,
                         size_t batch, uint8_t* shards, size_t bstride) {
  if (!c) return fail(NP_ERR_INVALID_ARGUMENT);
  int st = check_params(p);
  if (st) return st;
  if (len == 0) return fail(NP_ERR_PAYLOAD_SIZE_IS_ZERO);
  const size_t sl = np_shard_len(p, len), row_bytes = p->wanted_n * sl;
  if (!payloads || !shards || pstride < len || bstride < row_bytes) return fail(NP_ERR_INVALID_ARGUMENT);
  if (batch == 0) return NP_OK;
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipSetDevice(c->device);
  // pageable buffers pinned in place for the call (NP_PAGEABLE=pin): the
  // copies then run as DMA from / to pinned memory, at the PCIe rate
  const size_t span_in = (batch - 1) * pstride + len, span_out = (batch - 1) * bstride + row_bytes;
  void* pinned_in = nullptr;
  void* pinned_out = nullptr;
  if (pageable_pin()) {
    if (!mapped_host_range(payloads, span_in)) pinned_in = pin_range(payloads, span_in);
    if (!mapped_host_range(shards, span_out)) pinned_out = pin_range(shards, span_out);
  }
  hipError_t e = pipe_init(c);
  const size_t sb = std::min(batch, std::max<size_t>(1, kPipeSlotBytes / (len + row_bytes)));
  for (int i = 0; e == hipSuccess && i < np_ctx::kPipe; ++i) {
    e = c->pipe_in[i].ensure(sb * len);
    if (e == hipSuccess) e = c->pipe_out[i].ensure(sb * row_bytes);
  }
  size_t slot = 0;
  for (size_t b0 = 0; e == hipSuccess && b0 < batch; b0 += sb, slot = (slot + 1) % np_ctx::kPipe) {
    const size_t cnt = std::min(sb, batch - b0);
    hipStream_t s = c->pipe_s[slot];
    uint8_t* din = c->pipe_in[slot].as<uint8_t>();
    uint8_t* dout = c->pipe_out[slot].as<uint8_t>();
    e = hipMemcpy2DAsync(din, len, payloads + b0 * pstride, pstride, len, cnt, hipMemcpyHostToDevice, s);
    if (e == hipSuccess) e = launch_encode(c, enc_args(p, din, len, len, cnt, dout, row_bytes), s);
    if (e == hipSuccess)
      e = hipMemcpy2DAsync(shards + b0 * bstride, bstride, dout, row_bytes, row_bytes, cnt, hipMemcpyDeviceToHost, s);
  }
  e = pipe_sync(c, e);
  if (pinned_in) (void)hipHostUnregister(pinned_in);
  if (pinned_out) (void)hipHostUnregister(pinned_out);
  return dev_err(e);
}

int np_reconstruct_batch_host(np_ctx* c, const np_code_params* p, const uint8_t* shards, size_t shard_len,
                              size_t bstride, const uint8_t* present, size_t batch, uint8_t* out,
                              size_t out_stride) {
  if (!c || !present) return fail(NP_ERR_INVALID_ARGUMENT);
  int st = check_params(p);
  if (st) return st;
  for (size_t b = 0; b < batch; ++b) {  // mod.rs:171-180
    size_t have = 0;
    for (size_t v = 0; v < p->n; ++v) have += present[b * p->n + v] ? 1 : 0;
    if (have < p->k) return fail(NP_ERR_NEED_MORE_SHARDS, have, p->k, p->n);
  }
  if (shard_len == 0 || (shard_len & 1)) return fail(NP_ERR_EMPTY_SHARD);
  const size_t olen = (shard_len / 2) * 2 * p->k;
  if (!shards || !out || bstride < p->n * shard_len || out_stride < olen) return fail(NP_ERR_INVALID_ARGUMENT);
  if (batch == 0) return NP_OK;
  // only the rows the kernels read cross PCIe; the device stride stays n rows
  const size_t rows = rows_needed(p, shard_len, present, batch), in_bytes = rows * shard_len, dstride = p->n * shard_len;
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipSetDevice(c->device);
  // Pinned shards: a kernel reads only the present rows over PCIe (the
  // gather: 682 of 1024 rows at config 3, 1366 of 4096 at config 4); pageable
  // ones go by one 2-D DMA of the first `rows` rows of every payload.  The
  // outputs go by DMA either way (the link shares badly between
  // kernel reads of host memory and any D2H, but a DMA D2H is the best of it).
  // (4-byte aligned rows only: k_copy_rows moves 16- or 4-byte pieces there;
  // other layouts keep the DMA, which any alignment runs at full rate)
  const bool gather_ok = ((reinterpret_cast<uintptr_t>(shards) | bstride | shard_len) & 3) == 0;
  const size_t span_in = (batch - 1) * bstride + in_bytes, span_out = (batch - 1) * out_stride + olen;
  const uint8_t* mapped = gather_ok ? mapped_host_range(shards, span_in) : nullptr;
  // Pageable buffers pinned in place for the call (NP_PAGEABLE=pin): the
  // gather kernel then reads the present rows of the caller's own shards, and
  // the outputs go by DMA straight into the caller's buffer
  void* pinned_in = nullptr;
  void* pinned_out = nullptr;
  if (gather_ok && !mapped && !std::getenv("NP_NO_GATHER") && pageable_pin()) {
    pinned_in = pin_range(shards, span_in);
    if (pinned_in) mapped = mapped_host_range(shards, span_in);
    if (mapped && !mapped_host_range(out, span_out)) pinned_out = pin_range(out, span_out);
  }
  // Pageable shards of a decode (rows == n): host threads copy the present
  // rows into pinned staging, from where k_copy_rows gathers them as from
  // pinned shards; outputs come back through pinned staging as well.  Only
  // the present rows are read from the caller's memory and cross PCIe.
  const bool host_gather = !mapped && rows == p->n && !std::getenv("NP_NO_GATHER");
  // Outputs of the staged pageable path: through pinned staging and host
  // threads, or (NP_PAGEABLE_OUT=direct) by the runtime's pageable D2H, which
  // measured slower in the pipeline (profiles/r04_e2e_cfg4.json).
  const char* pout = std::getenv("NP_PAGEABLE_OUT");
  const bool staged_out = host_gather && !(pout && std::strcmp(pout, "direct") == 0);
  hipError_t e = pipe_init(c);
  const size_t sb = std::min(batch, std::max<size_t>(1, kPipeSlotBytes / (in_bytes + olen)));
  const size_t slot_in = (sb - 1) * dstride + in_bytes;
  for (int i = 0; e == hipSuccess && i < np_ctx::kPipe; ++i) {
    e = c->pipe_in[i].ensure(slot_in);
    if (e == hipSuccess) e = c->pipe_out[i].ensure(sb * olen);
    if (host_gather) {
      if (e == hipSuccess) e = c->pipe_hin[i].ensure(slot_in);
      if (e == hipSuccess && staged_out) e = c->pipe_hout[i].ensure(sb * olen);
      if (e == hipSuccess && !c->pipe_ev[i]) e = hipEventCreateWithFlags(&c->pipe_ev[i], hipEventDisableTiming);
    }
  }
  const uint8_t* hin_dev[np_ctx::kPipe] = {};
  for (int i = 0; host_gather && e == hipSuccess && i < np_ctx::kPipe; ++i) {
    hin_dev[i] = mapped_host_range(c->pipe_hin[i].as<uint8_t>(), slot_in);
    if (!hin_dev[i]) e = hipErrorInvalidValue;  // hipHostMalloc memory is mapped
  }
  // pend_cnt[sl]: payloads of slot sl whose pinned staging is still in use
  // (the gather kernel, and with staged outputs the D2H into pipe_hout)
  size_t pend_b0[np_ctx::kPipe] = {}, pend_cnt[np_ctx::kPipe] = {};
  auto drain = [&](int sl) {  // slot sl's staging is free again (its outputs -> the caller's buffer)
    if (!pend_cnt[sl]) return;
    const hipError_t r = hipEventSynchronize(c->pipe_ev[sl]);
    if (e == hipSuccess) e = r;
    if (r == hipSuccess && staged_out) {
      const uint8_t* src = c->pipe_hout[sl].as<uint8_t>();
      const size_t b0 = pend_b0[sl], pieces = (olen + (1u << 20) - 1) >> 20;
      parallel_for(pend_cnt[sl] * pieces, [&](size_t i) {
        const size_t b = i / pieces, off = (i % pieces) << 20, len = std::min<size_t>(olen - off, size_t(1) << 20);
        stream_copy(out + (b0 + b) * out_stride + off, src + b * olen + off, len);
      });
    }
    pend_cnt[sl] = 0;
  };
  // the whole present mask up front, synchronously: from pageable memory an
  // asynchronous copy per sub-batch would wait for its stream, and with it the
  // enqueueing of the next sub-batches
  if (e == hipSuccess) e = c->pipe_pres.ensure(batch * p->n);
  if (e == hipSuccess) e = hipMemcpy(c->pipe_pres.p, present, batch * p->n, hipMemcpyHostToDevice);
  size_t slot = 0;
  for (size_t b0 = 0; e == hipSuccess && b0 < batch; b0 += sb, slot = (slot + 1) % np_ctx::kPipe) {
    const size_t cnt = std::min(sb, batch - b0);
    hipStream_t s = c->pipe_s[slot];
    uint8_t* din = c->pipe_in[slot].as<uint8_t>();
    uint8_t* dout = c->pipe_out[slot].as<uint8_t>();
    const uint8_t* dpres = c->pipe_pres.as<uint8_t>() + b0 * p->n;
    if (host_gather) {
      drain(static_cast<int>(slot));  // the slot's previous sub-batch is done with its staging
      if (e != hipSuccess) break;
      uint8_t* hin = c->pipe_hin[slot].as<uint8_t>();
      const size_t nrows = cnt * p->n;
      parallel_for((nrows + 63) / 64, [&](size_t i) {  // 64 rows per task
        for (size_t r = 64 * i; r < std::min(nrows, 64 * i + 64); ++r) {
          const size_t b = r / p->n, v = r % p->n;
          if (present[(b0 + b) * p->n + v])
            stream_copy(hin + b * dstride + v * shard_len, shards + (b0 + b) * bstride + v * shard_len, shard_len);
        }
      });
      e = np::launch_copy_rows(hin_dev[slot], dstride, din, dstride, shard_len, dpres, static_cast<uint32_t>(p->n),
                               static_cast<uint32_t>(rows), cnt, kGatherBlocks, s);
      if (!staged_out) {  // the input staging is free once the gather kernel is done
        if (e == hipSuccess) e = hipEventRecord(c->pipe_ev[slot], s);
        if (e == hipSuccess) pend_b0[slot] = b0, pend_cnt[slot] = cnt;
      }
    } else {
    e = mapped ? np::launch_copy_rows(mapped + b0 * bstride, bstride, din, dstride, shard_len, dpres,
                                      static_cast<uint32_t>(p->n), static_cast<uint32_t>(rows), cnt, kGatherBlocks, s)
               : hipMemcpy2DAsync(din, dstride, shards + b0 * bstride, bstride, in_bytes, cnt, hipMemcpyHostToDevice,
                                  s);
    }
    if (e == hipSuccess) {
      np::ReconstructArgs a{};
      a.shards = din;
      a.shard_len = shard_len;
      a.batch_stride = dstride;
      a.present = dpres;
      a.locators = nullptr;  // computed on the device
      a.batch = cnt;
      a.n = static_cast<uint32_t>(p->n);
      a.k = static_cast<uint32_t>(p->k);
      a.out = dout;
      a.out_stride = olen;
      e = launch_reconstruct(c, a, s);
    }
    if (staged_out) {
      if (e == hipSuccess)
        e = hipMemcpyAsync(c->pipe_hout[slot].p, dout, cnt * olen, hipMemcpyDeviceToHost, s);
      if (e == hipSuccess) e = hipEventRecord(c->pipe_ev[slot], s);
      if (e == hipSuccess) pend_b0[slot] = b0, pend_cnt[slot] = cnt;
    } else if (e == hipSuccess) {
      e = hipMemcpy2DAsync(out + b0 * out_stride, out_stride, dout, olen, olen, cnt, hipMemcpyDeviceToHost, s);
    }
  }
  // the remaining slots in submission order (a failed call still waits for its streams)
  for (size_t i = 1; host_gather && i <= np_ctx::kPipe; ++i) drain(static_cast<int>((slot + i) % np_ctx::kPipe));
  e = pipe_sync(c, e);
  if (pinned_in) (void)hipHostUnregister(pinned_in);
  if (pinned_out) (void)hipHostUnregister(pinned_out);
  return dev_err(e);
}

// ---------------------------------------------------------- reconstruct ----
int np_error_locator_dev(np_ctx* c, size_t n, const uint8_t* d_present, size_t batch, uint16_t* d_loc,
                         void* stream) {
  if (!c || !d_present || !d_loc || !is_pow2(n) || n > np::kFieldSize) return fail(NP_ERR_INVALID_ARGUMENT);
  (void)hipSetDevice(c->device);
  return dev_err(np::launch_error_locator(c->T, static_cast<uint32_t>(n), d_present, batch, d_loc, pick(c, stream)));
}

namespace {

int reconstruct_dev2(np_ctx* c, const np_code_params* p, const uint8_t* d_shards, size_t shard_len, size_t bstride,
                     const uint8_t* d_present, const uint16_t* d_loc, size_t batch, uint8_t* d_out,
                     size_t out_stride, np_payload_status* d_status, void* stream, bool trusted) {
  if (!c) return fail(NP_ERR_INVALID_ARGUMENT);
  int st = check_params(p);
  if (st) return st;
  if (shard_len == 0 || (shard_len & 1)) return fail(NP_ERR_EMPTY_SHARD);
  if (!d_shards || !d_present || !d_out || bstride < p->n * shard_len || out_stride < (shard_len / 2) * 2 * p->k)
    return fail(NP_ERR_INVALID_ARGUMENT);
  static_assert(sizeof(np_payload_status) == 2 * sizeof(uint32_t), "status layout of ReconstructArgs::status");
  std::lock_guard<std::mutex> g(c->mu);  // context scratch
  (void)hipSetDevice(c->device);
  np::ReconstructArgs a{};
  a.shards = d_shards;
  a.shard_len = shard_len;
  a.batch_stride = bstride;
  a.present = d_present;
  a.locators = d_loc;
  a.batch = batch;
  a.n = static_cast<uint32_t>(p->n);
  a.k = static_cast<uint32_t>(p->k);
  a.out = d_out;
  a.out_stride = out_stride;
  a.status = reinterpret_cast<uint32_t*>(d_status);
  a.trusted = trusted;
  return dev_err(launch_reconstruct(c, a, pick(c, stream)));
}

}  // namespace

int np_reconstruct_batch_dev3(np_ctx* c, const np_code_params* p, const uint8_t* d_shards, size_t shard_len,
                              size_t bstride, const uint8_t* d_present, const uint16_t* d_loc, size_t batch,
                              uint8_t* d_out, size_t out_stride, np_payload_status* d_status, void* stream) {
  return reconstruct_dev2(c, p, d_shards, shard_len, bstride, d_present, d_loc, batch, d_out, out_stride, d_status,
                          stream, false);
}

// The 0.1.0 signature (no per-payload status), kept so that a caller built
// against the old header still passes its stream in the stream slot.
int np_reconstruct_batch_dev2(np_ctx* c, const np_code_params* p, const uint8_t* d_shards, size_t shard_len,
                              size_t bstride, const uint8_t* d_present, const uint16_t* d_loc, size_t batch,
                              uint8_t* d_out, size_t out_stride, void* stream) {
  return reconstruct_dev2(c, p, d_shards, shard_len, bstride, d_present, d_loc, batch, d_out, out_stride, nullptr,
                          stream, false);
}

int np_reconstruct_codewords_batch_dev(np_ctx* c, const np_code_params* p, const uint8_t* d_shards,
                                       size_t shard_len, size_t bstride, const uint8_t* d_present, size_t batch,
                                       uint8_t* d_out, size_t out_stride, np_payload_status* d_status,
                                       void* stream) {
  return reconstruct_dev2(c, p, d_shards, shard_len, bstride, d_present, nullptr, batch, d_out, out_stride,
                          d_status, stream, true);
}

int np_reconstruct_batch_dev(np_ctx* c, const np_code_params* p, const uint8_t* d_shards, size_t shard_len,
                             size_t bstride, const uint8_t* present, size_t batch, uint8_t* d_out, size_t out_stride,
                             void* stream) {
  if (!c || !present) return fail(NP_ERR_INVALID_ARGUMENT);
  int st = check_params(p);
  if (st) return st;
  for (size_t b = 0; b < batch; ++b) {  // mod.rs:171-180
    size_t have = 0;
    for (size_t v = 0; v < p->n; ++v) have += present[b * p->n + v] ? 1 : 0;
    if (have < p->k) return fail(NP_ERR_NEED_MORE_SHARDS, have, p->k, p->n);
  }
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipSetDevice(c->device);
  hipStream_t s = pick(c, stream);
  if (shard_len == 0 || (shard_len & 1)) return fail(NP_ERR_EMPTY_SHARD);
  if (!d_shards || !d_out || bstride < p->n * shard_len || out_stride < (shard_len / 2) * 2 * p->k)
    return fail(NP_ERR_INVALID_ARGUMENT);
  hipError_t e = c->d_present.ensure(std::max<size_t>(batch * p->n, 1));
  if (e != hipSuccess) return dev_err(e);
  e = hipMemcpyAsync(c->d_present.p, present, batch * p->n, hipMemcpyHostToDevice, s);
  if (e != hipSuccess) return dev_err(e);
  np::ReconstructArgs a{};
  a.shards = d_shards;
  a.shard_len = shard_len;
  a.batch_stride = bstride;
  a.present = c->d_present.as<uint8_t>();
  a.locators = nullptr;  // computed on the device
  a.batch = batch;
  a.n = static_cast<uint32_t>(p->n);
  a.k = static_cast<uint32_t>(p->k);
  a.out = d_out;
  a.out_stride = out_stride;
  e = launch_reconstruct(c, a, s);
  if (e != hipSuccess) return dev_err(e);
  // present mask was copied from pageable host memory: make the call
  // synchronous with respect to it before returning.
  return dev_err(hipStreamSynchronize(s));
}

int np_rs_reconstruct(np_ctx* c, const np_code_params* p, const uint8_t* const* shards, const size_t* lens,
                      size_t n_received, uint8_t* out, size_t cap, size_t* out_len) {
  if (!c || !p || (n_received && (!shards || !lens))) return fail(NP_ERR_INVALID_ARGUMENT);
  if (!is_pow2(p->n) && !is_pow2(p->k)) return fail(NP_ERR_PARAMETER_MUST_BE_POWER_OF_2, p->n, p->k);
  const size_t n = p->n, k = p->k;
  // mod.rs:163-180: pad/truncate to n, erasures, existential count
  std::vector<uint8_t> present(n, 0);
  size_t have = 0;
  for (size_t i = 0; i < n && i < n_received; ++i) {
    present[i] = shards[i] ? 1 : 0;
    have += present[i];
  }
  if (have < k) return fail(NP_ERR_NEED_MORE_SHARDS, have, k, n);
  // mod.rs:183-214: shard length from the first present shard
  size_t first = 0;
  while (!present[first]) ++first;
  const size_t syms = (lens[first] + 1) / 2;
  if (syms == 0) return fail(NP_ERR_EMPTY_SHARD);
  for (size_t i = first + 1; i < n; ++i)
    if (present[i] && (lens[i] + 1) / 2 != syms) return fail(NP_ERR_INCONSISTENT_SHARD_LENGTHS, syms, (lens[i] + 1) / 2);
  int st = check_params(p);
  if (st) return st;
  const size_t need = syms * 2 * k;
  if (!out || !out_len || cap < need) return fail(NP_ERR_INVALID_ARGUMENT, need);
  const size_t sl = 2 * syms;
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipSetDevice(c->device);
  hipError_t e = c->h_in.ensure(n * sl);
  if (e == hipSuccess) e = c->d_in.ensure(n * sl);
  if (e == hipSuccess) e = c->d_out.ensure(need);
  if (e == hipSuccess) e = c->h_out.ensure(need);
  if (e == hipSuccess) e = c->d_present.ensure(n);
  if (e != hipSuccess) return dev_err(e);
  uint8_t* stage = c->h_in.as<uint8_t>();
  for (size_t i = 0; i < n; ++i) {
    uint8_t* row = stage + i * sl;
    if (present[i]) {
      std::memcpy(row, shards[i], lens[i]);
      if (lens[i] < sl) std::memset(row + lens[i], 0, sl - lens[i]);  // WrappedShard zero pad
    } else {
      std::memset(row, 0, sl);
    }
  }
  hipStream_t s = c->stream;
  e = hipMemcpyAsync(c->d_in.p, stage, n * sl, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = hipMemcpyAsync(c->d_present.p, present.data(), n, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) {
    np::ReconstructArgs a{};
    a.shards = c->d_in.as<uint8_t>();
    a.shard_len = sl;
    a.batch_stride = n * sl;
    a.present = c->d_present.as<uint8_t>();
    a.locators = nullptr;  // computed on the device
    a.batch = 1;
    a.n = static_cast<uint32_t>(n);
    a.k = static_cast<uint32_t>(k);
    a.out = c->d_out.as<uint8_t>();
    a.out_stride = need;
    e = launch_reconstruct(c, a, s);
  }
  if (e == hipSuccess) e = hipMemcpyAsync(c->h_out.p, c->d_out.p, need, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return dev_err(e);
  std::memcpy(out, c->h_out.p, need);
  *out_len = need;
  return NP_OK;
}

int np_reconstruct(np_ctx* c, const uint8_t* const* shards, const size_t* lens, size_t n_received,
                   size_t validator_count, uint8_t* out, size_t cap, size_t* out_len) {
  // reconstruct.rs:4-9
  np_code_params p;
  int st = np_derive_parameters(validator_count, np_recoverability_subset_size(validator_count), &p);
  if (st) return st;
  return np_rs_reconstruct(c, &p, shards, lens, n_received, out, cap, out_len);
}

int np_rs_reconstruct_from_systematic(np_ctx* c, const np_code_params* p, const uint8_t* const* chunks,
                                      const size_t* lens, size_t n_chunks, uint8_t* out, size_t cap,
                                      size_t* out_len) {
  // mod.rs:247-285: validation as the crate, then the column gather of the
  // first k shards on the device (kernels_systematic.hip)
  if (!c || !p || (n_chunks && (!chunks || !lens))) return fail(NP_ERR_INVALID_ARGUMENT);
  if (n_chunks == 0) return fail(NP_ERR_NEED_MORE_SHARDS, 0, p->k, p->n);
  if (n_chunks < p->k) return fail(NP_ERR_NEED_MORE_SHARDS, n_chunks, p->k, p->n);
  const size_t syms = (lens[0] + 1) / 2;
  if (syms == 0) return fail(NP_ERR_EMPTY_SHARD);
  for (size_t i = 0; i < n_chunks; ++i)
    if ((lens[i] + 1) / 2 != syms) return fail(NP_ERR_INCONSISTENT_SHARD_LENGTHS, syms, (lens[i] + 1) / 2);
  const size_t k = p->k, need = syms * 2 * k, sl = 2 * syms;
  if (!out || !out_len || cap < need) return fail(NP_ERR_INVALID_ARGUMENT, need);
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipSetDevice(c->device);
  hipError_t e = c->h_in.ensure(k * sl);
  if (e == hipSuccess) e = c->d_in.ensure(k * sl);
  if (e == hipSuccess) e = c->d_out.ensure(need);
  if (e == hipSuccess) e = c->h_out.ensure(need);
  if (e != hipSuccess) return dev_err(e);
  uint8_t* stage = c->h_in.as<uint8_t>();
  for (size_t j = 0; j < k; ++j) {
    std::memcpy(stage + j * sl, chunks[j], lens[j]);
    if (lens[j] < sl) std::memset(stage + j * sl + lens[j], 0, sl - lens[j]);  // WrappedShard zero pad
  }
  hipStream_t s = c->stream;
  e = hipMemcpyAsync(c->d_in.p, stage, k * sl, hipMemcpyHostToDevice, s);
  if (e == hipSuccess) e = np::launch_systematic(c->d_in.as<uint8_t>(), sl, k * sl, static_cast<uint32_t>(k), 1,
                                                 c->d_out.as<uint8_t>(), need, s);
  if (e == hipSuccess) e = hipMemcpyAsync(c->h_out.p, c->d_out.p, need, hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e != hipSuccess) return dev_err(e);
  std::memcpy(out, c->h_out.p, need);
  *out_len = need;
  return NP_OK;
}

int np_reconstruct_from_systematic_batch_dev(np_ctx* c, const np_code_params* p, const uint8_t* d_shards,
                                             size_t shard_len, size_t bstride, size_t batch, uint8_t* d_out,
                                             size_t out_stride, void* stream) {
  if (!c) return fail(NP_ERR_INVALID_ARGUMENT);
  int st = check_params(p);
  if (st) return st;
  if (shard_len == 0 || (shard_len & 1)) return fail(NP_ERR_EMPTY_SHARD);
  if (!d_shards || !d_out || bstride < p->k * shard_len || out_stride < (shard_len / 2) * 2 * p->k)
    return fail(NP_ERR_INVALID_ARGUMENT);
  (void)hipSetDevice(c->device);
  return dev_err(np::launch_systematic(d_shards, shard_len, bstride, static_cast<uint32_t>(p->k), batch, d_out,
                                       out_stride, pick(c, stream)));
}

// ------------------------------------------------------------ multi-GPU ----
// payloads are independent, so a batch splits into contiguous
// ranges, one per device (context), with no exchange between devices; one
// host thread per context drives its range on that context's stream (the
// host-memory calls block in their pipeline, so the threads overlap them).
void np_batch_split(size_t batch, size_t ndev, size_t i, size_t* begin, size_t* count) {
  if (!begin || !count) return;
  if (ndev == 0 || i >= ndev) {
    *begin = batch;
    *count = 0;
    return;
  }
  const size_t base = batch / ndev, extra = batch % ndev;  // the first `extra` ranges hold one more
  *begin = i * base + std::min(i, extra);
  *count = base + (i < extra ? 1 : 0);
}

}  // extern "C"

namespace {

// Runs fn(i, begin, count) for every context on its own thread; returns the
// first failing status with its error detail on the calling thread.
template <class F>
int run_multi(np_ctx* const* ctxs, size_t nctx, size_t batch, F fn) {
  if (!ctxs || nctx == 0) return fail(NP_ERR_INVALID_ARGUMENT);
  for (size_t i = 0; i < nctx; ++i)
    if (!ctxs[i]) return fail(NP_ERR_INVALID_ARGUMENT);
  std::vector<int> st(nctx, NP_OK);
  std::vector<std::array<size_t, 3>> det(nctx);
  std::vector<std::thread> th;
  th.reserve(nctx);
  for (size_t i = 0; i < nctx; ++i) {
    size_t b0 = 0, cnt = 0;
    np_batch_split(batch, nctx, i, &b0, &cnt);
    th.emplace_back([&, i, b0, cnt] {
      st[i] = cnt ? fn(i, b0, cnt) : NP_OK;
      np_last_error_detail(det[i].data());
    });
  }
  for (auto& t : th) t.join();
  for (size_t i = 0; i < nctx; ++i)
    if (st[i] != NP_OK) return fail(st[i], det[i][0], det[i][1], det[i][2]);
  return NP_OK;
}

}  // namespace

extern "C" {

int np_encode_batch_multi(np_ctx* const* ctxs, size_t nctx, const np_code_params* p,
                          const uint8_t* const* d_payloads, size_t len, size_t pstride, size_t batch,
                          uint8_t* const* d_shards, size_t bstride) {
  if (!d_payloads || !d_shards) return fail(NP_ERR_INVALID_ARGUMENT);
  if (int st = check_params(p)) return st;
  return run_multi(ctxs, nctx, batch, [&](size_t i, size_t, size_t cnt) {
    int st = np_encode_batch_dev(ctxs[i], p, d_payloads[i], len, pstride, cnt, d_shards[i], bstride, nullptr);
    return st ? st : np_ctx_synchronize(ctxs[i]);
  });
}

int np_reconstruct_batch_multi(np_ctx* const* ctxs, size_t nctx, const np_code_params* p,
                               const uint8_t* const* d_shards, size_t shard_len, size_t bstride,
                               const uint8_t* const* d_present, size_t batch, uint8_t* const* d_out,
                               size_t out_stride, np_payload_status* const* d_status) {
  if (!d_shards || !d_present || !d_out) return fail(NP_ERR_INVALID_ARGUMENT);
  if (int st = check_params(p)) return st;
  return run_multi(ctxs, nctx, batch, [&](size_t i, size_t, size_t cnt) {
    int st = np_reconstruct_batch_dev3(ctxs[i], p, d_shards[i], shard_len, bstride, d_present[i], nullptr, cnt,
                                       d_out[i], out_stride, d_status ? d_status[i] : nullptr, nullptr);
    return st ? st : np_ctx_synchronize(ctxs[i]);
  });
}

int np_encode_batch_host_multi(np_ctx* const* ctxs, size_t nctx, const np_code_params* p, const uint8_t* payloads,
                               size_t len, size_t pstride, size_t batch, uint8_t* shards, size_t bstride) {
  if (!payloads || !shards) return fail(NP_ERR_INVALID_ARGUMENT);
  if (int st = check_params(p)) return st;
  return run_multi(ctxs, nctx, batch, [&](size_t i, size_t b0, size_t cnt) {
    return np_encode_batch_host(ctxs[i], p, payloads + b0 * pstride, len, pstride, cnt, shards + b0 * bstride,
                                bstride);
  });
}

int np_reconstruct_batch_host_multi(np_ctx* const* ctxs, size_t nctx, const np_code_params* p,
                                    const uint8_t* shards, size_t shard_len, size_t bstride, const uint8_t* present,
                                    size_t batch, uint8_t* out, size_t out_stride) {
  if (!shards || !present || !out || !p) return fail(NP_ERR_INVALID_ARGUMENT);
  if (int st = check_params(p)) return st;
  return run_multi(ctxs, nctx, batch, [&](size_t i, size_t b0, size_t cnt) {
    return np_reconstruct_batch_host(ctxs[i], p, shards + b0 * bstride, shard_len, bstride, present + b0 * p->n,
                                     cnt, out + b0 * out_stride, out_stride);
  });
}

// --------------------------------------------------------- parity hooks ----
int np_afft_dev(np_ctx* c, uint16_t* d, size_t size, size_t index, size_t cols, void* stream) {
  if (!c || !d || !is_pow2(size) || size > np::kFieldSize || index + size > np::kFieldSize)
    return fail(NP_ERR_INVALID_ARGUMENT);
  (void)hipSetDevice(c->device);
  return dev_err(np::launch_afft(c->T, d, static_cast<uint32_t>(size), static_cast<uint32_t>(index), cols, false,
                                 pick(c, stream)));
}

int np_inverse_afft_dev(np_ctx* c, uint16_t* d, size_t size, size_t index, size_t cols, void* stream) {
  if (!c || !d || !is_pow2(size) || size > np::kFieldSize || index + size > np::kFieldSize)
    return fail(NP_ERR_INVALID_ARGUMENT);
  (void)hipSetDevice(c->device);
  return dev_err(np::launch_afft(c->T, d, static_cast<uint32_t>(size), static_cast<uint32_t>(index), cols, true,
                                 pick(c, stream)));
}

int np_walsh_dev(np_ctx* c, uint16_t* d, size_t size, void* stream) {
  if (!c || !d || !is_pow2(size) || size > np::kFieldSize) return fail(NP_ERR_INVALID_ARGUMENT);
  (void)hipSetDevice(c->device);
  return dev_err(np::launch_walsh(d, static_cast<uint32_t>(size), pick(c, stream)));
}

int np_mul_dev(np_ctx* c, const uint16_t* a, const uint16_t* m, uint16_t* o, size_t count, void* stream) {
  if (!c || !a || !m || !o) return fail(NP_ERR_INVALID_ARGUMENT);
  (void)hipSetDevice(c->device);
  return dev_err(np::launch_mul(c->T, a, m, o, count, pick(c, stream)));
}

int np_encode_low_dev(np_ctx* c, const uint16_t* d, size_t k, uint16_t* cw, size_t n, size_t cols, void* stream) {
  if (!c || !d || !cw || !is_pow2(n) || !is_pow2(k) || 2 * k > n || n > np::kFieldSize)
    return fail(NP_ERR_INVALID_ARGUMENT);
  (void)hipSetDevice(c->device);
  return dev_err(
      np::launch_encode_low(c->T, d, static_cast<uint32_t>(k), cw, static_cast<uint32_t>(n), cols, pick(c, stream)));
}

int np_decode_main_dev(np_ctx* c, uint16_t* cw, size_t upto, const uint8_t* d_present, const uint16_t* d_loc,
                       size_t n, size_t cols, void* stream) {
  if (!c || !cw || !d_present || !d_loc || !is_pow2(n) || n > np::kFieldSize || upto > n)
    return fail(NP_ERR_INVALID_ARGUMENT);
  (void)hipSetDevice(c->device);
  return dev_err(np::launch_decode_main(c->T, cw, static_cast<uint32_t>(upto), d_present, d_loc,
                                        static_cast<uint32_t>(n), cols, pick(c, stream)));
}

}  // extern "C"
