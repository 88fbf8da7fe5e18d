// Host engine behind the C ABI (include/novelpoly.h): parameter derivation,
// validation with the crate's error behaviour, per-device contexts, staging
// and kernel dispatch.  Mirrors src/novel_poly_basis/mod.rs:24-285 of the
// reference crate; the per-chunk / per-column loops of mod.rs:144-154 and
// :221-236 are replaced by batched GPU kernels.
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <iterator>
#include <map>
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

thread_local char g_site_msg[192] = "";

// Every failure sets the detail and clears the call-site text; dev_err writes
// the text after this for NP_ERR_DEVICE / NP_ERR_ALLOC (a
// validation error, or a success, never reports an older failure's site).
int fail(int st, size_t a = 0, size_t b = 0, size_t c = 0) {
  g_detail[0] = a;
  g_detail[1] = b;
  g_detail[2] = c;
  g_site_msg[0] = '\0';
  return st;
}

// Call site of the first failing HIP call since the last status was reported
// (HIP(expr) below): its engine.cpp line and text.  dev_err turns it into the
// NP_ERR_DEVICE / NP_ERR_ALLOC detail {hipError_t, line, 0} and the text of
// np_last_error_site, so a failure names the call that returned it -- for an
// asynchronous kernel or copy fault that is the synchronisation that saw it
// (NP_SYNC_EACH=1 below makes the host pipeline synchronise after every step).
thread_local int g_site_line = 0;
thread_local const char* g_site_call = nullptr;

hipError_t at_site(hipError_t e, int line, const char* call) {
  if (e != hipSuccess && !g_site_line) {
    g_site_line = line;
    g_site_call = call;
  }
  return e;
}
#define HIP(x) at_site((x), __LINE__, #x)

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
    // engine.cpp big_scratch, np_ctx::big_cap)
    hipError_t e = hipMalloc(&p, bytes);
    if (e == hipSuccess)
      cap = bytes;
    else
      (void)hipGetLastError();  // returned here: not left behind for the next launch's hipGetLastError
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
    if (e == hipSuccess)
      cap = bytes;
    else
      (void)hipGetLastError();
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
  HostBuf h_pres;  // pinned staging of present masks (np_reconstruct_batch_dev / _host, np_rs_reconstruct)
  // Per-workgroup scratch of the k = 1024 kernels (kernels_big.hip).  Launches
  // on different streams are ordered through big_done so they never share it.
  DevBuf d_big;
  size_t big_cap = size_t(2) << 30;  // scratch_cap_for: set at creation
  hipEvent_t big_done = nullptr;
  bool big_used = false;
  // Host-memory batch pipeline (np_*_batch_host): per slot a stream and
  // device buffers for one sub-batch; created on first use.
  static constexpr int kPipe = 6;  // at most; pipe_slots() are used
  hipStream_t pipe_s[kPipe] = {};
  DevBuf pipe_in[kPipe], pipe_out[kPipe];
  DevBuf pipe_cin[kPipe];  // packed present rows and their offsets (np_reconstruct_batch_host)
  DevBuf pipe_pres;  // the present mask of a whole host reconstruct call
  // Pageable host reconstruct: pinned staging per slot for the present rows
  // (gathered by host threads) and for the outputs, and the slot's last event.
  HostBuf pipe_hin[kPipe], pipe_hout[kPipe];
  hipEvent_t pipe_ev[kPipe] = {};
};

namespace {

int dev_err(hipError_t e) {
  const int line = g_site_line;
  const char* call = g_site_call;
  g_site_line = 0;
  g_site_call = nullptr;
  if (e == hipSuccess) {
    g_site_msg[0] = '\0';
    return NP_OK;
  }
  const int st = fail(e == hipErrorOutOfMemory ? NP_ERR_ALLOC : NP_ERR_DEVICE, static_cast<size_t>(e),
                      static_cast<size_t>(line));
  if (line)
    std::snprintf(g_site_msg, sizeof g_site_msg, "engine.cpp:%d %s: %s", line, call, hipGetErrorName(e));
  else
    std::snprintf(g_site_msg, sizeof g_site_msg, "(call site not recorded): %s", hipGetErrorName(e));
  return st;
}

template <class T>
hipError_t upload(np_ctx* c, const std::vector<T>& v, const T** dst) {
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, v.size() * sizeof(T));
  if (e != hipSuccess) return e;
  c->table_allocs.push_back(p);
  e = HIP(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
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

// Bytes of big-kernel scratch per context (k = 2048 decode at n = 16384:
// 256 slots of 9.1 MiB; the sub-transform path: 512 x 1 MiB payloads in one
// slice at every validator count, 4.5 GiB of slots at 40,000 validators).
// 8 GiB against 4 measured 4-5 % faster at 20,000 and 40,000 validators
// (profiles/r05/huge/slices_ab.txt), 2.8 % of the 288 GB.  The cap follows the
// device's total memory (a 32nd, 8 GiB on an MI355X), never the memory free at
// context creation: which kernels run and how a batch is sliced are then the
// same from run to run.  It is never below kBigScratchMin, the
// size the path choices (rec_path, launch_encode) assume.
constexpr size_t kBigScratchMax = size_t(8) << 30;
constexpr size_t kBigScratchMin = size_t(2) << 30;
size_t scratch_cap_for(int device) {
  size_t total_b = 0;
  if (hipSetDevice(device) != hipSuccess || hipDeviceTotalMem(&total_b, device) != hipSuccess) {
    (void)hipGetLastError();
    return kBigScratchMin;
  }
  return std::min(kBigScratchMax, std::max(kBigScratchMin, total_b / 32));
}

// Payloads per slice of the sub-transform path when one payload costs
// `two / 2` bytes of slots plus `side`: even, so that pairs stay whole.
size_t huge_slice(const np_ctx* c, size_t two, size_t side) {
  const size_t per = c->big_cap / std::max<size_t>(1, (two + 1) / 2 + side);
  return per >= 2 ? per & ~size_t(1) : 1;
}

// Big-kernel scratch of `want` bytes (capped), ordered after every earlier
// big launch of this context on any stream.  Caller holds the context lock.
hipError_t big_scratch(np_ctx* c, size_t want, hipStream_t s, uint8_t** out, size_t* bytes) {
  want = std::min(want, c->big_cap);
  hipError_t e = hipSuccess;
  if (!c->big_done) e = HIP(hipEventCreateWithFlags(&c->big_done, hipEventDisableTiming));
  if (e == hipSuccess && c->big_used) {
    if (want > c->d_big.cap) e = HIP(hipEventSynchronize(c->big_done));  // about to free the old buffer
    if (e == hipSuccess) e = HIP(hipStreamWaitEvent(s, c->big_done, 0));
  }
  if (e == hipSuccess) e = HIP(c->d_big.ensure(want));
  *out = c->d_big.as<uint8_t>();
  *bytes = c->d_big.cap;
  return e;
}

hipError_t big_done(np_ctx* c, hipStream_t s, hipError_t e) {
  if (e != hipSuccess) return e;
  c->big_used = true;
  return HIP(hipEventRecord(c->big_done, s));
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
      np::huge_reconstruct_scratch_per_payload(shard_len, n, k) <= kBigScratchMin / 2)
    return RecPath::Huge;
  if (np::big_reconstruct_supported(n, k)) return RecPath::Big;
  return RecPath::Generic;
}

// Caller holds the context lock.
hipError_t launch_encode(np_ctx* c, const np::EncodeArgs& a, hipStream_t s) {
  if (np::fast_encode_supported(a.n, a.k)) return HIP(np::launch_encode_fast(c->T, a, s));
  if (np::res_encode_supported(a.n, a.k) && np::res_enabled()) return HIP(np::launch_encode_res(c->T, a, s));
  const size_t huge_per = np::huge_encode_scratch_per_payload(a.shard_len, a.n, a.k);
  if (np::huge_encode_supported(a.n, a.k) && huge_on(a.k) && huge_per <= kBigScratchMin) {
    // slices of the batch whose tile slots fit the context scratch
    const size_t per = huge_slice(c, np::huge_encode_scratch(2, a.payload_len, a.n, a.k), 0);
    for (size_t b0 = 0; b0 < a.batch; b0 += per) {
      np::EncodeArgs sub = a;
      sub.batch = std::min(per, a.batch - b0);
      sub.payloads = a.payloads + b0 * a.payload_stride;
      sub.shards = a.shards + b0 * a.batch_stride;
      uint8_t* scr = nullptr;
      size_t bytes = 0;
      hipError_t e = big_scratch(c, np::huge_encode_scratch(sub.batch, sub.payload_len, sub.n, sub.k), s, &scr, &bytes);
      if (e == hipSuccess) e = HIP(np::launch_encode_huge(c->T, sub, scr, s));
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
    if (e == hipSuccess) e = HIP(np::launch_encode_big(c->T, a, scr, bytes, s));
    return big_done(c, s, e);
  }
  return HIP(np::launch_encode_generic(c->T, a, s));
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
  const bool res = !np::fast_reconstruct_supported(a.n, a.k) || np::res256_reconstruct(a.n, a.k);
  if (path == RecPath::FastRes) {
    // per-payload decode rows + row multipliers and their tables (from the
    // caller's locators when given) and the status, then the decode
    const size_t stride = np::prefix_stride(a.n, a.k);
    const size_t per = std::max<size_t>(1, c->big_cap / (stride + own_status));
    for (size_t b0 = 0; b0 < a.batch; b0 += per) {
      np::ReconstructArgs sub = slice(a, b0, std::min(per, a.batch - b0));
      uint8_t* scr = nullptr;
      size_t bytes = 0;
      hipError_t e = big_scratch(c, sub.batch * (stride + own_status), s, &scr, &bytes);
      if (!a.status) sub.status = reinterpret_cast<uint32_t*>(scr + sub.batch * stride);
      if (e == hipSuccess) e = HIP(np::launch_prefix_locator(c->T, sub, scr, s));
      sub.prefix = scr;
      if (e == hipSuccess) e = res ? HIP(np::launch_reconstruct_res(c->T, sub, s)) : HIP(np::launch_reconstruct_fast(c->T, sub, s));
      e = big_done(c, s, e);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  if (path == RecPath::Huge) {
    // per payload: tile slots, mode byte and occupancy word, locators (unless
    // the caller's), status
    const size_t side = 32 + (a.locators ? 0 : 2 * static_cast<size_t>(a.n)) + own_status;
    const size_t per = huge_slice(c, np::huge_reconstruct_scratch(2, a.shard_len, a.n, a.k), side);
    for (size_t b0 = 0; b0 < a.batch; b0 += per) {
      np::ReconstructArgs sub = slice(a, b0, std::min(per, a.batch - b0));
      uint8_t* scr = nullptr;
      size_t bytes = 0;
      const size_t slots = np::huge_reconstruct_scratch(sub.batch, sub.shard_len, sub.n, sub.k);
      hipError_t e = big_scratch(c, slots + sub.batch * side, s, &scr, &bytes);
      uint8_t* side0 = scr + slots;  // a multiple of 128 KiB
      uint16_t* loc = reinterpret_cast<uint16_t*>(side0);
      uint8_t* mode = side0 + (a.locators ? 0 : 2 * static_cast<size_t>(a.n) * sub.batch);
      if (!a.status) sub.status = reinterpret_cast<uint32_t*>(mode + np::huge_side_bytes(sub.batch));
      if (e == hipSuccess) e = HIP(np::launch_reconstruct_huge(c->T, sub, scr, mode, loc, s));
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
    const size_t per = std::max<size_t>(1, c->big_cap / 4 / rstride);
    for (size_t b0 = 0; b0 < a.batch; b0 += per) {
      np::ReconstructArgs sub = slice(a, b0, std::min(per, a.batch - b0));
      const size_t rec_bytes = (sub.batch * rstride + 255) / 256 * 256;
      uint8_t* scr = nullptr;
      size_t bytes = 0;
      hipError_t e = big_scratch(c, rec_bytes + big_slots(c, sub.batch * tiles, sub.n, sub.k, true) * per_tile, s, &scr, &bytes);
      if (e == hipSuccess && bytes < rec_bytes + 8 * per_tile) e = hipErrorInvalidValue;
      if (!a.status) sub.status = reinterpret_cast<uint32_t*>(scr + sub.batch * np::big_record_stride(a.n));
      sub.prefix = scr;
      if (e == hipSuccess) e = HIP(np::launch_big_records(c->T, sub, scr, s));
      if (e == hipSuccess) e = HIP(np::launch_reconstruct_big(c->T, sub, scr + rec_bytes, bytes - rec_bytes, s));
      e = big_done(c, s, e);
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  // generic path: the status, and the locators unless the caller gave them,
  // into the ordered context scratch
  const size_t loc_bytes = a.locators ? 0 : a.n * sizeof(uint16_t);
  const size_t per = std::max<size_t>(1, c->big_cap / (loc_bytes + own_status + 1));
  for (size_t b0 = 0; b0 < a.batch; b0 += per) {
    np::ReconstructArgs b = slice(a, b0, std::min(per, a.batch - b0));
    uint8_t* scr = nullptr;
    size_t bytes = 0;
    hipError_t e = big_scratch(c, std::max<size_t>(1, b.batch * (loc_bytes + own_status)), s, &scr, &bytes);
    if (!a.status) b.status = reinterpret_cast<uint32_t*>(scr + b.batch * loc_bytes);
    if (e == hipSuccess) e = HIP(np::launch_payload_status(b, s));
    if (!a.locators) {
      b.locators = reinterpret_cast<uint16_t*>(scr);
      if (e == hipSuccess) e = HIP(np::launch_error_locator(c->T, a.n, b.present, b.batch, reinterpret_cast<uint16_t*>(scr), s));
    }
    if (e == hipSuccess) e = HIP(np::launch_reconstruct_generic(c->T, b, s));
    e = big_done(c, s, e);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// The stream of a `_dev` call: the caller's, where NULL is HIP's legacy null
// stream (the caller's default stream, e.g. torch's), as in every HIP / CUDA
// library -- work the caller queued there before the call is ordered before
// ours (verdict r05: NULL used to mean the context's non-blocking stream,
// which ran unordered with the caller's default-stream fills and copies).
// The host calls keep the context's own streams.
hipStream_t pick(np_ctx*, void* s) { return static_cast<hipStream_t>(s); }

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
// thread is one of them): the host side of the pageable calls' staging, which
// moves memcpy-sized row pieces.  The workers persist for the process (one
// pool; a staged call used to start and join 15 threads per step, twice per
// sub-batch); a caller that finds the pool busy -- another context's call on
// another thread -- starts threads of its own for that step as before.
constexpr unsigned kHostThreads = 16;

class HostPool {
 public:
  static HostPool& get() {
    static HostPool* p = new HostPool;  // never destroyed: workers may be waiting at exit
    return *p;
  }
  // false: busy (the caller falls back)
  template <class F>
  bool run(size_t count, F& f) {
    std::unique_lock<std::mutex> busy(run_mu_, std::try_to_lock);
    if (!busy.owns_lock()) return false;
    {
      std::lock_guard<std::mutex> g(mu_);
      job_ = [](void* ctx, size_t i) { (*static_cast<F*>(ctx))(i); };
      ctx_ = &f;
      count_ = count;
      next_.store(0);
      active_ = workers_.size();
      ++gen_;
    }
    cv_.notify_all();
    drain(job_, ctx_, count);
    stream_fence();
    std::unique_lock<std::mutex> g(mu_);
    done_cv_.wait(g, [&] { return active_ == 0; });
    return true;
  }
  size_t threads() const { return workers_.size() + 1; }

 private:
  using Job = void (*)(void*, size_t);
  HostPool() {
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const unsigned t = std::min(kHostThreads, hw);
    for (unsigned w = 1; w < t; ++w) workers_.emplace_back([this] { loop(); });
    for (auto& th : workers_) th.detach();
  }
  void drain(Job job, void* ctx, size_t count) {
    for (size_t i = next_.fetch_add(1); i < count; i = next_.fetch_add(1)) job(ctx, i);
  }
  void loop() {
    size_t seen = 0;
    for (;;) {
      Job job;
      void* ctx;
      size_t count;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [&] { return gen_ != seen; });
        seen = gen_;
        job = job_, ctx = ctx_, count = count_;
      }
      drain(job, ctx, count);
      stream_fence();
      std::lock_guard<std::mutex> g(mu_);
      if (--active_ == 0) done_cv_.notify_one();
    }
  }
  std::vector<std::thread> workers_;
  std::mutex run_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  Job job_ = nullptr;
  void* ctx_ = nullptr;
  size_t count_ = 0, active_ = 0, gen_ = 0;
  std::atomic<size_t> next_{0};
};

template <class F>
void parallel_for(size_t count, F f) {
  if (count == 0) return;
  if (count > 1 && HostPool::get().threads() > 1 && HostPool::get().run(count, f)) return;
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

const char* np_last_error_site(void) { return g_site_msg; }

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

int np_debug_bounds_check(np_ctx* c, uint32_t out[8]) {
  if (!c || !out) return fail(NP_ERR_INVALID_ARGUMENT);
  (void)hipSetDevice(c->device);
  for (int i = 0; i < 8; ++i) out[i] = 0;
  hipError_t e = HIP(hipDeviceSynchronize());
  if (e != hipSuccess) return dev_err(e);
  hipError_t (*const take[])(uint32_t*) = {np::bounds_take_generic, np::bounds_take_fast, np::bounds_take_res,
                                            np::bounds_take_small, np::bounds_take_big, np::bounds_take_huge};
  for (auto f : take) {
    uint32_t r[8];
    e = f(r);
    if (e == hipErrorNotSupported) return fail(NP_ERR_INVALID_ARGUMENT);  // the product build: no checks
    if (e != hipSuccess) return dev_err(HIP(e));
    if (r[0] && !out[0])
      for (int i = 1; i < 8; ++i) out[i] = r[i];
    out[0] += r[0];
  }
  return NP_OK;
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
  c->big_cap = scratch_cap_for(device);
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
    c->pipe_cin[i].release();
    c->pipe_hin[i].release();
    c->pipe_hout[i].release();
    if (c->pipe_ev[i]) (void)hipEventDestroy(c->pipe_ev[i]);
    if (c->pipe_s[i]) (void)hipStreamDestroy(c->pipe_s[i]);
  }
  c->pipe_pres.release();
  c->h_in.release();
  c->h_out.release();
  c->h_pres.release();
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
}

void* np_ctx_stream(np_ctx* c) { return c ? static_cast<void*>(c->stream) : nullptr; }
int np_ctx_device(np_ctx* c) { return c ? c->device : -1; }

int np_ctx_synchronize(np_ctx* c) {
  if (!c) return fail(NP_ERR_INVALID_ARGUMENT);
  (void)hipSetDevice(c->device);
  hipError_t e = HIP(hipStreamSynchronize(c->stream));
  if (e == hipSuccess) e = HIP(hipStreamSynchronize(nullptr));  // the `_dev` calls given a NULL stream
  return dev_err(e);
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
  hipError_t e = HIP(c->d_in.ensure(len));
  if (e == hipSuccess) e = HIP(c->d_out.ensure(std::max<size_t>(out_bytes, 1)));
  if (e == hipSuccess) e = HIP(c->h_in.ensure(len));
  if (e == hipSuccess) e = HIP(c->h_out.ensure(std::max<size_t>(out_bytes, 1)));
  if (e != hipSuccess) return dev_err(e);
  std::memcpy(c->h_in.p, payload, len);
  e = HIP(hipMemcpyAsync(c->d_in.p, c->h_in.p, len, hipMemcpyHostToDevice, c->stream));
  np::EncodeArgs a = enc_args(p, c->d_in.as<uint8_t>(), len, len, 1, c->d_out.as<uint8_t>(), out_bytes);
  if (e == hipSuccess) e = HIP(launch_encode(c, a, c->stream));
  if (e == hipSuccess) e = HIP(hipMemcpyAsync(c->h_out.p, c->d_out.p, out_bytes, hipMemcpyDeviceToHost, c->stream));
  if (e == hipSuccess) e = HIP(hipStreamSynchronize(c->stream));
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
  return dev_err(HIP(launch_encode(c, a, pick(c, stream))));
}

}  // extern "C"

// ------------------------------------------------- host-memory pipeline ----
// the caller's view of encode / reconstruct, buffers in host
// memory.  The batch goes in sub-batches of about kPipeSlotBytes over
// np_ctx::kPipe streams; each sub-batch is H2D -> kernel -> D2H on its
// stream, so the copies of one overlap the kernels and the opposite-direction
// copies of the others (PCIe is full duplex).
//
// No pageable pointer is ever handed to a HIP copy.  Every host span of a
// call is one of
//  - pinned by the caller (hipHostMalloc, torch pin_memory, hipHostRegister;
//    mapped_host_range finds it): DMA, or the present-row gather kernel,
//    straight from / to it;
//  - with NP_PAGEABLE=pin (opt-in), pinned in place for the call through the
//    process-wide PinRegistry (pageable spans of at least kPinMinBytes): the
//    same;
//  - staged: host threads copy it into / out of the context's pinned staging
//    slots, and the DMA or the gather runs from / to those.
// Round 4 still let the runtime copy pageable spans whose rows were not
// 4-byte aligned (hipMemcpy2DAsync from a numpy array, right after the same
// pages had been registered and unregistered), and one GPU run faulted in
// that call.  Round 5 saw one more illegal address in a
// process that had pinned numpy buffers in place earlier (in device-only
// calls, not traced to any kernel), so pinning in place is opt-in.
namespace {

constexpr size_t kPipeSlotBytes = size_t(64) << 20;  // encode: payloads + shard rows per sub-batch
constexpr size_t kPipeMovedBytes = size_t(24) << 20;         // reconstruct: PCIe bytes per sub-batch
// Pageable spans below this are staged: registering and unregistering them
// costs more than copying them.
constexpr size_t kPinMinBytes = size_t(1) << 20;

// Device address of [p, p + bytes) when the whole range lies in one pinned host
// allocation mapped into the device address space (hipHostMalloc, torch's
// pin_memory, hipHostRegister), else nullptr (pageable memory).
const uint8_t* mapped_host_range(const uint8_t* p, size_t bytes) {
  if (bytes == 0) return nullptr;
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

// The page ranges this library registered in place, process-wide.
// hipHostRegister pins whole pages, so the range pinned for one span can share
// its first and last page with a neighbouring span: the adjacent slice of the
// same caller buffer on another thread (np_*_host_multi), or another call's
// buffer.  Each registered range is refcounted under one lock: a span inside a
// registered range takes a reference, a span that only partly overlaps one is
// staged instead, and the range is unregistered when its last reference goes
// -- after the streams of every call that used it have drained.
class PinRegistry {
 public:
  // The device address of [p, p + bytes) for the length of a call, or nullptr
  // (stage it).  In this order, under the registry lock: a span inside a range
  // registered here takes a reference (*base = that range); else memory the
  // caller pinned itself (mapped_host_range; no reference, the caller owns
  // it); else, with `may_pin` and at least kPinMinBytes, the span's pages are
  // registered here (*base = the new range).  One lock over the lookup, the
  // attribute query and the reference: no other call can unregister a
  // registry range between this call finding it mapped and taking its
  // reference (the lookup used to come first, outside the lock).
  const uint8_t* acquire(const uint8_t* p, size_t bytes, bool may_pin, uintptr_t* base) {
    *base = 0;
    if (bytes == 0) return nullptr;
    const uintptr_t a = reinterpret_cast<uintptr_t>(p) & ~uintptr_t(4095);
    const uintptr_t z = (reinterpret_cast<uintptr_t>(p) + bytes + 4095) & ~uintptr_t(4095);
    std::lock_guard<std::mutex> g(mu_);
    auto it = ranges_.upper_bound(a);  // the first range starting above a
    bool overlap = it != ranges_.end() && it->first < z;
    if (it != ranges_.begin()) {
      auto pv = std::prev(it);
      if (pv->second.end >= z) {
        const uint8_t* d = mapped_host_range(p, bytes);
        if (!d) return nullptr;  // (cannot happen while registered; stage)
        ++pv->second.refs;
        *base = pv->first;
        return d;
      }
      overlap = overlap || pv->second.end > a;
    }
    if (overlap) return nullptr;  // partly inside a registry range: stage
    if (const uint8_t* d = mapped_host_range(p, bytes)) return d;  // pinned by the caller
    if (!may_pin || bytes < kPinMinBytes) return nullptr;
    if (hipHostRegister(reinterpret_cast<void*>(a), z - a, hipHostRegisterMapped | hipHostRegisterPortable) !=
        hipSuccess) {
      (void)hipGetLastError();  // refused (e.g. the caller registered an overlapping range): stage
      return nullptr;
    }
    const uint8_t* d = mapped_host_range(p, bytes);
    if (!d) {
      unregister(a);
      return nullptr;
    }
    ranges_[a] = Range{z, 1};
    *base = a;
    return d;
  }
  void release(uintptr_t base) {
    std::lock_guard<std::mutex> g(mu_);
    auto it = ranges_.find(base);
    if (it == ranges_.end() || --it->second.refs) return;
    unregister(base);
    ranges_.erase(it);
  }
  // Unregistrations the runtime refused (np_pin_registry_stats): a refused one
  // leaves pages registered that the caller may free and the allocator may
  // hand out again, so it is counted and reported, never ignored.
  size_t failed_unregisters() const { return failed_.load(); }
  size_t live_ranges() {
    std::lock_guard<std::mutex> g(mu_);
    return ranges_.size();
  }

 private:
  void unregister(uintptr_t base) {
    const hipError_t e = hipHostUnregister(reinterpret_cast<void*>(base));
    if (e != hipSuccess) {
      (void)hipGetLastError();
      if (failed_.fetch_add(1) == 0)
        std::fprintf(stderr, "novelpoly: hipHostUnregister(%p) failed: %s\n", reinterpret_cast<void*>(base),
                     hipGetErrorName(e));
    }
  }
  struct Range {
    uintptr_t end;
    size_t refs;
  };
  std::mutex mu_;
  std::map<uintptr_t, Range> ranges_;
  std::atomic<size_t> failed_{0};
};

PinRegistry& pins() {
  static PinRegistry* r = new PinRegistry;  // never destroyed: calls may run during static destruction
  return *r;
}

// Slots (streams) of the host pipeline: 4 (config-3 / 4 reconstruct from
// pageable buffers 16.6 / 22.1 GiB/s with 3, 17.7 / 22.8 with 4, no better
// with 6; profiles/r06/pipe_probe2_cfg{3,4}.txt); NP_PIPE_SLOTS overrides
// (experiments).
int pipe_slots() {
  const char* e = std::getenv("NP_PIPE_SLOTS");
  return e ? std::min(np_ctx::kPipe, std::max(1, std::atoi(e))) : 4;
}

hipError_t pipe_init(np_ctx* c, int npipe) {
  for (int i = 0; i < npipe; ++i) {
    if (!c->pipe_s[i]) {
      hipError_t e = HIP(hipStreamCreateWithFlags(&c->pipe_s[i], hipStreamNonBlocking));
      if (e != hipSuccess) return e;
    }
    if (!c->pipe_ev[i]) {
      hipError_t e = HIP(hipEventCreateWithFlags(&c->pipe_ev[i], hipEventDisableTiming));
      if (e != hipSuccess) return e;
    }
  }
  return hipSuccess;
}

hipError_t pipe_sync(np_ctx* c, hipError_t e) {
  for (int i = 0; i < np_ctx::kPipe; ++i) {
    if (!c->pipe_s[i]) continue;
    const hipError_t r = HIP(hipStreamSynchronize(c->pipe_s[i]));
    if (e == hipSuccess) e = r;
  }
  return e;
}

// NP_SYNC_EACH=1: the host pipeline waits for its stream after every step, so
// that an asynchronous fault is reported at the step that caused it (its line
// and name in np_last_error_site) instead of at the final synchronisation.
hipError_t after(hipError_t e, hipStream_t s, int line, const char* step) {
  if (e != hipSuccess || !std::getenv("NP_SYNC_EACH")) return e;
  return at_site(hipStreamSynchronize(s), line, step);
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
// Pinned callers' present rows: packed by host threads and DMA'd (true) or
// gathered by k_copy_rows from the caller's memory (false); NP_HOST_ROWS
// overrides per call.
constexpr bool kPinnedPack = true;

// Pageable buffers are staged through pinned memory by host threads
// (default), or with NP_PAGEABLE=pin pinned in place for the call (read per
// call).
bool pageable_pin() {
  const char* m = std::getenv("NP_PAGEABLE");
  return m && std::strcmp(m, "pin") == 0;
}

// A host span for the length of a call: its device address when the caller
// pinned it or it was pinned in place here, else nullptr (staged).  Holds its
// registry reference until destroyed, so it must outlive every stream
// operation on the span (the calls synchronise their streams before return).
class HostSpan {
 public:
  HostSpan(const void* p, size_t bytes, bool may_pin)
      : dev_(pins().acquire(static_cast<const uint8_t*>(p), bytes, may_pin, &base_)) {}
  ~HostSpan() {
    if (base_) pins().release(base_);
  }
  HostSpan(const HostSpan&) = delete;
  HostSpan& operator=(const HostSpan&) = delete;
  const uint8_t* dev() const { return dev_; }
  bool pinned() const { return dev_ != nullptr; }

 private:
  uintptr_t base_ = 0;
  const uint8_t* dev_ = nullptr;
};

// Per-slot bookkeeping of a staged pipeline: a slot's pinned staging may be
// refilled once the sub-batch that last used it is done (its event), whose
// staged outputs are then handed to the caller (copy_out(b0, cnt, slot)).
// NP_PIPE_STATS=1: the host pipeline's time split (waits for slots, host
// copies out, packing, the rest) on stderr per call -- the measurements of
// DESIGN.md §4.7.
struct PipeStats {
  bool on = std::getenv("NP_PIPE_STATS") != nullptr;
  double wait = 0, out = 0, pack = 0;
  std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
  static double ms(std::chrono::steady_clock::time_point a) {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - a).count();
  }
  void report(const char* what, size_t sb, size_t batch) const {
    if (on)
      std::fprintf(stderr, "np pipe %s: %.3f ms, %zu sub-batches of %zu: wait %.3f, copy-out %.3f, pack %.3f\n", what,
                   ms(t0), (batch + sb - 1) / sb, sb, wait, out, pack);
  }
};

struct SlotRing {
  np_ctx* c;
  PipeStats* st = nullptr;
  size_t b0[np_ctx::kPipe] = {}, cnt[np_ctx::kPipe] = {};
  template <class F>
  void drain(int sl, hipError_t& e, F copy_out) {
    if (!cnt[sl]) return;
    auto t = std::chrono::steady_clock::now();
    const hipError_t r = HIP(hipEventSynchronize(c->pipe_ev[sl]));
    if (st) st->wait += PipeStats::ms(t);
    if (e == hipSuccess) e = r;
    t = std::chrono::steady_clock::now();
    if (r == hipSuccess) copy_out(b0[sl], cnt[sl], sl);
    if (st) st->out += PipeStats::ms(t);
    cnt[sl] = 0;
  }
  hipError_t mark(int sl, hipStream_t s, size_t first, size_t count) {
    const hipError_t e = HIP(hipEventRecord(c->pipe_ev[sl], s));
    if (e == hipSuccess) b0[sl] = first, cnt[sl] = count;
    return e;
  }
};

// cnt blocks of `len` bytes, src + b * sstride -> dst + b * dstride, on host
// threads in pieces of at most 1 MiB.
void copy_blocks(uint8_t* dst, size_t dstride, const uint8_t* src, size_t sstride, size_t len, size_t cnt) {
  const size_t pieces = (len + (size_t(1) << 20) - 1) >> 20;
  parallel_for(cnt * pieces, [&](size_t i) {
    const size_t b = i / pieces, off = (i % pieces) << 20, l = std::min<size_t>(len - off, size_t(1) << 20);
    stream_copy(dst + b * dstride + off, src + b * sstride + off, l);
  });
}

}  // namespace

extern "C" {

void np_pin_registry_stats(size_t out[2]) {
  if (!out) return;
  out[0] = pins().live_ranges();
  out[1] = pins().failed_unregisters();
}

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
  const size_t span_in = (batch - 1) * pstride + len, span_out = (batch - 1) * bstride + row_bytes;
  const bool may_pin = pageable_pin();
  const HostSpan hin(payloads, span_in, may_pin), hout(shards, span_out, may_pin);
  const bool st_in = !hin.pinned(), st_out = !hout.pinned();
  const int npipe = pipe_slots();
  hipError_t e = pipe_init(c, npipe);
  const size_t sb = std::min(batch, std::max<size_t>(1, kPipeSlotBytes / (len + row_bytes)));
  for (int i = 0; e == hipSuccess && i < npipe; ++i) {
    e = HIP(c->pipe_in[i].ensure(sb * len));
    if (e == hipSuccess) e = HIP(c->pipe_out[i].ensure(sb * row_bytes));
    if (e == hipSuccess && st_in) e = HIP(c->pipe_hin[i].ensure(sb * len));
    if (e == hipSuccess && st_out) e = HIP(c->pipe_hout[i].ensure(sb * row_bytes));
  }
  SlotRing ring{c};
  auto copy_out = [&](size_t b0, size_t cnt, int sl) {  // staged shard rows -> the caller's buffer
    if (st_out) copy_blocks(shards + b0 * bstride, bstride, c->pipe_hout[sl].as<uint8_t>(), row_bytes, row_bytes, cnt);
  };
  int slot = 0;
  for (size_t b0 = 0; e == hipSuccess && b0 < batch; b0 += sb, slot = (slot + 1) % npipe) {
    const size_t cnt = std::min(sb, batch - b0);
    hipStream_t s = c->pipe_s[slot];
    uint8_t* din = c->pipe_in[slot].as<uint8_t>();
    uint8_t* dout = c->pipe_out[slot].as<uint8_t>();
    ring.drain(slot, e, copy_out);  // the slot's staging is free again
    if (e != hipSuccess) break;
    if (st_in) {
      uint8_t* h = c->pipe_hin[slot].as<uint8_t>();
      copy_blocks(h, len, payloads + b0 * pstride, pstride, len, cnt);
      e = HIP(hipMemcpyAsync(din, h, cnt * len, hipMemcpyHostToDevice, s));
    } else {
      e = HIP(hipMemcpy2DAsync(din, len, payloads + b0 * pstride, pstride, len, cnt, hipMemcpyHostToDevice, s));
    }
    e = after(e, s, __LINE__, "payloads H2D");
    if (e == hipSuccess) e = HIP(launch_encode(c, enc_args(p, din, len, len, cnt, dout, row_bytes), s));
    e = after(e, s, __LINE__, "encode kernels");
    if (e == hipSuccess)
      e = st_out ? HIP(hipMemcpyAsync(c->pipe_hout[slot].p, dout, cnt * row_bytes, hipMemcpyDeviceToHost, s))
                 : HIP(hipMemcpy2DAsync(shards + b0 * bstride, bstride, dout, row_bytes, row_bytes, cnt,
                                        hipMemcpyDeviceToHost, s));
    e = after(e, s, __LINE__, "shard rows D2H");
    if (e == hipSuccess && (st_in || st_out)) e = ring.mark(slot, s, b0, cnt);
  }
  // the pending slots, oldest first: `slot` is the next one the loop would
  // have used, i.e. the one used longest ago
  for (int i = 0; i < npipe; ++i) ring.drain((slot + i) % npipe, e, copy_out);
  return dev_err(pipe_sync(c, e));
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
  const size_t n = p->n, rows = rows_needed(p, shard_len, present, batch), in_bytes = rows * shard_len,
               dstride = n * shard_len;
  std::lock_guard<std::mutex> g(c->mu);
  (void)hipSetDevice(c->device);
  const size_t span_in = (batch - 1) * bstride + in_bytes, span_out = (batch - 1) * out_stride + olen;
  const bool may_pin = pageable_pin();
  const HostSpan hin(shards, span_in, may_pin), hout(out, span_out, may_pin);
  const bool st_in = !hin.pinned(), st_out = !hout.pinned();
  // How the present rows (682 of 1024 per payload at config 3, 1366 of 4096
  // at config 4) reach the device:
  //  - pack: host threads pack a sub-batch's present rows one after the other
  //    into the slot's pinned staging, with each row's device offset; one DMA
  //    moves both, and k_expand_rows puts the rows in place (HBM to HBM).
  //    Staged (pageable) spans always go this way: the host copy is needed
  //    anyway, and DMA in both directions shares PCIe better than kernel
  //    reads of host memory next to a DMA D2H;
  //  - gather: k_copy_rows reads the present rows straight from the caller's
  //    pinned rows (4-byte aligned), no host copy;
  //  - dma2d: the first `rows` rows of every payload by one 2-D DMA (pinned,
  //    unaligned rows).
  // Pinned callers: NP_HOST_ROWS=pack / gather picks (read per call; default
  // below, measured in DESIGN.md §4.7).
  enum class Rows { Pack, Gather, Dma2d };
  const bool aligned = ((reinterpret_cast<uintptr_t>(shards) | bstride | shard_len) & 3) == 0;
  const char* hr = std::getenv("NP_HOST_ROWS");
  const int npipe = pipe_slots();
  hipError_t e = pipe_init(c, npipe);
  // Sub-batches of about kPipeMovedBytes of PCIe traffic (the present rows in,
  // the outputs out): 7 payloads at config 3, 3 at config 4 (the best of
  // profiles/r06/pipe_probe2_cfg{3,4}.txt); NP_PIPE_SB (payloads) overrides.
  size_t moved = 0;  // present rows the kernels read, over the whole call
  for (size_t b = 0; b < batch; ++b)
    for (size_t v = 0; v < rows; ++v) moved += present[b * n + v] ? 1 : 0;
  const size_t per = moved * shard_len / batch + olen;
  size_t sb = std::min(batch, std::max<size_t>(1, (kPipeMovedBytes + per - 1) / per));
  if (const char* v = std::getenv("NP_PIPE_SB")) sb = std::min(batch, std::max<size_t>(1, std::strtoul(v, nullptr, 10)));
  // Pinned callers: packed when the call pipelines several sub-batches; a call
  // of one sub-batch has nothing to overlap the packing with, so its aligned
  // rows go by the gather (one payload at config 3: 0.20 ms against 0.29).
  const bool pinned_pack = hr ? std::strcmp(hr, "pack") == 0 : kPinnedPack && (batch > sb || !aligned);
  const Rows mode = st_in || pinned_pack ? Rows::Pack : aligned ? Rows::Gather : Rows::Dma2d;
  const size_t slot_in = (sb - 1) * dstride + in_bytes;
  const size_t nblk = (rows + 63) / 64;  // packing tasks per payload: 64 rows each
  const size_t pack_cap = (sb * rows * 8 + 255) / 256 * 256 + sb * rows * shard_len;  // offsets, then rows
  for (int i = 0; e == hipSuccess && i < npipe; ++i) {
    e = HIP(c->pipe_in[i].ensure(slot_in));
    if (e == hipSuccess) e = HIP(c->pipe_out[i].ensure(sb * olen));
    if (e == hipSuccess && mode == Rows::Pack) e = HIP(c->pipe_hin[i].ensure(pack_cap));
    if (e == hipSuccess && mode == Rows::Pack) e = HIP(c->pipe_cin[i].ensure(pack_cap));
    if (e == hipSuccess && st_out) e = HIP(c->pipe_hout[i].ensure(sb * olen));
  }
  // the whole present mask up front, through pinned staging, before any
  // sub-batch reads it
  if (e == hipSuccess) e = HIP(c->pipe_pres.ensure(batch * n));
  if (e == hipSuccess) e = HIP(c->h_pres.ensure(batch * n));
  if (e == hipSuccess) {
    std::memcpy(c->h_pres.p, present, batch * n);
    e = HIP(hipMemcpyAsync(c->pipe_pres.p, c->h_pres.p, batch * n, hipMemcpyHostToDevice, c->pipe_s[0]));
  }
  if (e == hipSuccess) e = HIP(hipStreamSynchronize(c->pipe_s[0]));
  PipeStats stats;
  SlotRing ring{c, &stats};
  auto copy_out = [&](size_t b0, size_t cnt, int sl) {  // staged outputs -> the caller's buffer
    if (st_out) copy_blocks(out + b0 * out_stride, out_stride, c->pipe_hout[sl].as<uint8_t>(), olen, olen, cnt);
  };
  std::vector<size_t> base;  // packed index of the first present row of each (payload, 64-row block)
  int slot = 0;
  for (size_t b0 = 0; e == hipSuccess && b0 < batch; b0 += sb, slot = (slot + 1) % npipe) {
    const size_t cnt = std::min(sb, batch - b0);
    hipStream_t s = c->pipe_s[slot];
    uint8_t* din = c->pipe_in[slot].as<uint8_t>();
    uint8_t* dout = c->pipe_out[slot].as<uint8_t>();
    const uint8_t* dpres = c->pipe_pres.as<uint8_t>() + b0 * n;
    ring.drain(slot, e, copy_out);  // the slot's staging is free again
    if (e != hipSuccess) break;
    const uint8_t* src = shards + b0 * bstride;
    if (mode == Rows::Pack) {
      base.assign(cnt * nblk + 1, 0);
      for (size_t t = 0; t < cnt * nblk; ++t) {
        const uint8_t* pr = present + (b0 + t / nblk) * n + 64 * (t % nblk);
        const size_t m = std::min<size_t>(64, rows - 64 * (t % nblk));
        size_t have = 0;
        for (size_t v = 0; v < m; ++v) have += pr[v] ? 1 : 0;
        base[t + 1] = base[t] + have;
      }
      const size_t total = base.back(), list_bytes = (total * 8 + 255) / 256 * 256;
      uint8_t* h = c->pipe_hin[slot].as<uint8_t>();
      uint64_t* list = reinterpret_cast<uint64_t*>(h);
      uint8_t* data = h + list_bytes;
      const auto tp = std::chrono::steady_clock::now();
      parallel_for(cnt * nblk, [&](size_t t) {
        const size_t b = t / nblk, v0 = 64 * (t % nblk), m = std::min<size_t>(64, rows - v0);
        const uint8_t* pr = present + (b0 + b) * n + v0;
        size_t j = base[t];
        for (size_t v = 0; v < m; ++v) {
          if (!pr[v]) continue;
          stream_copy(data + j * shard_len, src + b * bstride + (v0 + v) * shard_len, shard_len);
          list[j++] = b * dstride + (v0 + v) * shard_len;
        }
      });
      stats.pack += PipeStats::ms(tp);
      uint8_t* cin = c->pipe_cin[slot].as<uint8_t>();
      e = HIP(hipMemcpyAsync(cin, h, list_bytes + total * shard_len, hipMemcpyHostToDevice, s));
      e = after(e, s, __LINE__, "packed rows H2D");
      if (e == hipSuccess)
        e = HIP(np::launch_expand_rows(cin + list_bytes, reinterpret_cast<const uint64_t*>(cin), din, shard_len, total, s));
      e = after(e, s, __LINE__, "packed rows expand");
    } else if (mode == Rows::Gather) {
      e = HIP(np::launch_copy_rows(hin.dev() + b0 * bstride, bstride, din, dstride, shard_len, dpres,
                                   static_cast<uint32_t>(n), static_cast<uint32_t>(rows), cnt, kGatherBlocks, s));
      e = after(e, s, __LINE__, "present-row gather");
    } else {
      e = HIP(hipMemcpy2DAsync(din, dstride, src, bstride, in_bytes, cnt, hipMemcpyHostToDevice, s));
      e = after(e, s, __LINE__, "shard rows H2D");
    }
    if (e == hipSuccess) {
      np::ReconstructArgs a{};
      a.shards = din;
      a.shard_len = shard_len;
      a.batch_stride = dstride;
      a.present = dpres;
      a.locators = nullptr;  // computed on the device
      a.batch = cnt;
      a.n = static_cast<uint32_t>(n);
      a.k = static_cast<uint32_t>(p->k);
      a.out = dout;
      a.out_stride = olen;
      e = HIP(launch_reconstruct(c, a, s));
    }
    e = after(e, s, __LINE__, "reconstruct kernels");
    if (e == hipSuccess)
      e = st_out ? HIP(hipMemcpyAsync(c->pipe_hout[slot].p, dout, cnt * olen, hipMemcpyDeviceToHost, s))
                 : HIP(hipMemcpy2DAsync(out + b0 * out_stride, out_stride, dout, olen, olen, cnt,
                                        hipMemcpyDeviceToHost, s));
    e = after(e, s, __LINE__, "outputs D2H");
    if (e == hipSuccess && (mode == Rows::Pack || st_out)) e = ring.mark(slot, s, b0, cnt);
  }
  // the pending slots, oldest first (a failed call still waits for its streams)
  for (int i = 0; i < npipe; ++i) ring.drain((slot + i) % npipe, e, copy_out);
  e = pipe_sync(c, e);
  stats.report(mode == Rows::Pack ? "reconstruct (pack)" : mode == Rows::Gather ? "reconstruct (gather)" : "reconstruct (2-D DMA)", sb, batch);
  return dev_err(e);
}

// ---------------------------------------------------------- reconstruct ----
int np_error_locator_dev(np_ctx* c, size_t n, const uint8_t* d_present, size_t batch, uint16_t* d_loc,
                         void* stream) {
  if (!c || !d_present || !d_loc || !is_pow2(n) || n > np::kFieldSize) return fail(NP_ERR_INVALID_ARGUMENT);
  (void)hipSetDevice(c->device);
  return dev_err(HIP(np::launch_error_locator(c->T, static_cast<uint32_t>(n), d_present, batch, d_loc, pick(c, stream))));
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
#if NP_BOUNDS_CHECK
  if (const char* st = std::getenv("NP_BOUNDS_SELFTEST")) a.chk_shrink_out = static_cast<uint32_t>(std::atoi(st));
#endif
  return dev_err(HIP(launch_reconstruct(c, a, pick(c, stream))));
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
  // the present mask through pinned staging (no pageable pointer reaches a HIP copy, §4.7)
  hipError_t e = HIP(c->d_present.ensure(std::max<size_t>(batch * p->n, 1)));
  if (e == hipSuccess) e = HIP(c->h_pres.ensure(std::max<size_t>(batch * p->n, 1)));
  if (e != hipSuccess) return dev_err(e);
  std::memcpy(c->h_pres.p, present, batch * p->n);
  e = HIP(hipMemcpyAsync(c->d_present.p, c->h_pres.p, batch * p->n, hipMemcpyHostToDevice, s));
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
  e = HIP(launch_reconstruct(c, a, s));
  if (e != hipSuccess) return dev_err(e);
  // the staged present mask is the context's: the call returns once the
  // stream is done with it
  return dev_err(HIP(hipStreamSynchronize(s)));
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
  hipError_t e = HIP(c->h_in.ensure(n * sl));
  if (e == hipSuccess) e = HIP(c->d_in.ensure(n * sl));
  if (e == hipSuccess) e = HIP(c->d_out.ensure(need));
  if (e == hipSuccess) e = HIP(c->h_out.ensure(need));
  if (e == hipSuccess) e = HIP(c->d_present.ensure(n));
  if (e == hipSuccess) e = HIP(c->h_pres.ensure(n));
  if (e != hipSuccess) return dev_err(e);
  std::memcpy(c->h_pres.p, present.data(), n);
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
  e = HIP(hipMemcpyAsync(c->d_in.p, stage, n * sl, hipMemcpyHostToDevice, s));
  if (e == hipSuccess) e = HIP(hipMemcpyAsync(c->d_present.p, c->h_pres.p, n, hipMemcpyHostToDevice, s));
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
    e = HIP(launch_reconstruct(c, a, s));
  }
  if (e == hipSuccess) e = HIP(hipMemcpyAsync(c->h_out.p, c->d_out.p, need, hipMemcpyDeviceToHost, s));
  if (e == hipSuccess) e = HIP(hipStreamSynchronize(s));
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
  hipError_t e = HIP(c->h_in.ensure(k * sl));
  if (e == hipSuccess) e = HIP(c->d_in.ensure(k * sl));
  if (e == hipSuccess) e = HIP(c->d_out.ensure(need));
  if (e == hipSuccess) e = HIP(c->h_out.ensure(need));
  if (e != hipSuccess) return dev_err(e);
  uint8_t* stage = c->h_in.as<uint8_t>();
  for (size_t j = 0; j < k; ++j) {
    std::memcpy(stage + j * sl, chunks[j], lens[j]);
    if (lens[j] < sl) std::memset(stage + j * sl + lens[j], 0, sl - lens[j]);  // WrappedShard zero pad
  }
  hipStream_t s = c->stream;
  e = HIP(hipMemcpyAsync(c->d_in.p, stage, k * sl, hipMemcpyHostToDevice, s));
  if (e == hipSuccess) e = np::launch_systematic(c->d_in.as<uint8_t>(), sl, k * sl, static_cast<uint32_t>(k), 1,
                                                 c->d_out.as<uint8_t>(), need, s);
  if (e == hipSuccess) e = HIP(hipMemcpyAsync(c->h_out.p, c->d_out.p, need, hipMemcpyDeviceToHost, s));
  if (e == hipSuccess) e = HIP(hipStreamSynchronize(s));
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
  return dev_err(HIP(np::launch_systematic(d_shards, shard_len, bstride, static_cast<uint32_t>(p->k), batch, d_out,
                                       out_stride, pick(c, stream))));
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
  std::vector<std::string> site(nctx);  // the worker's np_last_error_site text (thread-local there)
  std::vector<std::thread> th;
  th.reserve(nctx);
  for (size_t i = 0; i < nctx; ++i) {
    size_t b0 = 0, cnt = 0;
    np_batch_split(batch, nctx, i, &b0, &cnt);
    th.emplace_back([&, i, b0, cnt] {
      st[i] = cnt ? fn(i, b0, cnt) : NP_OK;
      np_last_error_detail(det[i].data());
      site[i] = g_site_msg;
    });
  }
  for (auto& t : th) t.join();
  for (size_t i = 0; i < nctx; ++i)
    if (st[i] != NP_OK) {
      const int r = fail(st[i], det[i][0], det[i][1], det[i][2]);
      std::snprintf(g_site_msg, sizeof g_site_msg, "%s", site[i].c_str());
      return r;
    }
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
    int st = np_encode_batch_dev(ctxs[i], p, d_payloads[i], len, pstride, cnt, d_shards[i], bstride, ctxs[i]->stream);
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
                                       d_out[i], out_stride, d_status ? d_status[i] : nullptr, ctxs[i]->stream);
    return st ? st : np_ctx_synchronize(ctxs[i]);
  });
}

int np_encode_batch_host_multi(np_ctx* const* ctxs, size_t nctx, const np_code_params* p, const uint8_t* payloads,
                               size_t len, size_t pstride, size_t batch, uint8_t* shards, size_t bstride) {
  if (!payloads || !shards) return fail(NP_ERR_INVALID_ARGUMENT);
  if (int st = check_params(p)) return st;
  // Pageable spans pinned once for all devices' ranges: the
  // workers' spans then lie inside one registration, and adjacent ranges that
  // share a page never register or unregister it under each other's copies.
  const size_t sl = np_shard_len(p, len), row_bytes = p->wanted_n * sl;
  const bool whole = batch && len && pstride >= len && bstride >= row_bytes && pageable_pin();
  const HostSpan hin(payloads, whole ? (batch - 1) * pstride + len : 0, whole),
      hout(shards, whole ? (batch - 1) * bstride + row_bytes : 0, whole);
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
  // pinned once for all ranges, as in np_encode_batch_host_multi; a worker
  // ships at most the rows the whole batch needs
  const size_t olen = (shard_len / 2) * 2 * p->k;
  const bool whole = batch && shard_len && !(shard_len & 1) && bstride >= p->n * shard_len && out_stride >= olen &&
                     pageable_pin();
  const size_t rows = whole ? rows_needed(p, shard_len, present, batch) : 0;
  const HostSpan hin(shards, whole ? (batch - 1) * bstride + rows * shard_len : 0, whole),
      hout(out, whole ? (batch - 1) * out_stride + olen : 0, whole);
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
  return dev_err(HIP(np::launch_afft(c->T, d, static_cast<uint32_t>(size), static_cast<uint32_t>(index), cols, false,
                                 pick(c, stream))));
}

int np_inverse_afft_dev(np_ctx* c, uint16_t* d, size_t size, size_t index, size_t cols, void* stream) {
  if (!c || !d || !is_pow2(size) || size > np::kFieldSize || index + size > np::kFieldSize)
    return fail(NP_ERR_INVALID_ARGUMENT);
  (void)hipSetDevice(c->device);
  return dev_err(HIP(np::launch_afft(c->T, d, static_cast<uint32_t>(size), static_cast<uint32_t>(index), cols, true,
                                 pick(c, stream))));
}

int np_walsh_dev(np_ctx* c, uint16_t* d, size_t size, void* stream) {
  if (!c || !d || !is_pow2(size) || size > np::kFieldSize) return fail(NP_ERR_INVALID_ARGUMENT);
  (void)hipSetDevice(c->device);
  return dev_err(HIP(np::launch_walsh(d, static_cast<uint32_t>(size), pick(c, stream))));
}

int np_mul_dev(np_ctx* c, const uint16_t* a, const uint16_t* m, uint16_t* o, size_t count, void* stream) {
  if (!c || !a || !m || !o) return fail(NP_ERR_INVALID_ARGUMENT);
  (void)hipSetDevice(c->device);
  return dev_err(HIP(np::launch_mul(c->T, a, m, o, count, pick(c, stream))));
}

int np_encode_low_dev(np_ctx* c, const uint16_t* d, size_t k, uint16_t* cw, size_t n, size_t cols, void* stream) {
  if (!c || !d || !cw || !is_pow2(n) || !is_pow2(k) || 2 * k > n || n > np::kFieldSize)
    return fail(NP_ERR_INVALID_ARGUMENT);
  (void)hipSetDevice(c->device);
  return dev_err(HIP(
      np::launch_encode_low(c->T, d, static_cast<uint32_t>(k), cw, static_cast<uint32_t>(n), cols, pick(c, stream))));
}

int np_decode_main_dev(np_ctx* c, uint16_t* cw, size_t upto, const uint8_t* d_present, const uint16_t* d_loc,
                       size_t n, size_t cols, void* stream) {
  if (!c || !cw || !d_present || !d_loc || !is_pow2(n) || n > np::kFieldSize || upto > n)
    return fail(NP_ERR_INVALID_ARGUMENT);
  (void)hipSetDevice(c->device);
  return dev_err(HIP(np::launch_decode_main(c->T, cw, static_cast<uint32_t>(upto), d_present, d_loc,
                                        static_cast<uint32_t>(n), cols, pick(c, stream))));
}

}  // extern "C"
