// Generic gfx950 kernels: correct for every power-of-two n <= 65536 and
// k <= n/2 (any CodeParams the crate can derive).  One workgroup owns a
// tile of codeword columns held in LDS; its 256 threads sweep the butterflies
// of each transform level.  The multiply is the crate's LOG/EXP gather
// (inc_log_mul.rs:42-49) from L2-resident tables, so this path is the
// correctness fallback, not the fast path (kernels_fast.hip).
#include "device_common.hpp"
#include "launchers.hpp"

namespace np {
namespace {

constexpr int kThreads = 256;
constexpr uint32_t kLdsBudgetSyms = 32768;  // 64 KiB of u16 per workgroup by default

// One level of the additive FFT / inverse FFT over `nseg` segments of `size`
// symbols.  Segment g starts at lds + seg_base(g) and uses skew index offset
// seg_index(g) (inc_afft.rs:139-214 / 267-332).
struct Segs {
  uint32_t col_stride;  // symbols between columns
  uint32_t first_off;   // offset of segment 0 within a column
  uint32_t seg_per_col; // segments per column
  uint32_t size;        // symbols per segment
  uint32_t index0;      // skew index of segment 0
  uint32_t index_step;  // skew index increment per segment (= size for encode shifts)
};

template <bool INVERSE>
__device__ void lds_transform(const DevTables& T, uint16_t* lds, const Segs& sg, uint32_t ncols) {
  const uint32_t half = sg.size >> 1;
  const uint32_t total = ncols * sg.seg_per_col * half;
  for (uint32_t step = 0; (1u << step) < sg.size; ++step) {
    const uint32_t d = INVERSE ? (1u << step) : (half >> step);
    for (uint32_t b = threadIdx.x; b < total; b += blockDim.x) {
      const uint32_t seg = b / half, r = b - seg * half;
      const uint32_t col = seg / sg.seg_per_col, sc = seg - col * sg.seg_per_col;
      uint16_t* v = lds + col * sg.col_stride + sg.first_off + sc * sg.size;
      const uint32_t grp = r / d, off = r - grp * d;
      const uint32_t i = grp * 2 * d + off;
      const uint32_t j = grp * 2 * d + d;  // group key, inc_afft.rs:457 / 573
      const uint32_t sk = T.skew[j + sg.index0 + sc * sg.index_step - 1];
      uint32_t x = v[i], y = v[i + d];
      if (INVERSE) {
        y ^= x;
        if (sk != kQ) x ^= gf_mul_log(T, y, sk);
      } else {
        if (sk != kQ) x ^= gf_mul_log(T, y, sk);
        y ^= x;
      }
      v[i] = static_cast<uint16_t>(x);
      v[i + d] = static_cast<uint16_t>(y);
    }
    __syncthreads();
  }
}

// Formal derivative restricted to outputs [0, upto) of each column, in place
// (inc_afft.rs:17-31; closed form SURVEY F7).  Outputs are produced in
// increasing order in chunks of blockDim.x; a chunk only reads positions >= its
// own first position, so in-place update after a barrier is exact.
__device__ void lds_formal_derivative(uint16_t* lds, uint32_t col_stride, uint32_t n, uint32_t upto,
                                      uint32_t ncols) {
  const uint32_t total = ncols * upto;
  for (uint32_t base = 0; base < total; base += blockDim.x) {
    const uint32_t e = base + threadIdx.x;
    uint32_t acc = 0, col = 0, j = 0;
    if (e < total) {
      col = e / upto;
      j = e - col * upto;
      const uint16_t* v = lds + col * col_stride;
      acc = v[j];
      for (uint32_t l = 1; l < n; l <<= 1)
        if (!(j & l)) acc ^= v[j | l];
    }
    __syncthreads();
    if (e < total) lds[col * col_stride + j] = static_cast<uint16_t>(acc);
    __syncthreads();
  }
}

uint32_t cols_for(uint32_t syms_per_col) {
  uint32_t c = kLdsBudgetSyms / syms_per_col;
  if (c < 1) c = 1;
  if (c > 64) c = 64;
  return c;
}

// ---------------------------------------------------------------- encode ----
// grid = (tiles of chunks, batch).  mod.rs:144-154 + inc_encode.rs:165-208.
__global__ __launch_bounds__(kThreads) void k_encode_generic(DevTables T, EncodeArgs a, uint32_t nchunks,
                                                             uint32_t cols) {
  extern __shared__ uint16_t lds[];
  const size_t b = blockIdx.y;
  const uint32_t ch0 = blockIdx.x * cols;
  const uint32_t ncol = min(cols, nchunks - ch0);
  const uint32_t n = a.n, k = a.k;
  const uint8_t* p = a.payloads + b * a.payload_stride;
  uint8_t* out = a.shards + b * a.batch_stride;

  for (uint32_t e = threadIdx.x; e < ncol * k; e += blockDim.x) {
    const uint32_t c = e / k, i = e - c * k;
    lds[c * n + i] = be_sym(p, (static_cast<size_t>(ch0 + c) * k + i) * 2, a.payload_len);
  }
  __syncthreads();
  // systematic part: codeword[0..k) == data (inc_encode.rs:47)
  const uint32_t sys = min(k, a.wanted_n);
  for (uint32_t e = threadIdx.x; e < sys * ncol; e += blockDim.x) {
    const uint32_t v = e / ncol, c = e - v * ncol;
    const uint16_t s = lds[c * n + v];
    uint8_t* q = out + static_cast<size_t>(v) * a.shard_len + 2 * static_cast<size_t>(ch0 + c);
    q[0] = static_cast<uint8_t>(s >> 8);
    q[1] = static_cast<uint8_t>(s);
  }
  __syncthreads();
  lds_transform<true>(T, lds, Segs{n, 0, 1, k, 0, 0}, ncol);  // inverse_afft(k, 0)
  const uint32_t nseg = n / k - 1;
  for (uint32_t e = threadIdx.x; e < ncol * nseg * k; e += blockDim.x) {
    const uint32_t c = e / (nseg * k), r = e - c * nseg * k;
    lds[c * n + k + r] = lds[c * n + (r % k)];
  }
  __syncthreads();
  lds_transform<false>(T, lds, Segs{n, k, nseg, k, k, k}, ncol);  // afft(k, shift) per shift
  for (uint32_t e = threadIdx.x; e < (a.wanted_n > k ? a.wanted_n - k : 0) * ncol; e += blockDim.x) {
    const uint32_t v = k + e / ncol, c = e % ncol;
    const uint16_t s = lds[c * n + v];
    uint8_t* q = out + static_cast<size_t>(v) * a.shard_len + 2 * static_cast<size_t>(ch0 + c);
    q[0] = static_cast<uint8_t>(s >> 8);
    q[1] = static_cast<uint8_t>(s);
  }
}

// ----------------------------------------------------------- reconstruct ----
// grid = (tiles of symbol columns, batch).  mod.rs:221-236 + inc_reconstruct.rs:1-85.
// The forward FFT is pruned to the first k outputs: for index 0 the left
// group of every level >= k has the zero skew (skews[2^m - 1] == sentinel), so
// positions [0,k) only see afft(k, 0) -- bit-exact with decode_main.
__global__ __launch_bounds__(kThreads) void k_reconstruct_generic(DevTables T, ReconstructArgs a, uint32_t nsyms,
                                                                  uint32_t cols) {
  extern __shared__ uint16_t lds[];
  const size_t b = blockIdx.y;
  const uint32_t s0 = blockIdx.x * cols;
  const uint32_t ncol = min(cols, nsyms - s0);
  const uint32_t n = a.n, k = a.k;
  if (a.status && a.status[2 * b] != 0) return;  // fewer than k present rows (k_payload_status)
  const uint8_t* sh = a.shards + b * a.batch_stride;
  const uint8_t* pres = a.present + b * n;
  const uint16_t* loc = a.locators + b * n;

  for (uint32_t e = threadIdx.x; e < ncol * n; e += blockDim.x) {
    const uint32_t v = e / ncol, c = e - v * ncol;
    uint16_t w = 0;
    if (pres[v]) {
      const uint8_t* q = sh + static_cast<size_t>(v) * a.shard_len + 2 * static_cast<size_t>(s0 + c);
      w = gf_mul_log(T, (uint32_t(q[0]) << 8) | q[1], loc[v]);
    }
    lds[c * n + v] = w;
  }
  __syncthreads();
  lds_transform<true>(T, lds, Segs{n, 0, 1, n, 0, 0}, ncol);
  lds_formal_derivative(lds, n, n, k, ncol);
  lds_transform<false>(T, lds, Segs{n, 0, 1, k, 0, 0}, ncol);
  uint8_t* out = a.out + b * a.out_stride;
  for (uint32_t e = threadIdx.x; e < ncol * k; e += blockDim.x) {
    const uint32_t c = e / k, j = e - c * k;
    uint32_t w;
    if (pres[j]) {
      const uint8_t* q = sh + static_cast<size_t>(j) * a.shard_len + 2 * static_cast<size_t>(s0 + c);
      w = (uint32_t(q[0]) << 8) | q[1];
    } else {
      w = gf_mul_log(T, lds[c * n + j], loc[j]);
    }
    uint8_t* o = out + static_cast<size_t>(s0 + c) * 2 * k + 2 * j;
    o[0] = static_cast<uint8_t>(w >> 8);
    o[1] = static_cast<uint8_t>(w);
  }
}

// ------------------------------------------------------------- locator ----
// inc_reconstruct.rs:90-113 over the full field (mod.rs:217-218), one
// workgroup per erasure pattern, 128 KiB of LDS.
__device__ void lds_walsh(uint16_t* v, uint32_t size) {
  for (uint32_t h = 1; h < size; h <<= 1) {
    for (uint32_t b = threadIdx.x; b < size / 2; b += blockDim.x) {
      const uint32_t g = b / h, off = b - g * h;
      const uint32_t i = g * 2 * h + off;
      const uint32_t x = v[i], y = v[i + h];
      const uint32_t s = x + y, t = x + kQ - y;
      v[i] = static_cast<uint16_t>((s & 0xffffu) + (s >> 16));
      v[i + h] = static_cast<uint16_t>((t & 0xffffu) + (t >> 16));
    }
    __syncthreads();
  }
}

// The locator of one payload in registers: position i of the 65536-point
// Walsh transforms lives in thread t, register r of one of three layouts,
// each holding a different 6 (or 4) bits of i in r, so each pass of levels
// runs in registers and the passes meet through the LDS (four exchanges
// instead of one barrier per level):
//   A  i = 64 t + r                      levels 0-5   (r = bits 0-5)
//   B  i = 4096 w + 64 r + lane          levels 6-11  (t = 64 w + lane)
//   C  i = 1024 r + t                    levels 12-15 (r bits 2-5)
// The first transform (of 0 / 1 erasure flags) is exact in integers, so its
// levels run in any order (C, B, A) and one reduction mod 65535 follows
// (only its residue enters the product, inc_reconstruct.rs:103-106).  The
// second keeps the reference's per-level end-around-carry form and its level
// order 0..15 (inc_log_mul.rs:92-114), which decides whether a zero residue
// reads 0 or 65535.
// LDS slot of position i: i + 2 (i >> 6), one dword of padding per 64
// positions, so A's 64-position stride falls on distinct banks and every
// layout's address is a per-thread base plus a constant (65536 + 2048 u16 =
// 132 KiB).
constexpr uint32_t kLocLdsBytes = 2u * (65536u + 2048u);

template <int B0, int NB>
__device__ __forceinline__ void walsh_exact(int32_t (&v)[64]) {
#pragma unroll
  for (int b = B0; b < B0 + NB; ++b)
#pragma unroll
    for (int r = 0; r < 64; ++r)
      if (!(r & (1 << b))) {
        const int32_t x = v[r], y = v[r | (1 << b)];
        v[r] = x + y;
        v[r | (1 << b)] = x - y;
      }
}
template <int B0, int NB>
__device__ __forceinline__ void walsh_fold(uint32_t (&v)[64]) {
#pragma unroll
  for (int b = B0; b < B0 + NB; ++b)
#pragma unroll
    for (int r = 0; r < 64; ++r)
      if (!(r & (1 << b))) {
        const uint32_t x = v[r], y = v[r | (1 << b)];
        const uint32_t s = x + y, d = x + kQ - y;
        v[r] = static_cast<uint16_t>(s + (s >> 16));  // (s & 0xffff) + (s >> 16), at most 65535
        v[r | (1 << b)] = static_cast<uint16_t>(d + (d >> 16));
      }
}

// BLK: n is a multiple of 1024, so rows 1024 r + t < n for r < n / 1024 (a
// wave-uniform test); otherwise the test is per row.
template <bool BLK>
__global__ __launch_bounds__(1024) void k_error_locator(DevTables T, uint32_t n, const uint8_t* present,
                                                        uint16_t* locators) {
  extern __shared__ uint16_t lw[];
  const size_t b = blockIdx.x;
#if NP_BOUNDS_CHECK
  {
    BoundsSet bs{};
    bs.lo[kBkPresent] = reinterpret_cast<uint64_t>(present);
    bs.hi[kBkPresent] = bs.lo[kBkPresent] + static_cast<uint64_t>(gridDim.x) * n;
    bs.lo[kBkLocators] = reinterpret_cast<uint64_t>(locators);
    bs.hi[kBkLocators] = bs.lo[kBkLocators] + 2ull * gridDim.x * n;
    bounds_arm(bs);
  }
#endif
  const uint8_t* pres = present + b * n;
  const uint32_t t = threadIdx.x, w = t >> 6, lane = t & 63u;
  const uint32_t nr = BLK ? __builtin_amdgcn_readfirstlane(n >> 10) : (n > t ? (n - t + 1023u) >> 10 : 0u);
  auto in_n = [&](int r) { return static_cast<uint32_t>(r) < nr; };  // row 1024 r + t < n
  // LDS slots i + 2 (i >> 6) of the three layouts as a per-thread base (opaque,
  // so no phase keeps another's 64 addresses live) plus a constant per r
  auto base = [](uint32_t v) {
    asm volatile("" : "+v"(v));
    return v;
  };
  auto sa = [&](int r) { return base(66u * t) + r; };                 // A: i = 64 t + r
  auto sb = [&](int r) { return base(4224u * w + lane) + 66u * r; };  // B: i = 4096 w + 64 r + lane
  auto sc = [&](int r) { return base(t + 2u * w) + 1056u * r; };      // C: i = 1024 r + t
  // ---- Walsh of the erasure flags (i < n), exact: levels 12-15 in C, then B, A
  int32_t e[64];
  uint32_t er[2] = {0u, 0u};  // bit r: row 1024 r + t erased (kept for the output)
#pragma unroll
  for (int r = 0; r < 64; ++r) {
    e[r] = in_n(r) ? (*NP_BCHK(pres + (t + 1024u * r), 1, kBkPresent) == 0) : 0;
    er[r >> 5] |= static_cast<uint32_t>(e[r]) << (r & 31);
    if ((r & 15) == 15) __builtin_amdgcn_sched_barrier(0);  // 16 loads in flight, not 64 addresses live
  }
  asm volatile("" : "+v"(er[0]), "+v"(er[1]));  // the mask now, not 64 flags kept to the end
  walsh_exact<2, 4>(e);  // C: i bits 12-15 are r bits 2-5
#pragma unroll
  for (int r = 0; r < 64; ++r) lw[sc(r)] = static_cast<uint16_t>(e[r]);  // |e| <= 16
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 64; ++r) e[r] = static_cast<int16_t>(lw[sb(r)]);
  walsh_exact<0, 6>(e);  // B: levels 6-11
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 64; ++r) lw[sb(r)] = static_cast<uint16_t>(e[r]);  // |e| <= 1024
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 64; ++r) e[r] = static_cast<int16_t>(lw[sa(r)]);
  walsh_exact<0, 6>(e);  // A: levels 0-5; |e| <= 65536
  // ---- times LOG_WALSH mod 65535 (inc_reconstruct.rs:103-106), in A
  uint32_t v[64];
  const uint4* lwt = reinterpret_cast<const uint4*>(T.log_walsh + 64u * t);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const uint4 m = lwt[q];
    const uint32_t mm[4] = {m.x, m.y, m.z, m.w};
#pragma unroll
    for (int h = 0; h < 8; ++h) {
      const int r = 8 * q + h;
      const int32_t c = e[r] % static_cast<int32_t>(kQ);
      const uint32_t res = static_cast<uint32_t>(c < 0 ? c + static_cast<int32_t>(kQ) : c);
      v[r] = (res * ((mm[h >> 1] >> (16 * (h & 1))) & 0xffffu)) % kQ;
    }
  }
  // ---- second Walsh, the reference's form and order: A (0-5), B (6-11), C (12-15)
  walsh_fold<0, 6>(v);
  __syncthreads();  // every wave has read the first transform's A values
#pragma unroll
  for (int r = 0; r < 64; ++r) lw[sa(r)] = static_cast<uint16_t>(v[r]);
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 64; ++r) v[r] = lw[sb(r)];
  walsh_fold<0, 6>(v);
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 64; ++r) lw[sb(r)] = static_cast<uint16_t>(v[r]);
  __syncthreads();
#pragma unroll
  for (int r = 0; r < 64; ++r) v[r] = lw[sc(r)];
  walsh_fold<2, 4>(v);
  // erased rows: ONEMASK - value (inc_reconstruct.rs:108-112)
#pragma unroll
  for (int r = 0; r < 64; ++r) {
    if (in_n(r))
      *NP_BCHK(locators + (b * n + t + 1024u * r), 2, kBkLocators) =
          static_cast<uint16_t>(((er[r >> 5] >> (r & 31)) & 1u) ? kQ - v[r] : v[r]);
    if ((r & 15) == 15) __builtin_amdgcn_sched_barrier(0);
  }
}

// mod.rs:171-180: a payload with fewer than k present rows is NeedMoreShards
// {have, min: k, all: n}; one 256-thread workgroup per payload.
__global__ __launch_bounds__(256) void k_payload_status(ReconstructArgs a) {
  const size_t b = blockIdx.x;
  const uint8_t* pres = a.present + b * a.n;
  int have = 0;
  for (uint32_t r = 0; r < a.n; r += 256) {
    const uint32_t v = r + threadIdx.x;
    have += __syncthreads_count(v < a.n && pres[v] != 0);
  }
  if (threadIdx.x == 0) {
    a.status[2 * b] = have >= static_cast<int>(a.k) ? 0u : kStatusNeedMoreShards;
    a.status[2 * b + 1] = static_cast<uint32_t>(have);
  }
}

// ------------------------------------------------------------ parity hooks ----
template <bool INVERSE>
__global__ __launch_bounds__(kThreads) void k_afft_cols(DevTables T, uint16_t* data, uint32_t size,
                                                        uint32_t index, size_t cols_total, uint32_t cols) {
  extern __shared__ uint16_t lds[];
  const size_t c0 = static_cast<size_t>(blockIdx.x) * cols;
  const uint32_t ncol = static_cast<uint32_t>(min(static_cast<size_t>(cols), cols_total - c0));
  uint16_t* g = data + c0 * size;
  for (uint32_t e = threadIdx.x; e < ncol * size; e += blockDim.x) lds[e] = g[e];
  __syncthreads();
  lds_transform<INVERSE>(T, lds, Segs{size, 0, 1, size, index, 0}, ncol);
  for (uint32_t e = threadIdx.x; e < ncol * size; e += blockDim.x) g[e] = lds[e];
}

__global__ __launch_bounds__(1024) void k_walsh(uint16_t* data, uint32_t size) {
  extern __shared__ uint16_t lds[];
  for (uint32_t e = threadIdx.x; e < size; e += blockDim.x) lds[e] = data[e];
  __syncthreads();
  lds_walsh(lds, size);
  for (uint32_t e = threadIdx.x; e < size; e += blockDim.x) data[e] = lds[e];
}

__global__ void k_mul(DevTables T, const uint16_t* a, const uint16_t* m, uint16_t* out, size_t count) {
  const size_t i = static_cast<size_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i < count) out[i] = gf_mul_log(T, a[i], m[i]);
}

__global__ __launch_bounds__(kThreads) void k_encode_low(DevTables T, const uint16_t* data, uint32_t k,
                                                         uint16_t* codeword, uint32_t n, size_t cols_total,
                                                         uint32_t cols) {
  extern __shared__ uint16_t lds[];
  const size_t c0 = static_cast<size_t>(blockIdx.x) * cols;
  const uint32_t ncol = static_cast<uint32_t>(min(static_cast<size_t>(cols), cols_total - c0));
  for (uint32_t e = threadIdx.x; e < ncol * k; e += blockDim.x) {
    const uint32_t c = e / k, i = e - c * k;
    lds[c * n + i] = data[(c0 + c) * k + i];
  }
  __syncthreads();
  lds_transform<true>(T, lds, Segs{n, 0, 1, k, 0, 0}, ncol);
  const uint32_t nseg = n / k - 1;
  for (uint32_t e = threadIdx.x; e < ncol * nseg * k; e += blockDim.x) {
    const uint32_t c = e / (nseg * k), r = e - c * nseg * k;
    lds[c * n + k + r] = lds[c * n + (r % k)];
  }
  __syncthreads();
  lds_transform<false>(T, lds, Segs{n, k, nseg, k, k, k}, ncol);
  for (uint32_t e = threadIdx.x; e < ncol * n; e += blockDim.x) {
    const uint32_t c = e / n, i = e - c * n;
    codeword[(c0 + c) * n + i] = i < k ? data[(c0 + c) * k + i] : lds[c * n + i];
  }
}

__global__ __launch_bounds__(kThreads) void k_decode_main(DevTables T, uint16_t* codeword, uint32_t upto,
                                                          const uint8_t* present, const uint16_t* loc,
                                                          uint32_t n, size_t cols_total, uint32_t cols) {
  extern __shared__ uint16_t lds[];
  const size_t c0 = static_cast<size_t>(blockIdx.x) * cols;
  const uint32_t ncol = static_cast<uint32_t>(min(static_cast<size_t>(cols), cols_total - c0));
  uint16_t* g = codeword + c0 * n;
  for (uint32_t e = threadIdx.x; e < ncol * n; e += blockDim.x) {
    const uint32_t i = e % n;
    lds[e] = present[i] ? gf_mul_log(T, g[e], loc[i]) : 0;
  }
  __syncthreads();
  lds_transform<true>(T, lds, Segs{n, 0, 1, n, 0, 0}, ncol);
  lds_formal_derivative(lds, n, n, n, ncol);
  lds_transform<false>(T, lds, Segs{n, 0, 1, n, 0, 0}, ncol);
  for (uint32_t e = threadIdx.x; e < ncol * n; e += blockDim.x) {
    const uint32_t i = e % n;
    uint16_t w = lds[e];
    if (i < upto) w = present[i] ? 0 : gf_mul_log(T, w, loc[i]);
    g[e] = w;
  }
}

inline uint32_t grid_x(size_t total, uint32_t per) { return static_cast<uint32_t>((total + per - 1) / per); }

}  // namespace

hipError_t configure_generic_kernels() {
  const int lim = 160 * 1024;
  hipError_t e = hipSuccess;
  auto set = [&](const void* f) {
    hipError_t r = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, lim);
    if (r != hipSuccess && e == hipSuccess) e = r;
  };
  set(reinterpret_cast<const void*>(&k_encode_generic));
  set(reinterpret_cast<const void*>(&k_reconstruct_generic));
  set(reinterpret_cast<const void*>(&k_error_locator<true>));
  set(reinterpret_cast<const void*>(&k_error_locator<false>));
  set(reinterpret_cast<const void*>(&k_afft_cols<true>));
  set(reinterpret_cast<const void*>(&k_afft_cols<false>));
  set(reinterpret_cast<const void*>(&k_walsh));
  set(reinterpret_cast<const void*>(&k_encode_low));
  set(reinterpret_cast<const void*>(&k_decode_main));
  return e;
}

hipError_t launch_encode_generic(const DevTables& T, const EncodeArgs& a, hipStream_t s) {
  const size_t nchunks = (a.payload_len + 2 * a.k - 1) / (2 * a.k);
  if (nchunks == 0 || a.batch == 0) return hipSuccess;
  const uint32_t cols = cols_for(a.n);
  dim3 grid(grid_x(nchunks, cols), static_cast<uint32_t>(a.batch));
  k_encode_generic<<<grid, kThreads, cols * a.n * sizeof(uint16_t), s>>>(T, a, static_cast<uint32_t>(nchunks),
                                                                          cols);
  return hipGetLastError();
}

hipError_t launch_reconstruct_generic(const DevTables& T, const ReconstructArgs& a, hipStream_t s) {
  const size_t nsyms = a.shard_len / 2;
  if (nsyms == 0 || a.batch == 0) return hipSuccess;
  const uint32_t cols = cols_for(a.n);
  dim3 grid(grid_x(nsyms, cols), static_cast<uint32_t>(a.batch));
  k_reconstruct_generic<<<grid, kThreads, cols * a.n * sizeof(uint16_t), s>>>(T, a, static_cast<uint32_t>(nsyms),
                                                                               cols);
  return hipGetLastError();
}

hipError_t launch_error_locator(const DevTables& T, uint32_t n, const uint8_t* present, size_t batch,
                                uint16_t* locators, hipStream_t s) {
  if (batch == 0) return hipSuccess;
  if (n % 1024u == 0)
    k_error_locator<true><<<static_cast<uint32_t>(batch), 1024, kLocLdsBytes, s>>>(T, n, present, locators);
  else
    k_error_locator<false><<<static_cast<uint32_t>(batch), 1024, kLocLdsBytes, s>>>(T, n, present, locators);
  return hipGetLastError();
}

hipError_t launch_payload_status(const ReconstructArgs& a, hipStream_t s) {
  if (a.batch == 0 || !a.status) return hipSuccess;
  if (a.batch > 0x7fffffffu) return hipErrorInvalidValue;
  k_payload_status<<<static_cast<uint32_t>(a.batch), 256, 0, s>>>(a);
  return hipGetLastError();
}

hipError_t launch_afft(const DevTables& T, uint16_t* data, uint32_t size, uint32_t index, size_t cols,
                       bool inverse, hipStream_t s) {
  if (cols == 0 || size < 2) return hipSuccess;
  const uint32_t per = cols_for(size);
  const size_t lds = per * size * sizeof(uint16_t);
  if (inverse)
    k_afft_cols<true><<<grid_x(cols, per), kThreads, lds, s>>>(T, data, size, index, cols, per);
  else
    k_afft_cols<false><<<grid_x(cols, per), kThreads, lds, s>>>(T, data, size, index, cols, per);
  return hipGetLastError();
}

hipError_t launch_walsh(uint16_t* data, uint32_t size, hipStream_t s) {
  if (size < 2) return hipSuccess;
  k_walsh<<<1, 1024, size * sizeof(uint16_t), s>>>(data, size);
  return hipGetLastError();
}

hipError_t launch_mul(const DevTables& T, const uint16_t* a, const uint16_t* m, uint16_t* out, size_t count,
                      hipStream_t s) {
  if (count == 0) return hipSuccess;
  k_mul<<<grid_x(count, 256), 256, 0, s>>>(T, a, m, out, count);
  return hipGetLastError();
}

hipError_t launch_encode_low(const DevTables& T, const uint16_t* data, uint32_t k, uint16_t* codeword, uint32_t n,
                             size_t cols, hipStream_t s) {
  if (cols == 0) return hipSuccess;
  const uint32_t per = cols_for(n);
  k_encode_low<<<grid_x(cols, per), kThreads, per * n * sizeof(uint16_t), s>>>(T, data, k, codeword, n, cols,
                                                                                per);
  return hipGetLastError();
}

hipError_t launch_decode_main(const DevTables& T, uint16_t* codeword, uint32_t upto, const uint8_t* present,
                              const uint16_t* locator, uint32_t n, size_t cols, hipStream_t s) {
  if (cols == 0) return hipSuccess;
  const uint32_t per = cols_for(n);
  k_decode_main<<<grid_x(cols, per), kThreads, per * n * sizeof(uint16_t), s>>>(T, codeword, upto, present,
                                                                                 locator, n, cols, per);
  return hipGetLastError();
}

hipError_t bounds_take_generic(uint32_t out[8]) { return bounds_take_tu(out); }

}  // namespace np
