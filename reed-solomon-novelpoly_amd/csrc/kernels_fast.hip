// Specialised gfx950 kernels for the hot shapes (n = 4k style codes, k <= 256).
//
// Work mapping ("lanes <-> chunks").  A workgroup of 256 threads owns a tile of
// 256 consecutive chunks (encode) or symbol columns (reconstruct).  All lanes
// of a wave execute the same transform level and group at the same time, so
// every GF(2^16) multiplier is wave-uniform.
//
// GF multiply.  Multiplication by a fixed c is GF(2)-linear.  The
// symbols of four codewords / positions are kept "byte-planar": register L holds
// the four low bytes, H the four high bytes.  c*y is the XOR of 12 byte-table
// lookups (input byte plane x 3-bit group -> output byte) and one v_perm_b32
// performs one lookup for all four bytes.  The tables of c (20 dwords, built
// on the host: field_tables.cpp) are staged per transform into LDS and read
// with wave-uniform (broadcast) ds_read_b128.
//
// Levels.  Within one lane, position-quads (4 consecutive positions of one
// codeword) serve every level with butterfly distance d >= 4.  The two lowest
// levels (d = 1, 2) pair symbols inside a quad; they are done in a "chunk-quad"
// pass through LDS in which each lane holds the same 4 positions of 4 codewords,
// again with uniform multipliers.  That pass also produces the coalesced shard
// rows (encode) and consumes the coalesced shard rows (reconstruct).
//
// Reference: additive FFT inc_afft.rs:139-214 (inverse) / :267-332 (forward);
// encode inc_encode.rs:15-48 + mod.rs:117-157; reconstruct inc_reconstruct.rs:1-85
// + mod.rs:162-239.  Skew factor of group t at level d and index I is
// skews[(2t+1)d + I - 1] (inc_afft.rs:457, 573).
#include "device_common.hpp"
#include "launchers.hpp"

namespace np {
namespace {

constexpr int kTile = 256;
constexpr int kPoolWords = 20;

__device__ __forceinline__ uint32_t vperm(uint32_t s0, uint32_t s1, uint32_t sel) {
  return __builtin_amdgcn_perm(s0, s1, sel);
}

// Byte-table selectors of four byte-planar symbols: bits 0-2, 3-5, 6-7 of
// every byte of the low plane (s[0..2]) and of the high plane (s[3..5]).
// Written as one asm block so that the compiler cannot hoist the selector
// extraction of a whole transform level ahead of its use (that hoisting cost
// 6 live VGPRs per pending butterfly and blew the register budget).
__device__ __forceinline__ void selectors(uint32_t yl, uint32_t yh, uint32_t (&s)[6]) {
  asm volatile(
      "v_and_b32 %0, 0x07070707, %6\n\t"
      "v_lshrrev_b32 %1, 3, %6\n\t"
      "v_lshrrev_b32 %2, 6, %6\n\t"
      "v_and_b32 %3, 0x07070707, %7\n\t"
      "v_lshrrev_b32 %4, 3, %7\n\t"
      "v_lshrrev_b32 %5, 6, %7\n\t"
      "v_and_b32 %1, 0x07070707, %1\n\t"
      "v_and_b32 %2, 0x03030303, %2\n\t"
      "v_and_b32 %4, 0x07070707, %4\n\t"
      "v_and_b32 %5, 0x03030303, %5"
      : "=&v"(s[0]), "=&v"(s[1]), "=&v"(s[2]), "=&v"(s[3]), "=&v"(s[4]), "=&v"(s[5])
      : "v"(yl), "v"(yh));
}

// x ^= c*y on four byte-planar symbols.  Pool layout: field_tables.cpp.
__device__ __forceinline__ void qmul(uint32_t& xl, uint32_t& xh, uint32_t yl, uint32_t yh, const uint32_t (&p)[20]) {
  uint32_t s[6];
  selectors(yl, yh, s);
  uint32_t lo = xor3(vperm(p[1], p[0], s[0]), vperm(p[3], p[2], s[1]), vperm(p[4], p[4], s[2]));
  lo = xor3(lo, vperm(p[6], p[5], s[3]), vperm(p[8], p[7], s[4]));
  xl = xor3(xl, lo, vperm(p[9], p[9], s[5]));
  uint32_t hi = xor3(vperm(p[11], p[10], s[0]), vperm(p[13], p[12], s[1]), vperm(p[14], p[14], s[2]));
  hi = xor3(hi, vperm(p[16], p[15], s[3]), vperm(p[18], p[17], s[4]));
  xh = xor3(xh, hi, vperm(p[19], p[19], s[5]));
}

typedef const __attribute__((address_space(4))) uint32_t* cpool_t;

// Multiplier tables of the additive element c, read through the scalar cache
// (wave-uniform address -> s_load).
__device__ __forceinline__ void pool_of(const DevTables& T, uint32_t c, uint32_t (&p)[20]) {
  const cpool_t q = (cpool_t)(T.perm_pools) + c * kPoolWords;
#pragma unroll
  for (int i = 0; i < 20; ++i) p[i] = q[i];
}

// Additive skew of group t at level b of a transform at index I (a multiple
// of the transform size): skews[(2t+1)2^b + I - 1] is the field element with
// Cantor coordinates 2(t + I/2^(b+1)) = 2t + (I >> b)  (tests/test_oracle.py::
// test_skews_are_cantor_points pins this on the reference tables).
__device__ __forceinline__ uint32_t skew_c(int b, int t, uint32_t index) {
  return 2u * static_cast<uint32_t>(t) + (index >> b);
}

// --------------------------------------------------------------- LDS tile ----
// Row r (a chunk / a column) holds the K symbols of that codeword segment as
// K/4 8-byte blocks (4 big-endian symbols each).  Block slots are XOR-swizzled
// so that both the per-row sweep (lane = row) and the chunk-quad sweep (lane =
// 4 consecutive rows) hit distinct ds_read_b64 bank pairs for K >= 128.
template <int K>
__device__ __forceinline__ uint32_t tile_off(uint32_t row, uint32_t blk) {
  const uint32_t f = (row >> 2) ^ ((row & 3u) << 3);
  return row * (2u * K) + (((blk ^ f) & (K / 4 - 1)) << 3);
}

// Swizzled row base: tile_off(row, blk) == tile_base(row) ^ (blk << 3).  The
// asm keeps the compiler from hoisting K/4 precomputed addresses (one VGPR
// each) across the transforms: each access recomputes its address with one XOR.
template <int K>
__device__ __forceinline__ uint32_t tile_base(uint32_t row) {
  uint32_t base = row * (2u * K) + ((((row >> 2) ^ ((row & 3u) << 3)) & (K / 4 - 1)) << 3);
  asm volatile("" : "+v"(base));
  return base;
}

// 8-byte block (4 BE symbols) <-> byte-planar quad.
__device__ __forceinline__ void blk_to_quad(uint2 d, uint32_t& l, uint32_t& h) {
  l = vperm(d.y, d.x, 0x07050301u);
  h = vperm(d.y, d.x, 0x06040200u);
}
__device__ __forceinline__ uint2 quad_to_blk(uint32_t l, uint32_t h) {
  return make_uint2(vperm(l, h, 0x05010400u), vperm(l, h, 0x07030602u));
}

// 4 rows' blocks (d[i] = row i) -> chunk-quads: CL[p]/CH[p] hold position p of rows 0..3.
__device__ __forceinline__ void blks_to_cq(const uint2 (&d)[4], uint32_t (&cl)[4], uint32_t (&ch)[4]) {
  const uint32_t lx01 = vperm(d[1].x, d[0].x, 0x07030501u), lx23 = vperm(d[3].x, d[2].x, 0x07030501u);
  const uint32_t ly01 = vperm(d[1].y, d[0].y, 0x07030501u), ly23 = vperm(d[3].y, d[2].y, 0x07030501u);
  const uint32_t hx01 = vperm(d[1].x, d[0].x, 0x06020400u), hx23 = vperm(d[3].x, d[2].x, 0x06020400u);
  const uint32_t hy01 = vperm(d[1].y, d[0].y, 0x06020400u), hy23 = vperm(d[3].y, d[2].y, 0x06020400u);
  cl[0] = vperm(lx23, lx01, 0x05040100u);
  cl[1] = vperm(lx23, lx01, 0x07060302u);
  cl[2] = vperm(ly23, ly01, 0x05040100u);
  cl[3] = vperm(ly23, ly01, 0x07060302u);
  ch[0] = vperm(hx23, hx01, 0x05040100u);
  ch[1] = vperm(hx23, hx01, 0x07060302u);
  ch[2] = vperm(hy23, hy01, 0x05040100u);
  ch[3] = vperm(hy23, hy01, 0x07060302u);
}

// Shard-row bytes of position p for the lane's 4 rows: (h,l) pairs of rows 0..3.
__device__ __forceinline__ uint2 cq_row(uint32_t l, uint32_t h) {
  return make_uint2(vperm(l, h, 0x05010400u), vperm(l, h, 0x07030602u));
}

__device__ __forceinline__ void cq_to_blks(const uint32_t (&cl)[4], const uint32_t (&ch)[4], uint2 (&d)[4]) {
  const uint2 r0 = cq_row(cl[0], ch[0]), r1 = cq_row(cl[1], ch[1]);
  const uint2 r2 = cq_row(cl[2], ch[2]), r3 = cq_row(cl[3], ch[3]);
  d[0] = make_uint2(vperm(r1.x, r0.x, 0x05040100u), vperm(r3.x, r2.x, 0x05040100u));
  d[1] = make_uint2(vperm(r1.x, r0.x, 0x07060302u), vperm(r3.x, r2.x, 0x07060302u));
  d[2] = make_uint2(vperm(r1.y, r0.y, 0x05040100u), vperm(r3.y, r2.y, 0x05040100u));
  d[3] = make_uint2(vperm(r1.y, r0.y, 0x07060302u), vperm(r3.y, r2.y, 0x07060302u));
}

// Store 4 symbols (rows 4l..4l+3 of the tile) into shard row `row`.
__device__ __forceinline__ void store_row4(uint8_t* rowp, uint2 v, uint32_t col0, uint32_t ncols, bool aligned8) {
  if (col0 + 4 <= ncols && aligned8) {
    *reinterpret_cast<uint2*>(rowp + 2 * col0) = v;
    return;
  }
  const uint32_t w[2] = {v.x, v.y};
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (col0 + i < ncols) {
      uint16_t s = static_cast<uint16_t>(w[i >> 1] >> (16 * (i & 1)));
      *reinterpret_cast<uint16_t*>(rowp + 2 * (col0 + i)) = s;
    }
}

// ------------------------------------------------------ register transforms ----
template <int K, bool INDEX0>
__device__ __forceinline__ void ifft_reg(const DevTables& T, uint32_t index, uint32_t (&L)[K / 4], uint32_t (&H)[K / 4]) {
#pragma unroll
  for (int b = 2; (1 << b) < K; ++b) {
    const int D = 1 << (b - 2), G = K >> (b + 1);
#pragma unroll
    for (int t = 0; t < G; ++t) {
      if (INDEX0 && t == 0) {
#pragma unroll
        for (int u = 0; u < D; ++u) {
          L[u + D] ^= L[u];
          H[u + D] ^= H[u];
        }
        continue;
      }
      uint32_t p[20];
      pool_of(T, skew_c(b, t, index), p);
#pragma unroll
      for (int u = 0; u < D; ++u) {
        const int qx = t * 2 * D + u, qy = qx + D;
        L[qy] ^= L[qx];
        H[qy] ^= H[qx];
        qmul(L[qx], H[qx], L[qy], H[qy], p);
      }
    }
  }
}

template <int K>
constexpr int log2k() {
  int r = 0;
  while ((1 << r) < K) ++r;
  return r;
}

template <int K, bool INDEX0>
__device__ __forceinline__ void fft_reg(const DevTables& T, uint32_t index, uint32_t (&L)[K / 4], uint32_t (&H)[K / 4]) {
#pragma unroll
  for (int lv = log2k<K>() - 1; lv >= 2; --lv) {  // top level first
    const int D = 1 << (lv - 2), G = K >> (lv + 1);
#pragma unroll
    for (int t = 0; t < G; ++t) {
      if (INDEX0 && t == 0) {
#pragma unroll
        for (int u = 0; u < D; ++u) {
          L[u + D] ^= L[u];
          H[u + D] ^= H[u];
        }
        continue;
      }
      uint32_t p[20];
      pool_of(T, skew_c(lv, t, index), p);
#pragma unroll
      for (int u = 0; u < D; ++u) {
        const int qx = t * 2 * D + u, qy = qx + D;
        qmul(L[qx], H[qx], L[qy], H[qy], p);
        L[qy] ^= L[qx];
        H[qy] ^= H[qx];
      }
    }
  }
}

// Chunk-quad levels 0 and 1 for block m (positions 4m..4m+3) of 4 rows.
template <int K, bool INVERSE, bool INDEX0>
__device__ __forceinline__ void cq_levels(const DevTables& T, uint32_t index, uint32_t m, uint32_t (&cl)[4],
                                          uint32_t (&ch)[4]) {
  const bool skip = INDEX0 && m == 0;  // group t == 0 at index 0 has the zero skew
  uint32_t p[20];
  if (INVERSE) {
    cl[1] ^= cl[0]; ch[1] ^= ch[0];
    cl[3] ^= cl[2]; ch[3] ^= ch[2];
    if (!skip) {
      pool_of(T, skew_c(0, 2 * m, index), p);
      qmul(cl[0], ch[0], cl[1], ch[1], p);
    }
    pool_of(T, skew_c(0, 2 * m + 1, index), p);
    qmul(cl[2], ch[2], cl[3], ch[3], p);
    cl[2] ^= cl[0]; ch[2] ^= ch[0];
    cl[3] ^= cl[1]; ch[3] ^= ch[1];
    if (!skip) {
      pool_of(T, skew_c(1, m, index), p);
      qmul(cl[0], ch[0], cl[2], ch[2], p);
      qmul(cl[1], ch[1], cl[3], ch[3], p);
    }
  } else {
    if (!skip) {
      pool_of(T, skew_c(1, m, index), p);
      qmul(cl[0], ch[0], cl[2], ch[2], p);
      qmul(cl[1], ch[1], cl[3], ch[3], p);
    }
    cl[2] ^= cl[0]; ch[2] ^= ch[0];
    cl[3] ^= cl[1]; ch[3] ^= ch[1];
    if (!skip) {
      pool_of(T, skew_c(0, 2 * m, index), p);
      qmul(cl[0], ch[0], cl[1], ch[1], p);
    }
    cl[1] ^= cl[0]; ch[1] ^= ch[0];
    pool_of(T, skew_c(0, 2 * m + 1, index), p);
    qmul(cl[2], ch[2], cl[3], ch[3], p);
    cl[3] ^= cl[2]; ch[3] ^= ch[2];
  }
}

template <int K>
__device__ __forceinline__ void read_row(const uint8_t* tile, uint32_t row, uint32_t (&L)[K / 4], uint32_t (&H)[K / 4]) {
  const uint32_t base = tile_base<K>(row);
#pragma unroll
  for (int m = 0; m < K / 4; ++m)
    blk_to_quad(*reinterpret_cast<const uint2*>(tile + (base ^ (static_cast<uint32_t>(m) << 3))), L[m], H[m]);
}

template <int K>
__device__ __forceinline__ void write_row(uint8_t* tile, uint32_t row, const uint32_t (&L)[K / 4],
                                          const uint32_t (&H)[K / 4]) {
  const uint32_t base = tile_base<K>(row);
#pragma unroll
  for (int m = 0; m < K / 4; ++m)
    *reinterpret_cast<uint2*>(tile + (base ^ (static_cast<uint32_t>(m) << 3))) = quad_to_blk(L[m], H[m]);
}

// ----------------------------------------------------------------- encode ----
// One workgroup: 256 chunks of one payload.  mod.rs:144-154 / inc_encode.rs:15-48.
template <int K>
__global__ __launch_bounds__(256, 1) void k_encode_fast(DevTables T, EncodeArgs a, uint32_t nchunks,
                                                        uint32_t tiles) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* tile = smem;
  const uint32_t pb = blockIdx.x / tiles, tl = blockIdx.x - pb * tiles;
  const uint32_t ch0 = tl * kTile;
  const uint32_t ncols = min(static_cast<uint32_t>(kTile), nchunks - ch0);
  const uint8_t* pay = a.payloads + static_cast<size_t>(pb) * a.payload_stride;
  uint8_t* out = a.shards + static_cast<size_t>(pb) * a.batch_stride;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const bool al8 = (a.shard_len & 7u) == 0;

  // ---- load the tile: 256 chunks x 2K bytes, contiguous in the payload
  {
    const size_t base = static_cast<size_t>(ch0) * 2 * K;
    const size_t len = a.payload_len;
#pragma unroll 4
    for (uint32_t o = tid * 16u; o < kTile * 2u * K; o += 256u * 16u) {
      uint4 v = make_uint4(0, 0, 0, 0);
      const size_t g = base + o;
      if (g + 16 <= len) {
        v = *reinterpret_cast<const uint4*>(pay + g);
      } else if (g < len) {
        uint8_t tmp[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) tmp[i] = (g + i < len) ? pay[g + i] : 0;
        v = *reinterpret_cast<const uint4*>(tmp);
      }
      const uint32_t row = o / (2u * K), blk = (o % (2u * K)) / 8u;
      *reinterpret_cast<uint2*>(tile + tile_off<K>(row, blk)) = make_uint2(v.x, v.y);
      *reinterpret_cast<uint2*>(tile + tile_off<K>(row, blk + 1)) = make_uint2(v.z, v.w);
    }
  }
  __syncthreads();
  // ---- chunk-quad pass: systematic rows + inverse levels 0,1
  for (uint32_t m = wave; m < K / 4; m += 4) {
    uint2 d[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) d[i] = *reinterpret_cast<const uint2*>(tile + tile_off<K>(4 * lane + i, m));
    uint32_t cl[4], ch[4];
    blks_to_cq(d, cl, ch);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const uint32_t row = 4 * m + p;
      if (row < a.wanted_n) store_row4(out + static_cast<size_t>(row) * a.shard_len + 2 * static_cast<size_t>(ch0), cq_row(cl[p], ch[p]), 4 * lane,
                                       ncols, al8);
    }
    cq_levels<K, true, true>(T, 0, m, cl, ch);
    cq_to_blks(cl, ch, d);
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<uint2*>(tile + tile_off<K>(4 * lane + i, m)) = d[i];
  }
  __syncthreads();
  uint32_t WL[K / 4], WH[K / 4], ML[K / 4], MH[K / 4];
  read_row<K>(tile, tid, WL, WH);
  ifft_reg<K, true>(T, 0, WL, WH);
#pragma unroll
  for (int q = 0; q < K / 4; ++q) {
    ML[q] = WL[q];
    MH[q] = WH[q];
    asm volatile("" : "+v"(ML[q]), "+v"(MH[q]));  // materialise M here (no sinking into the loop)
  }
  const uint32_t nshift = a.n / K;
  for (uint32_t sh = 1; sh < nshift; ++sh) {
    if (sh * K >= a.wanted_n) break;
    __syncthreads();  // the previous chunk-quad pass is done with the tile
#pragma unroll
    for (int q = 0; q < K / 4; ++q) {
      WL[q] = ML[q];
      WH[q] = MH[q];
    }
    fft_reg<K, false>(T, sh * K, WL, WH);
    write_row<K>(tile, tid, WL, WH);
    __syncthreads();
    for (uint32_t m = wave; m < K / 4; m += 4) {
      uint2 d[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) d[i] = *reinterpret_cast<const uint2*>(tile + tile_off<K>(4 * lane + i, m));
      uint32_t cl[4], ch[4];
      blks_to_cq(d, cl, ch);
      cq_levels<K, false, false>(T, sh * K, m, cl, ch);
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const uint32_t row = sh * K + 4 * m + p;
        if (row < a.wanted_n)
          store_row4(out + static_cast<size_t>(row) * a.shard_len + 2 * static_cast<size_t>(ch0), cq_row(cl[p], ch[p]), 4 * lane, ncols, al8);
      }
    }
  }
}

template <int K>
size_t encode_lds_bytes() {
  return static_cast<size_t>(kTile) * 2 * K;
}

template <int K>
hipError_t launch_encode_k(const DevTables& T, const EncodeArgs& a, hipStream_t s) {
  const size_t nchunks = (a.payload_len + 2 * a.k - 1) / (2 * a.k);
  if (nchunks == 0 || a.batch == 0) return hipSuccess;
  const uint32_t tiles = static_cast<uint32_t>((nchunks + kTile - 1) / kTile);
  const size_t blocks = a.batch * tiles;
  if (blocks > 0x7fffffffu) return hipErrorInvalidValue;
  k_encode_fast<K><<<static_cast<uint32_t>(blocks), 256, encode_lds_bytes<K>(), s>>>(
      T, a, static_cast<uint32_t>(nchunks), tiles);
  return hipGetLastError();
}

}  // namespace

bool fast_encode_supported(uint32_t n, uint32_t k) {
  return (k == 64 || k == 128 || k == 256) && n >= 2 * k && n <= 65536;
}

bool fast_reconstruct_supported(uint32_t, uint32_t) { return false; }

hipError_t launch_encode_fast(const DevTables& T, const EncodeArgs& a, hipStream_t s) {
  switch (a.k) {
    case 64: return launch_encode_k<64>(T, a, s);
    case 128: return launch_encode_k<128>(T, a, s);
    case 256: return launch_encode_k<256>(T, a, s);
    default: return hipErrorNotSupported;
  }
}

hipError_t launch_reconstruct_fast(const DevTables&, const ReconstructArgs&, hipStream_t) {
  return hipErrorNotSupported;
}

hipError_t configure_fast_kernels() {
  hipError_t e = hipSuccess;
  auto set = [&](const void* f, size_t bytes) {
    hipError_t r = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(bytes));
    if (r != hipSuccess && e == hipSuccess) e = r;
  };
  set(reinterpret_cast<const void*>(&k_encode_fast<64>), encode_lds_bytes<64>());
  set(reinterpret_cast<const void*>(&k_encode_fast<128>), encode_lds_bytes<128>());
  set(reinterpret_cast<const void*>(&k_encode_fast<256>), encode_lds_bytes<256>());
  return e;
}

}  // namespace np
