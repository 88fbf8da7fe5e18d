// Shared building blocks of the specialised gfx950 kernels (kernels_fast.hip,
// kernels_big.hip): tile geometry and LDS swizzle, the v_perm GF(2^16)
// multiply, multiplier-table fetch and staging, the column-quad and high
// register layouts with their transform levels, and the folded erasure
// locator.  See kernels_fast.hip for the design.
#pragma once
#include <type_traits>

#include "device_common.hpp"
#include "launchers.hpp"

namespace np {
namespace {

constexpr int kTile = 256;  // columns per workgroup

// Experiment builds only (tools/exp_variants.sh; the product is built with 0):
// bit 0 skips the transform levels, bit 1 the shard stores, bit 2 the payload
// loads, so the phases of a kernel can be timed apart.
#ifndef NP_EXP
#define NP_EXP 0
#endif
constexpr int kExp = NP_EXP;

// Experiment builds with NP_EXP bit 6: thread 0 of a workgroup writes
// s_memtime stamps at phase boundaries to `dbg` (tools/phase_stamps.py).
// With bit 7 as well, lane 0 of every wave writes its own 32 stamps
// (dbg[32 * wave + slot], tools/wave_stamps.py).
__device__ __forceinline__ void stamp(uint64_t* dbg, int slot) {
  if constexpr ((kExp & 64) != 0 && (kExp & 128) != 0) {
    if ((threadIdx.x & 63u) == 0) dbg[32u * (threadIdx.x >> 6) + slot] = __builtin_amdgcn_s_memtime();
  } else if constexpr (kExp & 64) {
    if (threadIdx.x == 0) dbg[slot] = __builtin_amdgcn_s_memtime();
  }
}
constexpr int kPoolWords = 20;

// Prefix-locator record of one payload (k_prefix_locator, k_locator_records):
// header (byte 0 = prefix segments), one u16 row multiplier per row, then the
// v_perm tables (kPoolWords dwords, field_tables.cpp) of every row's
// multiplier, contiguous: the decode reads one 80-byte record per row and
// tile from a 40-80 KiB block instead of from the 5 MiB pool table, where the
// tiles of a payload would fetch the same scattered records again from HBM.
constexpr uint32_t kPrefixHeader = 16;
__host__ __device__ constexpr size_t prefix_pools_offset(uint32_t n) {
  return (kPrefixHeader + 2u * static_cast<size_t>(n) + 15u) & ~static_cast<size_t>(15);
}
__host__ __device__ constexpr size_t prefix_stride_c(uint32_t n, uint32_t k) {
  (void)k;
  return prefix_pools_offset(n) + 4u * kPoolWords * static_cast<size_t>(n);
}

__host__ __device__ constexpr int ilog2(int v) {
  int r = 0;
  while ((1 << r) < v) ++r;
  return r;
}

template <int K>
struct Geo {
  static constexpr int kLog = ilog2(K);
  static constexpr int Q = K / 4;              // 8-byte blocks (position quads) per column
  static constexpr int R = K / 64;             // lanes per column in the high layout
  static constexpr int kLogR = ilog2(R);
  static constexpr int kThreads = 4 * K;       // = kTile * Q / 16
  static constexpr int P = Q >= 32 ? 1 : 32 / Q;  // columns per 256-byte swizzle row
  static constexpr int W = Q >= 32 ? Q : 32;      // blocks per swizzle row
  static constexpr int kTileBytes = kTile * 2 * K;
  static constexpr int kVPWords = 8 * K;  // one staged transform: K - 1 slots of 8 dwords (rounded)
};

// Workgroup -> (batch entry, tile).  Workgroups are handed to the 8 XCDs
// round-robin (b % 8), so when the batch is a multiple of 8 all tiles of one
// batch entry go to the same XCD and share its L2 (per-entry data: multiplier
// tables of the locator values, the EXP gathers, present flags).  Any mapping
// is correct; this one only buys locality.
struct TileRef {
  uint32_t pb, tl;
};
__device__ __forceinline__ TileRef tile_of(uint32_t b, uint32_t tiles, bool xcd_major) {
  if (xcd_major) {
    const uint32_t slot = b >> 3;
    return TileRef{(slot / tiles) * 8 + (b & 7u), slot % tiles};
  }
  return TileRef{b / tiles, b % tiles};
}

// ------------------------------------------------------------ LDS tile ----
// Block (column c, quad m) lives at 8 * (cs * W + ((ci * Q + m) ^ f(cs))) with
// cs = c / P, ci = c % P and f a linear map of cs found by
// tools/lds_swizzle_search.py: conflict-free ds_read_b64 / ds_write_b64 for the
// cq sweep, the high-layout sweep and the row-major tile sweep.
__host__ __device__ constexpr uint32_t swz_row(int K, int b) {
  const uint8_t m64[8] = {29, 18, 1, 26, 6, 11, 18, 0};
  const uint8_t m128[8] = {21, 7, 24, 4, 14, 5, 17, 23};
  const uint8_t m256[8] = {13, 7, 27, 26, 7, 18, 17, 15};
  return K == 64 ? m64[b] : K == 128 ? m128[b] : m256[b];
}

template <int K>
__host__ __device__ constexpr uint32_t swz(uint32_t cs) {
  uint32_t v = 0;
  for (int b = 0; b < 8; ++b)
    if ((cs >> b) & 1u) v ^= swz_row(K, b);
  return v;
}

// Byte offset of block 0 of column c; block m is at col_base(c) ^ 8m.  The map
// is linear in the bits of c, so col_base(c1 | c2) == col_base(c1) ^ col_base(c2)
// for disjoint bit sets.
// EVEN: the swizzle with bit 0 cleared, so blocks 2i and 2i + 1 of a column
// stay a contiguous, 16-byte aligned pair (the multi-tile encode's payload
// tile with 16-byte LDS-DMA pieces, kernels_fast.hip NP_ENC_DMA_X4: its cq
// reads then conflict 2-way).
template <int K, bool EVEN = false>
__host__ __device__ constexpr uint32_t col_base_c(uint32_t c) {
  using G = Geo<K>;
  const uint32_t cs = c / G::P, ci = c % G::P;
  return 8u * cs * G::W + 8u * ((ci * G::Q) ^ (swz<K>(cs) & (EVEN ? ~1u : ~0u)));
}

// Runtime version; the asm keeps the compiler from materialising every block
// address of a sweep in its own VGPR.
template <int K, bool EVEN = false>
__device__ __forceinline__ uint32_t col_base(uint32_t c) {
  uint32_t b = col_base_c<K, EVEN>(c);
  asm volatile("" : "+v"(b));
  return b;
}

// ------------------------------------------------------------ GF multiply ----
__device__ __forceinline__ uint32_t vperm(uint32_t s0, uint32_t s1, uint32_t sel) {
  return __builtin_amdgcn_perm(s0, s1, sel);
}

// Byte-table selectors of four byte-planar symbols: bits 0-2, 3-5, 6-7 of
// every byte of the low plane (s[0..2]) and of the high plane (s[3..5]).  The
// two planes shift as one 64-bit value: the bits the high plane shifts into
// the low plane's top byte land above each byte's mask.  One asm block, so the
// extraction of a whole level is not hoisted ahead of use.
__device__ __forceinline__ void selectors(uint32_t yl, uint32_t yh, uint32_t (&s)[6]) {
  const uint64_t y = (static_cast<uint64_t>(yh) << 32) | yl;
  uint64_t t3, t6;
  asm volatile("v_lshrrev_b64 %0, 3, %2\n\tv_lshrrev_b64 %1, 6, %2" : "=&v"(t3), "=&v"(t6) : "v"(y));
  asm volatile(
      "v_and_b32 %0, 0x07070707, %6\n\t"
      "v_and_b32 %3, 0x07070707, %7\n\t"
      "v_and_b32 %1, 0x07070707, %8\n\t"
      "v_and_b32 %4, 0x07070707, %9\n\t"
      "v_and_b32 %2, 0x03030303, %10\n\t"
      "v_and_b32 %5, 0x03030303, %11"
      : "=&v"(s[0]), "=&v"(s[1]), "=&v"(s[2]), "=&v"(s[3]), "=&v"(s[4]), "=&v"(s[5])
      : "v"(yl), "v"(yh), "v"(static_cast<uint32_t>(t3)), "v"(static_cast<uint32_t>(t3 >> 32)),
        "v"(static_cast<uint32_t>(t6)), "v"(static_cast<uint32_t>(t6 >> 32)));
}

// One output byte plane of c*y: acc ^= XOR of the 6 table lookups (tables
// p[o..o+9] of pool layout field_tables.cpp).  v_perm reads at most one SGPR, so
// the S1 half of each 8-entry table comes in a VGPR copy (va..vd).  Written as
// asm so that the compiler keeps every product next to its pool fetch instead
// of sinking the lookups (and the 20 live SGPRs of their pool) far below it.
__device__ __forceinline__ void qplane(uint32_t& acc, const uint32_t (&s)[6], uint32_t va, uint32_t vb, uint32_t vc,
                                       uint32_t vd, uint32_t sa, uint32_t sb, uint32_t sc, uint32_t sd, uint32_t se,
                                       uint32_t sf) {
  uint32_t t0, t1, t2;
  asm volatile(
      "v_perm_b32 %[t0], %[sa], %[va], %[s0]\n\t"
      "v_perm_b32 %[t1], %[sb], %[vb], %[s1]\n\t"
      "v_perm_b32 %[t2], %[sc], %[sc], %[s2]\n\t"
      "v_bitop3_b32 %[t0], %[t0], %[t1], %[t2] bitop3:0x96\n\t"
      "v_perm_b32 %[t1], %[sd], %[vc], %[s3]\n\t"
      "v_perm_b32 %[t2], %[se], %[vd], %[s4]\n\t"
      "v_bitop3_b32 %[t0], %[t0], %[t1], %[t2] bitop3:0x96\n\t"
      "v_perm_b32 %[t1], %[sf], %[sf], %[s5]\n\t"
      "v_bitop3_b32 %[acc], %[acc], %[t0], %[t1] bitop3:0x96"
      : [acc] "+v"(acc), [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2)
      : [s0] "v"(s[0]), [s1] "v"(s[1]), [s2] "v"(s[2]), [s3] "v"(s[3]), [s4] "v"(s[4]), [s5] "v"(s[5]),
        [va] "v"(va), [vb] "v"(vb), [vc] "v"(vc), [vd] "v"(vd), [sa] "s"(sa), [sb] "s"(sb), [sc] "s"(sc),
        [sd] "s"(sd), [se] "s"(se), [sf] "s"(sf));
}

// One output byte plane of c*y, written (not accumulated): the last XOR3 takes
// the third partial sum instead of an accumulator, so no zeroing move.
__device__ __forceinline__ void qplane_set(uint32_t& out, const uint32_t (&s)[6], uint32_t va, uint32_t vb, uint32_t vc,
                                           uint32_t vd, uint32_t sa, uint32_t sb, uint32_t sc, uint32_t sd, uint32_t se,
                                           uint32_t sf) {
  uint32_t t0, t1, t2, t3;
  asm volatile(
      "v_perm_b32 %[t0], %[sa], %[va], %[s0]\n\t"
      "v_perm_b32 %[t1], %[sb], %[vb], %[s1]\n\t"
      "v_perm_b32 %[t2], %[sc], %[sc], %[s2]\n\t"
      "v_bitop3_b32 %[t0], %[t0], %[t1], %[t2] bitop3:0x96\n\t"
      "v_perm_b32 %[t1], %[sd], %[vc], %[s3]\n\t"
      "v_perm_b32 %[t2], %[se], %[vd], %[s4]\n\t"
      "v_perm_b32 %[t3], %[sf], %[sf], %[s5]\n\t"
      "v_bitop3_b32 %[out], %[t0], %[t1], %[t2] bitop3:0x96\n\t"
      "v_xor_b32 %[out], %[out], %[t3]"
      : [out] "=&v"(out), [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2), [t3] "=&v"(t3)
      : [s0] "v"(s[0]), [s1] "v"(s[1]), [s2] "v"(s[2]), [s3] "v"(s[3]), [s4] "v"(s[4]), [s5] "v"(s[5]),
        [va] "v"(va), [vb] "v"(vb), [vc] "v"(vc), [vd] "v"(vd), [sa] "s"(sa), [sb] "s"(sb), [sc] "s"(sc),
        [sd] "s"(sd), [se] "s"(se), [sf] "s"(sf));
}

// A multiplier ready for use: its 20 table dwords in SGPRs plus VGPR copies of
// the 8 dwords that v_perm must read from a VGPR.  The copies are made by an
// asm block where the butterfly group starts, so that they are neither hoisted
// next to the s_load of a prefetched table nor repeated per butterfly.
struct Mult {
  uint32_t s[12];  // SGPR operands (pool dwords 8..19)
  uint32_t v[8];   // VGPR operands (pool dwords 0..7)
};

// From a whole pool in SGPRs: VGPR copies made by an asm block where the
// butterfly group starts (neither hoisted next to the s_load nor repeated per
// butterfly).
__device__ __forceinline__ Mult make_mult(const uint32_t (&p)[20]) {
  Mult m;
#pragma unroll
  for (int i = 0; i < 12; ++i) m.s[i] = p[8 + i];
  // 64-bit moves: the pool's SGPRs come in aligned pairs from s_load_dwordx8
  uint64_t v01, v23, v45, v67;
  asm volatile(
      "v_mov_b64 %0, %4\n\tv_mov_b64 %1, %5\n\tv_mov_b64 %2, %6\n\tv_mov_b64 %3, %7"
      : "=v"(v01), "=v"(v23), "=v"(v45), "=v"(v67)
      : "s"((static_cast<uint64_t>(p[1]) << 32) | p[0]), "s"((static_cast<uint64_t>(p[3]) << 32) | p[2]),
        "s"((static_cast<uint64_t>(p[5]) << 32) | p[4]), "s"((static_cast<uint64_t>(p[7]) << 32) | p[6]));
  m.v[0] = static_cast<uint32_t>(v01), m.v[1] = static_cast<uint32_t>(v01 >> 32);
  m.v[2] = static_cast<uint32_t>(v23), m.v[3] = static_cast<uint32_t>(v23 >> 32);
  m.v[4] = static_cast<uint32_t>(v45), m.v[5] = static_cast<uint32_t>(v45 >> 32);
  m.v[6] = static_cast<uint32_t>(v67), m.v[7] = static_cast<uint32_t>(v67 >> 32);
  return m;
}

// From the SGPR half plus the VGPR half staged in LDS (two broadcast
// ds_read_b128, no VALU work).  SUB: a subfield pool (field_tables.hpp kSubV /
// kSubS), whose 6 SGPR and 4 VGPR dwords are all the multiply reads.
template <bool SUB = false>
__device__ __forceinline__ Mult staged_mult(const uint32_t (&sp)[12], const uint32_t* vp) {
  Mult m;
  constexpr int ns = SUB ? 6 : 12;
#pragma unroll
  for (int i = 0; i < ns; ++i) m.s[i] = sp[i];
  const uint4 a = *reinterpret_cast<const uint4*>(vp);
  m.v[0] = a.x, m.v[1] = a.y, m.v[2] = a.z, m.v[3] = a.w;
  if constexpr (!SUB) {
    const uint4 b = *reinterpret_cast<const uint4*>(vp + 4);
    m.v[4] = b.x, m.v[5] = b.y, m.v[6] = b.z, m.v[7] = b.w;
  }
  return m;
}

// x ^= c*y on four byte-planar symbols (pool layout: field_tables.cpp).
__device__ __forceinline__ void qmul(uint32_t& xl, uint32_t& xh, uint32_t yl, uint32_t yh, const Mult& m) {
  uint32_t s[6];
  selectors(yl, yh, s);
  qplane(xl, s, m.v[0], m.v[1], m.v[2], m.v[3], m.s[0], m.s[1], m.s[2], m.s[3], m.s[4], m.s[5]);
  qplane(xh, s, m.v[4], m.v[5], m.v[6], m.v[7], m.s[6], m.s[7], m.s[8], m.s[9], m.s[10], m.s[11]);
}

// (ol, oh) = c*y.
__device__ __forceinline__ void qmul_set(uint32_t& ol, uint32_t& oh, uint32_t yl, uint32_t yh, const Mult& m) {
  uint32_t s[6];
  selectors(yl, yh, s);
  qplane_set(ol, s, m.v[0], m.v[1], m.v[2], m.v[3], m.s[0], m.s[1], m.s[2], m.s[3], m.s[4], m.s[5]);
  qplane_set(oh, s, m.v[4], m.v[5], m.v[6], m.v[7], m.s[6], m.s[7], m.s[8], m.s[9], m.s[10], m.s[11]);
}

// ---- subfield multiply (tower coordinates, field_tables.hpp) ----
// For c in GF(2^8) both byte planes of a symbol in tower coordinates are
// GF(2^8) elements that c multiplies separately: per plane 3 lookups
// (bits 0-2, 3-5, 6-7) instead of the 6 of a full 16 x 16 map.  Pool layout
// kSubV / kSubS: VGPR dwords v[0..1] (plane a), v[2..3] (plane b); SGPR dwords
// s[0..2] (a), s[3..5] (b) of Mult.
__device__ __forceinline__ void qplane_sub(uint32_t& acc, uint32_t s0, uint32_t s1, uint32_t s2, uint32_t va,
                                           uint32_t vb, uint32_t sa, uint32_t sb, uint32_t sc) {
  uint32_t t0, t1, t2;
  asm volatile(
      "v_perm_b32 %[t0], %[sa], %[va], %[s0]\n\t"
      "v_perm_b32 %[t1], %[sb], %[vb], %[s1]\n\t"
      "v_perm_b32 %[t2], %[sc], %[sc], %[s2]\n\t"
      "v_bitop3_b32 %[acc], %[acc], %[t0], %[t1] bitop3:0x96\n\t"
      "v_xor_b32 %[acc], %[acc], %[t2]"
      : [acc] "+v"(acc), [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2)
      : [s0] "v"(s0), [s1] "v"(s1), [s2] "v"(s2), [va] "v"(va), [vb] "v"(vb), [sa] "s"(sa), [sb] "s"(sb),
        [sc] "s"(sc));
}

__device__ __forceinline__ void qplane_sub_set(uint32_t& out, uint32_t s0, uint32_t s1, uint32_t s2, uint32_t va,
                                               uint32_t vb, uint32_t sa, uint32_t sb, uint32_t sc) {
  uint32_t t0, t1, t2;
  asm volatile(
      "v_perm_b32 %[t0], %[sa], %[va], %[s0]\n\t"
      "v_perm_b32 %[t1], %[sb], %[vb], %[s1]\n\t"
      "v_perm_b32 %[t2], %[sc], %[sc], %[s2]\n\t"
      "v_bitop3_b32 %[out], %[t0], %[t1], %[t2] bitop3:0x96"
      : [out] "=&v"(out), [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2)
      : [s0] "v"(s0), [s1] "v"(s1), [s2] "v"(s2), [va] "v"(va), [vb] "v"(vb), [sa] "s"(sa), [sb] "s"(sb),
        [sc] "s"(sc));
}

// x ^= c*y, c in GF(2^8), tower coordinates.
__device__ __forceinline__ void qmul_sub(uint32_t& xl, uint32_t& xh, uint32_t yl, uint32_t yh, const Mult& m) {
  uint32_t s[6];
  selectors(yl, yh, s);
  qplane_sub(xl, s[0], s[1], s[2], m.v[0], m.v[1], m.s[0], m.s[1], m.s[2]);
  qplane_sub(xh, s[3], s[4], s[5], m.v[2], m.v[3], m.s[3], m.s[4], m.s[5]);
}

// (ol, oh) = c*y, c in GF(2^8), tower coordinates.
__device__ __forceinline__ void qmul_sub_set(uint32_t& ol, uint32_t& oh, uint32_t yl, uint32_t yh, const Mult& m) {
  uint32_t s[6];
  selectors(yl, yh, s);
  qplane_sub_set(ol, s[0], s[1], s[2], m.v[0], m.v[1], m.s[0], m.s[1], m.s[2]);
  qplane_sub_set(oh, s[3], s[4], s[5], m.v[2], m.v[3], m.s[3], m.s[4], m.s[5]);
}

// x ^= c*y: the subfield form (SUB) or the full 16 x 16 map.
template <bool SUB>
__device__ __forceinline__ void qmul_mode(uint32_t& xl, uint32_t& xh, uint32_t yl, uint32_t yh, const Mult& m) {
  if constexpr (SUB)
    qmul_sub(xl, xh, yl, yh, m);
  else
    qmul(xl, xh, yl, yh, m);
}

typedef const __attribute__((address_space(4))) uint32_t* cpool_t;

// Multiplier tables of the additive element c via the scalar cache (c is
// wave-uniform, so this is s_load); TW: tower coordinates (tower_pools).
template <bool TW = false>
__device__ __forceinline__ void pool_of(const DevTables& T, uint32_t c, uint32_t (&p)[20]) {
  // opaque index: two fetches of the same table (e.g. beta, or the index-0
  // skews shared by an IFFT and an FFT) must not be merged into one long-lived value
  asm volatile("" : "+s"(c));
  const cpool_t q = (cpool_t)(TW ? T.tower_pools : T.perm_pools) + c * kPoolWords;
#pragma unroll
  for (int i = 0; i < 20; ++i) p[i] = q[i];
}

// The skew tables of a transform: Cantor coordinates (perm_pools, the k = 1024
// kernels) or tower coordinates (tower_pools, TW: the fast kernels).
template <bool TW>
__device__ __forceinline__ const uint32_t* skew_pools(const DevTables& T) {
  return TW ? T.tower_pools : T.perm_pools;
}

// Only the SGPR half (dwords 8..19) of the tables of c.
// SUB: only the 6 dwords a subfield pool uses.
// OUT: out_pools (the level-0 groups of a kEncConv transform).
template <bool TW = false, bool SUB = false, bool OUT = false>
__device__ __forceinline__ void spool_of(const DevTables& T, uint32_t c, uint32_t (&p)[12]) {
  asm volatile("" : "+s"(c));
  const cpool_t q = (cpool_t)(OUT ? T.out_pools : skew_pools<TW>(T)) + c * kPoolWords + 8;
#pragma unroll
  for (int i = 0; i < (SUB ? 6 : 12); ++i) p[i] = q[i];
}

__device__ __forceinline__ uint32_t uniform(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
  return (static_cast<uint64_t>(uniform(static_cast<uint32_t>(v >> 32))) << 32) | uniform(static_cast<uint32_t>(v));
}

// A wave-uniform value the compiler must treat as new here: stops common
// subexpressions (row offsets, table indices) of different phases from being
// merged into values that stay live in SGPRs across the whole kernel.
__device__ __forceinline__ uint32_t fresh_v(uint32_t v) {  // same for a per-lane value
  asm volatile("" : "+v"(v));
  return v;
}

// This thread's lane (0..63), recomputed here (v_mbcnt): a loop that takes
// its lane per iteration from this keeps no thread-id VGPR live across the
// iterations (which the allocator may spill at its 128-VGPR budget, and a
// spill reload's vmcnt(0) waits for every load and store in flight).
__device__ __forceinline__ uint32_t lane_fresh() {
  uint32_t l;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
  return l;
}

template <typename T>
__device__ __forceinline__ T fresh(T v) {
  static_assert(sizeof(T) == 4 || sizeof(T) == 8, "scalar register value");
  if constexpr (sizeof(T) == 4) {
    uint32_t u;
    __builtin_memcpy(&u, &v, 4);
    asm volatile("" : "+s"(u));
    __builtin_memcpy(&v, &u, 4);
  } else {
    uint64_t u;
    __builtin_memcpy(&u, &v, 8);
    asm volatile("" : "+s"(u));
    __builtin_memcpy(&v, &u, 8);
  }
  return v;
}

// The table pointers as new values (see fresh): inside a loop over tiles,
// keeps the compiler from hoisting loads and addresses derived from them
// (staged tables, pool addresses) out of the loop into live registers.
__device__ __forceinline__ DevTables fresh_tables(const DevTables& T) {
  DevTables t = T;
  t.log = fresh(t.log);
  t.exp = fresh(t.exp);
  t.skew = fresh(t.skew);
  t.skew_add = fresh(t.skew_add);
  t.log_walsh = fresh(t.log_walsh);
  t.lw_fold = fresh(t.lw_fold);
  t.perm_pools = fresh(t.perm_pools);
  t.tower_pools = fresh(t.tower_pools);
  t.in_pools = fresh(t.in_pools);
  t.out_pools = fresh(t.out_pools);
  t.tower_full_sub = fresh(t.tower_full_sub);
  t.zeros = fresh(t.zeros);
  return t;
}

// ------------------------------------------------------ byte reshuffles ----
// 8-byte block (4 big-endian symbols) <-> byte-planar quad.
__device__ __forceinline__ void blk_to_quad(uint2 d, uint32_t& l, uint32_t& h) {
  l = vperm(d.y, d.x, 0x07050301u);
  h = vperm(d.y, d.x, 0x06040200u);
}
__device__ __forceinline__ uint2 quad_to_blk(uint32_t l, uint32_t h) {
  return make_uint2(vperm(l, h, 0x05010400u), vperm(l, h, 0x07030602u));
}

// Blocks of 4 columns (d[i] = column i, positions 4u..4u+3) -> cq registers
// cl[v] / ch[v] = position 4u+v of columns 0..3.
__device__ __forceinline__ void blks_to_cq(const uint2 (&d)[4], uint32_t* cl, uint32_t* ch) {
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

// Shard-row bytes of one position for the lane's 4 columns.
__device__ __forceinline__ uint2 cq_row(uint32_t l, uint32_t h) {
  return make_uint2(vperm(l, h, 0x05010400u), vperm(l, h, 0x07030602u));
}

__device__ __forceinline__ void cq_to_blks(const uint32_t* cl, const uint32_t* ch, uint2 (&d)[4]) {
  const uint2 r0 = cq_row(cl[0], ch[0]), r1 = cq_row(cl[1], ch[1]);
  const uint2 r2 = cq_row(cl[2], ch[2]), r3 = cq_row(cl[3], ch[3]);
  d[0] = make_uint2(vperm(r1.x, r0.x, 0x05040100u), vperm(r3.x, r2.x, 0x05040100u));
  d[1] = make_uint2(vperm(r1.x, r0.x, 0x07060302u), vperm(r3.x, r2.x, 0x07060302u));
  d[2] = make_uint2(vperm(r1.y, r0.y, 0x05040100u), vperm(r3.y, r2.y, 0x05040100u));
  d[3] = make_uint2(vperm(r1.y, r0.y, 0x07060302u), vperm(r3.y, r2.y, 0x07060302u));
}

// 4 symbols (columns 4l..4l+3 of one shard row) to / from global memory.
// `full` (wave-uniform) = whole 256-column tile present and 8-byte aligned rows.
// Partial tiles: lanes whose four columns all exist still use one 8-byte
// access (any even address, rows_vec_ok below).
// (The checked build does not instrument the encodes' shard-row stores here or
// in store_rows: a check in their per-lane branches made the compiler move the
// scalar table operands of the surrounding transforms into VGPRs, which it
// cannot compile.  The decode-side loads and copy-outs are checked.)
__device__ __forceinline__ void store4(uint8_t* rowp, uint2 v, uint32_t lane, uint32_t ncols, bool full) {
  if (full) {
    *reinterpret_cast<uint2*>(rowp + 8u * lane) = v;
    return;
  }
  const uint32_t w[2] = {v.x, v.y};
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (4 * lane + i < ncols) {
      const uint16_t s = static_cast<uint16_t>(w[i >> 1] >> (16 * (i & 1)));
      *reinterpret_cast<uint16_t*>(rowp + 8u * lane + 2 * i) = s;
    }
}

__device__ __forceinline__ uint2 load4(const uint8_t* rowp, uint32_t lane, uint32_t ncols, bool full) {
  if (full || 4 * lane + 4 <= ncols) return *reinterpret_cast<const uint2*>(NP_BCHK2(rowp + 8u * lane, 8, kBkShards, kBkZeros));
  uint32_t w[2] = {0, 0};
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (4 * lane + i < ncols)
      w[i >> 1] |= static_cast<uint32_t>(*reinterpret_cast<const uint16_t*>(NP_BCHK2(rowp + 8u * lane + 2 * i, 2, kBkShards, kBkZeros))) << (16 * (i & 1));
  return make_uint2(w[0], w[1]);
}

// Shard-row pieces of rows row0..row0+NR-1 for this lane.  Absent rows read
// the zero page instead (no branch, no HBM traffic).
template <int NR>
__device__ __forceinline__ void load_rows(uint2 (&raw)[NR], const uint8_t* sh, size_t shard_len, const uint8_t* PR,
                                          uint32_t row0, const uint8_t* zeros, uint32_t lane, uint32_t ncols,
                                          bool full) {
  const uint8_t* src[NR];
#pragma unroll
  for (int p = 0; p < NR; ++p)
    src[p] = uniform(PR[row0 + p]) ? sh + static_cast<size_t>(row0 + p) * shard_len : zeros;
  if (full) {
#pragma unroll
    for (int p = 0; p < NR; ++p) raw[p] = *reinterpret_cast<const uint2*>(NP_BCHK2(src[p] + 8u * lane, 8, kBkShards, kBkZeros));
  } else {
#pragma unroll
    for (int p = 0; p < NR; ++p) raw[p] = load4(src[p], lane, ncols, false);
  }
}

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));

// 8-byte accesses of data touched exactly once, with streaming (nt) cache
// policy: payload loads of the single-tile and k = 1024 encodes (config 4
// encode -5 %, config 2 neutral) and the k = 1024 reconstruct's output
// (whole lines; -1 %).
__device__ __forceinline__ uint2 load_once(const uint8_t* p) {
  const uint64_t v = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(NP_BCHK(p, 8, kBkPayloads)));
  return make_uint2(static_cast<uint32_t>(v), static_cast<uint32_t>(v >> 32));
}
__device__ __forceinline__ void store_once(uint8_t* p, uint2 v) {
  __builtin_nontemporal_store(static_cast<uint64_t>(v.x) | (static_cast<uint64_t>(v.y) << 32), reinterpret_cast<uint64_t*>(NP_BCHK(p, 8, kBkOut)));
}

// Raw buffer descriptor (V#) over [base, base + bytes): buffer loads and
// stores take the wave-uniform part of an address from SGPRs (base, soffset)
// and only the lane part from a VGPR, so row addressing costs no VALU.  A load
// at or beyond `bytes` returns zeros without touching memory.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, static_cast<int>(bytes), 0x00020000);
}

// A full tile's shard-row pieces move as 8-byte vector accesses, payload
// blocks and the decode's output as 8- / 16-byte ones, at any even (rows) / any (output) address:
// the KFD runs gfx9 queues in unaligned-access mode (SH_MEM_CONFIG alignment
// mode UNALIGNED; tools/microbench/unaligned.hip checks the bytes and the
// rates), so odd or 2-mod-4 chunk counts -- rows 2- or 4-byte aligned, e.g.
// the reference bench's 10 MB payloads at k = 512 -- keep the vector path
// instead of per-symbol accesses.  The parity tests with odd chunk counts pin
// it.
__device__ __forceinline__ bool rows_vec_ok(const void* p, size_t stride, size_t len) {
  return ((reinterpret_cast<uintptr_t>(p) | stride | len) & 1u) == 0;
}
// Streaming row stores for rows of whole 128-byte lines only (streaming partial
// lines made the 10 MB encode 3.8 ms instead of 2.3).
__device__ __forceinline__ bool rows_nt(const void* p, size_t stride, size_t len) {
  const uintptr_t v = reinterpret_cast<uintptr_t>(p) | stride | len;
  return (v & 127u) == 0;
}
__device__ __forceinline__ bool out_vec_ok(const void*, size_t) { return true; }  // any address (rows_vec_ok)

// Shard rows row0..row0+15 (those below wanted_n) from cq registers.
// Shard rows are written once and never read back by the encode: streaming
// (nontemporal, the nt bit of the buffer store) stores leave L2 to the tiles
// and tables; config 3 encode -3.3 %.
#ifndef kRowStoreCpol
#define kRowStoreCpol 2
#endif
// nt (rows_nt): streaming stores; otherwise the default policy.
__device__ __forceinline__ void store_rows(uint8_t* out, size_t shard_len, uint32_t row0, uint32_t wanted_n,
                                           const uint32_t (&L)[16], const uint32_t (&H)[16], uint32_t lane,
                                           uint32_t ncols, bool full, bool nt = true) {
  if (full && row0 + 16 <= wanted_n && 16 * shard_len < 0x7fffffffu) {
    const __amdgpu_buffer_rsrc_t r = buf_rsrc(out + static_cast<size_t>(row0) * shard_len, 16 * static_cast<uint32_t>(shard_len));
    if (nt) {
#pragma unroll
      for (int p = 0; p < 16; ++p) {
        const uint2 v = cq_row(L[p], H[p]);
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{v.x, v.y}, r, 8u * lane,
                                              static_cast<uint32_t>(p * shard_len), kRowStoreCpol);
      }
    } else {
#pragma unroll
      for (int p = 0; p < 16; ++p) {
        const uint2 v = cq_row(L[p], H[p]);
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{v.x, v.y}, r, 8u * lane, static_cast<uint32_t>(p * shard_len), 0);
      }
    }
  } else if (4 * lane + 4 <= ncols) {  // partial tile, lanes with all four columns
#pragma unroll
    for (int p = 0; p < 16; ++p)
      if (row0 + p < wanted_n) *reinterpret_cast<uint2*>(out + static_cast<size_t>(row0 + p) * shard_len + 8u * lane) = cq_row(L[p], H[p]);
  } else {
#pragma unroll
    for (int p = 0; p < 16; ++p)
      if (row0 + p < wanted_n) store4(out + static_cast<size_t>(row0 + p) * shard_len, cq_row(L[p], H[p]), lane, ncols, false);
  }
}

// ---------------------------------------------------------- transforms ----
// Software-pipelined multiplier fetch: group(f, pool) runs for f = 0..NG-1 and
// the 20 table dwords of group f+1 are requested before group f executes.  The
// scheduling barriers stop the compiler from hoisting the s_loads of a whole
// pass (20 SGPRs each) ahead of their use, which spills SGPRs into VGPRs.
template <int F>
using Int = std::integral_constant<int, F>;

template <int F, int NG, typename CF, typename GF>
__device__ __forceinline__ void pipe_step(const DevTables& T, CF& cval, GF& group, uint32_t (&cur)[20],
                                          uint32_t (&nxt)[20]) {
  if constexpr (F < NG) {
    if constexpr (F + 1 < NG) pool_of(T, cval(Int<F + 1>{}), nxt);
    __builtin_amdgcn_sched_barrier(0);
    group(Int<F>{}, make_mult(cur));
    __builtin_amdgcn_sched_barrier(0);
    pipe_step<F + 1, NG>(T, cval, group, nxt, cur);
  }
}

// cval(Int<f>) -> multiplier of group f; group(Int<f>, pool) runs group f.
template <int NG, typename CF, typename GF>
__device__ __forceinline__ void pipelined(const DevTables& T, CF cval, GF group) {
  uint32_t pa[20], pb[20];
  pool_of(T, cval(Int<0>{}), pa);
  pipe_step<0, NG>(T, cval, group, pa, pb);
}

// (Measured and not kept: an explicit lgkmcnt(0) wait at each group's start,
// so that the next group's table prefetch overlaps -- neutral, config 3
// +0.3 %; the row tables' VGPR half by vector loads -- +7 % on the decode.)

// Same with group f's tables at rec(Int<f>) (a wave-uniform global address).
__device__ __forceinline__ void pool_at(cpool_t q, uint32_t (&p)[20]) {
#pragma unroll
  for (int i = 0; i < 20; ++i) p[i] = q[i];
}

// need(f) (wave-uniform): group f multiplies; the tables of the others are
// not fetched (their group must not use the multiplier).
template <int F, int NG, typename RF, typename NF, typename GF>
__device__ __forceinline__ void rpipe_step(RF& rec, NF& need, GF& group, uint32_t (&cur)[20], uint32_t (&nxt)[20]) {
  if constexpr (F < NG) {
    if constexpr (F + 1 < NG) {
      if (need(Int<F + 1>{})) pool_at(rec(Int<F + 1>{}), nxt);
    }
    __builtin_amdgcn_sched_barrier(0);
    group(Int<F>{}, make_mult(cur));
    __builtin_amdgcn_sched_barrier(0);
    rpipe_step<F + 1, NG>(rec, need, group, nxt, cur);
  }
}

template <int NG, typename RF, typename NF, typename GF>
__device__ __forceinline__ void pipelined_rec(RF rec, NF need, GF group) {
  uint32_t pa[20], pb[20];
  if (need(Int<0>{})) pool_at(rec(Int<0>{}), pa);
  rpipe_step<0, NG>(rec, need, group, pa, pb);
}

// Same for a transform whose VGPR table halves are staged in LDS (VP, see
// stage_vpools): group f reads them at vaddr(f); only the SGPR half is
// prefetched with s_load.
// subf(Int<f>) -> std::integral_constant<bool, group f multiplies in the subfield form>.
// OUTF(f): integral_constant<bool>, group f's SGPR half from out_pools.
struct NoOut {
  template <typename FC>
  __device__ __forceinline__ std::false_type operator()(FC) const {
    return {};
  }
};
template <int F, int NG, bool TW, typename CF, typename VF, typename SF, typename GF, typename OF>
__device__ __forceinline__ void spipe_step(const DevTables& T, CF& cval, VF& vaddr, SF& subf, GF& group, OF& outf,
                                           uint32_t (&cur)[12], uint32_t (&nxt)[12]) {
  if constexpr (F < NG) {
    if constexpr (F + 1 < NG)
      spool_of<TW, decltype(subf(Int<F + 1>{}))::value, decltype(outf(Int<F + 1>{}))::value>(T, cval(Int<F + 1>{}),
                                                                                             nxt);
    __builtin_amdgcn_sched_barrier(0);
    group(Int<F>{}, staged_mult<decltype(subf(Int<F>{}))::value>(cur, vaddr(Int<F>{})));
    __builtin_amdgcn_sched_barrier(0);
    spipe_step<F + 1, NG, TW>(T, cval, vaddr, subf, group, outf, nxt, cur);
  }
}

template <int NG, bool TW = false, typename CF, typename VF, typename SF, typename GF, typename OF = NoOut>
__device__ __forceinline__ void pipelined_staged(const DevTables& T, CF cval, VF vaddr, SF subf, GF group,
                                                 OF outf = OF{}) {
  uint32_t pa[12], pb[12];
  spool_of<TW, decltype(subf(Int<0>{}))::value, decltype(outf(Int<0>{}))::value>(T, cval(Int<0>{}), pa);
  spipe_step<0, NG, TW>(T, cval, vaddr, subf, group, outf, pa, pb);
}

// LDS slot of the multiplier of group t at level b of a size-K transform:
// levels in order, K >> (b + 1) groups each (K - 1 slots of 8 dwords).
template <int K>
__host__ __device__ constexpr uint32_t vslot(int b, uint32_t t) {
  return static_cast<uint32_t>(K - (K >> b)) + t;
}

// Copies the VGPR halves (8 dwords) of every multiplier of a size-K transform
// at `index` into VP (K - 1 slots).  Caller synchronises.
// tw: tower_pools (the transform runs in tower coordinates), else perm_pools.
// l0_out (forward transforms whose outputs leave the tower, kEncConv): the
// level-0 slots from out_pools (tower in, Cantor out) instead.
template <int K, int NT>
__device__ __forceinline__ void stage_vpools(const DevTables& T, uint32_t index, uint32_t* VP, bool tw = false,
                                             bool l0_out = false) {
  // scalar base (a select the compiler may otherwise do per lane, in a VGPR
  // pair that gets spilled across the callers' loops)
  const uint32_t* pools = fresh(tw ? T.tower_pools : T.perm_pools);
  const uint32_t* pools0 = fresh(l0_out ? T.out_pools : pools);
  for (uint32_t i = fresh_v(threadIdx.x); i < 2u * (K - 1); i += NT) {
    const uint32_t slot = i >> 1, half = i & 1u;
    uint32_t b = 0;
    while (slot >= static_cast<uint32_t>(K - (K >> (b + 1)))) ++b;
    const uint32_t t = slot - static_cast<uint32_t>(K - (K >> b));
    const uint32_t c = 2u * t + (index >> b);
    *reinterpret_cast<uint4*>(VP + 8 * slot + 4 * half) =
        *reinterpret_cast<const uint4*>((b == 0 ? pools0 : pools) + static_cast<size_t>(c) * kPoolWords + 4 * half);
  }
}

struct GroupRef {
  int b, t;
};

// Flat group f of the cq levels (15 groups: 8, 4, 2, 1 per level).
template <bool INVERSE>
__host__ __device__ constexpr GroupRef cq_group(int f) {
  for (int s = 0; s < 4; ++s) {
    const int b = INVERSE ? s : 3 - s, n = 8 >> b;
    if (f < n) return GroupRef{b, f};
    f -= n;
  }
  return GroupRef{0, 0};
}

// Flat group f of the high levels (groups 16 / 2^(b-1-logR) per level b).
template <int K, bool INVERSE>
__host__ __device__ constexpr GroupRef hi_group(int f) {
  constexpr int logK = Geo<K>::kLog, logR = Geo<K>::kLogR;
  for (int s = 0; s < logK - 4; ++s) {
    const int b = INVERSE ? 4 + s : logK - 1 - s, n = 16 >> (b - 1 - logR);
    if (f < n) return GroupRef{b, f};
    f -= n;
  }
  return GroupRef{0, 0};
}

template <int K>
__host__ __device__ constexpr int hi_groups() {
  int n = 0;
  for (int b = 4; b < Geo<K>::kLog; ++b) n += 16 >> (b - 1 - Geo<K>::kLogR);
  return n;
}

// Levels 0..3 in the cq layout: CL/CH[p] = position 16g + p.  Group t of level
// b is g * (8 >> b) + (p >> (b + 1)).  `rows` (wave-uniform bit p = position
// 16g + p): inverse transforms skip the groups none of whose input rows is
// set (all-zero inputs stay zero), forward ones the groups none of whose
// output rows is set (outputs nobody reads); ~0u runs every group.
// Tower coordinates (field_tables.hpp HostTables::tower_a).  GEN >= 0: the
// transform runs in tower coordinates and its levels b >= GEN multiply in the
// subfield form (every skew of such a level lies in GF(2^8)), levels b < GEN
// with the full map; GEN = -1: Cantor coordinates (perm_pools).  For a size-K
// transform at index I the skews of level b are Cantor((I >> b) + 2t), all
// below 256 exactly when (I >> b) < 256 (I is a multiple of K), so the right
// GEN is gen_of(I).
template <int GEN>
constexpr bool kSubLevel(int b) {
  return GEN >= 0 && b >= GEN;
}

__host__ __device__ constexpr uint32_t gen_of(uint32_t index) {
  uint32_t g = 0;
  while ((index >> g) >= 256u) ++g;
  return g;
}

// f(Int<G>) for G = gen_of(index) when MING <= G <= MAXG (a wave-uniform
// branch over compile-time instances; the caller guarantees G >= MING);
// beyond MAXG f(Int<-1>) (Cantor coordinates, the caller converts) when
// FALLBACK, else f(Int<MAXG>) (the caller guarantees G <= MAXG).
template <int G, int MAXG, bool FALLBACK, typename F>
__device__ __forceinline__ void with_gen_from(uint32_t g, F& f) {
  if constexpr (G == MAXG) {
    if constexpr (FALLBACK) {
      if (g == MAXG) return f(Int<MAXG>{});
      return f(Int<-1>{});
    } else {
      return f(Int<MAXG>{});
    }
  } else {
    if (g == G) return f(Int<G>{});
    return with_gen_from<G + 1, MAXG, FALLBACK>(g, f);
  }
}

template <int MING, int MAXG, bool FALLBACK, typename F>
__device__ __forceinline__ void with_gen(uint32_t index, F&& f) {
  static_assert(MING <= MAXG, "gen range");
  const uint32_t g = __builtin_amdgcn_readfirstlane(gen_of(index));
  with_gen_from<(MING > 0 ? MING : 0), MAXG, FALLBACK>(g, f);
}

// The VGPR half (dwords 2..3) of the conversion's table, by a scalar load: the
// compiler otherwise reads it with a vector load (it cannot prove that the row
// stores do not alias the tables), and that load's vmcnt(0) wait also waits
// for every row store issued before it.
__device__ __forceinline__ uint64_t tower_conv_vhalf(cpool_t q) {
  uint64_t s23, vv;
  asm volatile("s_load_dwordx2 %0, %1, 0x8\n\ts_waitcnt lgkmcnt(0)" : "=s"(s23) : "s"(q) : "memory");
  asm volatile("v_mov_b64 %0, %1" : "=v"(vv) : "s"(s23));
  return vv;
}

// The conversion's tables (tower_pools[kFieldSize], b slots) for a fused
// conversion (qbfly_fwd_conv): 3 SGPR and 2 VGPR dwords.
struct ConvTab {
  uint32_t sa, sb, sc, va, vb;
};
__device__ __forceinline__ ConvTab conv_tab(const DevTables& T) {
  const cpool_t q = (cpool_t)(T.tower_pools) + 65536u * kPoolWords;
  const uint64_t vv = tower_conv_vhalf(q);
  return ConvTab{q[8 + 3], q[8 + 4], q[8 + 5], static_cast<uint32_t>(vv), static_cast<uint32_t>(vv >> 32)};
}

// The forward butterfly of a transform's last level fused with the tower ->
// Cantor conversion of both outputs (kEncConv).  With x' = x ^ c y, y' = y ^ x'
// (tower coordinates) and Tc(v) = (v_L ^ A(v_H), v_H), A the conversion's
// high -> low plane map (tower_convert):
//   Tc(x')_L = x_L ^ A(x_H) ^ Tc(c y)_L,   Tc(x')_H = x_H ^ (c y)_H,
//   Tc(y')   = Tc(x') ^ Tc(y),             Tc(y)_L = y_L ^ A(y_H),
// where m = out_pools[c] computes exactly (Tc(c y)_L, (c y)_H) from tower y,
// and A(y_H) reuses the high plane's selectors of the product: 43 VALU
// instead of a butterfly (28) and two conversions (2 x 10).
__device__ __forceinline__ void qbfly_fwd_conv(uint32_t& xl, uint32_t& xh, uint32_t& yl, uint32_t& yh, const Mult& m,
                                               const ConvTab& a) {
  uint32_t s[6];
  selectors(yl, yh, s);
  uint32_t x0, x1, x2;  // selectors of x_H (before x_H changes)
  asm volatile(
      "v_and_b32 %0, 0x07070707, %3\n\t"
      "v_lshrrev_b32 %1, 3, %3\n\t"
      "v_lshrrev_b32 %2, 6, %3\n\t"
      "v_and_b32 %1, 0x07070707, %1\n\t"
      "v_and_b32 %2, 0x03030303, %2"
      : "=&v"(x0), "=&v"(x1), "=&v"(x2)
      : "v"(xh));
  qplane_sub(xl, x0, x1, x2, a.va, a.vb, a.sa, a.sb, a.sc);  // x_L ^ A(x_H)
  qplane(xl, s, m.v[0], m.v[1], m.v[2], m.v[3], m.s[0], m.s[1], m.s[2], m.s[3], m.s[4], m.s[5]);
  qplane(xh, s, m.v[4], m.v[5], m.v[6], m.v[7], m.s[6], m.s[7], m.s[8], m.s[9], m.s[10], m.s[11]);
  qplane_sub(yl, s[3], s[4], s[5], a.va, a.vb, a.sa, a.sb, a.sc);  // y_L ^ A(y_H)
  yl ^= xl;
  yh ^= xh;
}

// Progress-based issue priority (PRIO != 0): a wave lowers its issue priority
// as it works through a transform pass (3 in the first quarter of the pass's
// groups, 0 in the last), so the waves of a SIMD that are behind issue first
// and the four reach the pass's closing barrier together, instead of in age
// order (a SIMD favours its older waves).  The callers choose per kernel
// (kernels_fast.hip kEncPrio / kRecPrio*).
// PRIO 1: 3, 2, 1, 0 over the pass's quarters; 2: 3 throughout; 3: 1, 1, 0, 0;
// 4: 3, 3, 2, 2 (passes inside a longer barrier-free span, kernels_fast.hip
// kRecPrioSpan / kEncPrio).
template <int F, int NG, int PRIO>
__device__ __forceinline__ void progress_prio() {
  if constexpr (PRIO != 0) {
    constexpr int q = F * 4 / NG, qp = F == 0 ? -1 : (F - 1) * 4 / NG;
    constexpr int pr = PRIO == 1 ? 3 - q : PRIO == 2 ? 3 : PRIO == 3 ? (q < 2 ? 1 : 0) : (q < 2 ? 3 : 2);
    constexpr int pp = qp < 0 ? -1 : PRIO == 1 ? 3 - qp : PRIO == 2 ? 3 : PRIO == 3 ? (qp < 2 ? 1 : 0) : (qp < 2 ? 3 : 2);
    if constexpr (pr != pp) __builtin_amdgcn_s_setprio(pr);
  }
}

// GEN: coordinates and subfield levels (kSubLevel).
// POST(t), when given, runs after group t of the forward transform's level 0
// (rows 2t and 2t + 1 are final there).
struct NoPost {
  __device__ __forceinline__ void operator()(int) const {}
};
// CONV (forward, tower coordinates): the last level leaves the outputs in
// Cantor coordinates (qbfly_fwd_conv; VP's level-0 slots staged from out_pools,
// stage_vpools l0_out).
template <int K, bool INVERSE, bool INDEX0, int GEN = -1, bool CONV = false, int PRIO = 0, typename POST = NoPost>
__device__ __forceinline__ void cq_levels(const DevTables& T, const uint32_t* VP, uint32_t index, uint32_t g,
                                          uint32_t (&L)[16], uint32_t (&H)[16], uint32_t rows = ~0u,
                                          POST post = POST{}) {
  if constexpr (kExp & 1) return;
  static_assert(!CONV || (!INVERSE && GEN >= 0 && !kSubLevel<GEN>(0)), "fused conversion: forward, tower, full level 0");
  auto cval = [&](auto fc) __attribute__((always_inline)) {
    constexpr GroupRef r = cq_group<INVERSE>(decltype(fc)::value);
    return 2u * (g * (8u >> r.b) + r.t) + (index >> r.b);
  };
  auto vaddr = [&](auto fc) __attribute__((always_inline)) {
    constexpr GroupRef r = cq_group<INVERSE>(decltype(fc)::value);
    return VP + 8u * vslot<K>(r.b, g * (8u >> r.b) + r.t);
  };
  ConvTab ct{};  // CONV: loaded at level 0's first group, live through that level only
  auto group = [&](auto fc, const Mult& p) __attribute__((always_inline)) {
    constexpr GroupRef r = cq_group<INVERSE>(decltype(fc)::value);
    constexpr int d = 1 << r.b;
    progress_prio<decltype(fc)::value, 15, PRIO>();
    if constexpr (CONV && r.b == 0 && r.t == 0) ct = conv_tab(T);
    constexpr uint32_t span = ((1u << (2 * d)) - 1u) << (r.t * 2 * d);  // the group's rows
    if ((rows & span) == 0) return;
    auto body = [&](auto sub_c) __attribute__((always_inline)) {
      constexpr bool SUB = decltype(sub_c)::value;
#pragma unroll
      for (int u = 0; u < d; ++u) {
        const int x = r.t * 2 * d + u, y = x + d;
        if constexpr (CONV && r.b == 0) {
          qbfly_fwd_conv(L[x], H[x], L[y], H[y], p, ct);
        } else if (INVERSE) {
          L[y] ^= L[x];
          H[y] ^= H[x];
          qmul_mode<SUB>(L[x], H[x], L[y], H[y], p);
        } else {
          qmul_mode<SUB>(L[x], H[x], L[y], H[y], p);
          L[y] ^= L[x];
          H[y] ^= H[x];
        }
      }
    };
    body(std::integral_constant<bool, kSubLevel<GEN>(r.b)>{});
    if constexpr (!INVERSE && r.b == 0) post(r.t);
  };
  auto subf = [&](auto fc) __attribute__((always_inline)) {
    return std::integral_constant<bool, kSubLevel<GEN>(cq_group<INVERSE>(decltype(fc)::value).b)>{};
  };
  auto outf = [&](auto fc) __attribute__((always_inline)) {
    return std::integral_constant<bool, CONV && cq_group<INVERSE>(decltype(fc)::value).b == 0>{};
  };
  pipelined_staged<15, (GEN >= 0)>(T, cval, vaddr, subf, group, outf);
}

// Levels 4..logK-1 in the high layout: quad j pairs with j + 2^(b-2-logR);
// group t = j >> (b-1-logR).  FIRST > 0 starts at flat group FIRST (the
// forward transform's top level, one group, done by the caller: fwd_top).
// HOOK (forward transforms): hook.pre() runs before the first group of level
// 4 (the last high level) and hook.post(t) after its group t (quads 2t and
// 2t + 1 are final there).
struct NoHiHook {
  __device__ __forceinline__ void pre() const {}
  __device__ __forceinline__ void post(int) const {}
};
template <int K, bool INVERSE, bool INDEX0, int FIRST = 0, int GEN = -1, int PRIO = 0, typename HOOK = NoHiHook>
__device__ __forceinline__ void hi_levels(const DevTables& T, const uint32_t* VP, uint32_t index, uint32_t (&L)[16],
                                          uint32_t (&H)[16], HOOK hook = HOOK{}) {
  if constexpr (kExp & 1) return;
  constexpr int logR = Geo<K>::kLogR;
  auto cval = [&](auto fc) __attribute__((always_inline)) {
    constexpr GroupRef r = hi_group<K, INVERSE>(decltype(fc)::value + FIRST);
    return 2u * r.t + (index >> r.b);
  };
  auto vaddr = [&](auto fc) __attribute__((always_inline)) {
    constexpr GroupRef r = hi_group<K, INVERSE>(decltype(fc)::value + FIRST);
    return VP + 8u * vslot<K>(r.b, r.t);
  };
  auto group = [&](auto fc, const Mult& p) __attribute__((always_inline)) {
    constexpr GroupRef r = hi_group<K, INVERSE>(decltype(fc)::value + FIRST);
    constexpr int dj = 1 << (r.b - 2 - logR);
    constexpr bool live = !INDEX0 || r.t != 0;
    progress_prio<decltype(fc)::value, hi_groups<K>() - FIRST, PRIO>();
    if constexpr (!INVERSE && r.b == 4 && r.t == 0) hook.pre();
    auto body = [&](auto sub_c) __attribute__((always_inline)) {
      constexpr bool SUB = decltype(sub_c)::value;
#pragma unroll
      for (int u = 0; u < dj; ++u) {
        const int x = r.t * 2 * dj + u, y = x + dj;
        if (INVERSE) {
          L[y] ^= L[x];
          H[y] ^= H[x];
          if (live) qmul_mode<SUB>(L[x], H[x], L[y], H[y], p);
        } else {
          if (live) qmul_mode<SUB>(L[x], H[x], L[y], H[y], p);
          L[y] ^= L[x];
          H[y] ^= H[x];
        }
      }
    };
    body(std::integral_constant<bool, kSubLevel<GEN>(r.b)>{});
    if constexpr (!INVERSE && r.b == 4) hook.post(r.t);
  };
  auto subf = [&](auto fc) __attribute__((always_inline)) {
    return std::integral_constant<bool, kSubLevel<GEN>(hi_group<K, INVERSE>(decltype(fc)::value + FIRST).b)>{};
  };
  pipelined_staged<hi_groups<K>() - FIRST, (GEN >= 0)>(T, cval, vaddr, subf, group);
}

// Top level (b = logK - 1, one group, quads j and j + 8) of the forward
// transform FFT(K, index) in the high layout, as the encode's shift loop runs
// it.  Its skew is Cantor(index >> b) = Cantor(2s) at index = sK: linear in s,
// so the products c_s * X[j + 8] of shift 3 are those of shifts 1 and 2 XORed
// (the inputs X = M are the same for every shift).  MODE 0: multiply; 1:
// multiply and keep the products in P; 2: multiply and XOR them into P; 3:
// take the products from P (no multiply).
template <int K, int MODE, int GEN = -1>
__device__ __forceinline__ void fwd_top(const DevTables& T, const uint32_t* VP, uint32_t index, uint32_t (&L)[16],
                                        uint32_t (&H)[16], uint32_t (&PL)[8], uint32_t (&PH)[8]) {
  if constexpr (kExp & 1) return;
  constexpr int b = Geo<K>::kLog - 1;
  static_assert(b - 2 - Geo<K>::kLogR == 3, "top level pairs quads j, j + 8");
  Mult m;
  if constexpr (MODE != 3) {
    uint32_t sp[12];
    spool_of<(GEN >= 0), kSubLevel<GEN>(b)>(T, index >> b, sp);
    m = staged_mult<kSubLevel<GEN>(b)>(sp, VP + 8u * vslot<K>(b, 0));
  }
  constexpr bool sub = kSubLevel<GEN>(b);
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    uint32_t pl, ph;
    if constexpr (MODE == 3) {
      pl = PL[u], ph = PH[u];
    } else {
      if constexpr (sub)
        qmul_sub_set(pl, ph, L[u + 8], H[u + 8], m);
      else
        qmul_set(pl, ph, L[u + 8], H[u + 8], m);
      if constexpr (MODE == 1) PL[u] = pl, PH[u] = ph;
      if constexpr (MODE == 2) PL[u] ^= pl, PH[u] ^= ph;
    }
    L[u] ^= pl;
    H[u] ^= ph;
    L[u + 8] ^= L[u];
    H[u + 8] ^= H[u];
  }
}

// A ^= D_K(X) for one byte plane in the high layout: D(x)[j] = x[j] ^ XOR over
// single bits l not in j of x[j | l] (inc_afft.rs:17-31, closed form SURVEY F7).
// l = 1, 2 live inside a quad, l = 4 (and 8 for R = 4) in the neighbour lanes
// of the column, larger l in other registers of the lane.
template <int K>
__device__ __forceinline__ void add_derivative(uint32_t (&A)[16], uint32_t (&X)[16], uint32_t r) {
  constexpr int logR = Geo<K>::kLogR;
  const uint32_t m0 = (r & 1u) ? 0u : ~0u, m1 = (r & 2u) ? 0u : ~0u;
  // in place, ascending j: X[j | l] (l not in j) is still the original value
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t x = X[j];
    uint32_t v = xor3(x, vperm(x, x, 0x0C030301u), vperm(x, x, 0x0C0C0C02u));
    if (logR >= 1) v ^= static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(x), 0xB1, 0xF, 0xF, false)) & m0;
    if (logR >= 2) v ^= static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(x), 0x4E, 0xF, 0xF, false)) & m1;
#pragma unroll
    for (int jb = 0; jb < 4; ++jb)
      if (!(j & (1 << jb))) v ^= X[j | (1 << jb)];
    A[j] ^= v;
    asm volatile("" : "+v"(A[j]));  // finish position j here (bounded temporaries)
    X[j] = 0;                       // dead from here on
  }
}

// Cantor <-> tower coordinates of NR quads (an involution, field_tables.hpp
// HostTables::tower_a): the low plane takes A(high plane), 3 byte lookups of
// the high plane through the b slots of tower_pools[kFieldSize].
template <int NR>
__device__ __forceinline__ void tower_convert(const DevTables& T, uint32_t (&L)[NR], const uint32_t (&H)[NR]) {
  const cpool_t q = (cpool_t)(T.tower_pools) + 65536u * kPoolWords;
  const uint32_t sa = q[8 + 3], sb = q[8 + 4], sc = q[8 + 5];
  const uint64_t vv = tower_conv_vhalf(q);
  const uint32_t va = static_cast<uint32_t>(vv), vb = static_cast<uint32_t>(vv >> 32);
#pragma unroll
  for (int p = 0; p < NR; ++p) {
    uint32_t s0, s1, s2;  // one asm block: no quad's selectors are computed far ahead of its lookups
    asm volatile(
        "v_and_b32 %0, 0x07070707, %3\n\t"
        "v_lshrrev_b32 %1, 3, %3\n\t"
        "v_lshrrev_b32 %2, 6, %3\n\t"
        "v_and_b32 %1, 0x07070707, %1\n\t"
        "v_and_b32 %2, 0x03030303, %2"
        : "=&v"(s0), "=&v"(s1), "=&v"(s2)
        : "v"(H[p]));
    qplane_sub(L[p], s0, s1, s2, va, vb, sa, sb, sc);
  }
}

// ---------------------------------------------------------- LDS sweeps ----
template <int K, bool EVEN = false>
__device__ __forceinline__ void cq_read(const uint8_t* tile, uint32_t base, uint32_t (&L)[16], uint32_t (&H)[16]) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    uint2 d[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      d[i] = *reinterpret_cast<const uint2*>(tile + (base ^ (col_base_c<K, EVEN>(i) ^ (8u * u))));
    blks_to_cq(d, &L[4 * u], &H[4 * u]);
  }
}

template <int K>
__device__ __forceinline__ void cq_write(uint8_t* tile, uint32_t base, const uint32_t (&L)[16], const uint32_t (&H)[16]) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    uint2 d[4];
    cq_to_blks(&L[4 * u], &H[4 * u], d);
#pragma unroll
    for (int i = 0; i < 4; ++i) *reinterpret_cast<uint2*>(tile + (base ^ (col_base_c<K>(i) ^ (8u * u)))) = d[i];
  }
}

template <int K>
__device__ __forceinline__ void hi_read(const uint8_t* tile, uint32_t base, uint32_t (&L)[16], uint32_t (&H)[16]) {
#pragma unroll
  for (int j = 0; j < 16; ++j)
    blk_to_quad(*reinterpret_cast<const uint2*>(tile + (base ^ (8u * Geo<K>::R * j))), L[j], H[j]);
}

template <int K>
__device__ __forceinline__ void hi_write(uint8_t* tile, uint32_t base, const uint32_t (&L)[16], const uint32_t (&H)[16]) {
#pragma unroll
  for (int j = 0; j < 16; ++j)
    *reinterpret_cast<uint2*>(tile + (base ^ (8u * Geo<K>::R * j))) = quad_to_blk(L[j], H[j]);
}

// Planar exchange between the two layouts (the transforms' own LDS round
// trips; the payload tile and the output copy-out keep the natural block
// format above): a block holds (low bytes, high bytes) of 4 positions of one
// column, so the high layout moves its quads with no byte shuffle and the cq
// side does only the 4 x 4 byte transpose (positions x columns) of each plane.
__device__ __forceinline__ void tr4x4(uint32_t a0, uint32_t a1, uint32_t a2, uint32_t a3, uint32_t* o) {
  const uint32_t t01 = vperm(a1, a0, 0x05010400u), u01 = vperm(a1, a0, 0x07030602u);
  const uint32_t t23 = vperm(a3, a2, 0x05010400u), u23 = vperm(a3, a2, 0x07030602u);
  o[0] = vperm(t23, t01, 0x05040100u);
  o[1] = vperm(t23, t01, 0x07060302u);
  o[2] = vperm(u23, u01, 0x05040100u);
  o[3] = vperm(u23, u01, 0x07060302u);
}

template <int K>
__device__ __forceinline__ void cq_read_p(const uint8_t* tile, uint32_t base, uint32_t (&L)[16], uint32_t (&H)[16]) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    uint2 d[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      d[i] = *reinterpret_cast<const uint2*>(tile + (base ^ (col_base_c<K>(i) ^ (8u * u))));
    tr4x4(d[0].x, d[1].x, d[2].x, d[3].x, &L[4 * u]);
    tr4x4(d[0].y, d[1].y, d[2].y, d[3].y, &H[4 * u]);
  }
}

template <int K>
__device__ __forceinline__ void cq_write_p(uint8_t* tile, uint32_t base, const uint32_t (&L)[16],
                                           const uint32_t (&H)[16]) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    uint32_t l[4], h[4];
    tr4x4(L[4 * u], L[4 * u + 1], L[4 * u + 2], L[4 * u + 3], l);
    tr4x4(H[4 * u], H[4 * u + 1], H[4 * u + 2], H[4 * u + 3], h);
#pragma unroll
    for (int i = 0; i < 4; ++i)
      *reinterpret_cast<uint2*>(tile + (base ^ (col_base_c<K>(i) ^ (8u * u)))) = make_uint2(l[i], h[i]);
  }
}

template <int K>
__device__ __forceinline__ void hi_read_p(const uint8_t* tile, uint32_t base, uint32_t (&L)[16], uint32_t (&H)[16]) {
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint2 d = *reinterpret_cast<const uint2*>(tile + (base ^ (8u * Geo<K>::R * j)));
    L[j] = d.x;
    H[j] = d.y;
  }
}

template <int K>
__device__ __forceinline__ void hi_write_p(uint8_t* tile, uint32_t base, const uint32_t (&L)[16],
                                           const uint32_t (&H)[16]) {
#pragma unroll
  for (int j = 0; j < 16; ++j) *reinterpret_cast<uint2*>(tile + (base ^ (8u * Geo<K>::R * j))) = make_uint2(L[j], H[j]);
}

// Quad exchange between the cq layout and a column-quad high layout (the
// fast encodes): LDS item (position p, column quad c) = the uint2 (low plane,
// high plane) of columns 4c..4c+3 at position p, at byte 8 (64 p + c).  cq
// side: wave g, lane c holds positions 16 g + i.  High side (nres = 256 / K
// residues per thread): wave w, lane c, register j' = r + nres j holds
// position nres w + r + 16 j, so level b >= 4 pairs registers j' and
// j' + 2^(b-2-logR) with group j' >> (b-1-logR), as hi_levels expects
// (R = K / 64), and no byte transpose is needed on either side (tr4x4).
// Every wave-instruction moves 512 contiguous bytes.
__device__ __forceinline__ void cq_write_q(uint8_t* tile, uint32_t g, uint32_t lane, const uint32_t (&L)[16],
                                           const uint32_t (&H)[16]) {
  uint8_t* b = tile + 8192u * g + fresh_v(8u * lane);
#pragma unroll
  for (int i = 0; i < 16; ++i) *reinterpret_cast<uint2*>(b + 512u * i) = make_uint2(L[i], H[i]);
}
__device__ __forceinline__ void cq_read_q(const uint8_t* tile, uint32_t g, uint32_t lane, uint32_t (&L)[16],
                                          uint32_t (&H)[16]) {
  const uint8_t* b = tile + 8192u * g + fresh_v(8u * lane);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const uint2 d = *reinterpret_cast<const uint2*>(b + 512u * i);
    L[i] = d.x;
    H[i] = d.y;
  }
}
// Byte offset of high-layout register j' from the thread's base (K / 64 = R).
template <int K>
__host__ __device__ constexpr uint32_t hi_q_off(int jj) {
  constexpr int nres = 256 / K;
  return 512u * static_cast<uint32_t>(jj % nres + 16 * (jj / nres));
}
template <int K = 256>
__device__ __forceinline__ void hi_write_q(uint8_t* tile, uint32_t w, uint32_t lane, const uint32_t (&L)[16],
                                           const uint32_t (&H)[16]) {
  uint8_t* b = tile + 512u * (256u / K) * w + fresh_v(8u * lane);
#pragma unroll
  for (int j = 0; j < 16; ++j) *reinterpret_cast<uint2*>(b + hi_q_off<K>(j)) = make_uint2(L[j], H[j]);
}
template <int K = 256>
__device__ __forceinline__ void hi_read_q(const uint8_t* tile, uint32_t w, uint32_t lane, uint32_t (&L)[16],
                                          uint32_t (&H)[16]) {
  const uint8_t* b = tile + 512u * (256u / K) * w + fresh_v(8u * lane);
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint2 d = *reinterpret_cast<const uint2*>(b + hi_q_off<K>(j));
    L[j] = d.x;
    H[j] = d.y;
  }
}

// ---------------------------------------------------------------- locator ----
// eval_error_polynomial (inc_reconstruct.rs:90-113, called over the whole field
// by mod.rs:217-218) for an erasure set inside [0, N), folded to N points
// (SURVEY F8): loc = WHT_N(WHT_N(e) * F_N mod 65535) mod 65535 with F_N the
// folded LOG_WALSH (field_tables.hpp).  Equal to the reference mod 65535, which
// is all a multiplier needs (EXP[65535] == EXP[0]).  Leaves E[v] = EXP[loc] for
// present rows and EXP[65535 - loc] for erased rows (the postmultiplier,
// inc_reconstruct.rs:108-112), and PR[v] = present flag.  W: N dwords of scratch.
// Walsh-Hadamard transform of W[0, N) in LDS, two levels per pass (each
// thread takes groups of 4 elements: levels b and b + 1 in registers), so a
// size-1024 transform has 5 barriers instead of 10.  MOD = false: exact in
// int32 (the 0/1 erasure vector, |x| <= N); MOD = true: mod 65535 with
// canonical residues in [0, 65534], so the level order does not matter (only
// the residue enters a multiplier: EXP[65535] == EXP[0]).
template <bool MOD>
__device__ __forceinline__ void wht_bfly(uint32_t& x, uint32_t& y) {
  if constexpr (MOD) {
    uint32_t s = x + y, d = x + 65535u - y;
    s -= s >= 65535u ? 65535u : 0u;
    d -= d >= 65535u ? 65535u : 0u;
    x = s;
    y = d;
  } else {
    const int32_t a = static_cast<int32_t>(x), b = static_cast<int32_t>(y);
    x = static_cast<uint32_t>(a + b);
    y = static_cast<uint32_t>(a - b);
  }
}
template <int N, int NT, bool MOD>
__device__ __forceinline__ void lds_wht(uint32_t* W) {
  const uint32_t tid = threadIdx.x;
  int b = 0;
#pragma unroll 1
  for (; (2 << b) < N; b += 2) {  // levels b, b + 1 (both below log2 N)
    const uint32_t h = 1u << b;
    for (uint32_t q = tid; q < N / 4; q += NT) {
      const uint32_t i = ((q & ~(h - 1u)) << 2) | (q & (h - 1u));
      uint32_t x0 = W[i], x1 = W[i + h], x2 = W[i + 2 * h], x3 = W[i + 3 * h];
      wht_bfly<MOD>(x0, x1);
      wht_bfly<MOD>(x2, x3);
      wht_bfly<MOD>(x0, x2);
      wht_bfly<MOD>(x1, x3);
      W[i] = x0, W[i + h] = x1, W[i + 2 * h] = x2, W[i + 3 * h] = x3;
    }
    __syncthreads();
  }
  if ((1 << b) < N) {  // log2 N odd: the last level alone
    const uint32_t h = 1u << b;
    for (uint32_t q = tid; q < N / 2; q += NT) {
      const uint32_t i = ((q & ~(h - 1u)) << 1) | (q & (h - 1u));
      uint32_t x = W[i], y = W[i + h];
      wht_bfly<MOD>(x, y);
      W[i] = x, W[i + h] = y;
    }
    __syncthreads();
  }
}

// The locator from the erasure indicator W[v] = (row v absent) and PR[v] (the
// present flag), both in LDS and synchronised: see fused_locator.
template <int N, int NT>
__device__ __forceinline__ void fused_locator_core(const DevTables& T, uint32_t* W, uint16_t* E, const uint8_t* PR) {
  const uint32_t tid = threadIdx.x;
  lds_wht<N, NT, false>(W);  // integer WHT of the 0/1 erasure vector
  const uint16_t* F = T.lw_fold + N;
  for (uint32_t v = tid; v < N; v += NT) {
    const int32_t x = static_cast<int32_t>(W[v]);  // |x| <= N
    const uint32_t m = x < 0 ? static_cast<uint32_t>(x + 65535) : static_cast<uint32_t>(x);
    W[v] = (m * static_cast<uint32_t>(F[v])) % 65535u;
  }
  __syncthreads();
  lds_wht<N, NT, true>(W);  // WHT mod 65535
  for (uint32_t v = tid; v < N; v += NT) *NP_BCHK(E + v, 2, kBkRecords) = T.exp[NP_ICHK(PR[v] ? W[v] : 65535u - W[v], 65536u)];
}

// The same, leaving each row's multiplier table (80 bytes: in_pools of
// EXP[loc] for a present row, out_pools of EXP[65535 - loc] for an erased one)
// at dst + 80 v instead of the u16 multipliers: the table loads follow the
// multiplier in registers (k_prefix_locator's records; write_row_pools'
// layout).
template <int N, int NT>
__device__ __forceinline__ void fused_locator_pools(const DevTables& T, uint32_t* W, const uint8_t* PR, uint8_t* dst) {
  const uint32_t tid = threadIdx.x;
  lds_wht<N, NT, false>(W);
  const uint16_t* F = T.lw_fold + N;
  for (uint32_t v = tid; v < N; v += NT) {
    const int32_t x = static_cast<int32_t>(W[v]);
    const uint32_t m = x < 0 ? static_cast<uint32_t>(x + 65535) : static_cast<uint32_t>(x);
    W[v] = (m * static_cast<uint32_t>(F[v])) % 65535u;
  }
  __syncthreads();
  lds_wht<N, NT, true>(W);
  // (the row's table follows its multiplier in registers; batching four rows'
  // table loads ahead of their stores measured 98 us per launch against 55.5,
  // config 3)
  for (uint32_t v = tid; v < N; v += NT) {
    const bool p = PR[v] != 0;
    const uint32_t e = T.exp[NP_ICHK(p ? W[v] : 65535u - W[v], 65536u)];
    const uint4* src = reinterpret_cast<const uint4*>((p ? T.in_pools : T.out_pools) + static_cast<size_t>(e) * kPoolWords);
    uint4* d = NP_BCHK(reinterpret_cast<uint4*>(dst + static_cast<size_t>(v) * 4 * kPoolWords), 4 * kPoolWords, kBkRecords);
    const uint4 a0 = src[0], a1 = src[1], a2 = src[2], a3 = src[3], a4 = src[4];
    d[0] = a0, d[1] = a1, d[2] = a2, d[3] = a3, d[4] = a4;
  }
}

template <int N, int NT>
__device__ __forceinline__ void fused_locator(const DevTables& T, const uint8_t* pres, uint32_t* W, uint16_t* E,
                                              uint8_t* PR) {
  const uint32_t tid = threadIdx.x;
  for (uint32_t v = tid; v < N; v += NT) {
    const uint8_t p = *NP_BCHK(pres + v, 1, kBkPresent);
    PR[v] = p;
    W[v] = p ? 0u : 1u;
  }
  __syncthreads();
  fused_locator_core<N, NT>(T, W, E, PR);
}

}  // namespace
}  // namespace np
