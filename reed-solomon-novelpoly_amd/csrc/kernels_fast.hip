// Specialised gfx950 kernels for the hot shapes: k = K in {64, 128, 256},
// encode for n >= 2K, reconstruct for n in {2K, 4K} (every BASELINE shape
// with k <= 256).
//
// Work mapping.  A workgroup owns a tile of 256 codeword columns (encode: 256
// payload chunks; reconstruct: 256 symbol columns of the shards).  A
// size-K transform (K = 2^logK positions) is split in two register layouts
// that meet in a 256 x K LDS tile:
//
//  * "column-quad" (cq) layout -- levels 0..3.  Wave g owns positions
//    16g..16g+15, lane l owns columns 4l..4l+3; register CL[p] / CH[p] hold
//    the low / high bytes of position 16g+p of those four columns.  Shard rows
//    are position-major, so this layout is also the one that reads and writes
//    shard rows with coalesced 8-byte accesses.
//  * "high" layout -- levels 4..logK-1.  R = K/64 adjacent lanes share a
//    column; lane (c, r) holds the 16 position-quads m = R*j + r (j = 0..15)
//    as byte-planar pairs (L[j], H[j]).  Butterflies of these levels pair
//    quads j and j + 2^(b-2-logR) of one lane.
//
// In both layouts every butterfly group is the same for all lanes of a wave,
// so each GF(2^16) multiplier is wave-uniform: c*y is the XOR of 12 v_perm
// byte-table lookups whose 20 table dwords are fetched with s_load
// (field_tables.cpp builds them).  Each lane keeps 32 state dwords, so a
// 4K-thread workgroup fits 4 waves per SIMD.
//
// Reference: additive FFT inc_afft.rs:139-214 (inverse) / :267-332 (forward);
// encode inc_encode.rs:15-48 + mod.rs:117-157; reconstruct inc_reconstruct.rs:1-85
// + mod.rs:162-239.  The skew of group t at level b and transform index I is
// the field element with Cantor coordinates 2t + (I >> b)
// (tests/test_oracle.py::test_skews_are_cantor_points).
#include "device_common.hpp"
#include "launchers.hpp"

#include <type_traits>

namespace np {
namespace {

constexpr int kTile = 256;  // columns per workgroup
constexpr int kPoolWords = 20;

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
};

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
template <int K>
__host__ __device__ constexpr uint32_t col_base_c(uint32_t c) {
  using G = Geo<K>;
  const uint32_t cs = c / G::P, ci = c % G::P;
  return 8u * cs * G::W + 8u * ((ci * G::Q) ^ swz<K>(cs));
}

// Runtime version; the asm keeps the compiler from materialising every block
// address of a sweep in its own VGPR.
template <int K>
__device__ __forceinline__ uint32_t col_base(uint32_t c) {
  uint32_t b = col_base_c<K>(c);
  asm volatile("" : "+v"(b));
  return b;
}

// ------------------------------------------------------------ GF multiply ----
__device__ __forceinline__ uint32_t vperm(uint32_t s0, uint32_t s1, uint32_t sel) {
  return __builtin_amdgcn_perm(s0, s1, sel);
}

// Byte-table selectors of four byte-planar symbols: bits 0-2, 3-5, 6-7 of
// every byte of the low plane (s[0..2]) and of the high plane (s[3..5]).  One
// asm block, so the extraction of a whole level is not hoisted ahead of use.
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

// A multiplier ready for use: its 20 table dwords in SGPRs plus VGPR copies of
// the 8 dwords that v_perm must read from a VGPR.  The copies are made by an
// asm block where the butterfly group starts, so that they are neither hoisted
// next to the s_load of a prefetched table nor repeated per butterfly.
struct Mult {
  uint32_t s[20];
  uint32_t v[8];
};

__device__ __forceinline__ Mult make_mult(const uint32_t (&p)[20]) {
  Mult m;
#pragma unroll
  for (int i = 0; i < 20; ++i) m.s[i] = p[i];
  asm volatile(
      "v_mov_b32 %0, %8\n\tv_mov_b32 %1, %9\n\tv_mov_b32 %2, %10\n\tv_mov_b32 %3, %11\n\t"
      "v_mov_b32 %4, %12\n\tv_mov_b32 %5, %13\n\tv_mov_b32 %6, %14\n\tv_mov_b32 %7, %15"
      : "=v"(m.v[0]), "=v"(m.v[1]), "=v"(m.v[2]), "=v"(m.v[3]), "=v"(m.v[4]), "=v"(m.v[5]), "=v"(m.v[6]),
        "=v"(m.v[7])
      : "s"(p[0]), "s"(p[2]), "s"(p[5]), "s"(p[7]), "s"(p[10]), "s"(p[12]), "s"(p[15]), "s"(p[17]));
  return m;
}

// x ^= c*y on four byte-planar symbols (pool layout: field_tables.cpp).
__device__ __forceinline__ void qmul(uint32_t& xl, uint32_t& xh, uint32_t yl, uint32_t yh, const Mult& m) {
  uint32_t s[6];
  selectors(yl, yh, s);
  qplane(xl, s, m.v[0], m.v[1], m.v[2], m.v[3], m.s[1], m.s[3], m.s[4], m.s[6], m.s[8], m.s[9]);
  qplane(xh, s, m.v[4], m.v[5], m.v[6], m.v[7], m.s[11], m.s[13], m.s[14], m.s[16], m.s[18], m.s[19]);
}

// (ol, oh) = c*y.
__device__ __forceinline__ void qmul_set(uint32_t& ol, uint32_t& oh, uint32_t yl, uint32_t yh, const Mult& m) {
  ol = 0;
  oh = 0;
  qmul(ol, oh, yl, yh, m);
}

typedef const __attribute__((address_space(4))) uint32_t* cpool_t;

// Multiplier tables of the additive element c via the scalar cache (c is
// wave-uniform, so this is s_load).
__device__ __forceinline__ void pool_of(const DevTables& T, uint32_t c, uint32_t (&p)[20]) {
  // opaque index: two fetches of the same table (e.g. beta, or the index-0
  // skews shared by an IFFT and an FFT) must not be merged into one long-lived value
  asm volatile("" : "+s"(c));
  const cpool_t q = (cpool_t)(T.perm_pools) + c * kPoolWords;
#pragma unroll
  for (int i = 0; i < 20; ++i) p[i] = q[i];
}

__device__ __forceinline__ uint32_t uniform(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

// A wave-uniform value the compiler must treat as new here: stops common
// subexpressions (row offsets, table indices) of different phases from being
// merged into values that stay live in SGPRs across the whole kernel.
__device__ __forceinline__ uint32_t fresh_v(uint32_t v) {  // same for a per-lane value
  asm volatile("" : "+v"(v));
  return v;
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
  if (full) return *reinterpret_cast<const uint2*>(rowp + 8u * lane);
  uint32_t w[2] = {0, 0};
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (4 * lane + i < ncols)
      w[i >> 1] |= static_cast<uint32_t>(*reinterpret_cast<const uint16_t*>(rowp + 8u * lane + 2 * i)) << (16 * (i & 1));
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
    for (int p = 0; p < NR; ++p) raw[p] = *reinterpret_cast<const uint2*>(src[p] + 8u * lane);
  } else {
#pragma unroll
    for (int p = 0; p < NR; ++p) raw[p] = load4(src[p], lane, ncols, false);
  }
}

// Shard rows row0..row0+15 (those below wanted_n) from cq registers.
__device__ __forceinline__ void store_rows(uint8_t* out, size_t shard_len, uint32_t row0, uint32_t wanted_n,
                                           const uint32_t (&L)[16], const uint32_t (&H)[16], uint32_t lane,
                                           uint32_t ncols, bool full) {
  if (full && row0 + 16 <= wanted_n) {
#pragma unroll
    for (int p = 0; p < 16; ++p)
      *reinterpret_cast<uint2*>(out + static_cast<size_t>(row0 + p) * shard_len + 8u * lane) = cq_row(L[p], H[p]);
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
// b is g * (8 >> b) + (p >> (b + 1)).
template <bool INVERSE, bool INDEX0>
__device__ __forceinline__ void cq_levels(const DevTables& T, uint32_t index, uint32_t g, uint32_t (&L)[16],
                                          uint32_t (&H)[16]) {
  auto cval = [&](auto fc) __attribute__((always_inline)) {
    constexpr GroupRef r = cq_group<INVERSE>(decltype(fc)::value);
    return 2u * (g * (8u >> r.b) + r.t) + (index >> r.b);
  };
  auto group = [&](auto fc, const Mult& p) __attribute__((always_inline)) {
    constexpr GroupRef r = cq_group<INVERSE>(decltype(fc)::value);
    constexpr int d = 1 << r.b;
    const bool live = !INDEX0 || r.t != 0 || g != 0;  // c == 0: the skew sentinel, no product
#pragma unroll
    for (int u = 0; u < d; ++u) {
      const int x = r.t * 2 * d + u, y = x + d;
      if (INVERSE) {
        L[y] ^= L[x];
        H[y] ^= H[x];
        if (live) qmul(L[x], H[x], L[y], H[y], p);
      } else {
        if (live) qmul(L[x], H[x], L[y], H[y], p);
        L[y] ^= L[x];
        H[y] ^= H[x];
      }
    }
  };
  pipelined<15>(T, cval, group);
}

// Levels 4..logK-1 in the high layout: quad j pairs with j + 2^(b-2-logR);
// group t = j >> (b-1-logR).
template <int K, bool INVERSE, bool INDEX0>
__device__ __forceinline__ void hi_levels(const DevTables& T, uint32_t index, uint32_t (&L)[16], uint32_t (&H)[16]) {
  constexpr int logR = Geo<K>::kLogR;
  auto cval = [&](auto fc) __attribute__((always_inline)) {
    constexpr GroupRef r = hi_group<K, INVERSE>(decltype(fc)::value);
    return 2u * r.t + (index >> r.b);
  };
  auto group = [&](auto fc, const Mult& p) __attribute__((always_inline)) {
    constexpr GroupRef r = hi_group<K, INVERSE>(decltype(fc)::value);
    constexpr int dj = 1 << (r.b - 2 - logR);
    constexpr bool live = !INDEX0 || r.t != 0;
#pragma unroll
    for (int u = 0; u < dj; ++u) {
      const int x = r.t * 2 * dj + u, y = x + dj;
      if (INVERSE) {
        L[y] ^= L[x];
        H[y] ^= H[x];
        if (live) qmul(L[x], H[x], L[y], H[y], p);
      } else {
        if (live) qmul(L[x], H[x], L[y], H[y], p);
        L[y] ^= L[x];
        H[y] ^= H[x];
      }
    }
  };
  pipelined<hi_groups<K>()>(T, cval, group);
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

// ---------------------------------------------------------- LDS sweeps ----
template <int K>
__device__ __forceinline__ void cq_read(const uint8_t* tile, uint32_t base, uint32_t (&L)[16], uint32_t (&H)[16]) {
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    uint2 d[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      d[i] = *reinterpret_cast<const uint2*>(tile + (base ^ (col_base_c<K>(i) ^ (8u * u))));
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

// ----------------------------------------------------------------- encode ----
// One workgroup: 256 chunks of one payload.  mod.rs:144-154 / inc_encode.rs:15-48.
template <int K>
__global__ __launch_bounds__(4 * K) __attribute__((amdgpu_waves_per_eu(4))) void k_encode_fast(DevTables T, EncodeArgs a, uint32_t nchunks, uint32_t tiles) {
  using G = Geo<K>;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* tile = smem;
  const uint32_t pb = blockIdx.x / tiles, tl = blockIdx.x - pb * tiles;
  const uint32_t ch0 = tl * kTile;
  const uint32_t ncols = min(static_cast<uint32_t>(kTile), nchunks - ch0);
  const uint8_t* pay = a.payloads + static_cast<size_t>(pb) * a.payload_stride;
  uint8_t* out = a.shards + static_cast<size_t>(pb) * a.batch_stride + 2 * static_cast<size_t>(ch0);
  const uint32_t tid = threadIdx.x, lane = tid & 63u, g = uniform(tid >> 6);
  const bool full =
      ncols == kTile && ((reinterpret_cast<uintptr_t>(a.shards) | a.batch_stride | a.shard_len) & 7u) == 0;

  // ---- tile load: thread tid moves blocks (c0 + 16 i, m0), i = 0..15
  {
    const uint32_t c0 = tid / G::Q, m0 = tid % G::Q;
    const uint32_t base = col_base<K>(c0) ^ (8u * m0);
    const size_t gbase = static_cast<size_t>(ch0 + c0) * 2 * K + 8u * m0;
    const bool fast = ((reinterpret_cast<uintptr_t>(pay) & 7u) == 0) &&
                      static_cast<size_t>(ch0 + kTile) * 2 * K <= a.payload_len;
    if (fast) {
      uint2 v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) v[i] = *reinterpret_cast<const uint2*>(pay + gbase + static_cast<size_t>(i) * 32 * K);
#pragma unroll
      for (int i = 0; i < 16; ++i) *reinterpret_cast<uint2*>(tile + (base ^ col_base_c<K>(16u * i))) = v[i];
    } else {
#pragma unroll 1
      for (uint32_t i = 0; i < 16; ++i) {
        const size_t g0 = gbase + static_cast<size_t>(i) * 32 * K;
        uint32_t w[2] = {0, 0};
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (g0 + e < a.payload_len) w[e >> 2] |= static_cast<uint32_t>(pay[g0 + e]) << (8 * (e & 3));
        *reinterpret_cast<uint2*>(tile + (base ^ col_base_c<K>(16u * i))) = make_uint2(w[0], w[1]);
      }
    }
  }
  __syncthreads();

  const uint32_t cqb = col_base<K>(4 * lane) ^ (32u * g);  // blocks 4g..4g+3 of columns 4l..4l+3
  // ---- cq pass: systematic rows, inverse levels 0..3
  {
    uint32_t CL[16], CH[16];
    cq_read<K>(tile, cqb, CL, CH);
    store_rows(out, a.shard_len, 16 * g, a.wanted_n, CL, CH, lane, ncols, full);
    cq_levels<true, true>(T, 0, g, CL, CH);
    cq_write<K>(tile, cqb, CL, CH);
  }
  __syncthreads();
  // ---- high layout: inverse levels 4.. -> coefficients M
  const uint32_t hb = col_base<K>(tid / G::R) ^ (8u * (tid % G::R));
  uint32_t ML[16], MH[16];
  hi_read<K>(tile, hb, ML, MH);
  hi_levels<K, true, true>(T, 0, ML, MH);
#pragma unroll
  for (int q = 0; q < 16; ++q) asm volatile("" : "+v"(ML[q]), "+v"(MH[q]));  // materialise M once

  const uint32_t nshift = a.n / K;
  for (uint32_t sh = 1; sh < nshift; ++sh) {
    const uint32_t index = sh * K;
    if (index >= a.wanted_n) break;
    uint32_t XL[16], XH[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      XL[q] = ML[q];
      XH[q] = MH[q];
    }
    hi_levels<K, false, false>(T, index, XL, XH);
    __syncthreads();  // the previous cq pass is done with the tile
    hi_write<K>(tile, fresh_v(hb), XL, XH);
    __syncthreads();
    cq_read<K>(tile, fresh_v(cqb), XL, XH);
    cq_levels<false, false>(T, index, g, XL, XH);
    store_rows(out, a.shard_len, index + 16 * g, a.wanted_n, XL, XH, lane, ncols, full);
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
template <int N, int NT>
__device__ __forceinline__ void fused_locator(const DevTables& T, const uint8_t* pres, uint32_t* W, uint16_t* E,
                                              uint8_t* PR) {
  const uint32_t tid = threadIdx.x;
  for (uint32_t v = tid; v < N; v += NT) {
    const uint8_t p = pres[v];
    PR[v] = p;
    W[v] = p ? 0u : 1u;
  }
  __syncthreads();
  for (uint32_t h = 1; h < N; h <<= 1) {  // integer WHT of the 0/1 erasure vector
    for (uint32_t b = tid; b < N / 2; b += NT) {
      const uint32_t i = (b / h) * 2 * h + (b % h), j = i + h;
      const int32_t x = static_cast<int32_t>(W[i]), y = static_cast<int32_t>(W[j]);
      W[i] = static_cast<uint32_t>(x + y);
      W[j] = static_cast<uint32_t>(x - y);
    }
    __syncthreads();
  }
  const uint16_t* F = T.lw_fold + N;
  for (uint32_t v = tid; v < N; v += NT) {
    const int32_t x = static_cast<int32_t>(W[v]);  // |x| <= N
    const uint32_t m = x < 0 ? static_cast<uint32_t>(x + 65535) : static_cast<uint32_t>(x);
    W[v] = (m * static_cast<uint32_t>(F[v])) % 65535u;
  }
  __syncthreads();
  for (uint32_t h = 1; h < N; h <<= 1) {  // WHT mod 65535
    for (uint32_t b = tid; b < N / 2; b += NT) {
      const uint32_t i = (b / h) * 2 * h + (b % h), j = i + h;
      const uint32_t x = W[i], y = W[j];
      uint32_t s = x + y, d = x + 65535u - y;
      s -= s >= 65535u ? 65535u : 0u;
      d -= d >= 65535u ? 65535u : 0u;
      W[i] = s;
      W[j] = d;
    }
    __syncthreads();
  }
  for (uint32_t v = tid; v < N; v += NT) E[v] = T.exp[PR[v] ? W[v] : 65535u - W[v]];
}

// ------------------------------------------------------------ reconstruct ----
struct RecCtx {
  const DevTables& T;
  size_t shard_len;
  uint8_t* tile;
  const uint16_t* E;
  const uint8_t* PR;
  const uint8_t* sh;
  uint32_t g, lane, tid, ncols;
  bool full;
  uint32_t cqb, hb;
};

// Step STEP of the segment sweep (segments 2, 3, 1, 0 for NQ = 4; 1, 0 for
// NQ = 2): x_q = IFFT(K, qK)(premultiplied segment q), folded into A.
template <int K, int NQ, int STEP>
__device__ __forceinline__ void rec_segment(const RecCtx& c, uint32_t (&AL)[16], uint32_t (&AH)[16]) {
  constexpr int q = NQ == 4 ? (STEP == 0 ? 2 : STEP == 1 ? 3 : 3 - STEP) : 1 - STEP;
  constexpr uint32_t index = static_cast<uint32_t>(q) * K;
  const DevTables& T = c.T;
  __builtin_amdgcn_sched_barrier(0);
  const uint32_t g = fresh(c.g);
  const uint8_t* sh = fresh(c.sh);
  const uint16_t* E = fresh(c.E);
  const uint8_t* PR = fresh(c.PR);
  const size_t shard_len = fresh(c.shard_len);
  const uint32_t cqb = fresh_v(c.cqb), hb = fresh_v(c.hb);
  uint32_t XL[16], XH[16];
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    uint2 raw[8];
    load_rows<8>(raw, sh, shard_len, PR, index + 16 * g + 8 * half, T.zeros, c.lane, c.ncols, c.full);
    pipelined<8>(
        T, [&](auto pc) __attribute__((always_inline)) { return uniform(E[index + 16 * g + 8 * half + decltype(pc)::value]); },
        [&](auto pc, const Mult& pool) __attribute__((always_inline)) {
          constexpr int p = decltype(pc)::value;
          const int x = 8 * half + p;
          XL[x] = 0;  // absent rows contribute zero
          XH[x] = 0;
          if (uniform(PR[index + 16 * g + x])) {
            uint32_t l, h;
            blk_to_quad(raw[p], l, h);
            qmul_set(XL[x], XH[x], l, h, pool);
          }
        });
  }
  cq_levels<true, q == 0>(T, index, g, XL, XH);
  if (STEP > 0) __syncthreads();  // the previous high pass is done with the tile
  cq_write<K>(c.tile, cqb, XL, XH);
  __syncthreads();
  hi_read<K>(c.tile, hb, XL, XH);
  hi_levels<K, true, q == 0>(T, index, XL, XH);
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (STEP == 0) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      AL[j] = XL[j];
      AH[j] = XH[j];
    }
  } else if constexpr (q == 0) {
    if constexpr (NQ == 2) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        AL[j] ^= XL[j];
        AH[j] ^= XH[j];
      }
    }
    add_derivative<K>(AL, XL, c.tid % Geo<K>::R);
    add_derivative<K>(AH, XH, c.tid % Geo<K>::R);
  } else if constexpr (NQ == 4 && q == 3) {
    uint32_t beta[20];
    pool_of(T, 2u, beta);  // beta = Cantor(2), the t = 1 skew of level logK at index 0
    const Mult pool = make_mult(beta);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      XL[j] ^= AL[j];
      XH[j] ^= AH[j];
      qmul(AL[j], AH[j], XL[j], XH[j], pool);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      AL[j] ^= XL[j];
      AH[j] ^= XH[j];
    }
  }
  __builtin_amdgcn_sched_barrier(0);
}


// One workgroup: 256 symbol columns of one batch entry.  NQ = n / K segments.
// The inverse transform of size n is NQ inverse transforms of size K (index
// qK) followed by log2(NQ) top levels whose skews at index 0 are 0 (t = 0) or
// beta = Cantor(2) (t = 1).  Only the first k = K outputs are needed; for them
//   NQ = 2:  d = D_K(x0) ^ x0 ^ x1
//   NQ = 4:  d = D_K(x0) ^ x1 ^ x2 ^ beta * (x2 ^ x3)
// where x_q = IFFT(K, qK)(premultiplied segment q) and D_K is the formal
// derivative of size K; then out = FFT(K, 0)(d) (the size-n forward transform
// restricted to its first K outputs is FFT(K, 0): its t = 0 skews are 0).
template <int K, int NQ>
__global__ __launch_bounds__(4 * K) __attribute__((amdgpu_waves_per_eu(4))) void k_reconstruct_fast(DevTables T, ReconstructArgs a, uint32_t nsyms,
                                                            uint32_t tiles) {
  using G = Geo<K>;
  constexpr int N = NQ * K;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* tile = smem;
  uint16_t* E = reinterpret_cast<uint16_t*>(smem + G::kTileBytes);  // multiplier element of every row
  uint8_t* PR = smem + G::kTileBytes + 2 * N;                        // present flags
  const uint32_t pb = blockIdx.x / tiles, tl = blockIdx.x - pb * tiles;
  const uint32_t col0 = tl * kTile;
  const uint32_t ncols = min(static_cast<uint32_t>(kTile), nsyms - col0);
  const uint8_t* sh = a.shards + static_cast<size_t>(pb) * a.batch_stride + 2 * static_cast<size_t>(col0);
  const uint8_t* pres = a.present + static_cast<size_t>(pb) * N;
  const uint16_t* loc = a.locators + static_cast<size_t>(pb) * N;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, g = uniform(tid >> 6);
  const bool full =
      ncols == kTile && ((reinterpret_cast<uintptr_t>(a.shards) | a.batch_stride | a.shard_len) & 7u) == 0;

  if (loc) {
    for (uint32_t v = tid; v < static_cast<uint32_t>(N); v += G::kThreads) {
      E[v] = T.exp[loc[v]];  // mul(x, log m) == x * EXP[m] (inc_log_mul.rs:42-49)
      PR[v] = pres[v];
    }
  } else {
    fused_locator<N, G::kThreads>(T, pres, reinterpret_cast<uint32_t*>(tile), E, PR);
  }
  __syncthreads();

  const uint32_t cqb = col_base<K>(4 * lane) ^ (32u * g);
  const uint32_t hb = col_base<K>(tid / G::R) ^ (8u * (tid % G::R));
  uint32_t AL[16], AH[16];

  // segment order: 2, 3, 1, 0 (NQ = 4) or 1, 0 (NQ = 2)
  RecCtx c{T, a.shard_len, tile, E, PR, sh, g, lane, tid, ncols, full, cqb, hb};
  rec_segment<K, NQ, 0>(c, AL, AH);
  rec_segment<K, NQ, 1>(c, AL, AH);
  if constexpr (NQ == 4) {
    rec_segment<K, NQ, 2>(c, AL, AH);
    rec_segment<K, NQ, 3>(c, AL, AH);
  }
  // ---- forward transform of size K at index 0, then postmultiply erased rows
  hi_levels<K, false, true>(T, 0, AL, AH);
  __syncthreads();
  hi_write<K>(tile, fresh_v(hb), AL, AH);
  __syncthreads();
  {
    const uint32_t cqbf = fresh_v(cqb);
    uint32_t XL[16], XH[16];
    cq_read<K>(tile, cqbf, XL, XH);
    cq_levels<false, true>(T, 0, g, XL, XH);
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      uint2 raw[8];
      load_rows<8>(raw, sh, a.shard_len, PR, 16 * g + 8 * half, T.zeros, lane, ncols, full);
      pipelined<8>(
          T, [&](auto pc) __attribute__((always_inline)) { return uniform(E[16 * g + 8 * half + decltype(pc)::value]); },
          [&](auto pc, const Mult& pool) __attribute__((always_inline)) {
            constexpr int p = decltype(pc)::value;
            const int x = 8 * half + p;
            // present: the received symbol (mod.rs:225-235); erased: the
            // postmultiplied recovered symbol (inc_reconstruct.rs:76-84)
            if (uniform(PR[16 * g + x])) {
              blk_to_quad(raw[p], XL[x], XH[x]);
            } else {
              const uint32_t l = XL[x], h = XH[x];
              qmul_set(XL[x], XH[x], l, h, pool);
            }
          });
    }
    __syncthreads();
    cq_write<K>(tile, cqbf, XL, XH);
  }
  __syncthreads();
  // ---- copy-out: column c of the tile is 2K contiguous bytes of the output
  {
    uint8_t* out = a.out + static_cast<size_t>(pb) * a.out_stride + static_cast<size_t>(col0) * 2 * K;
    const bool al_o = ((reinterpret_cast<uintptr_t>(a.out) | a.out_stride) & 7u) == 0;
    const uint32_t c0 = tid / G::Q, m0 = tid % G::Q;
    const uint32_t base = col_base<K>(c0) ^ (8u * m0);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint32_t c = c0 + 16u * i;
      if (c >= ncols) break;
      const uint2 v = *reinterpret_cast<const uint2*>(tile + (base ^ col_base_c<K>(16u * i)));
      uint8_t* o = out + static_cast<size_t>(c) * 2 * K + 8u * m0;
      if (al_o) {
        *reinterpret_cast<uint2*>(o) = v;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = static_cast<uint8_t>((e < 4 ? v.x : v.y) >> (8 * (e & 3)));
      }
    }
  }
}

// ------------------------------------------------------------- launchers ----
template <int K>
size_t encode_lds_bytes() {
  return static_cast<size_t>(Geo<K>::kTileBytes);
}

template <int K, int NQ>
size_t reconstruct_lds_bytes() {
  return static_cast<size_t>(Geo<K>::kTileBytes) + 3u * NQ * K;
}

template <int K>
hipError_t launch_encode_k(const DevTables& T, const EncodeArgs& a, hipStream_t s) {
  const size_t nchunks = (a.payload_len + 2 * a.k - 1) / (2 * a.k);
  if (nchunks == 0 || a.batch == 0) return hipSuccess;
  const uint32_t tiles = static_cast<uint32_t>((nchunks + kTile - 1) / kTile);
  const size_t blocks = a.batch * tiles;
  if (blocks > 0x7fffffffu || nchunks > 0xffffffffu) return hipErrorInvalidValue;
  k_encode_fast<K><<<static_cast<uint32_t>(blocks), Geo<K>::kThreads, encode_lds_bytes<K>(), s>>>(
      T, a, static_cast<uint32_t>(nchunks), tiles);
  return hipGetLastError();
}

template <int K, int NQ>
hipError_t launch_reconstruct_k(const DevTables& T, const ReconstructArgs& a, hipStream_t s) {
  const size_t nsyms = a.shard_len / 2;
  if (nsyms == 0 || a.batch == 0) return hipSuccess;
  const uint32_t tiles = static_cast<uint32_t>((nsyms + kTile - 1) / kTile);
  const size_t blocks = a.batch * tiles;
  if (blocks > 0x7fffffffu || nsyms > 0xffffffffu) return hipErrorInvalidValue;
  k_reconstruct_fast<K, NQ><<<static_cast<uint32_t>(blocks), Geo<K>::kThreads, reconstruct_lds_bytes<K, NQ>(), s>>>(
      T, a, static_cast<uint32_t>(nsyms), tiles);
  return hipGetLastError();
}

}  // namespace

bool fast_encode_supported(uint32_t n, uint32_t k) {
  return (k == 64 || k == 128 || k == 256) && n >= 2 * k && n <= 65536;
}

bool fast_reconstruct_supported(uint32_t n, uint32_t k) {
  return (k == 64 || k == 128 || k == 256) && (n == 2 * k || n == 4 * k);
}

hipError_t launch_encode_fast(const DevTables& T, const EncodeArgs& a, hipStream_t s) {
  switch (a.k) {
    case 64: return launch_encode_k<64>(T, a, s);
    case 128: return launch_encode_k<128>(T, a, s);
    case 256: return launch_encode_k<256>(T, a, s);
    default: return hipErrorNotSupported;
  }
}

hipError_t launch_reconstruct_fast(const DevTables& T, const ReconstructArgs& a, hipStream_t s) {
  const bool q4 = a.n == 4 * a.k;
  switch (a.k) {
    case 64: return q4 ? launch_reconstruct_k<64, 4>(T, a, s) : launch_reconstruct_k<64, 2>(T, a, s);
    case 128: return q4 ? launch_reconstruct_k<128, 4>(T, a, s) : launch_reconstruct_k<128, 2>(T, a, s);
    case 256: return q4 ? launch_reconstruct_k<256, 4>(T, a, s) : launch_reconstruct_k<256, 2>(T, a, s);
    default: return hipErrorNotSupported;
  }
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
  set(reinterpret_cast<const void*>(&k_reconstruct_fast<64, 2>), reconstruct_lds_bytes<64, 2>());
  set(reinterpret_cast<const void*>(&k_reconstruct_fast<64, 4>), reconstruct_lds_bytes<64, 4>());
  set(reinterpret_cast<const void*>(&k_reconstruct_fast<128, 2>), reconstruct_lds_bytes<128, 2>());
  set(reinterpret_cast<const void*>(&k_reconstruct_fast<128, 4>), reconstruct_lds_bytes<128, 4>());
  set(reinterpret_cast<const void*>(&k_reconstruct_fast<256, 2>), reconstruct_lds_bytes<256, 2>());
  set(reinterpret_cast<const void*>(&k_reconstruct_fast<256, 4>), reconstruct_lds_bytes<256, 4>());
  return e;
}

}  // namespace np
