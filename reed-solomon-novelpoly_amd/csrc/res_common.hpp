#pragma once
// Shared building blocks of the resident kernels (kernels_res.hip: k = 512 /
// 1024; kernels_huge.hip: k = 2048 .. 16384 as size-1024 sub-transforms):
// tile geometry and LDS swizzle, the CQ / HA / HD register layouts and their
// levels, per-lane multiplies, the formal derivative, shard-row I/O, row
// tables and the copy-out.  Included by those two translation units only
// (everything is in an anonymous namespace).
//
// k = 1024 (BASELINE config 4: n = 4096; 2,731-5,461 validators at n = 4096 /
// 8,192) and k = 512 (1,534-3,070 validators: n = 2048 / 4096, the reference's
// own 2,000-validator bench shape) with the whole size-K transform of a tile
// resident in one workgroup: no scratch round trips.
//
// A tile is 64 codeword columns (encode: 64 payload chunks of 2K bytes;
// decode: 64 symbol columns of the shards) x K positions = 128 KiB (K = 1024)
// or 64 KiB (K = 512, two workgroups per CU), the LDS tile.  The K threads
// (K / 64 waves) hold the tile in registers, 64 symbols each, in three layouts
// that meet in the LDS tile (written for K = 1024, position p = bits p0..p9,
// block m = p >> 2, column c < 64; K = 512 where it differs):
//
//  * CQ (levels 0-3; the shard rows): wave w, lane 16u + cq holds positions
//    P_i = 64 w + 16 u + i (i = 0..15) of columns 4 cq .. 4 cq + 3, byte-planar
//    quads L[i] / H[i] (fast_common.hpp's column-quad layout).  Shard rows are
//    read and written from here (8 bytes per lane and row).
//  * HA (levels 4-7): wave w, lane = column c holds the position quads
//    m = (w & 3) + 4 j + 64 (w >> 2), j = 0..15 (position bits 4-7 in j).
//  * HD (levels 8-9, the decode's formal derivative): wave w, lane l holds
//    column 4 w + (l >> 4), quads m = (l & 15) + 16 j (position bits 2-5 in the
//    16 lanes of a DPP row, bits 6-9 in j).  K = 512 (level 8): column
//    8 w + (l >> 3), quads (l & 7) + 8 j (bits 2-4 in 8 lanes, 5-8 in j).
//
// HA and HD see whole butterfly groups per register, so their multipliers are
// wave-uniform (s_load tables, as in the fast kernels).  In CQ the lane's
// position bits 4-5 (u) are part of the group index: the skew of group
// T = p >> (b + 1) at level b <= 3 is Cantor(2T + (I >> b)), and by the
// linearity of Cantor coordinates it splits into a wave-uniform element
// c_w = Cantor(w << (6 - b) | 2 (i >> (b + 1)) | I >> b) and a per-lane
// element delta = Cantor(u << (4 - b)) < 64, in GF(2^8).  Subfield levels
// multiply by (c_w + delta) through per-lane tables (the XOR of the two
// elements' tables: every table entry is linear in the multiplier); levels
// with full multipliers add delta * y to c_w * y, sharing the selectors.
//
// The LDS tile holds 8-byte position-quad items (column c, block m) at
// 2048 c + 8 (m ^ rsw(c)), rsw a linear swizzle (conflict-free for the CQ, HA
// and HD sweeps, see rsw).  The payload tile arrives there as natural blocks;
// the exchanges between layouts use planar items (low bytes, high bytes of
// the 4 positions), so only the CQ side transposes (tr4x4).
//
// Reference: inc_afft.rs:139-214 / :267-332 (transforms), inc_encode.rs:15-48
// and mod.rs:117-157 (encode), inc_reconstruct.rs:1-113 and mod.rs:162-239
// (reconstruct).  Decode algebra (the fold of the size-n transforms into
// size-K ones, kappa, D_K): kernels_fast.hip, DESIGN.md §4.3.


#include <algorithm>
#include <cstdlib>
#include <utility>

#include "fast_common.hpp"

namespace np {
namespace {


constexpr int kRC = 64;  // columns per tile
// Geometry of the size-K kernels (K = 512, 1024): K threads, K / 64 waves.
template <int K>
struct RGeo {
  static_assert(K == 256 || K == 512 || K == 1024, "resident kernels: k = 256 (decode A/B), 512 or 1024");
  static constexpr int kThreads = K;
  static constexpr uint32_t kTileBytes = kRC * 2 * K;  // 128 / 64 KiB
  static constexpr uint32_t kColBytes = 2 * K;
  static constexpr uint32_t kLPC = K / 64;  // HD: lanes per column
  static constexpr uint32_t kHD = 8 * kLPC;  // HD: item j at hdb ^ kHD j
  static constexpr int kLogK = K == 1024 ? 10 : K == 512 ? 9 : 8;
};

// ------------------------------------------------------------- LDS tile ----
// Swizzle of the block index by the column, linear in the bits of c.  K = 1024:
// c0 -> 24, c1 -> 4, c2 -> 1, c3 -> 2, c4 -> 20, c5 -> 8.  Conflict-free for
// ds_read_b64 (32-lane groups, bank (a / 4) mod 64) and ds_write_b64 (16-lane
// groups, bank (a / 4) mod 32) in the three sweeps:
//  HA: 32 consecutive columns at one block (rank {v0..v4} = 5), and 16 of
//      them for writes (rank {v0..v3} mod 16 = 4);
//  HD: 16 consecutive blocks of columns c, c + 1 (v0 has bit 4);
//  CQ: columns 4 cq + e over cq < 16 with block bit 2 (u) (rank {v2..v5, 4} =
//      5; writes: rank {v2..v5} mod 16 = 4).
// K = 512 (HD: 8 blocks of columns c .. c + 3): c0 -> 28, c1 -> 14, c2 -> 1,
// c3 -> 25, c4 -> 20, c5 -> 27, found and checked over every sweep of both
// sizes (and the payload tile's writes) by tools/res_swizzle.py.  K = 256 (the
// decode A/B of DESIGN.md §8; HD: 4 blocks of columns c .. c + 7): c0 -> 24,
// c1 -> 4, c2 -> 14, c3 -> 5, c4 -> 17, c5 -> 23, by the same search.
template <int K>
__host__ __device__ constexpr uint32_t rsw(uint32_t c) {
  if constexpr (K == 1024)
    return ((c & 1u) ? 24u : 0u) ^ ((c & 2u) ? 4u : 0u) ^ ((c & 4u) ? 1u : 0u) ^ ((c & 8u) ? 2u : 0u) ^
           ((c & 16u) ? 20u : 0u) ^ ((c & 32u) ? 8u : 0u);
  else if constexpr (K == 512)
    return ((c & 1u) ? 28u : 0u) ^ ((c & 2u) ? 14u : 0u) ^ ((c & 4u) ? 1u : 0u) ^ ((c & 8u) ? 25u : 0u) ^
           ((c & 16u) ? 20u : 0u) ^ ((c & 32u) ? 27u : 0u);
  else
    return ((c & 1u) ? 24u : 0u) ^ ((c & 2u) ? 4u : 0u) ^ ((c & 4u) ? 14u : 0u) ^ ((c & 8u) ? 5u : 0u) ^
           ((c & 16u) ? 17u : 0u) ^ ((c & 32u) ? 23u : 0u);
}
template <int K>
__host__ __device__ constexpr uint32_t pq_addr(uint32_t c, uint32_t m) {
  return RGeo<K>::kColBytes * c + 8u * (m ^ rsw<K>(c));
}

// Per-thread coordinates of the three layouts.
struct Res {
  uint32_t tid, w, l;
  // CQ
  uint32_t cq, u, cqb;  // cqb: pq_addr(4 cq, 16 w + 4 u); item (e, q) at (cqb | 2K e) ^ 8 (q ^ rsw(e))
  // HA: item j at hab ^ 32 j
  uint32_t hab;
  // HD: item j at hdb ^ kHD j
  uint32_t hdb;
};

template <int K>
__device__ __forceinline__ Res res_coords() {
  constexpr uint32_t lpc = RGeo<K>::kLPC;
  Res r;
  r.tid = fresh_v(threadIdx.x);
  r.w = uniform(r.tid >> 6);
  r.l = r.tid & 63u;
  r.cq = r.l & 15u;
  r.u = r.l >> 4;
  r.cqb = pq_addr<K>(4u * r.cq, 16u * r.w + 4u * r.u);
  r.hab = pq_addr<K>(r.l, (r.w & 3u) + 64u * (r.w >> 2));
  r.hdb = pq_addr<K>((64u / lpc) * r.w + r.l / lpc, r.l % lpc);
  return r;
}

template <int K>
__device__ __forceinline__ uint32_t cq_item(uint32_t cqb, uint32_t e, uint32_t q) {
  return (cqb | (RGeo<K>::kColBytes * e)) ^ (8u * (q ^ rsw<K>(e)));
}

// CQ from natural blocks (the payload tile).
template <int K>
__device__ __forceinline__ void rcq_read_nat(const uint8_t* tile, uint32_t cqb, uint32_t (&L)[16], uint32_t (&H)[16]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint2 d[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) d[e] = *reinterpret_cast<const uint2*>(tile + cq_item<K>(cqb, e, q));
    blks_to_cq(d, &L[4 * q], &H[4 * q]);
  }
}

// CQ <-> planar items (4 x 4 byte transposes of each plane).
template <int K>
__device__ __forceinline__ void rcq_write(uint8_t* tile, uint32_t cqb, const uint32_t (&L)[16], const uint32_t (&H)[16]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t l[4], h[4];
    tr4x4(L[4 * q], L[4 * q + 1], L[4 * q + 2], L[4 * q + 3], l);
    tr4x4(H[4 * q], H[4 * q + 1], H[4 * q + 2], H[4 * q + 3], h);
#pragma unroll
    for (int e = 0; e < 4; ++e) *reinterpret_cast<uint2*>(tile + cq_item<K>(cqb, e, q)) = make_uint2(l[e], h[e]);
  }
}
template <int K>
__device__ __forceinline__ void rcq_read(const uint8_t* tile, uint32_t cqb, uint32_t (&L)[16], uint32_t (&H)[16]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint2 d[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) d[e] = *reinterpret_cast<const uint2*>(tile + cq_item<K>(cqb, e, q));
    tr4x4(d[0].x, d[1].x, d[2].x, d[3].x, &L[4 * q]);
    tr4x4(d[0].y, d[1].y, d[2].y, d[3].y, &H[4 * q]);
  }
}

template <int STEP>
__device__ __forceinline__ void rh_write(uint8_t* tile, uint32_t base, const uint32_t (&L)[16], const uint32_t (&H)[16]) {
#pragma unroll
  for (int j = 0; j < 16; ++j) *reinterpret_cast<uint2*>(tile + (base ^ (STEP * j))) = make_uint2(L[j], H[j]);
}
template <int STEP>
__device__ __forceinline__ void rh_read(const uint8_t* tile, uint32_t base, uint32_t (&L)[16], uint32_t (&H)[16]) {
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint2 d = *reinterpret_cast<const uint2*>(tile + (base ^ (STEP * j)));
    L[j] = d.x;
    H[j] = d.y;
  }
}
constexpr int kHA = 32;  // HA: item j at hab ^ 32 j (block + 4 j)

// ------------------------------------------------------ per-lane multiply ----
// One output plane of c*y with all table dwords per lane (VGPRs): the subfield
// layout (field_tables.hpp kSubV / kSubS): t[0], t[1] entries 0-3 of the
// bit 0-2 / 3-5 tables, t[2], t[3] their entries 4-7, t[4] the bit 6-7 table
// (both byte planes use the same tables: e_i = 2^i, field_tables.cpp).
struct SubT {
  uint32_t t[5];
};
__device__ __forceinline__ void qplane_sub_vv(uint32_t& acc, uint32_t s0, uint32_t s1, uint32_t s2, const SubT& m) {
  uint32_t t0, t1, t2;
  asm volatile(
      "v_perm_b32 %[t0], %[a2], %[a0], %[s0]\n\t"
      "v_perm_b32 %[t1], %[a3], %[a1], %[s1]\n\t"
      "v_perm_b32 %[t2], %[a4], %[a4], %[s2]\n\t"
      "v_bitop3_b32 %[acc], %[acc], %[t0], %[t1] bitop3:0x96\n\t"
      "v_xor_b32 %[acc], %[acc], %[t2]"
      : [acc] "+v"(acc), [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2)
      : [s0] "v"(s0), [s1] "v"(s1), [s2] "v"(s2), [a0] "v"(m.t[0]), [a1] "v"(m.t[1]), [a2] "v"(m.t[2]),
        [a3] "v"(m.t[3]), [a4] "v"(m.t[4]));
}
__device__ __forceinline__ void qmul_sub_vv(uint32_t& xl, uint32_t& xh, uint32_t yl, uint32_t yh, const SubT& m) {
  uint32_t s[6];
  selectors(yl, yh, s);
  qplane_sub_vv(xl, s[0], s[1], s[2], m);
  qplane_sub_vv(xh, s[3], s[4], s[5], m);
}
// x ^= c_w*y ^ d*y: c_w a full multiplier (SGPR / VGPR halves), d a per-lane
// subfield one; the selectors of y serve both.
__device__ __forceinline__ void qmul_full_d(uint32_t& xl, uint32_t& xh, uint32_t yl, uint32_t yh, const Mult& m,
                                            const SubT& d) {
  uint32_t s[6];
  selectors(yl, yh, s);
  qplane(xl, s, m.v[0], m.v[1], m.v[2], m.v[3], m.s[0], m.s[1], m.s[2], m.s[3], m.s[4], m.s[5]);
  qplane(xh, s, m.v[4], m.v[5], m.v[6], m.v[7], m.s[6], m.s[7], m.s[8], m.s[9], m.s[10], m.s[11]);
  qplane_sub_vv(xl, s[0], s[1], s[2], d);
  qplane_sub_vv(xh, s[3], s[4], s[5], d);
}

// One output plane of c*y (written, not accumulated) with all 20 full-map
// table dwords per lane (pool layout field_tables.cpp build_pool: p[0..7] the
// VGPR half, p[8..19] the SGPR half).
__device__ __forceinline__ void qplane_set_vv(uint32_t& out, const uint32_t (&s)[6], uint32_t va, uint32_t vb,
                                              uint32_t vc, uint32_t vd, uint32_t sa, uint32_t sb, uint32_t sc,
                                              uint32_t sd, uint32_t se, uint32_t sf) {
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
        [va] "v"(va), [vb] "v"(vb), [vc] "v"(vc), [vd] "v"(vd), [sa] "v"(sa), [sb] "v"(sb), [sc] "v"(sc),
        [sd] "v"(sd), [se] "v"(se), [sf] "v"(sf));
}
struct FullT {
  uint32_t p[20];
};
// (ol, oh) = c*y with a per-lane full table.
__device__ __forceinline__ void qmul_set_vv(uint32_t& ol, uint32_t& oh, uint32_t yl, uint32_t yh, const FullT& m) {
  uint32_t s[6];
  selectors(yl, yh, s);
  qplane_set_vv(ol, s, m.p[0], m.p[1], m.p[2], m.p[3], m.p[8], m.p[9], m.p[10], m.p[11], m.p[12], m.p[13]);
  qplane_set_vv(oh, s, m.p[4], m.p[5], m.p[6], m.p[7], m.p[14], m.p[15], m.p[16], m.p[17], m.p[18], m.p[19]);
}

// x ^= c*y with a per-lane full table (qmul_set_vv's accumulating form).
__device__ __forceinline__ void qplane_vv(uint32_t& acc, const uint32_t (&s)[6], uint32_t va, uint32_t vb,
                                          uint32_t vc, uint32_t vd, uint32_t sa, uint32_t sb, uint32_t sc,
                                          uint32_t sd, uint32_t se, uint32_t sf) {
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
        [va] "v"(va), [vb] "v"(vb), [vc] "v"(vc), [vd] "v"(vd), [sa] "v"(sa), [sb] "v"(sb), [sc] "v"(sc),
        [sd] "v"(sd), [se] "v"(se), [sf] "v"(sf));
}
__device__ __forceinline__ void qmul_vv(uint32_t& xl, uint32_t& xh, uint32_t yl, uint32_t yh, const FullT& m) {
  uint32_t s[6];
  selectors(yl, yh, s);
  qplane_vv(xl, s, m.p[0], m.p[1], m.p[2], m.p[3], m.p[8], m.p[9], m.p[10], m.p[11], m.p[12], m.p[13]);
  qplane_vv(xh, s, m.p[4], m.p[5], m.p[6], m.p[7], m.p[14], m.p[15], m.p[16], m.p[17], m.p[18], m.p[19]);
}

// Full-layout tables of the per-lane deltas Cantor(u << (4 - b)), b, u < 4
// (tower_full_sub), staged once per kernel for the full CQ levels b >= 1:
// table (b, u) at DL + 20 (4 b + u).  Caller synchronises.
constexpr uint32_t kDeltaWords = 16u * kPoolWords;
__device__ __forceinline__ void stage_delta_tables(const DevTables& T, uint32_t* DL) {
  const uint32_t i = threadIdx.x;
  if (i < kDeltaWords / 4u) {
    const uint32_t slot = i / 5u, part = i % 5u, b = slot >> 2, u = slot & 3u;
    *reinterpret_cast<uint4*>(DL + kPoolWords * slot + 4u * part) = *reinterpret_cast<const uint4*>(
        T.tower_full_sub + static_cast<size_t>(u << (4 - b)) * kPoolWords + 4u * part);
  }
}

// The per-lane part delta = Cantor(u << (4 - b)) of the CQ skews at level b:
// its subfield tables (tower_pools, sub layout).
__device__ __forceinline__ SubT delta_tables(const DevTables& T, uint32_t u, int b) {
  const uint32_t* p = T.tower_pools + static_cast<size_t>(u << (4 - b)) * kPoolWords;
  SubT d;
  d.t[0] = p[0];
  d.t[1] = p[1];
  d.t[2] = p[8];
  d.t[3] = p[9];
  d.t[4] = p[10];
  return d;
}

// ------------------------------------------------------------ transforms ----
// Levels b < res_gen(I) of a size-K transform at index I hold skews outside
// GF(2^8): Cantor(2T + (I >> b)) with 2T < 2^(logK - b) lies in GF(2^8) for
// every group exactly when ((I + K) >> b) <= 256.  (fast_common.hpp gen_of is
// the size-256 form of this rule.)  K = 1024: index 0: 2; 1024: 3; 2048, 3072:
// 4.  K = 512: 0: 1; 512: 2; 1024, 1536: 3; 2048-3584 (n = 4096): 4.
template <int K>
__host__ __device__ constexpr int res_gen(uint32_t I) {
  int b = 0;
  while (((I + static_cast<uint32_t>(K)) >> b) > 256u) ++b;
  return b;
}
static_assert(res_gen<1024>(0) == 2 && res_gen<1024>(1024) == 3 && res_gen<1024>(2048) == 4 &&
                  res_gen<1024>(3072) == 4,
              "res_gen");
static_assert(res_gen<1024>(4096) == 5 && res_gen<1024>(7168) == 5, "res_gen, n = 8192: level 4 (HA) full");
static_assert(res_gen<512>(0) == 1 && res_gen<512>(512) == 2 && res_gen<512>(1536) == 3 && res_gen<512>(2048) == 4 &&
                  res_gen<512>(3584) == 4,
              "res_gen, k = 512");

// CQ levels 0-3 of a size-1024 transform at index I.  GEN: levels b < GEN
// have full multipliers (gen_of(I), fast_common.hpp kSubLevel).  Group t of
// level b in this thread is registers t 2^(b+1) .. + 2^(b+1).
// ST (kernels_res.hip): full levels b >= 1 multiply by c_w + delta through a
// per-lane full table, the XOR of c_w's (s_load) and delta's (staged in LDS at
// dl, stage_delta_tables): 20 XORs per group instead of a delta multiply (10
// instructions) per butterfly and the 4 v_mov copies of c_w's VGPR half.
template <bool INVERSE, int GEN, int B, int TG, bool ST = false>
__device__ __forceinline__ void rcq_group(const DevTables& T, uint32_t I, uint32_t w, const SubT& dt,
                                          uint32_t (&L)[16], uint32_t (&H)[16], const uint32_t* dl = nullptr) {
  constexpr int d = 1 << B;
  // uniform element of group TG: Cantor(w << (6 - B) | 2 TG | I >> B)
  const uint32_t cw = (w << (6 - B)) + 2u * TG + (I >> B);
  __builtin_amdgcn_sched_barrier(0);
  if constexpr (B >= GEN) {  // subfield: per-lane table of cw + delta
    uint32_t sp[12];
    spool_of<true, true>(T, cw, sp);  // SGPR dwords 8..13 (entries 4-7, the bit 6-7 table)
    const cpool_t q = (cpool_t)(T.tower_pools) + cw * kPoolWords;
    SubT m;
    m.t[0] = q[0] ^ dt.t[0];
    m.t[1] = q[1] ^ dt.t[1];
    m.t[2] = sp[0] ^ dt.t[2];
    m.t[3] = sp[1] ^ dt.t[3];
    m.t[4] = sp[2] ^ dt.t[4];
#pragma unroll
    for (int v = 0; v < d; ++v) {
      const int x = TG * 2 * d + v, y = x + d;
      if constexpr (INVERSE) {
        L[y] ^= L[x];
        H[y] ^= H[x];
        qmul_sub_vv(L[x], H[x], L[y], H[y], m);
      } else {
        qmul_sub_vv(L[x], H[x], L[y], H[y], m);
        L[y] ^= L[x];
        H[y] ^= H[x];
      }
    }
  } else if constexpr (ST && B >= 1) {  // per-lane full table of c_w + delta
    const uint32_t c = fresh(cw);
    const cpool_t q = (cpool_t)(c < 256u ? T.tower_full_sub : T.tower_pools) + c * kPoolWords;
    FullT m;
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const uint4 d = *reinterpret_cast<const uint4*>(dl + 4 * i);
      m.p[4 * i] = q[4 * i] ^ d.x;
      m.p[4 * i + 1] = q[4 * i + 1] ^ d.y;
      m.p[4 * i + 2] = q[4 * i + 2] ^ d.z;
      m.p[4 * i + 3] = q[4 * i + 3] ^ d.w;
    }
#pragma unroll
    for (int v = 0; v < d; ++v) {
      const int x = TG * 2 * d + v, y = x + d;
      if constexpr (INVERSE) {
        L[y] ^= L[x];
        H[y] ^= H[x];
        qmul_vv(L[x], H[x], L[y], H[y], m);
      } else {
        qmul_vv(L[x], H[x], L[y], H[y], m);
        L[y] ^= L[x];
        H[y] ^= H[x];
      }
    }
  } else {  // full c_w (tower coordinates) plus the per-lane subfield delta
    // a level with full skews can hold subfield ones too (index 0, levels
    // 0-1, waves 0-3): their full-layout tables are in tower_full_sub
    uint32_t p[20];
    const uint32_t c = fresh(cw);
    const cpool_t q = (cpool_t)(c < 256u ? T.tower_full_sub : T.tower_pools) + c * kPoolWords;
#pragma unroll
    for (int i = 0; i < 20; ++i) p[i] = q[i];
    const Mult m = make_mult(p);
#pragma unroll
    for (int v = 0; v < d; ++v) {
      const int x = TG * 2 * d + v, y = x + d;
      if constexpr (INVERSE) {
        L[y] ^= L[x];
        H[y] ^= H[x];
        qmul_full_d(L[x], H[x], L[y], H[y], m, dt);
      } else {
        qmul_full_d(L[x], H[x], L[y], H[y], m, dt);
        L[y] ^= L[x];
        H[y] ^= H[x];
      }
    }
  }
  __builtin_amdgcn_sched_barrier(0);
}

template <bool INVERSE, int GEN, int B, bool ST, int... TG>
__device__ __forceinline__ void rcq_level(const DevTables& T, uint32_t I, uint32_t w, uint32_t u, uint32_t (&L)[16],
                                          uint32_t (&H)[16], const uint32_t* DL, std::integer_sequence<int, TG...>) {
  if constexpr (ST && B >= 1 && B < GEN) {
    const uint32_t* dl = DL + kPoolWords * (4u * B + u);
    const SubT dt{};
    (rcq_group<INVERSE, GEN, B, TG, true>(T, I, w, dt, L, H, dl), ...);
  } else {
    const SubT dt = delta_tables(T, u, B);
    (rcq_group<INVERSE, GEN, B, TG>(T, I, w, dt, L, H), ...);
  }
}

// Experiment builds (NP_EXP, never the product): bit 8 skips the CQ levels,
// bit 9 the HA levels, bit 10 the HD levels (tools/res_debug.py).
// PRIO: progress-based issue priority over the pass's four levels
// (fast_common.hpp progress_prio).
template <bool INVERSE, int GEN, bool ST = false, int PRIO = 0>
__device__ __forceinline__ void rcq_levels(const DevTables& T, uint32_t I, const Res& r, uint32_t (&L)[16],
                                           uint32_t (&H)[16], const uint32_t* DL = nullptr) {
  if constexpr (kExp & (1 | 256)) return;
  if constexpr (INVERSE ? (kExp & 4096) != 0 : (kExp & 2048) != 0) return;  // experiment: one direction only
  const uint32_t w = fresh(r.w), u = fresh_v(r.u);
  // progress in butterfly groups (8 + 4 + 2 + 1)
  if constexpr (INVERSE) {
    progress_prio<0, 15, PRIO>();
    rcq_level<true, GEN, 0, ST>(T, I, w, u, L, H, DL, std::make_integer_sequence<int, 8>{});
    progress_prio<8, 15, PRIO>();
    rcq_level<true, GEN, 1, ST>(T, I, w, u, L, H, DL, std::make_integer_sequence<int, 4>{});
    progress_prio<12, 15, PRIO>();
    rcq_level<true, GEN, 2, ST>(T, I, w, u, L, H, DL, std::make_integer_sequence<int, 2>{});
    rcq_level<true, GEN, 3, ST>(T, I, w, u, L, H, DL, std::make_integer_sequence<int, 1>{});
  } else {
    progress_prio<0, 15, PRIO>();
    rcq_level<false, GEN, 3, ST>(T, I, w, u, L, H, DL, std::make_integer_sequence<int, 1>{});
    rcq_level<false, GEN, 2, ST>(T, I, w, u, L, H, DL, std::make_integer_sequence<int, 2>{});
    progress_prio<3, 15, PRIO>();
    rcq_level<false, GEN, 1, ST>(T, I, w, u, L, H, DL, std::make_integer_sequence<int, 4>{});
    progress_prio<7, 15, PRIO>();
    rcq_level<false, GEN, 0, ST>(T, I, w, u, L, H, DL, std::make_integer_sequence<int, 8>{});
  }
}

// Software-pipelined multiplier fetch over tower_pools (fast_common.hpp
// pipelined() reads perm_pools): group f + 1's tables are requested before
// group f runs.
template <int F, int NG, typename CF, typename GF>
__device__ __forceinline__ void tpipe_step(const DevTables& T, CF& cval, GF& group, uint32_t (&cur)[20],
                                           uint32_t (&nxt)[20]) {
  if constexpr (F < NG) {
    if constexpr (F + 1 < NG) pool_of<true>(T, cval(Int<F + 1>{}), nxt);
    __builtin_amdgcn_sched_barrier(0);
    group(Int<F>{}, make_mult(cur));
    __builtin_amdgcn_sched_barrier(0);
    tpipe_step<F + 1, NG>(T, cval, group, nxt, cur);
  }
}
template <int NG, typename CF, typename GF>
__device__ __forceinline__ void tpipelined(const DevTables& T, CF cval, GF group) {
  uint32_t pa[20], pb[20];
  pool_of<true>(T, cval(Int<0>{}), pa);
  tpipe_step<0, NG>(T, cval, group, pa, pb);
}

// Flat group f of levels R0..R1-1 of a register layout (ascending for the
// inverse transform, descending for the forward one).
template <int R0, int R1, bool INVERSE>
__host__ __device__ constexpr GroupRef rh_group(int f) {
  for (int s = 0; s < R1 - R0; ++s) {
    const int r = INVERSE ? R0 + s : R1 - 1 - s;
    const int n = 8 >> r;
    if (f < n) return GroupRef{r, f};
    f -= n;
  }
  return GroupRef{0, 0};
}
template <int R0, int R1>
__host__ __device__ constexpr int rh_groups() {
  int n = 0;
  for (int r = R0; r < R1; ++r) n += 8 >> r;
  return n;
}

// Staged VGPR halves of the HA / HD multipliers (kernels_res.hip), per
// transform of index I = blk K: kNH + 1 blocks of 15 slots of 8 dwords
// (pool dwords 0-7); block h < kNH holds the HA groups of hi = h (position
// bits 8-9 = w >> 2), block kNH the HD groups (hi = 0).  Level r (relative to
// the layout's first position bit), group t: slot rslot(r, t) of its block.
template <int K>
struct RStage {
  static constexpr uint32_t kNH = K / 256;
  static constexpr uint32_t kSlots = 15u * (kNH + 1);
  static constexpr uint32_t kWords = 8u * kSlots;  // per transform
};
__host__ __device__ constexpr uint32_t rslot(int r, int t) {
  return 16u - (16u >> r) + static_cast<uint32_t>(t);
}

// Copies the staged halves of the transforms at I = I0, I0 + K, ..,
// I0 + (nblk - 1) K into VS (nblk * RStage<K>::kWords dwords).  Caller
// synchronises.
template <int K>
__device__ __forceinline__ void stage_rh_tables(const DevTables& T, uint32_t* VS, uint32_t nblk, uint32_t I0 = 0) {
  using S = RStage<K>;
  constexpr int pbd = RGeo<K>::kLogK - 4;  // HD's first position bit
  const uint32_t* pools = fresh(T.tower_pools);
  const uint32_t total = 2u * S::kSlots * nblk;
  for (uint32_t i = fresh_v(threadIdx.x); i < total; i += K) {
    const uint32_t half = i & 1u, s = i >> 1;
    const uint32_t blk = s / S::kSlots, sl = s % S::kSlots;
    const uint32_t hb = sl / 15u, loc = sl % 15u;
    uint32_t r = 0;
    while (loc >= 16u - (8u >> r)) ++r;
    const uint32_t t = loc - (16u - (16u >> r)), I = I0 + blk * K;
    const uint32_t c = hb < S::kNH ? 2u * ((hb << (3 - r)) + t) + (I >> (4 + r)) : 2u * t + (I >> (pbd + r));
    *reinterpret_cast<uint4*>(VS + 8u * s + 4u * half) =
        *reinterpret_cast<const uint4*>(pools + static_cast<size_t>(c) * kPoolWords + 4u * half);
  }
}

// Levels PB0 + r, R0 <= r < R1, in a register layout whose register index j
// holds position bits PB0..PB0+3 and whose wave holds the bits above as `hi`:
// group T = (j >> (r + 1)) + (hi << (3 - r)).  Every multiplier is
// wave-uniform; levels below GEN (res_gen(I)) hold full ones (level 4 for
// I >= 4096, the shifts and segments of n = 8192), the others lie in GF(2^8).
//
// With vsb (the kernels_res.hip kernels) the VGPR halves of the multipliers
// come from the LDS block of the transform (RStage, stage_rh_tables) by
// ds_read instead of as v_mov copies of the s_loaded pool: 4 v_mov_b64 per
// group, i.e. up to a fifth of a level-4 butterfly.
template <int PB0, int R0, int R1, bool INVERSE, int GEN = 0, bool ST = false, int PRIO = 0>
__device__ __forceinline__ void rh_levels(const DevTables& T, uint32_t I, uint32_t hi, uint32_t (&L)[16],
                                          uint32_t (&H)[16], const uint32_t* vsb = nullptr) {
  if constexpr (kExp & 1) return;
  const uint32_t h = fresh(hi);
  auto cval = [&](auto fc) __attribute__((always_inline)) {
    constexpr GroupRef g = rh_group<R0, R1, INVERSE>(decltype(fc)::value);
    return 2u * ((h << (3 - g.b)) + g.t) + (I >> (PB0 + g.b));
  };
  auto group = [&](auto fc, const Mult& p) __attribute__((always_inline)) {
    constexpr GroupRef g = rh_group<R0, R1, INVERSE>(decltype(fc)::value);
    constexpr int d = 1 << g.b;
    constexpr bool SUB = PB0 + g.b >= GEN;
    progress_prio<decltype(fc)::value, rh_groups<R0, R1>(), PRIO>();
#pragma unroll
    for (int v = 0; v < d; ++v) {
      const int x = g.t * 2 * d + v, y = x + d;
      if constexpr (INVERSE) {
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
  if constexpr (ST) {
    auto vaddr = [&](auto fc) __attribute__((always_inline)) {
      constexpr GroupRef g = rh_group<R0, R1, INVERSE>(decltype(fc)::value);
      return vsb + 8u * rslot(g.b, g.t);
    };
    auto subf = [&](auto fc) __attribute__((always_inline)) {
      return std::integral_constant<bool, (PB0 + rh_group<R0, R1, INVERSE>(decltype(fc)::value).b >= GEN)>{};
    };
    pipelined_staged<rh_groups<R0, R1>(), true>(T, cval, vaddr, subf, group);
  } else {
    tpipelined<rh_groups<R0, R1>()>(T, cval, group);
  }
}

// HA: levels 4-7 (hi = position bits 8-9 = w >> 2; K = 512: bit 8).  HD:
// the levels above 7 (register bits j hold position bits logK-4 .. logK-1:
// K = 1024 levels 8-9 = j bits 2-3, K = 512 level 8 = j bit 3; hi = 0).
template <bool INVERSE, int GEN = 0>
__device__ __forceinline__ void ha_levels(const DevTables& T, uint32_t I, const Res& r, uint32_t (&L)[16],
                                          uint32_t (&H)[16]) {
  if constexpr (kExp & 512) return;
  rh_levels<4, 0, 4, INVERSE, GEN>(T, I, r.w >> 2, L, H);
}
template <int K, bool INVERSE>
__device__ __forceinline__ void hd_levels(const DevTables& T, uint32_t I, uint32_t (&L)[16], uint32_t (&H)[16]) {
  if constexpr (kExp & 1024) return;
  constexpr int pb0 = RGeo<K>::kLogK - 4;
  rh_levels<pb0, 8 - pb0, 4, INVERSE>(T, I, 0u, L, H);
}
// The same with the staged VGPR halves: vs = the transform's RStage block.
template <int K, bool INVERSE, int GEN = 0, int PRIO = 0>
__device__ __forceinline__ void ha_levels_st(const DevTables& T, uint32_t I, const Res& r, uint32_t (&L)[16],
                                             uint32_t (&H)[16], const uint32_t* vs) {
  if constexpr (kExp & 512) return;
  const uint32_t h = fresh(r.w >> 2);
  rh_levels<4, 0, 4, INVERSE, GEN, true, PRIO>(T, I, h, L, H, vs + 120u * h);
}
template <int K, bool INVERSE, int PRIO = 0>
__device__ __forceinline__ void hd_levels_st(const DevTables& T, uint32_t I, uint32_t (&L)[16], uint32_t (&H)[16],
                                             const uint32_t* vs) {
  if constexpr (kExp & 1024) return;
  constexpr int pb0 = RGeo<K>::kLogK - 4;
  rh_levels<pb0, 8 - pb0, 4, INVERSE, 0, true, PRIO>(T, I, 0u, L, H, vs + 120u * RStage<K>::kNH);
}

// A ^= D_K(X) in the HD layout for one byte plane (inc_afft.rs:17-31,
// closed form SURVEY F7: D(x)[p] = x[p] ^ XOR over single bits l not in p of
// x[p | l]): bits 0-1 inside the quad, bits 2-5 (K = 512: 2-4) in the lanes
// of a DPP row (l & 15: quad_perm for bits 2-3, row_shl 4 / 8 for bits 4-5),
// the rest (6-9; K = 512: 5-8) in the registers.  K = 256: bits 2-3 in the
// lanes (quad_perm), 4-7 in the registers.
template <int K>
__device__ __forceinline__ void add_derivative_hd(uint32_t (&A)[16], uint32_t (&X)[16], uint32_t lane) {
  const uint32_t r = lane & 15u;
  const uint32_t m0 = (r & 1u) ? 0u : ~0u, m1 = (r & 2u) ? 0u : ~0u;
  const uint32_t m2 = (r & 4u) ? 0u : ~0u, m3 = (r & 8u) ? 0u : ~0u;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t x = X[j];
    uint32_t v = xor3(x, vperm(x, x, 0x0C030301u), vperm(x, x, 0x0C0C0C02u));
    v ^= static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(x), 0xB1, 0xF, 0xF, false)) & m0;
    v ^= static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(x), 0x4E, 0xF, 0xF, false)) & m1;
    if constexpr (RGeo<K>::kLPC >= 8)
      v ^= static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(x), 0x104, 0xF, 0xF, false)) & m2;
    if constexpr (RGeo<K>::kLPC == 16)
      v ^= static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(x), 0x108, 0xF, 0xF, false)) & m3;
#pragma unroll
    for (int jb = 0; jb < 4; ++jb)
      if (!(j & (1 << jb))) v ^= X[j | (1 << jb)];
    A[j] ^= v;
    asm volatile("" : "+v"(A[j]));  // finish position j here (bounded temporaries)
    X[j] = 0;                       // dead from here on
  }
}

// ------------------------------------------------------------ payload tile ----
// Natural blocks of 64 chunks into the LDS tile: chunk ch0 + c supplies its
// bytes [off, off + 2K) (chunk_bytes apart; off = 0 and chunk_bytes = 2K for a
// whole chunk, off = 2048 m for sub-segment m of a size-k chunk); thread t
// moves block t mod K/4 of chunks t / (K/4) + 4 i.  Bytes past payload_len
// are zeros (the reference's zero padding, mod.rs:117-157).
template <int K>
__device__ __forceinline__ void load_pay_tile(uint8_t* tile, const uint8_t* pay, size_t payload_len, uint32_t ch0,
                                              size_t chunk_bytes, size_t off, uint32_t tid) {
  const uint32_t m = tid % (K / 4), c0 = tid / (K / 4);
  const bool fast = out_vec_ok(pay, 0) &&  // (8-byte loads at any address, see rows_vec_ok)
                    static_cast<size_t>(ch0 + kRC - 1) * chunk_bytes + off + 2 * K <= payload_len;
  const uint8_t* src = pay + static_cast<size_t>(ch0 + c0) * chunk_bytes + off + 8u * m;
  if (fast) {
    uint2 v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) v[i] = (kExp & 4) ? make_uint2(i, tid) : load_once(src + static_cast<size_t>(i) * 4 * chunk_bytes);
#pragma unroll
    for (int i = 0; i < 16; ++i) *reinterpret_cast<uint2*>(tile + pq_addr<K>(c0 + 4u * i, m)) = v[i];
  } else {
#pragma unroll 1
    for (uint32_t i = 0; i < 16; ++i) {
      const size_t g0 = static_cast<size_t>(ch0 + c0 + 4u * i) * chunk_bytes + off + 8u * m;
      uint32_t wv[2] = {0, 0};
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (g0 + e < payload_len) wv[e >> 2] |= static_cast<uint32_t>(*NP_BCHK(pay + (g0 + e), 1, kBkPayloads)) << (8 * (e & 3));
      *reinterpret_cast<uint2*>(tile + pq_addr<K>(c0 + 4u * i, m)) = make_uint2(wv[0], wv[1]);
    }
  }
}

// Two payloads in one tile (kernels_huge.hip, payloads of at most 32 columns:
// k = 16384 at 1 MiB): columns 0..31 are chunks 0..31 of pay0, columns
// 32..63 chunks 0..31 of pay1 (nullptr: the batch ended, zeros).  Bytes past
// payload_len, and chunks past the payload's last, are zeros as in
// load_pay_tile.
template <int K>
__device__ __forceinline__ void load_pay_tile_pair(uint8_t* tile, const uint8_t* pay0, const uint8_t* pay1,
                                                   size_t payload_len, size_t chunk_bytes, size_t off, uint32_t tid) {
  const uint32_t m = tid % (K / 4), c0 = tid / (K / 4);
#pragma unroll 1
  for (uint32_t i = 0; i < 16; ++i) {
    const uint32_t c = c0 + 4u * i;
    const uint8_t* pay = c < 32u ? pay0 : pay1;
    const size_t g0 = static_cast<size_t>(c & 31u) * chunk_bytes + off + 8u * m;
    uint2 v = make_uint2(0, 0);
    if (pay && g0 + 8 <= payload_len) {
      v = load_once(pay + g0);
    } else if (pay) {
      uint32_t wv[2] = {0, 0};
#pragma unroll
      for (int e = 0; e < 8; ++e)
        if (g0 + e < payload_len) wv[e >> 2] |= static_cast<uint32_t>(pay[g0 + e]) << (8 * (e & 3));
      v = make_uint2(wv[0], wv[1]);
    }
    *reinterpret_cast<uint2*>(tile + pq_addr<K>(c, m)) = v;
  }
}

// ------------------------------------------------------------ shard rows ----

// This lane's 8 bytes (columns 4 cq .. 4 cq + 3) of shard rows
// row0 + 64 w + 16 u + i, i = 0..15.  `out` = row 0, column 0 of the tile.
// nt: streaming stores (rows of whole 128-byte lines); rows that start
// inside a line (odd chunk counts) store with the default policy, so that L2
// merges the pieces of a line that neighbouring waves write.
__device__ __forceinline__ void rres_store_rows(uint8_t* out, size_t shard_len, uint32_t row0, uint32_t wanted_n,
                                                const uint32_t (&L)[16], const uint32_t (&H)[16], const Res& r,
                                                uint32_t ncols, bool full, bool nt) {
  const uint32_t rb = row0 + 64u * fresh(r.w);  // first row of this wave
  if (full && rb + 64u <= wanted_n && 64u * shard_len < 0x7fffffffu) {
    const __amdgpu_buffer_rsrc_t rs = buf_rsrc(out + static_cast<size_t>(rb) * shard_len, 64u * static_cast<uint32_t>(shard_len));
    const uint32_t vo = fresh_v(16u * r.u * static_cast<uint32_t>(shard_len) + 8u * r.cq);
    if (nt) {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const uint2 v = cq_row(L[i], H[i]);
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{v.x, v.y}, rs, vo, static_cast<uint32_t>(i * shard_len),
                                              kRowStoreCpol);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const uint2 v = cq_row(L[i], H[i]);
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{v.x, v.y}, rs, vo, static_cast<uint32_t>(i * shard_len), 0);
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    const uint32_t row = rb + 16u * r.u + i;
    if (row < wanted_n) store4(out + static_cast<size_t>(row) * shard_len, cq_row(L[i], H[i]), r.cq, ncols, full);
  }
}

// The same for a tile of two payloads (load_pay_tile_pair): lane 16 u + cq
// stores columns 4 (cq & 7) .. + 3 of payload cq >> 3 (out0 / out1 = row 0,
// column 0 of each; nullptr: none), ncols columns each.
__device__ __forceinline__ void rres_store_rows_pair(uint8_t* out0, uint8_t* out1, size_t shard_len, uint32_t row0,
                                                     uint32_t wanted_n, const uint32_t (&L)[16], const uint32_t (&H)[16],
                                                     const Res& r, uint32_t ncols) {
  uint8_t* out = r.cq < 8u ? out0 : out1;
  if (!out) return;
  const uint32_t lc = r.cq & 7u, rb = row0 + 64u * r.w + 16u * r.u;
  const bool whole = 4u * lc + 4u <= ncols;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (rb + i >= wanted_n) break;
    uint8_t* rowp = out + static_cast<size_t>(rb + i) * shard_len;
    const uint2 v = cq_row(L[i], H[i]);
    if (whole)
      *reinterpret_cast<uint2*>(rowp + 8u * lc) = v;
    else
      store4(rowp, v, lc, ncols, false);
  }
}

// ----------------------------------------------------------- reconstruct ----
// n = NQ * K, NQ in {2, 4, 8}.  As in k_reconstruct_fast (kernels_fast.hip,
// DESIGN.md §4.3) the first k outputs are FFT(K, 0)(d) with
//   NQ = 2: d = D(x0) ^ x0 ^ x1,   NQ = 4: d = D(x0) ^ x1 ^ x2 ^ beta (x2 ^ x3),
//   NQ = 8: d = D(x0) ^ sum_q kappa_q x_q (rec8_kappa_res),
// x_q = IFFT(K, K q)(premultiplied segment q), beta = Cantor(2) and D the
// size-K formal derivative -- here every x_q is computed whole in the
// workgroup (CQ -> HA -> HD) and d accumulates in the HD layout, where every
// position bit is reachable for D (add_derivative_hd).
//
// Row multipliers: the payload's prefix record (k_prefix_locator): one 80-byte
// table per row (the premultiply's Cantor -> tower map for present rows, the
// postmultiply's tower -> Cantor map for erased ones).  CQ lanes of one wave
// hold 4 different rows per register (u), so a segment's K tables are
// staged into the LDS tile (free between the HD read and the next exchange)
// and read per lane; absent rows get zero tables (their rows read as zeros).
constexpr uint32_t kRowSlot = 80;  // bytes per staged row table
// Row r (of a segment) -> its LDS table slot: groups of 16 rows with 16 bytes
// of padding after each (1296 bytes = 324 dwords, 4 banks apart), so the four
// rows r, r + 16, r + 32, r + 48 of one wave-instruction hit different banks.
constexpr uint32_t kRowGroup = 16 * kRowSlot + 16;
__host__ __device__ constexpr uint32_t row_slot(uint32_t r) { return kRowGroup * (r >> 4) + kRowSlot * (r & 15u); }
static_assert(row_slot(1023) + kRowSlot <= RGeo<1024>::kTileBytes, "row tables fit the tile");
static_assert(row_slot(511) + kRowSlot <= RGeo<512>::kTileBytes, "row tables fit the tile");
static_assert(row_slot(255) + kRowSlot <= RGeo<256>::kTileBytes, "row tables fit the tile");

// Thread t stages the table of row row0 + t (zeros for an absent row, so that
// its premultiplied zero row stays zero without a select).
__device__ __forceinline__ void stage_row_tables(uint8_t* tile, const uint8_t* pools, const uint8_t* pres,
                                                 uint32_t row0, uint32_t tid, bool erased_only) {
  const uint32_t row = row0 + tid;
  const bool p = pres[row] != 0;
  const bool take = erased_only ? !p : p;
  uint4 v[5];
  const uint4* src = reinterpret_cast<const uint4*>(pools + static_cast<size_t>(row) * kRowSlot);
#pragma unroll
  for (int i = 0; i < 5; ++i) v[i] = take ? src[i] : make_uint4(0, 0, 0, 0);
  uint4* dst = reinterpret_cast<uint4*>(tile + row_slot(tid));
#pragma unroll
  for (int i = 0; i < 5; ++i) dst[i] = v[i];
}

// The same by LDS-DMA, issued without waiting: rows row0 .. row0 + nrows - 1
// (nrows a multiple of 16) of the payload's record into their slots, every
// row's record table as it is (an absent row reads zeros, and a table maps
// zero to zero, so its premultiplied row stays zero).  A 16-row group is 1280
// contiguous record bytes = 5 pieces of 256 bytes (one global_load_lds_dword
// per wave: LDS byte M0 + 4 lane); the waves of the workgroup take the pieces
// in turn.  The caller waits (s_waitcnt vmcnt) and synchronises before the
// tables are read.  Written as asm (M0 set in the same statement,
// kernels_fast.hip dma_tile), so the compiler adds no vmcnt(0) of its own.
__device__ __forceinline__ void dma_row_tables(uint8_t* tile, const uint8_t* pools, uint32_t row0, uint32_t nrows,
                                               uint32_t w, uint32_t lane, uint32_t nwaves) {
  static_assert(16 * kRowSlot == 5 * 256, "five 256-byte pieces per 16-row group");
  const uint32_t lds0 = static_cast<uint32_t>(reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint8_t*)(tile)));
  const uint32_t pieces = (nrows / 16) * 5;
  const uint8_t* src0 = pools + static_cast<size_t>(row0) * kRowSlot + 4u * lane;
#pragma unroll 1
  for (uint32_t pc = w; pc < pieces; pc += nwaves) {
    const uint32_t g = pc / 5, part = pc - 5 * g;
    const uint8_t* src = NP_BCHK(src0 + 1280u * g + 256u * part, 4, kBkRecords);
    const uint32_t dst = uniform(lds0 + kRowGroup * g + 256u * part);
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(src), "s"(dst)
                 : "memory");
  }
}

// The same from the payload's locators (log form, all n rows: mul(x, log m) ==
// x * EXP[m], inc_log_mul.rs:42-49): the tables of EXP[loc] straight from the
// context's pools (present rows: in_pools, Cantor -> tower; erased rows:
// out_pools, tower -> Cantor), as k_locator_records / write_row_pools build them.
__device__ __forceinline__ void stage_row_tables_loc(uint8_t* tile, const DevTables& T, const uint16_t* loc,
                                                     const uint8_t* pres, uint32_t row0, uint32_t tid,
                                                     bool erased_only) {
  const uint32_t row = row0 + tid;
  const bool p = pres[row] != 0;
  const bool take = erased_only ? !p : p;
  uint4 v[5];
  const uint32_t e = T.exp[loc[row]];
  const uint4* src = reinterpret_cast<const uint4*>((p ? T.in_pools : T.out_pools) + static_cast<size_t>(e) * kPoolWords);
#pragma unroll
  for (int i = 0; i < 5; ++i) v[i] = take ? src[i] : make_uint4(0, 0, 0, 0);
  uint4* dst = reinterpret_cast<uint4*>(tile + row_slot(tid));
#pragma unroll
  for (int i = 0; i < 5; ++i) dst[i] = v[i];
}

__device__ __forceinline__ FullT row_table(const uint8_t* tile, uint32_t r) {
  FullT m;
  const uint4* src = reinterpret_cast<const uint4*>(tile + row_slot(r));
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const uint4 v = src[i];
    m.p[4 * i] = v.x, m.p[4 * i + 1] = v.y, m.p[4 * i + 2] = v.z, m.p[4 * i + 3] = v.w;
  }
  return m;
}

// Two payloads in one tile (kernels_huge.hip, HugeArgs::pair): the tables of
// both payloads' rows do not fit the tile at once (2 x 1024 x 80 bytes), so
// they are staged in two halves.  Half hf holds rows row0 + 16 g + 8 hf + i
// (g < 64, i < 8) of payload sel at slot sel * 512 + 8 g + i, in the 16-row
// groups of row_slot (83 KiB).  A CQ lane (wave w, u, cq) reads its row i of
// the half at pair_row_slot(cq >> 3, 4 w + u, i).
__host__ __device__ constexpr uint32_t pair_row_slot(uint32_t sel, uint32_t g, uint32_t i) {
  return row_slot(512u * sel + 8u * g + i);
}
static_assert(pair_row_slot(1, 63, 7) + kRowSlot <= RGeo<1024>::kTileBytes, "pair row tables fit the tile");

// Thread t stages half hf's table of payload t >> 9 (loc / pres of payload 0
// and 1; payload 1 may be absent: pres1 == nullptr, zero tables), as
// stage_row_tables_loc.
__device__ __forceinline__ void stage_row_tables_pair(uint8_t* tile, const DevTables& T, const uint16_t* loc0,
                                                      const uint8_t* pres0, const uint16_t* loc1,
                                                      const uint8_t* pres1, uint32_t row0, uint32_t hf, uint32_t tid,
                                                      bool erased_only) {
  const uint32_t sel = tid >> 9, g = (tid >> 3) & 63u, i = tid & 7u;
  const uint32_t row = row0 + 16u * g + 8u * hf + i;
  const uint8_t* pres = sel ? pres1 : pres0;
  const uint16_t* loc = sel ? loc1 : loc0;
  uint4 v[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) v[k] = make_uint4(0, 0, 0, 0);
  if (pres) {
    const bool p = pres[row] != 0;
    if (erased_only ? !p : p) {
      const uint32_t e = T.exp[loc[row]];
      const uint4* src = reinterpret_cast<const uint4*>((p ? T.in_pools : T.out_pools) + static_cast<size_t>(e) * kPoolWords);
#pragma unroll
      for (int k = 0; k < 5; ++k) v[k] = src[k];
    }
  }
  uint4* dst = reinterpret_cast<uint4*>(tile + pair_row_slot(sel, g, i));
#pragma unroll
  for (int k = 0; k < 5; ++k) dst[k] = v[k];
}

__device__ __forceinline__ FullT row_table_at(const uint8_t* tile, uint32_t addr) {
  FullT m;
  const uint4* src = reinterpret_cast<const uint4*>(tile + addr);
#pragma unroll
  for (int i = 0; i < 5; ++i) {
    const uint4 v = src[i];
    m.p[4 * i] = v.x, m.p[4 * i + 1] = v.y, m.p[4 * i + 2] = v.z, m.p[4 * i + 3] = v.w;
  }
  return m;
}

// Presence bits of this lane's 16 rows row0 + 64 w + 16 u + i (bit i).
__device__ __forceinline__ uint32_t lane_rows_present(const uint8_t* pres, uint32_t row0, const Res& r) {
  const uint8_t* p = NP_BCHK(pres + row0 + 64u * r.w + 16u * r.u, 16, kBkPresent);
  uint32_t m = 0;
  if ((reinterpret_cast<uintptr_t>(p) & 3u) == 0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t v = reinterpret_cast<const uint32_t*>(p)[i];
#pragma unroll
      for (int b = 0; b < 4; ++b)
        if ((v >> (8 * b)) & 0xffu) m |= 1u << (4 * i + b);
    }
  } else {
#pragma unroll
    for (int i = 0; i < 16; ++i)
      if (p[i]) m |= 1u << i;
  }
  return m;
}

// This lane's 8 bytes of rows row0 + 64 w + 16 u + i0 + i, i < NR (absent: zeros).
template <int NR = 16>
__device__ __forceinline__ void load_lane_rows(uint2 (&raw)[NR], const uint8_t* sh, size_t shard_len, uint32_t row0,
                                               uint32_t pm, const Res& r, uint32_t ncols, bool full,
                                               const uint8_t* zeros, int i0 = 0) {
  const uint8_t* base = sh + static_cast<size_t>(row0 + 64u * r.w + 16u * r.u + i0) * shard_len;
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const uint8_t* src = ((pm >> (i0 + i)) & 1u) ? base + static_cast<size_t>(i) * shard_len : zeros;
#if NP_BOUNDS_CHECK
    {  // the bytes load4 reads: columns 4 cq .. 4 cq + 3 below ncols
      const uint32_t nb = full ? 8u : 2u * static_cast<uint32_t>(min(4, max(0, static_cast<int>(ncols) - 4 * static_cast<int>(r.cq))));
      src = NP_BCHK2(src + 8u * r.cq, nb, kBkShards, kBkZeros) - 8u * r.cq;
    }
#endif
    raw[i] = load4(src, r.cq, ncols, full);
  }
}

// The merge's output: CQ registers (positions 64 w + 16 u + i of columns
// 4 cq .. + 3) -> bytes [2 (64 w + 16 u), + 32) of each of the 4 output
// columns (2K bytes each).
template <int K>
// col_bytes: the output's column stride (2K; 2k for a sub-segment of a size-k
// transform, kernels_huge.hip).
__device__ __forceinline__ void res_copy_out(uint8_t* out_tile, const uint32_t (&L)[16], const uint32_t (&H)[16],
                                             const Res& r, uint32_t ncols, bool aligned16,
                                             size_t col_bytes = 2 * K) {
  uint2 d[4][4];
#pragma unroll
  for (int q = 0; q < 4; ++q) cq_to_blks(&L[4 * q], &H[4 * q], d[q]);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const uint32_t c = 4u * r.cq + e;
    if (c >= ncols) break;
    uint8_t* o = NP_BCHK(out_tile + static_cast<size_t>(c) * col_bytes + 128u * r.w + 32u * r.u, 32, kBkOut);
    if (aligned16) {
      *reinterpret_cast<uint4*>(o) = make_uint4(d[0][e].x, d[0][e].y, d[1][e].x, d[1][e].y);
      *reinterpret_cast<uint4*>(o + 16) = make_uint4(d[2][e].x, d[2][e].y, d[3][e].x, d[3][e].y);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int b = 0; b < 8; ++b) o[8 * q + b] = static_cast<uint8_t>((b < 4 ? d[q][e].x : d[q][e].y) >> (8 * (b & 3)));
    }
  }
}

// NQ = 8: the fold coefficients of kernels_fast.hip rec8_kappa (Cantor
// coordinates, all in GF(16); tests/test_oracle.py::test_rec8_kappa).
__host__ __device__ constexpr uint32_t rec8_kappa_res(int q) {
  constexpr uint32_t k[8] = {1, 1, 3, 2, 12, 15, 10, 8};
  return k[q];
}

// ---------------------------------------------- encode: quad items ----
// After its payload read, the encode's tile (k_encode_res, and the huge
// encode's sub-transforms) holds quad items: column quad cq
// (4 columns, byte-planar: exactly a CQ register pair) at position p, at byte
// 128 pi(p) + 8 cq with pi(p) = p ^ ((p >> 4) & 1).  So the exchanges between
// its layouts move register pairs as they are: no tr4x4 (the decode keeps the
// planar items of res_common.hpp, whose HD layout its derivative needs).
// Layouts besides CQ (lane 16 a + cq, a = lane bits 4-5):
//  * HA': register j = position bits 4-7, a = bits 0-1, w & 3 = bits 2-3,
//    w >> 2 = bits 8-9 (the HA levels' hi, as in res_common's HA);
//  * HD': register j = position bits logK-4 .. logK-1, a = bits 0-1, w = the
//    bits between.
// Banks: a ds_write_b64 of 16 lanes covers one position's 128-byte row; the
// 32-lane halves of a ds_read_b64 cover two positions that differ in bit 4
// (CQ: u) or bit 0 (HA', HD': a), and pi puts those in opposite halves of a
// 256-byte bank row.
struct Qi {
  uint32_t cqe, cqo;  // CQ: item i at (i odd ? cqo : cqe) + 128 i
  uint32_t ha;        // HA': item j at (j odd ? ha ^ 128 : ha) + 2048 j
  uint32_t hd;        // HD': item j at hd + (128 << (logK - 4)) j
};
template <int K>
__device__ __forceinline__ Qi qi_coords(const Res& r) {
  Qi q;
  const uint32_t e = r.u & 1u;  // position bit 4 in CQ
  const uint32_t cqb = 128u * (64u * r.w + 16u * r.u) + 8u * r.cq;
  q.cqe = cqb + 128u * e;  // even i: i ^ e = i + e
  q.cqo = cqb - 128u * e;  // odd i: i ^ e = i - e
  q.ha = 128u * (((r.w >> 2) << 8) | ((r.w & 3u) << 2) | r.u) + 8u * r.cq;
  const uint32_t ph = (r.w << 2) | r.u;
  q.hd = 128u * (ph ^ ((ph >> 4) & 1u)) + 8u * r.cq;
  return q;
}
template <bool WRITE>
__device__ __forceinline__ void qi_item(uint8_t* tile, uint32_t addr, uint32_t& l, uint32_t& h) {
  if constexpr (WRITE) {
    *reinterpret_cast<uint2*>(tile + addr) = make_uint2(l, h);
  } else {
    const uint2 d = *reinterpret_cast<const uint2*>(tile + addr);
    l = d.x;
    h = d.y;
  }
}
template <bool WRITE>
__device__ __forceinline__ void qi_cq(uint8_t* tile, const Qi& q, uint32_t (&L)[16], uint32_t (&H)[16]) {
  const uint32_t be = fresh_v(q.cqe), bo = fresh_v(q.cqo);
#pragma unroll
  for (int i = 0; i < 16; ++i) qi_item<WRITE>(tile, ((i & 1) ? bo : be) + 128u * i, L[i], H[i]);
}
template <bool WRITE>
__device__ __forceinline__ void qi_ha(uint8_t* tile, const Qi& q, uint32_t (&L)[16], uint32_t (&H)[16]) {
  const uint32_t be = fresh_v(q.ha), bo = fresh_v(q.ha ^ 128u);
#pragma unroll
  for (int j = 0; j < 16; ++j) qi_item<WRITE>(tile, ((j & 1) ? bo : be) + 2048u * j, L[j], H[j]);
}
template <int K, bool WRITE>
__device__ __forceinline__ void qi_hd(uint8_t* tile, const Qi& q, uint32_t (&L)[16], uint32_t (&H)[16]) {
  constexpr uint32_t step = 128u << (RGeo<K>::kLogK - 4);
  const uint32_t b0 = fresh_v(q.hd), b1 = fresh_v(q.hd + 8u * step);  // two bases: ds offsets < 64 KiB
#pragma unroll
  for (int j = 0; j < 16; ++j) qi_item<WRITE>(tile, (j < 8 ? b0 : b1) + step * (j & 7), L[j], H[j]);
}

}  // namespace
}  // namespace np
