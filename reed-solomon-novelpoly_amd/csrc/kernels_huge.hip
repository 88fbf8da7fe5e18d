// k = 2048 .. 16384 (n = 4096 .. 65536; 8,193-65,536 validators): a size-k
// transform as M = k / 1024 size-1024 sub-transforms in the resident layouts
// of res_common.hpp plus its top log2(M) levels.
//
// For a size-k transform at index I (a multiple of k) and position
// p = 1024 m + p' (sub-segment m):
//  * a level b < 10 has the skew Cantor(2T + (I >> b)) of group T = p >> (b + 1)
//    = (m << (9 - b)) + (p' >> (b + 1)), i.e. Cantor(2 (p' >> (b + 1)) +
//    ((I + 1024 m) >> b)): the levels 0-9 on sub-segment m are the size-1024
//    transform at index I + 1024 m (inc_afft.rs:139-214 / :267-332);
//  * a level b = 10 + L >= 10 pairs sub-segments m and m + 2^L with the skew
//    Cantor(2 (m >> (L + 1)) + (I >> b)), the same for every p', and in GF(2^8)
//    ((I + k) >> 10 <= 64 for n <= 65536): a subfield multiply per quad.
// So IFFT(k, I) = Top^-1_I o (IFFT(1024, I + 1024 m) per m) and FFT(k, I) =
// (FFT(1024, I + 1024 m) per m) o Top_I.
//
// The sub-transforms hand their results to the top-level pass through a
// scratch in thread order: slot s of a tile holds the HD registers of the
// sub-transform's 1024 threads (quad j of thread t at (1024 j + t) * 8 bytes,
// 128 KiB), so (j, t) names the same 4 positions of the same column in every
// slot and the top-level pass runs per (j, t) with coalesced 8-byte accesses.
//
// Encode (mod.rs:144-154, inc_encode.rs:15-48), per batch slice:
//   k_huge_enc_inv  per m: payload sub-tile -> systematic rows, IFFT(1024,
//                   1024 m) -> slot m;
//   k_huge_enc_top  per (j, t): Top^-1_0 over slots 0..M-1 -> coefficients,
//                   then per shift s Top_{sk} -> slots s M + m;
//   k_huge_enc_fwd  per (s, m): FFT(1024, sk + 1024 m) of slot s M + m -> shard
//                   rows sk + 1024 m ...
// Reconstruct (inc_reconstruct.rs:1-113, mod.rs:162-239; the fold of
// kernels_fast.hip / DESIGN.md §4.3 with n = NQ k):
//   k_huge_records  status and mode per payload (skip / copy / decode), and
//                   which 1024-row blocks hold a present row;
//   locators        the generic 65536-point Walsh kernel (or the caller's);
//   k_huge_rec_inv  per (q, m): premultiplied rows q k + 1024 m ..,
//                   IFFT(1024, q k + 1024 m) -> slot q M + m; q = 0 also
//                   D_1024 of it -> slot NQ M + m; nothing for a block
//                   without a present row (zero: the rows past wanted_n);
//   k_huge_rec_top  per (j, t): x_q = Top^-1_{qk}, d = D_k(x_0) ^ sum kappa_q
//                   x_q with D_k = (D_1024 lifted) ^ the high single-bit
//                   terms x_0[m | 2^L] (kernels_big.hip's argument), then
//                   Top_0 -> slots 0..M-1;
//   k_huge_rec_fwd  per m: FFT(1024, 1024 m) of slot m, postmultiply of the
//                   erased rows, merge with the received ones, copy-out.
#include "res_common.hpp"

namespace np {
namespace {

// Age order (no s_setprio) in the sub-transforms' passes: progress-based
// priority (fast_common.hpp progress_prio) measured neutral at 10000
// validators (profiles/r04_ab.txt probe 23).
constexpr int kHugePrioEnc = 0, kHugePrioDec = 0;

constexpr int kSK = 1024;                             // sub-transform size
constexpr uint32_t kSlotBytes = 16u * 1024u * 8u;     // one sub-segment of a tile in thread order
constexpr uint32_t kHDS = RGeo<kSK>::kHD;
// Dynamic LDS of the sub-transform kernels: the tile, the CQ delta tables and
// the RStage block of the workgroup's transform index.
constexpr uint32_t kHugeLds = RGeo<kSK>::kTileBytes + 4u * (kDeltaWords + RStage<kSK>::kWords);

struct HugeArgs {
  uint8_t* scr;         // tile slots of the slice: tile (pb, tl) at (pb tiles + tl) slots kSlotBytes
  const uint16_t* loc;  // reconstruct: locators, batch x n (log form)
  const uint8_t* mode;  // reconstruct: per payload kHugeSkip / kHugeCopy / kHugeDecode
  const uint64_t* occ;  // reconstruct: per payload, bit u: rows 1024 u .. + 1023 hold a present row
  uint32_t tiles, slots, M, K, NQ;
  // encode, payloads of at most 32 columns: a tile holds two payloads
  // (columns 0-31 payload 2 pb, 32-63 payload 2 pb + 1; load_pay_tile_pair)
  uint32_t pair;
  uint32_t batch;  // payloads of the slice
  // this launch's sub-transforms: u0 .. u0 + (grid / per) - 1 (index 1024 u,
  // slot u; all of one res_gen), per = batch x tiles workgroups each
  uint32_t u0, per;
};
// Workgroup b of a launch: sub-transform u, batch entry and tile.
struct SubRef {
  uint32_t u, pb, tl;
};
__device__ __forceinline__ SubRef sub_of(const HugeArgs& h, uint32_t b, size_t batch) {
  const uint32_t u = uniform(h.u0 + b / h.per);
  const TileRef tr = tile_of(b % h.per, h.tiles, (batch & 7u) == 0);
  return SubRef{u, tr.pb, tr.tl};
}
constexpr uint8_t kHugeSkip = 0, kHugeCopy = 1, kHugeDecode = 2;
// Mode of tile pt's payload; a paired tile (HugeArgs::pair) runs the larger
// of its two payloads' modes (decode > copy > skip).
__device__ __forceinline__ uint32_t tile_mode(const HugeArgs& h, size_t pt) {
  if (!h.pair) return h.mode[pt / h.tiles];
  const uint32_t m0 = h.mode[2 * pt];
  const uint32_t m1 = 2 * pt + 1 < h.batch ? h.mode[2 * pt + 1] : kHugeSkip;
  return m0 > m1 ? m0 : m1;
}
// Blocks of tile pt's payload(s) with a present row (a paired tile: either
// payload's); the slots of the others are zero and never written.
__device__ __forceinline__ uint64_t tile_occ(const HugeArgs& h, size_t pt) {
  if (!h.pair) return h.occ[pt / h.tiles];
  return h.occ[2 * pt] | (2 * pt + 1 < h.batch ? h.occ[2 * pt + 1] : 0ull);
}
// The units a launch's workgroups enumerate per sub-transform: tiles, or
// pairs of payloads.
__device__ __forceinline__ uint32_t unit_count(const HugeArgs& h, uint32_t batch) {
  return h.pair ? (batch + 1) / 2 : batch;
}

__device__ __forceinline__ uint8_t* slot_at(const HugeArgs& h, uint32_t pb, uint32_t tl, uint32_t slot) {
  return h.scr + (static_cast<size_t>(pb) * h.tiles + tl) * h.slots * kSlotBytes + static_cast<size_t>(slot) * kSlotBytes;
}
__device__ __forceinline__ void slot_store(uint8_t* s, uint32_t tid, const uint32_t (&L)[16], const uint32_t (&H)[16]) {
#pragma unroll
  for (int j = 0; j < 16; ++j) *reinterpret_cast<uint2*>(s + (1024u * j + tid) * 8u) = make_uint2(L[j], H[j]);
}
__device__ __forceinline__ void slot_load(const uint8_t* s, uint32_t tid, uint32_t (&L)[16], uint32_t (&H)[16]) {
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint2 v = *reinterpret_cast<const uint2*>(s + (1024u * j + tid) * 8u);
    L[j] = v.x;
    H[j] = v.y;
  }
}

// ---------------------------------------------------------- top levels ----
// x ^= c y for one quad, c < 256 a Cantor index (subfield, tower coordinates).
__device__ __forceinline__ void top_mul(const DevTables& T, uint32_t c, uint2& x, const uint2& y) {
  uint32_t p[20];
  pool_of<true>(T, c, p);
  const Mult mm = make_mult(p);
  qmul_sub(x.x, x.y, y.x, y.y, mm);
}

// Levels 10 .. 10 + log2(M) - 1 of a size-1024 M transform at index I over the
// sub-segment quads y[m].  Inverse (ascending levels): hi ^= lo; lo ^= c hi.
template <int M>
__device__ __forceinline__ void top_inverse_h(const DevTables& T, uint2 (&y)[M], uint32_t I) {
#pragma unroll
  for (int L = 0; (1 << L) < M; ++L) {
#pragma unroll
    for (int g = 0; g < (M >> (L + 1)); ++g) {
      const uint32_t c = uniform(2u * g + (I >> (10 + L)));
#pragma unroll
      for (int v = 0; v < (1 << L); ++v) {
        const int lo = g * (2 << L) + v, hi = lo + (1 << L);
        y[hi].x ^= y[lo].x;
        y[hi].y ^= y[lo].y;
        top_mul(T, c, y[lo], y[hi]);
      }
    }
  }
}
// Forward (descending levels): lo ^= c hi; hi ^= lo.
template <int M>
__device__ __forceinline__ void top_forward_h(const DevTables& T, uint2 (&y)[M], uint32_t I) {
#pragma unroll
  for (int L = ilog2(M) - 1; L >= 0; --L) {
#pragma unroll
    for (int g = 0; g < (M >> (L + 1)); ++g) {
      const uint32_t c = uniform(2u * g + (I >> (10 + L)));
#pragma unroll
      for (int v = 0; v < (1 << L); ++v) {
        const int lo = g * (2 << L) + v, hi = lo + (1 << L);
        top_mul(T, c, y[lo], y[hi]);
        y[hi].x ^= y[lo].x;
        y[hi].y ^= y[lo].y;
      }
    }
  }
}

// ---------------------------------------------------------------- encode ----
// Shard rows I .. I + 1023 of the workgroup's tile from CQ registers: tile
// (pb, columns ch0 ..), or the two payloads 2 pb, 2 pb + 1 of a paired tile.
__device__ __forceinline__ void huge_store_rows(const EncodeArgs& a, const HugeArgs& h, uint32_t pb, uint32_t ch0,
                                                uint32_t I, const uint32_t (&L)[16], const uint32_t (&H)[16],
                                                const Res& r, uint32_t ncols, bool full, bool nt) {
  if (h.pair) {
    uint8_t* o0 = a.shards + static_cast<size_t>(2 * pb) * a.batch_stride;
    uint8_t* o1 = 2 * pb + 1 < a.batch ? o0 + a.batch_stride : nullptr;
    rres_store_rows_pair(o0, o1, a.shard_len, I, a.wanted_n, L, H, r, ncols);
  } else {
    rres_store_rows(a.shards + static_cast<size_t>(pb) * a.batch_stride + 2 * static_cast<size_t>(ch0), a.shard_len,
                    I, a.wanted_n, L, H, r, ncols, full, nt);
  }
}

template <int GEN>
__device__ __forceinline__ void huge_enc_inv_body(
    DevTables T, EncodeArgs a, HugeArgs h, uint32_t nchunks) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* tile = smem;
  const SubRef sr = sub_of(h, blockIdx.x, unit_count(h, a.batch));
  const uint32_t pb = sr.pb, tl = sr.tl, ch0 = tl * kRC;
  const uint32_t ncols = min(static_cast<uint32_t>(kRC), nchunks - ch0);
  const uint32_t I = kSK * sr.u;  // sub-segment u of IFFT(k, 0)
  const Res r = res_coords<kSK>();
  const bool full = ncols == kRC && rows_vec_ok(a.shards, a.batch_stride, a.shard_len);
  const bool nt = rows_nt(a.shards, a.batch_stride, a.shard_len);
  if (h.pair) {
    const bool two = 2 * pb + 1 < a.batch;
    load_pay_tile_pair<kSK>(tile, a.payloads + static_cast<size_t>(2 * pb) * a.payload_stride,
                            two ? a.payloads + static_cast<size_t>(2 * pb + 1) * a.payload_stride : nullptr,
                            a.payload_len, 2 * static_cast<size_t>(h.K), 2 * static_cast<size_t>(I), r.tid);
  } else {
    load_pay_tile<kSK>(tile, a.payloads + static_cast<size_t>(pb) * a.payload_stride, a.payload_len, ch0,
                       2 * static_cast<size_t>(h.K), 2 * static_cast<size_t>(I), r.tid);
  }
  uint32_t* DL = reinterpret_cast<uint32_t*>(smem + RGeo<kSK>::kTileBytes);
  uint32_t* VS = DL + kDeltaWords;
  stage_delta_tables(T, DL);
  stage_rh_tables<kSK>(T, VS, 1, I);
  const Qi qc = qi_coords<kSK>(r);
  __syncthreads();
  uint32_t L[16], H[16];
  rcq_read_nat<kSK>(tile, r.cqb, L, H);
  huge_store_rows(a, h, pb, ch0, I, L, H, r, ncols, full, nt);
  tower_convert(T, L, H);
  rcq_levels<true, GEN, true, kHugePrioEnc>(T, I, r, L, H, DL);
  __syncthreads();  // every wave has read its payload blocks
  qi_cq<true>(tile, qc, L, H);
  __syncthreads();
  qi_ha<false>(tile, qc, L, H);
  ha_levels_st<kSK, true, GEN, kHugePrioEnc>(T, I, r, L, H, VS);
  __syncthreads();
  qi_ha<true>(tile, qc, L, H);
  __syncthreads();
  qi_hd<kSK, false>(tile, qc, L, H);
  hd_levels_st<kSK, true, kHugePrioEnc>(T, I, L, H, VS);
  slot_store(slot_at(h, pb, tl, sr.u), r.tid, L, H);  // HD' registers in thread order
}

// Thread (tile, j, t): the coefficients of its quads, then every shift's
// top-level outputs W_s (only sub-segments with wanted rows).
template <int M>
__global__ __launch_bounds__(256) void k_huge_enc_top(DevTables T, HugeArgs h, uint32_t nshift, uint32_t wanted_n,
                                                      size_t units) {
#if NP_BOUNDS_CHECK
  bounds_arm(BoundsSet{});  // every kernel of an instrumented unit arms its extents (none here)
#endif
  const size_t gid = static_cast<size_t>(blockIdx.x) * 256u + threadIdx.x;
  if (gid >= units) return;
  uint8_t* base = h.scr + (gid >> 14) * h.slots * kSlotBytes + (gid & 16383u) * 8u;
  uint2 c[M];
#pragma unroll
  for (int m = 0; m < M; ++m) c[m] = *reinterpret_cast<const uint2*>(base + m * static_cast<size_t>(kSlotBytes));
  top_inverse_h<M>(T, c, 0u);
#pragma unroll 1
  for (uint32_t s = 1; s < nshift && s * h.K < wanted_n; ++s) {
    uint2 w[M];
#pragma unroll
    for (int m = 0; m < M; ++m) w[m] = c[m];
    top_forward_h<M>(T, w, uniform(s * h.K));
#pragma unroll
    for (int m = 0; m < M; ++m)
      if (s * h.K + kSK * m < wanted_n)
        *reinterpret_cast<uint2*>(base + (s * M + m) * static_cast<size_t>(kSlotBytes)) = w[m];
  }
}

template <int GEN>
__device__ __forceinline__ void huge_enc_fwd_body(
    DevTables T, EncodeArgs a, HugeArgs h, uint32_t nchunks) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* tile = smem;
  const SubRef sr = sub_of(h, blockIdx.x, unit_count(h, a.batch));
  const uint32_t pb = sr.pb, tl = sr.tl, ch0 = tl * kRC;
  const uint32_t ncols = min(static_cast<uint32_t>(kRC), nchunks - ch0);
  const uint32_t I = kSK * sr.u;  // shift u / M, sub-segment u % M
  const Res r = res_coords<kSK>();
  const bool full = ncols == kRC && rows_vec_ok(a.shards, a.batch_stride, a.shard_len);
  const bool nt = rows_nt(a.shards, a.batch_stride, a.shard_len);
  uint32_t* DL = reinterpret_cast<uint32_t*>(smem + RGeo<kSK>::kTileBytes);
  uint32_t* VS = DL + kDeltaWords;
  stage_delta_tables(T, DL);
  stage_rh_tables<kSK>(T, VS, 1, I);
  const Qi qc = qi_coords<kSK>(r);
  uint32_t L[16], H[16];
  slot_load(slot_at(h, pb, tl, sr.u), r.tid, L, H);
  __syncthreads();  // the staged tables
  hd_levels_st<kSK, false, kHugePrioEnc>(T, I, L, H, VS);
  qi_hd<kSK, true>(tile, qc, L, H);
  __syncthreads();
  qi_ha<false>(tile, qc, L, H);
  ha_levels_st<kSK, false, GEN, kHugePrioEnc>(T, I, r, L, H, VS);
  __syncthreads();
  qi_ha<true>(tile, qc, L, H);
  __syncthreads();
  qi_cq<false>(tile, qc, L, H);
  rcq_levels<false, GEN, true, kHugePrioEnc>(T, I, r, L, H, DL);
  tower_convert(T, L, H);  // back to Cantor coordinates for the shard rows
  huge_store_rows(a, h, pb, ch0, I, L, H, r, ncols, full, nt);
}

// ----------------------------------------------------------- reconstruct ----
// Status (mod.rs:178-180) and mode of each payload: fewer than k present rows:
// skip; all k systematic rows present: their copy (inc_reconstruct.rs:46-50);
// else the full decode from every present row.
// Thread t counts the present flags of rows 4 (t + 256 i) .. + 3 (one dword
// each; n is a multiple of 1024), then one block sum.
// Iteration i covers block i (rows 1024 i .. + 1023): its occupancy bit.
__global__ __launch_bounds__(256) void k_huge_records(ReconstructArgs a, uint8_t* mode, uint64_t* occ) {
#if NP_BOUNDS_CHECK
  bounds_arm(BoundsSet{});
#endif
  __shared__ int part[2][4];
  const uint32_t pb = blockIdx.x;
  const uint8_t* pres = a.present + static_cast<size_t>(pb) * a.n;
  int c1 = 0, c = 0;
  uint64_t oc = 0;
  for (uint32_t v = 4u * threadIdx.x, i = 0; v < a.n; v += 1024u, ++i) {
    const uint32_t w = *reinterpret_cast<const uint32_t*>(pres + v);  // the flags are 0 / 1 bytes
    const int cnt = ((w & 0xffu) != 0) + ((w & 0xff00u) != 0) + ((w & 0xff0000u) != 0) + ((w >> 24) != 0);
    c += cnt;
    if (v < a.k) c1 += cnt;
    if (__syncthreads_or(cnt)) oc |= 1ull << i;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    c += __shfl_xor(c, o);
    c1 += __shfl_xor(c1, o);
  }
  if ((threadIdx.x & 63u) == 0) part[0][threadIdx.x >> 6] = c1, part[1][threadIdx.x >> 6] = c;
  __syncthreads();
  const int have1 = part[0][0] + part[0][1] + part[0][2] + part[0][3];
  const int have = part[1][0] + part[1][1] + part[1][2] + part[1][3];
  const bool ok = have >= static_cast<int>(a.k);
  if (threadIdx.x == 0) {
    if (a.status) {
      a.status[2 * pb] = ok ? 0u : kStatusNeedMoreShards;
      a.status[2 * pb + 1] = static_cast<uint32_t>(have);
    }
    mode[pb] = !ok ? kHugeSkip : have1 == static_cast<int>(a.k) ? kHugeCopy : kHugeDecode;
    occ[pb] = oc;
  }
}

template <int GEN>
__device__ __forceinline__ void huge_rec_inv_body(
    DevTables T, ReconstructArgs a, HugeArgs h, uint32_t nsyms) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* tile = smem;
  const SubRef sr = sub_of(h, blockIdx.x, unit_count(h, a.batch));
  const uint32_t pb = sr.pb, tl = sr.tl;  // pb: the pair of payloads 2 pb, 2 pb + 1 (HugeArgs::pair)
  if (uniform(tile_mode(h, static_cast<size_t>(pb) * h.tiles + tl)) != kHugeDecode) return;
  // no present row: the slot is zero (k_huge_rec_top reads none)
  if (!((uniform64(tile_occ(h, static_cast<size_t>(pb) * h.tiles + tl)) >> sr.u) & 1u)) return;
  const uint32_t col0 = tl * kRC, ncols = min(static_cast<uint32_t>(kRC), nsyms - col0);
  const uint32_t I = kSK * sr.u;  // rows I .. I + 1023: segment u / M, sub-segment u % M
  const Res r = res_coords<kSK>();
  uint32_t* DL = reinterpret_cast<uint32_t*>(smem + RGeo<kSK>::kTileBytes);
  uint32_t* VS = DL + kDeltaWords;
  uint32_t XL[16], XH[16];
  if (h.pair) {
    // lane 16 u + cq: payload 2 pb + (cq >> 3), columns 4 (cq & 7) ..; the two
    // payloads' row tables in two halves of 8 rows per lane
    const bool two = 2 * pb + 1 < a.batch;
    const uint32_t sel = r.cq >> 3, pbl = 2 * pb + sel;
    const bool valid = sel == 0 || two;
    const size_t n = a.n;
    const uint8_t* pres0 = a.present + static_cast<size_t>(2 * pb) * n;
    const uint8_t* pres1 = two ? pres0 + n : nullptr;
    const uint16_t* loc0 = h.loc + static_cast<size_t>(2 * pb) * n;
    const uint16_t* loc1 = two ? loc0 + n : nullptr;
    const uint32_t pm = valid ? lane_rows_present(a.present + static_cast<size_t>(pbl) * n, I, r) : 0u;
    const uint8_t* sh = a.shards + static_cast<size_t>(valid ? pbl : 2 * pb) * a.batch_stride;
    Res rl = r;
    rl.cq = r.cq & 7u;
    uint2 raw[8];
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      load_lane_rows<8>(raw, sh, a.shard_len, I, pm, rl, ncols, false, T.zeros, 8 * hf);
      if (hf == 1) __syncthreads();  // every wave is done with half 0's tables
      stage_row_tables_pair(tile, T, loc0, pres0, loc1, pres1, I, hf, r.tid, false);
      if (hf == 0) {
        stage_delta_tables(T, DL);
        stage_rh_tables<kSK>(T, VS, 1, I);
      }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        uint32_t l, hh;
        blk_to_quad(raw[i], l, hh);
        const FullT m = row_table_at(tile, pair_row_slot(sel, 4u * r.w + r.u, i));
        qmul_set_vv(XL[8 * hf + i], XH[8 * hf + i], l, hh, m);
      }
    }
  } else {
    const uint8_t* pres = a.present + static_cast<size_t>(pb) * a.n;
    const uint16_t* loc = h.loc + static_cast<size_t>(pb) * a.n;
    const uint8_t* sh = a.shards + static_cast<size_t>(pb) * a.batch_stride + 2 * static_cast<size_t>(col0);
    const bool full = ncols == kRC && rows_vec_ok(a.shards, a.batch_stride, a.shard_len);
    const uint32_t pm = lane_rows_present(pres, I, r);
    uint2 raw[8];
    load_lane_rows<8>(raw, sh, a.shard_len, I, pm, r, ncols, full, T.zeros, 0);
    stage_row_tables_loc(tile, T, loc, pres, I, r.tid, false);
    stage_delta_tables(T, DL);
    stage_rh_tables<kSK>(T, VS, 1, I);
    __syncthreads();
    // premultiply (inc_reconstruct.rs:72-74; Cantor in, tower out), two halves
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      if (half == 1) load_lane_rows<8>(raw, sh, a.shard_len, I, pm, r, ncols, full, T.zeros, 8);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        uint32_t l, hh;
        blk_to_quad(raw[i], l, hh);
        const FullT m = row_table(tile, 64u * r.w + 16u * r.u + 8 * half + i);
        qmul_set_vv(XL[8 * half + i], XH[8 * half + i], l, hh, m);
      }
    }
  }
  rcq_levels<true, GEN, true, kHugePrioDec>(T, I, r, XL, XH, DL);
  __syncthreads();  // every wave has read its row tables
  rcq_write<kSK>(tile, fresh_v(r.cqb), XL, XH);
  __syncthreads();
  rh_read<kHA>(tile, fresh_v(r.hab), XL, XH);
  ha_levels_st<kSK, true, GEN, kHugePrioDec>(T, I, r, XL, XH, VS);
  __syncthreads();
  rh_write<kHA>(tile, fresh_v(r.hab), XL, XH);
  __syncthreads();
  rh_read<kHDS>(tile, fresh_v(r.hdb), XL, XH);
  hd_levels_st<kSK, true, kHugePrioDec>(T, I, XL, XH, VS);
  slot_store(slot_at(h, pb, tl, sr.u), r.tid, XL, XH);
  if (sr.u < h.M) {  // z = D_1024 of segment 0's sub-transform (the lifted low part of D_k)
    uint32_t AL[16], AH[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) AL[j] = AH[j] = 0;
    add_derivative_hd<kSK>(AL, XL, r.l);
    add_derivative_hd<kSK>(AH, XH, r.l);
    slot_store(slot_at(h, pb, tl, h.NQ * h.M + sr.u), r.tid, AL, AH);
  }
}

// Fold coefficients kappa_q (Cantor coordinates, kernels_fast.hip):
// NQ = 2: (1, 1); NQ = 4: (0, 1, 1 + beta, beta), beta = Cantor(2); NQ = 8:
// rec8_kappa.
template <int NQ>
__host__ __device__ constexpr uint32_t huge_kappa(int q) {
  return NQ == 2 ? 1u : NQ == 4 ? (q == 0 ? 0u : q == 1 ? 1u : q == 2 ? 3u : 2u) : rec8_kappa_res(q);
}

template <int M, int NQ>
__global__ __launch_bounds__(256) void k_huge_rec_top(DevTables T, HugeArgs h, size_t units) {
#if NP_BOUNDS_CHECK
  bounds_arm(BoundsSet{});
#endif
  const size_t gid = static_cast<size_t>(blockIdx.x) * 256u + threadIdx.x;
  if (gid >= units) return;
  const size_t pt = gid >> 14;  // tile of the slice
  if (uniform(tile_mode(h, pt)) != kHugeDecode) return;
  uint8_t* base = h.scr + pt * h.slots * kSlotBytes + (gid & 16383u) * 8u;
  auto at = [&](uint32_t slot) __attribute__((always_inline)) { return base + static_cast<size_t>(slot) * kSlotBytes; };
  // blocks without a present row: zero slots that k_huge_rec_inv skipped
  const uint64_t oc = uniform64(tile_occ(h, pt));
  auto ld = [&](uint32_t u, uint32_t slot) __attribute__((always_inline)) {
    return ((oc >> u) & 1u) ? *reinterpret_cast<const uint2*>(at(slot)) : make_uint2(0u, 0u);
  };
  uint2 d[M], x[M];
  // x_0 and the lifted D_1024(y_0)
#pragma unroll
  for (int m = 0; m < M; ++m) {
    x[m] = ld(m, m);
    d[m] = ld(m, NQ * M + m);
  }
  top_inverse_h<M>(T, x, 0u);
  top_inverse_h<M>(T, d, 0u);
  // D_k's high single-bit terms: position 1024 m + p' takes x_0 at 1024 (m | 2^L) + p'
#pragma unroll
  for (int m = 0; m < M; ++m)
#pragma unroll
    for (int L = 0; (1 << L) < M; ++L)
      if (!(m & (1 << L))) {
        d[m].x ^= x[m | (1 << L)].x;
        d[m].y ^= x[m | (1 << L)].y;
      }
  if constexpr (huge_kappa<NQ>(0) == 1u) {
#pragma unroll
    for (int m = 0; m < M; ++m) d[m].x ^= x[m].x, d[m].y ^= x[m].y;
  }
#pragma unroll
  for (int q = 1; q < NQ; ++q) {
    if (!((oc >> (q * M)) & ((1ull << M) - 1u))) continue;  // x_q = 0
#pragma unroll
    for (int m = 0; m < M; ++m) x[m] = ld(q * M + m, q * M + m);
    top_inverse_h<M>(T, x, uniform(q * h.K));
    const uint32_t kq = huge_kappa<NQ>(q);
    if (kq == 1u) {
#pragma unroll
      for (int m = 0; m < M; ++m) d[m].x ^= x[m].x, d[m].y ^= x[m].y;
    } else {
#pragma unroll
      for (int m = 0; m < M; ++m) top_mul(T, kq, d[m], x[m]);
    }
  }
  top_forward_h<M>(T, d, 0u);
#pragma unroll
  for (int m = 0; m < M; ++m) *reinterpret_cast<uint2*>(at(m)) = d[m];
}

template <int GEN>
__device__ __forceinline__ void huge_rec_fwd_body(
    DevTables T, ReconstructArgs a, HugeArgs h, uint32_t nsyms) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* tile = smem;
  const SubRef sr = sub_of(h, blockIdx.x, unit_count(h, a.batch));
  const uint32_t pb = sr.pb, tl = sr.tl;  // pb: the pair 2 pb, 2 pb + 1 (HugeArgs::pair)
  const uint32_t mode = uniform(tile_mode(h, static_cast<size_t>(pb) * h.tiles + tl));
  if (mode == kHugeSkip) return;
  const uint32_t col0 = tl * kRC, ncols = min(static_cast<uint32_t>(kRC), nsyms - col0);
  const uint32_t I = kSK * sr.u;  // output rows I .. I + 1023
  const bool out16 = out_vec_ok(a.out, a.out_stride);
  const Res r = res_coords<kSK>();
  uint32_t AL[16], AH[16];
  if (mode == kHugeDecode) {
    uint32_t* DL = reinterpret_cast<uint32_t*>(smem + RGeo<kSK>::kTileBytes);
    uint32_t* VS = DL + kDeltaWords;
    stage_delta_tables(T, DL);
    stage_rh_tables<kSK>(T, VS, 1, I);
    slot_load(slot_at(h, pb, tl, sr.u), r.tid, AL, AH);
    __syncthreads();  // the staged tables
    hd_levels_st<kSK, false, kHugePrioDec>(T, I, AL, AH, VS);
    rh_write<kHDS>(tile, fresh_v(r.hdb), AL, AH);
    __syncthreads();
    rh_read<kHA>(tile, fresh_v(r.hab), AL, AH);
    ha_levels_st<kSK, false, GEN, kHugePrioDec>(T, I, r, AL, AH, VS);
    __syncthreads();
    rh_write<kHA>(tile, fresh_v(r.hab), AL, AH);
    __syncthreads();
    rcq_read<kSK>(tile, fresh_v(r.cqb), AL, AH);
    rcq_levels<false, GEN, true, kHugePrioDec>(T, I, r, AL, AH, DL);
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j) AL[j] = AH[j] = 0;
  }
  // merge: received systematic rows, postmultiplied recovered ones
  // (inc_reconstruct.rs:46-50, :82-84; tower in, Cantor out)
  if (h.pair) {
    // lane 16 u + cq: payload 2 pb + (cq >> 3), whose own mode decides
    // whether it writes (a copy-mode payload has every systematic row
    // present, so the merge takes them all; a skipped one writes nothing)
    const bool two = 2 * pb + 1 < a.batch;
    const uint32_t sel = r.cq >> 3, pbl = 2 * pb + sel;
    const bool valid = sel == 0 || two;
    const size_t n = a.n;
    const uint8_t* pres0 = a.present + static_cast<size_t>(2 * pb) * n;
    const uint8_t* pres1 = two ? pres0 + n : nullptr;
    const uint16_t* loc0 = h.loc + static_cast<size_t>(2 * pb) * n;
    const uint16_t* loc1 = two ? loc0 + n : nullptr;
    const bool writes = valid && h.mode[pbl] != kHugeSkip;
    const uint32_t pm = valid ? lane_rows_present(a.present + static_cast<size_t>(pbl) * n, I, r) : 0u;
    Res rl = r;
    rl.cq = r.cq & 7u;
    uint2 raw[16];
    load_lane_rows(raw, a.shards + static_cast<size_t>(valid ? pbl : 2 * pb) * a.batch_stride, a.shard_len, I, pm, rl,
                   ncols, false, T.zeros);
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      if (mode == kHugeDecode) {
        __syncthreads();  // every wave has read the tile (hf = 0) / half 0's tables (hf = 1)
        stage_row_tables_pair(tile, T, loc0, pres0, loc1, pres1, I, hf, r.tid, true);
        __syncthreads();
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int x = 8 * hf + i;
        uint32_t l, hh;
        if ((pm >> x) & 1u) {
          blk_to_quad(raw[x], l, hh);
        } else {
          const FullT m = row_table_at(tile, pair_row_slot(sel, 4u * r.w + r.u, i));
          qmul_set_vv(l, hh, AL[x], AH[x], m);
        }
        AL[x] = l;
        AH[x] = hh;
      }
    }
    if (writes)
      res_copy_out<kSK>(a.out + static_cast<size_t>(pbl) * a.out_stride + 2 * I, AL, AH, rl, ncols, out16,
                        2 * static_cast<size_t>(h.K));
    return;
  }
  const uint8_t* pres = a.present + static_cast<size_t>(pb) * a.n;
  const uint8_t* sh = a.shards + static_cast<size_t>(pb) * a.batch_stride + 2 * static_cast<size_t>(col0);
  const bool full = ncols == kRC && rows_vec_ok(a.shards, a.batch_stride, a.shard_len);
  const uint32_t pm = lane_rows_present(pres, I, r);
  uint2 raw[16];
  load_lane_rows(raw, sh, a.shard_len, I, pm, r, ncols, full, T.zeros);
  __syncthreads();  // every wave has read the tile
  if (mode == kHugeDecode) stage_row_tables_loc(tile, T, h.loc + static_cast<size_t>(pb) * a.n, pres, I, r.tid, true);
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    uint32_t l, hh;
    if ((pm >> i) & 1u) {
      blk_to_quad(raw[i], l, hh);
    } else {
      const FullT m = row_table(tile, 64u * r.w + 16u * r.u + i);
      qmul_set_vv(l, hh, AL[i], AH[i], m);
    }
    AL[i] = l;
    AH[i] = hh;
  }
  res_copy_out<kSK>(a.out + static_cast<size_t>(pb) * a.out_stride + static_cast<size_t>(col0) * 2 * h.K + 2 * I, AL, AH,
                    r, ncols, out16, 2 * static_cast<size_t>(h.K));
}

// One launch per phase: workgroup b's sub-transform u picks its GEN
// (res_gen<1024>(1024 u)) at run time; the bodies are the same code as one
// launch per GEN range had run, without the launches' ramps and tails.
template <typename F>
__device__ __forceinline__ void with_gen_dev(uint32_t u, F&& f) {
  switch (res_gen<kSK>(kSK * u)) {
    case 2: f(Int<2>{}); break;
    case 3: f(Int<3>{}); break;
    case 4: f(Int<4>{}); break;
    case 5: f(Int<5>{}); break;
    case 6: f(Int<6>{}); break;
    case 7: f(Int<7>{}); break;
    default: f(Int<8>{}); break;
  }
}
#define NP_HUGE_PHASE(NAME, ARGS, CALL)                                                                              \
  __global__ __launch_bounds__(kSK) __attribute__((amdgpu_waves_per_eu(4))) void k_##NAME ARGS {                     \
    NP_HUGE_ARM();                                                                                                   \
    with_gen_dev(uniform(h.u0 + blockIdx.x / h.per), [&](auto g) { NAME##_body<decltype(g)::value> CALL; });       \
  }
#if NP_BOUNDS_CHECK
#define NP_HUGE_ARM() bounds_arm(bounds_for(a, T))
#else
#define NP_HUGE_ARM() ((void)0)
#endif
NP_HUGE_PHASE(huge_enc_inv, (DevTables T, EncodeArgs a, HugeArgs h, uint32_t nchunks), (T, a, h, nchunks))
NP_HUGE_PHASE(huge_enc_fwd, (DevTables T, EncodeArgs a, HugeArgs h, uint32_t nchunks), (T, a, h, nchunks))
NP_HUGE_PHASE(huge_rec_inv, (DevTables T, ReconstructArgs a, HugeArgs h, uint32_t nsyms), (T, a, h, nsyms))
NP_HUGE_PHASE(huge_rec_fwd, (DevTables T, ReconstructArgs a, HugeArgs h, uint32_t nsyms), (T, a, h, nsyms))
#undef NP_HUGE_PHASE

// ------------------------------------------------------------ dispatch ----
template <typename F>
hipError_t with_m(uint32_t M, F&& f) {
  switch (M) {
    case 2: return f(Int<2>{});
    case 4: return f(Int<4>{});
    case 8: return f(Int<8>{});
    case 16: return f(Int<16>{});
    default: return hipErrorInvalidValue;
  }
}
template <typename F>
hipError_t with_nq(uint32_t NQ, F&& f) {
  switch (NQ) {
    case 2: return f(Int<2>{});
    case 4: return f(Int<4>{});
    case 8: return f(Int<8>{});
    default: return hipErrorInvalidValue;
  }
}

// NP_HUGE_PAIR=0 (experiment knob, read once): one payload per tile always.
bool huge_pair_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("NP_HUGE_PAIR");
    return !(e && e[0] == '0');
  }();
  return on;
}

HugeArgs huge_args(uint8_t* scr, uint32_t n, uint32_t k, size_t tiles, uint32_t slots) {
  HugeArgs h{};
  h.scr = scr;
  h.tiles = static_cast<uint32_t>(tiles);
  h.slots = slots;
  h.K = k;
  h.M = k / kSK;
  h.NQ = n / k;
  return h;
}

}  // namespace

bool huge_encode_supported(uint32_t n, uint32_t k) { return k >= 2048 && k <= 16384 && n >= 2 * k && n <= 65536; }
bool huge_reconstruct_supported(uint32_t n, uint32_t k) {
  return k >= 2048 && k <= 16384 && (n == 2 * k || n == 4 * k || n == 8 * k) && n <= 65536;
}
size_t huge_encode_scratch_per_payload(size_t shard_len, uint32_t n, uint32_t k) {
  (void)k;
  const size_t tiles = (shard_len / 2 + kRC - 1) / kRC;
  return tiles * (n / kSK) * static_cast<size_t>(kSlotBytes);
}
// Tile slots of a slice of `batch` payloads of `cols` columns each, as the
// launchers lay them out: two payloads per tile when they pair them.
size_t huge_slice_units(size_t batch, size_t cols) {
  const bool pair = huge_pair_enabled() && cols <= kRC / 2 && batch > 1;
  return pair ? (batch + 1) / 2 : batch * ((cols + kRC - 1) / kRC);
}
size_t huge_encode_scratch(size_t batch, size_t payload_len, uint32_t n, uint32_t k) {
  return huge_slice_units(batch, (payload_len + 2 * k - 1) / (2 * k)) * (n / kSK) * static_cast<size_t>(kSlotBytes);
}
size_t huge_reconstruct_scratch(size_t batch, size_t shard_len, uint32_t n, uint32_t k) {
  return huge_slice_units(batch, shard_len / 2) * ((n + k) / kSK) * static_cast<size_t>(kSlotBytes);
}
size_t huge_reconstruct_scratch_per_payload(size_t shard_len, uint32_t n, uint32_t k) {
  const size_t tiles = (shard_len / 2 + kRC - 1) / kRC;
  return tiles * ((n + k) / kSK) * static_cast<size_t>(kSlotBytes);
}

hipError_t launch_encode_huge(const DevTables& T, const EncodeArgs& a, uint8_t* scratch, hipStream_t s) {
  if (!huge_encode_supported(a.n, a.k)) return hipErrorInvalidValue;
  const size_t nchunks = (a.payload_len + 2 * a.k - 1) / (2 * a.k);
  if (nchunks == 0 || a.batch == 0) return hipSuccess;
  if (nchunks > 0xffffffffu) return hipErrorInvalidValue;
  const size_t tiles = (nchunks + kRC - 1) / kRC;
  // payloads of at most 32 columns (k = 16384 at 1 MiB): two per tile
  const bool pair = huge_pair_enabled() && nchunks <= kRC / 2 && a.batch > 1;
  const size_t per = pair ? (a.batch + 1) / 2 : a.batch * tiles;
  if (per * (a.n / kSK) > 0x7fffffffu) return hipErrorInvalidValue;
  const uint32_t nc = static_cast<uint32_t>(nchunks);
  HugeArgs h = huge_args(scratch, a.n, a.k, tiles, a.n / kSK);
  h.per = static_cast<uint32_t>(per);
  h.pair = pair ? 1u : 0u;
  auto grid = [&](uint32_t u0, uint32_t u1) { return static_cast<uint32_t>(per * (u1 - u0)); };
  h.u0 = 0;
  k_huge_enc_inv<<<grid(0, h.M), kSK, kHugeLds, s>>>(T, a, h, nc);
  hipError_t e = hipGetLastError();
  const size_t units = per * 16 * kSK;
  if (e == hipSuccess)
    e = with_m(h.M, [&](auto mc) {
      k_huge_enc_top<decltype(mc)::value><<<static_cast<uint32_t>(units / 256), 256, 0, s>>>(T, h, h.NQ, a.wanted_n, units);
      return hipGetLastError();
    });
  // parity sub-segments holding wanted rows: u in [M, ceil(wanted_n / 1024))
  const uint32_t u_end = std::min(a.n, a.wanted_n + kSK - 1) / kSK;
  if (e == hipSuccess && u_end > h.M) {
    h.u0 = h.M;
    k_huge_enc_fwd<<<grid(h.M, u_end), kSK, kHugeLds, s>>>(T, a, h, nc);
    e = hipGetLastError();
  }
  return e;
}

hipError_t launch_reconstruct_huge(const DevTables& T, const ReconstructArgs& a, uint8_t* scratch, uint8_t* mode,
                                   uint16_t* locators, hipStream_t s) {
  if (!huge_reconstruct_supported(a.n, a.k)) return hipErrorInvalidValue;
  const size_t nsyms = a.shard_len / 2;
  if (a.batch == 0) return hipSuccess;
  if (a.batch > 0x7fffffffu || nsyms > 0xffffffffu) return hipErrorInvalidValue;
  uint64_t* occ = reinterpret_cast<uint64_t*>(mode + (a.batch + 15) / 16 * 16);
  k_huge_records<<<static_cast<uint32_t>(a.batch), 256, 0, s>>>(a, mode, occ);
  hipError_t e = hipGetLastError();
  if (nsyms == 0 || e != hipSuccess) return e;
  const uint16_t* loc = a.locators;
  if (!loc) {
    e = launch_error_locator(T, a.n, a.present, a.batch, locators, s);
    loc = locators;
  }
  const size_t tiles = (nsyms + kRC - 1) / kRC;
  // payloads of at most 32 columns: two per tile, as the encode
  const bool pair = huge_pair_enabled() && nsyms <= kRC / 2 && a.batch > 1;
  const size_t per = pair ? (a.batch + 1) / 2 : a.batch * tiles;
  if (per * (a.n / kSK) > 0x7fffffffu) return hipErrorInvalidValue;
  const uint32_t ns = static_cast<uint32_t>(nsyms);
  HugeArgs h = huge_args(scratch, a.n, a.k, tiles, (a.n + a.k) / kSK);
  h.loc = loc;
  h.mode = mode;
  h.occ = occ;
  h.per = static_cast<uint32_t>(per);
  h.pair = pair ? 1u : 0u;
  h.batch = static_cast<uint32_t>(a.batch);
  auto grid = [&](uint32_t u0, uint32_t u1) { return static_cast<uint32_t>(per * (u1 - u0)); };
  if (e == hipSuccess) {
    h.u0 = 0;
    k_huge_rec_inv<<<grid(0, a.n / kSK), kSK, kHugeLds, s>>>(T, a, h, ns);
    e = hipGetLastError();
  }
  const size_t units = per * 16 * kSK;
  if (e == hipSuccess)
    e = with_m(h.M, [&](auto mc) {
      return with_nq(h.NQ, [&](auto qc) {
        k_huge_rec_top<decltype(mc)::value, decltype(qc)::value>
            <<<static_cast<uint32_t>(units / 256), 256, 0, s>>>(T, h, units);
        return hipGetLastError();
      });
    });
  if (e == hipSuccess) {
    h.u0 = 0;
    k_huge_rec_fwd<<<grid(0, h.M), kSK, kHugeLds, s>>>(T, a, h, ns);
    e = hipGetLastError();
  }
  return e;
}

hipError_t configure_huge_kernels() {
  hipError_t e = hipSuccess;
  auto set = [&](const void* f) {
    const hipError_t r = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(kHugeLds));
    if (r != hipSuccess && e == hipSuccess) e = r;
  };
  set(reinterpret_cast<const void*>(&k_huge_enc_inv));
  set(reinterpret_cast<const void*>(&k_huge_enc_fwd));
  set(reinterpret_cast<const void*>(&k_huge_rec_inv));
  set(reinterpret_cast<const void*>(&k_huge_rec_fwd));
  return e;
}

hipError_t bounds_take_huge(uint32_t out[8]) { return bounds_take_tu(out); }

}  // namespace np
