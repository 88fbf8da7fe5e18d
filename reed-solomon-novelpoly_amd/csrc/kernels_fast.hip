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
#include <algorithm>
#include <cstdlib>

#include "fast_common.hpp"
// (The next tile's payload is read once: its LDS-DMA loads stream (nt),
// keeping L2 for the tables and the row stores; config 3 encode -4 %.)

namespace np {
namespace {

// ----------------------------------------------------------------- encode ----
// Encode shifts run in tower coordinates while gen_of(index) <= kEncMaxGen
// (index < 2048: n <= 8K at k = 256, every n the crate derives), their levels
// below gen_of(index) with the full map; farther shifts of larger explicit
// codes run in Cantor coordinates.
constexpr int kEncMaxGen = 3;
__device__ __forceinline__ bool enc_tower(uint32_t index) {
  return __builtin_amdgcn_readfirstlane(gen_of(index)) <= static_cast<uint32_t>(kEncMaxGen);
}

// Shifts 1..3 are compile-time (SH): tower coordinates, the top-level products
// shared between them (fwd_top), their cq levels below gen_of(SH * K) with the
// full map.  SH = 23: shift 2 or 3 (runtime sh; both have gen_of = 2 at
// K = 256).  SH = 0: a shift >= 4 (n > 4K) in Cantor coordinates.  A runtime
// choice between instances inside a pass makes the register allocator spill,
// so each call site is one instance.
// Issue priority (s_setprio, fast_common.hpp progress_prio; DESIGN.md §4.2,
// §4.3).  Encode: every transform pass by progress (priority 3 in its first
// quarter of butterfly groups down to 0 in the last): config-3 encode 1.601 /
// 1.602 -> 1.514 / 1.527 ms (-5 %, profiles/r04_ab.txt probe 18).  Decode: one
// schedule over each barrier-free span of the segment sweep (high levels of
// step s, fold, premultiply and cq levels of step s + 1): priority 2 in the
// high levels (progress schedule 2), 2 in the premultiply, 3 then 0 in the cq
// levels: config-3 reconstruct -3.2 % (probe 21); the forward transform's
// spans likewise (its high levels 3, its cq levels and the merge 2): -1.7 %
// (probe 22).  Per-pass priority in the decode measured +1.5 to +2.8 %, the
// encode's span schedule neutral, premultiply priorities 1 and 3 and high-level
// schedule 4 within noise (probes 24, 26).
constexpr int kEncPrio = 1, kEncPrioCq = 1;
constexpr int kRecPrioPremul = 2, kRecPrioCq = 3, kRecPrioHi = 2, kRecPrioFwdHi = 3, kRecPrioFwdCq = 2;

template <int K, int SH>
constexpr int kShiftGen = static_cast<int>(gen_of((SH == 23 ? 2 : SH) * K));

// X = M, then the forward high levels of shift sh (top level included).
template <int K, int SH, typename HOOK = NoHiHook>
__device__ __forceinline__ void shift_hi(const DevTables& T, const uint32_t* vp, uint32_t index,
                                         const uint32_t (&ML)[16], const uint32_t (&MH)[16], uint32_t (&XL)[16],
                                         uint32_t (&XH)[16], uint32_t (&PL)[8], uint32_t (&PH)[8], HOOK hook = HOOK{}) {
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    XL[q] = ML[q];
    XH[q] = MH[q];
  }
  if constexpr (SH == 0) {
    tower_convert(T, XL, XH);  // M is in tower coordinates
    fwd_top<K, 0, -1>(T, vp, index, XL, XH, PL, PH);
    hi_levels<K, false, false, 1, -1, kEncPrio>(T, vp, index, XL, XH);
  } else {
    if constexpr (SH == 23) {
      if (index == 2 * K)
        fwd_top<K, 2, 0>(T, vp, index, XL, XH, PL, PH);
      else
        fwd_top<K, 3, 0>(T, vp, index, XL, XH, PL, PH);
    } else {
      fwd_top<K, SH, 0>(T, vp, index, XL, XH, PL, PH);
    }
    hi_levels<K, false, false, 1, 0, kEncPrio>(T, vp, index, XL, XH, hook);  // hi levels: gen_of(index) <= 4
  }
}

// Shifts whose level 0 multiplies by full elements (gen_of(sK) >= 1: every
// shift at k = 256) leave the tower inside that level (cq_levels CONV,
// qbfly_fwd_conv) instead of converting the 16 rows after it.  Measured:
// config-3 encode 1.656 / 1.663 -> 1.629 / 1.631 ms (-1.8 %, profiles/r04_ab.txt).
// Whether shift sh of a size-K encode fuses its conversion; the staging of its
// tables must agree (stage_vpools l0_out).  SH = 23 stands for shifts 2 and 3.
__host__ __device__ constexpr bool enc_conv(int K, uint32_t sh) {
  return sh >= 1 && sh <= 3 && gen_of(sh * static_cast<uint32_t>(K)) >= 1;
}
template <int K, int SH>
constexpr bool kEncConv = SH != 0 && enc_conv(K, SH == 23 ? 2u : static_cast<uint32_t>(SH));

// The forward cq levels of shift sh, ending in Cantor coordinates.
template <int K, int SH, typename POST = NoPost>
__device__ __forceinline__ void shift_cq(const DevTables& T, const uint32_t* vp, uint32_t index, uint32_t g,
                                         uint32_t (&XL)[16], uint32_t (&XH)[16], POST post = POST{}) {
  if constexpr (SH == 0) {
    cq_levels<K, false, false, -1, false, kEncPrioCq>(T, vp, index, g, XL, XH, ~0u, post);
  } else {
    static_assert(SH != 23 || kShiftGen<K, 2> == kShiftGen<K, 3>, "shifts 2 and 3 share one instance");
    static_assert(SH != 23 || enc_conv(K, 2) == enc_conv(K, 3), "shifts 2 and 3 share one instance");
    cq_levels<K, false, false, kShiftGen<K, SH>, kEncConv<K, SH>, kEncPrioCq>(T, vp, index, g, XL, XH, ~0u, post);
    if constexpr (!kEncConv<K, SH>) tower_convert(T, XL, XH);  // back to Cantor coordinates for the shard rows
  }
}

// The fast encodes exchange layouts through quad items (cq_write_q ..
// hi_read_q, fast_common.hpp): no byte transposes.  The multi-tile encode
// writes each shift's high-layout quads to LDS right after their last
// (level-4) butterfly group instead of after the whole high pass: encode
// -1.9 % at config 3 (1.686 -> 1.655 ms, profiles/r04_ab.txt).

// One workgroup: 256 chunks of one payload.  mod.rs:144-154 / inc_encode.rs:15-48.
template <int K>
__global__ __launch_bounds__(4 * K) __attribute__((amdgpu_waves_per_eu(4))) void k_encode_fast(DevTables T, EncodeArgs a, uint32_t nchunks, uint32_t tiles) {
  using G = Geo<K>;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* tile = smem;
  uint32_t* VP = reinterpret_cast<uint32_t*>(smem + G::kTileBytes);  // 2 staged transforms
#if NP_BOUNDS_CHECK
  bounds_arm(bounds_of_enc(a));
#endif
  const TileRef tr = tile_of(blockIdx.x, tiles, (a.batch & 7u) == 0);
  const uint32_t pb = tr.pb, tl = tr.tl;
  const uint32_t ch0 = tl * kTile;
  const uint32_t ncols = min(static_cast<uint32_t>(kTile), nchunks - ch0);
  const uint8_t* pay = a.payloads + static_cast<size_t>(pb) * a.payload_stride;
  uint8_t* out = a.shards + static_cast<size_t>(pb) * a.batch_stride + 2 * static_cast<size_t>(ch0);
  const uint32_t tid = threadIdx.x, lane = tid & 63u, g = uniform(tid >> 6);
  const bool full =
      ncols == kTile && rows_vec_ok(a.shards, a.batch_stride, a.shard_len);

  // ---- tile load: thread tid moves blocks (c0 + 16 i, m0), i = 0..15
  {
    const uint32_t c0 = tid / G::Q, m0 = tid % G::Q;
    const uint32_t base = col_base<K>(c0) ^ (8u * m0);
    const size_t gbase = static_cast<size_t>(ch0 + c0) * 2 * K + 8u * m0;
    const bool fast = out_vec_ok(pay, 0) && static_cast<size_t>(ch0 + kTile) * 2 * K <= a.payload_len;
    if (fast) {
      uint2 v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i)
        v[i] = (kExp & 4) ? make_uint2(i, tid) : load_once(pay + gbase + static_cast<size_t>(i) * 32 * K);
#pragma unroll
      for (int i = 0; i < 16; ++i) *reinterpret_cast<uint2*>(tile + (base ^ col_base_c<K>(16u * i))) = v[i];
    } else {
#pragma unroll 1
      for (uint32_t i = 0; i < 16; ++i) {
        const size_t g0 = gbase + static_cast<size_t>(i) * 32 * K;
        uint32_t w[2] = {0, 0};
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (g0 + e < a.payload_len) w[e >> 2] |= static_cast<uint32_t>(*NP_BCHK(pay + (g0 + e), 1, kBkPayloads)) << (8 * (e & 3));
        *reinterpret_cast<uint2*>(tile + (base ^ col_base_c<K>(16u * i))) = make_uint2(w[0], w[1]);
      }
    }
  }
  const uint32_t nshift = a.n / K;
  const bool nt = rows_nt(a.shards, a.batch_stride, a.shard_len);
  const uint32_t wanted_store = ((kExp & 2) && a.k != 12345u) ? 0u : a.wanted_n;  // experiment: no stores
  // n <= 4K: the tables of every transform stay staged (one buffer each, as
  // k_encode_multi: no table load inside the shift loop, where it would wait
  // for the row stores issued before it); otherwise two buffers alternate
  const bool resident = nshift <= 4;
  if (resident) {
    for (uint32_t sh = 0; sh < nshift && sh * K < a.wanted_n; ++sh)
      stage_vpools<K, G::kThreads>(T, sh * K, VP + sh * G::kVPWords, true, enc_conv(K, sh));
  } else {
    stage_vpools<K, G::kThreads>(T, 0, VP, true);                                   // inverse transform, index 0
    if (nshift > 1) stage_vpools<K, G::kThreads>(T, K, VP + G::kVPWords, true, enc_conv(K, 1));  // first shift
  }
  __syncthreads();

  const uint32_t cqb = col_base<K>(4 * lane) ^ (32u * g);  // blocks 4g..4g+3 of columns 4l..4l+3
  // ---- cq pass: systematic rows, inverse levels 0..3
  {
    uint32_t CL[16], CH[16];
    cq_read<K>(tile, cqb, CL, CH);
    store_rows(out, a.shard_len, 16 * g, wanted_store, CL, CH, lane, ncols, full, nt);
    tower_convert(T, CL, CH);  // transforms run in tower coordinates
    cq_levels<K, true, true, 0, false, kEncPrioCq>(T, VP, 0, g, CL, CH);
    // the quad items overlay payload blocks that other waves read: wait for
    // every wave's cq_read
    __syncthreads();
    cq_write_q(tile, g, lane, CL, CH);
  }
  __syncthreads();
  // ---- high layout: inverse levels 4.. -> coefficients M
  uint32_t ML[16], MH[16];
  hi_read_q<K>(tile, g, lane, ML, MH);
  hi_levels<K, true, true, 0, 0, kEncPrio>(T, VP, 0, ML, MH);
#pragma unroll
  for (int q = 0; q < 16; ++q) asm volatile("" : "+v"(ML[q]), "+v"(MH[q]));  // materialise M once

  uint32_t PL[8], PH[8];  // top-level products of shift 1, then of shifts 1 ^ 2 (fwd_top)
  auto shift = [&](auto shc, uint32_t sh) __attribute__((always_inline)) {
    constexpr int SH = decltype(shc)::value;
    const uint32_t index = sh * K;
    uint32_t XL[16], XH[16];
    const uint32_t* vp = VP + (resident ? sh : (sh & 1u)) * G::kVPWords;
    shift_hi<K, SH>(T, vp, index, ML, MH, XL, XH, PL, PH);
    __syncthreads();  // the previous cq pass is done with the tile and with the other table buffer
    if (!resident && sh + 1 < nshift && (sh + 1) * K < a.wanted_n)
      stage_vpools<K, G::kThreads>(T, (sh + 1) * K, VP + ((sh + 1) & 1u) * G::kVPWords, sh + 1 < 4,
                                   enc_conv(K, sh + 1));
    hi_write_q<K>(tile, g, lane, XL, XH);
    __syncthreads();
    cq_read_q(tile, g, lane, XL, XH);
    shift_cq<K, SH>(T, vp, index, g, XL, XH);
    store_rows(out, a.shard_len, index + 16 * g, wanted_store, XL, XH, lane, ncols, full, nt);
  };
  if (nshift > 1 && K < a.wanted_n) shift(Int<1>{}, 1);
  if (nshift > 2 && 2 * K < a.wanted_n) shift(Int<2>{}, 2);
  if (nshift > 3 && 3 * K < a.wanted_n) shift(Int<3>{}, 3);
#pragma unroll 1
  for (uint32_t sh = 4; sh < nshift && sh * K < a.wanted_n; ++sh) shift(Int<0>{}, sh);
}

// ----------------------------------------------------- multi-tile encode ----
// k = 256: a workgroup encodes `tpw` consecutive tiles of one payload, and the
// payload blocks of the next tile flow into the LDS tile by LDS-DMA while the
// last shift's cq levels and row stores of this tile run (the tile is free
// once every wave has read it back for that last cq pass).  The launch record
// is re-read from the kernarg segment at every tile, so that none of it stays
// live in registers across the tile loop.
// Multi-tile workgroups (k = 256 only).  Tried for the k = 64 / 128 decodes
// too: 5-11 % slower at 190, 300 and 700 validators, neutral at config 2
// (profiles/r04_ab.txt probe 11) -- there four workgroups share a CU, and
// fewer, longer ones hid less.
template <int K>
constexpr bool kMultiTile = K == 256;

// Table buffers of the multi-tile encode: the inverse transform's and one per
// shift, staged once per workgroup (n <= 4K); with the 128 KiB tile they fill
// the 160 KiB of LDS.  Table loads inside the tile loop would wait (vmcnt
// counts in order) for the row stores issued before them.
constexpr int kEncBuffers = 4;

struct EncLaunch {
  DevTables T;
  EncodeArgs a;
  uint32_t nchunks, tiles, tpw;
};
typedef const __attribute__((address_space(4))) EncLaunch* enc_launch_ptr;

// The next tile's payload by 16-byte LDS-DMA pieces (8 per wave instead of 32
// of 4 bytes), which needs the payload tile's swizzle at 16-byte granularity
// (col_base EVEN; the tile's cq reads then conflict 2-way).  From the stamps
// (profiles/r04_encode_stamps_hiw.txt): 32 pieces per wave overfill the wave's
// memory queue and the DMA's issue stalls.  Measured: encode 1.625 / 1.630 /
// 1.625 -> 1.598 / 1.603 / 1.596 ms (-1.7 %, profiles/r04_ab.txt probe 15).
// The pieces' addresses are a scalar base plus a 32-bit lane offset (1 VALU per
// piece instead of 7 for 64-bit per-lane addresses; -0.5 %, probe 17).  Issuing
// all pieces from 4 waves after a barrier measured -0.8 % on top, neutral with
// the issue priority (probe 18).
template <int K>
constexpr bool kEncDmaX4 = K == 256;

// kEncDmaX4: wave w's columns 16w..16w+15 in 8 pieces of two columns (lanes
// 0-31 the first, 32-63 the second, 16 bytes each): lane l of a piece writes
// LDS blocks 2(l & 31), 2(l & 31) + 1 of its column, which hold the payload's
// contiguous blocks 2(l & 31) ^ sw, (2(l & 31) ^ sw) + 1 (sw even).
template <int K>
__device__ __forceinline__ void dma_tile_x4(const uint8_t* pay, uint32_t ch0, uint8_t* tile, uint32_t w, uint32_t lane) {
  static_assert(K == 256, "two 512-byte columns per 1 KiB piece");
  constexpr uint32_t kColBytes = 2 * K;
  const uint32_t lds0 = static_cast<uint32_t>(
      reinterpret_cast<uintptr_t>((__attribute__((address_space(3))) uint8_t*)(tile)));
  const uint32_t half = lane >> 5, li = lane & 31u;
  const uint32_t swh = half ? (swz<K>(1) & ~1u) : 0u;  // the odd column's part of the (linear) swizzle
  // scalar base per piece (column 16w + 2j), 32-bit lane offset: the swizzle
  // is linear, so piece j's offset is the lane's piece-0 offset XOR a constant
  const uint32_t off0 = 512u * half + 8u * ((2u * li) ^ (swz<K>(16u * w) & ~1u) ^ swh);
  const uint8_t* base = pay + static_cast<size_t>(ch0 + 16u * w) * kColBytes;
#pragma unroll
  for (uint32_t j = 0; j < 8; ++j) {
    const uint32_t off = off0 ^ (8u * (swz<K>(2u * j) & ~1u));
    const uint8_t* sb = base + 2u * j * kColBytes;
    NP_BNOTE(sb + off, 16, kBkPayloads);
    const uint32_t dst = uniform(lds0 + (16u * w + 2u * j) * kColBytes);
    uint32_t keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2 nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep)
                 : "v"(off), "s"(sb), "s"(dst)
                 : "memory");
  }
}

// One shift of the encode (rows sK .. sK+K-1), SH = 1..3.  With `dma_pay`,
// the last cq pass starts the next tile's payload DMA once every wave has read
// the tile.
template <int K, int SH>
__device__ __forceinline__ void encode_shift(const DevTables& T, const EncodeArgs& a, uint8_t* tile, uint32_t* VP,
                                             uint8_t* out, uint32_t sh, uint32_t g, uint32_t lane, uint32_t ncols,
                                             bool full, const uint32_t (&ML)[16],
                                             const uint32_t (&MH)[16], uint32_t (&PL)[8], uint32_t (&PH)[8],
                                             const uint8_t* dma_pay, uint32_t dma_ch0, uint64_t* dbg) {
  using G = Geo<K>;
  const uint32_t index = sh * K;
  uint32_t XL[16], XH[16];
  const uint32_t* vp = VP + sh * G::kVPWords;  // the tables of every shift stay staged (kEncBuffers)
  constexpr int st0 = 7 + 4 * (SH - 1);  // stamp slots of this shift
  {
    // the quads of each level-4 group go to LDS as soon as they are final,
    // among the level's VALU work; the barrier that frees the tile (every
    // wave's previous cq read) moves before level 4
    uint8_t* hb0 = tile + 512u * (256u / K) * g + fresh_v(8u * lane);
    struct Hook {
      uint8_t* b;
      uint32_t (&L)[16];
      uint32_t (&H)[16];
      __device__ __forceinline__ void pre() const { __syncthreads(); }
      __device__ __forceinline__ void post(int t) const {
        *reinterpret_cast<uint2*>(b + hi_q_off<K>(2 * t)) = make_uint2(L[2 * t], H[2 * t]);
        *reinterpret_cast<uint2*>(b + hi_q_off<K>(2 * t + 1)) = make_uint2(L[2 * t + 1], H[2 * t + 1]);
      }
    };
    shift_hi<K, SH>(T, vp, index, ML, MH, XL, XH, PL, PH, Hook{hb0, XL, XH});
    stamp(dbg, st0);
    __syncthreads();
    cq_read_q(tile, g, lane, XL, XH);
  }
  if (dma_pay) {
    // No workgroup barrier: wave g's quad items and its share of the next
    // payload tile are the same 8 KiB (cq_read_q, dma_tile_x4), so once its
    // own reads are back no other wave touches that region.  Measured: encode
    // 1.646 / 1.648 -> 1.638 / 1.638 ms (-0.6 %, profiles/r04_ab.txt probe 13).
    // Spreading the DMA pieces over the last cq pass measured +0.3 to +0.7 %.
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if constexpr (!(kExp & 4)) dma_tile_x4<K>(dma_pay, dma_ch0, tile, g, lane);
  }
  stamp(dbg, st0 + 1);
  const uint32_t row0 = index + 16 * g;
  const uint32_t wanted = (kExp & 2) ? 0u : a.wanted_n;
  const bool nt = rows_nt(a.shards, a.batch_stride, a.shard_len);
  shift_cq<K, SH>(T, vp, index, g, XL, XH);
  stamp(dbg, st0 + 2);
  store_rows(out, a.shard_len, row0, wanted, XL, XH, lane, ncols, full, nt);
  stamp(dbg, st0 + 3);
}

// One tile; returns whether the next tile's payload is on its way by DMA.
template <int K>
__device__ __forceinline__ bool encode_tile_multi(const DevTables& T, const EncodeArgs& a, uint8_t* smem, uint32_t pb,
                                                  uint32_t tl, uint32_t nchunks, bool first, bool have_dma,
                                                  bool stored16, uint32_t next_tl) {
  using G = Geo<K>;
  uint8_t* tile = smem;
  uint32_t* VP = reinterpret_cast<uint32_t*>(smem + G::kTileBytes);  // 2 staged transforms
  const uint32_t ch0 = tl * kTile;
  const uint32_t ncols = min(static_cast<uint32_t>(kTile), nchunks - ch0);
  const uint8_t* pay = a.payloads + static_cast<size_t>(pb) * a.payload_stride;
  uint8_t* out = a.shards + static_cast<size_t>(pb) * a.batch_stride + 2 * static_cast<size_t>(ch0);
  // opaque per tile: otherwise the lane-derived addresses of the loads, DMA and
  // row guards are hoisted out of the tile loop and spilled, and each reload
  // (a VMEM op) waits with vmcnt(0) for the DMA and every row store before it
  const uint32_t tid = fresh_v(threadIdx.x), lane = tid & 63u, g = uniform(tid >> 6);
  const bool full =
      ncols == kTile && rows_vec_ok(a.shards, a.batch_stride, a.shard_len);
  // experiment builds (NP_EXP bit 6): s_memtime stamps past the payload's shard
  // rows (tools/enc_stamps.py allocates batch_stride = n shard_len + 4 KiB per tile)
  uint64_t* dbg = (kExp & 64) ? reinterpret_cast<uint64_t*>(a.shards + static_cast<size_t>(pb) * a.batch_stride +
                                                             static_cast<size_t>(a.n) * a.shard_len + 4096u * tl)
                              : nullptr;
  stamp(dbg, 0);
  // whole tiles load by 8-byte vector loads at any address; the LDS-DMA of the
  // next tile's payload (4-byte pieces) only from 8-byte aligned payloads
  const bool aligned_pay = (reinterpret_cast<uintptr_t>(pay) & (kEncDmaX4<K> ? 15u : 7u)) == 0;
  auto tile_whole = [&](uint32_t t) __attribute__((always_inline)) {
    return static_cast<size_t>(t * kTile + kTile) * 2 * K <= a.payload_len;
  };
  auto tile_fast = [&](uint32_t t) __attribute__((always_inline)) { return aligned_pay && tile_whole(t); };
  if (have_dma) {
    // this wave's DMA pieces have landed; the previous tile's last 16 row
    // stores, issued after them, may still be in flight
    if (stored16)
      asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    const uint32_t c0 = tid / G::Q, m0 = tid % G::Q;
    const uint32_t base = col_base<K, kEncDmaX4<K>>(c0) ^ (8u * m0);
    const size_t gbase = static_cast<size_t>(ch0 + c0) * 2 * K + 8u * m0;
    if (out_vec_ok(pay, 0) && tile_whole(tl)) {
      uint2 v[16];
#pragma unroll
      for (int i = 0; i < 16; ++i)
        v[i] = (kExp & 4) ? make_uint2(i, tid) : load_once(pay + gbase + static_cast<size_t>(i) * 32 * K);
#pragma unroll
      for (int i = 0; i < 16; ++i) *reinterpret_cast<uint2*>(tile + (base ^ col_base_c<K, kEncDmaX4<K>>(16u * i))) = v[i];
    } else {
#pragma unroll 1
      for (uint32_t i = 0; i < 16; ++i) {
        const size_t g0 = gbase + static_cast<size_t>(i) * 32 * K;
        uint32_t w[2] = {0, 0};
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (g0 + e < a.payload_len) w[e >> 2] |= static_cast<uint32_t>(*NP_BCHK(pay + (g0 + e), 1, kBkPayloads)) << (8 * (e & 3));
        *reinterpret_cast<uint2*>(tile + (base ^ col_base_c<K, kEncDmaX4<K>>(16u * i))) = make_uint2(w[0], w[1]);
      }
    }
  }
  const uint32_t nshift = a.n / K;
  const uint32_t last = min(nshift, (a.wanted_n + K - 1) / K) - 1;  // last shift with wanted rows
  if (first) {  // tables of the inverse transform (index 0) and of every shift, kept for all tiles
    for (uint32_t sh = 0; sh <= last; ++sh)
      stage_vpools<K, G::kThreads>(T, sh * K, VP + sh * G::kVPWords, true, enc_conv(K, sh));
  }
  __syncthreads();
  stamp(dbg, 1);

  const uint32_t cqb = col_base<K, kEncDmaX4<K>>(4 * lane) ^ (32u * g);  // the payload tile's swizzle
  {
    uint32_t CL[16], CH[16];
    cq_read<K, kEncDmaX4<K>>(tile, cqb, CL, CH);
    store_rows(out, a.shard_len, 16 * g, (kExp & 2) ? 0u : a.wanted_n, CL, CH, lane, ncols, full,
               rows_nt(a.shards, a.batch_stride, a.shard_len));
    stamp(dbg, 2);
    tower_convert(T, CL, CH);  // transforms run in tower coordinates
    cq_levels<K, true, true, 0, false, kEncPrioCq>(T, VP, 0, g, CL, CH);
    stamp(dbg, 3);
    // the quad items overlay payload blocks that other waves read: wait for
    // every wave's cq_read
    __syncthreads();
    cq_write_q(tile, g, lane, CL, CH);
  }
  stamp(dbg, 4);
  __syncthreads();
  uint32_t ML[16], MH[16];
  hi_read_q<K>(tile, g, lane, ML, MH);
  stamp(dbg, 5);
  hi_levels<K, true, true, 0, 0, kEncPrio>(T, VP, 0, ML, MH);
#pragma unroll
  for (int q = 0; q < 16; ++q) asm volatile("" : "+v"(ML[q]), "+v"(MH[q]));  // materialise M once
  stamp(dbg, 6);
  uint32_t PL[8], PH[8];
  const bool dma = last >= 1 && next_tl != ~0u && tile_fast(next_tl);
  const uint8_t* dpay = dma ? pay : nullptr;
  const uint32_t dch0 = next_tl * kTile;
  if (last >= 1)
    encode_shift<K, 1>(T, a, tile, VP, out, 1, g, lane, ncols, full, ML, MH, PL, PH,
                       last == 1 ? dpay : nullptr, dch0, dbg);
  if (last >= 2)
    encode_shift<K, 2>(T, a, tile, VP, out, 2, g, lane, ncols, full, ML, MH, PL, PH,
                       last == 2 ? dpay : nullptr, dch0, dbg);
  if (last >= 3)
    encode_shift<K, 3>(T, a, tile, VP, out, 3, g, lane, ncols, full, ML, MH, PL, PH, dpay, dch0, dbg);
  return dma;
}

template <int K>
__global__ __launch_bounds__(4 * K) __attribute__((amdgpu_waves_per_eu(4))) void k_encode_multi(EncLaunch L) {
#if defined(__HIP_DEVICE_COMPILE__)  // (the host pass cannot bind the kernarg-segment record to references)
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
#if NP_BOUNDS_CHECK
  bounds_arm(bounds_of_enc(L.a));
#endif
  const uint32_t groups = (L.tiles + L.tpw - 1) / L.tpw;  // workgroups per batch entry
  const TileRef tr = tile_of(blockIdx.x, groups, (L.a.batch & 7u) == 0);
  const uint32_t pb = tr.pb, tl0 = tr.tl * L.tpw;
  const uint32_t ntl = min(L.tpw, L.tiles - tl0);
  const uint64_t kp = reinterpret_cast<uint64_t>(__builtin_amdgcn_kernarg_segment_ptr());
  bool dma = false;
#pragma unroll 1
  for (uint32_t t = 0; t < ntl; ++t) {
    if (t > 0) __syncthreads();  // the previous tile's last cq pass is done with the tables
    const enc_launch_ptr lp = reinterpret_cast<enc_launch_ptr>(fresh(kp));
    const DevTables T = lp->T;
    const EncodeArgs a = lp->a;
    // the previous tile's last shift stored 16 rows per wave (store_rows' full path)
    const uint32_t pch0 = (tl0 + t - 1) * kTile;
    const bool stored16 = t > 0 && pch0 + kTile <= lp->nchunks &&
                          rows_vec_ok(a.shards, a.batch_stride, a.shard_len) &&
                          (min(a.n / K, (a.wanted_n + K - 1) / K) - 1) * K + 16 * 16 <= a.wanted_n &&
                          16 * a.shard_len < 0x7fffffffu;
    dma = encode_tile_multi<K>(T, a, smem, fresh(pb), fresh(tl0) + t, lp->nchunks, t == 0, dma, stored16,
                               t + 1 < ntl ? tl0 + t + 1 : ~0u);
  }
#endif
}

// ------------------------------------------------------------ reconstruct ----
struct RecCtx {
  const DevTables& T;
  size_t shard_len;
  uint8_t* tile;
  const uint32_t* R;  // row table records of the payload (prefix record)
  const uint8_t* sh;
  uint32_t* VP;  // 2 staged transforms
  uint32_t g, lane, tid, ncols;
  bool full;
  uint32_t cqb, hb;
  uint64_t* dbg;  // experiment builds only (stamp)
  uint32_t occ;   // bit q: segment q holds a present row (k_prefix_locator, record byte 1)
};

// Segment q of the sweep at step `step` (segments 2, 3, 1, 0 for NQ = 4; 1, 0
// for NQ = 2; 7, 6, ..., 0 for NQ = 8).
template <int NQ>
__host__ __device__ constexpr int seg_of(int step) {
  return NQ == 8 ? 7 - step : NQ == 4 ? (step == 0 ? 2 : step == 1 ? 3 : 3 - step) : 1 - step;
}

// NQ = 8: the first K outputs of the size-8K decode need
//   d = D_K(x0) ^ sum_q kappa_q x_q,  x_q = IFFT(K, qK)(premultiplied segment q),
// the three top inverse levels of index 0 (skews 0, Cantor(2), Cantor(4),
// Cantor(6)) and the derivative's single-bit terms K, 2K, 4K folded into one
// coefficient per segment: kappa = (1, 1, 1+b1, b1, (1+b1)(1+b2), (1+b1) b2,
// b1 (1+b3), b1 b3) with b_i = Cantor(2i), in Cantor coordinates below (all in
// GF(16); tests/test_oracle.py::test_rec8_kappa re-derives them with the
// oracle).  One accumulator, one subfield multiply per segment and position.
__host__ __device__ constexpr uint32_t rec8_kappa(int q) {
  constexpr uint32_t k[8] = {1, 1, 3, 2, 12, 15, 10, 8};
  return k[q];
}

// Presence of rows row0..row0+15 as bits (wave-uniform): one byte load per
// lane and a ballot, so row sources can be chosen before the flags reach LDS.
__device__ __forceinline__ uint32_t row_mask16(const uint8_t* pres, uint32_t row0, uint32_t lane) {
  const bool p = lane < 16u && *NP_BCHK(pres + (row0 + lane), 1, kBkPresent) != 0;
  return static_cast<uint32_t>(__ballot(p));
}

// Row loads: streaming (nt) for rows read once -- the parity segments' rows
// and the merge's final read of the systematic rows -- and the default policy
// for segment 0's systematic rows, which the merge reads again, so that the
// parity rows do not push them (and the payload's row-table records, re-read
// by every tile) out of L2.  (Every load with the default policy measured
// +1.5 % on the decode, all-nt +0.5 % in round 1.)
// Issues the loads of the lane's pieces of rows row0..row0+15; the data is
// consumed later.  Full tiles: one buffer descriptor per row whose size is 0
// for an absent row, so that load returns zeros with no HBM traffic and no
// branch.  Partial tiles: absent rows read the zero page.
template <int CPOL>
__device__ __forceinline__ void issue_rows_c(uint2 (&raw)[16], const uint8_t* sh, size_t shard_len, uint32_t mask,
                                             uint32_t row0, const uint8_t* zeros, uint32_t lane, uint32_t ncols,
                                             bool full) {
  if (full) {
#pragma unroll
    for (int p = 0; p < 16; ++p) {
      if ((mask >> p) & 1u) NP_BNOTE(sh + static_cast<size_t>(row0 + p) * shard_len + 8u * lane, 8, kBkShards);
      const __amdgpu_buffer_rsrc_t r = buf_rsrc(sh + static_cast<size_t>(row0 + p) * shard_len, ((mask >> p) & 1u) ? 512u : 0u);
      const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, 8u * lane, 0, CPOL);
      raw[p] = make_uint2(v.x, v.y);
    }
  } else {
#pragma unroll
    for (int p = 0; p < 16; ++p) {
      const uint8_t* src = ((mask >> p) & 1u) ? sh + static_cast<size_t>(row0 + p) * shard_len : zeros;
      raw[p] = load4(src, lane, ncols, false);
    }
  }
}

// reread: the rows are read again later (segment 0 before the merge).
__device__ __forceinline__ void issue_rows(uint2 (&raw)[16], const uint8_t* sh, size_t shard_len, uint32_t mask,
                                           uint32_t row0, const uint8_t* zeros, uint32_t lane, uint32_t ncols,
                                           bool full, bool reread = false) {
  if (!reread)
    issue_rows_c<2>(raw, sh, shard_len, mask, row0, zeros, lane, ncols, full);
  else
    issue_rows_c<0>(raw, sh, shard_len, mask, row0, zeros, lane, ncols, full);
}

// Copy-out straight from the cq registers: lane l holds columns 4l..4l+3 at
// positions 16g..16g+15, i.e. bytes [32g, 32g + 32) of each of those four
// 2K-byte output columns (two 16-byte stores per column).  Full tiles with
// 16-byte aligned output only; saves the LDS round trip and its two barriers.
// (Streaming stores here cost +26 %: each wave writes a quarter of a line.)
template <int K>
__device__ __forceinline__ void copy_out_cq(uint8_t* out_tile, uint32_t lane, uint32_t g, const uint32_t (&L)[16],
                                            const uint32_t (&H)[16]) {
  uint2 d[4][4];
#pragma unroll
  for (int u = 0; u < 4; ++u) cq_to_blks(&L[4 * u], &H[4 * u], d[u]);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    uint8_t* o = NP_BCHK(out_tile + static_cast<size_t>(4u * lane + i) * 2 * K + 32u * g, 32, kBkOut);
    *reinterpret_cast<uint4*>(o) = make_uint4(d[0][i].x, d[0][i].y, d[1][i].x, d[1][i].y);
    *reinterpret_cast<uint4*>(o + 16) = make_uint4(d[2][i].x, d[2][i].y, d[3][i].x, d[3][i].y);
  }
}

// The merge's systematic rows (4- and 8-segment decodes) load before the
// forward transform's cq pass.  Measured: decode 0 to -2 % at config 3 (box to
// box), -4 % at n/k = 8, k = 64, against loading them at the merge; before the
// forward high pass instead: -0.9 %.

// Row loads run one step ahead of their use where the registers allow it
// (prefixes of up to 2 segments); the 4-segment decode, which keeps more
// state live, loads each step's rows where it uses them.
template <int NQ>
constexpr bool kRowPrefetch = NQ <= 2;

// The tables of all NQ segment transforms fit in LDS next to the tile (K = 256:
// 128 KiB + 4 x 8 KiB of the 160 KiB): staged once per workgroup and kept for
// all its tiles, instead of two buffers restaged per step.  Measured -1 % to
// +0.6 % at config 3 (noise), -1.2 % at config 2.  (An L2 prefetch of the next
// step's rows by LDS-DMA into a dummy LDS area measured +8 %: vector loads
// complete in order, so the wait for a step's last row also waited for the
// prefetch behind it.)
// Only where it keeps the workgroups per CU (4K threads each, four waves per
// SIMD): K = 64 / 128 with NQ = 8 would lose one of four / two (measured +24 %
// / +65 % decode time).
template <int K, int NQ>
constexpr bool kRecResident =
    NQ > 1 &&
    Geo<K>::kTileBytes + NQ * 4u * Geo<K>::kVPWords <= 160u * 1024u * Geo<K>::kThreads / 1024u;
// LDS buffer of segment q's tables at decode step `step`.
template <int K, int NQ>
__device__ __forceinline__ uint32_t vp_slot(int q, int step) {
  return kRecResident<K, NQ> ? static_cast<uint32_t>(q) : static_cast<uint32_t>(step & 1);
}

// Largest gen_of over the decode's segment transforms (index qK, q < NQ).
template <int K, int NQ>
constexpr int kRecMaxGen = static_cast<int>(gen_of(static_cast<uint32_t>((NQ - 1) * K)));

// Tables staged before the first step: every segment's (kRecResident, slot q)
// or those of steps 0 and 1 (slots 0 and 1).  Caller synchronises.
template <int K, int NQ>
__device__ __forceinline__ void stage_rec_tables(const DevTables& T, uint32_t* VP) {
  if constexpr (kRecResident<K, NQ>) {
#pragma unroll 1
    for (int q = 0; q < NQ; ++q)
      stage_vpools<K, Geo<K>::kThreads>(T, static_cast<uint32_t>(q) * K, VP + q * Geo<K>::kVPWords, true);
  } else {
    stage_vpools<K, Geo<K>::kThreads>(T, static_cast<uint32_t>(seg_of<NQ>(0)) * K, VP, true);
    stage_vpools<K, Geo<K>::kThreads>(T, static_cast<uint32_t>(seg_of<NQ>(1)) * K, VP + Geo<K>::kVPWords, true);
  }
}

// msk[step] (16-bit row masks, wave-uniform) through shifts of packed scalars:
// a select chain over msk[] becomes a dynamically indexed private array, i.e.
// a scratch load whose vmcnt(0) wait also waits for every row load and store
// issued before it.
template <int NQ>
__device__ __forceinline__ uint32_t seg_mask(const uint32_t (&msk)[NQ], int step) {
  if constexpr (NQ <= 2) return step == 0 ? msk[0] : msk[NQ - 1];  // one select (the packed form spills here)
  uint64_t lo = 0, hi = 0;
#pragma unroll
  for (int i = 0; i < NQ; ++i) {
    const uint64_t v = static_cast<uint64_t>(msk[i] & 0xffffu);
    if (i < 4)
      lo |= v << (16 * i);
    else
      hi |= v << (16 * (i - 4));
  }
  const uint32_t sh = 16u * static_cast<uint32_t>(step & 3);
  return static_cast<uint32_t>(((step < 4 ? lo : hi) >> sh) & 0xffffu);
}

// The segment sweep: x_q = IFFT(K, qK)(premultiplied segment q), folded into
// A.  With kRowPrefetch `raw` holds segment seg_of(0)'s rows on entry and the
// systematic rows (for the merge) on exit.  A runtime loop keeps
// the kernel small; at index 0 the t = 0 multipliers are the zero element,
// whose table yields 0 (the reference's skipped multiply).
// Tile prefetch: the multi-tile decodes that load each step's rows
// where they use them (NQ >= 4) load the next tile's first-step rows during
// this tile's copy-out (and the first tile's before the tables are staged), as
// the 2-segment decode does: at the tile boundary only the rows and the output
// registers are live.  Measured (profiles/r04_ab.txt): config-3 decode
// 2.78 -> 2.73 ms (-1.6 %); the 8-segment decode (1200 validators) +0.5 %, so
// 4 segments only.
template <int K, int NQ>
constexpr bool kTilePrefetch = NQ == 4 && kMultiTile<K>;

// PRE0: step 0's rows are in `raw` on entry (kTilePrefetch).
template <int NQ>
constexpr bool kSkipEmpty = NQ == 8;

template <int K, int NQ, bool PRE0 = false>
__device__ __forceinline__ void rec_segments(const RecCtx& c, const uint32_t (&msk)[NQ], uint2 (&raw)[16],
                                             uint32_t (&AL)[16], uint32_t (&AH)[16], bool after_tile) {
  const DevTables& T = c.T;
  uint32_t XL[16], XH[16];
  // A (+)= the fold of x_q (XL / XH in the high layout) for segment q at `step`
  auto fold = [&](int step, int q) __attribute__((always_inline)) {
    if (NQ == 8 && q != 0) {  // A ^= kappa_q x_q (kRec8Kappa, all in GF(2^8))
      const uint32_t kq = uniform(rec8_kappa(q));
      if (kq == 1u) {
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          AL[j] ^= XL[j];
          AH[j] ^= XH[j];
        }
      } else {
        uint32_t kp[20];
        pool_of<true>(T, kq, kp);
        const Mult pool = make_mult(kp);
        if (step == 0) {
#pragma unroll
          for (int j = 0; j < 16; ++j) qmul_sub_set(AL[j], AH[j], XL[j], XH[j], pool);
        } else {
#pragma unroll
          for (int j = 0; j < 16; ++j) qmul_sub(AL[j], AH[j], XL[j], XH[j], pool);
        }
      }
    } else if (step == 0) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        AL[j] = XL[j];
        AH[j] = XH[j];
      }
    } else if (q == 0) {
      if (NQ == 2 || NQ == 8) {  // kappa_0 = 1
#pragma unroll
        for (int j = 0; j < 16; ++j) {
          AL[j] ^= XL[j];
          AH[j] ^= XH[j];
        }
      }
      add_derivative<K>(AL, XL, c.tid % Geo<K>::R);
      add_derivative<K>(AH, XH, c.tid % Geo<K>::R);
    } else if (NQ == 4 && q == 3) {
      uint32_t beta[20];
      pool_of<true>(T, 2u, beta);  // beta = Cantor(2) in GF(2^8), the t = 1 skew of level logK at index 0
      const Mult pool = make_mult(beta);
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        XL[j] ^= AL[j];
        XH[j] ^= AH[j];
        qmul_sub(AL[j], AH[j], XL[j], XH[j], pool);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        AL[j] ^= XL[j];
        AH[j] ^= XH[j];
      }
    }
  };
#pragma unroll 1
  for (int step = 0; step < NQ; ++step) {
    const int q = seg_of<NQ>(step);
    // A segment without a present row contributes x_q = 0 (absent rows are
    // zeros): no loads, premultiply, transform or exchange, only the fold.
    // The 8-segment decodes only (n = 8k, e.g. 300, 700 and 1,200
    // validators: the segments above wanted_n are empty); the others are
    // compiled without the branch.  The next step's tables are still staged
    // here when they are not resident (in the other buffer, which the
    // previous step's high pass read).
    if (kSkipEmpty<NQ> && !((c.occ >> q) & 1u)) {
#pragma unroll
      for (int j = 0; j < 16; ++j) XL[j] = XH[j] = 0;
      if constexpr (!kRecResident<K, NQ>) {
        if (step > 0 && step + 1 < NQ) {
          __syncthreads();
          stage_vpools<K, Geo<K>::kThreads>(T, static_cast<uint32_t>(seg_of<NQ>(step + 1)) * K,
                                            c.VP + ((step + 1) & 1) * Geo<K>::kVPWords, true);
          __syncthreads();
        }
      }
    } else {
      const uint32_t index = uniform(static_cast<uint32_t>(q) * K);
      __builtin_amdgcn_sched_barrier(0);
      const uint32_t g = fresh(c.g);
      const uint8_t* sh = fresh(c.sh);
      const uint32_t* R = fresh(c.R);
      const size_t shard_len = fresh(c.shard_len);
      const uint32_t cqb = fresh_v(c.cqb), hb = fresh_v(c.hb);
      uint32_t m = uniform(seg_mask<NQ>(msk, step));
      if (!kRowPrefetch<NQ> && !(PRE0 && step == 0))
        issue_rows(raw, (kExp & 32) ? T.zeros : sh, (kExp & 32) ? 0 : shard_len, m, index + 16 * g, T.zeros, c.lane,
                   c.ncols, c.full, q == 0);
      stamp(c.dbg, 2 + 6 * step);
      __builtin_amdgcn_s_setprio(kRecPrioPremul);
      pipelined_rec<16>(
          [&](auto pc) __attribute__((always_inline)) {
            NP_BNOTE(reinterpret_cast<const uint8_t*>(R) + (index + 16 * g + decltype(pc)::value) * 4 * kPoolWords,
                     4 * kPoolWords, kBkRecords);
            return (cpool_t)(R) + (index + 16 * g + decltype(pc)::value) * kPoolWords;
          },
          [&](auto pc) __attribute__((always_inline)) { return ((m >> decltype(pc)::value) & 1u) != 0; },  // present
          [&](auto pc, const Mult& pool) __attribute__((always_inline)) {
            constexpr int x = decltype(pc)::value;
            XL[x] = 0;  // absent rows contribute zero
            XH[x] = 0;
            if ((m >> x) & 1u) {
              uint32_t l, h;
              blk_to_quad(raw[x], l, h);
              if constexpr (kExp & 16) {  // experiment: no premultiply
                XL[x] = l;
                XH[x] = h;
              } else {
                qmul_set(XL[x], XH[x], l, h, pool);
              }
            }
          });
      const uint32_t* vp = c.VP + vp_slot<K, NQ>(q, step) * Geo<K>::kVPWords;
      stamp(c.dbg, 3 + 6 * step);
      // absent rows are zero; segment q's transform has gen_of(qK) <= kRecMaxGen
      with_gen<0, kRecMaxGen<K, NQ>, false>(index, [&](auto gc) __attribute__((always_inline)) {
        cq_levels<K, true, false, decltype(gc)::value, false, kRecPrioCq>(T, vp, index, g, XL, XH, m);
      });
      stamp(c.dbg, 4 + 6 * step);
      if (step > 0 || after_tile) {
        __syncthreads();  // the previous high pass (or tile's copy-out) is done with the tile and the other table buffer
        if (!kRecResident<K, NQ> && step + 1 < NQ) {
          const int qn = seg_of<NQ>(step + 1);
          stage_vpools<K, Geo<K>::kThreads>(T, static_cast<uint32_t>(qn) * K, c.VP + ((step + 1) & 1) * Geo<K>::kVPWords, true);
        }
      }
      cq_write_p<K>(c.tile, cqb, XL, XH);
      // next step's rows (the systematic rows after the last step) load during
      // this step's high pass
      if constexpr (kRowPrefetch<NQ>) {
        uint32_t mn = msk[0];
        uint32_t qn = 0;
  #pragma unroll
        for (int i = 1; i < NQ; ++i) {
          if (step + 1 == i) {
            mn = msk[i];
            qn = static_cast<uint32_t>(seg_of<NQ>(i));
          }
        }
        if (step + 1 == NQ) mn = msk[NQ - 1], qn = 0;  // segment 0 is the last step's
        issue_rows(raw, (kExp & 32) ? T.zeros : sh, (kExp & 32) ? 0 : shard_len, uniform(mn), uniform(qn) * K + 16 * g,
                   T.zeros, c.lane, c.ncols, c.full, qn == 0 && step + 1 < NQ);
      }
      __syncthreads();
      stamp(c.dbg, 5 + 6 * step);
      hi_read_p<K>(c.tile, hb, XL, XH);
      // hi levels: gen_of(index) <= 4; segment 0 (index 0) skips the t = 0
      // groups, whose skew is the zero element (15 of the 32 quad multiplies)
      // (the 2-segment decode keeps its rows prefetch live here: no room for two instances)
      if (NQ == 4 && q == 0)  // -1.1 % (config 3)
        hi_levels<K, true, true, 0, 0, kRecPrioHi>(T, vp, 0, XL, XH);
      else
        hi_levels<K, true, false, 0, 0, kRecPrioHi>(T, vp, index, XL, XH);
      stamp(c.dbg, 6 + 6 * step);
    }
    __builtin_amdgcn_sched_barrier(0);
    fold(step, q);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (PRE0) {
      // raw is reloaded at every later step: an instruction-free definition
      // here ends its live range (the loop header's phi would otherwise keep
      // step 0's rows live through every step)
#pragma unroll
      for (int x = 0; x < 16; ++x) asm volatile("" : "=v"(raw[x].x), "=v"(raw[x].y));
    }
  }
}

// Decode of one tile (K < 256: see kMultiTile), as rec_tiles with ntl = 1.
template <int K, int NQ>
__device__ __forceinline__ void rec_tile(const DevTables& T, const ReconstructArgs& a, const uint8_t* sh,
                                         const uint8_t* pres, const uint32_t* rows, uint8_t* smem,
                                         uint32_t pb, uint32_t col0, uint32_t ncols, bool full, uint64_t* dbg,
                                         uint32_t occ) {
  using G = Geo<K>;
  uint8_t* tile = smem;
  uint32_t* VP = reinterpret_cast<uint32_t*>(smem + G::kTileBytes);  // 2 staged transforms
  const uint32_t tid = threadIdx.x, lane = tid & 63u, g = uniform(tid >> 6);
  const uint32_t cqb = col_base<K>(4 * lane) ^ (32u * g);

  // presence bits of this wave's rows in every segment of the prefix; the
  // first step's rows start loading before the tables are staged
  stamp(dbg, 0);
  uint32_t msk[NQ];
#pragma unroll
  for (int i = 0; i < NQ; ++i) msk[i] = row_mask16(pres, static_cast<uint32_t>(NQ == 1 ? 0 : seg_of<NQ>(i)) * K + 16 * g, lane);
  uint2 raw[16];
  if constexpr (kRowPrefetch<NQ>)
    issue_rows(raw, (NQ > 1 && (kExp & 32)) ? T.zeros : sh, (NQ > 1 && (kExp & 32)) ? 0 : a.shard_len, msk[0],
               static_cast<uint32_t>(NQ == 1 ? 0 : seg_of<NQ>(0)) * K + 16 * g, T.zeros, lane, ncols, full);

  uint32_t XL[16], XH[16];
  if constexpr (NQ > 1) {
    // multiplier tables of the first two segment transforms (indices 2K, 3K or
    // K, 0), or of all of them (kRecResident)
    stage_rec_tables<K, NQ>(T, VP);
    __syncthreads();
    stamp(dbg, 1);

    const uint32_t hb = col_base<K>(tid / G::R) ^ (8u * (tid % G::R));
    uint32_t AL[16], AH[16];
    RecCtx c{T, a.shard_len, tile, rows, sh, VP, g, lane, tid, ncols, full, cqb, hb, dbg, occ};
    rec_segments<K, NQ>(c, msk, raw, AL, AH, false);
    // ---- forward transform of size K at index 0
    const uint32_t* vp0 = VP + vp_slot<K, NQ>(0, NQ - 1) * G::kVPWords;  // segment 0's tables = FFT(K, 0)'s
    stamp(dbg, 26);
    hi_levels<K, false, true, 0, 0, kRecPrioFwdHi>(T, vp0, 0, AL, AH);
    stamp(dbg, 27);
    __syncthreads();
    hi_write<K>(tile, fresh_v(hb), AL, AH);
    __syncthreads();
    stamp(dbg, 28);
    if constexpr (!kRowPrefetch<NQ>)  // the merge's rows load during the FFT's cq pass
      issue_rows(raw, sh, a.shard_len, uniform(msk[NQ - 1]), 16 * g, T.zeros, lane, ncols, full);
    cq_read<K>(tile, fresh_v(cqb), XL, XH);
    cq_levels<K, false, true, 0, false, kRecPrioFwdCq>(T, vp0, 0, g, XL, XH, ~uniform(msk[NQ - 1]));  // erased rows only
    stamp(dbg, 29);
  }
  // ---- merge: received systematic rows, postmultiplied recovered ones
  const uint32_t cqbf = fresh_v(cqb);
  const uint32_t m0 = uniform(msk[NQ == 1 ? 0 : NQ - 1]);  // segment 0 = the last step's
  if constexpr (NQ == 1) {
#pragma unroll
    for (int p = 0; p < 16; ++p) blk_to_quad(raw[p], XL[p], XH[p]);
  } else {
    pipelined_rec<16>(
        [&](auto pc) __attribute__((always_inline)) {
          NP_BNOTE(reinterpret_cast<const uint8_t*>(rows) + (16 * g + decltype(pc)::value) * 4 * kPoolWords,
                   4 * kPoolWords, kBkRecords);
          return (cpool_t)(fresh(rows)) + (16 * g + decltype(pc)::value) * kPoolWords;
        },
        [&](auto pc) __attribute__((always_inline)) { return ((m0 >> decltype(pc)::value) & 1u) == 0; },  // erased
        [&](auto pc, const Mult& pool) __attribute__((always_inline)) {
          constexpr int x = decltype(pc)::value;
          // present: the received symbol (mod.rs:225-235); erased: the
          // postmultiplied recovered symbol (inc_reconstruct.rs:76-84)
          if ((m0 >> x) & 1u) {
            blk_to_quad(raw[x], XL[x], XH[x]);
          } else {
            const uint32_t l = XL[x], h = XH[x];
            qmul_set(XL[x], XH[x], l, h, pool);
          }
        });
  }
  stamp(dbg, 30);
  if (full && out_vec_ok(a.out, a.out_stride)) {
    copy_out_cq<K>(a.out + static_cast<size_t>(pb) * a.out_stride + static_cast<size_t>(col0) * 2 * K, lane, g, XL, XH);
    stamp(dbg, 31);
    return;
  }
  __syncthreads();
  cq_write<K>(tile, cqbf, XL, XH);
  __syncthreads();
  // ---- copy-out: column c of the tile is 2K contiguous bytes of the output
  {
    uint8_t* out = a.out + static_cast<size_t>(pb) * a.out_stride + static_cast<size_t>(col0) * 2 * K;
    const bool al_o = true;  // 8-byte stores at any address (rows_vec_ok)
    const uint32_t c0 = tid / G::Q, m0 = tid % G::Q;
    const uint32_t base = col_base<K>(c0) ^ (8u * m0);
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint32_t c = c0 + 16u * i;
      if (c >= ncols) break;
      const uint2 v = *reinterpret_cast<const uint2*>(tile + (base ^ col_base_c<K>(16u * i)));
      uint8_t* o = NP_BCHK(out + static_cast<size_t>(c) * 2 * K + 8u * m0, 8, kBkOut);
      if (al_o) {
        *reinterpret_cast<uint2*>(o) = v;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) o[e] = static_cast<uint8_t>((e < 4 ? v.x : v.y) >> (8 * (e & 3)));
      }
    }
  }
  stamp(dbg, 31);
}

// Decode of ntl consecutive tiles of one payload from the first NQ segments (NQ * K rows).  The inverse
// transform of size NQ * K is NQ inverse transforms of size K (index qK)
// followed by log2(NQ) top levels whose skews at index 0 are 0 (t = 0) or
// beta = Cantor(2) (t = 1).  Only the first k = K outputs are needed; for them
//   NQ = 2:  d = D_K(x0) ^ x0 ^ x1
//   NQ = 4:  d = D_K(x0) ^ x1 ^ x2 ^ beta * (x2 ^ x3)
// where x_q = IFFT(K, qK)(premultiplied segment q) and D_K is the formal
// derivative of size K; then out = FFT(K, 0)(d) (the size-n forward transform
// restricted to its first K outputs is FFT(K, 0): its t = 0 skews are 0).
// NQ = 1: every systematic row is present, the output is those rows.
//
// Decoding from a prefix (trusted codewords only, ReconstructArgs::trusted).
// The first NQ * K codeword symbols are the codeword of the same message
// under the (NQ * K, K) code: the size-n forward transform of the zero-padded
// coefficients copies its lower half into the upper half at every top level
// (inc_afft.rs:267-332 with x[i + d] = 0), so its first NQ * K outputs are
// FFT(NQ * K, 0) of the same coefficients.  A message of K symbols is
// determined by any K of its codeword symbols, so when the received shards
// ARE a codeword, decoding the prefix with the rows beyond it treated as
// erased yields the reference's output.  For any other input the reference's
// decode (a linear map of every present row) differs, so the crate-equivalent
// entry points always decode from all n rows (or copy, NQ = 1).
template <int K, int NQ>
__device__ __forceinline__ void rec_tiles(const DevTables& T, const ReconstructArgs& a, const uint8_t* pres,
                                          const uint32_t* rows, uint8_t* smem, uint32_t pb,
                                          uint32_t tl0, uint32_t ntl, uint32_t nsyms, uint32_t occ) {
  using G = Geo<K>;
  uint8_t* tile = smem;
  uint32_t* VP = reinterpret_cast<uint32_t*>(smem + G::kTileBytes);  // 2 staged transforms
  const uint32_t tid0 = threadIdx.x, g0 = uniform(tid0 >> 6);
  const bool aligned = rows_vec_ok(a.shards, a.batch_stride, a.shard_len);
  const uint8_t* shp = a.shards + static_cast<size_t>(pb) * a.batch_stride;

  // presence bits of this wave's rows in every segment of the prefix (the
  // same for every tile of the payload); the first tile's first-step rows
  // start loading before the tables are staged
  uint32_t msk0[NQ];
#pragma unroll
  for (int i = 0; i < NQ; ++i) msk0[i] = row_mask16(pres, static_cast<uint32_t>(NQ == 1 ? 0 : seg_of<NQ>(i)) * K + 16 * g0, tid0 & 63u);
  auto tile_cols = [&](uint32_t tl) __attribute__((always_inline)) {
    return min(static_cast<uint32_t>(kTile), nsyms - tl * kTile);
  };
  // Tile order rotated by the batch entry: the workgroups running at the same
  // time then read different 512-byte pieces of their rows, instead of every
  // one the same offset of 4 KiB-strided rows (L2 conflict misses).
  const uint32_t rot = pb % ntl;
  auto tile_at = [&](uint32_t t) __attribute__((always_inline)) {
    const uint32_t i = t + rot;
    return tl0 + (i >= ntl ? i - ntl : i);
  };
  uint2 raw[16];
  if constexpr (kRowPrefetch<NQ> || kTilePrefetch<K, NQ>) {
    const uint32_t nc = tile_cols(tile_at(0));
    issue_rows(raw, (NQ > 1 && (kExp & 32)) ? T.zeros : shp + 2u * static_cast<size_t>(tile_at(0)) * kTile,
               (NQ > 1 && (kExp & 32)) ? 0 : a.shard_len, msk0[0],
               static_cast<uint32_t>(NQ == 1 ? 0 : seg_of<NQ>(0)) * K + 16 * g0, T.zeros, tid0 & 63u, nc,
               nc == kTile && aligned);
  }
  if constexpr (NQ > 1) {
    // multiplier tables of the first two segment transforms (indices 2K, 3K or
    // K, 0), or of all of them (kRecResident): kept for every tile
    stage_rec_tables<K, NQ>(T, VP);
    __syncthreads();
  }

#pragma unroll 1
  for (uint32_t t = 0; t < ntl; ++t) {
    // per-tile copies the compiler must treat as new: otherwise it hoists the
    // row offsets, sizes and descriptors derived from them out of the tile loop
    // and keeps them live in (spilled) registers across it
    const uint32_t g = fresh(g0);
    // (a copy of threadIdx.x kept across the tile loop was the kernel's one
    // spilled VGPR, and its reload waited with vmcnt(0) for every load in flight)
    const uint32_t lane = lane_fresh(), tid = 64u * g + lane;
    const uint32_t cqb = col_base<K>(4 * lane) ^ (32u * g);
    const size_t shard_len = fresh(a.shard_len);
    uint32_t msk[NQ];
#pragma unroll
    for (int i = 0; i < NQ; ++i) msk[i] = fresh(msk0[i]);
    const uint32_t tl = tile_at(t), col0 = tl * kTile, ncols = tile_cols(tl);
    const bool full = ncols == kTile && aligned;
    const uint8_t* sh = shp + 2u * static_cast<size_t>(col0);
    uint64_t* dbg = (kExp & 64) ? reinterpret_cast<uint64_t*>(a.out + static_cast<size_t>(pb) * a.out_stride +
                                                               static_cast<size_t>(nsyms) * 2 * K + ((kExp & 128) ? 4096u : 256u) * tl)
                                 : nullptr;
    stamp(dbg, 0);
    if constexpr (NQ >= 4 && !kRecResident<K, NQ>) {
      if (t > 0) {  // the first two segments' tables were replaced during the previous tile
        __syncthreads();
        stage_vpools<K, G::kThreads>(T, static_cast<uint32_t>(seg_of<NQ>(0)) * K, VP, true);
        stage_vpools<K, G::kThreads>(T, static_cast<uint32_t>(seg_of<NQ>(1)) * K, VP + G::kVPWords, true);
        __syncthreads();
      }
    }
    stamp(dbg, 1);
    uint32_t XL[16], XH[16];
    if constexpr (NQ > 1) {
      const uint32_t hb = col_base<K>(tid / G::R) ^ (8u * (tid % G::R));
      uint32_t AL[16], AH[16];
      RecCtx c{T, shard_len, tile, rows, sh, VP, g, lane, tid, ncols, full, cqb, hb, dbg, occ};
      // t > 0: step 0 waits for the previous tile's last LDS reads (its FFT's
      // cq_read, the copy-out) before writing the tile
      rec_segments<K, NQ, kTilePrefetch<K, NQ>>(c, msk, raw, AL, AH, t > 0 && (NQ == 2 || kRecResident<K, NQ>));
      // ---- forward transform of size K at index 0
      const uint32_t* vp0 = VP + vp_slot<K, NQ>(0, NQ - 1) * G::kVPWords;  // segment 0's tables = FFT(K, 0)'s
      stamp(dbg, 26);
      hi_levels<K, false, true, 0, 0, kRecPrioFwdHi>(T, vp0, 0, AL, AH);
      stamp(dbg, 27);
      __syncthreads();
      hi_write<K>(tile, fresh_v(hb), AL, AH);
      __syncthreads();
      stamp(dbg, 28);
      if constexpr (!kRowPrefetch<NQ>)  // the merge's rows load during the FFT's cq pass
        issue_rows(raw, sh, shard_len, uniform(msk[NQ - 1]), 16 * g, T.zeros, lane, ncols, full);
      cq_read<K>(tile, fresh_v(cqb), XL, XH);
      cq_levels<K, false, true, 0, false, kRecPrioFwdCq>(T, vp0, 0, g, XL, XH, ~uniform(msk[NQ - 1]));  // erased rows only
      stamp(dbg, 29);
    }
    // ---- merge: received systematic rows, postmultiplied recovered ones
    const uint32_t cqbf = fresh_v(cqb);
    const uint32_t m0 = uniform(msk[NQ == 1 ? 0 : NQ - 1]);  // segment 0 = the last step's
    if constexpr (NQ == 1) {
#pragma unroll
      for (int p = 0; p < 16; ++p) blk_to_quad(raw[p], XL[p], XH[p]);
    } else {
      pipelined_rec<16>(
          [&](auto pc) __attribute__((always_inline)) {
            NP_BNOTE(reinterpret_cast<const uint8_t*>(rows) + (16 * g + decltype(pc)::value) * 4 * kPoolWords,
                     4 * kPoolWords, kBkRecords);
            return (cpool_t)(fresh(rows)) + (16 * g + decltype(pc)::value) * kPoolWords;
          },
          [&](auto pc) __attribute__((always_inline)) { return ((m0 >> decltype(pc)::value) & 1u) == 0; },  // erased
          [&](auto pc, const Mult& pool) __attribute__((always_inline)) {
            constexpr int x = decltype(pc)::value;
            // present: the received symbol (mod.rs:225-235); erased: the
            // postmultiplied recovered symbol (inc_reconstruct.rs:76-84)
            if ((m0 >> x) & 1u) {
              blk_to_quad(raw[x], XL[x], XH[x]);
            } else {
              const uint32_t l = XL[x], h = XH[x];
              qmul_set(XL[x], XH[x], l, h, pool);
            }
          });
    }
    stamp(dbg, 30);
    // the next tile's first-step rows load during this tile's copy-out
    if constexpr (kRowPrefetch<NQ> || kTilePrefetch<K, NQ>) {
      if (t + 1 < ntl) {
        const uint32_t tn = tile_at(t + 1), nc = tile_cols(tn);
        issue_rows(raw, (NQ > 1 && (kExp & 32)) ? T.zeros : shp + 2u * static_cast<size_t>(tn) * kTile,
                   (NQ > 1 && (kExp & 32)) ? 0 : shard_len,
                   msk[0], static_cast<uint32_t>(NQ == 1 ? 0 : seg_of<NQ>(0)) * K + 16 * g, T.zeros, lane, nc,
                   nc == kTile && aligned);
      }
    }
    if (full && out_vec_ok(a.out, a.out_stride)) {
      copy_out_cq<K>(a.out + static_cast<size_t>(pb) * a.out_stride + static_cast<size_t>(col0) * 2 * K, lane, g, XL,
                     XH);
      stamp(dbg, 31);
      continue;
    }
    __syncthreads();
    cq_write<K>(tile, cqbf, XL, XH);
    __syncthreads();
    // ---- copy-out: column c of the tile is 2K contiguous bytes of the output
    {
      uint8_t* out = a.out + static_cast<size_t>(pb) * a.out_stride + static_cast<size_t>(col0) * 2 * K;
      const bool al_o = true;  // 8-byte stores at any address (rows_vec_ok)
      const uint32_t c0 = tid / G::Q, q0 = tid % G::Q;
      const uint32_t base = col_base<K>(c0) ^ (8u * q0);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const uint32_t c = c0 + 16u * i;
        if (c >= ncols) break;
        const uint2 v = *reinterpret_cast<const uint2*>(tile + (base ^ col_base_c<K>(16u * i)));
        uint8_t* o = NP_BCHK(out + static_cast<size_t>(c) * 2 * K + 8u * q0, 8, kBkOut);
        if (al_o) {
          *reinterpret_cast<uint2*>(o) = v;
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = static_cast<uint8_t>((e < 4 ? v.x : v.y) >> (8 * (e & 3)));
        }
      }
    }
    stamp(dbg, 31);
  }
}

// One workgroup: `tpw` consecutive 256-column tiles of one batch entry (the
// row multipliers and the staged tables of a payload serve all of them, and
// the next tile's rows load during a tile's copy-out), n = NQ * K.  Without
// caller locators (a.locators == nullptr) the workgroup decodes from the rows
// that k_prefix_locator chose (NQ' = 1: the K systematic rows, all present;
// NQ' = NQ: all n rows; NQ' = 2 for trusted codewords only; NQ' = 0: fewer
// than K present rows, no decode) with its row multipliers.  Caller locators
// are over all n rows, so they pin the full decode.  An instance serves the
// payloads whose prefix has
// at most SERVE segments (SERVE = 2: prefixes of 1 and 2 segments; SERVE = 4:
// the 4-segment ones only), so each code path gets its own register allocation;
// for n = 4K the host launches both over the same grid.
template <int K, int NQ, int SERVE>
__global__ __launch_bounds__(4 * K) __attribute__((amdgpu_waves_per_eu(4))) void k_reconstruct_fast(
    DevTables T, ReconstructArgs a, uint32_t nsyms, uint32_t tiles, uint32_t tpw) {
  constexpr int N = NQ * K;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
#if NP_BOUNDS_CHECK
  bounds_arm(bounds_of(a, T, prefix_stride_c(N, K)));
#endif
  const uint32_t groups = (tiles + tpw - 1) / tpw;  // workgroups per batch entry
  const TileRef tr = tile_of(blockIdx.x, groups, (a.batch & 7u) == 0);
  const uint32_t pb = tr.pb, tl0 = tr.tl * tpw;
  const uint32_t ntl = min(tpw, tiles - tl0);
  const uint8_t* pres = a.present + static_cast<size_t>(pb) * N;
  // the payload's decode prefix and row tables (k_prefix_locator, or
  // k_locator_records for caller locators)
  const uint8_t* rec = NP_BCHK(a.prefix + static_cast<size_t>(pb) * prefix_stride_c(N, K), 2, kBkRecords);
  const int nq = uniform(rec[0]);
  const uint32_t occ = uniform(rec[1]);  // segments with a present row
  const uint32_t* rows = reinterpret_cast<const uint32_t*>(rec + prefix_pools_offset(N));
  if constexpr (kMultiTile<K>) {
    if constexpr (SERVE >= 4) {
      if (nq == SERVE) rec_tiles<K, SERVE>(T, a, pres, rows, smem, pb, tl0, ntl, nsyms, occ);
    } else if (nq == 1) {
      rec_tiles<K, 1>(T, a, pres, rows, smem, pb, tl0, ntl, nsyms, occ);
    } else if (NQ <= 4 && nq == 2) {
      rec_tiles<K, 2>(T, a, pres, rows, smem, pb, tl0, ntl, nsyms, occ);
    }
  } else {  // tpw == 1
    const uint32_t col0 = tl0 * kTile;
    const uint32_t ncols = min(static_cast<uint32_t>(kTile), nsyms - col0);
    const uint8_t* sh = a.shards + static_cast<size_t>(pb) * a.batch_stride + 2 * static_cast<size_t>(col0);
    const bool full =
        ncols == kTile && rows_vec_ok(a.shards, a.batch_stride, a.shard_len);
    uint64_t* dbg = (kExp & 64) ? reinterpret_cast<uint64_t*>(a.out + static_cast<size_t>(pb) * a.out_stride +
                                                               static_cast<size_t>(nsyms) * 2 * K + ((kExp & 128) ? 4096u : 256u) * tl0)
                                 : nullptr;
    if constexpr (SERVE >= 4) {
      if (nq == SERVE) rec_tile<K, SERVE>(T, a, sh, pres, rows, smem, pb, col0, ncols, full, dbg, occ);
    } else if (nq == 1) {
      rec_tile<K, 1>(T, a, sh, pres, rows, smem, pb, col0, ncols, full, dbg, occ);
    } else if (NQ <= 4 && nq == 2) {
      rec_tile<K, 2>(T, a, sh, pres, rows, smem, pb, col0, ncols, full, dbg, occ);
    }
  }
}

// ---------------------------------------------------------- prefix locator ----
// The v_perm tables of row multipliers E[0..rows) into the record (thread
// tid copies the rows it wrote E for: no barrier).
// Present rows get the premultiply's tables (Cantor in, tower out: in_pools),
// erased rows the postmultiply's (tower in, Cantor out: out_pools).
__device__ __forceinline__ void write_row_pools(const DevTables& T, const uint16_t* E, const uint8_t* PR,
                                                uint32_t rows, uint8_t* dst) {
  for (uint32_t v = threadIdx.x; v < rows; v += 256) {
    const uint32_t* pools = PR[v] ? T.in_pools : T.out_pools;
    const uint4* src = reinterpret_cast<const uint4*>(pools + static_cast<size_t>(NP_ICHK(*NP_BCHK(E + v, 2, kBkRecords), 65536u)) * kPoolWords);
    uint4* d = NP_BCHK(reinterpret_cast<uint4*>(dst + static_cast<size_t>(v) * 4 * kPoolWords), 4 * kPoolWords, kBkRecords);
    const uint4 a0 = src[0], a1 = src[1], a2 = src[2], a3 = src[3], a4 = src[4];
    d[0] = a0, d[1] = a1, d[2] = a2, d[3] = a3, d[4] = a4;
  }
}


// One workgroup per payload: the decode prefix (rec_tile) and the erasure
// locator folded to it (fused_locator, SURVEY F8: eval_error_polynomial
// inc_reconstruct.rs:90-113 over [0, NQ' * K)), as row multipliers EXP[loc]
// (present) / EXP[-loc] (erased).  Record: byte 0 = NQ' in {1, 2, NQ}, byte 1
// the segment occupancy, the rows' 80-byte multiplier tables from
// prefix_pools_offset (k_locator_records also leaves the u16 multipliers at
// kPrefixHeader; the decodes read only the tables).  Computed once per payload
// instead of once per column tile.
// Present rows of payload pb in [0, K), [0, 2K) and [0, N) (256 threads).
template <int K, int N>
__device__ __forceinline__ void count_present(const uint8_t* pres, int& have1, int& have2, int& have) {
  have1 = have2 = have = 0;
  for (int r = 0; r < N; r += 256) {
    const int v = static_cast<int>(threadIdx.x) + r;
    const bool p = v < N && *NP_BCHK(pres + v, 1, kBkPresent) != 0;
    if (r < K) have1 += __syncthreads_count(v < K && p);
    if (r < 2 * K) have2 += __syncthreads_count(v < 2 * K && p);
    have += __syncthreads_count(p);
  }
}

// Bit q: segment q (rows [qK, (q+1)K)) holds a present row (record byte 1:
// the decodes skip the transforms of empty segments).
template <int K, int N>
__device__ __forceinline__ uint32_t segment_occupancy(const uint8_t* pres) {
  uint32_t occ = 0;
#pragma unroll 1
  for (int q = 0; q < N / K; ++q) {
    int any = 0;
    for (int v = static_cast<int>(threadIdx.x); v < K; v += 256) any |= *NP_BCHK(pres + (q * K + v), 1, kBkPresent) != 0;
    if (__syncthreads_or(any)) occ |= 1u << q;
  }
  return occ;
}

// Status of payload pb (launchers.hpp ReconstructArgs::status); true if it
// decodes.
__device__ __forceinline__ bool write_status(const ReconstructArgs& a, uint32_t pb, int have) {
  const bool ok = have >= static_cast<int>(a.k);  // mod.rs:178-180
  if (threadIdx.x == 0 && a.status) {
    *NP_BCHK(a.status + 2 * pb, 4, kBkStatus) = ok ? 0u : kStatusNeedMoreShards;
    *NP_BCHK(a.status + 2 * pb + 1, 4, kBkStatus) = static_cast<uint32_t>(have);
  }
  return ok;
}

// Threads of k_prefix_locator for n = N rows: 512 from N = 512 on, so that
// each thread's chain of dependent loads (flag, multiplier, its 80-byte
// table) runs N / 512 times.  Config 3 (N = 1024), with the counters summed
// per wave before the LDS atomics: 256 threads 51.0 / 50.6 us per launch,
// 512 49.8 / 50.0, 1024 54.5 / 54.6 (two workgroups per CU instead of four;
// profiles/r06/prefix_threads.txt); 55.4 before the wave sums.
template <int N>
constexpr int kPrefixThreads = N >= 512 ? 512 : 256;

// NQ' = 0 marks a payload with fewer than K present rows: no decode.
template <int K, int NQ, int NT = kPrefixThreads<NQ * K>>
__global__ __launch_bounds__(NT) void k_prefix_locator(DevTables T, ReconstructArgs a, uint8_t* out) {
  constexpr int N = NQ * K;
  __shared__ uint32_t W[N];
  __shared__ uint8_t PR[N];
  const uint32_t pb = blockIdx.x, tid = threadIdx.x;
#if NP_BOUNDS_CHECK
  {
    ReconstructArgs ab = a;
    ab.prefix = out;
    bounds_arm(bounds_of(ab, T, prefix_stride_c(N, K)));
  }
#endif
  const uint8_t* pres = a.present + static_cast<size_t>(pb) * N;
  uint8_t* rec = out + static_cast<size_t>(pb) * prefix_stride_c(N, K);
  // One pass over the present flags: PR, the erasure indicator W for the
  // locator, the present rows in [0, K), [0, 2K), [0, N) and the segments
  // holding one (was count_present + segment_occupancy + the locator's own
  // load: 17 barriers fewer).
  __shared__ uint32_t acc[4];  // have1, have2, have, occupancy
  if (tid < 4) acc[tid] = 0;
  __syncthreads();
  {
    uint32_t c1 = 0, c2 = 0, c = 0, occ = 0;
    for (uint32_t v = tid; v < static_cast<uint32_t>(N); v += NT) {
      const uint8_t p = *NP_BCHK(pres + v, 1, kBkPresent);
      PR[v] = p;
      W[v] = p ? 0u : 1u;
      const uint32_t on = p ? 1u : 0u;
      c += on;
      c1 += v < static_cast<uint32_t>(K) ? on : 0u;
      c2 += v < 2u * K ? on : 0u;
      occ |= on << (v / K);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {  // wave sums first: one LDS atomic per wave and counter
      c1 += __shfl_xor(c1, o);
      c2 += __shfl_xor(c2, o);
      c += __shfl_xor(c, o);
      occ |= __shfl_xor(occ, o);
    }
    if ((tid & 63u) == 0) {
      atomicAdd(&acc[0], c1);
      atomicAdd(&acc[1], c2);
      atomicAdd(&acc[2], c);
      atomicOr(&acc[3], occ);
    }
  }
  __syncthreads();
  const int have1 = static_cast<int>(acc[0]), have2 = static_cast<int>(acc[1]), have = static_cast<int>(acc[2]);
  // All K systematic rows present: the output is those rows (the reference
  // copies received rows < k, inc_reconstruct.rs:46-50), exact for any input.
  // Otherwise the full decode from every present row, as the reference
  // (inc_reconstruct.rs:61-85); the 2K-row prefix only for trusted codewords.
  const int nq = !write_status(a, pb, have) ? 0 : have1 == K ? 1 : (a.trusted && NQ == 4 && have2 >= K) ? 2 : NQ;
  if (tid == 0) *NP_BCHK(rec, 2, kBkRecords) = static_cast<uint8_t>(nq), *NP_BCHK(rec + 1, 1, kBkRecords) = static_cast<uint8_t>(acc[3]);
  if (nq <= 1) return;
  // the row tables straight from the multipliers (the decodes read only the
  // tables, not the u16 multipliers)
  if (NQ == 4 && nq == 2) {
    fused_locator_pools<2 * K, NT>(T, W, PR, rec + prefix_pools_offset(N));  // the first 2K entries of W and PR
  } else {
    fused_locator_pools<N, NT>(T, W, PR, rec + prefix_pools_offset(N));
  }
}

// The record for caller locators (log form, all n rows: the full decode,
// NQ' = NQ): row multipliers EXP[loc] and their tables.  One workgroup per
// payload.
template <int K, int NQ>
__global__ __launch_bounds__(256) void k_locator_records(DevTables T, ReconstructArgs a, uint8_t* out) {
  constexpr int N = NQ * K;
  const uint32_t pb = blockIdx.x, tid = threadIdx.x;
#if NP_BOUNDS_CHECK
  {
    ReconstructArgs ab = a;
    ab.prefix = out;
    bounds_arm(bounds_of(ab, T, prefix_stride_c(N, K)));
  }
#endif
  const uint16_t* loc = a.locators + static_cast<size_t>(pb) * N;
  uint8_t* rec = out + static_cast<size_t>(pb) * prefix_stride_c(N, K);
  uint16_t* E = reinterpret_cast<uint16_t*>(rec + kPrefixHeader);
  int have1, have2, have;
  count_present<K, N>(a.present + static_cast<size_t>(pb) * N, have1, have2, have);
  const bool ok = write_status(a, pb, have);
  const uint32_t occ = segment_occupancy<K, N>(a.present + static_cast<size_t>(pb) * N);
  if (tid == 0) *NP_BCHK(rec, 2, kBkRecords) = static_cast<uint8_t>(ok ? NQ : 0), *NP_BCHK(rec + 1, 1, kBkRecords) = static_cast<uint8_t>(occ);
  if (!ok) return;
  // mul(x, log m) == x * EXP[m] (inc_log_mul.rs:42-49)
  for (uint32_t v = tid; v < static_cast<uint32_t>(N); v += 256) *NP_BCHK(E + v, 2, kBkRecords) = T.exp[*NP_BCHK(loc + v, 2, kBkLocators)];
  write_row_pools(T, E, a.present + static_cast<size_t>(pb) * N, N, rec + prefix_pools_offset(N));
}

// ------------------------------------------------------------- launchers ----
template <int K>
size_t encode_lds_bytes() {
  return static_cast<size_t>(Geo<K>::kTileBytes) + 4u * 4u * Geo<K>::kVPWords;  // up to 4 resident tables
}

template <int K>
size_t encode_multi_lds_bytes() {
  return static_cast<size_t>(Geo<K>::kTileBytes) + kEncBuffers * 4u * Geo<K>::kVPWords;
}


template <int K, int NQ>
size_t reconstruct_lds_bytes() {
  return static_cast<size_t>(Geo<K>::kTileBytes) + (kRecResident<K, NQ> ? NQ : 2) * 4u * Geo<K>::kVPWords;
}

// Tiles per workgroup (kMultiTile): as many as keep >= kWorkgroups
// workgroups (4 per CU on 256 CUs) in the grid.  `knob` names an environment
// variable that pins the count (tests).
constexpr size_t kWorkgroups = 1024;

template <int K>
uint32_t tiles_per_workgroup(size_t batch, uint32_t tiles, const char* knob) {
  if (!kMultiTile<K>) return 1;
  size_t want = batch * tiles / kWorkgroups;
  if (const char* e = std::getenv(knob)) want = std::strtoul(e, nullptr, 10);
  return static_cast<uint32_t>(std::max<size_t>(1, std::min<size_t>(tiles, want)));
}

template <int K>
hipError_t launch_encode_k(const DevTables& T, const EncodeArgs& a, hipStream_t s) {
  const size_t nchunks = (a.payload_len + 2 * a.k - 1) / (2 * a.k);
  if (nchunks == 0 || a.batch == 0) return hipSuccess;
  if (nchunks > 0xffffffffu) return hipErrorInvalidValue;
  const uint32_t tiles = static_cast<uint32_t>((nchunks + kTile - 1) / kTile);
  const uint32_t tpw = a.n <= kEncBuffers * K ? tiles_per_workgroup<K>(a.batch, tiles, "NP_ENC_TPW") : 1u;
  const size_t blocks = a.batch * ((tiles + tpw - 1) / tpw);
  if (blocks > 0x7fffffffu) return hipErrorInvalidValue;
  if constexpr (kMultiTile<K>) {
    if (a.n <= kEncBuffers * K) {
      k_encode_multi<K><<<static_cast<uint32_t>(blocks), Geo<K>::kThreads, encode_multi_lds_bytes<K>(), s>>>(
          EncLaunch{T, a, static_cast<uint32_t>(nchunks), tiles, tpw});
      return hipGetLastError();
    }
  }
  k_encode_fast<K><<<static_cast<uint32_t>(blocks), Geo<K>::kThreads, encode_lds_bytes<K>(), s>>>(
      T, a, static_cast<uint32_t>(nchunks), tiles);
  return hipGetLastError();
}

template <int K, int NQ>
hipError_t launch_prefix_k(const DevTables& T, const ReconstructArgs& a, uint8_t* out, hipStream_t s) {
  if (a.batch == 0) return hipSuccess;
  if (a.batch > 0x7fffffffu) return hipErrorInvalidValue;
  if (a.locators)
    k_locator_records<K, NQ><<<static_cast<uint32_t>(a.batch), 256, 0, s>>>(T, a, out);
  else
    k_prefix_locator<K, NQ><<<static_cast<uint32_t>(a.batch), kPrefixThreads<NQ * K>, 0, s>>>(T, a, out);
  return hipGetLastError();
}

template <int K, int NQ>
hipError_t launch_reconstruct_k(const DevTables& T, const ReconstructArgs& a, hipStream_t s) {
  const size_t nsyms = a.shard_len / 2;
  if (nsyms == 0 || a.batch == 0) return hipSuccess;
  if (nsyms > 0xffffffffu) return hipErrorInvalidValue;
  const uint32_t tiles = static_cast<uint32_t>((nsyms + kTile - 1) / kTile);
  const uint32_t tpw = tiles_per_workgroup<K>(a.batch, tiles, "NP_REC_TPW");
  const size_t blocks = a.batch * ((tiles + tpw - 1) / tpw);
  if (blocks > 0x7fffffffu) return hipErrorInvalidValue;
  k_reconstruct_fast<K, NQ, 2><<<static_cast<uint32_t>(blocks), Geo<K>::kThreads, reconstruct_lds_bytes<K, NQ>(), s>>>(
      T, a, static_cast<uint32_t>(nsyms), tiles, tpw);
  if constexpr (NQ >= 4)
    k_reconstruct_fast<K, NQ, NQ><<<static_cast<uint32_t>(blocks), Geo<K>::kThreads, reconstruct_lds_bytes<K, NQ>(), s>>>(
        T, a, static_cast<uint32_t>(nsyms), tiles, tpw);
  return hipGetLastError();
}

// f(K, NQ) with NQ = n / k in {2, 4, 8} as compile-time constants.
template <int K, typename F>
hipError_t by_nq(const ReconstructArgs& a, F f) {
  using KC = std::integral_constant<int, K>;
  if (a.n == 8u * K) return f(KC{}, std::integral_constant<int, 8>{});
  if (a.n == 4u * K) return f(KC{}, std::integral_constant<int, 4>{});
  return f(KC{}, std::integral_constant<int, 2>{});
}

}  // namespace

bool fast_encode_supported(uint32_t n, uint32_t k) {
  return ((k == 64 || k == 128 || k == 256) && n >= 2 * k && n <= 65536) || small_encode_supported(n, k);
}

bool fast_reconstruct_supported(uint32_t n, uint32_t k) {
  return ((k == 64 || k == 128 || k == 256) && (n == 2 * k || n == 4 * k || n == 8 * k)) ||
         small_reconstruct_supported(n, k);
}

hipError_t launch_encode_fast(const DevTables& T, const EncodeArgs& a, hipStream_t s) {
  switch (a.k) {
    case 64: return launch_encode_k<64>(T, a, s);
    case 128: return launch_encode_k<128>(T, a, s);
    case 256: return launch_encode_k<256>(T, a, s);
    case 1:
    case 2:
    case 4:
    case 8:
    case 16:
    case 32: return launch_encode_small(T, a, s);
    default: return hipErrorNotSupported;
  }
}

size_t prefix_stride(uint32_t n, uint32_t k) { return prefix_stride_c(n, k); }

hipError_t launch_prefix_locator(const DevTables& T, const ReconstructArgs& a, uint8_t* out, hipStream_t s) {
  switch (a.k) {
    case 64: return by_nq<64>(a, [&](auto K, auto NQ) { return launch_prefix_k<K.value, NQ.value>(T, a, out, s); });
    case 128: return by_nq<128>(a, [&](auto K, auto NQ) { return launch_prefix_k<K.value, NQ.value>(T, a, out, s); });
    case 256: return by_nq<256>(a, [&](auto K, auto NQ) { return launch_prefix_k<K.value, NQ.value>(T, a, out, s); });
    case 1: return by_nq<1>(a, [&](auto K, auto NQ) { return launch_prefix_k<K.value, NQ.value>(T, a, out, s); });
    case 2: return by_nq<2>(a, [&](auto K, auto NQ) { return launch_prefix_k<K.value, NQ.value>(T, a, out, s); });
    case 4: return by_nq<4>(a, [&](auto K, auto NQ) { return launch_prefix_k<K.value, NQ.value>(T, a, out, s); });
    case 8: return by_nq<8>(a, [&](auto K, auto NQ) { return launch_prefix_k<K.value, NQ.value>(T, a, out, s); });
    case 16: return by_nq<16>(a, [&](auto K, auto NQ) { return launch_prefix_k<K.value, NQ.value>(T, a, out, s); });
    case 32: return by_nq<32>(a, [&](auto K, auto NQ) { return launch_prefix_k<K.value, NQ.value>(T, a, out, s); });
    case 512: return by_nq<512>(a, [&](auto K, auto NQ) { return launch_prefix_k<K.value, NQ.value>(T, a, out, s); });  // kernels_res.hip
    case 1024: return by_nq<1024>(a, [&](auto K, auto NQ) { return launch_prefix_k<K.value, NQ.value>(T, a, out, s); });  // kernels_res.hip
    default: return hipErrorNotSupported;
  }
}

hipError_t launch_reconstruct_fast(const DevTables& T, const ReconstructArgs& a, hipStream_t s) {
  switch (a.k) {
    case 64: return by_nq<64>(a, [&](auto K, auto NQ) { return launch_reconstruct_k<K.value, NQ.value>(T, a, s); });
    case 128: return by_nq<128>(a, [&](auto K, auto NQ) { return launch_reconstruct_k<K.value, NQ.value>(T, a, s); });
    case 256: return by_nq<256>(a, [&](auto K, auto NQ) { return launch_reconstruct_k<K.value, NQ.value>(T, a, s); });
    case 1:
    case 2:
    case 4:
    case 8:
    case 16:
    case 32: return launch_reconstruct_small(T, a, s);
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
  set(reinterpret_cast<const void*>(&k_encode_multi<256>), encode_multi_lds_bytes<256>());
  set(reinterpret_cast<const void*>(&k_reconstruct_fast<64, 2, 2>), reconstruct_lds_bytes<64, 2>());
  set(reinterpret_cast<const void*>(&k_reconstruct_fast<64, 4, 2>), reconstruct_lds_bytes<64, 4>());
  set(reinterpret_cast<const void*>(&k_reconstruct_fast<64, 4, 4>), reconstruct_lds_bytes<64, 4>());
  set(reinterpret_cast<const void*>(&k_reconstruct_fast<128, 2, 2>), reconstruct_lds_bytes<128, 2>());
  set(reinterpret_cast<const void*>(&k_reconstruct_fast<128, 4, 2>), reconstruct_lds_bytes<128, 4>());
  set(reinterpret_cast<const void*>(&k_reconstruct_fast<128, 4, 4>), reconstruct_lds_bytes<128, 4>());
  set(reinterpret_cast<const void*>(&k_reconstruct_fast<256, 2, 2>), reconstruct_lds_bytes<256, 2>());
  set(reinterpret_cast<const void*>(&k_reconstruct_fast<256, 4, 2>), reconstruct_lds_bytes<256, 4>());
  set(reinterpret_cast<const void*>(&k_reconstruct_fast<256, 4, 4>), reconstruct_lds_bytes<256, 4>());
  set(reinterpret_cast<const void*>(&k_reconstruct_fast<64, 8, 2>), reconstruct_lds_bytes<64, 8>());
  set(reinterpret_cast<const void*>(&k_reconstruct_fast<64, 8, 8>), reconstruct_lds_bytes<64, 8>());
  set(reinterpret_cast<const void*>(&k_reconstruct_fast<128, 8, 2>), reconstruct_lds_bytes<128, 8>());
  set(reinterpret_cast<const void*>(&k_reconstruct_fast<128, 8, 8>), reconstruct_lds_bytes<128, 8>());
  set(reinterpret_cast<const void*>(&k_reconstruct_fast<256, 8, 2>), reconstruct_lds_bytes<256, 8>());
  set(reinterpret_cast<const void*>(&k_reconstruct_fast<256, 8, 8>), reconstruct_lds_bytes<256, 8>());
  return e;
}

hipError_t bounds_take_fast(uint32_t out[8]) { return bounds_take_tu(out); }

}  // namespace np
