// k = 512 and 1024 resident kernels: encode (k_encode_res) and reconstruct
// (k_reconstruct_res) of a 64-column tile with the whole size-K transform in
// the workgroup.  Layouts, levels and row I/O: res_common.hpp.
#include "res_common.hpp"

namespace np {
namespace {

// Progress-based issue priority in every transform pass of the resident
// kernels (fast_common.hpp progress_prio).  Measured (profiles/r04_ab.txt
// probe 23): config-4 encode 2.545 / 2.550 -> 2.422 / 2.424 ms, reconstruct
// 4.376 / 4.381 -> 4.168 / 4.166 ms (-4.8 % each); 2000 validators (k = 512)
// reconstruct -4.3 %, encode unchanged.  (One schedule over each decode step's
// span from the row tables' barrier to the CQ write, as the fast decode has,
// measured +2.4 % at config 4, probe 24.)
constexpr int kResPrioEnc = 1, kResPrioDec = 1, kResPrioDecCq = 1;

// ---------------------------------------------------------------- encode ----
// One workgroup: 64 chunks of one payload.  mod.rs:144-154 /
// inc_encode.rs:15-48: IFFT(K, 0) of each chunk -> coefficients M (HD
// layout, registers), then per shift s the FFT(K, K s) -> shard rows
// K s .. K s + K - 1; rows 0..K-1 are the payload itself.
template <int K>
__global__ __launch_bounds__(K) __attribute__((amdgpu_waves_per_eu(4))) void k_encode_res(
    DevTables T, EncodeArgs a, uint32_t nchunks, uint32_t tiles) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* tile = smem;
#if NP_BOUNDS_CHECK
  bounds_arm(bounds_of_enc(a));
#endif
  const TileRef tr = tile_of(blockIdx.x, tiles, (a.batch & 7u) == 0);
  const uint32_t pb = tr.pb, tl = tr.tl;
  const uint32_t ch0 = tl * kRC;
  const uint32_t ncols = min(static_cast<uint32_t>(kRC), nchunks - ch0);
  const uint8_t* pay = a.payloads + static_cast<size_t>(pb) * a.payload_stride;
  uint8_t* out = a.shards + static_cast<size_t>(pb) * a.batch_stride + 2 * static_cast<size_t>(ch0);
  const Res r = res_coords<K>();
  const Qi qc = qi_coords<K>(r);
  const bool full =
      ncols == kRC && rows_vec_ok(a.shards, a.batch_stride, a.shard_len);
  const bool nt = rows_nt(a.shards, a.batch_stride, a.shard_len);
  const uint32_t wanted_store = ((kExp & 2) && a.k != 12345u) ? 0u : a.wanted_n;  // experiment: no stores

  load_pay_tile<K>(tile, pay, a.payload_len, ch0, 2 * K, 0, r.tid);
  const uint32_t nshift = a.n / K;
  uint32_t* DL = reinterpret_cast<uint32_t*>(smem + RGeo<K>::kTileBytes);  // CQ delta tables
  uint32_t* VS = DL + kDeltaWords;                                           // HA / HD tables, RStage
  stage_delta_tables(T, DL);
  stage_rh_tables<K>(T, VS, nshift);
  __syncthreads();
  // ---- CQ: systematic rows, inverse levels 0-3 (index 0: every multiplier in GF(2^8))
  {
    uint32_t L[16], H[16];
    rcq_read_nat<K>(tile, r.cqb, L, H);
    rres_store_rows(out, a.shard_len, 0, wanted_store, L, H, r, ncols, full, nt);
    tower_convert(T, L, H);  // the transforms run in tower coordinates
    rcq_levels<true, res_gen<K>(0), true, kResPrioEnc>(T, 0, r, L, H, DL);
    __syncthreads();  // every wave has read its payload blocks
    qi_cq<true>(tile, qc, L, H);
  }
  __syncthreads();
  uint32_t ML[16], MH[16];
  {
    uint32_t L[16], H[16];
    qi_ha<false>(tile, qc, L, H);
    ha_levels_st<K, true, 0, kResPrioEnc>(T, 0, r, L, H, VS);
    __syncthreads();
    qi_ha<true>(tile, qc, L, H);
    __syncthreads();
    qi_hd<K, false>(tile, qc, ML, MH);
  }
  hd_levels_st<K, true, kResPrioEnc>(T, 0, ML, MH, VS);
#pragma unroll
  for (int q = 0; q < 16; ++q) asm volatile("" : "+v"(ML[q]), "+v"(MH[q]));  // materialise M once

  auto shift = [&](auto gc, uint32_t sh) __attribute__((always_inline)) {
    constexpr int GEN = decltype(gc)::value;
    const uint32_t I = sh * K;
    uint32_t L[16], H[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      L[q] = ML[q];
      H[q] = MH[q];
    }
    const uint32_t* vs = VS + sh * RStage<K>::kWords;
    hd_levels_st<K, false, kResPrioEnc>(T, I, L, H, vs);
    __syncthreads();  // the previous CQ pass is done with the tile
    qi_hd<K, true>(tile, qc, L, H);
    __syncthreads();
    qi_ha<false>(tile, qc, L, H);
    ha_levels_st<K, false, GEN, kResPrioEnc>(T, I, r, L, H, vs);
    __syncthreads();
    qi_ha<true>(tile, qc, L, H);
    __syncthreads();
    qi_cq<false>(tile, qc, L, H);
    rcq_levels<false, GEN, true, kResPrioEnc>(T, I, r, L, H, DL);
    tower_convert(T, L, H);  // back to Cantor coordinates for the shard rows
    rres_store_rows(out, a.shard_len, I, wanted_store, L, H, r, ncols, full, nt);
  };
  if (nshift > 1 && K < a.wanted_n) shift(Int<res_gen<K>(K)>{}, 1);
#pragma unroll 1
  for (uint32_t sh = 2; sh < 4 && sh < nshift && sh * K < a.wanted_n; ++sh) shift(Int<res_gen<K>(2 * K)>{}, sh);
#pragma unroll 1
  for (uint32_t sh = 4; sh < nshift && sh * K < a.wanted_n; ++sh) shift(Int<res_gen<K>(4 * K)>{}, sh);  // n = 8K
}

// Experiment builds (NP_EXP bit 6): lane 0 of every wave writes s_memtime to
// dbg[64 wave + slot] (tools/res_stamps.py; slots: 0 start, 1 tables, 2 + 8
// step + phase for the segment steps, 40.. the forward transform and merge).
__device__ __forceinline__ void rstamp(uint64_t* dbg, int slot) {
  if constexpr ((kExp & 64) != 0) {
    if ((threadIdx.x & 63u) == 0) dbg[64u * (threadIdx.x >> 6) + slot] = __builtin_amdgcn_s_memtime();
  }
}

// The decode's full CQ levels through per-lane full tables (rcq_group ST),
// except in the k = 1024, 8-segment instance, where the tables' 20 VGPRs
// made the allocator spill 60 dwords instead of 15.
template <int K, int NQ>
constexpr bool kRecDeltaST = !(K == 1024 && NQ == 8);

// A segment step's row tables arrive by LDS-DMA issued during the previous
// step's HD levels and fold (dma_row_tables), instead of by loads and LDS
// writes between two barriers at the start of the step.  Measured: config-4
// decode 4.37 / 4.38 ms with, 4.37 / 4.36 without (noise, profiles/r04_ab.txt);
// kept, it leaves the step start to the row loads.

// K = 256 (the decode A/B of DESIGN.md §8, NP_REC_RES256): 8 levels, CQ 0-3
// and HA 4-7, so there are no HD levels.  Each x_q stays in HA, and so does d
// (the folds are elementwise); only D(x0) goes through HD (its position bits
// 2-3 are in lanes there), and back.  One exchange per segment instead of two.
template <int K>
constexpr bool kResNoHD = (K == 256);

template <int NQ>
__host__ __device__ constexpr int res_seg(int step) {  // segments 2, 3, 1, 0 (NQ = 4); 1, 0 (NQ = 2); 7..0 (NQ = 8)
  return NQ == 8 ? 7 - step : NQ == 4 ? (step == 0 ? 2 : step == 1 ? 3 : 3 - step) : 1 - step;
}

// Step STEP of the segment sweep: x_q = IFFT(K, K q)(premultiplied
// segment q), folded into d (A, HD layout).  Steps are compile-time: each has
// one CQ instance (its GEN) and its own fold, with no runtime branch between
// instances (a branch over instances inside a loop made the allocator spill).

template <int K, int NQ, int STEP>
__device__ __forceinline__ bool res_step(const DevTables& T, const ReconstructArgs& a, uint8_t* tile,
                                         const uint8_t* pools, const uint8_t* pres, const uint8_t* sh,
                                         uint8_t* out_tile, uint32_t ncols, bool full, bool out16, uint32_t (&AL)[16],
                                         uint32_t (&AH)[16], uint64_t* dbg, uint32_t occ) {
  constexpr int q = res_seg<NQ>(STEP);
  constexpr int s0 = 2 + 8 * STEP;
  constexpr uint32_t I = static_cast<uint32_t>(q) * K;
  constexpr uint32_t kHD = RGeo<K>::kHD;
  const Res rr = res_coords<K>();  // opaque per step: lane-derived values are not hoisted across steps
  uint32_t XL[16], XH[16];
  // 8 segments: a segment without a present row gives x_q = 0 (record byte 1,
  // kernels_fast.hip segment_occupancy; e.g. the rows past wanted_n at 2,500,
  // 3,000 and 5,000 validators): no loads, transform or exchanges, only the
  // next step's row tables and the fold.
  if (NQ == 8 && !((occ >> q) & 1u)) {
#pragma unroll
    for (int j = 0; j < 16; ++j) XL[j] = XH[j] = 0;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this step's table pieces (LDS-DMA into the tile)
    if constexpr (STEP + 1 < NQ) {
      __syncthreads();  // every wave's
      dma_row_tables(tile, pools, static_cast<uint32_t>(res_seg<NQ>(STEP + 1)) * K, K, rr.w, rr.l, K / 64);
    }
  } else {
  {
    const uint32_t pm = lane_rows_present(pres, I, rr);
    uint2 raw[8];
    // this step's tables were issued by LDS-DMA during the previous step
    // (res_decode_tile for step 0): wait for this wave's pieces before the
    // row loads queue behind them, then for every wave's
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    load_lane_rows<8>(raw, sh, a.shard_len, I, pm, rr, ncols, full, T.zeros, 0);
    __syncthreads();
    rstamp(dbg, s0);
    // premultiply by the row multipliers (inc_reconstruct.rs:72-74; Cantor
    // in, tower out), in two halves of 8 rows (register pressure)
#pragma unroll
    for (int half = 0; half < 2; ++half) {
      if (half == 1) load_lane_rows<8>(raw, sh, a.shard_len, I, pm, rr, ncols, full, T.zeros, 8);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        uint32_t l, h;
        blk_to_quad(raw[i], l, h);
        const FullT m = row_table(tile, 64u * rr.w + 16u * rr.u + 8 * half + i);
        qmul_set_vv(XL[8 * half + i], XH[8 * half + i], l, h, m);
      }
    }
  }
  rstamp(dbg, s0 + 1);
  if constexpr ((kExp & 16384) != 0 && STEP == 0) {  // experiment: the first step's premultiplied rows
    res_copy_out<K>(out_tile, XL, XH, rr, ncols, out16);
    return false;
  }
  const uint32_t* DL = reinterpret_cast<const uint32_t*>(tile + RGeo<K>::kTileBytes);
  rcq_levels<true, res_gen<K>(I), kRecDeltaST<K, NQ>, kResPrioDecCq>(T, I, rr, XL, XH, DL);
  if constexpr ((kExp & 32768) != 0 && STEP == 0) {  // experiment: the first step after its CQ levels
    res_copy_out<K>(out_tile, XL, XH, rr, ncols, out16);
    return false;
  }
  rstamp(dbg, s0 + 2);
  __syncthreads();  // every wave has read its row tables
  rcq_write<K>(tile, fresh_v(rr.cqb), XL, XH);
  __syncthreads();
  rh_read<kHA>(tile, fresh_v(rr.hab), XL, XH);
  rstamp(dbg, s0 + 3);
  const uint32_t* vs = DL + kDeltaWords + q * RStage<K>::kWords;
  if constexpr (kResNoHD<K>) {
    // K = 256: HA holds every level above 3, x_q stays there and d with it
    if constexpr (STEP + 1 < NQ) {
      __syncthreads();  // every wave has read the tile: the next step's tables may land in it
      dma_row_tables(tile, pools, static_cast<uint32_t>(res_seg<NQ>(STEP + 1)) * K, K, rr.w, rr.l, K / 64);
    }
    ha_levels_st<K, true, res_gen<K>(I), kResPrioDec>(T, I, rr, XL, XH, vs);
    rstamp(dbg, s0 + 4);
    if constexpr (q == 0) {
      // D(x0) needs position bits 2-3 in one wave: through HD and back
      __syncthreads();  // every wave has read its HA items
      rh_write<kHA>(tile, fresh_v(rr.hab), XL, XH);
      __syncthreads();
      rh_read<kHD>(tile, fresh_v(rr.hdb), XL, XH);
      uint32_t YL[16], YH[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        YL[j] = (NQ == 2 || NQ == 8) ? XL[j] : 0u;  // d = D(x0) ^ x0 ^ ..
        YH[j] = (NQ == 2 || NQ == 8) ? XH[j] : 0u;
      }
      add_derivative_hd<K>(YL, XL, rr.l);
      add_derivative_hd<K>(YH, XH, rr.l);
      __syncthreads();
      rh_write<kHD>(tile, fresh_v(rr.hdb), YL, YH);
      __syncthreads();
      rh_read<kHA>(tile, fresh_v(rr.hab), YL, YH);
#pragma unroll
      for (int j = 0; j < 16; ++j) AL[j] ^= YL[j], AH[j] ^= YH[j];
      rstamp(dbg, s0 + 7);
      return true;
    }
  } else {
  ha_levels_st<K, true, res_gen<K>(I), kResPrioDec>(T, I, rr, XL, XH, vs);
  rstamp(dbg, s0 + 4);
  __syncthreads();
  rh_write<kHA>(tile, fresh_v(rr.hab), XL, XH);
  __syncthreads();
  rh_read<kHD>(tile, fresh_v(rr.hdb), XL, XH);
  if constexpr (STEP + 1 < NQ) {
    __syncthreads();  // every wave has read the tile: the next step's tables may land in it
    dma_row_tables(tile, pools, static_cast<uint32_t>(res_seg<NQ>(STEP + 1)) * K, K, rr.w, rr.l, K / 64);
  }
  rstamp(dbg, s0 + 5);
  hd_levels_st<K, true, kResPrioDec>(T, I, XL, XH, vs);
  rstamp(dbg, s0 + 6);
  }
  }
  // fold x_q into d (kernels_fast.hip rec_segments)
  if constexpr (NQ == 8 && q != 0 && rec8_kappa_res(q) != 1u) {  // d ^= kappa_q x_q, kappa_q in GF(16)
    uint32_t kp[20];
    pool_of<true>(T, rec8_kappa_res(q), kp);
    const Mult m = make_mult(kp);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if constexpr (STEP == 0)
        qmul_sub_set(AL[j], AH[j], XL[j], XH[j], m);
      else
        qmul_sub(AL[j], AH[j], XL[j], XH[j], m);
    }
  } else if constexpr (STEP == 0) {
#pragma unroll
    for (int j = 0; j < 16; ++j) AL[j] = XL[j], AH[j] = XH[j];
  } else if constexpr (q == 0) {
    if constexpr (NQ == 2 || NQ == 8) {
#pragma unroll
      for (int j = 0; j < 16; ++j) AL[j] ^= XL[j], AH[j] ^= XH[j];
    }
    add_derivative_hd<K>(AL, XL, rr.l);
    add_derivative_hd<K>(AH, XH, rr.l);
  } else if constexpr (NQ == 4 && q == 3) {  // A = x2 ^ beta (x2 ^ x3)
    uint32_t beta[20];
    pool_of<true>(T, 2u, beta);  // beta = Cantor(2), in GF(2^8)
    const Mult m = make_mult(beta);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      XL[j] ^= AL[j];
      XH[j] ^= AH[j];
      qmul_sub(AL[j], AH[j], XL[j], XH[j], m);
    }
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j) AL[j] ^= XL[j], AH[j] ^= XH[j];
  }
  rstamp(dbg, s0 + 7);
  return true;
}

template <int K, int NQ, int... STEP>
__device__ __forceinline__ bool res_sweep(const DevTables& T, const ReconstructArgs& a, uint8_t* tile,
                                          const uint8_t* pools, const uint8_t* pres, const uint8_t* sh,
                                          uint8_t* out_tile, uint32_t ncols, bool full, bool out16,
                                          uint32_t (&AL)[16], uint32_t (&AH)[16], uint64_t* dbg, uint32_t occ,
                                          std::integer_sequence<int, STEP...>) {
  return (res_step<K, NQ, STEP>(T, a, tile, pools, pres, sh, out_tile, ncols, full, out16, AL, AH, dbg, occ) && ...);
}

// One tile; NQ segments of K rows (a.n = NQ * K, or a trusted 2-segment
// prefix of n = 4K).
template <int K, int NQ>
__device__ __forceinline__ void res_decode_tile(const DevTables& T, const ReconstructArgs& a, uint8_t* tile,
                                                const uint8_t* pools, const uint8_t* pres, const uint8_t* sh,
                                                uint8_t* out_tile, uint32_t ncols, bool full, bool out16,
                                                uint64_t* dbg, uint32_t occ) {
  uint32_t AL[16], AH[16];
  uint32_t* DL = reinterpret_cast<uint32_t*>(tile + RGeo<K>::kTileBytes);  // CQ delta tables
  uint32_t* VS = DL + kDeltaWords;                                      // RStage blocks 0..NQ-1
  rstamp(dbg, 0);
  {  // the first step's row tables (the tile is free at the start)
    const Res r0 = res_coords<K>();
    dma_row_tables(tile, pools, static_cast<uint32_t>(res_seg<NQ>(0)) * K, K, r0.w, r0.l, K / 64);
  }
  stage_delta_tables(T, DL);  // the first step's barriers order both
  stage_rh_tables<K>(T, VS, NQ);
  rstamp(dbg, 1);
  if (!res_sweep<K, NQ>(T, a, tile, pools, pres, sh, out_tile, ncols, full, out16, AL, AH, dbg, occ,
                     std::make_integer_sequence<int, NQ>{}))
    return;
  constexpr uint32_t kHD = RGeo<K>::kHD, lpc = RGeo<K>::kLPC;
  const Res r = res_coords<K>();
  if constexpr ((kExp & 8192) != 0 && !kResNoHD<K>) {  // experiment (tools/res_debug_rec.py): d in natural blocks, tower coordinates
    const uint32_t c = (64u / lpc) * r.w + r.l / lpc;
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (c < ncols)
        *reinterpret_cast<uint2*>(out_tile + static_cast<size_t>(c) * 2 * K + 8u * (r.l % lpc + lpc * j)) =
            quad_to_blk(AL[j], AH[j]);
    return;
  }
  // ---- out = FFT(K, 0)(d), first k rows (inc_reconstruct.rs:80)
  if constexpr (!kResNoHD<K>) {  // (K = 256: d is in HA already)
    hd_levels_st<K, false, kResPrioDec>(T, 0, AL, AH, VS);
    rstamp(dbg, 40);
    __syncthreads();  // the last step's HD read is done
    rh_write<kHD>(tile, fresh_v(r.hdb), AL, AH);
    __syncthreads();
    rh_read<kHA>(tile, fresh_v(r.hab), AL, AH);
  }
  rstamp(dbg, 41);
  ha_levels_st<K, false, 0, kResPrioDec>(T, 0, r, AL, AH, VS);
  rstamp(dbg, 42);
  __syncthreads();
  rh_write<kHA>(tile, fresh_v(r.hab), AL, AH);
  __syncthreads();
  rcq_read<K>(tile, fresh_v(r.cqb), AL, AH);
  {  // the merge's tables land during the FFT's CQ levels
    __syncthreads();  // every wave has read the tile
    dma_row_tables(tile, pools, 0, K, r.w, r.l, K / 64);
  }
  rstamp(dbg, 43);
  rcq_levels<false, res_gen<K>(0), kRecDeltaST<K, NQ>, kResPrioDec>(T, 0, r, AL, AH, DL);
  rstamp(dbg, 44);
  // ---- merge: received systematic rows, postmultiplied recovered ones
  // (inc_reconstruct.rs:46-50, :82-84; tower in, Cantor out)
  const uint32_t pm = lane_rows_present(pres, 0, r);
  uint2 raw[16];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's table pieces
  load_lane_rows(raw, sh, a.shard_len, 0, pm, r, ncols, full, T.zeros);
  __syncthreads();  // every wave's
  rstamp(dbg, 45);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    uint32_t l, h;
    if ((pm >> i) & 1u) {
      blk_to_quad(raw[i], l, h);
    } else {
      const FullT m = row_table(tile, 64u * r.w + 16u * r.u + i);
      qmul_set_vv(l, h, AL[i], AH[i], m);
    }
    AL[i] = l;
    AH[i] = h;
  }
  rstamp(dbg, 46);
  res_copy_out<K>(out_tile, AL, AH, r, ncols, out16);
  rstamp(dbg, 47);
}

// Every systematic row present: the output is those rows (inc_reconstruct.rs:46-50).
template <int K>
__device__ __forceinline__ void res_copy_tile(const ReconstructArgs& a, const uint8_t* sh, uint8_t* out_tile,
                                              uint32_t ncols, bool full, bool out16, const DevTables& T) {
  const Res r = res_coords<K>();
  uint2 raw[16];
  load_lane_rows(raw, sh, a.shard_len, 0, 0xffffu, r, ncols, full, T.zeros);
  uint32_t L[16], H[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) blk_to_quad(raw[i], L[i], H[i]);
  res_copy_out<K>(out_tile, L, H, r, ncols, out16);
}

// One workgroup per 64-column tile.  SERVE = 1: payloads whose record says
// copy (nq = 1); 2: decodes from 2 segments (n = 2K, or a trusted prefix of
// n = 4K); 4 / 8: the 4- / 8-segment decodes.  The host launches the
// instances over the same grid (kernels_fast.hip's scheme).
template <int K, int SERVE>
__global__ __launch_bounds__(K) __attribute__((amdgpu_waves_per_eu(4))) void k_reconstruct_res(
    DevTables T, ReconstructArgs a, uint32_t nsyms, uint32_t tiles) {
  // SERVE = 1: copies (nq = 1); 2: 2-segment decodes; 4: 4-segment decodes
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
#if NP_BOUNDS_CHECK
  bounds_arm(bounds_of(a, T, prefix_stride_c(a.n, a.k)));
#endif
  const TileRef tr = tile_of(blockIdx.x, tiles, (a.batch & 7u) == 0);
  const uint32_t pb = tr.pb, tl = tr.tl;
  const uint8_t* rec = NP_BCHK(a.prefix + static_cast<size_t>(pb) * prefix_stride_c(a.n, a.k), 2, kBkRecords);
  const uint32_t nq = uniform(rec[0]);
  if (nq != static_cast<uint32_t>(SERVE)) return;
  const uint8_t* pools = rec + prefix_pools_offset(a.n);
  const uint8_t* pres = a.present + static_cast<size_t>(pb) * a.n;
  const uint32_t col0 = tl * kRC;
  const uint32_t ncols = min(static_cast<uint32_t>(kRC), nsyms - col0);
  const uint8_t* sh = a.shards + static_cast<size_t>(pb) * a.batch_stride + 2 * static_cast<size_t>(col0);
  uint8_t* out_tile = a.out + static_cast<size_t>(pb) * a.out_stride + static_cast<size_t>(col0) * 2 * K;
  const bool full =
      ncols == kRC && rows_vec_ok(a.shards, a.batch_stride, a.shard_len);
  const bool out16 = out_vec_ok(a.out, a.out_stride);
  // experiment builds (NP_EXP bit 6): stamps past the payload's output
  // (tools/res_stamps.py allocates out_stride = output + 8 KiB per tile)
  uint64_t* dbg = (kExp & 64) ? reinterpret_cast<uint64_t*>(a.out + static_cast<size_t>(pb) * a.out_stride +
                                                             static_cast<size_t>(nsyms) * 2 * K + 8192u * tl)
                              : nullptr;
  if constexpr (SERVE == 1)
    res_copy_tile<K>(a, sh, out_tile, ncols, full, out16, T);
  else
    res_decode_tile<K, SERVE>(T, a, smem, pools, pres, sh, out_tile, ncols, full, out16, dbg, uniform(rec[1]));
}

}  // namespace

bool res_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("NP_RES");
    return !(e && e[0] == '0');
  }();
  return on;
}

// k = 512 and 1024 with n / k in {2, 4, 8} (n <= 8K: res_gen <= 5).
bool res_encode_supported(uint32_t n, uint32_t k) { return (k == 512 || k == 1024) && (n == 2 * k || n == 4 * k || n == 8 * k); }
bool res_reconstruct_supported(uint32_t n, uint32_t k) { return res_encode_supported(n, k); }

namespace {
// Dynamic LDS of a kernel over nblk transform indices: the tile, the CQ delta
// tables and the RStage blocks.
template <int K>
constexpr uint32_t res_lds(uint32_t nblk) {
  return RGeo<K>::kTileBytes + 4u * (kDeltaWords + RStage<K>::kWords * nblk);
}
static_assert(res_lds<1024>(8) <= 160u * 1024u, "k = 1024: one workgroup per CU");
static_assert(res_lds<512>(8) <= 80u * 1024u, "k = 512: two workgroups per CU");
static_assert(res_lds<256>(4) <= 40u * 1024u, "k = 256, n = 4k: four workgroups per CU");

template <int K>
hipError_t launch_reconstruct_res_k(const DevTables& T, const ReconstructArgs& a, hipStream_t s) {
  using G = RGeo<K>;
  const size_t nsyms = a.shard_len / 2;
  if (nsyms == 0 || a.batch == 0) return hipSuccess;
  if (nsyms > 0xffffffffu) return hipErrorInvalidValue;
  const uint32_t tiles = static_cast<uint32_t>((nsyms + kRC - 1) / kRC);
  const size_t blocks = a.batch * tiles;
  if (blocks > 0x7fffffffu) return hipErrorInvalidValue;
  const uint32_t nb = static_cast<uint32_t>(blocks), ns = static_cast<uint32_t>(nsyms);
  k_reconstruct_res<K, 1><<<nb, G::kThreads, 0, s>>>(T, a, ns, tiles);
  if (a.n == 2u * K || a.trusted) k_reconstruct_res<K, 2><<<nb, G::kThreads, res_lds<K>(2), s>>>(T, a, ns, tiles);
  if (a.n == 4u * K) k_reconstruct_res<K, 4><<<nb, G::kThreads, res_lds<K>(4), s>>>(T, a, ns, tiles);
  if (a.n == 8u * K) k_reconstruct_res<K, 8><<<nb, G::kThreads, res_lds<K>(8), s>>>(T, a, ns, tiles);
  return hipGetLastError();
}

template <int K>
hipError_t launch_encode_res_k(const DevTables& T, const EncodeArgs& a, hipStream_t s) {
  using G = RGeo<K>;
  const size_t nchunks = (a.payload_len + 2 * a.k - 1) / (2 * a.k);
  if (nchunks == 0 || a.batch == 0) return hipSuccess;
  if (nchunks > 0xffffffffu) return hipErrorInvalidValue;
  const uint32_t tiles = static_cast<uint32_t>((nchunks + kRC - 1) / kRC);
  const size_t blocks = a.batch * tiles;
  if (blocks > 0x7fffffffu) return hipErrorInvalidValue;
  k_encode_res<K><<<static_cast<uint32_t>(blocks), G::kThreads, res_lds<K>(a.n / K), s>>>(T, a, static_cast<uint32_t>(nchunks), tiles);
  return hipGetLastError();
}

template <int K>
hipError_t configure_res_k() {
  hipError_t e = hipSuccess;
  const void* enc = nullptr;  // (no K = 256 encode: the fast one serves it)
  if constexpr (K != 256) enc = reinterpret_cast<const void*>(&k_encode_res<K>);
  for (const void* f : {enc, reinterpret_cast<const void*>(&k_reconstruct_res<K, 2>),
                        reinterpret_cast<const void*>(&k_reconstruct_res<K, 4>),
                        reinterpret_cast<const void*>(&k_reconstruct_res<K, 8>)}) {
    if (!f) continue;
    const hipError_t r = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(res_lds<K>(8)));
    if (r != hipSuccess && e == hipSuccess) e = r;
  }
  return e;
}
}  // namespace

hipError_t launch_reconstruct_res(const DevTables& T, const ReconstructArgs& a, hipStream_t s) {
  if (a.k == 256 && (a.n == 512 || a.n == 1024 || a.n == 2048)) return launch_reconstruct_res_k<256>(T, a, s);
  if (!res_reconstruct_supported(a.n, a.k)) return hipErrorInvalidValue;
  return a.k == 512 ? launch_reconstruct_res_k<512>(T, a, s) : launch_reconstruct_res_k<1024>(T, a, s);
}

// The k = 256 decode in the resident geometry instead of k_reconstruct_fast
// (the A/B of four 64-column workgroups per CU against one
// 256-column workgroup).  Experiment knob, read per call.
bool res256_reconstruct(uint32_t n, uint32_t k) {
  if (k != 256 || (n != 512 && n != 1024 && n != 2048)) return false;
  const char* e = std::getenv("NP_REC_RES256");
  return e && e[0] == '1';
}

hipError_t launch_encode_res(const DevTables& T, const EncodeArgs& a, hipStream_t s) {
  if (!res_encode_supported(a.n, a.k)) return hipErrorInvalidValue;
  return a.k == 512 ? launch_encode_res_k<512>(T, a, s) : launch_encode_res_k<1024>(T, a, s);
}

hipError_t configure_res_kernels() {
  const hipError_t e = configure_res_k<1024>();
  const hipError_t f = configure_res_k<512>();
  const hipError_t g = configure_res_k<256>();
  return e != hipSuccess ? e : f != hipSuccess ? f : g;
}

hipError_t bounds_take_res(uint32_t out[8]) { return bounds_take_tu(out); }

}  // namespace np
