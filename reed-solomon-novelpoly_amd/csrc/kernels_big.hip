// Specialised gfx950 kernels for k = 512, 1024 and 2048 (BASELINE config 4:
// n = 4096, k = 1024; 1,366-2,730 validators: k = 512; 6,144-8,192: k =
// 2048).
//
// A 256-column tile of a size-KB transform needs KB/2 KiB, more than the LDS
// holds, so a workgroup (1024 threads, the K = 256 register layouts of
// fast_common.hpp) runs the transform as SUBS = KB / 256 size-256 sub-segments
// plus the top levels (8, 9 for KB >= 1024, 10 for KB = 2048) that mix them:
//
//   phase 1  per sub-segment: LDS tile -> column-quad levels 0..3 -> high-layout
//            levels 4..7 -> registers -> per-workgroup scratch in HBM / L2;
//   phase 2  per position quad, across the sub-segments: the top levels (and for
//            reconstruct the segment combination, formal derivative and the
//            forward transform's top levels) -> scratch;
//   phase 3  per sub-segment: scratch -> high-layout levels 7..4 -> LDS ->
//            column-quad levels 3..0 -> shard rows / output.
//
// Scratch traffic stays in the workgroup (each thread reads back what it
// wrote), so no inter-workgroup synchronisation is needed.  The top-level
// skews of a size-KB transform at index I are Cantor((I >> 9) + 2t) for
// level 9 and Cantor((I >> 8) + 2t) for level 8 (fast_common.hpp, skew_c).
//
// Reference: inc_afft.rs:139-214 / :267-332, inc_encode.rs:15-48,
// inc_reconstruct.rs:1-113, mod.rs:117-239.
#include <map>
#include <mutex>

#include "fast_common.hpp"

namespace np {
namespace {

// Progress-based issue priority in the sub-segment transforms' passes, encode
// and decode (fast_common.hpp progress_prio).  Measured at 7000 validators
// (k = 2048, profiles/r04_ab.txt probe 25): encode 1.818 / 1.799 -> 1.715 /
// 1.745 ms (-4 %), reconstruct 2.807 / 2.815 -> 2.796 / 2.805 ms.
constexpr int kBigPrioEnc = 1, kBigPrioDec = 1;

constexpr int kS = 256;                   // sub-segment (register-layout) size
constexpr int kTB = Geo<kS>::kThreads;    // 1024 threads
constexpr size_t kSegScr = 16u * kTB * 8; // one sub-segment of a tile in thread order: 128 KiB

// Scratch of one sub-segment slot: quad j of thread t at ((j * kTB) + t) * 8 bytes.
// NT: nontemporal (streaming) accesses.  The reconstruct writes every scratch
// word once and reads it back once, far beyond what L2 holds in between (the
// resident workgroups' scratch is 640 MiB): streaming is -7 % there.  The
// encode re-reads its coefficients M once per shift and keeps plain accesses
// for them (streaming them cost it +5 %).
__device__ __forceinline__ uint64_t* scr_at(uint8_t* seg, uint32_t j, uint32_t tid) {
  return reinterpret_cast<uint64_t*>(seg + static_cast<uint32_t>((j * kTB + tid) * 8));
}
__device__ __forceinline__ const uint64_t* scr_at(const uint8_t* seg, uint32_t j, uint32_t tid) {
  return reinterpret_cast<const uint64_t*>(seg + static_cast<uint32_t>((j * kTB + tid) * 8));
}

template <bool NT>
__device__ __forceinline__ void scr_q_store(uint8_t* seg, uint32_t j, uint32_t tid, const uint2& x) {
  const uint64_t v = static_cast<uint64_t>(x.x) | (static_cast<uint64_t>(x.y) << 32);
  if constexpr (NT)
    __builtin_nontemporal_store(v, scr_at(seg, j, tid));
  else
    *scr_at(seg, j, tid) = v;
}
template <bool NT>
__device__ __forceinline__ uint2 scr_q(const uint8_t* seg, uint32_t j, uint32_t tid) {
  uint64_t v;
  if constexpr (NT)
    v = __builtin_nontemporal_load(scr_at(seg, j, tid));
  else
    v = *scr_at(seg, j, tid);
  return make_uint2(static_cast<uint32_t>(v), static_cast<uint32_t>(v >> 32));
}

template <bool NT>
__device__ __forceinline__ void scr_store(uint8_t* seg, uint32_t tid, const uint32_t (&L)[16],
                                          const uint32_t (&H)[16]) {
#pragma unroll
  for (int j = 0; j < 16; ++j) scr_q_store<NT>(seg, j, tid, make_uint2(L[j], H[j]));
}

template <bool NT>
__device__ __forceinline__ void scr_load(const uint8_t* seg, uint32_t tid, uint32_t (&L)[16], uint32_t (&H)[16]) {
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint2 v = scr_q<NT>(seg, j, tid);
    L[j] = v.x;
    H[j] = v.y;
  }
}

// Multiplier of a skew or segment coefficient c < 256 (Cantor index): every
// one the big kernels use outside the sub-segment transforms lies in GF(2^8),
// so it is a subfield multiply in tower coordinates (tower_pools, qmul_sub).
__device__ __forceinline__ Mult tmult(const DevTables& T, uint32_t c) {
  uint32_t p[20];
  pool_of<true>(T, c, p);
  return make_mult(p);
}

// x ^= c * y for one (L, H) quad pair, c from tmult.
__device__ __forceinline__ void qm(uint2& x, const uint2& y, const Mult& m) { qmul_sub(x.x, x.y, y.x, y.y, m); }
__device__ __forceinline__ void qx(uint2& x, const uint2& y) {
  x.x ^= y.x;
  x.y ^= y.y;
}

// The multipliers of the top levels of a size-(256 SUBS) transform at index
// 256 SUBS q: level 8 + L (L < log2 SUBS) has SUBS / 2^(L+1) groups, group t
// with skew Cantor(q SUBS / 2^L + 2t), at m[top_off(L) + t]; all in GF(2^8).
// Loaded once per pass over the 16 quads.
__host__ __device__ constexpr int top_off(int subs, int L) { return subs - (subs >> L); }
__host__ __device__ constexpr uint32_t top_skew(int subs, int L, uint32_t q, int t) {
  return q * static_cast<uint32_t>(subs >> L) + 2u * t;
}
template <int SUBS>
struct TopMults {
  Mult m[SUBS - 1];
};
template <int SUBS>
__device__ __forceinline__ TopMults<SUBS> top_mults(const DevTables& T, uint32_t q) {
  TopMults<SUBS> m;
#pragma unroll
  for (int L = 0; (1 << L) < SUBS; ++L)
#pragma unroll
    for (int t = 0; t < (SUBS >> (L + 1)); ++t)
      if (top_skew(SUBS, L, q, t)) m.m[top_off(SUBS, L) + t] = tmult(T, top_skew(SUBS, L, q, t));
  return m;
}

// Top inverse levels (8, 9, ...) on one position quad of each sub-segment:
// inverse butterfly hi ^= lo; lo ^= c hi.  q is a compile-time constant at
// the q = 0 calls, so their zero skews fold.
template <int SUBS>
__device__ __forceinline__ void top_inverse(uint2 (&y)[SUBS], uint32_t q, const TopMults<SUBS>& m) {
#pragma unroll
  for (int L = 0; (1 << L) < SUBS; ++L) {
    const int d = 1 << L;
#pragma unroll
    for (int t = 0; t < (SUBS >> (L + 1)); ++t)
#pragma unroll
      for (int u = 0; u < d; ++u) {
        const int x = 2 * d * t + u;
        qx(y[x + d], y[x]);
        if (top_skew(SUBS, L, q, t)) qm(y[x], y[x + d], m.m[top_off(SUBS, L) + t]);
      }
  }
}

// The same with each group's multiplier fetched where it is used (SUBS = 8:
// holding all seven across the pass would cost 28 VGPRs); T comes from
// fresh_tables at the call, so the fetches are not hoisted out of its loop.
template <int SUBS>
__device__ __forceinline__ void top_inverse_fetch(const DevTables& T, uint2 (&y)[SUBS], uint32_t q) {
#pragma unroll
  for (int L = 0; (1 << L) < SUBS; ++L) {
    const int d = 1 << L;
#pragma unroll
    for (int t = 0; t < (SUBS >> (L + 1)); ++t) {
      const uint32_t c = top_skew(SUBS, L, q, t);
      Mult m;
      if (c) m = tmult(T, c);
#pragma unroll
      for (int u = 0; u < d; ++u) {
        const int x = 2 * d * t + u;
        qx(y[x + d], y[x]);
        if (c) qm(y[x], y[x + d], m);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
}

// Top forward levels at index 256 SUBS c (highest first): lo ^= c hi; hi ^= lo.
template <int SUBS>
__device__ __forceinline__ void top_forward(uint2 (&w)[SUBS], uint32_t c, const TopMults<SUBS>& m) {
#pragma unroll
  for (int L = ilog2(SUBS) - 1; L >= 0; --L) {
    const int d = 1 << L;
#pragma unroll
    for (int t = 0; t < (SUBS >> (L + 1)); ++t)
#pragma unroll
      for (int u = 0; u < d; ++u) {
        const int x = 2 * d * t + u;
        if (top_skew(SUBS, L, c, t)) qm(w[x], w[x + d], m.m[top_off(SUBS, L) + t]);
        qx(w[x + d], w[x]);
      }
  }
}

// ------------------------------------------------------------------ encode ----
// The shift's top-level outputs W are written once and read once: streaming
// (-6 % on the encode); the coefficients M keep the default policy.
// Sub-segment transforms of the shifts run in tower coordinates while
// gen_of(index) <= kEncBigMaxGen (index < 4096: n <= 4096, config 4); their
// levels below gen_of(index) with the full map.  Farther shifts of larger codes
// run in Cantor coordinates.
constexpr int kEncBigMaxGen = 4;
// k = 2048 (n <= 8192): every shift in tower coordinates (index < 8192).
template <int KB>
constexpr int kEncBigMaxGenK = KB == 2048 ? 5 : kEncBigMaxGen;
// Highest gen_of of a sub-segment transform at index 256 s, s < SUBS (at
// least 2: the instances the k = 512 / 1024 kernels were tuned with).
template <int KB>
constexpr int kSubMaxGen = gen_of(KB - 256) > 2 ? static_cast<int>(gen_of(KB - 256)) : 2;


template <int KB>
constexpr size_t enc_scratch() {
  return (2u * (KB / kS) - 1u) * kSegScr;  // M (SUBS sub-segments) + W_1.. (SUBS - 1)
}

// The encode's sub-segment transforms exchange layouts through quad items
// (the high layout of k_encode_multi; the top levels and the scratch are
// per thread and position, so they follow it unchanged).  The decode keeps
// the natural format: D_256 needs position bits 0-3 in one wave.

template <int KB>
__global__ __launch_bounds__(kTB) __attribute__((amdgpu_waves_per_eu(4))) void k_encode_big(
    DevTables T, EncodeArgs a, uint32_t nchunks, uint32_t tiles, uint32_t tile0, uint8_t* scratch) {
  using G = Geo<kS>;
#if NP_BOUNDS_CHECK
  bounds_arm(bounds_of_enc(a));
#endif
  constexpr int SUBS = KB / kS;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* tile = smem;
  uint32_t* VP = reinterpret_cast<uint32_t*>(smem + G::kTileBytes);
  const uint32_t blk = tile0 + blockIdx.x;
  const TileRef tr = tile_of(blk, tiles, (a.batch & 7u) == 0);
  const uint32_t pb = tr.pb, tl = tr.tl;
  const uint32_t ch0 = tl * kTile;
  const uint32_t ncols = min(static_cast<uint32_t>(kTile), nchunks - ch0);
  const uint8_t* pay = a.payloads + static_cast<size_t>(pb) * a.payload_stride;
  uint8_t* out = a.shards + static_cast<size_t>(pb) * a.batch_stride + 2 * static_cast<size_t>(ch0);
  uint8_t* scrM = scratch + static_cast<size_t>(blockIdx.x) * enc_scratch<KB>();
  uint8_t* scrW = scrM + (SUBS - 1) * kSegScr;  // W_s at scrW + s slots, s >= 1
  const uint32_t tid = threadIdx.x, lane = tid & 63u, g = uniform(tid >> 6);
  const bool full =
      ncols == kTile && rows_vec_ok(a.shards, a.batch_stride, a.shard_len);
  const uint32_t cqb = col_base<kS>(4 * lane) ^ (32u * g);
  const bool fast_in = out_vec_ok(pay, 0) &&
                       static_cast<size_t>(ch0 + kTile) * 2 * KB <= a.payload_len;

  // ---- phase 1: x_s = IFFT(256, 256 s)(sub-segment s of every chunk)
#pragma unroll 1
  for (uint32_t s = 0; s < SUBS; ++s) {
    // per iteration, opaque: lane-derived addresses are not hoisted and spilled
    const uint32_t tid = fresh_v(threadIdx.x), lane = tid & 63u;
    const uint32_t index = 256u * s;
    __syncthreads();  // previous sub-segment is done with the tile and the tables
    stage_vpools<kS, kTB>(T, index, VP, true);
    {
      const uint32_t c0 = tid / G::Q, m0 = tid % G::Q;
      const uint32_t base = col_base<kS>(c0) ^ (8u * m0);
      const size_t gbase = static_cast<size_t>(ch0 + c0) * 2 * KB + 2u * index + 8u * m0;
      if (fast_in) {
        uint2 v[16];
#pragma unroll
        for (int i = 0; i < 16; ++i)
          v[i] = load_once(pay + gbase + static_cast<size_t>(i) * 16 * 2 * KB);
#pragma unroll
        for (int i = 0; i < 16; ++i) *reinterpret_cast<uint2*>(tile + (base ^ col_base_c<kS>(16u * i))) = v[i];
      } else {
#pragma unroll 1
        for (uint32_t i = 0; i < 16; ++i) {
          const size_t g0 = gbase + static_cast<size_t>(i) * 16 * 2 * KB;
          uint32_t w[2] = {0, 0};
#pragma unroll
          for (int e = 0; e < 8; ++e)
            if (g0 + e < a.payload_len) w[e >> 2] |= static_cast<uint32_t>(pay[g0 + e]) << (8 * (e & 3));
          *reinterpret_cast<uint2*>(tile + (base ^ col_base_c<kS>(16u * i))) = make_uint2(w[0], w[1]);
        }
      }
    }
    __syncthreads();
    {
      uint32_t CL[16], CH[16];
      const uint32_t cq = fresh_v(cqb);
      cq_read<kS>(tile, cq, CL, CH);
      store_rows(out, a.shard_len, index + 16 * g, a.wanted_n, CL, CH, lane, ncols, full,
                 rows_nt(a.shards, a.batch_stride, a.shard_len));  // systematic rows
      tower_convert(T, CL, CH);  // the transforms run in tower coordinates
      with_gen<0, kSubMaxGen<KB>, false>(index, [&](auto gc) __attribute__((always_inline)) {
        constexpr int GEN = decltype(gc)::value;  // 0 only at index 0
        cq_levels<kS, true, GEN == 0, GEN, false, kBigPrioEnc>(T, VP, index, g, CL, CH);
      });
      // quad items (fast_common.hpp cq_write_q): no byte transposes
      __syncthreads();  // they overlay payload blocks that other waves read
      cq_write_q(tile, g, lane, CL, CH);
    }
    __syncthreads();
    uint32_t XL[16], XH[16];
    hi_read_q(tile, g, lane, XL, XH);
    with_gen<0, kSubMaxGen<KB>, false>(index, [&](auto gc) __attribute__((always_inline)) {
      constexpr int GEN = decltype(gc)::value;
      hi_levels<kS, true, GEN == 0, 0, GEN, kBigPrioEnc>(T, VP, index, XL, XH);
    });
    if (s + 1 < static_cast<uint32_t>(SUBS)) {
      scr_store<false>(scrM + s * kSegScr, tid, XL, XH);
    } else {  // the last sub-segment waits in the LDS tile (thread order), not in the scratch
      __syncthreads();  // every wave has read the tile
      scr_store<false>(tile, tid, XL, XH);
    }
  }
  // ---- phase 2: top inverse levels at index 0 -> coefficients M (in place;
  // sub-segment 0 is unchanged: every level-8/9 butterfly at index 0 keeps lo).
  // Each thread reads back only what it wrote: no barrier.
  {
    const TopMults<SUBS> tm = top_mults<SUBS>(T, 0u);
#pragma unroll 1
    for (uint32_t j = 0; j < 16; ++j) {
      const uint32_t tid = fresh_v(threadIdx.x);
      uint2 x[SUBS];
#pragma unroll
      for (int r = 0; r + 1 < SUBS; ++r) x[r] = scr_q<false>(scrM + r * kSegScr, j, tid);
      x[SUBS - 1] = scr_q<false>(tile, j, tid);
      top_inverse<SUBS>(x, 0u, tm);
#pragma unroll
      for (int r = 1; r < SUBS; ++r) scr_q_store<false>(scrM + r * kSegScr, j, tid, x[r]);
    }
  }

  // ---- phase 3: every shift c = 1.. : top forward levels, then SUBS x FFT(256).
  // W_0 waits in the LDS tile (thread order) for the first sub-segment's
  // transform, W_1.. in the scratch: the kernel is bound by its scratch traffic.
  const uint32_t nshift = a.n / KB;
#pragma unroll 1
  for (uint32_t c = 1; c < nshift; ++c) {
    if (c * KB >= a.wanted_n) break;
    const TopMults<SUBS> tm = top_mults<SUBS>(T, c);
    __syncthreads();  // the previous transform is done with the tile
#pragma unroll 1
    for (uint32_t j = 0; j < 16; ++j) {
      const uint32_t tid = fresh_v(threadIdx.x);
      uint2 w[SUBS];
#pragma unroll
      for (int r = 0; r < SUBS; ++r) w[r] = scr_q<false>(scrM + r * kSegScr, j, tid);
      top_forward<SUBS>(w, c, tm);
      scr_q_store<false>(tile, j, tid, w[0]);
#pragma unroll
      for (int r = 1; r < SUBS; ++r) scr_q_store<true>(scrW + r * kSegScr, j, tid, w[r]);
    }
#pragma unroll 1
    for (uint32_t s = 0; s < SUBS; ++s) {
      const uint32_t index = c * KB + 256u * s;
      if (index >= a.wanted_n) break;
      const uint32_t tid = fresh_v(threadIdx.x), lane = tid & 63u;
      uint32_t XL[16], XH[16];
      if (s == 0) scr_load<false>(tile, tid, XL, XH);  // this thread's own W_0
      __syncthreads();  // the tile (W_0 read) and the tables are free
      stage_vpools<kS, kTB>(T, index, VP, gen_of(index) <= kEncBigMaxGenK<KB>);
      __syncthreads();
      if (s != 0) scr_load<true>(scrW + s * kSegScr, tid, XL, XH);
      with_gen<1, kEncBigMaxGenK<KB>, true>(index, [&](auto gc) __attribute__((always_inline)) {
        constexpr int GEN = decltype(gc)::value;
        if constexpr (GEN < 0) tower_convert(T, XL, XH);  // a far shift: Cantor coordinates
        hi_levels<kS, false, false, 0, GEN, kBigPrioEnc>(T, VP, index, XL, XH);
      });
      hi_write_q(tile, g, lane, XL, XH);
      __syncthreads();
      cq_read_q(tile, g, lane, XL, XH);
      with_gen<1, kEncBigMaxGenK<KB>, true>(index, [&](auto gc) __attribute__((always_inline)) {
        constexpr int GEN = decltype(gc)::value;
        cq_levels<kS, false, false, GEN, false, kBigPrioEnc>(T, VP, index, g, XL, XH);
        if constexpr (GEN >= 0) tower_convert(T, XL, XH);  // back to Cantor coordinates for the rows
      });
      store_rows(out, a.shard_len, index + 16 * g, a.wanted_n, XL, XH, lane, ncols, full,
                 rows_nt(a.shards, a.batch_stride, a.shard_len));
    }
  }
}

// ------------------------------------------------------------- reconstruct ----
// n = NQ * KB.  As in k_reconstruct_fast (kernels_fast.hip), the first KB
// outputs are out = FFT(KB, 0)(d) with
//   d = D_KB(x0) ^ sum_q kappa_q x_q,  x_q = IFFT(KB, KB q)(premultiplied segment q)
// (kappa: NQ = 2 (1, 1); NQ = 4 (0, 1, 3, 2); NQ = 8 rec8_kappa; Cantor
// coordinates, all in GF(16)).  The sum is formed per Cantor bit b of kappa,
// S_b = XOR of the x_q with bit b set, d ^= S_0 ^ sum_b Cantor(2^b) S_b: one
// multiply per bit rather than per segment.  Each x_q is SUBS sub-segment
// transforms y_qs = IFFT(256, KB q + 256 s) plus the top levels, and
// D_KB = (I (x) D_256) + (high single-bit terms l = 256, 512 < KB); the D_256
// part commutes with the top levels, so it is applied to y_0s in phase 1.
template <int NQ>
__host__ __device__ constexpr uint32_t big_kappa(int q) {
  if constexpr (NQ == 2) {
    return 1u;
  } else if constexpr (NQ == 4) {
    constexpr uint32_t k[4] = {0, 1, 3, 2};
    return k[q];
  } else {
    constexpr uint32_t k[8] = {1, 1, 3, 2, 12, 15, 10, 8};  // kernels_fast.hip rec8_kappa
    return k[q];
  }
}
template <int... Q, typename F>
__device__ __forceinline__ void for_each_q(std::integer_sequence<int, Q...>, F&& f) {
  (f(Int<Q>{}), ...);
}
template <int NQ>
__host__ __device__ constexpr bool kappa_bit_used(int b) {
  for (int q = 0; q < NQ; ++q)
    if ((big_kappa<NQ>(q) >> b) & 1u) return true;
  return false;
}

// Highest gen_of of a phase-1 sub-segment transform (index 256 (SUBS NQ - 1)).
template <int KB, int NQ>
constexpr int kRecBigMaxGen = static_cast<int>(gen_of(256u * (KB / kS * NQ - 1)));

// Per-payload record of the big reconstruct (k_big_records): a mode word, at
// byte 8 the occupancy of the 256-row sub-segments (bit i: rows [256 i,
// 256 i + 256) hold a present row; n <= 16384), then the row multipliers
// E[0..n) (u16: EXP[loc] of present rows, EXP[-loc] of erased ones) and the
// present flags PR[0..n) (bytes), as the kernel's LDS holds them.
constexpr uint32_t kBigSkip = 0;  // fewer than k present rows (NeedMoreShards)
constexpr uint32_t kBigCopy = 1;  // all k systematic rows present: a copy
constexpr uint32_t kBigDecode = 2;
constexpr size_t kBigRecHeader = 16;
__host__ __device__ constexpr size_t big_rec_stride(uint32_t n) { return kBigRecHeader + 3u * n; }

// The decode keeps E and PR in LDS next to the tile up to n = 8192 (which
// fills the 160 KiB exactly); beyond, it reads them from the record through
// the scalar cache (wave-uniform rows).
__host__ __device__ constexpr bool big_rows_global(uint32_t n) { return n > 8192u; }

// Row multiplier and present flag of row r: from LDS, or (G) from the record
// in global memory with dword scalar loads.
template <bool G>
struct RowView {
  const uint16_t* E;
  const uint8_t* PR;
  __device__ __forceinline__ uint32_t e(uint32_t r) const {
    if constexpr (G) {
      const uint32_t w = ((cpool_t)(E))[r >> 1];
      return (r & 1u) ? w >> 16 : w & 0xffffu;
    } else {
      return uniform(E[r]);
    }
  }
  __device__ __forceinline__ bool pr(uint32_t r) const {
    if constexpr (G) {
      return ((((cpool_t)(PR))[r >> 2] >> (8u * (r & 3u))) & 0xffu) != 0;
    } else {
      return uniform(PR[r]) != 0;
    }
  }
};

// Shard-row pieces of rows row0..row0+NR-1 for this lane (fast_common.hpp
// load_rows over a RowView).  Absent rows read the zero page.
template <int NR, bool G>
__device__ __forceinline__ void load_rows_v(uint2 (&raw)[NR], const uint8_t* sh, size_t shard_len, const RowView<G>& rv,
                                            uint32_t row0, const uint8_t* zeros, uint32_t lane, uint32_t ncols,
                                            bool full) {
  const uint8_t* src[NR];
#pragma unroll
  for (int p = 0; p < NR; ++p) src[p] = rv.pr(row0 + p) ? sh + static_cast<size_t>(row0 + p) * shard_len : zeros;
  if (full) {
#pragma unroll
    for (int p = 0; p < NR; ++p) raw[p] = *reinterpret_cast<const uint2*>(src[p] + 8u * lane);
  } else {
#pragma unroll
    for (int p = 0; p < NR; ++p) raw[p] = load4(src[p], lane, ncols, false);
  }
}

// Output column c, symbols 256 s .. 256 s + 255 (bytes [2 KB c + 512 s, +512))
// from the tile's natural blocks.
template <int KB>
__device__ __forceinline__ void tile_copy_out(const ReconstructArgs& a, const uint8_t* tile, uint32_t pb,
                                              uint32_t col0, uint32_t ncols, uint32_t s) {
  using G = Geo<kS>;
  uint8_t* outp = a.out + static_cast<size_t>(pb) * a.out_stride + static_cast<size_t>(col0) * 2 * KB + 512u * s;
  const bool al_o = true;  // 8-byte stores at any address (rows_vec_ok)
  // opaque thread id, one output pointer stepped per column: otherwise the 16
  // per-lane 64-bit column addresses are hoisted out of the callers' loops and
  // spilled, and every reload waits (vmcnt(0)) for the stores before it
  const uint32_t tid = fresh_v(threadIdx.x), c0 = tid / G::Q, m0 = tid % G::Q;
  const uint32_t base = col_base<kS>(c0) ^ (8u * m0);
  uint8_t* o = outp + static_cast<size_t>(c0) * 2 * KB + 8u * m0;
#pragma unroll
  for (int i = 0; i < 16; ++i, o += 16u * 2 * KB) {
    const uint32_t c = c0 + 16u * i;
    if (c >= ncols) break;
    const uint2 v = *reinterpret_cast<const uint2*>(tile + (base ^ col_base_c<kS>(16u * i)));
    if (al_o) {
      store_once(o, v);
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) o[e] = static_cast<uint8_t>((e < 4 ? v.x : v.y) >> (8 * (e & 3)));
    }
  }
}

// Every systematic row present: the reference returns them unchanged
// (inc_reconstruct.rs:46-50), so the output is their column gather.
template <int KB>
__device__ __forceinline__ void big_copy_systematic(const ReconstructArgs& a, const uint8_t* sh, uint8_t* tile,
                                                    uint32_t pb, uint32_t col0, uint32_t ncols, bool full) {
  const uint32_t tid = threadIdx.x, lane = tid & 63u, g = uniform(tid >> 6);
  const uint32_t cqb = col_base<kS>(4 * lane) ^ (32u * g);
#pragma unroll 1
  for (uint32_t s = 0; s < static_cast<uint32_t>(KB / kS); ++s) {
    uint32_t XL[16], XH[16];
#pragma unroll
    for (int p = 0; p < 16; ++p) {
      const uint32_t row = 256u * s + 16u * g + p;
      blk_to_quad(load4(sh + static_cast<size_t>(row) * a.shard_len, lane, ncols, full), XL[p], XH[p]);
    }
    __syncthreads();  // the previous sub-segment's copy-out is done with the tile
    cq_write<kS>(tile, cqb, XL, XH);
    __syncthreads();
    tile_copy_out<KB>(a, tile, pb, col0, ncols, s);
  }
}

// Quad positions whose scratch loads phase 2 issues together (NQ <= 4);
// 2 measured +3 % at config 4.
template <int NQ>
constexpr int kRecJB = 1;

template <int KB, int NQ>
__global__ __launch_bounds__(kTB) __attribute__((amdgpu_waves_per_eu(4))) void k_reconstruct_big(
    DevTables T, ReconstructArgs a, uint32_t nsyms, uint32_t tiles, uint32_t tile0, uint8_t* scratch) {
  using G = Geo<kS>;
#if NP_BOUNDS_CHECK
  bounds_arm(bounds_of(a, T, 0));
#endif
  constexpr int SUBS = KB / kS;
  constexpr int N = NQ * KB;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  constexpr bool RG = big_rows_global(N);
  uint8_t* tile = smem;
  uint32_t* VP = reinterpret_cast<uint32_t*>(smem + G::kTileBytes);
  uint16_t* E = reinterpret_cast<uint16_t*>(smem + G::kTileBytes + 4 * G::kVPWords);
  uint8_t* PR = smem + G::kTileBytes + 4 * G::kVPWords + 2 * N;
  const uint32_t blk = tile0 + blockIdx.x;
  const TileRef tr = tile_of(blk, tiles, (a.batch & 7u) == 0);
  const uint32_t pb = tr.pb, tl = tr.tl;
  // the payload's record (k_big_records): mode, row multipliers E, present flags
  const uint8_t* rec = a.prefix + static_cast<size_t>(pb) * big_rec_stride(N);
  const uint32_t mode = uniform(*reinterpret_cast<const uint32_t*>(rec));
  if (mode == kBigSkip) return;  // fewer than k present rows: status NeedMoreShards
  // sub-segments with a present row; the others are zero (absent rows are)
  const uint64_t occ = (static_cast<uint64_t>(uniform(reinterpret_cast<const uint32_t*>(rec)[3])) << 32) |
                       uniform(reinterpret_cast<const uint32_t*>(rec)[2]);
  auto seg_live = [&](int q) __attribute__((always_inline)) {
    return ((occ >> (SUBS * q)) & ((1ull << SUBS) - 1u)) != 0;
  };
  const uint32_t col0 = tl * kTile;
  const uint32_t ncols = min(static_cast<uint32_t>(kTile), nsyms - col0);
  const uint8_t* sh = a.shards + static_cast<size_t>(pb) * a.batch_stride + 2 * static_cast<size_t>(col0);
  // y_qs (SUBS NQ - 1 slots), then D_256(y_0s) (SUBS slots, reused for e_1..)
  // (the last y slot is unused: that sub-segment waits in the LDS tile)
  uint8_t* scrY = scratch + static_cast<size_t>(blockIdx.x) * (SUBS * NQ + SUBS - 1) * kSegScr;
  uint8_t* scrD = scrY + (SUBS * NQ - 1) * kSegScr;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, g = uniform(tid >> 6);
  const bool full =
      ncols == kTile && rows_vec_ok(a.shards, a.batch_stride, a.shard_len);
  const uint32_t cqb = col_base<kS>(4 * lane) ^ (32u * g);
  const uint32_t hb = col_base<kS>(tid / G::R) ^ (8u * (tid % G::R));

  if (mode == kBigCopy) {  // all k systematic rows present: the output is those rows
    big_copy_systematic<KB>(a, sh, tile, pb, col0, ncols, full);
    return;
  }
  if constexpr (!RG) {  // E (2N bytes) and PR (N bytes) are contiguous in the record and in LDS
    const uint4* src = reinterpret_cast<const uint4*>(rec + kBigRecHeader);
    uint4* dst = reinterpret_cast<uint4*>(E);
    for (uint32_t v = tid; v < 3u * N / 16u; v += kTB) dst[v] = src[v];
  }
  const RowView<RG> rv{RG ? reinterpret_cast<const uint16_t*>(rec + kBigRecHeader) : E,
                       RG ? rec + kBigRecHeader + 2u * N : PR};

  // ---- phase 1: y_qs for every segment q and sub-segment s
  __syncthreads();  // E, PR ready
#pragma unroll 1
  for (uint32_t qs = 0; qs < static_cast<uint32_t>(SUBS * NQ); ++qs) {
    const uint32_t index = 256u * qs;  // = KB q + 256 s
    const uint32_t gg = fresh(g);
    const uint32_t tid = fresh_v(threadIdx.x), lane = tid & 63u;  // opaque: not hoisted and spilled
    if (!((occ >> qs) & 1u)) {  // no present row: y_qs = 0 without loads, tables or transform
      uint32_t ZL[16] = {0}, ZH[16] = {0};
      if (qs + 1 < static_cast<uint32_t>(SUBS * NQ)) {
        scr_store<true>(scrY + qs * kSegScr, tid, ZL, ZH);
      } else {
        __syncthreads();  // every wave has read the tile
        scr_store<false>(tile, tid, ZL, ZH);
      }
      if (qs < static_cast<uint32_t>(SUBS)) scr_store<true>(scrD + qs * kSegScr, tid, ZL, ZH);
      continue;
    }
    // the sub-segment's present rows load while the tables are staged
    uint2 rows[2][8];
#pragma unroll
    for (int half = 0; half < 2; ++half)
      load_rows_v<8>(rows[half], sh, a.shard_len, rv, index + 16 * gg + 8 * half, T.zeros, lane, ncols, full);
    __syncthreads();  // tile / tables free
    stage_vpools<kS, kTB>(T, index, VP, true);
    __syncthreads();
    uint32_t XL[16], XH[16];
    {
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const uint2 (&raw)[8] = rows[half];
        const uint32_t r0 = index + 16 * gg + 8 * half;
        // premultiply (Cantor in, tower out: in_pools) of the present rows
        pipelined_rec<8>(
            [&](auto pc) __attribute__((always_inline)) {
              return (cpool_t)(T.in_pools) + rv.e(r0 + decltype(pc)::value) * kPoolWords;
            },
            [&](auto pc) __attribute__((always_inline)) { return rv.pr(r0 + decltype(pc)::value); },
            [&](auto pc, const Mult& pool) __attribute__((always_inline)) {
              constexpr int p = decltype(pc)::value;
              const int x = 8 * half + p;
              XL[x] = 0;
              XH[x] = 0;
              if (rv.pr(index + 16 * gg + x)) {
                uint32_t l, h;
                blk_to_quad(raw[p], l, h);
                qmul_set(XL[x], XH[x], l, h, pool);
              }
            });
      }
      with_gen<0, kRecBigMaxGen<KB, NQ>, false>(index, [&](auto gc) __attribute__((always_inline)) {
        constexpr int GEN = decltype(gc)::value;  // 0 only at index 0
        cq_levels<kS, true, GEN == 0, GEN, false, kBigPrioDec>(T, VP, index, gg, XL, XH);
      });
      cq_write<kS>(tile, fresh_v(cqb), XL, XH);
    }
    __syncthreads();
    hi_read<kS>(tile, fresh_v(hb), XL, XH);
    with_gen<0, kRecBigMaxGen<KB, NQ>, false>(index, [&](auto gc) __attribute__((always_inline)) {
      constexpr int GEN = decltype(gc)::value;
      hi_levels<kS, true, GEN == 0, 0, GEN, kBigPrioDec>(T, VP, index, XL, XH);
    });
    if (qs + 1 < static_cast<uint32_t>(SUBS * NQ)) {
      scr_store<true>(scrY + qs * kSegScr, tid, XL, XH);
    } else {  // the last sub-segment waits in the LDS tile (thread order), not in the scratch
      __syncthreads();  // every wave has read the tile
      scr_store<false>(tile, tid, XL, XH);
    }
    if (qs < static_cast<uint32_t>(SUBS)) {  // segment 0: also D_256(y_0s)
      uint32_t DL[16] = {0}, DH[16] = {0};
      add_derivative<kS>(DL, XL, tid % G::R);
      add_derivative<kS>(DH, XH, tid % G::R);
      scr_store<true>(scrD + qs * kSegScr, tid, DL, DH);
    }
  }

  // ---- phase 2: top levels of every x_q, the combination, the derivative's
  // high terms and the forward transform's top levels at index 0 -> e_s (over
  // D's slots)
  // One quad position j: x0, z = D_256(y_0.) and the other segments' quads in,
  // e_s out.
  const TopMults<SUBS> tm0 = top_mults<SUBS>(T, 0u);  // index 0: beta for SUBS = 4, nothing else
  auto fold = [&](uint32_t j, uint2 (&x0)[SUBS], uint2 (&z)[SUBS], uint2 (&yq)[NQ - 1][SUBS])
      __attribute__((always_inline)) {
    const uint32_t tid = fresh_v(threadIdx.x);
    uint2 d[SUBS];
    top_inverse<SUBS>(x0, 0u, tm0);
    top_inverse<SUBS>(z, 0u, tm0);  // D_256 lifted
    // D_KB(x0)_s = (lifted D_256)_s ^ x0_{s | 2^m} for each high bit 256 2^m < KB clear in s
#pragma unroll
    for (int s = 0; s < SUBS; ++s) {
      d[s] = z[s];
#pragma unroll
      for (int m = 1; m < SUBS; m <<= 1)
        if (!(s & m)) qx(d[s], x0[s | m]);
    }
    uint2 acc[4][SUBS];  // S_b, per Cantor bit b of kappa
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int s = 0; s < SUBS; ++s) acc[b][s] = make_uint2(0u, 0u);
    auto accumulate = [&](const uint2 (&y)[SUBS], uint32_t kq) __attribute__((always_inline)) {
#pragma unroll
      for (int b = 0; b < 4; ++b)
        if ((kq >> b) & 1u)
#pragma unroll
          for (int s = 0; s < SUBS; ++s) qx(acc[b][s], y[s]);
    };
    for_each_q(std::make_integer_sequence<int, NQ>{}, [&](auto qc) __attribute__((always_inline)) {
      constexpr int q = decltype(qc)::value;
      constexpr uint32_t kq = big_kappa<NQ>(q);
      if constexpr (kq != 0) {
        if constexpr (q == 0) {
          accumulate(x0, kq);
        } else if (seg_live(q)) {
          top_inverse<SUBS>(yq[q - 1], static_cast<uint32_t>(q), top_mults<SUBS>(T, static_cast<uint32_t>(q)));
          accumulate(yq[q - 1], kq);
        }
      }
    });
#pragma unroll
    for (int s = 0; s < SUBS; ++s) qx(d[s], acc[0][s]);
#pragma unroll
    for (int b = 1; b < 4; ++b) {
      if (!kappa_bit_used<NQ>(b)) continue;
      const Mult m = tmult(T, 1u << b);
#pragma unroll
      for (int s = 0; s < SUBS; ++s) qm(d[s], acc[b][s], m);
    }
    top_forward<SUBS>(d, 0u, tm0);
    scr_q_store<false>(tile, j, tid, d[0]);  // over the slot this thread just read: e_0 waits in the tile
#pragma unroll
    for (int s = 1; s < SUBS; ++s) scr_q_store<true>(scrD + s * kSegScr, j, tid, d[s]);
  };
  if constexpr (SUBS >= 8) {
    // k = 2048: the segments stream through the fold one at a time (the
    // per-bit sums and every segment's quads at once exceed the 128 VGPRs of
    // a 1024-thread workgroup): d ^= kappa_q y_q, one multiply per segment.
#pragma unroll 1
    for (uint32_t j = 0; j < 16; ++j) {
      const uint32_t tid = fresh_v(threadIdx.x);
      uint2 d[SUBS];
      {
        uint2 x0[SUBS], z[SUBS];
#pragma unroll
        for (int s = 0; s < SUBS; ++s) {
          x0[s] = scr_q<true>(scrY + s * kSegScr, j, tid);
          z[s] = scr_q<true>(scrD + s * kSegScr, j, tid);
        }
        top_inverse<SUBS>(x0, 0u, tm0);
        top_inverse<SUBS>(z, 0u, tm0);  // D_256 lifted
#pragma unroll
        for (int s = 0; s < SUBS; ++s) {
          d[s] = z[s];
#pragma unroll
          for (int m = 1; m < SUBS; m <<= 1)
            if (!(s & m)) qx(d[s], x0[s | m]);
          if constexpr (big_kappa<NQ>(0) == 1u) qx(d[s], x0[s]);  // kappa_0 in {0, 1}
        }
      }
      for_each_q(std::make_integer_sequence<int, NQ>{}, [&](auto qc) __attribute__((always_inline)) {
        constexpr int q = decltype(qc)::value;
        constexpr uint32_t kq = big_kappa<NQ>(q);
        if (q > 0 && kq != 0 && seg_live(q)) {
          __builtin_amdgcn_sched_barrier(0);
          const DevTables Tq = fresh_tables(T);
          uint2 y[SUBS];
#pragma unroll
          for (int s = 0; s < SUBS; ++s)
            y[s] = (q == NQ - 1 && s == SUBS - 1) ? scr_q<false>(tile, j, tid)  // this thread's own
                                                   : scr_q<true>(scrY + (SUBS * q + s) * kSegScr, j, tid);
          top_inverse_fetch<SUBS>(Tq, y, static_cast<uint32_t>(q));
          if constexpr (kq == 1u) {
#pragma unroll
            for (int s = 0; s < SUBS; ++s) qx(d[s], y[s]);
          } else {
            const Mult m = tmult(Tq, kq);
#pragma unroll
            for (int s = 0; s < SUBS; ++s) qm(d[s], y[s], m);
          }
        }
      });
      top_forward<SUBS>(d, 0u, tm0);
      scr_q_store<false>(tile, j, tid, d[0]);  // over the slot this thread just read: e_0 waits in the tile
#pragma unroll
      for (int s = 1; s < SUBS; ++s) scr_q_store<true>(scrD + s * kSegScr, j, tid, d[s]);
    }
  } else {
  constexpr int JB = kRecJB<NQ>;
#pragma unroll 1
  for (uint32_t j0 = 0; j0 < 16; j0 += JB) {
    const uint32_t tid = fresh_v(threadIdx.x);
    // every quad of JB positions in flight at once (one latency per JB positions)
    uint2 x0[JB][SUBS], z[JB][SUBS], yq[JB][NQ - 1][SUBS];
#pragma unroll
    for (int u = 0; u < JB; ++u) {
#pragma unroll
      for (int s = 0; s < SUBS; ++s) {
        x0[u][s] = scr_q<true>(scrY + s * kSegScr, j0 + u, tid);
        z[u][s] = scr_q<true>(scrD + s * kSegScr, j0 + u, tid);
      }
#pragma unroll
      for (int q = 1; q < NQ; ++q) {  // (zeros for empty segments: skipping them here spills at k = 1024)
#pragma unroll
        for (int s = 0; s < SUBS; ++s)
          yq[u][q - 1][s] = (q == NQ - 1 && s == SUBS - 1) ? scr_q<false>(tile, j0 + u, tid)  // this thread's own
                                                           : scr_q<true>(scrY + (SUBS * q + s) * kSegScr, j0 + u, tid);
      }
    }
#pragma unroll
    for (int u = 0; u < JB; ++u) fold(j0 + u, x0[u], z[u], yq[u]);
  }
  }

  // ---- phase 3: FFT(256, 256 s) of e_s, postmultiply erased rows, copy out
#pragma unroll 1
  for (uint32_t s = 0; s < SUBS; ++s) {
    const uint32_t index = 256u * s;
    const uint32_t tid = fresh_v(threadIdx.x), lane = tid & 63u;
    uint32_t XL[16], XH[16];
    if (s == 0) scr_load<false>(tile, tid, XL, XH);  // this thread's own e_0
    __syncthreads();  // the tile (e_0 read) and the tables are free
    stage_vpools<kS, kTB>(T, index, VP, true);
    __syncthreads();
    if (s != 0) scr_load<true>(scrD + s * kSegScr, tid, XL, XH);
    with_gen<0, kSubMaxGen<KB>, false>(index, [&](auto gc) __attribute__((always_inline)) {
      constexpr int GEN = decltype(gc)::value;
      hi_levels<kS, false, GEN == 0, 0, GEN, kBigPrioDec>(T, VP, index, XL, XH);
    });
    hi_write<kS>(tile, fresh_v(hb), XL, XH);
    __syncthreads();
    {
      const uint32_t gg = fresh(g), cq = fresh_v(cqb);
      cq_read<kS>(tile, cq, XL, XH);
      with_gen<0, kSubMaxGen<KB>, false>(index, [&](auto gc) __attribute__((always_inline)) {
        constexpr int GEN = decltype(gc)::value;
        cq_levels<kS, false, GEN == 0, GEN, false, kBigPrioDec>(T, VP, index, gg, XL, XH);
      });
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        uint2 raw[8];
        const uint32_t r0 = index + 16 * gg + 8 * half;
        load_rows_v<8>(raw, sh, a.shard_len, rv, r0, T.zeros, lane, ncols, full);
        // received symbol (present) or postmultiplied (erased; tower in, Cantor out: out_pools)
        pipelined_rec<8>(
            [&](auto pc) __attribute__((always_inline)) {
              return (cpool_t)(T.out_pools) + rv.e(r0 + decltype(pc)::value) * kPoolWords;
            },
            [&](auto pc) __attribute__((always_inline)) { return !rv.pr(r0 + decltype(pc)::value); },
            [&](auto pc, const Mult& pool) __attribute__((always_inline)) {
              constexpr int p = decltype(pc)::value;
              const int x = 8 * half + p;
              if (rv.pr(index + 16 * gg + x)) {
                blk_to_quad(raw[p], XL[x], XH[x]);
              } else {
                const uint32_t l = XL[x], h = XH[x];
                qmul_set(XL[x], XH[x], l, h, pool);
              }
            });
      }
      __syncthreads();
      cq_write<kS>(tile, cq, XL, XH);
    }
    __syncthreads();
    tile_copy_out<KB>(a, tile, pb, col0, ncols, s);
  }
}

// One workgroup per payload: the status (mod.rs:178-180), the mode, and for a
// decode the erasure locator (fused_locator: eval_error_polynomial,
// inc_reconstruct.rs:90-113, folded to the n rows; or the caller's
// locators) as row multipliers E and present flags PR.  Once per payload
// instead of once per column tile.
// n = 16384: the Walsh scratch W alone is 64 KiB, so E and PR go straight to
// the record (big_rows_global) instead of through LDS.
template <int K, int N>
__global__ __launch_bounds__(256) void k_big_records(DevTables T, ReconstructArgs a, uint8_t* out) {
#if NP_BOUNDS_CHECK
  bounds_arm(bounds_of(a, T, 0));  // (E and PR may live in LDS here: records unchecked)
#endif
  constexpr bool RG = big_rows_global(N);
  __shared__ uint32_t W[N];
  __shared__ __attribute__((aligned(16))) uint16_t El[RG ? 8 : N];
  __shared__ __attribute__((aligned(16))) uint8_t PRl[RG ? 16 : N];
  const uint32_t pb = blockIdx.x, tid = threadIdx.x;
  const uint8_t* pres = a.present + static_cast<size_t>(pb) * N;
  uint8_t* rec = out + static_cast<size_t>(pb) * big_rec_stride(N);
  uint16_t* E = RG ? reinterpret_cast<uint16_t*>(rec + kBigRecHeader) : El;
  uint8_t* PR = RG ? rec + kBigRecHeader + 2u * N : PRl;
  int have1 = 0, have = 0;  // present rows in [0, K) and [0, N)
  uint64_t occ = 0;          // 256-row sub-segments with a present row
  for (int r = 0; r < N; r += 256) {
    const bool p = pres[r + static_cast<int>(tid)] != 0;
    if (r < K) have1 += __syncthreads_count(p);
    const int c = __syncthreads_count(p);
    have += c;
    if (c) occ |= 1ull << (r / 256);
  }
  const bool ok = have >= K;
  if (tid == 0 && a.status) {
    a.status[2 * pb] = ok ? 0u : kStatusNeedMoreShards;
    a.status[2 * pb + 1] = static_cast<uint32_t>(have);
  }
  const uint32_t mode = !ok ? kBigSkip : have1 == K ? kBigCopy : kBigDecode;
  if (tid == 0) {
    reinterpret_cast<uint32_t*>(rec)[0] = mode;
    reinterpret_cast<uint32_t*>(rec)[2] = static_cast<uint32_t>(occ);
    reinterpret_cast<uint32_t*>(rec)[3] = static_cast<uint32_t>(occ >> 32);
  }
  if (mode != kBigDecode) return;
  if (a.locators) {  // mul(x, log m) == x * EXP[m] (inc_log_mul.rs:42-49)
    const uint16_t* loc = a.locators + static_cast<size_t>(pb) * N;
    for (uint32_t v = tid; v < static_cast<uint32_t>(N); v += 256) {
      E[v] = T.exp[loc[v]];
      PR[v] = pres[v];
    }
  } else {
    fused_locator<N, 256>(T, pres, W, E, PR);
  }
  if constexpr (!RG) {
    __syncthreads();
    uint4* dst = reinterpret_cast<uint4*>(rec + kBigRecHeader);
    for (uint32_t v = tid; v < 2u * N / 16u; v += 256) dst[v] = reinterpret_cast<const uint4*>(E)[v];
    dst += 2u * N / 16u;
    for (uint32_t v = tid; v < static_cast<uint32_t>(N) / 16u; v += 256) dst[v] = reinterpret_cast<const uint4*>(PR)[v];
  }
}

constexpr size_t enc_big_lds() { return static_cast<size_t>(Geo<kS>::kTileBytes) + 4u * Geo<kS>::kVPWords; }
constexpr size_t rec_big_lds(uint32_t n) {  // tile, tables, E (2 n bytes), PR (n bytes) up to n = 8192
  return static_cast<size_t>(Geo<kS>::kTileBytes) + 4u * Geo<kS>::kVPWords + (big_rows_global(n) ? 0u : 3u * n);
}
// Dynamic LDS of every instance fits the CU's 160 KiB (n = 8192 exactly fills it).
static_assert(enc_big_lds() <= 160u * 1024u, "encode LDS");
static_assert(16384 / 256 <= 64, "sub-segment occupancy is one u64");
static_assert(rec_big_lds(8192) <= 160u * 1024u, "largest reconstruct instance (k = 1024 / 2048, n = 8192) LDS");

// Calls f(reconstruct kernel, record kernel) for the instances of (n, k);
// false if none.
template <typename F>
bool with_rec_big(uint32_t n, uint32_t k, F&& f) {
  if (k == 512) {
    if (n == 1024) return f(&k_reconstruct_big<512, 2>, &k_big_records<512, 1024>), true;
    if (n == 2048) return f(&k_reconstruct_big<512, 4>, &k_big_records<512, 2048>), true;
    if (n == 4096) return f(&k_reconstruct_big<512, 8>, &k_big_records<512, 4096>), true;
  } else if (k == 1024) {
    if (n == 2048) return f(&k_reconstruct_big<1024, 2>, &k_big_records<1024, 2048>), true;
    if (n == 4096) return f(&k_reconstruct_big<1024, 4>, &k_big_records<1024, 4096>), true;
    if (n == 8192) return f(&k_reconstruct_big<1024, 8>, &k_big_records<1024, 8192>), true;
  } else if (k == 2048) {
    if (n == 4096) return f(&k_reconstruct_big<2048, 2>, &k_big_records<2048, 4096>), true;
    if (n == 8192) return f(&k_reconstruct_big<2048, 4>, &k_big_records<2048, 8192>), true;
    if (n == 16384) return f(&k_reconstruct_big<2048, 8>, &k_big_records<2048, 16384>), true;
  }
  return false;
}

}  // namespace

bool big_encode_supported(uint32_t n, uint32_t k) {
  return (k == 512 || k == 1024 || k == 2048) && n >= 2 * k && n <= 65536;
}
bool big_reconstruct_supported(uint32_t n, uint32_t k) {
  return with_rec_big(n, k, [](auto, auto) {});
}
size_t big_encode_scratch_per_tile(uint32_t k) {
  return k == 512 ? enc_scratch<512>() : k == 1024 ? enc_scratch<1024>() : enc_scratch<2048>();
}
size_t big_reconstruct_scratch_per_tile(uint32_t n, uint32_t k) {
  const uint32_t subs = k / kS;
  return static_cast<size_t>(subs) * (n / k + 1) * kSegScr - kSegScr;
}

// Workgroups of the big kernels resident on the device at once (one per CU:
// 1024 threads and 130-160 KiB of LDS each), rounded down to a multiple of 8.
// Each launch covers at most that many tiles, so a launch is one full round of
// workgroups on the CUs (no partial last round) and its scratch stays that of
// the resident workgroups.
int current_device() {
  int d = 0;
  return hipGetDevice(&d) == hipSuccess ? d : 0;
}

// Cached per (device, kernel instance) under a lock (contexts on different
// threads may ask at once); the occupancy is that of the instance launched.
size_t resident_slots_of(int device, const void* kern, size_t lds) {
  static std::mutex mu;
  static std::map<std::pair<int, const void*>, size_t> cache;
  std::lock_guard<std::mutex> g(mu);
  const auto key = std::make_pair(device, kern);
  const auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  int cus = 0, per = 0, prev = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
  // the occupancy query runs on the current device: switch to `device` for it
  const bool sw = hipGetDevice(&prev) == hipSuccess && prev != device && hipSetDevice(device) == hipSuccess;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, kTB, lds) != hipSuccess || per <= 0) per = 1;
  if (sw) (void)hipSetDevice(prev);
  const size_t slots = std::max<size_t>(8, static_cast<size_t>(cus) * per / 8 * 8);
  cache[key] = slots;
  return slots;
}

size_t big_resident_slots(int device, uint32_t n, uint32_t k, bool reconstruct) {
  const void* kern = nullptr;
  if (reconstruct) {
    with_rec_big(n, k, [&](auto kf, auto) { kern = reinterpret_cast<const void*>(kf); });
    return kern ? resident_slots_of(device, kern, rec_big_lds(n)) : 8;
  }
  kern = k == 512 ? reinterpret_cast<const void*>(&k_encode_big<512>)
         : k == 1024 ? reinterpret_cast<const void*>(&k_encode_big<1024>)
                     : reinterpret_cast<const void*>(&k_encode_big<2048>);
  return resident_slots_of(device, kern, enc_big_lds());
}

hipError_t launch_encode_big(const DevTables& T, const EncodeArgs& a, uint8_t* scratch, size_t scratch_bytes,
                             hipStream_t s) {
  if (!big_encode_supported(a.n, a.k)) return hipErrorInvalidValue;
  const size_t nchunks = (a.payload_len + 2 * a.k - 1) / (2 * a.k);
  if (nchunks == 0 || a.batch == 0) return hipSuccess;
  const uint32_t tiles = static_cast<uint32_t>((nchunks + kTile - 1) / kTile);
  const size_t total = a.batch * tiles;
  // multiple of 8 keeps tile0 % 8 == 0 (tile_of)
  const size_t per_tile = big_encode_scratch_per_tile(a.k);
  const void* kern = a.k == 512 ? reinterpret_cast<const void*>(&k_encode_big<512>)
                     : a.k == 1024 ? reinterpret_cast<const void*>(&k_encode_big<1024>)
                                   : reinterpret_cast<const void*>(&k_encode_big<2048>);
  const size_t per_launch = std::min(resident_slots_of(current_device(), kern, enc_big_lds()), scratch_bytes / per_tile / 8 * 8);
  if (per_launch == 0 || total > 0xffffffffu) return hipErrorInvalidValue;
  for (size_t t0 = 0; t0 < total; t0 += per_launch) {
    const uint32_t blocks = static_cast<uint32_t>(std::min(per_launch, total - t0));
    if (a.k == 512)
      k_encode_big<512><<<blocks, kTB, enc_big_lds(), s>>>(T, a, static_cast<uint32_t>(nchunks), tiles,
                                                            static_cast<uint32_t>(t0), scratch);
    else if (a.k == 1024)
      k_encode_big<1024><<<blocks, kTB, enc_big_lds(), s>>>(T, a, static_cast<uint32_t>(nchunks), tiles,
                                                             static_cast<uint32_t>(t0), scratch);
    else
      k_encode_big<2048><<<blocks, kTB, enc_big_lds(), s>>>(T, a, static_cast<uint32_t>(nchunks), tiles,
                                                             static_cast<uint32_t>(t0), scratch);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

size_t big_record_stride(uint32_t n) { return big_rec_stride(n); }

hipError_t launch_big_records(const DevTables& T, const ReconstructArgs& a, uint8_t* records, hipStream_t s) {
  if (!big_reconstruct_supported(a.n, a.k) || a.batch > 0x7fffffffu) return hipErrorInvalidValue;
  if (a.batch == 0) return hipSuccess;
  with_rec_big(a.n, a.k, [&](auto, auto recs) {
    recs<<<static_cast<uint32_t>(a.batch), 256, 0, s>>>(T, a, records);
  });
  return hipGetLastError();
}

hipError_t launch_reconstruct_big(const DevTables& T, const ReconstructArgs& a, uint8_t* scratch,
                                  size_t scratch_bytes, hipStream_t s) {
  if (!big_reconstruct_supported(a.n, a.k)) return hipErrorInvalidValue;
  const size_t nsyms = a.shard_len / 2;
  if (nsyms == 0 || a.batch == 0) return hipSuccess;
  const uint32_t tiles = static_cast<uint32_t>((nsyms + kTile - 1) / kTile);
  const size_t total = a.batch * tiles;
  const size_t per_tile = big_reconstruct_scratch_per_tile(a.n, a.k);
  const void* kern = nullptr;
  with_rec_big(a.n, a.k, [&](auto k, auto) { kern = reinterpret_cast<const void*>(k); });
  const size_t per_launch =
      std::min(resident_slots_of(current_device(), kern, rec_big_lds(a.n)), scratch_bytes / per_tile / 8 * 8);
  if (per_launch == 0 || total > 0xffffffffu) return hipErrorInvalidValue;
  for (size_t t0 = 0; t0 < total; t0 += per_launch) {
    const uint32_t blocks = static_cast<uint32_t>(std::min(per_launch, total - t0));
    with_rec_big(a.n, a.k, [&](auto kern, auto) {
      kern<<<blocks, kTB, rec_big_lds(a.n), s>>>(T, a, static_cast<uint32_t>(nsyms), tiles, static_cast<uint32_t>(t0),
                                                 scratch);
    });
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t configure_big_kernels() {
  hipError_t e = hipSuccess;
  auto set = [&](const void* f, size_t bytes) {
    hipError_t r = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(bytes));
    if (r != hipSuccess && e == hipSuccess) e = r;
  };
  set(reinterpret_cast<const void*>(&k_encode_big<512>), enc_big_lds());
  set(reinterpret_cast<const void*>(&k_encode_big<1024>), enc_big_lds());
  set(reinterpret_cast<const void*>(&k_encode_big<2048>), enc_big_lds());
  for (uint32_t k : {512u, 1024u, 2048u})
    for (uint32_t nq : {2u, 4u, 8u})
      with_rec_big(nq * k, k, [&](auto kern, auto) { set(reinterpret_cast<const void*>(kern), rec_big_lds(nq * k)); });
  return e;
}

hipError_t bounds_take_big(uint32_t out[8]) { return bounds_take_tu(out); }

}  // namespace np
