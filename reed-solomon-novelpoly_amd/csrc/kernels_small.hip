// Specialised gfx950 kernels for small codes: k = K in {1, 2, 4, 8, 16, 32},
// encode for 2K <= n <= 8K, reconstruct for n in {2K, 4K, 8K} -- the shapes
// of 2 to 191 validators (n_wanted / k_wanted ~ 3), which the generic path
// served at ~13 GiB/s.  K < 8: a column is 2K bytes, loaded and stored whole;
// the 4-position blocks of the register layout are padded.
//
// Work mapping.  One wave owns a tile of 256 codeword columns and holds ALL K
// positions of its lane's four columns in registers: Q[p] = the low / high
// bytes of position p of columns 4l..4l+3 (the column-quad layout of
// kernels_fast.hip with every position in one lane).  Every butterfly of a
// size-K transform then pairs two registers of the same lane with a
// wave-uniform multiplier: no LDS tile, no barrier, no cross-lane traffic.
// Shard rows are position-major, so row p of the tile is register pair p:
// coalesced 8-byte row loads and stores, as on the fast path.  Four waves of a
// workgroup are four independent tiles; the workgroup only shares the staged
// multiplier tables.  Every transform index here is below 256 (n <= 8K <=
// 256), so all transforms run in tower coordinates with subfield multipliers.
//
// Reference: additive FFT inc_afft.rs:139-214 (inverse) / :267-332 (forward);
// encode inc_encode.rs:15-48 + mod.rs:117-157; reconstruct inc_reconstruct.rs:1-85
// + mod.rs:162-239.  The decode folds the size-n inverse transform into
// per-segment transforms exactly as kernels_fast.hip rec_segments (its
// derivation: the comment above rec_tiles there).
#include "fast_common.hpp"

namespace np {
namespace {

constexpr int kSmallMaxSeg = 8;  // n / k at most

// A position's quad lives in one 64-bit value (low plane in the low dword):
// the multiply's selector extraction shifts both planes as one 64-bit value
// (fast_common.hpp selectors), which needs them in an aligned register pair;
// with separate L[] / H[] arrays the allocator kept a paired copy of every
// position (235 VGPRs at K = 32).
__device__ __forceinline__ uint32_t lo(uint64_t q) { return static_cast<uint32_t>(q); }
__device__ __forceinline__ uint32_t hi(uint64_t q) { return static_cast<uint32_t>(q >> 32); }
__device__ __forceinline__ uint64_t quad(uint32_t l, uint32_t h) { return (static_cast<uint64_t>(h) << 32) | l; }

// x ^= c * y (subfield multiplier)
__device__ __forceinline__ void qmul_q(uint64_t& x, uint64_t y, const Mult& m) {
  uint32_t xl = lo(x), xh = hi(x);
  qmul_sub(xl, xh, lo(y), hi(y), m);
  x = quad(xl, xh);
}

// Flat group f of a whole size-K transform: levels 0..logK-1 (inverse) or
// logK-1..0 (forward), K >> (b + 1) groups each.
template <int K, bool INVERSE>
__host__ __device__ constexpr GroupRef reg_group(int f) {
  constexpr int lg = ilog2(K);
  for (int s = 0; s < lg; ++s) {
    const int b = INVERSE ? s : lg - 1 - s, n = K >> (b + 1);
    if (f < n) return GroupRef{b, f};
    f -= n;
  }
  return GroupRef{0, 0};
}

// The size-K transform at `index` (< 256) on the lane's registers, tower
// coordinates.  Group t of level b pairs positions t * 2^(b+1) + u and that +
// 2^b; its skew is Cantor(2t + (index >> b)).  `rows` (wave-uniform bit p =
// position p): inverse transforms skip the groups none of whose input rows is
// set, forward ones the groups none of whose output rows is set.  INDEX0: the
// t = 0 skews of index 0 are the zero element (the reference's skipped
// multiply, inc_afft.rs:170 / :300).
template <int K, bool INVERSE, bool INDEX0>
__device__ __forceinline__ void reg_levels(const DevTables& T, const uint32_t* VP, uint32_t index, uint64_t (&Q)[K],
                                           uint32_t rows = ~0u) {
  auto cval = [&](auto fc) __attribute__((always_inline)) {
    constexpr GroupRef r = reg_group<K, INVERSE>(decltype(fc)::value);
    return 2u * r.t + (index >> r.b);
  };
  auto vaddr = [&](auto fc) __attribute__((always_inline)) {
    constexpr GroupRef r = reg_group<K, INVERSE>(decltype(fc)::value);
    return VP + 8u * vslot<K>(r.b, r.t);
  };
  auto group = [&](auto fc, const Mult& p) __attribute__((always_inline)) {
    constexpr GroupRef r = reg_group<K, INVERSE>(decltype(fc)::value);
    constexpr int d = 1 << r.b;
    constexpr bool live = !INDEX0 || r.t != 0;
    constexpr uint64_t span = ((1ull << (2 * d)) - 1ull) << (r.t * 2 * d);
    if ((rows & span) == 0) return;
#pragma unroll
    for (int u = 0; u < d; ++u) {
      const int x = r.t * 2 * d + u, y = x + d;
      if (INVERSE) {
        Q[y] ^= Q[x];
        if (live) qmul_q(Q[x], Q[y], p);
      } else {
        if (live) qmul_q(Q[x], Q[y], p);
        Q[y] ^= Q[x];
      }
    }
  };
  auto subf = [&](auto) __attribute__((always_inline)) { return std::true_type{}; };
  pipelined_staged<K - 1, true>(T, cval, vaddr, subf, group);
}

// A ^= D_K(X): D(x)[j] = x[j] ^ XOR over single bits l not in j of x[j | l]
// (inc_afft.rs:17-31, closed form SURVEY F7); every position is a register.
template <int K>
__device__ __forceinline__ void add_derivative_reg(uint64_t (&A)[K], const uint64_t (&X)[K]) {
#pragma unroll
  for (int j = 0; j < K; ++j) {
    uint64_t v = X[j];
#pragma unroll
    for (int l = 1; l < K; l <<= 1)
      if (!(j & l)) v ^= X[j | l];
    A[j] ^= v;
  }
}

// Cantor <-> tower coordinates of NR quads (fast_common.hpp tower_convert).
template <int NR>
__device__ __forceinline__ void tower_convert_q(const DevTables& T, uint64_t (&Q)[NR]) {
  const cpool_t q = (cpool_t)(T.tower_pools) + 65536u * kPoolWords;
  const uint32_t sa = q[8 + 3], sb = q[8 + 4], sc = q[8 + 5];
  const uint64_t vv = tower_conv_vhalf(q);
  const uint32_t va = static_cast<uint32_t>(vv), vb = static_cast<uint32_t>(vv >> 32);
#pragma unroll
  for (int p = 0; p < NR; ++p) {
    uint32_t s0, s1, s2, l = lo(Q[p]);
    const uint32_t h = hi(Q[p]);
    asm volatile(
        "v_and_b32 %0, 0x07070707, %3\n\t"
        "v_lshrrev_b32 %1, 3, %3\n\t"
        "v_lshrrev_b32 %2, 6, %3\n\t"
        "v_and_b32 %1, 0x07070707, %1\n\t"
        "v_and_b32 %2, 0x03030303, %2"
        : "=&v"(s0), "=&v"(s1), "=&v"(s2)
        : "v"(h));
    qplane_sub(l, s0, s1, s2, va, vb, sa, sb, sc);
    Q[p] = quad(l, h);
  }
}

// Shard rows row0..row0+NR-1 (those below wanted_n) from the registers;
// streaming stores as store_rows.
template <int NR>
__device__ __forceinline__ void store_rows_k(uint8_t* out, size_t shard_len, uint32_t row0, uint32_t wanted_n,
                                             const uint64_t (&Q)[NR], uint32_t lane, uint32_t ncols, bool full,
                                             bool nt) {
  if (full && row0 + NR <= wanted_n && NR * shard_len < 0x7fffffffu) {
    const __amdgpu_buffer_rsrc_t r = buf_rsrc(out + static_cast<size_t>(row0) * shard_len, NR * static_cast<uint32_t>(shard_len));
#pragma unroll
    for (int p = 0; p < NR; ++p) {
      const uint2 v = cq_row(lo(Q[p]), hi(Q[p]));
      if (nt)
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{v.x, v.y}, r, 8u * lane, static_cast<uint32_t>(p * shard_len),
                                              kRowStoreCpol);
      else
        __builtin_amdgcn_raw_buffer_store_b64(u32x2{v.x, v.y}, r, 8u * lane, static_cast<uint32_t>(p * shard_len), 0);
      __builtin_amdgcn_sched_barrier(0);  // one row at a time: no K rows of temporaries
    }
  } else {
#pragma unroll
    for (int p = 0; p < NR; ++p)
      if (row0 + p < wanted_n) store4(out + static_cast<size_t>(row0 + p) * shard_len, cq_row(lo(Q[p]), hi(Q[p])), lane, ncols, full);
  }
}

// The lane's pieces of rows row0..row0+NR-1; absent rows (mask bit clear)
// read as zeros.  Full tiles: one buffer descriptor over the NR rows, an
// absent row's load offset past its end (returns zeros: no traffic, no
// branch); CPOL 2 = streaming (rows read once).
template <int NR, int CPOL>
__device__ __forceinline__ void load_rows_k(uint2 (&raw)[NR], const uint8_t* sh, size_t shard_len, uint32_t mask,
                                            uint32_t row0, const uint8_t* zeros, uint32_t lane, uint32_t ncols,
                                            bool full) {
  if (full && NR * shard_len < 0x7fffffffu) {
    const __amdgpu_buffer_rsrc_t r = buf_rsrc(sh + static_cast<size_t>(row0) * shard_len, NR * static_cast<uint32_t>(shard_len));
#pragma unroll
    for (int p = 0; p < NR; ++p) {
      const uint32_t so = ((mask >> p) & 1u) ? static_cast<uint32_t>(p * shard_len) : 0x80000000u;
      const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, 8u * lane, so, CPOL);
      raw[p] = make_uint2(v.x, v.y);
    }
  } else {
#pragma unroll
    for (int p = 0; p < NR; ++p) {
      const uint8_t* src = ((mask >> p) & 1u) ? sh + static_cast<size_t>(row0 + p) * shard_len : zeros;
      raw[p] = load4(src, lane, ncols, false);
    }
  }
}

// Wave-tile gt -> (batch entry, tile); false past the batch.
__device__ __forceinline__ bool wave_tile(size_t batch, uint32_t tiles, uint32_t& pb, uint32_t& tl) {
  const uint32_t gt = uniform(blockIdx.x * 4u + (threadIdx.x >> 6));
  pb = gt / tiles;
  tl = gt % tiles;
  return pb < batch;
}

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// Blocks of 4 columns (d[i] = column i, positions 4u..4u+3) <-> quads Q[v] =
// position 4u+v of columns 0..3 (fast_common.hpp blks_to_cq / cq_to_blks).
__device__ __forceinline__ void blks_to_q(const uint2 (&d)[4], uint64_t* Q) {
  uint32_t cl[4], ch[4];
  blks_to_cq(d, cl, ch);
#pragma unroll
  for (int v = 0; v < 4; ++v) Q[v] = quad(cl[v], ch[v]);
}
__device__ __forceinline__ void q_to_blks(const uint64_t* Q, uint2 (&d)[4]) {
  uint32_t cl[4], ch[4];
#pragma unroll
  for (int v = 0; v < 4; ++v) cl[v] = lo(Q[v]), ch[v] = hi(Q[v]);
  cq_to_blks(cl, ch, d);
}
__device__ __forceinline__ uint64_t blk_quad(uint2 d) {
  uint32_t l, h;
  blk_to_quad(d, l, h);
  return quad(l, h);
}

// ----------------------------------------------------------------- encode ----
// mod.rs:144-154 / inc_encode.rs:15-48: chunk c of the payload (K symbols,
// big-endian) is column c; M = IFFT(K, 0)(column), shard rows sK..sK+K-1 =
// FFT(K, sK)(M) for the shifts s below wanted_n / K, rows 0..K-1 the payload.
template <int K>
__global__ __launch_bounds__(256) void k_encode_small(DevTables T, EncodeArgs a, uint32_t nchunks, uint32_t tiles) {
  using G = Geo<K>;
#if NP_BOUNDS_CHECK
  bounds_arm(bounds_of_enc(a));
#endif
  __shared__ __attribute__((aligned(16))) uint32_t VP[kSmallMaxSeg * G::kVPWords];
  const uint32_t nshift = a.n / K;  // <= kSmallMaxSeg (small_encode_supported)
  for (uint32_t s = 0; s < nshift && s * K < a.wanted_n; ++s) stage_vpools<K, 256>(T, s * K, VP + s * G::kVPWords, true);
  __syncthreads();
  uint32_t pb, tl;
  if (!wave_tile(a.batch, tiles, pb, tl)) return;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t ch0 = tl * kTile;
  const uint32_t ncols = min(static_cast<uint32_t>(kTile), nchunks - ch0);
  const uint8_t* pay = a.payloads + static_cast<size_t>(pb) * a.payload_stride;
  uint8_t* out = a.shards + static_cast<size_t>(pb) * a.batch_stride + 2 * static_cast<size_t>(ch0);
  const bool full =
      ncols == kTile && rows_vec_ok(a.shards, a.batch_stride, a.shard_len);

  // ---- the lane's four columns: 2K contiguous payload bytes each
  uint64_t M[K];
  {
    const size_t c0 = static_cast<size_t>(ch0 + 4u * lane) * 2 * K;
    const bool fast = out_vec_ok(pay, 0) &&  // 16-byte loads at any address (rows_vec_ok)
                      static_cast<size_t>(ch0 + kTile) * 2 * K <= a.payload_len;
    if (fast && K < 8) {  // k in {1, 2, 4}: the lane's four columns are 8K contiguous bytes
      uint2 d[4];
      if constexpr (K == 4) {
        const u32x4 v0 = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(pay + c0));
        const u32x4 v1 = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(pay + c0 + 16));
        d[0] = make_uint2(v0.x, v0.y), d[1] = make_uint2(v0.z, v0.w), d[2] = make_uint2(v1.x, v1.y),
        d[3] = make_uint2(v1.z, v1.w);
      } else if constexpr (K == 2) {  // a column is one dword: positions 2, 3 of the blocks are padding
        const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(pay + c0));
        d[0] = make_uint2(v.x, 0), d[1] = make_uint2(v.y, 0), d[2] = make_uint2(v.z, 0), d[3] = make_uint2(v.w, 0);
      } else {  // K == 1: a column is one symbol
        const uint2 v = *reinterpret_cast<const uint2*>(pay + c0);
        d[0] = make_uint2(v.x & 0xffffu, 0), d[1] = make_uint2(v.x >> 16, 0), d[2] = make_uint2(v.y & 0xffffu, 0),
        d[3] = make_uint2(v.y >> 16, 0);
      }
      uint64_t Q4[4];
      blks_to_q(d, Q4);
#pragma unroll
      for (int p = 0; p < K; ++p) M[p] = Q4[p];
    } else if (fast) {
#pragma unroll
      for (int u2 = 0; u2 < K / 8; ++u2) {  // positions 8u2..8u2+7: 16 bytes per column
        uint2 d0[4], d1[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(pay + c0 + i * 2 * K + 16 * u2));
          d0[i] = make_uint2(v.x, v.y);
          d1[i] = make_uint2(v.z, v.w);
        }
        blks_to_q(d0, &M[8 * u2]);
        blks_to_q(d1, &M[8 * u2 + 4]);
      }
    } else {  // the payload's last tile: bytes past payload_len are zeros (mod.rs:135-141)
      constexpr int kBlk = K < 4 ? 1 : K / 4, kBytes = K < 4 ? 2 * K : 8;  // 8-byte blocks per column
#pragma unroll
      for (int u = 0; u < kBlk; ++u) {  // unrolled: M stays in registers
        uint2 d[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const size_t g0 = c0 + static_cast<size_t>(i) * 2 * K + 8u * u;
          uint32_t w[2] = {0, 0};
#pragma unroll
          for (int e = 0; e < kBytes; ++e)
            if (g0 + e < a.payload_len) w[e >> 2] |= static_cast<uint32_t>(pay[g0 + e]) << (8 * (e & 3));
          d[i] = make_uint2(w[0], w[1]);
        }
        if constexpr (K >= 4) {
          blks_to_q(d, &M[4 * u]);
        } else {
          uint64_t Q4[4];
          blks_to_q(d, Q4);
#pragma unroll
          for (int p = 0; p < K; ++p) M[p] = Q4[p];
        }
      }
    }
  }
  store_rows_k<K>(out, a.shard_len, 0, a.wanted_n, M, lane, ncols, full, rows_nt(a.shards, a.batch_stride, a.shard_len));
  tower_convert_q(T, M);  // the transforms run in tower coordinates
  reg_levels<K, true, true>(T, VP, 0, M);
#pragma unroll
  for (int p = 0; p < K; ++p) asm volatile("" : "+v"(M[p]));  // materialise M once

#pragma unroll 1
  for (uint32_t s = 1; s < nshift && s * K < a.wanted_n; ++s) {
    const uint32_t index = uniform(s * K);
    const uint32_t live = a.wanted_n - index;  // rows of this shift that are kept
    const uint32_t rows = live >= static_cast<uint32_t>(K) ? ~0u : (1u << live) - 1u;
    uint64_t X[K];
#pragma unroll
    for (int p = 0; p < K; ++p) X[p] = M[p];
    reg_levels<K, false, false>(T, VP + s * G::kVPWords, index, X, uniform(rows));
    tower_convert_q(T, X);  // back to Cantor coordinates for the shard rows
    store_rows_k<K>(out, a.shard_len, index, a.wanted_n, X, lane, ncols, full, rows_nt(a.shards, a.batch_stride, a.shard_len));
  }
}

// ------------------------------------------------------------ reconstruct ----
// Coefficient kappa_q (Cantor coordinates) of segment q in the first K
// outputs' fold d = D_K(x0) ^ sum_q kappa_q x_q of a decode from nq segments
// (kernels_fast.hip rec_segments / rec8_kappa; tests/test_oracle.py
// test_rec8_kappa).
__device__ __forceinline__ uint32_t small_kappa(int nq, int q) {
  if (nq == 2) return 1u;
  if (nq == 4) return q == 0 ? 0u : q == 1 ? 1u : q == 2 ? 3u : 2u;
  return q < 2 ? 1u : q == 2 ? 3u : q == 3 ? 2u : q == 4 ? 12u : q == 5 ? 15u : q == 6 ? 10u : 8u;
}

// One wave: 256 symbol columns of one payload.  The payload's record
// (kernels_fast.hip k_prefix_locator / k_locator_records) gives nq' (0: fewer
// than k present rows, skipped; 1: every systematic row present, copied; 2 or
// NQ: decode from that many segments) and the premultiply (present rows) /
// postmultiply (erased rows) tables of every row.
template <int K, int NQ>
__global__ __launch_bounds__(256) void k_reconstruct_small(DevTables T, ReconstructArgs a, uint32_t nsyms,
                                                           uint32_t tiles) {
  using G = Geo<K>;
  constexpr int N = NQ * K;
#if NP_BOUNDS_CHECK
  bounds_arm(bounds_of(a, T, prefix_stride_c(N, K)));
#endif
  __shared__ __attribute__((aligned(16))) uint32_t VP[NQ * G::kVPWords];
  for (int q = 0; q < NQ; ++q) stage_vpools<K, 256>(T, static_cast<uint32_t>(q) * K, VP + q * G::kVPWords, true);
  __syncthreads();
  uint32_t pb, tl;
  if (!wave_tile(a.batch, tiles, pb, tl)) return;
  const uint8_t* rec = a.prefix + static_cast<size_t>(pb) * prefix_stride_c(N, K);
  const int nq = uniform(rec[0]);
  if (nq == 0) return;  // NeedMoreShards: output untouched
  const uint32_t* R = reinterpret_cast<const uint32_t*>(rec + prefix_pools_offset(N));
  const uint8_t* pres = a.present + static_cast<size_t>(pb) * N;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t col0 = tl * kTile;
  const uint32_t ncols = min(static_cast<uint32_t>(kTile), nsyms - col0);
  const uint8_t* sh = a.shards + static_cast<size_t>(pb) * a.batch_stride + 2 * static_cast<size_t>(col0);
  const bool full =
      ncols == kTile && rows_vec_ok(a.shards, a.batch_stride, a.shard_len);
  const uint32_t m0 = uniform(static_cast<uint32_t>(__ballot(lane < K && pres[lane] != 0)));

  uint64_t X[K];
  if (nq == 1) {
    uint2 raw[K];
    load_rows_k<K, 2>(raw, sh, a.shard_len, m0, 0, T.zeros, lane, ncols, full);
#pragma unroll
    for (int p = 0; p < K; ++p) X[p] = blk_quad(raw[p]);
  } else {
    uint64_t A[K];
#pragma unroll
    for (int p = 0; p < K; ++p) A[p] = 0;
#pragma unroll 1
    for (int q = nq - 1; q >= 0; --q) {
      const uint32_t row0 = uniform(static_cast<uint32_t>(q) * K);
      const uint32_t m = q == 0 ? m0 : uniform(static_cast<uint32_t>(__ballot(lane < K && pres[row0 + lane] != 0)));
      if (m == 0) continue;  // x_q = 0
      {
        uint2 raw[K];
        if (q == 0)  // read again by the merge
          load_rows_k<K, 0>(raw, sh, a.shard_len, m, 0, T.zeros, lane, ncols, full);
        else
          load_rows_k<K, 2>(raw, sh, a.shard_len, m, row0, T.zeros, lane, ncols, full);
        pipelined_rec<K>(
            [&](auto pc) __attribute__((always_inline)) { return (cpool_t)(R) + (row0 + decltype(pc)::value) * kPoolWords; },
            [&](auto pc) __attribute__((always_inline)) { return ((m >> decltype(pc)::value) & 1u) != 0; },
            [&](auto pc, const Mult& pool) __attribute__((always_inline)) {
              constexpr int x = decltype(pc)::value;
              X[x] = 0;  // absent rows contribute zero
              if ((m >> x) & 1u) {
                uint32_t l, h, xl, xh;
                blk_to_quad(raw[x], l, h);
                qmul_set(xl, xh, l, h, pool);  // Cantor in, tower out (in_pools)
                X[x] = quad(xl, xh);
              }
            });
      }
      const uint32_t* vp = VP + q * G::kVPWords;
      if (q == 0) {
        reg_levels<K, true, true>(T, vp, 0, X, m);
        add_derivative_reg<K>(A, X);
      } else {
        reg_levels<K, true, false>(T, vp, row0, X, m);
      }
      const uint32_t kq = uniform(small_kappa(nq, q));
      if (kq == 1u) {
#pragma unroll
        for (int p = 0; p < K; ++p) A[p] ^= X[p];
      } else if (kq != 0u) {
        uint32_t kp[20];
        pool_of<true>(T, kq, kp);
        const Mult pool = make_mult(kp);
#pragma unroll
        for (int p = 0; p < K; ++p) qmul_q(A[p], X[p], pool);
      }
    }
    // FFT(K, 0): only the erased systematic rows' outputs are needed
    reg_levels<K, false, true>(T, VP, 0, A, ~m0);
    // merge: received systematic rows (mod.rs:225-235), postmultiplied
    // recovered ones (inc_reconstruct.rs:76-84)
    uint2 raw[K];
    load_rows_k<K, 2>(raw, sh, a.shard_len, m0, 0, T.zeros, lane, ncols, full);
    pipelined_rec<K>(
        [&](auto pc) __attribute__((always_inline)) { return (cpool_t)(R) + decltype(pc)::value * kPoolWords; },
        [&](auto pc) __attribute__((always_inline)) { return ((m0 >> decltype(pc)::value) & 1u) == 0; },
        [&](auto pc, const Mult& pool) __attribute__((always_inline)) {
          constexpr int x = decltype(pc)::value;
          if ((m0 >> x) & 1u) {
            X[x] = blk_quad(raw[x]);
          } else {
            uint32_t xl, xh;
            qmul_set(xl, xh, lo(A[x]), hi(A[x]), pool);  // tower in, Cantor out (out_pools)
            X[x] = quad(xl, xh);
          }
        });
  }
  // ---- copy-out: column c of the tile is 2K contiguous output bytes
  uint8_t* out = a.out + static_cast<size_t>(pb) * a.out_stride + static_cast<size_t>(col0) * 2 * K;
  const bool al16 = full && out_vec_ok(a.out, a.out_stride);
  const bool al8 = true;  // 8-byte stores at any address (rows_vec_ok)
  if constexpr (K < 8) {  // k in {1, 2, 4}: 2K output bytes per column
    uint64_t Q4[4] = {0, 0, 0, 0};
#pragma unroll
    for (int p = 0; p < K; ++p) Q4[p] = X[p];
    uint2 d[4];
    q_to_blks(Q4, d);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t c = 4u * lane + i;
      uint8_t* o = out + static_cast<size_t>(c) * 2 * K;
      if (c < ncols) {
        if constexpr (K == 4) {
          if (al8) {
            *reinterpret_cast<uint2*>(o) = d[i];
          } else {
#pragma unroll
            for (int e = 0; e < 8; ++e) o[e] = static_cast<uint8_t>((e < 4 ? d[i].x : d[i].y) >> (8 * (e & 3)));
          }
        } else {
#pragma unroll
          for (int e = 0; e < 2 * K; ++e) o[e] = static_cast<uint8_t>(d[i].x >> (8 * e));
        }
      }
    }
    return;
  }
#pragma unroll
  for (int u2 = 0; u2 < K / 8; ++u2) {
    uint2 d0[4], d1[4];
    q_to_blks(&X[8 * u2], d0);
    q_to_blks(&X[8 * u2 + 4], d1);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t c = 4u * lane + i;
      uint8_t* o = out + static_cast<size_t>(c) * 2 * K + 16u * u2;
      if (al16) {
        *reinterpret_cast<uint4*>(o) = make_uint4(d0[i].x, d0[i].y, d1[i].x, d1[i].y);
      } else if (c < ncols) {
        if (al8) {
          *reinterpret_cast<uint2*>(o) = d0[i];
          *reinterpret_cast<uint2*>(o + 8) = d1[i];
        } else {
          const uint32_t w[4] = {d0[i].x, d0[i].y, d1[i].x, d1[i].y};
#pragma unroll
          for (int e = 0; e < 16; ++e) o[e] = static_cast<uint8_t>(w[e >> 2] >> (8 * (e & 3)));
        }
      }
    }
  }
}

template <int K>
hipError_t launch_encode_k(const DevTables& T, const EncodeArgs& a, hipStream_t s) {
  const size_t nchunks = (a.payload_len + 2 * a.k - 1) / (2 * a.k);
  if (nchunks == 0 || a.batch == 0) return hipSuccess;
  if (nchunks > 0xffffffffu) return hipErrorInvalidValue;
  const uint32_t tiles = static_cast<uint32_t>((nchunks + kTile - 1) / kTile);
  const size_t blocks = (a.batch * tiles + 3) / 4;
  if (a.batch * tiles > 0xffffffffu || blocks > 0x7fffffffu) return hipErrorInvalidValue;
  k_encode_small<K><<<static_cast<uint32_t>(blocks), 256, 0, s>>>(T, a, static_cast<uint32_t>(nchunks), tiles);
  return hipGetLastError();
}

template <int K, int NQ>
hipError_t launch_reconstruct_k(const DevTables& T, const ReconstructArgs& a, hipStream_t s) {
  const size_t nsyms = a.shard_len / 2;
  if (nsyms == 0 || a.batch == 0) return hipSuccess;
  if (nsyms > 0xffffffffu) return hipErrorInvalidValue;
  const uint32_t tiles = static_cast<uint32_t>((nsyms + kTile - 1) / kTile);
  const size_t blocks = (a.batch * tiles + 3) / 4;
  if (a.batch * tiles > 0xffffffffu || blocks > 0x7fffffffu) return hipErrorInvalidValue;
  k_reconstruct_small<K, NQ><<<static_cast<uint32_t>(blocks), 256, 0, s>>>(T, a, static_cast<uint32_t>(nsyms), tiles);
  return hipGetLastError();
}

template <int K>
hipError_t reconstruct_by_nq(const DevTables& T, const ReconstructArgs& a, hipStream_t s) {
  if (a.n == 8u * K) return launch_reconstruct_k<K, 8>(T, a, s);
  if (a.n == 4u * K) return launch_reconstruct_k<K, 4>(T, a, s);
  return launch_reconstruct_k<K, 2>(T, a, s);
}

}  // namespace

bool small_encode_supported(uint32_t n, uint32_t k) {
  return (k == 1 || k == 2 || k == 4 || k == 8 || k == 16 || k == 32) && n >= 2 * k &&
         n <= kSmallMaxSeg * k;
}

bool small_reconstruct_supported(uint32_t n, uint32_t k) {
  return (k == 1 || k == 2 || k == 4 || k == 8 || k == 16 || k == 32) &&
         (n == 2 * k || n == 4 * k || n == 8 * k);
}

hipError_t launch_encode_small(const DevTables& T, const EncodeArgs& a, hipStream_t s) {
  switch (a.k) {
    case 1: return launch_encode_k<1>(T, a, s);
    case 2: return launch_encode_k<2>(T, a, s);
    case 4: return launch_encode_k<4>(T, a, s);
    case 8: return launch_encode_k<8>(T, a, s);
    case 16: return launch_encode_k<16>(T, a, s);
    case 32: return launch_encode_k<32>(T, a, s);
    default: return hipErrorNotSupported;
  }
}

hipError_t launch_reconstruct_small(const DevTables& T, const ReconstructArgs& a, hipStream_t s) {
  switch (a.k) {
    case 1: return reconstruct_by_nq<1>(T, a, s);
    case 2: return reconstruct_by_nq<2>(T, a, s);
    case 4: return reconstruct_by_nq<4>(T, a, s);
    case 8: return reconstruct_by_nq<8>(T, a, s);
    case 16: return reconstruct_by_nq<16>(T, a, s);
    case 32: return reconstruct_by_nq<32>(T, a, s);
    default: return hipErrorNotSupported;
  }
}

hipError_t bounds_take_small(uint32_t out[8]) { return bounds_take_tu(out); }

}  // namespace np
