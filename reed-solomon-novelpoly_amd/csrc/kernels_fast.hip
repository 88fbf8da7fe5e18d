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
#include "fast_common.hpp"

namespace np {
namespace {

// ----------------------------------------------------------------- encode ----
// One workgroup: 256 chunks of one payload.  mod.rs:144-154 / inc_encode.rs:15-48.
template <int K>
__global__ __launch_bounds__(4 * K) __attribute__((amdgpu_waves_per_eu(4))) void k_encode_fast(DevTables T, EncodeArgs a, uint32_t nchunks, uint32_t tiles) {
  using G = Geo<K>;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* tile = smem;
  uint32_t* VP = reinterpret_cast<uint32_t*>(smem + G::kTileBytes);  // 2 staged transforms
  const TileRef tr = tile_of(blockIdx.x, tiles, (a.batch & 7u) == 0);
  const uint32_t pb = tr.pb, tl = tr.tl;
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
  const uint32_t nshift = a.n / K;
  stage_vpools<K, G::kThreads>(T, 0, VP);                              // inverse transform, index 0
  if (nshift > 1) stage_vpools<K, G::kThreads>(T, K, VP + G::kVPWords);  // first shift
  __syncthreads();

  const uint32_t cqb = col_base<K>(4 * lane) ^ (32u * g);  // blocks 4g..4g+3 of columns 4l..4l+3
  // ---- cq pass: systematic rows, inverse levels 0..3
  {
    uint32_t CL[16], CH[16];
    cq_read<K>(tile, cqb, CL, CH);
    store_rows(out, a.shard_len, 16 * g, a.wanted_n, CL, CH, lane, ncols, full);
    cq_levels<K, true, true>(T, VP, 0, g, CL, CH);
    cq_write<K>(tile, cqb, CL, CH);
  }
  __syncthreads();
  // ---- high layout: inverse levels 4.. -> coefficients M
  const uint32_t hb = col_base<K>(tid / G::R) ^ (8u * (tid % G::R));
  uint32_t ML[16], MH[16];
  hi_read<K>(tile, hb, ML, MH);
  hi_levels<K, true, true>(T, VP, 0, ML, MH);
#pragma unroll
  for (int q = 0; q < 16; ++q) asm volatile("" : "+v"(ML[q]), "+v"(MH[q]));  // materialise M once

  for (uint32_t sh = 1; sh < nshift; ++sh) {
    const uint32_t index = sh * K;
    if (index >= a.wanted_n) break;
    uint32_t XL[16], XH[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      XL[q] = ML[q];
      XH[q] = MH[q];
    }
    const uint32_t* vp = VP + (sh & 1u) * G::kVPWords;
    hi_levels<K, false, false>(T, vp, index, XL, XH);
    __syncthreads();  // the previous cq pass is done with the tile and with the other table buffer
    if (sh + 1 < nshift && (sh + 1) * K < a.wanted_n)
      stage_vpools<K, G::kThreads>(T, (sh + 1) * K, VP + ((sh + 1) & 1u) * G::kVPWords);
    hi_write<K>(tile, fresh_v(hb), XL, XH);
    __syncthreads();
    cq_read<K>(tile, fresh_v(cqb), XL, XH);
    cq_levels<K, false, false>(T, vp, index, g, XL, XH);
    store_rows(out, a.shard_len, index + 16 * g, a.wanted_n, XL, XH, lane, ncols, full);
  }
}

// ------------------------------------------------------------ reconstruct ----
struct RecCtx {
  const DevTables& T;
  size_t shard_len;
  uint8_t* tile;
  const uint16_t* E;
  const uint8_t* PR;
  const uint8_t* sh;
  uint32_t* VP;  // 2 staged transforms
  uint32_t g, lane, tid, ncols;
  bool full;
  uint32_t cqb, hb;
};

// The segment sweep (segments 2, 3, 1, 0 for NQ = 4; 1, 0 for NQ = 2): x_q =
// IFFT(K, qK)(premultiplied segment q), folded into A.  A runtime loop keeps the
// kernel small; at index 0 the t = 0 multipliers are the zero element, whose
// table yields 0 (the reference's skipped multiply).
template <int K, int NQ>
__device__ __forceinline__ void rec_segments(const RecCtx& c, uint32_t (&AL)[16], uint32_t (&AH)[16]) {
  const DevTables& T = c.T;
#pragma unroll 1
  for (int step = 0; step < NQ; ++step) {
    const int q = NQ == 4 ? (step == 0 ? 2 : step == 1 ? 3 : 3 - step) : 1 - step;
    const uint32_t index = uniform(static_cast<uint32_t>(q) * K);
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
    const uint32_t* vp = c.VP + (step & 1) * Geo<K>::kVPWords;
    cq_levels<K, true, false>(T, vp, index, g, XL, XH);
    if (step > 0) {
      __syncthreads();  // the previous high pass is done with the tile and the other table buffer
      if (step + 1 < NQ) {
        const int qn = NQ == 4 ? (step + 1 == 1 ? 3 : 2 - step) : 0;
        stage_vpools<K, Geo<K>::kThreads>(T, static_cast<uint32_t>(qn) * K, c.VP + ((step + 1) & 1) * Geo<K>::kVPWords);
      }
    }
    cq_write<K>(c.tile, cqb, XL, XH);
    __syncthreads();
    hi_read<K>(c.tile, hb, XL, XH);
    hi_levels<K, true, false>(T, vp, index, XL, XH);
    __builtin_amdgcn_sched_barrier(0);
    if (step == 0) {
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        AL[j] = XL[j];
        AH[j] = XH[j];
      }
    } else if (q == 0) {
      if (NQ == 2) {
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
}

// Decode of one tile from the first NQ segments (NQ * K rows).  The inverse
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
// Decoding from a prefix.  The first NQ * K codeword symbols are the
// codeword of the same message under the (NQ * K, K) code: the size-n forward
// transform of the zero-padded coefficients copies its lower half into the
// upper half at every top level (inc_afft.rs:267-332 with x[i + d] = 0), so its
// first NQ * K outputs are FFT(NQ * K, 0) of the same coefficients.  A message
// of K symbols is determined by any K of its codeword symbols, so decoding the
// prefix with the rows beyond it treated as erased yields the reference's
// output whenever the prefix holds at least K present rows.
template <int K, int NQ>
__device__ __forceinline__ void rec_tile(const DevTables& T, const ReconstructArgs& a, const uint8_t* sh,
                                         const uint8_t* pres, const uint16_t* loc, uint8_t* smem, uint32_t pb,
                                         uint32_t col0, uint32_t ncols, bool full) {
  using G = Geo<K>;
  constexpr int N = NQ * K;
  uint8_t* tile = smem;
  uint32_t* VP = reinterpret_cast<uint32_t*>(smem + G::kTileBytes);  // 2 staged transforms
  uint16_t* E = reinterpret_cast<uint16_t*>(smem + G::kTileBytes + 8 * G::kVPWords);  // multiplier of every row
  uint8_t* PR = smem + G::kTileBytes + 8 * G::kVPWords + 2 * 4 * K;                    // present flags
  const uint32_t tid = threadIdx.x, lane = tid & 63u, g = uniform(tid >> 6);
  const uint32_t cqb = col_base<K>(4 * lane) ^ (32u * g);

  uint32_t XL[16], XH[16];
  if constexpr (NQ == 1) {
    for (uint32_t v = tid; v < static_cast<uint32_t>(K); v += G::kThreads) PR[v] = 1;
    __syncthreads();
  } else {
    if (loc) {
      for (uint32_t v = tid; v < static_cast<uint32_t>(N); v += G::kThreads) {
        E[v] = T.exp[loc[v]];  // mul(x, log m) == x * EXP[m] (inc_log_mul.rs:42-49)
        PR[v] = pres[v];
      }
    } else {
      fused_locator<N, G::kThreads>(T, pres, reinterpret_cast<uint32_t*>(tile), E, PR);
    }
    // multiplier tables of the first two segment transforms (indices 2K, 3K or K, 0)
    stage_vpools<K, G::kThreads>(T, (NQ == 4 ? 2u : 1u) * K, VP);
    stage_vpools<K, G::kThreads>(T, (NQ == 4 ? 3u : 0u) * K, VP + G::kVPWords);
    __syncthreads();

    const uint32_t hb = col_base<K>(tid / G::R) ^ (8u * (tid % G::R));
    uint32_t AL[16], AH[16];
    // segment order: 2, 3, 1, 0 (NQ = 4) or 1, 0 (NQ = 2)
    RecCtx c{T, a.shard_len, tile, E, PR, sh, VP, g, lane, tid, ncols, full, cqb, hb};
    rec_segments<K, NQ>(c, AL, AH);
    // ---- forward transform of size K at index 0
    const uint32_t* vp0 = VP + ((NQ - 1) & 1) * G::kVPWords;  // segment 0's tables = FFT(K, 0)'s
    hi_levels<K, false, true>(T, vp0, 0, AL, AH);
    __syncthreads();
    hi_write<K>(tile, fresh_v(hb), AL, AH);
    __syncthreads();
    cq_read<K>(tile, fresh_v(cqb), XL, XH);
    cq_levels<K, false, true>(T, vp0, 0, g, XL, XH);
  }
  // ---- merge: received systematic rows, postmultiplied recovered ones
  const uint32_t cqbf = fresh_v(cqb);
#pragma unroll
  for (int half = 0; half < 2; ++half) {
    uint2 raw[8];
    load_rows<8>(raw, sh, a.shard_len, PR, 16 * g + 8 * half, T.zeros, lane, ncols, full);
    if constexpr (NQ == 1) {
#pragma unroll
      for (int p = 0; p < 8; ++p) blk_to_quad(raw[p], XL[8 * half + p], XH[8 * half + p]);
    } else {
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
  }
  __syncthreads();
  cq_write<K>(tile, cqbf, XL, XH);
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

// One workgroup: 256 symbol columns of one batch entry, n = NQ * K.  With the
// locator computed here (a.locators == nullptr) the workgroup decodes from the
// shortest prefix of K, 2K or n rows holding K present rows (rec_tile).
// Precomputed locators are over all n rows, so they pin the full decode.
template <int K, int NQ>
__global__ __launch_bounds__(4 * K) __attribute__((amdgpu_waves_per_eu(4))) void k_reconstruct_fast(DevTables T, ReconstructArgs a, uint32_t nsyms,
                                                            uint32_t tiles) {
  constexpr int N = NQ * K;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const TileRef tr = tile_of(blockIdx.x, tiles, (a.batch & 7u) == 0);
  const uint32_t pb = tr.pb, tl = tr.tl;
  const uint32_t col0 = tl * kTile;
  const uint32_t ncols = min(static_cast<uint32_t>(kTile), nsyms - col0);
  const uint8_t* sh = a.shards + static_cast<size_t>(pb) * a.batch_stride + 2 * static_cast<size_t>(col0);
  const uint8_t* pres = a.present + static_cast<size_t>(pb) * N;
  const uint16_t* loc = a.locators ? a.locators + static_cast<size_t>(pb) * N : nullptr;
  const bool full =
      ncols == kTile && ((reinterpret_cast<uintptr_t>(a.shards) | a.batch_stride | a.shard_len) & 7u) == 0;

  int nq = NQ;
  if (!loc) {
    const uint32_t tid = threadIdx.x;  // 4K threads cover rows [0, 2K) twice over
    const int have1 = __syncthreads_count(tid < static_cast<uint32_t>(K) && pres[tid] != 0);
    const int have2 = __syncthreads_count(tid < static_cast<uint32_t>(2 * K) && pres[tid] != 0);
    nq = have1 == K ? 1 : (NQ == 4 && have2 >= K) ? 2 : NQ;
  }
  if (nq == 1) {
    rec_tile<K, 1>(T, a, sh, pres, loc, smem, pb, col0, ncols, full);
  } else if (NQ == 4 && nq == 2) {
    rec_tile<K, 2>(T, a, sh, pres, loc, smem, pb, col0, ncols, full);
  } else {
    rec_tile<K, NQ>(T, a, sh, pres, loc, smem, pb, col0, ncols, full);
  }
}

// ------------------------------------------------------------- launchers ----
template <int K>
size_t encode_lds_bytes() {
  return static_cast<size_t>(Geo<K>::kTileBytes) + 2u * 4u * Geo<K>::kVPWords;
}

template <int K, int NQ>
size_t reconstruct_lds_bytes() {
  return static_cast<size_t>(Geo<K>::kTileBytes) + 2u * 4u * Geo<K>::kVPWords + 3u * 4 * K;
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
