// Specialised gfx950 kernels for k = 1024 (BASELINE config 4: n = 4096).
//
// A 256-column tile of a size-1024 transform needs 512 KiB, more than the LDS
// holds, so a workgroup (1024 threads, the K = 256 register layouts of
// fast_common.hpp) runs the transform as four size-256 sub-segments plus the
// two top levels (8, 9) that mix them:
//
//   phase 1  per sub-segment: LDS tile -> column-quad levels 0..3 -> high-layout
//            levels 4..7 -> registers -> per-workgroup scratch in HBM / L2;
//   phase 2  per position quad, across the sub-segments: levels 8, 9 (and for
//            reconstruct the segment combination, formal derivative and the
//            forward transform's top levels) -> scratch;
//   phase 3  per sub-segment: scratch -> high-layout levels 7..4 -> LDS ->
//            column-quad levels 3..0 -> shard rows / output.
//
// Scratch traffic stays in the workgroup (each thread reads back what it
// wrote), so no inter-workgroup synchronisation is needed.  The top-level
// skews of a size-1024 transform at index I are Cantor((I >> 9) + 2t) for
// level 9 and Cantor((I >> 8) + 2t) for level 8 (fast_common.hpp, skew_c).
//
// Reference: inc_afft.rs:139-214 / :267-332, inc_encode.rs:15-48,
// inc_reconstruct.rs:1-113, mod.rs:117-239.
#include <map>
#include <mutex>

#include "fast_common.hpp"

namespace np {
namespace {

constexpr int kS = 256;                   // sub-segment (register-layout) size
constexpr int kKB = 1024;                 // k served here
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
__device__ __forceinline__ void scr_q_store(uint8_t* seg, uint32_t j, uint32_t tid, uint32_t l, uint32_t h) {
  const uint64_t v = static_cast<uint64_t>(l) | (static_cast<uint64_t>(h) << 32);
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
  for (int j = 0; j < 16; ++j) scr_q_store<NT>(seg, j, tid, L[j], H[j]);
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

__device__ __forceinline__ Mult mult_of(const DevTables& T, uint32_t c) {
  uint32_t p[20];
  pool_of(T, c, p);
  return make_mult(p);
}

// x ^= c * y for one (L, H) quad pair.
__device__ __forceinline__ void qm(uint2& x, const uint2& y, const Mult& m) { qmul(x.x, x.y, y.x, y.y, m); }
__device__ __forceinline__ void qx(uint2& x, const uint2& y) {
  x.x ^= y.x;
  x.y ^= y.y;
}

// ------------------------------------------------------------------ encode ----
// The shift's top-level outputs W are written once and read once: streaming
// (-6 % on the encode); the coefficients M keep the default policy.
#ifndef NP_W_NT
#define NP_W_NT true
#endif
constexpr size_t kEncScratch = 8 * kSegScr;  // M (4 sub-segments) + W (4 sub-segments)

__global__ __launch_bounds__(kTB) __attribute__((amdgpu_waves_per_eu(4))) void k_encode_big(
    DevTables T, EncodeArgs a, uint32_t nchunks, uint32_t tiles, uint32_t tile0, uint8_t* scratch) {
  using G = Geo<kS>;
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
  uint8_t* scrM = scratch + static_cast<size_t>(blockIdx.x) * kEncScratch;
  uint8_t* scrW = scrM + 4 * kSegScr;
  const uint32_t tid = threadIdx.x, lane = tid & 63u, g = uniform(tid >> 6);
  const bool full =
      ncols == kTile && ((reinterpret_cast<uintptr_t>(a.shards) | a.batch_stride | a.shard_len) & 7u) == 0;
  const uint32_t cqb = col_base<kS>(4 * lane) ^ (32u * g);
  const uint32_t hb = col_base<kS>(tid / G::R) ^ (8u * (tid % G::R));
  const bool fast_in = ((reinterpret_cast<uintptr_t>(pay) & 7u) == 0) &&
                       static_cast<size_t>(ch0 + kTile) * 2 * kKB <= a.payload_len;

  // ---- phase 1: x_s = IFFT(256, 256 s)(sub-segment s of every chunk), s = 0..3
#pragma unroll 1
  for (uint32_t s = 0; s < 4; ++s) {
    const uint32_t index = 256u * s;
    __syncthreads();  // previous sub-segment is done with the tile and the tables
    stage_vpools<kS, kTB>(T, index, VP);
    {
      const uint32_t c0 = tid / G::Q, m0 = tid % G::Q;
      const uint32_t base = col_base<kS>(c0) ^ (8u * m0);
      const size_t gbase = static_cast<size_t>(ch0 + c0) * 2 * kKB + 2u * index + 8u * m0;
      if (fast_in) {
        uint2 v[16];
#pragma unroll
        for (int i = 0; i < 16; ++i)
          v[i] = load_once(pay + gbase + static_cast<size_t>(i) * 16 * 2 * kKB);
#pragma unroll
        for (int i = 0; i < 16; ++i) *reinterpret_cast<uint2*>(tile + (base ^ col_base_c<kS>(16u * i))) = v[i];
      } else {
#pragma unroll 1
        for (uint32_t i = 0; i < 16; ++i) {
          const size_t g0 = gbase + static_cast<size_t>(i) * 16 * 2 * kKB;
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
      store_rows(out, a.shard_len, index + 16 * g, a.wanted_n, CL, CH, lane, ncols, full);  // systematic rows
      cq_levels<kS, true, false>(T, VP, index, g, CL, CH);
      cq_write<kS>(tile, cq, CL, CH);
    }
    __syncthreads();
    uint32_t XL[16], XH[16];
    hi_read<kS>(tile, fresh_v(hb), XL, XH);
    hi_levels<kS, true, false>(T, VP, index, XL, XH);
    scr_store<false>(scrM + s * kSegScr, tid, XL, XH);
  }

  // ---- phase 2: top inverse levels at index 0 -> coefficients M (in place)
  {
    const Mult beta = mult_of(T, 2u);  // level 8, t = 1; the t = 0 skews at index 0 are zero
#pragma unroll 1
    for (uint32_t j = 0; j < 16; ++j) {
      uint2 x0 = scr_q<false>(scrM, j, tid), x1 = scr_q<false>(scrM + kSegScr, j, tid);
      uint2 x2 = scr_q<false>(scrM + 2 * kSegScr, j, tid), x3 = scr_q<false>(scrM + 3 * kSegScr, j, tid);
      qx(x1, x0);     // level 8, t = 0: hi ^= lo
      qx(x3, x2);     // level 8, t = 1
      qm(x2, x3, beta);
      qx(x2, x0);     // level 9, t = 0
      qx(x3, x1);
      scr_q_store<false>(scrM + kSegScr, j, tid, x1.x, x1.y);
      scr_q_store<false>(scrM + 2 * kSegScr, j, tid, x2.x, x2.y);
      scr_q_store<false>(scrM + 3 * kSegScr, j, tid, x3.x, x3.y);
    }
  }

  // ---- phase 3: every shift c = 1.. : top forward levels, then 4 x FFT(256)
  const uint32_t nshift = a.n / kKB;
#pragma unroll 1
  for (uint32_t c = 1; c < nshift; ++c) {
    if (c * kKB >= a.wanted_n) break;
    {
      const Mult m9 = mult_of(T, 2u * c), m80 = mult_of(T, 4u * c), m81 = mult_of(T, 4u * c + 2u);
#pragma unroll 1
      for (uint32_t j = 0; j < 16; ++j) {
        uint2 w0 = scr_q<false>(scrM, j, tid), w1 = scr_q<false>(scrM + kSegScr, j, tid);
        uint2 w2 = scr_q<false>(scrM + 2 * kSegScr, j, tid), w3 = scr_q<false>(scrM + 3 * kSegScr, j, tid);
        qm(w0, w2, m9);  // level 9: lo ^= c9 * hi; hi ^= lo
        qx(w2, w0);
        qm(w1, w3, m9);
        qx(w3, w1);
        qm(w0, w1, m80);  // level 8, t = 0
        qx(w1, w0);
        qm(w2, w3, m81);  // level 8, t = 1
        qx(w3, w2);
        scr_q_store<NP_W_NT>(scrW, j, tid, w0.x, w0.y);
        scr_q_store<NP_W_NT>(scrW + kSegScr, j, tid, w1.x, w1.y);
        scr_q_store<NP_W_NT>(scrW + 2 * kSegScr, j, tid, w2.x, w2.y);
        scr_q_store<NP_W_NT>(scrW + 3 * kSegScr, j, tid, w3.x, w3.y);
      }
    }
#pragma unroll 1
    for (uint32_t s = 0; s < 4; ++s) {
      const uint32_t index = c * kKB + 256u * s;
      if (index >= a.wanted_n) break;
      __syncthreads();  // the tile and the tables are free
      stage_vpools<kS, kTB>(T, index, VP);
      __syncthreads();
      uint32_t XL[16], XH[16];
      scr_load<NP_W_NT>(scrW + s * kSegScr, tid, XL, XH);
      hi_levels<kS, false, false>(T, VP, index, XL, XH);
      hi_write<kS>(tile, fresh_v(hb), XL, XH);
      __syncthreads();
      cq_read<kS>(tile, fresh_v(cqb), XL, XH);
      cq_levels<kS, false, false>(T, VP, index, g, XL, XH);
      store_rows(out, a.shard_len, index + 16 * g, a.wanted_n, XL, XH, lane, ncols, full);
    }
  }
}

// ------------------------------------------------------------- reconstruct ----
// n = NQ * 1024.  As in k_reconstruct_fast (kernels_fast.hip), for the first
// k = 1024 outputs d = D_1024(x0) ^ x1 ^ x2 ^ beta (x2 ^ x3) (NQ = 4) or
// D_1024(x0) ^ x0 ^ x1 (NQ = 2) with x_q = IFFT(1024, 1024 q)(premultiplied
// segment q), then out = FFT(1024, 0)(d).  Here each x_q is 4 sub-segment
// transforms y_qs = IFFT(256, 1024 q + 256 s) plus levels 8, 9, and
// D_1024 = (I (x) D_256) + (high single-bit terms l = 256, 512); the D_256 part
// commutes with levels 8, 9, so it is applied to y_0s in phase 1.
template <int NQ>
__global__ __launch_bounds__(kTB) __attribute__((amdgpu_waves_per_eu(4))) void k_reconstruct_big(
    DevTables T, ReconstructArgs a, uint32_t nsyms, uint32_t tiles, uint32_t tile0, uint8_t* scratch) {
  using G = Geo<kS>;
  constexpr int N = NQ * kKB;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* tile = smem;
  uint32_t* VP = reinterpret_cast<uint32_t*>(smem + G::kTileBytes);
  uint16_t* E = reinterpret_cast<uint16_t*>(smem + G::kTileBytes + 4 * G::kVPWords);
  uint8_t* PR = smem + G::kTileBytes + 4 * G::kVPWords + 2 * N;
  const uint32_t blk = tile0 + blockIdx.x;
  const TileRef tr = tile_of(blk, tiles, (a.batch & 7u) == 0);
  const uint32_t pb = tr.pb, tl = tr.tl;
  if (a.status && uniform(a.status[2 * pb]) != 0) return;  // fewer than k present rows (k_payload_status)
  const uint32_t col0 = tl * kTile;
  const uint32_t ncols = min(static_cast<uint32_t>(kTile), nsyms - col0);
  const uint8_t* sh = a.shards + static_cast<size_t>(pb) * a.batch_stride + 2 * static_cast<size_t>(col0);
  const uint8_t* pres = a.present + static_cast<size_t>(pb) * N;
  const uint16_t* loc = a.locators ? a.locators + static_cast<size_t>(pb) * N : nullptr;
  uint8_t* scrY = scratch + static_cast<size_t>(blockIdx.x) * (4 * NQ + 4) * kSegScr;  // y_qs, then D_256(y_0s)
  uint8_t* scrD = scrY + 4 * NQ * kSegScr;                                               // reused for e_s
  const uint32_t tid = threadIdx.x, lane = tid & 63u, g = uniform(tid >> 6);
  const bool full =
      ncols == kTile && ((reinterpret_cast<uintptr_t>(a.shards) | a.batch_stride | a.shard_len) & 7u) == 0;
  const uint32_t cqb = col_base<kS>(4 * lane) ^ (32u * g);
  const uint32_t hb = col_base<kS>(tid / G::R) ^ (8u * (tid % G::R));

  if (loc) {
    for (uint32_t v = tid; v < static_cast<uint32_t>(N); v += kTB) {
      E[v] = T.exp[loc[v]];
      PR[v] = pres[v];
    }
  } else {
    fused_locator<N, kTB>(T, pres, reinterpret_cast<uint32_t*>(tile), E, PR);
  }

  // ---- phase 1: y_qs for every segment q and sub-segment s
  __syncthreads();  // E, PR ready
#pragma unroll 1
  for (uint32_t qs = 0; qs < 4u * NQ; ++qs) {
    const uint32_t index = 256u * qs;  // = 1024 q + 256 s
    const uint32_t gg = fresh(g);
    // the sub-segment's present rows load while the tables are staged
    uint2 rows[2][8];
#pragma unroll
    for (int half = 0; half < 2; ++half)
      load_rows<8>(rows[half], sh, a.shard_len, PR, index + 16 * gg + 8 * half, T.zeros, lane, ncols, full);
    __syncthreads();  // tile / tables free
    stage_vpools<kS, kTB>(T, index, VP);
    __syncthreads();
    uint32_t XL[16], XH[16];
    {
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        const uint2 (&raw)[8] = rows[half];
        pipelined<8>(
            T, [&](auto pc) __attribute__((always_inline)) { return uniform(E[index + 16 * gg + 8 * half + decltype(pc)::value]); },
            [&](auto pc, const Mult& pool) __attribute__((always_inline)) {
              constexpr int p = decltype(pc)::value;
              const int x = 8 * half + p;
              XL[x] = 0;
              XH[x] = 0;
              if (uniform(PR[index + 16 * gg + x])) {
                uint32_t l, h;
                blk_to_quad(raw[p], l, h);
                qmul_set(XL[x], XH[x], l, h, pool);
              }
            });
      }
      cq_levels<kS, true, false>(T, VP, index, gg, XL, XH);
      cq_write<kS>(tile, fresh_v(cqb), XL, XH);
    }
    __syncthreads();
    hi_read<kS>(tile, fresh_v(hb), XL, XH);
    hi_levels<kS, true, false>(T, VP, index, XL, XH);
    scr_store<true>(scrY + qs * kSegScr, tid, XL, XH);
    if (qs < 4) {  // segment 0: also D_256(y_0s)
      uint32_t DL[16] = {0}, DH[16] = {0};
      add_derivative<kS>(DL, XL, tid % G::R);
      add_derivative<kS>(DH, XH, tid % G::R);
      scr_store<true>(scrD + qs * kSegScr, tid, DL, DH);
    }
  }

  // ---- phase 2: levels 8, 9 of every x_q, the combination, the derivative's
  // high terms and the forward transform's levels 9, 8 -> e_s (over D's slots)
  {
    const Mult beta = mult_of(T, 2u);
#pragma unroll 1
    for (uint32_t j = 0; j < 16; ++j) {
      uint2 d[4], x0[4];
      // x_0 and D_256 lifted: level 8 (t = 0 skew 0, t = 1 beta), level 9 (skew 0)
      {
        uint2 y[4], z[4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          y[s] = scr_q<true>(scrY + s * kSegScr, j, tid);
          z[s] = scr_q<true>(scrD + s * kSegScr, j, tid);
        }
        qx(y[1], y[0]);
        qx(y[3], y[2]);
        qm(y[2], y[3], beta);
        qx(y[2], y[0]);
        qx(y[3], y[1]);
        qx(z[1], z[0]);
        qx(z[3], z[2]);
        qm(z[2], z[3], beta);
        qx(z[2], z[0]);
        qx(z[3], z[1]);
#pragma unroll
        for (int s = 0; s < 4; ++s) x0[s] = y[s];
        // D_1024(x0)_s = (lifted D_256)_s ^ x0_{s|1} (s even) ^ x0_{s|2} (s < 2)
        d[0] = z[0];
        qx(d[0], x0[1]);
        qx(d[0], x0[2]);
        d[1] = z[1];
        qx(d[1], x0[3]);
        d[2] = z[2];
        qx(d[2], x0[3]);
        d[3] = z[3];
        if (NQ == 2) {
#pragma unroll
          for (int s = 0; s < 4; ++s) qx(d[s], x0[s]);
        }
      }
      uint2 yq[NQ - 1][4];  // every segment's quads in flight at once (one latency per j)
#pragma unroll
      for (int q = 1; q < NQ; ++q)
#pragma unroll
        for (int s = 0; s < 4; ++s) yq[q - 1][s] = scr_q<true>(scrY + (4 * q + s) * kSegScr, j, tid);
#pragma unroll
      for (uint32_t q = 1; q < static_cast<uint32_t>(NQ); ++q) {
        uint2 (&y)[4] = yq[q - 1];
        // levels 8 (t = 0: Cantor(4q), t = 1: Cantor(4q + 2)) and 9 (Cantor(2q)): hi ^= lo; lo ^= c hi
        {
          const Mult m80 = mult_of(T, 4u * q), m81 = mult_of(T, 4u * q + 2u);
          qx(y[1], y[0]);
          qm(y[0], y[1], m80);
          qx(y[3], y[2]);
          qm(y[2], y[3], m81);
        }
        {
          const Mult m9 = mult_of(T, 2u * q);
          qx(y[2], y[0]);
          qm(y[0], y[2], m9);
          qx(y[3], y[1]);
          qm(y[1], y[3], m9);
        }
        if (NQ == 2 || q == 1) {
#pragma unroll
          for (int s = 0; s < 4; ++s) qx(d[s], y[s]);  // ^ x1 (and for NQ = 4: x1)
        } else if (q == 2) {
#pragma unroll
          for (int s = 0; s < 4; ++s) qx(d[s], y[s]);  // ^ x2 (kept in yq[1] for q = 3)
        } else {  // q == 3: ^ beta (x2 ^ x3)
#pragma unroll
          for (int s = 0; s < 4; ++s) {
            qx(y[s], yq[1][s]);
            qm(d[s], y[s], beta);
          }
        }
      }
      // forward levels 9 (t = 0: skew 0) and 8 (t = 0: 0, t = 1: beta) at index 0
      qx(d[2], d[0]);
      qx(d[3], d[1]);
      qx(d[1], d[0]);
      qm(d[2], d[3], beta);
      qx(d[3], d[2]);
#pragma unroll
      for (int s = 0; s < 4; ++s) scr_q_store<true>(scrD + s * kSegScr, j, tid, d[s].x, d[s].y);
    }
  }

  // ---- phase 3: FFT(256, 256 s) of e_s, postmultiply erased rows, copy out
#pragma unroll 1
  for (uint32_t s = 0; s < 4; ++s) {
    const uint32_t index = 256u * s;
    __syncthreads();
    stage_vpools<kS, kTB>(T, index, VP);
    __syncthreads();
    uint32_t XL[16], XH[16];
    scr_load<true>(scrD + s * kSegScr, tid, XL, XH);
    hi_levels<kS, false, false>(T, VP, index, XL, XH);
    hi_write<kS>(tile, fresh_v(hb), XL, XH);
    __syncthreads();
    {
      const uint32_t gg = fresh(g), cq = fresh_v(cqb);
      cq_read<kS>(tile, cq, XL, XH);
      cq_levels<kS, false, false>(T, VP, index, gg, XL, XH);
#pragma unroll
      for (int half = 0; half < 2; ++half) {
        uint2 raw[8];
        load_rows<8>(raw, sh, a.shard_len, PR, index + 16 * gg + 8 * half, T.zeros, lane, ncols, full);
        pipelined<8>(
            T, [&](auto pc) __attribute__((always_inline)) { return uniform(E[index + 16 * gg + 8 * half + decltype(pc)::value]); },
            [&](auto pc, const Mult& pool) __attribute__((always_inline)) {
              constexpr int p = decltype(pc)::value;
              const int x = 8 * half + p;
              if (uniform(PR[index + 16 * gg + x])) {
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
    {  // output column c, symbols 256 s .. 256 s + 255: bytes [2048 c + 512 s, +512)
      uint8_t* outp = a.out + static_cast<size_t>(pb) * a.out_stride + static_cast<size_t>(col0) * 2 * kKB + 512u * s;
      const bool al_o = ((reinterpret_cast<uintptr_t>(a.out) | a.out_stride) & 7u) == 0;
      const uint32_t c0 = tid / G::Q, m0 = tid % G::Q;
      const uint32_t base = col_base<kS>(c0) ^ (8u * m0);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const uint32_t c = c0 + 16u * i;
        if (c >= ncols) break;
        const uint2 v = *reinterpret_cast<const uint2*>(tile + (base ^ col_base_c<kS>(16u * i)));
        uint8_t* o = outp + static_cast<size_t>(c) * 2 * kKB + 8u * m0;
        if (al_o) {
          store_once(o, v);
        } else {
#pragma unroll
          for (int e = 0; e < 8; ++e) o[e] = static_cast<uint8_t>((e < 4 ? v.x : v.y) >> (8 * (e & 3)));
        }
      }
    }
  }
}

size_t enc_big_lds() { return static_cast<size_t>(Geo<kS>::kTileBytes) + 4u * Geo<kS>::kVPWords; }
template <int NQ>
size_t rec_big_lds() {
  return static_cast<size_t>(Geo<kS>::kTileBytes) + 4u * Geo<kS>::kVPWords + 3u * NQ * kKB;
}

}  // namespace

bool big_encode_supported(uint32_t n, uint32_t k) { return k == kKB && n >= 2 * k && n <= 65536; }
bool big_reconstruct_supported(uint32_t n, uint32_t k) {
  return k == kKB && (n == 2 * k || n == 4 * k);
}
size_t big_encode_scratch_per_tile() { return kEncScratch; }
size_t big_reconstruct_scratch_per_tile(uint32_t n) { return (4u * (n / kKB) + 4u) * kSegScr; }

// Workgroups of the k = 1024 kernels resident on the device at once (one per
// CU: 1024 threads and ~150 KiB of LDS each), rounded down to a multiple of 8.
// Each launch covers at most that many tiles, so a launch is one full round of
// workgroups on the CUs (no partial last round) and its scratch stays that of
// the resident workgroups.
int current_device() {
  int d = 0;
  return hipGetDevice(&d) == hipSuccess ? d : 0;
}

// Cached per device under a lock (contexts on different threads may ask at once).
size_t big_resident_slots(int device) {
  static std::mutex mu;
  static std::map<int, size_t> cache;
  std::lock_guard<std::mutex> g(mu);
  const auto it = cache.find(device);
  if (it != cache.end()) return it->second;
  int cus = 0, per = 0, prev = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || cus <= 0) cus = 256;
  // the occupancy query runs on the current device: switch to `device` for it
  const bool sw = hipGetDevice(&prev) == hipSuccess && prev != device && hipSetDevice(device) == hipSuccess;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, reinterpret_cast<const void*>(&k_reconstruct_big<4>), kTB,
                                                   rec_big_lds<4>()) != hipSuccess ||
      per <= 0)
    per = 1;
  if (sw) (void)hipSetDevice(prev);
  const size_t slots = std::max<size_t>(8, static_cast<size_t>(cus) * per / 8 * 8);
  cache[device] = slots;
  return slots;
}

hipError_t launch_encode_big(const DevTables& T, const EncodeArgs& a, uint8_t* scratch, size_t scratch_bytes,
                             hipStream_t s) {
  const size_t nchunks = (a.payload_len + 2 * a.k - 1) / (2 * a.k);
  if (nchunks == 0 || a.batch == 0) return hipSuccess;
  const uint32_t tiles = static_cast<uint32_t>((nchunks + kTile - 1) / kTile);
  const size_t total = a.batch * tiles;
  // multiple of 8 keeps tile0 % 8 == 0 (tile_of)
  const size_t per_launch = std::min(big_resident_slots(current_device()), scratch_bytes / kEncScratch / 8 * 8);
  if (per_launch == 0 || total > 0xffffffffu) return hipErrorInvalidValue;
  for (size_t t0 = 0; t0 < total; t0 += per_launch) {
    const uint32_t blocks = static_cast<uint32_t>(std::min(per_launch, total - t0));
    k_encode_big<<<blocks, kTB, enc_big_lds(), s>>>(T, a, static_cast<uint32_t>(nchunks), tiles,
                                                     static_cast<uint32_t>(t0), scratch);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_reconstruct_big(const DevTables& T, const ReconstructArgs& a, uint8_t* scratch,
                                  size_t scratch_bytes, hipStream_t s) {
  const size_t nsyms = a.shard_len / 2;
  if (nsyms == 0 || a.batch == 0) return hipSuccess;
  const uint32_t tiles = static_cast<uint32_t>((nsyms + kTile - 1) / kTile);
  const size_t total = a.batch * tiles;
  const size_t per_tile = big_reconstruct_scratch_per_tile(a.n);
  const size_t per_launch = std::min(big_resident_slots(current_device()), scratch_bytes / per_tile / 8 * 8);
  if (per_launch == 0 || total > 0xffffffffu) return hipErrorInvalidValue;
  for (size_t t0 = 0; t0 < total; t0 += per_launch) {
    const uint32_t blocks = static_cast<uint32_t>(std::min(per_launch, total - t0));
    if (a.n == 4 * kKB)
      k_reconstruct_big<4><<<blocks, kTB, rec_big_lds<4>(), s>>>(T, a, static_cast<uint32_t>(nsyms), tiles,
                                                                 static_cast<uint32_t>(t0), scratch);
    else
      k_reconstruct_big<2><<<blocks, kTB, rec_big_lds<2>(), s>>>(T, a, static_cast<uint32_t>(nsyms), tiles,
                                                                 static_cast<uint32_t>(t0), scratch);
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
  set(reinterpret_cast<const void*>(&k_encode_big), enc_big_lds());
  set(reinterpret_cast<const void*>(&k_reconstruct_big<2>), rec_big_lds<2>());
  set(reinterpret_cast<const void*>(&k_reconstruct_big<4>), rec_big_lds<4>());
  return e;
}

}  // namespace np
