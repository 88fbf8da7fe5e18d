// Store-rate calibration for the encode's memory floor (verdict
// r05 item 5): 1 GiB of coalesced stores at 4, 8, 16 and 32 waves per CU,
// 256 / 512 / 1024 contiguous bytes per wave-instruction (4 / 8 / 16 B per
// lane), default and non-temporal policies; and the config-3 encode's own mix
// (1 byte read for every 4 written: 1 GiB of payload in, 4 GiB of shard rows
// out, 8-byte stores per lane) at zero arithmetic.  Best of 5 launches each,
// HIP events.  Not product code: make -C tools/microbench calib_store.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef unsigned int v2u __attribute__((ext_vector_type(2)));
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <int W, bool NT>
__global__ __launch_bounds__(256) void store_k(uint8_t* __restrict__ out, size_t bytes) {
  const size_t per = 256u * W;  // bytes per wave-instruction
  const size_t waves = static_cast<size_t>(gridDim.x) * 4;
  const uint32_t lane = threadIdx.x & 63u;
  size_t wv = static_cast<size_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  for (size_t off = wv * per; off < bytes; off += waves * per) {
    uint8_t* p = out + off + W * 4u * lane;
    if constexpr (W == 1) {
      const uint32_t v = static_cast<uint32_t>(off) ^ lane;
      if constexpr (NT)
        __builtin_nontemporal_store(v, reinterpret_cast<uint32_t*>(p));
      else
        *reinterpret_cast<uint32_t*>(p) = v;
    } else if constexpr (W == 2) {
      const v2u v = {static_cast<uint32_t>(off), lane};
      if constexpr (NT)
        __builtin_nontemporal_store(v, reinterpret_cast<v2u*>(p));
      else
        *reinterpret_cast<v2u*>(p) = v;
    } else {
      const v4u v = {static_cast<uint32_t>(off), lane, 1u, 2u};
      if constexpr (NT)
        __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(p));
      else
        *reinterpret_cast<v4u*>(p) = v;
    }
  }
}

// The encode's shape at zero arithmetic: a wave reads 512 B of payload (8 B
// per lane) and writes 4 x 512 B of shard rows (8 B per lane, four rows 1 MiB
// apart, the shifts' rows); NT as the encode's row stores.
template <bool NT>
__global__ __launch_bounds__(256) void mix_k(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                            size_t in_bytes) {
  const size_t waves = static_cast<size_t>(gridDim.x) * 4;
  const uint32_t lane = threadIdx.x & 63u;
  const size_t quarter = in_bytes;  // out = 4 rows of in_bytes each
  size_t wv = static_cast<size_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  for (size_t off = wv * 512; off < in_bytes; off += waves * 512) {
    const v2u x = *reinterpret_cast<const v2u*>(in + off + 8u * lane);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      v2u y = x;
      y.x ^= r;
      uint8_t* p = out + r * quarter + off + 8u * lane;
      if constexpr (NT)
        __builtin_nontemporal_store(y, reinterpret_cast<v2u*>(p));
      else
        *reinterpret_cast<v2u*>(p) = y;
    }
  }
}

// Variants of the mix: each wave takes U x 512 B of payload (8-byte loads, all
// U in flight) and writes the same bytes to 4 rows with SW-byte stores per
// lane.
template <int SW, int U, bool NT>
__global__ __launch_bounds__(256) void mixv_k(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                             size_t in_bytes) {
  constexpr size_t C = 512u * U;
  const size_t waves = static_cast<size_t>(gridDim.x) * 4;
  const uint32_t lane = threadIdx.x & 63u;
  size_t wv = static_cast<size_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  for (size_t off = wv * C; off < in_bytes; off += waves * C) {
    uint32_t acc = 0;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const v2u x = *reinterpret_cast<const v2u*>(in + off + 512u * u + 8u * lane);
      acc ^= x.x ^ x.y;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      uint8_t* o = out + r * in_bytes + off;
#pragma unroll
      for (size_t i = 0; i < C / (64u * SW); ++i) {
        uint8_t* q = o + i * 64u * SW + SW * lane;
        if constexpr (SW == 4) {
          if constexpr (NT) __builtin_nontemporal_store(acc + r, reinterpret_cast<uint32_t*>(q));
          else *reinterpret_cast<uint32_t*>(q) = acc + r;
        } else if constexpr (SW == 8) {
          const v2u v = {acc, static_cast<uint32_t>(r)};
          if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<v2u*>(q));
          else *reinterpret_cast<v2u*>(q) = v;
        } else {
          const v4u v = {acc, static_cast<uint32_t>(r), 1u, 2u};
          if constexpr (NT) __builtin_nontemporal_store(v, reinterpret_cast<v4u*>(q));
          else *reinterpret_cast<v4u*>(q) = v;
        }
      }
    }
  }
}

int main() {
  const size_t gib = size_t(1) << 30;
  uint8_t *in = nullptr, *out = nullptr;
  if (hipMalloc(&in, gib) != hipSuccess || hipMalloc(&out, 4 * gib) != hipSuccess) return 1;
  (void)hipMemset(in, 1, gib);
  (void)hipMemset(out, 0, 4 * gib);
  (void)hipDeviceSynchronize();
  hipDeviceProp_t prop;
  (void)hipGetDeviceProperties(&prop, 0);
  const int cus = prop.multiProcessorCount;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto timed = [&](auto launch) {
    float best = 1e30f;
    for (int it = 0; it < 6; ++it) {
      (void)hipEventRecord(e0, 0);
      launch();
      (void)hipEventRecord(e1, 0);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (it > 0 && ms < best) best = ms;  // the first launch warms
    }
    return best;
  };
  printf("CUs %d; 1 GiB of stores per launch (GB/s = 1e9 B/s), best of 5\n", cus);
  printf("%-10s %-4s %12s %12s %12s %12s\n", "B/lane", "nt", "4 waves/CU", "8 waves/CU", "16 waves/CU", "32 waves/CU");
  auto row = [&](const char* name, bool nt, auto kern) {
    printf("%-10s %-4s", name, nt ? "nt" : "-");
    for (int wpc : {4, 8, 16, 32}) {
      const int grid = cus * wpc / 4;
      const float ms = timed([&] { hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, out, gib); });
      printf(" %12.0f", gib / (ms * 1e-3) / 1e9);
    }
    printf("\n");
  };
  row("4", false, store_k<1, false>);
  row("4", true, store_k<1, true>);
  row("8", false, store_k<2, false>);
  row("8", true, store_k<2, true>);
  row("16", false, store_k<4, false>);
  row("16", true, store_k<4, true>);
  printf("\nencode mix: 1 GiB read + 4 GiB written (8 B per lane), zero arithmetic; combined GB/s and ms\n");
  for (bool nt : {false, true}) {
    printf("%-15s", nt ? "stores nt" : "stores plain");
    for (int wpc : {4, 8, 16, 32}) {
      const int grid = cus * wpc / 4;
      const float ms = timed([&] {
        if (nt)
          hipLaunchKernelGGL(mix_k<true>, dim3(grid), dim3(256), 0, 0, in, out, gib);
        else
          hipLaunchKernelGGL(mix_k<false>, dim3(grid), dim3(256), 0, 0, in, out, gib);
      });
      printf("  %2d w/CU %6.0f GB/s (%.3f ms)", wpc, 5.0 * gib / (ms * 1e-3) / 1e9, ms);
    }
    printf("\n");
  }
  printf("\nencode mix variants (1 GiB read + 4 GiB written), combined GB/s at 4 / 8 / 16 waves per CU\n");
  auto mixrow = [&](const char* name, auto kern) {
    printf("%-28s", name);
    for (int wpc : {4, 8, 16}) {
      const int grid = cus * wpc / 4;
      const float ms = timed([&] { hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, in, out, gib); });
      printf("  %6.0f (%.3f ms)", 5.0 * gib / (ms * 1e-3) / 1e9, ms);
    }
    printf("\n");
  };
  mixrow("st 4 B, 4 loads in flight", mixv_k<4, 4, false>);
  mixrow("st 8 B, 4 loads in flight", mixv_k<8, 4, false>);
  mixrow("st 16 B, 4 loads in flight", mixv_k<16, 4, false>);
  mixrow("st 16 B nt, 4 loads", mixv_k<16, 4, true>);
  mixrow("st 4 B, 8 loads in flight", mixv_k<4, 8, false>);
  mixrow("st 16 B, 8 loads in flight", mixv_k<16, 8, false>);
  mixrow("st 8 B, 1 load", mixv_k<8, 1, false>);
  (void)hipFree(in);
  (void)hipFree(out);
  return 0;
}
