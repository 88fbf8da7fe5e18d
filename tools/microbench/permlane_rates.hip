// Microbenchmark: cycles per wave-instruction of the cross-lane moves a
// register-only layout change would use instead of an LDS exchange
// (the resident decode's HA -> HD step): v_permlane32_swap and
// v_permlane16_swap (gfx950; each swaps half of one VGPR's lanes with half of
// another's), a DPP row rotate and, for scale, v_xor_b32 and v_perm_b32, at
// 1, 2, 4 and 8 waves per SIMD on all CUs.  Not product code.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);         \
      return 1;                                                               \
    }                                                                         \
  } while (0)

constexpr int ITERS = 4096;
constexpr int NR = 16;  // registers per thread (8 independent pairs)

// One step over the NR registers: 8 instructions (one per register pair).
template <int OP>
__device__ __forceinline__ void step(uint32_t (&r)[NR], uint32_t k) {
#pragma unroll
  for (int i = 0; i < NR; i += 2) {
    if constexpr (OP == 0)
      asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(r[i]), "+v"(r[i + 1]));
    else if constexpr (OP == 1)
      asm volatile("v_permlane16_swap_b32 %0, %1" : "+v"(r[i]), "+v"(r[i + 1]));
    else if constexpr (OP == 2)
      asm volatile("v_mov_b32_dpp %0, %1 row_ror:4 row_mask:0xf bank_mask:0xf" : "=v"(r[i]) : "v"(r[i + 1]));
    else if constexpr (OP == 3)
      asm volatile("v_xor_b32 %0, %0, %1" : "+v"(r[i]) : "v"(r[i + 1]));
    else
      asm volatile("v_perm_b32 %0, %1, %0, %2" : "+v"(r[i]) : "v"(r[i + 1]), "v"(k));
  }
}

template <int OP>
__global__ __launch_bounds__(256) void k_lane(uint32_t* out, uint32_t seed) {
  uint32_t r[NR];
#pragma unroll
  for (int i = 0; i < NR; ++i) r[i] = threadIdx.x * seed + 977u * i;
  const uint32_t k = (seed & 0x07070707u) | 0x00010203u;
  for (int it = 0; it < ITERS; ++it) step<OP>(r, k);
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < NR; ++i) acc ^= r[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int OP>
int run(const char* name, int cus, uint32_t* out) {
  printf("%-34s", name);
  for (int w : {1, 2, 4, 8}) {  // 256-thread blocks: one wave per SIMD each
    k_lane<OP><<<cus * w, 256>>>(out, 7);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e9;
    for (int rep = 0; rep < 5; ++rep) {
      CK(hipEventRecord(e0));
      k_lane<OP><<<cus * w, 256>>>(out, 7);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    const double instrs = static_cast<double>(w) * ITERS * (NR / 2);  // wave-instructions per SIMD
    printf(" | %d w/SIMD %5.2f cyc/instr", w, best * 1e-3 * 2.4e9 / instrs);
  }
  printf("\n");
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  uint32_t* out;
  CK(hipMalloc(&out, sizeof(uint32_t) * 256 * 8 * cus));
  printf("cross-lane moves, 8 independent register pairs per thread, %d CUs, cycles at 2.4 GHz per SIMD\n", cus);
  run<0>("v_permlane32_swap (2 VGPRs)", cus, out);
  run<1>("v_permlane16_swap (2 VGPRs)", cus, out);
  run<2>("v_mov_b32_dpp row_ror:4", cus, out);
  run<3>("v_xor_b32", cus, out);
  run<4>("v_perm_b32", cus, out);
  return 0;
}
