// Microbenchmark: does the SIMD overlap v_perm from one wave with full-rate
// ops (v_and / v_xor) from another?  Waves with even id run only v_perm, odd
// ids only v_and (SPLIT), vs every wave running the 1:1 mix (MIX), vs one
// kind alone.  Not product code.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
constexpr int ITERS = 4096;

#define PERM8 "v_perm_b32 %0, %8, %1, %0\n\tv_perm_b32 %1, %8, %2, %1\n\tv_perm_b32 %2, %8, %3, %2\n\tv_perm_b32 %3, %8, %4, %3\n\tv_perm_b32 %4, %8, %5, %4\n\tv_perm_b32 %5, %8, %6, %5\n\tv_perm_b32 %6, %8, %7, %6\n\tv_perm_b32 %7, %8, %0, %7"
#define AND8 "v_and_b32 %0, 0x07070707, %1\n\tv_and_b32 %1, 0x07070707, %2\n\tv_and_b32 %2, 0x07070707, %3\n\tv_and_b32 %3, 0x07070707, %4\n\tv_and_b32 %4, 0x07070707, %5\n\tv_and_b32 %5, 0x07070707, %6\n\tv_and_b32 %6, 0x07070707, %7\n\tv_and_b32 %7, 0x07070707, %0"
#define MIX8 "v_perm_b32 %0, %8, %1, %0\n\tv_and_b32 %1, 0x07070707, %2\n\tv_perm_b32 %2, %8, %3, %2\n\tv_and_b32 %3, 0x07070707, %4\n\tv_perm_b32 %4, %8, %5, %4\n\tv_and_b32 %5, 0x07070707, %6\n\tv_perm_b32 %6, %8, %7, %6\n\tv_and_b32 %7, 0x07070707, %0"
#define REGS "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s)

template <int MODE>  // 0 perm only, 1 and only, 2 split by wave parity, 3 mix in every wave
__global__ __launch_bounds__(1024) void k(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  const bool odd = (threadIdx.x >> 6) & 1;
  for (int it = 0; it < ITERS; ++it) {
    if (MODE == 0 || (MODE == 2 && !odd)) asm volatile(PERM8 : REGS);
    else if (MODE == 1 || (MODE == 2 && odd)) asm volatile(AND8 : REGS);
    else asm volatile(MIX8 : REGS);
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

template <int MODE>
int run(const char* name, int cus, uint32_t* out) {
  k<MODE><<<cus, 1024>>>(out, 7);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e9;
  for (int r = 0; r < 3; ++r) {
    CK(hipEventRecord(e0));
    k<MODE><<<cus, 1024>>>(out, 7);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = ms < best ? ms : best;
  }
  // 4 waves per SIMD, ITERS * 8 instructions each
  printf("%-28s %.3f ms  %.2f cyc per wave-instruction per SIMD @2.4GHz\n", name, best,
         best * 1e6 * 2.4 / (4.0 * ITERS * 8));
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  uint32_t* out;
  CK(hipMalloc(&out, sizeof(uint32_t) * 1024 * p.multiProcessorCount));
  run<0>("perm only", p.multiProcessorCount, out);
  run<1>("and only", p.multiProcessorCount, out);
  run<2>("split: perm waves + and waves", p.multiProcessorCount, out);
  run<3>("mix 1:1 in every wave", p.multiProcessorCount, out);
  return 0;
}
