// Microbenchmark: issue throughput of single VALU instructions on gfx950 at 4
// and 8 waves per SIMD (8 independent register chains, wall clock over
// ITERS x 8 instructions).  Used to price the GF(2^16) multiply designs
// (DESIGN.md).  Not product code.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
constexpr int ITERS = 8192;
__global__ __launch_bounds__(1024) void k_perm_svv(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_perm_b32 %0, %8, %1, %0\n\tv_perm_b32 %1, %8, %2, %1\n\tv_perm_b32 %2, %8, %3, %2\n\tv_perm_b32 %3, %8, %4, %3\n\tv_perm_b32 %4, %8, %5, %4\n\tv_perm_b32 %5, %8, %6, %5\n\tv_perm_b32 %6, %8, %7, %6\n\tv_perm_b32 %7, %8, %0, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(1024) void k_perm_vvv(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_perm_b32 %0, %2, %1, %0\n\tv_perm_b32 %1, %3, %2, %1\n\tv_perm_b32 %2, %4, %3, %2\n\tv_perm_b32 %3, %5, %4, %3\n\tv_perm_b32 %4, %6, %5, %4\n\tv_perm_b32 %5, %7, %6, %5\n\tv_perm_b32 %6, %0, %7, %6\n\tv_perm_b32 %7, %1, %0, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(1024) void k_bitop3_vvv(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_bitop3_b32 %0, %1, %2, %0 bitop3:0x96\n\tv_bitop3_b32 %1, %2, %3, %1 bitop3:0x96\n\tv_bitop3_b32 %2, %3, %4, %2 bitop3:0x96\n\tv_bitop3_b32 %3, %4, %5, %3 bitop3:0x96\n\tv_bitop3_b32 %4, %5, %6, %4 bitop3:0x96\n\tv_bitop3_b32 %5, %6, %7, %5 bitop3:0x96\n\tv_bitop3_b32 %6, %7, %0, %6 bitop3:0x96\n\tv_bitop3_b32 %7, %0, %1, %7 bitop3:0x96" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(1024) void k_bitop3_svv(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_bitop3_b32 %0, %8, %1, %0 bitop3:0x96\n\tv_bitop3_b32 %1, %8, %2, %1 bitop3:0x96\n\tv_bitop3_b32 %2, %8, %3, %2 bitop3:0x96\n\tv_bitop3_b32 %3, %8, %4, %3 bitop3:0x96\n\tv_bitop3_b32 %4, %8, %5, %4 bitop3:0x96\n\tv_bitop3_b32 %5, %8, %6, %5 bitop3:0x96\n\tv_bitop3_b32 %6, %8, %7, %6 bitop3:0x96\n\tv_bitop3_b32 %7, %8, %0, %7 bitop3:0x96" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(1024) void k_and_lit_vop2(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_and_b32 %0, 0x07070707, %1\n\tv_and_b32 %1, 0x07070707, %2\n\tv_and_b32 %2, 0x07070707, %3\n\tv_and_b32 %3, 0x07070707, %4\n\tv_and_b32 %4, 0x07070707, %5\n\tv_and_b32 %5, 0x07070707, %6\n\tv_and_b32 %6, 0x07070707, %7\n\tv_and_b32 %7, 0x07070707, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(1024) void k_and_sgpr_vop2(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_and_b32_e32 %0, %8, %1\n\tv_and_b32_e32 %1, %8, %2\n\tv_and_b32_e32 %2, %8, %3\n\tv_and_b32_e32 %3, %8, %4\n\tv_and_b32_e32 %4, %8, %5\n\tv_and_b32_e32 %5, %8, %6\n\tv_and_b32_e32 %6, %8, %7\n\tv_and_b32_e32 %7, %8, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(1024) void k_and_sgpr_vop3(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_and_b32_e64 %0, %8, %1\n\tv_and_b32_e64 %1, %8, %2\n\tv_and_b32_e64 %2, %8, %3\n\tv_and_b32_e64 %3, %8, %4\n\tv_and_b32_e64 %4, %8, %5\n\tv_and_b32_e64 %5, %8, %6\n\tv_and_b32_e64 %6, %8, %7\n\tv_and_b32_e64 %7, %8, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(1024) void k_and_vvv_vop3(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_and_b32_e64 %0, %2, %1\n\tv_and_b32_e64 %1, %3, %2\n\tv_and_b32_e64 %2, %4, %3\n\tv_and_b32_e64 %3, %5, %4\n\tv_and_b32_e64 %4, %6, %5\n\tv_and_b32_e64 %5, %7, %6\n\tv_and_b32_e64 %6, %0, %7\n\tv_and_b32_e64 %7, %1, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(1024) void k_xor_vop2(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_xor_b32 %0, %1, %0\n\tv_xor_b32 %1, %2, %1\n\tv_xor_b32 %2, %3, %2\n\tv_xor_b32 %3, %4, %3\n\tv_xor_b32 %4, %5, %4\n\tv_xor_b32 %5, %6, %5\n\tv_xor_b32 %6, %7, %6\n\tv_xor_b32 %7, %0, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(1024) void k_lshr_vop2(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_lshrrev_b32 %0, 3, %1\n\tv_lshrrev_b32 %1, 3, %2\n\tv_lshrrev_b32 %2, 3, %3\n\tv_lshrrev_b32 %3, 3, %4\n\tv_lshrrev_b32 %4, 3, %5\n\tv_lshrrev_b32 %5, 3, %6\n\tv_lshrrev_b32 %6, 3, %7\n\tv_lshrrev_b32 %7, 3, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(1024) void k_lshr_vop3(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_lshrrev_b32_e64 %0, 3, %1\n\tv_lshrrev_b32_e64 %1, 3, %2\n\tv_lshrrev_b32_e64 %2, 3, %3\n\tv_lshrrev_b32_e64 %3, 3, %4\n\tv_lshrrev_b32_e64 %4, 3, %5\n\tv_lshrrev_b32_e64 %5, 3, %6\n\tv_lshrrev_b32_e64 %6, 3, %7\n\tv_lshrrev_b32_e64 %7, 3, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(1024) void k_and_or(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_and_or_b32 %0, %1, %2, %0\n\tv_and_or_b32 %1, %2, %3, %1\n\tv_and_or_b32 %2, %3, %4, %2\n\tv_and_or_b32 %3, %4, %5, %3\n\tv_and_or_b32 %4, %5, %6, %4\n\tv_and_or_b32 %5, %6, %7, %5\n\tv_and_or_b32 %6, %7, %0, %6\n\tv_and_or_b32 %7, %0, %1, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(1024) void k_bfi(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_bfi_b32 %0, %1, %2, %0\n\tv_bfi_b32 %1, %2, %3, %1\n\tv_bfi_b32 %2, %3, %4, %2\n\tv_bfi_b32 %3, %4, %5, %3\n\tv_bfi_b32 %4, %5, %6, %4\n\tv_bfi_b32 %5, %6, %7, %5\n\tv_bfi_b32 %6, %7, %0, %6\n\tv_bfi_b32 %7, %0, %1, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(1024) void k_lshl_or(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_lshl_or_b32 %0, %1, 3, %0\n\tv_lshl_or_b32 %1, %2, 3, %1\n\tv_lshl_or_b32 %2, %3, 3, %2\n\tv_lshl_or_b32 %3, %4, 3, %3\n\tv_lshl_or_b32 %4, %5, 3, %4\n\tv_lshl_or_b32 %5, %6, 3, %5\n\tv_lshl_or_b32 %6, %7, 3, %6\n\tv_lshl_or_b32 %7, %0, 3, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(1024) void k_cndmask_vcc(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_cndmask_b32 %0, %1, %2, vcc\n\tv_cndmask_b32 %1, %2, %3, vcc\n\tv_cndmask_b32 %2, %3, %4, vcc\n\tv_cndmask_b32 %3, %4, %5, vcc\n\tv_cndmask_b32 %4, %5, %6, vcc\n\tv_cndmask_b32 %5, %6, %7, vcc\n\tv_cndmask_b32 %6, %7, %0, vcc\n\tv_cndmask_b32 %7, %0, %1, vcc" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(1024) void k_mov_dpp(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %1, %2 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %2, %3 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %3, %4 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %4, %5 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %5, %6 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %6, %7 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %7, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(1024) void k_alignbit(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_alignbit_b32 %0, %1, %2, 3\n\tv_alignbit_b32 %1, %2, %3, 3\n\tv_alignbit_b32 %2, %3, %4, 3\n\tv_alignbit_b32 %3, %4, %5, 3\n\tv_alignbit_b32 %4, %5, %6, 3\n\tv_alignbit_b32 %5, %6, %7, 3\n\tv_alignbit_b32 %6, %7, %0, 3\n\tv_alignbit_b32 %7, %0, %1, 3" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(1024) void k_bfe(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_bfe_u32 %0, %1, 3, 3\n\tv_bfe_u32 %1, %2, 3, 3\n\tv_bfe_u32 %2, %3, 3, 3\n\tv_bfe_u32 %3, %4, 3, 3\n\tv_bfe_u32 %4, %5, 3, 3\n\tv_bfe_u32 %5, %6, 3, 3\n\tv_bfe_u32 %6, %7, 3, 3\n\tv_bfe_u32 %7, %0, 3, 3" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(1024) void k_mov_b32(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_mov_b32 %0, %1\n\tv_mov_b32 %1, %2\n\tv_mov_b32 %2, %3\n\tv_mov_b32 %3, %4\n\tv_mov_b32 %4, %5\n\tv_mov_b32 %5, %6\n\tv_mov_b32 %6, %7\n\tv_mov_b32 %7, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ __launch_bounds__(1024) void k_mix_perm_and_1_1(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_perm_b32 %0, %8, %1, %0\n\tv_and_b32 %1, 0x07070707, %2\n\tv_perm_b32 %2, %8, %3, %2\n\tv_and_b32 %3, 0x07070707, %4\n\tv_perm_b32 %4, %8, %5, %4\n\tv_and_b32 %5, 0x07070707, %6\n\tv_perm_b32 %6, %8, %7, %6\n\tv_and_b32 %7, 0x07070707, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(1024) void k_mix_perm_and_1_2(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_perm_b32 %0, %8, %1, %0\n\tv_and_b32 %1, 0x07070707, %2\n\tv_xor_b32 %2, %3, %2\n\tv_perm_b32 %3, %8, %4, %3\n\tv_and_b32 %4, 0x07070707, %5\n\tv_xor_b32 %5, %6, %5\n\tv_perm_b32 %6, %8, %7, %6\n\tv_and_b32 %7, 0x07070707, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(1024) void k_mix_perm_bitop3_1_1(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_perm_b32 %0, %8, %1, %0\n\tv_bitop3_b32 %1, %2, %3, %1 bitop3:0x96\n\tv_perm_b32 %2, %8, %3, %2\n\tv_bitop3_b32 %3, %4, %5, %3 bitop3:0x96\n\tv_perm_b32 %4, %8, %5, %4\n\tv_bitop3_b32 %5, %6, %7, %5 bitop3:0x96\n\tv_perm_b32 %6, %8, %7, %6\n\tv_bitop3_b32 %7, %0, %1, %7 bitop3:0x96" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(1024) void k_mix_permvvv_and_1_1(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_perm_b32 %0, %2, %1, %0\n\tv_and_b32 %1, 0x07070707, %2\n\tv_perm_b32 %2, %4, %3, %2\n\tv_and_b32 %3, 0x07070707, %4\n\tv_perm_b32 %4, %6, %5, %4\n\tv_and_b32 %5, 0x07070707, %6\n\tv_perm_b32 %6, %0, %7, %6\n\tv_and_b32 %7, 0x07070707, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(1024) void k_mix_and_xor(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_and_b32 %0, 0x07070707, %1\n\tv_xor_b32 %1, %2, %1\n\tv_and_b32 %2, 0x07070707, %3\n\tv_xor_b32 %3, %4, %3\n\tv_and_b32 %4, 0x07070707, %5\n\tv_xor_b32 %5, %6, %5\n\tv_and_b32 %6, 0x07070707, %7\n\tv_xor_b32 %7, %0, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__device__ __forceinline__ void qm(uint32_t& xl, uint32_t& xh, uint32_t yl, uint32_t yh, uint32_t va, uint32_t vb,
                                   uint32_t vc, uint32_t vd, uint32_t ve, uint32_t vf, uint32_t vg, uint32_t vh,
                                   uint32_t s0, uint32_t s1, uint32_t s2) {
  uint32_t a, b, c, d, e, f, t0, t1, t2;
  asm volatile(
      "v_and_b32 %[a], 0x07070707, %[yl]\n\tv_lshrrev_b32 %[b], 3, %[yl]\n\tv_lshrrev_b32 %[c], 6, %[yl]\n\t"
      "v_and_b32 %[d], 0x07070707, %[yh]\n\tv_lshrrev_b32 %[e], 3, %[yh]\n\tv_lshrrev_b32 %[f], 6, %[yh]\n\t"
      "v_and_b32 %[b], 0x07070707, %[b]\n\tv_and_b32 %[c], 0x03030303, %[c]\n\t"
      "v_and_b32 %[e], 0x07070707, %[e]\n\tv_and_b32 %[f], 0x03030303, %[f]\n\t"
      "v_perm_b32 %[t0], %[s0], %[va], %[a]\n\tv_perm_b32 %[t1], %[s1], %[vb], %[b]\n\tv_perm_b32 %[t2], %[s2], %[s2], %[c]\n\t"
      "v_bitop3_b32 %[t0], %[t0], %[t1], %[t2] bitop3:0x96\n\t"
      "v_perm_b32 %[t1], %[s0], %[vc], %[d]\n\tv_perm_b32 %[t2], %[s1], %[vd], %[e]\n\t"
      "v_bitop3_b32 %[t0], %[t0], %[t1], %[t2] bitop3:0x96\n\t"
      "v_perm_b32 %[t1], %[s2], %[s2], %[f]\n\tv_bitop3_b32 %[xl], %[xl], %[t0], %[t1] bitop3:0x96\n\t"
      "v_perm_b32 %[t0], %[s0], %[ve], %[a]\n\tv_perm_b32 %[t1], %[s1], %[vf], %[b]\n\tv_perm_b32 %[t2], %[s2], %[s2], %[c]\n\t"
      "v_bitop3_b32 %[t0], %[t0], %[t1], %[t2] bitop3:0x96\n\t"
      "v_perm_b32 %[t1], %[s0], %[vg], %[d]\n\tv_perm_b32 %[t2], %[s1], %[vh], %[e]\n\t"
      "v_bitop3_b32 %[t0], %[t0], %[t1], %[t2] bitop3:0x96\n\t"
      "v_perm_b32 %[t1], %[s2], %[s2], %[f]\n\tv_bitop3_b32 %[xh], %[xh], %[t0], %[t1] bitop3:0x96"
      : [xl] "+v"(xl), [xh] "+v"(xh), [a] "=&v"(a), [b] "=&v"(b), [c] "=&v"(c), [d] "=&v"(d), [e] "=&v"(e),
        [f] "=&v"(f), [t0] "=&v"(t0), [t1] "=&v"(t1), [t2] "=&v"(t2)
      : [yl] "v"(yl), [yh] "v"(yh), [va] "v"(va), [vb] "v"(vb), [vc] "v"(vc), [vd] "v"(vd), [ve] "v"(ve), [vf] "v"(vf),
        [vg] "v"(vg), [vh] "v"(vh), [s0] "s"(s0), [s1] "s"(s1), [s2] "s"(s2));
}
// 4 independent quads per iteration, each x ^= c * y then y ^= x (the butterfly)
__global__ __launch_bounds__(1024) void k_qmul(uint32_t* out, uint32_t seed) {
  uint32_t x[8], y[8], v[8];
  for (int i = 0; i < 8; ++i) { x[i] = threadIdx.x * seed + i; y[i] = x[i] * 747796405u; v[i] = seed * (i + 3); }
  const uint32_t s0 = seed | 0x01020304u, s1 = seed ^ 0x05060708u, s2 = seed + 7;
  for (int it = 0; it < ITERS / 16; ++it) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      qm(x[2 * q], x[2 * q + 1], y[2 * q], y[2 * q + 1], v[0], v[1], v[2], v[3], v[4], v[5], v[6], v[7], s0, s1, s2);
      y[2 * q] ^= x[2 * q];
      y[2 * q + 1] ^= x[2 * q + 1];
    }
  }
  uint32_t acc = 0;
  for (int i = 0; i < 8; ++i) acc ^= x[i] ^ y[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

__global__ __launch_bounds__(1024) void k_blk_pppp_aaaa(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_perm_b32 %0, %8, %1, %0\n\tv_perm_b32 %1, %8, %2, %1\n\tv_perm_b32 %2, %8, %3, %2\n\tv_perm_b32 %3, %8, %4, %3\n\tv_and_b32 %4, 0x07070707, %5\n\tv_and_b32 %5, 0x07070707, %6\n\tv_and_b32 %6, 0x07070707, %7\n\tv_and_b32 %7, 0x07070707, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(1024) void k_blk_pp_aa(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_perm_b32 %0, %8, %1, %0\n\tv_perm_b32 %1, %8, %2, %1\n\tv_and_b32 %2, 0x07070707, %3\n\tv_and_b32 %3, 0x07070707, %4\n\tv_perm_b32 %4, %8, %5, %4\n\tv_perm_b32 %5, %8, %6, %5\n\tv_and_b32 %6, 0x07070707, %7\n\tv_and_b32 %7, 0x07070707, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(1024) void k_mix_perm_xorvop2(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_perm_b32 %0, %8, %1, %0\n\tv_xor_b32 %1, %2, %1\n\tv_perm_b32 %2, %8, %3, %2\n\tv_xor_b32 %3, %4, %3\n\tv_perm_b32 %4, %8, %5, %4\n\tv_xor_b32 %5, %6, %5\n\tv_perm_b32 %6, %8, %7, %6\n\tv_xor_b32 %7, %0, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(1024) void k_mix_bfi_and(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_bfi_b32 %0, %1, %2, %0\n\tv_and_b32 %1, 0x07070707, %2\n\tv_bfi_b32 %2, %3, %4, %2\n\tv_and_b32 %3, 0x07070707, %4\n\tv_bfi_b32 %4, %5, %6, %4\n\tv_and_b32 %5, 0x07070707, %6\n\tv_bfi_b32 %6, %7, %0, %6\n\tv_and_b32 %7, 0x07070707, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(1024) void k_mix_bitop3s_and(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_bitop3_b32 %0, %8, %1, %0 bitop3:0x96\n\tv_and_b32 %1, 0x07070707, %2\n\tv_bitop3_b32 %2, %8, %3, %2 bitop3:0x96\n\tv_and_b32 %3, 0x07070707, %4\n\tv_bitop3_b32 %4, %8, %5, %4 bitop3:0x96\n\tv_and_b32 %5, 0x07070707, %6\n\tv_bitop3_b32 %6, %8, %7, %6 bitop3:0x96\n\tv_and_b32 %7, 0x07070707, %0" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

__global__ __launch_bounds__(1024) void k_perm4_salu4(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_perm_b32 %0, %8, %1, %0\n\ts_add_u32 s100, s100, 1\n\tv_perm_b32 %1, %8, %2, %1\n\ts_add_u32 s100, s100, 1\n\tv_perm_b32 %2, %8, %3, %2\n\ts_add_u32 s100, s100, 1\n\tv_perm_b32 %3, %8, %4, %3\n\ts_add_u32 s100, s100, 1" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc", "s100", "scc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(1024) void k_perm4_salu2(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_perm_b32 %0, %8, %1, %0\n\tv_perm_b32 %1, %8, %2, %1\n\ts_add_u32 s100, s100, 1\n\tv_perm_b32 %2, %8, %3, %2\n\tv_perm_b32 %3, %8, %4, %3\n\ts_add_u32 s100, s100, 1\n\tv_perm_b32 %4, %8, %5, %4\n\tv_perm_b32 %5, %8, %6, %5\n\ts_add_u32 s100, s100, 1\n\tv_perm_b32 %6, %8, %7, %6\n\tv_perm_b32 %7, %8, %0, %7\n\ts_add_u32 s100, s100, 1" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc", "s100", "scc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}
__global__ __launch_bounds__(1024) void k_perm_only_ref(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x * seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t s = seed | 0x01020304u;
  for (int it = 0; it < ITERS; ++it)
    asm volatile("v_perm_b32 %0, %8, %1, %0\n\tv_perm_b32 %1, %8, %2, %1\n\tv_perm_b32 %2, %8, %3, %2\n\tv_perm_b32 %3, %8, %4, %3\n\tv_perm_b32 %4, %8, %5, %4\n\tv_perm_b32 %5, %8, %6, %5\n\tv_perm_b32 %6, %8, %7, %6\n\tv_perm_b32 %7, %8, %0, %7" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "s"(s) : "vcc", "s100", "scc");
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

template <typename F>
int run(const char* name, F kern, int cus, uint32_t* out) {
  printf("%-16s", name);
  for (int per_cu : {1, 2}) {  // 1024-thread blocks: 4 or 8 waves per SIMD
    kern<<<cus * per_cu, 1024>>>(out, 7);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e9;
    for (int r = 0; r < 3; ++r) {
      CK(hipEventRecord(e0));
      kern<<<cus * per_cu, 1024>>>(out, 7);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    const double per_simd = 4.0 * per_cu * ITERS * 8;  // wave-instructions per SIMD
    printf("   %d w/SIMD: %.2f cyc@2.4GHz", 4 * per_cu, best * 1e6 / per_simd * 2.4);
  }
  printf("\n");
  return 0;
}

template <typename F>
int run_q(const char* name, F kern, int cus, uint32_t* out) {
  printf("%-28s", name);
  for (int per_cu : {1, 2}) {
    kern<<<cus * per_cu, 1024>>>(out, 7);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e9;
    for (int r = 0; r < 3; ++r) {
      CK(hipEventRecord(e0));
      kern<<<cus * per_cu, 1024>>>(out, 7);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    const double quads = 4.0 * per_cu * (ITERS / 16) * 4;  // quad-multiplies per SIMD
    printf("   %d w/SIMD: %.1f cyc/quad-mul@2.4GHz", 4 * per_cu, best * 1e6 / quads * 2.4);
  }
  printf("\n");
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  uint32_t* out;
  CK(hipMalloc(&out, sizeof(uint32_t) * 2048 * cus));
  run("perm_svv", k_perm_svv, cus, out);
  run("perm_vvv", k_perm_vvv, cus, out);
  run("bitop3_vvv", k_bitop3_vvv, cus, out);
  run("bitop3_svv", k_bitop3_svv, cus, out);
  run("and_lit_vop2", k_and_lit_vop2, cus, out);
  run("and_sgpr_vop2", k_and_sgpr_vop2, cus, out);
  run("and_sgpr_vop3", k_and_sgpr_vop3, cus, out);
  run("and_vvv_vop3", k_and_vvv_vop3, cus, out);
  run("xor_vop2", k_xor_vop2, cus, out);
  run("lshr_vop2", k_lshr_vop2, cus, out);
  run("lshr_vop3", k_lshr_vop3, cus, out);
  run("and_or", k_and_or, cus, out);
  run("bfi", k_bfi, cus, out);
  run("lshl_or", k_lshl_or, cus, out);
  run("cndmask_vcc", k_cndmask_vcc, cus, out);
  run("mov_dpp", k_mov_dpp, cus, out);
  run("alignbit", k_alignbit, cus, out);
  run("bfe", k_bfe, cus, out);
  run("mov_b32", k_mov_b32, cus, out);
  run("mix_perm_and_1_1", k_mix_perm_and_1_1, cus, out);
  run("mix_perm_and_1_2", k_mix_perm_and_1_2, cus, out);
  run("mix_perm_bitop3_1_1", k_mix_perm_bitop3_1_1, cus, out);
  run("mix_permvvv_and_1_1", k_mix_permvvv_and_1_1, cus, out);
  run("mix_and_xor", k_mix_and_xor, cus, out);
  run_q("qmul (28+2 instr per quad)", k_qmul, cus, out);
  run("blk_pppp_aaaa", k_blk_pppp_aaaa, cus, out);
  run("blk_pp_aa", k_blk_pp_aa, cus, out);
  run("mix_perm_xorvop2", k_mix_perm_xorvop2, cus, out);
  run("mix_bfi_and", k_mix_bfi_and, cus, out);
  run("mix_bitop3s_and", k_mix_bitop3s_and, cus, out);
  run("perm4_salu4 (4 valu/iter)", k_perm4_salu4, cus, out);
  run("perm4_salu2 (8 valu/iter)", k_perm4_salu2, cus, out);
  run("perm_only_ref (8 valu/iter)", k_perm_only_ref, cus, out);
  return 0;
}
