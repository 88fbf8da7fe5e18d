// Microbenchmark (not product code): the quad multiply x ^= c*y followed by the
// butterfly y ^= x, in the asm-statement splits the kernels can use.  hipcc
// pads one wait state after every asm statement whose outputs the next VALU
// touches (cdna_hip_programming.md §5.7 item 2), so the split decides how many
// s_nop run per multiply:
//   product : fast_common.hpp's qmul (shift | and | plane | plane: 4 statements)
//   two     : shift statement + one statement for ands, perms and XOR3s
//   one     : one statement with 32-bit shifts (2 more instructions)
#include <cstdio>

#include "fast_common.hpp"

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
constexpr int ITERS = 8192;

namespace np {
namespace {

__device__ __forceinline__ void qmul_two(uint32_t& xl, uint32_t& xh, uint32_t yl, uint32_t yh, const Mult& m) {
  const uint64_t y = (static_cast<uint64_t>(yh) << 32) | yl;
  uint64_t t3, t6;
  asm volatile("v_lshrrev_b64 %0, 3, %2\n\tv_lshrrev_b64 %1, 6, %2" : "=&v"(t3), "=&v"(t6) : "v"(y));
  uint32_t s0, s1, s2, s3, s4, s5, a, b, c;
  asm volatile(
      "v_and_b32 %[s0], 0x07070707, %[yl]\n\t"
      "v_and_b32 %[s1], 0x07070707, %[t3l]\n\t"
      "v_and_b32 %[s2], 0x03030303, %[t6l]\n\t"
      "v_perm_b32 %[a], %[sa], %[va], %[s0]\n\t"
      "v_and_b32 %[s3], 0x07070707, %[yh]\n\t"
      "v_perm_b32 %[b], %[sb], %[vb], %[s1]\n\t"
      "v_and_b32 %[s4], 0x07070707, %[t3h]\n\t"
      "v_perm_b32 %[c], %[sc], %[sc], %[s2]\n\t"
      "v_and_b32 %[s5], 0x03030303, %[t6h]\n\t"
      "v_bitop3_b32 %[a], %[a], %[b], %[c] bitop3:0x96\n\t"
      "v_perm_b32 %[b], %[sd], %[vc], %[s3]\n\t"
      "v_perm_b32 %[c], %[se], %[vd], %[s4]\n\t"
      "v_bitop3_b32 %[a], %[a], %[b], %[c] bitop3:0x96\n\t"
      "v_perm_b32 %[b], %[sf], %[sf], %[s5]\n\t"
      "v_bitop3_b32 %[xl], %[xl], %[a], %[b] bitop3:0x96\n\t"
      "v_perm_b32 %[a], %[sg], %[ve], %[s0]\n\t"
      "v_perm_b32 %[b], %[sh], %[vf], %[s1]\n\t"
      "v_perm_b32 %[c], %[si], %[si], %[s2]\n\t"
      "v_bitop3_b32 %[a], %[a], %[b], %[c] bitop3:0x96\n\t"
      "v_perm_b32 %[b], %[sj], %[vg], %[s3]\n\t"
      "v_perm_b32 %[c], %[sk], %[vh], %[s4]\n\t"
      "v_bitop3_b32 %[a], %[a], %[b], %[c] bitop3:0x96\n\t"
      "v_perm_b32 %[b], %[sl], %[sl], %[s5]\n\t"
      "v_bitop3_b32 %[xh], %[xh], %[a], %[b] bitop3:0x96"
      : [xl] "+v"(xl), [xh] "+v"(xh), [s0] "=&v"(s0), [s1] "=&v"(s1), [s2] "=&v"(s2), [s3] "=&v"(s3), [s4] "=&v"(s4),
        [s5] "=&v"(s5), [a] "=&v"(a), [b] "=&v"(b), [c] "=&v"(c)
      : [yl] "v"(yl), [yh] "v"(yh), [t3l] "v"(static_cast<uint32_t>(t3)), [t3h] "v"(static_cast<uint32_t>(t3 >> 32)),
        [t6l] "v"(static_cast<uint32_t>(t6)), [t6h] "v"(static_cast<uint32_t>(t6 >> 32)), [va] "v"(m.v[0]),
        [vb] "v"(m.v[1]), [vc] "v"(m.v[2]), [vd] "v"(m.v[3]), [ve] "v"(m.v[4]), [vf] "v"(m.v[5]), [vg] "v"(m.v[6]),
        [vh] "v"(m.v[7]), [sa] "s"(m.s[0]), [sb] "s"(m.s[1]), [sc] "s"(m.s[2]), [sd] "s"(m.s[3]), [se] "s"(m.s[4]),
        [sf] "s"(m.s[5]), [sg] "s"(m.s[6]), [sh] "s"(m.s[7]), [si] "s"(m.s[8]), [sj] "s"(m.s[9]), [sk] "s"(m.s[10]),
        [sl] "s"(m.s[11]));
}

__device__ __forceinline__ void qmul_one(uint32_t& xl, uint32_t& xh, uint32_t yl, uint32_t yh, const Mult& m) {
  uint32_t s0, s1, s2, s3, s4, s5, a, b, c;
  asm volatile(
      "v_and_b32 %[s0], 0x07070707, %[yl]\n\t"
      "v_lshrrev_b32 %[s1], 3, %[yl]\n\t"
      "v_lshrrev_b32 %[s2], 6, %[yl]\n\t"
      "v_and_b32 %[s3], 0x07070707, %[yh]\n\t"
      "v_lshrrev_b32 %[s4], 3, %[yh]\n\t"
      "v_lshrrev_b32 %[s5], 6, %[yh]\n\t"
      "v_and_b32 %[s1], 0x07070707, %[s1]\n\t"
      "v_and_b32 %[s2], 0x03030303, %[s2]\n\t"
      "v_perm_b32 %[a], %[sa], %[va], %[s0]\n\t"
      "v_and_b32 %[s4], 0x07070707, %[s4]\n\t"
      "v_perm_b32 %[b], %[sb], %[vb], %[s1]\n\t"
      "v_and_b32 %[s5], 0x03030303, %[s5]\n\t"
      "v_perm_b32 %[c], %[sc], %[sc], %[s2]\n\t"
      "v_bitop3_b32 %[a], %[a], %[b], %[c] bitop3:0x96\n\t"
      "v_perm_b32 %[b], %[sd], %[vc], %[s3]\n\t"
      "v_perm_b32 %[c], %[se], %[vd], %[s4]\n\t"
      "v_bitop3_b32 %[a], %[a], %[b], %[c] bitop3:0x96\n\t"
      "v_perm_b32 %[b], %[sf], %[sf], %[s5]\n\t"
      "v_bitop3_b32 %[xl], %[xl], %[a], %[b] bitop3:0x96\n\t"
      "v_perm_b32 %[a], %[sg], %[ve], %[s0]\n\t"
      "v_perm_b32 %[b], %[sh], %[vf], %[s1]\n\t"
      "v_perm_b32 %[c], %[si], %[si], %[s2]\n\t"
      "v_bitop3_b32 %[a], %[a], %[b], %[c] bitop3:0x96\n\t"
      "v_perm_b32 %[b], %[sj], %[vg], %[s3]\n\t"
      "v_perm_b32 %[c], %[sk], %[vh], %[s4]\n\t"
      "v_bitop3_b32 %[a], %[a], %[b], %[c] bitop3:0x96\n\t"
      "v_perm_b32 %[b], %[sl], %[sl], %[s5]\n\t"
      "v_bitop3_b32 %[xh], %[xh], %[a], %[b] bitop3:0x96"
      : [xl] "+v"(xl), [xh] "+v"(xh), [s0] "=&v"(s0), [s1] "=&v"(s1), [s2] "=&v"(s2), [s3] "=&v"(s3), [s4] "=&v"(s4),
        [s5] "=&v"(s5), [a] "=&v"(a), [b] "=&v"(b), [c] "=&v"(c)
      : [yl] "v"(yl), [yh] "v"(yh), [va] "v"(m.v[0]), [vb] "v"(m.v[1]), [vc] "v"(m.v[2]), [vd] "v"(m.v[3]),
        [ve] "v"(m.v[4]), [vf] "v"(m.v[5]), [vg] "v"(m.v[6]), [vh] "v"(m.v[7]), [sa] "s"(m.s[0]), [sb] "s"(m.s[1]),
        [sc] "s"(m.s[2]), [sd] "s"(m.s[3]), [se] "s"(m.s[4]), [sf] "s"(m.s[5]), [sg] "s"(m.s[6]), [sh] "s"(m.s[7]),
        [si] "s"(m.s[8]), [sj] "s"(m.s[9]), [sk] "s"(m.s[10]), [sl] "s"(m.s[11]));
}

template <int FORM>
__global__ __launch_bounds__(1024) void k_form(uint32_t* out, uint32_t seed) {
  uint32_t x[8], y[8];
  for (int i = 0; i < 8; ++i) { x[i] = threadIdx.x * seed + i; y[i] = x[i] * 747796405u; }
  Mult m;
  for (int i = 0; i < 12; ++i) m.s[i] = uniform(seed * (i + 11) | 0x01000100u);
  for (int i = 0; i < 8; ++i) m.v[i] = fresh_v(seed * (i + 3));
  for (int it = 0; it < ITERS / 16; ++it) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (FORM == 0) qmul(x[2 * q], x[2 * q + 1], y[2 * q], y[2 * q + 1], m);
      if (FORM == 1) qmul_two(x[2 * q], x[2 * q + 1], y[2 * q], y[2 * q + 1], m);
      if (FORM == 2) qmul_one(x[2 * q], x[2 * q + 1], y[2 * q], y[2 * q + 1], m);
      y[2 * q] ^= x[2 * q];
      y[2 * q + 1] ^= x[2 * q + 1];
    }
  }
  uint32_t acc = 0;
  for (int i = 0; i < 8; ++i) acc ^= x[i] ^ y[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

}  // namespace
}  // namespace np

template <typename F>
int run_q(const char* name, F kern, int cus, uint32_t* out) {
  printf("%-10s", name);
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
  CK(hipMalloc(&out, sizeof(uint32_t) * cus * 2048));
  run_q("product", np::k_form<0>, cus, out);
  run_q("two", np::k_form<1>, cus, out);
  run_q("one", np::k_form<2>, cus, out);
  return 0;
}
