// Microbenchmark: cycles per quad-butterfly of the GF(2^16) v_perm multiply
// sequences the codec kernels ship (fast_common.hpp qmul_sub / qmul, the
// IFFT butterfly y ^= x; x ^= c * y on four byte-planar symbols), and
// variants of them, at 1, 2, 4 and 8 waves per SIMD.  Every thread runs 4
// independent butterflies per iteration (a level of a transform gives 8).
// Prints wall-clock cycles (at 2.4 GHz) per butterfly per SIMD and per
// instruction.  Not product code (DESIGN.md §5 prices the kernels with it).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e = (x);                                                               \
    if (e != hipSuccess) {                                                            \
      printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);                 \
      return 1;                                                                       \
    }                                                                                 \
  } while (0)

constexpr int ITERS = 2048;
constexpr int NB = 4;  // butterflies per iteration and thread

// Selectors as the product (fast_common.hpp selectors): two 64-bit shifts, six ands.
#define SEL64                                                                                         \
  "v_lshrrev_b64 %[t34], 3, %[y01]\n\t"                                                              \
  "v_lshrrev_b64 %[t56], 6, %[y01]\n\t"                                                              \
  "v_and_b32 %[s0], 0x07070707, %[yl]\n\t"                                                           \
  "v_and_b32 %[s3], 0x07070707, %[yh]\n\t"                                                           \
  "v_and_b32 %[s1], 0x07070707, %[t3]\n\t"                                                           \
  "v_and_b32 %[s4], 0x07070707, %[t4]\n\t"                                                           \
  "v_and_b32 %[s2], 0x03030303, %[t5]\n\t"                                                           \
  "v_and_b32 %[s5], 0x03030303, %[t6]\n\t"
// Selectors with 32-bit shifts (fast_common.hpp NP_SEL_ASM).
#define SEL32                                                                                         \
  "v_and_b32 %[s0], 0x07070707, %[yl]\n\t"                                                           \
  "v_lshrrev_b32 %[s1], 3, %[yl]\n\t"                                                                \
  "v_lshrrev_b32 %[s2], 6, %[yl]\n\t"                                                                \
  "v_and_b32 %[s3], 0x07070707, %[yh]\n\t"                                                           \
  "v_lshrrev_b32 %[s4], 3, %[yh]\n\t"                                                                \
  "v_lshrrev_b32 %[s5], 6, %[yh]\n\t"                                                                \
  "v_and_b32 %[s1], 0x07070707, %[s1]\n\t"                                                           \
  "v_and_b32 %[s2], 0x03030303, %[s2]\n\t"                                                           \
  "v_and_b32 %[s4], 0x07070707, %[s4]\n\t"                                                           \
  "v_and_b32 %[s5], 0x03030303, %[s5]\n\t"
// Subfield lookups of both planes, SGPR + VGPR table halves (qplane_sub).
#define SUBLOOK(TA, TB, TC)                                                                           \
  "v_perm_b32 %[p0], " TA ", %[va], %[s0]\n\t"                                                       \
  "v_perm_b32 %[p1], " TB ", %[vb], %[s1]\n\t"                                                       \
  "v_perm_b32 %[p2], " TC ", " TC ", %[s2]\n\t"                                                      \
  "v_bitop3_b32 %[xl], %[xl], %[p0], %[p1] bitop3:0x96\n\t"                                          \
  "v_xor_b32 %[xl], %[xl], %[p2]\n\t"                                                                \
  "v_perm_b32 %[p0], " TA ", %[va], %[s3]\n\t"                                                       \
  "v_perm_b32 %[p1], " TB ", %[vb], %[s4]\n\t"                                                       \
  "v_perm_b32 %[p2], " TC ", " TC ", %[s5]\n\t"                                                      \
  "v_bitop3_b32 %[xh], %[xh], %[p0], %[p1] bitop3:0x96\n\t"                                          \
  "v_xor_b32 %[xh], %[xh], %[p2]\n\t"
#define YXOR "v_xor_b32 %[yl], %[yl], %[xl]\n\tv_xor_b32 %[yh], %[yh], %[xh]\n\t"

#define OUTS                                                                                          \
  [xl] "+v"(xl), [xh] "+v"(xh), [yl] "+v"(y01.x), [yh] "+v"(y01.y), [s0] "=&v"(s0), [s1] "=&v"(s1),  \
      [s2] "=&v"(s2), [s3] "=&v"(s3), [s4] "=&v"(s4), [s5] "=&v"(s5), [p0] "=&v"(p0), [p1] "=&v"(p1), \
      [p2] "=&v"(p2)

struct U2 {
  uint32_t x, y;
};

// VARIANT: 0 product (SEL64, SGPR tables), 1 SEL32, 2 VGPR-only tables,
// 3 full 16x16 multiply (12 lookups), 4 perms and xors only (no selectors:
// the floor of the lookups), 5 selectors and xors only (no perms).
template <int VARIANT>
__device__ __forceinline__ void bfly(uint32_t& xl, uint32_t& xh, uint32_t& yl, uint32_t& yh, uint32_t va, uint32_t vb,
                                     uint32_t vc, uint32_t vd, uint32_t sa, uint32_t sb, uint32_t sc) {
  uint32_t s0, s1, s2, s3, s4, s5, p0, p1, p2;
  uint64_t t34, t56;
  U2 y01{yl, yh};
  (void)t34, (void)t56;
  if constexpr (VARIANT == 0) {  // as fast_common.hpp: y ^= x, selectors(), qplane_sub x2
    yl ^= xl;
    yh ^= xh;
    const uint64_t y = (static_cast<uint64_t>(yh) << 32) | yl;
    asm volatile("v_lshrrev_b64 %0, 3, %2\n\tv_lshrrev_b64 %1, 6, %2" : "=&v"(t34), "=&v"(t56) : "v"(y));
    asm volatile(
        "v_and_b32 %[s0], 0x07070707, %[yl]\n\t"
        "v_and_b32 %[s3], 0x07070707, %[yh]\n\t"
        "v_and_b32 %[s1], 0x07070707, %[t3]\n\t"
        "v_and_b32 %[s4], 0x07070707, %[t4]\n\t"
        "v_and_b32 %[s2], 0x03030303, %[t5]\n\t"
        "v_and_b32 %[s5], 0x03030303, %[t6]\n\t" SUBLOOK("%[sa]", "%[sb]", "%[sc]")
        : [xl] "+v"(xl), [xh] "+v"(xh), [s0] "=&v"(s0), [s1] "=&v"(s1), [s2] "=&v"(s2), [s3] "=&v"(s3),
          [s4] "=&v"(s4), [s5] "=&v"(s5), [p0] "=&v"(p0), [p1] "=&v"(p1), [p2] "=&v"(p2)
        : [yl] "v"(static_cast<uint32_t>(y)), [yh] "v"(static_cast<uint32_t>(y >> 32)),
          [t3] "v"(static_cast<uint32_t>(t34)), [t4] "v"(static_cast<uint32_t>(t34 >> 32)),
          [t5] "v"(static_cast<uint32_t>(t56)), [t6] "v"(static_cast<uint32_t>(t56 >> 32)), [va] "v"(va),
          [vb] "v"(vb), [sa] "s"(sa), [sb] "s"(sb), [sc] "s"(sc));
    return;
  }
  if constexpr (VARIANT == 1) {
    asm volatile(YXOR SEL32 SUBLOOK("%[sa]", "%[sb]", "%[sc]")
                 : OUTS
                 : [va] "v"(va), [vb] "v"(vb), [sa] "s"(sa), [sb] "s"(sb), [sc] "s"(sc));
  } else if constexpr (VARIANT == 2) {
    asm volatile(YXOR SEL32 SUBLOOK("%[vc]", "%[vd]", "%[vd]")
                 : OUTS
                 : [va] "v"(va), [vb] "v"(vb), [vc] "v"(vc), [vd] "v"(vd));
  } else if constexpr (VARIANT == 3) {
    asm volatile(YXOR SEL32 SUBLOOK("%[sa]", "%[sb]", "%[sc]") SUBLOOK("%[sc]", "%[sa]", "%[sb]")
                 : OUTS
                 : [va] "v"(va), [vb] "v"(vb), [sa] "s"(sa), [sb] "s"(sb), [sc] "s"(sc));
  } else if constexpr (VARIANT == 4) {
    s0 = yl, s1 = yh, s2 = yl ^ 1u, s3 = yh, s4 = yl, s5 = yh;
    asm volatile(YXOR SUBLOOK("%[sa]", "%[sb]", "%[sc]")
                 : [xl] "+v"(xl), [xh] "+v"(xh), [yl] "+v"(y01.x), [yh] "+v"(y01.y), [p0] "=&v"(p0), [p1] "=&v"(p1),
                   [p2] "=&v"(p2)
                 : [s0] "v"(s0), [s1] "v"(s1), [s2] "v"(s2), [s3] "v"(s3), [s4] "v"(s4), [s5] "v"(s5), [va] "v"(va),
                   [vb] "v"(vb), [sa] "s"(sa), [sb] "s"(sb), [sc] "s"(sc));
  } else {
    asm volatile(YXOR SEL32
                 "v_bitop3_b32 %[xl], %[xl], %[s0], %[s1] bitop3:0x96\n\t"
                 "v_xor_b32 %[xl], %[xl], %[s2]\n\t"
                 "v_bitop3_b32 %[xh], %[xh], %[s3], %[s4] bitop3:0x96\n\t"
                 "v_xor_b32 %[xh], %[xh], %[s5]\n\t"
                 : OUTS
                 : [va] "v"(va), [vb] "v"(vb), [sa] "s"(sa), [sb] "s"(sb), [sc] "s"(sc));
  }
  yl = y01.x;
  yh = y01.y;
}

template <int VARIANT>
__global__ __launch_bounds__(256) void k_bfly(uint32_t* out, uint32_t seed) {
  uint32_t xl[NB], xh[NB], yl[NB], yh[NB];
  for (int i = 0; i < NB; ++i) {
    xl[i] = threadIdx.x * seed + i;
    xh[i] = xl[i] * 747796405u;
    yl[i] = xh[i] ^ seed;
    yh[i] = yl[i] + 17u * i;
  }
  const uint32_t va = seed * 3u, vb = seed * 5u, vc = seed * 7u, vd = seed * 11u;
  const uint32_t sa = __builtin_amdgcn_readfirstlane(seed | 0x01020304u),
                 sb = __builtin_amdgcn_readfirstlane(seed ^ 0x05060708u), sc = __builtin_amdgcn_readfirstlane(seed + 7u);
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int i = 0; i < NB; ++i) bfly<VARIANT>(xl[i], xh[i], yl[i], yh[i], va, vb, vc, vd, sa, sb, sc);
  }
  uint32_t acc = 0;
  for (int i = 0; i < NB; ++i) acc ^= xl[i] ^ xh[i] ^ yl[i] ^ yh[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

template <int VARIANT>
int run(const char* name, int instrs, int cus, uint32_t* out) {
  printf("%-44s %2d instr", name, instrs);
  for (int w : {1, 2, 4, 8}) {  // 256-thread blocks: one wave per SIMD each
    k_bfly<VARIANT><<<cus * w, 256>>>(out, 7);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best = 1e9;
    for (int r = 0; r < 5; ++r) {
      CK(hipEventRecord(e0));
      k_bfly<VARIANT><<<cus * w, 256>>>(out, 7);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
    }
    const double bf = static_cast<double>(w) * ITERS * NB;  // butterflies per SIMD
    const double cyc = best * 1e-3 * 2.4e9 / bf;
    printf(" | %d w/SIMD %6.1f cyc/bfly %4.2f cyc/instr", w, cyc, cyc / instrs);
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
  printf("quad butterfly y ^= x; x ^= c*y (4 symbols), %d CUs, cycles at 2.4 GHz per SIMD\n", cus);
  run<0>("subfield, product (sel b64, SGPR tables)", 20, cus, out);
  run<1>("subfield, 32-bit shift selectors", 22, cus, out);
  run<2>("subfield, VGPR-only tables", 22, cus, out);
  run<3>("full 16x16 (12 lookups)", 32, cus, out);
  run<4>("lookups + xors only (no selectors)", 12, cus, out);
  run<5>("selectors + xors only (no lookups)", 16, cus, out);
  return 0;
}
