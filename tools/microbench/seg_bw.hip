// Microbenchmark: HBM bandwidth of shard-row stores/loads by access shape.
// A "matrix" of R rows x 4096 B (1 GiB).  Shape S: each wave-instruction
// covers 64/S rows x 8S bytes (lanes 8 B each), i.e. S = 64: one 512-B row
// segment; S = 4: 16 rows x 32 B.  Waves take adjacent column segments, so
// a 128-B line is completed by 128/(8S) consecutive waves.  Not product code.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr size_t ROW = 4096;
constexpr size_t ROWS = (size_t(1) << 30) / ROW;

// wave w owns column segment cs = w % (ROW / (8S)) of row block rb = w / (ROW / (8S)); a row block is 64/S rows x ITER
template <int S, bool STORE>
__global__ __launch_bounds__(256) void k_seg(uint8_t* buf, size_t nwaves) {
  constexpr int ROWS_PER_INST = 64 / S;
  constexpr int SEG = 8 * S;
  constexpr int SEGS = ROW / SEG;
  constexpr int ITER = 16;
  const size_t w = (size_t(blockIdx.x) * blockDim.x + threadIdx.x) / 64;
  const uint32_t lane = threadIdx.x & 63;
  if (w >= nwaves) return;
  const size_t cs = w % SEGS, rb = w / SEGS;
  const uint32_t r_in = lane / S, c_in = lane % S;
  uint2 acc = make_uint2(lane, (uint32_t)w);
  for (int i = 0; i < ITER; ++i) {
    const size_t row = (rb * ITER + i) * ROWS_PER_INST + r_in;
    uint2* p = reinterpret_cast<uint2*>(buf + row * ROW + cs * SEG + 8 * c_in);
    if (STORE) {
      *p = acc;
    } else {
      uint2 v = *p;
      acc.x ^= v.x;
      acc.y += v.y;
    }
  }
  if (!STORE && acc.x == 0x12345678u) buf[0] = 1;
}

template <int S, bool STORE>
int run(uint8_t* buf) {
  constexpr int ROWS_PER_INST = 64 / S;
  const size_t nwaves = ROWS / (ROWS_PER_INST * 16) * (ROW / (8 * S));
  const size_t blocks = (nwaves + 3) / 4;
  k_seg<S, STORE><<<blocks, 256>>>(buf, nwaves);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e9;
  for (int r = 0; r < 3; ++r) {
    CK(hipEventRecord(e0));
    k_seg<S, STORE><<<blocks, 256>>>(buf, nwaves);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = ms < best ? ms : best;
  }
  printf("%s %2d rows x %4d B per instruction: %7.1f GB/s\n", STORE ? "store" : "load ", ROWS_PER_INST, 8 * S,
         (double)(size_t(1) << 30) / best / 1e6);
  return 0;
}

// 16 B per lane: each wave-instruction covers 64/S rows x 16S bytes.
template <int S, bool STORE>
__global__ __launch_bounds__(256) void k_seg16(uint8_t* buf, size_t nwaves) {
  constexpr int ROWS_PER_INST = 64 / S;
  constexpr int SEG = 16 * S;
  constexpr int SEGS = ROW / SEG;
  constexpr int ITER = 16;
  const size_t w = (size_t(blockIdx.x) * blockDim.x + threadIdx.x) / 64;
  const uint32_t lane = threadIdx.x & 63;
  if (w >= nwaves) return;
  const size_t cs = w % SEGS, rb = w / SEGS;
  const uint32_t r_in = lane / S, c_in = lane % S;
  uint4 acc = make_uint4(lane, (uint32_t)w, 1, 2);
  for (int i = 0; i < ITER; ++i) {
    const size_t row = (rb * ITER + i) * ROWS_PER_INST + r_in;
    uint4* p = reinterpret_cast<uint4*>(buf + row * ROW + cs * SEG + 16 * c_in);
    if (STORE) {
      *p = acc;
    } else {
      uint4 v = *p;
      acc.x ^= v.x;
      acc.y += v.y;
      acc.z ^= v.z;
      acc.w += v.w;
    }
  }
  if (!STORE && (acc.x ^ acc.z) == 0x12345678u) buf[0] = 1;
}

template <int S, bool STORE>
int run16(uint8_t* buf) {
  constexpr int ROWS_PER_INST = 64 / S;
  const size_t nwaves = ROWS / (ROWS_PER_INST * 16) * (ROW / (16 * S));
  const size_t blocks = (nwaves + 3) / 4;
  k_seg16<S, STORE><<<blocks, 256>>>(buf, nwaves);
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  float best = 1e9;
  for (int r = 0; r < 3; ++r) {
    CK(hipEventRecord(e0));
    k_seg16<S, STORE><<<blocks, 256>>>(buf, nwaves);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    best = ms < best ? ms : best;
  }
  printf("%s %2d rows x %4d B per instruction (16 B/lane): %7.1f GB/s\n", STORE ? "store" : "load ", ROWS_PER_INST,
         16 * S, (double)(size_t(1) << 30) / best / 1e6);
  return 0;
}

int main() {
  uint8_t* buf;
  CK(hipMalloc(&buf, size_t(1) << 30));
  CK(hipMemset(buf, 1, size_t(1) << 30));
  run<64, true>(buf);
  run<32, true>(buf);
  run<16, true>(buf);
  run<8, true>(buf);
  run<4, true>(buf);
  run<2, true>(buf);
  run16<64, true>(buf);
  run16<32, true>(buf);
  run16<16, true>(buf);
  run16<8, true>(buf);
  run16<64, false>(buf);
  run16<32, false>(buf);
  run16<16, false>(buf);
  run<64, false>(buf);
  run<32, false>(buf);
  run<16, false>(buf);
  run<8, false>(buf);
  run<4, false>(buf);
  run<2, false>(buf);
  return 0;
}
