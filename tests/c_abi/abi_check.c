/*
 * C-language check of the drop-in boundary (include/novelpoly.h): built with
 * `gcc -std=c99 -pedantic -Wall -Wextra -Werror` against the header and linked
 * to libnovelpoly_hip.so, the way the reference's bindgen route
 * (/root/reference/reed-solomon-novelpoly/build.rs:18-41, src/cxx.rs:13-31)
 * would bind it -- C types, not ctypes.  tests/test_c_abi.py builds and runs
 * it on the GPU and compares the digests it prints with
 * tests/golden/digests.json (generated from the reference C build).
 *
 * Workload: BASELINE config 2 (n_wanted 256, k_wanted 86 -> n 256, k 64),
 * payload 0 of the synthetic generator (novelpoly_amd/synth.py: splitmix64,
 * seed 0x5EED0000), 192 erasures by partial Fisher-Yates (seed 0xE7A50000).
 * Prints one line per entry point: "<name> <sha256 hex>".
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "novelpoly.h"

/* ---- SHA-256 (FIPS 180-4), for the digests ---- */
typedef struct {
  uint32_t h[8];
  uint64_t len;
  uint8_t buf[64];
  size_t fill;
} sha256_t;

static const uint32_t K256[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

static uint32_t ror(uint32_t x, int r) { return (x >> r) | (x << (32 - r)); }

static void sha_block(sha256_t* s, const uint8_t* p) {
  uint32_t w[64], a, b, c, d, e, f, g, h;
  int i;
  for (i = 0; i < 16; ++i)
    w[i] = ((uint32_t)p[4 * i] << 24) | ((uint32_t)p[4 * i + 1] << 16) | ((uint32_t)p[4 * i + 2] << 8) | p[4 * i + 3];
  for (i = 16; i < 64; ++i) {
    const uint32_t s0 = ror(w[i - 15], 7) ^ ror(w[i - 15], 18) ^ (w[i - 15] >> 3);
    const uint32_t s1 = ror(w[i - 2], 17) ^ ror(w[i - 2], 19) ^ (w[i - 2] >> 10);
    w[i] = w[i - 16] + s0 + w[i - 7] + s1;
  }
  a = s->h[0], b = s->h[1], c = s->h[2], d = s->h[3], e = s->h[4], f = s->h[5], g = s->h[6], h = s->h[7];
  for (i = 0; i < 64; ++i) {
    const uint32_t t1 = h + (ror(e, 6) ^ ror(e, 11) ^ ror(e, 25)) + ((e & f) ^ (~e & g)) + K256[i] + w[i];
    const uint32_t t2 = (ror(a, 2) ^ ror(a, 13) ^ ror(a, 22)) + ((a & b) ^ (a & c) ^ (b & c));
    h = g, g = f, f = e, e = d + t1, d = c, c = b, b = a, a = t1 + t2;
  }
  s->h[0] += a, s->h[1] += b, s->h[2] += c, s->h[3] += d, s->h[4] += e, s->h[5] += f, s->h[6] += g, s->h[7] += h;
}

static void sha_init(sha256_t* s) {
  static const uint32_t h0[8] = {0x6a09e667, 0xbb67ae85, 0x3c6ef372, 0xa54ff53a,
                                 0x510e527f, 0x9b05688c, 0x1f83d9ab, 0x5be0cd19};
  memcpy(s->h, h0, sizeof h0);
  s->len = 0;
  s->fill = 0;
}

static void sha_update(sha256_t* s, const uint8_t* p, size_t n) {
  s->len += n;
  while (n) {
    size_t t = 64 - s->fill < n ? 64 - s->fill : n;
    memcpy(s->buf + s->fill, p, t);
    s->fill += t, p += t, n -= t;
    if (s->fill == 64) sha_block(s, s->buf), s->fill = 0;
  }
}

static void sha_hex(sha256_t* s, char out[65]) {
  const uint64_t bits = s->len * 8;
  uint8_t pad = 0x80, z = 0, lb[8];
  int i;
  sha_update(s, &pad, 1);
  while (s->fill != 56) sha_update(s, &z, 1);
  for (i = 0; i < 8; ++i) lb[i] = (uint8_t)(bits >> (56 - 8 * i));
  sha_update(s, lb, 8);
  for (i = 0; i < 8; ++i) sprintf(out + 8 * i, "%08x", s->h[i]);
}

static void print_digest(const char* name, const uint8_t* p, size_t n) {
  sha256_t s;
  char hex[65];
  sha_init(&s);
  sha_update(&s, p, n);
  sha_hex(&s, hex);
  printf("%s %s\n", name, hex);
}

/* ---- synthetic inputs (novelpoly_amd/synth.py) ---- */
static uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static void synth_payload(uint64_t index, uint8_t* out, size_t n) {
  size_t i;
  for (i = 0; i < n; ++i) {
    const uint64_t w = mix64((0x5EED0000ull + index) + (uint64_t)(i / 8 + 1) * 0x9E3779B97F4A7C15ull);
    out[i] = (uint8_t)(w >> (8 * (i % 8)));
  }
}

static void synth_present(uint64_t index, size_t n, size_t erase, uint8_t* present) {
  uint64_t state = 0xE7A50000ull + index;
  size_t* perm = (size_t*)malloc(n * sizeof *perm);
  size_t i;
  for (i = 0; i < n; ++i) perm[i] = i, present[i] = 1;
  for (i = 0; i < erase; ++i) {
    size_t j, t;
    state += 0x9E3779B97F4A7C15ull;
    j = i + (size_t)(mix64(state) % (uint64_t)(n - i));
    t = perm[i], perm[i] = perm[j], perm[j] = t;
  }
  for (i = 0; i < erase; ++i) present[perm[i]] = 0;
  free(perm);
}

#define CHECK(x)                                                               \
  do {                                                                         \
    int st_ = (x);                                                             \
    if (st_ != 0) {                                                            \
      fprintf(stderr, "%s:%d: %s -> %d (%s)\n", __FILE__, __LINE__, #x, st_, \
              np_status_message(st_));                                         \
      return 1;                                                                \
    }                                                                          \
  } while (0)
#define HCHECK(x)                                                                 \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d: %s -> %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

int main(void) {
  const size_t n_wanted = 256, k_wanted = 86, plen = 65536, erase = 192;
  np_code_params p;
  np_ctx* ctx = NULL;
  size_t sl, n, k, olen, out_len = 0, v, detail[3];
  uint8_t *payload, *shards, *present, *out, *d_pay, *d_sh, *d_out, *d_pres, *h_sh;
  const uint8_t** recv;
  size_t* lens;

  printf("version %s\n", np_version());
  CHECK(np_derive_parameters(n_wanted, k_wanted, &p));
  n = p.n, k = p.k;
  sl = np_shard_len(&p, plen);
  printf("params n=%zu k=%zu wanted_n=%zu shard_len=%zu fast=%d\n", n, k, p.wanted_n, sl, np_is_fast_path(&p));
  if (np_derive_parameters(1, 1, &p) != NP_ERR_WANTED_SHARD_COUNT_TOO_LOW) return 2; /* mod.rs:44-46 */
  np_last_error_detail(detail);
  if (detail[0] != 1) return 2;
  CHECK(np_derive_parameters(n_wanted, k_wanted, &p));

  payload = (uint8_t*)malloc(plen);
  shards = (uint8_t*)malloc(n * sl);
  present = (uint8_t*)malloc(n);
  olen = (sl / 2) * 2 * k;
  out = (uint8_t*)malloc(olen);
  h_sh = (uint8_t*)malloc(n * sl);
  recv = (const uint8_t**)malloc(n * sizeof *recv);
  lens = (size_t*)malloc(n * sizeof *lens);
  synth_payload(0, payload, plen);
  synth_present(0, n, erase, present);
  print_digest("payload", payload, plen);
  print_digest("present", present, n);
  fflush(stdout);
  CHECK(np_ctx_create(0, &ctx));

  /* encode.rs:6-11 */
  CHECK(np_encode(ctx, payload, plen, n_wanted, shards, sl));
  print_digest("np_encode", shards, p.wanted_n * sl);

  /* reconstruct.rs:4-9: NULL marks a missing shard */
  for (v = 0; v < n; ++v) {
    recv[v] = present[v] ? shards + v * sl : NULL;
    lens[v] = present[v] ? sl : 0;
  }
  CHECK(np_reconstruct(ctx, recv, lens, n, n_wanted, out, olen, &out_len));
  print_digest("np_reconstruct", out, out_len);

  /* too few shards: Error::NeedMoreShards{have, min, all} (mod.rs:178-180) */
  for (v = 0; v < n; ++v) recv[v] = v < k - 1 ? shards + v * sl : NULL, lens[v] = v < k - 1 ? sl : 0;
  if (np_reconstruct(ctx, recv, lens, n, n_wanted, out, olen, &out_len) != NP_ERR_NEED_MORE_SHARDS) return 3;
  np_last_error_detail(detail);
  printf("need_more_shards have=%zu min=%zu all=%zu\n", detail[0], detail[1], detail[2]);

  /* device batch API (hipMalloc'd buffers, the context's stream) */
  HCHECK(hipMalloc((void**)&d_pay, plen));
  HCHECK(hipMalloc((void**)&d_sh, n * sl));
  HCHECK(hipMalloc((void**)&d_out, olen));
  HCHECK(hipMalloc((void**)&d_pres, n));
  HCHECK(hipMemcpy(d_pay, payload, plen, hipMemcpyHostToDevice));
  HCHECK(hipMemcpy(d_pres, present, n, hipMemcpyHostToDevice));
  CHECK(np_encode_batch_dev(ctx, &p, d_pay, plen, plen, 1, d_sh, n * sl, NULL));
  CHECK(np_reconstruct_batch_dev2(ctx, &p, d_sh, sl, n * sl, d_pres, NULL, 1, d_out, olen, NULL));
  CHECK(np_ctx_synchronize(ctx));
  HCHECK(hipMemcpy(h_sh, d_sh, n * sl, hipMemcpyDeviceToHost));
  HCHECK(hipMemcpy(out, d_out, olen, hipMemcpyDeviceToHost));
  print_digest("np_encode_batch_dev", h_sh, p.wanted_n * sl);
  print_digest("np_reconstruct_batch_dev2", out, olen);

  HCHECK(hipFree(d_pay));
  HCHECK(hipFree(d_sh));
  HCHECK(hipFree(d_out));
  HCHECK(hipFree(d_pres));
  np_ctx_destroy(ctx);
  free(payload), free(shards), free(present), free(out), free(h_sh), free((void*)recv), free(lens);
  printf("done\n");
  return 0;
}
