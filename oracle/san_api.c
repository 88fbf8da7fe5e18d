/*
 * san_api.c -- drives the restatement's crate-level glue (np_oracle.c:
 * derive_parameters, encode, reconstruct, reconstruct_from_systematic) under
 * AddressSanitizer + UBSan.  TEST INFRASTRUCTURE ONLY: built by
 * `make -C oracle san`, run by tests/test_cpu_bench.py::test_oracle_api_sanitized.
 *
 * Cases follow the reference's own feeds: the reconstruct fuzz target
 * (reed-solomon-novelpoly-fuzzit/src/reconstruct.rs:15-43: validator counts,
 * arbitrary shard bytes and lengths, missing shards), the roundtrip tests
 * (reed-solomon-novelpoly/src/novel_poly_basis/tests.rs), and the error paths of
 * errors.rs (zero payload, too few shards, inconsistent / empty shards).
 *
 * usage: san_api SEED ITERATIONS ; prints one JSON line, exit 1 on a mismatch.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "np_oracle.h"

static uint64_t rng;
static uint64_t next(void) {
  uint64_t z = (rng += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static size_t below(size_t m) { return m ? (size_t)(next() % m) : 0; }

static int failures;
#define CHECK(c, ...)                   \
  do {                                  \
    if (!(c)) {                         \
      fprintf(stderr, __VA_ARGS__);     \
      fputc('\n', stderr);              \
      ++failures;                       \
    }                                   \
  } while (0)

/* encode -> drop shards -> reconstruct (and from_systematic) round trip */
static void roundtrip(size_t validators, size_t len, int corrupt) {
  const size_t kw = npo_recoverability_subset_size(validators);
  size_t n, k, wn;
  if (npo_derive_parameters(validators, kw, &n, &k, &wn) != NPO_OK) return;
  uint8_t* pay = malloc(len ? len : 1);
  for (size_t i = 0; i < len; ++i) pay[i] = (uint8_t)next();
  const size_t sl = npo_shard_len(k, len);
  uint8_t* sh = malloc(wn * sl + 1);
  int st = npo_encode(pay, len, n, k, wn, sh, sl);
  if (len == 0) {
    CHECK(st == NPO_PAYLOAD_SIZE_IS_ZERO, "encode of an empty payload: %d", st);
    free(pay), free(sh);
    return;
  }
  CHECK(st == NPO_OK, "encode(%zu validators, %zu bytes): %d", validators, len, st);
  const uint8_t** rows = calloc(wn, sizeof(*rows));
  size_t* lens = calloc(wn, sizeof(size_t));
  size_t have = 0;
  for (size_t v = 0; v < wn; ++v) {
    if (below(3) != 0) rows[v] = sh + v * sl, lens[v] = sl, ++have;
  }
  if (corrupt && have) {  /* non-codeword input: the decode stays defined */
    size_t v = below(wn);
    while (!rows[v]) v = (v + 1) % wn;
    sh[v * sl + below(sl)] ^= (uint8_t)(1 + below(255));
  }
  const size_t cap = (sl / 2) * 2 * k + 16;
  uint8_t* out = malloc(cap);
  size_t out_len = 0, detail[3] = {0, 0, 0};
  st = npo_reconstruct(rows, lens, wn, n, k, out, cap, &out_len, detail);
  if (have < k) {
    CHECK(st == NPO_NEED_MORE_SHARDS, "reconstruct with %zu < %zu rows: %d", have, k, st);
  } else {
    CHECK(st == NPO_OK, "reconstruct(%zu validators): %d", validators, st);
    if (!corrupt) CHECK(out_len >= len && memcmp(out, pay, len) == 0, "round trip differs (%zu validators)", validators);
  }
  /* from_systematic: the first k rows, all present */
  for (size_t v = 0; v < k && v < wn; ++v) rows[v] = sh + v * sl, lens[v] = sl;
  st = npo_reconstruct_from_systematic(rows, lens, k < wn ? k : wn, n, k, out, cap, &out_len, detail);
  if (!corrupt) CHECK(st == NPO_OK && memcmp(out, pay, len) == 0, "from_systematic (%zu validators): %d", validators, st);
  free(out), free(rows), free(lens), free(pay), free(sh);
}

/* the fuzz target's feed: arbitrary bytes and lengths in arbitrary rows */
static void fuzz(size_t validators) {
  const size_t kw = npo_recoverability_subset_size(validators);
  size_t n, k, wn;
  if (npo_derive_parameters(validators, kw, &n, &k, &wn) != NPO_OK) return;
  const size_t rows_n = below(wn + 2);
  const uint8_t** rows = calloc(rows_n + 1, sizeof(*rows));
  size_t* lens = calloc(rows_n + 1, sizeof(size_t));
  uint8_t* pool = malloc(rows_n * 64 + 1);
  const size_t common = below(64);
  for (size_t v = 0; v < rows_n; ++v) {
    if (below(4) == 0) continue;
    lens[v] = below(8) == 0 ? below(64) : common;
    for (size_t i = 0; i < lens[v]; ++i) pool[v * 64 + i] = (uint8_t)next();
    rows[v] = pool + v * 64;
  }
  const size_t cap = 64 * k + 16;
  uint8_t* out = malloc(cap);
  size_t out_len = 0, detail[3] = {0, 0, 0};
  const int st = npo_reconstruct(rows, lens, rows_n, n, k, out, cap, &out_len, detail);
  CHECK(st >= NPO_OK && st <= NPO_INVALID_ARGUMENT, "fuzz status %d", st);
  CHECK(st != NPO_OK || out_len <= cap, "fuzz output overruns");
  free(out), free(pool), free(rows), free(lens);
}

int main(int argc, char** argv) {
  if (argc != 3) {
    fprintf(stderr, "usage: %s SEED ITERATIONS\n", argv[0]);
    return 2;
  }
  rng = strtoull(argv[1], 0, 10);
  const long iters = atol(argv[2]);
  npo_init();
  static const size_t fixed[] = {2, 3, 4, 5, 10, 24, 40, 100, 191, 300, 1024, 2000, 2200};
  for (size_t i = 0; i < sizeof fixed / sizeof fixed[0]; ++i) {
    roundtrip(fixed[i], 1 + below(5000), 0);
    roundtrip(fixed[i], 0, 0);
    roundtrip(fixed[i], 1 + below(3000), 1);
  }
  for (long it = 0; it < iters; ++it) {
    const size_t validators = 1 + below(2200);
    roundtrip(validators, below(4) == 0 ? 1 + below(7) : 1 + below(4000), (int)below(2));
    fuzz(validators);
  }
  /* parameter derivation over every validator count the fuzz target draws */
  for (size_t v = 0; v <= 70000; v += 1 + below(97)) {
    size_t n, k, wn;
    const int st = npo_derive_parameters(v, npo_recoverability_subset_size(v), &n, &k, &wn);
    CHECK(st != NPO_OK || (n <= 65536 && k * 2 <= n && wn <= n), "derive_parameters(%zu)", v);
  }
  printf("{\"iterations\": %ld, \"failures\": %d}\n", iters, failures);
  return failures ? 1 : 0;
}
