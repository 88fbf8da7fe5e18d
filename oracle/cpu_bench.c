/*
 * cpu_bench.c -- CPU baseline for bench.py (TEST INFRASTRUCTURE ONLY).
 *
 * Times the whole-payload encode + reconstruct of one BASELINE config on the
 * host cores, with the crate's per-payload glue restated here (paths relative
 * to /root/reference/reed-solomon-novelpoly):
 *   encode        chunk loop + BE packing + shard scatter  mod.rs:117-157, inc_encode.rs:165-208
 *   reconstruct   erasure vector, locator once per payload mod.rs:162-239
 *                 per-column gather / decode / merge       inc_reconstruct.rs:1-55
 * around one of two field/transform back ends, chosen at compile time:
 *   -DNP_BENCH_REF : the reference's own C implementation cxx/RSErasureCode.c
 *                    (encodeL :175-183, decode_init :200-209, decode_main :211-240),
 *                    compiled from /root/reference by oracle/Makefile into
 *                    oracle/_ref/cpu_bench_ref (never copied into the repo);
 *   default        : the restatement np_oracle.c (oracle/cpu_bench_port).
 * Payloads are independent, so T threads take payloads from a shared counter
 * (the caller-side parallelism the crate leaves to its users).
 * Every payload's reconstruction is checked against its input.
 *
 * usage: cpu_bench N K PAYLOAD_BYTES ERASURES THREADS SECONDS
 * prints one JSON object: payloads, seconds, gib_s, threads, kind.
 */
#include <pthread.h>
#include <stdatomic.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define FIELD 65536

#ifdef NP_BENCH_REF
#include "RSErasureCode.h"
static const char* KIND = "reference";
static void be_init(void) { setup(); }
static void be_encode_low(const uint16_t* data, size_t k, uint16_t* cw, size_t n) {
  encodeL((GFSymbol*)data, (int)k, cw, (int)n);
}
/* decode_init reads log_walsh2[n..FIELD) as input of its walsh: the caller zeroes it */
static void be_locator(const int* erased, const uint8_t* erased8, size_t n, uint16_t* loc) {
  (void)erased8;
  memset(loc, 0, FIELD * sizeof(uint16_t));
  (void)n;  /* called over the whole field, as mod.rs:217-218 calls eval_error_polynomial */
  decode_init((Boolean*)erased, loc, FIELD);
}
static void be_decode(uint16_t* cw, size_t k, const int* erased, const uint8_t* erased8, const uint16_t* loc,
                      size_t n) {
  (void)erased8;
  decode_main(cw, (int)k, (Boolean*)erased, (GFSymbol*)loc, (int)n);
}
#else
#include "np_oracle.h"
static const char* KIND = "port";
static void be_init(void) { npo_init(); }
static void be_encode_low(const uint16_t* data, size_t k, uint16_t* cw, size_t n) { npo_encode_low(data, k, cw, n); }
static void be_locator(const int* erased, const uint8_t* erased8, size_t n, uint16_t* loc) {
  (void)erased;
  npo_eval_error_polynomial(erased8, n, loc);
}
static void be_decode(uint16_t* cw, size_t k, const int* erased, const uint8_t* erased8, const uint16_t* loc,
                      size_t n) {
  (void)erased;
  npo_decode_main(cw, k, erased8, loc, n);
}
#endif

static size_t N, K, PLEN, ERASE, SHARD_LEN, CHUNKS;
static atomic_long next_payload;
static long stop_after;
static double deadline;
static atomic_int failures;

static double now(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + 1e-9 * ts.tv_nsec;
}

static uint64_t splitmix64(uint64_t* s) {
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

typedef struct {
  uint8_t *payload, *shards, *out;
  uint16_t *data, *cw, *loc;
  int* erased;
  uint8_t* erased8;
  uint32_t* perm;
  long done;
} Worker;

static void one_payload(Worker* w, long idx) {
  uint64_t s = 0x5EED0000ull + (uint64_t)idx;
  for (size_t i = 0; i < PLEN; i += 8) {
    const uint64_t v = splitmix64(&s);
    for (size_t b = 0; b < 8 && i + b < PLEN; ++b) w->payload[i + b] = (uint8_t)(v >> (8 * b));
  }
  /* encode: chunk c = payload bytes [2kc, 2k(c+1)), BE u16, zero padded */
  for (size_t c = 0; c < CHUNKS; ++c) {
    for (size_t i = 0; i < K; ++i) {
      const size_t o = 2 * K * c + 2 * i;
      const uint8_t hi = o < PLEN ? w->payload[o] : 0, lo = o + 1 < PLEN ? w->payload[o + 1] : 0;
      w->data[i] = (uint16_t)(hi << 8 | lo);
    }
    be_encode_low(w->data, K, w->cw, N);
    for (size_t v = 0; v < N; ++v) {
      w->shards[v * SHARD_LEN + 2 * c] = (uint8_t)(w->cw[v] >> 8);
      w->shards[v * SHARD_LEN + 2 * c + 1] = (uint8_t)w->cw[v];
    }
  }
  /* erasures: partial Fisher-Yates over [0, N) */
  uint64_t e = 0xE7A50000ull + (uint64_t)idx;
  for (size_t i = 0; i < N; ++i) w->perm[i] = (uint32_t)i, w->erased[i] = 0, w->erased8[i] = 0;
  for (size_t i = 0; i < ERASE; ++i) {
    const size_t j = i + (size_t)(splitmix64(&e) % (N - i));
    const uint32_t t = w->perm[i];
    w->perm[i] = w->perm[j], w->perm[j] = t;
    w->erased[w->perm[i]] = 1, w->erased8[w->perm[i]] = 1;
  }
  /* reconstruct: locator once per payload, then every symbol column */
  be_locator(w->erased, w->erased8, N, w->loc);
  for (size_t c = 0; c < CHUNKS; ++c) {
    for (size_t v = 0; v < N; ++v)
      w->cw[v] = w->erased8[v] ? 0 : (uint16_t)(w->shards[v * SHARD_LEN + 2 * c] << 8 | w->shards[v * SHARD_LEN + 2 * c + 1]);
    memcpy(w->data, w->cw, K * sizeof(uint16_t));
    be_decode(w->cw, K, w->erased, w->erased8, w->loc, N);
    for (size_t i = 0; i < K; ++i) {
      const uint16_t v = w->erased8[i] ? w->cw[i] : w->data[i];
      w->out[2 * K * c + 2 * i] = (uint8_t)(v >> 8);
      w->out[2 * K * c + 2 * i + 1] = (uint8_t)v;
    }
  }
  if (memcmp(w->out, w->payload, PLEN) != 0) atomic_fetch_add(&failures, 1);
}

static void* run(void* arg) {
  Worker* w = (Worker*)arg;
  for (;;) {
    if (now() > deadline) break;
    const long idx = atomic_fetch_add(&next_payload, 1);
    if (idx >= stop_after) break;
    one_payload(w, idx);
    ++w->done;
  }
  return NULL;
}

int main(int argc, char** argv) {
  if (argc != 7) {
    fprintf(stderr, "usage: %s N K PAYLOAD_BYTES ERASURES THREADS SECONDS\n", argv[0]);
    return 2;
  }
  N = strtoull(argv[1], 0, 10), K = strtoull(argv[2], 0, 10), PLEN = strtoull(argv[3], 0, 10);
  ERASE = strtoull(argv[4], 0, 10);
  const int threads = atoi(argv[5]);
  const double seconds = atof(argv[6]);
  if (N < 2 || K < 1 || K * 2 > N || N > FIELD || PLEN == 0 || ERASE > N - K || threads < 1) {
    fprintf(stderr, "bad arguments\n");
    return 2;
  }
  CHUNKS = (PLEN + 2 * K - 1) / (2 * K);
  SHARD_LEN = 2 * CHUNKS;
  be_init();
  Worker* ws = calloc((size_t)threads, sizeof(Worker));
  for (int t = 0; t < threads; ++t) {
    Worker* w = &ws[t];
    w->payload = malloc(PLEN), w->out = malloc(2 * K * CHUNKS), w->shards = malloc(N * SHARD_LEN);
    /* data: n symbols, zero beyond k (encode_low reads n: inc_encode.rs:18, :193-196) */
    w->data = calloc(N, sizeof(uint16_t)), w->cw = malloc(N * sizeof(uint16_t));
    w->loc = malloc(FIELD * sizeof(uint16_t)), w->erased = calloc(FIELD, sizeof(int));
    w->erased8 = calloc(FIELD, 1), w->perm = malloc(N * sizeof(uint32_t));
  }
  stop_after = 100000;
  const double t0 = now();
  deadline = t0 + seconds;
  pthread_t* th = malloc((size_t)threads * sizeof(pthread_t));
  for (int t = 0; t < threads; ++t) pthread_create(&th[t], NULL, run, &ws[t]);
  long done = 0;
  for (int t = 0; t < threads; ++t) pthread_join(th[t], NULL), done += ws[t].done;
  const double dt = now() - t0;
  printf("{\"kind\": \"%s\", \"payloads\": %ld, \"seconds\": %.3f, \"threads\": %d, \"gib_s\": %.6f, \"failures\": %d}\n",
         KIND, done, dt, threads, done * (double)PLEN / dt / (1024.0 * 1024.0 * 1024.0), atomic_load(&failures));
  for (int t = 0; t < threads; ++t) {
    Worker* w = &ws[t];
    free(w->payload), free(w->out), free(w->shards), free(w->data), free(w->cw);
    free(w->loc), free(w->erased), free(w->erased8), free(w->perm);
  }
  free(ws), free(th);
  return atomic_load(&failures) ? 1 : 0;
}
