/*
 * np_oracle.c -- scalar CPU restatement of the novel-polynomial-basis RS
 * hot path.  TEST INFRASTRUCTURE ONLY (see np_oracle.h for the rules and
 * for the reference file:line map).  Written from the published algorithm
 * (Lin, Han, Chung, FOCS'14) as the reference crate applies it; the code
 * is deliberately plain so that it is easy to audit against the reference.
 */
#include "np_oracle.h"

#include <stdlib.h>
#include <string.h>

#define Q 65535u          /* order of the multiplicative group, also "log zero" */
#define FSZ 65536u

static uint16_t g_log[FSZ];      /* Cantor-coordinate element -> discrete log     */
static uint16_t g_exp[FSZ];      /* discrete log -> Cantor-coordinate element     */
static uint16_t g_skew[FSZ];     /* skew factors (log form); [65535] unused       */
static uint16_t g_lwalsh[FSZ];   /* walsh(LOG with [0]=0)                         */
static int g_ready = 0;

/* Field constants: f2e16.rs:4-12 (generator 0x2D of x^16+x^5+x^3+x^2+1 and
 * the 16-element Cantor basis). */
static const uint16_t kCantor[16] = {1,     44234, 15374, 5694,  50562, 60718, 37196, 16402,
                                     27800, 4312,  27250, 47360, 64952, 64308, 65336, 39198};

uint16_t npo_mul(uint16_t a, uint16_t m) {
  /* inc_log_mul.rs:42-49: zero stays zero; otherwise add logs with an
   * end-around carry so that 65535 acts as 0 (g^65535 == 1). */
  if (a == 0) return 0;
  uint32_t t = (uint32_t)g_log[a] + (uint32_t)m;
  return g_exp[(t & 0xffffu) + (t >> 16)];
}

/* Walsh-Hadamard over Z/65535 with end-around carries, inc_log_mul.rs:92-114.
 * Values may come out as 65535 (the second representative of zero); the
 * reference keeps that representative, so do we. */
void npo_walsh(uint16_t* v, size_t size) {
  for (size_t h = 1; h < size; h <<= 1)
    for (size_t blk = 0; blk < size; blk += 2 * h)
      for (size_t i = blk; i < blk + h; ++i) {
        uint32_t a = v[i], b = v[i + h];
        uint32_t s = a + b, d = a + Q - b;
        v[i] = (uint16_t)((s & 0xffffu) + (s >> 16));
        v[i + h] = (uint16_t)((d & 0xffffu) + (d >> 16));
      }
}

static void build_tables(void) {
  /* poly -> log via the LFSR of the generator (inc_gen_field_tables.rs:33-45) */
  static uint16_t poly_log[FSZ];
  uint32_t st = 1;
  for (uint32_t e = 0; e < Q; ++e) {
    poly_log[st] = (uint16_t)e;
    st <<= 1;
    if (st & 0x10000u) st ^= 0x1002du;
  }
  poly_log[0] = (uint16_t)Q;
  /* Cantor coordinates -> polynomial element, then log (:47-58) */
  static uint16_t cant[FSZ];
  cant[0] = 0;
  for (unsigned b = 0; b < 16; ++b)
    for (uint32_t j = 0; j < (1u << b); ++j) cant[j | (1u << b)] = cant[j] ^ kCantor[b];
  for (uint32_t i = 0; i < FSZ; ++i) g_log[i] = poly_log[cant[i]];
  for (uint32_t i = 0; i < FSZ; ++i) g_exp[g_log[i]] = (uint16_t)i;
  g_exp[Q] = g_exp[0];
  /* LOG_WALSH (:64-70) */
  memcpy(g_lwalsh, g_log, sizeof g_lwalsh);
  g_lwalsh[0] = 0;
  npo_walsh(g_lwalsh, FSZ);
}

static void build_skews(void) {
  /* inc_afft.rs:386-445: skew factors s_j built additively over a basis that
   * is renormalised after every level m, then converted to log form. */
  uint16_t basis[15];
  for (unsigned i = 0; i < 15; ++i) basis[i] = (uint16_t)(1u << (i + 1));
  static uint16_t add[FSZ];
  memset(add, 0, sizeof add);
  for (unsigned m = 0; m < 15; ++m) {
    size_t stride = (size_t)1 << (m + 1);
    add[((size_t)1 << m) - 1] = 0;
    for (unsigned i = m; i < 15; ++i) {
      size_t span = (size_t)1 << (i + 1);
      for (size_t j = ((size_t)1 << m) - 1; j < span; j += stride) add[j + span] = add[j] ^ basis[i];
    }
    uint16_t prod = npo_mul(basis[m], g_log[basis[m] ^ 1]);
    basis[m] = (uint16_t)(Q - g_log[prod]);
    for (unsigned i = m + 1; i < 15; ++i) {
      uint32_t e = ((uint32_t)g_log[basis[i] ^ 1] + basis[m]) % Q;
      basis[i] = npo_mul(basis[i], (uint16_t)e);
    }
  }
  for (size_t i = 0; i < Q; ++i) g_skew[i] = g_log[add[i]];
  g_skew[Q] = (uint16_t)Q;
}

void npo_init(void) {
  if (g_ready) return;
  build_tables();
  build_skews();
  g_ready = 1;
}

const uint16_t* npo_log_table(void) { npo_init(); return g_log; }
const uint16_t* npo_exp_table(void) { npo_init(); return g_exp; }
const uint16_t* npo_skews(void) { npo_init(); return g_skew; }
const uint16_t* npo_log_walsh(void) { npo_init(); return g_lwalsh; }

/* inverse additive FFT, inc_afft.rs:139-214: bottom-up, per group first the
 * XOR then the (skippable) skew multiply. */
void npo_inverse_afft(uint16_t* v, size_t size, size_t index) {
  npo_init();
  for (size_t h = 1; h < size; h <<= 1) {
    for (size_t grp = h; grp < size; grp += 2 * h) {
      uint16_t s = g_skew[grp + index - 1];
      for (size_t i = grp - h; i < grp; ++i) v[i + h] ^= v[i];
      if (s != Q)
        for (size_t i = grp - h; i < grp; ++i) v[i] ^= npo_mul(v[i + h], s);
    }
  }
}

/* forward additive FFT, inc_afft.rs:267-332: top-down, multiply then XOR. */
void npo_afft(uint16_t* v, size_t size, size_t index) {
  npo_init();
  for (size_t h = size >> 1; h > 0; h >>= 1) {
    for (size_t grp = h; grp < size; grp += 2 * h) {
      uint16_t s = g_skew[grp + index - 1];
      if (s != Q)
        for (size_t i = grp - h; i < grp; ++i) v[i] ^= npo_mul(v[i + h], s);
      for (size_t i = grp - h; i < grp; ++i) v[i + h] ^= v[i];
    }
  }
}

/* formal derivative, inc_afft.rs:17-31 (the tweaked variant's B factors are
 * all the identity). */
void npo_formal_derivative(uint16_t* v, size_t size) {
  for (size_t i = 1; i < size; ++i) {
    size_t low = i & (~i + 1);
    for (size_t j = i - low; j < i; ++j) v[j] ^= (j + low < size) ? v[j + low] : 0;
  }
}

/* inc_encode.rs:15-48 */
void npo_encode_low(const uint16_t* data, size_t k, uint16_t* cw, size_t n) {
  memcpy(cw, data, n * sizeof(uint16_t));
  npo_inverse_afft(cw, k, 0);
  for (size_t shift = k; shift < n; shift += k) {
    memcpy(cw + shift, cw, k * sizeof(uint16_t));
    npo_afft(cw + shift, k, shift);
  }
  memcpy(cw, data, k * sizeof(uint16_t));
}

static int is_pow2(size_t x) { return x && !(x & (x - 1)); }

/* inc_encode.rs:165-208: big-endian packing, odd tail gets a zero low byte. */
int npo_encode_sub(const uint8_t* bytes, size_t len, size_t n, size_t k, uint16_t* cw) {
  if (!is_pow2(n) || !is_pow2(k) || len > 2 * k || 2 * k > n) return NPO_INVALID_ARGUMENT;
  uint16_t* elm = (uint16_t*)calloc(n, sizeof(uint16_t));
  if (!elm) return NPO_INVALID_ARGUMENT;
  for (size_t i = 0; i < (len + 1) / 2; ++i) {
    uint16_t hi = bytes[2 * i];
    uint16_t lo = (2 * i + 1 < len) ? bytes[2 * i + 1] : 0;
    elm[i] = (uint16_t)((hi << 8) | lo);
  }
  npo_encode_low(elm, k, cw, n);
  free(elm);
  return NPO_OK;
}

/* inc_reconstruct.rs:90-113, always evaluated over the full field. */
void npo_eval_error_polynomial(const uint8_t* er, size_t n_er, uint16_t* lw) {
  npo_init();
  memset(lw, 0, FSZ * sizeof(uint16_t));
  size_t z = n_er < FSZ ? n_er : FSZ;
  for (size_t i = 0; i < z; ++i) lw[i] = er[i] ? 1 : 0;
  npo_walsh(lw, FSZ);
  for (size_t i = 0; i < FSZ; ++i) lw[i] = (uint16_t)(((uint32_t)lw[i] * (uint32_t)g_lwalsh[i]) % Q);
  npo_walsh(lw, FSZ);
  for (size_t i = 0; i < z; ++i)
    if (er[i]) lw[i] = (uint16_t)(Q - lw[i]);
}

/* inc_reconstruct.rs:61-85 */
void npo_decode_main(uint16_t* cw, size_t upto, const uint8_t* er, const uint16_t* lw, size_t n) {
  for (size_t i = 0; i < n; ++i) cw[i] = er[i] ? 0 : npo_mul(cw[i], lw[i]);
  npo_inverse_afft(cw, n, 0);
  npo_formal_derivative(cw, n);
  npo_afft(cw, n, 0);
  for (size_t i = 0; i < upto; ++i) cw[i] = er[i] ? npo_mul(cw[i], lw[i]) : 0;
}

/* ---------------- API glue (novel_poly_basis/mod.rs, util.rs) ---------------- */

static size_t prev_pow2(size_t x) { size_t p = 1; while (p * 2 <= x) p *= 2; return p; }
static size_t next_pow2(size_t x) { size_t p = 1; while (p < x) p *= 2; return p; }

size_t npo_recoverability_subset_size(size_t n) { return (n ? (n - 1) / 3 : 0) + 1; }

int npo_derive_parameters(size_t n_w, size_t k_w, size_t* n, size_t* k, size_t* wn) {
  if (n_w < 2) return NPO_WANTED_SHARD_COUNT_TOO_LOW;
  if (k_w < 1) return NPO_WANTED_PAYLOAD_SHARD_COUNT_TOO_LOW;
  size_t kp = prev_pow2(k_w), np = next_pow2(n_w);
  if (np > FSZ) return NPO_WANTED_SHARD_COUNT_TOO_HIGH;
  *n = np; *k = kp; *wn = n_w;
  return NPO_OK;
}

size_t npo_shard_len(size_t k, size_t len) {
  size_t syms = (len + 1) / 2;
  return ((syms + k - 1) / k) * 2;
}

int npo_encode(const uint8_t* p, size_t len, size_t n, size_t k, size_t wn, uint8_t* out, size_t sl) {
  if (len == 0) return NPO_PAYLOAD_SIZE_IS_ZERO;
  if (sl != npo_shard_len(k, len) || wn > n) return NPO_INVALID_ARGUMENT;
  uint16_t* cw = (uint16_t*)malloc(n * sizeof(uint16_t));
  if (!cw) return NPO_INVALID_ARGUMENT;
  size_t chunk = 0;
  for (size_t off = 0; off < len; off += 2 * k, ++chunk) {
    size_t piece = len - off < 2 * k ? len - off : 2 * k;
    int st = npo_encode_sub(p + off, piece, n, k, cw);
    if (st) { free(cw); return st; }
    for (size_t v = 0; v < wn; ++v) {
      out[v * sl + 2 * chunk] = (uint8_t)(cw[v] >> 8);
      out[v * sl + 2 * chunk + 1] = (uint8_t)(cw[v] & 0xff);
    }
  }
  free(cw);
  return NPO_OK;
}

int npo_encode_batch(const uint8_t* p, size_t len, size_t batch, size_t n, size_t k, uint8_t* out) {
  size_t sl = npo_shard_len(k, len);
  for (size_t b = 0; b < batch; ++b) {
    int st = npo_encode(p + b * len, len, n, k, n, out + b * n * sl, sl);
    if (st) return st;
  }
  return NPO_OK;
}

/* shard length in symbols of a WrappedShard built from `bytes` bytes */
static size_t syms_of(size_t bytes) { return (bytes + 1) / 2; }

static uint16_t sym_at(const uint8_t* s, size_t bytes, size_t i) {
  uint16_t hi = (2 * i < bytes) ? s[2 * i] : 0;
  uint16_t lo = (2 * i + 1 < bytes) ? s[2 * i + 1] : 0;
  return (uint16_t)((hi << 8) | lo);
}

int npo_reconstruct(const uint8_t* const* shards, const size_t* lens, size_t nrecv, size_t n, size_t k,
                    uint8_t* out, size_t cap, size_t* out_len, size_t* det) {
  /* mod.rs:162-239 */
  uint8_t* er = (uint8_t*)malloc(n);
  if (!er) return NPO_INVALID_ARGUMENT;
  size_t have = 0;
  for (size_t i = 0; i < n; ++i) {
    er[i] = (i >= nrecv || shards[i] == NULL) ? 1 : 0;
    have += !er[i];
  }
  if (have < k) {
    if (det) { det[0] = have; det[1] = k; det[2] = n; }
    free(er);
    return NPO_NEED_MORE_SHARDS;
  }
  size_t first = 0;
  while (er[first]) ++first;
  size_t syms = syms_of(lens[first]);
  if (syms == 0) { free(er); return NPO_EMPTY_SHARD; }
  for (size_t i = first + 1; i < n; ++i)
    if (!er[i] && syms_of(lens[i]) != syms) {
      if (det) { det[0] = syms; det[1] = syms_of(lens[i]); det[2] = 0; }
      free(er);
      return NPO_INCONSISTENT_SHARD_LENGTHS;
    }
  size_t need = syms * 2 * k;
  if (cap < need) { free(er); return NPO_INVALID_ARGUMENT; }
  uint16_t* lw = (uint16_t*)malloc(FSZ * sizeof(uint16_t));
  uint16_t* cw = (uint16_t*)malloc(n * sizeof(uint16_t));
  npo_eval_error_polynomial(er, n, lw);
  for (size_t s = 0; s < syms; ++s) {
    for (size_t i = 0; i < n; ++i) cw[i] = er[i] ? 0 : sym_at(shards[i], lens[i], s);
    /* inc_reconstruct.rs:20-50: present data symbols are passed through */
    uint16_t* keep = (uint16_t*)malloc(k * sizeof(uint16_t));
    memcpy(keep, cw, k * sizeof(uint16_t));
    npo_decode_main(cw, k, er, lw, n);
    for (size_t i = 0; i < k; ++i) {
      uint16_t v = er[i] ? cw[i] : keep[i];
      out[s * 2 * k + 2 * i] = (uint8_t)(v >> 8);
      out[s * 2 * k + 2 * i + 1] = (uint8_t)(v & 0xff);
    }
    free(keep);
  }
  *out_len = need;
  free(cw); free(lw); free(er);
  return NPO_OK;
}

int npo_reconstruct_from_systematic(const uint8_t* const* shards, const size_t* lens, size_t nch, size_t n,
                                    size_t k, uint8_t* out, size_t cap, size_t* out_len, size_t* det) {
  /* mod.rs:247-285 */
  if (nch == 0 || nch < k) {
    if (det) { det[0] = nch; det[1] = k; det[2] = n; }
    return NPO_NEED_MORE_SHARDS;
  }
  size_t syms = syms_of(lens[0]);
  if (syms == 0) return NPO_EMPTY_SHARD;
  for (size_t i = 0; i < nch; ++i)
    if (syms_of(lens[i]) != syms) {
      if (det) { det[0] = syms; det[1] = syms_of(lens[i]); det[2] = 0; }
      return NPO_INCONSISTENT_SHARD_LENGTHS;
    }
  size_t need = syms * 2 * k;
  if (cap < need) return NPO_INVALID_ARGUMENT;
  for (size_t s = 0; s < syms; ++s)
    for (size_t c = 0; c < k; ++c) {
      uint16_t v = sym_at(shards[c], lens[c], s);
      out[s * 2 * k + 2 * c] = (uint8_t)(v >> 8);
      out[s * 2 * k + 2 * c + 1] = (uint8_t)(v & 0xff);
    }
  *out_len = need;
  return NPO_OK;
}
