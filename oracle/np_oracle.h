/*
 * np_oracle.h -- CPU restatement of the reed-solomon-novelpoly hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This library is the parity checker for the
 * MI355X engine: only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it.  The product (libnovelpoly_hip.so) never
 * links or calls it.
 *
 * It restates, from scratch and in plain C, the algorithm of the reference
 * crate (paths relative to /root/reference/reed-solomon-novelpoly):
 *   field tables   inc_gen_field_tables.rs:29-72   (C twin cxx/RSErasureCode.c:106-129)
 *   skew factors   src/field/inc_afft.rs:386-445   (C twin cxx/RSErasureCode.c:132-151)
 *   mul            src/field/inc_log_mul.rs:42-49  (C twin mulE :43-45)
 *   walsh          src/field/inc_log_mul.rs:92-114 (C twin walsh :47-58)
 *   inverse_afft   src/field/inc_afft.rs:139-214   (C twin IFLT :75-88)
 *   afft           src/field/inc_afft.rs:267-332   (C twin FLT :91-103)
 *   formal deriv.  src/field/inc_afft.rs:17-58     (C twin :60-73; B factors are identity)
 *   encode_low     src/field/inc_encode.rs:15-48   (C twin encodeL :175-183)
 *   encode_sub     src/field/inc_encode.rs:165-208
 *   error locator  src/field/inc_reconstruct.rs:90-113 (C twin decode_init :200-209)
 *   decode_main    src/field/inc_reconstruct.rs:61-85  (C twin :211-240)
 *   reconstruct_sub src/field/inc_reconstruct.rs:1-55
 *   API glue       src/novel_poly_basis/mod.rs:43-285, src/util.rs:1-42
 *
 * Parity of this restatement is pinned against the reference's own C
 * implementation compiled from /root/reference (oracle/Makefile ->
 * oracle/_ref/librsec_ref.so) and against the known-answer tests that the
 * reference's test-suite holds (see tests/test_oracle.py).
 */
#ifndef NP_ORACLE_H
#define NP_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes: same numbering as include/novelpoly.h (errors.rs:4-28 order) */
#define NPO_OK 0
#define NPO_WANTED_SHARD_COUNT_TOO_HIGH 1
#define NPO_WANTED_SHARD_COUNT_TOO_LOW 2
#define NPO_WANTED_PAYLOAD_SHARD_COUNT_TOO_LOW 3
#define NPO_PAYLOAD_SIZE_IS_ZERO 4
#define NPO_NEED_MORE_SHARDS 5
#define NPO_PARAMETER_MUST_BE_POWER_OF_2 6
#define NPO_INCONSISTENT_SHARD_LENGTHS 7
#define NPO_EMPTY_SHARD 8
#define NPO_INVALID_ARGUMENT 100

void npo_init(void);
const uint16_t* npo_log_table(void);   /* 65536 entries */
const uint16_t* npo_exp_table(void);   /* 65536 entries */
const uint16_t* npo_skews(void);       /* 65535 entries, log form, 65535 = skip */
const uint16_t* npo_log_walsh(void);   /* 65536 entries */

uint16_t npo_mul(uint16_t additive, uint16_t multiplier);
void npo_walsh(uint16_t* data, size_t size);
void npo_afft(uint16_t* data, size_t size, size_t index);
void npo_inverse_afft(uint16_t* data, size_t size, size_t index);
void npo_formal_derivative(uint16_t* data, size_t size);
/* data holds n symbols (the message zero-padded from k to n, inc_encode.rs:18) */
void npo_encode_low(const uint16_t* data, size_t k, uint16_t* codeword, size_t n);
int  npo_encode_sub(const uint8_t* bytes, size_t len, size_t n, size_t k, uint16_t* codeword_out);
void npo_eval_error_polynomial(const uint8_t* erasures, size_t n_erasures, uint16_t* locator_out /*65536*/);
void npo_decode_main(uint16_t* codeword, size_t recover_up_to, const uint8_t* erasures,
                     const uint16_t* locator, size_t n);

/* API glue (mod.rs / util.rs) */
size_t npo_recoverability_subset_size(size_t n_wanted);
int    npo_derive_parameters(size_t n_wanted, size_t k_wanted, size_t* n, size_t* k, size_t* wanted_n);
size_t npo_shard_len(size_t k, size_t payload_len);
/* shards_out: wanted_n rows of shard_len bytes (row-major) */
int npo_encode(const uint8_t* payload, size_t len, size_t n, size_t k, size_t wanted_n,
               uint8_t* shards_out, size_t shard_len);
/* shards[i] == NULL -> missing; lens in bytes (odd lengths are zero padded like WrappedShard).
 * out must hold (max shard symbols)*2*k bytes; *out_len receives the produced length.
 * detail[3] receives the error payload (have,min,all / first,other). */
int npo_reconstruct(const uint8_t* const* shards, const size_t* lens, size_t n_received,
                    size_t n, size_t k, uint8_t* out, size_t out_cap, size_t* out_len, size_t* detail);
int npo_reconstruct_from_systematic(const uint8_t* const* shards, const size_t* lens, size_t n_chunks,
                                    size_t n, size_t k, uint8_t* out, size_t out_cap, size_t* out_len,
                                    size_t* detail);

/* Batch helpers used by bench.py's CPU baseline (single thread). */
int npo_encode_batch(const uint8_t* payloads, size_t payload_len, size_t batch, size_t n, size_t k,
                     uint8_t* shards_out /* batch * n * shard_len */);

#ifdef __cplusplus
}
#endif
#endif
