// Host-side construction of the GF(2^16) tables the kernels consume.
//
// Generated from scratch at context creation (the crate generates them at
// build time: reed-solomon-novelpoly/inc_gen_field_tables.rs:29-93, skew
// factors at src/field/inc_afft.rs:386-445).  Field constants:
// src/field/f2e16.rs:4-12.
#pragma once
#include <cstdint>
#include <vector>

namespace np {

constexpr uint32_t kFieldSize = 65536;
constexpr uint32_t kOneMask = 65535;  // ONEMASK: group order, also the "skip" skew sentinel

struct HostTables {
  std::vector<uint16_t> log;        // Cantor coordinates -> discrete log   (LOG_TABLE)
  std::vector<uint16_t> exp;        // discrete log -> Cantor coordinates   (EXP_TABLE)
  std::vector<uint16_t> skew;       // 65536 entries, log form, [i]==65535 -> multiply skipped (AFFT.skews)
  std::vector<uint16_t> skew_add;   // additive (field element) form of skew, 0 for the sentinel
  std::vector<uint16_t> log_walsh;  // LOG_WALSH
  // LOG_WALSH folded to n points for every power of two n: entries [n, 2n) hold
  // F_n[j] = sum_h LOG_WALSH[j + n*h] mod 65535 (the 65536-point
  // Walsh pair of eval_error_polynomial restricted to an erasure set inside
  // [0, n) equals two n-point Walsh transforms around F_n, mod 65535).
  std::vector<uint16_t> lw_fold;
  // Per additive multiplier c (65536 of them): byte tables for the v_perm
  // multiplier (kernels_fast.hip, "GF multiply"); 20 dwords each.
  std::vector<uint32_t> perm_pools;
};

// Built once, thread-safe.
const HostTables& host_tables();

// a * g^m with the crate's conventions (inc_log_mul.rs:42-49).
uint16_t host_mul(const HostTables& t, uint16_t a, uint16_t m);
// a * c for two field elements in additive (Cantor coordinate) form.
uint16_t host_mul_add(const HostTables& t, uint16_t a, uint16_t c);

constexpr int kPermPoolWords = 20;
constexpr int kPoolVWords = 8;  // VGPR half, stored first

}  // namespace np
