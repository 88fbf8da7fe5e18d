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

  // Tower coordinates of the fast kernels.  GF(2^16) = GF(2^8) + gamma GF(2^8)
  // with gamma = beta_8 (the Cantor basis element of bit 8); beta_{8+i} =
  // a_i + gamma e_i with a_i, e_i in GF(2^8) = span(beta_0..beta_7).  A symbol
  // with Cantor coordinates (lo, hi) has tower coordinates (lo ^ A(hi), hi):
  // the low byte is its GF(2^8) part a over beta_0..beta_7, the high byte its
  // gamma part b over e_0..e_7.  The map is an involution (to_tower).  Every
  // skew factor Cantor(v) with v < 256 lies in GF(2^8), where it multiplies a
  // and b separately: 6 byte lookups instead of 12 (fast_common.hpp qmul_sub).
  uint8_t tower_a[8] = {0}, tower_e[8] = {0};
  // Per multiplier c, 20 dwords each, kernels in tower coordinates:
  //  tower_pools: x -> c x, tower -> tower; c < 256: the subfield layout
  //               (kSubV / kSubS); entry kFieldSize: the conversion's
  //               high-plane -> low-plane tables in the subfield b slots;
  //  in_pools:    Cantor -> tower (the decode's premultiply);
  //  out_pools:   tower -> Cantor (the decode's postmultiply).
  std::vector<uint32_t> tower_pools, in_pools, out_pools;
  // The full 16 x 16 map layout (build_pool, tower -> tower) of the 256
  // subfield elements, whose tower_pools entries hold the subfield layout:
  // for transforms whose levels mix skews inside and outside GF(2^8) (the
  // k = 1024 resident kernels' level 0-1 groups at index 0).
  std::vector<uint32_t> tower_full_sub;
};

// Built once, thread-safe.
const HostTables& host_tables();

// a * g^m with the crate's conventions (inc_log_mul.rs:42-49).
uint16_t host_mul(const HostTables& t, uint16_t a, uint16_t m);
// a * c for two field elements in additive (Cantor coordinate) form.
uint16_t host_mul_add(const HostTables& t, uint16_t a, uint16_t c);

constexpr int kPermPoolWords = 20;
constexpr int kPoolVWords = 8;  // VGPR half, stored first
// Subfield layout inside a 20-dword pool: VGPR dwords kSubV + 2 plane + g
// (entries 0-3 of the 8-entry tables g = 0, 1), SGPR dwords kSubS + 3 plane + g
// (entries 4-7 of tables 0, 1; the 4-entry table g = 2); plane 0 = a (low
// byte), 1 = b (high byte).
constexpr int kSubV = 0;
constexpr int kSubS = 8;

// Cantor <-> tower coordinates (an involution, see HostTables::tower_a).
uint16_t to_tower(const HostTables& t, uint16_t x);

}  // namespace np
