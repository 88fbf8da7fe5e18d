// Host construction of field tables, skews and multiplier lookup tables.
// See field_tables.hpp for the reference citations.
#include "field_tables.hpp"

#include <mutex>

namespace np {
namespace {

// Cantor basis of GF(2^16) over GF(2) used by the crate (f2e16.rs:6).
constexpr uint16_t kCantorBasis[16] = {1,     44234, 15374, 5694,  50562, 60718, 37196, 16402,
                                       27800, 4312,  27250, 47360, 64952, 64308, 65336, 39198};
constexpr uint32_t kReductionPoly = 0x1002d;  // x^16 + x^5 + x^3 + x^2 + 1 (GENERATOR 0x2D)

void fwht_mod_onemask(uint16_t* v, uint32_t n) {
  // inc_log_mul.rs:92-114: butterflies (a+b, a-b) over Z/65535 with end-around carry.
  for (uint32_t half = 1; half < n; half <<= 1) {
    for (uint32_t base = 0; base < n; base += half << 1) {
      for (uint32_t i = base; i < base + half; ++i) {
        uint32_t a = v[i], b = v[i + half];
        uint32_t sum = a + b, dif = a + kOneMask - b;
        v[i] = static_cast<uint16_t>((sum & 0xffffu) + (sum >> 16));
        v[i + half] = static_cast<uint16_t>((dif & 0xffffu) + (dif >> 16));
      }
    }
  }
}

// v_perm pools of a GF(2)-linear map f of 16-bit symbols: input byte plane P
// (0 = low byte, 1 = high byte), bit group G (bits 0-2, 3-5, 6-7 of that byte)
// -> contribution to output byte O.  Logical order: for O in {lo, hi}:
// [P0G0 a,b][P0G1 a,b][P0G2][P1G0 a,b][P1G1 a,b][P1G2] where a = entries 0-3
// (v_perm S1, read from a VGPR) and b = entries 4-7 (S0, an SGPR).  Stored as
// the 8 "a" dwords first (kPoolVWords, staged in LDS by the kernels) and then
// the 12 SGPR dwords.
template <class F>
void build_pool(F f, uint32_t* pool) {
  uint32_t logical[kPermPoolWords];
  int w = 0;
  for (int out_byte = 0; out_byte < 2; ++out_byte) {
    for (int plane = 0; plane < 2; ++plane) {
      const int shifts[3] = {0, 3, 6};
      const int widths[3] = {3, 3, 2};
      for (int g = 0; g < 3; ++g) {
        uint8_t entries[8] = {0};
        for (int v = 0; v < (1 << widths[g]); ++v) {
          const uint16_t in = static_cast<uint16_t>((v << shifts[g]) << (8 * plane));
          const uint16_t prod = f(in);
          entries[v] = static_cast<uint8_t>(out_byte ? (prod >> 8) : (prod & 0xff));
        }
        // v_perm_b32(S0, S1, sel): selector 0..3 -> bytes of S1, 4..7 -> bytes of S0.
        const uint32_t lo = entries[0] | (entries[1] << 8) | (entries[2] << 16) | (uint32_t(entries[3]) << 24);
        const uint32_t hi = entries[4] | (entries[5] << 8) | (entries[6] << 16) | (uint32_t(entries[7]) << 24);
        logical[w++] = lo;
        if (widths[g] == 3) logical[w++] = hi;  // 4-entry tables use S0 == S1
      }
    }
  }
  static constexpr int kV[8] = {0, 2, 5, 7, 10, 12, 15, 17};
  static constexpr int kS[12] = {1, 3, 4, 6, 8, 9, 11, 13, 14, 16, 18, 19};
  for (int i = 0; i < 8; ++i) pool[i] = logical[kV[i]];
  for (int i = 0; i < 12; ++i) pool[8 + i] = logical[kS[i]];
}

// Subfield pool (field_tables.hpp kSub*): two 8-bit maps, fa on the low
// (a) plane and fb on the high (b) plane, 3 byte tables each.
template <class FA, class FB>
void build_sub_pool(FA fa, FB fb, uint32_t* pool) {
  const int shifts[3] = {0, 3, 6};
  const int widths[3] = {3, 3, 2};
  for (int plane = 0; plane < 2; ++plane) {
    for (int g = 0; g < 3; ++g) {
      uint8_t entries[8] = {0};
      for (int v = 0; v < (1 << widths[g]); ++v) {
        const uint8_t in = static_cast<uint8_t>(v << shifts[g]);
        entries[v] = plane ? fb(in) : fa(in);
      }
      const uint32_t lo = entries[0] | (entries[1] << 8) | (entries[2] << 16) | (uint32_t(entries[3]) << 24);
      const uint32_t hi = entries[4] | (entries[5] << 8) | (entries[6] << 16) | (uint32_t(entries[7]) << 24);
      if (g < 2) {
        pool[kSubV + 2 * plane + g] = lo;
        pool[kSubS + 3 * plane + g] = hi;
      } else {
        pool[kSubS + 3 * plane + 2] = lo;
      }
    }
  }
}

void build(HostTables& t) {
  t.log.assign(kFieldSize, 0);
  t.exp.assign(kFieldSize, 0);
  // polynomial-basis element -> log, by stepping powers of the generator.
  std::vector<uint16_t> log_of_poly(kFieldSize, 0);
  uint32_t power = 1;
  for (uint32_t e = 0; e < kOneMask; ++e) {
    log_of_poly[power] = static_cast<uint16_t>(e);
    power <<= 1;
    if (power >> 16) power ^= kReductionPoly;
  }
  log_of_poly[0] = static_cast<uint16_t>(kOneMask);
  // Cantor coordinates -> polynomial element (XOR of the selected basis vectors).
  std::vector<uint16_t> poly_of(kFieldSize, 0);
  for (int bit = 0; bit < 16; ++bit) {
    const uint32_t top = 1u << bit;
    for (uint32_t low = 0; low < top; ++low) poly_of[top | low] = poly_of[low] ^ kCantorBasis[bit];
  }
  for (uint32_t a = 0; a < kFieldSize; ++a) t.log[a] = log_of_poly[poly_of[a]];
  for (uint32_t a = 0; a < kFieldSize; ++a) t.exp[t.log[a]] = static_cast<uint16_t>(a);
  t.exp[kOneMask] = t.exp[0];

  t.log_walsh = t.log;
  t.log_walsh[0] = 0;
  fwht_mod_onemask(t.log_walsh.data(), kFieldSize);
  t.lw_fold.assign(2 * static_cast<size_t>(kFieldSize), 0);
  for (uint32_t n = 1; n <= kFieldSize; n <<= 1)
    for (uint32_t j = 0; j < n; ++j) {
      uint64_t acc = 0;
      for (uint32_t h = j; h < kFieldSize; h += n) acc += t.log_walsh[h];
      t.lw_fold[n + j] = static_cast<uint16_t>(acc % kOneMask);
    }

  // Skew factors (inc_afft.rs:386-445).
  std::vector<uint16_t> sk(kFieldSize, 0);
  uint16_t basis[15];
  for (int i = 0; i < 15; ++i) basis[i] = static_cast<uint16_t>(2u << i);
  for (int m = 0; m < 15; ++m) {
    const uint32_t first = (1u << m) - 1, stride = 2u << m;
    sk[first] = 0;
    for (int i = m; i < 15; ++i) {
      const uint32_t span = 2u << i;
      for (uint32_t j = first; j < span; j += stride) sk[j + span] = sk[j] ^ basis[i];
    }
    const uint16_t prod = host_mul(t, basis[m], t.log[basis[m] ^ 1]);
    basis[m] = static_cast<uint16_t>(kOneMask - t.log[prod]);
    for (int i = m + 1; i < 15; ++i) {
      const uint32_t e = (static_cast<uint32_t>(t.log[basis[i] ^ 1]) + basis[m]) % kOneMask;
      basis[i] = host_mul(t, basis[i], static_cast<uint16_t>(e));
    }
  }
  t.skew.assign(kFieldSize, static_cast<uint16_t>(kOneMask));
  t.skew_add.assign(kFieldSize, 0);
  for (uint32_t i = 0; i < kOneMask; ++i) {
    t.skew[i] = t.log[sk[i]];
    t.skew_add[i] = sk[i];
  }

  // Multiplier lookup tables, indexed by the additive multiplier c.
  t.perm_pools.assign(static_cast<size_t>(kFieldSize) * kPermPoolWords, 0);
  for (uint32_t c = 0; c < kFieldSize; ++c)
    build_pool([&](uint16_t x) { return host_mul_add(t, x, static_cast<uint16_t>(c)); },
               &t.perm_pools[static_cast<size_t>(c) * kPermPoolWords]);

  // Tower coordinates (field_tables.hpp): beta_{8+i} = a_i + gamma e_i with
  // gamma = beta_8 and a_i, e_i in GF(2^8) (the elements whose Cantor
  // coordinates have a zero high byte).
  const uint16_t gamma = 256;
  for (int i = 0; i < 8; ++i) {
    for (uint32_t e = 0; e < 256; ++e) {
      const uint32_t rest = static_cast<uint32_t>(1u << (8 + i)) ^ host_mul_add(t, gamma, static_cast<uint16_t>(e));
      if (rest < 256) {
        t.tower_a[i] = static_cast<uint8_t>(rest);
        t.tower_e[i] = static_cast<uint8_t>(e);
        break;
      }
    }
  }
  uint8_t einv[256];  // element of GF(2^8) -> coordinates over e_0..e_7
  for (uint32_t h = 0; h < 256; ++h) {
    uint32_t el = 0;
    for (int i = 0; i < 8; ++i)
      if ((h >> i) & 1u) el ^= t.tower_e[i];
    einv[el] = static_cast<uint8_t>(h);
  }
  auto conv = [&](uint16_t x) { return to_tower(t, x); };  // an involution: T == T^-1
  t.tower_pools.assign((static_cast<size_t>(kFieldSize) + 1) * kPermPoolWords, 0);
  t.in_pools.assign(static_cast<size_t>(kFieldSize) * kPermPoolWords, 0);
  t.out_pools.assign(static_cast<size_t>(kFieldSize) * kPermPoolWords, 0);
  for (uint32_t c = 0; c < kFieldSize; ++c) {
    const uint16_t cc = static_cast<uint16_t>(c);
    const size_t at = static_cast<size_t>(c) * kPermPoolWords;
    if (c < 256) {  // c in GF(2^8): acts on (a, b) as two GF(2^8) products
      build_sub_pool([&](uint8_t a) { return static_cast<uint8_t>(host_mul_add(t, a, cc)); },
                     [&](uint8_t h) {
                       uint32_t el = 0;
                       for (int i = 0; i < 8; ++i)
                         if ((h >> i) & 1u) el ^= t.tower_e[i];
                       return einv[host_mul_add(t, static_cast<uint16_t>(el), cc)];
                     },
                     &t.tower_pools[at]);
    } else {
      build_pool([&](uint16_t x) { return conv(host_mul_add(t, conv(x), cc)); }, &t.tower_pools[at]);
    }
    build_pool([&](uint16_t x) { return conv(host_mul_add(t, x, cc)); }, &t.in_pools[at]);
    build_pool([&](uint16_t x) { return host_mul_add(t, conv(x), cc); }, &t.out_pools[at]);
  }
  t.tower_full_sub.assign(256u * kPermPoolWords, 0);
  for (uint32_t c = 0; c < 256; ++c) {
    const uint16_t cc = static_cast<uint16_t>(c);
    build_pool([&](uint16_t x) { return conv(host_mul_add(t, conv(x), cc)); },
               &t.tower_full_sub[static_cast<size_t>(c) * kPermPoolWords]);
  }
  // entry kFieldSize: the conversion's high-plane -> low-plane tables (b slots)
  build_sub_pool([](uint8_t) { return static_cast<uint8_t>(0); },
                 [&](uint8_t h) { return static_cast<uint8_t>(to_tower(t, static_cast<uint16_t>(h << 8)) & 0xff); },
                 &t.tower_pools[static_cast<size_t>(kFieldSize) * kPermPoolWords]);
}

}  // namespace

uint16_t host_mul(const HostTables& t, uint16_t a, uint16_t m) {
  if (a == 0) return 0;
  const uint32_t s = static_cast<uint32_t>(t.log[a]) + m;
  return t.exp[(s & 0xffffu) + (s >> 16)];
}

uint16_t to_tower(const HostTables& t, uint16_t x) {
  uint32_t lo = x & 0xffu;
  for (int i = 0; i < 8; ++i)
    if ((x >> (8 + i)) & 1u) lo ^= t.tower_a[i];
  return static_cast<uint16_t>((x & 0xff00u) | lo);
}

uint16_t host_mul_add(const HostTables& t, uint16_t a, uint16_t c) {
  if (a == 0 || c == 0) return 0;
  return host_mul(t, a, t.log[c]);
}

const HostTables& host_tables() {
  static HostTables tables;
  static std::once_flag once;
  std::call_once(once, [] { build(tables); });
  return tables;
}

}  // namespace np
