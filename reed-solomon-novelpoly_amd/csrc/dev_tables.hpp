// Device table pointers shared by host engine and kernels (no device code here).
#pragma once
#include <cstddef>
#include <cstdint>

namespace np {

constexpr size_t kZeroPageBytes = 4096;

// Device copies of the tables of field_tables.hpp (one set per context).
struct DevTables {
  const uint16_t* log;         // 65536
  const uint16_t* exp;         // 65536
  const uint16_t* skew;        // 65536, log form, 65535 = skip
  const uint16_t* skew_add;    // 65536, additive form, 0 = skip
  const uint16_t* log_walsh;   // 65536
  const uint16_t* lw_fold;     // 2 x 65536, F_n at [n, 2n) (field_tables.hpp)
  const uint32_t* perm_pools;  // 65536 x 20 dwords (Cantor coordinates)
  // tower coordinates (field_tables.hpp HostTables::tower_pools etc.)
  const uint32_t* tower_pools;  // (65536 + 1) x 20 dwords: c < 256 subfield layout; [65536] = conversion
  const uint32_t* in_pools;     // 65536 x 20: Cantor -> tower
  const uint32_t* out_pools;    // 65536 x 20: tower -> Cantor
  const uint32_t* tower_full_sub;  // 256 x 20: the full-map layout of the subfield elements (tower -> tower)
  const uint8_t* zeros;        // kZeroPageBytes of zeros (stand-in source for absent rows)
};

}  // namespace np
