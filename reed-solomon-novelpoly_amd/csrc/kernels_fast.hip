// Specialised gfx950 kernels (filled in below the generic path).
#include "device_common.hpp"
#include "launchers.hpp"

namespace np {
bool fast_encode_supported(uint32_t, uint32_t) { return false; }
bool fast_reconstruct_supported(uint32_t, uint32_t) { return false; }
hipError_t launch_encode_fast(const DevTables&, const EncodeArgs&, hipStream_t) { return hipErrorNotSupported; }
hipError_t launch_reconstruct_fast(const DevTables&, const ReconstructArgs&, hipStream_t) {
  return hipErrorNotSupported;
}
hipError_t configure_fast_kernels() { return hipSuccess; }
}  // namespace np
