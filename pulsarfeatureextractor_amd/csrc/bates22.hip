// bates22.hip — placeholder launcher (filled in by the Bates-score kernels).
#include <hip/hip_runtime.h>
#include "../../include/pfe.h"
namespace pfe {
size_t bates22_workspace_bytes(const pfe_bates_in*) { return 0; }
hipError_t launch_bates22(const pfe_bates_in*, double*, uint32_t*, void*, size_t, hipStream_t) {
  return hipErrorNotSupported;
}
}  // namespace pfe
