// pfd.h — arguments of the PFD kernel (pfd.hip) shared with the C-ABI layer (capi.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/pfe.h"

namespace pfe {

struct PfdArgs {
  const double* profs;     // n x npart x nsub x L
  const double* subfreqs;  // n x nsub
  const double* scal;      // n x PFE_PFD_NSCAL
  int npart, nsub, L;
  int64_t n;
  double* profile;  // n x L or null
  float* chis;      // n x PFE_PFD_NDM or null
  double* lyon8;    // n x 8 or null
  uint32_t* status;
};

size_t pfd_lds_bytes(int nsub, int L);
hipError_t launch_pfd_dmprof(const PfdArgs& a, hipStream_t st);

}  // namespace pfe
