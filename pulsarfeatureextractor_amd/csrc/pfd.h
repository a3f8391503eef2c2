// pfd.h — arguments of the PFD kernel (pfd.hip) shared with the C-ABI layer (capi.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/pfe.h"
#include "options.h"

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
  // the 22-score path (pfd22.hip): scores 12-15 and 20-22 into out22 (n x 22), and the
  // DM-fit inputs [period, snr, dm, width, dm_start, dm_end] into par22 (n x 8); both or none
  double* out22 = nullptr;
  double* par22 = nullptr;
  int waves = 4;  // handle option PFE_OPT_PFD_WAVES: the four-wave kernel (<= 128 bins) or one wave
  // the folds' part sums T (n x nsub x L, k_pfd_parts) read from global memory instead of
  // reduced in the kernel (split pipeline), or null (fused)
  const double* tin = nullptr;
};

// split pipeline of pfe_pfd_dmprof: k_pfd_parts streams chunks of `chunk` folds' part sums
// into the two halves of ws (2 x chunk x nsub x L doubles) on `side` while k_pfd_dmprof4
// sweeps the previous chunk on `st`; ev: four events (two per buffer).  False when the
// shape takes the fused kernels (> 128 bins or the four-wave LDS limit).
bool pfd_split_ok(const PfdArgs& a);
hipError_t launch_pfd_dmprof_split(const PfdArgs& a, hipStream_t st, hipStream_t side, double* ws,
                                   int64_t chunk, hipEvent_t (&ev)[4]);

size_t pfd_lds_bytes(int nsub, int L);
hipError_t launch_pfd_dmprof(const PfdArgs& a, hipStream_t st);
// the 22-score chain (pfd22.hip); work: pfd22_workspace_bytes(n, L) bytes of device memory
size_t pfd22_workspace_bytes(int64_t n, int L);
struct Fork;
hipError_t launch_pfd22(PfdArgs a, double* out, uint32_t* status, void* work, size_t work_bytes,
                        hipStream_t st, const Fork* fk, const Options& o);

}  // namespace pfe
