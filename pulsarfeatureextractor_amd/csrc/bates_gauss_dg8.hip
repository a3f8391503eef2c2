// bates_gauss_dg8.hip — last stage of the Gaussian chain: the 8-parameter double-Gaussian
// fit and the combination rule (s10, s11; k_gdg8g pooled, k_gdg8b batched, k_gdg8 wave per
// fit).  Kernels: bates_gauss.h.
#include "bates_gauss.h"

namespace pfe {

hipError_t launch_gauss_dg8(const BatesArgs& a, hipStream_t st) {
  const int L = a.lp;
  const bool use_blm = a.solver != PFE_SOLVER_WAVE;
  const bool use_glm = a.solver == PFE_SOLVER_POOLED && L <= GLM_MAX_LP;
  const dim3 pool((unsigned)a.pwaves);
#define PFE_GAUSS_LAUNCH(P)                                                             \
  do {                                                                                  \
    if (use_glm)                                                                        \
      hipLaunchKernelGGL((k_gdg8g<(P <= 4 ? P : 4)>), pool, dim3(64), 0, st, a);        \
    else if (use_blm)                                                                   \
      hipLaunchKernelGGL((k_gdg8b<P, BLM_FPW>), dim3((unsigned)((a.n + a.fpw - 1) / a.fpw)), \
                         dim3(64), 0, st, a);                                           \
    else                                                                                \
      hipLaunchKernelGGL((k_gdg8<P>), gw(a.n), dim3(BLOCK), 0, st, a);                  \
  } while (0)
  if (L <= 64)
    PFE_GAUSS_LAUNCH(1);
  else if (L <= 128)
    PFE_GAUSS_LAUNCH(2);
  else if (L <= 256)
    PFE_GAUSS_LAUNCH(4);
  else
    PFE_GAUSS_LAUNCH(16);
#undef PFE_GAUSS_LAUNCH
  return hipGetLastError();
}

}  // namespace pfe

PFE_LM_PROFILE_EXPORT(gauss_dg8)
