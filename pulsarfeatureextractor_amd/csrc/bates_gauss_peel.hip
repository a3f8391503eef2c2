// bates_gauss_peel.hip — second stage of the Gaussian chain: the T1 fit (s8, s9) and the
// double-Gaussian peel passes (k_gt1g / k_gdgg pooled, k_gt1b / k_gdgb batched, k_gt1 /
// k_gdg wave per fit).  Kernels: bates_gauss.h.
#include "bates_gauss.h"

namespace pfe {

hipError_t launch_gauss_peel(const BatesArgs& a, hipStream_t st) {
  const int L = a.lp;
  // batched lmdif (lm_batch.h) unless the handle selects the wave-per-fit kernels
  const bool use_blm = a.solver != PFE_SOLVER_WAVE;
  const bool use_glm = a.solver == PFE_SOLVER_POOLED && L <= GLM_MAX_LP;
  const dim3 pool((unsigned)a.pwaves);
#define PFE_GAUSS_LAUNCH(P)                                                             \
  do {                                                                                  \
    if (use_glm)                                                                        \
      hipLaunchKernelGGL((k_gt1g<(P <= 4 ? P : 4)>), pool, dim3(64), 0, st, a);         \
    else if (use_blm)                                                                   \
      hipLaunchKernelGGL((k_gt1b<P>), dim3((unsigned)((a.n + a.fpw - 1) / a.fpw)),      \
                         dim3(64), 0, st, a);                                           \
    else                                                                                \
      hipLaunchKernelGGL((k_gt1<P>), gw(a.n), dim3(BLOCK), 0, st, a);                   \
    if (use_glm)                                                                        \
      hipLaunchKernelGGL((k_gdgg<(P <= 4 ? P : 4)>), pool, dim3(64), 0, st, a);         \
    else if (use_blm)                                                                   \
      hipLaunchKernelGGL((k_gdgb<P>), dim3((unsigned)a.pwaves), dim3(64), 0, st, a);    \
    else                                                                                \
      hipLaunchKernelGGL((k_gdg<P>), gw(a.n), dim3(BLOCK), 0, st, a);                   \
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

PFE_LM_PROFILE_EXPORT(gauss_peel)
