// bates_gauss.hip — the Gaussian chain's launcher (s5-s11) and its first stage: the
// Freedman-Diaconis histograms and their fits (k_ghistg / k_gfixg / k_ghist / k_ghist_wide).
// Kernels: bates_gauss.h; later stages: bates_gauss_peel.hip, bates_gauss_dg8.hip.
#include "bates_gauss.h"

namespace pfe {

hipError_t launch_gauss_hist(const BatesArgs& a, hipStream_t st) {
  const int L = a.lp;
  // pooled group-LM kernels (lm_group.h) for <= 256 bins (the default solver)
  const bool use_glm = a.solver == PFE_SOLVER_POOLED && L <= GLM_MAX_LP;
  const dim3 pool((unsigned)a.pwaves);
#define PFE_GAUSS_LAUNCH(P)                                                             \
  do {                                                                                  \
    if (use_glm && a.fprof) {                                                           \
      hipLaunchKernelGGL((k_ghistg<(P <= 4 ? P : 4), true>), pool, dim3(64), 0, st, a); \
      hipLaunchKernelGGL((k_gfixg<(P <= 4 ? P : 4), true>), pool, dim3(64), 0, st, a);  \
      hipLaunchKernelGGL((k_ghist<P, 4, false, true, true>), gw(a.n), dim3(BLOCK), 0, st, a); \
      hipLaunchKernelGGL((k_ghist<P, 16, true, true>), gw(a.n), dim3(BLOCK), 0, st, a);  \
    } else if (use_glm) {                                                               \
      hipLaunchKernelGGL((k_ghistg<(P <= 4 ? P : 4), false>), pool, dim3(64), 0, st, a); \
      hipLaunchKernelGGL((k_gfixg<(P <= 4 ? P : 4), false>), pool, dim3(64), 0, st, a);  \
      hipLaunchKernelGGL((k_ghist<P, 4, false, false, true>), gw(a.n), dim3(BLOCK), 0, st, a); \
      hipLaunchKernelGGL((k_ghist<P, 16, true, false>), gw(a.n), dim3(BLOCK), 0, st, a); \
    } else if (a.fprof) {                                                               \
      hipLaunchKernelGGL((k_ghist<P, 4, false, true>), gw(a.n), dim3(BLOCK), 0, st, a);  \
      hipLaunchKernelGGL((k_ghist<P, 16, true, true>), gw(a.n), dim3(BLOCK), 0, st, a);  \
    } else {                                                                            \
      hipLaunchKernelGGL((k_ghist<P, 4, false, false>), gw(a.n), dim3(BLOCK), 0, st, a); \
      hipLaunchKernelGGL((k_ghist<P, 16, true, false>), gw(a.n), dim3(BLOCK), 0, st, a); \
    }                                                                                   \
    /* > 1024 bins: the queue k_ghist<BIG> filled */                                    \
    if (a.fprof)                                                                        \
      hipLaunchKernelGGL((k_ghist_wide<P, true>), dim3((unsigned)a.wide_waves), dim3(64), 0, st, a); \
    else                                                                                \
      hipLaunchKernelGGL((k_ghist_wide<P, false>), dim3((unsigned)a.wide_waves), dim3(64), 0, st, a); \
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

// the whole chain, in order on one stream
hipError_t launch_gauss(const BatesArgs& a, hipStream_t st) {
  hipError_t e;
  if ((e = launch_gauss_hist(a, st)) != hipSuccess) return e;
  if ((e = launch_gauss_peel(a, st)) != hipSuccess) return e;
  return launch_gauss_dg8(a, st);
}

}  // namespace pfe

PFE_LM_PROFILE_EXPORT(gauss)
