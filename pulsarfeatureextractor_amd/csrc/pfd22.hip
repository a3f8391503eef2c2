// pfd22.hip — the 22-score path for PFD files (PFDFile.compute, PFDFile.py:587-613) on gfx950.
//
// PFDFile scores a float profile (getprofile + scale, 0..255) through the same
// ProfileOperations fits as PHCX files, with PFD versions of the candidate parameters and the
// DM-curve fit (PFDOperations.py:93-393) and the sub-band scores over the dedispersed fold
// (PFDOperations.py:401-466).  The chain, on the caller's stream:
//   k_pfd_dmprof (pfd.hip)   dedispersion, profile, chi^2-vs-DM curve, s12-s15, s20-s22
//   k_sine<F>                 s1-s4 on the float profile        (bates_sine_dm_sub.hip)
//   k_ghist<F>, k_gt1b, k_gdgb, k_gdg8b   s5-s11                (bates_gauss.hip)
//   k_pfd_dmfitb              s16-s19: the clamped 4-parameter DM-curve fit (below)
#include <cmath>

#include "bates_common.h"
#include "lm_batch.h"
#include "lm_group.h"
#include "pfd.h"

namespace pfe {

#pragma clang fp contract(off)

hipError_t launch_sine(const BatesArgs& a, hipStream_t st);
hipError_t launch_gauss(const BatesArgs& a, hipStream_t st);
size_t bates22_workspace_bytes(const pfe_bates_in* in);
void bates_setup(BatesArgs& a, int64_t n, int lp, void* work, const Options& o);
void launch_clear_internal(uint32_t* status, int64_t n, hipStream_t st);
bool fork_begin(const Fork* fk, hipStream_t st);
hipError_t fork_end(const Fork* fk, hipStream_t st);

constexpr double KDM_PFD = 8.3 * 1000000.0;  // 8.3*10**6      (PFDOperations.py:342)
constexpr double DF_PFD = 32.0;              // df = 32         (:343)
constexpr double F3_PFD = 2460375.0;         // pow(135, 3), an exact integer (:344)
static_assert(F3_PFD == 2460375.0, "div_const<2460375> in PfdDMFn::weff is this divisor");

// residuals of getDMFittings (:302-310): y - (Up + Amp*sqrt((P - w)/w)), w clamped to P
template <int MPL>
struct PfdDMFn {
  double x[MPL], y[MPL];
  bool ok[MPL];
  double wint, dm, period;
  __device__ __forceinline__ double weff(double prop, double shift, int k) const {
    const double t = div_const<2460375LL>(prop * KDM_PFD * fabs((dm + shift) - x[k]) * DF_PFD);
    double w = dm_sqrt(wint + t * t);
    if (w > period) w = period;                                        // :305-307
    return w;
  }
  __device__ __forceinline__ double model(const double (&p)[4], int k) const {
    const double w = weff(p[1], p[2], k);
    return p[3] + p[0] * dm_sqrt((period - w) / w);                    // :308
  }
  __device__ __forceinline__ void operator()(const double (&p)[4], double (&f)[MPL]) const {
#pragma unroll
    for (int k = 0; k < MPL; ++k) f[k] = ok[k] ? y[k] - model(p, k) : 0.0;
  }
};

struct PfdDMArgs {
  BatesArgs a;
  const float* chis;  // n x PFE_PFD_NDM
};

// the fit data of candidate c (:322-352): yData = 255./max(chis)*chis in float32 (numpy's
// scalar rules, as the reference runs under the numpy this build is pinned against)
__device__ __forceinline__ float pfd_dm_scale(const PfdDMArgs& d, int64_t c) {
  const float* ch = d.chis + c * PFE_PFD_NDM;
  float m = ch[0];  // Python max() over the float32 array
  for (int i = 1; i < PFE_PFD_NDM; ++i)
    if (ch[i] > m) m = ch[i];
  return 255.0f / m;
}

// rows i = lb + STRIDE*k: the wave layout (lane, 64) or the group layout (glane, 16); s is
// pfd_dm_scale(d, c)
template <int MPL, int STRIDE = 64>
__device__ __forceinline__ void pfd_dm_functor(const PfdDMArgs& d, int64_t c, PfdDMFn<MPL>& fn,
                                               float s, int lb = lane_id()) {
  const double* q = d.a.scal + c * 8;
  const float* ch = d.chis + c * PFE_PFD_NDM;
  const double dm_start = q[4], dm_end = q[5];
  const double step = fabs(dm_start - dm_end) / (double)PFE_PFD_NDM;   // :338
  fn.period = q[0];
  fn.dm = q[2];
  fn.wint = (q[3] * q[0]) * (q[3] * q[0]);                              // :341
#pragma unroll
  for (int k = 0; k < MPL; ++k) {
    const int i = lb + STRIDE * k;
    fn.ok[k] = i < PFE_PFD_NDM;
    fn.y[k] = fn.ok[k] ? (double)(s * ch[fn.ok[k] ? i : 0]) : 0.0;
    fn.x[k] = dm_start + (double)i * step;                              // :349-352
  }
}

// the theoretical curve (:355-366); false = 255./max(_help) divides by zero
template <int MPL>
__device__ __forceinline__ bool pfd_dm_theo(const PfdDMFn<MPL>& fn, double (&theo)[MPL],
                                            double& amp0) {
  double help[MPL];
  double hmax = -INFINITY;
#pragma unroll
  for (int k = 0; k < MPL; ++k) {
    const double t = KDM_PFD * fabs(fn.dm - fn.x[k]) * DF_PFD / F3_PFD;
    double w = sqrt(fn.wint + t * t);
    if (w > fn.period) w = fn.period;
    help[k] = sqrt((fn.period - w) / w);
    if (fn.ok[k]) hmax = fmax(hmax, help[k]);
  }
  hmax = wmax(hmax);
  const double h0 = bcast(help[0], 0);  // Python max(): a leading NaN wins
  if (h0 != h0) hmax = h0;
  if (hmax == 0.0) return false;
  amp0 = 255.0 / hmax;
#pragma unroll
  for (int k = 0; k < MPL; ++k) theo[k] = amp0 * help[k];
  return true;
}

template <int MPL>
struct PfdDMLoader {
  PfdDMArgs d;
  int64_t base;
  __device__ __forceinline__ PfdDMFn<MPL> operator()(int f) const {
    PfdDMFn<MPL> fn;
    pfd_dm_functor<MPL>(d, base + f, fn, pfd_dm_scale(d, base + f));
    return fn;
  }
};

// s16-s19 (:346, :377-393): chi^2 of the theoretical curve over the bins where it is > 0,
// a Python loop (sequential, lane 0 over LDS terms)
template <int MPL, int FPW>
__global__ __launch_bounds__(64) void k_pfd_dmfitb(PfdDMArgs d) {
  __shared__ BlmState<4, FPW> S;
  __shared__ double term[64 * MPL];
  __shared__ int used[64 * MPL];
  const BatesArgs& a = d.a;
  const int64_t base = (int64_t)blockIdx.x * a.fpw;
  const int lane = lane_id();
  bool live = false;
  if (lane < a.fpw && base + lane < a.n) {
    uint32_t* st = a.status + base + lane;
    if (*st & PFE_ST_PFD_DMCURVE_FAIL) {  // numdms == 1: dms[0] raises in getDMFittings
      atomicAnd(st, ~(uint32_t)PFE_ST_PFD_DMCURVE_FAIL);  // (other score groups may be
      atomicOr(st, (uint32_t)PFE_ST_DMFIT_FAIL);           // updating status concurrently)
    } else
      live = true;
  }
  uint64_t fits = __ballot(live);
  if (fits == 0) return;
  for (uint64_t m = fits; m; m &= m - 1) {
    const int f = __builtin_ctzll(m);
    PfdDMFn<MPL> fn;
    pfd_dm_functor<MPL>(d, base + f, fn, pfd_dm_scale(d, base + f));
    double theo[MPL], amp0 = 0.0;
    if (!pfd_dm_theo<MPL>(fn, theo, amp0)) {  // ZeroDivisionError
      if (lane == 0) atomicOr(&a.status[base + f], (uint32_t)(PFE_ST_DMFIT_FAIL));
      fits &= ~(1ull << f);
      continue;
    }
    if (lane == 0) {
      S.x[0][f] = amp0;
      S.x[1][f] = 1.0;
      S.x[2][f] = 0.0;
      S.x[3][f] = 0.0;
    }
  }
  if (fits == 0) return;
  const PfdDMLoader<MPL> load{d, base};
  blm_run<4, MPL, FPW>(load, S, fits, 200 * 5);
  for (uint64_t m = fits; m; m &= m - 1) {
    const int f = __builtin_ctzll(m);
    const int64_t c = base + f;
    PfdDMFn<MPL> fn;
    pfd_dm_functor<MPL>(d, c, fn, pfd_dm_scale(d, c));
    double theo[MPL], amp0 = 0.0;
    pfd_dm_theo<MPL>(fn, theo, amp0);
#pragma unroll
    for (int k = 0; k < MPL; ++k) {
      const int i = lane + 64 * k;
      if (fn.ok[k]) {
        const double dd = fn.y[k] - theo[k];
        used[i] = theo[k] > 0.0;                                        // :381
        term[i] = (dd * dd) / theo[k];                                  // :383
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) {
      const double* q = a.scal + c * 8;
      const double period = q[0], snr = q[1];
      const double wint = fn.wint;
      double chi = 0.0;
      int ndeg = 0;
      for (int i = 0; i < PFE_PFD_NDM; ++i)
        if (used[i]) {
          chi += term[i];
          ++ndeg;
        }
      double* o = a.out + c * 22;
      o[15] = snr / sqrt((period - sqrt(wint)) / sqrt(wint));          // s16 (:346)
      o[16] = fabs(1.0 - S.x[1][f]);                                   // s17 (:391)
      o[17] = fabs(S.x[2][f]);                                         // s18, filterScore(18)
      o[18] = ndeg ? chi / (double)ndeg : 0.0;                         // s19 (:387)
      if (!ndeg) atomicOr(&a.status[c], (uint32_t)(PFE_ST_DMFIT_FAIL));                     // ZeroDivisionError
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

// s16-s19 of candidate c after the fit (whole wave): chi^2 of the theoretical curve over
// the bins where it is > 0, a Python loop (sequential, lane 0 over LDS terms)
template <int MPL>
__device__ __forceinline__ void pfd_dm_finish(const PfdDMArgs& d, int64_t c, double prop,
                                              double shift, double* term, int* used) {
  const BatesArgs& a = d.a;
  const int lane = lane_id();
  PfdDMFn<MPL> fn;
  pfd_dm_functor<MPL>(d, c, fn, pfd_dm_scale(d, c));
  double theo[MPL], amp0 = 0.0;
  pfd_dm_theo<MPL>(fn, theo, amp0);
#pragma unroll
  for (int k = 0; k < MPL; ++k) {
    const int i = lane + 64 * k;
    if (fn.ok[k]) {
      const double dd = fn.y[k] - theo[k];
      used[i] = theo[k] > 0.0;                                        // :381
      term[i] = (dd * dd) / theo[k];                                  // :383
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if (lane == 0) {
    const double* q = a.scal + c * 8;
    const double period = q[0], snr = q[1];
    const double wint = fn.wint;
    double chi = 0.0;
    int ndeg = 0;
    for (int i = 0; i < PFE_PFD_NDM; ++i)
      if (used[i]) {
        chi += term[i];
        ++ndeg;
      }
    double* o = a.out + c * 22;
    o[15] = snr / sqrt((period - sqrt(wint)) / sqrt(wint));          // s16 (:346)
    o[16] = fabs(1.0 - prop);                                        // s17 (:391)
    o[17] = fabs(shift);                                             // s18, filterScore(18)
    o[18] = ndeg ? chi / (double)ndeg : 0.0;                         // s19 (:387)
    if (!ndeg) atomicOr(&a.status[c], (uint32_t)(PFE_ST_DMFIT_FAIL));                     // ZeroDivisionError
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// pooled group-LM form (lm_group.h) of the clamped 4-parameter DM fit
template <int MPL, int FPW>
struct PfdDMProb {
  static constexpr int MG = 4 * MPL;
  PfdDMArgs d;
  SlotTab<FPW>& T;  // d0 = 255/max(chis) of the slot's candidate
  double* term;
  int* used;
  int nslots;
  __device__ __forceinline__ bool refill(int f, BlmState<4, FPW>& S) {
    const BatesArgs& a = d.a;
    const int lane = lane_id();
    const int64_t c0 = T.cand[f];
    if (c0 >= 0) pfd_dm_finish<MPL>(d, c0, S.x[1][f], S.x[2][f], term, used);
    if (f < nslots) {
      for (;;) {
        const int64_t c = queue_next(a.counters + CTR_PFDDMG);
        if (c >= a.n) break;
        const uint32_t st = a.status[c];
        if (st & PFE_ST_PFD_DMCURVE_FAIL) {  // numdms == 1: dms[0] raises in getDMFittings
          if (lane == 0) {
            atomicAnd(&a.status[c], ~(uint32_t)PFE_ST_PFD_DMCURVE_FAIL);
            atomicOr(&a.status[c], (uint32_t)PFE_ST_DMFIT_FAIL);
          }
          continue;
        }
        const float sc = pfd_dm_scale(d, c);
        PfdDMFn<MPL> fn;
        pfd_dm_functor<MPL>(d, c, fn, sc);
        double theo[MPL], amp0 = 0.0;
        if (!pfd_dm_theo<MPL>(fn, theo, amp0)) {  // ZeroDivisionError
          if (lane == 0) atomicOr(&a.status[c], (uint32_t)(PFE_ST_DMFIT_FAIL));
          continue;
        }
        if (lane == 0) {
          T.cand[f] = c;
          T.d0[f] = (double)sc;
          S.x[0][f] = amp0;
          S.x[1][f] = 1.0;
          S.x[2][f] = 0.0;
          S.x[3][f] = 0.0;
        }
        blm_sync();
        return true;
      }
    }
    if (lane == 0) T.cand[f] = -1;
    blm_sync();
    return false;
  }
  __device__ __forceinline__ PfdDMFn<MG> load(int f) const {
    PfdDMFn<MG> fn;
    pfd_dm_functor<MG, GLM_G>(d, T.cand[f], fn, (float)T.d0[f], glane());
    return fn;
  }
  __device__ __forceinline__ int maxfev(int) const { return 200 * 5; }
};

template <int MPL>
__global__ __launch_bounds__(64, 2) void k_pfd_dmfitg(PfdDMArgs d) {
  constexpr int FPW = GLM_FPW;
  __shared__ BlmState<4, FPW> S;
  __shared__ SlotTab<FPW> T;
  __shared__ double term[64 * MPL];
  __shared__ int used[64 * MPL];
  if (lane_id() < FPW) T.cand[lane_id()] = -1;
  blm_sync();
  PfdDMProb<MPL, FPW> prob{d, T, term, used, d.a.gslots};
  glm_engine<4, 4 * MPL, FPW>(prob, S, T.ph, T.list, d.a.hand[HAND_DM], HAND_K_DM);
}

size_t pfd22_workspace_bytes(int64_t n, int L) {
  pfe_bates_in in{};
  in.n = n;
  in.lp = L;
  const size_t al = 255;
  return bates22_workspace_bytes(&in) + ((size_t)n * L * sizeof(double) + al) +
         ((size_t)n * PFE_PFD_NDM * sizeof(float) + al) + ((size_t)n * 8 * sizeof(double) + al) +
         256;
}

static char* carve(char*& p, size_t bytes) {
  char* r = (char*)(((uintptr_t)p + 255) & ~(uintptr_t)255);
  p = r + bytes;
  return r;
}

// pa: the PFD inputs (profs, subfreqs, scal, shape, n); out n x 22, status n (device)
hipError_t launch_pfd22(PfdArgs pa, double* out, uint32_t* status, void* work, size_t work_bytes,
                        hipStream_t st, const Fork* fk, const Options& o) {
  const int64_t n = pa.n;
  const int L = pa.L;
  if (work_bytes < pfd22_workspace_bytes(n, L)) return hipErrorInvalidValue;
  char* p = (char*)work;
  double* profile = (double*)carve(p, (size_t)n * L * sizeof(double));
  float* chis = (float*)carve(p, (size_t)n * PFE_PFD_NDM * sizeof(float));
  double* par22 = (double*)carve(p, (size_t)n * 8 * sizeof(double));
  char* bwork = carve(p, 0);
  hipError_t e = hipMemsetAsync(out, 0, (size_t)n * 22 * sizeof(double), st);
  if (e != hipSuccess) return e;
  pa.profile = profile;
  pa.chis = chis;
  pa.lyon8 = nullptr;
  pa.status = status;
  pa.out22 = out;
  pa.par22 = par22;
  if ((e = launch_pfd_dmprof(pa, st)) != hipSuccess) return e;
  BatesArgs a;
  bates_setup(a, n, L, bwork, o);
  a.prof = nullptr;
  a.fprof = profile;
  a.sub = nullptr;
  a.nsub = 0;
  a.lsb = 0;
  a.dmcurve = nullptr;
  a.ndm = PFE_PFD_NDM;
  a.scal = par22;
  a.out = out;
  a.status = status;
  e = hipMemsetAsync(a.counters, 0, BATES_NCOUNTERS * sizeof(unsigned), st);
  if (e != hipSuccess) return e;
  const bool forked = fork_begin(fk, st);
  const hipStream_t sg = forked ? fk->side[0] : st, sd = forked ? fk->side[1] : st;
  if ((e = launch_gauss(a, sg)) != hipSuccess) return e;
  const PfdDMArgs d{a, chis};
  if (a.solver == PFE_SOLVER_POOLED)  // pooled group-LM unless the handle selects another solver
    hipLaunchKernelGGL((k_pfd_dmfitg<2>), dim3((unsigned)a.pwaves), dim3(64), 0, sd, d);
  else
    hipLaunchKernelGGL((k_pfd_dmfitb<2, BLM_FPW>), dim3((unsigned)((n + a.fpw - 1) / a.fpw)),
                       dim3(64), 0, sd, d);
  if ((e = launch_sine(a, st)) != hipSuccess) return e;
  if (forked && (e = fork_end(fk, st)) != hipSuccess) return e;
  launch_clear_internal(status, n, st);
  return hipGetLastError();
}

}  // namespace pfe

PFE_LM_PROFILE_EXPORT(pfd22)
