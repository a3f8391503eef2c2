// bates_common.h — shared pieces of the 22-score kernels (one wavefront per candidate).
#pragma once

#include "../../include/pfe.h"
#include "lm_wave.h"
#include "options.h"

namespace pfe {

#pragma clang fp contract(off)

constexpr double TWO_PI = 6.283185307179586;          // Python's 2*pi (numpy.pi * 2)
constexpr double FWHM_C = 2.3548200450309493;         // 2*sqrt(2*log(2)) as numpy computes it
// One wave (= one candidate) per workgroup: the fit lengths are heavy-tailed (median ~200,
// p90 ~900 function evaluations for the 8-parameter fit), and a multi-wave workgroup holds
// its CU slots until its slowest wave retires.
constexpr int BLOCK = 64;
constexpr int WAVES_PER_BLOCK = BLOCK / 64;

// internal status bits (not exported)
constexpr uint32_t ST_DEFER_HIST = 0x10000u;  // histogram has more bins than the kernel's slots
constexpr uint32_t ST_DEFER_HIST64 = 0x20000u;  // > 64 bins: the pooled histogram kernels pass it on
constexpr uint32_t ST_DEFER_WIDE = 0x40000u;    // > 1024 bins: queued for k_ghist_wide
constexpr uint32_t ST_GAUSS_UNSUP = 0x80000u;   // the histogram group's own PFE_ST_UNSUPPORTED
// failure bits the Gaussian chain skips a candidate on: only bits the chain sets itself, so
// its work (and every output bit, failed rows included) never depends on how far the
// concurrently running sine / DM / sub-band groups have got
constexpr uint32_t GAUSS_SKIP = PFE_ST_GAUSS_FAIL | ST_GAUSS_UNSUP;
// widest Freedman-Diaconis histogram scored (k_ghist_wide; rows in global scratch): the
// uint8 profiles of <= 256 bins need at most ~10k (range 510 over an IQR of 1/4)
constexpr int WIDE_MAX_BINS = 16384;

// per-candidate workspace passed between the Gaussian-group kernels
struct GaussWS {
  double p_mu;      // mu of the Gaussian fit to the profile histogram   (:681-682)
  double minbg;     // min(p_mu, mean(profile))                          (:724)
  double pstd;      // profile.std()
  double t1[4];     // fitGaussianT1 parameters (sigma, mu, A, bg)       (:739, :1246)
  double fd_mu;     // mu of the derivative-histogram fit (pooled histogram kernels)
  double dg[8];     // store_p1 ++ store_p2 of fitDoubleGaussian's passes 8 and 7 (:1402-1408)
  double fp_amp;    // amplitude of the profile-histogram fit (pooled histogram kernels)
  double h_min, h_max;  // profile histogram range and bin count (pooled histogram kernels)
  int hb;
};

struct BatesArgs {
  const uint8_t* prof;
  const double* fprof;  // float profiles (the PFD path, pfd22.hip) instead of prof, or null
  int lp;
  const uint8_t* sub;
  int nsub, lsb;
  const double* dmcurve;
  int ndm;
  const double* scal;
  int64_t n;
  double* out;       // n x 22
  uint32_t* status;  // n
  GaussWS* ws;       // n
  double c_lp;       // pow(lp, -0.3333333)     (ProfileOperationsInterface.py:151)
  double c_lp1;      // pow(lp-1, -0.3333333)
  unsigned* counters;  // BATES_NCOUNTERS work-queue counters, zeroed before the chain
  double* wscr;        // per-wave scratch of the persistent batched kernels
  int pwaves;          // number of persistent waves wscr is sized for
  int fpw;             // fits per wave of the batched kernels (<= BLM_FPW): small batches
                       // use fewer so that there are several waves per wave slot
  int gslots;          // fit slots per wave of the pooled kernels (<= GLM_FPW)
  int cus;             // compute units of the device
  double* hand[3];     // hand-over scratch of the pooled kernels per stream (HAND_*), or null
  int solver;          // PFE_SOLVER_* (handle option PFE_OPT_SOLVER)
  int* wide_list;      // candidates queued for k_ghist_wide (n entries)
  double* wide_scr;    // per-wave row scratch of k_ghist_wide (wide_waves slabs)
  int wide_waves;
  void* sub_work;       // scratch of the any-shape sub-band kernel (subband_work_bytes), or null
  int raw_dm;           // 1: column 17 holds getDMFittings' signed shift, not filterScore(18, .)
};

// score groups of the chain (launch_bates_groups): the ProfileOperationsInterface methods
enum : unsigned { BG_SINE = 1u, BG_GAUSS = 2u, BG_DM = 4u, BG_SUB = 8u, BG_ALL = 15u };

constexpr int BATES_NCOUNTERS = 16;
// Hand-over scratch (lm_group.h HandOver): one region per concurrently running chain, sized
// for HAND_K doubles per group lane per slot (residuals + cached model terms) and up to
// hand_waves() waves; a kernel whose functor needs more re-evaluates instead.
enum : int { HAND_GAUSS = 0, HAND_DM = 1, HAND_SINE = 2 };
constexpr int HAND_K_GAUSS = 24, HAND_K_DM = 24, HAND_K_SINE = 8;
// lanes per group of the pooled profile fits (lm_group.h): 16 up to 128 bins, 32 (8 rows per
// lane) up to 256 -- larger profiles use the batched solver
__host__ __device__ constexpr int glm_group_lanes(int lp) { return lp > 128 ? 32 : 16; }
constexpr int GLM_MAX_LP = 256;

// Side streams of a handle: the score groups that do not depend on each other run on them
// concurrently with the caller's stream (sine fits | Gaussian chain | DM fit + sub-bands), so
// one kernel's drain tail overlaps another's work.  Status bits are set with atomics.
struct Fork {
  hipStream_t side[2] = {nullptr, nullptr};
  hipEvent_t ev[3] = {nullptr, nullptr, nullptr};
  int serial = 0;  // handle option PFE_OPT_SERIAL: groups in order on the caller's stream
};
constexpr int CTR_GDG = 0;  // batch queue of k_gdgb
constexpr int BLM_FPW = 32;  // most fits per wave in the batched kernels (LDS state size)
constexpr int GLM_FPW = 32;  // fit slots per wave of the pooled group-LM kernels (lm_group.h)
static_assert(GLM_FPW == BLM_FPW, "per-wave scratch is sized by BLM_FPW");
// fit slots per wave of k_gdg8g: its SIMT phase (lmpar, one slot per lane) is the largest
// share of the 8-parameter kernel, which runs one wave per SIMD (registers), so as many slots
// as the LDS admits at 4 waves per CU: BlmState<8, 53> + slot table = 40 928 B of 40 960
// (round 6: 48 -> 53 slots, k_gdg8g 273.5 -> 271.3 ms per 1M, every output bit-identical,
// profiles/r06_ab_slots53.txt)
#ifndef PFE_GDG8_FPW
#define PFE_GDG8_FPW 53
#endif
constexpr int GDG8_FPW = PFE_GDG8_FPW;
// waves per SIMD k_gdg8g is compiled for (its registers: 1)
#ifndef PFE_GDG8_WPE
#define PFE_GDG8_WPE 1
#endif
// fit slots per wave of the 4-parameter pooled kernels k_gt1g / k_gdgg up to 128 bins (two
// waves per SIMD: BlmState<4, 44> + slot table + peel rows = 19 KB, 8 waves = 153 KB of LDS
// per CU; their SIMT phase also runs one slot per lane)
#ifndef PFE_GLM4_FPW
#define PFE_GLM4_FPW 44
#endif
constexpr int GLM4_FPW = PFE_GLM4_FPW;
// work queues of the pooled kernels (BatesArgs::counters)
constexpr int CTR_GT1G = 1, CTR_GDGG = 2, CTR_GDG8G = 3, CTR_DMG = 4, CTR_SINEG = 5, CTR_PFDDMG = 6,
              CTR_GHISTG = 7, CTR_GFIXG = 8, CTR_WIDE = 9, CTR_WIDEQ = 10;
// one k_ghist_wide wave's scratch: the rows of a 3-parameter solve (5 arrays) + the counts
constexpr size_t WIDE_SLAB_BYTES = (size_t)WIDE_MAX_BINS * (5 * sizeof(double) + sizeof(int));

// rows per lane (MPL) the kernels use for a profile of lp bins
__host__ __device__ constexpr int profile_mpl(int lp) {
  return lp <= 64 ? 1 : lp <= 128 ? 2 : lp <= 256 ? 4 : 16;
}
// per-wave scratch of k_gdgb: x and y of FPW fits, 64*MPL rows each
__host__ __device__ constexpr size_t gdg_wave_scratch_doubles(int lp) {
  return (size_t)(GLM4_FPW > BLM_FPW ? GLM4_FPW : BLM_FPW) * 64 * profile_mpl(lp) * 2;
}

// persistent waves of a pooled kernel without per-wave scratch that holds `per_simd` waves
// per SIMD: enough to fill the device, never more than the slots the batch needs
static inline dim3 pool_grid(const BatesArgs& a, int per_simd) {
  const int64_t need = (a.n + a.gslots - 1) / a.gslots;
  const int64_t cap = (int64_t)a.cus * 4 * per_simd;
  return dim3((unsigned)(need < cap ? (need > 0 ? need : 1) : cap));
}

static inline dim3 grid_for_candidates(int64_t n) {
  return dim3((unsigned)((n + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK));
}

__device__ __forceinline__ int64_t wave_candidate() {
  return ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
}

// one profile value as fp64: the uint8 PHCX row, or the float PFD row when fprof is set
// (a uniform branch on a kernel argument)
__device__ __forceinline__ double prof_at(const BatesArgs& a, int64_t idx) {
  return a.fprof ? a.fprof[idx] : (double)a.prof[idx];
}

// Profile row of candidate c into MPL slots (rows beyond lp read 0).
template <int MPL>
__device__ __forceinline__ void load_row_u8(const uint8_t* row, int len, int lane, int (&v)[MPL]) {
#pragma unroll
  for (int k = 0; k < MPL; ++k) {
    const int i = lane + 64 * k;
    v[k] = (i < len) ? (int)row[i] : 0;
  }
}

// numpy mean / std (ddof=0) of an integer row from exact integer sums.
struct MeanStd {
  double mean, std;
};
template <int MPL>
__device__ __forceinline__ MeanStd int_mean_std(const int (&v)[MPL], int len, int lane) {
  long long s1 = 0, s2 = 0;
#pragma unroll
  for (int k = 0; k < MPL; ++k)
    if (lane + 64 * k < len) {
      s1 += v[k];
      s2 += (long long)v[k] * v[k];
    }
  s1 = wsum_ll(s1);
  s2 = wsum_ll(s2);
  const double n = (double)len;
  const double mean = (double)s1 / n;
  const long long N2 = (long long)len * s2 - s1 * s1;  // exact for len*255^2*len < 2^63
  return {mean, sqrt((double)N2 / (n * n))};
}

// numpy mean / std of a distributed float vector (two-pass, tree sums)
struct FMeanStd {
  double mean, std;
};
template <int MPL>
__device__ __forceinline__ FMeanStd f_mean_std(const double (&v)[MPL], const bool (&ok)[MPL], int len) {
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < MPL; ++k)
    if (ok[k]) s += v[k];
  const double mean = wsum(s) / (double)len;
  double q = 0.0;
#pragma unroll
  for (int k = 0; k < MPL; ++k)
    if (ok[k]) {
      const double d = v[k] - mean;
      q += d * d;
    }
  return {mean, sqrt(wsum(q) / (double)len)};
}

// Python's builtin min(a, b): returns a unless b < a
__device__ __forceinline__ double py_min(double a, double b) { return (b < a) ? b : a; }

// ---- the DM-curve models' per-row arithmetic, bit-exact and cheaper -------------------------
// a / B for a constant B, correctly rounded: with Y = RN(1/B), q = RN(a Y), r = fma(-q, B, a)
// (exact) and fma(r, Y, q) = RN(a / B) by Markstein's theorem whenever nothing under- or
// overflows (|a| in [2^-900, 2^900]; tests/test_recipdiv.py checks both divisors), three
// instructions instead of an IEEE division's ~11; a row outside that range (0, inf, NaN, a
// diverging fit) takes the division -- a wave branch around it, so the common case carries
// none of the division's instructions.
#ifndef PFE_DM_DIVF3
#define PFE_DM_DIVF3 1
#endif
template <int64_t B>
__device__ __forceinline__ double div_const(double a) {
#if PFE_DM_DIVF3
  constexpr double D = (double)B, Y = 1.0 / (double)B;
  const double q = a * Y;
  double t = __builtin_fma(__builtin_fma(-q, D, a), Y, q);
  const double aa = __builtin_fabs(a);
  const bool ok = aa >= 0x1p-900 && aa <= 0x1p900;
  if (__builtin_expect(__ballot(!ok) != 0, 0)) t = ok ? t : a / D;
  return t;
#else
  return a / (double)B;
#endif
}

// the DM models' square roots: sqrt_rn (wave.h) unless PFE_DM_SQRT=0
#ifndef PFE_DM_SQRT
#define PFE_DM_SQRT 1
#endif
__device__ __forceinline__ double dm_sqrt(double x) { return PFE_DM_SQRT ? sqrt_rn(x) : sqrt(x); }

}  // namespace pfe
