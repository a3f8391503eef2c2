// lm_wave.h — MINPACK lmdif (Levenberg-Marquardt, forward-difference Jacobian) for one
// wavefront, as used by scipy.optimize.leastsq (the reference's only optimiser,
// ProfileOperations.py:449,549,949,1045,1246,1379,1473; PHCXOperations.py:212).
//
// Restated from the published MINPACK-1 algorithm (More, Garbow, Hillstrom 1980: lmdif,
// fdjac2, qrfac, lmpar, qrsolv, enorm) with scipy's leastsq defaults:
//   ftol = xtol = 1.49012e-8, gtol = 0, maxfev = 200*(n+1), epsfcn = DBL_EPSILON,
//   factor = 100, mode = 1 (diag from the column norms of the first Jacobian).
//
// Parallel decomposition (one candidate per wave):
//   * the m residuals / Jacobian rows are spread over the 64 lanes, MPL rows per lane
//     (row i -> lane i%64, slot i/64): function evaluations, forward differences, the
//     Householder updates of qrfac and Q^T f are lane-parallel, every dot product / norm
//     over rows is a wave reduction (DPP butterflies, identical result in all lanes);
//   * the n-sized state (x, diag, qtf, R, ipvt, lmpar/qrsolv) is replicated in every lane
//     and updated with identical arithmetic, so all control flow is wave-uniform.
// Differences from a sequential MINPACK: sums over the m rows are formed in tree order
// (last-bit differences), n-vector norms follow MINPACK's enorm exactly.
#pragma once

#include "wave.h"

// The solver's own linear algebra (qrfac, Q^T f, lmpar, qrsolv, the norms) is contracted
// into fused multiply-adds: these sums run in another order than MINPACK's sequential loops
// anyway (tree sums over the m rows), so their last bits are not the reference's either way,
// and an FMA shortens the serial dependency chains of qrsolv / lmpar (one slot per lane).
// The residual models and every bit-exact score keep -ffp-contract=off (numpy evaluates each
// operation rounded).  -DPFE_LA_NOFMA restores the uncontracted solver (A/B builds).
// For the same reason the quotients by one per-column divisor (the forward-difference step h
// of fdjac2, the Householder norm of qrfac and its column updates, lmpar's dxnorm, the gtol
// test's fnorm) are products with its reciprocal, qrsolv's Givens rotations take 0.5 *
// rsqrt, qrfac's norm-loss test compares squares, and enorm of an n-vector whose elements all
// lie in MINPACK's intermediate range is sqrt(sum x^2) without per-element branches.
#ifdef PFE_LA_NOFMA
#define PFE_LA_CONTRACT
constexpr bool LA_EXACT_QUOTIENTS = true;
#else
#define PFE_LA_CONTRACT _Pragma("clang fp contract(fast)")
constexpr bool LA_EXACT_QUOTIENTS = false;
#endif

namespace pfe {

constexpr double LM_FTOL = 1.49012e-08;
constexpr double LM_XTOL = 1.49012e-08;
constexpr double LM_GTOL = 0.0;
constexpr double LM_FACTOR = 100.0;
constexpr double EPSMCH = 2.220446049250313e-16;
constexpr double DWARF = 2.2250738585072014e-308;

// x / d of the solver's linear algebra, given rinv = 1 / d (see LA_EXACT_QUOTIENTS)
__device__ __forceinline__ double la_quot(double x, double d, double rinv) {
  return LA_EXACT_QUOTIENTS ? x / d : x * rinv;
}
// qrfac's test that a downdated column norm lost too much to be trusted,
// 0.05 (rdiag / wa)^2 <= epsmch: without the quotient in the contracted build (wa > 0)
__device__ __forceinline__ bool la_norm_lost(double rdiag, double wa) {
  if (LA_EXACT_QUOTIENTS) {
    const double q = rdiag / wa;
    return 0.05 * (q * q) <= EPSMCH;
  }
  return 0.05 * (rdiag * rdiag) <= EPSMCH * (wa * wa);
}
// 0.5 / sqrt(t) of qrsolv's Givens rotations (t in [0.25, 0.5]): 0.5 * rsqrt(t) in the
// contracted build
__device__ __forceinline__ double la_half_rsqrt(double t) {
  return LA_EXACT_QUOTIENTS ? 0.5 / sqrt(t) : 0.5 * rsqrt(t);
}

// ---- optional phase-cycle profiler (instrumented builds only: -DPFE_LM_PROFILE) ----------
// Per translation unit, per parameter count N (slot 0..3 for N = 2, 3, 4, 8): counters
//   0 lmdif calls, 1 outer iterations, 2 lmpar calls, 3 qrsolv calls, 4 function evaluations,
//   5 fdjac2 cycles, 6 qrfac cycles, 7 Q^T f / R / gnorm cycles, 8 lmpar cycles,
//   9 trial evaluation cycles, 10 total lmdif cycles
#ifdef PFE_LM_PROFILE
// (single global counter set: the atomics of many resident waves contend on it, so absolute
// cycle counts are inflated; use the ratios and the event counts)
static __device__ unsigned long long pfe_lm_prof[4][16];
__device__ __forceinline__ long long lm_clock() { return clock64(); }
template <int N>
__device__ __forceinline__ void lm_prof_add(int k, long long v) {
  constexpr int slot = N == 2 ? 0 : N == 3 ? 1 : N == 4 ? 2 : 3;
  if (lane_id() == 0) atomicAdd(&pfe_lm_prof[slot][k], (unsigned long long)v);
}
#define PFE_LM_PROFILE_EXPORT(tag)                                                      \
  extern "C" int pfe_lmprof_##tag(unsigned long long* out, int reset) {                 \
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(pfe::pfe_lm_prof), sizeof(pfe::pfe_lm_prof)) != \
        hipSuccess)                                                                     \
      return -1;                                                                        \
    if (reset) {                                                                        \
      static unsigned long long z[4][16];                                               \
      if (hipMemcpyToSymbol(HIP_SYMBOL(pfe::pfe_lm_prof), z, sizeof(z)) != hipSuccess)  \
        return -1;                                                                      \
    }                                                                                   \
    return 0;                                                                           \
  }
#define LM_T0(v) const long long v = lm_clock()
#define LM_ADD(k, v) lm_prof_add<N>((k), (v))
__device__ __forceinline__ long long lm_clock_p() { return clock64(); }
#else
#define PFE_LM_PROFILE_EXPORT(tag)
#define LM_T0(v) \
  do {           \
  } while (0)
#define LM_ADD(k, v) \
  do {               \
  } while (0)
__device__ __forceinline__ long long lm_clock_p() { return 0; }
#endif

// MINPACK enorm of a replicated n-vector (sequential, with the dwarf/giant scaling)
template <int N>
__device__ __forceinline__ double enorm_u(const double (&x)[N]) {
  PFE_LA_CONTRACT
  const double rdwarf = 3.834e-20, rgiant = 1.304e19;
  const double agiant = rgiant / (double)N;
  if constexpr (!LA_EXACT_QUOTIENTS) {
    // every non-zero element in MINPACK's intermediate range (the common case): enorm is
    // sqrt(sum x^2) there, with no per-element branches
    double s = 0.0;
    bool mid = true;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const double xabs = fabs(x[i]);
      s += xabs * xabs;
      mid = mid && ((xabs > rdwarf && xabs < agiant) || xabs == 0.0);
    }
    if (mid) return sqrt(s);
  }
  double s1 = 0, s2 = 0, s3 = 0, x1max = 0, x3max = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const double xabs = fabs(x[i]);
    if (xabs > rdwarf && xabs < agiant) {
      s2 += xabs * xabs;
    } else if (xabs <= rdwarf) {
      if (xabs > x3max) {
        const double r = x3max / xabs;
        s3 = 1.0 + s3 * (r * r);
        x3max = xabs;
      } else if (xabs != 0.0) {
        const double r = xabs / x3max;
        s3 += r * r;
      }
    } else {
      if (xabs > x1max) {
        const double r = x1max / xabs;
        s1 = 1.0 + s1 * (r * r);
        x1max = xabs;
      } else {
        const double r = xabs / x1max;
        s1 += r * r;
      }
    }
  }
  if (s1 != 0.0) return x1max * sqrt(s1 + (s2 / x1max) / x1max);
  if (s2 != 0.0) {
    if (s2 >= x3max) return sqrt(s2 * (1.0 + (x3max / s2) * (x3max * s3)));
    return sqrt(x3max * ((s2 / x3max) + (x3max * s3)));
  }
  return x3max * sqrt(s3);
}

// Euclidean norm of a distributed m-vector (rows outside [0,m) must hold 0)
template <int MPL>
__device__ __forceinline__ double enorm_w(const double (&f)[MPL]) {
  PFE_LA_CONTRACT
  double p = 0.0;
#pragma unroll
  for (int k = 0; k < MPL; ++k) p += f[k] * f[k];
  return sqrt(wsum(p));
}

// row i = lane + 64*k is >= j (j < 64)
__device__ __forceinline__ bool row_ge(int lane, int k, int j) { return k > 0 || lane >= j; }

// ---- qrfac (pivot = true) on the distributed m x N matrix a -------------------------------
template <int N, int MPL>
__device__ __forceinline__ void qrfac(double (&a)[MPL][N], int (&ipvt)[N], double (&rdiag)[N], double (&acnorm)[N]) {
  PFE_LA_CONTRACT
  const int lane = lane_id();
  double wa[N];
  {
    double s[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
      double p = 0.0;
#pragma unroll
      for (int k = 0; k < MPL; ++k) p += a[k][j] * a[k][j];
      s[j] = p;
    }
    wsum_arr(s);
#pragma unroll
    for (int j = 0; j < N; ++j) {
      acnorm[j] = sqrt(s[j]);
      rdiag[j] = acnorm[j];
      wa[j] = acnorm[j];
      ipvt[j] = j;
    }
  }
#pragma unroll
  for (int j = 0; j < N; ++j) {
    // bring the column of largest norm into the pivot position
    int kmax = j;
    double rmax = rdiag[j];
#pragma unroll
    for (int k = j + 1; k < N; ++k)
      if (rdiag[k] > rmax) {
        kmax = k;
        rmax = rdiag[k];
      }
    if (kmax != j) {
#pragma unroll
      for (int k2 = j + 1; k2 < N; ++k2) {
        if (kmax == k2) {
#pragma unroll
          for (int s = 0; s < MPL; ++s) {
            const double t = a[s][j];
            a[s][j] = a[s][k2];
            a[s][k2] = t;
          }
          rdiag[k2] = rdiag[j];
          wa[k2] = wa[j];
          const int t = ipvt[j];
          ipvt[j] = ipvt[k2];
          ipvt[k2] = t;
        }
      }
    }
    // Householder transformation reducing column j to a multiple of e_j
    double p = 0.0;
#pragma unroll
    for (int k = 0; k < MPL; ++k)
      if (row_ge(lane, k, j)) p += a[k][j] * a[k][j];
    double ajnorm = sqrt(wsum(p));
    if (ajnorm != 0.0) {
      if (bcast(a[0][j], j) < 0.0) ajnorm = -ajnorm;
      const double rinv = 1.0 / ajnorm;
#pragma unroll
      for (int k = 0; k < MPL; ++k)
        if (row_ge(lane, k, j)) a[k][j] = la_quot(a[k][j], ajnorm, rinv);
      if (lane == j) a[0][j] = a[0][j] + 1.0;
      if constexpr (true) {
        double d[N];
#pragma unroll
        for (int c = 0; c < N; ++c) {
          double q = 0.0;
          if (c > j) {
#pragma unroll
            for (int k = 0; k < MPL; ++k)
              if (row_ge(lane, k, j)) q += a[k][j] * a[k][c];
          }
          d[c] = q;
        }
        wsum_from(d, j + 1);
        const double ajj = bcast(a[0][j], j);
        const double rajj = 1.0 / ajj;
#pragma unroll
        for (int c = j + 1; c < N; ++c) {
          const double temp = la_quot(d[c], ajj, rajj);
#pragma unroll
          for (int k = 0; k < MPL; ++k)
            if (row_ge(lane, k, j)) a[k][c] = a[k][c] - temp * a[k][j];
          if (rdiag[c] != 0.0) {
            const double t2 = bcast(a[0][c], j) / rdiag[c];
            rdiag[c] = rdiag[c] * sqrt(fmax(0.0, 1.0 - t2 * t2));
            if (la_norm_lost(rdiag[c], wa[c])) {
              double r = 0.0;
#pragma unroll
              for (int k = 0; k < MPL; ++k)
                if (row_ge(lane, k, j + 1)) r += a[k][c] * a[k][c];
              rdiag[c] = sqrt(wsum(r));
              wa[c] = rdiag[c];
            }
          }
        }
      }
    }
    rdiag[j] = -ajnorm;
  }
}

// ---- qrsolv (replicated n x n) --------------------------------------------------------
template <int N>
__device__ __forceinline__ void qrsolv(double (&r)[N][N], const int (&ipvt)[N],
                                       const double (&diag)[N], const double (&qtb)[N],
                                       double (&x)[N], double (&sdiag)[N]) {
  PFE_LA_CONTRACT
  double wa[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
#pragma unroll
    for (int i = j; i < N; ++i) r[i][j] = r[j][i];
    x[j] = r[j][j];
    wa[j] = qtb[j];
  }
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const double dl = sel(diag, ipvt[j]);
    if (dl != 0.0) {
#pragma unroll
      for (int k = j; k < N; ++k) sdiag[k] = 0.0;
      sdiag[j] = dl;
      double qtbpj = 0.0;
#pragma unroll
      for (int k = j; k < N; ++k) {
        if (sdiag[k] != 0.0) {
          double sn, cs;
          if (fabs(r[k][k]) < fabs(sdiag[k])) {
            const double cotan = r[k][k] / sdiag[k];
            sn = la_half_rsqrt(0.25 + 0.25 * (cotan * cotan));
            cs = sn * cotan;
          } else {
            const double tn = sdiag[k] / r[k][k];
            cs = la_half_rsqrt(0.25 + 0.25 * (tn * tn));
            sn = cs * tn;
          }
          r[k][k] = cs * r[k][k] + sn * sdiag[k];
          const double temp = cs * wa[k] + sn * qtbpj;
          qtbpj = -sn * wa[k] + cs * qtbpj;
          wa[k] = temp;
#pragma unroll
          for (int i = k + 1; i < N; ++i) {
            const double t = cs * r[i][k] + sn * sdiag[i];
            sdiag[i] = -sn * r[i][k] + cs * sdiag[i];
            r[i][k] = t;
          }
        }
      }
    }
    sdiag[j] = r[j][j];
    r[j][j] = x[j];
  }
  int nsing = N;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    if (sdiag[j] == 0.0 && nsing == N) nsing = j;
    if (nsing < N) wa[j] = 0.0;
  }
#pragma unroll
  for (int j = N - 1; j >= 0; --j) {
    if (j < nsing) {
      double sum = 0.0;
#pragma unroll
      for (int i = j + 1; i < N; ++i)
        if (i < nsing) sum += r[i][j] * wa[i];
      wa[j] = (wa[j] - sum) / sdiag[j];
    }
  }
#pragma unroll
  for (int j = 0; j < N; ++j) put(x, ipvt[j], wa[j]);
}

// ---- lmpar (replicated) -----------------------------------------------------------------
// MINPACK's lmpar step for step (the uncontracted build's; lmpar below)
template <int N>
__device__ __forceinline__ void lmpar_literal(double (&r)[N][N], const int (&ipvt)[N],
                                              const double (&diag)[N], const double (&qtb)[N],
                                              double delta, double& par, double (&x)[N],
                                              double (&sdiag)[N]) {
  PFE_LA_CONTRACT
  double wa1[N], wa2[N];
  int nsing = N;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    wa1[j] = qtb[j];
    if (r[j][j] == 0.0 && nsing == N) nsing = j;
    if (nsing < N) wa1[j] = 0.0;
  }
#pragma unroll
  for (int j = N - 1; j >= 0; --j) {
    if (j < nsing) {
      wa1[j] = wa1[j] / r[j][j];
      const double temp = wa1[j];
#pragma unroll
      for (int i = 0; i < j; ++i) wa1[i] = wa1[i] - r[i][j] * temp;
    }
  }
#pragma unroll
  for (int j = 0; j < N; ++j) put(x, ipvt[j], wa1[j]);
  int iter = 0;
#pragma unroll
  for (int j = 0; j < N; ++j) wa2[j] = diag[j] * x[j];
  double dxnorm = enorm_u(wa2);
  double fp = dxnorm - delta;
  if (fp <= 0.1 * delta) {
    par = 0.0;  // iter == 0
    return;
  }
  double parl = 0.0;
  if (nsing >= N) {
    const double rdx = 1.0 / dxnorm;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const int l = ipvt[j];
      wa1[j] = sel(diag, l) * la_quot(sel(wa2, l), dxnorm, rdx);
    }
#pragma unroll
    for (int j = 0; j < N; ++j) {
      double sum = 0.0;
#pragma unroll
      for (int i = 0; i < j; ++i) sum += r[i][j] * wa1[i];
      wa1[j] = (wa1[j] - sum) / r[j][j];
    }
    const double temp = enorm_u(wa1);
    parl = ((fp / delta) / temp) / temp;
  }
#pragma unroll
  for (int j = 0; j < N; ++j) {
    double sum = 0.0;
#pragma unroll
    for (int i = 0; i <= j; ++i) sum += r[i][j] * qtb[i];
    wa1[j] = sum / sel(diag, ipvt[j]);
  }
  const double gnorm = enorm_u(wa1);
  double paru = gnorm / delta;
  if (paru == 0.0) paru = DWARF / fmin(delta, 0.1);
  par = fmax(par, parl);
  par = fmin(par, paru);
  if (par == 0.0) par = gnorm / dxnorm;
  for (;;) {
    ++iter;
    if (par == 0.0) par = fmax(DWARF, 0.001 * paru);
    const double sp = sqrt(par);
#pragma unroll
    for (int j = 0; j < N; ++j) wa1[j] = sp * diag[j];
    qrsolv<N>(r, ipvt, wa1, qtb, x, sdiag);
    LM_ADD(3, 1);
#pragma unroll
    for (int j = 0; j < N; ++j) wa2[j] = diag[j] * x[j];
    dxnorm = enorm_u(wa2);
    const double temp = fp;
    fp = dxnorm - delta;
    if (fabs(fp) <= 0.1 * delta || (parl == 0.0 && fp <= temp && temp < 0.0) || iter == 10) break;
    const double rdx = 1.0 / dxnorm;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const int l = ipvt[j];
      wa1[j] = sel(diag, l) * la_quot(sel(wa2, l), dxnorm, rdx);
    }
#pragma unroll
    for (int j = 0; j < N; ++j) {
      wa1[j] = wa1[j] / sdiag[j];
      const double t = wa1[j];
#pragma unroll
      for (int i = j + 1; i < N; ++i) wa1[i] = wa1[i] - r[i][j] * t;
    }
    const double t = enorm_u(wa1);
    const double parc = ((fp / delta) / t) / t;
    if (fp > 0.0) parl = fmax(parl, par);
    if (fp < 0.0) paru = fmin(paru, par);
    par = fmax(parl, par + parc);
  }
}

// qrsolv in the pivoted basis: dp[j] = diag[ipvt[j]], and xp[j] = x[ipvt[j]] on return (the
// same values as qrsolv's, without its permutation selects)
template <int N>
__device__ __forceinline__ void qrsolv_p(double (&r)[N][N], const double (&dp)[N],
                                         const double (&qtb)[N], double (&xp)[N],
                                         double (&sdiag)[N]) {
  PFE_LA_CONTRACT
  double wa[N], rd[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
#pragma unroll
    for (int i = j; i < N; ++i) r[i][j] = r[j][i];
    rd[j] = r[j][j];
    wa[j] = qtb[j];
  }
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const double dl = dp[j];
    if (dl != 0.0) {
#pragma unroll
      for (int k = j; k < N; ++k) sdiag[k] = 0.0;
      sdiag[j] = dl;
      double qtbpj = 0.0;
#pragma unroll
      for (int k = j; k < N; ++k) {
        if (sdiag[k] != 0.0) {
          double sn, cs;
          if (fabs(r[k][k]) < fabs(sdiag[k])) {
            const double cotan = r[k][k] / sdiag[k];
            sn = la_half_rsqrt(0.25 + 0.25 * (cotan * cotan));
            cs = sn * cotan;
          } else {
            const double tn = sdiag[k] / r[k][k];
            cs = la_half_rsqrt(0.25 + 0.25 * (tn * tn));
            sn = cs * tn;
          }
          r[k][k] = cs * r[k][k] + sn * sdiag[k];
          const double temp = cs * wa[k] + sn * qtbpj;
          qtbpj = -sn * wa[k] + cs * qtbpj;
          wa[k] = temp;
#pragma unroll
          for (int i = k + 1; i < N; ++i) {
            const double t = cs * r[i][k] + sn * sdiag[i];
            sdiag[i] = -sn * r[i][k] + cs * sdiag[i];
            r[i][k] = t;
          }
        }
      }
    }
    sdiag[j] = r[j][j];
    r[j][j] = rd[j];
  }
  int nsing = N;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    if (sdiag[j] == 0.0 && nsing == N) nsing = j;
    if (nsing < N) wa[j] = 0.0;
  }
#pragma unroll
  for (int j = N - 1; j >= 0; --j) {
    if (j < nsing) {
      double sum = 0.0;
#pragma unroll
      for (int i = j + 1; i < N; ++i)
        if (i < nsing) sum += r[i][j] * wa[i];
      wa[j] = (wa[j] - sum) / sdiag[j];
    }
  }
#pragma unroll
  for (int j = 0; j < N; ++j) xp[j] = wa[j];
}

// lmpar.  x: the Levenberg-Marquardt step (natural order), xp[j] = x[ipvt[j]].  The contracted
// build works in the pivoted basis throughout -- diag[ipvt[j]] selected once, qrsolv_p, the
// scaled step and its norm in pivoted order (a norm does not depend on the order but for its
// rounding) -- and scatters x once at the end, instead of MINPACK's per-iteration
// permutations (on a replicated register array each is an n-way select chain: for n = 8
// about 500 instructions per iteration)
template <int N>
__device__ __forceinline__ void lmpar(double (&r)[N][N], const int (&ipvt)[N],
                                      const double (&diag)[N], const double (&qtb)[N],
                                      double delta, double& par, double (&x)[N],
                                      double (&sdiag)[N], double (&xp)[N]) {
  PFE_LA_CONTRACT
  if constexpr (LA_EXACT_QUOTIENTS) {
    lmpar_literal<N>(r, ipvt, diag, qtb, delta, par, x, sdiag);
#pragma unroll
    for (int j = 0; j < N; ++j) xp[j] = sel(x, ipvt[j]);
    return;
  }
  double dp[N], wa1[N], wa2[N];
#pragma unroll
  for (int j = 0; j < N; ++j) dp[j] = sel(diag, ipvt[j]);
  int nsing = N;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    wa1[j] = qtb[j];
    if (r[j][j] == 0.0 && nsing == N) nsing = j;
    if (nsing < N) wa1[j] = 0.0;
  }
#pragma unroll
  for (int j = N - 1; j >= 0; --j) {
    if (j < nsing) {
      wa1[j] = wa1[j] / r[j][j];
      const double temp = wa1[j];
#pragma unroll
      for (int i = 0; i < j; ++i) wa1[i] = wa1[i] - r[i][j] * temp;
    }
  }
#pragma unroll
  for (int j = 0; j < N; ++j) {
    xp[j] = wa1[j];
    wa2[j] = dp[j] * xp[j];
  }
  int iter = 0;
  double dxnorm = enorm_u(wa2);
  double fp = dxnorm - delta;
  if (fp <= 0.1 * delta) {
    par = 0.0;  // iter == 0
  } else {
    double parl = 0.0;
    if (nsing >= N) {
      const double rdx = 1.0 / dxnorm;
#pragma unroll
      for (int j = 0; j < N; ++j) wa1[j] = dp[j] * (wa2[j] * rdx);
#pragma unroll
      for (int j = 0; j < N; ++j) {
        double sum = 0.0;
#pragma unroll
        for (int i = 0; i < j; ++i) sum += r[i][j] * wa1[i];
        wa1[j] = (wa1[j] - sum) / r[j][j];
      }
      const double temp = enorm_u(wa1);
      parl = ((fp / delta) / temp) / temp;
    }
#pragma unroll
    for (int j = 0; j < N; ++j) {
      double sum = 0.0;
#pragma unroll
      for (int i = 0; i <= j; ++i) sum += r[i][j] * qtb[i];
      wa1[j] = sum / dp[j];
    }
    const double gnorm = enorm_u(wa1);
    double paru = gnorm / delta;
    if (paru == 0.0) paru = DWARF / fmin(delta, 0.1);
    par = fmax(par, parl);
    par = fmin(par, paru);
    if (par == 0.0) par = gnorm / dxnorm;
    for (;;) {
      ++iter;
      if (par == 0.0) par = fmax(DWARF, 0.001 * paru);
      const double sp = sqrt(par);
#pragma unroll
      for (int j = 0; j < N; ++j) wa1[j] = sp * dp[j];
      qrsolv_p<N>(r, wa1, qtb, xp, sdiag);
      LM_ADD(3, 1);
#pragma unroll
      for (int j = 0; j < N; ++j) wa2[j] = dp[j] * xp[j];
      dxnorm = enorm_u(wa2);
      const double temp = fp;
      fp = dxnorm - delta;
      if (fabs(fp) <= 0.1 * delta || (parl == 0.0 && fp <= temp && temp < 0.0) || iter == 10) break;
      const double rdx = 1.0 / dxnorm;
#pragma unroll
      for (int j = 0; j < N; ++j) wa1[j] = dp[j] * (wa2[j] * rdx);
#pragma unroll
      for (int j = 0; j < N; ++j) {
        wa1[j] = wa1[j] / sdiag[j];
        const double t = wa1[j];
#pragma unroll
        for (int i = j + 1; i < N; ++i) wa1[i] = wa1[i] - r[i][j] * t;
      }
      const double t = enorm_u(wa1);
      const double parc = ((fp / delta) / t) / t;
      if (fp > 0.0) parl = fmax(parl, par);
      if (fp < 0.0) paru = fmin(paru, par);
      par = fmax(parl, par + parc);
    }
  }
#pragma unroll
  for (int j = 0; j < N; ++j) put(x, ipvt[j], xp[j]);
}
template <int N>
__device__ __forceinline__ void lmpar(double (&r)[N][N], const int (&ipvt)[N],
                                      const double (&diag)[N], const double (&qtb)[N],
                                      double delta, double& par, double (&x)[N],
                                      double (&sdiag)[N]) {
  double xp[N];
  lmpar<N>(r, ipvt, diag, qtb, delta, par, x, sdiag, xp);
}

// ---- lmdif ----------------------------------------------------------------------------
// fcn(p, f): fill f[k] with the residual of this lane's row i = lane + 64*k for i < m and
// with 0 for i >= m.  Returns MINPACK's info (1-8); x holds the solution.
struct LMResult {
  int info;
  int nfev;
};

template <int N, int MPL, class Fn>
__device__ __forceinline__ LMResult lmdif(const Fn& fcn, double (&x)[N], int maxfev) {
  const double eps = 1.4901161193847656e-08;  // sqrt(max(epsfcn, epsmch)) = 2^-26
  double fvec[MPL], wa4[MPL];
  double fjac[MPL][N];
  double diag[N], qtf[N], wa1[N], wa2[N], wa3[N];
  double r[N][N];
  int ipvt[N];
  int info = 0;
  LM_T0(t_start);
  fcn(x, fvec);
  int nfev = 1;
  double fnorm = enorm_w(fvec);
  double par = 0.0, xnorm = 0.0, delta = 0.0;
  int iter = 1;
  const int lane = lane_id();
  for (;;) {
    LM_ADD(1, 1);
    LM_T0(t_fd);
    // forward-difference Jacobian (fdjac2)
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const double temp = x[j];
      double h = eps * fabs(temp);
      if (h == 0.0) h = eps;
      x[j] = temp + h;
      fcn(x, wa4);
      x[j] = temp;
      const double rh = 1.0 / h;
#pragma unroll
      for (int k = 0; k < MPL; ++k) fjac[k][j] = la_quot(wa4[k] - fvec[k], h, rh);
    }
    nfev += N;
    LM_T0(t_qr);
    LM_ADD(5, t_qr - t_fd);
    qrfac<N, MPL>(fjac, ipvt, wa1, wa2);
    LM_T0(t_qt);
    LM_ADD(6, t_qt - t_qr);
    if (iter == 1) {
#pragma unroll
      for (int j = 0; j < N; ++j) {
        diag[j] = wa2[j];
        if (wa2[j] == 0.0) diag[j] = 1.0;
      }
#pragma unroll
      for (int j = 0; j < N; ++j) wa3[j] = diag[j] * x[j];
      xnorm = enorm_u(wa3);
      delta = LM_FACTOR * xnorm;
      if (delta == 0.0) delta = LM_FACTOR;
    }
    // (Q^T) fvec -> qtf; restore the diagonal of R
#pragma unroll
    for (int k = 0; k < MPL; ++k) wa4[k] = fvec[k];
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const double ajj = bcast(fjac[0][j], j);
      if (ajj != 0.0) {
        double p = 0.0;
#pragma unroll
        for (int k = 0; k < MPL; ++k)
          if (row_ge(lane, k, j)) p += fjac[k][j] * wa4[k];
        const double sum = wsum(p);
        const double temp = -sum / ajj;
#pragma unroll
        for (int k = 0; k < MPL; ++k)
          if (row_ge(lane, k, j)) wa4[k] = wa4[k] + fjac[k][j] * temp;
      }
      if (lane == j) fjac[0][j] = wa1[j];
      qtf[j] = bcast(wa4[0], j);
    }
#pragma unroll
    for (int j = 0; j < N; ++j) {
#pragma unroll
      for (int i = 0; i < N; ++i) r[i][j] = (i <= j) ? bcast(fjac[0][j], i) : 0.0;
    }
    // scaled gradient norm
    double gnorm = 0.0;
    if (fnorm != 0.0) {
#pragma unroll
      for (int j = 0; j < N; ++j) {
        const double wl = sel(wa2, ipvt[j]);
        if (wl != 0.0) {
          double sum = 0.0;
#pragma unroll
          for (int i = 0; i <= j; ++i) sum += r[i][j] * (qtf[i] / fnorm);
          gnorm = fmax(gnorm, fabs(sum / wl));
        }
      }
    }
    LM_T0(t_gn);
    LM_ADD(7, t_gn - t_qt);
    if (gnorm <= LM_GTOL) info = 4;
    if (info != 0) break;
#pragma unroll
    for (int j = 0; j < N; ++j) diag[j] = fmax(diag[j], wa2[j]);
    // inner loop
    double ratio;
    do {
      LM_T0(t_lp);
      lmpar<N>(r, ipvt, diag, qtf, delta, par, wa1, wa2);
      LM_T0(t_tr);
      LM_ADD(8, t_tr - t_lp);
      LM_ADD(2, 1);
#pragma unroll
      for (int j = 0; j < N; ++j) {
        wa1[j] = -wa1[j];
        wa2[j] = x[j] + wa1[j];
        wa3[j] = diag[j] * wa1[j];
      }
      const double pnorm = enorm_u(wa3);
      if (iter == 1) delta = fmin(delta, pnorm);
      fcn(wa2, wa4);
      ++nfev;
      const double fnorm1 = enorm_w(wa4);
      LM_ADD(9, lm_clock() - t_tr);
      double actred = -1.0;
      if (0.1 * fnorm1 < fnorm) {
        const double q = fnorm1 / fnorm;
        actred = 1.0 - q * q;
      }
      double temp = 0.0;
#pragma unroll
      for (int j = 0; j < N; ++j) wa3[j] = 0.0;
#pragma unroll
      for (int j = 0; j < N; ++j) {
        temp = sel(wa1, ipvt[j]);
#pragma unroll
        for (int i = 0; i <= j; ++i) wa3[i] = wa3[i] + r[i][j] * temp;
      }
      const double temp1 = enorm_u(wa3) / fnorm;
      const double temp2 = (sqrt(par) * pnorm) / fnorm;
      const double prered = temp1 * temp1 + (temp2 * temp2) / 0.5;
      const double dirder = -(temp1 * temp1 + temp2 * temp2);
      ratio = 0.0;
      if (prered != 0.0) ratio = actred / prered;
      if (ratio <= 0.25) {
        if (actred >= 0.0) temp = 0.5;
        if (actred < 0.0) temp = 0.5 * dirder / (dirder + 0.5 * actred);
        if (0.1 * fnorm1 >= fnorm || temp < 0.1) temp = 0.1;
        delta = temp * fmin(delta, pnorm / 0.1);
        par = par / temp;
      } else if (par == 0.0 || ratio >= 0.75) {
        delta = pnorm / 0.5;
        par = 0.5 * par;
      }
      if (ratio >= 1e-4) {
#pragma unroll
        for (int j = 0; j < N; ++j) {
          x[j] = wa2[j];
          wa2[j] = diag[j] * x[j];
        }
#pragma unroll
        for (int k = 0; k < MPL; ++k) fvec[k] = wa4[k];
        xnorm = enorm_u(wa2);
        fnorm = fnorm1;
        ++iter;
      }
      if (fabs(actred) <= LM_FTOL && prered <= LM_FTOL && 0.5 * ratio <= 1.0) info = 1;
      if (delta <= LM_XTOL * xnorm) info = 2;
      if (fabs(actred) <= LM_FTOL && prered <= LM_FTOL && 0.5 * ratio <= 1.0 && info == 2) info = 3;
      if (info != 0) break;
      if (nfev >= maxfev) info = 5;
      if (fabs(actred) <= EPSMCH && prered <= EPSMCH && 0.5 * ratio <= 1.0) info = 6;
      if (delta <= EPSMCH * xnorm) info = 7;
      if (gnorm <= EPSMCH) info = 8;
      if (info != 0) break;
    } while (ratio < 1e-4);
    if (info != 0) break;
  }
  LM_ADD(0, 1);
  LM_ADD(4, nfev);
  LM_ADD(10, lm_clock() - t_start);
  return {info, nfev};
}

}  // namespace pfe
