// lm_global.h — MINPACK lmdif for one wavefront with the m rows in global memory.
//
// The same algorithm and arithmetic as lm_wave.h (fdjac2, qrfac with pivoting, Q^T f,
// lmpar / qrsolv on the replicated n x n state, scipy's leastsq defaults), for problems whose
// m rows do not fit in registers: the Freedman-Diaconis histograms of profiles with a tiny
// interquartile range (thousands of bins, ProfileOperationsInterface.py:138-166).  Row
// i = lane + 64 k of every m-vector lives at buf[k * 64 + lane] of its array, so each access
// of a slot is one coalesced 512-B wave transaction; sums over rows are formed per lane over
// the slots in order, then by the wave butterfly (wsum), exactly as lm_wave.h does with
// MPL = nsl slots.  The arrays of one solve (fvec, wa4, fjac[N]) take (N + 2) * 64 * nsl
// doubles of per-wave scratch; the data stay L2-resident for the length of a solve.
#pragma once

#include "lm_wave.h"

namespace pfe {

// per-wave row storage of one solve: nsl slots of 64 rows per array
template <int N>
struct RowStore {
  double* base;
  int nsl;
  __device__ __forceinline__ double* fvec() const { return base; }
  __device__ __forceinline__ double* wa4() const { return base + (size_t)nsl * 64; }
  __device__ __forceinline__ double* fjac(int j) const { return base + (size_t)(2 + j) * nsl * 64; }
  static __host__ __device__ constexpr size_t doubles_per_slot() { return (size_t)(N + 2) * 64; }
};

__device__ __forceinline__ double enorm_g(const double* f, int nsl, int lane) {
  double p = 0.0;
  for (int k = 0; k < nsl; ++k) {
    const double v = f[k * 64 + lane];
    p += v * v;
  }
  return sqrt(wsum(p));
}

template <int N>
__device__ void qrfac_g(const RowStore<N>& rs, int (&ipvt)[N], double (&rdiag)[N], double (&acnorm)[N]) {
  const int lane = lane_id();
  const int nsl = rs.nsl;
  double wa[N];
  {
    double s[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const double* a = rs.fjac(j);
      double p = 0.0;
      for (int k = 0; k < nsl; ++k) p += a[k * 64 + lane] * a[k * 64 + lane];
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
    // bring the column of largest norm into the pivot position (the rows move in memory)
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
          double* a = rs.fjac(j);
          double* b = rs.fjac(k2);
          for (int k = 0; k < nsl; ++k) {
            const double t = a[k * 64 + lane];
            a[k * 64 + lane] = b[k * 64 + lane];
            b[k * 64 + lane] = t;
          }
          rdiag[k2] = rdiag[j];
          wa[k2] = wa[j];
          const int t = ipvt[j];
          ipvt[j] = ipvt[k2];
          ipvt[k2] = t;
        }
      }
    }
    double* aj = rs.fjac(j);
    double p = 0.0;
    for (int k = 0; k < nsl; ++k)
      if (row_ge(lane, k, j)) p += aj[k * 64 + lane] * aj[k * 64 + lane];
    double ajnorm = sqrt(wsum(p));
    if (ajnorm != 0.0) {
      if (bcast(aj[lane], j) < 0.0) ajnorm = -ajnorm;
      for (int k = 0; k < nsl; ++k)
        if (row_ge(lane, k, j)) aj[k * 64 + lane] = aj[k * 64 + lane] / ajnorm;
      if (lane == j) aj[lane] = aj[lane] + 1.0;
      double d[N];
#pragma unroll
      for (int c = 0; c < N; ++c) {
        double q = 0.0;
        if (c > j) {
          const double* ac = rs.fjac(c);
          for (int k = 0; k < nsl; ++k)
            if (row_ge(lane, k, j)) q += aj[k * 64 + lane] * ac[k * 64 + lane];
        }
        d[c] = q;
      }
      wsum_from(d, j + 1);
      const double ajj = bcast(aj[lane], j);
#pragma unroll
      for (int c = j + 1; c < N; ++c) {
        double* ac = rs.fjac(c);
        const double temp = d[c] / ajj;
        for (int k = 0; k < nsl; ++k)
          if (row_ge(lane, k, j)) ac[k * 64 + lane] = ac[k * 64 + lane] - temp * aj[k * 64 + lane];
        if (rdiag[c] != 0.0) {
          const double t2 = bcast(ac[lane], j) / rdiag[c];
          rdiag[c] = rdiag[c] * sqrt(fmax(0.0, 1.0 - t2 * t2));
          const double q = rdiag[c] / wa[c];
          if (0.05 * (q * q) <= EPSMCH) {
            double r = 0.0;
            for (int k = 0; k < nsl; ++k)
              if (row_ge(lane, k, j + 1)) r += ac[k * 64 + lane] * ac[k * 64 + lane];
            rdiag[c] = sqrt(wsum(r));
            wa[c] = rdiag[c];
          }
        }
      }
    }
    rdiag[j] = -ajnorm;
  }
}

// fcn(p, f): f[k * 64 + lane] = residual of row lane + 64 k (0 for rows >= m)
template <int N, class Fn>
__device__ LMResult lmdif_g(const Fn& fcn, double (&x)[N], int maxfev, const RowStore<N>& rs) {
  const double eps = 1.4901161193847656e-08;
  const int lane = lane_id();
  const int nsl = rs.nsl;
  double* fvec = rs.fvec();
  double* wa4 = rs.wa4();
  double diag[N], qtf[N], wa1[N], wa2[N], wa3[N];
  double r[N][N];
  int ipvt[N];
  int info = 0;
  fcn(x, fvec);
  int nfev = 1;
  double fnorm = enorm_g(fvec, nsl, lane);
  double par = 0.0, xnorm = 0.0, delta = 0.0;
  int iter = 1;
  for (;;) {
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const double temp = x[j];
      double h = eps * fabs(temp);
      if (h == 0.0) h = eps;
      x[j] = temp + h;
      fcn(x, wa4);
      x[j] = temp;
      double* fj = rs.fjac(j);
      for (int k = 0; k < nsl; ++k) fj[k * 64 + lane] = (wa4[k * 64 + lane] - fvec[k * 64 + lane]) / h;
    }
    nfev += N;
    qrfac_g<N>(rs, ipvt, wa1, wa2);
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
    for (int k = 0; k < nsl; ++k) wa4[k * 64 + lane] = fvec[k * 64 + lane];
#pragma unroll
    for (int j = 0; j < N; ++j) {
      double* fj = rs.fjac(j);
      const double ajj = bcast(fj[lane], j);
      if (ajj != 0.0) {
        double p = 0.0;
        for (int k = 0; k < nsl; ++k)
          if (row_ge(lane, k, j)) p += fj[k * 64 + lane] * wa4[k * 64 + lane];
        const double sum = wsum(p);
        const double temp = -sum / ajj;
        for (int k = 0; k < nsl; ++k)
          if (row_ge(lane, k, j)) wa4[k * 64 + lane] = wa4[k * 64 + lane] + fj[k * 64 + lane] * temp;
      }
      if (lane == j) fj[lane] = wa1[j];
      qtf[j] = bcast(wa4[lane], j);
    }
#pragma unroll
    for (int j = 0; j < N; ++j) {
      const double* fj = rs.fjac(j);
      const double v = fj[lane];
#pragma unroll
      for (int i = 0; i < N; ++i) r[i][j] = (i <= j) ? bcast(v, i) : 0.0;
    }
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
    if (gnorm <= LM_GTOL) info = 4;
    if (info != 0) break;
#pragma unroll
    for (int j = 0; j < N; ++j) diag[j] = fmax(diag[j], wa2[j]);
    double ratio;
    do {
      lmpar<N>(r, ipvt, diag, qtf, delta, par, wa1, wa2);
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
      const double fnorm1 = enorm_g(wa4, nsl, lane);
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
        for (int k = 0; k < nsl; ++k) fvec[k * 64 + lane] = wa4[k * 64 + lane];
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
  return {info, nfev};
}

}  // namespace pfe
