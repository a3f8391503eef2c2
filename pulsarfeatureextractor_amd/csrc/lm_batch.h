// lm_batch.h — MINPACK lmdif for a batch of up to FPW independent fits owned by one wave.
//
// The wave-per-fit lmdif of lm_wave.h executes the n-sized half of MINPACK (lmpar, qrsolv,
// the step bookkeeping) redundantly in all 64 lanes; for n = 4..8 that half is 2/3 or more of
// the instructions a solve issues.  Here a wave owns a batch of fits and alternates two kinds
// of phases:
//
//   * m-phase ("visit"): the wave works on ONE fit with all 64 lanes — residual evaluations,
//     the forward-difference Jacobian, Householder QR with column pivoting, Q^T f, the
//     acceptance test of a trial step — exactly the wave-parallel code of lm_wave.h.  Fits are
//     visited one after another; only fits that still iterate are visited, so the m-parallel
//     work costs what the fits need, however unequal their iteration counts are.
//   * SIMT phase: every lane runs lmpar (+ qrsolv) and the predicted-reduction terms for its
//     own fit (lane f <-> fit f), i.e. the serial half is executed once per fit, not 64 times.
//
// Between phases the per-fit state lives in LDS, structure-of-arrays ([element][fit]), so the
// SIMT phase reads it conflict-free and the m-phase reads one fit's values as broadcasts.
// The arithmetic is that of lmdif in lm_wave.h operation for operation (and thus of MINPACK,
// up to the tree-ordered m-sums), so results are bit-identical to the wave-per-fit solver.
#pragma once

#include <type_traits>

#include "lm_wave.h"

namespace pfe {

// packed upper triangle of R, by columns: element (i, j), i <= j
__host__ __device__ constexpr int tri_idx(int i, int j) { return j * (j + 1) / 2 + i; }

template <int N, int FPW>
struct BlmState {
  double x[N][FPW];      // current point
  double trial[N][FPW];  // x + step of the last lmpar
  double diag[N][FPW];   // scaling (mode 1: running max of the Jacobian column norms)
  double qtf[N][FPW];    // first n elements of Q^T fvec
  double acn[N][FPW];    // column norms of the last Jacobian (qrfac acnorm)
  double r[N * (N + 1) / 2][FPW];
  double fnorm[FPW], par[FPW], delta[FPW], xnorm[FPW], gnorm[FPW];
  double pnorm[FPW], prered[FPW], dirder[FPW], tstale[FPW];
  int ipvt[N][FPW];
  int iter[FPW], nfev[FPW], info[FPW];
};

// Functors with kCols = true keep reusable terms of a full evaluation (Cache) and evaluate
// forward-difference columns from them; others are evaluated in full every time.
template <class Fn, class = void>
struct FnCache {
  struct type {};
};
template <class Fn>
struct FnCache<Fn, decltype((void)Fn::kCols)> {
  using type = typename Fn::Cache;
};
template <class Fn, class = void>
struct HasCols : std::false_type {};
template <class Fn>
struct HasCols<Fn, decltype((void)Fn::kCols)> : std::integral_constant<bool, Fn::kCols> {};

template <class Fn, int N, int MPL>
__device__ __forceinline__ void fn_eval(const Fn& fn, const double (&p)[N], double (&f)[MPL],
                                        typename FnCache<Fn>::type& c) {
  if constexpr (HasCols<Fn>::value)
    fn.eval(p, f, c);
  else
    fn(p, f);
}
// p = the base point with parameter j moved from pj0 to pj0 + h (the forward-difference
// column j); pj0 lets a functor rebuild the base point's intermediate terms
template <class Fn, int N, int MPL>
__device__ __forceinline__ void fn_eval_col(const Fn& fn, const double (&p)[N], int j, double pj0,
                                            double (&f)[MPL], const typename FnCache<Fn>::type& c) {
  if constexpr (HasCols<Fn>::value)
    fn.eval_col(p, j, pj0, f, c);
  else
    fn(p, f);
}

__device__ __forceinline__ void blm_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// The outer-iteration body of lmdif for fit f (m-phase): forward-difference Jacobian at
// S.x[.][f] with residuals fvec, QR, (first iteration: diag, xnorm, delta), Q^T f, R, gnorm,
// the gtol test and the diag update.  Writes everything the SIMT phase needs.
template <int N, int MPL, int FPW, class Fn>
__device__ __forceinline__ void blm_outer(const Fn& fcn, const double (&fvec)[MPL],
                                          const typename FnCache<Fn>::type& cache, double fnorm,
                                          int f, BlmState<N, FPW>& S, int iter, int nfev) {
  const double eps = 1.4901161193847656e-08;  // sqrt(max(epsfcn, epsmch)) = 2^-26
  const int lane = lane_id();
  LM_ADD(1, 1);
  LM_T0(t_fd);
  double x[N];
#pragma unroll
  for (int j = 0; j < N; ++j) x[j] = S.x[j][f];
  double fjac[MPL][N], wa4[MPL];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const double temp = x[j];
    double h = eps * fabs(temp);
    if (h == 0.0) h = eps;
    x[j] = temp + h;
    fn_eval_col<Fn, N, MPL>(fcn, x, j, temp, wa4, cache);
    x[j] = temp;
    const double rh = 1.0 / h;
#pragma unroll
    for (int k = 0; k < MPL; ++k) fjac[k][j] = la_quot(wa4[k] - fvec[k], h, rh);
  }
  nfev += N;
  int ipvt[N];
  double rdiag[N], acn[N];
  LM_T0(t_qr);
  LM_ADD(5, t_qr - t_fd);
  qrfac<N, MPL>(fjac, ipvt, rdiag, acn);
  LM_T0(t_qt);
  LM_ADD(6, t_qt - t_qr);
  double diag[N];
  if (iter == 1) {
    double wa3[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
      diag[j] = acn[j];
      if (acn[j] == 0.0) diag[j] = 1.0;
    }
#pragma unroll
    for (int j = 0; j < N; ++j) wa3[j] = diag[j] * x[j];
    const double xnorm = enorm_u(wa3);
    double delta = LM_FACTOR * xnorm;
    if (delta == 0.0) delta = LM_FACTOR;
    if (lane == 0) {
      S.xnorm[f] = xnorm;
      S.delta[f] = delta;
    }
  } else {
#pragma unroll
    for (int j = 0; j < N; ++j) diag[j] = S.diag[j][f];
  }
  // (Q^T) fvec -> qtf; restore the diagonal of R
  double qtf[N];
#pragma unroll
  for (int k = 0; k < MPL; ++k) wa4[k] = fvec[k];
  {
  PFE_LA_CONTRACT
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
    if (lane == j) fjac[0][j] = rdiag[j];
    qtf[j] = bcast(wa4[0], j);
  }
  }
  // R (upper triangle) -> LDS: row i lives in lane i
#pragma unroll
  for (int j = 0; j < N; ++j)
    if (lane <= j) S.r[tri_idx(0, j) + lane][f] = fjac[0][j];
  // the scaled gradient norm and the gtol test run in the next SIMT phase (blm_simt), one
  // fit per lane, from R, qtf, acnorm and ipvt in LDS; info = -1 marks "not yet tested"
  const int info = -1;
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < N; ++j) {
      S.diag[j][f] = fmax(diag[j], acn[j]);
      S.qtf[j][f] = qtf[j];
      S.acn[j][f] = acn[j];
      S.ipvt[j][f] = ipvt[j];
    }
    S.info[f] = info;
    S.nfev[f] = nfev;
    S.iter[f] = iter;
    S.fnorm[f] = fnorm;
  }
  LM_ADD(7, lm_clock_p() - t_qt);
}

// first visit of fit f: residuals at the start point, then the first outer iteration
template <int N, int MPL, int FPW, class Fn>
__device__ __forceinline__ void blm_init(const Fn& fcn, int f, BlmState<N, FPW>& S) {
  double x[N], fvec[MPL];
  typename FnCache<Fn>::type cache;
#pragma unroll
  for (int j = 0; j < N; ++j) x[j] = S.x[j][f];
  fn_eval<Fn, N, MPL>(fcn, x, fvec, cache);
  const double fnorm = enorm_w(fvec);
  if (lane_id() == 0) {
    S.par[f] = 0.0;
    S.xnorm[f] = 0.0;
    S.delta[f] = 0.0;
  }
  blm_outer<N, MPL, FPW>(fcn, fvec, cache, fnorm, f, S, 1, 1);
}

// SIMT phase for this lane's fit: lmpar, the trial point and the predicted-reduction terms.
// ACN_SQ (the pooled engine's contracted build): S.acn holds the squared column norms of the
// new Jacobian, and the scaling MINPACK updates after qrfac (diag = max(diag, acnorm); at
// the first iteration diag = acnorm, xnorm and delta) is done here, one fit per lane
template <int N, int FPW, bool ACN_SQ = false>
__device__ __forceinline__ void blm_simt(int f, BlmState<N, FPW>& S) {
  PFE_LA_CONTRACT
  double r[N][N], diag[N], qtf[N], x[N];
  int ipvt[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
#pragma unroll
    for (int i = 0; i < N; ++i) r[i][j] = (i <= j) ? S.r[tri_idx(i, j)][f] : 0.0;
    diag[j] = S.diag[j][f];
    qtf[j] = S.qtf[j][f];
    x[j] = S.x[j][f];
    ipvt[j] = S.ipvt[j][f];
  }
  double delta = S.delta[f], par = S.par[f];
  const double fnorm = S.fnorm[f];
  const int iter = S.iter[f];
  if (S.info[f] < 0) {
    // scaled gradient norm of the new Jacobian and the gtol test (lmdif's outer loop)
    double acn[N];
#pragma unroll
    for (int j = 0; j < N; ++j) acn[j] = ACN_SQ ? sqrt(S.acn[j][f]) : S.acn[j][f];
    if constexpr (ACN_SQ) {
      if (iter == 1) {
        double wa3[N];
#pragma unroll
        for (int j = 0; j < N; ++j) {
          diag[j] = acn[j] == 0.0 ? 1.0 : acn[j];
          wa3[j] = diag[j] * x[j];
        }
        const double xnorm = enorm_u(wa3);
        delta = LM_FACTOR * xnorm;
        if (delta == 0.0) delta = LM_FACTOR;
        S.xnorm[f] = xnorm;
        S.delta[f] = delta;
      }
#pragma unroll
      for (int j = 0; j < N; ++j) {
        diag[j] = fmax(diag[j], acn[j]);
        S.diag[j][f] = diag[j];
      }
    }
    double gnorm = 0.0;
    if (fnorm != 0.0) {
      const double rfn = 1.0 / fnorm;
#pragma unroll
      for (int j = 0; j < N; ++j) {
        const double wl = sel(acn, ipvt[j]);
        if (wl != 0.0) {
          double sum = 0.0;
#pragma unroll
          for (int i = 0; i <= j; ++i) sum += r[i][j] * la_quot(qtf[i], fnorm, rfn);
          gnorm = fmax(gnorm, fabs(sum / wl));
        }
      }
    }
    S.gnorm[f] = gnorm;
    const int info = (gnorm <= LM_GTOL) ? 4 : 0;
    S.info[f] = info;
    if (info != 0) return;
  }
  double wa1[N], wa2[N], wa3[N], wp[N];
  lmpar<N>(r, ipvt, diag, qtf, delta, par, wa1, wa2, wp);
#pragma unroll
  for (int j = 0; j < N; ++j) {
    wa1[j] = -wa1[j];
    wa2[j] = x[j] + wa1[j];
    wa3[j] = diag[j] * wa1[j];
  }
  const double pnorm = enorm_u(wa3);
  if (iter == 1) delta = fmin(delta, pnorm);
  double temp = 0.0;
#pragma unroll
  for (int j = 0; j < N; ++j) wa3[j] = 0.0;
#pragma unroll
  for (int j = 0; j < N; ++j) {
    temp = -wp[j];  // wa1[ipvt[j]]
#pragma unroll
    for (int i = 0; i <= j; ++i) wa3[i] = wa3[i] + r[i][j] * temp;
  }
  const double temp1 = enorm_u(wa3) / fnorm;
  const double temp2 = (sqrt(par) * pnorm) / fnorm;
#pragma unroll
  for (int j = 0; j < N; ++j) S.trial[j][f] = wa2[j];
  S.pnorm[f] = pnorm;
  S.delta[f] = delta;
  S.par[f] = par;
  S.prered[f] = temp1 * temp1 + (temp2 * temp2) / 0.5;
  S.dirder[f] = -(temp1 * temp1 + temp2 * temp2);
  S.tstale[f] = temp;
}

// m-phase visit after a SIMT phase: evaluate the trial point, update delta/par, accept or
// reject, convergence tests; on an accepted step that does not finish the fit, the next
// outer iteration follows immediately (the new residuals are still in registers).
template <int N, int MPL, int FPW, class Fn>
__device__ __forceinline__ void blm_trial(const Fn& fcn, int f, BlmState<N, FPW>& S, int maxfev) {
  const int lane = lane_id();
  double wa2[N], wa4[MPL];
  typename FnCache<Fn>::type cache;
#pragma unroll
  for (int j = 0; j < N; ++j) wa2[j] = S.trial[j][f];
  fn_eval<Fn, N, MPL>(fcn, wa2, wa4, cache);
  int nfev = S.nfev[f] + 1;
  const double fnorm1 = enorm_w(wa4);
  double fnorm = S.fnorm[f];
  double delta = S.delta[f], par = S.par[f], xnorm = S.xnorm[f];
  const double pnorm = S.pnorm[f], prered = S.prered[f], dirder = S.dirder[f];
  const double gnorm = S.gnorm[f];
  int iter = S.iter[f];
  double actred = -1.0;
  if (0.1 * fnorm1 < fnorm) {
    const double q = fnorm1 / fnorm;
    actred = 1.0 - q * q;
  }
  double temp = S.tstale[f];
  double ratio = 0.0;
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
  const bool accepted = ratio >= 1e-4;
  if (accepted) {
    double wa3[N];
#pragma unroll
    for (int j = 0; j < N; ++j) wa3[j] = S.diag[j][f] * wa2[j];
    xnorm = enorm_u(wa3);
    fnorm = fnorm1;
    ++iter;
  }
  int info = 0;
  if (fabs(actred) <= LM_FTOL && prered <= LM_FTOL && 0.5 * ratio <= 1.0) info = 1;
  if (delta <= LM_XTOL * xnorm) info = 2;
  if (fabs(actred) <= LM_FTOL && prered <= LM_FTOL && 0.5 * ratio <= 1.0 && info == 2) info = 3;
  if (info == 0) {
    if (nfev >= maxfev) info = 5;
    if (fabs(actred) <= EPSMCH && prered <= EPSMCH && 0.5 * ratio <= 1.0) info = 6;
    if (delta <= EPSMCH * xnorm) info = 7;
    if (gnorm <= EPSMCH) info = 8;
  }
  if (lane == 0) {
    S.delta[f] = delta;
    S.par[f] = par;
    S.nfev[f] = nfev;
    S.info[f] = info;
    if (accepted) {
#pragma unroll
      for (int j = 0; j < N; ++j) S.x[j][f] = wa2[j];
      S.xnorm[f] = xnorm;
      S.fnorm[f] = fnorm;
      S.iter[f] = iter;
    }
  }
  if (accepted && info == 0) {
    blm_sync();
    blm_outer<N, MPL, FPW>(fcn, wa4, cache, fnorm, f, S, iter, nfev);
  }
}

// Run lmdif on the fits whose bits are set in `fits` (lane f <-> fit f, f < FPW).  The caller
// has stored each fit's start point in S.x[.][f]; on return S.x holds the solutions and
// S.info / S.nfev MINPACK's info and evaluation counts.  load(f) returns the residual functor
// of fit f (it is called inside every m-phase visit, so it should read its data cheaply).
template <int N, int MPL, int FPW, class Loader>
__device__ __forceinline__ void blm_run(const Loader& load, BlmState<N, FPW>& S, uint64_t fits,
                                        int maxfev) {
  static_assert(FPW <= 64, "one fit per lane");
  const int lane = lane_id();
  LM_T0(t_start);
  blm_sync();
  for (uint64_t m = fits; m; m &= m - 1) {
    const int f = __builtin_ctzll(m);
    const auto fn = load(f);
    blm_init<N, MPL, FPW>(fn, f, S);
    blm_sync();
  }
  LM_ADD(11, lm_clock_p() - t_start);
  for (;;) {
    blm_sync();
    const bool mine = lane < FPW && ((fits >> lane) & 1ull) && S.info[lane < FPW ? lane : 0] <= 0;
    if (__ballot(mine) == 0) break;
    LM_T0(t_simt);
    if (mine) blm_simt<N, FPW>(lane, S);
    blm_sync();
    // fits still iterating after the gtol test: evaluate their trial points
    const uint64_t act = __ballot(mine && S.info[lane < FPW ? lane : 0] == 0);
    LM_T0(t_trial);
    LM_ADD(12, t_trial - t_simt);
    LM_ADD(14, 1);
    LM_ADD(15, __builtin_popcountll(__ballot(mine)));
    LM_ADD(2, __builtin_popcountll(act));
    for (uint64_t m = act; m; m &= m - 1) {
      const int f = __builtin_ctzll(m);
      const auto fn = load(f);
      blm_trial<N, MPL, FPW>(fn, f, S, maxfev);
      blm_sync();
    }
    LM_ADD(9, lm_clock_p() - t_trial);
  }
  LM_ADD(0, __builtin_popcountll(fits));
#ifdef PFE_LM_PROFILE
  {
    int nf = 0;
    for (uint64_t m = fits; m; m &= m - 1) nf += S.nfev[__builtin_ctzll(m)];
    LM_ADD(4, nf);
  }
#endif
  LM_ADD(10, lm_clock_p() - t_start);
}

}  // namespace pfe
