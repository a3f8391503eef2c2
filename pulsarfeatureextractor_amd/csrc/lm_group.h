// lm_group.h — MINPACK lmdif for a pool of fits owned by one wave, worked in 16-lane groups.
//
// lm_batch.h visits one fit at a time with all 64 lanes (m = 128 rows -> 2 rows per lane),
// so every per-fit scalar step of the m-parallel half (pivot choice, Householder scaling,
// divisions and square roots of qrfac, the step bookkeeping of a trial) and every 64-lane
// reduction is paid once per fit by the whole wave, and a batch runs until its slowest fit
// is done (its SIMT phases then carry few fits).  Here:
//
//   * a wave owns FPW fit SLOTS; the state of each lives in LDS (BlmState, [element][slot]);
//   * the m-parallel half runs in GROUPS of G = 16 lanes (one DPP row): NG = 4 fits are
//     worked at once, row r of a fit in group-lane r % 16, register slot r / 16; reductions
//     are 4 DPP steps inside the row and broadcasts are row_newbcast -- no cross-row traffic.
//     G = 32 (two DPP rows, NG = 2) halves the rows each lane holds (the 8-parameter fit's
//     registers, 256-bin profiles): one v_permlane16_swap step joins the two rows;
//   * the serial half (gtol test, lmpar, predicted reduction) runs one fit per lane (SIMT,
//     blm_simt of lm_batch.h, unchanged);
//   * slots are refilled as soon as their fit ends (Problem::refill, wave-cooperative), so
//     the pool stays full until the work queue drains: no batch waits for its slowest fit.
//
// Each loop iteration is: refill finished slots -> O-phase (function value at x, the
// forward-difference Jacobian, QR, Q^T f: fresh fits and accepted steps) -> SIMT phase
// (lmpar) -> T-phase (trial point evaluation, acceptance and convergence tests).  A phase
// hands its slots to the groups through a compacted list, NG per round.
//
// The arithmetic is MINPACK's (as lm_wave.h / lm_batch.h) with m-sums ordered per lane over
// its rows and then as a butterfly over the 16 lanes: results differ from lm_batch.h only
// in that summation order (last-bit), i.e. like any other non-sequential lmdif.
#pragma once

#include <type_traits>

#include "lm_batch.h"

namespace pfe {

constexpr int GLM_G = 16;  // lanes per group: one DPP row (default; 32 = two rows)

enum : int { PH_EMPTY = 0, PH_INIT = 1, PH_OUTER = 2, PH_LMPAR = 3, PH_TRIAL = 4, PH_DONE = 5 };

template <int G = GLM_G>
__device__ __forceinline__ int glane() {
  static_assert(G == 16 || G == 32, "groups of one or two DPP rows");
  return lane_id() & (G - 1);
}

// v_permlane16_swap of v with itself: .even holds the even row's value of each row pair
// (rows 0,1 -> row 0's), .odd the odd row's
struct RowPair {
  double even, odd;
};
__device__ __forceinline__ RowPair row_pair(double v) {
  const long long b = __double_as_longlong(v);
  const unsigned lo = (unsigned)b, hi = (unsigned)((unsigned long long)b >> 32);
  const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return {__longlong_as_double((long long)(((unsigned long long)h[0] << 32) | l[0])),
          __longlong_as_double((long long)(((unsigned long long)h[1] << 32) | l[1]))};
}

// sum over the G lanes of a group; every lane of the group gets the same bits (IEEE
// addition is commutative, so the mirrored butterflies agree, and both rows of a pair add
// the same two row sums)
template <int G = GLM_G>
__device__ __forceinline__ double gsum(double v) {
  v += dpp_f64<DPP_QUAD_XOR1>(v);
  v += dpp_f64<DPP_QUAD_XOR2>(v);
  v += dpp_f64<DPP_ROW_HALF_MIRROR>(v);
  v += dpp_f64<DPP_ROW_MIRROR>(v);
  if constexpr (G == 32) {
    const RowPair r = row_pair(v);
    v = r.even + r.odd;
  }
  return v;
}
template <int K, int G = GLM_G>
__device__ __forceinline__ void gsum_from(double (&v)[K], int lo) {
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (k >= lo) v[k] += dpp_f64<DPP_QUAD_XOR1>(v[k]);
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (k >= lo) v[k] += dpp_f64<DPP_QUAD_XOR2>(v[k]);
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (k >= lo) v[k] += dpp_f64<DPP_ROW_HALF_MIRROR>(v[k]);
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (k >= lo) v[k] += dpp_f64<DPP_ROW_MIRROR>(v[k]);
  if constexpr (G == 32) {
#pragma unroll
    for (int k = 0; k < K; ++k)
      if (k >= lo) {
        const RowPair r = row_pair(v[k]);
        v[k] = r.even + r.odd;
      }
  }
}

// value of group-lane j (row_newbcast; j folds to a constant inside unrolled loops)
template <int J>
__device__ __forceinline__ double nbc(double v) {
  return __longlong_as_double(
      __builtin_amdgcn_mov_dpp(__double_as_longlong(v), 0x150 + J, 0xF, 0xF, true));
}
__device__ __forceinline__ double gbcast16(double v, int j) {
  switch (j) {
    case 0: return nbc<0>(v);
    case 1: return nbc<1>(v);
    case 2: return nbc<2>(v);
    case 3: return nbc<3>(v);
    case 4: return nbc<4>(v);
    case 5: return nbc<5>(v);
    case 6: return nbc<6>(v);
    case 7: return nbc<7>(v);
    case 8: return nbc<8>(v);
    case 9: return nbc<9>(v);
    case 10: return nbc<10>(v);
    case 11: return nbc<11>(v);
    case 12: return nbc<12>(v);
    case 13: return nbc<13>(v);
    case 14: return nbc<14>(v);
    default: return nbc<15>(v);
  }
}
// value of group-lane j < 16 (a row of the group's first DPP row) in every lane of the group
template <int G = GLM_G>
__device__ __forceinline__ double gbcast(double v, int j) {
  const double w = gbcast16(v, j);
  if constexpr (G == 32)
    return row_pair(w).even;
  else
    return w;
}

// Euclidean norm of a group-distributed m-vector (rows outside [0,m) hold 0)
template <int MPL, int G = GLM_G>
__device__ __forceinline__ double enorm_g(const double (&f)[MPL]) {
  PFE_LA_CONTRACT
  double p = 0.0;
#pragma unroll
  for (int k = 0; k < MPL; ++k) p += f[k] * f[k];
  return sqrt(gsum<G>(p));
}

// qrfac (pivot = true) on the group-distributed m x N matrix a (row r: lane r%G, slot r/G)
// rajjv[j] = 1 / a[j][j] of step j's Householder vector (0 for a zero column): the divisor
// Q^T f divides by in glm_outer, so the contracted build takes it from here instead of a
// second division
template <int N, int MPL, int G = GLM_G>
__device__ __forceinline__ void qrfac_g(double (&a)[MPL][N], int (&ipvt)[N], double (&rdiag)[N],
                                        double (&acnorm)[N], double (&rajjv)[N]) {
  PFE_LA_CONTRACT
  static_assert(N <= 16, "diagonal rows must sit in slot 0 of the group's first DPP row");
  const int gl = glane<G>();
  // nrm: the partial column norms MINPACK keeps in rdiag while it factors (literal build), or
  // their squares (contracted build: the downdate r^2 - a^2, the pivot choice and the
  // norm-loss test need no square root; only the columns' own norms ajnorm and acnorm do)
  constexpr bool SQ = !LA_EXACT_QUOTIENTS;
  double nrm[N], wa[N];
  {
    double s[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
      double p = 0.0;
#pragma unroll
      for (int k = 0; k < MPL; ++k) p += a[k][j] * a[k][j];
      s[j] = p;
    }
    gsum_from<N, G>(s, 0);
#pragma unroll
    for (int j = 0; j < N; ++j) {
      acnorm[j] = SQ ? s[j] : sqrt(s[j]);  // squared in the contracted build (blm_simt roots it)
      nrm[j] = acnorm[j];
      wa[j] = nrm[j];
      ipvt[j] = j;
    }
  }
#pragma unroll
  for (int j = 0; j < N; ++j) {
    int kmax = j;
    double rmax = nrm[j];
#pragma unroll
    for (int k = j + 1; k < N; ++k)
      if (nrm[k] > rmax) {
        kmax = k;
        rmax = nrm[k];
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
          nrm[k2] = nrm[j];
          wa[k2] = wa[j];
          const int t = ipvt[j];
          ipvt[j] = ipvt[k2];
          ipvt[k2] = t;
        }
      }
    }
    double p = 0.0;
#pragma unroll
    for (int k = 0; k < MPL; ++k)
      if (row_ge(gl, k, j)) p += a[k][j] * a[k][j];
    // the column's norm and its reciprocal: sqrt and a division (literal build, or a sum of
    // squares outside [1e-280, 1e280]), else one rsqrt and a product
    const double pp = gsum<G>(p);
    double ajnorm, rinv;
    if (SQ && pp > 1e-280 && pp < 1e280) {
      rinv = rsqrt(pp);
      ajnorm = pp * rinv;
    } else {
      ajnorm = sqrt(pp);
      rinv = 1.0 / ajnorm;
    }
    rajjv[j] = 0.0;
    if (ajnorm != 0.0) {
      if (gbcast<G>(a[0][j], j) < 0.0) {
        ajnorm = -ajnorm;
        rinv = -rinv;
      }
#pragma unroll
      for (int k = 0; k < MPL; ++k)
        if (row_ge(gl, k, j)) a[k][j] = la_quot(a[k][j], ajnorm, rinv);
      if (gl == j) a[0][j] = a[0][j] + 1.0;
      double d[N];
#pragma unroll
      for (int c = 0; c < N; ++c) {
        double q = 0.0;
        if (c > j) {
#pragma unroll
          for (int k = 0; k < MPL; ++k)
            if (row_ge(gl, k, j)) q += a[k][j] * a[k][c];
        }
        d[c] = q;
      }
      gsum_from<N, G>(d, j + 1);
      const double ajj = gbcast<G>(a[0][j], j);
      const double rajj = 1.0 / ajj;
      rajjv[j] = rajj;
#pragma unroll
      for (int c = j + 1; c < N; ++c) {
        const double temp = la_quot(d[c], ajj, rajj);
#pragma unroll
        for (int k = 0; k < MPL; ++k)
          if (row_ge(gl, k, j)) a[k][c] = a[k][c] - temp * a[k][j];
        if (nrm[c] != 0.0) {
          const double ajc = gbcast<G>(a[0][c], j);
          bool lost;
          if constexpr (SQ) {  // r^2 - a^2, and 0.05 (r / wa)^2 <= epsmch on the squares
            nrm[c] = fmax(0.0, nrm[c] - ajc * ajc);
            lost = 0.05 * nrm[c] <= EPSMCH * wa[c];
          } else {
            const double t2 = ajc / nrm[c];
            nrm[c] = nrm[c] * sqrt(fmax(0.0, 1.0 - t2 * t2));
            lost = la_norm_lost(nrm[c], wa[c]);
          }
          if (lost) {
            double r = 0.0;
#pragma unroll
            for (int k = 0; k < MPL; ++k)
              if (row_ge(gl, k, j + 1)) r += a[k][c] * a[k][c];
            r = gsum<G>(r);
            nrm[c] = SQ ? r : sqrt(r);
            wa[c] = nrm[c];
          }
        }
      }
    }
    rdiag[j] = -ajnorm;
  }
}

// Hand-over of an accepted trial's residuals (and the functor's cached terms, e.g. the exp
// factors) to the slot's next O-phase, through per-wave global scratch laid out
// [slot][word][group lane]: MINPACK's fvec = wa4 after a successful step, instead of
// evaluating the function at the new x once more.  nullptr: re-evaluate (same bits).
template <int MPL, class Fn, int G = GLM_G>
struct HandOver {
  using Cache = typename FnCache<Fn>::type;
  static constexpr int CW = HasCols<Fn>::value ? (int)(sizeof(Cache) / sizeof(double)) : 0;
  static constexpr int K = MPL + CW;  // doubles per group lane per slot
  static constexpr int WORDS = K * G;  // doubles per slot
  __device__ static __forceinline__ void put(double* hand, int f, const double (&fv)[MPL],
                                             const Cache& c) {
    double* h = hand + (size_t)f * WORDS + glane<G>();
#pragma unroll
    for (int k = 0; k < MPL; ++k) h[k * G] = fv[k];
    if constexpr (CW > 0) {
      double w[CW > 0 ? CW : 1];
      __builtin_memcpy(w, &c, sizeof(Cache));
#pragma unroll
      for (int i = 0; i < CW; ++i) h[(MPL + i) * G] = w[i];
    }
  }
  __device__ static __forceinline__ void get(const double* hand, int f, double (&fv)[MPL],
                                             Cache& c) {
    const double* h = hand + (size_t)f * WORDS + glane<G>();
#pragma unroll
    for (int k = 0; k < MPL; ++k) fv[k] = h[k * G];
    if constexpr (CW > 0) {
      double w[CW > 0 ? CW : 1];
#pragma unroll
      for (int i = 0; i < CW; ++i) w[i] = h[(MPL + i) * G];
      __builtin_memcpy(&c, w, sizeof(Cache));
    }
  }
};

// Cost probes (timing builds only, never the product): -DPFE_DUP_EVAL evaluates every trial
// point twice, -DPFE_DUP_COLS every Jacobian column twice, -DPFE_DUP_QR factors every
// Jacobian twice (the copies' results are kept live and dropped), so the time each adds is
// the cost of that part of the solver (tools/ab_lib_bates.sh)
template <int M>
__device__ __forceinline__ void probe_keep(const double (&a)[M]) {
#pragma unroll
  for (int k = 0; k < M; ++k) asm volatile("" ::"v"(a[k]));
}

// O-phase for slot f (one group): residuals at S.x (a fresh fit also initialises par, delta,
// xnorm, the counters and fnorm), the forward-difference Jacobian, QR, Q^T f, R -> LDS.
// Leaves info = -1 (the gtol test runs in the next SIMT phase).
template <int N, int MPL, int FPW, int G = GLM_G, class Fn>
__device__ __forceinline__ void glm_outer(const Fn& fcn, int f, BlmState<N, FPW>& S, bool fresh,
                                          const double* hand) {
  const double eps = 1.4901161193847656e-08;  // sqrt(max(epsfcn, epsmch)) = 2^-26
  const int gl = glane<G>();
  double x[N], fvec[MPL];
  typename FnCache<Fn>::type cache;
#pragma unroll
  for (int j = 0; j < N; ++j) x[j] = S.x[j][f];
  // the residuals at x: for an accepted step the trial's residuals, handed over or
  // recomputed (same function, same operands: the same bits)
  if (!fresh && hand)
    HandOver<MPL, Fn, G>::get(hand, f, fvec, cache);
  else
    fn_eval<Fn, N, MPL>(fcn, x, fvec, cache);
  int iter, nfev;
  double fnorm;
  if (fresh) {
    fnorm = enorm_g<MPL, G>(fvec);
    iter = 1;
    nfev = 1;
  } else {
    fnorm = S.fnorm[f];
    iter = S.iter[f];
    nfev = S.nfev[f];
  }
  double fjac[MPL][N], wa4[MPL];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const double temp = x[j];
    double h = eps * fabs(temp);
    if (h == 0.0) h = eps;
    x[j] = temp + h;
#ifdef PFE_DUP_COLS
    {
      double w2[MPL];
      fn_eval_col<Fn, N, MPL>(fcn, x, j, temp, w2, cache);
      probe_keep(w2);
    }
#endif
    fn_eval_col<Fn, N, MPL>(fcn, x, j, temp, wa4, cache);
    x[j] = temp;
    const double rh = 1.0 / h;
#pragma unroll
    for (int k = 0; k < MPL; ++k) fjac[k][j] = la_quot(wa4[k] - fvec[k], h, rh);
  }
  nfev += N;
  int ipvt[N];
  double rdiag[N], acn[N], rajjv[N];
#ifdef PFE_DUP_QR
  {
    double a2[MPL][N], r2[N], c2[N], j2[N];
    int p2[N];
#pragma unroll
    for (int k = 0; k < MPL; ++k)
#pragma unroll
      for (int j = 0; j < N; ++j) a2[k][j] = fjac[k][j];
    qrfac_g<N, MPL, G>(a2, p2, r2, c2, j2);
    probe_keep(r2);
    probe_keep(j2);
  }
#endif
  qrfac_g<N, MPL, G>(fjac, ipvt, rdiag, acn, rajjv);
  // the contracted build leaves acn squared and the scaling (diag, and xnorm / delta of a
  // fresh fit) to the next SIMT phase, one fit per lane (blm_simt<.., true>)
  constexpr bool SQ = !LA_EXACT_QUOTIENTS;
  double diag[N];
  double xnorm = 0.0, delta = 0.0;
  if (SQ) {
  } else if (iter == 1) {
    double wa3[N];
#pragma unroll
    for (int j = 0; j < N; ++j) {
      diag[j] = acn[j];
      if (acn[j] == 0.0) diag[j] = 1.0;
    }
#pragma unroll
    for (int j = 0; j < N; ++j) wa3[j] = diag[j] * x[j];
    xnorm = enorm_u(wa3);
    delta = LM_FACTOR * xnorm;
    if (delta == 0.0) delta = LM_FACTOR;
  } else {
#pragma unroll
    for (int j = 0; j < N; ++j) diag[j] = S.diag[j][f];
  }
  double qtf[N];
#pragma unroll
  for (int k = 0; k < MPL; ++k) wa4[k] = fvec[k];
  {
  PFE_LA_CONTRACT
#pragma unroll
  for (int j = 0; j < N; ++j) {
    const double ajj = gbcast<G>(fjac[0][j], j);
    if (ajj != 0.0) {
      double p = 0.0;
#pragma unroll
      for (int k = 0; k < MPL; ++k)
        if (row_ge(gl, k, j)) p += fjac[k][j] * wa4[k];
      const double sum = gsum<G>(p);
      const double temp = la_quot(-sum, ajj, rajjv[j]);
#pragma unroll
      for (int k = 0; k < MPL; ++k)
        if (row_ge(gl, k, j)) wa4[k] = wa4[k] + fjac[k][j] * temp;
    }
    if (gl == j) fjac[0][j] = rdiag[j];
    qtf[j] = gbcast<G>(wa4[0], j);
  }
  }
#pragma unroll
  for (int j = 0; j < N; ++j)
    if (gl <= j) S.r[tri_idx(0, j) + gl][f] = fjac[0][j];
  if (gl == 0) {
#pragma unroll
    for (int j = 0; j < N; ++j) {
      if (!SQ) S.diag[j][f] = fmax(diag[j], acn[j]);
      S.qtf[j][f] = qtf[j];
      S.acn[j][f] = acn[j];
      S.ipvt[j][f] = ipvt[j];
    }
    if (!SQ && iter == 1) {
      S.xnorm[f] = xnorm;
      S.delta[f] = delta;
    }
    if (fresh) S.par[f] = 0.0;
    S.info[f] = -1;
    S.nfev[f] = nfev;
    S.iter[f] = iter;
    S.fnorm[f] = fnorm;
  }
}

// T-phase for slot f (one group): evaluate the trial point, update delta/par, accept or
// reject, convergence tests.  Returns the slot's next phase.
template <int N, int MPL, int FPW, int G = GLM_G, class Fn>
__device__ __forceinline__ int glm_trial(const Fn& fcn, int f, BlmState<N, FPW>& S, int maxfev,
                                         double* hand) {
  const int gl = glane<G>();
  double wa2[N], wa4[MPL];
  typename FnCache<Fn>::type cache;
#pragma unroll
  for (int j = 0; j < N; ++j) wa2[j] = S.trial[j][f];
#ifdef PFE_DUP_EVAL
  {
    double w2[MPL];
    typename FnCache<Fn>::type c2;
    fn_eval<Fn, N, MPL>(fcn, wa2, w2, c2);
    probe_keep(w2);
  }
#endif
  fn_eval<Fn, N, MPL>(fcn, wa2, wa4, cache);
  const int nfev = S.nfev[f] + 1;
  const double fnorm1 = enorm_g<MPL, G>(wa4);
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
  if (hand && accepted && info == 0) HandOver<MPL, Fn, G>::put(hand, f, wa4, cache);
  if (gl == 0) {
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
  return info != 0 ? PH_DONE : accepted ? PH_OUTER : PH_LMPAR;
}

// Per-slot bookkeeping of a pooled kernel (LDS): the candidate a slot works on, the stage
// of its fit sequence and a few per-fit values; ph/list belong to the engine.
template <int FPW>
struct SlotTab {
  long long cand[FPW];  // candidate of the slot's fit, -1 = none
  int pass[FPW];        // stage of the candidate's fit sequence
  int mpad[FPW];        // rows [0, mpad) take part
  double d0[FPW], d1[FPW], d2[FPW];  // per-fit values of the problem
  int ph[FPW];          // engine phase
  int list[FPW];        // engine scratch
};

// next item of a work queue (whole wave; wave-uniform)
__device__ __forceinline__ int64_t queue_next(unsigned* ctr) {
  unsigned c = 0;
  if (lane_id() == 0) c = atomicAdd(ctr, 1u);
  return (int64_t)(unsigned)__builtin_amdgcn_readfirstlane((int)c);
}

// Hand the slots of `mask` to the groups, NG = 64/G per round; body(f) runs in the group
// that owns slot f (lanes of other groups are masked off).
template <int G, class Body>
__device__ __forceinline__ void glm_rounds(uint64_t mask, int* list, const Body& body) {
  const int lane = lane_id();
  const int cnt = __builtin_popcountll(mask);
  if ((mask >> lane) & 1ull) list[__builtin_popcountll(mask & ((1ull << lane) - 1ull))] = lane;
  blm_sync();
  const int g = lane / G;
  for (int base = 0; base < cnt; base += 64 / G) {
    const int idx = base + g;
    if (idx < cnt) body(list[idx]);
  }
  blm_sync();
}

// The engine.  Prob provides (all called by the whole wave unless noted):
//   bool refill(int f, S)   -- finish slot f's previous fit if it had one (prob keeps that
//                              state), then set up its next fit: start point in S.x[.][f];
//                              false when the slot stays empty (work exhausted)
//   Fn   load(int f) const  -- (one group) the residual functor of slot f, rows r = gl + G k
//   int  maxfev(int f) const
// ph / list: LDS int[FPW] each.  hand_region: hand-over scratch of FPW x hand_k x G doubles
// per wave (block), or nullptr.  G: lanes per group (16 or 32; Prob::load lays the rows out
// for the same G).
template <int N, int MPL, int FPW, int G = GLM_G, class Prob>
__device__ __forceinline__ void glm_engine(Prob& prob, BlmState<N, FPW>& S, int* ph, int* list,
                                           double* hand_region = nullptr, int hand_k = 0) {
  static_assert(FPW <= 64, "one slot per lane in the SIMT phase");
  const int lane = lane_id();
  using Fn = std::decay_t<decltype(prob.load(0))>;
  using HO = HandOver<MPL, Fn, G>;
  double* const hand = (hand_region && HO::K <= hand_k)
                           ? hand_region + (size_t)blockIdx.x * FPW * hand_k * G
                           : nullptr;
  if (lane < FPW) ph[lane] = PH_DONE;  // every slot takes its first fit in the refill step
  blm_sync();
#ifdef PFE_LM_PROFILE
  // per-wave phase cycles, added to the global counters once at the end (slots 9 T-phase,
  // 10 total, 11 refill, 12 SIMT, 13 O-phase; 14/15 fits per O / T round x 1000)
  long long c_ref = 0, c_o = 0, c_s = 0, c_t = 0, n_o = 0, n_t = 0, r_o = 0, r_t = 0;
  const long long c_start = lm_clock();
#endif
  for (;;) {
    // refill slots whose fit has ended
#ifdef PFE_LM_PROFILE
    long long t0 = lm_clock();
#endif
    const uint64_t done = __ballot(lane < FPW && ph[lane < FPW ? lane : 0] == PH_DONE);
    for (uint64_t m = done; m; m &= m - 1) {
      const int f = __builtin_ctzll(m);
      const bool got = prob.refill(f, S);
      if (lane == 0) ph[f] = got ? PH_INIT : PH_EMPTY;
      blm_sync();
    }
    blm_sync();
    const int myph = lane < FPW ? ph[lane] : PH_EMPTY;
    if (__ballot(myph != PH_EMPTY) == 0) break;
#ifdef PFE_LM_PROFILE
    long long t1 = lm_clock();
    c_ref += t1 - t0;
    t0 = t1;
#endif
    // O-phase: fresh fits and accepted steps
    const uint64_t mo = __ballot(myph == PH_INIT || myph == PH_OUTER);
    if (mo) {
      glm_rounds<G>(mo, list, [&](int f) {
        const auto fn = prob.load(f);
        glm_outer<N, MPL, FPW, G>(fn, f, S, ph[f] == PH_INIT, hand);
      });
      if ((mo >> lane) & 1ull) ph[lane] = PH_LMPAR;
      blm_sync();
    }
#ifdef PFE_LM_PROFILE
    t1 = lm_clock();
    c_o += t1 - t0;
    t0 = t1;
    n_o += __builtin_popcountll(mo);
    r_o += (__builtin_popcountll(mo) + 3) / 4;
#endif
    // SIMT phase: the gtol test after a new Jacobian, lmpar, the trial point
    if (lane < FPW && ph[lane] == PH_LMPAR) {
      blm_simt<N, FPW, !LA_EXACT_QUOTIENTS>(lane, S);
      ph[lane] = S.info[lane] != 0 ? PH_DONE : PH_TRIAL;
    }
    blm_sync();
#ifdef PFE_LM_PROFILE
    t1 = lm_clock();
    c_s += t1 - t0;
    t0 = t1;
#endif
    // T-phase
    const uint64_t mt = __ballot(lane < FPW && ph[lane < FPW ? lane : 0] == PH_TRIAL);
    if (mt) {
      glm_rounds<G>(mt, list, [&](int f) {
        const auto fn = prob.load(f);
        const int nph = glm_trial<N, MPL, FPW, G>(fn, f, S, prob.maxfev(f), hand);
        if (glane<G>() == 0) ph[f] = nph;
      });
      // slots change groups between phases: the hand-over stores precede the next loads
      if (hand) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    }
#ifdef PFE_LM_PROFILE
    c_t += lm_clock() - t0;
    n_t += __builtin_popcountll(mt);
    r_t += (__builtin_popcountll(mt) + 3) / 4;
#endif
  }
#ifdef PFE_LM_PROFILE
  LM_ADD(9, c_t);
  LM_ADD(10, lm_clock() - c_start);
  LM_ADD(11, c_ref);
  LM_ADD(12, c_s);
  LM_ADD(13, c_o);
  LM_ADD(14, r_o ? 1000 * n_o / r_o : 0);
  LM_ADD(15, r_t ? 1000 * n_t / r_t : 0);
  LM_ADD(0, 1);  // waves
#endif
}

}  // namespace pfe
