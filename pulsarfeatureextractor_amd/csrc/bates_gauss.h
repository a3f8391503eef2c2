// bates_gauss.h — scores 5-11 (Gaussian fits) on gfx950: the kernels.  They are
// instantiated by three translation units, one per launch stage of the chain (the stages
// compile in parallel): bates_gauss.hip (histogram fits + the chain's launcher),
// bates_gauss_peel.hip (T1 fit and peel passes), bates_gauss_dg8.hip (8-parameter fit).
//
// Reference: ProfileOperations.getGaussianFittings (PulsarFeatureExtractor/src/
// ProfileOperations.py:595-770) with freedmanDiaconisRule / getDerivative
// (ProfileOperationsInterface.py:138-186), numpy.histogram, fitGaussian :774-983,
// fitGaussianFixedWidthBins :988-1057, fitGaussianT1 :1061-1132 ->
// fitGaussianWithBackground :1194-1264, fitDoubleGaussianT2 :1136-1190 ->
// fitDoubleGaussian :1268-1428 -> fitDoubleGaussianWithBackground :1432-1483.
//
// Three kernels (launched in this order on one stream):
//   k_ghist  : Freedman-Diaconis bin counts, the two histograms and their Gaussian fits
//              -> s5, s6, s7 and mu of the profile-histogram fit (workspace)
//   k_gt1    : background-subtracted, half-rotated profile, 4-parameter fit -> s8, s9
//   k_gdg    : peak peeling, 8 single-Gaussian passes with subtraction, the 8-parameter
//              fit and the combination rule -> s10, s11
#pragma once

#include "bates_common.h"
#include <type_traits>

#include "lm_batch.h"
#include "lm_global.h"
#include "lm_group.h"
#include "np_sum.h"

namespace pfe {
// t = (x - mu) / sigma for every row of a fit.  With y = RN(1/sigma), q = RN(a*y) is within
// an ulp of a/sigma, r = a - q*sigma is exact in an fma, and q + r*y rounds to RN(a/sigma)
// (Markstein's theorem) whenever nothing under- or overflows: three instructions per row
// instead of the ~11 of an IEEE division, the same bits.  The Gaussian models only use t*t:
// with |sigma| in [2^-500, 2^500] and |mu|, |x| <= 2^400 every quotient is either correctly
// rounded or smaller than 2^-400, where t*t is 0 either way; outside that range (diverging
// fits) the rows divide.
struct RecipDiv {
  double b, y;
  __device__ __forceinline__ double operator()(double a) const {
    const double q = a * y;
    const double r = fma(-q, b, a);
    return fma(r, y, q);
  }
};
struct PlainDiv {
  double b;
  __device__ __forceinline__ double operator()(double a) const { return a / b; }
};
// exp(-(t*t) / 2), the Gaussian models' only exponential, with the device library's own
// algorithm (ocml exp_f64: n = rint(x log2 e), the two-part reduction, its degree-12
// polynomial, ldexp) minus its x > 1024 -> +inf select, which an argument <= 0 (or NaN) never
// takes: the same bits, two instructions fewer per row and evaluation.
#ifndef PFE_GAUSS_EXP
#define PFE_GAUSS_EXP 1
#endif
__device__ __forceinline__ double exp_neg_half_sq(double t) {
  const double x = -(t * t) / 2.0;
#if PFE_GAUSS_EXP
  const double dn = __builtin_rint(x * 0x1.71547652b82fep+0);
  double f = __builtin_fma(-dn, 0x1.62e42fefa39efp-1, x);
  f = __builtin_fma(-dn, 0x1.abc9e3b39803fp-56, f);
  double p = __builtin_fma(f, 0x1.ade156a5dcb37p-26, 0x1.28af3fca7ab0cp-22);
  p = __builtin_fma(f, p, 0x1.71dee623fde64p-19);
  p = __builtin_fma(f, p, 0x1.a01997c89e6b0p-16);
  p = __builtin_fma(f, p, 0x1.a01a014761f6ep-13);
  p = __builtin_fma(f, p, 0x1.6c16c1852b7b0p-10);
  p = __builtin_fma(f, p, 0x1.1111111122322p-7);
  p = __builtin_fma(f, p, 0x1.55555555502a1p-5);
  p = __builtin_fma(f, p, 0x1.5555555555511p-3);
  p = __builtin_fma(f, p, 0x1.000000000000bp-1);
  p = __builtin_fma(f, p, 1.0);
  p = __builtin_fma(f, p, 1.0);
  const double e = __builtin_ldexp(p, (int)dn);
  return x < -1075.0 ? 0.0 : e;
#else
  return exp(x);
#endif
}

template <class Body>
__device__ __forceinline__ void with_div(double sigma, double mu, const Body& body) {
  const double as = fabs(sigma);
  if (as >= 0x1p-500 && as <= 0x1p500 && fabs(mu) <= 0x1p400)
    body(RecipDiv{sigma, 1.0 / sigma});
  else
    body(PlainDiv{sigma});
}
}  // namespace pfe

namespace pfe {

#pragma clang fp contract(off)

// ---------------------------------------------------------------------------------------
// order statistics of small integer data by bisection over the value range (ballots)
// ---------------------------------------------------------------------------------------
template <int MPL>
__device__ int kth_smallest(const int (&v)[MPL], const bool (&ok)[MPL], int k, int lo, int hi) {
  // smallest x in [lo, hi] with #(v <= x) >= k+1
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;  // floor (arithmetic shift)
    int cnt = 0;
#pragma unroll
    for (int s = 0; s < MPL; ++s) cnt += __popcll(__ballot(ok[s] && v[s] <= mid));
    if (cnt >= k + 1)
      hi = mid;
    else
      lo = mid + 1;
  }
  return lo;
}

// scipy.stats.scoreatpercentile(data, per), interpolation 'fraction'
template <int MPL>
__device__ double score_at_percentile(const int (&v)[MPL], const bool (&ok)[MPL], int n, double per,
                                      int lo, int hi) {
  const double idx = per / 100.0 * (double)(n - 1);
  const int i = (int)idx;
  if ((double)i == idx) return (double)kth_smallest<MPL>(v, ok, i, lo, hi);
  const double w0 = (double)(i + 1) - idx, w1 = idx - (double)i;
  const double si = (double)kth_smallest<MPL>(v, ok, i, lo, hi);
  const double sj = (double)kth_smallest<MPL>(v, ok, i + 1, lo, hi);
  return (si * w0 + sj * w1) / (w0 + w1);
}

// freedmanDiaconisRule (ProfileOperationsInterface.py:138-166).  c = pow(n, -0.3333333)
// computed on the host with the C library pow, as Python does.
template <int MPL>
__device__ int fd_bins(const int (&v)[MPL], const bool (&ok)[MPL], int n, double c, int vmin, int vmax) {
  const double iqr = score_at_percentile<MPL>(v, ok, n, 75.0, vmin, vmax) -
                     score_at_percentile<MPL>(v, ok, n, 25.0, vmin, vmax);
  const double bw = 2.0 * iqr * c;
  const int rng = vmax - vmin;
  if (bw <= 0.0) return rng / 60;  // binwidth = 60 (int); Py2 int '/' floors
  const double q = ceil((double)rng / bw);
  return q > 1e9 ? 1000000000 : (int)q;
}

// ---- the same for float data (PFD profiles) ----
// doubles ordered as unsigned keys (finite data)
__device__ __forceinline__ uint64_t okey(double v) {
  const uint64_t u = (uint64_t)__double_as_longlong(v);
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ double from_okey(uint64_t k) {
  const uint64_t u = (k >> 63) ? (k & 0x7FFFFFFFFFFFFFFFull) : ~k;
  return __longlong_as_double((long long)u);
}

// k-th smallest (0-based) value of v[ok] by bisection over the key range (64 ballots rounds)
template <int MPL>
__device__ double kth_smallest_f(const double (&v)[MPL], const bool (&ok)[MPL], int k) {
  uint64_t kv[MPL];
  uint64_t lo = ~0ull, hi = 0;
#pragma unroll
  for (int s = 0; s < MPL; ++s) {
    kv[s] = okey(v[s]);
    if (ok[s]) {
      lo = kv[s] < lo ? kv[s] : lo;
      hi = kv[s] > hi ? kv[s] : hi;
    }
  }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t a = (uint64_t)__shfl_xor((long long)lo, o), b = (uint64_t)__shfl_xor((long long)hi, o);
    lo = a < lo ? a : lo;
    hi = b > hi ? b : hi;
  }
  while (lo < hi) {  // smallest key K with #(key <= K) >= k+1
    const uint64_t mid = lo + ((hi - lo) >> 1);
    int cnt = 0;
#pragma unroll
    for (int s = 0; s < MPL; ++s) cnt += __popcll(__ballot(ok[s] && kv[s] <= mid));
    if (cnt >= k + 1)
      hi = mid;
    else
      lo = mid + 1;
  }
  return from_okey(lo);
}

template <int MPL>
__device__ double score_at_percentile_f(const double (&v)[MPL], const bool (&ok)[MPL], int n,
                                        double per) {
  const double idx = per / 100.0 * (double)(n - 1);
  const int i = (int)idx;
  if ((double)i == idx) return kth_smallest_f<MPL>(v, ok, i);
  const double w0 = (double)(i + 1) - idx, w1 = idx - (double)i;
  const double si = kth_smallest_f<MPL>(v, ok, i);
  const double sj = kth_smallest_f<MPL>(v, ok, i + 1);
  return (si * w0 + sj * w1) / (w0 + w1);
}

// freedmanDiaconisRule on float data: rnge / binwidth is a true division (binwidth 60 too);
// a NaN bin count (int(nan) raises ValueError) or one beyond int range returns -1
template <int MPL>
__device__ int fd_bins_f(const double (&v)[MPL], const bool (&ok)[MPL], int n, double c,
                         double vmin, double vmax) {
  const double iqr = score_at_percentile_f<MPL>(v, ok, n, 75.0) -
                     score_at_percentile_f<MPL>(v, ok, n, 25.0);
  double bw = 2.0 * iqr * c;
  if (bw <= 0.0) bw = 60.0;
  const double q = ceil((vmax - vmin) / bw);
  if (!(q == q)) return -1;
  return q > 1e9 ? 1000000000 : (int)q;
}

// numpy.histogram(data, nbins) into per-wave LDS counters
struct HistSpec {
  double first, last, step;
  int nb;
  __device__ double edge(int i) const { return i >= nb ? last : (double)i * step + first; }
};

__device__ __forceinline__ HistSpec hist_spec(double vmin, double vmax, int nb) {
  HistSpec h;
  h.first = vmin;
  h.last = vmax;
  if (vmin == vmax) {
    h.first -= 0.5;
    h.last += 0.5;
  }
  h.nb = nb;
  h.step = (h.last - h.first) / (double)nb;  // numpy.linspace: delta/div, then i*step + start
  return h;
}

__device__ __forceinline__ int hist_bin(const HistSpec& h, double v) {
  const double denom = (double)(h.last - h.first);
  int idx = (int)(((v - h.first) / denom) * (double)h.nb);
  if (idx == h.nb) idx -= 1;
  if (v < h.edge(idx)) idx -= 1;
  if (v >= h.edge(idx + 1) && idx != h.nb - 1) idx += 1;
  return idx;
}

// ---------------------------------------------------------------------------------------
// Gaussian fit to a histogram (fitGaussian :774-983)
// ---------------------------------------------------------------------------------------
template <int MPL>
struct GaussFn {  // y - |A| exp(-((x-mu)/sigma)^2 / 2)
  double x[MPL], y[MPL];
  bool ok[MPL];
  template <class D>
  __device__ __forceinline__ double model(const D& dv, const double (&p)[3], int k) const {
    const double t = dv(x[k] - p[1]);
    return fabs(p[2]) * exp_neg_half_sq(t);
  }
  __device__ __forceinline__ double model(const double (&p)[3], int k) const {
    return model(PlainDiv{p[0]}, p, k);
  }
  __device__ __forceinline__ void operator()(const double (&p)[3], double (&f)[MPL]) const {
    with_div(p[0], p[1], [&](const auto& dv) {
#pragma unroll
      for (int k = 0; k < MPL; ++k) f[k] = ok[k] ? y[k] - model(dv, p, k) : 0.0;
    });
  }
};

template <int MPL>
struct GaussFixedFn {  // mu fixed at xmax; parameters (sigma, A)
  double x[MPL], y[MPL];
  bool ok[MPL];
  double xmax;
  template <class D>
  __device__ __forceinline__ double model(const D& dv, const double (&p)[2], int k) const {
    const double t = dv(x[k] - xmax);
    return fabs(p[1]) * exp_neg_half_sq(t);
  }
  __device__ __forceinline__ double model(const double (&p)[2], int k) const {
    return model(PlainDiv{p[0]}, p, k);
  }
  __device__ __forceinline__ void operator()(const double (&p)[2], double (&f)[MPL]) const {
    with_div(p[0], xmax, [&](const auto& dv) {
#pragma unroll
      for (int k = 0; k < MPL; ++k) f[k] = ok[k] ? y[k] - model(dv, p, k) : 0.0;
    });
  }
};

struct HistFit {
  double sigma, mu, amp;
  bool fail;  // IndexError / ValueError / TypeError in the reference
};

// counts in y (nb bins, left edges in x); returns the final parameters
template <int MPL>
__device__ HistFit fit_gaussian_hist(GaussFn<MPL>& fn, int nb, int lane) {
  HistFit r{0, 0, 0, false};
  // statistics of the (unpadded) counts
  double cmax = -1.0;
  int imax = 1 << 30;
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < MPL; ++k)
    if (lane + 64 * k < nb) {
      s += fn.y[k];
      if (fn.y[k] > cmax) {
        cmax = fn.y[k];
        imax = lane + 64 * k;
      }
    }
  const ArgMax am = wargmax(cmax, imax);
  const int idx = am.i;
  const double a0 = am.v;
  const double mean = wsum(s) / (double)nb;
  double q = 0.0;
#pragma unroll
  for (int k = 0; k < MPL; ++k)
    if (lane + 64 * k < nb) {
      const double d = fn.y[k] - mean;
      q += d * d;
    }
  const double s0 = sqrt(wsum(q) / (double)nb);
  const double meansq = mean * mean;
  const int nx = nb;
  const int m = nb < 3 ? 3 : nb;  // zero-padded to the parameter count (:943-947)
#pragma unroll
  for (int k = 0; k < MPL; ++k) {
    const int i = lane + 64 * k;
    fn.ok[k] = i < m;
    if (i >= nb) {
      fn.x[k] = 0.0;
      fn.y[k] = 0.0;
    }
  }
  // left edge of bin idx (x values live in lanes)
  auto xat = [&](int i) -> double {
    double v = 0.0;
#pragma unroll
    for (int k = 0; k < MPL; ++k)
      if (i >> 6 == k) v = bcast(fn.x[k], i & 63);
    return v;
  };
  double mu0 = xat(idx);
  int retry = 0;
  double p[3];
  for (;;) {
    p[0] = s0;
    p[1] = mu0;
    p[2] = a0;
    lmdif<3, MPL>(fn, p, 200 * 4);
    double cs = 0.0;
#pragma unroll
    for (int k = 0; k < MPL; ++k)
      if (lane + 64 * k < nx) {
        const double d = fn.y[k] - fn.model(p, k);
        cs += d * d;
      }
    const double chisq = wsum(cs) / (double)m;
    if ((chisq > meansq * (double)nx) && (p[0] < 0.2 * (double)nx)) {
      ++retry;
      // temp = delete(temp, idx): after r deletions temp = counts[:idx] + counts[idx+r:]
      if (idx + retry > nb) {  // numpy.delete index out of bounds
        r.fail = true;
        return r;
      }
      double bv = -1.0;
      int bi = 1 << 30;
#pragma unroll
      for (int k = 0; k < MPL; ++k) {
        const int i = lane + 64 * k;
        if (i < nb && (i < idx || i >= idx + retry) && fn.y[k] > bv) {
          bv = fn.y[k];
          bi = i;
        }
      }
      const ArgMax t = wargmax(bv, bi);
      if (t.i >= (1 << 30)) {  // argmax of an empty array
        r.fail = true;
        return r;
      }
      const int pos = t.i < idx ? t.i : t.i - retry;
      if (pos + retry >= m) {  // xData[pos+counter] out of range
        r.fail = true;
        return r;
      }
      mu0 = xat(pos + retry);
      if (retry > 5) break;
    } else {
      break;
    }
  }
  r.sigma = p[0];
  r.mu = p[1];
  r.amp = p[2];
  return r;
}

template <int MPL>
__device__ void load_hist(GaussFn<MPL>& fn, const int* hist, const HistSpec& h, int lane) {
#pragma unroll
  for (int k = 0; k < MPL; ++k) {
    const int i = lane + 64 * k;
    fn.ok[k] = i < h.nb;
    fn.x[k] = i < h.nb ? h.edge(i) : 0.0;
    fn.y[k] = i < h.nb ? (double)hist[i] : 0.0;
  }
}

// The profile, its derivative (getDerivative :170-186) and their Freedman-Diaconis bin
// counts (:654-656) for candidate c.  F = float profiles (the PFD path): float order
// statistics and true-division bin counts; nan = the profile holds a NaN (numpy.histogram
// raises on the non-finite range).
template <int P, bool F>
struct GhPre {
  using V = typename std::conditional<F, double, int>::type;
  V v[P], d[P];
  bool okv[P], okd[P];
  int hb, db;
  double vmin, vmax, dmin, dmax;
  bool nan;
};

template <int P, bool F>
__device__ __forceinline__ void ghist_prologue(const BatesArgs& a, int64_t c, GhPre<P, F>& g) {
  const int lane = lane_id();
  const int lp = a.lp;
  g.nan = false;
#pragma unroll
  for (int k = 0; k < P; ++k) {
    const int i = lane + 64 * k;
    g.okv[k] = i < lp;
    g.okd[k] = i < lp - 1;
    if constexpr (F) {
      const double* row = a.fprof + c * lp;
      g.v[k] = g.okv[k] ? row[i] : 0.0;
      g.d[k] = g.okd[k] ? row[i] - row[i + 1] : 0.0;  // getDerivative (:170-186)
    } else {
      const uint8_t* row = a.prof + c * lp;
      g.v[k] = g.okv[k] ? (int)row[i] : 0;
      g.d[k] = g.okd[k] ? (int)row[i] - (int)row[i + 1] : 0;
    }
  }
  if constexpr (F) {
    double vmin = INFINITY, vmax = -INFINITY, dmin = INFINITY, dmax = -INFINITY;
    bool nan = false;
#pragma unroll
    for (int k = 0; k < P; ++k) {
      if (g.okv[k]) {
        nan |= !(g.v[k] == g.v[k]);
        vmin = fmin(vmin, g.v[k]);
        vmax = fmax(vmax, g.v[k]);
      }
      if (g.okd[k]) {
        dmin = fmin(dmin, g.d[k]);
        dmax = fmax(dmax, g.d[k]);
      }
    }
    g.vmin = wmin(vmin);
    g.vmax = wmax(vmax);
    g.dmin = wmin(dmin);
    g.dmax = wmax(dmax);
    if (__ballot(nan)) {
      g.nan = true;
      g.hb = g.db = 0;
      return;
    }
    g.hb = fd_bins_f<P>(g.v, g.okv, lp, a.c_lp, g.vmin, g.vmax);        // :654
    g.db = fd_bins_f<P>(g.d, g.okd, lp - 1, a.c_lp1, g.dmin, g.dmax);   // :656
  } else {
    int vmin = 1 << 30, vmax = -(1 << 30), dmin = 1 << 30, dmax = -(1 << 30);
#pragma unroll
    for (int k = 0; k < P; ++k) {
      if (g.okv[k]) {
        vmin = min(vmin, g.v[k]);
        vmax = max(vmax, g.v[k]);
      }
      if (g.okd[k]) {
        dmin = min(dmin, g.d[k]);
        dmax = max(dmax, g.d[k]);
      }
    }
    vmin = wmin_i(vmin);
    vmax = wmax_i(vmax);
    dmin = wmin_i(dmin);
    dmax = wmax_i(dmax);
    g.hb = fd_bins<P>(g.v, g.okv, lp, a.c_lp, vmin, vmax);        // :654
    g.db = fd_bins<P>(g.d, g.okd, lp - 1, a.c_lp1, dmin, dmax);   // :656
    g.vmin = vmin;
    g.vmax = vmax;
    g.dmin = dmin;
    g.dmax = dmax;
  }
}

// numpy.histogram counts of val[ok] into LDS hist[0, h.nb)
template <int P, class V>
__device__ __forceinline__ void build_hist(int* hist, const HistSpec& h, const V (&val)[P],
                                           const bool (&ok)[P]) {
  const int lane = lane_id();
  __builtin_amdgcn_wave_barrier();
  for (int i = lane; i < h.nb; i += 64) hist[i] = 0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int k = 0; k < P; ++k)
    if (ok[k]) atomicAdd(&hist[hist_bin(h, val[k])], 1);
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// profile.mean(), profile.std() (:724, :730): exact integer sums, or numpy's pairwise sums
// of a float profile (sg: LDS stage of 64P doubles)
template <int P, bool F>
__device__ __forceinline__ MeanStd ghist_meanstd(const GhPre<P, F>& g, int lp, double* sg) {
  const int lane = lane_id();
  MeanStd ms;
  if constexpr (F) {
#pragma unroll
    for (int k = 0; k < P; ++k)
      if (g.okv[k]) sg[lane + 64 * k] = g.v[k];
    lds_sync();
    ms.mean = np_pairwise<4>(sg, lp, lane) / (double)lp;
    lds_sync();
#pragma unroll
    for (int k = 0; k < P; ++k)
      if (g.okv[k]) {
        const double t = g.v[k] - ms.mean;
        sg[lane + 64 * k] = t * t;
      }
    lds_sync();
    ms.std = sqrt(np_pairwise<4>(sg, lp, lane) / (double)lp);
    lds_sync();
  } else {
    ms = int_mean_std<P>(g.v, lp, lane);
  }
  return ms;
}

// P = slots of the profile (lp <= 64*P), H = histogram-bin slots (nb <= 64*H);
// BIG: only candidates deferred with ST_DEFER_HIST (more than 256 bins);
// D64: only candidates the pooled kernels deferred with ST_DEFER_HIST64 (more than 64 bins);
// F = float profiles (the PFD path): float order statistics, true-division bin counts and
// numpy's pairwise mean / std instead of the exact integer forms
template <int P, int H, bool BIG, bool F, bool D64 = false>
__global__ __launch_bounds__(BLOCK) void k_ghist(BatesArgs a) {
  __shared__ int hist_all[BLOCK / 64][64 * H];
  __shared__ double stage_all[BLOCK / 64][F ? 64 * P : 1];
  const int64_t c = wave_candidate();
  if (c >= a.n) return;
  if constexpr (BIG) {
    if (!(a.status[c] & ST_DEFER_HIST)) return;
  }
  if constexpr (D64) {
    if (!(a.status[c] & ST_DEFER_HIST64)) return;
  }
  const int lane = lane_id();
  const int wv = threadIdx.x >> 6;
  int* hist = hist_all[wv];
  const int lp = a.lp;
  GhPre<P, F> g;
  ghist_prologue<P, F>(a, c, g);
  if (D64 && lane == 0) atomicAnd(&a.status[c], ~(uint32_t)(ST_DEFER_HIST64));
  if (g.nan) {  // numpy.histogram: autodetected range is not finite (ValueError)
    if (lane == 0) atomicOr(&a.status[c], (uint32_t)(PFE_ST_GAUSS_FAIL));
    return;
  }
  const int hb = g.hb, db = g.db;
  uint32_t st = 0;
  if (hb <= 0 || db <= 0) st = PFE_ST_GAUSS_FAIL;                  // histogram(bins=0) raises
  if (!st && (hb > 64 * H || db > 64 * H)) {
    if (!BIG)
      st = ST_DEFER_HIST;
    else if (hb > WIDE_MAX_BINS || db > WIDE_MAX_BINS)
      st = PFE_ST_UNSUPPORTED | ST_GAUSS_UNSUP;
    else {  // queue for k_ghist_wide (rows in global scratch)
      st = ST_DEFER_WIDE;
      if (lane == 0) a.wide_list[atomicAdd(a.counters + CTR_WIDE, 1u)] = (int)c;
    }
  }
  if (BIG && lane == 0) atomicAnd(&a.status[c], ~(uint32_t)(ST_DEFER_HIST));
  if (st) {
    if (lane == 0) atomicOr(&a.status[c], (uint32_t)(st));
    return;
  }
  // ---- derivative histogram and its fit (:657-661)
  const HistSpec hd = hist_spec(g.dmin, g.dmax, db);
  build_hist<P>(hist, hd, g.d, g.okd);
  GaussFn<H> fn;
  load_hist<H>(fn, hist, hd, lane);
  const HistFit fd = fit_gaussian_hist<H>(fn, db, lane);
  // ---- profile histogram and its fits (:678-705)
  const HistSpec hp = hist_spec(g.vmin, g.vmax, hb);
  build_hist<P>(hist, hp, g.v, g.okv);
  load_hist<H>(fn, hist, hp, lane);
  GaussFixedFn<H> fx;
#pragma unroll
  for (int k = 0; k < H; ++k) {
    fx.x[k] = fn.x[k];
    fx.y[k] = fn.y[k];
    fx.ok[k] = fn.ok[k];
  }
  const HistFit fp = fit_gaussian_hist<H>(fn, hb, lane);
  if (fd.fail || fp.fail || hb < 2) {  // hb < 2: leastsq(m=1 < n=2) raises TypeError
    if (lane == 0) atomicOr(&a.status[c], (uint32_t)(PFE_ST_GAUSS_FAIL));
    return;
  }
  // fixed-mean fit (:1034-1045): xmax = xData[int(bins/2)-1] (index -1 = last bin)
  int xi = hb / 2 - 1;
  if (xi < 0) xi += hb;
  fx.xmax = hp.edge(xi);
  double cmax = -1.0, s = 0.0;
#pragma unroll
  for (int k = 0; k < H; ++k)
    if (fx.ok[k]) {
      cmax = fmax(cmax, fx.y[k]);
      s += fx.y[k];
    }
  cmax = wmax(cmax);
  const double mean = wsum(s) / (double)hb;
  double q = 0.0;
#pragma unroll
  for (int k = 0; k < H; ++k)
    if (fx.ok[k]) q += (fx.y[k] - mean) * (fx.y[k] - mean);
  double pf[2] = {sqrt(wsum(q) / (double)hb), cmax};
  lmdif<2, H>(fx, pf, 200 * 3);
  const MeanStd ms = ghist_meanstd<P, F>(g, lp, stage_all[wv]);
  if (lane == 0) {
    double* o = a.out + c * 22;
    o[4] = fabs(fx.xmax - fp.mu);          // s5 (:715)
    o[5] = fabs(pf[1] / fp.amp);           // s6 (:716)
    o[6] = fabs(fd.mu - fp.mu);            // s7 (:717)
    GaussWS* w = a.ws + c;
    w->p_mu = fp.mu;
    w->minbg = py_min(fp.mu, ms.mean);     // :724
    w->pstd = ms.std;
  }
}

// ---------------------------------------------------------------------------------------
// Histograms wider than 1024 bins (k_ghist_wide): the profile histogram of a near-flat
// quantised profile has thousands of Freedman-Diaconis bins (an IQR of 1/4 over a range of
// 255).  Same fits as k_ghist, with the m rows of each solve in per-wave global scratch
// (lm_global.h) and the counts in global memory; the bin edges are recomputed from the
// HistSpec on every evaluation.  Candidates arrive through a queue filled by k_ghist<BIG>.
// ---------------------------------------------------------------------------------------
struct WideHist {  // counts of nb bins (rows >= nb are the zero padding up to m)
  const int* cnt;
  HistSpec h;
  int nb, m;
  __device__ __forceinline__ double x(int i) const { return i < nb ? h.edge(i) : 0.0; }
  __device__ __forceinline__ double y(int i) const { return i < nb ? (double)cnt[i] : 0.0; }
};

struct GaussFnWide {  // y - |A| exp(-((x-mu)/sigma)^2 / 2) over the rows of a WideHist
  WideHist w;
  int nsl;
  template <class D>
  __device__ __forceinline__ double model(const D& dv, const double (&p)[3], double xv) const {
    const double t = dv(xv - p[1]);
    return fabs(p[2]) * exp_neg_half_sq(t);
  }
  __device__ __forceinline__ void operator()(const double (&p)[3], double* f) const {
    const int lane = lane_id();
    with_div(p[0], p[1], [&](const auto& dv) {
      for (int k = 0; k < nsl; ++k) {
        const int i = lane + 64 * k;
        f[k * 64 + lane] = i < w.m ? w.y(i) - model(dv, p, w.x(i)) : 0.0;
      }
    });
  }
};

struct GaussFixedFnWide {  // mu fixed at xmax; parameters (sigma, A)
  WideHist w;
  int nsl;
  double xmax;
  __device__ __forceinline__ void operator()(const double (&p)[2], double* f) const {
    const int lane = lane_id();
    with_div(p[0], xmax, [&](const auto& dv) {
      for (int k = 0; k < nsl; ++k) {
        const int i = lane + 64 * k;
        double v = 0.0;
        if (i < w.m) {
          const double t = dv(w.x(i) - xmax);
          v = w.y(i) - fabs(p[1]) * exp_neg_half_sq(t);
        }
        f[k * 64 + lane] = v;
      }
    });
  }
};

// fitGaussian (:774-983) on a wide histogram: fit_gaussian_hist with the rows in memory
__device__ HistFit fit_gaussian_hist_wide(const WideHist& w, double* scr, int lane) {
  HistFit r{0, 0, 0, false};
  const int nb = w.nb;
  const int nsl = (w.m + 63) / 64;
  double cmax = -1.0, s = 0.0;
  int imax = 1 << 30;
  for (int k = 0; k < nsl; ++k) {
    const int i = lane + 64 * k;
    if (i < nb) {
      const double v = w.y(i);
      s += v;
      if (v > cmax) {
        cmax = v;
        imax = i;
      }
    }
  }
  const ArgMax am = wargmax(cmax, imax);
  const int idx = am.i;
  const double a0 = am.v;
  const double mean = wsum(s) / (double)nb;
  double q = 0.0;
  for (int k = 0; k < nsl; ++k) {
    const int i = lane + 64 * k;
    if (i < nb) {
      const double d = w.y(i) - mean;
      q += d * d;
    }
  }
  const double s0 = sqrt(wsum(q) / (double)nb);
  const double meansq = mean * mean;
  GaussFnWide fn{w, nsl};
  const RowStore<3> rs{scr, nsl};
  double mu0 = w.x(idx);
  int retry = 0;
  double p[3];
  for (;;) {
    p[0] = s0;
    p[1] = mu0;
    p[2] = a0;
    lmdif_g<3>(fn, p, 200 * 4, rs);
    double cs = 0.0;
    for (int k = 0; k < nsl; ++k) {
      const int i = lane + 64 * k;
      if (i < nb) {
        const double d = w.y(i) - fn.model(PlainDiv{p[0]}, p, w.x(i));
        cs += d * d;
      }
    }
    const double chisq = wsum(cs) / (double)w.m;
    if ((chisq > meansq * (double)nb) && (p[0] < 0.2 * (double)nb)) {
      ++retry;
      if (idx + retry > nb) {  // numpy.delete index out of bounds
        r.fail = true;
        return r;
      }
      double bv = -1.0;
      int bi = 1 << 30;
      for (int k = 0; k < nsl; ++k) {
        const int i = lane + 64 * k;
        if (i < nb && (i < idx || i >= idx + retry) && w.y(i) > bv) {
          bv = w.y(i);
          bi = i;
        }
      }
      const ArgMax t = wargmax(bv, bi);
      if (t.i >= (1 << 30)) {
        r.fail = true;
        return r;
      }
      const int pos = t.i < idx ? t.i : t.i - retry;
      if (pos + retry >= w.m) {
        r.fail = true;
        return r;
      }
      mu0 = w.x(pos + retry);
      if (retry > 5) break;
    } else {
      break;
    }
  }
  r.sigma = p[0];
  r.mu = p[1];
  r.amp = p[2];
  return r;
}

// numpy.histogram counts of val[ok] into global cnt[0, nb)
template <int P, class V>
__device__ __forceinline__ void build_hist_wide(int* cnt, const HistSpec& h, const V (&val)[P],
                                                const bool (&ok)[P]) {
  const int lane = lane_id();
  for (int i = lane; i < h.nb; i += 64) cnt[i] = 0;
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int k = 0; k < P; ++k)
    if (ok[k]) atomicAdd(&cnt[hist_bin(h, val[k])], 1);
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "agent");
  __builtin_amdgcn_wave_barrier();
}

template <int P, bool F>
__global__ __launch_bounds__(64) void k_ghist_wide(BatesArgs a) {
  __shared__ double stage[F ? 64 * P : 1];
  const int lane = lane_id();
  const unsigned total = a.counters[CTR_WIDE];
  char* slab = (char*)a.wide_scr + (size_t)blockIdx.x * WIDE_SLAB_BYTES;
  double* scr = (double*)slab;
  int* cnt = (int*)(slab + (size_t)WIDE_MAX_BINS * 5 * sizeof(double));
  for (;;) {
    const int64_t q = queue_next(a.counters + CTR_WIDEQ);
    if (q >= (int64_t)total) break;
    const int64_t c = a.wide_list[q];
    GhPre<P, F> g;
    ghist_prologue<P, F>(a, c, g);
    const int hb = g.hb, db = g.db;
    // ---- derivative histogram and its fit (:657-661)
    const HistSpec hd = hist_spec(g.dmin, g.dmax, db);
    build_hist_wide<P>(cnt, hd, g.d, g.okd);
    const HistFit fd = fit_gaussian_hist_wide(WideHist{cnt, hd, db, db < 3 ? 3 : db}, scr, lane);
    // ---- profile histogram and its fits (:678-705)
    const HistSpec hp = hist_spec(g.vmin, g.vmax, hb);
    build_hist_wide<P>(cnt, hp, g.v, g.okv);
    const WideHist wp{cnt, hp, hb, hb < 3 ? 3 : hb};
    const HistFit fp = fit_gaussian_hist_wide(wp, scr, lane);
    uint32_t st = 0;
    if (fd.fail || fp.fail || hb < 2) st = PFE_ST_GAUSS_FAIL;
    if (!st) {
      // fixed-mean fit (:1034-1045): xmax = xData[int(bins/2)-1]
      int xi = hb / 2 - 1;
      if (xi < 0) xi += hb;
      const int nsl = (hb + 63) / 64;
      GaussFixedFnWide fx{WideHist{cnt, hp, hb, hb}, nsl, hp.edge(xi)};
      double cmax = -1.0, s = 0.0;
      for (int k = 0; k < nsl; ++k) {
        const int i = lane + 64 * k;
        if (i < hb) {
          cmax = fmax(cmax, fx.w.y(i));
          s += fx.w.y(i);
        }
      }
      cmax = wmax(cmax);
      const double mean = wsum(s) / (double)hb;
      double qq = 0.0;
      for (int k = 0; k < nsl; ++k) {
        const int i = lane + 64 * k;
        if (i < hb) qq += (fx.w.y(i) - mean) * (fx.w.y(i) - mean);
      }
      double pf[2] = {sqrt(wsum(qq) / (double)hb), cmax};
      lmdif_g<2>(fx, pf, 200 * 3, RowStore<2>{scr, nsl});
      const MeanStd ms = ghist_meanstd<P, F>(g, a.lp, stage);
      if (lane == 0) {
        double* o = a.out + c * 22;
        o[4] = fabs(fx.xmax - fp.mu);          // s5 (:715)
        o[5] = fabs(pf[1] / fp.amp);           // s6 (:716)
        o[6] = fabs(fd.mu - fp.mu);            // s7 (:717)
        GaussWS* w = a.ws + c;
        w->p_mu = fp.mu;
        w->minbg = py_min(fp.mu, ms.mean);     // :724
        w->pstd = ms.std;
      }
    }
    if (lane == 0) {
      if (st) atomicOr(&a.status[c], st);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      atomicAnd(&a.status[c], ~ST_DEFER_WIDE);
    }
  }
}

// ---------------------------------------------------------------------------------------
// Pooled group-LM forms (lm_group.h) of the histogram fits, for histograms of <= 64 bins
// (one 64-lane row in the wave layout, 4 rows per lane in a 16-lane group):
//   k_ghistg  -- fitGaussian on the derivative histogram, then on the profile histogram,
//                with the reference's retries (:949-978); each retry is a new fit in the slot
//   k_gfixg   -- fitGaussianFixedWidthBins on the profile histogram, s5-s7
// Candidates with wider histograms are marked ST_DEFER_HIST64 for k_ghist<.., D64>.
// ---------------------------------------------------------------------------------------
// the statistics fitGaussian starts from (:912-948): first argmax, its count, mean, std
struct HStats {
  int idx;
  double a0, mean, s0;
};
__device__ __forceinline__ HStats hist_stats(const GaussFn<1>& fn, int nb) {
  const int lane = lane_id();
  const bool in = lane < nb;
  const ArgMax am = wargmax(in ? fn.y[0] : -1.0, in ? lane : (1 << 30));
  const double mean = wsum(in ? fn.y[0] : 0.0) / (double)nb;
  const double d = in ? fn.y[0] - mean : 0.0;
  const double s0 = sqrt(wsum(d * d) / (double)nb);
  return {am.i, am.v, mean, s0};
}

template <int FPW>
struct HistSlots {  // per slot and stage (0 = derivative, 1 = profile histogram)
  double first[2][FPW], step[2][FPW], last[2][FPW];
  int nb[2][FPW];
};

template <int P, bool F, int FPW>
struct GhistProb {
  BatesArgs a;
  SlotTab<FPW>& T;    // pass = stage << 4 | retry
  HistSlots<FPW>& HS;
  double* cnt;        // wave scratch: counts [FPW][2][64]
  int* hist;          // LDS [64]
  double* sg;         // LDS stage (F)
  int nslots;
  __device__ __forceinline__ HistSpec spec(int st, int f) const {
    HistSpec h;
    h.first = HS.first[st][f];
    h.step = HS.step[st][f];
    h.last = HS.last[st][f];
    h.nb = HS.nb[st][f];
    return h;
  }
  // wave layout: the data rows of slot f's stage st (as load_hist + the zero padding)
  __device__ __forceinline__ GaussFn<1> wave_rows(int st, int f) const {
    GaussFn<1> fn;
    const int lane = lane_id();
    const HistSpec h = spec(st, f);
    const int m = h.nb < 3 ? 3 : h.nb;
    fn.ok[0] = lane < m;
    fn.x[0] = lane < h.nb ? h.edge(lane) : 0.0;
    fn.y[0] = lane < h.nb ? cnt[((size_t)f * 2 + st) * 64 + lane] : 0.0;
    return fn;
  }
  __device__ __forceinline__ void start(int st, int f, BlmState<3, FPW>& S, int retry, double mu0) {
    const GaussFn<1> fn = wave_rows(st, f);
    const HStats hs = hist_stats(fn, HS.nb[st][f]);
    const double mu = retry ? mu0 : bcast(fn.x[0], hs.idx);
    if (lane_id() == 0) {
      T.pass[f] = st << 4 | retry;
      S.x[0][f] = hs.s0;
      S.x[1][f] = mu;
      S.x[2][f] = hs.a0;
    }
  }
  __device__ __forceinline__ bool refill(int f, BlmState<3, FPW>& S) {
    const int lane = lane_id();
    const int64_t c0 = T.cand[f];
    if (c0 >= 0) {
      const int st = T.pass[f] >> 4;
      int retry = T.pass[f] & 15;
      const int nb = HS.nb[st][f];
      const int m = nb < 3 ? 3 : nb;
      const GaussFn<1> fn = wave_rows(st, f);
      const double p[3] = {S.x[0][f], S.x[1][f], S.x[2][f]};
      const HStats hs = hist_stats(fn, nb);
      // the retry rule of fitGaussian (:970-978), as fit_gaussian_hist
      const double r = (lane < nb) ? fn.y[0] - fn.model(p, 0) : 0.0;
      const double chisq = wsum(r * r) / (double)m;
      bool fail = false, again = false;
      double mu0 = 0.0;
      if ((chisq > hs.mean * hs.mean * (double)nb) && (p[0] < 0.2 * (double)nb)) {
        ++retry;
        if (hs.idx + retry > nb) {
          fail = true;
        } else {
          const bool in = lane < nb && (lane < hs.idx || lane >= hs.idx + retry);
          const ArgMax t = wargmax(in ? fn.y[0] : -1.0, in ? lane : (1 << 30));
          if (t.i >= (1 << 30)) {
            fail = true;
          } else {
            const int pos = t.i < hs.idx ? t.i : t.i - retry;
            if (pos + retry >= m) {
              fail = true;
            } else {
              mu0 = bcast(fn.x[0], pos + retry);
              again = retry <= 5;
            }
          }
        }
      }
      if (again) {
        start(st, f, S, retry, mu0);
        blm_sync();
        return true;
      }
      if (fail) {
        if (lane == 0) atomicOr(&a.status[c0], (uint32_t)(PFE_ST_GAUSS_FAIL));
      } else if (st == 0) {
        if (lane == 0) a.ws[c0].fd_mu = p[1];
        start(1, f, S, 0, 0.0);
        blm_sync();
        return true;
      } else {  // the profile-histogram fit: what k_gfixg and the later kernels need
        GhPre<P, F> g;
        ghist_prologue<P, F>(a, c0, g);  // (the profile rows again, for its mean / std)
        const MeanStd ms = ghist_meanstd<P, F>(g, a.lp, sg);
        if (lane == 0) {
          GaussWS* w = a.ws + c0;
          w->p_mu = p[1];
          w->fp_amp = p[2];
          w->minbg = py_min(p[1], ms.mean);  // :724
          w->pstd = ms.std;
        }
      }
    }
    if (f < nslots) {
      for (;;) {
        const int64_t c = queue_next(a.counters + CTR_GHISTG);
        if (c >= a.n) break;
        GhPre<P, F> g;
        ghist_prologue<P, F>(a, c, g);
        uint32_t stt = 0;
        if (g.nan || g.hb <= 0 || g.db <= 0 || g.hb < 2) stt = PFE_ST_GAUSS_FAIL;
        else if (g.hb > 64 || g.db > 64) stt = ST_DEFER_HIST64;
        if (stt) {
          if (lane == 0) atomicOr(&a.status[c], (uint32_t)(stt));
          continue;
        }
        const HistSpec hd = hist_spec(g.dmin, g.dmax, g.db);
        const HistSpec hp = hist_spec(g.vmin, g.vmax, g.hb);
        double* cf = cnt + (size_t)f * 2 * 64;
        build_hist<P>(hist, hd, g.d, g.okd);
        cf[lane] = lane < hd.nb ? (double)hist[lane] : 0.0;
        build_hist<P>(hist, hp, g.v, g.okv);
        cf[64 + lane] = lane < hp.nb ? (double)hist[lane] : 0.0;
        if (lane == 0) {
          T.cand[f] = c;
          HS.first[0][f] = hd.first;
          HS.step[0][f] = hd.step;
          HS.last[0][f] = hd.last;
          HS.nb[0][f] = hd.nb;
          HS.first[1][f] = hp.first;
          HS.step[1][f] = hp.step;
          HS.last[1][f] = hp.last;
          HS.nb[1][f] = hp.nb;
          GaussWS* w = a.ws + c;
          w->h_min = g.vmin;
          w->h_max = g.vmax;
          w->hb = g.hb;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        blm_sync();
        start(0, f, S, 0, 0.0);
        blm_sync();
        return true;
      }
    }
    if (lane == 0) T.cand[f] = -1;
    blm_sync();
    return false;
  }
  __device__ __forceinline__ GaussFn<4> load(int f) const {
    GaussFn<4> fn;
    const int gl = glane();
    const int st = T.pass[f] >> 4;
    const HistSpec h = spec(st, f);
    const int m = h.nb < 3 ? 3 : h.nb;
    const double* cf = cnt + ((size_t)f * 2 + st) * 64;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = gl + GLM_G * k;
      fn.ok[k] = i < m;
      fn.x[k] = i < h.nb ? h.edge(i) : 0.0;
      fn.y[k] = i < h.nb ? cf[i] : 0.0;
    }
    return fn;
  }
  __device__ __forceinline__ int maxfev(int) const { return 200 * 4; }
};

template <int P, bool F>
__global__ __launch_bounds__(64, 2) void k_ghistg(BatesArgs a) {
  constexpr int FPW = GLM_FPW;
  __shared__ BlmState<3, FPW> S;
  __shared__ SlotTab<FPW> T;
  __shared__ HistSlots<FPW> HS;
  __shared__ int hist[64];
  __shared__ double stage[F ? 64 * P : 1];
  if (lane_id() < FPW) T.cand[lane_id()] = -1;
  blm_sync();
  double* cnt = a.wscr + (size_t)blockIdx.x * gdg_wave_scratch_doubles(a.lp);
  GhistProb<P, F, FPW> prob{a, T, HS, cnt, hist, stage, a.gslots};
  glm_engine<3, 4, FPW>(prob, S, T.ph, T.list, a.hand[HAND_GAUSS], HAND_K_GAUSS);
}

template <int P, bool F, int FPW>
struct GfixProb {
  BatesArgs a;
  SlotTab<FPW>& T;  // d0 = first, d1 = step, d2 = last, mpad = nb of the profile histogram
  double* cnt;      // wave scratch: counts [FPW][64]
  int* hist;        // LDS [64]
  int nslots;
  __device__ __forceinline__ HistSpec spec(int f) const {
    HistSpec h;
    h.first = T.d0[f];
    h.step = T.d1[f];
    h.last = T.d2[f];
    h.nb = T.mpad[f];
    return h;
  }
  __device__ __forceinline__ double xmax_of(const HistSpec& h) const {
    int xi = h.nb / 2 - 1;  // xData[int(bins/2)-1] (index -1 = last bin) (:1041)
    if (xi < 0) xi += h.nb;
    return h.edge(xi);
  }
  __device__ __forceinline__ bool refill(int f, BlmState<2, FPW>& S) {
    const int lane = lane_id();
    const int64_t c0 = T.cand[f];
    if (c0 >= 0 && lane == 0) {
      const GaussWS* w = a.ws + c0;
      const double xmax = xmax_of(spec(f));
      double* o = a.out + c0 * 22;
      o[4] = fabs(xmax - w->p_mu);         // s5 (:715)
      o[5] = fabs(S.x[1][f] / w->fp_amp);  // s6 (:716)
      o[6] = fabs(w->fd_mu - w->p_mu);     // s7 (:717)
    }
    if (f < nslots) {
      for (;;) {
        const int64_t c = queue_next(a.counters + CTR_GFIXG);
        if (c >= a.n) break;
        if (a.status[c] & (PFE_ST_GAUSS_FAIL | ST_DEFER_HIST64)) continue;
        const GaussWS* w = a.ws + c;
        const HistSpec hp = hist_spec(w->h_min, w->h_max, w->hb);
        GhPre<P, F> g;  // the profile rows (the bin counts are not needed again)
#pragma unroll
        for (int k = 0; k < P; ++k) {
          const int i = lane + 64 * k;
          g.okv[k] = i < a.lp;
          if constexpr (F)
            g.v[k] = g.okv[k] ? a.fprof[c * a.lp + i] : 0.0;
          else
            g.v[k] = g.okv[k] ? (int)a.prof[c * a.lp + i] : 0;
        }
        build_hist<P>(hist, hp, g.v, g.okv);
        const bool in = lane < hp.nb;
        const double y = in ? (double)hist[lane] : 0.0;
        cnt[(size_t)f * 64 + lane] = y;
        // start point (:1034-1045): std of the counts, their maximum
        const double cmax = wmax(in ? y : -1.0);
        const double mean = wsum(y) / (double)hp.nb;
        const double d = in ? y - mean : 0.0;
        const double s0 = sqrt(wsum(d * d) / (double)hp.nb);
        if (lane == 0) {
          T.cand[f] = c;
          T.d0[f] = hp.first;
          T.d1[f] = hp.step;
          T.d2[f] = hp.last;
          T.mpad[f] = hp.nb;
          S.x[0][f] = s0;
          S.x[1][f] = cmax;
        }
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
        blm_sync();
        return true;
      }
    }
    if (lane == 0) T.cand[f] = -1;
    blm_sync();
    return false;
  }
  __device__ __forceinline__ GaussFixedFn<4> load(int f) const {
    GaussFixedFn<4> fn;
    const int gl = glane();
    const HistSpec h = spec(f);
    const double* cf = cnt + (size_t)f * 64;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int i = gl + GLM_G * k;
      fn.ok[k] = i < h.nb;
      fn.x[k] = i < h.nb ? h.edge(i) : 0.0;
      fn.y[k] = i < h.nb ? cf[i] : 0.0;
    }
    fn.xmax = xmax_of(h);
    return fn;
  }
  __device__ __forceinline__ int maxfev(int) const { return 200 * 3; }
};

template <int P, bool F>
__global__ __launch_bounds__(64, 2) void k_gfixg(BatesArgs a) {
  constexpr int FPW = GLM_FPW;
  __shared__ BlmState<2, FPW> S;
  __shared__ SlotTab<FPW> T;
  __shared__ int hist[64];
  if (lane_id() < FPW) T.cand[lane_id()] = -1;
  blm_sync();
  double* cnt = a.wscr + (size_t)blockIdx.x * gdg_wave_scratch_doubles(a.lp);
  GfixProb<P, F, FPW> prob{a, T, cnt, hist, a.gslots};
  glm_engine<2, 4, FPW>(prob, S, T.ph, T.list, a.hand[HAND_GAUSS], HAND_K_GAUSS);
}

// ---------------------------------------------------------------------------------------
// s8, s9: fitGaussianT1 -> fitGaussianWithBackground
// ---------------------------------------------------------------------------------------
template <int MPL>
struct GaussBgFn {  // y - (|A| exp(-((x-mu)/|sigma|)^2/2) + bg)      (:1226)
  static constexpr bool kCols = true;  // amplitude / background columns reuse the exp
  struct Cache {
    double e[MPL];
  };
  double x[MPL], y[MPL];
  bool ok[MPL];
  template <class D>
  __device__ __forceinline__ double term(const D& dv, const double (&p)[4], int k) const {
    const double t = dv(x[k] - p[1]);
    return exp_neg_half_sq(t);
  }
  __device__ __forceinline__ double model(const double (&p)[4], int k) const {
    return fabs(p[2]) * term(PlainDiv{fabs(p[0])}, p, k) + p[3];
  }
  __device__ __forceinline__ void operator()(const double (&p)[4], double (&f)[MPL]) const {
    with_div(fabs(p[0]), p[1], [&](const auto& dv) {
#pragma unroll
      for (int k = 0; k < MPL; ++k)
        f[k] = ok[k] ? y[k] - (fabs(p[2]) * term(dv, p, k) + p[3]) : 0.0;
    });
  }
  __device__ __forceinline__ void eval(const double (&p)[4], double (&f)[MPL], Cache& c) const {
    with_div(fabs(p[0]), p[1], [&](const auto& dv) {
#pragma unroll
      for (int k = 0; k < MPL; ++k) {
        c.e[k] = ok[k] ? term(dv, p, k) : 0.0;
        f[k] = ok[k] ? y[k] - (fabs(p[2]) * c.e[k] + p[3]) : 0.0;
      }
    });
  }
  __device__ __forceinline__ void eval_col(const double (&p)[4], int j, double,
                                           double (&f)[MPL], const Cache& c) const {
    if (j < 2) {
      with_div(fabs(p[0]), p[1], [&](const auto& dv) {
#pragma unroll
        for (int k = 0; k < MPL; ++k)
          f[k] = ok[k] ? y[k] - (fabs(p[2]) * term(dv, p, k) + p[3]) : 0.0;
      });
    } else {
#pragma unroll
      for (int k = 0; k < MPL; ++k) f[k] = ok[k] ? y[k] - (fabs(p[2]) * c.e[k] + p[3]) : 0.0;
    }
  }
};

// fitGaussianT1's data (:1097-1132): the halves-rotated, background-shifted profile, and the
// start point of fitGaussianWithBackground (:1239-1245)
template <int P>
__device__ __forceinline__ void gt1_setup(const BatesArgs& a, int64_t c, const GaussWS& w,
                                          GaussBgFn<P>& fn) {
  const int lane = lane_id();
  const int lp = a.lp;
  const int cut = lp / 2;  // Py2: ceil(L/2) of an int division is L//2
#pragma unroll
  for (int k = 0; k < P; ++k) {
    const int i = lane + 64 * k;
    const bool ok = i < lp;
    fn.ok[k] = ok;
    fn.x[k] = (double)i;
    double y = 0.0;
    if (ok) {
      const int src = (i + cut) % lp;  // rotated: part2 + part1 (:1107-1109)
      const double pv = prof_at(a, c * lp + src);
      if (w.minbg > 0.0) {
        y = pv - w.minbg + w.pstd;      // :730
        if (y < 0.0) y = 0.0;
      } else {
        y = pv;
      }
    }
    fn.y[k] = y;
  }
}

template <int P>
__device__ __forceinline__ void gt1_start(const GaussBgFn<P>& fn, int lp, double (&p)[4]) {
  const int lane = lane_id();
  double bv = -INFINITY;
  int bi = 1 << 30;
#pragma unroll
  for (int k = 0; k < P; ++k)
    if (fn.ok[k] && (bi == (1 << 30) || fn.y[k] > bv)) {
      bv = fn.y[k];
      bi = lane + 64 * k;
    }
  const ArgMax am = wargmax(bv, bi);
  bool ok[P];
#pragma unroll
  for (int k = 0; k < P; ++k) ok[k] = fn.ok[k];
  const FMeanStd fs = f_mean_std<P>(fn.y, ok, lp);
  p[0] = fs.std;
  p[1] = (double)am.i;
  p[2] = am.v;
  p[3] = 1.0;
}

template <int P>
__device__ __forceinline__ void gt1_finish(const BatesArgs& a, int64_t c, const GaussBgFn<P>& fn,
                                           const double (&p)[4]) {
  const int lane = lane_id();
  double cs = 0.0;
#pragma unroll
  for (int k = 0; k < P; ++k)
    if (fn.ok[k]) {
      const double dd = fn.y[k] - fn.model(p, k);
      cs += dd * dd;
    }
  const double chisq = wsum(cs) / (double)a.lp;
  if (lane == 0) {
    double* o = a.out + c * 22;
    o[7] = fabs(FWHM_C * p[0]);  // s8 (:1247)
    o[8] = chisq;                // s9
    GaussWS* wp = a.ws + c;
    wp->t1[0] = p[0];
    wp->t1[1] = p[1];
    wp->t1[2] = p[2];
    wp->t1[3] = p[3];
  }
}

template <int P>
__global__ __launch_bounds__(BLOCK) void k_gt1(BatesArgs a) {
  const int64_t c = wave_candidate();
  if (c >= a.n) return;
  if (a.status[c] & (GAUSS_SKIP | ST_DEFER_HIST)) return;
  const GaussWS w = a.ws[c];
  GaussBgFn<P> fn;
  gt1_setup<P>(a, c, w, fn);
  double p[4];
  gt1_start<P>(fn, a.lp, p);
  lmdif<4, P>(fn, p, 200 * 5);
  gt1_finish<P>(a, c, fn, p);
}

// batched form (lm_batch.h); bit-identical to k_gt1
template <int P>
struct Gt1Loader {
  BatesArgs a;
  int64_t base;
  __device__ __forceinline__ GaussBgFn<P> operator()(int f) const {
    GaussBgFn<P> fn;
    gt1_setup<P>(a, base + f, a.ws[base + f], fn);
    return fn;
  }
};

template <int P>
__global__ __launch_bounds__(64) void k_gt1b(BatesArgs a) {
  constexpr int FPW = BLM_FPW;
  __shared__ BlmState<4, FPW> S;
  const int fpw = a.fpw;
  const int64_t base = (int64_t)blockIdx.x * fpw;
  const int lane = lane_id();
  const bool live = lane < fpw && base + lane < a.n &&
                    !(a.status[base + (lane < fpw ? lane : 0)] & (GAUSS_SKIP | ST_DEFER_HIST));
  const uint64_t fits = __ballot(live);
  if (fits == 0) return;
  const Gt1Loader<P> load{a, base};
  for (uint64_t m = fits; m; m &= m - 1) {
    const int f = __builtin_ctzll(m);
    const GaussBgFn<P> fn = load(f);
    double p[4];
    gt1_start<P>(fn, a.lp, p);
    if (lane == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) S.x[j][f] = p[j];
    }
  }
  blm_run<4, P, FPW>(load, S, fits, 200 * 5);
  for (uint64_t m = fits; m; m &= m - 1) {
    const int f = __builtin_ctzll(m);
    const GaussBgFn<P> fn = load(f);
    const double p[4] = {S.x[0][f], S.x[1][f], S.x[2][f], S.x[3][f]};
    gt1_finish<P>(a, base + f, fn, p);
  }
}

// ---------------------------------------------------------------------------------------
// s10, s11: fitDoubleGaussianT2 -> fitDoubleGaussian -> fitDoubleGaussianWithBackground
// ---------------------------------------------------------------------------------------
// Residual functors used by the batched solver also provide eval (full evaluation that
// keeps the exp terms) and eval_col (evaluation at a point that differs from the cached one
// only in parameter j): forward-difference columns of amplitude/background parameters then
// reuse the exp terms.  Same operations on the same operands, so bit-identical residuals.
template <int MPL>
struct GaussAbsBgFn {  // y - (|A| exp(-((x-mu)/sigma)^2/2) + |bg|)     (:1296)
  static constexpr bool kCols = true;
  struct Cache {
    double e[MPL];
  };
  double x[MPL], y[MPL];
  bool ok[MPL];
  template <class D>
  __device__ __forceinline__ double term(const D& dv, const double (&p)[4], int k) const {
    const double t = dv(x[k] - p[1]);
    return exp_neg_half_sq(t);
  }
  __device__ __forceinline__ void operator()(const double (&p)[4], double (&f)[MPL]) const {
    with_div(p[0], p[1], [&](const auto& dv) {
#pragma unroll
      for (int k = 0; k < MPL; ++k)
        f[k] = ok[k] ? y[k] - (fabs(p[2]) * term(dv, p, k) + fabs(p[3])) : 0.0;
    });
  }
  __device__ __forceinline__ void eval(const double (&p)[4], double (&f)[MPL], Cache& c) const {
    with_div(p[0], p[1], [&](const auto& dv) {
#pragma unroll
      for (int k = 0; k < MPL; ++k) {
        c.e[k] = ok[k] ? term(dv, p, k) : 0.0;
        f[k] = ok[k] ? y[k] - (fabs(p[2]) * c.e[k] + fabs(p[3])) : 0.0;
      }
    });
  }
  __device__ __forceinline__ void eval_col(const double (&p)[4], int j, double,
                                           double (&f)[MPL], const Cache& c) const {
    if (j < 2) {
      with_div(p[0], p[1], [&](const auto& dv) {
#pragma unroll
        for (int k = 0; k < MPL; ++k)
          f[k] = ok[k] ? y[k] - (fabs(p[2]) * term(dv, p, k) + fabs(p[3])) : 0.0;
      });
    } else {
#pragma unroll
      for (int k = 0; k < MPL; ++k)
        f[k] = ok[k] ? y[k] - (fabs(p[2]) * c.e[k] + fabs(p[3])) : 0.0;
    }
  }
};
__device__ __forceinline__ double g_absbg(double x, const double (&p)[4]) {
  const double t = (x - p[1]) / p[0];
  return fabs(p[2]) * exp_neg_half_sq(t) + fabs(p[3]);
}

template <int MPL>
struct DoubleGaussFn {  // :1459-1460
  static constexpr bool kCols = true;
  struct Cache {
    double e1[MPL], e2[MPL];
  };
  double x[MPL], y[MPL];
  bool ok[MPL];
  template <class D>
  __device__ __forceinline__ double term1(const D& dv, const double (&p)[8], int k) const {
    const double t1 = dv(x[k] - p[1]);
    return exp_neg_half_sq(t1);
  }
  template <class D>
  __device__ __forceinline__ double term2(const D& dv, const double (&p)[8], int k) const {
    const double t2 = dv(x[k] - p[5]);
    return exp_neg_half_sq(t2);
  }
  __device__ __forceinline__ double term1(const double (&p)[8], int k) const {
    return term1(PlainDiv{fabs(p[0])}, p, k);
  }
  __device__ __forceinline__ double term2(const double (&p)[8], int k) const {
    return term2(PlainDiv{fabs(p[4])}, p, k);
  }
  __device__ __forceinline__ double combine(const double (&p)[8], double e1, double e2) const {
    return (fabs(p[2]) * e1) + (fabs(p[6]) * e2) + (fabs(p[3]) + fabs(p[7])) / 2.0;
  }
  __device__ __forceinline__ double model(const double (&p)[8], int k) const {
    return combine(p, term1(p, k), term2(p, k));
  }
  __device__ __forceinline__ void operator()(const double (&p)[8], double (&f)[MPL]) const {
    Cache c;
    eval(p, f, c);
  }
  __device__ __forceinline__ void eval(const double (&p)[8], double (&f)[MPL], Cache& c) const {
    with_div(fabs(p[0]), p[1], [&](const auto& dv) {
#pragma unroll
      for (int k = 0; k < MPL; ++k) c.e1[k] = ok[k] ? term1(dv, p, k) : 0.0;
    });
    with_div(fabs(p[4]), p[5], [&](const auto& dv) {
#pragma unroll
      for (int k = 0; k < MPL; ++k) c.e2[k] = ok[k] ? term2(dv, p, k) : 0.0;
    });
#pragma unroll
    for (int k = 0; k < MPL; ++k) f[k] = ok[k] ? y[k] - combine(p, c.e1[k], c.e2[k]) : 0.0;
  }
  __device__ __forceinline__ void eval_col(const double (&p)[8], int j, double,
                                           double (&f)[MPL], const Cache& c) const {
    double e[MPL];
    if (j == 0 || j == 1) {
      with_div(fabs(p[0]), p[1], [&](const auto& dv) {
#pragma unroll
        for (int k = 0; k < MPL; ++k) e[k] = ok[k] ? term1(dv, p, k) : 0.0;
      });
    } else if (j == 4 || j == 5) {
      with_div(fabs(p[4]), p[5], [&](const auto& dv) {
#pragma unroll
        for (int k = 0; k < MPL; ++k) e[k] = ok[k] ? term2(dv, p, k) : 0.0;
      });
    }
#pragma unroll
    for (int k = 0; k < MPL; ++k) {
      const double e1 = (j == 0 || j == 1) ? e[k] : c.e1[k];
      const double e2 = (j == 4 || j == 5) ? e[k] : c.e2[k];
      f[k] = ok[k] ? y[k] - combine(p, e1, e2) : 0.0;
    }
  }
};

// numpy.delete on the "kept" index list represented as a bit mask over original positions
template <int P>
struct KeptSet {
  uint64_t w[P];
  int len;
  __device__ void init(int L) {
#pragma unroll
    for (int j = 0; j < P; ++j) {
      const int lo = 64 * j;
      w[j] = (L >= lo + 64) ? ~0ull : (L > lo ? ((1ull << (L - lo)) - 1ull) : 0ull);
    }
    len = L;
  }
  // remove the element at (possibly negative) position pos of the compacted list;
  // false = IndexError
  __device__ bool del(int pos) {
    if (pos < -len || pos >= len) return false;
    if (pos < 0) pos += len;
    int acc = 0;
    bool done = false;
#pragma unroll
    for (int j = 0; j < P; ++j) {
      const int cnt = __popcll(w[j]);
      if (!done && pos < acc + cnt) {
        uint64_t x = w[j];
        for (int r = pos - acc; r > 0; --r) x &= x - 1;  // drop the r lowest set bits
        w[j] &= ~(x & (~x + 1));                        // clear the next set bit
        done = true;
      }
      acc += cnt;
    }
    --len;
    return true;
  }
};

// fitDoubleGaussianT2 (:1162-1170) and the peak removal of fitDoubleGaussian (:1305-1354)
// for candidate c: y/ok = the rotated integer profile (also in ys, LDS); the kept points'
// positions are compacted into cx[0..m1) (LDS).  Returns m1, or -1 on the reference's
// IndexError (then s10 = s11 = 1e6 are written and the status bit is set).
template <int P>
__device__ __forceinline__ int gdg_peel(const BatesArgs& a, int64_t c, double* ys, double* cx,
                                        double (&y)[P], bool (&ok)[P]) {
  const int lane = lane_id();
  const int L = a.lp;
  const int cut = L / 2;
#pragma unroll
  for (int k = 0; k < P; ++k) {
    const int i = lane + 64 * k;
    ok[k] = i < L;
    y[k] = ok[k] ? prof_at(a, c * L + (ok[k] ? (i + cut) % L : 0)) : -1.0;
    if (ok[k]) ys[i] = y[k];
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
  // argmax (first maximum; the profile values are >= 0)
  double bv = -1.0;
  int bi = 1 << 30;
#pragma unroll
  for (int k = 0; k < P; ++k)
    if (ok[k] && y[k] > bv) {
      bv = y[k];
      bi = lane + 64 * k;
    }
#pragma unroll
  for (int s = 1; s < 64; s <<= 1) {
    const double ov = __shfl_xor(bv, s);
    const int oi = __shfl_xor(bi, s);
    if (ov > bv || (ov == bv && oi < bi)) {
      bv = ov;
      bi = oi;
    }
  }
  const int pos = uni(bi);
  // ---- neighbour peeling (:1305-1354), simulated on the kept-index mask
  KeptSet<P> ks;
  ks.init(L);
  bool index_error = !ks.del(pos);
  {
    int tol = 0;
    const int lim = 5;
    int i = 1;
    while (!index_error && i < L) {
      if ((pos - i) > 0 && (pos + i) < L) {
        const bool A = ys[pos - i] >= ys[pos - i + 1];
        const bool B = ys[pos + i] >= ys[pos + i - 1];
        if (!A && !B) {
          index_error = !ks.del(pos - i) || !ks.del(pos - i);
        } else if (A || (B && (tol < lim))) {
          index_error = !ks.del(pos - i) || !ks.del(pos - i);
          ++tol;
        } else {
          break;
        }
      } else if ((pos - i) < 0) {
        if (pos + i >= L) {  // y[pos+i] out of range
          index_error = true;
          break;
        }
        if (ys[pos + i] < ys[pos + i - 1]) {
          index_error = !ks.del(pos - i + 1);
        } else if (tol < lim) {
          index_error = !ks.del(pos - i + 1);
          ++tol;
        } else {
          break;
        }
      } else if ((pos + i) > L) {
        if (ys[pos - i] < ys[pos - i + 1]) {
          index_error = !ks.del(pos - i + 1);
        } else if (tol < lim) {
          index_error = !ks.del(pos - i);
          ++tol;
        } else {
          break;
        }
      }
      ++i;
    }
  }
  if (index_error) {  // getGaussianFittings catches IndexError: s10 = s11 = 1e6 (:762-764)
    if (lane == 0) {
      a.out[c * 22 + 9] = 1000000.0;
      a.out[c * 22 + 10] = 1000000.0;
      atomicOr(&a.status[c], (uint32_t)(PFE_ST_DGF_INDEXERROR));
    }
    return -1;
  }
  // compaction through LDS: x of the kept points to rows 0..len-1
  {
    int rank_base = 0;
#pragma unroll
    for (int j = 0; j < P; ++j) {
      const uint64_t wj = ks.w[j];
      const int i = 64 * j + lane;
      if ((wj >> lane) & 1ull) {
        const int r = rank_base + __popcll(wj & ((1ull << lane) - 1ull));
        cx[r] = (double)i;
      }
      rank_base += __popcll(wj);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
  __builtin_amdgcn_wave_barrier();
  return ks.len;
}

// start point of a peel pass from the current data rows [0, nlen) (:1361-1367)
template <int P>
__device__ __forceinline__ void peel_start(const GaussAbsBgFn<P>& fn, int nlen, double (&p)[4]) {
  const int lane = lane_id();
  double bvd = -INFINITY;
  int bid = 1 << 30;
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < P; ++k) {
    const int r = lane + 64 * k;
    if (r < nlen) {
      s += fn.y[k];
      if (bid == (1 << 30) || fn.y[k] > bvd) {
        bvd = fn.y[k];
        bid = r;
      }
    }
  }
  const ArgMax am = wargmax(bvd, bid);
  const double mean = wsum(s) / (double)nlen;
  double q = 0.0;
#pragma unroll
  for (int k = 0; k < P; ++k)
    if (lane + 64 * k < nlen) q += (fn.y[k] - mean) * (fn.y[k] - mean);
  double xe = 0.0;
#pragma unroll
  for (int k = 0; k < P; ++k)
    if (am.i >> 6 == k) xe = bcast(fn.x[k], am.i & 63);
  p[0] = sqrt(wsum(q) / (double)nlen);
  p[1] = xe;
  p[2] = am.v;
  p[3] = mean;
}

// subtraction of a peel pass's fit from the rotated profile y (:1389-1399; the window is
// centred on p[2], the amplitude): new data rows into fn
template <int P>
__device__ __forceinline__ void peel_subtract(const double (&y)[P], const bool (&ok)[P],
                                              const double (&p)[4], GaussAbsBgFn<P>& fn) {
  const int lane = lane_id();
  const double nfwhm = fabs(FWHM_C * p[0]);
#pragma unroll
  for (int k = 0; k < P; ++k) {
    const int i = lane + 64 * k;
    const double xi = (double)i;
    const double yi = y[k];
    double ny = yi;
    if (ok[k]) {
      const double ev = g_absbg(xi, p);
      if (ev <= yi)
        ny = yi - ev + p[3];
      else if ((ev > yi) && (xi > (p[2] - (1.5 * nfwhm) / 2.0)) && (xi < (p[2] + (1.5 * nfwhm) / 2.0)))
        ny = p[3];
    }
    fn.x[k] = xi;
    fn.y[k] = ok[k] ? ny : 0.0;
    fn.ok[k] = ok[k];
  }
}

template <int P>
__global__ __launch_bounds__(BLOCK) void k_gdg(BatesArgs a) {
  __shared__ double ys_all[BLOCK / 64][64 * P];
  __shared__ double cx_all[BLOCK / 64][64 * P];
  const int64_t c = wave_candidate();
  if (c >= a.n) return;
  if (a.status[c] & (GAUSS_SKIP | ST_DEFER_HIST)) return;
  const int lane = lane_id();
  const int L = a.lp;
  double* ys = ys_all[threadIdx.x >> 6];
  double* cx = cx_all[threadIdx.x >> 6];
  double y[P];
  bool ok[P];
  const int m1 = gdg_peel<P>(a, c, ys, cx, y, ok);
  if (m1 < 0) return;
  GaussAbsBgFn<P> fn;
  // ---- pass 1 on the compacted kept points, passes 2..8 on all L points
  double cy[P];
  bool cok[P];
#pragma unroll
  for (int k = 0; k < P; ++k) {
    const int r = lane + 64 * k;
    cok[k] = r < m1;
    fn.x[k] = cok[k] ? cx[r] : 0.0;
    cy[k] = cok[k] ? ys[(int)fn.x[k]] : 0.0;
    fn.y[k] = cy[k];
    fn.ok[k] = r < (m1 < 4 ? 4 : m1);  // zero padding to 4 points (:1373-1377)
  }
  double p[4], p1[4], p2[4];
  int nlen = m1;
  for (int pass = 1; pass <= 8; ++pass) {
    peel_start<P>(fn, nlen, p);
    lmdif<4, P>(fn, p, 200 * 5);
    peel_subtract<P>(y, ok, p, fn);
    nlen = L;
    if (pass == 7) {
#pragma unroll
      for (int j = 0; j < 4; ++j) p2[j] = p[j];
    } else if (pass == 8) {
#pragma unroll
      for (int j = 0; j < 4; ++j) p1[j] = p[j];
    }
  }
  if (lane == 0) {
    GaussWS* wp = a.ws + c;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      wp->dg[j] = p1[j];
      wp->dg[4 + j] = p2[j];
    }
  }
}

// Batched form of k_gdg: persistent waves take batches of BLM_FPW candidates from a queue;
// the 8 peel passes run as 8 batched lmdif calls (lm_batch.h) over the batch's fits.  Each
// fit's data rows (x, y) live in the wave's scratch between m-phase visits.
template <int P>
struct PeelLoader {
  const double* xs;  // [FPW][64P]
  const double* ys;
  const int* mpad;   // LDS [FPW]: rows [0, mpad) take part (zero padding included)
  __device__ __forceinline__ GaussAbsBgFn<P> operator()(int f) const {
    GaussAbsBgFn<P> fn;
    const int lane = lane_id();
    const int mp = mpad[f];
    const double* X = xs + (size_t)f * 64 * P;
    const double* Y = ys + (size_t)f * 64 * P;
#pragma unroll
    for (int k = 0; k < P; ++k) {
      const int r = lane + 64 * k;
      fn.x[k] = X[r];
      fn.y[k] = Y[r];
      fn.ok[k] = r < mp;
    }
    return fn;
  }
};

__device__ __forceinline__ void scratch_sync() { __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup"); }

template <int P>
__device__ __forceinline__ void store_rows(double* X, double* Y, const GaussAbsBgFn<P>& fn) {
  const int lane = lane_id();
#pragma unroll
  for (int k = 0; k < P; ++k) {
    X[lane + 64 * k] = fn.x[k];
    Y[lane + 64 * k] = fn.y[k];
  }
}

template <int P>
__global__ __launch_bounds__(64) void k_gdgb(BatesArgs a) {
  constexpr int FPW = BLM_FPW;
  __shared__ BlmState<4, FPW> S;
  __shared__ double ys[64 * P];
  __shared__ double cx[64 * P];
  __shared__ int mpad[FPW];
  const int lane = lane_id();
  const int L = a.lp;
  double* xs = a.wscr + (size_t)blockIdx.x * gdg_wave_scratch_doubles(L);
  double* yv = xs + (size_t)FPW * 64 * P;
  const PeelLoader<P> load{xs, yv, mpad};
  const int fpw = a.fpw;
  const int64_t nb = (a.n + fpw - 1) / fpw;
  for (;;) {
    int b = 0;
    if (lane == 0) b = (int)atomicAdd(a.counters + CTR_GDG, 1u);
    b = __builtin_amdgcn_readfirstlane(b);
    if (b >= nb) break;
    const int64_t base = (int64_t)b * fpw;
    // candidates of this batch that reach the double-Gaussian fit
    const bool live = lane < fpw && base + lane < a.n &&
                      !(a.status[base + (lane < fpw ? lane : 0)] & (GAUSS_SKIP | ST_DEFER_HIST));
    uint64_t fits = __ballot(live);
    // prologue: peak removal, pass-1 rows and start points
    for (uint64_t m = fits; m; m &= m - 1) {
      const int f = __builtin_ctzll(m);
      const int64_t c = base + f;
      double y[P];
      bool ok[P];
      const int m1 = gdg_peel<P>(a, c, ys, cx, y, ok);
      if (m1 < 0) {
        fits &= ~(1ull << f);
        continue;
      }
      GaussAbsBgFn<P> fn;
#pragma unroll
      for (int k = 0; k < P; ++k) {
        const int r = lane + 64 * k;
        const bool cok = r < m1;
        fn.x[k] = cok ? cx[r] : 0.0;
        fn.y[k] = cok ? ys[(int)fn.x[k]] : 0.0;
        fn.ok[k] = r < (m1 < 4 ? 4 : m1);  // zero padding to 4 points (:1373-1377)
      }
      store_rows<P>(xs + (size_t)f * 64 * P, yv + (size_t)f * 64 * P, fn);
      double p[4];
      peel_start<P>(fn, m1, p);
      if (lane == 0) {
        mpad[f] = m1 < 4 ? 4 : m1;
#pragma unroll
        for (int j = 0; j < 4; ++j) S.x[j][f] = p[j];
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
      __builtin_amdgcn_wave_barrier();
    }
    if (fits == 0) continue;
    scratch_sync();
    for (int pass = 1; pass <= 8; ++pass) {
      blm_run<4, P, FPW>(load, S, fits, 200 * 5);
      for (uint64_t m = fits; m; m &= m - 1) {
        const int f = __builtin_ctzll(m);
        const int64_t c = base + f;
        double p[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) p[j] = S.x[j][f];
        if (pass >= 7 && lane == 0) {
          GaussWS* wp = a.ws + c;
#pragma unroll
          for (int j = 0; j < 4; ++j) wp->dg[(pass == 8 ? 0 : 4) + j] = p[j];
        }
        if (pass == 8) continue;
        double y[P];
        bool ok[P];
        const int cut = L / 2;
#pragma unroll
        for (int k = 0; k < P; ++k) {
          const int i = lane + 64 * k;
          ok[k] = i < L;
          y[k] = ok[k] ? prof_at(a, c * L + (ok[k] ? (i + cut) % L : 0)) : -1.0;
        }
        GaussAbsBgFn<P> fn;
        peel_subtract<P>(y, ok, p, fn);
        store_rows<P>(xs + (size_t)f * 64 * P, yv + (size_t)f * 64 * P, fn);
        double q[4];
        peel_start<P>(fn, L, q);
        if (lane == 0) {
          mpad[f] = L;
#pragma unroll
          for (int j = 0; j < 4; ++j) S.x[j][f] = q[j];
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
      }
      scratch_sync();
    }
  }
}

// the combination rule (:1413-1428) and the s10/s11 selection (:747-768) after the final fit
template <int P>
__device__ __forceinline__ void gdg8_finish(const BatesArgs& a, int64_t c, const DoubleGaussFn<P>& dg,
                                            const bool (&ok)[P], const double (&q8)[8],
                                            const GaussWS& w) {
  const int lane = lane_id();
  const int L = a.lp;
  double p1[4], p2[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    p1[j] = w.dg[j];
    p2[j] = w.dg[4 + j];
  }
  const double f_fwhm1 = fabs(FWHM_C * q8[0]), f_fwhm2 = fabs(FWHM_C * q8[4]);
  double fchi = 0.0, cchi = 0.0;
  double ffit[P], cfit[P];
#pragma unroll
  for (int k = 0; k < P; ++k) {
    ffit[k] = dg.model(q8, k);
    const double x = dg.x[k];
    cfit[k] = g_absbg(x, p1) + g_absbg(x, p2) - p1[3] - p2[3] + (p1[3] + p2[3]) / 2.0;
    if (ok[k]) {
      if (ffit[k] >= 1.0) fchi += (dg.y[k] - ffit[k]) * (dg.y[k] - ffit[k]) / (double)L;
      if (cfit[k] >= 1.0) cchi += (dg.y[k] - cfit[k]) * (dg.y[k] - cfit[k]) / (double)L;
    }
  }
  fchi = wsum(fchi);
  cchi = wsum(cchi);
  const bool use_final = fchi <= cchi;
  const double fw1 = use_final ? f_fwhm1 : fabs(FWHM_C * p2[0]);  // combi_fwhm2
  const double fw2 = use_final ? f_fwhm2 : fabs(FWHM_C * p1[0]);                   // combi_fwhm1
  const double dchi = use_final ? fchi : cchi;
  // gf_dgf_std = std(dgf_fit - (gf_fit + minbg - std))  (:755-756)
  const double t1p[4] = {w.t1[0], w.t1[1], w.t1[2], w.t1[3]};
  double dd[P];
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < P; ++k) {
    const double x = dg.x[k];
    const double tt = (x - t1p[1]) / fabs(t1p[0]);
    const double gf = fabs(t1p[2]) * exp_neg_half_sq(tt) + t1p[3];
    dd[k] = (use_final ? ffit[k] : cfit[k]) - (gf + w.minbg - w.pstd);
    if (ok[k]) s += dd[k];
  }
  const double mu = wsum(s) / (double)L;
  double q = 0.0;
#pragma unroll
  for (int k = 0; k < P; ++k)
    if (ok[k]) q += (dd[k] - mu) * (dd[k] - mu);
  const double gstd = fabs(sqrt(wsum(q) / (double)L));
  if (lane == 0) {
    double* o = a.out + c * 22;
    o[9] = (gstd < 3.0) ? o[7] : py_min(fw1, fw2);  // s10 (:758-761)
    o[10] = dchi;                                   // s11
  }
}

// final 8-parameter fit (:1411, :1432-1483), the combination rule (:1413-1428) and the
// s10/s11 selection of getGaussianFittings (:747-768)
template <int P>
__global__ __launch_bounds__(BLOCK) void k_gdg8(BatesArgs a) {
  const int64_t c = wave_candidate();
  if (c >= a.n) return;
  if (a.status[c] & (GAUSS_SKIP | ST_DEFER_HIST | PFE_ST_DGF_INDEXERROR)) return;
  const int lane = lane_id();
  const int L = a.lp;
  const int cut = L / 2;
  const GaussWS w = a.ws[c];
  bool ok[P];
  DoubleGaussFn<P> dg;
#pragma unroll
  for (int k = 0; k < P; ++k) {
    const int i = lane + 64 * k;
    ok[k] = i < L;
    dg.x[k] = (double)i;
    dg.y[k] = ok[k] ? prof_at(a, c * L + (i + cut) % L) : 0.0;
    dg.ok[k] = ok[k];
  }
  double p1[4], p2[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    p1[j] = w.dg[j];
    p2[j] = w.dg[4 + j];
  }
  double q8[8] = {p1[0], p1[1], p1[2], p1[3], p2[0], p2[1], p2[2], p2[3]};
  lmdif<8, P>(dg, q8, 200 * 9);
  gdg8_finish<P>(a, c, dg, ok, q8, w);
}

// Batched form of k_gdg8: one wave owns FPW candidates and runs their 8-parameter fits
// through the batched lmdif (lm_batch.h); bit-identical to k_gdg8.
template <int P>
struct Gdg8Loader {
  const uint8_t* prof;
  const double* fprof;
  int64_t base;
  int L, cut;
  __device__ __forceinline__ DoubleGaussFn<P> operator()(int f) const {
    DoubleGaussFn<P> dg;
    const int lane = lane_id();
    const int64_t row = (base + f) * L;
#pragma unroll
    for (int k = 0; k < P; ++k) {
      const int i = lane + 64 * k;
      const bool ok = i < L;
      const int64_t idx = row + (ok ? (i + cut) % L : 0);
      dg.x[k] = (double)i;
      dg.y[k] = ok ? (fprof ? fprof[idx] : (double)prof[idx]) : 0.0;
      dg.ok[k] = ok;
    }
    return dg;
  }
};

template <int P, int FPW>
__global__ __launch_bounds__(64) void k_gdg8b(BatesArgs a) {
  __shared__ BlmState<8, FPW> S;
  const int64_t base = (int64_t)blockIdx.x * a.fpw;
  const int lane = lane_id();
  bool part = false;
  if (lane < a.fpw) {
    const int64_t c = base + lane;
    if (c < a.n && !(a.status[c] & (GAUSS_SKIP | ST_DEFER_HIST | PFE_ST_DGF_INDEXERROR))) {
      part = true;
      const GaussWS* w = a.ws + c;
#pragma unroll
      for (int j = 0; j < 8; ++j) S.x[j][lane] = w->dg[j];
    }
  }
  const uint64_t fits = __ballot(part);
  if (fits == 0) return;
  const int L = a.lp;
  const Gdg8Loader<P> load{a.prof, a.fprof, base, L, L / 2};
  blm_run<8, P, FPW>(load, S, fits, 200 * 9);
  for (uint64_t m = fits; m; m &= m - 1) {
    const int f = __builtin_ctzll(m);
    const int64_t c = base + f;
    const DoubleGaussFn<P> dg = load(f);
    bool ok[P];
#pragma unroll
    for (int k = 0; k < P; ++k) ok[k] = dg.ok[k];
    double q8[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) q8[j] = S.x[j][f];
    const GaussWS w = a.ws[c];
    gdg8_finish<P>(a, c, dg, ok, q8, w);
  }
}

// ---------------------------------------------------------------------------------------
// Pooled group-LM forms (lm_group.h) of the three fit kernels, for profiles of <= 256 bins:
// persistent waves keep GLM_FPW fit slots busy from a work queue of candidates; the
// m-parallel half of lmdif runs in groups of G lanes (16 up to 128 bins: 4 fits at a time;
// 32 above: 2 fits at a time, glm_group_lanes), the serial half one fit per lane.  Data rows
// of the fits in group layout: row r -> group-lane r % G, slot r / G.
// ---------------------------------------------------------------------------------------
// ---- s8, s9 -----------------------------------------------------------------------------
template <int P, int FPW, int G>
struct Gt1Prob {
  static constexpr int MG = 64 * P / G;
  BatesArgs a;
  SlotTab<FPW>& T;
  int nslots;
  __device__ __forceinline__ bool refill(int f, BlmState<4, FPW>& S) {
    const int lane = lane_id();
    const int64_t c0 = T.cand[f];
    if (c0 >= 0) {  // s8, s9 and the T1 parameters of the fit that ended
      GaussBgFn<P> fn;
      gt1_setup<P>(a, c0, a.ws[c0], fn);
      const double p[4] = {S.x[0][f], S.x[1][f], S.x[2][f], S.x[3][f]};
      gt1_finish<P>(a, c0, fn, p);
    }
    if (f < nslots) {
      for (;;) {
        const int64_t c = queue_next(a.counters + CTR_GT1G);
        if (c >= a.n) break;
        if (a.status[c] & (GAUSS_SKIP | ST_DEFER_HIST)) continue;
        GaussBgFn<P> fn;
        gt1_setup<P>(a, c, a.ws[c], fn);
        double p[4];
        gt1_start<P>(fn, a.lp, p);
        if (lane == 0) {
          T.cand[f] = c;
#pragma unroll
          for (int j = 0; j < 4; ++j) S.x[j][f] = p[j];
        }
        blm_sync();
        return true;
      }
    }
    if (lane == 0) T.cand[f] = -1;
    blm_sync();
    return false;
  }
  __device__ __forceinline__ GaussBgFn<MG> load(int f) const {  // gt1_setup, group layout
    GaussBgFn<MG> fn;
    const int64_t c = T.cand[f];
    const double minbg = a.ws[c].minbg, pstd = a.ws[c].pstd;
    const int lp = a.lp, cut = lp / 2, gl = glane<G>();
#pragma unroll
    for (int k = 0; k < MG; ++k) {
      const int i = gl + G * k;
      const bool ok = i < lp;
      fn.ok[k] = ok;
      fn.x[k] = (double)i;
      double y = 0.0;
      if (ok) {
        const double pv = prof_at(a, c * lp + (i + cut) % lp);
        if (minbg > 0.0) {
          y = pv - minbg + pstd;
          if (y < 0.0) y = 0.0;
        } else {
          y = pv;
        }
      }
      fn.y[k] = y;
    }
    return fn;
  }
  __device__ __forceinline__ int maxfev(int) const { return 200 * 5; }
};

template <int P>
#ifndef PFE_GT1G_WPE
#define PFE_GT1G_WPE 2
#endif
#ifndef PFE_GDGG_WPE
#define PFE_GDGG_WPE 2
#endif
__global__ __launch_bounds__(64, PFE_GT1G_WPE) void k_gt1g(BatesArgs a) {
  constexpr int FPW = P <= 2 ? GLM4_FPW : GLM_FPW;  // LDS: 256-bin peel rows keep 32
  constexpr int G = glm_group_lanes(64 * P);
  __shared__ BlmState<4, FPW> S;
  __shared__ SlotTab<FPW> T;
  if (lane_id() < FPW) T.cand[lane_id()] = -1;
  blm_sync();
  Gt1Prob<P, FPW, G> prob{a, T, a.gslots * FPW / GLM_FPW};
  glm_engine<4, 64 * P / G, FPW, G>(prob, S, T.ph, T.list, a.hand[HAND_GAUSS], HAND_K_GAUSS);
}

// ---- s10, s11: the 8 peel passes ----------------------------------------------------------
template <int P, int FPW, int G>
struct PeelProb {
  static constexpr int MG = 64 * P / G;
  BatesArgs a;
  SlotTab<FPW>& T;
  double* xs;  // wave scratch: x rows of the slots, [FPW][64P]
  double* yv;  // y rows
  double* ys;  // LDS [64P] (gdg_peel)
  double* cx;  // LDS [64P]
  int nslots;
  __device__ __forceinline__ bool refill(int f, BlmState<4, FPW>& S) {
    const int lane = lane_id();
    const int L = a.lp;
    double* X = xs + (size_t)f * 64 * P;
    double* Y = yv + (size_t)f * 64 * P;
    const int64_t c0 = T.cand[f];
    if (c0 >= 0) {
      const int ps = T.pass[f];
      double p[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) p[j] = S.x[j][f];
      if (ps >= 7 && lane == 0) {  // store_p2 (pass 7), store_p1 (pass 8) (:1402-1408)
        GaussWS* wp = a.ws + c0;
#pragma unroll
        for (int j = 0; j < 4; ++j) wp->dg[(ps == 8 ? 0 : 4) + j] = p[j];
      }
      if (ps < 8) {  // subtract this pass's fit, start the next one on all L points
        const int cut = L / 2;
        double y[P];
        bool ok[P];
#pragma unroll
        for (int k = 0; k < P; ++k) {
          const int i = lane + 64 * k;
          ok[k] = i < L;
          y[k] = ok[k] ? prof_at(a, c0 * L + (ok[k] ? (i + cut) % L : 0)) : -1.0;
        }
        GaussAbsBgFn<P> fn;
        peel_subtract<P>(y, ok, p, fn);
        store_rows<P>(X, Y, fn);
        double q[4];
        peel_start<P>(fn, L, q);
        if (lane == 0) {
          T.mpad[f] = L;
          T.pass[f] = ps + 1;
#pragma unroll
          for (int j = 0; j < 4; ++j) S.x[j][f] = q[j];
        }
        scratch_sync();
        blm_sync();
        return true;
      }
    }
    if (f < nslots) {
      for (;;) {
        const int64_t c = queue_next(a.counters + CTR_GDGG);
        if (c >= a.n) break;
        if (a.status[c] & (GAUSS_SKIP | ST_DEFER_HIST)) continue;
        double y[P];
        bool ok[P];
        const int m1 = gdg_peel<P>(a, c, ys, cx, y, ok);
        if (m1 < 0) continue;
        GaussAbsBgFn<P> fn;
#pragma unroll
        for (int k = 0; k < P; ++k) {
          const int r = lane + 64 * k;
          const bool cok = r < m1;
          fn.x[k] = cok ? cx[r] : 0.0;
          fn.y[k] = cok ? ys[(int)fn.x[k]] : 0.0;
          fn.ok[k] = r < (m1 < 4 ? 4 : m1);  // zero padding to 4 points (:1373-1377)
        }
        store_rows<P>(X, Y, fn);
        double p[4];
        peel_start<P>(fn, m1, p);
        if (lane == 0) {
          T.mpad[f] = m1 < 4 ? 4 : m1;
          T.cand[f] = c;
          T.pass[f] = 1;
#pragma unroll
          for (int j = 0; j < 4; ++j) S.x[j][f] = p[j];
        }
        scratch_sync();
        blm_sync();
        return true;
      }
    }
    if (lane == 0) T.cand[f] = -1;
    blm_sync();
    return false;
  }
  __device__ __forceinline__ GaussAbsBgFn<MG> load(int f) const {
    GaussAbsBgFn<MG> fn;
    const int gl = glane<G>();
    const int mp = T.mpad[f];
    const double* X = xs + (size_t)f * 64 * P;
    const double* Y = yv + (size_t)f * 64 * P;
#pragma unroll
    for (int k = 0; k < MG; ++k) {
      const int r = gl + G * k;
      fn.x[k] = X[r];
      fn.y[k] = Y[r];
      fn.ok[k] = r < mp;
    }
    return fn;
  }
  __device__ __forceinline__ int maxfev(int) const { return 200 * 5; }
};

template <int P>
__global__ __launch_bounds__(64, PFE_GDGG_WPE) void k_gdgg(BatesArgs a) {
  constexpr int FPW = P <= 2 ? GLM4_FPW : GLM_FPW;  // LDS: 256-bin peel rows keep 32
  __shared__ BlmState<4, FPW> S;
  __shared__ SlotTab<FPW> T;
  __shared__ double ys[64 * P];
  __shared__ double cx[64 * P];
  if (lane_id() < FPW) T.cand[lane_id()] = -1;
  blm_sync();
  double* xs = a.wscr + (size_t)blockIdx.x * gdg_wave_scratch_doubles(a.lp);
  double* yv = xs + (size_t)FPW * 64 * P;
  constexpr int G = glm_group_lanes(64 * P);
  PeelProb<P, FPW, G> prob{a, T, xs, yv, ys, cx, a.gslots * FPW / GLM_FPW};
  glm_engine<4, 64 * P / G, FPW, G>(prob, S, T.ph, T.list, a.hand[HAND_GAUSS], HAND_K_GAUSS);
}

// ---- s10, s11: the final 8-parameter fit ----------------------------------------------
// G lanes per group: 16 keeps 4P rows per lane (8 at 128 bins: the 8 x 8 Jacobian block,
// residuals and both exp caches), 32 halves that.
template <int P, int FPW, int G>
struct Gdg8Prob {
  static constexpr int MG = 64 * P / G;
  BatesArgs a;
  SlotTab<FPW>& T;
  int nslots;
  __device__ __forceinline__ bool refill(int f, BlmState<8, FPW>& S) {
    const int lane = lane_id();
    const int L = a.lp;
    const int64_t c0 = T.cand[f];
    if (c0 >= 0) {
      const DoubleGaussFn<P> dg = Gdg8Loader<P>{a.prof, a.fprof, c0, L, L / 2}(0);
      bool ok[P];
#pragma unroll
      for (int k = 0; k < P; ++k) ok[k] = dg.ok[k];
      double q8[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) q8[j] = S.x[j][f];
      const GaussWS w = a.ws[c0];
      gdg8_finish<P>(a, c0, dg, ok, q8, w);
    }
    if (f < nslots) {
      for (;;) {
        const int64_t c = queue_next(a.counters + CTR_GDG8G);
        if (c >= a.n) break;
        if (a.status[c] & (GAUSS_SKIP | ST_DEFER_HIST | PFE_ST_DGF_INDEXERROR)) continue;
        if (lane < 8) S.x[lane][f] = a.ws[c].dg[lane];
        if (lane == 0) T.cand[f] = c;
        blm_sync();
        return true;
      }
    }
    if (lane == 0) T.cand[f] = -1;
    blm_sync();
    return false;
  }
  __device__ __forceinline__ DoubleGaussFn<MG> load(int f) const {
    DoubleGaussFn<MG> dg;
    const int L = a.lp, cut = L / 2, gl = glane<G>();
    const int64_t row = T.cand[f] * L;
#pragma unroll
    for (int k = 0; k < MG; ++k) {
      const int i = gl + G * k;
      const bool ok = i < L;
      dg.x[k] = (double)i;
      dg.y[k] = ok ? prof_at(a, row + (i + cut) % L) : 0.0;
      dg.ok[k] = ok;
    }
    return dg;
  }
  __device__ __forceinline__ int maxfev(int) const { return 200 * 9; }
};

template <int P>
__global__ __launch_bounds__(64, PFE_GDG8_WPE) void k_gdg8g(BatesArgs a) {
  constexpr int FPW = GDG8_FPW;
  // 16 lanes (8 rows each) at 128 bins: 32 lanes measured 7 % slower there
  // (profiles/r02_gdg8_g32_ab.txt); 32 lanes (8 rows each) at 256 bins
  constexpr int G = glm_group_lanes(64 * P);
  __shared__ BlmState<8, FPW> S;
  __shared__ SlotTab<FPW> T;
  if (lane_id() < FPW) T.cand[lane_id()] = -1;
  blm_sync();
  Gdg8Prob<P, FPW, G> prob{a, T, a.gslots * GDG8_FPW / GLM_FPW};
  glm_engine<8, 64 * P / G, FPW, G>(prob, S, T.ph, T.list, a.hand[HAND_GAUSS], HAND_K_GAUSS);
}

static inline dim3 gw(int64_t n) { return grid_for_candidates(n); }

// the chain's launch stages (one translation unit each)
hipError_t launch_gauss_hist(const BatesArgs& a, hipStream_t st);
hipError_t launch_gauss_peel(const BatesArgs& a, hipStream_t st);
hipError_t launch_gauss_dg8(const BatesArgs& a, hipStream_t st);

}  // namespace pfe
