// bates_sine_dm_sub.hip — scores 1-4 (sinusoid fits) and 12-19 (candidate parameters and
// DM-curve fit) on gfx950 (scores 20-22: subband.hip).
//
// Reference (PulsarFeatureExtractor/src/):
//   s1-s4   ProfileOperations.getSinusoidFittings :190-376, fitSine :380-491,
//           fitSineSqr :495-587;                         PHCXFile.py:454-459
//   s12-s15 PHCXOperations.getCandidateParameters :81-112; filterScore
//           CandidateFileInterface.py:84-149;              PHCXFile.py:569-574
//   s16-s19 PHCXOperations.getDMFittings :121-233;       PHCXFile.py:613-618
#include "bates_common.h"
#include "lm_batch.h"
#include "lm_group.h"
#include "np_sum.h"

namespace pfe {

#pragma clang fp contract(off)

// ======================================================================================
// scores 1-4
// ======================================================================================
// sin(c * x_k + phi) over a lane's rows x_k = x_0 + STRIDE k (STRIDE a power of two).
// The residual models evaluate these at every function evaluation of the sine fits, and a
// library sin is ~80-150 VALU instructions (its large-argument branch is if-converted).
// Rows are walked by angle addition instead: one sincos at the anchor row (the reference's
// own argument fl(fl(c x_0) + phi)), one of the exact step STRIDE * c, then per row
//   s' = s C + c S,  c' = c C - s S                       (4 fp64 operations)
// re-anchored every R rows.  Each rotation adds ~1 ulp, so a row's value differs from the
// library sin of the reference's rounded argument by a few ulp of 1 -- the same order as
// that argument's own rounding (ulp(c x_k)) once |c x_k| > 4, and the class of residual
// perturbation the golden envelopes sample (tests/golden_util.py).  -DPFE_SIN_DIRECT builds
// the per-row library sin for A/B.
template <int M, int STRIDE, int R = 8>
__device__ __forceinline__ void sin_rows(double c, double phi, const double (&x)[M],
                                         double (&s)[M]) {
#ifdef PFE_SIN_DIRECT
#pragma unroll
  for (int k = 0; k < M; ++k) s[k] = sin(c * x[k] + phi);
#else
  static_assert((STRIDE & (STRIDE - 1)) == 0, "an exact step needs a power-of-two stride");
  double sd, cd;
  sincos(c * (double)STRIDE, &sd, &cd);
  double sk = 0.0, ck = 1.0;
#pragma unroll
  for (int k = 0; k < M; ++k) {
    if (k % R == 0) {
      sincos(c * x[k] + phi, &sk, &ck);
    } else {
      const double ns = fma(sk, cd, ck * sd);
      const double nc = fma(ck, cd, -(sk * sd));
      sk = ns;
      ck = nc;
    }
    s[k] = sk;
  }
#endif
}

template <int MPL, bool SQR>
struct SineFn {
  double x[MPL], y[MPL];
  bool ok[MPL];
  double amp, bg;
  __device__ __forceinline__ void operator()(const double (&p)[2], double (&f)[MPL]) const {
    double sv[MPL];
    sin_rows<MPL, 64>(TWO_PI * p[0], p[1], x, sv);
#pragma unroll
    for (int k = 0; k < MPL; ++k) {
      if (ok[k]) {
        const double s = sv[k];
        if constexpr (!SQR)
          f[k] = y[k] - (fabs(amp) * s + fabs(bg));               // :418
        else
          f[k] = (y[k] - (fabs(amp) * (s * s))) + fabs(bg);      // :522 (sign bug kept)
      } else {
        f[k] = 0.0;
      }
    }
  }
  __device__ __forceinline__ double model(const double (&p)[2], int k) const {
    const double s = sin(TWO_PI * p[0] * x[k] + p[1]);
    if constexpr (!SQR) return fabs(amp) * s + fabs(bg);          // :425
    return fabs(amp) * (s * s) + fabs(bg);                        // :529
  }
};

// block of 5-zero peak counting (:294-334) on the clipped profile: the zero counter is
// never reset by a non-zero bin, so a block closes at every 5th zero
template <int MPL>
__device__ __forceinline__ int count_peak_blocks(const uint64_t (&nz)[MPL], int len) {
  int blocks = 0, zeros = 0;
  bool cur = false;
#pragma unroll
  for (int w = 0; w < MPL; ++w) {
    const uint64_t word = nz[w];
    const int n = min(64, len - 64 * w);
    for (int b = 0; b < n; ++b) {
      if ((word >> b) & 1ull) {
        cur = true;
      } else if (zeros < 4) {
        ++zeros;
      } else {
        blocks += cur;
        cur = false;
        zeros = 0;
      }
    }
  }
  return blocks + cur;
}

// start point of fitSine (:398-438) / fitSineSqr (:535-541)
template <bool SQR>
__device__ __forceinline__ void sine_start(int maxima, int lp, double amp, double y0, double (&p)[2]) {
  double f0, phi0;
  if constexpr (!SQR) {
    f0 = (double)maxima / ((double)lp - 1.0);                     // :398
    if (y0 == amp)
      phi0 = 0.0;
    else if (y0 < amp)
      phi0 = (f0 != 0.0) ? -1.0 / (4.0 * f0) : -1.0 / (4.0 * 0.00000000001);
    else
      phi0 = (f0 != 0.0) ? 1.0 / (4.0 * f0) : 1.0 / (4.0 * 0.00000000001);
  } else {
    f0 = (double)maxima / ((double)lp - 1.0) / 2.0;               // :535
    if (y0 == 0.0)
      phi0 = 0.0;
    else
      phi0 = (f0 != 0.0) ? -1.0 / (4.0 * f0) : -1.0 / (4.0 * 0.00000000001);
  }
  p[0] = f0;
  p[1] = phi0;
}

template <int MPL, bool SQR>
__device__ __forceinline__ SineFn<MPL, SQR> sine_fn(const double (&yi)[MPL], int lp, int lane,
                                                    double amp) {
  SineFn<MPL, SQR> fn;
#pragma unroll
  for (int k = 0; k < MPL; ++k) {
    const int i = lane + 64 * k;
    fn.ok[k] = i < lp;
    fn.x[k] = (double)i;
    fn.y[k] = yi[k];
  }
  fn.amp = amp;
  fn.bg = amp;
  return fn;
}

// mean squared residual of the fitted model (:453-458)
template <int MPL, bool SQR>
__device__ __forceinline__ double sine_chi(const SineFn<MPL, SQR>& fn, const double (&p)[2], int lp) {
  double s = 0.0;
#pragma unroll
  for (int k = 0; k < MPL; ++k)
    if (fn.ok[k]) {
      const double d = fn.y[k] - fn.model(p, k);
      s += d * d;
    }
  return wsum(s) / (double)lp;
}

template <int MPL, bool SQR>
__device__ double sine_chisq(const double (&yi)[MPL], int lp, int lane, double amp, int maxima,
                             double y0) {
  const SineFn<MPL, SQR> fn = sine_fn<MPL, SQR>(yi, lp, lane, amp);
  double p[2];
  sine_start<SQR>(maxima, lp, amp, y0, p);
  lmdif<2, MPL>(fn, p, 200 * 3);
  return sine_chi<MPL, SQR>(fn, p, lp);
}

// everything of getSinusoidFittings before the fits: s4, the amplitude h = |max-min|/2, the
// peak count, y[0]; the profile as doubles in yv (wave layout).  fail: fitSine would raise.
struct SinePre {
  double h, s4, y0;
  int maxima;
  bool fail;
};
template <int MPL, bool F>
__device__ __forceinline__ SinePre sine_prologue(const BatesArgs& a, int64_t c, double* sg,
                                                 double (&yv)[MPL]) {
  const int lane = lane_id();
  const int lp = a.lp;
  SinePre r;
  r.fail = false;
  MeanStd ms;
  if constexpr (F) {
    const double* row = a.fprof + c * lp;
    double mx = -INFINITY, mn = INFINITY;
    bool nan = false;
#pragma unroll
    for (int k = 0; k < MPL; ++k) {
      const int i = lane + 64 * k;
      yv[k] = (i < lp) ? row[i] : 0.0;
      if (i < lp) {
        sg[i] = yv[k];
        nan |= !(yv[k] == yv[k]);
        mx = fmax(mx, yv[k]);
        mn = fmin(mn, yv[k]);
      }
    }
    mx = wmax(mx);
    mn = wmin(mn);
    if (__ballot(nan)) mx = mn = NAN;  // profile.max() / .min() propagate NaN
    r.h = fabs(mx - mn) / 2.0;
    lds_sync();
    // s4 = sum over the profile of (|max-min|/2 - p_i), a Python loop (:246-247)
    double t = 0.0;
    if (lane == 0)
      for (int i = 0; i < lp; ++i) t += r.h - sg[i];
    r.s4 = bcast(t, 0);
    ms.mean = np_pairwise<4>(sg, lp, lane) / (double)lp;
    lds_sync();
#pragma unroll
    for (int k = 0; k < MPL; ++k) {
      const int i = lane + 64 * k;
      if (i < lp) {
        const double d = yv[k] - ms.mean;
        sg[i] = d * d;
      }
    }
    lds_sync();
    ms.std = sqrt(np_pairwise<4>(sg, lp, lane) / (double)lp);
    lds_sync();
    r.y0 = row[0];
    if (!(r.y0 == r.y0)) {  // phi0 never assigned: fitSine raises (Sinusoid fitting exception)
      r.fail = true;
      r.maxima = 0;
      return r;
    }
  } else {
    int v[MPL];
    load_row_u8<MPL>(a.prof + c * lp, lp, lane, v);
    ms = int_mean_std<MPL>(v, lp, lane);
    int vmax = -1, vmin = 1 << 30;
#pragma unroll
    for (int k = 0; k < MPL; ++k)
      if (lane + 64 * k < lp) {
        vmax = max(vmax, v[k]);
        vmin = min(vmin, v[k]);
      }
    vmax = wmax_i(vmax);
    vmin = wmin_i(vmin);
    // s4 = sum((|max-min|/2) - p_i): every partial sum is exact, so = lp*h - sum(p)
    r.h = (double)abs(vmax - vmin) / 2.0;
    long long s1 = 0;
#pragma unroll
    for (int k = 0; k < MPL; ++k)
      if (lane + 64 * k < lp) s1 += v[k];
    s1 = wsum_ll(s1);
    r.s4 = (double)lp * r.h - (double)s1;
#pragma unroll
    for (int k = 0; k < MPL; ++k) yv[k] = (double)v[k];
    r.y0 = (double)__builtin_amdgcn_readfirstlane(v[0]);
  }
  // peaks of (p - mean) - std clipped at 0
  uint64_t nz[MPL];
#pragma unroll
  for (int k = 0; k < MPL; ++k) {
    const bool pos = (lane + 64 * k < lp) && ((yv[k] - ms.mean) - ms.std > 0.0);
    nz[k] = __ballot(pos);
  }
  r.maxima = count_peak_blocks<MPL>(nz, lp);
  return r;
}

// F = float profiles (the PFD path): numpy's pairwise mean / std, the sequential Python sum
// for s4, and the UnboundLocalError of fitSine when y[0] is NaN (:427-441)
template <int MPL, bool F>
__global__ __launch_bounds__(BLOCK) void k_sine(BatesArgs a) {
  __shared__ double stage_all[BLOCK / 64][F ? 64 * MPL : 1];
  const int64_t c = wave_candidate();
  if (c >= a.n) return;
  const int lane = lane_id();
  const int lp = a.lp;
  double yv[MPL];
  const SinePre pre = sine_prologue<MPL, F>(a, c, stage_all[threadIdx.x >> 6], yv);
  if (pre.fail) {
    if (lane == 0) atomicOr(&a.status[c], (uint32_t)(PFE_ST_SINE_FAIL));
    return;
  }
  const double c1 = sine_chisq<MPL, false>(yv, lp, lane, pre.h, pre.maxima, pre.y0);
  const double c2 = sine_chisq<MPL, true>(yv, lp, lane, pre.h, pre.maxima, pre.y0);
  if (lane == 0) {
    double* o = a.out + c * 22;
    o[0] = c1 / (double)pre.maxima;                               // :373 (inf/nan at 0)
    o[1] = c2 / (double)pre.maxima;                               // :374
    o[2] = (double)(pre.maxima > 0 ? pre.maxima - 1 : 0);         // :376 len(diff)
    o[3] = pre.s4;
  }
}

// pooled group-LM form (lm_group.h): a slot runs a candidate's sine fit, then its sine^2 fit
template <int MPL, int STRIDE>
struct SineAnyFn {  // SineFn<MPL, sqr> with the model chosen per slot (rows gl + STRIDE k)
  double x[MPL], y[MPL];
  bool ok[MPL];
  double amp, bg;
  bool sqr;
  __device__ __forceinline__ void operator()(const double (&p)[2], double (&f)[MPL]) const {
    double sv[MPL];
    sin_rows<MPL, STRIDE>(TWO_PI * p[0], p[1], x, sv);
#pragma unroll
    for (int k = 0; k < MPL; ++k) {
      if (ok[k]) {
        const double s = sv[k];
        f[k] = sqr ? (y[k] - (fabs(amp) * (s * s))) + fabs(bg)   // :522 (sign bug kept)
                   : y[k] - (fabs(amp) * s + fabs(bg));          // :418
      } else {
        f[k] = 0.0;
      }
    }
  }
};

template <int MPL, bool F, int FPW, int G>
struct SineProb {
  static constexpr int MG = 64 * MPL / G;
  BatesArgs a;
  SlotTab<FPW>& T;  // d0 = h, d1 = y0, mpad = maxima, pass = 0 (sine) / 1 (sine^2)
  double* sg;       // LDS stage (F)
  int nslots;
  __device__ __forceinline__ void profile(int64_t c, double (&yv)[MPL]) const {
    const int lane = lane_id();
#pragma unroll
    for (int k = 0; k < MPL; ++k) {
      const int i = lane + 64 * k;
      yv[k] = (i < a.lp) ? prof_at(a, c * a.lp + i) : 0.0;
    }
  }
  __device__ __forceinline__ bool refill(int f, BlmState<2, FPW>& S) {
    const int lane = lane_id();
    const int lp = a.lp;
    const int64_t c0 = T.cand[f];
    if (c0 >= 0) {
      const int stage = T.pass[f];
      const double h = T.d0[f];
      const int maxima = T.mpad[f];
      const double p[2] = {S.x[0][f], S.x[1][f]};
      double yv[MPL];
      profile(c0, yv);
      if (stage == 0) {
        const double c1 = sine_chi<MPL, false>(sine_fn<MPL, false>(yv, lp, lane, h), p, lp);
        double q[2];
        sine_start<true>(maxima, lp, h, T.d1[f], q);
        if (lane == 0) {
          a.out[c0 * 22 + 0] = c1 / (double)maxima;  // :373 (inf/nan at 0)
          T.pass[f] = 1;
          S.x[0][f] = q[0];
          S.x[1][f] = q[1];
        }
        blm_sync();
        return true;
      }
      const double c2 = sine_chi<MPL, true>(sine_fn<MPL, true>(yv, lp, lane, h), p, lp);
      if (lane == 0) a.out[c0 * 22 + 1] = c2 / (double)maxima;  // :374
    }
    if (f < nslots) {
      for (;;) {
        const int64_t c = queue_next(a.counters + CTR_SINEG);
        if (c >= a.n) break;
        double yv[MPL];
        const SinePre pre = sine_prologue<MPL, F>(a, c, sg, yv);
        if (pre.fail) {
          if (lane == 0) atomicOr(&a.status[c], (uint32_t)(PFE_ST_SINE_FAIL));
          continue;
        }
        double q[2];
        sine_start<false>(pre.maxima, lp, pre.h, pre.y0, q);
        if (lane == 0) {
          double* o = a.out + c * 22;
          o[2] = (double)(pre.maxima > 0 ? pre.maxima - 1 : 0);  // :376 len(diff)
          o[3] = pre.s4;
          T.cand[f] = c;
          T.pass[f] = 0;
          T.d0[f] = pre.h;
          T.d1[f] = pre.y0;
          T.mpad[f] = pre.maxima;
          S.x[0][f] = q[0];
          S.x[1][f] = q[1];
        }
        blm_sync();
        return true;
      }
    }
    if (lane == 0) T.cand[f] = -1;
    blm_sync();
    return false;
  }
  __device__ __forceinline__ SineAnyFn<MG, G> load(int f) const {
    SineAnyFn<MG, G> fn;
    const int64_t c = T.cand[f];
    const int lp = a.lp, gl = glane<G>();
#pragma unroll
    for (int k = 0; k < MG; ++k) {
      const int i = gl + G * k;
      fn.ok[k] = i < lp;
      fn.x[k] = (double)i;
      fn.y[k] = fn.ok[k] ? prof_at(a, c * lp + i) : 0.0;
    }
    fn.amp = T.d0[f];
    fn.bg = fn.amp;
    fn.sqr = T.pass[f] != 0;
    return fn;
  }
  __device__ __forceinline__ int maxfev(int) const { return 200 * 3; }
};

template <int MPL, bool F>
__global__ __launch_bounds__(64, 3) void k_sineg(BatesArgs a) {
  constexpr int FPW = GLM_FPW;
  __shared__ BlmState<2, FPW> S;
  __shared__ SlotTab<FPW> T;
  __shared__ double stage[F ? 64 * MPL : 1];
  if (lane_id() < FPW) T.cand[lane_id()] = -1;
  blm_sync();
  constexpr int G = glm_group_lanes(64 * MPL);
  SineProb<MPL, F, FPW, G> prob{a, T, stage, a.gslots};
  glm_engine<2, 64 * MPL / G, FPW, G>(prob, S, T.ph, T.list, a.hand[HAND_SINE], HAND_K_SINE);
}

// ======================================================================================
// scores 12-19
// ======================================================================================
constexpr double KDM = 8.3 * 1000000.0;   // 8.3*10**6 (PHCXOperations.py:187)
constexpr double DF = 400.0;
constexpr double F3 = 2593941624.0;       // pow(1374, 3), an exact integer

static_assert(F3 == 2593941624.0, "div_f3 is this divisor");
__device__ __forceinline__ double div_f3(double a) { return div_const<2593941624LL>(a); }

template <int MPL>
struct DMFn {
  static constexpr bool kCols = true;  // the amplitude column reuses sqrt((P - w)/w)
  struct Cache {
    double s[MPL];
  };
  double x[MPL], y[MPL];
  bool ok[MPL];
  double wint, dm, period;
  __device__ __forceinline__ double shape(const double (&p)[3], int k) const {
    const double t = div_f3(p[1] * KDM * fabs((dm + p[2]) - x[k]) * DF);   // :152
    const double weff = dm_sqrt(wint + t * t);
    return dm_sqrt((period - weff) / weff);
  }
  __device__ __forceinline__ double model(const double (&p)[3], int k) const {
    return p[0] * shape(p, k);                                         // :153
  }
  __device__ __forceinline__ void operator()(const double (&p)[3], double (&f)[MPL]) const {
#pragma unroll
    for (int k = 0; k < MPL; ++k) f[k] = ok[k] ? y[k] - model(p, k) : 0.0;
  }
  __device__ __forceinline__ void eval(const double (&p)[3], double (&f)[MPL], Cache& c) const {
#pragma unroll
    for (int k = 0; k < MPL; ++k) {
      c.s[k] = ok[k] ? shape(p, k) : 0.0;
      f[k] = ok[k] ? y[k] - p[0] * c.s[k] : 0.0;
    }
  }
  __device__ __forceinline__ void eval_col(const double (&p)[3], int j, double,
                                           double (&f)[MPL], const Cache& c) const {
#pragma unroll
    for (int k = 0; k < MPL; ++k) {
      const double sh = (j == 0) ? c.s[k] : (ok[k] ? shape(p, k) : 0.0);
      f[k] = ok[k] ? y[k] - p[0] * sh : 0.0;
    }
  }
};

__device__ __forceinline__ double filter_neg(double v) {
  // CandidateFileInterface.filterScore(13|14): isEqual(v, 0, 5e-6) == -1 -> 0.0
  return (fabs(v - 0.0) > 0.000005 && v < 0.0) ? 0.0 : v;
}

// the DM-curve fit data of candidate c (:160-209): residual functor, theoretical curve
// shape help[] and the start amplitude 255/max(help)
template <int MPL>
struct DMSetup {
  DMFn<MPL> fn;
  double help[MPL];
  double amp0;
};

// the residual functor alone (what an m-phase visit of the batched solver rebuilds)
// rows i = lb + STRIDE*k: the wave layout (lane, 64) or the group layout (glane, 16)
template <int MPL, int STRIDE = 64>
__device__ __forceinline__ void dm_functor(const BatesArgs& a, int64_t c, DMFn<MPL>& fn,
                                           int lb = lane_id()) {
  const double* sc = a.scal + c * PFE_NSCAL;
  const double period = sc[PFE_SCAL_PERIOD_MS], dm = sc[PFE_SCAL_DM],
               width = sc[PFE_SCAL_WIDTH], dm_start = sc[PFE_SCAL_DM_START],
               dm_end = sc[PFE_SCAL_DM_END], length_all = sc[PFE_SCAL_LENGTH_ALL];
  const int n = a.ndm;
  const double step = fabs(dm_start - dm_end) / length_all;          // :183
  fn.wint = (width * period) * (width * period);                     // :186
  fn.dm = dm;
  fn.period = period;
#pragma unroll
  for (int k = 0; k < MPL; ++k) {
    const int i = lb + STRIDE * k;
    fn.ok[k] = i < n;
    fn.y[k] = fn.ok[k] ? a.dmcurve[c * n + (fn.ok[k] ? i : 0)] : 0.0;
    fn.x[k] = dm_start + (double)(128 * i - 1) * step;               // :196 (x = 128k-1)
  }
}

template <int MPL>
__device__ __forceinline__ void dm_setup(const BatesArgs& a, int64_t c, DMSetup<MPL>& d) {
  dm_functor<MPL>(a, c, d.fn);
  const double wint = d.fn.wint, dm = d.fn.dm, period = d.fn.period;
  double hmax = -INFINITY;
#pragma unroll
  for (int k = 0; k < MPL; ++k) {
    const double t = KDM * fabs(dm - d.fn.x[k]) * DF / F3;
    const double weff = sqrt(wint + t * t);                          // :202
    d.help[k] = sqrt((period - weff) / weff);                        // :203
    if (d.fn.ok[k]) hmax = fmax(hmax, d.help[k]);
  }
  hmax = wmax(hmax);
  // Python max(): a leading NaN wins, later NaNs are skipped
  const double h0 = bcast(d.help[0], 0);
  if (h0 != h0) hmax = h0;
  d.amp0 = 255.0 / hmax;                                             // :206-209
}

template <int MPL>
__device__ __forceinline__ void dm_finish(const BatesArgs& a, int64_t c, const DMSetup<MPL>& d,
                                          const double (&p)[3]) {
  const int lane = lane_id();
  const double* sc = a.scal + c * PFE_NSCAL;
  const double period = sc[PFE_SCAL_PERIOD_MS], snr = sc[PFE_SCAL_SNR], dm = sc[PFE_SCAL_DM],
               width = sc[PFE_SCAL_WIDTH];
  const double wint = d.fn.wint;
  double chi = 0.0;
#pragma unroll
  for (int k = 0; k < MPL; ++k)
    if (d.fn.ok[k]) {
      const double fit = d.fn.model(p, k);
      if (fit >= 1.0) {
        const double dd = d.fn.y[k] - d.amp0 * d.help[k];            // theo (:206)
        chi += dd * dd;
      }
    }
  chi = wsum(chi) / (double)a.ndm;                                   // :222-229
  if (lane == 0) {
    double* o = a.out + c * 22;
    o[11] = period;                                                  // s12
    o[12] = filter_neg(snr);                                         // s13
    o[13] = filter_neg(dm);                                          // s14
    o[14] = width;                                                   // s15
    o[15] = snr / sqrt((period - sqrt(wint)) / sqrt(wint));          // s16 (:191)
    o[16] = fabs(1.0 - p[1]);                                        // s17
    // s18 = filterScore(18, shift) = |shift|; getDMFittings itself returns the signed shift
    o[17] = a.raw_dm ? p[2] : fabs(p[2]);
    o[18] = chi;                                                     // s19
  }
}

template <int MPL>
__global__ __launch_bounds__(BLOCK) void k_dmfit(BatesArgs a) {
  const int64_t c = wave_candidate();
  if (c >= a.n) return;
  DMSetup<MPL> d;
  dm_setup<MPL>(a, c, d);
  double p[3] = {d.amp0, 1.0, 0.0};
  lmdif<3, MPL>(d.fn, p, 200 * 4);
  dm_finish<MPL>(a, c, d, p);
}

// batched form: one wave owns BLM_FPW candidates' DM fits (lm_batch.h); bit-identical
template <int MPL>
struct DMLoader {
  BatesArgs a;
  int64_t base;
  __device__ __forceinline__ DMFn<MPL> operator()(int f) const {
    DMFn<MPL> fn;
    dm_functor<MPL>(a, base + f, fn);
    return fn;
  }
};

template <int MPL>
__global__ __launch_bounds__(64) void k_dmfitb(BatesArgs a) {
  constexpr int FPW = BLM_FPW;
  __shared__ BlmState<3, FPW> S;
  const int64_t base = (int64_t)blockIdx.x * a.fpw;
  const int lane = lane_id();
  const bool live = lane < a.fpw && base + lane < a.n;
  const uint64_t fits = __ballot(live);
  if (fits == 0) return;
  for (uint64_t m = fits; m; m &= m - 1) {
    const int f = __builtin_ctzll(m);
    DMSetup<MPL> d;
    dm_setup<MPL>(a, base + f, d);
    if (lane == 0) {
      S.x[0][f] = d.amp0;
      S.x[1][f] = 1.0;
      S.x[2][f] = 0.0;
    }
  }
  const DMLoader<MPL> load{a, base};
  blm_run<3, MPL, FPW>(load, S, fits, 200 * 4);
  for (uint64_t m = fits; m; m &= m - 1) {
    const int f = __builtin_ctzll(m);
    DMSetup<MPL> d;
    dm_setup<MPL>(a, base + f, d);
    const double p[3] = {S.x[0][f], S.x[1][f], S.x[2][f]};
    dm_finish<MPL>(a, base + f, d, p);
  }
}

// pooled group-LM form (lm_group.h): persistent waves keep GLM_FPW DM fits in flight
template <int MPL, int FPW>
struct DMProb {
  static constexpr int MG = 4 * MPL;  // rows per lane of a 16-lane group
  BatesArgs a;
  SlotTab<FPW>& T;
  int nslots;
  __device__ __forceinline__ bool refill(int f, BlmState<3, FPW>& S) {
    const int lane = lane_id();
    const int64_t c0 = T.cand[f];
    if (c0 >= 0) {
      DMSetup<MPL> d;
      dm_setup<MPL>(a, c0, d);
      const double p[3] = {S.x[0][f], S.x[1][f], S.x[2][f]};
      dm_finish<MPL>(a, c0, d, p);
    }
    if (f < nslots) {
      const int64_t c = queue_next(a.counters + CTR_DMG);
      if (c < a.n) {
        DMSetup<MPL> d;
        dm_setup<MPL>(a, c, d);
        if (lane == 0) {
          T.cand[f] = c;
          S.x[0][f] = d.amp0;
          S.x[1][f] = 1.0;
          S.x[2][f] = 0.0;
        }
        blm_sync();
        return true;
      }
    }
    if (lane == 0) T.cand[f] = -1;
    blm_sync();
    return false;
  }
  __device__ __forceinline__ DMFn<MG> load(int f) const {
    DMFn<MG> fn;
    dm_functor<MG, GLM_G>(a, T.cand[f], fn, glane());
    return fn;
  }
  __device__ __forceinline__ int maxfev(int) const { return 200 * 4; }
};

template <int MPL>
__global__ __launch_bounds__(64, 3) void k_dmfitg(BatesArgs a) {
  constexpr int FPW = GLM_FPW;
  __shared__ BlmState<3, FPW> S;
  __shared__ SlotTab<FPW> T;
  if (lane_id() < FPW) T.cand[lane_id()] = -1;
  blm_sync();
  DMProb<MPL, FPW> prob{a, T, a.gslots};
  glm_engine<3, 4 * MPL, FPW>(prob, S, T.ph, T.list, a.hand[HAND_DM], HAND_K_DM);
}

// ---- launchers -----------------------------------------------------------------------
static inline dim3 grid_waves(int64_t n) { return grid_for_candidates(n); }

// pooled group-LM kernels (lm_group.h) unless the handle selects another solver
static bool glm_on(const BatesArgs& a) { return a.solver == PFE_SOLVER_POOLED; }

template <bool F>
static void launch_sine_t(const BatesArgs& a, hipStream_t st) {
  if (glm_on(a) && a.lp <= GLM_MAX_LP) {
    if (a.lp <= 64)
      hipLaunchKernelGGL((k_sineg<1, F>), pool_grid(a, 3), dim3(64), 0, st, a);
    else if (a.lp <= 128)
      hipLaunchKernelGGL((k_sineg<2, F>), pool_grid(a, 3), dim3(64), 0, st, a);
    else
      hipLaunchKernelGGL((k_sineg<4, F>), pool_grid(a, 3), dim3(64), 0, st, a);
    return;
  }
  if (a.lp <= 64)
    hipLaunchKernelGGL((k_sine<1, F>), grid_waves(a.n), dim3(BLOCK), 0, st, a);
  else if (a.lp <= 128)
    hipLaunchKernelGGL((k_sine<2, F>), grid_waves(a.n), dim3(BLOCK), 0, st, a);
  else if (a.lp <= 256)
    hipLaunchKernelGGL((k_sine<4, F>), grid_waves(a.n), dim3(BLOCK), 0, st, a);
  else
    hipLaunchKernelGGL((k_sine<16, F>), grid_waves(a.n), dim3(BLOCK), 0, st, a);
}

hipError_t launch_sine(const BatesArgs& a, hipStream_t st) {
  if (a.fprof)
    launch_sine_t<true>(a, st);
  else
    launch_sine_t<false>(a, st);
  return hipGetLastError();
}

hipError_t launch_dmfit(const BatesArgs& a, hipStream_t st) {
  if (glm_on(a) && a.ndm <= 128) {
    if (a.ndm <= 64)
      hipLaunchKernelGGL(k_dmfitg<1>, pool_grid(a, 3), dim3(64), 0, st, a);
    else
      hipLaunchKernelGGL(k_dmfitg<2>, pool_grid(a, 3), dim3(64), 0, st, a);
    return hipGetLastError();
  }
  if (a.solver != PFE_SOLVER_WAVE) {  // batched lmdif (lm_batch.h)
    const dim3 g((unsigned)((a.n + a.fpw - 1) / a.fpw));
    if (a.ndm <= 64)
      hipLaunchKernelGGL(k_dmfitb<1>, g, dim3(64), 0, st, a);
    else if (a.ndm <= 128)
      hipLaunchKernelGGL(k_dmfitb<2>, g, dim3(64), 0, st, a);
    else if (a.ndm <= 256)
      hipLaunchKernelGGL(k_dmfitb<4>, g, dim3(64), 0, st, a);
    else
      hipLaunchKernelGGL(k_dmfitb<16>, g, dim3(64), 0, st, a);
    return hipGetLastError();
  }
  if (a.ndm <= 64)
    hipLaunchKernelGGL(k_dmfit<1>, grid_waves(a.n), dim3(BLOCK), 0, st, a);
  else if (a.ndm <= 128)
    hipLaunchKernelGGL(k_dmfit<2>, grid_waves(a.n), dim3(BLOCK), 0, st, a);
  else if (a.ndm <= 256)
    hipLaunchKernelGGL(k_dmfit<4>, grid_waves(a.n), dim3(BLOCK), 0, st, a);
  else
    hipLaunchKernelGGL(k_dmfit<16>, grid_waves(a.n), dim3(BLOCK), 0, st, a);
  return hipGetLastError();
}

}  // namespace pfe

PFE_LM_PROFILE_EXPORT(sine_dm_sub)
