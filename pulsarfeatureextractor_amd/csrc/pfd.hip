// pfd.hip — PRESTO-fold (PFD) preprocessing and PFD Lyon features on gfx950.
//
// One 64-lane workgroup per candidate does what a freshly loaded PFDFile does for the
// dmprof path (paths relative to PulsarFeatureExtractor/src/):
//   dedisperse at the best DM                   PFDFile.py:330-374  (integer-bin rotations)
//   getprofile + scale                          PFDFile.py:256-310  ((sumprof-min)/mean -> 0..255)
//   plot_chi2_vs_DM(dms[0], dms[-1], 100)       PFDFile.py:378-423  (rotations accumulate; float32)
//   computeProfileStatScores                    PFDFile.py:522-551  (float64 numpy/scipy stats)
//   computeDMCurveStatScores                    PFDFile.py:553-583  (float32 numpy/scipy stats)
// Every reduction is numpy's own: axis reductions over parts / sub-bands add sequentially,
// contiguous sums use numpy's pairwise summation (8 accumulators per block of <= 128, blocks
// split at n/2 rounded down to a multiple of 8), and the DM-curve statistics run in float32
// as numpy does on a float32 array.  The sub-band profiles of the candidate live in LDS.
#include <cmath>
#include <cstdlib>

#include "np_sum.h"
#include "pfd.h"
#include "wave.h"

namespace pfe {

#pragma clang fp contract(off)

__device__ __forceinline__ int pymod(long long v, int m) {
  long long r = v % m;
  if (r < 0) r += m;
  return (int)r;
}

__device__ __forceinline__ double delay_from_dm(double dm, double f) {  // PFDOperations.py:474-488
  return f > 0.0 ? dm / (0.000241 * f * f) : 0.0;
}

// numpy's pairwise sum of an LDS row with the leaf's loads issued before its adds when the
// row is a single leaf (np_leaf128: the same order of additions, so the same bits)
// NC (the four-wave kernel, rows of <= np_inl_max(3) = 968 values): every level inlined, no call -- a call
// in a kernel makes the backend assume the callee's register needs (212 VGPRs and 2 waves per
// SIMD for k_pfd_dmprof4 with the recursive call in it, 123 without)
template <bool NC = false>
__device__ __forceinline__ double np_sum_row(const double* a, int n, int lane) {
  if (n >= 8 && n <= 128) return np_leaf128(a, n, lane);
  if constexpr (NC)
    return np_pairwise_inl<3>(a, n, lane);
  else
    return np_pairwise<12>(a, n, lane);
}

// Python's builtin min (MAX = false) / max over an LDS row as a wave reduction: a[0] when
// a[0] is NaN, else the first element equal (==) to the extreme of the rest -- what the
// sequential scan with strict comparisons returns (py_min_seq / py_max_seq), ties and the
// sign of zero included, since the pair (value, first index) is carried
template <bool MAX>
__device__ __forceinline__ double py_ext_wave(const double* a, int n, int lane) {
  const double a0 = a[0];
  if (!(a0 == a0)) return a0;
  double bv = a0;
  int bi = 0;
  for (int i = lane; i < n; i += 64) {
    const double v = a[i];
    if (MAX ? v > bv : v < bv) {
      bv = v;
      bi = i;
    }
  }
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) {
    const double ov = __shfl_xor(bv, m);
    const int oi = __shfl_xor(bi, m);
    if ((MAX ? ov > bv : ov < bv) || (ov == bv && oi < bi)) {
      bv = ov;
      bi = oi;
    }
  }
  return bv;
}

// numpy's float32 leaf sum of a short LDS row (np_leaf_f32) with the 8 accumulators in lanes
// 0-7: the same additions in the same order, the result in every lane
__device__ __forceinline__ float np_leaf_f32_wave(const float* a, int n, int lane) {
  if (n < 8) return np_leaf_f32(a, n);
  const int nb = n - (n % 8);
  float r = 0.0f;
  if (lane < 8) {
    r = a[lane];
    for (int i = 8 + lane; i < nb; i += 8) r += a[i];
  }
  float q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) q[j] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, r), j));
  float res = ((q[0] + q[1]) + (q[2] + q[3])) + ((q[4] + q[5]) + (q[6] + q[7]));
  for (int i = nb; i < n; ++i) res += a[i];
  return res;
}

// mean, std, skew, kurtosis of x[0..n) (LDS) as numpy.mean / numpy.std / scipy.stats.skew /
// scipy.stats.kurtosis compute them in float64; tmp: n doubles of LDS scratch
template <bool NC>
__device__ __forceinline__ void stats4_f64(const double* x, double* tmp, int n, int lane, double (&o)[4]) {
  const double mean = np_sum_row<NC>(x, n, lane) / (double)n;
  for (int i = lane; i < n; i += 64) {
    const double d = x[i] - mean;
    tmp[i] = d * d;
  }
  lds_sync();
  const double m2 = np_sum_row<NC>(tmp, n, lane) / (double)n;
  lds_sync();
  for (int i = lane; i < n; i += 64) {
    const double d = x[i] - mean;
    tmp[i] = (d * d) * d;
  }
  lds_sync();
  const double m3 = np_sum_row<NC>(tmp, n, lane) / (double)n;
  lds_sync();
  for (int i = lane; i < n; i += 64) {
    const double d = x[i] - mean;
    const double d2 = d * d;
    tmp[i] = d2 * d2;
  }
  lds_sync();
  const double m4 = np_sum_row<NC>(tmp, n, lane) / (double)n;
  lds_sync();
  const double eps = 2.220446049250313e-16;
  const double zl = eps * mean;
  const bool zero = m2 <= zl * zl;
  o[0] = mean;
  o[1] = sqrt(m2);
  o[2] = zero ? NAN : m3 / pow(m2, 1.5);
  o[3] = zero ? NAN : m4 / (m2 * m2) - 3.0;
}

// the same in float32 (numpy on a float32 array): the element passes spread over the lanes,
// the leaf sums in lanes 0-7, the result in every lane
__device__ __forceinline__ void stats4_f32_wave(const float* a, float* tmp, int n, int lane, double (&o)[4]) {
  const float mean = np_leaf_f32_wave(a, n, lane) / (float)n;
  for (int i = lane; i < n; i += 64) {
    const float d = a[i] - mean;
    tmp[i] = d * d;
  }
  lds_sync();
  const float m2 = np_leaf_f32_wave(tmp, n, lane) / (float)n;
  lds_sync();
  for (int i = lane; i < n; i += 64) {
    const float d = a[i] - mean;
    tmp[i] = (d * d) * d;
  }
  lds_sync();
  const float m3 = np_leaf_f32_wave(tmp, n, lane) / (float)n;
  lds_sync();
  for (int i = lane; i < n; i += 64) {
    const float d = a[i] - mean;
    const float d2 = d * d;
    tmp[i] = d2 * d2;
  }
  lds_sync();
  const float m4 = np_leaf_f32_wave(tmp, n, lane) / (float)n;
  lds_sync();
  const float zl = 1.1920929e-07f * mean;
  const bool zero = m2 <= zl * zl;
  o[0] = (double)mean;
  o[1] = (double)sqrtf(m2);
  o[2] = zero ? NAN : (double)(m3 / powf(m2, 1.5f));
  o[3] = zero ? NAN : (double)(m4 / (m2 * m2) - 3.0f);
}

// ---- the 22-score path: candidate parameters and sub-band scores ---------------------
// CandidateFileInterface.filterScore(13|14) (CandidateFileInterface.py:97-107)
__device__ __forceinline__ double filter_neg_pfd(double v) {
  return (fabs(v - 0.0) > 0.000005 && v < 0.0) ? 0.0 : v;
}

// numpy.argmax over i of a[(i + shift) mod n] - sub (|shift| < n) as a wave reduction: the
// first NaN if there is one, else the first maximum (the values are the same roundings a
// sequential scan compares; ties go to the smaller i, so +0 / -0 ties too)
__device__ __forceinline__ int np_argmax_wave(const double* a, int n, int shift, double sub, int lane) {
  int nan_i = 1 << 30, bi = 1 << 30;
  double bv = 0.0;
  for (int i = lane; i < n; i += 64) {
    int j = i + shift;
    if (j >= n) j -= n;
    if (j < 0) j += n;
    const double v = a[j] - sub;
    if (!(v == v)) {
      if (i < nan_i) nan_i = i;
    } else if (bi == (1 << 30) || v > bv) {
      bv = v;
      bi = i;
    }
  }
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) {
    const int on = __shfl_xor(nan_i, m);
    const double ov = __shfl_xor(bv, m);
    const int oi = __shfl_xor(bi, m);
    nan_i = on < nan_i ? on : nan_i;
    if (oi != (1 << 30) && (bi == (1 << 30) || ov > bv || (ov == bv && oi < bi))) {
      bv = ov;
      bi = oi;
    }
  }
  return nan_i != (1 << 30) ? nan_i : (bi != (1 << 30) ? bi : 0);
}

// PFDOperations.getCandidateParameters (PFDOperations.py:130-231): the S/N of the profile
// against the mean / variance of its bins within 3 sigma, and the width between the half-
// maximum crossings of the profile rotated to put its peak at the centre.  The reference
// rotates with fft_rotate (:490-500) by an integer number of bins; this is the exact
// rotation, which pocketfft's round-off (~1e-13) can differ from only when a bin lies within
// that of the half maximum.
template <bool NC>
__device__ __forceinline__ void pfd_params(const double* prof, double* tmp, int L, int lane, double& snr,
                           double& width) {
  const double avg = np_sum_row<NC>(prof, L, lane) / (double)L;          // :130
  for (int b = lane; b < L; b += 64) {
    const double d = prof[b] - avg;
    tmp[b] = d * d;
  }
  lds_sync();
  const double var = np_sum_row<NC>(tmp, L, lane) / (double)L;          // :131
  lds_sync();
  const double sigma = sqrt(var);
  const double lo = avg - 3.0 * sigma, hi = avg + 3.0 * sigma;
  int m = 0;                                                              // :141-146
  for (int b0 = 0; b0 < L; b0 += 64) {
    const int b = b0 + lane;
    const bool keep = b < L && prof[b] > lo && prof[b] < hi;
    const uint64_t bal = __ballot(keep);
    if (keep) tmp[m + __popcll(bal & ((1ull << lane) - 1ull))] = prof[b];
    m += __popcll(bal);
  }
  lds_sync();
  const double avg2 = np_sum_row<NC>(tmp, m, lane) / (double)m;         // :148 (empty: NaN)
  lds_sync();
  for (int i = lane; i < m; i += 64) {
    const double d = tmp[i] - avg2;
    tmp[i] = d * d;
  }
  lds_sync();
  const double var2 = np_sum_row<NC>(tmp, m, lane) / (double)m;         // :149
  lds_sync();
  const double sd2 = sqrt(var2);
  for (int b = lane; b < L; b += 64) tmp[b] = (prof[b] - avg2) / sd2;
  lds_sync();
  snr = np_sum_row<NC>(tmp, L, lane);                                    // :151
  lds_sync();
  if (snr < 0.0) snr = 0.1;                                              // :152-153
  // width (:194-231): the sequential scans of the reference as wave reductions over the
  // same values (the rotated profile minus its Python min)
  const int peak0 = np_argmax_wave(prof, L, 0, 0.0, lane);
  const int shift = peak0 - L / 2;                                        // Py2 int '/'
  const double pmin = py_ext_wave<false>(prof, L, lane);
  auto rot = [&](int i) { int j = i + shift; if (j >= L) j -= L; if (j < 0) j += L; return prof[j] - pmin; };
  const int peak = np_argmax_wave(prof, L, shift, pmin, lane);
  // rmax: rot(0), raised by every later rot(i) > rmax -- NaN when rot(0) is, else the
  // largest non-NaN value (fmax skips NaN)
  const double r0 = rot(0);
  double rm = r0;
  for (int i = lane; i < L; i += 64) rm = fmax(rm, rot(i));
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) rm = fmax(rm, __shfl_xor(rm, m));
  const double rmax = (r0 == r0) ? rm : r0;
  const double half = rmax / 2.0;
  // left: the largest l in [1, peak] with rot(l) < half, else 0; right: the smallest r in
  // [peak, L) with rot(r) < half, else L (where the reference's walks stop)
  int left = 0, right = L;
  for (int i = lane; i < L; i += 64) {
    const bool below = rot(i) < half;
    if (below && i >= 1 && i <= peak && i > left) left = i;
    if (below && i >= peak && i < right) right = i;
  }
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) {
    const int ol = __shfl_xor(left, m), orr = __shfl_xor(right, m);
    left = ol > left ? ol : left;
    right = orr < right ? orr : right;
  }
  width = (1.0 * ((double)(right - left) - 1.0)) / (double)L;           // :231
}

// Pearson correlation as numpy.corrcoef computes it (see bates_sine_dm_sub.hip)
__device__ __forceinline__ double corr_pfd(double cxy, double cxx, double cyy) {
  double r = (cxy / sqrt(cxx)) / sqrt(cyy);
  if (r > 1.0) r = 1.0;
  if (r < -1.0) r = -1.0;
  return r;
}

// lane-strided partial sums then the wave tree (the order the PHCX kernels use for dots)
template <typename Fn>
__device__ __forceinline__ double wdot(int n, int lane, Fn f) {
  double s = 0.0;
  for (int j = lane; j < n; j += 64) s += f(j);
  return wsum(s);
}

// numpy's leaf sum (8 <= n <= 128) of eight rows at once: row g = lane / 8 in lanes
// 8g..8g+7, accumulator t = lane & 7 (its loads issued before its adds), combined
// ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) by DPP inside the 8 lanes, then the remainder in
// order: np_leaf's additions, so np_leaf's bits, in every lane of the group
__device__ __forceinline__ double np_leaf_rows8(const double* row, int n, int t) {
  const int nb = n - (n % 8);
  double v[16];
#pragma unroll
  for (int m = 0; m < 16; ++m) v[m] = row[min(t + 8 * m, n - 1)];
  double r = v[0];
#pragma unroll
  for (int m = 1; m < 16; ++m)
    if (8 * m < nb) r += v[m];
  r += dpp_f64<DPP_QUAD_XOR1>(r);
  r += dpp_f64<DPP_QUAD_XOR2>(r);
  r += dpp_f64<DPP_ROW_HALF_MIRROR>(r);
  for (int i = nb; i < n; ++i) r += row[i];
  return r;
}
// sum over the 8 lanes of a group (the per-band dots of s21 / s22, held to 1e-12)
__device__ __forceinline__ double sum8(double v) {
  v += dpp_f64<DPP_QUAD_XOR1>(v);
  v += dpp_f64<DPP_QUAD_XOR2>(v);
  v += dpp_f64<DPP_ROW_HALF_MIRROR>(v);
  return v;
}

// PFDOperations.getSubbandParameters (PFDOperations.py:401-441): s20 / s21 from
// ProfileOperations.getSubband_scores (ProfileOperations.py:1585-1686) over the dedispersed
// sub-band profiles T (nsub x L, profs.sum(0), PFDFile.plot_subbands :442-456) and s22 from
// getProfileCorr (:445-466).  T is overwritten (boxcar sums).  mb, mean, var: nsub doubles.
// false = the reference raises (max_bin unbound, width_bins == 0, no valid pair).
template <bool NC>
__device__ __forceinline__ bool pfd_subband_scores(double* T, const double* prof, double* tmp, double* mb,
                                   double* bmean, double* bvar, int NS, int L, int lane,
                                   double width, double (&o)[3]) {
  // s22 first, while T holds the sub-band profiles
  const double pm = np_sum_row<NC>(prof, L, lane) / (double)L;
  for (int b = lane; b < L; b += 64) tmp[b] = prof[b] - pm;
  lds_sync();
  const double inv2 = 1.0 / (double)(L - 1);
  const double pvar = wdot(L, lane, [&](int b) { return tmp[b] * tmp[b]; });
  double integ = 0.0;
  const bool rows8 = L >= 8 && L <= 128;
  if (rows8) {
    // eight bands per step (band j0 + lane / 8); the |cc| of each band in bvar, then summed
    // in band order
    const int g = lane >> 3, t = lane & 7;
    for (int j0 = 0; j0 < NS; j0 += 8) {
      const int j = min(j0 + g, NS - 1);
      const double* r = T + (size_t)j * L;
      const double mj = np_leaf_rows8(r, L, t) / (double)L;
      double dl_ = 0.0, ql_ = 0.0;
      for (int b = t; b < L; b += 8) {
        const double e = r[b] - mj;
        dl_ += e * tmp[b];
        ql_ += e * e;
      }
      const double d = sum8(dl_), q = sum8(ql_);
      if (t == 0 && j0 + g < NS) bvar[j] = fabs(corr_pfd(d * inv2, q * inv2, pvar * inv2));
    }
    lds_sync();
    for (int j = 0; j < NS; ++j)
      if (bvar[j] > 0.0055) integ += bvar[j];                          // :463-464, :437-439
  } else {
    for (int j = 0; j < NS; ++j) {
      const double* r = T + (size_t)j * L;
      const double mj = np_sum_row<NC>(r, L, lane) / (double)L;
      double dl_ = 0.0, ql_ = 0.0;  // wdot's order for both sums, in one pass
      for (int b = lane; b < L; b += 64) {
        const double e = r[b] - mj;
        dl_ += e * tmp[b];
        ql_ += e * e;
      }
      const double d = wsum(dl_);
      const double q = wsum(ql_);
      const double cc = fabs(corr_pfd(d * inv2, q * inv2, pvar * inv2));
      if (cc > 0.0055) integ += cc;                                    // :463-464, :437-439
    }
  }
  lds_sync();
  const int wb = (int)ceil(width * (double)L);                          // :1603
  const int nw = L - wb + 1;
  if (nw <= 0 || wb <= 0) return false;  // no windows: max_bin unbound; wb == 0: ZeroDivision
  // boxcar sums, a Python loop per window (:1608-1617), in place of each band's row
  bool have = false;
  double last_mb = 0.0;
  // packed: the boxcar rows are stored at an odd stride RS <= L (rows rewritten in band order
  // never reach a row not yet read), so the pair loop's lanes, all at the same j of different
  // rows, read distinct LDS banks
  const bool packed = rows8 && nw >= 8 && (nw | 1) <= L;
  const int RS = packed ? (nw | 1) : L;
  if (rows8) {
    // eight bands per step (band i0 + lane / 8, windows j = t mod 8 in registers until every
    // lane has read the row): the same sums in the same order; each band's first strict
    // maximum above -10000.0 by an 8-lane (value, first index) reduction; bmean holds the
    // band's max_bin or -1 (none), resolved in band order below
    const int g = lane >> 3, t = lane & 7;
    for (int i0 = 0; i0 < NS; i0 += 8) {
      const int i = i0 + g;
      const bool own = i < NS;
      double* r = T + (size_t)(own ? i : NS - 1) * L;
      double sv[16];
      double bvv = -10000.0;
      int bj = 1 << 30;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int j = t + 8 * q;
        double sm = 0.0;
        if (j < nw) {
          int b = 0;
          for (; b + 8 <= wb; b += 8) {
            double v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) v[u] = r[j + b + u];
#pragma unroll
            for (int u = 0; u < 8; ++u) sm += v[u];
          }
          for (; b < wb; ++b) sm += r[j + b];
          if (sm > bvv) {
            bvv = sm;
            bj = j;
          }
        }
        sv[q] = sm;
      }
      {
        double ov = dpp_f64<DPP_QUAD_XOR1>(bvv);
        int oj = dpp_i32<DPP_QUAD_XOR1>(bj);
        if (ov > bvv || (ov == bvv && oj < bj)) { bvv = ov; bj = oj; }
        ov = dpp_f64<DPP_QUAD_XOR2>(bvv);
        oj = dpp_i32<DPP_QUAD_XOR2>(bj);
        if (ov > bvv || (ov == bvv && oj < bj)) { bvv = ov; bj = oj; }
        ov = dpp_f64<DPP_ROW_HALF_MIRROR>(bvv);
        oj = dpp_i32<DPP_ROW_HALF_MIRROR>(bj);
        if (ov > bvv || (ov == bvv && oj < bj)) { bvv = ov; bj = oj; }
      }
      if (own && t == 0) bmean[i] = bj < (1 << 30) ? (double)(bj + wb / 2) : -1.0;  // Py2 wb/2
      lds_sync();
      if (own) {
        double* w = T + (size_t)i * RS;
#pragma unroll
        for (int q = 0; q < 16; ++q)
          if (t + 8 * q < nw) w[t + 8 * q] = sv[q];
      }
      lds_sync();
    }
    for (int i = 0; i < NS; ++i) {  // max_bin is one local across the bands
      const double v = bmean[i];
      if (v >= 0.0) {
        have = true;
        last_mb = v;
      }
      if (!have) return false;
      if (lane == 0) mb[i] = last_mb;
    }
    lds_sync();
  }
  for (int i = 0; !rows8 && i < NS; ++i) {
    double* r = T + (size_t)i * L;
    for (int j = lane; j < nw; j += 64) {
      double s = 0.0;  // r[j] + r[j+1] + ... in order; loads issued 8 at a time
      int b = 0;
      for (; b + 8 <= wb; b += 8) {
        double v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = r[j + b + u];
#pragma unroll
        for (int u = 0; u < 8; ++u) s += v[u];
      }
      for (; b < wb; ++b) s += r[j + b];
      tmp[j] = s;
    }
    lds_sync();
    // first strict maximum above -10000.0 (:1619-1628); a band without one repeats the
    // previous band's position (max_bin is one local across the bands)
    double bvv = -10000.0;
    int bj = 1 << 30;
    for (int j = lane; j < nw; j += 64)
      if (tmp[j] > bvv) {
        bvv = tmp[j];
        bj = j;
      }
#pragma unroll
    for (int s = 1; s < 64; s <<= 1) {
      const double ov = __shfl_xor(bvv, s);
      const int oj = __shfl_xor(bj, s);
      if (ov > bvv || (ov == bvv && oj < bj)) {
        bvv = ov;
        bj = oj;
      }
    }
    if (bj < (1 << 30)) {
      have = true;
      last_mb = (double)(bj + wb / 2);                                  // Py2 wb/2
    }
    if (!have) return false;
    if (lane == 0) mb[i] = last_mb;
    for (int j = lane; j < nw; j += 64) r[j] = tmp[j];
    lds_sync();
  }
  // RMS scatter of the maxima (:1629-1651)
  const double med = np_sum_row<NC>(mb, NS, lane) / (double)NS;
  int count = 0;
  double var_med = 0.0;
  for (int i = 0; i < NS; ++i)
    if (fabs(mb[i] - med) <= (double)wb) {
      ++count;
      var_med += (mb[i] - med) * (mb[i] - med);
    }
  double var;
  if (count > 1) {
    var = var_med / (double)(count - 1);
  } else {
    double mu = 0.0;
    for (int i = 0; i < NS; ++i) mu += mb[i];
    mu /= (double)NS;
    var = 0.0;
    for (int i = 0; i < NS; ++i) var += (mb[i] - mu) * (mb[i] - mu);
    var /= (double)(NS - 1);
  }
  const double rms = sqrt(var) / (double)wb;
  // mean pairwise correlation of the boxcar sums, pairs (i < k) in order (:1653-1677)
  if (rows8 && nw >= 8) {
    // eight bands per step: numpy's mean of the boxcar row, centred in place by the lanes
    // that own the elements (j = t mod 8), then the sum of squares
    const int g = lane >> 3, t = lane & 7;
    for (int i0 = 0; i0 < NS; i0 += 8) {
      const int i = i0 + g;
      const bool own = i < NS;
      double* r = T + (size_t)(own ? i : NS - 1) * RS;
      const double m = np_leaf_rows8(r, nw, t) / (double)nw;
      lds_sync();
      double v = 0.0;
      for (int j = t; j < nw; j += 8) {
        const double c = r[j] - m;
        if (own) r[j] = c;
        v += c * c;
      }
      v = sum8(v);
      if (own && t == 0) bvar[i] = v;
      lds_sync();
    }
  } else {
    for (int i = 0; i < NS; ++i) {
      double* r = T + (size_t)i * L;
      const double m = np_sum_row<NC>(r, nw, lane) / (double)nw;
      lds_sync();
      for (int j = lane; j < nw; j += 64) r[j] = r[j] - m;
      lds_sync();
      const double v = wdot(nw, lane, [&](int j) { return r[j] * r[j]; });
      if (lane == 0) bvar[i] = v;
    }
  }
  lds_sync();
  // one pair per lane at a time (rows at the odd stride RS, or from a lane-dependent start
  // when not packed, so the 64 lanes' LDS reads of one step spread over the banks), and the
  // pairs' correlations are summed as a wave reduction (s21 is held to 1e-12: numpy's
  // own dots run in BLAS order)
  const double inv = 1.0 / (double)(nw - 1);
  double csum_l = 0.0;
  int m_l = 0;
  const int npairs = NS * (NS - 1) / 2;
  for (int p = lane; p < npairs; p += 64) {
    int i = 0, rem = p;
    while (rem >= NS - 1 - i) {
      rem -= NS - 1 - i;
      ++i;
    }
    const int k = i + 1 + rem;
    const double* ri = T + (size_t)i * RS;
    const double* rk = T + (size_t)k * RS;
    double d = 0.0;
    if (packed) {  // every lane at the same j: four chains, loads first
      double d0 = 0.0, d1 = 0.0, d2 = 0.0, d3 = 0.0;
      int j = 0;
      for (; j + 4 <= nw; j += 4) {
        const double a0 = ri[j], a1 = ri[j + 1], a2 = ri[j + 2], a3 = ri[j + 3];
        const double b0 = rk[j], b1 = rk[j + 1], b2 = rk[j + 2], b3 = rk[j + 3];
        d0 += a0 * b0;
        d1 += a1 * b1;
        d2 += a2 * b2;
        d3 += a3 * b3;
      }
      for (; j < nw; ++j) d0 += ri[j] * rk[j];
      d = (d0 + d1) + (d2 + d3);
    } else {
      int j = lane % nw;
      for (int t = 0; t < nw; ++t) {
        d += ri[j] * rk[j];
        j = (j + 1 == nw) ? 0 : j + 1;
      }
    }
    const double cc = corr_pfd(d * inv, bvar[i] * inv, bvar[k] * inv);
    if (cc == cc) {
      csum_l += cc;
      ++m_l;
    }
  }
  const double csum = wsum(csum_l);
  const int m = wsum_i(m_l);
  if (m == 0) return false;                                             // ZeroDivisionError
  o[0] = rms;
  o[1] = csum / (double)m;
  o[2] = integ;
  return true;
}

// the rest of a fold after the chi^2 sweep (one wave): DM-curve statistics, the 22-score
// parameters and sub-band scores, status
template <bool NC>
__device__ __forceinline__ void pfd_finish(const PfdArgs& a, int64_t c, double* T, double* buf,
                                        double* tmp, double* dl, double* sdb, double* bv,
                                        float* chs, float* ftmp, const double (&po)[4],
                                        bool dm_ok, int lane) {
  const double* sc = a.scal + c * PFE_PFD_NSCAL;
  const double bestdm = sc[PFE_PFD_BESTDM];
  const double dm_lo = sc[PFE_PFD_DM_LO], dm_hi = sc[PFE_PFD_DM_HI];
  const int NS = a.nsub, L = a.L;
  if (a.lyon8) {
    double dmo[4] = {0.0, 0.0, 0.0, 0.0};
    if (dm_ok) stats4_f32_wave(chs, ftmp, PFE_PFD_NDM, lane, dmo);
    if (lane == 0) {
      double* o = a.lyon8 + c * 8;
      for (int i = 0; i < 4; ++i) {
        o[i] = po[i];
        o[4 + i] = dm_ok ? dmo[i] : NAN;
      }
    }
  }
  uint32_t st = dm_ok ? 0u : PFE_ST_PFD_DMCURVE_FAIL;
  if (a.out22) {
    double snr, width;
    pfd_params<NC>(buf, tmp, L, lane, snr, width);
    const double period = sc[PFE_PFD_BARY_P1] * 1000.0;            // PFDOperations.py:127
    const double span1 = dm_lo + ((dm_hi - dm_lo) * 1.0) / (double)(PFE_PFD_NDM - 1);
    const double span_last =
        dm_lo + ((dm_hi - dm_lo) * (double)(PFE_PFD_NDM - 1)) / (double)(PFE_PFD_NDM - 1);
    double sb[3];
    const bool sb_ok = pfd_subband_scores<NC>(T, buf, tmp, dl, sdb, bv, NS, L, lane, width, sb);
    if (!sb_ok) st |= PFE_ST_SUBBAND_FAIL;
    if (lane == 0) {
      double* o = a.out22 + c * 22;
      o[11] = period;                                                 // s12 (PFDFile.py:776)
      o[12] = filter_neg_pfd(snr);                                    // s13 (:777)
      o[13] = filter_neg_pfd(bestdm);                                 // s14 (:778)
      o[14] = width;                                                  // s15
      o[19] = sb[0];                                                  // s20 (:861-863)
      o[20] = sb[1];                                                  // s21
      o[21] = sb[2];                                                  // s22
      double* q = a.par22 + c * 8;
      q[0] = period;
      q[1] = snr;
      q[2] = bestdm;
      q[3] = width;
      q[4] = span1;      // float(dm_index[1])            (PFDOperations.py:337)
      q[5] = span_last;  // float(dm_index[len - 1])
      q[6] = 0.0;
      q[7] = 0.0;
    }
  }
  if (lane == 0) a.status[c] = st;
}

__global__ __launch_bounds__(64) void k_pfd_dmprof(PfdArgs a) {
  extern __shared__ double lds[];
  const int64_t c = blockIdx.x;
  if (c >= a.n) return;
  const int lane = lane_id();
  const int NP = a.npart, NS = a.nsub, L = a.L;
  double* T = lds;                  // NS x L: sub-band profiles summed over parts, dedispersed
  double* buf = T + (size_t)NS * L;  // L
  double* tmp = buf + L;             // L
  double* dl = tmp + L;              // NS delays
  double* sdb = dl + NS;             // NS subdelays_bins
  double* bv = sdb + NS;             // NS (22-score path: per-band variances)
  int* cum = (int*)(bv + NS);        // NS rotations applied since the dedispersion
  __shared__ float chs[PFE_PFD_NDM], ftmp[PFE_PFD_NDM];
  const double* sc = a.scal + c * PFE_PFD_NSCAL;
  const double bestdm = sc[PFE_PFD_BESTDM], bps = sc[PFE_PFD_BINSPERSEC];
  const double avgprof = sc[PFE_PFD_AVGPROF], varprof = sc[PFE_PFD_VARPROF];
  const double dm_lo = sc[PFE_PFD_DM_LO], dm_hi = sc[PFE_PFD_DM_HI];
  const double numdms = sc[PFE_PFD_NUMDMS];
  const double* fr = a.subfreqs + c * NS;
  const double* P = a.profs + c * (int64_t)NP * NS * L;
  // ---- dedisperse at the best DM (PFDFile.py:346-373, interp = 0)
  for (int j = lane; j < NS; j += 64) dl[j] = delay_from_dm(bestdm, fr[j]);
  lds_sync();
  {
    const double hif = dl[NS - 1];
    for (int j = lane; j < NS; j += 64) {
      const double delaybins = (dl[j] - hif) * bps - 0.0;
      const double nw = floor(delaybins + 0.5);
      sdb[j] = 0.0 + nw;
      cum[j] = pymod((long long)nw, L);  // rotation of the dedispersion itself
    }
  }
  lds_sync();
  // T[j][b] = sum over parts of the rotated sub-integration profiles (profs.sum(0))
  for (int j = 0; j < NS; ++j) {
    const int r = cum[j];
    for (int b = lane; b < L; b += 64) {
      const int src = b + r < L ? b + r : b + r - L;
      double s = P[(int64_t)j * L + src];
      for (int p = 1; p < NP; ++p) s += P[((int64_t)p * NS + j) * L + src];
      T[(size_t)j * L + b] = s;
    }
  }
  lds_sync();
  // sumprof = T.sum(0); the profile (getprofile + scale)
  for (int b = lane; b < L; b += 64) {
    double s = T[b];
    for (int j = 1; j < NS; ++j) s += T[(size_t)j * L + b];
    buf[b] = s;
  }
  lds_sync();
  {
    const double mn = py_ext_wave<false>(buf, L, lane);
    for (int b = lane; b < L; b += 64) buf[b] = buf[b] - mn;  // normprof
    lds_sync();
    const double mean = np_sum_row<false>(buf, L, lane) / (double)L;
    lds_sync();
    for (int b = lane; b < L; b += 64) buf[b] = buf[b] / mean;  // s
    lds_sync();
    const double smin = py_ext_wave<false>(buf, L, lane), smax = py_ext_wave<true>(buf, L, lane);
    lds_sync();
    for (int b = lane; b < L; b += 64) {
      const double t = (buf[b] - smin) / (smax - smin);
      buf[b] = (0.0 * (1.0 - t)) + (255.0 * t);
      if (a.profile) a.profile[c * L + b] = buf[b];
    }
    lds_sync();
  }
  double po[4] = {0.0, 0.0, 0.0, 0.0};
  if (a.lyon8) stats4_f64<false>(buf, tmp, L, lane, po);
  // ---- chi^2 versus DM over span(dms[0], dms[-1], 100) (PFDFile.py:378-423)
  const bool dm_ok = numdms > 1.0;  // numdms == 1: dms is a scalar and dms[0] raises
  if (dm_ok && (a.chis || a.lyon8)) {
    for (int j = lane; j < NS; j += 64) cum[j] = 0;
    lds_sync();
    for (int k = 0; k < PFE_PFD_NDM; ++k) {
      const double dm = dm_lo + ((dm_hi - dm_lo) * (double)k) / (double)(PFE_PFD_NDM - 1);
      for (int j = lane; j < NS; j += 64) dl[j] = delay_from_dm(dm, fr[j]);
      lds_sync();
      const double hif = dl[NS - 1];
      for (int j = lane; j < NS; j += 64) {
        const double delaybins = (dl[j] - hif) * bps - sdb[j];
        const double nw = floor(delaybins + 0.5);
        cum[j] = pymod((long long)cum[j] + (long long)nw, L);
        sdb[j] = sdb[j] + nw;
      }
      lds_sync();
      for (int b = lane; b < L; b += 64) {
        double s = 0.0;
        for (int j = 0; j < NS; ++j) {
          int src = b + cum[j];
          if (src >= L) src -= L;
          const double v = T[(size_t)j * L + src];
          s = (j == 0) ? v : s + v;
        }
        const double d = s - avgprof;
        tmp[b] = (d * d) / varprof;
      }
      lds_sync();
      const double chi = np_pairwise<12>(tmp, L, lane) / ((double)L - 1.0);
      lds_sync();
      if (lane == 0) chs[k] = (float)chi;
      if (a.chis && lane == 0) a.chis[c * PFE_PFD_NDM + k] = (float)chi;
    }
    lds_sync();
  }
  pfd_finish<false>(a, c, T, buf, tmp, dl, sdb, bv, chs, ftmp, po, dm_ok, lane);
}

#ifndef PFE_PFD4_E
#define PFE_PFD4_E 8
#endif
constexpr int PFD4_E = PFE_PFD4_E;  // fold elements per thread and load step of k_pfd_dmprof4

// the accumulated sub-band rotations of the 100 trial DMs (PFDFile.py:395-416), one lane
// per sub-band: rot[k][j] (the sweep of the single-wave kernel keeps them in cum / sdb)
__device__ __forceinline__ void sweep_rotations(uint16_t* rot, const double* sdb, const double* fr,
                                                int NS, int L, double bps, double dm_lo,
                                                double dm_hi, int lane) {
  for (int j = lane; j < NS; j += 64) {
    int cu = 0;
    double sd = sdb[j];
    for (int k = 0; k < PFE_PFD_NDM; ++k) {
      const double dm = dm_lo + ((dm_hi - dm_lo) * (double)k) / (double)(PFE_PFD_NDM - 1);
      const double hif = delay_from_dm(dm, fr[NS - 1]);
      const double delaybins = (delay_from_dm(dm, fr[j]) - hif) * bps - sd;
      const double nw = floor(delaybins + 0.5);
      cu = pymod((long long)cu + (long long)nw, L);
      sd = sd + nw;
      rot[k * NS + j] = (uint16_t)cu;  // 0 <= cu < L <= 128
    }
  }
}

// The 100-DM chi^2 sweep of k_pfd_dmprof4 for L = 64 / 128 and nsub a multiple of 8 (the
// PRESTO fold shapes): the same additions in the same order as the general loop below, with
// less issue per LDS read.  A trial DM's rotation of sub-band j is wave-uniform, so lanes
// 0-15 read the rotations of two DMs for 8 sub-bands at once and readlane makes them scalar;
// the wrap (b + r) mod L is a mask; and each wave sweeps two DMs at a time (k, k + 4), four
// independent ordered chains per lane.  numpy's pairwise leaf of the two chi^2 rows runs in
// lanes 0-7 (DM k) and 8-15 (DM k + 4) together.
template <int L>
__device__ __forceinline__ void sweep_pow2(const double* T, const uint16_t* rot, int NS, int wv,
                                           int lane, double avgprof, double varprof,
                                           double* xb, float* chs, float* chis) {
  constexpr int B = L / 64;  // bins per lane
  static_assert(B == 1 || B == 2, "L = 64 or 128");
  for (int k0 = wv; k0 < PFE_PFD_NDM; k0 += 8) {
    const bool two = k0 + 4 < PFE_PFD_NDM;  // wave-uniform
    const int k1 = two ? k0 + 4 : k0;
    const uint16_t* ra = rot + k0 * NS;
    const uint16_t* rb = rot + k1 * NS;
    double s[2][B];
    for (int j0 = 0; j0 < NS; j0 += 8) {
      const int rv = lane < 8 ? (int)ra[j0 + lane] : lane < 16 ? (int)rb[j0 + lane - 8] : 0;
      // two halves of 4 sub-bands (the same adds in the same order as one step of 8; half
      // the registers for the row reads in flight)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        double v[2][4][B];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int r0 = __builtin_amdgcn_readlane(rv, 4 * h + u);
          const int r1 = __builtin_amdgcn_readlane(rv, 8 + 4 * h + u);
          const double* row = T + (size_t)(j0 + 4 * h + u) * L;
#pragma unroll
          for (int q = 0; q < B; ++q) {
            const int b = lane + 64 * q;
            v[0][u][q] = row[(b + r0) & (L - 1)];
            v[1][u][q] = row[(b + r1) & (L - 1)];
          }
        }
#pragma unroll
        for (int d = 0; d < 2; ++d)
#pragma unroll
          for (int q = 0; q < B; ++q) {
            double t = (j0 == 0 && h == 0) ? v[d][0][q] : s[d][q] + v[d][0][q];
#pragma unroll
            for (int u = 1; u < 4; ++u) t = t + v[d][u][q];
            s[d][q] = t;
          }
      }
    }
    // chi^2 terms of both DMs, then numpy's leaf: r_i = x[i] + x[i+8] + ... (L multiple of 8)
#pragma unroll
    for (int d = 0; d < 2; ++d)
#pragma unroll
      for (int q = 0; q < B; ++q) {
        const double e = s[d][q] - avgprof;
        xb[d * 128 + lane + 64 * q] = (e * e) / varprof;
      }
    lds_sync();
    const double* xr = xb + ((lane >> 3) & 1) * 128;
    double w[L / 8];
#pragma unroll
    for (int m = 0; m < L / 8; ++m) w[m] = xr[(lane & 7) + 8 * m];
    double r = w[0];
#pragma unroll
    for (int m = 1; m < L / 8; ++m) r += w[m];
    const double den = (double)L - 1.0;
#pragma unroll
    for (int d = 0; d < 2; ++d) {
      const int o = 8 * d;
      const double r0 = bcast(r, o), r1 = bcast(r, o + 1), r2 = bcast(r, o + 2), r3 = bcast(r, o + 3);
      const double r4 = bcast(r, o + 4), r5 = bcast(r, o + 5), r6 = bcast(r, o + 6), r7 = bcast(r, o + 7);
      const double chi = (((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7))) / den;
      const int k = d ? k1 : k0;
      if (lane == 0 && (d == 0 || two)) {
        chs[k] = (float)chi;
        if (chis) chis[k] = (float)chi;
      }
    }
    lds_sync();
  }
}

// Four-wave form of k_pfd_dmprof for profiles of <= 128 bins (the same arithmetic, bit for
// bit).  The single-wave kernel streamed the fold with one dependent load per lane at a time
// and swept the 100 trial DMs one after another; here
//   * all 256 threads reduce the fold over its parts, 8 elements x 2 parts of loads in
//     flight per thread (each element still sums its parts in order, as numpy);
//   * wave 3 tabulates the accumulated sub-band rotations of all 100 trial DMs while its
//     first loads are in flight;
//   * the sweep runs 4 trial DMs at a time, one per wave: the lanes sum the rotated sub-band
//     rows bin by bin (64 consecutive doubles of a row per read, so the LDS reads are
//     conflict-free) and numpy's pairwise leaf sums the chi^2 terms;
//   * wave 0 builds the profile and finishes the fold (statistics, 22-score parameters) as
//     the single-wave kernel.
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3, 3))) void k_pfd_dmprof4(PfdArgs a) {
  extern __shared__ double lds[];
  const int64_t c = blockIdx.x;
  if (c >= a.n) return;
  const int tid = threadIdx.x;
  const int wv = tid >> 6;
  const int lane = lane_id();
  const int NP = a.npart, NS = a.nsub, L = a.L;
  double* T = lds;                   // NS x L
  double* buf = T + (size_t)NS * L;  // L
  double* tmp = buf + L;             // L
  double* dl = tmp + L;              // NS
  double* sdb = dl + NS;             // NS
  double* bv = sdb + NS;             // NS
  int* cum = (int*)(bv + NS);        // NS
  uint16_t* rot = (uint16_t*)(cum + NS);  // PFE_PFD_NDM x NS accumulated rotations (< L)
  double* xbuf = bv + NS + (4 * NS + 2 * PFE_PFD_NDM * NS + 7) / 8;  // 4 x 256, after cum, rot
  __shared__ float chs[PFE_PFD_NDM], ftmp[PFE_PFD_NDM];
  const double* sc = a.scal + c * PFE_PFD_NSCAL;
  const double bestdm = sc[PFE_PFD_BESTDM], bps = sc[PFE_PFD_BINSPERSEC];
  const double avgprof = sc[PFE_PFD_AVGPROF], varprof = sc[PFE_PFD_VARPROF];
  const double dm_lo = sc[PFE_PFD_DM_LO], dm_hi = sc[PFE_PFD_DM_HI];
  const double numdms = sc[PFE_PFD_NUMDMS];
  const double* fr = a.subfreqs + c * NS;
  const double* P = a.profs + c * (int64_t)NP * NS * L;
  const bool dm_ok = numdms > 1.0;  // numdms == 1: dms is a scalar and dms[0] raises
  const bool sweep = dm_ok && (a.chis || a.lyon8);
  // ---- dedisperse at the best DM (PFDFile.py:346-373, interp = 0)
  if (wv == 0) {
    for (int j = lane; j < NS; j += 64) dl[j] = delay_from_dm(bestdm, fr[j]);
    lds_sync();
    const double hif = dl[NS - 1];
    for (int j = lane; j < NS; j += 64) {
      const double delaybins = (dl[j] - hif) * bps - 0.0;
      const double nw = floor(delaybins + 0.5);
      sdb[j] = 0.0 + nw;
      cum[j] = pymod((long long)nw, L);
    }
  }
  __syncthreads();
  // T[j][b] = sum over parts of the rotated sub-integration profiles (profs.sum(0)): each
  // thread keeps PFD4_E elements and walks the parts, so PFD4_E loads are in flight per
  // thread and step; wave 3 first tabulates the sweep's rotations (below), overlapping them
  // with its first loads.  Split pipeline: T comes from k_pfd_parts (the same sums).
  if (a.tin) {
    const int total = NS * L;
    const double* tg = a.tin + c * (int64_t)total;
    if (wv == 3 && sweep) sweep_rotations(rot, sdb, fr, NS, L, bps, dm_lo, dm_hi, lane);
    for (int e = tid; e < total; e += 256) T[e] = tg[e];
  } else {
    const int total = NS * L;
    const int64_t pstride = (int64_t)NS * L;
    for (int e0 = tid; e0 < total; e0 += 256 * PFD4_E) {
      int src[PFD4_E];
      bool ok[PFD4_E];
      double acc[PFD4_E];
#pragma unroll
      for (int u = 0; u < PFD4_E; ++u) {
        const int e = e0 + 256 * u;
        ok[u] = e < total;
        const int j = ok[u] ? e / L : 0;
        const int b = ok[u] ? e - j * L : 0;
        const int r = cum[j];
        src[u] = j * L + (b + r < L ? b + r : b + r - L);
        acc[u] = ok[u] ? P[src[u]] : 0.0;
      }
      if (wv == 3 && sweep && e0 == tid) sweep_rotations(rot, sdb, fr, NS, L, bps, dm_lo, dm_hi, lane);
#pragma unroll 2
      for (int p = 1; p < NP; ++p) {
        double v[PFD4_E];
#pragma unroll
        for (int u = 0; u < PFD4_E; ++u) v[u] = ok[u] ? P[p * pstride + src[u]] : 0.0;
#pragma unroll
        for (int u = 0; u < PFD4_E; ++u) acc[u] += v[u];
      }
#pragma unroll
      for (int u = 0; u < PFD4_E; ++u)
        if (ok[u]) T[e0 + 256 * u] = acc[u];
    }
    if (wv == 3 && sweep && tid >= total) sweep_rotations(rot, sdb, fr, NS, L, bps, dm_lo, dm_hi, lane);
  }
  __syncthreads();
  // ---- chi^2 versus DM over span(dms[0], dms[-1], 100) (PFDFile.py:378-423): each wave
  // takes every 4th trial DM; its lanes sum the rotated sub-band rows over the bins (a wave
  // reads 64 consecutive doubles of a row at a time), the chi^2 terms go to the wave's LDS
  // row and numpy's pairwise leaf sums them (np_leaf, lanes 0-7)
#if defined(PFE_PFD_PROBE) && PFE_PFD_PROBE == 1  // instrumented build: no sweep
  if (sweep) {
  } else if (false) {
#else
  if (sweep && (L == 128 || L == 64) && NS % 8 == 0) {
#endif
    double* xb = xbuf + wv * 256;
    float* chis = a.chis ? a.chis + c * PFE_PFD_NDM : nullptr;
    if (L == 128)
      sweep_pow2<128>(T, rot, NS, wv, lane, avgprof, varprof, xb, chs, chis);
    else
      sweep_pow2<64>(T, rot, NS, wv, lane, avgprof, varprof, xb, chs, chis);
  } else if (sweep) {
    double* xb = xbuf + wv * 256;
    const int b0 = lane, b1 = lane + 64;
    for (int k = wv; k < PFE_PFD_NDM; k += 4) {
      const uint16_t* rk = rot + k * NS;
      // 8 sub-bands per step: their rotations, then all 16 row reads, then the ordered adds
      // (unconditional reads at clamped indices keep every load of a step in flight)
      double s0 = 0.0, s1 = 0.0;
      const int b0c = b0 < L ? b0 : 0, b1c = b1 < L ? b1 : 0;
      for (int j0 = 0; j0 < NS; j0 += 8) {
        int r[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) r[u] = rk[min(j0 + u, NS - 1)];
        double v0[8], v1[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const double* row = T + (size_t)min(j0 + u, NS - 1) * L;
          int i0 = b0c + r[u];
          if (i0 >= L) i0 -= L;
          int i1 = b1c + r[u];
          if (i1 >= L) i1 -= L;
          v0[u] = row[i0];
          v1[u] = row[i1];
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (j0 + u < NS) {
            s0 = (j0 + u == 0) ? v0[u] : s0 + v0[u];
            s1 = (j0 + u == 0) ? v1[u] : s1 + v1[u];
          }
      }
      if (b0 < L) {
        const double d = s0 - avgprof;
        xb[b0] = (d * d) / varprof;
      }
      if (b1 < L) {
        const double d = s1 - avgprof;
        xb[b1] = (d * d) / varprof;
      }
      lds_sync();
      const double chi = (L >= 8 ? np_leaf128(xb, L, lane) : np_leaf(xb, L, lane)) / ((double)L - 1.0);
      if (lane == 0) {
        chs[k] = (float)chi;
        if (a.chis) a.chis[c * PFE_PFD_NDM + k] = (float)chi;
      }
      lds_sync();
    }
  }
  __syncthreads();
#if defined(PFE_PFD_PROBE) && PFE_PFD_PROBE == 2  // instrumented build: no wave-0 tail
  return;
#endif
  if (wv != 0) return;
  // (the profile is built after the sweep: it does not feed it, and the wave-0-only calls it
  // makes kept out of the divergent part before the sweep)
  double po[4] = {0.0, 0.0, 0.0, 0.0};
  {
    // sumprof = T.sum(0); the profile (getprofile + scale)
    for (int b = lane; b < L; b += 64) {
      double s = T[b];
      for (int j = 1; j < NS; ++j) s += T[(size_t)j * L + b];
      buf[b] = s;
    }
    lds_sync();
    const double mn = py_ext_wave<false>(buf, L, lane);
    for (int b = lane; b < L; b += 64) buf[b] = buf[b] - mn;  // normprof
    lds_sync();
    const double mean = np_sum_row<true>(buf, L, lane) / (double)L;
    lds_sync();
    for (int b = lane; b < L; b += 64) buf[b] = buf[b] / mean;  // s
    lds_sync();
    const double smin = py_ext_wave<false>(buf, L, lane), smax = py_ext_wave<true>(buf, L, lane);
    lds_sync();
    for (int b = lane; b < L; b += 64) {
      const double t = (buf[b] - smin) / (smax - smin);
      buf[b] = (0.0 * (1.0 - t)) + (255.0 * t);
      if (a.profile) a.profile[c * L + b] = buf[b];
    }
    lds_sync();
    if (a.lyon8) stats4_f64<true>(buf, tmp, L, lane, po);
  }
  pfd_finish<true>(a, c, T, buf, tmp, dl, sdb, bv, chs, ftmp, po, dm_ok, lane);
}

// Split pipeline, stage 1: the fold's part sums T (as k_pfd_dmprof4 reduces them: the
// dedispersion rotations of wave 0, then each element summing its parts in order) streamed
// to global memory.  Little LDS and no sweep state, so many blocks per CU keep enough loads
// in flight to stream the folds at HBM rate while k_pfd_dmprof4 sweeps the previous chunk.
__global__ __launch_bounds__(256) void k_pfd_parts(PfdArgs a, double* __restrict__ tout) {
  extern __shared__ double lds[];
  const int64_t c = blockIdx.x;
  if (c >= a.n) return;
  const int tid = threadIdx.x;
  const int lane = lane_id();
  const int NP = a.npart, NS = a.nsub, L = a.L;
  double* dl = lds;               // NS
  int* cum = (int*)(dl + NS);     // NS
  const double* sc = a.scal + c * PFE_PFD_NSCAL;
  const double bestdm = sc[PFE_PFD_BESTDM], bps = sc[PFE_PFD_BINSPERSEC];
  const double* fr = a.subfreqs + c * NS;
  const double* P = a.profs + c * (int64_t)NP * NS * L;
  if ((tid >> 6) == 0) {  // PFDFile.py:346-373 (interp = 0), as k_pfd_dmprof4's wave 0
    for (int j = lane; j < NS; j += 64) dl[j] = delay_from_dm(bestdm, fr[j]);
    lds_sync();
    const double hif = dl[NS - 1];
    for (int j = lane; j < NS; j += 64) {
      const double delaybins = (dl[j] - hif) * bps - 0.0;
      const double nw = floor(delaybins + 0.5);
      cum[j] = pymod((long long)nw, L);
    }
  }
  __syncthreads();
  const int total = NS * L;
  const int64_t pstride = (int64_t)NS * L;
  double* tg = tout + c * (int64_t)total;
  for (int e0 = tid; e0 < total; e0 += 256 * PFD4_E) {
    int src[PFD4_E];
    bool ok[PFD4_E];
    double acc[PFD4_E];
#pragma unroll
    for (int u = 0; u < PFD4_E; ++u) {
      const int e = e0 + 256 * u;
      ok[u] = e < total;
      const int j = ok[u] ? e / L : 0;
      const int b = ok[u] ? e - j * L : 0;
      const int r = cum[j];
      src[u] = j * L + (b + r < L ? b + r : b + r - L);
      acc[u] = ok[u] ? __builtin_nontemporal_load(P + src[u]) : 0.0;
    }
#pragma unroll 2
    for (int p = 1; p < NP; ++p) {
      double v[PFD4_E];
#pragma unroll
      for (int u = 0; u < PFD4_E; ++u)
        v[u] = ok[u] ? __builtin_nontemporal_load(P + p * pstride + src[u]) : 0.0;
#pragma unroll
      for (int u = 0; u < PFD4_E; ++u) acc[u] += v[u];
    }
#pragma unroll
    for (int u = 0; u < PFD4_E; ++u)
      if (ok[u]) tg[e0 + 256 * u] = acc[u];
  }
}

size_t pfd_lds_bytes(int nsub, int L) {
  return ((size_t)nsub * L + 2 * (size_t)L + 3 * (size_t)nsub) * sizeof(double) +
         (size_t)nsub * sizeof(int) + 64;
}

static size_t pfd4_lds_bytes(int nsub, int L) {
  return pfd_lds_bytes(nsub, L) + (size_t)PFE_PFD_NDM * nsub * sizeof(uint16_t) + 8 +
         4 * 256 * sizeof(double);
}

// the four-wave kernel: <= 128 bins, the fold in LDS, and rows of <= 968 values (its
// pairwise sums are inlined three levels deep, np_sum_row<true>)
static bool pfd4_ok(const PfdArgs& a) {
  // nsub: the sub-band sums go through np_pairwise_inl<3>, numpy's order up to np_inl_max(3)
  return a.L <= 128 && a.nsub <= np_inl_max(3) && pfd4_lds_bytes(a.nsub, a.L) <= 64 * 1024 &&
         a.waves == 4;
}

bool pfd_split_ok(const PfdArgs& a) {
  return pfd4_ok(a);
}

// the folds [c0, c0 + cn) of a batch: every per-fold pointer moved to fold c0
static PfdArgs pfd_chunk(const PfdArgs& a, int64_t c0, int64_t cn) {
  PfdArgs b = a;
  b.n = cn;
  b.profs = a.profs + c0 * (int64_t)a.npart * a.nsub * a.L;
  b.subfreqs = a.subfreqs + c0 * a.nsub;
  b.scal = a.scal + c0 * PFE_PFD_NSCAL;
  if (a.profile) b.profile = a.profile + c0 * a.L;
  if (a.chis) b.chis = a.chis + c0 * PFE_PFD_NDM;
  if (a.lyon8) b.lyon8 = a.lyon8 + c0 * 8;
  if (a.status) b.status = a.status + c0;
  if (a.out22) b.out22 = a.out22 + c0 * 22;
  if (a.par22) b.par22 = a.par22 + c0 * 8;
  return b;
}

hipError_t launch_pfd_dmprof_split(const PfdArgs& a, hipStream_t st, hipStream_t side, double* ws,
                                   int64_t chunk, hipEvent_t (&ev)[4]) {
  const size_t lds4 = pfd4_lds_bytes(a.nsub, a.L);
  hipError_t e = ensure_dyn_lds<k_pfd_dmprof4>(lds4);
  if (e != hipSuccess) return e;
  const size_t ldsp = (size_t)a.nsub * (sizeof(double) + sizeof(int)) + 16;
  const int64_t per = (int64_t)a.nsub * a.L;
  // side waits for everything queued on st before the call (the inputs may come from it)
  if ((e = hipEventRecord(ev[2], st)) != hipSuccess) return e;
  if ((e = hipStreamWaitEvent(side, ev[2], 0)) != hipSuccess) return e;
  int k = 0;
  for (int64_t c0 = 0; c0 < a.n; c0 += chunk, ++k) {
    const int64_t cn = a.n - c0 < chunk ? a.n - c0 : chunk;
    const int buf = k & 1;
    double* t = ws + (size_t)buf * chunk * per;
    const PfdArgs b = pfd_chunk(a, c0, cn);
    // buffer reuse: chunk k - 2's sweep (on st) has read this half
    if (k >= 2 && (e = hipStreamWaitEvent(side, ev[2 + buf], 0)) != hipSuccess) return e;
    hipLaunchKernelGGL(k_pfd_parts, dim3((unsigned)cn), dim3(256), ldsp, side, b, t);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = hipEventRecord(ev[buf], side)) != hipSuccess) return e;
    if ((e = hipStreamWaitEvent(st, ev[buf], 0)) != hipSuccess) return e;
    PfdArgs d = b;
    d.tin = t;
    hipLaunchKernelGGL(k_pfd_dmprof4, dim3((unsigned)cn), dim3(256), lds4, st, d);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = hipEventRecord(ev[2 + buf], st)) != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_pfd_dmprof(const PfdArgs& a, hipStream_t st) {
  if (pfd4_ok(a)) {
    const size_t lds4 = pfd4_lds_bytes(a.nsub, a.L);
    hipError_t e = ensure_dyn_lds<k_pfd_dmprof4>(lds4);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_pfd_dmprof4, dim3((unsigned)a.n), dim3(256), lds4, st, a);
    return hipGetLastError();
  }
  const size_t lds = pfd_lds_bytes(a.nsub, a.L);
  hipError_t e = ensure_dyn_lds<k_pfd_dmprof>(lds);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_pfd_dmprof, dim3((unsigned)a.n), dim3(64), lds, st, a);
  return hipGetLastError();
}

}  // namespace pfe
