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

#include "pfd.h"
#include "wave.h"

namespace pfe {

#pragma clang fp contract(off)

// ---- numpy pairwise summation ---------------------------------------------------------
// a leaf (n <= 128): r[j] = a[j] + a[j+8] + ... over the largest multiple of 8, combined as
// ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), then the remainder in order; n < 8: 0 + a0 + a1 ...
__device__ double np_leaf(const double* a, int n, int lane) {
  if (n < 8) {
    double r = 0.0;
    for (int i = 0; i < n; ++i) r += a[i];
    return r;
  }
  const int nb = n - (n % 8);
  double r = 0.0;
  if (lane < 8) {
    r = a[lane];
    for (int i = 8 + lane; i < nb; i += 8) r += a[i];
  }
  const double r0 = bcast(r, 0), r1 = bcast(r, 1), r2 = bcast(r, 2), r3 = bcast(r, 3);
  const double r4 = bcast(r, 4), r5 = bcast(r, 5), r6 = bcast(r, 6), r7 = bcast(r, 7);
  double res = ((r0 + r1) + (r2 + r3)) + ((r4 + r5) + (r6 + r7));
  for (int i = nb; i < n; ++i) res += a[i];
  return res;
}

template <int D>
__device__ __noinline__ double np_pairwise(const double* a, int n, int lane) {
  if (n <= 128) return np_leaf(a, n, lane);
  int n2 = n / 2;
  n2 -= n2 % 8;
  return np_pairwise<D - 1>(a, n2, lane) + np_pairwise<D - 1>(a + n2, n - n2, lane);
}
template <>
__device__ __noinline__ double np_pairwise<0>(const double* a, int n, int lane) {
  return np_leaf(a, n, lane);
}

// float32 pairwise sum of a short array (n <= 128), evaluated identically in every lane
__device__ float np_leaf_f32(const float* a, int n) {
  if (n < 8) {
    float r = 0.0f;
    for (int i = 0; i < n; ++i) r += a[i];
    return r;
  }
  const int nb = n - (n % 8);
  float r[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = a[j];
  for (int i = 8; i < nb; i += 8)
#pragma unroll
    for (int j = 0; j < 8; ++j) r[j] += a[i + j];
  float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  for (int i = nb; i < n; ++i) res += a[i];
  return res;
}

// Python's builtin min / max over a sequence (first element wins ties and NaN)
__device__ double py_min_seq(const double* a, int n) {
  double m = a[0];
  for (int i = 1; i < n; ++i)
    if (a[i] < m) m = a[i];
  return m;
}
__device__ double py_max_seq(const double* a, int n) {
  double m = a[0];
  for (int i = 1; i < n; ++i)
    if (a[i] > m) m = a[i];
  return m;
}

__device__ __forceinline__ int pymod(long long v, int m) {
  long long r = v % m;
  if (r < 0) r += m;
  return (int)r;
}

__device__ __forceinline__ double delay_from_dm(double dm, double f) {  // PFDOperations.py:474-488
  return f > 0.0 ? dm / (0.000241 * f * f) : 0.0;
}

__device__ __forceinline__ void lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// mean, std, skew, kurtosis of x[0..n) (LDS) as numpy.mean / numpy.std / scipy.stats.skew /
// scipy.stats.kurtosis compute them in float64; tmp: n doubles of LDS scratch
__device__ void stats4_f64(const double* x, double* tmp, int n, int lane, double (&o)[4]) {
  const double mean = np_pairwise<12>(x, n, lane) / (double)n;
  for (int i = lane; i < n; i += 64) {
    const double d = x[i] - mean;
    tmp[i] = d * d;
  }
  lds_sync();
  const double m2 = np_pairwise<12>(tmp, n, lane) / (double)n;
  lds_sync();
  for (int i = lane; i < n; i += 64) {
    const double d = x[i] - mean;
    tmp[i] = (d * d) * d;
  }
  lds_sync();
  const double m3 = np_pairwise<12>(tmp, n, lane) / (double)n;
  lds_sync();
  for (int i = lane; i < n; i += 64) {
    const double d = x[i] - mean;
    const double d2 = d * d;
    tmp[i] = d2 * d2;
  }
  lds_sync();
  const double m4 = np_pairwise<12>(tmp, n, lane) / (double)n;
  lds_sync();
  const double eps = 2.220446049250313e-16;
  const double zl = eps * mean;
  const bool zero = m2 <= zl * zl;
  o[0] = mean;
  o[1] = sqrt(m2);
  o[2] = zero ? NAN : m3 / pow(m2, 1.5);
  o[3] = zero ? NAN : m4 / (m2 * m2) - 3.0;
}

// the same in float32 (numpy on a float32 array), evaluated identically in every lane
__device__ void stats4_f32(const float* a, float* tmp, int n, double (&o)[4]) {
  const float mean = np_leaf_f32(a, n) / (float)n;
  for (int i = 0; i < n; ++i) {
    const float d = a[i] - mean;
    tmp[i] = d * d;
  }
  const float m2 = np_leaf_f32(tmp, n) / (float)n;
  for (int i = 0; i < n; ++i) {
    const float d = a[i] - mean;
    tmp[i] = (d * d) * d;
  }
  const float m3 = np_leaf_f32(tmp, n) / (float)n;
  for (int i = 0; i < n; ++i) {
    const float d = a[i] - mean;
    const float d2 = d * d;
    tmp[i] = d2 * d2;
  }
  const float m4 = np_leaf_f32(tmp, n) / (float)n;
  const float zl = 1.1920929e-07f * mean;
  const bool zero = m2 <= zl * zl;
  o[0] = (double)mean;
  o[1] = (double)sqrtf(m2);
  o[2] = zero ? NAN : (double)(m3 / powf(m2, 1.5f));
  o[3] = zero ? NAN : (double)(m4 / (m2 * m2) - 3.0f);
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
  int* cum = (int*)(sdb + NS);       // NS rotations applied since the dedispersion
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
    const double mn = py_min_seq(buf, L);
    for (int b = lane; b < L; b += 64) buf[b] = buf[b] - mn;  // normprof
    lds_sync();
    const double mean = np_pairwise<12>(buf, L, lane) / (double)L;
    lds_sync();
    for (int b = lane; b < L; b += 64) buf[b] = buf[b] / mean;  // s
    lds_sync();
    const double smin = py_min_seq(buf, L), smax = py_max_seq(buf, L);
    lds_sync();
    for (int b = lane; b < L; b += 64) {
      const double t = (buf[b] - smin) / (smax - smin);
      buf[b] = (0.0 * (1.0 - t)) + (255.0 * t);
      if (a.profile) a.profile[c * L + b] = buf[b];
    }
    lds_sync();
  }
  double po[4] = {0.0, 0.0, 0.0, 0.0};
  if (a.lyon8) stats4_f64(buf, tmp, L, lane, po);
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
  if (a.lyon8) {
    double dmo[4] = {0.0, 0.0, 0.0, 0.0};
    if (dm_ok) stats4_f32(chs, ftmp, PFE_PFD_NDM, dmo);
    if (lane == 0) {
      double* o = a.lyon8 + c * 8;
      for (int i = 0; i < 4; ++i) {
        o[i] = po[i];
        o[4 + i] = dm_ok ? dmo[i] : NAN;
      }
    }
  }
  if (lane == 0) a.status[c] = dm_ok ? 0u : PFE_ST_PFD_DMCURVE_FAIL;
}

size_t pfd_lds_bytes(int nsub, int L) {
  return ((size_t)nsub * L + 2 * (size_t)L + 2 * (size_t)nsub) * sizeof(double) +
         (size_t)nsub * sizeof(int) + 64;
}

hipError_t launch_pfd_dmprof(const PfdArgs& a, hipStream_t st) {
  const size_t lds = pfd_lds_bytes(a.nsub, a.L);
  static size_t configured = 0;
  if (lds > 48 * 1024 && lds > configured) {
    hipError_t e = hipFuncSetAttribute((const void*)k_pfd_dmprof,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    configured = lds;
  }
  hipLaunchKernelGGL(k_pfd_dmprof, dim3((unsigned)a.n), dim3(64), lds, st, a);
  return hipGetLastError();
}

}  // namespace pfe
