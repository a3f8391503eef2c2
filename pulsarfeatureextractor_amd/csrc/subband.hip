// subband.hip — scores 20-22: the sub-band scores of a candidate.
//
// Reference: PHCXOperations.getSubbandParameters (PHCXOperations.py:305-349), which calls
// ProfileOperations.getSubband_scores (ProfileOperations.py:1585-1686) and getProfileCorr
// (PHCXOperations.py:387-415):
//   s20  RMS scatter of the boxcar-maximum positions of the sub-bands, over the boxcar
//        width wb = int(ceil(width * nBins))                     (:1603-1659, :1678)
//   s21  mean numpy.corrcoef of every pair (i < k) of boxcar-sum vectors, NaN pairs
//        skipped, ZeroDivisionError when none is left            (:1663-1675)
//   s22  sum of |corrcoef(sub-band j, profile)| over the values > 0.0055 (:403-415, :345-347)
//
// Design (one wave per candidate; nsub 2-256, nBins up to 1024 on chip, any other shape up
// to 65536 x 16384 through k_subband_g and global scratch):
//   * The candidate's nsub x lsb sub-band bytes are read once (16 B per lane, coalesced) and
//     turned into per-band exclusive prefix sums E[i][t] = sum_{u<t} x[i][u] in LDS (u16 up
//     to 256 bins, else u32): a 16-byte piece is prefixed in the lane with v_dot4, the
//     pieces of one band by a segmented lane scan.  Every boxcar sum is then
//     b[i][j] = E[i][j+wb] - E[i][j] (two LDS reads) and every raw byte E[i][j+1] - E[i][j].
//   * s20 and the maxima are integer-exact: the first strict maximum over j is the maximum
//     of the 32-bit key (b << 10) | (1023 - j).
//   * s21 without the nsub^2 pair loop: the boxcar sums are integers, so per band
//     S = sum b and N = nw * sum b^2 - S^2 are exact, and z = (nw b - S) / sqrt(nw N) has
//     <z_i, z_k> = corrcoef(b_i, b_k) (zero-variance bands, the reference's NaN pairs, are
//     left out: N = 0 exactly when numpy's variance is 0).  Hence
//         sum_{i<k} cc_ik = (sum_j (sum_i z_ij)^2 - sum_i |z_i|^2) / 2,
//     over the m = v(v-1)/2 pairs of the v valid bands: O(nsub nw) work instead of
//     O(nsub^2 nw).  It equals numpy's pair loop to rounding (~1e-15 relative; the parity
//     bar for s21 is 1e-5).
//   * s22 keeps numpy's arithmetic: centred fp64 values, per-lane partials over the slots in
//     order and the fixed butterfly (wsum), which is bit-identical to the reference's
//     corrcoef at 64/128/256 bins.
#include <hip/hip_runtime.h>

#include <cmath>
#include <type_traits>

#include "../../include/pfe.h"
#include "bates_common.h"
#include "wave.h"

namespace pfe {

struct SubArgs {
  const uint8_t* prof;  // n x lp
  int lp;
  const uint8_t* sub;   // n x nsub x lsb
  int nsub, lsb;
  const double* scal;   // n x PFE_NSCAL (width at PFE_SCAL_WIDTH)
  int64_t n;
  double* out;          // scores 20-22 of candidate c at out[c * ldo + 0..2]
  int ldo;
  uint32_t* status;
};

constexpr int SB_NB = 16;  // bands per register block
constexpr int SB_PK_WB = 32;  // widest boxcar of the fast kernel's packed pass 1
typedef unsigned short us2v __attribute__((ext_vector_type(2)));

// LDS row stride (elements) of the prefix array: 16-B aligned rows of lsb + 1 entries
template <typename PT>
__host__ __device__ constexpr int sb_stride(int lsb) {
  return sizeof(PT) == 2 ? ((lsb + 1 + 7) & ~7) : ((lsb + 1 + 3) & ~3);
}
template <typename PT>
__host__ __device__ constexpr size_t sb_wave_lds(int nsub, int lsb) {
  return ((size_t)nsub * sb_stride<PT>(lsb) * sizeof(PT) + 15) / 16 * 16 + ((size_t)nsub * 4 + 15) / 16 * 16;
}

// 16 bytes -> their 16 exclusive prefixes (packed into the 8/16 dwords of a PT row piece)
// plus the piece total
__device__ __forceinline__ uint32_t piece_prefix(const uint32_t (&w)[4], uint32_t (&e)[16]) {
  uint32_t run = 0;
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const uint32_t x = w[d];
    e[4 * d + 0] = run;
    e[4 * d + 1] = run + __builtin_amdgcn_udot4(x, 0x00000001u, 0u, false);
    e[4 * d + 2] = run + __builtin_amdgcn_udot4(x, 0x00000101u, 0u, false);
    e[4 * d + 3] = run + __builtin_amdgcn_udot4(x, 0x00010101u, 0u, false);
    run += __builtin_amdgcn_udot4(x, 0x01010101u, 0u, false);
  }
  return run;
}

// Fill E (this wave's prefix rows) for the fast layout: lsb a power of two in [16, 1024] and a
// 16-B aligned block: pieces of 16 bytes never cross a band, a band is seg = lsb/16 lanes.
template <typename PT>
__device__ __forceinline__ void fill_prefix_fast(const uint8_t* sb, int nsub, int lsb, PT* E, int lane) {
  const int stride = sb_stride<PT>(lsb);
  const int seg = lsb >= 1024 ? 64 : lsb / 16;
  const int64_t total = (int64_t)nsub * lsb;
  for (int64_t base = 0; base < total; base += 1024) {
    const int64_t off = base + 16 * lane;
    const bool ok = off < total;
    uint32_t w[4] = {0, 0, 0, 0};
    if (ok) {
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(sb + off));
      w[0] = v.x;
      w[1] = v.y;
      w[2] = v.z;
      w[3] = v.w;
    }
    uint32_t e[16];
    const uint32_t tot = piece_prefix(w, e);
    // exclusive scan of the piece totals inside the band's lane segment
    uint32_t x = tot;
    const int pos = lane & (seg - 1);
#pragma unroll
    for (int s = 1; s < 64; s <<= 1) {
      if (s >= seg) break;
      const uint32_t o = (uint32_t)__shfl_up((int)x, s);
      if (pos >= s) x += o;
    }
    const uint32_t excl = x - tot;
    if (ok) {
      const int band = (int)(off / lsb);
      const int t0 = (int)(off - (int64_t)band * lsb);
      PT* row = E + (size_t)band * stride + t0;
      if constexpr (sizeof(PT) == 2) {
        uint32_t pk[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) pk[q] = ((e[2 * q] + excl) & 0xFFFFu) | ((e[2 * q + 1] + excl) << 16);
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        reinterpret_cast<u32x4*>(row)[0] = (u32x4){pk[0], pk[1], pk[2], pk[3]};
        reinterpret_cast<u32x4*>(row)[1] = (u32x4){pk[4], pk[5], pk[6], pk[7]};
      } else {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
        for (int q = 0; q < 4; ++q)
          reinterpret_cast<u32x4*>(row)[q] =
              (u32x4){e[4 * q] + excl, e[4 * q + 1] + excl, e[4 * q + 2] + excl, e[4 * q + 3] + excl};
      }
      if (t0 + 16 == lsb) row[16] = (PT)(excl + tot);  // E[band][lsb]
    }
  }
}

// Fill E for any lsb / alignment: one band at a time, ceil(lsb/64) contiguous bytes per lane.
template <typename PT>
__device__ __forceinline__ void fill_prefix_generic(const uint8_t* sb, int nsub, int lsb, PT* E, int lane) {
  const int stride = sb_stride<PT>(lsb);
  const int ch = (lsb + 63) / 64;
  for (int i = 0; i < nsub; ++i) {
    const uint8_t* src = sb + (size_t)i * lsb;
    const int t0 = lane * ch;
    uint32_t run = 0;
    for (int u = 0; u < ch; ++u)
      if (t0 + u < lsb) run += src[t0 + u];
    const uint32_t excl = (uint32_t)wscan_excl((int)run);
    PT* row = E + (size_t)i * stride;
    uint32_t acc = excl;
    for (int u = 0; u < ch; ++u)
      if (t0 + u < lsb) {
        row[t0 + u] = (PT)acc;
        acc += src[t0 + u];
      }
    if (t0 < lsb && t0 + ch >= lsb) row[lsb] = (PT)acc;
  }
}

// numpy.corrcoef's off-diagonal entry from the centred sums (clip keeps NaN)
__device__ __forceinline__ double sb_corr(double cxy, double cxx, double cyy) {
  double r = (cxy / sqrt(cxx)) / sqrt(cyy);
  if (r > 1.0) r = 1.0;
  if (r < -1.0) r = -1.0;
  return r;
}

// s20: RMS scatter of the boxcar-maximum positions (:1633-1659, :1678); wave-uniform
__device__ __forceinline__ double rms_of_maxbins(const int* maxbin, int nsub, int wb) {
  double msum = 0.0;
  for (int i = 0; i < nsub; ++i) msum += (double)maxbin[i];
  const double med = msum / (double)nsub;
  int count = 0;
  double var_med = 0.0;
  for (int i = 0; i < nsub; ++i) {
    const double v = (double)maxbin[i];
    if (fabs(v - med) <= (double)wb) {
      ++count;
      var_med += (v - med) * (v - med);
    }
  }
  double var;
  if (count > 1) {
    var = var_med / (double)(count - 1);
  } else {
    double mu = 0.0;
    for (int i = 0; i < nsub; ++i) mu += (double)maxbin[i];
    mu /= (double)nsub;
    var = 0.0;
    for (int i = 0; i < nsub; ++i) var += ((double)maxbin[i] - mu) * ((double)maxbin[i] - mu);
    var /= (double)(nsub - 1);
  }
  return sqrt(var) / (double)wb;
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// acc + v(lane 0) + v(lane 1) + ... + v(lane cnt-1), left to right (a reference loop's order),
// through a 64-double LDS scratch: every lane reads the same 16 B (a broadcast), so each term
// costs one v_add_f64 instead of two v_readlane and an add
__device__ __forceinline__ double fold_lanes(double acc, double v, int cnt, double* scratch) {
  scratch[lane_id()] = v;
  wave_lds_sync();
  int t = 0;
  for (; t + 2 <= cnt; t += 2) {
    const double2 p = *reinterpret_cast<const double2*>(scratch + t);
    acc += p.x;
    acc += p.y;
  }
  if (t < cnt) acc += scratch[t];
  wave_lds_sync();
  return acc;
}

// rms_of_maxbins with band i in lane i % 64 (chunks of 64 bands), the same bits: the means are
// sums of integers (exact in any order), the two sums of squares are folded in band order, and
// a band outside |v - med| <= wb adds +0.0 to a non-negative sum, which leaves its bits alone
__device__ __forceinline__ double rms_of_maxbins_wave(const int* maxbin, int nsub, int wb, double* scratch) {
  const int lane = lane_id();
  int isum = 0;
  for (int i0 = 0; i0 < nsub; i0 += 64) isum += i0 + lane < nsub ? maxbin[i0 + lane] : 0;
  isum = wsum_i(isum);  // <= 65536 bands x 17 bits: no overflow
  const double msum = (double)isum;
  const double med = msum / (double)nsub;
  int count = 0;
  double var_med = 0.0;
  for (int i0 = 0; i0 < nsub; i0 += 64) {
    const int cnt = nsub - i0 < 64 ? nsub - i0 : 64;
    const double v = lane < cnt ? (double)maxbin[i0 + lane] : 0.0;
    const bool in = lane < cnt && fabs(v - med) <= (double)wb;
    count += __builtin_popcountll(__ballot(in));
    var_med = fold_lanes(var_med, in ? (v - med) * (v - med) : 0.0, cnt, scratch);
  }
  double var;
  if (count > 1) {
    var = var_med / (double)(count - 1);
  } else {
    const double mu = msum / (double)nsub;
    var = 0.0;
    for (int i0 = 0; i0 < nsub; i0 += 64) {
      const int cnt = nsub - i0 < 64 ? nsub - i0 : 64;
      const double v = lane < cnt ? (double)maxbin[i0 + lane] : 0.0;
      var = fold_lanes(var, (v - mu) * (v - mu), cnt, scratch);
    }
    var /= (double)(nsub - 1);
  }
  return sqrt(var) / (double)wb;
}

// SL = ceil(lsb / 64) window / bin slots per lane; WPB waves (candidates) per block
template <int SL, typename PT, int WPB>
__global__ __launch_bounds__(64 * WPB) void k_subband2(SubArgs a) {
  extern __shared__ __align__(16) unsigned char sb_lds[];
  const int lane = lane_id();
  const int w = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * WPB + w;
  if (c >= a.n) return;
  const int nsub = a.nsub, lsb = a.lsb;
  const size_t wave_bytes = sb_wave_lds<PT>(nsub, lsb);
  PT* E = reinterpret_cast<PT*>(sb_lds + w * wave_bytes);
  int* maxbin = reinterpret_cast<int*>(sb_lds + w * wave_bytes +
                                       ((size_t)nsub * sb_stride<PT>(lsb) * sizeof(PT) + 15) / 16 * 16);
  const int stride = sb_stride<PT>(lsb);

  const double width = a.scal[c * PFE_NSCAL + PFE_SCAL_WIDTH];
  const double wbd = ceil(width * (double)lsb);                      // :1603
  // wb <= 0: rms = stdev / 0 or no valid pair; wb > lsb: no window, max_bin unbound;
  // lp != lsb: corrcoef of different lengths raises (:403)
  if (!(wbd >= 1.0) || wbd > (double)lsb || a.lp != lsb) {
    if (lane == 0) atomicOr(&a.status[c], PFE_ST_SUBBAND_FAIL);
    return;
  }
  const int wb = (int)wbd;
  const int nw = lsb - wb + 1;                                        // windows per band
  const uint8_t* sb = a.sub + c * (int64_t)nsub * lsb;
  const bool fast = ((lsb & (lsb - 1)) == 0) && lsb >= 16 && (((uintptr_t)sb & 15) == 0);
  if (fast)
    fill_prefix_fast<PT>(sb, nsub, lsb, E, lane);
  else
    fill_prefix_generic<PT>(sb, nsub, lsb, E, lane);
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

  // the profile, centred as numpy.corrcoef centres it (s22)
  double pv[SL];
  double pm = 0.0;
#pragma unroll
  for (int k = 0; k < SL; ++k) {
    const int j = lane + 64 * k;
    pv[k] = (j < lsb) ? (double)a.prof[c * a.lp + j] : 0.0;
    pm += pv[k];
  }
  pm = wsum(pm) / (double)lsb;
  double pvar = 0.0;
#pragma unroll
  for (int k = 0; k < SL; ++k) {
    pv[k] = (lane + 64 * k < lsb) ? pv[k] - pm : 0.0;
    pvar += pv[k] * pv[k];
  }
  pvar = wsum(pvar);
  const double inv2 = 1.0 / (double)(lsb - 1);

  const double dnw = (double)nw;
  double Z[SL];      // sum over the valid bands of z_ij, window j = lane + 64k
#pragma unroll
  for (int k = 0; k < SL; ++k) Z[k] = 0.0;
  double zz = 0.0;   // sum of z_ij^2
  int valid = 0;     // bands with non-zero variance
  double integ = 0.0;

  for (int blk = 0; blk < nsub; blk += SB_NB) {
    const int nb = nsub - blk < SB_NB ? nsub - blk : SB_NB;
    // ---- boxcar statistics: S, sum b^2, first strict maximum -------------------------
    long long S[SB_NB], Q[SB_NB];
    int key[SB_NB];
#pragma unroll
    for (int ii = 0; ii < SB_NB; ++ii) {
      long long s = 0, q = 0;
      int kmax = 0;
      if (ii < nb) {
        const PT* row = E + (size_t)(blk + ii) * stride;
#pragma unroll
        for (int k = 0; k < SL; ++k) {
          const int j = lane + 64 * k;
          if (j < nw) {
            const int b = (int)row[j + wb] - (int)row[j];
            s += b;
            q += (long long)b * b;
            const int kk = (b << 10) | (1023 - j);
            kmax = kk > kmax ? kk : kmax;
          }
        }
      }
      S[ii] = s;
      Q[ii] = q;
      key[ii] = kmax;
    }
#pragma unroll
    for (int ii = 0; ii < SB_NB; ++ii) {
      S[ii] = wsum_ll(S[ii]);
      Q[ii] = wsum_ll(Q[ii]);
      key[ii] = wmax_i(key[ii]);
    }
    double r[SB_NB];
#pragma unroll
    for (int ii = 0; ii < SB_NB; ++ii) {
      const long long N = (long long)nw * Q[ii] - S[ii] * S[ii];  // exact: nw^2 var(b)
      r[ii] = (ii < nb && N > 0) ? 1.0 / sqrt(dnw * (double)N) : 0.0;
      valid += (ii < nb && N > 0) ? 1 : 0;
      if (ii < nb && lane == 0) maxbin[blk + ii] = 1023 - (key[ii] & 1023) + wb / 2;  // :1628
    }
    // ---- z-scores of the valid bands; centred bytes against the profile ---------------
    double sv[SB_NB], d[SB_NB];
#pragma unroll
    for (int ii = 0; ii < SB_NB; ++ii) {
      int bs = 0;
      if (ii < nb) {
        const PT* row = E + (size_t)(blk + ii) * stride;
        bs = (int)row[lsb];
#pragma unroll
        for (int k = 0; k < SL; ++k) {
          const int j = lane + 64 * k;
          if (j < nw && r[ii] != 0.0) {
            const int b = (int)row[j + wb] - (int)row[j];
            const double z = (double)((long long)nw * b - S[ii]) * r[ii];
            Z[k] += z;
            zz += z * z;
          }
        }
      }
      // numpy: mu = mean(sub_j); t = sub_j - mu; d = sum t * pv; q = sum t^2 (per-lane slots
      // in order, then the fixed butterfly)
      const double mu = (double)bs / (double)lsb;
      double dd = 0.0, q = 0.0;
      if (ii < nb) {
        const PT* row = E + (size_t)(blk + ii) * stride;
#pragma unroll
        for (int k = 0; k < SL; ++k) {
          const int j = lane + 64 * k;
          if (j < lsb) {
            const double t = (double)((int)row[j + 1] - (int)row[j]) - mu;
            dd += t * pv[k];
            q += t * t;
          }
        }
      }
      sv[ii] = q;
      d[ii] = dd;
    }
    wsum_arr(sv);
    wsum_arr(d);
#pragma unroll
    for (int ii = 0; ii < SB_NB; ++ii) {
      if (ii < nb) {
        const double cc = fabs(sb_corr(d[ii] * inv2, sv[ii] * inv2, pvar * inv2));
        if (cc > 0.0055) integ += cc;                                 // in band order
      }
    }
  }
  // ---- s21 -----------------------------------------------------------------------------
  double zs = 0.0;
#pragma unroll
  for (int k = 0; k < SL; ++k) zs += Z[k] * Z[k];
  zs = wsum(zs);
  zz = wsum(zz);
  const long long m = (long long)valid * (valid - 1) / 2;
  if (m == 0) {  // ZeroDivisionError (:1681)
    if (lane == 0) atomicOr(&a.status[c], PFE_ST_SUBBAND_FAIL);
    return;
  }
  const double mean_corr = (0.5 * (zs - zz)) / (double)m;
  // ---- s20 ------------------------------------------------------------------------------
  wave_lds_sync();
  const double rms = rms_of_maxbins(maxbin, nsub, wb);
  if (lane == 0) {
    double* o = a.out + c * a.ldo;
    o[0] = rms;
    o[1] = mean_corr;
    o[2] = integ;
  }
}

// ---- fast path: power-of-two nBins in [16, 256], 16-B aligned rows ---------------------
// Every sum the three scores need is an exact integer here, so the kernel works in integers
// and packed byte dot products and still returns numpy's bits:
//   * s22: with L a power of two, mu = T/L and pm = P/L are exact, every centred product
//     (x - mu)(p - pm) = (Lx - T)(Lp - P)/L^2 is exact and so is every partial sum, whatever
//     the order -- numpy's d = sum (x-mu)(p-pm) equals (L XP - T P)/L exactly, with
//     XP = sum x p, T = sum x, P = sum p (likewise sum (x-mu)^2 and the profile's): three
//     v_dot4 sums per 16-byte piece, taken in the same pass that builds the prefix sums;
//   * s20 / s21 in two passes over each block of 16 bands (round 5): pass 1 puts a band in
//     each lane (16 bands x 4 quarter lanes), so S = sum b, sum b^2 and the first maximum of
//     a band need two cross-lane steps; pass 2 (lane = window) forms the s21 identity of
//     k_subband2, W_j = sum_i r_i b_ij in band order, by fma;
//   * no masks in either pass: the prefix rows are padded with zero rows to a multiple of 16
//     bands and carry a zero tail; a pass-1 window past the last one reads the tail (its
//     saturated difference is 0), a pass-2 window reads the same prefix twice, so its boxcar
//     sum is 0 and its key (0 << 10 | 1023 - j) loses to every real window (smaller j).
__host__ __device__ constexpr int sb_pad16(int nsub) { return (nsub + 15) & ~15; }
// the fast kernel's u16 row pitch: lsb + 1 prefixes and a zero tail to lsb + 31 (read by the
// band-per-lane pass past the last window), 16-B aligned rows, and a pitch of 4 x odd dwords so
// that the 16 bands of a block read by one row of lanes land in 16 distinct bank groups
__host__ __device__ constexpr int sb_stride_fast(int lsb) {
  return ((lsb + 32 + 15) & ~15) + 8;  // = 8 (mod 16)
}
template <int LSB>
__host__ __device__ constexpr size_t fast_wave_lds(int nsub) {
  return ((size_t)sb_pad16(nsub) * sb_stride_fast(LSB) * 2 + 15) / 16 * 16 +
         ((size_t)nsub * 4 * sizeof(int) + 15) / 16 * 16 + 64 * sizeof(double);
}

// inclusive scan of x over the SEG-lane segments of a DPP row (SEG <= 16): row_shr reads
// 0 from outside the row, the select keeps a segment's scan inside it
template <int SEG>
__device__ __forceinline__ uint32_t seg_scan_incl(uint32_t x, int pos) {
  if constexpr (SEG >= 2) {
    const uint32_t o = (uint32_t)dpp_i32<0x111>((int)x);  // row_shr:1
    x += (SEG == 16 || pos >= 1) ? o : 0u;
  }
  if constexpr (SEG >= 4) {
    const uint32_t o = (uint32_t)dpp_i32<0x112>((int)x);  // row_shr:2
    x += (SEG == 16 || pos >= 2) ? o : 0u;
  }
  if constexpr (SEG >= 8) {
    const uint32_t o = (uint32_t)dpp_i32<0x114>((int)x);  // row_shr:4
    x += (SEG == 16 || pos >= 4) ? o : 0u;
  }
  if constexpr (SEG >= 16) x += (uint32_t)dpp_i32<0x118>((int)x);  // row_shr:8
  return x;
}

template <int M>
__device__ __forceinline__ int xor_i32(int v) {
  if constexpr (M == 1)
    return dpp_i32<DPP_QUAD_XOR1>(v);
  else if constexpr (M == 2)
    return dpp_i32<DPP_QUAD_XOR2>(v);
  else
    return __shfl_xor(v, M);
}
template <int M>
__device__ __forceinline__ unsigned long long xor_u64(unsigned long long v) {
  const int lo = xor_i32<M>((int)(uint32_t)v);
  const int hi = xor_i32<M>((int)(uint32_t)(v >> 32));
  return ((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo;
}
#ifndef PFE_SUBBAND_WPE
#define PFE_SUBBAND_WPE 3  // register cap (168 VGPRs); the two-pass kernel uses 64-74
#endif
template <int LSB, int WPB>
__global__ __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(PFE_SUBBAND_WPE)))
void k_subband_fast(SubArgs a) {
  constexpr int SL = LSB >= 64 ? LSB / 64 : 1;  // window slots per lane
  constexpr int SEG = LSB / 16;                 // lanes per band in the 16-byte piece layout
  constexpr int STRIDE = sb_stride_fast(LSB);
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  extern __shared__ __align__(16) unsigned char sb_lds[];
  const int lane = lane_id();
  // the wave's candidate, and everything derived from it, in scalar registers
  const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t c = (int64_t)blockIdx.x * WPB + w;
  if (c >= a.n) return;
  const int nsub = a.nsub;
  const int npad = sb_pad16(nsub);
  unsigned char* wbase = sb_lds + w * fast_wave_lds<LSB>(nsub);
  uint16_t* E = reinterpret_cast<uint16_t*>(wbase);
  int* bstat = reinterpret_cast<int*>(wbase + ((size_t)npad * STRIDE * 2 + 15) / 16 * 16);
  int* maxbin = bstat + 3 * nsub;
  double* fold = reinterpret_cast<double*>(reinterpret_cast<unsigned char*>(bstat) +
                                           ((size_t)nsub * 4 * sizeof(int) + 15) / 16 * 16);

  const double width = a.scal[c * PFE_NSCAL + PFE_SCAL_WIDTH];
  const double wbd = ceil(width * (double)LSB);                      // :1603
  if (!(wbd >= 1.0) || wbd > (double)LSB || a.lp != LSB) {
    if (lane == 0) atomicOr(&a.status[c], PFE_ST_SUBBAND_FAIL);
    return;
  }
  const int wb = __builtin_amdgcn_readfirstlane((int)wbd);
  const int nw = LSB - wb + 1;
  const uint8_t* sb = a.sub + c * (int64_t)nsub * LSB;
  const int pos = lane & (SEG - 1);
  // zero rows after the last band (read by the window loop's partial last block)
  for (int t = nsub * STRIDE / 8 + lane; t < npad * STRIDE / 8; t += 64)
    reinterpret_cast<uint32_t __attribute__((ext_vector_type(4)))*>(E)[t] =
        (uint32_t __attribute__((ext_vector_type(4)))){0, 0, 0, 0};
  // the zero tails E[band][LSB .. LSB + 31] of the real bands, 64 B each (the prefix pass
  // then stores E[band][LSB] = T): one 16-B store per lane per 16 bands
  for (int t = lane; t < nsub * 4; t += 64)
    reinterpret_cast<u32x4*>(E + (t >> 2) * STRIDE + LSB)[t & 3] = (u32x4){0, 0, 0, 0};
  // this lane's 16 profile bytes (a piece sits at the same offset of its band every pass)
  uint32_t pw[4];
  {
    const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(a.prof + c * LSB + 16 * pos));
    pw[0] = v.x;
    pw[1] = v.y;
    pw[2] = v.z;
    pw[3] = v.w;
  }
  int P = 0, P2 = 0;
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    P = (int)__builtin_amdgcn_udot4(pw[d], 0x01010101u, (uint32_t)P, false);
    P2 = (int)__builtin_amdgcn_udot4(pw[d], pw[d], (uint32_t)P2, false);
  }
  P = group_sum_i32<SEG>(P);
  P2 = group_sum_i32<SEG>(P2);

  // ---- prefix sums and the s22 sums, four 1 KiB passes per load burst ---------------------
  const int total = nsub * LSB;
  for (int base = 0; base < total; base += 4096) {
    u32x4 q[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int off = base + 1024 * u + 16 * lane;
      q[u] = off < total ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(sb + off))
                         : (u32x4){0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int off = base + 1024 * u + 16 * lane;
      if (base + 1024 * u >= total) break;  // wave-uniform
      const uint32_t wv[4] = {q[u].x, q[u].y, q[u].z, q[u].w};
      // the piece total first, then the 16 prefixes as one running chain of byte adds from
      // the band offset (a v_dot4 issues at about a quarter of the rate of an add on gfx950,
      // profiles/r04_ubench_op_rates.txt); each u16 pair is one v_lshl_or (every E of a band
      // is < 2^16 at <= 256 bins, so no carry crosses the halves)
      uint32_t tot = 0;
#pragma unroll
      for (int d = 0; d < 4; ++d) tot = __builtin_amdgcn_sad_u8(wv[d], 0u, tot);
      uint32_t e = seg_scan_incl<SEG>(tot, pos) - tot;
      uint32_t pk[8];
#ifndef PFE_SB_NOSDWA
      // the chain straight into the packed u16 pairs, one SDWA add per prefix: WORD_1 of a
      // pair = its WORD_0 + the next byte (the low half kept), WORD_0 of the next pair = the
      // previous WORD_1 + the byte after (the high half zeroed) -- 16 adds per 16 bytes, no
      // shifts or ors (every prefix is < 2^16 at <= 256 bins, so a half holds it exactly)
      const uint32_t excl = e;
      {
        uint32_t c = e;  // WORD_0 = the running prefix, WORD_1 = 0
#pragma unroll
        for (int d = 0; d < 4; ++d) {
          const uint32_t x = wv[d];
          uint32_t n;
          asm("v_add_u32_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:BYTE_0"
              : "+v"(c) : "v"(x));
          asm("v_add_u32_sdwa %0, %1, %2 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:BYTE_1"
              : "=v"(n) : "v"(c), "v"(x));
          asm("v_add_u32_sdwa %0, %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0 src1_sel:BYTE_2"
              : "+v"(n) : "v"(x));
          pk[2 * d] = c;
          pk[2 * d + 1] = n;
          asm("v_add_u32_sdwa %0, %1, %2 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:BYTE_3"
              : "=v"(c) : "v"(n), "v"(x));
        }
      }
#else
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const uint32_t x = wv[d];
        const uint32_t e0 = e;
        const uint32_t e1 = e0 + (x & 0xFFu);
        const uint32_t e2 = e1 + ((x >> 8) & 0xFFu);
        const uint32_t e3 = e2 + ((x >> 16) & 0xFFu);
        e = e3 + (x >> 24);
        pk[2 * d] = e0 | (e1 << 16);
        pk[2 * d + 1] = e2 | (e3 << 16);
      }
      const uint32_t excl = e - tot;
#endif
      int X2 = 0, XP = 0;
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        X2 = (int)__builtin_amdgcn_udot4(wv[d], wv[d], (uint32_t)X2, false);
        XP = (int)__builtin_amdgcn_udot4(wv[d], pw[d], (uint32_t)XP, false);
      }
      X2 = group_sum_i32<SEG>(X2);
      XP = group_sum_i32<SEG>(XP);
      if (off < total) {
        const int band = off / LSB;
        uint16_t* row = E + band * STRIDE + 16 * pos;
#if !defined(PFE_SB_NOSWZ) && !defined(PFE_SB_NOSWZ_ST)
        // a lane's 32 B go out as two 16-B stores; ds_write_b128 banks (dword mod 32) over 8
        // contiguous lanes, and lanes pos and pos + 4 (32 B apart) would hit the same 4 banks
        // if both stored their low half first: the upper four lanes of each eight store their
        // halves in the other order (2-way conflicts -> none, same bytes)
        const bool sw = (pos & 4) != 0;
        reinterpret_cast<u32x4*>(row)[sw ? 1 : 0] =
            sw ? (u32x4){pk[4], pk[5], pk[6], pk[7]} : (u32x4){pk[0], pk[1], pk[2], pk[3]};
        reinterpret_cast<u32x4*>(row)[sw ? 0 : 1] =
            sw ? (u32x4){pk[0], pk[1], pk[2], pk[3]} : (u32x4){pk[4], pk[5], pk[6], pk[7]};
#else
        reinterpret_cast<u32x4*>(row)[0] = (u32x4){pk[0], pk[1], pk[2], pk[3]};
        reinterpret_cast<u32x4*>(row)[1] = (u32x4){pk[4], pk[5], pk[6], pk[7]};
#endif
        if (pos == SEG - 1) {
          row[16] = (uint16_t)(excl + tot);  // E[band][LSB] = T (in the zeroed tail)
          bstat[3 * band + 0] = (int)(excl + tot);
          bstat[3 * band + 1] = X2;
          bstat[3 * band + 2] = XP;
        }
      }
    }
  }
  wave_lds_sync();

  // ---- s22: one band per lane, then the reference's sum in band order -----------------------
  const double inv2 = 1.0 / (double)(LSB - 1);
  const double pvar = (double)((long long)LSB * P2 - (long long)P * P) / (double)LSB;
  double integ = 0.0;
  for (int i0 = 0; i0 < nsub; i0 += 64) {
    double v = 0.0;
    const int i = i0 + lane;
    if (i < nsub) {
      const int T = bstat[3 * i], X2 = bstat[3 * i + 1], XP = bstat[3 * i + 2];
      const double d = (double)((long long)LSB * XP - (long long)T * P) / (double)LSB;
      const double q2 = (double)((long long)LSB * X2 - (long long)T * T) / (double)LSB;
      const double cc = fabs(sb_corr(d * inv2, q2 * inv2, pvar * inv2));
      v = cc > 0.0055 ? cc : 0.0;  // adding 0.0 leaves the running sum's bits unchanged
    }
    integ = fold_lanes(integ, v, nsub - i0 < 64 ? nsub - i0 : 64, fold);
  }

  // ---- s20 / s21 over blocks of 16 bands --------------------------------------------------
  const double dnw = (double)nw;
  double W[SL];
#pragma unroll
  for (int k = 0; k < SL; ++k) W[k] = 0.0;
  uint32_t zh[SL];  // held zeros: the high halves of pass 2's denormal byte-sum operands
#pragma unroll
  for (int k = 0; k < SL; ++k) {
    zh[k] = 0u;
    asm volatile("" : "+v"(zh[k]));
  }
  double C = 0.0;
  int valid = 0;
  // pass 2's window slots (lane = window): the prefix indices, band-independent (a window
  // past the last one reads E[lo] twice: b = 0)
  int lo_k[SL], hi_k[SL];
#pragma unroll
  for (int k = 0; k < SL; ++k) {
    const int j = lane + 64 * k;
    lo_k[k] = j < LSB ? j : LSB;
    hi_k[k] = j < nw ? j + wb : lo_k[k];
  }
  // pass 1's layout (lane = band): band bi of the block; its quarter lane qtr takes the windows
  // j = 8s + 2 qtr + p (step u = 2s + p), so at every step the four quarter lanes of a band
  // read four distinct dwords and the 64 lanes 64 distinct banks (the row pitch is 4 x odd
  // dwords); the steps run in chunks of 4 (skipped past the last window), and a window
  // j >= nw of the last chunk reads E[j + wb] from the zero tail of its row (indices up to
  // lsb + 22), so its saturated difference is 0: no masks
#ifndef PFE_SB_NOSWZ
  // u16 reads bank on (dword mod 32) per 32-lane half: with a row pitch of 4 x odd dwords,
  // bands bi and bi + 8 start on the same bank, so the half's two quarter lanes of each band
  // would collide 2-way; bands 8-15 take the quarters in the order 2, 3, 0, 1, which puts the
  // 32 lanes of a half on 32 distinct dwords (the four quarter lanes of a band still cover
  // every window once; sums and maxima are order-free integers: the same results)
  const int bi = lane & 15, qtr = (lane >> 4) ^ ((bi >> 3) << 1);
#else
  const int bi = lane & 15, qtr = lane >> 4;
#endif
  const int U = 2 * ((nw + 7) >> 3);
  constexpr int NCH = (LSB / 4 + 3) / 4;
  for (int blk = 0; blk < nsub; blk += SB_NB) {
    const int nb = nsub - blk < SB_NB ? nsub - blk : SB_NB;
    const uint16_t* rows = E + blk * STRIDE;  // bands past nsub are the zero rows
    // ---- pass 1: S = sum b, sum b^2 and the first maximum of each band -------------------
    const uint16_t* plo = rows + bi * STRIDE + 2 * qtr;
    const uint16_t* phi = plo + wb;
    int sv = 0, key = 0;
    unsigned long long qv = 0;
#ifndef PFE_SB_NOPK
    if (wb <= SB_PK_WB) {
      // packed: the lane's two windows of a step pair s, j = 8s + 2 qtr + {0, 1}, as the u16
      // halves of one register: (E[j], E[j + 1]) is an aligned dword (j even), and so is
      // (E[j + wb], E[j + 1 + wb]) for an even wb (an odd one takes the two dwords around it,
      // joined by one v_alignbit).  Per pair: one saturating v_pk_sub_u16 (b of both windows),
      // two v_dot2_u32_u16 (S, sum b^2) and a v_lshl_or + v_pk_max_u16 for the maxima -- 5
      // VALU for two windows instead of 7 for one.  Exact while wb <= 32: b <= 255 wb < 2^13,
      // so (b << 3) | step fits a half, and a lane's <= 64 squares stay below 2^32.
      int sq = 0;
      const uint32_t* dlo = reinterpret_cast<const uint32_t*>(plo);
      const uint32_t* dhi = reinterpret_cast<const uint32_t*>(plo + (wb & ~1));
      const int S2 = (U >> 1);  // step pairs (ceil(nw / 8))
      // IB bits of step index per key half: chunks of 2^IB step pairs, folded to the band key
      // once per chunk; b < 2^(16 - IB), so IB = 4 (half the folds) for wb <= 16
      auto pairs = [&](auto odd_c, auto ib_c) {
        constexpr bool ODD = decltype(odd_c)::value;
        constexpr int IB = decltype(ib_c)::value, CP = 1 << IB;
#pragma unroll
        for (int g = 0; g < (2 * NCH + CP - 1) / CP; ++g) {
          if (CP * g < S2) {  // wave-uniform
            uint32_t km = 0;
#pragma unroll
            for (int t = 0; t < CP; t += 2) {
              if (t > 0 && CP * g + t >= S2) break;  // wave-uniform, two pairs at a time
#pragma unroll
              for (int e = 0; e < 2; ++e) {
                const int sp = CP * g + t + e;
                const uint32_t lo = dlo[4 * sp];
                const uint32_t hi = ODD ? __builtin_amdgcn_alignbit(dhi[4 * sp + 1], dhi[4 * sp], 16)
                                        : dhi[4 * sp];
                const us2v b2 = __builtin_elementwise_sub_sat(__builtin_bit_cast(us2v, hi),
                                                              __builtin_bit_cast(us2v, lo));
                sv = (int)__builtin_amdgcn_udot2(b2, (us2v){1, 1}, (uint32_t)sv, false);
                sq = (int)__builtin_amdgcn_udot2(b2, b2, (uint32_t)sq, false);
                // both halves' keys (b << IB) | (CP - 1 - step): ties go to the smaller step
                const uint32_t k2 = (__builtin_bit_cast(uint32_t, b2) << IB) |
                                    (uint32_t)((CP - 1 - t - e) * 0x10001);
                km = __builtin_bit_cast(uint32_t,
                                        __builtin_elementwise_max(__builtin_bit_cast(us2v, k2),
                                                                  __builtin_bit_cast(us2v, km)));
              }
            }
            // the chunk's two half maxima as band-wide keys (b << 10) | (1023 - j)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
              const uint32_t kh = (km >> (16 * h)) & 0xFFFFu;
              const int j = 8 * (CP * g + CP - 1 - (int)(kh & (CP - 1u))) + 2 * qtr + h;
              const int kk = (int)((kh >> IB) << 10) | (1023 - j);
              key = kk > key ? kk : key;
            }
          }
        }
      };
      using I3 = std::integral_constant<int, 3>;
      using I4 = std::integral_constant<int, 4>;
      if (wb <= 16) {  // wave-uniform
        if (wb & 1)
          pairs(std::true_type{}, I4{});
        else
          pairs(std::false_type{}, I4{});
      } else {
        if (wb & 1)
          pairs(std::true_type{}, I3{});
        else
          pairs(std::false_type{}, I3{});
      }
      qv = (uint32_t)sq;
    } else
#endif
    {
      int kl = 0;
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
        if (4 * ch < U) {  // wave-uniform
#pragma unroll
          for (int v = 0; v < 4; ++v) {
            const int u = 4 * ch + v;
            const int o = 8 * (u >> 1) + (u & 1);
            const uint32_t b = __builtin_elementwise_sub_sat((uint32_t)phi[o], (uint32_t)plo[o]);
            // the lane's own key: ties go to the smaller step (the smaller j of this lane)
            const int kk = (int)((b << 6) | (uint32_t)(63 - u));
            kl = kk > kl ? kk : kl;
            sv += (int)b;
            // b < 2^16: the 24-bit multiply is exact; HIP declares __umul24 as returning int,
            // so the cast keeps a product >= 2^31 (b >= 46 341) from being sign-extended
            qv += (uint32_t)__umul24(b, b);
          }
        }
      }
      // the lane's best window as the band-wide key (b << 10) | (1023 - j)
      const int ub = 63 - (kl & 63);
      key = ((kl >> 6) << 10) | (1023 - (8 * (ub >> 1) + 2 * qtr + (ub & 1)));
    }
    // the band's four quarter lanes (bi, bi + 16, bi + 32, bi + 48) combined: integer sums
    // and a maximum
    sv += __shfl_xor(sv, 16);
    qv += xor_u64<16>(qv);
    key = max(key, __shfl_xor(key, 16));
    sv += __shfl_xor(sv, 32);
    qv += xor_u64<32>(qv);
    key = max(key, __shfl_xor(key, 32));
    const bool inb = bi < nb;
    const long long N = (long long)nw * (long long)qv - (long long)sv * sv;
    const bool ok = inb && N > 0;
    const double rl = ok ? 1.0 / sqrt(dnw * (double)N) : 0.0;
    const double cl = (double)sv * rl;
    if (lane < 16 && inb) maxbin[blk + bi] = 1023 - (key & 1023) + wb / 2;  // :1628
    valid += __builtin_popcountll(__ballot(lane < 16 && ok));
    // ---- pass 2: W_j += r_i b_ij in band order (the 16 bands' r and S r through LDS,
    // broadcast reads; C summed in band order) ---------------------------------------------
#ifndef PFE_SB_NODENORM
    // the boxcar sum b (an integer < 2^17) enters the fma as the denormal b * 2^-1074: its
    // 32 bits in the low half of a register pair whose high half is a held zero (no
    // conversion instruction), against r * 2^1022, so every product and partial sum is
    // numpy's times 2^-52 exactly (all terms are >= 0 and >= 2^-79 when non-zero: no
    // subnormal rounding) and W is scaled back once at the end
    if (lane < 16) {
      fold[bi] = rl * 0x1p1022;
      fold[16 + bi] = cl;
    }
#else
    if (lane < 16) {
      fold[bi] = rl;
      fold[16 + bi] = cl;
    }
#endif
    wave_lds_sync();
#pragma unroll
    for (int ii = 0; ii < SB_NB; ii += 2) {
      const double2 r2 = *reinterpret_cast<const double2*>(fold + ii);
      const double2 c2 = *reinterpret_cast<const double2*>(fold + 16 + ii);
      C += c2.x;
      C += c2.y;
      const uint16_t* row0 = rows + ii * STRIDE;
      const uint16_t* row1 = row0 + STRIDE;
#ifndef PFE_SB_NODENORM
#pragma unroll
      for (int k = 0; k < SL; ++k)
        W[k] = __builtin_fma(r2.x, __builtin_bit_cast(double, ((uint64_t)zh[k] << 32) |
                             (uint32_t)((int)row0[hi_k[k]] - (int)row0[lo_k[k]])), W[k]);
#pragma unroll
      for (int k = 0; k < SL; ++k)
        W[k] = __builtin_fma(r2.y, __builtin_bit_cast(double, ((uint64_t)zh[k] << 32) |
                             (uint32_t)((int)row1[hi_k[k]] - (int)row1[lo_k[k]])), W[k]);
#else
#pragma unroll
      for (int k = 0; k < SL; ++k)
        W[k] = __builtin_fma(r2.x, (double)((int)row0[hi_k[k]] - (int)row0[lo_k[k]]), W[k]);
#pragma unroll
      for (int k = 0; k < SL; ++k)
        W[k] = __builtin_fma(r2.y, (double)((int)row1[hi_k[k]] - (int)row1[lo_k[k]]), W[k]);
#endif
    }
    wave_lds_sync();
  }
#ifndef PFE_SB_NODENORM
#pragma unroll
  for (int k = 0; k < SL; ++k) W[k] *= 0x1p52;  // exact
#endif
  // s21: sum_{i<k} cc_ik = (sum_j Z_j^2 - v) / 2 with Z_j = nw W_j - C, |z_i|^2 = 1
  double zs = 0.0;
#pragma unroll
  for (int k = 0; k < SL; ++k) {
    const double z = (lane + 64 * k < nw) ? dnw * W[k] - C : 0.0;
    zs += z * z;
  }
  zs = wsum(zs);
  const long long m = (long long)valid * (valid - 1) / 2;
  if (m == 0) {  // ZeroDivisionError (:1681)
    if (lane == 0) atomicOr(&a.status[c], PFE_ST_SUBBAND_FAIL);
    return;
  }
  const double mean_corr = (0.5 * (zs - (double)valid)) / (double)m;
  wave_lds_sync();
  const double rms = rms_of_maxbins_wave(maxbin, nsub, wb, fold);
  if (lane == 0) {
    double* o = a.out + c * a.ldo;
    o[0] = rms;
    o[1] = mean_corr;
    o[2] = integ;
  }
}

// ---- any shape: prefix rows in global scratch -------------------------------------------
// The LDS-resident kernels above hold a candidate's nsub x (lsb + 1) prefix sums on chip
// (nsub 2-256, nBins 1-1024, nsub (nBins + 1) <= 32768).  Every other shape the reference
// scores (getSubband_scores takes any nsub x nBins) goes here: persistent waves, each with a
// slab of global scratch holding ONE band's prefix row at a time (E, lsb + 1 u32), the s21
// window sums Z (nw doubles, lane-owned) and the boxcar-maximum positions (nsub ints).  The
// arithmetic is k_subband2's, band by band: integer boxcar sums and keys (64-bit here, any
// window index), exact S / nw sum b^2 - S^2 (128-bit), the same z-score identity for s21, and
// s22's centred fp64 sums in the same per-lane slot order and butterfly.
constexpr int SBG_MAX_NSUB = 65536, SBG_MAX_LSB = 16384;

__host__ __device__ inline size_t sbg_slab_bytes(int nsub, int lsb) {
  return ((size_t)(lsb + 1) * 4 + 15) / 16 * 16 + (size_t)lsb * 8 + ((size_t)nsub * 4 + 15) / 16 * 16;
}
static int64_t sbg_waves(int64_t n) { return n < 1024 ? (n > 0 ? n : 1) : 1024; }

__device__ __forceinline__ unsigned long long wmax_u64(unsigned long long v) {
#pragma unroll
  for (int s = 1; s < 64; s <<= 1) {
    const unsigned long long o = (unsigned long long)__shfl_xor((long long)v, s);
    v = o > v ? o : v;
  }
  return v;
}

__device__ __forceinline__ void sbg_sync() {  // the wave's global-scratch stores -> its loads
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}

__global__ __launch_bounds__(64) void k_subband_g(SubArgs a, unsigned char* work) {
  const int lane = lane_id();
  const int nsub = a.nsub, lsb = a.lsb;
  unsigned char* slab = work + (size_t)blockIdx.x * sbg_slab_bytes(nsub, lsb);
  uint32_t* E = reinterpret_cast<uint32_t*>(slab);
  double* Zg = reinterpret_cast<double*>(slab + ((size_t)(lsb + 1) * 4 + 15) / 16 * 16);
  int* maxbin = reinterpret_cast<int*>(reinterpret_cast<unsigned char*>(Zg) + (size_t)lsb * 8);
  for (int64_t c = blockIdx.x; c < a.n; c += gridDim.x) {
    sbg_sync();  // the previous candidate's reads of Zg / maxbin precede this one's stores
    const double width = a.scal[c * PFE_NSCAL + PFE_SCAL_WIDTH];
    const double wbd = ceil(width * (double)lsb);                    // :1603
    if (!(wbd >= 1.0) || wbd > (double)lsb || a.lp != lsb) {
      if (lane == 0) atomicOr(&a.status[c], PFE_ST_SUBBAND_FAIL);
      continue;
    }
    const int wb = (int)wbd;
    const int nw = lsb - wb + 1;
    const uint8_t* sb = a.sub + c * (int64_t)nsub * lsb;
    const uint8_t* pr = a.prof + c * a.lp;
    // the profile, centred as numpy.corrcoef centres it (s22): slots j = lane + 64 k in order
    double pm = 0.0;
    for (int j = lane; j < lsb; j += 64) pm += (double)pr[j];
    pm = wsum(pm) / (double)lsb;
    double pvar = 0.0;
    for (int j = lane; j < lsb; j += 64) {
      const double v = (double)pr[j] - pm;
      pvar += v * v;
    }
    pvar = wsum(pvar);
    const double inv2 = 1.0 / (double)(lsb - 1);
    for (int j = lane; j < nw; j += 64) Zg[j] = 0.0;
    const double dnw = (double)nw;
    double zz = 0.0, integ = 0.0;
    int valid = 0;
    for (int i = 0; i < nsub; ++i) {
      const uint8_t* row = sb + (size_t)i * lsb;
      sbg_sync();  // every lane is done with the previous band's E
      uint32_t carry = 0;
      for (int base = 0; base < lsb; base += 64) {
        const int t = base + lane;
        const int x = t < lsb ? (int)row[t] : 0;
        const int ex = wscan_excl(x);
        if (t < lsb) E[t] = carry + (uint32_t)ex;
        carry += (uint32_t)__shfl(ex + x, 63);
      }
      if (lane == 0) E[lsb] = carry;
      sbg_sync();
      // boxcar statistics: S, sum b^2, first strict maximum
      long long S = 0, Q = 0;
      unsigned long long key = 0;
      for (int j = lane; j < nw; j += 64) {
        const long long b = (long long)E[j + wb] - (long long)E[j];
        S += b;
        Q += b * b;
        const unsigned long long kk = ((unsigned long long)b << 32) | (0xFFFFFFFFull - (unsigned)j);
        key = kk > key ? kk : key;
      }
      S = wsum_ll(S);
      Q = wsum_ll(Q);
      key = wmax_u64(key);
      const __int128 N = (__int128)nw * Q - (__int128)S * S;          // exact: nw^2 var(b)
      const double r = N > 0 ? 1.0 / sqrt(dnw * (double)N) : 0.0;
      valid += N > 0 ? 1 : 0;
      if (lane == 0) maxbin[i] = (int)(0xFFFFFFFFull - (key & 0xFFFFFFFFull)) + wb / 2;  // :1628
      if (r != 0.0) {
        for (int j = lane; j < nw; j += 64) {
          const long long b = (long long)E[j + wb] - (long long)E[j];
          const double z = (double)((long long)nw * b - S) * r;
          Zg[j] += z;
          zz += z * z;
        }
      }
      const double mu = (double)E[lsb] / (double)lsb;
      double dd = 0.0, q = 0.0;
      for (int j = lane; j < lsb; j += 64) {
        const double t = (double)((int)E[j + 1] - (int)E[j]) - mu;
        dd += t * ((double)pr[j] - pm);
        q += t * t;
      }
      dd = wsum(dd);
      q = wsum(q);
      const double cc = fabs(sb_corr(dd * inv2, q * inv2, pvar * inv2));
      if (cc > 0.0055) integ += cc;                                   // in band order
    }
    double zs = 0.0;
    for (int j = lane; j < nw; j += 64) zs += Zg[j] * Zg[j];
    zs = wsum(zs);
    zz = wsum(zz);
    const long long m = (long long)valid * (valid - 1) / 2;
    if (m == 0) {  // ZeroDivisionError (:1681)
      if (lane == 0) atomicOr(&a.status[c], PFE_ST_SUBBAND_FAIL);
      continue;
    }
    const double mean_corr = (0.5 * (zs - zz)) / (double)m;
    sbg_sync();
    const double rms = rms_of_maxbins(maxbin, nsub, wb);
    if (lane == 0) {
      double* o = a.out + c * a.ldo;
      o[0] = rms;
      o[1] = mean_corr;
      o[2] = integ;
    }
  }
}

// ---- launchers -------------------------------------------------------------------------
// the LDS-resident kernels' shapes
static bool subband_lds_shape(int nsub, int lsb) {
  return nsub >= 2 && nsub <= 256 && lsb >= 1 && lsb <= 1024 && (int64_t)nsub * (lsb + 1) <= 32768;
}

// nullptr when the shape is scored, else why not (checked by the C-ABI before any launch)
const char* subband_shape_error(int nsub, int lsb) {
  if (nsub < 1 || nsub > SBG_MAX_NSUB) return "nsub outside [1, 65536]";
  if (lsb < 1 || lsb > SBG_MAX_LSB) return "lsb outside [1, 16384]";
  return nullptr;
}

// global scratch of the any-shape kernel for n candidates (0: the LDS kernels take the shape)
size_t subband_work_bytes(int64_t n, int nsub, int lsb) {
  if (subband_lds_shape(nsub, lsb) || subband_shape_error(nsub, lsb)) return 0;
  return (size_t)sbg_waves(n) * sbg_slab_bytes(nsub, lsb);
}

template <int SL, typename PT>
static hipError_t launch_sl(const SubArgs& s, hipStream_t st) {
  const size_t wave = sb_wave_lds<PT>(s.nsub, s.lsb);
  if (wave * 4 <= 40 * 1024) {
    hipLaunchKernelGGL((k_subband2<SL, PT, 4>), dim3((unsigned)((s.n + 3) / 4)), dim3(256),
                       wave * 4, st, s);
  } else {
    hipError_t e = ensure_dyn_lds<k_subband2<SL, PT, 1>>(wave);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_subband2<SL, PT, 1>), dim3((unsigned)s.n), dim3(64), wave, st, s);
  }
  return hipGetLastError();
}

template <int LSB>
static hipError_t launch_fast(const SubArgs& s, hipStream_t st) {
  const size_t wave = fast_wave_lds<LSB>(s.nsub);
  if (wave * 4 <= 40 * 1024) {
    hipLaunchKernelGGL((k_subband_fast<LSB, 4>), dim3((unsigned)((s.n + 3) / 4)), dim3(256),
                       wave * 4, st, s);
  } else {
    hipError_t e = ensure_dyn_lds<k_subband_fast<LSB, 1>>(wave);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_subband_fast<LSB, 1>), dim3((unsigned)s.n), dim3(64), wave, st, s);
  }
  return hipGetLastError();
}

static hipError_t launch_sub(const SubArgs& s, void* work, hipStream_t st) {
  if (s.n <= 0) return hipSuccess;
  if (subband_shape_error(s.nsub, s.lsb)) return hipErrorInvalidValue;
  if (!subband_lds_shape(s.nsub, s.lsb)) {
    if (!work) return hipErrorInvalidValue;
    hipLaunchKernelGGL(k_subband_g, dim3((unsigned)sbg_waves(s.n)), dim3(64), 0, st, s,
                       (unsigned char*)work);
    return hipGetLastError();
  }
  const int L = s.lsb;
  const bool aligned = (((uintptr_t)s.sub | (uintptr_t)s.prof) & 15) == 0;
  if (aligned && s.lp == L) {
    switch (L) {
      case 16: return launch_fast<16>(s, st);
      case 32: return launch_fast<32>(s, st);
      case 64: return launch_fast<64>(s, st);
      case 128: return launch_fast<128>(s, st);
      case 256: return launch_fast<256>(s, st);
      default: break;
    }
  }
  if (L <= 64) return launch_sl<1, uint16_t>(s, st);
  if (L <= 128) return launch_sl<2, uint16_t>(s, st);
  if (L <= 256) return launch_sl<4, uint16_t>(s, st);
  if (L <= 512) return launch_sl<8, uint32_t>(s, st);
  return launch_sl<16, uint32_t>(s, st);
}

__global__ void k_mark_unsupported(uint32_t* status, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) atomicOr(&status[i], PFE_ST_UNSUPPORTED);
}

// the 22-score chain: scores 20-22 into columns 19-21 of out (n x 22).  A sub-band shape
// beyond every kernel (subband_shape_error: nsub > 65536 or nBins > 16384) fails its rows,
// not the call: the other groups' scores are still computed and every row gets
// PFE_ST_UNSUPPORTED.  a.sub_work: the any-shape kernel's scratch (subband_work_bytes)
hipError_t launch_subband(const BatesArgs& a, hipStream_t st) {
  if (a.n <= 0) return hipSuccess;
  if (subband_shape_error(a.nsub, a.lsb)) {
    hipLaunchKernelGGL(k_mark_unsupported, dim3((unsigned)((a.n + 255) / 256)), dim3(256), 0,
                       st, a.status, a.n);
    return hipGetLastError();
  }
  SubArgs s{a.prof, a.lp, a.sub, a.nsub, a.lsb, a.scal, a.n, a.out + 19, 22, a.status};
  return launch_sub(s, a.sub_work, st);
}

// pfe_subband3: out n x 3; status zeroed here; work: subband_work_bytes(n, nsub, lsb) bytes
hipError_t launch_subband3(const pfe_bates_in* in, double* out, uint32_t* status, void* work,
                           hipStream_t st) {
  hipError_t e = hipMemsetAsync(status, 0, (size_t)in->n * sizeof(uint32_t), st);
  if (e != hipSuccess) return e;
  e = hipMemsetAsync(out, 0, (size_t)in->n * 3 * sizeof(double), st);
  if (e != hipSuccess) return e;
  SubArgs s{in->prof, in->lp, in->sub, in->nsub, in->lsb, in->scal, in->n, out, 3, status};
  return launch_sub(s, work, st);
}

}  // namespace pfe
