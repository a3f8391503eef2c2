// lyon8.hip — the 8 Lyon statistical-moment features on gfx950.
//
// Reference: PHCXFile.computeProfileStatScores / computeDMCurveStatScores
// (PulsarFeatureExtractor/src/PHCXFile.py:320-379) compute, per candidate,
//     [mean(bins), std(bins), skew(bins), kurtosis(bins)]
// of the integrated profile and of the DM array, with numpy (mean: sum/n; std: ddof=0)
// and scipy.stats (biased skew g1 = m3/m2^1.5, biased Fisher kurtosis g2 = m4/m2^2 - 3,
// NaN when m2 <= (eps*mean)^2).  The dmprof driver concatenates profile then DM
// (DataProcessor.py:884-886).
//
// Design (HBM-bound streaming reduction, no MFMA):
//   * PHCX bins are 02X bytes, so all power sums are EXACT integers: sum x and sum x^2 with
//     v_dot4_u32_u8, and with y = x - 128 unpacked to 16-bit halves, sum y^3 and sum y^4
//     with v_dot2_{i32_i16,u32_u16} on packed 16-bit squares.  ~3.3 VALU ops per byte.
//   * The exact central-moment numerators n^k*m_k come from T1..T4 in 64-bit modular
//     integer arithmetic (exact for n <= 430; a 128-bit variant covers long DM arrays),
//     so each m_k is correctly rounded from its exact rational value: mean and std match
//     numpy bit-for-bit whenever numpy's own sums are exact (n a power of two <= 256),
//     skew/kurt to a few ulp.
//   * Fast path (lp == ld == L in {64,128,256}, 16-B aligned rows): L/32 lanes per
//     candidate, each lane streams 32 B of the profile row and 32 B of the DM row with
//     dwordx4 loads; the group reduces with DPP quad/half-row butterflies; each lane then
//     finalises 8/(L/32) of the candidate's 8 outputs and stores them as one contiguous
//     16/32/8-byte vector, so a wave writes a dense 1 KiB span of the output matrix.
//   * Generic path (any lengths/alignment): one wave per (candidate,row), byte loads,
//     64-bit per-lane sums, 128-bit finalisation.

#include "options.h"
#include "pfe_common.h"

namespace pfe {

typedef short short2v __attribute__((ext_vector_type(2)));
typedef unsigned short ushort2v __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

// Exact central-moment numerators from shifted power sums (y = x - 128):
//   N2 = n^2 m2 = n T2 - T1^2
//   N3 = n^3 m3 = n^2 T3 - 3 n T1 T2 + 2 T1^3
//   N4 = n^4 m4 = n^3 T4 - 4 n^2 T1 T3 + 6 n T1^2 T2 - 3 T1^4
// Evaluated modulo 2^64; every true value is < 2^63 for n <= 430, so the result is exact.
struct Moments {
  double mean, m2, m3, m4;
};

__device__ __forceinline__ Moments moments_i64(long long n, long long T1, long long T2,
                                               long long T3, unsigned long long T4) {
  typedef unsigned long long u64;
  const u64 un = (u64)n, t1 = (u64)T1, t2 = (u64)T2, t3 = (u64)T3;
  const u64 n2 = un * un, n3 = n2 * un;
  const u64 t1s = t1 * t1;
  const long long N2 = (long long)(un * t2 - t1s);
  const long long N3 = (long long)(n2 * t3 - 3ull * un * t1 * t2 + 2ull * t1s * t1);
  const u64 N4 = n3 * T4 - 4ull * n2 * t1 * t3 + 6ull * un * t1s * t2 - 3ull * t1s * t1s;
  const double dn = (double)n;
  Moments m;
  m.mean = (double)(T1 + 128ll * n) / dn;
  m.m2 = (double)N2 / (dn * dn);
  m.m3 = (double)N3 / (dn * dn * dn);
  m.m4 = (double)N4 / ((dn * dn) * (dn * dn));
  return m;
}

// 128-bit variant for long rows (PHCX DataBlock: nDM*128 values).  Requires n < 2^24.
__device__ __forceinline__ double i128_to_f64(__int128 v) {
  const bool neg = v < 0;
  unsigned __int128 u = neg ? (unsigned __int128)(-v) : (unsigned __int128)v;
  const uint64_t hi = (uint64_t)(u >> 64), lo = (uint64_t)u;
  // hi*2^64 + lo with a single final rounding when hi < 2^53 (always true here)
  double r = (double)hi * 18446744073709551616.0 + (double)lo;
  return neg ? -r : r;
}

__device__ __forceinline__ Moments moments_i128(long long n, long long T1, long long T2,
                                                long long T3, unsigned long long T4) {
  typedef __int128 i128;
  const i128 in = n, t1 = T1, t2 = T2, t3 = T3, t4 = (i128)T4;
  const i128 n2 = in * in, n3 = n2 * in;
  const i128 t1s = t1 * t1;
  const i128 N2 = in * t2 - t1s;
  const i128 N3 = n2 * t3 - 3 * in * t1 * t2 + 2 * t1s * t1;
  const i128 N4 = n3 * t4 - 4 * n2 * t1 * t3 + 6 * in * t1s * t2 - 3 * t1s * t1s;
  const double dn = (double)n;
  Moments m;
  m.mean = (double)(T1 + 128ll * n) / dn;
  m.m2 = i128_to_f64(N2) / (dn * dn);
  m.m3 = i128_to_f64(N3) / (dn * dn * dn);
  m.m4 = i128_to_f64(N4) / ((dn * dn) * (dn * dn));
  return m;
}

// scipy.stats.skew / kurtosis (bias=True, Fisher) zero-variance rule:
//   zero = m2 <= (eps * mean)^2  ->  NaN
__device__ __forceinline__ bool zero_var(const Moments& m) {
  const double e = 2.220446049250313e-16 * m.mean;
  return m.m2 <= e * e;
}

__device__ __forceinline__ double stat_k(const Moments& m, int k) {
  // k: 0 mean, 1 std, 2 skew, 3 kurt
  if (k == 0) return m.mean;
  if (k == 1) return sqrt(m.m2);
  if (zero_var(m)) return __builtin_nan("");
  if (k == 2) return m.m3 / (m.m2 * sqrt(m.m2));
  return m.m4 / (m.m2 * m.m2) - 3.0;
}

// ---- fast path: per-lane accumulation --------------------------------------------------
// L in {64,128,256}; LPC = L/32 lanes per candidate, each streams 32 B of each row.  Per 4
// bytes: S1 = sum x and S2 = sum x^2 by unsigned v_dot4, the shifted y = x-128 only for
// y^3/y^4 (v_perm unpack, packed i16 sub/mul, v_dot2); branch-free finalisation with compile-time powers of 1/L (exact for
// L = 2^k, so mean and m2..m4 are the correctly rounded rationals with no division).
struct Acc2 {
  uint32_t s1, s2;
  int t3;
  uint64_t t4;
};

__device__ __forceinline__ void acc2_dword(uint32_t x, Acc2& a, uint32_t& t4a) {
  a.s1 = __builtin_amdgcn_udot4(x, 0x01010101u, a.s1, false);
  a.s2 = __builtin_amdgcn_udot4(x, x, a.s2, false);
  const uint32_t lo = __builtin_amdgcn_perm(0u, x, 0x0c020c00u);  // [b0,0,b2,0]
  const uint32_t hi = __builtin_amdgcn_perm(0u, x, 0x0c030c01u);  // [b1,0,b3,0]
  short2v ylo = __builtin_bit_cast(short2v, lo) - (short2v){128, 128};
  short2v yhi = __builtin_bit_cast(short2v, hi) - (short2v){128, 128};
  ushort2v qlo = __builtin_bit_cast(ushort2v, ylo) * __builtin_bit_cast(ushort2v, ylo);
  ushort2v qhi = __builtin_bit_cast(ushort2v, yhi) * __builtin_bit_cast(ushort2v, yhi);
  a.t3 = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2v, qlo), ylo, a.t3, false);
  a.t3 = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2v, qhi), yhi, a.t3, false);
  t4a = __builtin_amdgcn_udot2(qlo, qlo, t4a, false);
  t4a = __builtin_amdgcn_udot2(qhi, qhi, t4a, false);
}

__device__ __forceinline__ void acc2_x4(const u32x4 q, Acc2& a) {
  uint32_t u = 0, v = 0;  // each <= 2 dwords * 4 * 2^28 = 2^31
  acc2_dword(q.x, a, u);
  acc2_dword(q.y, a, u);
  acc2_dword(q.z, a, v);
  acc2_dword(q.w, a, v);
  a.t4 += (uint64_t)u + (uint64_t)v;
}

template <int G>
__device__ __forceinline__ void acc2_reduce(Acc2& a) {
  a.s1 = (uint32_t)group_sum_i32<G>((int)a.s1);
  a.s2 = (uint32_t)group_sum_i32<G>((int)a.s2);
  a.t3 = group_sum_i32<G>(a.t3);
  a.t4 = group_sum_u64<G>(a.t4);
}

// the four statistics of one row from its exact sums; n = L (a power of two)
template <int L>
__device__ __forceinline__ void stats4(const Acc2& a, double (&st)[4]) {
  constexpr double IN1 = 1.0 / L, IN2 = IN1 * IN1, IN3 = IN2 * IN1, IN4 = IN2 * IN2;
  const long long S1 = (long long)a.s1;
  const long long T1 = S1 - 128ll * L;                                    // sum y
  const long long T2 = (long long)a.s2 - 256ll * S1 + 16384ll * L;         // sum y^2
  const long long T3 = a.t3;
  typedef unsigned long long u64;
  const long long N2 = (long long)L * T2 - T1 * T1;
  const long long T1s = T1 * T1;
  const long long N3 = (long long)L * L * T3 - 3ll * L * T1 * T2 + 2ll * T1s * T1;
  const u64 N4 = (u64)L * L * L * a.t4 - 4ull * (u64)L * L * (u64)(T1 * T3) +
                 6ull * (u64)L * (u64)(T1s * T2) - 3ull * (u64)T1s * (u64)T1s;
  const double mean = (double)S1 * IN1;
  const double m2 = (double)N2 * IN2;
  const double m3 = (double)N3 * IN3;
  const double m4 = (double)N4 * IN4;
  const double sd = sqrt(m2);
  const double e = 2.220446049250313e-16 * mean;
  const bool zero = m2 <= e * e;                                          // scipy's rule
  st[0] = mean;
  st[1] = sd;
  st[2] = zero ? __builtin_nan("") : m3 / (m2 * sd);
  st[3] = zero ? __builtin_nan("") : m4 / (m2 * m2) - 3.0;
}

// ---- fast path: the stream kernel ------------------------------------------------------
// Each wave step covers U consecutive groups of CPW candidates, so a
// wave reads U*CPW*L contiguous bytes of each input in one burst (8 KiB per array at
// L = 128, U = 4: measured +5% HBM throughput over one group, tools/membw.hip), and all
// 4*U dwordx4 loads are issued unconditionally (out-of-range groups re-read the last row)
// before any is consumed, so the compiler's vmcnt counting keeps them all in flight.
template <int L, int U>
__global__ __launch_bounds__(256) void lyon8_u8_fast3(const uint8_t* __restrict__ prof,
                                                      int64_t ps,
                                                      const uint8_t* __restrict__ dm,
                                                      int64_t ds, int64_t n,
                                                      double* __restrict__ out) {
  constexpr int LPC = L / 32;
  constexpr int CPW = 64 / LPC;
  constexpr int SPL = 8 / LPC;
  const int lane = threadIdx.x & 63;
  const int sub = lane % LPC;
  const int cw = lane / LPC;
  const int j0 = sub * SPL;
  const bool is_dm = j0 >= 4;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t step = (int64_t)CPW * U;
  const int64_t stride = (((int64_t)gridDim.x * blockDim.x) >> 6) * step;
  for (int64_t base = wave * step; base < n; base += stride) {
    u32x4 p[U][2], d[U][2];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      int64_t c = base + u * CPW + cw;
      c = c < n ? c : n - 1;
      const u32x4* pp = reinterpret_cast<const u32x4*>(prof + c * ps + sub * 32);
      const u32x4* dp = reinterpret_cast<const u32x4*>(dm + c * ds + sub * 32);
      p[u][0] = __builtin_nontemporal_load(pp);
      p[u][1] = __builtin_nontemporal_load(pp + 1);
      d[u][0] = __builtin_nontemporal_load(dp);
      d[u][1] = __builtin_nontemporal_load(dp + 1);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t c = base + u * CPW + cw;
      Acc2 sp = {0, 0, 0, 0}, sd = {0, 0, 0, 0};
      acc2_x4(p[u][0], sp);
      acc2_x4(p[u][1], sp);
      acc2_x4(d[u][0], sd);
      acc2_x4(d[u][1], sd);
      acc2_reduce<LPC>(sp);
      acc2_reduce<LPC>(sd);
      Acc2 s;
      s.s1 = is_dm ? sd.s1 : sp.s1;
      s.s2 = is_dm ? sd.s2 : sp.s2;
      s.t3 = is_dm ? sd.t3 : sp.t3;
      s.t4 = is_dm ? sd.t4 : sp.t4;
      double st[4];
      stats4<L>(s, st);
      if (c < n) {
        double* o = out + c * 8 + j0;
        if constexpr (SPL == 4) {
          __builtin_nontemporal_store((f64x2){st[0], st[1]}, reinterpret_cast<f64x2*>(o));
          __builtin_nontemporal_store((f64x2){st[2], st[3]}, reinterpret_cast<f64x2*>(o) + 1);
        } else if constexpr (SPL == 2) {
          const bool hi2 = (j0 & 3) != 0;
          __builtin_nontemporal_store((f64x2){hi2 ? st[2] : st[0], hi2 ? st[3] : st[1]},
                                      reinterpret_cast<f64x2*>(o));
        } else {
          const int k = j0 & 3;
          const double v = k == 0 ? st[0] : k == 1 ? st[1] : k == 2 ? st[2] : st[3];
          __builtin_nontemporal_store(v, o);
        }
      }
    }
  }
}

// ---- generic path ----------------------------------------------------------------------
// One wave per (candidate,row).  Rows of any length/alignment.
__global__ __launch_bounds__(256) void lyon8_u8_generic(const uint8_t* __restrict__ prof,
                                                        int64_t ps, int lp,
                                                        const uint8_t* __restrict__ dm,
                                                        int64_t ds, int ld, int64_t n,
                                                        double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t w = wave; w < 2 * n; w += nwaves) {
    const int64_t c = w >> 1;
    const int row = (int)(w & 1);
    const uint8_t* p = row ? dm + c * ds : prof + c * ps;
    const int len = row ? ld : lp;
    long long t1 = 0, t2 = 0, t3 = 0;
    unsigned long long t4 = 0;
    for (int i = lane; i < len; i += 64) {
      const int y = (int)p[i] - 128;
      const int y2 = y * y;
      t1 += y;
      t2 += y2;
      t3 += (long long)(y2 * y);
      t4 += (unsigned long long)((uint32_t)y2 * (uint32_t)y2);
    }
    t1 = wave_sum_i64(t1);
    t2 = wave_sum_i64(t2);
    t3 = wave_sum_i64(t3);
    t4 = (unsigned long long)wave_sum_i64((long long)t4);
    if (lane < 4) {
      const Moments m = len <= 430 ? moments_i64(len, t1, t2, t3, t4)
                                   : moments_i128(len, t1, t2, t3, t4);
      out[c * 8 + row * 4 + lane] = stat_k(m, lane);
    }
  }
}

// ---- long DM rows: the real PHCX shape -------------------------------------------------
// PHCX's Lyon DM array is the whole section-0 DataBlock (PHCXOperations.getDMCurveData
// :528-539): nDM x 128 bytes (15 360 at nDM = 120, 16 384 at 128) next to a 64/128/256-bin
// profile.  One wave per candidate.
//   * skew / kurt (and mean): exact integer power sums (v_dot4 / v_dot2 as the fast path),
//     reduced over the wave, then the exact rational moments (128-bit numerators).
//   * std: numpy's own arithmetic, so it is bit-identical to numpy.std of the row.  mean =
//     the exact sum / n correctly rounded (numpy's float64 sum of bytes is exact); then
//     d = x - mean and d*d rounded per element, and the squares summed the way numpy's
//     reduction does it: the array in buffered chunks of 8192 elements, each chunk a
//     pairwise sum (leaves of <= 128 values as eight strided running sums combined
//     ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), halves split at a multiple of 8), the chunk sums
//     added in order to 0.  (Measured: this, not one pairwise tree over the whole row, is
//     numpy.std's order for a 15 360-element row.)
//   * Rows whose pairwise trees are perfect -- a chunk of length 2^k * M, M a multiple of 8
//     in (64, 128] -- are laid out so the wave's butterfly IS the tree: the first chunk's
//     leaves sit in lanes 0-31, the second's in lanes 32-63 (a row of <= 8192 values is one
//     chunk whose halves take the two half-waves), leaf i of a half in lane i / L (L = 1 or
//     2 leaves per lane, combined in-lane), lanes past the last leaf hold 0 (x + 0 = x for the
//     non-negative sums), and wave_sum_f64 adds lanes as xor-1, 2, 4, ... partners (IEEE
//     addition is commutative), ending with half-wave 0 + half-wave 1 = chunk 0 + chunk 1.
//     LongShape (host) decides whether ld qualifies; other lengths take lyon8_u8_generic.
//   * the profile row (LP = 64/128/256 bytes) is read by lanes 0..LP/16-1, 16 B each; its
//     power sums are exact and LP a power of two, so stats4<LP> is numpy's value bit for bit.
struct LongShape {
  int ld;         // row length
  int base[2];    // first byte of each half-wave's part
  int m[2];       // leaf length (a multiple of 8 in (64, 128])
  int l[2];       // leaves per lane (1 or 2)
  int lanes[2];   // lanes of the half holding leaves
};

// numpy pairwise leaf of the 16 words w (8 bytes each, leaf length 8 * count words; words
// past it are 0x80 bytes and contribute 0)
__device__ __forceinline__ double leaf_sumsq(const uint64_t (&w)[16], int nwords, double mean) {
  double r[8];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const double d = (double)(uint32_t)((w[k] >> (8 * j)) & 0xFF) - mean;
      const double sq = k < nwords ? d * d : 0.0;
      if (k == 0)
        r[j] = sq;
      else
        r[j] += sq;
    }
  }
  return ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
}

template <int LP>
__global__ __launch_bounds__(256) void lyon8_u8_long(const uint8_t* __restrict__ prof,
                                                     int64_t ps,
                                                     const uint8_t* __restrict__ dm,
                                                     int64_t ds, int64_t n,
                                                     double* __restrict__ out, LongShape sh) {
  constexpr int PL = LP / 16;  // lanes holding the profile
  const int lane = threadIdx.x & 63;
  const int h = lane >> 5, li = lane & 31;
  const int M = sh.m[h], L = sh.l[h];
  const bool has = li < sh.lanes[h];
  const int off0 = sh.base[h] + li * L * M;
  const int nw0 = has ? M / 8 : 0;
  const int nw1 = has && L == 2 ? M / 8 : 0;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t c = wave; c < n; c += nwaves) {
    // ---- one burst of loads: the lane's (up to) two leaves, 8 B words, and 16 B of profile
    const uint8_t* drow = dm + c * ds;
    uint64_t w0[16], w1[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int a0 = k < nw0 ? off0 + 8 * k : 0;
      const int a1 = k < nw1 ? off0 + M + 8 * k : 0;
      w0[k] = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(drow + a0));
      w1[k] = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(drow + a1));
    }
    const int pl = lane < PL ? lane : 0;
    const u32x4 pq = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(prof + c * ps) + pl);
#pragma unroll
    for (int k = 0; k < 16; ++k) {  // words outside the leaves: bytes 0x80, y = 0
      if (k >= nw0) w0[k] = 0x8080808080808080ull;
      if (k >= nw1) w1[k] = 0x8080808080808080ull;
    }
    // ---- exact power sums (0x80 bytes add 128 / 128^2 to S1 / S2, nothing to T3 / T4)
    Acc2 sd = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 16; k += 2) {
      acc2_x4((u32x4){(uint32_t)w0[k], (uint32_t)(w0[k] >> 32), (uint32_t)w0[k + 1],
                      (uint32_t)(w0[k + 1] >> 32)}, sd);
      acc2_x4((u32x4){(uint32_t)w1[k], (uint32_t)(w1[k] >> 32), (uint32_t)w1[k + 1],
                      (uint32_t)(w1[k + 1] >> 32)}, sd);
    }
    const int pad = 8 * (32 - nw0 - nw1);  // 0x80 bytes counted above
    Acc2 sp = {0, 0, 0, 0};
    if (lane < PL) acc2_x4(pq, sp);
    const long long S1 = wave_sum_i64((long long)sd.s1 - 128ll * pad);
    const long long S2 = wave_sum_i64((long long)sd.s2 - 16384ll * pad);
    const long long T3 = wave_sum_i64((long long)sd.t3);
    const unsigned long long T4 = (unsigned long long)wave_sum_i64((long long)sd.t4);
    sp.s1 = (uint32_t)wave_sum_i64((long long)sp.s1);
    sp.s2 = (uint32_t)wave_sum_i64((long long)sp.s2);
    sp.t3 = (int)wave_sum_i64((long long)sp.t3);
    sp.t4 = (uint64_t)wave_sum_i64((long long)sp.t4);
    // ---- numpy's std of the DM row
    const double dn = (double)sh.ld;
    const double mean = (double)S1 / dn;
    const double ssq = wave_sum_f64(leaf_sumsq(w0, nw0, mean) + leaf_sumsq(w1, nw1, mean));
    // ---- finalise: lanes 0-3 the profile statistics, lanes 4-7 the DM row's
    if (lane < 8) {
      double v;
      if (lane < 4) {
        double st[4];
        stats4<LP>(sp, st);
        v = lane == 0 ? st[0] : lane == 1 ? st[1] : lane == 2 ? st[2] : st[3];
      } else {
        const long long T1 = S1 - 128ll * sh.ld;
        const long long T2 = S2 - 256ll * S1 + 16384ll * sh.ld;
        const Moments mo = moments_i128(sh.ld, T1, T2, T3, T4);
        const int k = lane - 4;
        v = k == 0 ? mean : k == 1 ? sqrt(ssq / dn) : stat_k(mo, k);
      }
      __builtin_nontemporal_store(v, out + c * 8 + lane);
    }
  }
}

// ---- long DM rows of 2^k bytes: coalesced, no per-byte floating point -------------------
// nDM = 64 / 128 DataBlock rows (ld = 8192 / 16384 = 1024 * NI).  With n = 2^k the mean
// S1 / 2^k is exact, and so are d = x - mean (a multiple of 2^-k below 256), d*d and every
// partial sum inside one 128-value leaf of numpy's pairwise tree (< 2^23 in units of 2^-2k):
// numpy's leaf sum is the exact rational
//     2^2k * sum_leaf d^2 = 2^2k B - 2^(k+1) S1 A + 128 S1^2     (A = sum x, B = sum x^2)
// evaluated here in 64-bit integers and converted exactly (< 2^53).  Only the tree levels
// above the leaves round, and those follow numpy's order: the two 8192-value chunks (ld =
// 16384) are each a perfect tree over 64 leaves, added as (0 + c0) + c1 = c0 + c1.
//   * loads: wave instruction i reads bytes [1024 i, 1024 i + 1024) of the row, 16 B per
//     lane (fully coalesced dwordx4, all NI issued before any is consumed); lanes 8g..8g+7
//     hold leaf 8i + g.
//   * per leaf, A and B over its 8 lanes by a reduce-scatter: for the leaves of instructions
//     8s..8s+7 lane t = lane & 7 ends with the sums of instruction 8s + t (exact integers),
//     so each lane converts two leaves (s = 0, 1), not sixteen.
//   * set s's leaf index within its chunk is 8t + g: numpy's tree pairs leaf bits 0-2 (lane
//     bits 3-5: row_ror 8, permlane16 / permlane32 swaps) and then leaf bits 3-5 (lane bits
//     0-2: quad and half-row DPP).  IEEE addition is commutative, so both lanes of every pair
//     hold the bits numpy's pair sum has.
//   * skew / kurt / mean as lyon8_u8_long (exact power sums, 128-bit numerators).
constexpr int DPP_ROW_ROR8 = 0x128;

template <int CTRL>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
  return (uint32_t)dpp_i32<CTRL>((int)v);
}

// lane t (= lane & 7) of each 8-lane group gets sum over the group of v[t]
__device__ __forceinline__ uint32_t reduce_scatter8(const uint32_t (&v)[8], int t) {
  const bool b2 = t & 4, b1 = t & 2, b0 = t & 1;
  uint32_t a[4], b[2];
#pragma unroll
  for (int k = 0; k < 4; ++k)  // partner 7 - t: opposite bit 2
    a[k] = (b2 ? v[k + 4] : v[k]) + dpp_u32<DPP_ROW_HALF_MIRROR>(b2 ? v[k] : v[k + 4]);
#pragma unroll
  for (int k = 0; k < 2; ++k)  // partner t ^ 2
    b[k] = (b1 ? a[k + 2] : a[k]) + dpp_u32<DPP_QUAD_XOR2>(b1 ? a[k] : a[k + 2]);
  return (b0 ? b[1] : b[0]) + dpp_u32<DPP_QUAD_XOR1>(b0 ? b[0] : b[1]);
}

__device__ __forceinline__ double swap16_sum(double v) {  // v + (v of lane ^ 16)
  const long long x = __double_as_longlong(v);
  const unsigned lo = (unsigned)x, hi = (unsigned)((unsigned long long)x >> 32);
  const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  return __longlong_as_double((long long)(((unsigned long long)h[0] << 32) | l[0])) +
         __longlong_as_double((long long)(((unsigned long long)h[1] << 32) | l[1]));
}
__device__ __forceinline__ double swap32_sum(double v) {  // v + (v of lane ^ 32)
  const long long x = __double_as_longlong(v);
  const unsigned lo = (unsigned)x, hi = (unsigned)((unsigned long long)x >> 32);
  const auto l = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  const auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  return __longlong_as_double((long long)(((unsigned long long)h[0] << 32) | l[0])) +
         __longlong_as_double((long long)(((unsigned long long)h[1] << 32) | l[1]));
}

// numpy's pairwise tree over the 64 leaves of a set (leaf 8t + g in lane 8g + t)
__device__ __forceinline__ double leaf_tree64(double v) {
  v += dpp_f64<DPP_ROW_ROR8>(v);  // leaf bit 0 = lane bit 3
  v = swap16_sum(v);              // leaf bit 1 = lane bit 4
  v = swap32_sum(v);              // leaf bit 2 = lane bit 5
  v += dpp_f64<DPP_QUAD_XOR1>(v);  // leaf bit 3 = lane bit 0
  v += dpp_f64<DPP_QUAD_XOR2>(v);  // leaf bit 4 = lane bit 1
  v += dpp_f64<DPP_ROW_HALF_MIRROR>(v);  // leaf bit 5 = lane bit 2
  return v;
}

// y^3 / y^4 power sums of one dword (y = x - 128), as acc2_dword without the udot4 sums
__device__ __forceinline__ void acc34_dword(uint32_t x, int& t3, uint32_t& t4a) {
  const uint32_t lo = __builtin_amdgcn_perm(0u, x, 0x0c020c00u);
  const uint32_t hi = __builtin_amdgcn_perm(0u, x, 0x0c030c01u);
  short2v ylo = __builtin_bit_cast(short2v, lo) - (short2v){128, 128};
  short2v yhi = __builtin_bit_cast(short2v, hi) - (short2v){128, 128};
  ushort2v qlo = __builtin_bit_cast(ushort2v, ylo) * __builtin_bit_cast(ushort2v, ylo);
  ushort2v qhi = __builtin_bit_cast(ushort2v, yhi) * __builtin_bit_cast(ushort2v, yhi);
  t3 = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2v, qlo), ylo, t3, false);
  t3 = __builtin_amdgcn_sdot2(__builtin_bit_cast(short2v, qhi), yhi, t3, false);
  t4a = __builtin_amdgcn_udot2(qlo, qlo, t4a, false);
  t4a = __builtin_amdgcn_udot2(qhi, qhi, t4a, false);
}

template <int LP, int NI>
__global__ __launch_bounds__(256) void lyon8_u8_pow2(const uint8_t* __restrict__ prof,
                                                     int64_t ps,
                                                     const uint8_t* __restrict__ dm,
                                                     int64_t ds, int64_t n,
                                                     double* __restrict__ out) {
  static_assert(NI == 8 || NI == 16, "ld = 8192 or 16384");
  constexpr int PL = LP / 16;
  constexpr int K = NI == 16 ? 14 : 13;  // ld = 2^K
  constexpr int LD = 1 << K;
  constexpr double SCALE = 1.0 / (double)(1ll << (2 * K));  // 2^-2K
  const int lane = threadIdx.x & 63;
  const int t = lane & 7;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t c = wave; c < n; c += nwaves) {
    const u32x4* drow = reinterpret_cast<const u32x4*>(dm + c * ds) + lane;
    u32x4 q[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) q[i] = __builtin_nontemporal_load(drow + 64 * i);
    const int pl = lane < PL ? lane : 0;
    const u32x4 pq = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(prof + c * ps) + pl);
    // per instruction: this lane's 16 bytes' sum x and sum x^2; the row's y^3 / y^4 sums
    uint32_t A[NI], B[NI];
    uint32_t s1 = 0, s2 = 0;
    int t3 = 0;
    uint64_t t4 = 0;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      uint32_t a = __builtin_amdgcn_udot4(q[i].x, 0x01010101u, 0u, false);
      a = __builtin_amdgcn_udot4(q[i].y, 0x01010101u, a, false);
      a = __builtin_amdgcn_udot4(q[i].z, 0x01010101u, a, false);
      a = __builtin_amdgcn_udot4(q[i].w, 0x01010101u, a, false);
      uint32_t b = __builtin_amdgcn_udot4(q[i].x, q[i].x, 0u, false);
      b = __builtin_amdgcn_udot4(q[i].y, q[i].y, b, false);
      b = __builtin_amdgcn_udot4(q[i].z, q[i].z, b, false);
      b = __builtin_amdgcn_udot4(q[i].w, q[i].w, b, false);
      A[i] = a;
      B[i] = b;
      s1 += a;
      s2 += b;
      uint32_t u = 0, v = 0;  // each <= 2 dwords * 4 * 2^28 = 2^31
      acc34_dword(q[i].x, t3, u);
      acc34_dword(q[i].y, t3, u);
      acc34_dword(q[i].z, t3, v);
      acc34_dword(q[i].w, t3, v);
      t4 += (uint64_t)u + (uint64_t)v;
    }
    Acc2 sp = {0, 0, 0, 0};
    if (lane < PL) acc2_x4(pq, sp);
    const long long S1 = wave_sum_i64((long long)s1);
    const long long S2 = wave_sum_i64((long long)s2);
    const long long T3 = wave_sum_i64((long long)t3);
    const unsigned long long T4 = (unsigned long long)wave_sum_i64((long long)t4);
    sp.s1 = (uint32_t)wave_sum_i64((long long)sp.s1);
    sp.s2 = (uint32_t)wave_sum_i64((long long)sp.s2);
    sp.t3 = (int)wave_sum_i64((long long)sp.t3);
    sp.t4 = (uint64_t)wave_sum_i64((long long)sp.t4);
    // ---- numpy's std of the DM row: exact leaf sums, numpy's tree above them
    double ssq = 0.0;
#pragma unroll
    for (int s = 0; s < NI / 8; ++s) {
      uint32_t va[8], vb[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        va[k] = A[8 * s + k];
        vb[k] = B[8 * s + k];
      }
      const long long la = reduce_scatter8(va, t), lb = reduce_scatter8(vb, t);
      const long long v2k = (lb << (2 * K)) - ((2 * S1 * la) << K) + 128ll * S1 * S1;
      const double chunk = leaf_tree64((double)v2k * SCALE);
      ssq = s == 0 ? chunk : ssq + chunk;
    }
    // ---- finalise: lanes 0-3 the profile statistics, lanes 4-7 the DM row's
    if (lane < 8) {
      double v;
      if (lane < 4) {
        double st[4];
        stats4<LP>(sp, st);
        v = lane == 0 ? st[0] : lane == 1 ? st[1] : lane == 2 ? st[2] : st[3];
      } else {
        const double dn = (double)LD;
        const long long T1 = S1 - 128ll * LD;
        const long long T2 = S2 - 256ll * S1 + 16384ll * LD;
        const Moments mo = moments_i128(LD, T1, T2, T3, T4);
        const int k = lane - 4;
        v = k == 0 ? (double)S1 / dn : k == 1 ? sqrt(ssq / dn) : stat_k(mo, k);
      }
      __builtin_nontemporal_store(v, out + c * 8 + lane);
    }
  }
}

// ---- long DM rows of 8192 + 2^j * M1 bytes: coalesced loads, leaves through LDS ---------
// e.g. nDM = 120 (15 360 bytes: chunk 0 = 64 leaves of 128, chunk 1 = 64 leaves of 112).
// The mean is not exact there, so numpy's leaf sums round and every d*d is added in numpy's
// order as in lyon8_u8_long -- but the row is read with coalesced dwordx4 loads (16 B per
// lane, 1 KiB per wave instruction, all issued up front) and each chunk is staged through a
// wave-private LDS image, one leaf per lane, so a lane's 16 words come from LDS instead of 16
// scattered global loads.
//   * image: leaf l of a chunk at l * S, S = M + pad with S / 16 odd, so the ds_read_b128 of
//     the 16 lanes of a bank group start on 16 distinct 16-B bank slots (conflict-free);
//     M is a multiple of 16, so every 16-B piece lies in one leaf.
//   * leaves of a chunk are a perfect pairwise tree in lane order (lanes past the last leaf
//     hold 0), summed by wave_sum_f64's butterflies; the chunk sums are added in order.
constexpr int L8_LDS_WAVE_BYTES = 64 * 144;  // 64 leaves at S <= 144

// the LDS image is wave-private: order the wave's own stores and loads
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__host__ __device__ constexpr int lds_leaf_stride(int m) { return m + ((m / 16) % 2 == 0 ? 16 : 32); }

template <int M>
__device__ __forceinline__ double leaf_sumsq_lds(const uint8_t* img, int leaf, double mean) {
  constexpr int S = lds_leaf_stride(M);
  uint64_t w[16];
  const u32x4* p = reinterpret_cast<const u32x4*>(img + leaf * S);
#pragma unroll
  for (int k = 0; k < M / 16; ++k) {
    const u32x4 v = p[k];
    w[2 * k] = ((uint64_t)v.y << 32) | v.x;
    w[2 * k + 1] = ((uint64_t)v.w << 32) | v.z;
  }
  return leaf_sumsq(w, M / 8, mean);
}

// write the chunk's pieces held in q[0..NP) (piece p = lane + 64 i, 16 B at chunk offset 16p)
// into the image: leaf = 16p / M
template <int M, int NP>
__device__ __forceinline__ void stage_chunk(uint8_t* img, const u32x4 (&q)[NP], int lane, int len) {
  constexpr int S = lds_leaf_stride(M);
#pragma unroll
  for (int i = 0; i < NP; ++i) {
    const int o = 16 * (lane + 64 * i);
    if (o < len) {
      const int leaf = o / M;  // M a compile-time constant: a multiply-shift
      *reinterpret_cast<u32x4*>(img + leaf * S + (o - leaf * M)) = q[i];
    }
  }
}

template <int LP, int M1>
__global__ __launch_bounds__(256) void lyon8_u8_lds(const uint8_t* __restrict__ prof, int64_t ps,
                                                    const uint8_t* __restrict__ dm, int64_t ds,
                                                    int64_t n, double* __restrict__ out, int ld) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[4][L8_LDS_WAVE_BYTES];
  constexpr int PL = LP / 16;
  const int lane = threadIdx.x & 63;
  uint8_t* img = lds[threadIdx.x >> 6];
  const int len1 = ld - 8192;                 // chunk 1: 2^j leaves of M1 bytes
  const int leaves1 = len1 / M1;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t c = wave; c < n; c += nwaves) {
    const u32x4* drow = reinterpret_cast<const u32x4*>(dm + c * ds);
    u32x4 q0[8], q1[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) q0[i] = __builtin_nontemporal_load(drow + lane + 64 * i);
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // clamped: out-of-row pieces re-read the last one
      const int p = lane + 64 * i;
      q1[i] = __builtin_nontemporal_load(drow + 512 + (16 * p < len1 ? p : len1 / 16 - 1));
    }
    const int pl = lane < PL ? lane : 0;
    const u32x4 pq = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(prof + c * ps) + pl);
    // ---- exact power sums (pieces past the row count as 0x80 bytes, removed below)
    Acc2 sd = {0, 0, 0, 0};
    int pad = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc2_x4(q0[i], sd);
    stage_chunk<128>(img, q0, lane, 8192);  // chunk 0's image (q0 dies here)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const bool in = 16 * (lane + 64 * i) < len1;
      const u32x4 h = (u32x4){0x80808080u, 0x80808080u, 0x80808080u, 0x80808080u};
      acc2_x4(in ? q1[i] : h, sd);
      pad += in ? 0 : 16;
    }
    Acc2 sp = {0, 0, 0, 0};
    if (lane < PL) acc2_x4(pq, sp);
    const long long S1 = wave_sum_i64((long long)sd.s1 - 128ll * pad);
    const long long S2 = wave_sum_i64((long long)sd.s2 - 16384ll * pad);
    const long long T3 = wave_sum_i64((long long)sd.t3);
    const unsigned long long T4 = (unsigned long long)wave_sum_i64((long long)sd.t4);
    sp.s1 = (uint32_t)wave_sum_i64((long long)sp.s1);
    sp.s2 = (uint32_t)wave_sum_i64((long long)sp.s2);
    sp.t3 = (int)wave_sum_i64((long long)sp.t3);
    sp.t4 = (uint64_t)wave_sum_i64((long long)sp.t4);
    const double dn = (double)ld;
    const double mean = (double)S1 / dn;
    // ---- numpy's std: chunk 0 (64 leaves of 128), then chunk 1, each staged through LDS
    wave_lds_sync();
    const double c0 = wave_sum_f64(leaf_sumsq_lds<128>(img, lane, mean));
    wave_lds_sync();
    stage_chunk<M1>(img, q1, lane, len1);
    wave_lds_sync();
    const double c1 = wave_sum_f64(lane < leaves1 ? leaf_sumsq_lds<M1>(img, lane, mean) : 0.0);
    wave_lds_sync();
    const double ssq = c0 + c1;
    if (lane < 8) {
      double v;
      if (lane < 4) {
        double st[4];
        stats4<LP>(sp, st);
        v = lane == 0 ? st[0] : lane == 1 ? st[1] : lane == 2 ? st[2] : st[3];
      } else {
        const long long T1 = S1 - 128ll * ld;
        const long long T2 = S2 - 256ll * S1 + 16384ll * ld;
        const Moments mo = moments_i128(ld, T1, T2, T3, T4);
        const int k = lane - 4;
        v = k == 0 ? mean : k == 1 ? sqrt(ssq / dn) : stat_k(mo, k);
      }
      __builtin_nontemporal_store(v, out + c * 8 + lane);
    }
  }
}

// ---- DataBlock rows, round 4: per-byte numpy chains at 3 fp64 operations per byte --------
// lyon8_u8_lds spent ~3.1 k VALU wave-instructions per 15 360-byte row (VALU-bound at 37 %
// of HBM): byte extraction from 64-bit words, per-row 128-bit finalisation in every lane,
// 64-bit wave reductions.  This kernel keeps numpy's arithmetic and removes the rest:
//   * each byte of a leaf is read from the wave's padded LDS image with ds_read_u8 (the LDS
//     unit zero-extends it: no VALU extraction), then one fma, one mul, one add (dm_leaf) --
//     numpy's fl(fl(x - mean)^2) added to the leaf's running sum j = i mod 8 in order;
//   * the exact power sums (mean, skew, kurt) come from the coalesced registers the row was
//     loaded into, as the other Lyon-8 kernels compute them (v_dot4 / v_dot2);
//   * the per-row totals are reduced as 32-bit halves (DPP in-row, permlane swaps across
//     rows) and parked in lane (row mod 64); the 8 statistics of a batch of <= 64 rows are
//     finalised once, one row per lane, and stored as one 4 KiB span -- the divisions,
//     square roots and 128-bit numerators run once per 64 rows instead of once per row;
//   * the profile row (64-256 bytes) is summed there too, by the lane that finalises it;
//   * each wave owns a contiguous range of rows (no grid-stride tail imbalance).
// Row layout (numpy's reduction of nDM x 128 values): NCH chunks of 8192, the first NCH-1
// full (64 leaves of 128), the last one numpy's pairwise tree of <= 64 leaves of 64..128
// values (multiples of 8) whose leaves all sit at one depth (a perfect binary tree; their
// lengths may differ, e.g. nDM = 127: 120, 128, 128, 128, ...), so the wave butterfly over
// lane-ordered leaves is numpy's tree.  That covers every nDM in 3..256 but 33, 97, 161, 225
// (host: dm_shape).  LDS image per wave: leaf l at l * 132 (132 = 4 * 33: the 32 lanes of a
// ds_read_u8 group hit 32 distinct banks), written with ds_write_b32 (the padded stride is
// only 4-byte aligned); the last chunk's 8-byte halves go where a per-block table says.
constexpr int DM_MAX_LEAVES = 64;
struct DmShape {
  int lp;          // profile length (64 / 128 / 256)
  int ld;          // DataBlock row length (multiple of 16)
  int len_last;    // bytes of the last chunk
  int leaves_last; // leaves of the last chunk (power of two <= 64; 48 in the tri form)
  int tri;         // 1: the last chunk is 4224 bytes (nDM = 33 mod 64), numpy's one tree
                   // with leaves at two depths: 16 blocks of 264 = 128 + (64 + 72)
  uint16_t start[DM_MAX_LEAVES + 1];  // leaf starts of the last chunk (+ its length)
};

// lane of leaf L of the last chunk: L itself, or in the tri form lane 4b + i for leaf i of
// block b (lane 4b + 3 idle), so that a quad holds one 264-byte block
__host__ __device__ inline int dm_leaf_lane(const DmShape& sh, int L) {
  return sh.tri ? 4 * (L / 3) + L % 3 : L;
}

// numpy's sum of the last chunk's 48 leaves in the tri form: each quad's block as
// L0 + (L64 + L72) (quad broadcasts, every lane of the quad gets the same bits), then the
// 16 blocks pairwise as wave_sum_f64's upper levels
__device__ __forceinline__ double wave_sum_tri_f64(double v) {
  const double l0 = dpp_f64<0x00>(v), l1 = dpp_f64<0x55>(v), l2 = dpp_f64<0xAA>(v);
  v = l0 + (l1 + l2);
  v += dpp_f64<DPP_ROW_HALF_MIRROR>(v);
  v += dpp_f64<DPP_ROW_MIRROR>(v);
  return row_total_f64(v);
}

constexpr int DM_S = 132;                     // LDS leaf stride
constexpr int DM_IMG_BYTES = 64 * DM_S;       // one chunk image per wave (8448 B)
// two one-chunk tri rows per wave (G == 32 of lyon8_u8_dm): a lane's slot holds a block's
// 128-byte leaf (even lane) or its 64- and 72-byte leaves back to back (odd lane, 136 B); the
// stride 140 = 4 x 35 (odd dwords) keeps a ds_read_u8 group's 32 lanes on 32 banks
constexpr int DM_S_T = 140;
constexpr int DM_IMG_T = 64 * DM_S_T;         // 8960 B

// 64-lane sum of a 32-bit value: DPP within rows, then the four row sums through the
// permlane swaps.  Exact; every lane ends with the total.
__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
  v += (uint32_t)dpp_i32<DPP_QUAD_XOR1>((int)v);
  v += (uint32_t)dpp_i32<DPP_QUAD_XOR2>((int)v);
  v += (uint32_t)dpp_i32<DPP_ROW_HALF_MIRROR>((int)v);
  v += (uint32_t)dpp_i32<DPP_ROW_MIRROR>((int)v);
  const auto a = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  v = a[0] + a[1];
  const auto b = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  return b[0] + b[1];
}

// numpy's 8 leaf chains over the words k < nw (8..16) of the leaf at lb (LDS): each byte
// fl(fl(x - mean)^2) added to chain j = i mod 8 in order, then ((r0+r1)+(r2+r3))+((r4+r5)+
// (r6+r7)).  Three VALU per byte, all of numpy's roundings kept, in a scaled domain:
//   * the byte is read with ds_read_u8 (volatile, so it stays one zero-extended byte per read
//     instead of a dword that needs a VALU extraction per byte) into the low half of a VGPR
//     pair whose high half is a zero kept in a register for the whole kernel (z[j]); the pair
//     read as a double is the denormal x * 2^-1074 (fp64 denormals are not flushed:
//     .amdhsa_float_denorm_mode_16_64 3);
//   * d' = fma(2^1023, X, -mean * 2^-51) = fl(x - mean) * 2^-51: the product is exact and
//     the one rounding is the rounding of x - mean, scaled by a power of two (no conversion,
//     no separate subtraction);
//   * sq' = d' * d' = fl(d^2) * 2^-102 and every chain sum likewise (all values stay normal),
//     so the leaf sum is numpy's times 2^-102 exactly (the caller scales it back).
// FPM adds scipy's d^3 = d^2 * d and d^4 = (d^2)^2 as fused running sums (scaled 2^-153 and
// 2^-204), in any order.  Words past the leaf (k >= nw) are read inside the image, not added.
//
// NC < 8 (round 5, the last chunk of a row whose <= 32 leaves would leave lanes idle): the
// lane takes only the NC chains c0 .. c0 + NC - 1 of its leaf (G = 8 / NC lanes per leaf) and
// returns their part of the leaf's tree -- (r0+r1)+(r2+r3) of its four chains, r0+r1 of two,
// r0 of one -- so the first log2(G) steps of the wave butterfly that follows complete each
// leaf's ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) with numpy's bits and the remaining steps are the
// tree over the leaves, as before: the pass reads and squares 128/G bytes per lane.
template <bool FPM, int NC = 8>
__device__ __forceinline__ double dm_leaf(const uint8_t* lb, int c0, double nm, double sc,
                                          const uint32_t (&z)[8], int nw, double& a3, double& a4) {
  static_assert(NC == 1 || NC == 2 || NC == 4 || NC == 8, "chains per lane");
  typedef const volatile __attribute__((address_space(3))) uint8_t lds_u8;
  lds_u8* vb = (lds_u8*)(lb + c0);
  double r[NC];
  double c3[2] = {0.0, 0.0}, c4[2] = {0.0, 0.0};
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    uint32_t x[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) x[j] = vb[8 * k + j];
    if (k < 8 || k < nw) {  // leaves hold >= 8 words: the first eight need no lane test
#pragma unroll
      for (int j = 0; j < NC; ++j) {
        const double X = __builtin_bit_cast(double, ((uint64_t)z[j] << 32) | x[j]);
        const double d = __builtin_fma(sc, X, nm);
        const double sq = d * d;
        r[j] = k == 0 ? sq : r[j] + sq;
        if constexpr (FPM) {
          c3[j & 1] = __builtin_fma(sq, d, c3[j & 1]);
          c4[j & 1] = __builtin_fma(sq, sq, c4[j & 1]);
        }
      }
    }
    // pin word k's arithmetic before word k+1's reads (empty asm ordered with the volatile
    // reads; without it every read of the leaf is hoisted, one VGPR each)
#pragma unroll
    for (int j = 0; j < NC; ++j) asm volatile("" : "+v"(r[j]));
    if constexpr (FPM) asm volatile("" : "+v"(c3[0]), "+v"(c3[1]), "+v"(c4[0]), "+v"(c4[1]));
  }
  a3 = c3[0] + c3[1];
  a4 = c4[0] + c4[1];
  if constexpr (NC == 8) return ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  if constexpr (NC == 4) return (r[0] + r[1]) + (r[2] + r[3]);
  if constexpr (NC == 2) return r[0] + r[1];
  return r[0];
}

// The tri form's last chunk split by chains (G == 3 of lyon8_u8_dm): block b's quad takes
//   q0: the 128-byte leaf's chains 0-3, q3: its chains 4-7 (16 words of 4 bytes each),
//   q1: the 64-byte leaf, chains 0-3 over its 8 words then chains 4-7 (restart at step 8),
//   q2: the 72-byte leaf, chains 0-3 over its 9 words then chains 4-7 (restart at step 9),
// one loop of 18 steps of 4 bytes (q2's 72 bytes; the others' steps past 16 add nothing)
// instead of one lane reading all 128 bytes of the big leaf.  Every chain still adds its
// bytes in order; q0 returns A = (r0+r1)+(r2+r3), q3 B = (r4+r5)+(r6+r7) (the big leaf is
// A + B), q1 / q2 their whole leaves.  Image slots as the tri stab has them: the big leaf at
// 4b (read by q0 and q3), the others at 4b + 1, 4b + 2.
template <bool FPM>
__device__ __forceinline__ double dm_leaf_tri(const uint8_t* img, int lane, double nm, double sc,
                                              const uint32_t (&z)[8], double& a3, double& a4) {
  typedef const volatile __attribute__((address_space(3))) uint8_t lds_u8;
  const int q = lane & 3;
  const uint8_t* leaf = img + (q == 3 ? lane - 3 : lane) * DM_S;
  // step k reads 4 bytes at: b1 + 8k (k < 8), base8 (k = 8), base9 + 8(k - 9) (k >= 9).  The
  // chains 0-3 stream (b1 + 8k) runs until the lane's restart R, then chains 4-7 of word
  // k - R are at leaf + 4 + 8(k - R) (R = 8 for q1, 9 for q2; none for q0 / q3)
  const uint8_t* b1 = leaf + (q == 3 ? 4 : 0);
  const uint8_t* base8 = q == 1 ? leaf + 4 : b1 + 64;
  const uint8_t* base9 = q == 1 ? leaf + 12 : q == 2 ? leaf + 4 : b1 + 72;
  double r[4], sv[4] = {0.0, 0.0, 0.0, 0.0};
  double c3[2] = {0.0, 0.0}, c4[2] = {0.0, 0.0};
#pragma unroll
  for (int k = 0; k < 18; ++k) {
    lds_u8* vb = (lds_u8*)(k < 8 ? b1 + 8 * k : k == 8 ? base8 : base9 + 8 * (k - 9));
    uint32_t x[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = vb[i];
    if (k == 8 || k == 9) {  // the 64 / 72-byte leaf's restart: chains 0-3 done
      const bool rs = q == k - 7;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        sv[i] = rs ? r[i] : sv[i];
        r[i] = rs ? 0.0 : r[i];
      }
    }
    const bool valid = k < 16 || q == 2;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const double X = __builtin_bit_cast(double, ((uint64_t)z[i] << 32) | x[i]);
      const double d = __builtin_fma(sc, X, nm);
      double sq = d * d;
      if (k >= 16) sq = valid ? sq : 0.0;  // +0.0 leaves a non-negative sum's bits alone
      r[i] = k == 0 ? sq : r[i] + sq;
      if constexpr (FPM) {
        c3[i & 1] = __builtin_fma(sq, d, c3[i & 1]);
        c4[i & 1] = __builtin_fma(sq, sq, c4[i & 1]);
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) asm volatile("" : "+v"(r[i]), "+v"(sv[i]));
    if constexpr (FPM) asm volatile("" : "+v"(c3[0]), "+v"(c3[1]), "+v"(c4[0]), "+v"(c4[1]));
  }
  a3 = c3[0] + c3[1];
  a4 = c4[0] + c4[1];
  const double tr = (r[0] + r[1]) + (r[2] + r[3]);
  const double ts = (sv[0] + sv[1]) + (sv[2] + sv[3]);
  return (q == 1 || q == 2) ? ts + tr : tr;
}

// numpy's sum of the tri form's 48 leaves from dm_leaf_tri's parts: the big leaf as q0 + q3
// and the pair as q1 + q2 (quad_perm [3,2,1,0]), the block as big + pair -- the bits of
// wave_sum_tri_f64's l0 + (l1 + l2) -- then the 16 blocks pairwise
__device__ __forceinline__ double wave_sum_tri_split_f64(double v) {
  v += dpp_f64<0x1B>(v);
  v = dpp_f64<0x00>(v) + dpp_f64<0x55>(v);
  v += dpp_f64<DPP_ROW_HALF_MIRROR>(v);
  v += dpp_f64<DPP_ROW_MIRROR>(v);
  return row_total_f64(v);
}

// Two one-chunk tri rows per wave (G == 32 of lyon8_u8_dm; nDM = 33): each half-wave holds
// a row's 16 blocks, block b in lanes 2b (its 128-byte leaf) and 2b + 1 (the 64- and 72-byte
// leaves, 136 bytes in a row of the image).  One loop of 17 words of 8 bytes, all 8 chains per
// lane: the even lane adds its 16 words (the 17th adds +0.0, which leaves a non-negative sum's
// bits alone); the odd lane adds the 64-byte leaf's 8 words, parks its chains at word 8 and
// restarts them for the 72-byte leaf's 9.  Returns the big leaf's tree, or L64 + L72 -- so the
// half-wave butterfly's first step (lane ^ 1) forms numpy's block L0 + (L64 + L72) and its
// remaining steps the perfect tree over the 16 blocks (half_sum_f64).
template <bool FPM>
__device__ __forceinline__ double dm_leaf_tri_pair(const uint8_t* img, int lane, double nm,
                                                   double sc, const uint32_t (&z)[8], double& a3,
                                                   double& a4) {
  typedef const volatile __attribute__((address_space(3))) uint8_t lds_u8;
  const bool odd = (lane & 1) != 0;
  lds_u8* vb = (lds_u8*)(img + lane * DM_S_T);
  double r[8], sv[8];
  double c3[2] = {0.0, 0.0}, c4[2] = {0.0, 0.0};
#pragma unroll
  for (int k = 0; k < 17; ++k) {
    uint32_t x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = vb[8 * k + j];
    if (k == 8) {  // the odd lane: the 64-byte leaf is done, its chains restart
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        sv[j] = r[j];
        r[j] = odd ? 0.0 : r[j];
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const double X = __builtin_bit_cast(double, ((uint64_t)z[j] << 32) | x[j]);
      const double d = __builtin_fma(sc, X, nm);
      double sq = d * d;
      if (k == 16) sq = odd ? sq : 0.0;
      r[j] = k == 0 ? sq : r[j] + sq;
      if constexpr (FPM) {
        c3[j & 1] = __builtin_fma(sq, d, c3[j & 1]);
        c4[j & 1] = __builtin_fma(sq, sq, c4[j & 1]);
      }
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) asm volatile("" : "+v"(r[j]));
    if (k >= 8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) asm volatile("" : "+v"(sv[j]));
    }
    if constexpr (FPM) asm volatile("" : "+v"(c3[0]), "+v"(c3[1]), "+v"(c4[0]), "+v"(c4[1]));
  }
  a3 = c3[0] + c3[1];
  a4 = c4[0] + c4[1];
  const double tr = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
  const double ts = ((sv[0] + sv[1]) + (sv[2] + sv[3])) + ((sv[4] + sv[5]) + (sv[6] + sv[7]));
  return odd ? ts + tr : tr;
}

// Sums over each 32-lane half of the wave (two rows per wave, G == 16 of lyon8_u8_dm): the
// in-row DPP steps of wave_sum_* and one exchange with lane ^ 16 -- for 32 leaves numpy's
// (tree of 0..15) + (tree of 16..31), for fewer the rows past them add +0.0
// (the exchange between the two DPP rows of a half is a v_permlane16_swap per dword, not a
// ds_bpermute: every lane of the row pair adds even row + odd row, the same bits)
__device__ __forceinline__ uint32_t half_sum_u32(uint32_t v) {
  v += (uint32_t)dpp_i32<DPP_QUAD_XOR1>((int)v);
  v += (uint32_t)dpp_i32<DPP_QUAD_XOR2>((int)v);
  v += (uint32_t)dpp_i32<DPP_ROW_HALF_MIRROR>((int)v);
  v += (uint32_t)dpp_i32<DPP_ROW_MIRROR>((int)v);
  const auto a = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  return a[0] + a[1];
}
__device__ __forceinline__ double half_sum_f64(double v) {
  v += dpp_f64<DPP_QUAD_XOR1>(v);
  v += dpp_f64<DPP_QUAD_XOR2>(v);
  v += dpp_f64<DPP_ROW_HALF_MIRROR>(v);
  v += dpp_f64<DPP_ROW_MIRROR>(v);
  return swap16_sum(v);
}

// write chunk ch of the row (its pieces q[8ch .. 8ch+7]) into the wave's LDS image.  Full
// chunks: leaf lane/8 + 8j at offset 16 (lane % 8).  The last chunk: each 8-byte half at the
// address of the block's table stab (0xFFFF: past the chunk).
template <int NCH, int NPMAX>
__device__ __forceinline__ void dm_stage(uint8_t* img, const u32x4 (&q)[NPMAX], int ch, int lane,
                                         uint32_t full_base, const uint16_t* stab) {
  constexpr int NPL = NPMAX - 8 * (NCH - 1);  // pieces of the last chunk (9: tri pairs)
  typedef volatile __attribute__((address_space(3))) uint32_t lds_u32;
  if (ch < NCH - 1) {
    // (volatile: single ds_write_b32 with 16-bit immediate offsets from one base register,
    // not ds_write2_b32 pairs whose 8-bit offsets need a base register per piece)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      lds_u32* dst = (lds_u32*)(img + full_base + 1056 * j);
      const u32x4 v = q[8 * ch + j];
      dst[0] = v.x;
      dst[1] = v.y;
      dst[2] = v.z;
      dst[3] = v.w;
    }
  } else {
#pragma unroll
    for (int j = 0; j < NPL; ++j) {
      const u32x4 v = q[8 * ch + j];
      const uint32_t a0 = stab[(2 * j) * 64 + lane], a1 = stab[(2 * j + 1) * 64 + lane];
      if (a0 != 0xFFFFu) {
        lds_u32* dst = (lds_u32*)(img + a0);
        dst[0] = v.x;
        dst[1] = v.y;
      }
      if (a1 != 0xFFFFu) {
        lds_u32* dst = (lds_u32*)(img + a1);
        dst[0] = v.z;
        dst[1] = v.w;
      }
    }
  }
}

// FPM (the default): skew / kurt from fp64 d^3 / d^4 sums fused into the byte loop (2 fp64
// FMAs per byte) instead of the exact integer power sums (3 packed integer ops per byte).
// Both run at half the VALU rate on gfx950 (profiles/r04_ubench_op_rates.txt: ~5.1 and ~4.4
// cycles per wave-instruction per SIMD), and the fp64 form frees the registers of the 16-bit
// unpacking: 4.20 vs 4.47 ms per 1M rows at nDM = 120, and 6.40 vs 7.01 ms at nDM = 160 with
// the 3- and 4-chunk forms at 3 waves per SIMD (profiles/r04_ab_dm_long.txt).
#ifndef PFE_DM_WPE_LONG
#define PFE_DM_WPE_LONG 3  // waves per SIMD of the 3- and 4-chunk forms (nDM > 128)
#endif
// G: lanes per leaf of the last chunk (1; or 2 / 4 / 8 when it has <= 32 / 16 / 8 leaves,
// see dm_leaf)
template <int NCH, bool FPM, int G = 1>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(NCH <= 2 ? 4 : PFE_DM_WPE_LONG, NCH <= 2 ? 4 : PFE_DM_WPE_LONG)))
void lyon8_u8_dm(const uint8_t* __restrict__ prof, int64_t ps, const uint8_t* __restrict__ dm,
                 int64_t ds, int64_t n, double* __restrict__ out, DmShape sh) {
  static_assert(NCH >= 1 && NCH <= 4, "DataBlocks of up to 4 numpy chunks (nDM <= 256)");
  static_assert(G == 1 || G == 2 || G == 4 || G == 8 || G == 3 || G == 16 || G == 32,
                "lanes per leaf (3: the tri form split; 16: two one-chunk rows per wave; 32: two "
                "one-chunk tri rows per wave)");
  // G == 16: one-chunk rows of <= 32 leaves two at a time, row c in lanes 0-31 and row c + 1
  // in lanes 32-63 (one leaf per lane, every per-row step shared by two rows); G == 32 the
  // same for one-chunk tri rows (nDM = 33, 4224 bytes: nine 16-byte pieces per lane, two lanes
  // per 264-byte block, dm_leaf_tri_pair)
  constexpr bool PAIRT = G == 32;
  constexpr bool PAIR = G == 16 || PAIRT;
  static_assert(!PAIR || (NCH == 1 && FPM), "pairs: one-chunk rows, fp64 moments");
  constexpr int NPMAX = PAIRT ? 9 : 8 * NCH;
  constexpr int NPL = NPMAX - 8 * (NCH - 1);  // 16-byte pieces of the last chunk per lane
  __shared__ __attribute__((aligned(16))) uint8_t lds[4][PAIRT ? DM_IMG_T : DM_IMG_BYTES];
  __shared__ uint16_t stab[2 * NPL * 64];  // last chunk: LDS address of half h of piece j, lane l
  const int lane = threadIdx.x & 63;
  uint8_t* img = lds[threadIdx.x >> 6];
  // the block's staging table (row-invariant): half h of lane l's piece j holds chunk bytes
  // o = 16 l + 1024 j + 8 h, i.e. bytes o - start(L) of leaf L (pairs: o = 16 (l % 32) +
  // 512 j + 8 h of the half's row, its leaf L at slot 32 (l / 32) + L; tri pairs: block
  // b = o / 264 at slots 2b (bytes 0-127) and 2b + 1 (bytes 128-263) of stride DM_S_T)
  for (int e = threadIdx.x; e < 2 * NPL * 64; e += blockDim.x) {
    const int jh = e >> 6, l = e & 63;
    const int o = PAIR ? 16 * (l & 31) + 512 * (jh >> 1) + 8 * (jh & 1)
                       : 16 * l + 1024 * (jh >> 1) + 8 * (jh & 1);
    uint16_t a = 0xFFFFu;
    if (o < sh.len_last) {
      if constexpr (PAIRT) {
        const int b = o / 264, w = o % 264;
        a = (uint16_t)((32 * (l >> 5) + 2 * b + (w < 128 ? 0 : 1)) * DM_S_T + (w < 128 ? w : w - 128));
      } else {
        int L = 0;
        while (L + 1 < sh.leaves_last && sh.start[L + 1] <= o) ++L;
        a = (uint16_t)(((PAIR ? 32 * (l >> 5) : 0) + dm_leaf_lane(sh, L)) * DM_S + (o - sh.start[L]));
      }
    }
    stab[e] = a;
  }
  __syncthreads();
  const int64_t nwaves = (int64_t)gridDim.x * 4;
  // wave-uniform by construction; readfirstlane makes it provable (scalar row loop, SGPR
  // buffer descriptors)
  const int64_t wave = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const int64_t r0 = n * wave / nwaves, r1 = n * (wave + 1) / nwaves;
  const int ppl = sh.lp >> 4;  // 16-byte pieces of the profile
  int zpad = 0;  // zero bytes this lane reads past the row
#pragma unroll
  for (int k = 0; k < NPMAX; ++k) zpad += 16 * (lane + 64 * k) >= sh.ld ? 16 : 0;
  const uint32_t full_base = 16u * lane + 4u * (lane >> 3);  // leaf lane/8, offset 16*(lane%8)
  // this lane's leaf of the last chunk (-1: none) and its 8-byte words
  const int leaf_last = (G == 3 || PAIRT) ? 0  // every lane of the split / paired tri form holds a part
                      : PAIR ? ((lane & 31) < sh.leaves_last ? (lane & 31) : -1)
                      : sh.tri ? ((lane & 3) < 3 ? 3 * (lane >> 2) + (lane & 3) : -1)
                               : (lane / G < sh.leaves_last ? lane / G : -1);
  const int nw_last = leaf_last >= 0 ? (sh.start[leaf_last + 1] - sh.start[leaf_last]) >> 3 : 16;
  // dm_leaf's constants: eight zeros held in registers (the high halves of the byte pairs)
  // and 2^1023 in an SGPR pair (a VOP3 operand; as a literal it would cost a move per byte)
  uint32_t z[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    z[j] = 0u;
    asm volatile("" : "+v"(z[j]));
  }
  double sc = 0x1p1023;
  asm volatile("" : "+s"(sc));
  for (int64_t base = r0; base < r1; base += 64) {
    const int cnt = (int)((r1 - base) < 64 ? (r1 - base) : 64);
    uint32_t kS1 = 0, kS2 = 0, kT3l = 0, kT3h = 0, kT4l = 0, kT4h = 0;
    double kssq = 0.0;
    for (int i = 0; i < cnt; i += PAIR ? 2 : 1) {
      const int64_t c = base + i;
      const bool two = PAIR && i + 1 < cnt;  // pairs: is there a row c + 1 (lanes 32-63)?
      u32x4 q[NPMAX];
      if constexpr (PAIR) {
        // piece p = lane % 32 + 32 k of the half's row (a lone last row: both halves read it)
        const uint8_t* rowp = dm + (c + (two ? (lane >> 5) : 0)) * ds;
#pragma unroll
        for (int k = 0; k < NPMAX; ++k) {
          const int p = (lane & 31) + 32 * k;
          q[k] = 16 * p < sh.ld ? __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(rowp) + p)
                                : (u32x4){0u, 0u, 0u, 0u};
        }
      } else {
        // ---- loads: piece p = lane + 64 k (16 B) through a buffer descriptor of the row's
        // ld bytes, so pieces past the row read as zero bytes (corrected below)
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t*>(dm + c * ds), 0, sh.ld, 0x00020000);
#pragma unroll
        for (int k = 0; k < NPMAX; ++k)
          q[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, 16 * lane, 1024 * k, 2));
      }
      // ---- exact power sums of the DM row; a zero byte past the row adds y^3 = -2^21 and
      // y^4 = 2^28 (y = x - 128) and nothing to sum x, sum x^2
      Acc2 sd = {0, 0, 0, 0};
      if constexpr (FPM) {
#pragma unroll
        for (int k = 0; k < NPMAX; ++k) {
          sd.s1 = __builtin_amdgcn_udot4(q[k].x, 0x01010101u, sd.s1, false);
          sd.s1 = __builtin_amdgcn_udot4(q[k].y, 0x01010101u, sd.s1, false);
          sd.s1 = __builtin_amdgcn_udot4(q[k].z, 0x01010101u, sd.s1, false);
          sd.s1 = __builtin_amdgcn_udot4(q[k].w, 0x01010101u, sd.s1, false);
        }
      } else {
#pragma unroll
        for (int k = 0; k < NPMAX; ++k) acc2_x4(q[k], sd);
        sd.t3 += zpad << 21;
        sd.t4 -= (uint64_t)zpad << 28;
      }
      // ---- numpy's sum of squared deviations, chunk by chunk through the LDS image
      // (chunk 0 is staged before the mean is known, so its registers die early)
      dm_stage<NCH>(img, q, 0, lane, full_base, stab);
      const uint32_t S1 = PAIR ? half_sum_u32(sd.s1) : wave_sum_u32(sd.s1);
      const double mean = (double)S1 / (double)sh.ld;
      const double nm = -__builtin_ldexp(mean, -51);  // exact
      // ---- the integer row totals (exact 32-bit halves) are reduced and parked in lane i
      // now, so their registers are free during the byte loop
      // park row c's value in lane i (pairs: row c + 1's, from lane 32, in lane i + 1)
      const bool mine = lane == i;
      const bool mine2 = two && lane == i + 1;
      auto park_u32 = [&](uint32_t& k, uint32_t v) {
        if constexpr (PAIR) {
          const uint32_t va = (uint32_t)__builtin_amdgcn_readlane((int)v, 0);
          const uint32_t vb = (uint32_t)__builtin_amdgcn_readlane((int)v, 32);
          k = mine ? va : mine2 ? vb : k;
        } else {
          k = mine ? v : k;
        }
      };
      park_u32(kS1, S1);
      if constexpr (!FPM) {
        const uint32_t S2 = wave_sum_u32(sd.s2);
        const uint32_t T3l = wave_sum_u32((uint32_t)sd.t3 & 0xFFFFu);
        const uint32_t T3h = wave_sum_u32((uint32_t)(sd.t3 >> 16));
        const uint32_t T4l = wave_sum_u32((uint32_t)sd.t4 & 0xFFFFFFu);
        const uint32_t T4h = wave_sum_u32((uint32_t)(sd.t4 >> 24));
        kS2 = mine ? S2 : kS2;
        kT3l = mine ? T3l : kT3l;
        kT3h = mine ? T3h : kT3h;
        kT4l = mine ? T4l : kT4l;
        kT4h = mine ? T4h : kT4h;
      }
      double ssq = 0.0, a3 = 0.0, a4 = 0.0;
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
        if (ch > 0) dm_stage<NCH>(img, q, ch, lane, full_base, stab);
        wave_lds_sync();
        double l3, l4;
        double leaf;
        if (PAIRT)  // two tri rows per wave, two lanes per block
          leaf = dm_leaf_tri_pair<FPM>(img, lane, nm, sc, z, l3, l4);
        else if (G == 3 && ch == NCH - 1)  // the tri form, its big leaf split by chains
          leaf = dm_leaf_tri<FPM>(img, lane, nm, sc, z, l3, l4);
        else if (G == 2 || G == 4 || G == 8) {  // the last chunk's leaf lane / G, chains of this lane
          if (ch == NCH - 1)
            leaf = dm_leaf<FPM, (G == 2 || G == 4 || G == 8) ? 8 / G : 8>(img + (lane / G) * DM_S,
                                                                       (8 / G) * (lane % G), nm, sc, z, nw_last, l3, l4);
          else
            leaf = dm_leaf<FPM>(img + lane * DM_S, 0, nm, sc, z, 16, l3, l4);
        }
        else
          leaf = dm_leaf<FPM>(img + lane * DM_S, 0, nm, sc, z, ch < NCH - 1 ? 16 : nw_last, l3, l4);
        if (ch == NCH - 1) {
          const bool in = leaf_last >= 0;
          leaf = in ? leaf : 0.0;
          l3 = in ? l3 : 0.0;
          l4 = in ? l4 : 0.0;
        }
        a3 += l3;
        a4 += l4;
        // numpy's tree over the lane-ordered leaves (the tri form: two depths)
        const double cs = PAIR ? half_sum_f64(leaf)
                          : (ch == NCH - 1 && G == 3) ? wave_sum_tri_split_f64(leaf)
                          : (ch == NCH - 1 && sh.tri) ? wave_sum_tri_f64(leaf) : wave_sum_f64(leaf);
        ssq = ch == 0 ? cs : ssq + cs;         // chunk sums in order (all scaled by 2^-102)
        wave_lds_sync();
      }
      ssq = __builtin_ldexp(ssq, 102);  // exact: numpy's sum of squared deviations
      if constexpr (FPM) {  // the fp64 d^3 / d^4 sums, parked as their two 32-bit halves
        const double s3 = __builtin_ldexp(a3, 153), s4 = __builtin_ldexp(a4, 204);
        const uint64_t b3 = (uint64_t)__double_as_longlong(PAIR ? half_sum_f64(s3) : wave_sum_f64(s3));
        const uint64_t b4 = (uint64_t)__double_as_longlong(PAIR ? half_sum_f64(s4) : wave_sum_f64(s4));
        park_u32(kT3l, (uint32_t)b3);
        park_u32(kT3h, (uint32_t)(b3 >> 32));
        park_u32(kT4l, (uint32_t)b4);
        park_u32(kT4h, (uint32_t)(b4 >> 32));
      }
      if constexpr (PAIR) {
        const double va = lane_f64(ssq, 0), vb = lane_f64(ssq, 32);
        kssq = mine ? va : mine2 ? vb : kssq;
      } else {
        kssq = mine ? ssq : kssq;
      }
    }
    // ---- finalise the batch: lane i -> row base + i
    if (lane < cnt) {
      // profile: lane i sums row base + i's lp bytes itself (exact power sums, once per 64
      // rows; lp a power of two: every moment is the correctly rounded exact rational)
      Acc2 sp = {0, 0, 0, 0};
      const u32x4* pr = reinterpret_cast<const u32x4*>(prof + (base + lane) * ps);
      for (int k = 0; k < ppl; ++k) acc2_x4(__builtin_nontemporal_load(pr + k), sp);
      const long long L = sh.lp;
      const long long S1p = (long long)sp.s1;
      const long long T1p = S1p - 128ll * L;
      const long long T2p = (long long)sp.s2 - 256ll * S1p + 16384ll * L;
      const long long T3p = (long long)sp.t3;
      const uint64_t T4p = sp.t4;
      const Moments mp = moments_i64(L, T1p, T2p, T3p, T4p);
      const double sdp = sqrt(mp.m2);
      const bool zp = zero_var(mp);
      // DM row: mean exact, std = numpy's sqrt(ssq / n), skew / kurt from the exact
      // third / fourth moments over scipy's m2 = ssq / n
      const long long D = sh.ld;
      const long long S1 = (long long)kS1;
      const double dn = (double)D;
      Moments md;
      if constexpr (FPM) {
        md.mean = (double)S1 / dn;
        md.m3 = __longlong_as_double((long long)(((uint64_t)kT3h << 32) | kT3l)) / dn;
        md.m4 = __longlong_as_double((long long)(((uint64_t)kT4h << 32) | kT4l)) / dn;
      } else {
        const long long T1 = S1 - 128ll * D;
        const long long T2 = (long long)kS2 - 256ll * S1 + 16384ll * D;
        const long long T3 = (long long)(int)kT3h * 65536ll + (long long)kT3l;
        const uint64_t T4 = ((uint64_t)kT4h << 24) + (uint64_t)kT4l;
        md = moments_i128(D, T1, T2, T3, T4);
      }
      const double m2 = kssq / dn;
      const double e = 2.220446049250313e-16 * md.mean;
      const bool zd = m2 <= e * e;
      const double sdd = sqrt(m2);
      f64x2* o = reinterpret_cast<f64x2*>(out + (base + lane) * 8);
      __builtin_nontemporal_store((f64x2){mp.mean, sdp}, o);
      __builtin_nontemporal_store(
          (f64x2){zp ? __builtin_nan("") : mp.m3 / (mp.m2 * sdp),
                  zp ? __builtin_nan("") : mp.m4 / (mp.m2 * mp.m2) - 3.0}, o + 1);
      __builtin_nontemporal_store((f64x2){md.mean, sdd}, o + 2);
      __builtin_nontemporal_store(
          (f64x2){zd ? __builtin_nan("") : md.m3 / (m2 * sdd),
                  zd ? __builtin_nan("") : md.m4 / (m2 * m2) - 3.0}, o + 3);
    }
  }
}

// ---- fp64 rows (PFD) -------------------------------------------------------------------
// Two-pass fp64, as numpy/scipy: mean = sum/n; m_k = mean((x-mean)^k) with d^3 = d^2*d and
// d^4 = (d^2)^2 (scipy.stats._moment exponentiation by squares).  One wave per row.
__global__ __launch_bounds__(256) void lyon8_f64_generic(const double* __restrict__ prof,
                                                         int64_t ps, int lp,
                                                         const double* __restrict__ dm,
                                                         int64_t ds, int ld, int64_t n,
                                                         double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t w = wave; w < 2 * n; w += nwaves) {
    const int64_t c = w >> 1;
    const int row = (int)(w & 1);
    const double* p = row ? dm + c * ds : prof + c * ps;
    const int len = row ? ld : lp;
    double s = 0.0;
    for (int i = lane; i < len; i += 64) s += p[i];
    s = wave_sum_f64(s);
    const double mean = s / (double)len;
    double a2 = 0.0, a3 = 0.0, a4 = 0.0;
    for (int i = lane; i < len; i += 64) {
      const double d = p[i] - mean;
      const double d2 = d * d;
      a2 += d2;
      a3 += d2 * d;
      a4 += d2 * d2;
    }
    a2 = wave_sum_f64(a2);
    a3 = wave_sum_f64(a3);
    a4 = wave_sum_f64(a4);
    if (lane < 4) {
      Moments m;
      m.mean = mean;
      m.m2 = a2 / (double)len;
      m.m3 = a3 / (double)len;
      m.m4 = a4 / (double)len;
      out[c * 8 + row * 4 + lane] = stat_k(m, lane);
    }
  }
}

}  // namespace pfe

// ---- launchers (called from capi.cpp) ---------------------------------------------------
namespace pfe {

static inline int grid_for(int64_t work_waves, int cap) {
  // 4 waves per block; capped (handle option PFE_OPT_LYON8_BLOCKS, default 256 CUs x 64
  // blocks: 7 resident waves per SIMD at 71 VGPRs; 32 blocks per CU were +1-2 % over 8
  // (tools/ab_lyon8_grid.sh), 64 a further 1.3 % over 32 (profiles/r03_ab_lyon8_grid.txt))
  // and grid-stride the rest
  int64_t blocks = (work_waves + 3) / 4;
  if (blocks < 1) blocks = 1;
  if (blocks > cap) blocks = cap;
  return (int)blocks;
}

// one chunk of numpy's reduction as a perfect pairwise tree: len = 2^k * m, m a multiple
// of 8 in (64, 128]; -> (m, leaves) or false
static bool perfect_chunk(int len, int& m, int& leaves) {
  leaves = 1;
  while (len > 128) {
    if (len % 16) return false;  // halves must stay multiples of 8
    len /= 2;
    leaves *= 2;
  }
  m = len;
  return len > 64 && len % 8 == 0;
}

// place a chunk's (or half-chunk's) leaves on the 32 lanes of half-wave h
static bool place_half(LongShape& sh, int h, int base, int len) {
  int m, leaves;
  if (!perfect_chunk(len, m, leaves) || leaves > 64) return false;
  sh.base[h] = base;
  sh.m[h] = m;
  sh.l[h] = leaves > 32 ? 2 : 1;
  sh.lanes[h] = leaves > 32 ? 32 : leaves;
  return true;
}

// lyon8_u8_long's layout of a DM row of ld bytes (numpy: chunks of 8192, each pairwise)
static bool long_row_shape(int ld, LongShape& sh) {
  sh.ld = ld;
  if (ld <= 256) return false;  // short rows: the fast / generic kernels
  if (ld <= 8192) {             // one chunk: its two halves take the two half-waves
    return ld % 16 == 0 && place_half(sh, 0, 0, ld / 2) && place_half(sh, 1, ld / 2, ld / 2);
  }
  if (ld <= 16384) return place_half(sh, 0, 0, 8192) && place_half(sh, 1, 8192, ld - 8192);
  return false;
}

// numpy's pairwise leaves of a contiguous sum of n values (numpy/core pairwise_sum: blocks
// of <= 128 values; larger ranges split at n/2 rounded down to a multiple of 8): appends
// (start, length, depth)
static void np_leaves(int off, int n, int depth, int* start, int* len, int* dep, int& cnt, int cap) {
  if (n <= 128) {
    if (cnt < cap) {
      start[cnt] = off;
      len[cnt] = n;
      dep[cnt] = depth;
    }
    ++cnt;
    return;
  }
  int n2 = n / 2;
  n2 -= n2 % 8;
  np_leaves(off, n2, depth + 1, start, len, dep, cnt, cap);
  np_leaves(off + n2, n - n2, depth + 1, start, len, dep, cnt, cap);
}

// lyon8_u8_dm's layout of a DataBlock row of ld bytes: nch chunks of 8192 values, the last
// one a perfect pairwise tree (all leaves at one depth) of <= 64 leaves of 64..128 values
// (the one imperfect last chunk of a DataBlock, 4224 bytes at nDM = 33 mod 64, takes the
// tri form: its 48 leaves are 16 blocks of 128 @ depth 5 + (64 + 72) @ depth 6)
static bool dm_shape(int lp, int ld, DmShape& sh, int& nch) {
  if (ld <= 256 || ld > 4 * 8192 || ld % 16) return false;
  nch = (ld + 8191) / 8192;
  const int len = ld - 8192 * (nch - 1);
  int start[DM_MAX_LEAVES], lens[DM_MAX_LEAVES], dep[DM_MAX_LEAVES], cnt = 0;
  np_leaves(0, len, 0, start, lens, dep, cnt, DM_MAX_LEAVES);
  if (cnt > DM_MAX_LEAVES) return false;
  bool tri = false;
  if (cnt == 48) {  // the tri form, checked leaf by leaf
    tri = true;
    for (int i = 0; i < cnt; ++i) {
      const int b = i / 3, k = i % 3;
      tri = tri && start[i] == 264 * b + (k == 0 ? 0 : k == 1 ? 128 : 192) &&
            lens[i] == (k == 0 ? 128 : k == 1 ? 64 : 72) && dep[i] == dep[0] + (k == 0 ? 0 : 1);
    }
    if (!tri) return false;
  } else {
    if ((cnt & (cnt - 1)) != 0) return false;
    for (int i = 0; i < cnt; ++i)
      if (dep[i] != dep[0] || lens[i] % 8 || lens[i] < 64 || lens[i] > 128) return false;
  }
  sh.lp = lp;
  sh.ld = ld;
  sh.len_last = len;
  sh.leaves_last = cnt;
  sh.tri = tri ? 1 : 0;
  for (int i = 0; i < cnt; ++i) sh.start[i] = (uint16_t)start[i];
  for (int i = cnt; i <= DM_MAX_LEAVES; ++i) sh.start[i] = (uint16_t)len;
  return true;
}

// blocks of K that fit on the device at once (occupancy x CUs), cached per kernel
template <auto K>
static int resident_blocks() {
  static int cached[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 1024;
  if (cached[dev] > 0) return cached[dev];
  int per_cu = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reinterpret_cast<const void*>(K), 256, 0) !=
          hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) {
    (void)hipGetLastError();
    return 1024;
  }
  cached[dev] = (per_cu > 0 ? per_cu : 1) * (cus > 0 ? cus : 1);
  return cached[dev];
}

// rows of up to PFE_DM_FPM_MAXCH numpy chunks take the fp64-moment form by default
#ifndef PFE_DM_FPM_MAXCH
#define PFE_DM_FPM_MAXCH 4
#endif
template <int NCH, bool FPM, int G = 1>
static void launch_dm_kernel(const uint8_t* prof, int64_t ps, const uint8_t* dm, int64_t ds,
                             int64_t n, double* out, const DmShape& sh, hipStream_t st, int cap) {
  constexpr auto K = lyon8_u8_dm<NCH, FPM, G>;
  int64_t blocks = resident_blocks<K>();
  const int64_t need = (n + 3) / 4;  // at least one row per wave
  if (blocks > need) blocks = need;
  if (blocks > cap) blocks = cap;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(K, dim3((unsigned)blocks), dim3(256), 0, st, prof, ps, dm, ds, n, out, sh);
}

hipError_t launch_lyon8_u8(const uint8_t* prof, int64_t ps, int lp, const uint8_t* dm,
                           int64_t ds, int ld, int64_t n, double* out, hipStream_t st,
                           const Options& o) {
  if (n <= 0) return hipSuccess;
  const bool aligned = ((uintptr_t)prof % 16 == 0) && ((uintptr_t)dm % 16 == 0) &&
                       (ps % 16 == 0) && (ds % 16 == 0) && ((uintptr_t)out % 16 == 0);
  DmShape dsh{};
  int dnch = 0;
  if (o.lyon8_dm != 1 && aligned && (lp == 64 || lp == 128 || lp == 256) && ld != 8192 &&
      ld != 16384 && dm_shape(lp, ld, dsh, dnch)) {
    // DataBlock rows (PHCX nDM x 128 bytes) other than the 2^k lengths: lyon8_u8_dm (DESIGN
    // §3.1c), skew / kurt from fp64 d^3 / d^4 sums (the faster form at every length
    // measured), from the exact power sums with option 2
    const int cap = o.lyon8_blocks;
    // lanes per leaf of the last chunk: a last chunk of <= 32 leaves is split by chains
    // (PFE_OPT_LYON8_DM_SPLIT = 0 keeps one lane per leaf)
    const int G = !o.lyon8_dm_split ? 1
                  // one-chunk tri rows (nDM = 33) two per wave, as the 17-32-leaf rows below
                  : (dsh.tri && dnch == 1 && o.lyon8_dm_split == 1) ? 32
                  : dsh.tri ? 3  // the tri form's big leaf split by chains
                  // two one-chunk rows per wave where a chain split would only halve the
                  // leaves' work (32 leaves); at <= 16 the 4- and 8-lane splits are faster
                  // (profiles/r05_lyon8_dm_pairs.txt)
                  : (dnch == 1 && dsh.leaves_last > 16 && dsh.leaves_last <= 32 && o.lyon8_dm_split == 1) ? 16
                  : dsh.leaves_last <= 8 ? 8 : dsh.leaves_last <= 16 ? 4 : dsh.leaves_last <= 32 ? 2 : 1;
    if (o.lyon8_dm == 0 && dnch <= PFE_DM_FPM_MAXCH) {
#define PFE_DMK(C)                                                                   \
  switch (G) {                                                                       \
    case 8: launch_dm_kernel<C, true, 8>(prof, ps, dm, ds, n, out, dsh, st, cap); break; \
    case 4: launch_dm_kernel<C, true, 4>(prof, ps, dm, ds, n, out, dsh, st, cap); break; \
    case 2: launch_dm_kernel<C, true, 2>(prof, ps, dm, ds, n, out, dsh, st, cap); break; \
    case 3: launch_dm_kernel<C, true, 3>(prof, ps, dm, ds, n, out, dsh, st, cap); break; \
    case 16: if constexpr (C == 1) launch_dm_kernel<1, true, 16>(prof, ps, dm, ds, n, out, dsh, st, cap); break; \
    case 32: if constexpr (C == 1) launch_dm_kernel<1, true, 32>(prof, ps, dm, ds, n, out, dsh, st, cap); break; \
    default: launch_dm_kernel<C, true, 1>(prof, ps, dm, ds, n, out, dsh, st, cap); break; \
  }
      switch (dnch) {
        case 1: PFE_DMK(1) break;
        case 2: PFE_DMK(2) break;
#if PFE_DM_FPM_MAXCH > 2
        case 3: PFE_DMK(3) break;
        default: PFE_DMK(4) break;
#endif
      }
#undef PFE_DMK
    } else {
      switch (dnch) {
        case 1: launch_dm_kernel<1, false>(prof, ps, dm, ds, n, out, dsh, st, cap); break;
        case 2: launch_dm_kernel<2, false>(prof, ps, dm, ds, n, out, dsh, st, cap); break;
        case 3: launch_dm_kernel<3, false>(prof, ps, dm, ds, n, out, dsh, st, cap); break;
        default: launch_dm_kernel<4, false>(prof, ps, dm, ds, n, out, dsh, st, cap); break;
      }
    }
    return hipGetLastError();
  }
  if (aligned && lp == ld && (lp == 64 || lp == 128 || lp == 256)) {
    const int U = o.lyon8_burst;  // 1, 2 (default) or 4 candidate groups per wave step
    const int cpw = 64 / (lp / 32) * U;
    const int grid = grid_for((n + cpw - 1) / cpw, o.lyon8_blocks);
#define PFE_L8(LL, UU) \
  hipLaunchKernelGGL((lyon8_u8_fast3<LL, UU>), dim3(grid), dim3(256), 0, st, prof, ps, dm, ds, n, out)
#define PFE_L8U(LL)          \
  do {                       \
    if (U == 1)              \
      PFE_L8(LL, 1);         \
    else if (U == 4)         \
      PFE_L8(LL, 4);         \
    else                     \
      PFE_L8(LL, 2);         \
  } while (0)
    if (lp == 64)
      PFE_L8U(64);
    else if (lp == 128)
      PFE_L8U(128);
    else
      PFE_L8U(256);
#undef PFE_L8U
#undef PFE_L8
  } else if (aligned && (lp == 64 || lp == 128 || lp == 256) && (ld == 8192 || ld == 16384)) {
    // nDM = 64 / 128 DataBlock rows: exact leaf sums, coalesced loads (lyon8_u8_pow2)
    const int grid = grid_for(n, o.lyon8_blocks);
#define PFE_L8P(LL, NN) \
  hipLaunchKernelGGL((lyon8_u8_pow2<LL, NN>), dim3(grid), dim3(256), 0, st, prof, ps, dm, ds, n, out)
    if (ld == 16384) {
      if (lp == 64)
        PFE_L8P(64, 16);
      else if (lp == 128)
        PFE_L8P(128, 16);
      else
        PFE_L8P(256, 16);
    } else {
      if (lp == 64)
        PFE_L8P(64, 8);
      else if (lp == 128)
        PFE_L8P(128, 8);
      else
        PFE_L8P(256, 8);
    }
#undef PFE_L8P
  } else if (int m1 = 0, l1 = 0; aligned && (lp == 64 || lp == 128 || lp == 256) && ld > 8192 &&
                                  ld < 16384 && ld % 16 == 0 && perfect_chunk(ld - 8192, m1, l1) &&
                                  m1 % 16 == 0) {
    // 8192 + 2^j * M1 bytes (nDM = 120: 15 360): coalesced loads, leaves through LDS
    const int grid = grid_for(n, o.lyon8_blocks);
#define PFE_L8S(LL, MM) \
  hipLaunchKernelGGL((lyon8_u8_lds<LL, MM>), dim3(grid), dim3(256), 0, st, prof, ps, dm, ds, n, out, ld)
#define PFE_L8SM(LL)          \
  do {                        \
    if (m1 == 80)             \
      PFE_L8S(LL, 80);        \
    else if (m1 == 96)        \
      PFE_L8S(LL, 96);        \
    else if (m1 == 112)       \
      PFE_L8S(LL, 112);       \
    else                      \
      PFE_L8S(LL, 128);       \
  } while (0)
    if (lp == 64)
      PFE_L8SM(64);
    else if (lp == 128)
      PFE_L8SM(128);
    else
      PFE_L8SM(256);
#undef PFE_L8SM
#undef PFE_L8S
  } else if (LongShape sh{}; aligned && (lp == 64 || lp == 128 || lp == 256) &&
                                long_row_shape(ld, sh)) {
    // real PHCX shape: short profile + the whole DataBlock (lyon8_u8_long)
    const int grid = grid_for(n, o.lyon8_blocks);
    if (lp == 64)
      hipLaunchKernelGGL(lyon8_u8_long<64>, dim3(grid), dim3(256), 0, st, prof, ps, dm, ds, n, out, sh);
    else if (lp == 128)
      hipLaunchKernelGGL(lyon8_u8_long<128>, dim3(grid), dim3(256), 0, st, prof, ps, dm, ds, n, out, sh);
    else
      hipLaunchKernelGGL(lyon8_u8_long<256>, dim3(grid), dim3(256), 0, st, prof, ps, dm, ds, n, out, sh);
  } else {
    const int grid = grid_for(2 * n, o.lyon8_blocks);
    hipLaunchKernelGGL(lyon8_u8_generic, dim3(grid), dim3(256), 0, st, prof, ps, lp, dm, ds, ld, n, out);
  }
  return hipGetLastError();
}

hipError_t launch_lyon8_f64(const double* prof, int64_t ps, int lp, const double* dm,
                            int64_t ds, int ld, int64_t n, double* out, hipStream_t st,
                            const Options& o) {
  if (n <= 0) return hipSuccess;
  const int grid = grid_for(2 * n, o.lyon8_blocks);
  hipLaunchKernelGGL(lyon8_f64_generic, dim3(grid), dim3(256), 0, st, prof, ps, lp, dm, ds, ld, n, out);
  return hipGetLastError();
}

}  // namespace pfe
