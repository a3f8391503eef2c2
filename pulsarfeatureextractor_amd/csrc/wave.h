// wave.h — wave64 building blocks for the Bates-score kernels (one wavefront per candidate).
//
// Data layout convention: a wave owns one candidate; point i of an m-point vector lives in
// lane (i % 64), slot (i / 64) of a per-lane register array of MPL slots.  "Uniform" values
// (fit parameters, small n x n matrices) are replicated in every lane.
#pragma once

#include "pfe_common.h"

namespace pfe {

__device__ __forceinline__ int lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }

// value of v held by lane `src` (src must be wave-uniform)
__device__ __forceinline__ double bcast(double v, int src) { return lane_f64(v, src); }
__device__ __forceinline__ int bcast_i(int v, int src) { return __builtin_amdgcn_readlane(v, src); }

// make a value that is uniform in fact also uniform for the compiler (SGPR)
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ double uni(double v) { return bcast(v, 0); }

// full-wave sum of doubles, identical in all lanes (fixed butterfly order)
__device__ __forceinline__ double wsum(double v) { return wave_sum_f64(v); }

template <int K>
__device__ __forceinline__ void wsum_arr(double (&v)[K]) {
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] += dpp_f64<DPP_QUAD_XOR1>(v[k]);
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] += dpp_f64<DPP_QUAD_XOR2>(v[k]);
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] += dpp_f64<DPP_ROW_HALF_MIRROR>(v[k]);
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] += dpp_f64<DPP_ROW_MIRROR>(v[k]);
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = row_total_f64(v[k]);
}

// wsum_arr restricted to v[lo..K) (lo folds to a constant inside unrolled loops)
template <int K>
__device__ __forceinline__ void wsum_from(double (&v)[K], int lo) {
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
#pragma unroll
  for (int k = 0; k < K; ++k)
    if (k >= lo) v[k] = row_total_f64(v[k]);
}

__device__ __forceinline__ int wsum_i(int v) {
  v += __shfl_xor(v, 1);
  v += __shfl_xor(v, 2);
  v += __shfl_xor(v, 4);
  v += __shfl_xor(v, 8);
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 32);
  return v;
}
__device__ __forceinline__ long long wsum_ll(long long v) { return wave_sum_i64(v); }

__device__ __forceinline__ double wmax(double v) {
#pragma unroll
  for (int s = 1; s < 64; s <<= 1) v = fmax(v, __shfl_xor(v, s));
  return v;
}
__device__ __forceinline__ double wmin(double v) {
#pragma unroll
  for (int s = 1; s < 64; s <<= 1) v = fmin(v, __shfl_xor(v, s));
  return v;
}
__device__ __forceinline__ int wmax_i(int v) {
#pragma unroll
  for (int s = 1; s < 64; s <<= 1) v = max(v, __shfl_xor(v, s));
  return v;
}
__device__ __forceinline__ int wmin_i(int v) {
#pragma unroll
  for (int s = 1; s < 64; s <<= 1) v = min(v, __shfl_xor(v, s));
  return v;
}

// (value, index) argmax with numpy semantics: the FIRST index of the maximum.  NaN is
// treated as the maximum (numpy.argmax returns the first NaN).
struct ArgMax {
  double v;
  int i;
};
__device__ __forceinline__ bool am_better(double a, int ia, double b, int ib) {
  // is (a,ia) preferred over (b,ib)?
  const bool an = a != a, bn = b != b;
  if (an || bn) return an && (!bn || ia < ib);
  return a > b || (a == b && ia < ib);
}
__device__ __forceinline__ ArgMax wargmax(double v, int i) {
#pragma unroll
  for (int s = 1; s < 64; s <<= 1) {
    const double ov = __shfl_xor(v, s);
    const int oi = __shfl_xor(i, s);
    if (am_better(ov, oi, v, i)) {
      v = ov;
      i = oi;
    }
  }
  return {v, i};
}

// exclusive prefix sum of an int over lanes 0..63
__device__ __forceinline__ int wscan_excl(int v) {
  const int l = lane_id();
  int x = v;
#pragma unroll
  for (int s = 1; s < 64; s <<= 1) {
    const int o = __shfl_up(x, s);
    if (l >= s) x += o;
  }
  return x - v;
}

// Value the optimiser cannot see through: keeps a select chain over register-array elements
// from being folded back into a load through a runtime index (which would demote the whole
// array to scratch memory).
template <typename T>
__device__ __forceinline__ T opaque(T v) {
  asm("" : "+v"(v));
  return v;
}

// select arr[idx] for a small uniform runtime idx without dynamic register indexing
template <int N, typename T>
__device__ __forceinline__ T sel(const T (&a)[N], int idx) {
  T r = opaque(a[0]);
#pragma unroll
  for (int k = 1; k < N; ++k) r = (idx == k) ? opaque(a[k]) : r;
  return r;
}
template <int N, typename T>
__device__ __forceinline__ void put(T (&a)[N], int idx, T v) {
#pragma unroll
  for (int k = 0; k < N; ++k) a[k] = (idx == k) ? v : opaque(a[k]);
}

// sqrt(x), correctly rounded: the compiler's own gfx950 expansion (v_rsq_f64, then two
// Goldschmidt / Newton steps by fma) without its pre-scaling of x < 2^-767 by 2^256 and its
// +-0 / +inf fix-up, so the same bits for every x in [2^-767, inf) in 10 instructions instead
// of 18; a wave with any other x (0, inf, NaN, negative, tiny) takes sqrt() for those lanes
// (a ballot over the active lanes, so it may sit in divergent code).
__device__ __forceinline__ double sqrt_rn(double x) {
  const double y = __builtin_amdgcn_rsq(x);
  double g = x * y;
  double h = y * 0.5;
  const double r = __builtin_fma(-h, g, 0.5);
  h = __builtin_fma(h, r, h);
  g = __builtin_fma(g, r, g);
  double d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  d = __builtin_fma(-g, g, x);
  g = __builtin_fma(d, h, g);
  const bool ok = x >= 0x1p-767 && x < __builtin_inf();
  if (__builtin_expect(__ballot(!ok) != 0, 0)) g = ok ? g : __builtin_sqrt(x);
  return g;
}

}  // namespace pfe
