// np_sum.h — numpy's own reduction orders on one wavefront (device helpers shared by the
// PFD kernels and the float-profile variants of the 22-score kernels).
#pragma once

#include "wave.h"

namespace pfe {

#pragma clang fp contract(off)

// ---- numpy pairwise summation ---------------------------------------------------------
// a leaf (n <= 128): r[j] = a[j] + a[j+8] + ... over the largest multiple of 8, combined as
// ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)), then the remainder in order; n < 8: 0 + a0 + a1 ...
__device__ __forceinline__ double np_leaf(const double* a, int n, int lane) {
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

// np_leaf for 8 <= n <= 128 with every load of a lane issued before its adds (the same
// order of additions, so the same bits)
__device__ __forceinline__ double np_leaf128(const double* a, int n, int lane) {
  const int nb = n - (n % 8);
  double v[16];
#pragma unroll
  for (int m = 0; m < 16; ++m) v[m] = a[min((lane & 7) + 8 * m, n - 1)];
  double r = v[0];
#pragma unroll
  for (int m = 1; m < 16; ++m)
    if (8 * m < nb) r += v[m];
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

// np_pairwise with every level inlined (no call).  numpy splits at floor8(n/2), so the larger
// half n - floor8(n/2) can exceed n/2 (969 -> 489 -> 249 -> 129): D levels reproduce numpy's
// order exactly for n <= np_inl_max(D) = 128, 248, 488, 968, 1928 (D = 0..4), not 128 * 2^D
__host__ __device__ constexpr int np_inl_max(int D) { return D == 0 ? 128 : 2 * (np_inl_max(D - 1) - 4); }
static_assert(np_inl_max(1) == 248 && np_inl_max(3) == 968, "numpy pairwise split bound");
template <int D>
__device__ __forceinline__ double np_pairwise_inl(const double* a, int n, int lane) {
  if (n <= 128 || D == 0) return np_leaf(a, n, lane);
  if constexpr (D > 0) {
    int n2 = n / 2;
    n2 -= n2 % 8;
    return np_pairwise_inl<D - 1>(a, n2, lane) + np_pairwise_inl<D - 1>(a + n2, n - n2, lane);
  }
  return 0.0;
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

__device__ __forceinline__ void lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace pfe
