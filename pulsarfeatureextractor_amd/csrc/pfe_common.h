// pfe_common.h — shared device helpers for the gfx950 kernels of libpfe.so.
//
// Wave-level (64-lane) reductions are written with DPP row operations
// (__builtin_amdgcn_update_dpp) for the in-row steps and ds_swizzle/readlane-free
// cross-row steps, so no LDS round trip is needed.  Everything here assumes wave64.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>

#define PFE_WAVE 64

namespace pfe {

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) for kernel K before a launch with `bytes`
// of dynamic LDS (> 48 KiB): the attribute is per device, and several handles or host
// threads may launch at once, so the size already set is tracked per device under a lock.
template <auto K>
inline hipError_t ensure_dyn_lds(size_t bytes) {
  if (bytes <= 48 * 1024) return hipSuccess;
  static std::mutex mu;
  static size_t done[64] = {};
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  const bool track = dev >= 0 && dev < 64;
  std::lock_guard<std::mutex> lock(mu);
  if (track && done[dev] >= bytes) return hipSuccess;
  e = hipFuncSetAttribute(reinterpret_cast<const void*>(K),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
  if (e == hipSuccess && track) done[dev] = bytes;
  return e;
}

// ---- DPP controls (gfx9 encoding) ----------------------------------------------------
// quad_perm selectors: ctrl = p0 | p1<<2 | p2<<4 | p3<<6
constexpr int DPP_QUAD_XOR1 = 0xB1;  // [1,0,3,2]
constexpr int DPP_QUAD_XOR2 = 0x4E;  // [2,3,0,1]
constexpr int DPP_ROW_HALF_MIRROR = 0x141;  // lane i <-> 7-i within each 8-lane half-row
constexpr int DPP_ROW_MIRROR = 0x140;       // lane i <-> 15-i within each 16-lane row

// Full row / bank masks and bound_ctrl = 1: a lane whose source is outside its row (the
// shift controls) reads 0, every other lane the selected source -- the result of
// update_dpp(0, v, ..., bound_ctrl = 0), but with no `old` operand, so the compiler does not
// materialise a zero into the destination before every v_mov_b32_dpp (two v_mov_b32 per
// 64-bit step of every group reduction; the same bits)
template <int CTRL>
__device__ __forceinline__ int dpp_i32(int v) {
  return __builtin_amdgcn_mov_dpp(v, CTRL, 0xF, 0xF, true);
}

template <int CTRL>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v) {
  const int lo = dpp_i32<CTRL>((int)(uint32_t)v);
  const int hi = dpp_i32<CTRL>((int)(uint32_t)(v >> 32));
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
  return __longlong_as_double((long long)dpp_u64<CTRL>((uint64_t)__double_as_longlong(v)));
}

// Butterfly all-reduce (sum) over aligned groups of G lanes, G in {1,2,4,8,16}.
// After the call every lane of the group holds the group total.
template <int G>
__device__ __forceinline__ int group_sum_i32(int v) {
  if constexpr (G >= 2) v += dpp_i32<DPP_QUAD_XOR1>(v);
  if constexpr (G >= 4) v += dpp_i32<DPP_QUAD_XOR2>(v);
  if constexpr (G >= 8) v += dpp_i32<DPP_ROW_HALF_MIRROR>(v);
  if constexpr (G >= 16) v += dpp_i32<DPP_ROW_MIRROR>(v);
  return v;
}

template <int G>
__device__ __forceinline__ uint64_t group_sum_u64(uint64_t v) {
  if constexpr (G >= 2) v += dpp_u64<DPP_QUAD_XOR1>(v);
  if constexpr (G >= 4) v += dpp_u64<DPP_QUAD_XOR2>(v);
  if constexpr (G >= 8) v += dpp_u64<DPP_ROW_HALF_MIRROR>(v);
  if constexpr (G >= 16) v += dpp_u64<DPP_ROW_MIRROR>(v);
  return v;
}

// Full-wave sums (64 lanes).  The in-row part uses DPP; the two cross-row steps use
// __shfl_xor (ds_bpermute), which is exact for integers and fixed-order for doubles, so
// the result is identical in every lane and deterministic run to run.
__device__ __forceinline__ long long wave_sum_i64(long long v) {
  uint64_t u = group_sum_u64<16>((uint64_t)v);
  u += (uint64_t)__shfl_xor((long long)u, 16);
  u += (uint64_t)__shfl_xor((long long)u, 32);
  return (long long)u;
}

// Combine the four 16-lane row sums of a wave (each row holds its sum in every lane) as
// (row0 + row1) + (row2 + row3) -- the same tree as xor-16 then xor-32 butterflies -- through
// lane reads, so the result is provably wave-uniform (scalar branches downstream) and no
// LDS-routed permutes are on the critical path.  Requires every lane active.
__device__ __forceinline__ double lane_f64(double v, int src) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(uint32_t)b, src);
  const int hi = __builtin_amdgcn_readlane((int)(uint32_t)((unsigned long long)b >> 32), src);
  return __longlong_as_double((long long)(((unsigned long long)(uint32_t)hi << 32) | (uint32_t)lo));
}
__device__ __forceinline__ double row_total_f64(double v) {
  return (lane_f64(v, 0) + lane_f64(v, 16)) + (lane_f64(v, 32) + lane_f64(v, 48));
}

__device__ __forceinline__ double wave_sum_f64(double v) {
  v += dpp_f64<DPP_QUAD_XOR1>(v);
  v += dpp_f64<DPP_QUAD_XOR2>(v);
  v += dpp_f64<DPP_ROW_HALF_MIRROR>(v);
  v += dpp_f64<DPP_ROW_MIRROR>(v);
  return row_total_f64(v);
}

}  // namespace pfe
