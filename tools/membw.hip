// membw.hip — HBM ceiling for the Lyon-8 traffic mix on MI355X (diagnostic, not product).
// Reads R bytes (two arrays, like prof+dm) and writes W = R/4 bytes, with several access
// shapes, timed with hipEvents.  Build: hipcc --offload-arch=gfx950 -O3 tools/membw.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));

#define CK(x)                                                                      \
  do {                                                                             \
    hipError_t e = (x);                                                            \
    if (e != hipSuccess) {                                                         \
      printf("%s: %s\n", #x, hipGetErrorString(e));                                \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

// shape 0: fully coalesced 16 B/lane over each input, 1 output dword4 per 4 input dword4s
template <bool NT>
__global__ __launch_bounds__(256) void k_coalesced(const u32x4* a, const u32x4* b, u32x4* o,
                                                    long n16) {  // n16 = #16B chunks per input
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long stride = (long)gridDim.x * blockDim.x;
  for (; i < n16 / 4; i += stride) {
    u32x4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      u32x4 x = NT ? __builtin_nontemporal_load(a + i + k * (n16 / 4)) : a[i + k * (n16 / 4)];
      u32x4 y = NT ? __builtin_nontemporal_load(b + i + k * (n16 / 4)) : b[i + k * (n16 / 4)];
      acc += x ^ y;
    }
    if (NT)
      __builtin_nontemporal_store(acc, o + i);
    else
      o[i] = acc;
  }
}

// shape 1: the lyon8 mapping (4 lanes x 32 B per 128-B row, two rows per lane group)
template <bool NT>
__global__ __launch_bounds__(256) void k_rows(const unsigned char* a, const unsigned char* b,
                                              double* o, long n) {
  const int lane = threadIdx.x & 63, sub = lane & 3, cw = lane >> 2;
  const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long nw = ((long)gridDim.x * blockDim.x) >> 6;
  for (long base = wave * 16; base < n; base += nw * 16) {
    const long c = base + cw;
    const u32x4* pa = (const u32x4*)(a + c * 128 + sub * 32);
    const u32x4* pb = (const u32x4*)(b + c * 128 + sub * 32);
    u32x4 x0 = NT ? __builtin_nontemporal_load(pa) : pa[0];
    u32x4 x1 = NT ? __builtin_nontemporal_load(pa + 1) : pa[1];
    u32x4 y0 = NT ? __builtin_nontemporal_load(pb) : pb[0];
    u32x4 y1 = NT ? __builtin_nontemporal_load(pb + 1) : pb[1];
    u32x4 s = x0 ^ x1 ^ y0 ^ y1;
    f64x2 v = {(double)s.x, (double)(s.y ^ s.z ^ s.w)};
    if (NT)
      __builtin_nontemporal_store(v, (f64x2*)(o + c * 8 + sub * 2));
    else
      *(f64x2*)(o + c * 8 + sub * 2) = v;
  }
}

// shape 2: 8 lanes x 16 B per row, each instruction a contiguous 1 KiB
template <bool NT>
__global__ __launch_bounds__(256) void k_rows8(const unsigned char* a, const unsigned char* b,
                                               double* o, long n) {
  const int lane = threadIdx.x & 63;
  const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long nw = ((long)gridDim.x * blockDim.x) >> 6;
  for (long base = wave * 16; base < n; base += nw * 16) {
    const u32x4* pa = (const u32x4*)(a + base * 128);
    const u32x4* pb = (const u32x4*)(b + base * 128);
    u32x4 x0 = NT ? __builtin_nontemporal_load(pa + lane) : pa[lane];
    u32x4 x1 = NT ? __builtin_nontemporal_load(pa + 64 + lane) : pa[64 + lane];
    u32x4 y0 = NT ? __builtin_nontemporal_load(pb + lane) : pb[lane];
    u32x4 y1 = NT ? __builtin_nontemporal_load(pb + 64 + lane) : pb[64 + lane];
    u32x4 s = x0 ^ x1 ^ y0 ^ y1;
    f64x2 v = {(double)s.x, (double)(s.y ^ s.z ^ s.w)};
    // 16 candidates x 64 B = 1 KiB of output per wave, 16 B per lane
    if (NT)
      __builtin_nontemporal_store(v, (f64x2*)(o + base * 8) + lane);
    else
      ((f64x2*)(o + base * 8))[lane] = v;
  }
}


// shape 3: rows32B mapping, but each lane group walks Q distant regions (Q candidates per
// lane group per iteration, one from each 1/Q of the range)
template <int Q>
__global__ __launch_bounds__(256) void k_rowsQ(const unsigned char* a, const unsigned char* b,
                                               double* o, long n) {
  const int lane = threadIdx.x & 63, sub = lane & 3, cw = lane >> 2;
  const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long nw = ((long)gridDim.x * blockDim.x) >> 6;
  const long part = n / Q;
  for (long base = wave * 16; base < part; base += nw * 16) {
    u32x4 x[Q][2], y[Q][2];
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const long c = q * part + base + cw;
      const u32x4* pa = (const u32x4*)(a + c * 128 + sub * 32);
      const u32x4* pb = (const u32x4*)(b + c * 128 + sub * 32);
      x[q][0] = __builtin_nontemporal_load(pa);
      x[q][1] = __builtin_nontemporal_load(pa + 1);
      y[q][0] = __builtin_nontemporal_load(pb);
      y[q][1] = __builtin_nontemporal_load(pb + 1);
    }
#pragma unroll
    for (int q = 0; q < Q; ++q) {
      const long c = q * part + base + cw;
      u32x4 s = x[q][0] ^ x[q][1] ^ y[q][0] ^ y[q][1];
      f64x2 v = {(double)s.x, (double)(s.y ^ s.z ^ s.w)};
      __builtin_nontemporal_store(v, (f64x2*)(o + c * 8 + sub * 2));
    }
  }
}

// shape 4: pure reads, coalesced (ceiling for the read side)
__global__ __launch_bounds__(256) void k_readonly(const u32x4* a, const u32x4* b, u32x4* o, long n16) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long stride = (long)gridDim.x * blockDim.x;
  u32x4 acc = {0, 0, 0, 0};
  for (; i < n16 / 4; i += stride) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      acc += __builtin_nontemporal_load(a + i + k * (n16 / 4));
      acc += __builtin_nontemporal_load(b + i + k * (n16 / 4));
    }
  }
  if (acc.x == 0x12345678u) o[0] = acc;
}

// shape 5: rows32B with independent load/store cache policies and U iterations in flight
template <bool NTL, bool NTS, int U>
__global__ __launch_bounds__(256) void k_rowsU(const unsigned char* a, const unsigned char* b,
                                               double* o, long n) {
  const int lane = threadIdx.x & 63, sub = lane & 3, cw = lane >> 2;
  const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long nw = ((long)gridDim.x * blockDim.x) >> 6;
  for (long base = wave * 16 * U; base < n; base += nw * 16 * U) {
    u32x4 x[U][2], y[U][2];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long c = base + u * 16 + cw;
      const u32x4* pa = (const u32x4*)(a + c * 128 + sub * 32);
      const u32x4* pb = (const u32x4*)(b + c * 128 + sub * 32);
      if (c < n) {
        x[u][0] = NTL ? __builtin_nontemporal_load(pa) : pa[0];
        x[u][1] = NTL ? __builtin_nontemporal_load(pa + 1) : pa[1];
        y[u][0] = NTL ? __builtin_nontemporal_load(pb) : pb[0];
        y[u][1] = NTL ? __builtin_nontemporal_load(pb + 1) : pb[1];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long c = base + u * 16 + cw;
      if (c < n) {
        u32x4 s = x[u][0] ^ x[u][1] ^ y[u][0] ^ y[u][1];
        f64x2 v = {(double)s.x, (double)(s.y ^ s.z ^ s.w)};
        if (NTS)
          __builtin_nontemporal_store(v, (f64x2*)(o + c * 8 + sub * 2));
        else
          *(f64x2*)(o + c * 8 + sub * 2) = v;
      }
    }
  }
}

// shape 5b: the same mapping with only one side of the traffic: MODE 1 reads the 256 B of a
// candidate and stores nothing (the result escapes through an impossible branch), MODE 2
// stores the 64 B of a candidate and reads nothing -- the read and write parts of the
// Lyon-8 kernel's traffic, timed apart
template <int MODE, int U>
__global__ __launch_bounds__(256) void k_rows_half(const unsigned char* a, const unsigned char* b,
                                                   double* o, long n) {
  const int lane = threadIdx.x & 63, sub = lane & 3, cw = lane >> 2;
  const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long nw = ((long)gridDim.x * blockDim.x) >> 6;
  u32x4 acc = {0, 0, 0, 0};
  for (long base = wave * 16 * U; base < n; base += nw * 16 * U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      long c = base + u * 16 + cw;
      c = c < n ? c : n - 1;
      if constexpr (MODE == 1) {
        const u32x4* pa = (const u32x4*)(a + c * 128 + sub * 32);
        const u32x4* pb = (const u32x4*)(b + c * 128 + sub * 32);
        acc ^= __builtin_nontemporal_load(pa) ^ __builtin_nontemporal_load(pa + 1) ^
               __builtin_nontemporal_load(pb) ^ __builtin_nontemporal_load(pb + 1);
      } else {
        f64x2 v = {(double)(c + sub), (double)c};
        __builtin_nontemporal_store(v, (f64x2*)(o + c * 8 + sub * 2));
      }
    }
  }
  if (MODE == 1 && acc.x == 0x12345678u && acc.y == 0x9abcdef0u) o[0] = (double)acc.z;
}

// shape 6: plain float4 copy (calibration against MI355X_MICROARCH.md's 6.29 TB/s)
__global__ __launch_bounds__(256) void k_copy(const u32x4* a, u32x4* o, long n16) {
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  const long stride = (long)gridDim.x * blockDim.x;
  for (; i < n16; i += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(a + i), o + i);
}

// shape 7: one interleaved stream [prof 128 B | dm 128 B] per candidate, U groups per step
template <int U>
__global__ __launch_bounds__(256) void k_inter(const unsigned char* a, double* o, long n) {
  const int lane = threadIdx.x & 63, sub = lane & 3, cw = lane >> 2;
  const long wave = ((long)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const long nw = ((long)gridDim.x * blockDim.x) >> 6;
  for (long base = wave * 16 * U; base < n; base += nw * 16 * U) {
    u32x4 x[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      long c = base + u * 16 + cw;
      c = c < n ? c : n - 1;
      const u32x4* pa = (const u32x4*)(a + c * 256 + sub * 32);
      x[u][0] = __builtin_nontemporal_load(pa);
      x[u][1] = __builtin_nontemporal_load(pa + 1);
      x[u][2] = __builtin_nontemporal_load(pa + 8);
      x[u][3] = __builtin_nontemporal_load(pa + 9);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long c = base + u * 16 + cw;
      if (c < n) {
        u32x4 s = x[u][0] ^ x[u][1] ^ x[u][2] ^ x[u][3];
        f64x2 v = {(double)s.x, (double)(s.y ^ s.z ^ s.w)};
        __builtin_nontemporal_store(v, (f64x2*)(o + c * 8 + sub * 2));
      }
    }
  }
}

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 10000000;  // candidates
  const int reps = 20;
  unsigned char *a, *b;
  double* o;
  CK(hipMalloc(&a, n * 256));
  CK(hipMalloc(&b, n * 256));
  CK(hipMalloc(&o, n * 64));
  CK(hipMemset(a, 1, n * 256));
  CK(hipMemset(b, 2, n * 128));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const double bytes = (double)n * 320;
  auto run = [&](const char* name, auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    printf("%-28s %8.4f ms  %7.1f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
  };
  // the Lyon-8 kernel's traffic split: read side alone, write side alone, both (grid 16384
  // as lyon8_u8_fast3's cap; GB/s over the 320 B of a candidate in every line)
  for (int rep = 0; rep < 2; ++rep) {
    run("split: read 256 B only g16384", [&] { hipLaunchKernelGGL((k_rows_half<1, 2>), dim3(16384), dim3(256), 0, 0, a, b, o, n); });
    run("split: write 64 B only g16384", [&] { hipLaunchKernelGGL((k_rows_half<2, 2>), dim3(16384), dim3(256), 0, 0, a, b, o, n); });
    run("split: read+write g16384", [&] { hipLaunchKernelGGL((k_rowsU<1, 1, 2>), dim3(16384), dim3(256), 0, 0, a, b, o, n); });
    run("split: read+write, plain stores", [&] { hipLaunchKernelGGL((k_rowsU<1, 0, 2>), dim3(16384), dim3(256), 0, 0, a, b, o, n); });
    run("split: read+write, plain loads", [&] { hipLaunchKernelGGL((k_rowsU<0, 1, 2>), dim3(16384), dim3(256), 0, 0, a, b, o, n); });
    run("split: read+write, U4", [&] { hipLaunchKernelGGL((k_rowsU<1, 1, 4>), dim3(16384), dim3(256), 0, 0, a, b, o, n); });
    run("split: read+write g8192", [&] { hipLaunchKernelGGL((k_rowsU<1, 1, 2>), dim3(8192), dim3(256), 0, 0, a, b, o, n); });
    run("split: read+write g32768", [&] { hipLaunchKernelGGL((k_rowsU<1, 1, 2>), dim3(32768), dim3(256), 0, 0, a, b, o, n); });
    run("copy (3.2GB moved) g16384", [&] { hipLaunchKernelGGL(k_copy, dim3(16384), dim3(256), 0, 0, (const u32x4*)a, (u32x4*)b, n * 10); });
  }
  for (int rep = 0; rep < 2; ++rep)
  for (int grid : {1024, 2048}) {
    char nm[64];
    snprintf(nm, 64, "copy (3.2GB moved) g%d", grid);
    run(nm, [&] { hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, (const u32x4*)a, (u32x4*)b, n * 10); });
    snprintf(nm, 64, "rowsU L1 S1 U2 g%d", grid);
    run(nm, [&] { hipLaunchKernelGGL((k_rowsU<1, 1, 2>), dim3(grid), dim3(256), 0, 0, a, b, o, n); });
    snprintf(nm, 64, "interleaved U1 g%d", grid);
    run(nm, [&] { hipLaunchKernelGGL((k_inter<1>), dim3(grid), dim3(256), 0, 0, a, o, n); });
    snprintf(nm, 64, "interleaved U2 g%d", grid);
    run(nm, [&] { hipLaunchKernelGGL((k_inter<2>), dim3(grid), dim3(256), 0, 0, a, o, n); });
  }
  return 0;
}
