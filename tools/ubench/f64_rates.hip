// Microbenchmark: issue rates of the instructions the DataBlock kernel is made of, on
// gfx950 -- independent v_fma_f64 / v_mul_f64 / v_add_f64 streams, a dependent v_add_f64
// chain, the integer ops of the sub-band kernel, and ds_read_u8 -- per SIMD at 1, 2, 4 and 8
// waves per SIMD (check the op's ISA with --save-temps: the count per element is assumed).
//   hipcc --offload-arch=gfx950 -O3 -o f64_rates f64_rates.hip && ./f64_rates
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr int ITERS = 4096;

template <int OP>
__global__ __launch_bounds__(256) void k_valu(double* out, double s) {
  double a[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = threadIdx.x * 1e-3 + j;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if constexpr (OP == 0) a[j] = __builtin_fma(a[j], s, 1.0);   // independent fma
      if constexpr (OP == 1) a[j] = a[j] * s;                       // independent mul
      if constexpr (OP == 2) a[j] = a[j] + s;                       // independent add
      if constexpr (OP == 3) a[0] = a[0] + s;                       // dependent add chain
      if constexpr (OP == 4) a[j] = __builtin_bit_cast(double, __builtin_bit_cast(unsigned long long, a[j]) + 1ull);  // 2x u32 adds
      if constexpr (OP == 5) {  // v_dot4_u32_u8 x2 (both halves)
        typedef unsigned u2 __attribute__((ext_vector_type(2)));
        u2 v = __builtin_bit_cast(u2, a[j]);
        v.x = __builtin_amdgcn_udot4(v.y, 0x01010101u, v.x, false);
        v.y = __builtin_amdgcn_udot4(v.x, v.x, v.y, false);
        a[j] = __builtin_bit_cast(double, v);
      }
      if constexpr (OP == 6) {  // v_pk_mul_lo_u16 x2
        typedef unsigned short s2 __attribute__((ext_vector_type(2)));
        typedef unsigned u2 __attribute__((ext_vector_type(2)));
        u2 v = __builtin_bit_cast(u2, a[j]);
        s2 p = __builtin_bit_cast(s2, v.x), q = __builtin_bit_cast(s2, v.y);
        p = p * q; q = q * p;
        v.x = __builtin_bit_cast(unsigned, p); v.y = __builtin_bit_cast(unsigned, q);
        a[j] = __builtin_bit_cast(double, v);
      }
      if constexpr (OP == 7) {  // v_dot2_u32_u16 x2
        typedef unsigned short s2 __attribute__((ext_vector_type(2)));
        typedef unsigned u2 __attribute__((ext_vector_type(2)));
        u2 v = __builtin_bit_cast(u2, a[j]);
        v.x = __builtin_amdgcn_udot2(__builtin_bit_cast(s2, v.y), __builtin_bit_cast(s2, v.y), v.x, false);
        v.y = __builtin_amdgcn_udot2(__builtin_bit_cast(s2, v.x), __builtin_bit_cast(s2, v.x), v.y, false);
        a[j] = __builtin_bit_cast(double, v);
      }
      if constexpr (OP == 9) {  // v_add_u32 x2 (independent halves)
        typedef unsigned u2 __attribute__((ext_vector_type(2)));
        u2 v = __builtin_bit_cast(u2, a[j]);
        v.x += 0x9e3779b9u; v.y += 0x7f4a7c15u;
        a[j] = __builtin_bit_cast(double, v);
      }
      if constexpr (OP == 10) {  // v_mad_u64_u32 x1
        typedef unsigned u2 __attribute__((ext_vector_type(2)));
        unsigned long long u = __builtin_bit_cast(unsigned long long, a[j]);
        const unsigned b = (unsigned)u;
        u = (unsigned long long)b * (unsigned)(b >> 3) + u;
        a[j] = __builtin_bit_cast(double, u);
      }
      if constexpr (OP == 11) {  // v_sad_u8 x2
        typedef unsigned u2 __attribute__((ext_vector_type(2)));
        u2 v = __builtin_bit_cast(u2, a[j]);
        v.x = __builtin_amdgcn_sad_u8(v.y, 0u, v.x);
        v.y = __builtin_amdgcn_sad_u8(v.x, 0u, v.y);
        a[j] = __builtin_bit_cast(double, v);
      }
      if constexpr (OP == 12) {  // v_cvt_f64_i32 x1
        const int b = (int)__builtin_bit_cast(unsigned long long, a[j]);
        a[j] = (double)(b ^ 5);
      }
      if constexpr (OP == 13) {  // v_add_u32_sdwa (byte-select add) x2
        typedef unsigned u2 __attribute__((ext_vector_type(2)));
        u2 v = __builtin_bit_cast(u2, a[j]);
        v.x = v.x + ((v.y >> 8) & 0xFFu);
        v.y = v.y + ((v.x >> 16) & 0xFFu);
        a[j] = __builtin_bit_cast(double, v);
      }
      if constexpr (OP == 14) {  // v_cndmask_b32 x2
        typedef unsigned u2 __attribute__((ext_vector_type(2)));
        u2 v = __builtin_bit_cast(u2, a[j]);
        const bool c = (threadIdx.x & 1) != 0;
        const unsigned x = c ? v.x : v.y, y = c ? v.y : v.x;
        v.x = x; v.y = y;
        a[j] = __builtin_bit_cast(double, v);
      }
      if constexpr (OP == 8) {  // v_perm_b32 x2
        typedef unsigned u2 __attribute__((ext_vector_type(2)));
        u2 v = __builtin_bit_cast(u2, a[j]);
        v.x = __builtin_amdgcn_perm(v.y, v.x, 0x0c020c00u);
        v.y = __builtin_amdgcn_perm(v.x, v.y, 0x0c030c01u);
        a[j] = __builtin_bit_cast(double, v);
      }
    }
    asm volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]));
  }
  double t = 0;
#pragma unroll
  for (int j = 0; j < 8; ++j) t += a[j];
  if (t == 12345.0) out[threadIdx.x] = t;
}

__global__ __launch_bounds__(256) void k_ds_u8(double* out, int stride) {
  __shared__ unsigned char img[4][64 * 132];
  typedef const volatile __attribute__((address_space(3))) unsigned char lds_u8;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (int e = threadIdx.x; e < 4 * 64 * 132; e += 256) (&img[0][0])[e] = (unsigned char)e;
  __syncthreads();
  lds_u8* vb = (lds_u8*)(img[w] + lane * stride);
  unsigned acc = 0;
  for (int i = 0; i < ITERS; ++i) {
    unsigned x[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) x[j] = vb[(i & 15) * 8 + j];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += x[j];
  }
  if (acc == 12345u) out[threadIdx.x] = acc;
}

int main() {
  double* out;
  hipMalloc(&out, 1 << 20);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const char* names[] = {"v_fma_f64 indep", "v_mul_f64 indep", "v_add_f64 indep", "v_add_f64 dep chain", "v_lshl_add_u64 (u64 +)",
                         "v_dot4_u32_u8", "v_pk_mul_lo_u16", "v_dot2_u32_u16", "v_perm_b32",
                         "v_add_u32", "mad_u64_u32+lshrrev", "v_sad_u8", "v_cvt_f64_i32+xor", "v_add_u32_sdwa", "v_cndmask_b32"};
  // VALU instructions per element and step, as the gfx950 ISA of each loop has them (the
  // u64 add is one v_lshl_add_u64; ops 10 and 12 time a pair of different instructions)
  const int per[] = {1, 1, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2};
  for (int op = 0; op < 15; ++op) {
    for (int wps = 1; wps <= 8; wps *= 2) {
      const int blocks = cus * wps;  // 4 waves per block = one per SIMD
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(a);
        switch (op) {
          case 0: hipLaunchKernelGGL(k_valu<0>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001); break;
          case 1: hipLaunchKernelGGL(k_valu<1>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001); break;
          case 2: hipLaunchKernelGGL(k_valu<2>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001); break;
          case 3: hipLaunchKernelGGL(k_valu<3>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001); break;
          case 4: hipLaunchKernelGGL(k_valu<4>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001); break;
          case 5: hipLaunchKernelGGL(k_valu<5>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001); break;
          case 6: hipLaunchKernelGGL(k_valu<6>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001); break;
          case 7: hipLaunchKernelGGL(k_valu<7>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001); break;
          case 8: hipLaunchKernelGGL(k_valu<8>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001); break;
          case 9: hipLaunchKernelGGL(k_valu<9>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001); break;
          case 10: hipLaunchKernelGGL(k_valu<10>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001); break;
          case 11: hipLaunchKernelGGL(k_valu<11>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001); break;
          case 12: hipLaunchKernelGGL(k_valu<12>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001); break;
          case 13: hipLaunchKernelGGL(k_valu<13>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001); break;
          case 14: hipLaunchKernelGGL(k_valu<14>, dim3(blocks), dim3(256), 0, 0, out, 1.0000001); break;
        }
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        if (rep == 1) {
          // wave-instructions per SIMD: wps waves x ITERS x 8 (op 4: 2 VALU per element)
          const double ins = (double)wps * ITERS * 8 * per[op];
          const double cyc = ms * 1e-3 * 2.4e9;
          printf("%-22s waves/SIMD %d: %.2f cycles per wave-instruction per SIMD (at 2.4 GHz)\n",
                 names[op], wps, cyc / ins);
        }
      }
    }
  }
  for (int stride = 132; stride <= 136; stride += 4) {
    for (int wps = 1; wps <= 8; wps *= 2) {
      const int blocks = cus * wps;
      for (int rep = 0; rep < 2; ++rep) {
        hipEventRecord(a);
        hipLaunchKernelGGL(k_ds_u8, dim3(blocks), dim3(256), 0, 0, out, stride);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        if (rep == 1) {
          const double ins = (double)4 * wps * ITERS * 8;  // per CU
          printf("ds_read_u8 stride %d waves/SIMD %d: %.2f cycles per wave-instruction per CU\n",
                 stride, wps, ms * 1e-3 * 2.4e9 / ins);
        }
      }
    }
  }
  return 0;
}
