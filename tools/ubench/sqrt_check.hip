// sqrt_rn (wave.h) against the compiler's sqrt, bit for bit, over random doubles of every
// exponent (and a contracted caller, as the LM solvers compile it).  hipcc --offload-arch=gfx950
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>
#include <vector>
#include "../../pulsarfeatureextractor_amd/csrc/wave.h"
using namespace pfe;
__global__ void k(const double* x, double* a, double* b, double* c, double* d, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  a[i] = sqrt(x[i]);
  b[i] = sqrt_rn(x[i]);
  {
    _Pragma("clang fp contract(fast)")
    c[i] = 3.0 * sqrt(x[i]) + x[i];
    d[i] = 3.0 * sqrt_rn(x[i]) + x[i];
  }
}
static uint64_t s = 0x9E3779B97F4A7C15ull;
static uint64_t nx() { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
int main() {
  const int n = 1 << 24;
  std::vector<double> x(n);
  for (int i = 0; i < n; ++i) {
    uint64_t m = nx() & ((1ull << 52) - 1);
    int e = (int)(nx() % 2046) + 1;               // every normal exponent
    if (i % 8 == 1) e = 1023 + (int)(nx() % 80) - 40;  // the fits' usual range
    uint64_t bits = ((uint64_t)e << 52) | m;
    if (i % 64 == 3) bits = nx() & ((1ull << 52) - 1);  // subnormals
    std::memcpy(&x[i], &bits, 8);
  }
  x[0] = 0.0; x[5] = -1.0; x[6] = 1.0 / 0.0;
  double *dx, *da, *db, *dc, *dd;
  hipMalloc(&dx, n * 8); hipMalloc(&da, n * 8); hipMalloc(&db, n * 8); hipMalloc(&dc, n * 8); hipMalloc(&dd, n * 8);
  hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
  k<<<n / 256, 256>>>(dx, da, db, dc, dd, n);
  std::vector<double> a(n), b(n), c(n), d(n);
  hipMemcpy(a.data(), da, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(b.data(), db, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(c.data(), dc, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(d.data(), dd, n * 8, hipMemcpyDeviceToHost);
  long bad = 0, badc = 0;
  for (int i = 0; i < n; ++i) {
    if (std::memcmp(&a[i], &b[i], 8) != 0) { if (bad < 5) printf("sqrt  x=%a sqrt=%a sqrt_rn=%a\n", x[i], a[i], b[i]); ++bad; }
    if (std::memcmp(&c[i], &d[i], 8) != 0) { if (badc < 5) printf("contr x=%a sqrt=%a sqrt_rn=%a\n", x[i], c[i], d[i]); ++badc; }
  }
  printf("n %d mismatches %ld contracted %ld\n", n, bad, badc);
  return bad || badc;
}
