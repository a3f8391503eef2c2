/* ORACLE (test infrastructure only) -- C restatement of the 8 Lyon features, OpenMP over
 * candidates.  Only tests/ and bench.py's cpu_baseline leg load it (as a checker / the
 * multi-core CPU baseline of SURVEY.md section 8(d)(ii)); the product path never does.
 *
 * Per row, what PHCXFile.computeProfileStatScores / computeDMCurveStatScores compute
 * (PulsarFeatureExtractor/src/PHCXFile.py:320-379): numpy.mean, numpy.std (ddof 0),
 * scipy.stats.skew and scipy.stats.kurtosis (biased, Fisher), with scipy's zero-variance
 * rule m2 <= (eps * mean)^2 -> NaN.  Two-pass float64 moments, summed sequentially; the sum
 * of a uint8 row is an exact integer, so the mean agrees with numpy to the last bit, and so
 * does the std for power-of-two row lengths (all squared deviations and partial sums are then
 * exact); otherwise, and for skew / kurtosis, within 1e-12 (tests/test_oracle_c.py).
 */
#include <math.h>
#include <stdint.h>

static void stats_u8(const uint8_t* x, int n, double* o) {
  long long s = 0;
  for (int i = 0; i < n; ++i) s += x[i];
  const double mean = (double)s / (double)n;
  double m2 = 0.0, m3 = 0.0, m4 = 0.0;
  for (int i = 0; i < n; ++i) {
    const double d = (double)x[i] - mean;
    const double d2 = d * d;
    m2 += d2;
    m3 += d2 * d;
    m4 += d2 * d2;
  }
  m2 /= (double)n;
  m3 /= (double)n;
  m4 /= (double)n;
  const double e = 2.220446049250313e-16 * mean;
  const int zero = m2 <= e * e;
  o[0] = mean;
  o[1] = sqrt(m2);
  o[2] = zero ? NAN : m3 / pow(m2, 1.5);
  o[3] = zero ? NAN : m4 / (m2 * m2) - 3.0;
}

/* prof: n x lp, dm: n x ld (row-major uint8); out: n x 8; threads <= 0: OpenMP default */
int pfe_oracle_lyon8_u8(const uint8_t* prof, int lp, const uint8_t* dm, int ld, long long n,
                        double* out, int threads) {
  if (n < 0 || lp <= 0 || ld <= 0) return -1;
#pragma omp parallel for schedule(static) num_threads(threads > 0 ? threads : 1) if (threads != 1)
  for (long long i = 0; i < n; ++i) {
    stats_u8(prof + i * lp, lp, out + i * 8);
    stats_u8(dm + i * ld, ld, out + i * 8 + 4);
  }
  return 0;
}
