// phcx_io_driver.cpp — host-only driver of the native PHCX reader (include/pfe_io.h) for the
// ASan + UBSan build in tests/test_phcx_sanitize.py.  Parses the files named on the command
// line with several threads, fetches every field of every parsed file, packs all parsed
// files that share the first parsed file's shape, and prints one line per file:
//   <index> <status> <lp> <nsub> <lsb> <ndm> <ld> <lfit> <fnv64 of the fetched fields>
// so that the test can compare the sanitized reader's results with the product library's.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "pfe_io.h"

static uint64_t fnv(uint64_t h, const void* p, size_t n) {
  const unsigned char* c = static_cast<const unsigned char*>(p);
  for (size_t i = 0; i < n; ++i) h = (h ^ c[i]) * 1099511628211ull;
  return h;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: %s <threads> <file>...\n", argv[0]);
    return 2;
  }
  const int threads = std::atoi(argv[1]);
  const int64_t n = argc - 2;
  pfe_phcx_batch* b = nullptr;
  if (pfe_phcx_parse(argv + 2, n, -1, threads, &b) != 0 || !b) return 3;
  if (pfe_phcx_count(b) != n) return 4;
  std::vector<int64_t> rows;
  pfe_phcx_info first{};
  for (int64_t i = 0; i < n; ++i) {
    pfe_phcx_info inf{};
    if (pfe_phcx_info_get(b, i, &inf) != 0) return 5;
    uint64_t h = 1469598103934665603ull;
    if (inf.status == PFE_IO_OK) {
      const int64_t caps[5] = {inf.lp, inf.ld, (int64_t)inf.nsub * inf.lsb, inf.ndm, inf.lfit};
      for (int f = 0; f < 5; ++f) {
        const size_t esz = f == PFE_PHCX_DM_CURVE ? sizeof(double) : 1;
        std::vector<unsigned char> buf((size_t)caps[f] * esz + 1);
        if (pfe_phcx_fetch(b, i, f, buf.data(), caps[f]) != 0) return 6;
        h = fnv(h, buf.data(), (size_t)caps[f] * esz);
        // one element too few must be refused, never written past
        if (caps[f] > 0 && pfe_phcx_fetch(b, i, f, buf.data(), caps[f] - 1) == 0) return 7;
      }
      h = fnv(h, inf.scal, sizeof(inf.scal));
      if (rows.empty()) first = inf;
      if (inf.lp == first.lp && inf.ld == first.ld && inf.nsub == first.nsub &&
          inf.lsb == first.lsb && inf.ndm == first.ndm)
        rows.push_back(i);
    }
    std::printf("%lld %d %d %d %d %d %lld %lld %016llx\n", (long long)i, inf.status, inf.lp,
                inf.nsub, inf.lsb, inf.ndm, (long long)inf.ld, (long long)inf.lfit,
                (unsigned long long)h);
  }
  // out-of-range queries are refused
  pfe_phcx_info junk{};
  if (pfe_phcx_info_get(b, n, &junk) == 0 || pfe_phcx_info_get(b, -1, &junk) == 0) return 8;
  if (!rows.empty()) {
    const int64_t r = (int64_t)rows.size();
    const int64_t sl = (int64_t)first.nsub * first.lsb;
    std::vector<uint8_t> prof(r * first.lp), dm(r * first.ld), sub(r * sl);
    std::vector<double> dmc(r * (first.ndm > 0 ? first.ndm : 1)), scal(r * 8);
    if (pfe_phcx_pack(b, rows.data(), r, threads, prof.data(), first.lp, dm.data(), first.ld,
                      sub.data(), sl, dmc.data(), first.ndm > 0 ? first.ndm : 1, scal.data()) != 0)
      return 9;
    // strides one short must be refused
    if (first.lp > 0 && pfe_phcx_pack(b, rows.data(), r, threads, prof.data(), first.lp - 1,
                                      nullptr, 0, nullptr, 0, nullptr, 0, nullptr) == 0)
      return 10;
    uint64_t h = fnv(1469598103934665603ull, prof.data(), prof.size());
    h = fnv(h, sub.data(), sub.size());
    h = fnv(h, dmc.data(), dmc.size() * sizeof(double));
    std::printf("pack %lld %016llx\n", (long long)r, (unsigned long long)h);
  }
  pfe_phcx_free(b);
  return 0;
}
