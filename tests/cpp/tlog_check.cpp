// CPU twin of the device logarithm (airice_tlog.hpp compiled by g++): writes tlog() of the
// deterministic inputs for the bit comparison with the GPU, and reports the error against
// long double logl over the finite, positive inputs.
//   tlog_check N seed out.bin [lean]   (lean: tlog_lean on the finite positive normal inputs)
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../airiceraytracing_amd/csrc/airice_tlog.hpp"
#include "tlog_inputs.hpp"

int main(int argc, char** argv) {
  if (argc < 4) return 2;
  const uint64_t n = std::strtoull(argv[1], nullptr, 10), seed = std::strtoull(argv[2], nullptr, 10);
  const bool lean = argc > 4 && std::string(argv[4]) == "lean";
  std::vector<double> y(n);
  double max_ulp = 0, worst_x = 0;
  // error in ulps of max(|log x|, 1): the absolute accuracy the ray kernels' log ratios need
  // (their outputs are differences of O(1) terms)
  double max_ulp1 = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const double x = tlog_input(i, seed);
    const bool normal = x >= 0x1p-1022 && x < __builtin_inf();
    y[i] = (lean && normal) ? airice::tlog_lean(x) : airice::tlog(x);
    if (x > 0 && std::isfinite(x)) {
      const long double ref = logl((long double)x);
      const double rd = (double)ref;
      if (rd == 0) continue;
      const double ulp = std::ldexp(1.0, std::ilogb(rd) - 52);
      const double e = (double)std::fabs((long double)y[i] - ref) / ulp;
      if (e > max_ulp) { max_ulp = e; worst_x = x; }
      const double e1 = (double)std::fabs((long double)y[i] - ref) / std::fmax(ulp, 0x1p-52);
      if (e1 > max_ulp1) max_ulp1 = e1;
    } else {
      const double ref = std::log(x);
      const bool same = (std::isnan(ref) && std::isnan(y[i])) || ref == y[i];
      if (!same) { std::printf("special mismatch x=%a got %a want %a\n", x, y[i], ref); return 1; }
    }
  }
  std::FILE* f = std::fopen(argv[3], "wb");
  if (!f) return 3;
  std::fwrite(y.data(), sizeof(double), n, f);
  std::fclose(f);
  std::printf("{\"n\": %llu, \"max_ulp\": %.4f, \"max_ulp_floor1\": %.4f, \"worst_x\": \"%a\"}\n",
              (unsigned long long)n, max_ulp, max_ulp1, worst_x);
  return 0;
}
