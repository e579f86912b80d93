// Golden rows of the cfg3 / cfg5 query generators (tests/parity.py mt19937_64_uniform):
// std::mt19937_64 + std::uniform_real_distribution<double> under libstdc++.
//   g++ -O2 -o /tmp/make_mt_golden tests/golden/make_mt_golden.cpp && /tmp/make_mt_golden \
//     > tests/golden/mt19937_64_golden.json
#include <cstdio>
#include <random>

int main() {
  std::printf("{\n \"cfg3_seed12345\": [\n");
  {
    std::mt19937_64 g(12345);
    std::uniform_real_distribution<double> uh(3001, 100000), ud(0, 50000), uz(0, 300);
    for (int i = 0; i < 400; ++i) {
      const double a = uh(g), b = ud(g), c = -uz(g);
      std::printf("  [%.17g, %.17g, %.17g]%s\n", a, b, c, i < 399 ? "," : "");
    }
  }
  std::printf(" ],\n \"cfg5_seed777\": [\n");
  {
    std::mt19937_64 g(777);
    std::uniform_real_distribution<double> uz(1, 300), uh(3001, 20000), ud(0, 30000);
    for (int i = 0; i < 400; ++i) {
      const double a = -uz(g), b = uh(g), c = ud(g);
      std::printf("  [%.17g, %.17g, %.17g]%s\n", a, b, c, i < 399 ? "," : "");
    }
  }
  std::printf(" ]\n}\n");
  return 0;
}
