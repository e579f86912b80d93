// Accuracy of the raw gfx950 v_rcp_f64 / v_rsq_f64 (the seeds of the Markstein quotient and the
// Goldschmidt square roots in airice_device.hpp): writes x, rcp(x), rsq(x) for random x; the
// host side (tools/rcp_rsq_accuracy.py) measures the relative errors in long double.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>

__global__ void k(const double* x, double* r, double* s, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    r[i] = __builtin_amdgcn_rcp(x[i]);
    s[i] = __builtin_amdgcn_rsq(x[i]);
  }
}

int main(int argc, char** argv) {
  const int n = 1 << 22;
  std::vector<double> x(n), r(n), s(n);
  std::mt19937_64 g(1);
  std::uniform_real_distribution<double> u(-30.0, 30.0);
  for (int i = 0; i < n; ++i) x[i] = std::exp2(u(g));
  double *dx, *dr, *ds;
  hipMalloc(&dx, n * 8); hipMalloc(&dr, n * 8); hipMalloc(&ds, n * 8);
  hipMemcpy(dx, x.data(), n * 8, hipMemcpyHostToDevice);
  k<<<(n + 255) / 256, 256>>>(dx, dr, ds, n);
  hipMemcpy(r.data(), dr, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(s.data(), ds, n * 8, hipMemcpyDeviceToHost);
  long double er = 0, es = 0;
  for (int i = 0; i < n; ++i) {
    long double X = x[i];
    long double e1 = fabsl((long double)r[i] * X - 1.0L);
    long double e2 = fabsl((long double)s[i] * (long double)s[i] * X - 1.0L) / 2;
    if (e1 > er) er = e1;
    if (e2 > es) es = e2;
  }
  printf("{\"n\": %d, \"rcp_max_rel\": %.3Le, \"rcp_bits\": %.2f, \"rsq_max_rel\": %.3Le, \"rsq_bits\": %.2f}\n",
         n, er, (double)-log2l(er), es, (double)-log2l(es));
  return 0;
}
