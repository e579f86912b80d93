// GPU side of the tlog check: the device tlog() (airice_tlog.hpp, as the kernels inline it) over
// the same deterministic inputs as tests/cpp/tlog_check.cpp, written for a bitwise comparison.
//   tlog_gpu N seed out.bin [lean]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../airiceraytracing_amd/csrc/airice_tlog.hpp"
#include "tlog_inputs.hpp"

__global__ void tlog_kernel(uint64_t n, uint64_t seed, int lean, double* y) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    const double x = tlog_input(i, seed);
    const bool normal = x >= 0x1p-1022 && x < __builtin_inf();
    y[i] = (lean && normal) ? airice::tlog_lean(x) : airice::tlog(x);
  }
}

int main(int argc, char** argv) {
  if (argc < 4) return 2;
  const uint64_t n = std::strtoull(argv[1], nullptr, 10), seed = std::strtoull(argv[2], nullptr, 10);
  const int lean = argc > 4 && argv[4][0] == 'l';
  double* d = nullptr;
  if (hipMalloc(&d, sizeof(double) * n) != hipSuccess) return 3;
  hipLaunchKernelGGL(tlog_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, n, seed, lean, d);
  std::vector<double> y(n);
  if (hipMemcpy(y.data(), d, sizeof(double) * n, hipMemcpyDeviceToHost) != hipSuccess) return 4;
  (void)hipFree(d);
  std::FILE* f = std::fopen(argv[3], "wb");
  if (!f) return 5;
  std::fwrite(y.data(), sizeof(double), n, f);
  std::fclose(f);
  return 0;
}
