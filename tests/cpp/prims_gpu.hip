// Device math primitives of the ray kernels (airiceraytracing_amd/csrc/airice_device.hpp) on
// host-given inputs, for the accuracy checks of tests/test_device_prims.py:
//   prims_gpu in.bin out.bin n
// in.bin: n x {q, a, b, x} doubles; out.bin: n x {fast_sqrt(q), sqrt_rsqrt(q).s, .rs,
// div_pos(a, b), asin_fast(x), log_ratio(a, b)} doubles.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../airiceraytracing_amd/csrc/airice_device.hpp"

__global__ void prims_kernel(const double* in, double* out, long n) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double q = in[4 * i], a = in[4 * i + 1], b = in[4 * i + 2], x = in[4 * i + 3];
  double s, rs;
  airice::sqrt_rsqrt(q, s, rs);
  double* o = out + 6 * i;
  o[0] = airice::fast_sqrt(q);
  o[1] = s;
  o[2] = rs;
  o[3] = airice::div_pos(a, b);
  o[4] = airice::asin_fast(x);
  o[5] = airice::log_ratio(a, b);
}

int main(int argc, char** argv) {
  if (argc < 4) return 2;
  const long n = std::atol(argv[3]);
  std::vector<double> in(4 * n), out(6 * n);
  std::FILE* f = std::fopen(argv[1], "rb");
  if (!f || std::fread(in.data(), sizeof(double), 4 * n, f) != (size_t)(4 * n)) return 3;
  std::fclose(f);
  double *din = nullptr, *dout = nullptr;
  if (hipMalloc(&din, sizeof(double) * 4 * n) != hipSuccess) return 4;
  if (hipMalloc(&dout, sizeof(double) * 6 * n) != hipSuccess) return 4;
  if (hipMemcpy(din, in.data(), sizeof(double) * 4 * n, hipMemcpyHostToDevice) != hipSuccess) return 5;
  hipLaunchKernelGGL(prims_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, din, dout, n);
  if (hipMemcpy(out.data(), dout, sizeof(double) * 6 * n, hipMemcpyDeviceToHost) != hipSuccess) return 6;
  (void)hipFree(din);
  (void)hipFree(dout);
  f = std::fopen(argv[2], "wb");
  if (!f) return 7;
  std::fwrite(out.data(), sizeof(double), 6 * n, f);
  std::fclose(f);
  return 0;
}
