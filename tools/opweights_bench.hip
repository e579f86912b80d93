// opweights_bench.hip -- measures the executed FP64 VALU cost of each ocml function on
// gfx950.  One kernel per function: every lane evaluates f on 16 arguments in the range
// the ray solver uses and accumulates; a baseline kernel does the same loop without f.
// Run under `rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 ... SQ_WAVES`; per call
// cost = (counter_f - counter_base) / (waves * 16).  tools/measure_opweights.py drives it.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

#define KERNEL(NAME, EXPR)                                                           \
  __global__ __launch_bounds__(256) void k_##NAME(const double* __restrict__ in,    \
                                                  double* __restrict__ out) {       \
    const int i = blockIdx.x * 256 + threadIdx.x;                                    \
    const double a0 = in[i];                                                         \
    double acc = 0.0;                                                                \
    _Pragma("unroll 1") for (int k = 0; k < 16; ++k) {                               \
      const double a = a0 + k * 1.0e-3;                                              \
      acc += (EXPR);                                                                 \
    }                                                                                \
    out[i] = acc;                                                                    \
  }

KERNEL(base, a)
KERNEL(exp, exp(-a))
KERNEL(log, log(1.0 + a))
KERNEL(sqrt, sqrt(a))
KERNEL(asin, asin(0.9 * a))
KERNEL(sin, sin(1.5 * a))
KERNEL(cos, cos(1.5 * a))
KERNEL(atan, atan(30.0 * a))
KERNEL(div, 1.2345 / (0.5 + a))

int main() {
  const int n = 256 * 1024;
  std::vector<double> h(n);
  for (int i = 0; i < n; ++i) h[i] = 0.05 + 0.9 * (double)((i * 2654435761u) % 1000003u) / 1000003.0;
  double *din, *dout;
  if (hipMalloc(&din, n * sizeof(double)) != hipSuccess) return 1;
  if (hipMalloc(&dout, n * sizeof(double)) != hipSuccess) return 1;
  if (hipMemcpy(din, h.data(), n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) return 1;
  dim3 g(n / 256), b(256);
  hipLaunchKernelGGL(k_base, g, b, 0, 0, din, dout);
  hipLaunchKernelGGL(k_exp, g, b, 0, 0, din, dout);
  hipLaunchKernelGGL(k_log, g, b, 0, 0, din, dout);
  hipLaunchKernelGGL(k_sqrt, g, b, 0, 0, din, dout);
  hipLaunchKernelGGL(k_asin, g, b, 0, 0, din, dout);
  hipLaunchKernelGGL(k_sin, g, b, 0, 0, din, dout);
  hipLaunchKernelGGL(k_cos, g, b, 0, 0, din, dout);
  hipLaunchKernelGGL(k_atan, g, b, 0, 0, din, dout);
  hipLaunchKernelGGL(k_div, g, b, 0, 0, din, dout);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  std::printf("opweights_bench: %d lanes x 16 evaluations per kernel\n", n);
  (void)hipFree(din);
  (void)hipFree(dout);
  return 0;
}
