// VALU issue-rate calibration on the GPU box (not part of the library): throughput of FP64 FMA,
// v_rcp_f64 / v_rsq_f64, 32-bit integer ops and v_cndmask chains at 8 waves/SIMD over the whole
// chip, timed with HIP events.  Prints one line per probe: wave-instructions/s per SIMD and
// cycles per wave-instruction at the clock implied by the FP64 FMA probe's 4-cycle issue.
//   hipcc -O3 --offload-arch=gfx950 -o tools/valu_rates tools/valu_rates.hip && tools/valu_rates
#include <hip/hip_runtime.h>

#include <cstdio>

#define CHECK(x)                                                              \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      return 1;                                                               \
    }                                                                         \
  } while (0)

constexpr int kIters = 2048;
constexpr int kChains = 8;

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void fma_probe(
    double* out, double s) {
  double a[kChains];
#pragma unroll
  for (int c = 0; c < kChains; ++c) a[c] = threadIdx.x * 1e-3 + c;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int c = 0; c < kChains; ++c) a[c] = __builtin_fma(a[c], s, 0.5);
  }
  double r = 0;
#pragma unroll
  for (int c = 0; c < kChains; ++c) r += a[c];
  if (r == 12345.0) out[threadIdx.x] = r;
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void fma_dep_probe(
    double* out, double s) {
  double a = threadIdx.x * 1e-3;
  for (int i = 0; i < kIters * kChains; ++i) a = __builtin_fma(a, s, 0.5);
  if (a == 12345.0) out[threadIdx.x] = a;
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void rcp_probe(
    double* out, double s) {
  double a[kChains];
#pragma unroll
  for (int c = 0; c < kChains; ++c) a[c] = threadIdx.x * 1e-3 + c + 1;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int c = 0; c < kChains; ++c) a[c] = __builtin_amdgcn_rcp(a[c]);
  }
  double r = 0;
#pragma unroll
  for (int c = 0; c < kChains; ++c) r += a[c];
  if (r == 12345.0) out[threadIdx.x] = r;
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void rsq_probe(
    double* out, double s) {
  double a[kChains];
#pragma unroll
  for (int c = 0; c < kChains; ++c) a[c] = threadIdx.x * 1e-3 + c + 1;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int c = 0; c < kChains; ++c) a[c] = __builtin_amdgcn_rsq(a[c]);
  }
  double r = 0;
#pragma unroll
  for (int c = 0; c < kChains; ++c) r += a[c];
  if (r == 12345.0) out[threadIdx.x] = r;
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void int_probe(
    double* out, double s) {
  unsigned a[kChains];
#pragma unroll
  for (int c = 0; c < kChains; ++c) a[c] = threadIdx.x * 7u + c;
  const unsigned k = (unsigned)s;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int c = 0; c < kChains; ++c) a[c] = (a[c] ^ k) + 0x9e3779b9u;  // v_xor + v_add
  }
  unsigned r = 0;
#pragma unroll
  for (int c = 0; c < kChains; ++c) r += a[c];
  if (r == 12345u) out[threadIdx.x] = r;
}

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void mix_probe(
    double* out, double s) {
  // one FP64 fma + two 32-bit ops per chain step: does 32-bit work hide under FP64 issue?
  double a[kChains];
  unsigned b[kChains];
#pragma unroll
  for (int c = 0; c < kChains; ++c) {
    a[c] = threadIdx.x * 1e-3 + c;
    b[c] = threadIdx.x + c;
  }
  const unsigned k = (unsigned)s;
  for (int i = 0; i < kIters; ++i) {
#pragma unroll
    for (int c = 0; c < kChains; ++c) {
      a[c] = __builtin_fma(a[c], s, 0.5);
      b[c] = (b[c] ^ k) + 0x9e3779b9u;  // v_xor_b32 + v_add_u32
    }
  }
  double r = 0;
#pragma unroll
  for (int c = 0; c < kChains; ++c) r += a[c] + b[c];
  if (r == 12345.0) out[threadIdx.x] = r;
}

int main() {
  double* out;
  CHECK(hipMalloc(&out, 4096 * sizeof(double)));
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  const int blocks = cus * 8 * 16;  // 8 blocks (32 waves) per CU resident, 16 rounds
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  struct Probe {
    const char* name;
    void (*k)(double*, double);
    double insts_per_iter;  // wave-instructions per lane-iteration of the probed kind
  } probes[] = {
      {"fp64_fma_indep8", fma_probe, 1.0},  {"fp64_fma_dep1", fma_dep_probe, 1.0},
      {"fp64_rcp", rcp_probe, 1.0},         {"fp64_rsq", rsq_probe, 1.0},
      {"u32_xor_add", int_probe, 2.0},      {"fma+u32mad", mix_probe, 1.0},
  };
  double clk_ghz = 0;
  for (auto& pr : probes) {
    for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(pr.k, dim3(blocks), dim3(256), 0, 0, out, 1.0000001);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    const int reps = 5;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(pr.k, dim3(blocks), dim3(256), 0, 0, out, 1.0000001);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    const double s = ms * 1e-3 / reps;
    const double waves = blocks * 4.0;
    const double wave_insts = waves * (double)kIters * kChains * pr.insts_per_iter;
    const double simds = cus * 4.0;
    const double per_simd = wave_insts / simds / s;  // wave-instructions per second per SIMD
    if (clk_ghz == 0) clk_ghz = per_simd * 4.0 / 1e9;  // FP64 FMA: 4 cycles per wave64 instruction
    std::printf("%-16s %8.3f ms  %.4g wave-inst/s/SIMD  %.2f cyc/inst at %.3f GHz  lane-ops %.4g /s\n",
                pr.name, s * 1e3, per_simd, clk_ghz * 1e9 / per_simd, clk_ghz,
                wave_insts * 64 / s);
  }
  return 0;
}
