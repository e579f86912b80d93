// Occupancy probe: what the runtime says vs what the hardware holds (tools/, debug only).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int V, int S>
__global__ void spin(unsigned long long* out, long long cycles) {
  if (V == 1) asm volatile("v_mov_b32 v57, 0" ::: "v57");
  if (V == 2) asm volatile("v_mov_b32 v63, 0" ::: "v63");
  if (V == 3) asm volatile("v_mov_b32 v64, 0" ::: "v64");
  if (S == 1) asm volatile("s_mov_b32 s70, 0" ::: "s70");
  if (S == 2) asm volatile("s_mov_b32 s90, 0" ::: "s90");
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while ((long long)(__builtin_amdgcn_s_memrealtime() - t0) < cycles) {}
  if ((threadIdx.x & 63) == 0) {
    const unsigned hw = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));
    const unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));
    const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
    const size_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    out[3 * w] = t0;
    out[3 * w + 1] = t1;
    out[3 * w + 2] = ((unsigned long long)xcc << 32) | hw;
  }
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  int maxw = 0;
  hipDeviceGetAttribute(&maxw, hipDeviceAttributeMaxThreadsPerMultiProcessor, 0);
  printf("CUs %d max threads/CU %d\n", cus, maxw);
  const int bs = 256;
  void (*ks[])(unsigned long long*, long long) = {spin<0, 0>, spin<1, 0>, spin<2, 0>, spin<3, 0>,
                                                  spin<0, 1>, spin<0, 2>, spin<1, 1>};
  const char* names[] = {"plain", "v57", "v63", "v64", "s70", "s90", "v57+s70"};
  for (int ki = 0; ki < 7; ++ki) {
    auto spin_k = ks[ki];
    int nb = 0;
    hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, spin_k, bs, 0);
    // launch 10 waves per SIMD worth of blocks, each spinning 20 us: count concurrent waves
    const long long waves = 10LL * cus * 4;
    const int blocks = (int)(waves * 64 / bs);
    unsigned long long* d;
    hipMalloc(&d, sizeof(unsigned long long) * 3 * waves);
    hipLaunchKernelGGL(spin_k, dim3(blocks), dim3(bs), 0, 0, d, 2000);  // 20 us at 100 MHz
    hipDeviceSynchronize();
    unsigned long long* h = new unsigned long long[3 * waves];
    hipMemcpy(h, d, sizeof(unsigned long long) * 3 * waves, hipMemcpyDeviceToHost);
    unsigned long long tmin = ~0ULL;
    for (long long i = 0; i < waves; ++i) tmin = h[3 * i] < tmin ? h[3 * i] : tmin;
    // waves that started within the first 10 us = first round
    long long first = 0;
    for (long long i = 0; i < waves; ++i) first += (h[3 * i] - tmin) < 1000;
    printf("%-8s block %4d: occupancy API %d blocks/CU (%d waves/SIMD); first-round waves %lld "
           "= %.2f per SIMD\n", names[ki], bs, nb, nb * bs / 64 / 4, first, (double)first / (cus * 4));
    hipFree(d);
    delete[] h;
  }
  return 0;
}
