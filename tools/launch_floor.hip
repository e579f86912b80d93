// Debug probe (GPU box): the floor of a one-query call -- launch + stream synchronisation of a
// one-wave kernel on a non-blocking stream, with its argument in device memory or in pinned,
// device-mapped host memory (the scalar slot), and with a host spin on a flag the kernel writes
// instead of hipStreamSynchronize.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

__global__ void touch(const double* in, double* out) {
  if (threadIdx.x == 0) out[0] = in[0] + 1.0;
}
__global__ void touch_flag(const double* in, double* out, volatile unsigned* flag, unsigned seq) {
  if (threadIdx.x == 0) {
    out[0] = in[0] + 1.0;
    __threadfence_system();
    flag[0] = seq;
  }
}

template <class F>
double med_us(F f) {
  std::vector<double> t;
  for (int i = 0; i < 420; ++i) {
    auto a = std::chrono::steady_clock::now();
    f(i);
    auto b = std::chrono::steady_clock::now();
    if (i >= 20) t.push_back(std::chrono::duration<double, std::micro>(b - a).count());
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main() {
  hipStream_t st;
  (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  double *d, *h, *hd;
  unsigned *fh, *fd;
  (void)hipMalloc(&d, 64);
  (void)hipHostMalloc(&h, 64, hipHostMallocMapped);
  (void)hipHostGetDevicePointer((void**)&hd, h, 0);
  (void)hipHostMalloc(&fh, 64, hipHostMallocMapped);
  (void)hipHostGetDevicePointer((void**)&fd, fh, 0);
  fh[0] = 0;
  const double dev_arg = med_us([&](int) {
    hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, st, d, d + 1);
    (void)hipStreamSynchronize(st);
  });
  const double host_arg = med_us([&](int) {
    hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, st, hd, hd + 1);
    (void)hipStreamSynchronize(st);
  });
  const double spin = med_us([&](int i) {
    const unsigned seq = (unsigned)i + 1;
    hipLaunchKernelGGL(touch_flag, dim3(1), dim3(64), 0, st, hd, hd + 1, fd, seq);
    while (__atomic_load_n(&fh[0], __ATOMIC_ACQUIRE) != seq) {
    }
  });
  (void)hipStreamSynchronize(st);
  // the signal written by the command processor after the kernel (no kernel change), then a
  // stream synchronisation that finds the work done
  const double cp_write = med_us([&](int i) {
    const unsigned seq = 100000u + (unsigned)i;
    hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, st, hd, hd + 1);
    (void)hipStreamWriteValue32(st, fd, seq, 0);
    while (__atomic_load_n(&fh[0], __ATOMIC_ACQUIRE) != seq) {
    }
  });
  const double cp_write_sync = med_us([&](int i) {
    const unsigned seq = 200000u + (unsigned)i;
    hipLaunchKernelGGL(touch, dim3(1), dim3(64), 0, st, hd, hd + 1);
    (void)hipStreamWriteValue32(st, fd, seq, 0);
    while (__atomic_load_n(&fh[0], __ATOMIC_ACQUIRE) != seq) {
    }
    (void)hipStreamSynchronize(st);
  });
  (void)hipStreamSynchronize(st);
  std::printf("{\"cp_write_spin_us\": %.2f, \"cp_write_spin_then_sync_us\": %.2f}\n", cp_write,
              cp_write_sync);
  std::printf("{\"launch_sync_device_arg_us\": %.2f, \"launch_sync_mapped_arg_us\": %.2f, "
              "\"launch_spin_flag_us\": %.2f}\n", dev_arg, host_arg, spin);
  return 0;
}
