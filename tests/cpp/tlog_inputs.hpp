// Deterministic inputs for the tlog checks (CPU twin and GPU kernel generate the same set).
#pragma once
#include <cstdint>
#include <cstring>

__host__ __device__ static inline uint64_t tlog_splitmix(uint64_t& s) {
  uint64_t z = (s += 0x9e3779b97f4a7c15ULL);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

// i-th input: a quarter each of random bit patterns over positive normals, values near 1
// (|x-1| < 2^-6), values in [0.5, 4) (the range of the ray kernels' ratios) and denormals / specials.
__host__ __device__ static inline double tlog_input(uint64_t i, uint64_t seed) {
  uint64_t s = seed ^ (i * 0x632be59bd9b4e019ULL);
  const uint64_t u = tlog_splitmix(s);
  double x;
  switch (i & 3) {
    case 0: {
      uint64_t b = (u % (0x7fefffffffffffffULL - 0x0010000000000000ULL)) + 0x0010000000000000ULL;
      std::memcpy(&x, &b, 8);
      break;
    }
    case 1:
      x = 1.0 + ((double)(u >> 11) * 0x1p-53 - 0.5) * 0x1p-5;
      break;
    case 2:
      x = 0.5 + (double)(u >> 11) * 0x1p-53 * 3.5;
      break;
    default: {
      const uint64_t k = u % 16;
      if (k == 0) { x = 0.0; break; }
      if (k == 1) { x = -1.5; break; }
      if (k == 2) { x = __builtin_inf(); break; }
      if (k == 3) { x = __builtin_nan(""); break; }
      uint64_t b = (u >> 12) | 1;  // positive denormal
      std::memcpy(&x, &b, 8);
    }
  }
  return x;
}
