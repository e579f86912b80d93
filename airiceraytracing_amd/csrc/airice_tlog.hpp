// airice_tlog.hpp -- table-driven natural logarithm for the device (and, compiled by g++, its
// bit-exact CPU twin used by tests/cpp/tlog_check.cpp).
//
// x = 2^k z, z in [0.6875, 1.375) (bit offset 0x3fe6000000000000); i = top 8 bits of the offset
// mantissa; r = fma(z, 1/c_i, -1) (|r| <= 2^-8, one rounding); log x = k ln2 + log c_i + log1p(r)
// with log1p(r) - r by a degree-7 Taylor polynomial (truncation <= 2^-67) and the k ln2 + log c_i
// + r sum kept in hi + lo form.  No division; ~16 FP64 + ~6 integer VALU ops and one 16-byte table
// load (airice_logtab.h, tools/gen_log_table.py) against ~45 for the fdlibm form with its divide.
// Error < 1 ulp (tests/test_tlog.py measures it against mpmath on the CPU twin and checks that
// the GPU returns the same bits).
#pragma once

#include <cstdint>
#include <cstring>

#ifndef __HIPCC__
#include <cmath>
#define __host__
#define __device__
#define AIRICE_FMA(a, b, c) std::fma((a), (b), (c))
#define AIRICE_INLINE inline
#else
#define AIRICE_FMA(a, b, c) __builtin_fma((a), (b), (c))
#define AIRICE_INLINE __forceinline__
#endif

#include "airice_logtab.h"

namespace airice {

// A polynomial coefficient held in an SGPR pair: the fma then issues as one VOP3 v_fma_f64 with the
// scalar operand, instead of two v_mov_b32 materialising the constant for v_fmac_f64 (what the
// compiler otherwise emits for Horner steps).  Value unchanged.
#if defined(__HIP_DEVICE_COMPILE__)
__device__ __forceinline__ double kc(double c) {
  asm("" : "+s"(c));
  return c;
}
#else
__host__ __device__ AIRICE_INLINE constexpr double kc(double c) { return c; }
#endif

__host__ __device__ AIRICE_INLINE uint64_t dbits(double x) {
  uint64_t u;
  std::memcpy(&u, &x, sizeof(u));
  return u;
}

__host__ __device__ AIRICE_INLINE double bitsd(uint64_t u) {
  double x;
  std::memcpy(&x, &u, sizeof(x));
  return x;
}

// log(x) for x positive, normal and finite.  `tab` is kLogTable or a copy of it (the table
// kernel stages it in LDS); any other x returns garbage without reading outside the table.
__host__ __device__ AIRICE_INLINE double tlog_pos(double x, const double* tab = &kLogTable[0][0]) {
  const double Ln2hi = 0x1.62e42fefa3800p-1;  // ln 2 with 11 low zero bits: k*Ln2hi is exact
  const double Ln2lo = 0x1.ef35793c76730p-45;
  const double A0 = -0x1p-1, A1 = 0x1.5555555555555p-2, A2 = -0x1p-2, A3 = 0x1.999999999999ap-3,
               A4 = -0x1.5555555555555p-3, A5 = 0x1.2492492492492p-3;  // -1/2, 1/3, ..., 1/7
  // the reduction touches only the high word (the offset has a zero low word); 32-bit integer
  // ops throughout so the exponent converts with one v_cvt_f64_i32
  const uint64_t ix = dbits(x);
  const uint32_t hx = (uint32_t)(ix >> 32);
  const uint32_t htmp = hx - 0x3fe60000u;
  const int i = (int)((htmp >> (20 - kLogTableBits)) & ((1u << kLogTableBits) - 1));
  const int k = (int32_t)htmp >> 20;
  const double z = bitsd(((uint64_t)(hx - (htmp & 0xfff00000u)) << 32) | (ix & 0xffffffffULL));
  const double invc = tab[2 * i], logc = tab[2 * i + 1];
  const double r = AIRICE_FMA(z, invc, -1.0);
  const double kd = (double)k;
  // w = k Ln2hi + logc in hi + lo form: k Ln2hi is exact and, when k != 0, larger than |logc|
  // (< 0.38), so Fast2Sum gives the rounding error of w exactly
  const double t = kd * Ln2hi;
  const double w = t + logc;
  const double we = (t - w) + logc;
  const double hi = w + r;
  const double lo = AIRICE_FMA(kd, Ln2lo, ((w - hi) + r) + we);
  const double r2 = r * r;
  // Horner: one constant per fma (no constant materialised in VGPRs but A5)
  double q = AIRICE_FMA(r, A5, kc(A4));
  q = AIRICE_FMA(r, q, kc(A3));
  q = AIRICE_FMA(r, q, kc(A2));
  q = AIRICE_FMA(r, q, kc(A1));
  q = AIRICE_FMA(r, q, kc(A0));
  return AIRICE_FMA(r2, q, lo) + hi;
}

// log(x) for x positive, normal and finite, without the hi + lo bookkeeping: w = k ln2 + log c_i
// by one fma, then w + (r + r^2 q) with q of degree 3 in r.  ~8 FP64 ops
// instead of ~19.  Error bounded in ABSOLUTE terms: <= ~3 ulp of max(|log x|, 1) at degree 5
// (truncation |r|^6/6 <= 2^-50.6 for |r| <= 2^-8, plus the roundings of w and the final sum;
// 2 ulp at degree 7), measured in tests/test_tlog.py.  The ray kernels' log ratios use this
// form: their outputs are built from differences of O(1) terms, so the absolute error of one
// logarithm is what reaches them.
__host__ __device__ AIRICE_INLINE double tlog_lean(double x, const double* tab = &kLogTable[0][0]) {
  const double Ln2 = 0x1.62e42fefa39efp-1;
  const double A0 = -0x1p-1, A1 = 0x1.5555555555555p-2, A2 = -0x1p-2, A3 = 0x1.999999999999ap-3;
  const uint64_t ix = dbits(x);
  const uint32_t hx = (uint32_t)(ix >> 32);
  const uint32_t htmp = hx - 0x3fe60000u;
  const int k = (int32_t)htmp >> 20;
  const double z = bitsd(((uint64_t)(hx - (htmp & 0xfff00000u)) << 32) | (ix & 0xffffffffULL));
  // the table address as one shift and one mask of the high word (the byte offset of entry i)
  const uint32_t off = (htmp >> (20 - kLogTableBits - 4)) & (((1u << kLogTableBits) - 1) << 4);
  const double* ent = reinterpret_cast<const double*>(reinterpret_cast<const char*>(tab) + off);
  const double invc = ent[0], logc = ent[1];
  const double r = AIRICE_FMA(z, invc, -1.0);
  const double w = AIRICE_FMA((double)k, Ln2, logc);
  const double r2 = r * r;
  // through r^5: truncation |r|^6 / 6 <= 2^-50.6 absolute (degree 7 measured 2.8 % slower on
  // the cfg2 table with the float table bit-identical; an Estrin form no faster than Horner)
  double q = AIRICE_FMA(r, kc(A3), kc(A2));
  q = AIRICE_FMA(r, q, kc(A1));
  q = AIRICE_FMA(r, q, kc(A0));
  return AIRICE_FMA(r2, q, r) + w;
}

// log(x) for any x with log()'s IEEE special values: denormals are scaled by 2^54 (exact) and
// 0 / negative / NaN / inf are selected at the end, so the code is branch-free.
__host__ __device__ AIRICE_INLINE double tlog(double x_in) {
  const bool tiny = x_in < 0x1p-1022;
  const double x = tiny ? x_in * 0x1p54 : x_in;
  const double y = tlog_pos(x) - (tiny ? 54 * 0x1.62e42fefa39efp-1 : 0.0);
  const double inf = __builtin_inf();
  const double special = (x_in == 0.0) ? -inf : (x_in > 0.0 ? x_in : __builtin_nan(""));
  return (x_in > 0.0 && x_in < inf) ? y : special;
}

}  // namespace airice
