// airice_lookup.hip -- batched GetHorizontalDistanceToIntersectionPoint_Table on gfx950.
//
//  lookup_kernel : one lane per (Tx height, horizontal distance, Rx depth) query against one
//                  antenna's HBM-resident table (11 float columns, SoA).  The lane runs the
//                  reference's bin search and two-level linear interpolation:
//                    FindClosestAirTxHeight (.cc:1033-1126)  row of the Tx height and the
//                                                            valid-THD span of that row,
//                    FindClosestTHD         (.cc:1128-1169)  8 bisection steps + linear scan,
//                    GetParValues           (.cc:1172-1302)  10 columns at 2 heights
//                                                            (one 48-byte packed record per
//                                                            entry when the table is packed),
//                    _Table                 (.cc:1305-1462)  interpolation in height, checks.
//                  Lanes that hit the one-sided extrapolation case (.cc:1418) are flagged and
//                  finished by the masked minimizer pass (launch_lookup_fallback,
//                  airice_kernels.hip), which reproduces the reference's fallback call.
//
// Cost model: ~20-40 dependent 4-byte gathers per query (2 rows x (bisection over ~900
// THD entries + 10 columns x 2 entries)), so the kernel is gather-latency bound; the table
// (11 x 4 B x rays, ~38 MB for the default grid) stays L2/MALL-resident across a batch.
// Reads the reference makes outside the table (a row with no valid THD, index -1 in
// FindClosestTHD) are bounded here and reported as AIRICE_LOOKUP_UNPINNED.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "airice.h"
#include "airice_internal.h"

namespace airice {
namespace {

constexpr int kLkBlock = 256;

struct LkTable {
  const float* t;
  const float* e;  // packed entries (airice_lookup_pack) or nullptr
  long long ld, n;
  double stop_h, step_h;
  int hsteps, asteps;
};

// One table entry's 11 columns, from the packed copy when there is one (three 16-byte loads of
// one 48-byte record) or else column by column.  Out-of-range entries: NaN, flagged, as lk_at.
struct LkRec {
  float c[AIRICE_LOOKUP_ENTRY_FLOATS];
};

__device__ __forceinline__ LkRec lk_rec(const LkTable& T, long long i, int& fl) {
  LkRec r;
  if (i < 0 || i >= T.n) {
    fl |= AIRICE_LOOKUP_UNPINNED;
#pragma unroll
    for (int c = 0; c < AIRICE_LOOKUP_ENTRY_FLOATS; ++c) r.c[c] = __builtin_nanf("");
    return r;
  }
  if (T.e != nullptr) {
    const float4* p = reinterpret_cast<const float4*>(T.e + (long long)AIRICE_LOOKUP_ENTRY_FLOATS * i);
    const float4 a = p[0], b = p[1], d = p[2];
    r.c[0] = a.x, r.c[1] = a.y, r.c[2] = a.z, r.c[3] = a.w;
    r.c[4] = b.x, r.c[5] = b.y, r.c[6] = b.z, r.c[7] = b.w;
    r.c[8] = d.x, r.c[9] = d.y, r.c[10] = d.z, r.c[11] = d.w;
    return r;
  }
#pragma unroll
  for (int c = 0; c < 11; ++c) r.c[c] = T.t[(long long)c * T.ld + i];
  r.c[11] = 0.0f;
  return r;
}

__device__ __forceinline__ double lk_at(const LkTable& T, int c, long long i, int& fl) {
  if (i < 0 || i >= T.n) {
    fl |= AIRICE_LOOKUP_UNPINNED;
    return __builtin_nan("");
  }
  return (double)T.t[(long long)c * T.ld + i];
}

// oneDLinearInterpolation (.cc:992-995)
__device__ __forceinline__ double lk_interp(double x, double xa, double ya, double xb, double yb) {
  return ya + (yb - ya) * ((x - xa) / (xb - xa));
}

// FindClosestAirTxHeight (.cc:1033-1126): the row of height P and the span of entries with a
// usable THD (not NaN, not in (−inf, 0.01) except exactly 0), scanned inwards from both ends.
struct TxhBins {
  long long s1, e1, s2, e2;
  double c1;
};

__device__ __forceinline__ TxhBins closest_txh(const LkTable& T, double P, int& fl) {
  const long long step = (long long)floor((P - T.stop_h) / T.step_h);
  const long long index = T.hsteps - step - 1;
  const long long max_bin = index * T.asteps + T.asteps - 1;
  const long long min_bin = index * T.asteps;
  double val = -0.001;
  long long start_bin = max_bin;
  bool went = false;
  while ((val != 0 && val < 0.01) || isnan(val)) {
    if (start_bin < 0) {  // the reference reads before the table
      fl |= AIRICE_LOOKUP_UNPINNED;
      break;
    }
    val = lk_at(T, 1, start_bin, fl);
    --start_bin;
    went = true;
  }
  if (went) ++start_bin;
  val = -0.001;
  long long end_bin = min_bin;
  went = false;
  while ((val != 0 && val < 0.01) || isnan(val)) {
    if (end_bin >= T.n) {  // ... or past its end
      fl |= AIRICE_LOOKUP_UNPINNED;
      break;
    }
    val = lk_at(T, 1, end_bin, fl);
    ++end_bin;
    went = true;
  }
  if (went) --end_bin;
  TxhBins b;
  b.s1 = end_bin;
  b.e1 = start_bin;
  b.c1 = fabs(lk_at(T, 0, index, fl) - P);  // sic (.cc:1076): row index used as an entry index
  b.s2 = b.s1 - T.asteps;
  b.e2 = b.e1 - T.asteps;
  if (b.s2 < 0) b.s2 = b.s1 + T.asteps;
  if (b.e2 < 0) b.e2 = b.e1 + T.asteps;
  return b;
}

// FindClosestTHD (.cc:1128-1169)
struct ThdBins {
  long long s, e;
  double c;
};

__device__ __forceinline__ ThdBins closest_thd(const LkTable& T, double P, long long s, long long e,
                                               int& fl) {
#pragma unroll 1
  for (int i = 0; i < 8; ++i) {
    if (e - s >= 3) {
      const long long mid = (s + e) / 2;
      const double v = lk_at(T, 1, mid, fl);
      if (v - P > 0) s = mid;
      if (v - P < 0) e = mid;
    }
  }
  double minimum = 100000000000.0;
  long long index2 = 0;
#pragma unroll 1
  for (long long ip = s; ip < e + 1; ++ip) {
    const double v = lk_at(T, 1, ip, fl);
    const double minval = fabs(v - P);
    if (minval < minimum && v > P) {
      minimum = minval;
    } else {
      index2 = ip;
      break;
    }
  }
  const long long index1 = index2 - 1;
  const double v2 = lk_at(T, 1, index2, fl);
  const double v1 = lk_at(T, 1, index1, fl);
  minimum = fabs(P - v2);
  if (minimum > fabs(P - v1)) minimum = fabs(P - v1);
  return ThdBins{index1, index2, minimum};
}

// The 10 parameters of one table row at horizontal distance D (.cc:1199-1240 / 1250-1289).
__device__ __forceinline__ void row_params(const LkTable& T, double D, long long s, long long e,
                                           double par[10], double* closest, int& fl) {
  const double max_thd = lk_at(T, 1, s, fl);
  if (D <= max_thd) {
    const ThdBins b = closest_thd(T, D, s, e, fl);
    *closest = b.c;
    if (b.c != 0) {
      const double x1 = lk_at(T, 1, b.s, fl), x2 = lk_at(T, 1, b.e, fl);
      const LkRec rs = lk_rec(T, b.s, fl), re = lk_rec(T, b.e, fl);
#pragma unroll
      for (int ip = 0; ip < 10; ++ip)
        par[ip] = lk_interp(D, x1, (double)rs.c[1 + ip], x2, (double)re.c[1 + ip]);
    } else {
      const LkRec r = lk_rec(T, b.s + 1, fl);
#pragma unroll
      for (int ip = 0; ip < 10; ++ip) par[ip] = (double)r.c[1 + ip];
    }
  } else {
#pragma unroll
    for (int ip = 0; ip < 10; ++ip) par[ip] = -1e9;
  }
}

__global__ __launch_bounds__(kLkBlock) void lookup_kernel(LkTable T, const double* __restrict__ src,
                                                          const double* __restrict__ dist,
                                                          double ice_cm, long long n, double d2r,
                                                          double* __restrict__ out, size_t ld,
                                                          uint8_t* __restrict__ ok,
                                                          uint8_t* __restrict__ flags) {
  const long long k = (long long)blockIdx.x * kLkBlock + threadIdx.x;
  if (k >= n) return;
  int fl = 0;
  const double H = src[k] / 100;
  const double D = dist[k] / 100;
  (void)ice_cm;  // the table path never reads the ice height (.cc:1309 converts it, unused)
  const double max_h = lk_at(T, 0, 0, fl);
  const double min_h = lk_at(T, 0, T.n - 1, fl);
  double x1 = 0, x2 = 0, y1 = 0, y2 = 0;
  double piv[10];
  unsigned set = 0;
#pragma unroll
  for (int i = 0; i < 10; ++i) piv[i] = 0;
  if (H <= max_h && H >= min_h && H > 0) {
    // GetParValues (.cc:1172-1302)
    const TxhBins b = closest_txh(T, H, fl);
    double par1[10], par2[10];
    double c1 = 0;
    const double h1 = lk_at(T, 0, b.s1, fl);
    row_params(T, D, b.s1, b.e1, par1, &c1, fl);
    double h2 = h1;
    if (b.c1 != 0 && H > min_h && b.s2 < T.n - 1) {
      h2 = lk_at(T, 0, b.s2, fl);
      double c2 = 0;
      row_params(T, D, b.s2, b.e2, par2, &c2, fl);
    } else {
#pragma unroll
      for (int ip = 0; ip < 10; ++ip) par2[ip] = par1[ip];
    }
    // interpolation in height (.cc:1376-1401); a parameter missing at both heights ends the
    // loop writing its value into slot 9 (the reference sets ipar = 9 before the store)
    x1 = h1;
    x2 = h2;
    bool done = false;
#pragma unroll
    for (int ip = 0; ip < 10; ++ip) {
      if (!done) {
        y1 = par1[ip];
        y2 = par2[ip];
        double v = 0;
        const bool missing = (y1 == -1e9 || y2 == -1e9);
        if (x1 != x2 && !missing) {
          v = lk_interp(H, x1, y1, x2, y2);
        } else if (x1 == x2 && y1 == y2) {
          v = par1[ip];
        }
        if ((x1 == x2 || missing) && y2 == -1e9 && y1 == -1e9) {
          piv[9] = v;
          set |= 1u << 9;
          done = true;
        } else {
          piv[ip] = v;
          set |= 1u << ip;
        }
      }
    }
  }
  if (set != 0x3ffu) fl |= AIRICE_LOOKUP_UNPINNED;
  const double thd = piv[0];
  const bool one_sided = (y1 == -1e9 && y2 != -1e9) || (y2 == -1e9 && y1 != -1e9);
  bool good = true;
  if (y2 == -1e9 && y1 == -1e9) good = false;
  if (H > max_h) good = false;
  if (H < min_h) good = false;
  if (H < 0) good = false;
  if ((fabs(thd - D) / D > 0.01 && D <= 100) || (fabs(thd - D) > 1 && D > 100)) good = false;
  if (one_sided) {
    // finished by launch_lookup_fallback: every output slot is rewritten there, and the
    // checks above are completed with CheckSolBool and launchAngle < 0
    fl |= AIRICE_LOOKUP_FALLBACK;
    ok[k] = good ? 1 : 0;
    flags[k] = (uint8_t)fl;
    return;
  }
  const double la = piv[3] * d2r;  // pi/180 (.cc:1410)
  if (la < 0) good = false;
  out[0 * ld + k] = good ? piv[1] * 100 : 0.0;  // opticalPathLengthInIce
  out[1 * ld + k] = good ? piv[2] * 100 : 0.0;  // opticalPathLengthInAir
  out[2 * ld + k] = piv[8] * 100;               // geometricalPathLengthInIce
  out[3 * ld + k] = piv[7] * 100;               // geometricalPathLengthInAir
  out[4 * ld + k] = good ? la : 0.0;            // launchAngle
  out[5 * ld + k] = good ? piv[4] * 100 : 0.0;  // horizontalDistanceToIntersectionPoint
  out[6 * ld + k] = piv[5];                     // transmissionCoefficientS
  out[7 * ld + k] = piv[6];                     // transmissionCoefficientP
  out[8 * ld + k] = piv[9] * d2r;               // RecievedAngleInIce
  ok[k] = good ? 1 : 0;
  flags[k] = (uint8_t)fl;
}

// airice_lookup_pack: one lane per entry; each column read is coalesced across the wave and each
// wave writes one contiguous 3 KB run of records.
__global__ __launch_bounds__(kLkBlock) void lookup_pack_kernel(const float* __restrict__ t,
                                                               long long ld, long long n,
                                                               float* __restrict__ e) {
  const long long i = (long long)blockIdx.x * kLkBlock + threadIdx.x;
  if (i >= n) return;
  float c[AIRICE_LOOKUP_ENTRY_FLOATS];
#pragma unroll
  for (int k = 0; k < 11; ++k) c[k] = t[(long long)k * ld + i];
  c[11] = 0.0f;
  float4* p = reinterpret_cast<float4*>(e + (long long)AIRICE_LOOKUP_ENTRY_FLOATS * i);
  p[0] = make_float4(c[0], c[1], c[2], c[3]);
  p[1] = make_float4(c[4], c[5], c[6], c[7]);
  p[2] = make_float4(c[8], c[9], c[10], c[11]);
}

}  // namespace

int launch_lookup_pack(const airice_lookup_table* t, float* e, hipStream_t st) {
  const long long n = (long long)t->n_entries;
  if (n == 0) return AIRICE_OK;
  hipLaunchKernelGGL(lookup_pack_kernel, dim3((unsigned)((n + kLkBlock - 1) / kLkBlock)),
                     dim3(kLkBlock), 0, st, t->table, (long long)t->ld, n, e);
  return hipGetLastError() == hipSuccess ? AIRICE_OK : AIRICE_EHIP;
}

int launch_lookup(const DevMedium& M, const IceConsts& I, const airice_lookup_table* t,
                  const double* src, const double* dist, const double* depth, double ice_cm,
                  size_t n, double* out, size_t ld, uint8_t* ok, uint8_t* flags, hipStream_t st) {
  if (n == 0) return AIRICE_OK;
  LkTable T;
  T.t = t->table;
  T.e = t->entries;
  T.ld = (long long)t->ld;
  T.n = (long long)t->n_entries;
  T.stop_h = t->loop_stop_height;
  T.step_h = t->height_step;
  T.hsteps = t->total_height_steps;
  T.asteps = t->total_angle_steps;
  const unsigned grid = (unsigned)((n + kLkBlock - 1) / kLkBlock);
  ktimer_begin(KT_LOOKUP, st);
  hipLaunchKernelGGL(lookup_kernel, dim3(grid), dim3(kLkBlock), 0, st, T, src, dist, ice_cm,
                     (long long)n, M.d2r, out, ld, ok, flags);
  ktimer_end(KT_LOOKUP, st);
  if (hipGetLastError() != hipSuccess) return AIRICE_EHIP;
  return launch_lookup_fallback(M, I, src, dist, depth, ice_cm, n, out, ld, ok, flags, st);
}

}  // namespace airice
