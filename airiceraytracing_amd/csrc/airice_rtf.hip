// airice_rtf.hip -- the RayTracingFunctions:: layer of the reference (RayTracingFunctions.cc, the
// library behind the cfg1 CLI) on gfx950: GetLayerHitPointPar, GetRayOpticalPath,
// GetRayPropagationTime, GetAirPropagationPar, GetIcePropagationPar, fDnfR, ftimeD and
// MinimizeforLaunchAngle, evaluated on the device with the reference's own expressions (these
// are the per-call scalar entry points of a drop-in, not a batch path: one lane per call;
// batches go through the table / solve / single-ray kernels).
//
// Differences from MultiRayAirIceRefraction's forms: 4-wide outputs {THD, receive angle (deg), L,
// time (s)} (no geometric path), GetAirPropagationPar's count at [4*MaxLayers]
// (RayTracingFunctions.cc:529-659), and GetIcePropagationPar without the transition branch.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "airice.h"
#include "airice_internal.h"


namespace airice {

namespace {

constexpr double kSpeedC = 299792458.0;  // RayTracingFunctions.h spedc

// GetB_air / GetC_air layer scan (RayTracingFunctions.cc:172-213)
__host__ __device__ int rtf_layer(const DevMedium& M, double z) {
  const double zabs = fabs(z);
  int which = 0;
  for (int il = 0; il < M.ml - 1; il++) {
    if (zabs < M.atm[il + 1] && zabs >= M.atm[il]) {
      which = il;
      break;
    }
  }
  if (zabs >= M.atm[M.ml - 1]) which = M.ml - 1;
  return which;
}
__host__ __device__ double rtf_B_air(const DevMedium& M, double z) { return M.B[rtf_layer(M, z)]; }
__host__ __device__ double rtf_C_air(const DevMedium& M, double z) { return -M.negC[rtf_layer(M, z)]; }
// Getnz_air (.cc:215-220), Getnz_ice (.cc:144-147)
__host__ __device__ double rtf_nz_air(const DevMedium& M, double z) {
  const double zabs = fabs(z);
  return M.A_air + rtf_B_air(M, zabs) * exp(-rtf_C_air(M, zabs) * zabs);
}
__host__ __device__ double rtf_nz_ice(const DevMedium& M, double z) {
  z = fabs(z);
  return M.A_ice + M.B_ice * exp(M.negC_ice * z);
}
__host__ __device__ double rtf_B(const DevMedium& M, double z, int air) { return air ? rtf_B_air(M, z) : M.B_ice; }
__host__ __device__ double rtf_C(const DevMedium& M, double z, int air) {
  return air ? rtf_C_air(M, z) : -M.negC_ice;
}
__host__ __device__ double rtf_nz(const DevMedium& M, double z, int air) {
  return air ? rtf_nz_air(M, z) : rtf_nz_ice(M, z);
}

// fDnfR (.cc:293-303)
__host__ __device__ double rtf_fDnfR(double x, double A, double B, double C, double L) {
  const double y = A + B * exp(C * x);
  return (L / C) * (1.0 / sqrt(A * A - L * L)) *
         (C * x - log(A * (A + B * exp(C * x)) - L * L + sqrt(A * A - L * L) * sqrt(y * y - L * L)));
}

// ftimeD (.cc:328-347); B is not used by the reference's formula
__host__ __device__ double rtf_ftimeD(const DevMedium& M, double x, double A, double C, double Speedc,
                             double L, int air) {
  const double n = rtf_nz(M, x, air);
  const double n2 = n * n;  // pow(Getnz(x), 2)
  return (1.0 / (Speedc * C * sqrt(n2 - L * L))) *
         (n2 - L * L +
          (C * x - log(A * n - L * L + sqrt(A * A - L * L) * sqrt(n2 - L * L))) *
              (A * A * sqrt(n2 - L * L)) / sqrt(A * A - L * L) +
          A * sqrt(n2 - L * L) * log(n + sqrt(n2 - L * L)));
}

// GetRayOpticalPath (.cc:349-369): the horizontal distance between two heights
__host__ __device__ double rtf_optical_path(const DevMedium& M, double A, double Rx, double Tx, double L,
                                   int air) {
  double x1 = +rtf_fDnfR(Rx, A, rtf_B(M, Rx, air), -rtf_C(M, Rx, air), L) -
              rtf_fDnfR(Tx, A, rtf_B(M, Tx, air), -rtf_C(M, Tx, air), L);
  if (air) x1 *= -1;
  return x1;
}

// GetRayPropagationTime (.cc:371-397)
__host__ __device__ double rtf_prop_time(const DevMedium& M, double A, double Rx, double Tx, double L,
                                int air) {
  double t = +rtf_ftimeD(M, Rx, A, -rtf_C(M, Rx, air), kSpeedC, L, air) -
             rtf_ftimeD(M, Tx, A, -rtf_C(M, Tx, air), kSpeedC, L, air);
  if (air) t *= -1;
  return t;
}

// The Snell part of GetLayerHitPointPar (.cc:399-454): the receive angle (radians) and L.
__host__ __device__ void rtf_hit_L(const DevMedium& M, double n_layer1, double Rx, double Tx,
                          double IncidentAng, int air, double& ReceiveAngle, double& Lvalue) {
  const double SurfaceRayIncidentAngle = IncidentAng * M.d2r;
  const double nzRx = rtf_nz(M, Rx, air);
  const double nzTx = rtf_nz(M, Tx, air);
  const double Lang = asin((n_layer1 / nzTx) * sin(SurfaceRayIncidentAngle));
  ReceiveAngle = asin((rtf_nz(M, Tx, air) * sin(Lang)) / rtf_nz(M, Rx, air));
  Lvalue = nzRx * sin(ReceiveAngle);
}

// GetLayerHitPointPar (.cc:399-527): {x1, ReceiveAngle (deg), L, time}
__host__ __device__ void rtf_hit_point(const DevMedium& M, double n_layer1, double Rx, double Tx,
                              double IncidentAng, int air, double out[4]) {
  const double A = air ? M.A_air : M.A_ice;
  double ReceiveAngle, Lvalue;
  rtf_hit_L(M, n_layer1, Rx, Tx, IncidentAng, air, ReceiveAngle, Lvalue);
  out[0] = rtf_optical_path(M, A, Rx, Tx, Lvalue, air);
  out[1] = ReceiveAngle * M.r2d;
  out[2] = Lvalue;
  out[3] = rtf_prop_time(M, A, Rx, Tx, Lvalue, air);
}

// Layer-skip scans of GetAirPropagationPar (.cc:531-559)
__host__ __device__ int rtf_skip_above(const DevMedium& M, double txh) {
  int skip = 0;
  for (int il = M.ml; il > -1; il--) {
    // ATMLAY[il-1] is read only when txh < ATMLAY[il]/100 (at il = 0 that is txh < 0)
    if (txh < M.atm[il] && (il >= 1 ? txh >= M.atm[il - 1] : false)) il = -100;
    if (il > -1) skip++;
  }
  return skip;
}
__host__ __device__ int rtf_skip_below(const DevMedium& M, double ice) {
  int skip = 0;
  for (int il = 0; il < M.ml; il++) {
    if (ice >= M.atm[il] && ice < M.atm[il + 1]) il = 100;
    if (il < M.ml) skip++;
  }
  return skip;
}

// GetAirPropagationPar (.cc:529-659): out[4*MaxLayers + 1], per layer {THD, Recv, L, t}, count
// at [4*MaxLayers]
__host__ __device__ int rtf_air_prop(const DevMedium& M, double LaunchAngleAir, double AirTxHeight,
                            double IceLayerHeight, double* out) {
  const int SkipLayersAbove = rtf_skip_above(M, AirTxHeight);
  const int SkipLayersBelow = rtf_skip_below(M, IceLayerHeight);
  const int top = M.ml - SkipLayersAbove - 1;
  double StartAngle = 0, StartHeight = 0, Start_nh = 0, StopHeight = 0, L0 = 0;
  int nf = 0;
  for (int il = top; il > SkipLayersBelow - 1; il--) {
    StartHeight = (il == top) ? AirTxHeight : M.atm[il + 1] - 0.00001;
    Start_nh = rtf_nz_air(M, StartHeight);
    StopHeight = (il == (SkipLayersBelow - 1) + 1) ? IceLayerHeight : M.atm[il];
    if (il == top) {
      StartAngle = 180 - LaunchAngleAir;
      double hp[4];
      rtf_hit_point(M, Start_nh, StopHeight, StartHeight, StartAngle, 1, hp);
      for (int j = 0; j < 4; j++) out[4 * nf + j] = hp[j];
      L0 = hp[2];
      StartAngle = hp[1];
    } else {
      const double nzStopHeight = rtf_nz_air(M, StopHeight);
      const double RecAng = asin(L0 / nzStopHeight) * M.r2d;
      out[4 * nf + 0] = rtf_optical_path(M, M.A_air, StopHeight, StartHeight, L0, 1);
      out[4 * nf + 1] = RecAng;
      out[4 * nf + 2] = L0;
      out[4 * nf + 3] = rtf_prop_time(M, M.A_air, StopHeight, StartHeight, L0, 1);
      StartAngle = RecAng;
    }
    nf++;
  }
  out[4 * M.ml] = nf;
  return nf;
}

// GetIcePropagationPar (.cc:661-681)
__host__ __device__ void rtf_ice_prop(const DevMedium& M, double AntennaDepth, double Lvalue,
                             double out[4]) {
  const double nzStopDepth = rtf_nz_ice(M, AntennaDepth);
  out[0] = rtf_optical_path(M, M.A_ice, AntennaDepth, 0.0, Lvalue, 0);
  out[1] = asin(Lvalue / nzStopDepth) * M.r2d;
  out[2] = Lvalue;
  out[3] = rtf_prop_time(M, M.A_ice, AntennaDepth, 0.0, Lvalue, 0);
}

// MinimizeforLaunchAngle (.cc:683-731)
__host__ __device__ double rtf_min_launch(const DevMedium& M, double x, double AirTxHeight,
                                 double IceLayerHeight, double AntennaDepth, double D) {
  double air[4 * kMaxLayers + 1];
  const int nf = rtf_air_prop(M, x, AirTxHeight, IceLayerHeight, air);
  double thd_air = 0;
  for (int i = 0; i < nf; i++) thd_air += air[i * 4];
  // no air layer (Tx above 150 km or below the ice): the reference reads an unset slot (UB),
  // modelled as NaN like the oracle
  const double Lvalue = nf > 0 ? air[2] : __builtin_nan("");
  double thd_ice = 0;
  if (AntennaDepth != 0) {
    double ice[4];
    rtf_ice_prop(M, AntennaDepth, Lvalue, ice);
    thd_ice = ice[0];
  }
  return D - (thd_ice + thd_air);
}

// gsl_root_fsolver_brent (GNU GSL 2.x roots/brent.c: brent_init / brent_iterate) driven by
// RayTracingFunctions::FindFunctionRoot (RayTracingFunctions.cc:256-290: set, then
// {iterate; root; x_lower; x_upper; gsl_root_test_interval(lo, hi, 0, tol)} while CONTINUE and
// iter < max_iter, the last root returned).  As for the bisection: a
// non-finite f at a bracket end makes brent_init return before the state is stored (the
// reference then iterates on uninitialised malloc memory) -- modelled as a zero state and flagged
// AIRICE_SOLVE_NONFINITE_END; a non-finite f at an iterate returns EBADFUNC with nothing stored
// (AIRICE_SOLVE_STALE_MID); lower > upper makes gsl_root_fsolver_set fail (AIRICE_SOLVE_BAD_BRACKET,
// root 0).  The test oracle restates it the same way (or_brent).
struct RtfBrent {
  double root;
  int status, iters;
};

template <class F>
__host__ __device__ RtfBrent gsl_brent(F f, double x_lo, double x_hi, double tolerance, int max_iter) {
  const double kEps = 2.2204460492503131e-16;  // GSL_DBL_EPSILON
  RtfBrent R{0.0, 0, 0};
  if (x_lo > x_hi) {
    R.status |= AIRICE_SOLVE_BAD_BRACKET;
    return R;
  }
  double root = 0.5 * (x_lo + x_hi);
  double lo = x_lo, hi = x_hi;
  double a = 0, b = 0, c = 0, d = 0, e = 0, fa = 0, fb = 0, fc = 0;
  const double f_lower = f(x_lo);
  double f_upper = 0;
  bool ok = __builtin_isfinite(f_lower);
  if (ok) {
    f_upper = f(x_hi);
    ok = __builtin_isfinite(f_upper);
  }
  if (!ok) {
    R.status |= AIRICE_SOLVE_NONFINITE_END;
  } else {
    a = x_lo, fa = f_lower;
    b = x_hi, fb = f_upper;
    c = x_hi, fc = f_upper;
    d = x_hi - x_lo;
    e = x_hi - x_lo;
  }
  int iter = 0;
  bool cont = true;
  do {
    iter++;
    // brent_iterate on local copies; the state is stored only when the new point is finite
    double la = a, lb = b, lc = c, ld = d, le = e, lfa = fa, lfb = fb, lfc = fc;
    bool ac_equal = false;
    if ((lfb < 0 && lfc < 0) || (lfb > 0 && lfc > 0)) {
      ac_equal = true;
      lc = la;
      lfc = lfa;
      ld = lb - la;
      le = lb - la;
    }
    if (fabs(lfc) < fabs(lfb)) {
      ac_equal = true;
      la = lb;
      lb = lc;
      lc = la;
      lfa = lfb;
      lfb = lfc;
      lfc = lfa;
    }
    const double tol = 0.5 * kEps * fabs(lb);
    const double m = 0.5 * (lc - lb);
    if (lfb == 0) {
      root = lb;
      lo = lb;
      hi = lb;
    } else if (fabs(m) <= tol) {
      root = lb;
      if (lb < lc) {
        lo = lb;
        hi = lc;
      } else {
        lo = lc;
        hi = lb;
      }
    } else {
      if (fabs(le) < tol || fabs(lfa) <= fabs(lfb)) {
        ld = m;  // bisection
        le = m;
      } else {
        double p, q, r;  // inverse cubic interpolation
        const double sr = lfb / lfa;
        if (ac_equal) {
          p = 2 * m * sr;
          q = 1 - sr;
        } else {
          q = lfa / lfc;
          r = lfb / lfc;
          p = sr * (2 * m * q * (q - r) - (lb - la) * (r - 1));
          q = (q - 1) * (r - 1) * (sr - 1);
        }
        if (p > 0)
          q = -q;
        else
          p = -p;
        const double t1 = 3 * m * q - fabs(tol * q), t2 = fabs(le * q);
        if (2 * p < (t1 < t2 ? t1 : t2)) {  // GSL_MIN
          le = ld;
          ld = p / q;
        } else {
          ld = m;
          le = m;
        }
      }
      la = lb;
      lfa = lfb;
      if (fabs(ld) > tol)
        lb += ld;
      else
        lb += (m > 0 ? +tol : -tol);
      const double fnew = f(lb);
      if (!__builtin_isfinite(fnew)) {
        R.status |= AIRICE_SOLVE_STALE_MID;
      } else {
        lfb = fnew;
        a = la, b = lb, c = lc, d = ld, e = le, fa = lfa, fb = lfb, fc = lfc;
        root = lb;
        double cc = lc;
        if ((lfb < 0 && lfc < 0) || (lfb > 0 && lfc > 0)) cc = la;
        if (lb < cc) {
          lo = lb;
          hi = cc;
        } else {
          lo = cc;
          hi = lb;
        }
      }
    }
    // gsl_root_test_interval(lo, hi, 0, tolerance)
    if (lo > hi) {
      cont = false;
    } else {
      const double min_abs = ((lo > 0.0 && hi > 0.0) || (lo < 0.0 && hi < 0.0))
                                 ? (fabs(lo) < fabs(hi) ? fabs(lo) : fabs(hi))
                                 : 0.0;
      cont = !(fabs(hi - lo) < 0 + tolerance * min_abs);
    }
  } while (cont && iter < max_iter);
  if (cont) R.status |= AIRICE_SOLVE_MAXITER;
  R.root = root;
  R.iters = iter;
  return R;
}

// Air2IceRayTracing CLI solve (Air2IceRayTracing.C:56-185; StoreRayPath is false there).
__host__ __device__ void rtf_air2ice(const DevMedium& M, double AirTxHeight, double HorizontalDistance,
                            double IceLayerHeight, double AntennaDepth, double* o) {
  const double StraightAngle =
      180 - (atan(HorizontalDistance / (AirTxHeight - IceLayerHeight + AntennaDepth)) * M.r2d);
  double startanglelim = StraightAngle - 16;
  double endanglelim = StraightAngle;
  int probes = 0;
  double air[4 * kMaxLayers + 1];
  if (startanglelim < 90.00) {
    startanglelim = 90.05;
    bool checknan = false;
    while (!checknan && startanglelim > 89.9) {
      const int nf = rtf_air_prop(M, startanglelim, AirTxHeight, IceLayerHeight, air);
      double thd = 0;
      for (int i = 0; i < nf; i++) thd += air[i * 4];
      if ((!__builtin_isnan(thd) && thd > 0) || startanglelim > endanglelim - 1) {
        checknan = true;
      } else {
        startanglelim = startanglelim + 0.05;
        ++probes;
      }
    }
  }
  if (endanglelim < 90.001 && endanglelim > 90.00) endanglelim = 90.05;
  const RtfBrent br = gsl_brent(
      [&](double x) {
        return rtf_min_launch(M, x, AirTxHeight, IceLayerHeight, AntennaDepth, HorizontalDistance);
      },
      startanglelim, endanglelim, 0.000000001, 20);
  const double LaunchAngleAir = br.root;
  const int nf = rtf_air_prop(M, LaunchAngleAir, AirTxHeight, IceLayerHeight, air);
  double thd_air = 0, t_air = 0;
  for (int i = 0; i < nf; i++) {
    thd_air += air[i * 4];
    t_air += air[3 + i * 4] * 1e9;  // pow(10, 9)
  }
  // nf == 0: the reference reads unset slots (UB); NaN here, as the oracle
  const double Lvalue = nf > 0 ? air[2] : __builtin_nan("");
  const double inc = nf > 0 ? air[1 + (nf - 1) * 4] : __builtin_nan("");
  double ice[4];
  rtf_ice_prop(M, AntennaDepth, Lvalue, ice);
  const double t_ice = ice[3] * 1e9;
  o[0] = startanglelim;
  o[1] = endanglelim;
  o[2] = LaunchAngleAir;
  o[3] = thd_air;
  o[4] = inc;
  o[5] = Lvalue;
  o[6] = t_air;
  o[7] = ice[0];
  o[8] = ice[1];
  o[9] = t_ice;
  o[10] = ice[0] + thd_air;
  o[11] = t_ice + t_air;
  o[12] = br.status | (nf == 0 ? AIRICE_SOLVE_NO_AIR_LAYER : 0);
  o[13] = br.iters;
  o[14] = probes;
  o[15] = nf;
}

// ---- MultiRayAirIceRefraction:: forms (MultiRayAirIceRefraction.cc:377-917): the same
// expressions plus the geometric path, 5-wide outputs {THD, Recv deg, L, t, geo} ----------------

// fpathD (.cc:434-447), the reference's expression
__host__ __device__ double mr_fpathD(double x, double A, double B, double C, double L) {
  return (log((A + B * exp(C * x)) *
              (sqrt((A * A + 2 * A * B * exp(C * x) + B * B * exp(2 * C * x) - L * L) /
                    ((A + B * exp(C * x)) * (A + B * exp(C * x)))) +
               1)) -
          (A * log(A * sqrt(A * A - L * L) *
                       sqrt((A * A + 2 * A * B * exp(C * x) + B * B * exp(2 * C * x) - L * L) /
                            ((A + B * exp(C * x)) * (A + B * exp(C * x)))) +
                   B * sqrt(A * A - L * L) * exp(C * x) *
                       sqrt((A * A + 2 * A * B * exp(C * x) + B * B * exp(2 * C * x) - L * L) /
                            ((A + B * exp(C * x)) * (A + B * exp(C * x)))) +
                   A * A + A * B * exp(C * x) - L * L)) /
              sqrt(A * A - L * L) +
          (A * C * x) / sqrt(A * A - L * L)) /
         C;
}

// GetRayGeometricPath (.cc:494-513)
__host__ __device__ double mr_geo_path(const DevMedium& M, double A, double Rx, double Tx, double L,
                              int air) {
  double g = mr_fpathD(Rx, A, rtf_B(M, Rx, air), -rtf_C(M, Rx, air), L) -
             mr_fpathD(Tx, A, rtf_B(M, Tx, air), -rtf_C(M, Tx, air), L);
  if (air) g *= -1;
  return g;
}

// GetLayerHitPointPar (.cc:521-646): {x1, ReceiveAngle (deg), L, time, x1_Geo}
__host__ __device__ void mr_hit_point(const DevMedium& M, double n_layer1, double Rx, double Tx,
                             double IncidentAng, int air, double out[5]) {
  rtf_hit_point(M, n_layer1, Rx, Tx, IncidentAng, air, out);
  out[4] = mr_geo_path(M, air ? M.A_air : M.A_ice, Rx, Tx, out[2], air);
}

// GetAirPropagationPar (.cc:661-804): out[5*MaxLayers + 2], per layer {THD, Recv, L, t, geo},
// the filled-layer count at [5*MaxLayers+1] ([5*MaxLayers] is never written by the reference;
// 0 here)
__host__ __device__ int mr_air_prop(const DevMedium& M, double LaunchAngleAir, double AirTxHeight,
                           double IceLayerHeight, double* out) {
  const int SkipLayersAbove = rtf_skip_above(M, AirTxHeight);
  const int SkipLayersBelow = rtf_skip_below(M, IceLayerHeight);
  const int top = M.ml - SkipLayersAbove - 1;
  double StartAngle = 0, StartHeight = 0, Start_nh = 0, StopHeight = 0, L0 = 0;
  int nf = 0;
  for (int il = top; il > SkipLayersBelow - 1; il--) {
    StartHeight = (il == top) ? AirTxHeight : M.atm[il + 1] - 0.00001;
    Start_nh = rtf_nz_air(M, StartHeight);
    StopHeight = (il == (SkipLayersBelow - 1) + 1) ? IceLayerHeight : M.atm[il];
    if (il == top) {
      StartAngle = 180 - LaunchAngleAir;
      double hp[5];
      mr_hit_point(M, Start_nh, StopHeight, StartHeight, StartAngle, 1, hp);
      for (int j = 0; j < 5; j++) out[5 * nf + j] = hp[j];
      L0 = hp[2];
      StartAngle = hp[1];
    } else {
      const double nzStopHeight = rtf_nz_air(M, StopHeight);
      const double RecAng = asin(L0 / nzStopHeight) * M.r2d;
      out[5 * nf + 0] = rtf_optical_path(M, M.A_air, StopHeight, StartHeight, L0, 1);
      out[5 * nf + 1] = RecAng;
      out[5 * nf + 2] = L0;
      out[5 * nf + 3] = rtf_prop_time(M, M.A_air, StopHeight, StartHeight, L0, 1);
      out[5 * nf + 4] = mr_geo_path(M, M.A_air, StopHeight, StartHeight, L0, 1);
      StartAngle = RecAng;
    }
    nf++;
  }
  out[5 * M.ml + 1] = nf;
  return nf;
}

// GetIcePropagationPar (.cc:807-869), TransitionBoundary == 0 (.h:70)
__host__ __device__ void mr_ice_prop(const DevMedium& M, double AntennaDepth, double Lvalue,
                            double out[5]) {
  rtf_ice_prop(M, AntennaDepth, Lvalue, out);
  out[4] = mr_geo_path(M, M.A_ice, AntennaDepth, 0.0, Lvalue, 0);
}

// MinimizeforLaunchAngle (.cc:873-917)
__host__ __device__ double mr_min_launch(const DevMedium& M, double x, double AirTxHeight,
                                double IceLayerHeight, double AntennaDepth, double D) {
  double air[5 * kMaxLayers + 2];
  const int nf = mr_air_prop(M, x, AirTxHeight, IceLayerHeight, air);
  double thd_air = 0;
  for (int i = 0; i < nf; i++) thd_air += air[i * 5];
  // no air layer: the reference reads air[-4] and an unset air[2] (UB), modelled as NaN
  const double Lvalue = nf > 0 ? air[2] : __builtin_nan("");
  double thd_ice = 0;
  if (AntennaDepth != 0) {
    double ice[5];
    mr_ice_prop(M, AntennaDepth, Lvalue, ice);
    thd_ice += ice[0];
  }
  return D - (thd_ice + thd_air);
}

// ---- one call spread over a wave (GetAirPropagationPar, MinimizeforLaunchAngle) ------------
// The reference's layer loop (.cc:529-659 / MultiRay .cc:661-804) derives L in its first layer
// and reuses it below (.cc:757-771), so once L is known the layers are independent: every lane
// derives L (the cheap Snell part of the first layer), then lane j evaluates layer
// il = top - j -- the same functions on the same arguments as the loop, all layers at once.
// W = 4: RayTracingFunctions {THD, Recv deg, L, t}; W = 5: MultiRay, + geometric path.
// Lane `ice_lane` (>= 0) evaluates the in-ice segment with the same path functions instead
// (GetIcePropagationPar's THD, .cc:661-681 / :807-869), for MinimizeforLaunchAngle.
struct LayerLane {
  int nf;     // layers filled
  double L0;  // Lvalue[0]
  double o[5];
};

template <int W>
__device__ LayerLane air_prop_lane(const DevMedium& M, double LaunchAngleAir, double AirTxHeight,
                                   double IceLayerHeight, int j, bool full, int ice_lane,
                                   double AntennaDepth) {
  LayerLane R;
  const int SkipLayersAbove = rtf_skip_above(M, AirTxHeight);
  const int SkipLayersBelow = rtf_skip_below(M, IceLayerHeight);
  const int top = M.ml - SkipLayersAbove - 1;
  R.nf = top >= SkipLayersBelow ? top - SkipLayersBelow + 1 : 0;
  // the first layer's Snell step (every lane): L
  const int t0 = top < 0 ? 0 : (top > 4 ? 4 : top);
  const double StopH0 = (top == (SkipLayersBelow - 1) + 1) ? IceLayerHeight : sel5(M.atm, t0);
  const double Start_nh0 = rtf_nz_air(M, AirTxHeight);
  double Recv0, L;
  rtf_hit_L(M, Start_nh0, StopH0, AirTxHeight, 180 - LaunchAngleAir, 1, Recv0, L);
  R.L0 = L;
  // this lane's layer
  const int il = top - j;
  const int ic = il < 0 ? 0 : (il > 3 ? 3 : il);
  const double StartH = (j == 0) ? AirTxHeight : sel5(M.atm, ic + 1) - 0.00001;
  const double StopH = (il == (SkipLayersBelow - 1) + 1) ? IceLayerHeight : sel5(M.atm, ic);
  const bool ice = j == ice_lane;
  const double A = ice ? M.A_ice : M.A_air;
  const double Rx = ice ? AntennaDepth : StopH, Tx = ice ? 0.0 : StartH;
  const int air = ice ? 0 : 1;
  // the layer's two ends on two lanes (lane j: Rx, lane j + 8: Tx; the partner's values come back
  // by shuffle): each antiderivative of GetRayOpticalPath / GetRayPropagationTime /
  // GetRayGeometricPath once per lane, differenced in the reference's order (+Rx - Tx, sign flip
  // in air)
  const bool tx_side = (threadIdx.x & 8) != 0;
  const double h = tx_side ? Tx : Rx;
  const double fD = rtf_fDnfR(h, A, rtf_B(M, h, air), -rtf_C(M, h, air), L);
  const double fD_tx = __shfl_down(fD, 8);
  double x1 = +fD - fD_tx;
  if (air) x1 *= -1;
  R.o[0] = x1;
  if (full) {
    const double nzStopHeight = rtf_nz_air(M, StopH);
    R.o[1] = (j == 0) ? Recv0 * M.r2d : asin(L / nzStopHeight) * M.r2d;
    R.o[2] = L;
    const double ft = rtf_ftimeD(M, h, A, -rtf_C(M, h, air), kSpeedC, L, air);
    double fp = 0.0;
    if (W == 5) fp = mr_fpathD(h, A, rtf_B(M, h, air), -rtf_C(M, h, air), L);
    const double ft_tx = __shfl_down(ft, 8);
    double t = +ft - ft_tx;
    if (air) t *= -1;
    R.o[3] = t;
    if (W == 5) {
      const double fp_tx = __shfl_down(fp, 8);
      double g = fp - fp_tx;
      if (air) g *= -1;
      R.o[4] = g;
    }
  }
  return R;
}

// GetAirPropagationPar on a wave: lane j < MaxLayers writes its layer's W slots (zeros past the
// filled layers, as the one-lane form leaves them), lane 0 the count.
template <int W>
__device__ void air_prop_wave(const DevMedium& M, double LaunchAngleAir, double AirTxHeight,
                              double IceLayerHeight, double* __restrict__ out) {
  const int lane = (int)(threadIdx.x & 63);
  const LayerLane R = air_prop_lane<W>(M, LaunchAngleAir, AirTxHeight, IceLayerHeight,
                                       (lane & 7), true, -1, 0.0);
  if (lane < M.ml)
    for (int k = 0; k < W; k++) out[W * lane + k] = lane < R.nf ? R.o[k] : 0.0;
  if (lane == 0) {
    if (W == 5) out[W * M.ml] = 0.0;
    out[W * M.ml + (W == 5 ? 1 : 0)] = R.nf;
  }
}

// MinimizeforLaunchAngle on a wave: the air layers on lanes 0-3, the in-ice THD on lane 4, the
// sums in the one-lane form's order.  rtf_min_launch: thd_ice = ice[0]; mr_min_launch:
// thd_ice += ice[0] (from 0).
template <int W>
__device__ double min_launch_wave(const DevMedium& M, double x, double AirTxHeight,
                                  double IceLayerHeight, double AntennaDepth, double D) {
  const int lane = (int)(threadIdx.x & 63);
  const LayerLane R = air_prop_lane<W>(M, x, AirTxHeight, IceLayerHeight,
                                       (lane & 7), false, 4, AntennaDepth);
  double thd_air = 0;
  for (int i = 0; i < kMaxLayers; i++) {
    const double a = __shfl(R.o[0], i);
    if (i < R.nf) thd_air += a;
  }
  const double ice0 = __shfl(R.o[0], 4);
  double thd_ice = 0;
  if (AntennaDepth != 0 && R.nf > 0) {
    if (W == 5)
      thd_ice += ice0;
    else
      thd_ice = ice0;
  } else if (AntennaDepth != 0) {
    // no air layer: L is the reference's unset slot (UB), modelled as NaN (the one-lane form)
    double ice[4];
    rtf_ice_prop(M, AntennaDepth, __builtin_nan(""), ice);
    if (W == 5)
      thd_ice += ice[0];
    else
      thd_ice = ice[0];
  }
  return D - (thd_ice + thd_air);
}

}  // namespace

struct RtfCall {
  int op, n_out;
  double a[8];
};
constexpr int kRtfMaxOut = AIRICE_RTF_AIR2ICE_FIELDS > 5 * kMaxLayers + 2 ? AIRICE_RTF_AIR2ICE_FIELDS
                                                                         : 5 * kMaxLayers + 2;
__host__ __device__ void rtf_eval_one(const DevMedium& M, const RtfCall& c, double* r);

namespace {

__global__ void rtf_kernel(DevMedium M, RtfCall c, double* __restrict__ out, Signal sig) {
  prefetch_kernargs<sizeof(DevMedium) + sizeof(RtfCall)>();
  // the layer-loop ops run on the whole wave (air_prop_wave, min_launch_wave); the rest on lane 0
  if (c.op == AIRICE_RTF_AIR_PROPAGATION || c.op == AIRICE_MR_AIR_PROPAGATION) {
    if (c.op == AIRICE_RTF_AIR_PROPAGATION)
      air_prop_wave<4>(M, c.a[0], c.a[1], c.a[2], out);
    else
      air_prop_wave<5>(M, c.a[0], c.a[1], c.a[2], out);
    __syncthreads();  // every lane's slots are written before lane 0 signals
    if (threadIdx.x == 0) signal_done(sig);
    return;
  }
  if (c.op == AIRICE_RTF_MIN_LAUNCH || c.op == AIRICE_MR_MIN_LAUNCH) {
    const double f = c.op == AIRICE_RTF_MIN_LAUNCH
                         ? min_launch_wave<4>(M, c.a[0], c.a[1], c.a[2], c.a[3], c.a[4])
                         : min_launch_wave<5>(M, c.a[0], c.a[1], c.a[2], c.a[3], c.a[4]);
    if (threadIdx.x == 0) {
      out[0] = f;
      signal_done(sig);
    }
    return;
  }
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double r[kRtfMaxOut];
  rtf_eval_one(M, c, r);
  for (int i = 0; i < c.n_out; i++) out[i] = r[i];
  signal_done(sig);
}

}  // namespace

// One call of any op on one lane (the kernel's lane 0 and the host form, rtf_host): r receives
// kRtfMaxOut values, zeros past the op's outputs.
__host__ __device__ void rtf_eval_one(const DevMedium& M, const RtfCall& c, double* r) {
  for (int i = 0; i < kRtfMaxOut; i++) r[i] = 0;
  switch (c.op) {
    case AIRICE_RTF_HIT_POINT:
      rtf_hit_point(M, c.a[0], c.a[1], c.a[2], c.a[3], (int)c.a[4], r);
      break;
    case AIRICE_RTF_OPTICAL_PATH:
      r[0] = rtf_optical_path(M, c.a[0], c.a[1], c.a[2], c.a[3], (int)c.a[4]);
      break;
    case AIRICE_RTF_PROPAGATION_TIME:
      r[0] = rtf_prop_time(M, c.a[0], c.a[1], c.a[2], c.a[3], (int)c.a[4]);
      break;
    case AIRICE_RTF_AIR_PROPAGATION:
      rtf_air_prop(M, c.a[0], c.a[1], c.a[2], r);
      break;
    case AIRICE_RTF_ICE_PROPAGATION:  // (IncidentAngleonIce, IceLayerHeight unused, .cc:664)
      rtf_ice_prop(M, c.a[2], c.a[3], r);
      break;
    case AIRICE_RTF_FDNFR:
      r[0] = rtf_fDnfR(c.a[0], c.a[1], c.a[2], c.a[3], c.a[4]);
      break;
    case AIRICE_RTF_FTIMED:
      r[0] = rtf_ftimeD(M, c.a[0], c.a[1], c.a[3], c.a[4], c.a[5], (int)c.a[6]);
      break;
    case AIRICE_RTF_MIN_LAUNCH:
      r[0] = rtf_min_launch(M, c.a[0], c.a[1], c.a[2], c.a[3], c.a[4]);
      break;
    case AIRICE_RTF_AIR2ICE:
      rtf_air2ice(M, c.a[0], c.a[1], c.a[2], c.a[3], r);
      break;
    case AIRICE_MR_FPATHD:  // (x, a, b, c, speedc, l): speedc unused by the formula
      r[0] = mr_fpathD(c.a[0], c.a[1], c.a[2], c.a[3], c.a[5]);
      break;
    case AIRICE_MR_GEOMETRIC_PATH:
      r[0] = mr_geo_path(M, c.a[0], c.a[1], c.a[2], c.a[3], (int)c.a[4]);
      break;
    case AIRICE_MR_HIT_POINT:
      mr_hit_point(M, c.a[0], c.a[1], c.a[2], c.a[3], (int)c.a[4], r);
      break;
    case AIRICE_MR_AIR_PROPAGATION:
      mr_air_prop(M, c.a[0], c.a[1], c.a[2], r);
      break;
    case AIRICE_MR_ICE_PROPAGATION:  // (IncidentAngleonIce, IceLayerHeight unused, .cc:807)
      mr_ice_prop(M, c.a[2], c.a[3], r);
      break;
    case AIRICE_MR_MIN_LAUNCH:
      r[0] = mr_min_launch(M, c.a[0], c.a[1], c.a[2], c.a[3], c.a[4]);
      break;
    default:
      break;
  }
}

int rtf_outputs(int op, int max_layers) {
  switch (op) {
    case AIRICE_RTF_HIT_POINT:
    case AIRICE_RTF_ICE_PROPAGATION:
      return 4;
    case AIRICE_RTF_AIR_PROPAGATION:
      return 4 * max_layers + 1;
    case AIRICE_RTF_OPTICAL_PATH:
    case AIRICE_RTF_PROPAGATION_TIME:
    case AIRICE_RTF_FDNFR:
    case AIRICE_RTF_FTIMED:
    case AIRICE_RTF_MIN_LAUNCH:
      return 1;
    case AIRICE_RTF_AIR2ICE:
      return AIRICE_RTF_AIR2ICE_FIELDS;
    case AIRICE_MR_FPATHD:
    case AIRICE_MR_GEOMETRIC_PATH:
    case AIRICE_MR_MIN_LAUNCH:
      return 1;
    case AIRICE_MR_HIT_POINT:
    case AIRICE_MR_ICE_PROPAGATION:
      return 5;
    case AIRICE_MR_AIR_PROPAGATION:
      return 5 * max_layers + 2;
    default:
      return -1;
  }
}

// The one call on the host (airice_rtf_eval's default for these one-query entry points): the
// same expressions compiled for the CPU (the host's libm in place of ocml: the same functions to
// within an ulp or so), with no kernel dispatch and completion wait (~8 us of a GPU call).
int rtf_host(const DevMedium& M, int op, const double* args, size_t n_args, double* out) {
  RtfCall c;
  c.op = op;
  c.n_out = rtf_outputs(op, M.ml);
  if (c.n_out < 0) return AIRICE_EINVAL;
  for (int i = 0; i < 8; i++) c.a[i] = (size_t)i < n_args ? args[i] : 0.0;
  double r[kRtfMaxOut];
  rtf_eval_one(M, c, r);
  for (int i = 0; i < c.n_out; i++) out[i] = r[i];
  return AIRICE_OK;
}

int launch_rtf(const DevMedium& M, int op, const double* args, size_t n_args, double* d_out,
               hipStream_t st) {
  RtfCall c;
  c.op = op;
  c.n_out = rtf_outputs(op, M.ml);
  for (int i = 0; i < 8; i++) c.a[i] = (size_t)i < n_args ? args[i] : 0.0;
  count_launch(LC_RTF);
  hipLaunchKernelGGL(rtf_kernel, dim3(1), dim3(64), 0, st, M, c, d_out, take_scalar_signal());
  return hipGetLastError() == hipSuccess ? AIRICE_OK : AIRICE_EHIP;
}

}  // namespace airice
