// airice_kernels.hip -- gfx950 kernels + stream-ordered launchers of libairice.so.
//
//  table_kernel   : one lane per (TxHeight, launch angle) ray of MakeRayTracingTable
//                   (MultiRayAirIceRefraction.cc:2079-2122 loop body -> GetRayTracingSolutions
//                   .cc:1796-2017), writes the 11 float table columns (.cc:2101-2111) and,
//                   optionally, the 18 doubles of dummy[] for parity checks.
//  rays_kernel    : same ray for arbitrary (angle, height) lists.
//  solve_kernel   : one lane per query of Air2IceRayTracing (.cc:1464-1616): bracket set-up,
//                   the 0.05-degree probe loop, GSL-bisection emulation (tolerance 1e-9,
//                   40 iterations) over a THD-only evaluator, and one full evaluation at the root.
//                   VARIANT selects MultiRay (dummy[17]) / pythonwrapper (dummy[15]) outputs.
//  hdtip_kernel   : GetHorizontalDistanceToIntersectionPoint (.cc:945-989), cm in/out.
//  trace_kernel   : pythonwrapper TraceIceToAir (TraceIceToAir.C:5-73) rows of 10.
//
// Data layout in HBM: structure-of-arrays, column c of item i at out[c*ld + i], so each
// wave's store of one column is one contiguous 256 B (f32) / 512 B (f64) segment.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>

#include "airice.h"
#include "airice_device.hpp"
#include "airice_internal.h"

namespace airice {

constexpr double kSpeedC = 299792458.0;  // .h:30
constexpr int kBlock = 256;

// ---------------------------------------------------------------------------
// Forward ray: GetRayTracingSolutions (.cc:1796-2017).  d[] = dummy[0..17].
// ---------------------------------------------------------------------------
struct RayOut {
  double d[18];
};

__device__ __forceinline__ void ray_solution(const DevMedium& M, const IceConsts& I, double theta,
                                             double H, bool in_ice, int bot, double* d) {
  const int top = top_layer(M, H);
  const Endpoint tx = air_endpoint(M, H);
  double start_angle = 0.0, thd_air = 0.0, t_air = 0.0, geo_air = 0.0;
#pragma unroll
  for (int il = kMaxLayers - 1; il >= 0; --il) {
    if (il > top || il < bot) continue;
    const bool first = (il == top);
    const Endpoint T = pick(first, tx, M.start[il]);
    const Endpoint R = pick(il == bot, I.ice_air, M.stop[il]);
    if (first) start_angle = 180 - theta;
    // n_layer1 = Getnz_air(StartHeight) = T.n (.cc:1850, 1871)
    const Segment s = segment_full(M, M.A_air, T, R, T.n, start_angle, true);
    thd_air += s.thd;
    start_angle = s.recv_deg;
    t_air += s.t;
    geo_air += s.geo;
  }
  const double inc = start_angle;
  double thd_ice = 0.0, t_ice = 0.0, geo_ice = 0.0, recv_ice = 0.0;
  if (in_ice) {
    // .cc:1897-1922: n_layer1 = Getnz_air(IceLayerHeight), Rx = -AntennaDepth, Tx = 0
    const Segment s = segment_full(M, M.A_ice, I.ice0, I.ice_rx, I.ice_air.n, inc, false);
    thd_ice += s.thd;
    t_ice += s.t;
    geo_ice += s.geo;
    recv_ice = s.recv_deg;
  }
  double tS, tP;
  fresnel_trans(I.ice_air.n, I.ice0.n, inc * M.d2r, tS, tP);
  d[0] = 0;
  d[1] = H;
  d[2] = thd_air + thd_ice;
  d[3] = thd_air;
  d[4] = thd_ice;
  d[5] = (t_ice + t_air) * kSpeedC;
  d[6] = t_air * kSpeedC;
  d[7] = t_ice * kSpeedC;
  d[8] = (t_ice + t_air) * 1e9;
  d[9] = t_air * 1e9;
  d[10] = t_ice * 1e9;
  d[11] = theta;
  d[12] = inc;
  d[13] = recv_ice;
  d[14] = tS;
  d[15] = tP;
  d[16] = geo_air;
  d[17] = geo_ice;
}

struct TableArgs {
  double start_h, stop_h, step_h;
  double start_a, stop_a, step_a;
  int hsteps, asteps;
  int row0, in_ice;
  long long n;
  size_t ld;
};

__global__ __launch_bounds__(kBlock) void table_kernel(DevMedium M, IceConsts I, TableArgs G,
                                                       float* __restrict__ table,
                                                       double* __restrict__ full) {
  const long long k = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (k >= G.n) return;
  const int r = (int)(k / G.asteps);
  const int iang = (int)(k - (long long)r * G.asteps);
  const int ihei = G.row0 + r;
  // .cc:2080, 2085, 2089-2094 (separate mul and add: no contraction)
  double H = G.start_h - G.step_h * ihei;
  double th = G.start_a + G.step_a * iang;
  if (H != G.stop_h && ihei == G.hsteps - 1) H = G.stop_h;
  if (iang == G.asteps - 1) th = G.stop_a;
  const int bot = bottom_layer(M, I.ice_h);
  double d[18];
  ray_solution(M, I, th, H, G.in_ice != 0, bot, d);
  const size_t ld = G.ld;
  // AllTableAllAntData columns (.cc:2101-2111)
  table[0 * ld + k] = (float)d[1];
  table[1 * ld + k] = (float)d[2];
  table[2 * ld + k] = (float)d[7];
  table[3 * ld + k] = (float)d[6];
  table[4 * ld + k] = (float)d[11];
  table[5 * ld + k] = (float)d[3];
  table[6 * ld + k] = (float)d[14];
  table[7 * ld + k] = (float)d[15];
  table[8 * ld + k] = (float)d[16];
  table[9 * ld + k] = (float)d[17];
  table[10 * ld + k] = (float)d[13];
  if (full != nullptr) {
#pragma unroll
    for (int c = 0; c < 18; ++c) full[c * ld + k] = d[c];
  }
}

__global__ __launch_bounds__(kBlock) void rays_kernel(DevMedium M, IceConsts I,
                                                      const double* __restrict__ launch,
                                                      const double* __restrict__ txh, int in_ice,
                                                      long long n, double* __restrict__ out,
                                                      size_t ld) {
  const long long k = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (k >= n) return;
  const int bot = bottom_layer(M, I.ice_h);
  double d[18];
  ray_solution(M, I, launch[k], txh[k], in_ice != 0, bot, d);
#pragma unroll
  for (int c = 0; c < 18; ++c) out[c * ld + k] = d[c];
}

// ---------------------------------------------------------------------------
// Minimizer: per-query air path (GetAirPropagationPar .cc:661-804 semantics).
// ---------------------------------------------------------------------------
struct AirPath {
  Endpoint tx;      // Tx height endpoint
  Endpoint iceair;  // air model at the (possibly depth-shifted) ice height
  Endpoint rtop;    // Rx endpoint of the top layer
  int top, bot;
};

__device__ __forceinline__ Endpoint stop_of(const DevMedium& M, int l) {
  Endpoint r = M.stop[0];
  r = pick(l == 1, M.stop[1], r);
  r = pick(l == 2, M.stop[2], r);
  r = pick(l == 3, M.stop[3], r);
  return r;
}

__device__ __forceinline__ AirPath make_air_path(const DevMedium& M, double H, double ice) {
  AirPath P;
  P.top = top_layer(M, H);
  P.bot = bottom_layer(M, ice);
  P.tx = air_endpoint(M, H);
  P.iceair = air_endpoint(M, ice);
  P.rtop = pick(P.top == P.bot, P.iceair, stop_of(M, P.top));
  P.rtop = pick(P.rtop.x == P.tx.x, P.tx, P.rtop);  // zero-length top segment
  return P;
}

// L of the first layer (GetLayerHitPointPar .cc:562-589 with n_layer1 == nzTx).
__device__ __forceinline__ double first_layer_L(const DevMedium& M, const AirPath& P, double theta) {
  const double sria = (180 - theta) * M.d2r;
  // (n_layer1/nzTx) is Getnz_air(Start)/Getnz_air(Start) == 1.0 exactly
  const double lang = asin(sin(sria));
  const double recv = asin((P.tx.n * sin(lang)) / P.rtop.n);
  return P.rtop.n * sin(recv);
}

// Sum of per-layer horizontal distances in air for launch angle theta (THD only:
// the time and geometric-path terms of the reference do not enter f).  Returns L0.
__device__ __forceinline__ double air_thd(const DevMedium& M, const AirPath& P, double theta,
                                          double& L0) {
  if (P.top < P.bot) {  // no layer: reference reads unset output slots (UB)
    L0 = __builtin_nan("");
    return 0.0;
  }
  const double L = first_layer_L(M, P, theta);
  L0 = L;
  const double LL = L * L;
  const double sAL = sqrt(M.A_air * M.A_air - LL);
  double thd = 0.0;
#pragma unroll
  for (int il = kMaxLayers - 1; il >= 0; --il) {
    if (il > P.top || il < P.bot) continue;
    const Endpoint T = pick(il == P.top, P.tx, M.start[il]);
    const Endpoint R = pick(il == P.top, P.rtop, pick(il == P.bot, P.iceair, M.stop[il]));
    double x1 = +prim_D(R, M.A_air, L, LL, sAL) - prim_D(T, M.A_air, L, LL, sAL);
    x1 *= -1;
    thd += x1;
  }
  return thd;
}

struct Query {
  AirPath P;
  Endpoint rx;      // ice endpoint at the antenna depth (if in ice)
  double dist;
  double depth_pos; // MinforLAng_params.antennadepth (> 0 in ice, 0 in air)
};

// MinimizeforLaunchAngle (.cc:873-917)
__device__ __forceinline__ double fmin_eval(const DevMedium& M, const IceConsts& I, const Query& q,
                                            double x) {
  double L;
  const double thd_air = air_thd(M, q.P, x, L);
  double thd_ice = 0;
  if (q.depth_pos != 0) {
    const double LL = L * L;
    const double sAL = sqrt(M.A_ice * M.A_ice - LL);
    thd_ice += +prim_D(q.rx, M.A_ice, L, LL, sAL) - prim_D(I.ice0, M.A_ice, L, LL, sAL);
  }
  return (q.dist - (thd_ice + thd_air));
}

struct SolveResult {
  double root;
  int status;
};

// FindFunctionRoot (.cc:340-374) with gsl_root_fsolver_bisection + gsl_root_test_interval
// semantics; an uninitialised solver state (non-finite endpoint) is modelled as zeros.
__device__ __forceinline__ SolveResult bisect(const DevMedium& M, const IceConsts& I,
                                              const Query& q, double x_lo, double x_hi) {
  SolveResult res{0.0, 0};
  if (x_lo > x_hi) {
    res.status |= AIRICE_SOLVE_BAD_BRACKET;
    return res;
  }
  double lo = x_lo, hi = x_hi;
  double root = 0.5 * (x_lo + x_hi);
  double f_lower = 0.0, f_upper = 0.0;
  const double fl = fmin_eval(M, I, q, lo);
  if (!isfinite(fl)) {
    res.status |= AIRICE_SOLVE_NONFINITE_END;
  } else {
    const double fu = fmin_eval(M, I, q, hi);
    if (!isfinite(fu)) {
      res.status |= AIRICE_SOLVE_NONFINITE_END;
    } else {
      f_lower = fl;
      f_upper = fu;
    }
  }
  const double tol = 0.000000001;
  bool cont = true;
  for (int iter = 1; iter <= 40 && cont; ++iter) {
    if (f_lower == 0.0) {
      root = lo;
      hi = lo;
    } else if (f_upper == 0.0) {
      root = hi;
      lo = hi;
    } else {
      const double xb = (lo + hi) / 2.0;
      const double fb = fmin_eval(M, I, q, xb);
      if (!isfinite(fb)) {
        // EBADFUNC leaves the state unchanged: every later iterate repeats this one,
        // so the driver ends at max_iter with the same root.
        res.status |= AIRICE_SOLVE_STALE_MID | AIRICE_SOLVE_MAXITER;
        break;
      } else if (fb == 0.0) {
        root = xb;
        lo = xb;
        hi = xb;
      } else if ((f_lower > 0.0 && fb < 0.0) || (f_lower < 0.0 && fb > 0.0)) {
        root = 0.5 * (lo + xb);
        hi = xb;
        f_upper = fb;
      } else {
        root = 0.5 * (xb + hi);
        lo = xb;
        f_lower = fb;
      }
    }
    if (lo > hi) {
      cont = false;
    } else {
      const double min_abs = ((lo > 0.0 && hi > 0.0) || (lo < 0.0 && hi < 0.0))
                                 ? (fabs(lo) < fabs(hi) ? fabs(lo) : fabs(hi))
                                 : 0.0;
      const double tolerance = 0 + tol * min_abs;
      cont = !(fabs(hi - lo) < tolerance);
    }
    if (cont && iter == 40) res.status |= AIRICE_SOLVE_MAXITER;
  }
  res.root = root;
  return res;
}

struct Solved {
  double launch, thd_air, t_air, geo_air, inc, thd_ice, t_ice, geo_ice, ant;
  double ice_h;  // IceLayerHeight after the Rx-in-air shift
  int status;
};

// Air2IceRayTracing (.cc:1464-1616) up to the outputs.
__device__ __forceinline__ Solved air2ice(const DevMedium& M, const IceConsts& I, double H,
                                          double D, double ice, double depth, double thR) {
  Solved S;
  S.status = 0;
  Query q;
  if (depth >= 0) {
    ice = depth + ice;
    depth = 0;
    q.depth_pos = depth;
  } else {
    q.depth_pos = -depth;
  }
  q.dist = D;
  q.P = make_air_path(M, H, ice);
  q.rx = ice_endpoint(M, q.depth_pos);
  S.ice_h = ice;

  double lo = thR - 16;
  double hi = thR;
  if (lo < 90.001) {
    lo = 90.001;
    bool checknan = false;
    while (!checknan && lo > 89.9) {
      double Ld;
      const double s = air_thd(M, q.P, lo, Ld);
      if ((!isnan(s) && s > 0) || lo > hi - 0.1) {
        checknan = true;
      } else {
        lo = lo + 0.05;
        S.status |= AIRICE_SOLVE_PROBED;
      }
    }
  }
  if (hi < 90.001 && hi > 90.00) hi = 90.05;
  const SolveResult r = bisect(M, I, q, lo, hi);
  S.status |= r.status;
  const double x = r.root;
  S.launch = x;

  // Final evaluation (GetAirPropagationPar + GetIcePropagationPar, .cc:1524-1566).
  S.thd_air = 0.0;
  S.t_air = 0.0;
  S.geo_air = 0.0;
  S.inc = __builtin_nan("");
  double L0 = __builtin_nan("");
  const AirPath& P = q.P;
  if (P.top < P.bot) S.status |= AIRICE_SOLVE_NO_AIR_LAYER;
  for (int il = P.top; il > P.bot - 1; --il) {
    Segment sg;
    if (il == P.top) {
      sg = segment_full(M, M.A_air, P.tx, P.rtop, P.tx.n, 180 - x, true);
      L0 = sg.L;
    } else {
      const Endpoint T = M.start[il];
      const Endpoint R = pick(il == P.bot, P.iceair, stop_of(M, il));
      sg = segment_with_L(M, M.A_air, T, R, L0, true);
    }
    S.thd_air += sg.thd;
    S.t_air += sg.t;
    S.geo_air += sg.geo;
    S.inc = sg.recv_deg;
  }
  S.thd_ice = 0.0;
  S.t_ice = 0.0;
  S.geo_ice = 0.0;
  S.ant = 0.0;
  if (depth < 0) {
    const Segment sg = segment_with_L(M, M.A_ice, I.ice0, q.rx, L0, false);
    S.thd_ice = sg.thd;
    S.ant = sg.recv_deg;
    S.t_ice = sg.t;
    S.geo_ice = sg.geo;
  }
  return S;
}

__device__ __forceinline__ double straight_angle(const DevMedium& M, double H, double D, double ice,
                                                 double depth) {
  double thR = 0;
  if (depth < 0) thR = 180 - (atan(D / (H - ice - depth)) * M.r2d);
  if (depth >= 0) thR = 180 - (atan(D / (H - (ice + depth))) * M.r2d);
  return thR;
}

template <int VARIANT>
__global__ __launch_bounds__(kBlock) void solve_kernel(DevMedium M, IceConsts I,
                                                       const double* __restrict__ txh,
                                                       const double* __restrict__ dist,
                                                       const double* __restrict__ depth,
                                                       const double* __restrict__ thr_in,
                                                       long long n, double* __restrict__ out,
                                                       size_t ld, uint8_t* __restrict__ status) {
  const long long k = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (k >= n) return;
  const double H = txh[k], D = dist[k], dep = depth[k];
  // StraightAngle argument of Air2IceRayTracing (.cc:1464); default: the thR that
  // GetHorizontalDistanceToIntersectionPoint forms (.cc:952-958).
  const double thR = thr_in != nullptr ? thr_in[k] : straight_angle(M, H, D, I.ice_h, dep);
  const Solved S = air2ice(M, I, H, D, I.ice_h, dep, thR);
  const double thd = S.thd_ice + S.thd_air;
  const double tt = S.t_ice + S.t_air;
  out[0 * ld + k] = H;
  out[1 * ld + k] = thd;
  out[2 * ld + k] = S.thd_air;
  out[3 * ld + k] = S.thd_ice;
  out[4 * ld + k] = tt * kSpeedC;
  out[5 * ld + k] = S.t_ice * kSpeedC;
  out[6 * ld + k] = S.t_air * kSpeedC;
  out[7 * ld + k] = tt;
  out[8 * ld + k] = S.t_ice;
  out[9 * ld + k] = S.t_air;
  out[10 * ld + k] = S.launch;
  const Endpoint iceair = air_endpoint(M, S.ice_h);
  if (VARIANT == AIRICE_VARIANT_MULTIRAY) {
    double tS, tP;
    fresnel_trans(iceair.n, I.ice0.n, S.inc * M.d2r, tS, tP);
    out[11 * ld + k] = S.ant;
    out[12 * ld + k] = tS;
    out[13 * ld + k] = tP;
    out[14 * ld + k] = S.geo_air;
    out[15 * ld + k] = S.geo_ice;
    out[16 * ld + k] = S.inc;
  } else {
    // pythonwrapper AirIceRayTracing.cc:1081-1084
    out[11 * ld + k] = asin((iceair.n / I.ice0.n) * sin(S.inc * M.d2r)) * M.r2d;
    out[12 * ld + k] = S.ant;
    out[13 * ld + k] = S.geo_air;
    out[14 * ld + k] = S.geo_ice;
  }
  if (status != nullptr) status[k] = (uint8_t)S.status;
}

// GetHorizontalDistanceToIntersectionPoint (.cc:945-989), cm in, 9 outputs + bool.
__global__ __launch_bounds__(kBlock) void hdtip_kernel(DevMedium M, IceConsts I,
                                                       const double* __restrict__ src_cm,
                                                       const double* __restrict__ dist_cm,
                                                       const double* __restrict__ depth_cm,
                                                       double ice_cm, long long n,
                                                       double* __restrict__ out, size_t ld,
                                                       uint8_t* __restrict__ ok) {
  const long long k = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (k >= n) return;
  const double H = src_cm[k] / 100, D = dist_cm[k] / 100, ice = ice_cm / 100,
               dep = depth_cm[k] / 100;
  const double thR = straight_angle(M, H, D, ice, dep);
  const Solved S = air2ice(M, I, H, D, ice, dep, thR);
  const double thd = S.thd_ice + S.thd_air;
  const Endpoint iceair = air_endpoint(M, S.ice_h);
  double tS, tP;
  fresnel_trans(iceair.n, I.ice0.n, S.inc * M.d2r, tS, tP);
  out[0 * ld + k] = (S.t_ice * kSpeedC) * 100;
  out[1 * ld + k] = (S.t_air * kSpeedC) * 100;
  out[2 * ld + k] = S.geo_ice * 100;
  out[3 * ld + k] = S.geo_air * 100;
  out[4 * ld + k] = S.launch * M.d2r;
  out[5 * ld + k] = S.thd_air * 100;
  out[6 * ld + k] = tS;
  out[7 * ld + k] = tP;
  out[8 * ld + k] = S.ant * M.d2r;
  bool good = false;
  if ((fabs(thd - D) / D < 0.01 && D <= 100) || (fabs(thd - D) < 1 && D > 100)) good = true;
  if (thd < 0) good = false;
  ok[k] = good ? 1 : 0;
}

// pythonwrapper TraceIceToAir (TraceIceToAir.C:5-73) with GetRayTracingSolution
// (AirIceRayTracing.cc:884-927); per-query ice height.
__global__ __launch_bounds__(kBlock) void trace_kernel(DevMedium M, IceConsts I,
                                                       const double* __restrict__ depth,
                                                       const double* __restrict__ iceh,
                                                       const double* __restrict__ txh,
                                                       const double* __restrict__ dist,
                                                       long long n, double* __restrict__ out10) {
  const long long k = (long long)blockIdx.x * kBlock + threadIdx.x;
  if (k >= n) return;
  const double H = txh[k], D = dist[k], ice = iceh[k], dep = depth[k];
  const double thR = straight_angle(M, H, D, ice, dep);
  const Solved S = air2ice(M, I, H, D, ice, dep, thR);
  const double thd = S.thd_ice + S.thd_air;
  const Endpoint iceair = air_endpoint(M, S.ice_h);
  const double aoi = asin((iceair.n / I.ice0.n) * sin(S.inc * M.d2r)) * M.r2d;
  bool good = false;
  if ((fabs(thd - D) / D < 0.01 && D <= 100) || (fabs(thd - D) < 1 && D > 100)) good = true;
  if (thd < 0) good = false;
  double* o = out10 + 10 * k;
  if (good) {
    // swap(launch, received); received = 180 - received (TraceIceToAir.C:33-34)
    o[0] = H;
    o[1] = D;
    o[2] = S.geo_ice;
    o[3] = S.geo_air;
    o[4] = S.ant;
    o[5] = 180 - S.launch;
    o[6] = S.thd_air;
    o[7] = aoi;
    o[8] = 0;
    o[9] = 0;
  } else {
#pragma unroll
    for (int c = 0; c < 10; ++c) o[c] = -1000;
  }
}

// ---------------------------------------------------------------------------
// Host launchers
// ---------------------------------------------------------------------------
static inline unsigned grid_for(long long n) { return (unsigned)((n + kBlock - 1) / kBlock); }

int launch_table(const DevMedium& M, const IceConsts& I, const airice_grid* g, int row_begin,
                 int row_count, float* d_table, double* d_full, size_t ld, hipStream_t st) {
  TableArgs A;
  A.start_h = g->start_height;
  A.stop_h = g->stop_height;
  A.step_h = g->height_step;
  A.start_a = g->start_angle;
  A.stop_a = g->stop_angle;
  A.step_a = g->angle_step;
  A.hsteps = g->height_steps;
  A.asteps = g->angle_steps;
  A.row0 = row_begin;
  A.in_ice = g->in_ice;
  A.n = (long long)row_count * g->angle_steps;
  A.ld = ld;
  if (A.n == 0) return AIRICE_OK;
  hipLaunchKernelGGL(table_kernel, dim3(grid_for(A.n)), dim3(kBlock), 0, st, M, I, A, d_table,
                     d_full);
  return hipGetLastError() == hipSuccess ? AIRICE_OK : AIRICE_EHIP;
}

int launch_rays(const DevMedium& M, const IceConsts& I, const double* launch, const double* txh,
                int in_ice, size_t n, double* out, size_t ld, hipStream_t st) {
  if (n == 0) return AIRICE_OK;
  hipLaunchKernelGGL(rays_kernel, dim3(grid_for((long long)n)), dim3(kBlock), 0, st, M, I, launch,
                     txh, in_ice, (long long)n, out, ld);
  return hipGetLastError() == hipSuccess ? AIRICE_OK : AIRICE_EHIP;
}

int launch_solve(const DevMedium& M, const IceConsts& I, int variant, const double* txh,
                 const double* dist, const double* depth, const double* thr, size_t n,
                 double* out, size_t ld, uint8_t* status, hipStream_t st) {
  if (n == 0) return AIRICE_OK;
  if (variant == AIRICE_VARIANT_MULTIRAY)
    hipLaunchKernelGGL(solve_kernel<AIRICE_VARIANT_MULTIRAY>, dim3(grid_for((long long)n)),
                       dim3(kBlock), 0, st, M, I, txh, dist, depth, thr, (long long)n, out, ld,
                       status);
  else
    hipLaunchKernelGGL(solve_kernel<AIRICE_VARIANT_PYWRAPPER>, dim3(grid_for((long long)n)),
                       dim3(kBlock), 0, st, M, I, txh, dist, depth, thr, (long long)n, out, ld,
                       status);
  return hipGetLastError() == hipSuccess ? AIRICE_OK : AIRICE_EHIP;
}

int launch_hdtip(const DevMedium& M, const IceConsts& I, const double* src, const double* dist,
                 const double* depth, double ice_cm, size_t n, double* out, size_t ld,
                 uint8_t* ok, hipStream_t st) {
  if (n == 0) return AIRICE_OK;
  hipLaunchKernelGGL(hdtip_kernel, dim3(grid_for((long long)n)), dim3(kBlock), 0, st, M, I, src,
                     dist, depth, ice_cm, (long long)n, out, ld, ok);
  return hipGetLastError() == hipSuccess ? AIRICE_OK : AIRICE_EHIP;
}

int launch_trace(const DevMedium& M, const IceConsts& I, const double* depth, const double* ice,
                 const double* txh, const double* dist, size_t n, double* out10, hipStream_t st) {
  if (n == 0) return AIRICE_OK;
  hipLaunchKernelGGL(trace_kernel, dim3(grid_for((long long)n)), dim3(kBlock), 0, st, M, I, depth,
                     ice, txh, dist, (long long)n, out10);
  return hipGetLastError() == hipSuccess ? AIRICE_OK : AIRICE_EHIP;
}

}  // namespace airice
