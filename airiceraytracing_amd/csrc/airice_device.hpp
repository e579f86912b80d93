// airice_device.hpp -- FP64 device math of the air->ice ray solver (gfx950).
//
// One ray (table) or one query (minimizer) per lane.  Every expression keeps the
// reference's evaluation order (MultiRayAirIceRefraction.cc:377-447 antiderivatives,
// :521-646 segment, :661-869 propagation, :1796-2017 forward ray) and is compiled with
// -ffp-contract=off, so device results differ from the CPU/GSL path only by the
// ulp-level differences of ocml vs glibc transcendentals.
//
// What is NOT a translation: identical pure sub-expressions are computed once
// (exp(C x) is shared by n(z), fDnfR, ftimeD, fpathD; sqrt(n^2-L^2) and the first
// log are shared by fDnfR and ftimeD), and every endpoint that does not depend on
// the ray (layer boundaries, the ice surface, the antenna depth of a table) is
// evaluated once on the host and passed in the kernel-argument block (SGPRs), so
// only the Tx endpoint needs device exp() -- the reference re-evaluates n(z) and
// the layer scan ~hundreds of times per ray.
#pragma once
#include <hip/hip_runtime.h>

namespace airice {

constexpr int kMaxLayers = 4;  // ATMLAY has 5 bounds -> at most 4 air layers

// One endpoint of a segment: the analytic antiderivatives need, at height/depth x,
//   C = the "c" parameter (= -C_layer, .cc:455-461), B, e = exp(C x), e2 = exp(2 C x),
//   y = A + B e (fDnfR/fpathD form) and n = Getnz(x) (ftimeD form; == y for x >= 0).
struct Endpoint {
  double x, C, B, e, e2, y, n;
};

struct DevMedium {
  double atm[5];    // ATMLAY[i]/100, m
  double B[5];      // B_air
  double negC[5];   // -C_air
  double A_air, A_ice, B_ice, negC_ice;
  double d2r;       // pi/180.0   (.cc:537)
  double r2d;       // 180/pi     (.cc:640)
  int ml;           // MaxLayers
  int pad_;
  Endpoint start[kMaxLayers];  // layer l start: x = ATMLAY[l+1]/100 - 1e-5 (.cc:1846)
  Endpoint stop[kMaxLayers];   // layer l stop:  x = ATMLAY[l]/100          (.cc:1858)
};

// Per-launch endpoints that are uniform over the batch.
struct IceConsts {
  double ice_h;        // IceLayerHeight (m) of the launch
  Endpoint ice_air;    // air model at the ice height (stop of the lowest air layer)
  Endpoint ice0;       // ice model at depth 0 (.cc:1899)
  Endpoint ice_rx;     // ice model at the antenna depth (table: uniform)
  double n1_over_n2;   // Getnz_air(ice)/Getnz_ice(0) (Trans_S/P, .cc:287-292)
};

__device__ __forceinline__ double sel4(const double (&a)[5], int l) {
  double r = a[0];
  r = (l == 1) ? a[1] : r;
  r = (l == 2) ? a[2] : r;
  r = (l == 3) ? a[3] : r;
  r = (l == 4) ? a[4] : r;
  return r;
}

// Air layer of |z| (GetB_air/GetC_air scan, .cc:221-230).
__device__ __forceinline__ int air_layer(const DevMedium& M, double zabs) {
  int which = 0;
  bool found = false;
#pragma unroll
  for (int l = 0; l < kMaxLayers; ++l) {
    if (l < M.ml - 1 && !found && zabs < M.atm[l + 1] && zabs >= M.atm[l]) {
      which = l;
      found = true;
    }
  }
  if (zabs >= sel4(M.atm, M.ml - 1)) which = M.ml - 1;
  return which;
}

__device__ __forceinline__ Endpoint air_endpoint(const DevMedium& M, double x) {
  Endpoint p;
  const double zabs = fabs(x);
  const int l = air_layer(M, zabs);
  p.x = x;
  p.B = sel4(M.B, l);
  p.C = sel4(M.negC, l);
  const double eabs = exp(p.C * zabs);
  p.n = M.A_air + p.B * eabs;
  if (x >= 0.0) {
    p.e = eabs;
    p.y = p.n;
  } else {
    p.e = exp(p.C * x);
    p.y = M.A_air + p.B * p.e;
  }
  p.e2 = exp(2 * p.C * x);
  return p;
}

__device__ __forceinline__ Endpoint ice_endpoint(const DevMedium& M, double x) {
  Endpoint p;
  const double zabs = fabs(x);
  p.x = x;
  p.B = M.B_ice;
  p.C = M.negC_ice;
  const double eabs = exp(p.C * zabs);
  p.n = M.A_ice + p.B * eabs;
  if (x >= 0.0) {
    p.e = eabs;
    p.y = p.n;
  } else {
    p.e = exp(p.C * x);
    p.y = M.A_ice + p.B * p.e;
  }
  p.e2 = exp(2 * p.C * x);
  return p;
}

__device__ __forceinline__ Endpoint pick(bool c, const Endpoint& a, const Endpoint& b) {
  Endpoint r;
  r.x = c ? a.x : b.x;
  r.C = c ? a.C : b.C;
  r.B = c ? a.B : b.B;
  r.e = c ? a.e : b.e;
  r.e2 = c ? a.e2 : b.e2;
  r.y = c ? a.y : b.y;
  r.n = c ? a.n : b.n;
  return r;
}

// Antiderivatives at one endpoint for a ray parameter L (sAL = sqrt(A*A-L*L), LL = L*L).
// fDnfR .cc:385, ftimeD .cc:424/427, fpathD .cc:445 -- operand order kept.
struct Prims {
  double D, T, G;
};

__device__ __forceinline__ double prim_D(const Endpoint& P, double A, double L, double LL,
                                         double sAL) {
  const double s = sqrt(P.y * P.y - LL);
  const double lg = log(A * P.y - LL + sAL * s);
  return (L / P.C) * (1.0 / sAL) * (P.C * P.x - lg);
}

__device__ __forceinline__ Prims prim_all(const Endpoint& P, double A, double L, double LL,
                                          double sAL, double speedc) {
  Prims r;
  // fDnfR
  const double sy = sqrt(P.y * P.y - LL);
  const double lgy = log(A * P.y - LL + sAL * sy);
  const double Cx = P.C * P.x;
  r.D = (L / P.C) * (1.0 / sAL) * (Cx - lgy);
  // ftimeD: same sqrt/log when n == y (x >= 0)
  double sn = sy, lgn = lgy;
  if (P.n != P.y) {
    sn = sqrt(P.n * P.n - LL);
    lgn = log(A * P.n - LL + sAL * sn);
  }
  r.T = (1.0 / (speedc * P.C * sn)) *
        (P.n * P.n - LL + (Cx - lgn) * (A * A * sn) / sAL + A * sn * log(P.n + sn));
  // fpathD
  const double Q = (A * A + 2 * A * P.B * P.e + P.B * P.B * P.e2 - LL) / (P.y * P.y);
  const double sq = sqrt(Q);
  r.G = (log(P.y * (sq + 1)) -
         (A * log(A * sAL * sq + P.B * sAL * P.e * sq + A * A + A * P.B * P.e - LL)) / sAL +
         (A * P.C * P.x) / sAL) /
        P.C;
  return r;
}

struct Segment {
  double thd, recv_deg, L, t, geo;
};

// GetLayerHitPointPar (.cc:521-646): Tx endpoint T, Rx endpoint R, incoming index n1,
// incidence angle in degrees.  air: results negated (.cc:464-466, 486-488, 508-510).
__device__ __forceinline__ Segment segment_full(const DevMedium& M, double A, const Endpoint& T,
                                                const Endpoint& R_, double n1, double inc_deg,
                                                bool air) {
  const double speedc = 299792458.0;
  // Same height -> the reference evaluates the same function of the same x at both
  // ends (zero-length segment, exactly 0 or NaN); endpoints built on host and device
  // can differ by an ulp, so reuse one.
  const Endpoint R = pick(R_.x == T.x, T, R_);
  const double sria = inc_deg * M.d2r;
  const double lang = asin((n1 / T.n) * sin(sria));
  const double recv = asin((T.n * sin(lang)) / R.n);
  const double L = R.n * sin(recv);
  const double LL = L * L;
  const double sAL = sqrt(A * A - LL);
  const Prims pr = prim_all(R, A, L, LL, sAL, speedc);
  const Prims pt = prim_all(T, A, L, LL, sAL, speedc);
  Segment s;
  s.thd = +pr.D - pt.D;
  s.t = +pr.T - pt.T;
  s.geo = pr.G - pt.G;
  if (air) {
    s.thd *= -1;
    s.t *= -1;
    s.geo *= -1;
  }
  s.recv_deg = recv * M.r2d;
  s.L = L;
  return s;
}

// Segment with a given L (GetAirPropagationPar lower layers .cc:757-771, GetIcePropagationPar
// .cc:820-827): receive angle asin(L/n(Rx)).
__device__ __forceinline__ Segment segment_with_L(const DevMedium& M, double A, const Endpoint& T,
                                                  const Endpoint& R_, double L, bool air) {
  const double speedc = 299792458.0;
  const Endpoint R = pick(R_.x == T.x, T, R_);  // zero-length segment, see segment_full
  const double LL = L * L;
  const double sAL = sqrt(A * A - LL);
  const Prims pr = prim_all(R, A, L, LL, sAL, speedc);
  const Prims pt = prim_all(T, A, L, LL, sAL, speedc);
  Segment s;
  s.thd = +pr.D - pt.D;
  s.t = +pr.T - pt.T;
  s.geo = pr.G - pt.G;
  if (air) {
    s.thd *= -1;
    s.t *= -1;
    s.geo *= -1;
  }
  s.recv_deg = asin(L / R.n) * M.r2d;
  s.L = L;
  return s;
}

// Layer-skip scans (.cc:1798-1825): top = MaxLayers-SkipLayersAbove-1, bottom = SkipLayersBelow.
__device__ __forceinline__ int top_layer(const DevMedium& M, double txh) {
  int skip = 0;
  for (int il = M.ml; il > -1; il--) {
    const bool hit = (txh < sel4(M.atm, il)) && (il >= 1 ? (txh >= sel4(M.atm, il - 1)) : false);
    if (hit) break;
    skip++;
  }
  return M.ml - skip - 1;
}

__device__ __forceinline__ int bottom_layer(const DevMedium& M, double ice_h) {
  int skip = 0;
  for (int il = 0; il < M.ml; il++) {
    if (ice_h >= sel4(M.atm, il) && ice_h < sel4(M.atm, il + 1)) break;
    skip++;
  }
  return skip;
}

// Fresnel amplitude transmission (.cc:285-337), thetai in radians.
__device__ __forceinline__ void fresnel_trans(double n1, double n2, double thetai, double& tS,
                                              double& tP) {
  const double a = (n1 / n2) * (sin(thetai));
  const double sqterm = sqrt(1 - a * a);
  const double ct = cos(thetai);
  double num = n1 * ct - n2 * sqterm;
  double den = n1 * ct + n2 * sqterm;
  tS = 1 + (num / den);
  if (isnan(tS)) tS = 0;
  num = n1 * sqterm - n2 * ct;
  den = n1 * sqterm + n2 * ct;
  tP = (1 - (num / den)) * (n1 / n2);
  if (isnan(tP)) tP = 0;
}

}  // namespace airice
