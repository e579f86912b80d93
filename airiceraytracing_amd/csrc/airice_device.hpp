// airice_device.hpp -- FP64 device math of the air->ice ray solver (gfx950).
//
// One ray (table) or one query (minimizer) per lane; FP64 throughout, compiled with
// -ffp-contract=off.  The closed forms are those of the reference
// (MultiRayAirIceRefraction.cc: fDnfR :377-386, ftimeD :412-431, fpathD :434-447,
// GetLayerHitPointPar :521-646), evaluated with fewer operations; every rewrite below is an
// exact identity whose only effect is ulp-level rounding (parity <= 1e-9 relative is checked
// on the full BASELINE grids in tests/test_gpu_parity.py):
//
//  (1) fpathD.  With y = A + B e^{Cx} and e^{2Cx} = (e^{Cx})^2 its radicand is
//      Q = (A^2 + 2ABe + B^2e^2 - L^2)/y^2 = (y^2 - L^2)/y^2, so sqrt(Q) = s/y with
//      s = sqrt(y^2 - L^2), and its two logarithms are log(y + s) (== ftimeD's log(n + s))
//      and log(A y - L^2 + sqrt(A^2-L^2) s) (== fDnfR's log).  fpathD costs no extra
//      transcendental; exp(2Cx) disappears.
//  (2) sin(asin(u)) == u for |u| <= 1 (NaN otherwise).  The reference's per-layer chain
//      angle -> sin -> asin -> sin -> asin -> sin -> degrees -> next layer collapses to one
//      running sine v: L = n_Rx * v_Rx, v_next = v_Rx.  asin is evaluated only where an angle
//      is an output (incidence on the ice, receive angle at the antenna).
//  (3) Divisions by per-segment / per-layer constants become products with their reciprocal
//      (1/sqrt(A^2-L^2) is already a factor of fDnfR; 1/C is precomputed per layer).
//  (5) Both ends of every segment lie in one layer (same C), so F(R) - F(T) of each
//      antiderivative needs log(a_R / a_T) instead of log(a_R) - log(a_T), and ftimeD's
//      (n^2 - L^2)/sqrt(n^2 - L^2) term is sqrt(n^2 - L^2): per segment 2 logarithms instead
//      of the reference's 12 (3 functions x 2 logs x 2 ends).
//  (4) Endpoint quantities that do not depend on the ray (layer boundaries, the ice surface,
//      a table's antenna depth) are evaluated once on the host and passed in the kernel-argument
//      block (SGPRs / scalar cache); only the Tx endpoint costs a device exp().
#pragma once
#include <hip/hip_runtime.h>

#include <cmath>

#include "airice_tlog.hpp"

namespace airice {

constexpr int kMaxLayers = 4;  // ATMLAY has 5 bounds -> at most 4 air layers

// One end of a segment at height/depth x in a medium n(z) = A + B exp(C |z|) (C < 0 here:
// C is the "c" parameter the reference passes, -C_layer, .cc:455-461).
//   y = A + B exp(C x)   (fDnfR / fpathD form),   n = Getnz(x) = A + B exp(C |x|)  (ftimeD form)
struct Endpoint {
  double x, C, invC, y, n;
  double Ay, y2, n2, An, Cx, ACx;  // A*y, y*y, n*n, A*n, C*x, (A*C)*x
};

__host__ __device__ inline Endpoint make_endpoint(double A, double B, double C, double x,
                                                  double e_abs, double e_x) {
  Endpoint p;
  p.x = x;
  p.C = C;
  p.invC = 1.0 / C;
  p.n = A + B * e_abs;
  p.y = (x >= 0.0) ? p.n : A + B * e_x;
  p.Ay = A * p.y;
  p.y2 = p.y * p.y;
  p.n2 = p.n * p.n;
  p.An = A * p.n;
  p.Cx = C * x;
  p.ACx = (A * C) * x;
  return p;
}

struct DevMedium {
  double atm[5];    // ATMLAY[i]/100, m
  double B[5];      // B_air
  double negC[5];   // -C_air
  double A_air, A_ice, B_ice, negC_ice;
  double d2r;       // pi/180.0   (.cc:537)
  double r2d;       // 180/pi     (.cc:640)
  int ml;           // MaxLayers
  int const_air;   // pythonwrapper UseConstantRefractiveIndex: bracket [90, thR], no probe
  Endpoint start[kMaxLayers];  // layer l start: x = ATMLAY[l+1]/100 - 1e-5 (.cc:1846)
  Endpoint stop[kMaxLayers];   // layer l stop:  x = ATMLAY[l]/100          (.cc:1858)
};

// A segment whose two ends are known before launch (the lower air layers of a ray, a table's
// ice segment): everything the closed forms need from the ends, folded on the host so the
// kernel reads them as scalars (no SGPR-SGPR arithmetic, no selects).
struct SegConst {
  double Tn, Ty2, TAy;  // start end: n, y^2, A*y
  double Rn, Ry2, RAy;  // stop end
  double ratio;         // Tn / Rn: Snell step sin(recv) = (Tn/Rn) sin(lang)
  double invC, invCc;   // 1/C, 1/(C c)
  double dCx, dACx;     // R.Cx - T.Cx, R.ACx - T.ACx
};

// Stop end of the first (Tx) layer of a ray, indexed by that layer: the layer's lower bound,
// or the ice when the layer is the lowest one.
struct TopEnd {
  double x, n, y2, Ay, invC, invCc, Cx, ACx;
};

// Per-launch constants that are uniform over the batch.
struct IceConsts {
  double ice_h;        // IceLayerHeight (m) of the launch
  Endpoint ice_air;    // air model at the ice height (stop of the lowest air layer)
  Endpoint ice0;       // ice model at depth 0 (.cc:1899)
  Endpoint ice_rx;     // ice model at the antenna depth (table: uniform)
  int bot;             // lowest air layer (layer of the ice height, .cc:1815-1825)
  int pad_;
  SegConst lower[kMaxLayers];  // layer l as a lower layer: start[l] -> (l == bot ? ice : stop[l])
  TopEnd topend[kMaxLayers];   // layer l as the Tx layer: its stop end
  SegConst iceseg;             // ice surface -> antenna (table)
  double n_air_ice, n_ice0;    // Getnz_air(ice), Getnz_ice(0) (Snell into the ice, Fresnel)
  double n_ratio;              // n_air_ice / n_ice0 (IEEE quotient, folded on the host)
};

__host__ __device__ inline SegConst make_segconst(const Endpoint& T, const Endpoint& R) {
  const double speedc = 299792458.0;
  SegConst s;
  s.Tn = T.n;
  s.Ty2 = T.y2;
  s.TAy = T.Ay;
  s.Rn = R.n;
  s.Ry2 = R.y2;
  s.RAy = R.Ay;
  s.ratio = T.n / R.n;
  s.invC = R.invC;
  s.invCc = R.invC * (1.0 / speedc);
  s.dCx = R.Cx - T.Cx;
  s.dACx = R.ACx - T.ACx;
  return s;
}

__host__ __device__ inline TopEnd make_topend(const Endpoint& R) {
  const double speedc = 299792458.0;
  return TopEnd{R.x, R.n, R.y2, R.Ay, R.invC, R.invC * (1.0 / speedc), R.Cx, R.ACx};
}

__host__ __device__ __forceinline__ double sel5(const double (&a)[5], int l) {
  double r = a[0];
  r = (l == 1) ? a[1] : r;
  r = (l == 2) ? a[2] : r;
  r = (l == 3) ? a[3] : r;
  r = (l == 4) ? a[4] : r;
  return r;
}

// Air layer of |z| (GetB_air/GetC_air scan, .cc:221-230).
__host__ __device__ __forceinline__ int air_layer(const DevMedium& M, double zabs) {
  int which = 0;
  bool found = false;
#pragma unroll
  for (int l = 0; l < kMaxLayers; ++l) {
    if (l < M.ml - 1 && !found && zabs < M.atm[l + 1] && zabs >= M.atm[l]) {
      which = l;
      found = true;
    }
  }
  if (zabs >= sel5(M.atm, M.ml - 1)) which = M.ml - 1;
  return which;
}

__host__ __device__ __forceinline__ Endpoint air_endpoint(const DevMedium& M, double x) {
  const double zabs = fabs(x);
  const int l = air_layer(M, zabs);
  const double B = sel5(M.B, l), C = sel5(M.negC, l);
  const double e_abs = exp(C * zabs);
  const double e_x = (x >= 0.0) ? e_abs : exp(C * x);
  return make_endpoint(M.A_air, B, C, x, e_abs, e_x);
}

__host__ __device__ __forceinline__ Endpoint ice_endpoint(const DevMedium& M, double x) {
  const double zabs = fabs(x);
  const double e_abs = exp(M.negC_ice * zabs);
  const double e_x = (x >= 0.0) ? e_abs : exp(M.negC_ice * x);
  return make_endpoint(M.A_ice, M.B_ice, M.negC_ice, x, e_abs, e_x);
}

__host__ __device__ __forceinline__ Endpoint pick(bool c, const Endpoint& a, const Endpoint& b) {
  Endpoint r;
  r.x = c ? a.x : b.x;
  r.C = c ? a.C : b.C;
  r.invC = c ? a.invC : b.invC;
  r.y = c ? a.y : b.y;
  r.n = c ? a.n : b.n;
  r.Ay = c ? a.Ay : b.Ay;
  r.y2 = c ? a.y2 : b.y2;
  r.n2 = c ? a.n2 : b.n2;
  r.An = c ? a.An : b.An;
  r.Cx = c ? a.Cx : b.Cx;
  r.ACx = c ? a.ACx : b.ACx;
  return r;
}

// A result store at agent scope (device: a relaxed atomic store, i.e. global_store ... sc1, a
// vector store); the host pass stores plainly.  Used for the kernels' streamed output columns.
template <typename T>
__host__ __device__ __forceinline__ void st_agent(T* p, T v) {
#if defined(__HIP_DEVICE_COMPILE__)
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
  *p = v;
#endif
}

// sin(asin(u)): u on the domain of asin, NaN outside it (identity (2)).
__host__ __device__ __forceinline__ double sin_asin(double u) { return (fabs(u) <= 1.0) ? u : __builtin_nan(""); }

// Per-segment constants of the ray parameter L.
struct RayL {
  double L, LL, sAL, rsAL;  // L, L^2, sqrt(A^2-L^2), 1/sqrt(A^2-L^2)
};

// High 32 bits (sign, exponent, top of the mantissa) of a double.
__host__ __device__ __forceinline__ uint32_t hi_word(double x) {
  return (uint32_t)(__builtin_bit_cast(uint64_t, x) >> 32);
}

// sqrt(q) and 1/sqrt(q) together from one v_rsq_f64 and Goldschmidt/Newton refinement (the
// iteration ocml's sqrt uses, without its denormal rescaling: q here is a difference of squares of
// O(1) refractive indices); both within ~1 ulp.  q = 0 gives (0, +inf) and q < 0 / NaN gives NaNs,
// as sqrt() and 1/sqrt() do.
__host__ __device__ __forceinline__ void sqrt_rsqrt(double q, double& s, double& rs) {
#if !defined(__HIP_DEVICE_COMPILE__)
  // host (the one-query calls, AIRICE_SCALAR): the correctly rounded forms (<= 1 ulp from the
  // device iteration)
  s = std::sqrt(q);
  rs = 1.0 / s;
  return;
#else
  const double y = __builtin_amdgcn_rsq(q);
  double g = q * y, h = 0.5 * y;
  double e = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, e, g);
  h = __builtin_fma(h, e, h);
  double d = __builtin_fma(-g, g, q);
  g = __builtin_fma(d, h, g);
  e = __builtin_fma(-h, g, 0.5);
  h = __builtin_fma(h, e, h);
  s = (q == 0.0) ? q : g;
  rs = (q == 0.0) ? __builtin_inf() : 2.0 * h;
#endif
}

// sqrt(q) (same iteration, no reciprocal): within ~1 ulp; q = 0 -> 0, q < 0 / NaN -> NaN.
// The q = 0 case needs no select: v_rsq_f64(q + 2^-1074) is finite at q = 0, and the added
// 2^-1074 leaves every q >= 2^-1020 (and every q <= 0, NaN) unchanged.
__host__ __device__ __forceinline__ double fast_sqrt(double q) {
#if !defined(__HIP_DEVICE_COMPILE__)
  return std::sqrt(q);  // host: correctly rounded (the device iteration is within ~1 ulp of it)
#else
  const double y = __builtin_amdgcn_rsq(q + 0x1p-1074);
  double g = q * y, h = 0.5 * y;
  const double e = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, e, g);
  h = __builtin_fma(h, e, h);
  const double d = __builtin_fma(-g, g, q);
  g = __builtin_fma(d, h, g);
  return g;  // q = 0: y finite, so g = 0 * y = 0 through every step
#endif
}

// a / b for b positive and normal (2^-1000 <= b < 2^1000): v_rcp_f64 (24 bits, measured by
// tools/rcp_rsq_accuracy.hip), one Newton step (48 bits), quotient and one residual correction
// (Markstein) -- the IEEE quotient but for rare last-bit cases.  Other b, and a non-finite
// result (an infinite or NaN a, an overflowing quotient: the residual is then NaN), take the IEEE
// division (tests/test_device_prims.py forces each case).
__host__ __device__ __forceinline__ double div_pos(double a, double b) {
#if !defined(__HIP_DEVICE_COMPILE__)
  return a / b;  // host: the IEEE quotient (the device form's value but for rare last bits)
#else
  if (!(hi_word(b) - 0x01700000u < 0x7D000000u)) return a / b;
  double y = __builtin_amdgcn_rcp(b);
  y = __builtin_fma(y, __builtin_fma(-b, y, 1.0), y);
  const double q0 = a * y;
  const double q = __builtin_fma(__builtin_fma(-b, q0, a), y, q0);
  if (__builtin_expect(!__builtin_isfinite(q), 0)) return a / b;
  return q;
#endif
}

// asin(x) (radians): t + t^3 P(t^2) on |x| < 1/2 (P: degree-12 fit, tools/gen_asin_poly.py, error
// 1.2e-16 relative), pi/2 - 2 asin(sqrt((1 - |x|)/2)) above (1 - |x| exact there); NaN for
// |x| > 1 or NaN, as asin().  ~25 FP64 ops against ~64 for ocml's asin (tools/opweights.json).
__host__ __device__ __forceinline__ double asin_fast(double x) {
  const double ax = fabs(x);
  const bool big = ax >= 0.5;
  const double s = big ? 0.5 * (1.0 - ax) : ax * ax;
  const double t = big ? fast_sqrt(s) : ax;
  double p = __builtin_fma(s, kc(0x1.d72b2bc8155f8p-6), kc(-0x1.e6aaa8a0a04ccp-7));
  p = __builtin_fma(s, p, kc(0x1.1d189408314eep-6));
  p = __builtin_fma(s, p, kc(0x1.65a9c4dfcf8b2p-8));
  p = __builtin_fma(s, p, kc(0x1.52420b04b37bep-7));
  p = __builtin_fma(s, p, kc(0x1.782651caa6547p-7));
  p = __builtin_fma(s, p, kc(0x1.c9cf07674736ap-7));
  p = __builtin_fma(s, p, kc(0x1.1c4d35cf95421p-6));
  p = __builtin_fma(s, p, kc(0x1.6e8bb1c8209a2p-6));
  p = __builtin_fma(s, p, kc(0x1.f1c71c1db0623p-6));
  p = __builtin_fma(s, p, kc(0x1.6db6db6e31f13p-5));
  p = __builtin_fma(s, p, kc(0x1.3333333332ecap-4));
  p = __builtin_fma(s, p, kc(0x1.5555555555556p-3));
  const double r = __builtin_fma(t * s, p, t);
  const double y = big ? __builtin_fma(-2.0, r, 0x1.921fb54442d18p+0) : r;
  return __builtin_copysign(y, x);
}

// asin for the kernels' angle outputs
__host__ __device__ __forceinline__ double k_asin(double x) { return asin_fast(x); }

__host__ __device__ __forceinline__ RayL ray_L(double A2, double L) {
  RayL r;
  r.L = L;
  r.LL = L * L;
  sqrt_rsqrt(A2 - r.LL, r.sAL, r.rsAL);
  return r;
}

struct Segment {
  double thd, t, geo;
};

// F(R) - F(T) for the three antiderivatives; air results negated (.cc:464-466, 486-488,
// 508-510).  A segment whose ends are at the same height is exactly 0 (or NaN) in the
// reference: the same function of the same x at both ends.  Endpoints built on the host
// and on the device can differ by an ulp, so one endpoint is reused.
// Natural log: the table-driven tlog() of airice_tlog.hpp (< 1 ulp, no division, IEEE special
// values; its g++-compiled twin is the bit reference in tests/test_tlog.py).
__host__ __device__ __forceinline__ double fast_log(double x) { return tlog(x); }

// log(a) - log(b) as one logarithm (identity (5)).  Fast path -- a, b and a/b positive and
// within 2^+-1000, i.e. every ray except special values -- takes the quotient from v_rcp_f64
// refined by two Newton steps and one residual correction (Markstein; the IEEE quotient in all
// but rare last-bit cases) and the table log without its special-value handling.  Otherwise:
// the IEEE division and the IEEE value of log(a) - log(b) (-inf - finite, finite - (-inf), NaN).
__host__ __device__ __forceinline__ double log_ratio_fast(double a, double b, const double* tab, bool& ok) {
#if !defined(__HIP_DEVICE_COMPILE__)
  // host: the IEEE quotient, the same positive-normal test
  const double qh = a / b;
  ok = std::fpclassify(b) == FP_NORMAL && b > 0.0 && std::fpclassify(qh) == FP_NORMAL && qh > 0.0;
  return tlog_lean(qh, tab);
#else
  double y = __builtin_amdgcn_rcp(b);
  y = __builtin_fma(y, __builtin_fma(-b, y, 1.0), y);
  const double q0 = a * y;
  const double q = __builtin_fma(__builtin_fma(-b, q0, a), y, q0);
  // a > 0 and q in range cover a (a tiny / huge / inf / NaN shows in q or in a > 0); b in range
  // keeps v_rcp_f64 and the Newton steps clear of overflow and denormals
  // b and q positive normal (class mask 1 << 8): a <= 0 or NaN, b <= 0, NaN, denormal or so
  // large that v_rcp_f64 leaves the normal range, and q zero, denormal, infinite or NaN all fail;
  // with b > 0 and q > 0 also a > 0
  ok = __builtin_amdgcn_class(b, 1 << 8) && __builtin_amdgcn_class(q, 1 << 8);
  return tlog_lean(q, tab);  // garbage, and unused, when !ok
#endif
}

__host__ __device__ __forceinline__ double log_ratio_ieee(double a, double b) {
  const double special = (a == 0.0 && b > 0.0)   ? -__builtin_inf()
                         : (b == 0.0 && a > 0.0) ? __builtin_inf()
                                                 : __builtin_nan("");
  return (a > 0.0 && b > 0.0) ? tlog(a / b) : special;
}

__host__ __device__ __forceinline__ double log_ratio(double a, double b,
                                            const double* tab = &kLogTable[0][0]) {
  bool ok;
  const double r = log_ratio_fast(a, b, tab, ok);
  if (ok) return r;
  return log_ratio_ieee(a, b);
}

// The two log-ratios of a segment: both fast paths straight-line (so their table loads and
// polynomials overlap), then one rarely taken branch for special values.
__host__ __device__ __forceinline__ void log_ratio2(double a1, double b1, double a2, double b2,
                                           const double* tab, double& d1, double& d2) {
  bool ok1, ok2;
  d1 = log_ratio_fast(a1, b1, tab, ok1);
  d2 = log_ratio_fast(a2, b2, tab, ok2);
  if (!(ok1 && ok2)) {
    if (!ok1) d1 = log_ratio_ieee(a1, b1);
    if (!ok2) d2 = log_ratio_ieee(a2, b2);
  }
}

__host__ __device__ __forceinline__ Segment segment(const Endpoint& T, const Endpoint& R_, double A,
                                           double A2, const RayL& RL, bool air,
                                           const double* tab = &kLogTable[0][0]) {
  const double speedc = 299792458.0;
  const Endpoint R = pick(R_.x == T.x, T, R_);
  // Both ends lie in one layer (same C) at x >= 0 -- true of every segment the table and
  // minimizer paths form (layer bounds come from the same scans; heights and depths are
  // validated >= 0 at the API).  Identity (5): each antiderivative difference needs
  // log(a_R/a_T) instead of two logarithms, and
  // ftimeD = (s + A^2 (Cx - lg1)/sqrt(A^2-L^2) + A lg2) / (c C) since (n^2-L^2)/s = s.
  Segment s;
  const double syR = fast_sqrt(R.y2 - RL.LL), syT = fast_sqrt(T.y2 - RL.LL);
  double d1, d2;
  log_ratio2(R.Ay - RL.LL + RL.sAL * syR, T.Ay - RL.LL + RL.sAL * syT, R.n + syR, T.n + syT, tab,
             d1, d2);
  const double dCx = R.Cx - T.Cx;
  s.thd = (RL.L * R.invC) * RL.rsAL * (dCx - d1);
  s.t = ((syR - syT) + A2 * RL.rsAL * (dCx - d1) + A * d2) * (R.invC * (1.0 / speedc));
  s.geo = (d2 - (A * d1) * RL.rsAL + (R.ACx - T.ACx) * RL.rsAL) * R.invC;
  if (air) {
    s.thd *= -1;
    s.t *= -1;
    s.geo *= -1;
  }
  return s;
}

// Segment with both ends folded on the host (SegConst), identity (5).  sin_in is the sine of
// the incidence inside the start end (sin(lang)); returns the sine of the receive angle.
__host__ __device__ __forceinline__ Segment segment_const(const SegConst& S, double A, double A2, double sin_in,
                                                 bool air, double& v_out,
                                                 const double* tab = &kLogTable[0][0]) {
  const double v2 = sin_asin(S.ratio * sin_in);
  const RayL RL = ray_L(A2, S.Rn * v2);
  const double syR = fast_sqrt(S.Ry2 - RL.LL), syT = fast_sqrt(S.Ty2 - RL.LL);
  double d1, d2;
  log_ratio2(S.RAy - RL.LL + RL.sAL * syR, S.TAy - RL.LL + RL.sAL * syT, S.Rn + syR, S.Tn + syT,
             tab, d1, d2);
  Segment s;
  s.thd = (RL.L * S.invC) * RL.rsAL * (S.dCx - d1);
  s.t = ((syR - syT) + A2 * RL.rsAL * (S.dCx - d1) + A * d2) * S.invCc;
  s.geo = (d2 - (A * d1) * RL.rsAL + S.dACx * RL.rsAL) * S.invC;
  if (air) {
    s.thd *= -1;
    s.t *= -1;
    s.geo *= -1;
  }
  v_out = v2;
  return s;
}

// Layer-skip scans (.cc:1798-1825): top = MaxLayers-SkipLayersAbove-1, bottom = SkipLayersBelow.
__host__ __device__ __forceinline__ int top_layer(const DevMedium& M, double txh) {
  int skip = 0;
  for (int il = M.ml; il > -1; il--) {
    const bool hit = (txh < sel5(M.atm, il)) && (il >= 1 ? (txh >= sel5(M.atm, il - 1)) : false);
    if (hit) break;
    skip++;
  }
  return M.ml - skip - 1;
}

__host__ __device__ __forceinline__ int bottom_layer(const DevMedium& M, double ice_h) {
  int skip = 0;
  for (int il = 0; il < M.ml; il++) {
    if (ice_h >= sel5(M.atm, il) && ice_h < sel5(M.atm, il + 1)) break;
    skip++;
  }
  return skip;
}

// Fresnel amplitude transmission (.cc:285-337), thetai in radians.
__host__ __device__ __forceinline__ void fresnel_trans(double n1, double n2, double thetai, double& tS,
                                              double& tP) {
  const double st = sin(thetai), ct = cos(thetai);
  const double a = (n1 / n2) * st;
  const double sqterm = sqrt(1 - a * a);
  double num = n1 * ct - n2 * sqterm;
  double den = n1 * ct + n2 * sqterm;
  tS = 1 + (num / den);
  if (isnan(tS)) tS = 0;
  num = n1 * sqterm - n2 * ct;
  den = n1 * sqterm + n2 * ct;
  tP = (1 - (num / den)) * (n1 / n2);
  if (isnan(tP)) tP = 0;
}

// Completion signal of a one-query launch (ScalarCall::arm, airice_runtime.cpp): the thread that
// wrote the call's last output makes its stores visible to the host, then stores seq into the
// pinned, device-mapped flag the calling host thread spins on.  flag == nullptr: no signal.
// n_in > 0: the query's inputs (the values the call also wrote to the slot) travel here, in the
// kernel arguments, so the kernel does not read them back from host memory over PCIe.
struct Signal {
  unsigned* flag;
  unsigned seq;
  int n_in;
  double in[4];
};
// One-wave launches (the scalar entry points): the kernel arguments -- KBs of host-folded medium
// constants -- are read with scalar loads where they are used (the build keeps loop-invariant
// loads in place, -disable-machine-licm), and in a kernel that runs once each first touch of a
// 64-byte line is a miss to device memory inside a chain of dependent work.  Touching every line
// of the first BYTES of the argument block at entry makes those misses one round of independent
// loads; the later reads hit the scalar cache.  (Values unchanged: the same loads, earlier.)
template <unsigned BYTES>
__device__ __forceinline__ void prefetch_kernargs() {
  typedef const __attribute__((address_space(4))) unsigned KU;
  KU* ka = (KU*)__builtin_amdgcn_kernarg_segment_ptr();
  unsigned acc = 0;
#pragma unroll
  for (unsigned i = 0; i < BYTES / 64; ++i) acc += ka[i * 16];
  __asm__ volatile("" ::"s"(acc));
}

__device__ __forceinline__ void signal_done(const Signal& s) {
  if (s.flag == nullptr) return;
  __threadfence_system();
  *static_cast<volatile unsigned*>(s.flag) = s.seq;
}

}  // namespace airice
