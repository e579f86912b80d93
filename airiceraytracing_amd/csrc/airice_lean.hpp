// airice_lean.hpp -- the guarded bisection's evaluation-free steps in closed form (device, and
// compiled by g++ for tests/cpp/lean_check.cpp, which checks it against the step-by-step form).
//
// solve_root (airice_kernels.hip) replays GSL's bisection (gsl_root_fsolver_bisection +
// gsl_root_test_interval(lo, hi, 0, 1e-9) + max_iter 40, MultiRayAirIceRefraction.cc:340-374).
// Between two evaluations it runs the steps whose midpoint lies in a guard region -- xm <= gl
// (f has f(lo)'s sign there: lo moves) or xm >= gr (hi moves) -- until a midpoint falls strictly
// between the guards (it must be evaluated) or the driver stops (interval test, max_iter).  Run
// step by step that is ~25 compare-and-select steps per solve, a fifth of the root finder's VALU
// issue (tools/solve_blocks.py).
//
// When every midpoint the run can form is exact -- the bracket width w = hi - lo a power of two,
// the finest spacing w 2^-R (R = 40 - iter steps left) no finer than hi's ulp, lo on hi's ulp grid:
// true of every bracket that starts as [thR - 16, thR], i.e. every query the probe loop did not
// move -- the midpoints are the dyadic points lo + M w 2^-R, M an integer, and the run is a
// descent in a binary trie: with a = floor((gl - lo) 2^R / w) and b = ceil((gr - lo) 2^R / w) - 1
// (clipped to [0, 2^R - 1]) it goes right while a's next bit is 1, left while b's is 0, and stops
// at the first bit where a has 0 and b has 1: after k = clz(a ^ b) - (64 - R) steps, with lo at
// a's k-bit prefix.  The interval test w 2^-j < tol lo_j first holds at j0 or j0 + 1 (j0 from
// tol hi, j0 + 1 from tol lo: hi < 2 lo), decided by one test at lo_j0.  Everything is exact, so
// the result is the step-by-step form's bit for bit; brackets that fail the exactness test (the
// probed ones) take the step-by-step form.
#pragma once

#include <cstdint>

#include "airice_tlog.hpp"

namespace airice {

struct LeanRun {
  double lo, hi;
  int steps;     // bisection steps taken (the driver's iteration count grows by this)
  bool done;     // the interval test or max_iter ended the run
  bool maxiter;  // ... at max_iter with the interval test still failing
};

__host__ __device__ AIRICE_INLINE int lean_exp(double x) {
  return (int)((dbits(x) >> 52) & 0x7ff) - 1023;
}
__host__ __device__ AIRICE_INLINE bool lean_pow2(double x) {
  return (dbits(x) & 0x000fffffffffffffULL) == 0;
}
// x * 2^n for |n| < 1000 and normal x, x * 2^n normal (exact)
__host__ __device__ AIRICE_INLINE double lean_scale(double x, int n) {
  return x * bitsd((uint64_t)(1023 + n) << 52);
}
// smallest j >= 1 with 2^(e - j) < t (t positive, normal)
__host__ __device__ AIRICE_INLINE int lean_first_below(int e, double t) {
  const int j = e - lean_exp(t) + (lean_pow2(t) ? 1 : 0);
  return j < 1 ? 1 : j;
}
// a's top j bits of R, as an integer times the finest spacing
__host__ __device__ AIRICE_INLINE uint64_t lean_prefix(uint64_t a, int R, int j) {
  return (a >> (R - j)) << (R - j);
}
// an integer-valued double in [0, 2^52) as an integer
__host__ __device__ AIRICE_INLINE uint64_t lean_u64(double v) {
  return dbits(v + 0x1p52) & 0x000fffffffffffffULL;
}
__host__ __device__ AIRICE_INLINE double lean_f64(uint64_t v) {
  return bitsd(v | 0x4330000000000000ULL) - 0x1p52;
}
__host__ __device__ AIRICE_INLINE int lean_clz64(uint64_t d) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __clzll((long long)d);
#else
  return __builtin_clzll(d);
#endif
}

// The step-by-step form (solve_root's semantics, one step at a time).  iter < 40.
__host__ __device__ AIRICE_INLINE LeanRun lean_steps(double lo, double hi, int iter, double gl,
                                                     double gr, double tol) {
  LeanRun o{lo, hi, 0, false, false};
  for (;;) {
    const double xm = (o.lo + o.hi) / 2.0;
    const bool inL = xm <= gl, inR = !inL && xm >= gr;
    if (!(inL || inR)) break;
    if (inL)
      o.lo = xm;
    else
      o.hi = xm;
    ++o.steps;
    const bool cont = !(((o.hi - o.lo) < 0 ? -(o.hi - o.lo) : (o.hi - o.lo)) < 0 + tol * o.lo);
    if (!cont || iter + o.steps == 40) {
      o.done = true;
      o.maxiter = cont;
      break;
    }
  }
  return o;
}

// The closed form.  gl / gr: the guard bounds (okL / okR false: no guard on that side).  Returns
// false, leaving o unset, when the bracket fails the exactness conditions above.
__host__ __device__ AIRICE_INLINE bool lean_closed(double lo, double hi, int iter, double gl,
                                                   double gr, bool okL, bool okR, double tol,
                                                   LeanRun& o) {
  const double w = hi - lo;
  const int R = 40 - iter;
  const int e = lean_exp(w), Ehi = lean_exp(hi), Elo = lean_exp(lo);
  const int shift = Ehi - Elo;
  const bool exact = w > 0.0 && lean_pow2(w) && R >= 1 && R <= 40 && e - R >= Ehi - 52 &&
                     shift >= 0 && shift < 52 &&
                     (dbits(lo) & ((1ULL << shift) - 1)) == 0 && lo > 0.0 && hi < 0x1p1000 &&
                     // gl - lo and gr - lo exact (Sterbenz)
                     (!okL || (gl >= 0.5 * lo && gl <= 2.0 * lo)) &&
                     (!okR || (gr >= 0.5 * lo && gr <= 2.0 * lo));
  if (!exact) return false;
  const double top = lean_scale(1.0, R) - 1.0;  // 2^R - 1
  double fa = okL ? floor(lean_scale(gl - lo, R - e)) : 0.0;
  double fb = okR ? ceil(lean_scale(gr - lo, R - e)) - 1.0 : top;
  fa = fa < 0.0 ? 0.0 : (fa > top ? top : fa);
  fb = fb < 0.0 ? 0.0 : (fb > top ? top : fb);
  const uint64_t a = lean_u64(fa), b = lean_u64(fb);
  const uint64_t d = a ^ b;
  const int k = d == 0 ? R : R - 64 + lean_clz64(d);  // steps before a midpoint needs f
  // first step whose interval passes the test: j0 or j1 = j0 + 1
  const int j0 = lean_first_below(e, tol * hi), j1 = lean_first_below(e, tol * lo);
  if (j1 - j0 > 1) return false;
  int js = j1;
  if (j0 < j1) {
    const double loj = lo + lean_scale(lean_f64(lean_prefix(a, R, j0 < R ? j0 : R)), e - R);
    if (lean_scale(1.0, e - j0) < 0 + tol * loj) js = j0;
  }
  const int s = js < R ? js : R;
  const int n = s <= k ? s : k;
  o.lo = lo + lean_scale(lean_f64(lean_prefix(a, R, n)), e - R);
  o.hi = o.lo + lean_scale(w, -n);
  o.steps = n;
  o.done = s <= k;
  o.maxiter = s <= k && js > R;
  return true;
}

// The probe's evaluation-free steps (solve_root; Air2IceRayTracing's probe loop,
// MultiRayAirIceRefraction.cc:1496-1509, where the loop's outcome needs no evaluation):
//   while ((!use_thr || lo < thr) && !(lo > T)) lo = lo + c;
// `stepped`: a step was taken.  Inside a binade [2^e, 2^(e+1)) every lo on that binade's grid
// (spacing u = 2^(e-52)) has lo + c rounded by the same amount, unless c's remainder modulo u is
// exactly u/2 (a tie, which depends on lo's last bit): there the steps are the exact arithmetic
// sequence x1 + m d (d = fl(x1 + c) - x1; m d exact while d < 2^(e-10) and m < 2^11), and the
// stopping step comes from one division, confirmed on exact values (the loop condition is monotone
// in lo for finite bounds).  A step that leaves the binade, a tie, or non-finite bounds go one step
// at a time.  The no-air-layer probe of the lookup's x100 fallback runs up to ~900 such steps.
__host__ __device__ AIRICE_INLINE double probe_steps(double lo, double c, double T, double thr,
                                                     bool use_thr, bool& stepped) {
  auto cont = [&](double x) { return (!use_thr || x < thr) && !(x > T); };
  stepped = false;
  const bool finite = __builtin_isfinite(T) && (!use_thr || __builtin_isfinite(thr)) && c > 0.0;
  while (cont(lo)) {
    lo = lo + c;
    stepped = true;
    if (!finite || !cont(lo)) continue;
    const double x2 = lo + c;
    const double d = x2 - lo;  // exact (x2 and lo within a factor 2)
    const int e = lean_exp(lo);
    if (lean_exp(x2) != e || !(lo > 0.0)) continue;
    const double u = lean_scale(1.0, e - 52);
    const double r = c - d;
    if ((r < 0 ? -r : r) == 0.5 * u || !(d < lean_scale(1.0, e - 10)) || !(d > 0.0)) continue;
    // steps m = 1 .. mmax stay inside the binade (x1 + m d < 2^(e+1)), m < 2^11
    const double top = lean_scale(1.0, e + 1);
    double mmax = floor((top - lo) / d);
    if (mmax > 2047.0) mmax = 2047.0;
    while (mmax >= 1.0 && !(lo + mmax * d < top)) mmax -= 1.0;
    if (mmax < 1.0) continue;
    // first m with !cont(x1 + m d): from the bounds, then confirmed
    double m = mmax;
    const double mT = floor((T - lo) / d) + 1.0;
    if (mT < m) m = mT;
    if (use_thr) {
      const double mthr = ceil((thr - lo) / d);
      if (mthr < m) m = mthr;
    }
    if (m < 1.0) m = 1.0;
    while (m > 1.0 && !cont(lo + (m - 1.0) * d)) m -= 1.0;
    while (m < mmax && cont(lo + m * d)) m += 1.0;
    lo = lo + m * d;
  }
  return lo;
}

}  // namespace airice
