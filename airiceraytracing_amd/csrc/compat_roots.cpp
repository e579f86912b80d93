// compat_roots.cpp -- FindFunctionRoot of the three reference namespaces
// (MultiRayAirIceRefraction.cc:340-374, max_iter 40; RayTracingFunctions.cc:256-290, max_iter 20;
// pythonwrapper/AirIceRayTracing.cc:315-353, max_iter = iterations) on the caller's host function.
//
// The reference drives GNU GSL's gsl_root_fsolver (alloc, error handler off, set, then
// {iterate; root; x_lower; x_upper; gsl_root_test_interval(lo, hi, 0, tolerance)} while
// GSL_CONTINUE and iter < max_iter, returning the last root).  GSL is not part of this build
// (airice_gsl_roots.h), so the two solvers the reference uses are restated here from GSL 2.x:
// roots/bisection.c (the Air2Ice minimizer, .cc:1521) and roots/brent.c (the RTF CLIs,
// Air2IceRayTracing.C:137), with roots/fsolver.c's set and roots/convergence.c's interval test.
// The search calls a host function pointer, so it runs on the host; the GPU kernels carry their
// own device forms of the same two machines (airice_kernels.hip, airice_rtf.hip).
//
// Undefined reference behaviour is modelled as the device and the test oracle model it: when
// f(x_lo) or f(x_hi) is not finite, GSL's set returns before storing its state and iterate then
// reads uninitialised malloc memory -- here that state is zero; x_lo > x_hi makes set fail before
// anything is stored -- here the root is 0 and the loop runs on the zero state.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "AirIceRayTracing.h"
#include "MultiRayAirIceRefraction.h"
#include "RayTracingFunctions.h"
#include "airice_gsl_roots.h"

#ifndef AIRICE_HAVE_GSL
// this library's solver types: only the name is read (set/iterate are GSL's own, not provided)
static const gsl_root_fsolver_type kBisection = {"bisection", 0, nullptr, nullptr};
static const gsl_root_fsolver_type kBrent = {"brent", 0, nullptr, nullptr};
extern "C" const gsl_root_fsolver_type* const airice_root_fsolver_bisection = &kBisection;
extern "C" const gsl_root_fsolver_type* const airice_root_fsolver_brent = &kBrent;
#endif

namespace {

constexpr double kDblEpsilon = 2.2204460492503131e-16;  // GSL_DBL_EPSILON

enum { GSL_OK = 0, GSL_CONT = -2, GSL_BADFUNC = 9, GSL_INVAL = 4, GSL_BADTOL = 13 };

struct Fn {
  gsl_function F;
  double operator()(double x) const { return F.function(x, F.params); }
};

// gsl_root_test_interval(x_lower, x_upper, 0, epsrel) (roots/convergence.c)
int test_interval(double lo, double hi, double epsrel) {
  if (epsrel < 0.0) return GSL_BADTOL;
  if (lo > hi) return GSL_INVAL;
  const double min_abs = ((lo > 0.0 && hi > 0.0) || (lo < 0.0 && hi < 0.0))
                             ? std::fmin(std::fabs(lo), std::fabs(hi))
                             : 0.0;
  return std::fabs(hi - lo) < 0.0 + epsrel * min_abs ? GSL_OK : GSL_CONT;
}

// fsolver record: the three values the driver reads back after each iterate
struct Solver {
  double root = 0, x_lower = 0, x_upper = 0;
};

// roots/bisection.c
double bisection(const Fn& f, double x_lo, double x_hi, double tolerance, int max_iter) {
  Solver s;
  double f_lower = 0, f_upper = 0;  // state (zero when set leaves it unwritten)
  if (!(x_lo > x_hi)) {            // gsl_root_fsolver_set
    s.root = 0.5 * (x_lo + x_hi);
    s.x_lower = x_lo;
    s.x_upper = x_hi;
    const double fl = f(x_lo);
    if (std::isfinite(fl)) {
      const double fu = f(x_hi);
      if (std::isfinite(fu)) {  // stored even when the ends do not straddle 0 (EINVAL ignored)
        f_lower = fl;
        f_upper = fu;
      }
    }
  }
  int iter = 0, status;
  do {
    iter++;
    // bisection_iterate
    const double xl = s.x_lower, xu = s.x_upper;
    if (f_lower == 0.0) {
      s.root = xl;
      s.x_upper = xl;
    } else if (f_upper == 0.0) {
      s.root = xu;
      s.x_lower = xu;
    } else {
      const double xb = (xl + xu) / 2.0;
      const double fb = f(xb);
      if (std::isfinite(fb)) {  // EBADFUNC: nothing stored
        if (fb == 0.0) {
          s.root = xb;
          s.x_lower = xb;
          s.x_upper = xb;
        } else if ((f_lower > 0.0 && fb < 0.0) || (f_lower < 0.0 && fb > 0.0)) {
          s.root = 0.5 * (xl + xb);
          s.x_upper = xb;
          f_upper = fb;
        } else {
          s.root = 0.5 * (xb + xu);
          s.x_lower = xb;
          f_lower = fb;
        }
      }
    }
    status = test_interval(s.x_lower, s.x_upper, tolerance);
  } while (status == GSL_CONT && iter < max_iter);
  return s.root;
}

// roots/brent.c
double brent(const Fn& f, double x_lo, double x_hi, double tolerance, int max_iter) {
  Solver s;
  double a = 0, b = 0, c = 0, d = 0, e = 0, fa = 0, fb = 0, fc = 0;  // state
  if (!(x_lo > x_hi)) {  // gsl_root_fsolver_set -> brent_init
    s.root = 0.5 * (x_lo + x_hi);
    s.x_lower = x_lo;
    s.x_upper = x_hi;
    const double fl = f(x_lo);
    if (std::isfinite(fl)) {
      const double fu = f(x_hi);
      if (std::isfinite(fu)) {
        a = x_lo, fa = fl;
        b = x_hi, fb = fu;
        c = x_hi, fc = fu;
        d = x_hi - x_lo;
        e = x_hi - x_lo;
      }
    }
  }
  int iter = 0, status;
  do {
    iter++;
    // brent_iterate on copies of the state; it is stored back only after a finite new point
    double la = a, lb = b, lc = c, ld = d, le = e, lfa = fa, lfb = fb, lfc = fc;
    bool ac_equal = false;
    if ((lfb < 0 && lfc < 0) || (lfb > 0 && lfc > 0)) {
      ac_equal = true;
      lc = la;
      lfc = lfa;
      ld = lb - la;
      le = lb - la;
    }
    if (std::fabs(lfc) < std::fabs(lfb)) {
      ac_equal = true;
      la = lb;
      lb = lc;
      lc = la;
      lfa = lfb;
      lfb = lfc;
      lfc = lfa;
    }
    const double tol = 0.5 * kDblEpsilon * std::fabs(lb);
    const double m = 0.5 * (lc - lb);
    if (lfb == 0) {
      s.root = lb;
      s.x_lower = lb;
      s.x_upper = lb;
    } else if (std::fabs(m) <= tol) {
      s.root = lb;
      if (lb < lc) {
        s.x_lower = lb;
        s.x_upper = lc;
      } else {
        s.x_lower = lc;
        s.x_upper = lb;
      }
    } else {
      if (std::fabs(le) < tol || std::fabs(lfa) <= std::fabs(lfb)) {
        ld = m;  // bisection step
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
        const double t1 = 3 * m * q - std::fabs(tol * q), t2 = std::fabs(le * q);
        if (2 * p < (t1 < t2 ? t1 : t2)) {
          le = ld;
          ld = p / q;
        } else {
          ld = m;
          le = m;
        }
      }
      la = lb;
      lfa = lfb;
      if (std::fabs(ld) > tol)
        lb += ld;
      else
        lb += (m > 0 ? +tol : -tol);
      const double fnew = f(lb);
      if (std::isfinite(fnew)) {  // EBADFUNC: nothing stored
        lfb = fnew;
        a = la, b = lb, c = lc, d = ld, e = le, fa = lfa, fb = lfb, fc = lfc;
        s.root = lb;
        const double cc = ((lfb < 0 && lfc < 0) || (lfb > 0 && lfc > 0)) ? la : lc;
        if (lb < cc) {
          s.x_lower = lb;
          s.x_upper = cc;
        } else {
          s.x_lower = cc;
          s.x_upper = lb;
        }
      }
    }
    status = test_interval(s.x_lower, s.x_upper, tolerance);
  } while (status == GSL_CONT && iter < max_iter);
  return s.root;
}

double find_root(const char* who, gsl_function F, double x_lo, double x_hi,
                 const gsl_root_fsolver_type* T, double tolerance, int max_iter) {
  if (T == nullptr || T->name == nullptr || F.function == nullptr) {
    std::fprintf(stderr, "%s::FindFunctionRoot: null solver type or function\n", who);
    std::abort();  // gsl_root_fsolver_alloc / GSL_FN_EVAL would crash
  }
  const Fn f{F};
  if (std::strcmp(T->name, "bisection") == 0) return bisection(f, x_lo, x_hi, tolerance, max_iter);
  if (std::strcmp(T->name, "brent") == 0) return brent(f, x_lo, x_hi, tolerance, max_iter);
  std::fprintf(stderr, "%s::FindFunctionRoot: solver '%s' is not provided (bisection, brent)\n",
               who, T->name);
  std::abort();
}

}  // namespace

double MultiRayAirIceRefraction::FindFunctionRoot(gsl_function F, double x_lo, double x_hi,
                                                  const gsl_root_fsolver_type* T,
                                                  double tolerance) {
  return find_root("MultiRayAirIceRefraction", F, x_lo, x_hi, T, tolerance, 40);
}

double RayTracingFunctions::FindFunctionRoot(gsl_function F, double x_lo, double x_hi,
                                             const gsl_root_fsolver_type* T, double tolerance) {
  return find_root("RayTracingFunctions", F, x_lo, x_hi, T, tolerance, 20);
}

double AirIceRayTracing::FindFunctionRoot(gsl_function F, double x_lo, double x_hi,
                                          const gsl_root_fsolver_type* T, double tolerance,
                                          int iterations) {
  return find_root("AirIceRayTracing", F, x_lo, x_hi, T, tolerance, iterations);
}
