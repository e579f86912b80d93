// Fuzz check of the guarded bisection's closed-form lean run (airice_lean.hpp, lean_closed)
// against its step-by-step form (lean_steps) on brackets built the way solve_root builds them:
// [thR - 16, thR], or a probe-moved lo (90.001 + 0.05 k), then some evaluated bisection steps,
// with guard bounds around a random root.  Prints the cases, how many took the closed form, and
// the mismatches (must be 0).  tests/test_lean.py runs it.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>

#include "airice_lean.hpp"

using namespace airice;

int main(int argc, char** argv) {
  const long n = argc > 1 ? atol(argv[1]) : 1000000;
  std::mt19937_64 rng(20261017);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  const double tol = 0.000000001;
  long closed = 0, bad = 0, done = 0, maxiter = 0;
  for (long c = 0; c < n; ++c) {
    const double thR = 90.0 + 90.0 * U(rng);
    double lo = thR - 16, hi = thR;
    if (lo < 90.001 || c % 11 == 0) {  // the probe moved lo
      lo = 90.001;
      const int k = (int)(U(rng) * 300);
      for (int i = 0; i < k && !(lo > hi - 0.1); ++i) lo = lo + 0.05;
      if (lo >= hi) continue;
    }
    if (hi < 90.001 && hi > 90.00) hi = 90.05;
    int iter = 0;
    const double root = lo + (hi - lo) * U(rng);
    // evaluated bisection steps before this run (the root's side decides)
    const int pre = (int)(U(rng) * (c % 3 == 0 ? 30 : 6));
    for (int i = 0; i < pre && iter < 39; ++i) {
      const double xm = (lo + hi) / 2.0;
      if (xm < root)
        lo = xm;
      else
        hi = xm;
      ++iter;
    }
    if (!(lo > 0.0) || !(fabs(hi - lo) >= tol * lo)) continue;  // the driver would have stopped
    // guards around the root: widths from 1e-13 to ~10 degrees, sometimes past the bracket
    const double dl = pow(10.0, -16 + 17 * U(rng)), dr = pow(10.0, -16 + 17 * U(rng));
    double gl = root - dl, gr = root + dr;
    const int mode = (int)(U(rng) * 10);
    bool okL = mode != 1, okR = mode != 2;
    if (mode == 3) gl = hi;           // no sign change: every midpoint has the ends' sign
    if (mode == 4) gl = lo - 1e-3;    // lo moved past the left guard
    if (mode == 5) gr = hi + 1e-3;
    if (gl < lo && mode != 4) gl = lo;
    if (gr > hi && mode != 5) gr = hi;
    if (!(gl < gr) && mode != 3) continue;
    if (mode == 3) { okR = false; }
    const LeanRun ref = lean_steps(lo, hi, iter, okL ? gl : -1.0, okR ? gr : INFINITY, tol);
    LeanRun got;
    if (!lean_closed(lo, hi, iter, gl, gr, okL, okR, tol, got)) continue;
    ++closed;
    done += ref.done;
    maxiter += ref.maxiter;
    const bool same = dbits(got.lo) == dbits(ref.lo) && dbits(got.hi) == dbits(ref.hi) &&
                      got.steps == ref.steps && got.done == ref.done &&
                      got.maxiter == ref.maxiter;
    if (!same) {
      if (++bad <= 10)
        printf("MISMATCH lo=%.17g hi=%.17g iter=%d gl=%.17g gr=%.17g okL=%d okR=%d: ref "
               "(%.17g %.17g %d %d %d) got (%.17g %.17g %d %d %d)\n",
               lo, hi, iter, gl, gr, okL, okR, ref.lo, ref.hi, ref.steps, ref.done, ref.maxiter,
               got.lo, got.hi, got.steps, got.done, got.maxiter);
    }
  }
  printf("cases %ld closed %ld done %ld maxiter %ld mismatches %ld\n", n, closed, done, maxiter,
         bad);
  return bad == 0 ? 0 : 1;
}
