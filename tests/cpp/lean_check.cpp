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
  // the probe's steps (probe_steps) against the loop: lo from 90.001 (or anywhere), stop bound
  // T = hi - 0.1 with hi = thR over the whole angle range (binade 64-128 and 128-256 crossings),
  // with and without the Snell bound thr; plus odd steps and bounds (ties, non-finite)
  long pcases = 0, pbad = 0, psteps = 0;
  for (long c = 0; c < n / 4; ++c) {
    const double thR = (c % 7 == 0) ? 60.0 + 300.0 * U(rng) : 90.0 + 90.0 * U(rng);
    double lo = (c % 5 == 0) ? 90.0 * U(rng) + 30.0 : 90.001;
    const double T = thR - 0.1;
    const bool use_thr = c % 2 == 0;
    double thr = 90.0 + 90.0 * U(rng);
    double step = 0.05;
    if (c % 13 == 0) step = pow(2.0, -3 - (int)(U(rng) * 20)) * (1 + U(rng));
    if (c % 17 == 0) step = 0.05 * (1 + 1e-3 * U(rng));
    if (c % 101 == 0) thr = NAN;
    if (c % 103 == 0) lo = INFINITY;
    // the loop, step by step (capped: a non-finite bound may never stop it)
    double ref = lo;
    bool ref_stepped = false;
    long k = 0;
    while (((!use_thr || ref < thr) && !(ref > T)) && k < 100000) {
      ref = ref + step;
      ref_stepped = true;
      ++k;
    }
    if (k >= 100000) continue;
    bool st = false;
    const double got = probe_steps(lo, step, T, thr, use_thr, st);
    ++pcases;
    psteps += k;
    if (dbits(got) != dbits(ref) || st != ref_stepped) {
      if (++pbad <= 10)
        printf("PROBE MISMATCH lo=%.17g step=%.17g T=%.17g thr=%.17g use_thr=%d: ref %.17g (%d) "
               "got %.17g (%d)\n", lo, step, T, thr, (int)use_thr, ref, (int)ref_stepped, got,
               (int)st);
    }
  }
  printf("cases %ld closed %ld done %ld maxiter %ld mismatches %ld probe_cases %ld probe_steps %ld "
         "probe_mismatches %ld\n", n, closed, done, maxiter, bad, pcases, psteps, pbad);
  return bad == 0 && pbad == 0 ? 0 : 1;
}
