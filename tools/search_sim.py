"""CPU simulation of the minimizer's root search (solve_root, airice_kernels.hip) to count
f-evaluations per solve for alternative search / guard strategies (tools only; the GPU's own counts
come from tools/solve_stats.py).  f(theta) = D - THD(theta) is taken from the oracle's forward ray
(GetRayTracingSolutions), a close stand-in for MinimizeforLaunchAngle's f; unprobed cfg3 queries.

    python tools/search_sim.py [n]
"""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import oracle  # noqa: E402
from tests.parity import cfg3_queries  # noqa: E402

TOL = 1e-9
D2R, R2D = 3.1415927 / 180.0, 180.0 / 3.1415927


def f32(x):
    return float(np.float32(x))


def gsl_midpoint_evals(lo, hi, gl, gr, f, fL_sign, counter):
    """GSL bisection from [lo, hi]; midpoints in (gl, gr) are evaluated (counted), others take the
    guard region's sign.  Returns the final bracket."""
    it = 0
    f_lower_neg = fL_sign < 0
    while it < 40:
        xm = (lo + hi) / 2.0
        if xm <= gl:
            lo = xm
        elif xm >= gr:
            hi = xm
        else:
            counter[0] += 1
            v = f(xm)
            if v == 0.0:
                return xm, xm
            if (v < 0) != f_lower_neg:
                hi = xm
                if abs(v) >= counter[1]:
                    gr = xm
            else:
                lo = xm
                if abs(v) >= counter[1]:
                    gl = xm
        it += 1
        if abs(hi - lo) < TOL * lo:
            break
    return lo, hi


def solve(f, lo, hi, tau, strategy):
    n = 0

    def ev(x):
        nonlocal n
        n += 1
        return f(x)

    fL, fR = ev(lo), ev(hi)
    if not (math.isfinite(fL) and math.isfinite(fR)):
        return n, None, float("nan")
    if (fL < 0) == (fR < 0) or abs(fL) < tau or abs(fR) < tau:
        return n, None, float("nan")
    gL, gR = lo, hi
    ul, uh = f32(math.tan(f32((180 - lo) * D2R))), f32(math.tan(f32((180 - hi) * D2R)))
    un = f32(uh - f32(fR) * f32(f32(uh - ul) / f32(fR - fL)))
    x2 = 180 - math.atan(un) * R2D
    x0, f0, x1, f1 = lo, fL, hi, fR
    f2 = None
    est = 0
    W = 16.0 / 2 ** 27
    while True:
        if est > 0:
            x = x2 - f2 * (x2 - x1) / (f2 - f1)
            if est >= 1:
                d1 = (x2 - x1) / (f2 - f1)
                d0 = (x1 - x0) / (f1 - f0)
                x += f1 * f2 * ((d1 - d0) / (f2 - f0))
            if not (gL < x < gR):
                x = 0.5 * (gL + gR)
            if strategy == "merge" and abs(x - x2) < W / 16 and abs(f2) >= tau:
                # x2 is a guard on its side (already recorded); one guard on the other side
                slope = abs((x2 - x1) / (f2 - f1))
                dl = 4 * tau * slope
                xo = x + (dl if (f2 < 0) == (fL < 0) else -dl)
                v = ev(xo)
                if math.isfinite(v) and abs(v) >= tau and gL < xo < gR:
                    if (v < 0) == (fL < 0):
                        gL = xo
                    else:
                        gR = xo
                break
        else:
            x = x2
        if est > 0:
            x0, f0, x1, f1 = x1, f1, x2, f2
        x2 = x
        f2 = ev(x)
        est += 1
        if not math.isfinite(f2):
            break
        if abs(f2) < tau:
            dlt = 4.0 * tau * abs((x2 - x1) / (f2 - f1))
            if strategy == "model" and 0 < dlt < gR - gL and est >= 2:
                # solve_root since round 4: guards placed by the secant slope, not evaluated
                # (f(x2 -+ dlt) ~ f2 -+ 4 tau sign(slope))
                left_neg = ((f2 - f1) / (x2 - x1)) > 0
                for xg, neg in ((x2 - dlt, left_neg), (x2 + dlt, not left_neg)):
                    if gL < xg < gR:
                        if neg == (fL < 0):
                            gL = xg
                        else:
                            gR = xg
                break
            if 0 < dlt < gR - gL:
                for xg in (x2 - dlt, x2 + dlt):
                    v = ev(xg)
                    if math.isfinite(v) and abs(v) >= tau and gL < xg < gR:
                        if (v < 0) == (fL < 0):
                            gL = xg
                        else:
                            gR = xg
            break
        if gL < x2 < gR:
            if (f2 < 0) == (fL < 0):
                gL = x2
            else:
                gR = x2
        if est >= 12:
            break
    cnt = [0, tau]
    blo, bhi = gsl_midpoint_evals(lo, hi, gL, gR, f, fL, cnt)
    return n + cnt[0], est, 0.5 * (blo + bhi)


def model_guess(m, H, D, ice, depth, iters=3):
    """Launch angle (deg) from a two-medium model without evaluating f: straight in air at n(Tx),
    straight in the ice at n(|depth| / 2), Snell at the surface; Newton on the launch angle."""
    h = H - ice
    d = abs(depth)
    n_tx = oracle.getnz_air(m, H)
    n_e = oracle.getnz_ice(m, -d / 2) if d > 0 else oracle.getnz_ice(m, 0.0)
    a = math.atan2(D, h + d)
    for _ in range(iters):
        L = n_tx * math.sin(a)
        if L >= n_e:
            break
        q = math.sqrt(n_e * n_e - L * L)
        g = h * math.tan(a) + d * L / q - D
        gp = h / math.cos(a) ** 2 + d * n_tx * math.cos(a) * n_e * n_e / q ** 3
        a = a - g / gp
    return 180 - a * R2D


def straddle_trips(m, H, D, d, f, lo, hi, tau, b):
    """Trips (the paired first evaluation counted 1.3) of a search that evaluates f at the model
    guess -+ b instead of at the bracket ends, takes the ends' signs from monotonicity when the
    pair straddles the root, then steps by secant / IQI; None when the pair does not straddle."""
    xm = model_guess(m, H, D, 3000.0, d)
    xa, xb = max(lo, xm - b), min(hi, xm + b)
    fa, fb = f(xa), f(xb)
    if not (math.isfinite(fa) and math.isfinite(fb) and (fa < 0) != (fb < 0) and
            abs(fa) >= tau and abs(fb) >= tau):
        return None
    pts = [(xa, fa), (xb, fb)]
    steps = 0
    while steps < 12:
        (xB, fB), (xC, fC) = pts[-2:]
        x2 = xC - fC * (xC - xB) / (fC - fB)
        if len(pts) >= 3:
            xA, fA = pts[-3]
            d1 = (xC - xB) / (fC - fB)
            d0 = (xB - xA) / (fB - fA)
            x2 += fB * fC * ((d1 - d0) / (fC - fA))
        f2 = f(x2)
        steps += 1
        pts.append((x2, f2))
        if not math.isfinite(f2) or abs(f2) < tau:
            break
    return 1.3 + steps


def paired_first_trips(f, lo, hi, tau, pair_h=None):
    """Trips (a paired evaluation counted 1.3) of the kept search from the paired bracket ends to
    |f| < tau, with the first search point evaluated alone (pair_h None, the kernel) or together
    with a second point pair_h degrees above it (both in one paired evaluation), the search then
    stepping by IQI through the last three points; None when the ends do not bracket a root."""
    fL, fR = f(lo), f(hi)
    if not (math.isfinite(fL) and math.isfinite(fR)) or (fL < 0) == (fR < 0) or \
            abs(fL) < tau or abs(fR) < tau:
        return None
    trips = 1.3
    ul, uh = f32(math.tan(f32((180 - lo) * D2R))), f32(math.tan(f32((180 - hi) * D2R)))
    un = f32(uh - f32(fR) * f32(f32(uh - ul) / f32(fR - fL)))
    x2 = 180 - math.atan(un) * R2D
    pts = [(lo, fL), (hi, fR)]
    if pair_h is None:
        fa = f(x2)
        trips += 1
        pts.append((x2, fa))
        if abs(fa) < tau:
            return trips
    else:
        fa, fb = f(x2), f(x2 + pair_h)
        trips += 1.3
        pts += [(x2, fa), (x2 + pair_h, fb)]
        if abs(fa) < tau or abs(fb) < tau:
            return trips
    for _ in range(12):
        (xA, fA), (xB, fB), (xC, fC) = pts[-3:]
        x = xC - fC * (xC - xB) / (fC - fB)
        d1 = (xC - xB) / (fC - fB)
        d0 = (xB - xA) / (fB - fA)
        x += fB * fC * ((d1 - d0) / (fC - fA))
        v = f(x)
        trips += 1
        pts.append((x, v))
        if not math.isfinite(v) or abs(v) < tau:
            break
    return trips


def main_pair(n):
    m = oracle.load_atmosphere(os.path.join(ROOT, "airiceraytracing_amd", "data",
                                            "Atmosphere.dat.gz"))
    txh, dst, dep = cfg3_queries(4 * n, seed=2024)
    hs = (None, 1e-5, 1e-4, 1e-3, 1e-2)
    res = {h: [] for h in hs}
    k = 0
    for i in range(len(txh)):
        H, D, d = txh[i], dst[i], dep[i]
        thR = oracle.straight_angle_of(m, H, D, 3000.0, d)
        lo, hi = thR - 16, thR
        if lo < 90.001:
            continue

        def f(t):
            return D - oracle.ray_solution(m, t, H, 3000.0, d)[2]

        tau = 1e-6 + 1e-10 * abs(D)
        out = {h: paired_first_trips(f, lo, hi, tau, h) for h in hs}
        if any(v is None for v in out.values()):
            continue
        for h, v in out.items():
            res[h].append(v)
        k += 1
        if k >= n:
            break
    for h, v in res.items():
        print(f"first point {'alone' if h is None else f'paired, +{h} deg'}: {np.mean(v):.3f} "
              f"trips per solve (p90 {np.percentile(v, 90):.2f}, max {max(v):.1f})")


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--pair":
        main_pair(int(sys.argv[2]) if len(sys.argv) > 2 else 300)
        return
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 300
    m = oracle.load_atmosphere(os.path.join(ROOT, "airiceraytracing_amd", "data",
                                            "Atmosphere.dat.gz"))
    txh, dst, dep = cfg3_queries(4 * n, seed=2024)
    res = {"base": [], "merge": [], "model": []}
    roots = {k: [] for k in res}
    exact = []
    ests = []
    used = 0
    for i in range(len(txh)):
        H, D, d = txh[i], dst[i], dep[i]
        thR = oracle.straight_angle_of(m, H, D, 3000.0, d)
        lo, hi = thR - 16, thR
        if lo < 90.001:
            continue

        def f(t):
            return D - oracle.ray_solution(m, t, H, 3000.0, d)[2]

        tau = 1e-6 + 1e-10 * abs(D)
        for s in res:
            k, e, r = solve(f, lo, hi, tau, s)
            res[s].append(k)
            roots[s].append(r)
            if s == "base" and e is not None:
                ests.append(e)
        # GSL's bisection evaluating every midpoint (the reference's root)
        c = [0, float("inf")]
        elo, ehi = gsl_midpoint_evals(lo, hi, -1e300, 1e300, f, f(lo), c)
        exact.append(0.5 * (elo + ehi))
        used += 1
        if used >= n:
            break
    ex = np.array(exact)
    for s, v in res.items():
        rr = np.array(roots[s], dtype=float)
        ok = np.isfinite(rr)
        same = int(np.sum(rr[ok] == ex[ok]))
        print(f"{s}: {np.mean(v):.3f} evaluations per solve over {len(v)} queries; root equal to "
              f"the every-midpoint bisection on {same}/{int(ok.sum())}")
    print(f"search steps (base) {np.mean(ests):.3f}")
    # the straddling model pair: trips per solve against the kept search's
    # (paired ends 1.3 + its search steps), a pair that does not straddle re-running the kept search
    txh, dst, dep = cfg3_queries(4 * n, seed=2024)
    for b in (0.003, 0.006, 0.012, 0.025):
        base, new, miss, k = [], [], 0, 0
        for i in range(len(txh)):
            H, D, d = txh[i], dst[i], dep[i]
            thR = oracle.straight_angle_of(m, H, D, 3000.0, d)
            lo, hi = thR - 16, thR
            if lo < 90.001:
                continue

            def f(t):
                return D - oracle.ray_solution(m, t, H, 3000.0, d)[2]

            tau = 1e-6 + 1e-10 * abs(D)
            _, e, _ = solve(f, lo, hi, tau, "model")
            if e is None:
                continue
            t = straddle_trips(m, H, D, d, f, lo, hi, tau, b)
            miss += t is None
            base.append(1.3 + e)
            new.append(t if t is not None else 2.6 + e)
            k += 1
            if k >= n:
                break
        print(f"straddle b={b} deg: {np.mean(new):.3f} trips per solve against {np.mean(base):.3f} "
              f"(pair not straddling: {miss / k:.3f})")


if __name__ == "__main__":
    main()
