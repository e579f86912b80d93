"""Coefficients of the device asin for t in [0, 1/2] (airice_device.hpp asin_small):
asin(t) = t + t^3 P(t^2), P of degree D fitted in mpmath (Chebyshev nodes on s = t^2 in
[0, 1/4], then a few Remez-style reweighting passes are unnecessary at this degree: the fit's
error is checked below and is far under 2^-53 relative to asin(t)).  Prints C hex floats.
    python tools/gen_asin_poly.py [D]"""
import sys

import mpmath as mp

mp.mp.prec = 200
D = int(sys.argv[1]) if len(sys.argv) > 1 else 11


def f(s):
    if s == 0:
        return mp.mpf(1) / 6
    t = mp.sqrt(s)
    return (mp.asin(t) - t) / (t ** 3)


def fit(D):
    a, b = mp.mpf(0), mp.mpf(1) / 4
    n = D + 1
    nodes = [(a + b) / 2 + (b - a) / 2 * mp.cos(mp.pi * (2 * k + 1) / (2 * n)) for k in range(n)]
    A = mp.matrix([[x ** j for j in range(n)] for x in nodes])
    y = mp.matrix([f(x) for x in nodes])
    return mp.lu_solve(A, y)


def check(c):
    import numpy as np
    cd = [float(x) for x in c]
    worst = 0.0
    for i in range(20001):
        t = 0.5 * i / 20000
        s = t * t
        p = cd[-1]
        for cj in reversed(cd[:-1]):
            p = float(np.fma(s, p, cj)) if hasattr(np, "fma") else s * p + cj
        t3 = t * s
        r = t + t3 * p
        ref = mp.asin(mp.mpf(t))
        if ref != 0:
            worst = max(worst, float(abs(mp.mpf(r) - ref) / ref))
    return worst


if __name__ == "__main__":
    c = fit(D)
    print(f"// degree {D} in t^2, max rel err (double Horner) {check(c):.3e}")
    for j, x in enumerate(c):
        print(f"  {float(x).hex()},  // c{j}")
