"""Premise check behind the guarded bisection's sign inference: on the
queries of tests/test_gpu_bisect_replay.py::test_replay_wide_ranges' second block (TxH 3000.5-3300 m,
D 0-5 m, antenna -5..500 m) -- where the deferred-f(lo) variant of round 1 mismatched -- sample
f(theta) = D - THD(theta) (the oracle's MinimizeforLaunchAngle, .cc:873-917) on 801 points of each
bracket [thR - 16, thR] and classify the queries.  CPU only.

    PYTHONPATH=. python tools/flo_premise.py [stride]
"""
import sys

import numpy as np

import oracle


def main():
    stride = int(sys.argv[1]) if len(sys.argv) > 1 else 100
    m = oracle.load_atmosphere("airiceraytracing_amd/data/Atmosphere.dat.gz")
    rng = np.random.default_rng(7)  # the replay test's generator, both blocks drawn in order
    n = 100000
    txh = np.concatenate([rng.uniform(3001, 100000, n // 2), rng.uniform(3000.5, 3300, n // 2)])
    dist = np.concatenate([rng.uniform(0, 300000, n // 2), rng.uniform(0, 5, n // 2)])
    depth = np.concatenate([-rng.uniform(0, 300, n // 2), rng.uniform(-5, 500, n // 2)])
    c = dict(queries=0, rx_above_tx=0, thR_above_180=0, no_air_layer_f_const=0,
             root_within_1e6_deg_of_hi=0, nonmonotone=0, nonfinite=0, f_lo_below_tau=0,
             f_hi_below_tau=0)
    for i in range(50000, 100000, stride):
        H, D, dep = txh[i], dist[i], depth[i]
        thR = oracle.straight_angle_of(m, H, D, 3000.0, dep)
        ice, dpos = (3000.0 + dep, 0.0) if dep >= 0 else (3000.0, -dep)
        lo, hi = max(thR - 16, 90.001), thR
        xs = np.linspace(lo, hi, 801)
        f = np.array([oracle.rtf_eval(m, 14, [x, H, ice, dpos, D])[0] for x in xs])
        tau = 1e-6 + 1e-10 * abs(D)
        fin = np.isfinite(f)
        d = np.diff(f[fin])
        c["queries"] += 1
        c["rx_above_tx"] += ice > H
        c["thR_above_180"] += thR > 180
        c["no_air_layer_f_const"] += bool(fin.all() and np.all(f == D))
        c["nonmonotone"] += not (np.all(d >= -1e-9) or np.all(d <= 1e-9))
        c["nonfinite"] += not fin.all()
        c["f_lo_below_tau"] += bool(fin[0] and abs(f[0]) < tau)
        c["f_hi_below_tau"] += bool(fin[-1] and abs(f[-1]) < tau)
        if fin.all() and np.sign(f[0]) != np.sign(f[-1]):
            # root position by bisection on the sampled neighbourhood of hi
            a, b = xs[-2], xs[-1]
            for _ in range(60):
                mid = 0.5 * (a + b)
                fm = oracle.rtf_eval(m, 14, [mid, H, ice, dpos, D])[0]
                if np.sign(fm) == np.sign(f[0]):
                    a = mid
                else:
                    b = mid
            c["root_within_1e6_deg_of_hi"] += (hi - a) < 1e-6
    print({k: int(v) for k, v in c.items()})


if __name__ == "__main__":
    main()
