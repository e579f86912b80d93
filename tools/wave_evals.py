"""Evaluation counts of the grouped root finder in the order its waves run them (debug, GPU box).

Needs a library built with -DAIRICE_SORTED_STATS=1 (AB_LIB=<that .so>) and AIRICE_GROUP_MIN=1 (the
batch-wide grouping, since round 4 the default of the trace source only): the per-query counts are
then recorded by sorted position, so 64 consecutive entries are one wave of roots_sorted_kernel.
Prints the mean evaluations per query, the mean of the per-wave maxima (a wave runs until its last
lane is done) and what a trip cap with a continuation pass would leave for each cap.

    AB_LIB=/tmp/stats.so python tools/wave_evals.py [n]
"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
    path = "/tmp/wave_evals.bin"
    if os.path.exists(path):
        os.remove(path)
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "solve_stats.py"), "--child",
                    "sorted", str(n), path], check=True, timeout=300)
    a = np.fromfile(path, dtype=np.int32).reshape(-1, 3)
    ev = a[:, 0]
    live = ev > 0
    ev = ev[: int(np.nonzero(live)[0].max()) + 1] if live.any() else ev
    m = (len(ev) // 64) * 64
    w = ev[:m].reshape(-1, 64)
    wmax = w.max(axis=1)
    # a trip evaluates once per lane; the paired ends (2 evaluations) take ~1.3 trips
    def trips(e):
        return np.where(e >= 2, e - 2 + 1.3, e)
    useful = trips(ev[ev > 0]).mean()
    print(f"queries {len(ev)}  evals mean {ev[ev > 0].mean():.3f}  wave-max mean {wmax.mean():.3f}"
          f"  trips/query {useful:.3f}  wave trips {trips(wmax).mean():.3f}"
          f"  lane efficiency {useful / trips(wmax).mean():.3f}", flush=True)
    print("wave-max histogram: " + " ".join(f"{i}:{c}" for i, c in enumerate(np.bincount(wmax))
                                           if c), flush=True)
    base = trips(wmax).sum()
    for cap in (6, 7, 8, 9):
        # pass 1: every wave stops at the cap; pass 2: the unfinished lanes, packed densely in the
        # same order, run their remaining evaluations
        p1 = trips(np.minimum(wmax, cap)).sum()
        rest = ev[:m][ev[:m] > cap] - cap
        k = (len(rest) // 64) * 64
        p2 = rest[:k].reshape(-1, 64).max(axis=1).sum() + (rest[k:].max() if k < len(rest) else 0)
        print(f"cap {cap}: continuing {len(rest)} ({len(rest) / m:.3f})  wave-trips "
              f"{(p1 + p2) / base:.3f} of now", flush=True)


if __name__ == "__main__":
    main()
