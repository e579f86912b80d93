"""Phase timing of the one-query solve kernel (debug build with -DAIRICE_SCALAR_STAMP=1, GPU box):
in-kernel s_memtime deltas for set-up (log table staging), root finding and the stage-2 body,
and the shader clock from s_memrealtime, medians over cfg3 queries.

    AB_LIB=ab/stamp.so python tools/scalar_stamps.py [n]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from airiceraytracing_amd import _lib
    _lib.LIB_PATH = os.path.abspath(os.environ["AB_LIB"])
    from airiceraytracing_amd import AirIceSolver
    from tests import parity
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    s = AirIceSolver()
    dev = torch.device("cuda:0")
    txh, dist, dep = [torch.from_numpy(a).to(dev) for a in parity.cfg3_queries(n)]
    out = torch.zeros((28, 1), dtype=torch.float64, device=dev)
    st = torch.empty(1, dtype=torch.uint8, device=dev)
    rows = []
    for i in range(n):
        s.solve_device(txh[i:i + 1], dist[i:i + 1], dep[i:i + 1], 3000.0, out, st, ld=1)
        torch.cuda.synchronize()
        rows.append(out[17:28, 0].cpu().numpy().copy())
    a = np.array(rows)
    ghz = a[:, 3] / (a[:, 4] * 10.0)  # ticks per 10 ns
    names = ["setup", "roots", "stage2", "total"]
    med = {k: float(np.median(a[:, j])) for j, k in enumerate(names)}
    print({"ticks_median": med, "clock_ghz_median": float(np.median(ghz)),
           "us_median": {k: v / np.median(ghz) / 1e3 for k, v in med.items()},
           "evals_mean": float(a[:, 5].mean()),
           "eval_us_median": float(np.median(a[:, 6] / ghz / 1e3)),
           "solve_setup_us_median": float(np.median(a[:, 7] / ghz / 1e3)),
           "lean_bisect_us_median": float(np.median(a[:, 8] / ghz / 1e3)),
           "pre_eval_us_median": float(np.median(a[:, 9] / ghz / 1e3)),
           "post_eval_us_median": float(np.median(a[:, 10] / ghz / 1e3))})


if __name__ == "__main__":
    main()
