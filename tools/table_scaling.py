"""Table-kernel throughput vs grid size (tail / ramp effects): times airice_table_launch with HIP
events on the launch stream for several grids, prints one line per grid."""
import sys
import time

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])

from airiceraytracing_amd import AirIceSolver, make_grid  # noqa: E402

GRIDS = [  # (label, depth_cm, hstep, a0, a1, astep)
    ("cfg2 20m x 0.5deg", -20000.0, 20.0, 92.0, 180.0, 0.5),
    ("1/8 rows", -20000.0, 160.0, 92.0, 180.0, 0.5),
    ("1/4 rows", -20000.0, 80.0, 92.0, 180.0, 0.5),
    ("1/2 rows", -20000.0, 40.0, 92.0, 180.0, 0.5),
    ("4x rows", -20000.0, 5.0, 92.0, 180.0, 0.5),
    ("2x rows", -20000.0, 10.0, 92.0, 180.0, 0.5),
    ("default 10m x 0.1deg", -20000.0, 10.0, 90.1, 180.0, 0.1),
    ("cfg4 rows 1m x 0.1deg", -20000.0, 1.0, 90.1, 180.0, 0.1),
]


def main():
    s = AirIceSolver()
    st = torch.cuda.Stream()
    ngrids = int(sys.argv[1]) if len(sys.argv) > 1 else len(GRIDS)
    for label, d, hs, a0, a1, ast in GRIDS[:ngrids]:
        g = make_grid(d, 300000.0, hs, a0, a1, ast)
        n = g.n_rays
        table = torch.empty((11, n), dtype=torch.float32, device="cuda:0")
        reps = max(3, int(2e8 // n))
        with torch.cuda.stream(st):
            for _ in range(3):
                s.table_device(g, table, stream=st)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(reps):
                s.table_device(g, table, stream=st)
            e1.record(st)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        print(f"{label:24s} rays={n:11d} ms={ms:9.4f} rays/s={n / ms * 1e3:.4g}", flush=True)
        del table
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
