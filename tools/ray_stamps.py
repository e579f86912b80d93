"""Debug probe (GPU box): where a one-ray GetRayTracingSolutions launch spends its time.  Needs a
build with -DAIRICE_RAY_STAMP=1 (AB_LIB): scalar_ray_kernel then writes shader-clock deltas from
its entry into out[18..22] (row constants, sine chain, segment, sums, stores).

    AB_LIB=ab/raystamp.so python tools/ray_stamps.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from airiceraytracing_amd import _lib
    if os.environ.get("AB_LIB"):
        _lib.LIB_PATH = os.path.abspath(os.environ["AB_LIB"])
    from airiceraytracing_amd import AirIceSolver
    s = AirIceSolver()
    dev = torch.device("cuda:0")
    rows = []
    for th, h in ((150.0, 20000.0), (120.0, 80000.0), (170.0, 5000.0), (100.0, 40000.0)) * 50:
        a = torch.tensor([th], dtype=torch.float64, device=dev)
        b = torch.tensor([h], dtype=torch.float64, device=dev)
        out = torch.zeros((24, 1), dtype=torch.float64, device=dev)
        s.rays_device(a, b, 3000.0, -200.0, True, out, ld=1)
        torch.cuda.synchronize()
        rows.append(out[18:23, 0].cpu().numpy())
    r = np.array(rows[8:])
    names = ["row consts", "sine chain", "segment", "sums", "stores"]
    med = np.median(r, axis=0)
    prev = 0.0
    for nm, v in zip(names, med):
        print(f"{nm:12s} at {v:8.0f} ticks (+{v - prev:6.0f})")
        prev = v


if __name__ == "__main__":
    main()
