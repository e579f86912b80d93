"""Time table_multi_kernel against table_kernel: one antenna through each, then 1..8 cfg2 antennas
in one multi launch (HIP events, 100 reps).  GPU box: python tools/multi_probe.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from airiceraytracing_amd import AirIceSolver, make_grid
    s = AirIceSolver()
    st = torch.cuda.current_stream()
    res = {}

    def timeit(fn, reps=100):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            fn()
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3

    grids = [make_grid(-20000.0 - 1000.0 * a, 300000.0, 20.0, 92.0, 180.0, 0.5) for a in range(8)]
    tabs = [torch.empty((11, g.n_rays), dtype=torch.float32, device="cuda:0") for g in grids]
    res["single_table_kernel_us"] = timeit(lambda: s.table_device(grids[0], tabs[0], stream=st))
    for n in (1, 2, 3, 4, 8):
        us = timeit(lambda: s.tables_device(grids[:n], tabs[:n], stream=st))
        res[f"multi_{n}_us"] = us
        res[f"multi_{n}_rays_per_s"] = sum(g.n_rays for g in grids[:n]) / (us * 1e-6)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
