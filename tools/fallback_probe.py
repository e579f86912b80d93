"""Debug probe (GPU box): the table lookup's fallback pass in isolation -- the lookup of 256
queries of which 0, 1 or 64 take the minimizer fallback, and of the whole 1e6 cfg3 batch (about
200 fallback lanes) -- HIP-event time per call.  AB_LIB: time another libairice.so build.

    python tools/fallback_probe.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    if os.environ.get("AB_LIB"):
        from airiceraytracing_amd import _lib
        _lib.LIB_PATH = os.path.abspath(os.environ["AB_LIB"])
    from airiceraytracing_amd import AirIceSolver, make_grid
    from tests.parity import cfg3_queries
    dev = torch.device("cuda:0")
    s = AirIceSolver()
    st = torch.cuda.current_stream()
    g = make_grid(-20000.0, 300000.0, 20.0, 92.0, 180.0, 0.5)
    table = torch.empty((11, g.n_rays), dtype=torch.float32, device=dev)
    s.table_device(g, table, stream=st)
    lt = s.lookup_table(table, g)
    s.lookup_pack(lt, stream=st)
    txh, dst, _ = cfg3_queries(1000000, seed=4242)

    def run(h, d, reps=20):
        n = len(h)
        src = torch.from_numpy(h * 100).to(dev)
        dcm = torch.from_numpy(d * 100).to(dev)
        dep = torch.full((n,), -20000.0, dtype=torch.float64, device=dev)
        out = torch.empty((9, n), dtype=torch.float64, device=dev)
        ok = torch.empty(n, dtype=torch.uint8, device=dev)
        fl = torch.empty(n, dtype=torch.uint8, device=dev)
        for _ in range(2):
            s.table_lookup_device(lt, src, dcm, dep, 300000.0, out, ok, fl, stream=st)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            s.table_lookup_device(lt, src, dcm, dep, 300000.0, out, ok, fl, stream=st)
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3, fl.cpu().numpy()

    t, fl = run(txh, dst)
    fb = np.flatnonzero(fl & 1)
    nofb = np.flatnonzero((fl & 1) == 0)
    print(f"1e6 batch: {t:.1f} us, {len(fb)} fallback lanes", flush=True)
    for k in (0, 1, 64):
        idx = np.concatenate([fb[:k], nofb[:256 - k]])
        t, f2 = run(txh[idx], dst[idx])
        print(f"256 queries, {int((f2 & 1).sum())} fallback: {t:.1f} us", flush=True)


if __name__ == "__main__":
    main()
