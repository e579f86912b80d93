"""Debug probe (GPU box): table-lookup time for the same 1e6 cfg3 queries in random order, sorted
by Tx height, sorted by (Tx height, distance), and counting-sorted into 16-1024 height classes --
how much of lookup_kernel's time is the scatter of its gathers over the table.  With AB_LIB and
--random-only it times one library build (tools/gpu_ab_lookup.sh).

    python tools/lookup_order_probe.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    if os.environ.get("AB_LIB"):  # time another libairice.so build
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
    n = 1000000
    txh, dst, _ = cfg3_queries(n, seed=4242)
    span = 100000.0 - 3000.0
    orders = {"random": np.arange(n), "by_txh": np.argsort(txh, kind="stable"),
              "by_txh_dist": np.lexsort((dst, np.floor(txh / 2000)))}
    if "--random-only" in sys.argv:
        orders = {"random": orders["random"]}
    for nb in (() if "--random-only" in sys.argv else (16, 64, 256, 1024)):  # counting sort into nb height buckets, k order within
        orders[f"bucket{nb}"] = np.argsort(np.floor((txh - 3000.0) / span * nb), kind="stable")
    for name, o in orders.items():
        src = torch.from_numpy(txh[o] * 100).to(dev)
        dcm = torch.from_numpy(dst[o] * 100).to(dev)
        dep = torch.full((n,), -20000.0, dtype=torch.float64, device=dev)
        out = torch.empty((9, n), dtype=torch.float64, device=dev)
        ok = torch.empty(n, dtype=torch.uint8, device=dev)
        fl = torch.empty(n, dtype=torch.uint8, device=dev)
        for _ in range(2):
            s.table_lookup_device(lt, src, dcm, dep, 300000.0, out, ok, fl, stream=st)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(10):
            s.table_lookup_device(lt, src, dcm, dep, 300000.0, out, ok, fl, stream=st)
        e1.record(st)
        torch.cuda.synchronize()
        import hashlib
        h = hashlib.sha1(out.cpu().numpy().tobytes() + ok.cpu().numpy().tobytes() +
                         fl.cpu().numpy().tobytes()).hexdigest()[:12]
        print(f"{name}: {e0.elapsed_time(e1) / 10 * 1e3:.1f} us per 1e6 lookups sha1 {h}", flush=True)


if __name__ == "__main__":
    main()
