"""BASELINE cfg4 (97,001 x 8,991 = 872,135,991 rays, 38.4 GB of float columns) built on the GPU
and compared with the oracle on EVERY row (tests/test_gpu_cfg4.py checks every 13th row inside
the -m gpu suite's time budget; this is the whole table, ~2 minutes on the box's 16 CPUs).

The oracle (oracle/airice_oracle.c or_table_rows, MakeRayTracingTable .cc:2019-2158 restated)
builds one chunk of rows on the host while the GPU compares the previous chunk: the oracle's
floats go to the device and the comparison (float ulps on the sign-magnitude line, NaN pattern)
runs there.  The bar is tests/test_gpu_cfg4.py's: <= 1 float ulp, identical NaN positions.

    python tools/cfg4_full_parity.py [out.json] [--rows-per-chunk R] [--threads T]   (GPU box)
"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CFG4 = (-20000.0, 300000.0, 1.0, 90.1, 180.0, 0.01)  # tests/test_gpu_cfg4.py, BASELINE cfg4


def ordered(x):
    """float32 bits (as int32) -> a monotone integer line (int64), as tests/parity.py."""
    import torch
    i = x.view(torch.int32).to(torch.int64)
    return torch.where(i < 0, -(i & 0x7FFFFFFF), i)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("out", nargs="?")
    ap.add_argument("--rows-per-chunk", type=int, default=2000)
    ap.add_argument("--threads", type=int, default=16)
    a = ap.parse_args()
    import torch
    import oracle
    from airiceraytracing_amd import AirIceSolver, make_grid
    t0 = time.perf_counter()
    import gzip
    with open(os.path.join(ROOT, "airiceraytracing_amd", "data", "Atmosphere.dat.gz"), "rb") as f:
        m = oracle.parse_atmosphere(gzip.decompress(f.read()), oracle.PI_MULTIRAY)
    s = AirIceSolver()
    g = make_grid(*CFG4)
    og = oracle.grid_init(*CFG4)
    H, A = g.height_steps, g.angle_steps
    assert (H, A) == (97001, 8991) and int(og.table_rows) == H
    dev = torch.device("cuda:0")
    table = torch.empty((11, H * A), dtype=torch.float32, device=dev)
    s.table_device(g, table, stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    t_build = time.perf_counter() - t0
    tab3 = table.view(11, H, A)
    chunks = [(r, min(r + a.rows_per_chunk, H)) for r in range(0, H, a.rows_per_chunk)]
    hist = torch.zeros((11, 3), dtype=torch.int64, device=dev)  # per column: 0 ulp, 1 ulp, > 1
    nan_mismatch = torch.zeros(11, dtype=torch.int64, device=dev)
    nan_count = torch.zeros(11, dtype=torch.int64, device=dev)
    worst = torch.zeros(11, dtype=torch.int64, device=dev)
    worst_at = None
    t_oracle = 0.0

    def build(c):
        t = time.perf_counter()
        ref = oracle.table_rows(m, og, c[0], c[1], nthreads=a.threads)
        return ref, time.perf_counter() - t

    with ThreadPoolExecutor(1) as ex:
        fut = ex.submit(build, chunks[0])
        for k, (r0, r1) in enumerate(chunks):
            ref, dt = fut.result()
            t_oracle += dt
            if k + 1 < len(chunks):
                fut = ex.submit(build, chunks[k + 1])
            rg = torch.from_numpy(ref).to(dev).view(11, r1 - r0, A)
            gg = tab3[:, r0:r1, :]
            ng, nr = torch.isnan(gg), torch.isnan(rg)
            nan_mismatch += (ng != nr).flatten(1).sum(1)
            nan_count += ng.flatten(1).sum(1)
            d = (ordered(gg.contiguous()) - ordered(rg)).abs()
            d = torch.where(ng | nr, torch.zeros_like(d), d).flatten(1)
            hist[:, 0] += (d == 0).sum(1)
            hist[:, 1] += (d == 1).sum(1)
            hist[:, 2] += (d > 1).sum(1)
            cmax = d.max(1).values
            if worst_at is None and bool((cmax > 1).any()):
                col = int(torch.argmax(cmax))
                flat = int(torch.argmax(d[col]))
                worst_at = {"column": col, "row": r0 + flat // A, "angle_index": flat % A,
                            "gpu": float(gg[col].flatten()[flat]),
                            "oracle": float(rg[col].flatten()[flat])}
            worst = torch.maximum(worst, cmax)
            if k % 5 == 0 or k + 1 == len(chunks):
                print(f"rows {r1}/{H}: max ulp {int(worst.max())}, "
                      f"oracle {t_oracle:.0f} s, wall {time.perf_counter() - t0:.0f} s", flush=True)
    torch.cuda.synchronize()
    n = H * A
    rep = {
        "_source": "tools/cfg4_full_parity.py: BASELINE cfg4 on the GPU against the oracle's "
                   "or_table_rows on every row",
        "grid": {"rows": H, "angles": A, "rays": n, "depth_cm": CFG4[0], "ice_cm": CFG4[1]},
        "max_ulp": int(worst.max()),
        "max_ulp_per_column": worst.tolist(),
        "entries_0ulp": int(hist[:, 0].sum()),
        "entries_1ulp": int(hist[:, 1].sum()),
        "entries_over_1ulp": int(hist[:, 2].sum()),
        "per_column_0_1_over": hist.tolist(),
        "nan_position_mismatches": int(nan_mismatch.sum()),
        "nan_entries": int(nan_count.sum()),
        "first_over_1ulp": worst_at,
        "gpu_build_s": t_build,
        "oracle_s": t_oracle,
        "oracle_threads": a.threads,
        "wall_s": time.perf_counter() - t0,
        "passed": int(worst.max()) <= 1 and int(nan_mismatch.sum()) == 0,
    }
    text = json.dumps(rep, indent=1)
    print(text)
    if a.out:
        with open(a.out, "w") as f:
            f.write(text + "\n")
    return 0 if rep["passed"] else 1


if __name__ == "__main__":
    sys.exit(main())
