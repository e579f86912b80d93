"""A/B timing of table-kernel builds: each library (a libairice.so variant) times the cfg2 table
launch in its own subprocess (HIP events on the launch stream), in alternating order over several
rounds, and the float tables are compared bit for bit against the first library's.

    python tools/ab_table.py libA.so libB.so [...] [--rounds 3] [--reps 300]
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(lib_path, reps, grid):
    sys.path.insert(0, ROOT)
    import torch
    from airiceraytracing_amd import _lib
    _lib.LIB_PATH = os.path.abspath(lib_path)
    from airiceraytracing_amd import AirIceSolver, make_grid
    s = AirIceSolver()
    g = make_grid(*grid)
    table = torch.empty((11, g.n_rays), dtype=torch.float32, device="cuda:0")
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        for _ in range(10):
            s.table_device(g, table, stream=st)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            s.table_device(g, table, stream=st)
        e1.record(st)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / reps
    tnp = table.cpu().numpy()
    h = hashlib.sha1(tnp.tobytes()).hexdigest()
    rec = {"lib": lib_path, "ms": ms, "rays_per_s": g.n_rays / ms * 1e3, "sha1": h}
    if os.environ.get("AB_PARITY"):
        # float table vs the oracle (max ulps, differing entries) and the double outputs of a
        # row sample vs the oracle (max relative difference, SURVEY.md §8(d) floors)
        import oracle
        from tests import parity
        om = oracle.load_atmosphere(os.path.join(ROOT, "airiceraytracing_amd", "data",
                                                 "Atmosphere.dat.gz"))
        og = oracle.grid_init(*grid)
        ot = oracle.table_rows(om, og, 0, og.height_steps, nthreads=16)
        rec["max_ulps"] = int(parity.float_ulp_diff(tnp, ot))
        rec["n_diff"] = int(np.count_nonzero(tnp.view(np.int32) != ot.view(np.int32)))
        worst = 0.0
        fh = hashlib.sha1()
        for r0 in range(0, g.height_steps, g.height_steps // 7):
            rr = min(200, g.height_steps - r0)
            full = torch.empty((18, rr * g.angle_steps), dtype=torch.float64, device="cuda:0")
            tt = torch.empty((11, rr * g.angle_steps), dtype=torch.float32, device="cuda:0")
            s.table_device(g, tt, full, row_begin=r0, row_count=rr)
            torch.cuda.synchronize()
            _, of = oracle.table_rows(om, og, r0, r0 + rr, full=True, nthreads=16)
            fnp = full.cpu().numpy()
            fh.update(fnp.tobytes())
            rep = parity.compare_columns(fnp, of, parity.RAY_FLOORS)
            assert rep["ok"], rep
            worst = max(worst, rep["max_rel"])
        rec["full_max_rel"] = worst
        rec["full_sha1"] = fh.hexdigest()[:12]
    print(json.dumps(rec))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("libs", nargs="*")
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--reps", type=int, default=300)
    p.add_argument("--one", default=None)
    p.add_argument("--grid", default="-20000,300000,20,92,180,0.5")
    a = p.parse_args()
    grid = [float(x) for x in a.grid.split(",")]
    if a.one:
        one(a.one, a.reps, grid)
        return
    res = {lib: [] for lib in a.libs}
    sha = {}
    for r in range(a.rounds):
        order = a.libs if r % 2 == 0 else a.libs[::-1]
        for lib in order:
            pr = subprocess.run([sys.executable, __file__, "--one", lib, "--reps", str(a.reps),
                                 f"--grid={a.grid}"], capture_output=True, text=True, timeout=300)
            if pr.returncode != 0:
                sys.exit(f"{lib}: exit {pr.returncode}\n{pr.stderr[-3000:]}")
            out = pr.stdout
            d = json.loads(out.strip().splitlines()[-1])
            res[lib].append(d["ms"])
            sha[lib] = d["sha1"]
            print(json.dumps(d), flush=True)
    ref = sha[a.libs[0]]
    for lib in a.libs:
        ms = sorted(res[lib])
        print(f"{lib}: min {ms[0] * 1e3:.2f} us  median {ms[len(ms) // 2] * 1e3:.2f} us  "
              f"table {'identical' if sha[lib] == ref else 'DIFFERS'}", flush=True)


if __name__ == "__main__":
    main()
