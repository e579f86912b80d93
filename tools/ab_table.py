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
    h = hashlib.sha1(table.cpu().numpy().tobytes()).hexdigest()
    print(json.dumps({"lib": lib_path, "ms": ms, "rays_per_s": g.n_rays / ms * 1e3, "sha1": h}))


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
