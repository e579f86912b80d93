"""A/B of minimizer builds on the three batch entries whose second stage is one full evaluation
at the parked root (solve_out_kernel, hdtip_out_kernel, trace_out_kernel): the cfg3 Air2Ice call
(1e6), the CoREAS hdtip call on the same queries (cm) and the cfg5 pythonwrapper trace (1e7);
whole-call times (HIP events on the launch stream) and sha1 of each call's outputs.  Each library
runs in its own subprocess, in alternating order over the rounds.

    python tools/ab_stage2.py libA.so libB.so [...] [--rounds 3]      (GPU box)
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(lib_path, reps):
    sys.path.insert(0, ROOT)
    import torch
    from airiceraytracing_amd import _lib
    _lib.LIB_PATH = os.path.abspath(lib_path)
    from airiceraytracing_amd import AirIceSolver, VARIANT_PYWRAPPER
    from tests.parity import cfg3_queries, cfg5_queries
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream()
    rec = {"lib": lib_path}

    def timed(name, call, outs):
        with torch.cuda.stream(st):
            for _ in range(2):
                call()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(reps):
                call()
            e1.record(st)
        torch.cuda.synchronize()
        rec[name + "_ms"] = e0.elapsed_time(e1) / reps
        h = hashlib.sha1()
        for o in outs:
            h.update(o.cpu().numpy().tobytes())
        rec[name + "_sha1"] = h.hexdigest()[:12]

    s = AirIceSolver()
    n3 = 1000000
    txh, dst, dep = (torch.from_numpy(a).to(dev) for a in cfg3_queries(n3))
    out = torch.empty((17, n3), dtype=torch.float64, device=dev)
    stt = torch.empty(n3, dtype=torch.uint8, device=dev)
    timed("solve", lambda: s.solve_device(txh, dst, dep, 3000.0, out, stt, stream=st), (out, stt))
    src, dcm, pcm = txh * 100, dst * 100, dep * 100
    o9 = torch.empty((9, n3), dtype=torch.float64, device=dev)
    ok = torch.empty(n3, dtype=torch.uint8, device=dev)
    timed("hdtip", lambda: s.hdtip_device(src, dcm, pcm, 300000.0, o9, ok, stream=st), (o9, ok))
    ps = AirIceSolver(variant=VARIANT_PYWRAPPER)
    n5 = 10000000
    q = [torch.from_numpy(a).to(dev) for a in cfg5_queries(n5)]
    tout = torch.empty((n5, 10), dtype=torch.float64, device=dev)
    timed("trace", lambda: ps.trace_ice_to_air_device(*q, tout, stream=st), (tout,))
    print(json.dumps(rec))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("libs", nargs="*")
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--one", default=None)
    a = p.parse_args()
    if a.one:
        one(a.one, a.reps)
        return
    res = {lib: [] for lib in a.libs}
    for r in range(a.rounds):
        for lib in (a.libs if r % 2 == 0 else a.libs[::-1]):
            pr = subprocess.run([sys.executable, __file__, "--one", lib, "--reps", str(a.reps)],
                                capture_output=True, text=True, timeout=300)
            if pr.returncode != 0:
                sys.exit(f"{lib}: exit {pr.returncode}\n{pr.stderr[-3000:]}")
            d = json.loads(pr.stdout.strip().splitlines()[-1])
            res[lib].append(d)
            print(json.dumps(d), flush=True)
    ref = res[a.libs[0]][0]
    for lib in a.libs:
        line = [lib]
        for k in ("solve", "hdtip", "trace"):
            ms = sorted(d[k + "_ms"] for d in res[lib])
            same = all(d[k + "_sha1"] == ref[k + "_sha1"] for d in res[lib])
            line.append(f"{k} {ms[0]:.4f}-{ms[-1]:.4f} ms {'same' if same else 'DIFFERS'}")
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
