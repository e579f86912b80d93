"""Root-finder evaluation counts on cfg3 (debug, GPU box): per query and per wave (the wave runs
until its slowest lane is done), guarded bisection vs every-midpoint bisection, plus the
roots_kernel time of each form.

    python tools/solve_stats.py [n]
"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def child(mode, n, path):
    import torch
    if os.environ.get("AB_LIB"):  # time another libairice.so build
        from airiceraytracing_amd import _lib
        _lib.LIB_PATH = os.path.abspath(os.environ["AB_LIB"])
    from airiceraytracing_amd import AirIceSolver
    from tests import parity
    s = AirIceSolver()
    txh, dist, depth = parity.cfg3_queries(n)
    dev = torch.device("cuda:0")
    t = [torch.from_numpy(a).to(dev) for a in (txh, dist, depth)]
    out = torch.empty((17, n), dtype=torch.float64, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    if path:
        os.environ["AIRICE_SOLVE_STATS"] = path
        s.solve_device(t[0], t[1], t[2], 3000.0, out, st)
        torch.cuda.synchronize()
        return
    for _ in range(3):
        s.solve_device(t[0], t[1], t[2], 3000.0, out, st)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        s.solve_device(t[0], t[1], t[2], 3000.0, out, st)
    e1.record()
    torch.cuda.synchronize()
    import hashlib
    h = hashlib.sha1(out.cpu().numpy().tobytes() + st.cpu().numpy().tobytes()).hexdigest()[:12]
    print(f"{mode}: solve {e0.elapsed_time(e1) / 10:.4f} ms for {n} queries sha1 {h}", flush=True)


def main():
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        mode, n, path = sys.argv[2], int(sys.argv[3]), (sys.argv[4] if len(sys.argv) > 4 else "")
        child(mode, n, path)
        return
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1000000
    for mode in ("fast", "exact"):
        env = dict(os.environ)
        env.pop("AIRICE_BISECT_EXACT", None)
        if mode == "exact":
            env["AIRICE_BISECT_EXACT"] = "1"
        path = f"/tmp/solve_stats_{mode}.bin"
        if os.path.exists(path):
            os.remove(path)
        subprocess.run([sys.executable, __file__, "--child", mode, str(n), path], env=env,
                       check=True, timeout=300)
        subprocess.run([sys.executable, __file__, "--child", mode, str(n)], env=env, check=True,
                       timeout=300)
        a = np.fromfile(path, dtype=np.int32).reshape(-1, 3)
        ev, est, ins = a[:, 0], a[:, 1], a[:, 2]
        m = (len(ev) // 64) * 64
        wave = ev[:m].reshape(-1, 64).max(axis=1)
        print(f"{mode}: evals mean {ev.mean():.2f} p50 {np.median(ev):.0f} p99 "
              f"{np.percentile(ev, 99):.0f} max {ev.max()}  wave-max mean {wave.mean():.2f}  "
              f"secant mean {est.mean():.2f} max {est.max()}  midpoints mean "
              f"{ins.mean():.2f} p99 {np.percentile(ins, 99):.0f}", flush=True)
        hist = np.bincount(ev, minlength=45)
        print("  evals histogram: " + " ".join(f"{i}:{c}" for i, c in enumerate(hist) if c),
              flush=True)
        if mode == "fast":
            eh = np.bincount(est)
            print("  secant histogram: " + " ".join(f"{i}:{c}" for i, c in enumerate(eh) if c))
            from tests import parity
            txh, dist, depth = parity.cfg3_queries(n)
            np.savez_compressed(os.path.join(ROOT, "gpurun_out", "solve_counts.npz"),
                                ev=ev.astype(np.int8), est=est.astype(np.int8),
                                ins=ins.astype(np.int8))
            for lo_, hi_ in ((0, 7), (7, 10), (10, 13), (13, 99)):
                m_ = (ev >= lo_) & (ev < hi_)
                if m_.any():
                    print(f"  evals [{lo_},{hi_}): n={m_.sum()} txh med {np.median(txh[m_]):.0f} "
                          f"dist med {np.median(dist[m_]):.0f} D/(H-3000) med "
                          f"{np.median(dist[m_] / (txh[m_] - 3000)):.3f}", flush=True)


if __name__ == "__main__":
    main()
