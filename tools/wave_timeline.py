"""Wave timeline of one table launch (AIRICE_TABLE_TRACE, debug only): per-wave start/end on the
100 MHz s_memrealtime clock plus HW_ID / XCC_ID -> resident waves per SIMD over time, round
boundaries, how long SIMDs sit with few waves.  Usage on the GPU box:
    python tools/wave_timeline.py [hstep]   (cfg2 grid by default)"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(hstep):
    path = "/tmp/airice_wave_trace.bin"
    if os.path.exists(path):
        os.remove(path)
    os.environ["AIRICE_TABLE_TRACE"] = path
    import torch
    from airiceraytracing_amd import AirIceSolver, make_grid
    s = AirIceSolver()
    g = make_grid(-20000.0, 300000.0, hstep, 92.0, 180.0, 0.5)
    t = torch.empty((11, g.n_rays), dtype=torch.float32, device="cuda:0")
    for _ in range(3):  # the last launch is analysed
        if os.path.exists(path):
            os.remove(path)
        s.table_device(g, t)
    torch.cuda.synchronize()
    dt = np.dtype([("t0", "<u8"), ("t1", "<u8"), ("c0", "<u8"), ("c1", "<u8"), ("hw", "<u4"),
                   ("xcc", "<u4")])
    return np.fromfile(path, dtype=dt), g


def main():
    hstep = float(sys.argv[1]) if len(sys.argv) > 1 else 20.0
    w, g = run(hstep)
    t0 = w["t0"].min()
    start = (w["t0"] - t0) * 10e-3  # us (100 MHz)
    end = (w["t1"] - t0) * 10e-3
    hw = w["hw"].astype(np.int64)
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    xcc = w["xcc"].astype(np.int64) & 0xF
    key = (((xcc * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd
    nsimd = len(np.unique(key))
    dur = end - start
    out = os.environ.get("AIRICE_TRACE_NPZ")
    if out:
        np.savez_compressed(out, start=start, end=end, key=key)
    print(f"waves={len(w)} simds={nsimd} waves/simd={len(w) / nsimd:.2f} "
          f"kernel span={end.max():.2f}us first-start spread={np.percentile(start, 99):.2f}us")
    # in-kernel shader clock (s_memtime ticks per 100 MHz s_memrealtime tick), long waves only
    dt_real = (w["t1"] - w["t0"]).astype(np.float64)
    dt_core = (w["c1"] - w["c0"]).astype(np.float64)
    long = dt_real > np.percentile(dt_real, 50)
    print(f"in-kernel clock GHz: median {np.median(dt_core[long] / dt_real[long]) * 0.1:.3f}")
    print(f"wave duration us: min {dur.min():.2f} p10 {np.percentile(dur, 10):.2f} "
          f"median {np.median(dur):.2f} p90 {np.percentile(dur, 90):.2f} max {dur.max():.2f}")
    # resident waves per SIMD over time, averaged over SIMDs
    grid = np.linspace(0, end.max(), 60)
    occ = [(np.count_nonzero((start <= t) & (end > t)) / nsimd) for t in grid]
    print("t(us) : mean resident waves per SIMD")
    for t, o in zip(grid[::3], occ[::3]):
        print(f"{t:7.2f} : {o:5.2f} " + "#" * int(round(o * 4)))
    # per-SIMD completion time spread
    last = np.zeros(key.max() + 1)
    np.maximum.at(last, key, end)
    last = last[np.unique(key)]
    print(f"per-SIMD finish us: min {last.min():.2f} median {np.median(last):.2f} "
          f"max {last.max():.2f}")
    # by row group (layers): duration of waves vs Tx height
    wave_row = (np.arange(len(w)) * 64) // g.angle_steps
    H = 100000 - hstep * wave_row
    for lo, hi in ((23141.75, 1e9), (8363.54, 23141.75), (3217.48, 8363.54), (0, 3217.48)):
        m = (H >= lo) & (H < hi)
        if m.any():
            print(f"TxH [{lo:8.1f},{hi:9.1f}): waves {m.sum():6d} median dur {np.median(dur[m]):.2f}us")


if __name__ == "__main__":
    main()
