"""The reference's validation harness RunMultiRayCode_loop.C (ROOT macro, :6-189) without ROOT:
the table lookup against the minimizer over its (Tx height x straight-line angle) grid, on the
GPU (tools only; tests/test_gpu_loop_validation.py checks it against the oracle).

RunMultiRayCode_loop.C builds the reference default table for one antenna 200 m below the
3000 m ice (:9-38), then walks Tx heights from the ice + 1 m to 100 km in 123 m steps and
straight-line angles from 90.2 to 179.8 deg in 0.23 deg steps (:40-60), sets the horizontal
distance so that the straight line hits the antenna (:89-95), and compares
GetHorizontalDistanceToIntersectionPoint (the minimizer, :112) with
GetHorizontalDistanceToIntersectionPoint_Table (:134) on horizontalDistanceToIntersectionPoint:
-1000 marks a failed / NaN / > 1e10 result (and a table result of exactly 0, :139-141); it
histograms the percent and absolute differences where both succeed (:159-176) and counts the
points where only the table has an answer (:180-183).  The reference records no results of its
own, so these statistics are the harness's output here, not a pinned value.

    python tools/table_vs_minimizer.py [out.json]      (GPU box)
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

PI_MULTIRAY = 3.1415927  # MultiRayAirIceRefraction.h:29
ANTENNA_DEPTH_CM = -200 * 100.0  # RunMultiRayCode_loop.C:9
ICE_CM = 3000 * 100.0  # :10


def harness_queries(antenna_depth_cm=ANTENNA_DEPTH_CM, ice_cm=ICE_CM):
    """(hR cm, TotalHorizontalDistance cm, straight-line angle deg) of every grid point, in the
    macro's loop order (RunMultiRayCode_loop.C:40-95)."""
    step_h, step_th = 123 * 100.0, 0.23
    start_th, stop_th = 90.2, 179.8
    width_th = stop_th - start_th
    start_h = ice_cm + 1 * 100.0
    stop_h = 100000 * 100.0
    if antenna_depth_cm >= 0:
        start_h = antenna_depth_cm + ice_cm + 1 * 100.0
    width_h = stop_h - start_h
    steps_h = int((width_h / step_h) + 1)  # int TotalStepsHb=(GridWidthHb/GridStepSizeHb)+1
    steps_th = int((width_th / step_th) + 1)
    ih, ith = np.meshgrid(np.arange(steps_h), np.arange(steps_th), indexing="ij")
    hR = start_h + step_h * ih.ravel().astype(np.float64)
    thR = start_th + step_th * ith.ravel().astype(np.float64)
    if antenna_depth_cm < 0:
        D = (hR - ice_cm - antenna_depth_cm) * np.tan((180 - thR) * (PI_MULTIRAY / 180.0))
    else:
        D = (hR - (ice_cm + antenna_depth_cm)) * np.tan((180 - thR) * (PI_MULTIRAY / 180.0))
    return hR, D, thR, (steps_h, steps_th)


def harness_values(hdtip_cm, ok, table_cm, table_ok):
    """rtresult / interresult of RunMultiRayCode_loop.C:116-141 (metres, -1000 = no result)."""
    ok = np.asarray(ok).astype(bool)
    table_ok = np.asarray(table_ok).astype(bool)
    rt = hdtip_cm / 100
    rt = np.where((~ok) | np.isnan(rt) | (rt > 1e10), -1000.0, rt)
    it = table_cm / 100
    it = np.where((~table_ok) | np.isnan(it) | (it > 1e10) | (it == 0), -1000.0, it)
    return rt, it


def summarize(rt, it):
    """The macro's counters and histograms (:143-187) as numbers."""
    v1, v2 = rt != -1000, it != -1000
    both = v1 & v2
    pct = np.abs(rt[both] - it[both]) / rt[both] * 100
    absd = np.abs(rt[both] - it[both])
    hist_pct, _ = np.histogram(pct, bins=200, range=(0, 100))  # h1error_dRR (:76)
    hist_abs, _ = np.histogram(absd, bins=200, range=(0, 100))  # h1error (:77)
    q = [50, 90, 99, 99.9]
    return {
        "points": int(rt.size),
        "count1_minimizer_solved": int(v1.sum()),
        "count2_table_solved": int(v2.sum()),
        "count3_both": int(both.sum()),
        "count4_table_only": int((~v1 & v2).sum()),
        "minimizer_only": int((v1 & ~v2).sum()),
        "minb": float(rt[v1].min()) if v1.any() else None,
        "minc": float(it[v2].min()) if v2.any() else None,
        "percent_error": {"mean": float(pct.mean()), **{f"p{p}": float(np.percentile(pct, p))
                                                           for p in q}, "max": float(pct.max())},
        "abs_error_m": {"mean": float(absd.mean()), **{f"p{p}": float(np.percentile(absd, p))
                                                          for p in q}, "max": float(absd.max())},
        "percent_error_under_1pct": float((pct < 1).mean()),
        "h1error_dRR_counts": hist_pct.tolist(),
        "h1error_counts": hist_abs.tolist(),
    }


def run_gpu(solver, hR, D, antenna_depth_cm=ANTENNA_DEPTH_CM, ice_cm=ICE_CM):
    """The minimizer (airice_hdtip_launch) and the lookup (airice_table_lookup_launch on the
    default table, packed) for every point; returns host arrays (out9 cm, ok) of each, and the
    table (host copy) with its grid."""
    import torch
    from airiceraytracing_amd import make_grid
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    g = make_grid(antenna_depth_cm, ice_cm)  # MakeRayTracingTable defaults (.cc:12-21)
    table = torch.empty((11, g.n_rays), dtype=torch.float32, device=dev)
    solver.table_device(g, table, stream=st)
    n = hR.size
    src = torch.from_numpy(np.ascontiguousarray(hR)).to(dev)
    dst = torch.from_numpy(np.ascontiguousarray(D)).to(dev)
    dep = torch.full((n,), antenna_depth_cm, dtype=torch.float64, device=dev)
    mo = torch.empty((9, n), dtype=torch.float64, device=dev)
    mok = torch.empty(n, dtype=torch.uint8, device=dev)
    solver.hdtip_device(src, dst, dep, ice_cm, mo, mok, stream=st)
    lt = solver.lookup_table(table, g)
    solver.lookup_pack(lt, stream=st)
    lo = torch.empty((9, n), dtype=torch.float64, device=dev)
    lok = torch.empty(n, dtype=torch.uint8, device=dev)
    lfl = torch.empty(n, dtype=torch.uint8, device=dev)
    solver.table_lookup_device(lt, src, dst, dep, ice_cm, lo, lok, lfl, stream=st)
    torch.cuda.synchronize()
    return ((mo.cpu().numpy(), mok.cpu().numpy().astype(bool)),
            (lo.cpu().numpy(), lok.cpu().numpy().astype(bool), lfl.cpu().numpy()),
            table.cpu().numpy(), g)


def main():
    from airiceraytracing_amd import AirIceSolver
    hR, D, thR, shape = harness_queries()
    (mo, mok), (lo, lok, lfl), _, g = run_gpu(AirIceSolver(), hR, D)
    rt, it = harness_values(mo[5], mok, lo[5], lok)
    rep = {"_source": "tools/table_vs_minimizer.py: RunMultiRayCode_loop.C's grid and comparison "
                      "on the GPU (minimizer: airice_hdtip_launch; table: the reference default "
                      "grid, airice_table_lookup_launch)",
           "grid": {"tx_heights": shape[0], "angles": shape[1],
                    "table": f"{g.height_steps} x {g.angle_steps} (10 m x 0.1 deg)"},
           "lookup_fallback_lanes": int(np.count_nonzero(lfl & 1)),
           **summarize(rt, it)}
    rep.pop("h1error_counts")
    text = json.dumps(rep, indent=1)
    print(text)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
