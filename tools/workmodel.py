"""Algorithmic FP64 work per table ray.

W_ray = sum_f n_f * w_f + n_arith, where n_f counts the UNIQUE transcendental / divide
evaluations a table ray needs for its 11 output columns (airice_kernels.hip ray_solution_row,
airice_device.hpp segment_const), w_f is the gfx950 ocml FP64 instruction cost of f
(tools/opweights.json, measured with rocprofv3 --pmc) and n_arith the add/mul/fma count.
Work that depends on the Tx height only (row constants) is amortised over the row's angles;
per-launch constants (Snell ratios between fixed layer bounds, n_air/n_ice) count zero.
Selects, compares and integer index math are not counted.
"""
from __future__ import annotations

import numpy as np

# per air/ice segment (identities (1)-(5)): sqrt(A^2-L^2) and its reciprocal (1 sqrt + 1 div),
# the two ends' sqrt(y^2-L^2) (2 sqrt), two log ratios (2 div + 2 log), ~31 add/mul forming
# the Snell step, L, the log arguments and THD / time / geometric path
SEGMENT = {"sqrt": 3, "log": 2, "div": 3, "arith": 31}
PER_SEGMENT_ACC = {"arith": 3}  # THD/time/geo accumulation
# per ray: launch sine, receive asin in ice, Fresnel T_S / T_P (2 sqrt, 2 div), launch angle
# and output scaling (the incidence asin is dummy[12], not a table column)
PER_RAY = {"sin": 1, "asin": 1, "sqrt": 2, "div": 2, "arith": 24}
# per table row (Tx height): Tx endpoint exp, 1/C and the top segment's Snell ratio, ~20 ops
PER_ROW = {"exp": 1, "div": 2, "arith": 20}


def _layers_m(medium):
    return [medium.atmlay_cm[i] / 100 for i in range(5)], int(medium.max_layers)


def _top(atm, ml, h):
    skip = 0
    for il in range(ml, -1, -1):
        if h < atm[il] and (il >= 1 and h >= atm[il - 1]):
            break
        skip += 1
    return ml - skip - 1


def _bot(atm, ml, ice):
    skip = 0
    for il in range(ml):
        if atm[il] <= ice < atm[il + 1]:
            break
        skip += 1
    return skip


def segments_per_ray(grid, medium=None) -> dict:
    if medium is None:
        from airiceraytracing_amd import load_medium
        medium = load_medium()
    atm, ml = _layers_m(medium)
    hs = grid.start_height - grid.height_step * np.arange(grid.height_steps)
    hs[-1] = grid.stop_height
    bot = _bot(atm, ml, grid.stop_height)
    n_air = np.array([max(0, _top(atm, ml, h) - bot + 1) for h in hs], dtype=np.float64)
    return {"mean_air": float(n_air.mean()), "ice": 1.0 if grid.in_ice else 0.0}


def ray_ops(segs: dict, w: dict, rays_per_row: int = 1) -> dict:
    nseg = segs["mean_air"] + segs["ice"]
    counts = {}
    for k, v in PER_ROW.items():
        counts[k] = counts.get(k, 0.0) + v / max(1, rays_per_row)
    for k, v in SEGMENT.items():
        counts[k] = counts.get(k, 0.0) + v * nseg
    for k, v in PER_SEGMENT_ACC.items():
        counts[k] = counts.get(k, 0.0) + v * nseg
    for k, v in PER_RAY.items():
        counts[k] = counts.get(k, 0.0) + v
    W = sum(counts[k] * w[k] for k in counts)
    return {"W": W, "counts_per_ray": counts, "weights_source": w.get("source", "?")}
