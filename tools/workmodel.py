"""Algorithmic FP64 work per table ray.

W_ray = sum_f n_f * w_f + n_arith, where n_f counts the UNIQUE transcendental / divide
evaluations of the CSE'd device code per ray (airice_device.hpp: segment_full, prim_all,
air_endpoint, fresnel_trans) and w_f is the gfx950 ocml lane-op cost of f
(tools/opweights.json).  Selects, compares and integer index math are not counted.
"""
from __future__ import annotations

import numpy as np

# per air/ice segment (airice_device.hpp segment(), identities (1)-(5)): Snell step 1 div,
# ray parameter 1 sqrt + 1 div, two ends x (1 sqrt), two log ratios (2 div + 2 log), and
# ~40 add/mul forming THD, time and geometric path from them
SEGMENT = {"sqrt": 3, "log": 2, "div": 4, "arith": 40}
# per ray: Tx endpoint (1 exp + 1 div + 8 products), launch sine, incidence asin, ice-segment
# Snell ratio and receive asin, Fresnel T_S/T_P (sin, cos, sqrt, 4 div), output scaling
PER_RAY = {"exp": 1, "sin": 2, "cos": 1, "asin": 2, "sqrt": 1, "div": 6, "arith": 40}
PER_SEGMENT_ACC = {"arith": 3}  # THD/time/geo accumulation


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


def ray_ops(segs: dict, w: dict) -> dict:
    nseg = segs["mean_air"] + segs["ice"]
    counts = {}
    for k, v in SEGMENT.items():
        counts[k] = counts.get(k, 0.0) + v * nseg
    for k, v in PER_SEGMENT_ACC.items():
        counts[k] = counts.get(k, 0.0) + v * nseg
    for k, v in PER_RAY.items():
        counts[k] = counts.get(k, 0.0) + v
    W = sum(counts[k] * w[k] for k in counts)
    return {"W": W, "counts_per_ray": counts, "weights_source": w.get("source", "?")}
