"""The one-query calls on the host (airice_rays_host, airice_rtf_eval in AIRICE_SCALAR_HOST mode,
the library's default): the drop-ins' one-ray GetRayTracingSolutions, the ray layer
(RayTracingFunctions:: / MultiRayAirIceRefraction:: fDnfR ... MinimizeforLaunchAngle) and the
one-query solves (Air2IceRayTracing, the CoREAS entry, TraceIceToAir, the lookup fallback) run on
the CPU from the same source as the device kernels.  These run here without a GPU: every output
against the oracle at the parity tolerance (1e-9 relative, per-quantity floors, NaN positions
equal).  Host against device is tests/test_gpu_rtf.py::test_host_matches_device."""
import numpy as np
import pytest

import oracle
from tests import parity


@pytest.fixture(scope="module")
def solver():
    from airiceraytracing_amd import AirIceSolver, _lib
    assert _lib.lib().airice_scalar_mode(-1) == _lib.SCALAR_HOST  # the default
    return AirIceSolver()


def _close(got, ref, floor=1e-12, rtol=1e-9):
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    assert got.shape == ref.shape
    nan = np.isnan(ref)
    assert np.array_equal(np.isnan(got), nan), (got, ref)
    err = np.abs(got[~nan] - ref[~nan])
    lim = rtol * np.maximum(np.abs(ref[~nan]), floor)
    assert np.all(err <= lim), (got, ref, err / np.maximum(np.abs(ref[~nan]), floor))


@pytest.mark.parametrize("ice,depth", [(3000.0, -200.0), (3000.0, 100.0), (2000.0, -5.0),
                                       (0.0, -300.0)])
def test_host_rays_vs_oracle(solver, oracle_medium, ice, depth):
    """Launch angles 90..180 deg, Tx heights across every layer, on layer bounds, just above the
    ice and above the atmosphere, Rx in the ice and in the air, grazing (NaN) rays."""
    rng = np.random.default_rng(5)
    la = np.concatenate([rng.uniform(90.0, 180.0, 300), [90.0, 90.1, 92.0, 179.99, 180.0, 135.0]])
    h = np.concatenate([rng.uniform(ice + 1, 100000.0, 300),
                        [8363.53902, 23141.7538, ice + 0.0001, 150000.0, 3217.48275, 50000.0]])
    got = solver.rays_host(la, h, ice, depth, depth < 0)
    ref = np.stack([oracle.ray_solution(oracle_medium, a, t, ice, depth, depth < 0)
                    for a, t in zip(la, h)], axis=1)
    # the Tx 0.1 mm above the ice: its air segment is a difference of antiderivatives of O(1e4)
    # whose values agree to 1e-7, so the oracle's own two-logarithm form carries ~1e-12 m of
    # rounding in a 3 mm THD, and its geometric path (fpathD's longer expression) ~1e-8 m (the
    # log-ratio form here is the more accurate one): checked to 1e-10 m and 1e-7 m
    near = np.isclose(h, ice + 0.0001)
    rep = parity.compare_columns(got[:, ~near], ref[:, ~near], parity.RAY_FLOORS)
    assert rep["ok"], rep
    for c, tol in ((2, 1e-10), (3, 1e-10), (16, 1e-7)):
        assert np.all(np.abs(got[c, near] - ref[c, near]) <= tol), (c, got[c, near], ref[c, near])
    assert np.isnan(ref[2]).any() and np.isfinite(ref[2]).any()


def test_host_rays_table_rows(solver, oracle_medium):
    """Whole cfg2 table rows: the host rays against the oracle's table rows (f32 within 1 ulp)."""
    g = oracle.grid_init(-20000.0, 300000.0, 20.0, 92.0, 180.0, 0.5)
    for row in (0, 1, 2000, 4850):
        t = oracle.table_rows(oracle_medium, g, row, row + 1)
        ang = t[4].astype(np.float64)
        # the table's launch angles are the grid's (column 4 holds them as floats)
        a = 92.0 + 0.5 * np.arange(g.angle_steps)
        a[-1] = 180.0
        assert np.array_equal(a.astype(np.float32), ang.astype(np.float32))
        got = solver.rays_host(a, np.full(a.size, float(t[0][0])), g.stop_height, g.depth_m, True)
        cols = [1, 2, 7, 6, 11, 3, 14, 15, 16, 17, 13]
        assert parity.float_ulp_diff(got[cols].astype(np.float32), t) <= 1


def test_host_rtf_ops_vs_oracle(solver, oracle_medium):
    """Every RayTracingFunctions:: op on random arguments (as tests/test_gpu_rtf.py's device
    test draws them) against the oracle."""
    from airiceraytracing_amd import _lib
    m = oracle_medium
    rng = np.random.default_rng(3)
    for _ in range(150):
        txh = rng.uniform(3001, 99000)
        ice = rng.choice([3000.0, rng.uniform(0, 3500)])
        la = rng.uniform(91, 180)
        air = int(rng.integers(0, 2))
        if air:
            tx, rx = rng.uniform(0, 60000), rng.uniform(0, 60000)
            n1 = oracle.getnz_air(m, tx) * rng.uniform(0.9999, 1.0001)
        else:
            tx, rx = -rng.uniform(0, 300), -rng.uniform(0, 300)
            n1 = rng.uniform(1.0, 1.78)
        L = rng.uniform(0, 1.0)
        cases = [
            (_lib.RTF_HIT_POINT, [n1, rx, tx, rng.uniform(0, 89.9), air]),
            (_lib.RTF_OPTICAL_PATH, [1.0 if air else 1.78, rx, tx, L, air]),
            (_lib.RTF_PROPAGATION_TIME, [1.0 if air else 1.78, rx, tx, L, air]),
            (_lib.RTF_AIR_PROPAGATION, [la, txh, ice]),
            (_lib.RTF_ICE_PROPAGATION, [rng.uniform(0, 60), ice, rng.uniform(0, 300), L]),
            (_lib.RTF_FDNFR, [rng.uniform(-300, 60000), 1.0, rng.uniform(1e-4, 4e-4),
                              -rng.uniform(1e-4, 2e-4), L]),
            (_lib.RTF_FTIMED, [rng.uniform(-300, 60000), 1.0 if air else 1.78, 0.0,
                               -rng.uniform(1e-4, 0.02), 299792458.0, L, air]),
            (_lib.RTF_MIN_LAUNCH, [la, txh, ice, rng.uniform(0, 300), rng.uniform(0, 50000)]),
        ]
        for op, args in cases:
            got = solver.rtf_eval(op, args)
            ref = oracle.rtf_eval(m, op, args)
            floor = 1e-15 if op in (_lib.RTF_PROPAGATION_TIME, _lib.RTF_FTIMED) else 1e-6
            _close(got, ref, floor=floor)


def test_host_rtf_cfg1_kat(solver, oracle_medium):
    """The cfg1 KAT through the host ray layer: THD in air of SingleRayAirIceRefraction 200 170
    20000 3000 prints as 2997.35."""
    from airiceraytracing_amd import _lib
    air = solver.rtf_eval(_lib.RTF_AIR_PROPAGATION, [170.0, 20000.0, 3000.0])
    assert f"{air[0] + air[4] + air[8]:g}" == "2997.35"
    _close(air, oracle.rtf_eval(oracle_medium, _lib.RTF_AIR_PROPAGATION, [170.0, 20000.0, 3000.0]))


def test_scalar_mode_switch():
    from airiceraytracing_amd import _lib
    from airiceraytracing_amd.solver import scalar_mode
    L = _lib.lib()
    assert L.airice_scalar_mode(-1) == _lib.SCALAR_HOST
    with scalar_mode(_lib.SCALAR_DEVICE):
        assert L.airice_scalar_mode(-1) == _lib.SCALAR_DEVICE
    assert L.airice_scalar_mode(-1) == _lib.SCALAR_HOST


@pytest.mark.parametrize("variant", ["multiray", "pywrapper"])
def test_host_one_query_solves_vs_oracle(oracle_medium, oracle_medium_py, variant):
    """Air2IceRayTracing one query at a time (airice_solve_host with n = 1: the host root finder,
    the GSL bisection replay with its guards, and the stage-2 body) against the oracle's solves:
    status bits equal, outputs within 1e-9 (rows whose GSL state is uninitialised excluded)."""
    from airiceraytracing_amd import AirIceSolver, VARIANT_MULTIRAY, VARIANT_PYWRAPPER
    py = variant == "pywrapper"
    s = AirIceSolver(variant=VARIANT_PYWRAPPER if py else VARIANT_MULTIRAY)
    txh, dist, dep = parity.cfg3_queries(400, seed=31)
    outs, sts = [], []
    for i in range(txh.size):
        o, st = s.solve_host(txh[i:i + 1], dist[i:i + 1], dep[i:i + 1], 3000.0)
        outs.append(o[:, 0])
        sts.append(st[0])
    got, gst = np.stack(outs, 1), np.array(sts)
    if py:
        thr = np.array([oracle.straight_angle_of(oracle_medium_py, a, b, 3000.0, c)
                        for a, b, c in zip(txh, dist, dep)])
        rows = [oracle.py_air2ice(oracle_medium_py, a, b, 3000.0, c, t)
                for a, b, c, t in zip(txh, dist, dep, thr)]
        ref = np.stack([r[0] for r in rows], 1)
        rst = np.array([r[1] for r in rows])
        floors = parity.PYSOLVE_FLOORS
    else:
        ref, rst = oracle.solve_batch(oracle_medium, txh, dist, dep, 3000.0)
        floors = parity.SOLVE_FLOORS
    mask = (rst & oracle.SOLVE_UNPINNED) == 0
    assert mask.mean() > 0.95
    assert np.array_equal(gst[mask], rst[mask])
    rep = parity.compare_columns(got, ref, floors, mask=mask)
    assert rep["ok"], rep


def test_host_one_query_trace_vs_oracle(oracle_medium_py):
    """Py_TraceIceToAir one query at a time on the host (airice_trace_ice_to_air_host, n = 1)."""
    from airiceraytracing_amd import AirIceSolver, VARIANT_PYWRAPPER
    s = AirIceSolver(variant=VARIANT_PYWRAPPER)
    d, ice, txh, dist = parity.cfg5_queries(300, seed=17)
    got = np.stack([s.trace_ice_to_air_host(d[i:i + 1], ice[i:i + 1], txh[i:i + 1],
                                            dist[i:i + 1])[0] for i in range(d.size)])
    ref = oracle.py_trace_batch(oracle_medium_py, d, ice, txh, dist)
    rep = parity.compare_columns(got.T, np.asarray(ref).reshape(-1, 10).T, parity.TRACE_FLOORS)
    assert rep["ok"], rep
