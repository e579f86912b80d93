"""The one-query calls on the host (airice_rays_host, airice_rtf_eval in AIRICE_SCALAR_HOST mode,
the library's default): the drop-ins' one-ray GetRayTracingSolutions and the ray layer
(RayTracingFunctions:: / MultiRayAirIceRefraction:: fDnfR ... MinimizeforLaunchAngle) run on the
CPU from the same source as the device kernels.  These run here without a GPU: every output
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
