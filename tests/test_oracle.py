"""CPU tests of the oracle: pinned against the known-answer values recorded in SURVEY.md §4
(tests/golden/kat.json; provenance in tests/golden/README.md), scipy's natural cubic spline,
and the GSL 2.x bisection semantics."""
import json
import math
import os

import numpy as np
import pytest

import oracle
from tests.conftest import GOLDEN


@pytest.fixture(scope="module")
def kat():
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        return json.load(f)


def rel(a, b):
    return abs(a - b) / max(abs(b), 1e-300)


# --------------------------------------------------------------- atmosphere
def test_atmosphere_parameters(oracle_medium, kat):
    k = kat["atmosphere"]
    m = oracle_medium
    assert m.max_layers == k["MaxLayers"]
    assert [m.atmlay[i] / 100 for i in range(5)] == pytest.approx(k["ATMLAY_m"], rel=1e-15)
    assert m.N0 == k["N0"]  # bitwise
    assert [m.C_air[i] for i in range(4)] == k["C_air"]
    assert [m.B_air[i] for i in range(4)] == k["B_air"]
    assert [m.layer_sizes[i] for i in range(3)] == k["layer_sizes"]


def test_spline_n0_matches_scipy(atmosphere_text, oracle_medium):
    from scipy.interpolate import CubicSpline
    lines = atmosphere_text.decode().splitlines()[6:]
    h, n = np.array([[float(t) for t in ln.split()[:2]] for ln in lines if ln.strip()]).T
    keep = h > -1
    cs = CubicSpline(h[keep], n[keep], bc_type="natural")
    assert abs(float(cs(0.0)) - oracle_medium.N0) <= 2e-16


def test_spline_reproduces_cubic_polynomial_knots():
    # natural spline of a straight line is the line itself
    x = np.linspace(-3, 7, 41)
    y = 0.25 * x + 1.0
    xa, ya = np.ascontiguousarray(x), np.ascontiguousarray(y)
    v = oracle.lib().or_spline_eval_at(oracle._ptr(xa), oracle._ptr(ya), len(x), 1.2345)
    assert v == pytest.approx(0.25 * 1.2345 + 1.0, rel=1e-14)


def test_refractive_index_model(oracle_medium):
    m = oracle_medium
    assert oracle.getnz_ice(m, 0.0) == pytest.approx(1.35, abs=1e-15)
    assert oracle.getnz_ice(m, -200.0) == oracle.getnz_ice(m, 200.0)
    assert oracle.getnz_air(m, 0.0) == pytest.approx(m.N0, rel=1e-15)
    # continuity across the layer boundaries (B_air chained, .cc:200-205)
    for b in (3217.48275, 8363.53902, 23141.7538):
        lo, hi = oracle.getnz_air(m, b - 1e-9), oracle.getnz_air(m, b)
        assert abs(lo - hi) < 1e-12


# --------------------------------------------------------------- known answers
def test_kat_ray_solution(oracle_medium, kat):
    k = kat["GetRayTracingSolutions"]
    d = oracle.ray_solution(oracle_medium, *k["args"], True)
    for idx, v in k["dummy"].items():
        assert rel(d[int(idx)], v) <= 1e-14, (idx, d[int(idx)], v)


def test_kat_air2ice(oracle_medium, kat):
    k = kat["Air2IceRayTracing"]
    out, st = oracle.air2ice(oracle_medium, *k["args"])
    assert st == 0
    for idx, v in k["dummy"].items():
        assert rel(out[int(idx)], v) <= 1e-15, (idx, out[int(idx)], v)


def test_kat_py_trace_ice_to_air(oracle_medium_py, kat):
    k = kat["Py_TraceIceToAir"]
    ok, a = oracle.py_trace_ice_to_air(oracle_medium_py, *k["args"])
    assert ok
    np.testing.assert_allclose(a, k["ArrayParameters"], rtol=1e-15, atol=0)


def test_kat_single_ray_cli_thd(oracle_medium, kat):
    # SingleRayAirIceRefraction 200 170 20000 3000 prints THD_air = 2997.35 (README.md)
    d = oracle.ray_solution(oracle_medium, 170.0, 20000.0, 3000.0, -200.0, True)
    assert round(d[3], 2) == kat["SingleRayAirIceRefraction"]["THD_air_printed"]


def test_golden_table_rows(oracle_medium):
    """Regression: committed oracle table rows (tests/golden/table_cfg2_rows.npz)."""
    g = np.load(os.path.join(GOLDEN, "table_cfg2_rows.npz"))
    og = oracle.grid_init(-20000.0, 300000.0, 20.0, 92.0, 180.0, 0.5)
    for r, full in zip(g["rows"], g["full"]):
        _, f = oracle.table_rows(oracle_medium, og, int(r), int(r) + 1, full=True)
        np.testing.assert_array_equal(f, full)


# --------------------------------------------------------------- grid
def test_grid_sizes():
    g = oracle.grid_init(-20000.0, 300000.0, 20.0, 92.0, 180.0, 0.5)
    assert (g.height_steps, g.angle_steps) == (4851, 177)
    g = oracle.grid_init(-20000.0, 300000.0)  # reference defaults (.cc:12-21)
    assert (g.height_steps, g.angle_steps) == (9701, 900)
    g = oracle.grid_init(-20000.0, 300000.0, 1.0, 90.1, 180.0, 0.01)  # cfg4
    assert g.height_steps * g.angle_steps == 872135991
    g = oracle.grid_init(+5000.0, 300000.0)  # Rx in air: stop at ice + depth
    assert not g.in_ice and g.stop_height == 3050.0


def test_table_last_row_and_column_forced(oracle_medium):
    og = oracle.grid_init(-20000.0, 300000.0, 20.0, 92.0, 180.0, 0.5)
    t = oracle.table_rows(oracle_medium, og, og.height_steps - 1, og.height_steps)
    assert np.all(t[0] == 3000.0)                       # AirTxHeight = LoopStopHeight
    assert t[4][-1] == 180.0 and t[4][0] == np.float32(92.0)
    # Tx on the ice: zero-length air path (exact 0, not a rounding residue)
    assert np.all(t[5][~np.isnan(t[5])] == 0.0)


# --------------------------------------------------------------- bisection semantics
def test_bisect_converges_and_counts():
    r, st, calls = oracle.bisect(lambda x: 150.0 - x, 140.0, 160.0)
    assert st == 0 and abs(r - 150.0) < 1e-9 * 150
    assert calls[:2] == [140.0, 160.0]        # set(): f(lo) then f(hi)
    assert calls[2] == 150.0                  # first midpoint is exactly the root here
    assert len(calls) == 3                    # f(mid)==0 -> root=lo=hi=mid -> converged


def test_bisect_non_straddling_walks_to_upper():
    # same-sign bracket: set() returns EINVAL but keeps the state; every iterate keeps the
    # upper half, so the root walks to x_hi
    r, st, _ = oracle.bisect(lambda x: x + 1.0, 100.0, 110.0)
    assert st == 0 and abs(r - 110.0) < 1e-6


def test_bisect_nonfinite_endpoint_zero_state():
    r, st, calls = oracle.bisect(lambda x: math.nan if x < 101 else 105.0 - x, 100.0, 110.0)
    assert st & oracle.SOLVE_NONFINITE_END
    assert len(calls) == 1 and r == 100.0     # modelled zero state: f_lower == 0 -> root = lo


def test_bisect_nonfinite_midpoint_freezes_root():
    r, st, calls = oracle.bisect(lambda x: math.nan if 104.9 < x < 105.1 else 107.0 - x,
                                 100.0, 110.0)
    assert st & oracle.SOLVE_STALE_MID and st & oracle.SOLVE_MAXITER
    assert r == 105.0 and len(calls) == 2 + 40  # same midpoint re-evaluated to max_iter


def test_bisect_exact_zero_at_endpoint():
    r, st, calls = oracle.bisect(lambda x: 0.0 if x == 100.0 else 1.0, 100.0, 110.0)
    assert r == 100.0 and len(calls) == 2


def test_bisect_relative_interval_test():
    # |hi-lo| < 1e-9 * min(|lo|,|hi|): at ~1e5 the loop stops near 1e-4 absolute width
    r, st, calls = oracle.bisect(lambda x: 123456.0 - x, 100000.0, 200000.0)
    assert abs(r - 123456.0) < 1e-9 * 123456 and st == 0
    assert len(calls) - 2 < 40


def test_bisect_max_iter():
    r, st, calls = oracle.bisect(lambda x: 0.5 - x, 0.0, 1.0, tol=1e-300)
    assert len(calls) <= 2 + 40


# --------------------------------------------------------------- properties
def test_snell_at_interface_and_layers(oracle_medium):
    m = oracle_medium
    th = 150.0
    d = oracle.ray_solution(m, th, 50000.0, 3000.0, -200.0, True)
    inc, refr = math.radians(d[12] * 3.1415927 / math.pi), None
    n_air = oracle.getnz_air(m, 3000.0)
    # receive angle in ice at the antenna: L = n_ice(200) sin(recv) = n_air(ice) sin(inc)
    L_air = n_air * math.sin(d[12] * 3.1415927 / 180)
    L_ice = oracle.getnz_ice(m, 200.0) * math.sin(d[13] * 3.1415927 / 180)
    assert abs(L_air - L_ice) < 1e-12
    # L invariant along the air path: n(H) sin(180-theta) == n(ice) sin(inc)
    L_top = oracle.getnz_air(m, 50000.0) * math.sin((180 - th) * 3.1415927 / 180)
    assert abs(L_top - L_air) < 1e-11


def test_thd_monotone_in_launch_angle(oracle_medium):
    ths = np.linspace(100, 179.5, 200)
    thd = [oracle.ray_solution(oracle_medium, t, 30000.0, 3000.0, -200.0, True)[2] for t in ths]
    assert np.all(np.diff(thd) < 0)


def test_nan_pattern_is_total_reflection(oracle_medium):
    m = oracle_medium
    # grazing launch from low altitude: L = n(H) sin(180-theta) > A_air=1 -> NaN
    d = oracle.ray_solution(m, 90.1, 3500.0, 3000.0, -200.0, True)
    L = oracle.getnz_air(m, 3500.0) * math.sin((180 - 90.1) * 3.1415927 / 180)
    assert (L > 1.0) == bool(np.isnan(d[2]))


def test_cfg3_statistics(oracle_medium):
    """~99% solved, ~0.7% bracket non-finite (reference UB)."""
    from tests.parity import cfg3_queries
    txh, dist, depth = cfg3_queries(3000)
    out, st = oracle.solve_batch(oracle_medium, txh, dist, depth, 3000.0, nthreads=4)
    unpinned = (st & oracle.SOLVE_UNPINNED) != 0
    assert unpinned.mean() < 0.02
    ok = np.abs(out[1] - dist) < 1
    assert ok.mean() > 0.97


def test_mt19937_64_known_answer_and_libstdcxx_golden():
    """The cfg3/cfg5 generators are std::mt19937_64 + std::uniform_real_distribution (BASELINE.md
    §3): the C++ standard's known answer, then rows printed by g++ (tests/golden/make_mt_golden.cpp)."""
    import json
    from tests import parity
    assert int(parity._mt19937_64_raw(5489, 10000)[-1]) == 9981545732273789042
    with open(os.path.join(os.path.dirname(__file__), "golden", "mt19937_64_golden.json")) as f:
        gold = json.load(f)
    g3 = np.array(gold["cfg3_seed12345"])
    np.testing.assert_array_equal(np.stack(parity.cfg3_queries(len(g3)), axis=1), g3)
    g5 = np.array(gold["cfg5_seed777"])
    d, ice, txh, dist = parity.cfg5_queries(len(g5))
    np.testing.assert_array_equal(np.stack([d, txh, dist], axis=1), g5)
    assert np.all(ice == 3000.0)


def test_root_window_rule():
    """tests/parity.compare_with_root_window: a row over 1e-9 passes only with both roots inside
    one GSL tolerance window and outputs within 1e-8, and such rows must stay rare."""
    import numpy as np
    from tests import parity
    n = 2_000_000
    ref = np.ones((2, n))
    gpu = ref.copy()
    th = np.full(n, 150.0)
    gpu[1, 7] = 1 + 3e-9                       # over 1e-9, roots equal: a window row
    rep = parity.compare_with_root_window(gpu, ref, np.array([1e-9, 1e-9]), th, th)
    assert rep["ok"] and rep["window_rows"] == 1 and rep["n_bad"] == 0
    thg = th.copy()
    thg[7] = 150.0 * (1 + 2e-9)                # roots two windows apart: unexplained
    rep = parity.compare_with_root_window(gpu, ref, np.array([1e-9, 1e-9]), thg, th)
    assert not rep["ok"] and rep["n_bad"] == 1
    gpu[1, 7] = 1 + 2e-8                       # beyond 1e-8: unexplained
    rep = parity.compare_with_root_window(gpu, ref, np.array([1e-9, 1e-9]), th, th)
    assert not rep["ok"]
    gpu[1, :5] = 1 + 3e-9                      # too many window rows for 2e6 queries
    gpu[1, 7] = 1.0
    rep = parity.compare_with_root_window(gpu, ref, np.array([1e-9, 1e-9]), th, th)
    assert rep["window_rows"] == 5 and not rep["ok"]
