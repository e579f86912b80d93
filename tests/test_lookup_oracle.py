"""CPU checks of the table-lookup restatement (oracle/airice_oracle.c or_table_lookup,
following MultiRayAirIceRefraction.cc:992-1462) on a coarse oracle-built table.

Parity pin: the reference's lookup is pure float->double interpolation over the table, so
the restatement is pinned by (i) exact reproduction of table entries at table nodes,
(ii) agreement with the independently pinned minimizer (SURVEY §4 KATs) to interpolation
accuracy, and (iii) the reference's documented quirks, each asserted directly.  No golden
output of the reference's lookup exists (it needs GSL + ROOT to run): parity of the
lookup's arithmetic against the reference itself is unpinned beyond (i)-(iii)."""
import numpy as np
import pytest

import oracle
from tests import parity

DEPTH_CM, ICE_CM = -20000.0, 300000.0


@pytest.fixture(scope="module")
def coarse(oracle_medium):
    g = oracle.grid_init(DEPTH_CM, ICE_CM, height_step=250.0, angle_step=0.2)
    tab = oracle.table_rows(oracle_medium, g, 0, g.height_steps, nthreads=8)
    return g, tab, oracle.lookup_table(tab, g)


def test_nodes_reproduce_table_entries(oracle_medium, coarse):
    g, tab, lt = coarse
    rng = np.random.default_rng(3)
    thd = tab[1].astype(np.float64)
    cand = np.flatnonzero(np.isfinite(thd) & (thd > 10.0))
    hits = 0
    for i in rng.choice(cand, 200, replace=False):
        H, D = float(tab[0, i]), float(tab[1, i])
        ok, o, fl = oracle.table_lookup(oracle_medium, lt, H * 100, D * 100, DEPTH_CM, ICE_CM)
        if not ok or fl:
            continue
        hits += 1
        # optical path in ice (col 2), launch angle (col 4 -> rad), THD in air (col 5)
        np.testing.assert_allclose(o[0], tab[2, i] * 100.0, rtol=1e-6)
        np.testing.assert_allclose(o[4], tab[4, i] * (oracle.PI_MULTIRAY / 180), rtol=1e-6)
        np.testing.assert_allclose(o[5], tab[5, i] * 100.0, rtol=1e-6, atol=1e-3)
    assert hits > 150


def test_agrees_with_minimizer(oracle_medium, coarse):
    g, tab, lt = coarse
    rng = np.random.default_rng(11)
    n = 300
    H = rng.uniform(3500, 99000, n)
    D = rng.uniform(10, 40000, n)
    out, ok, fl = oracle.table_lookup_batch(oracle_medium, lt, H * 100, D * 100, DEPTH_CM, ICE_CM)
    rel = []
    for i in np.flatnonzero((ok == 1) & (fl == 0)):
        ok2, o2 = oracle.hdtip(oracle_medium, H[i] * 100, D[i] * 100, DEPTH_CM, ICE_CM)
        if ok2:
            rel.append(abs(out[4, i] - o2[4]) / o2[4])
    rel = np.array(rel)
    assert rel.size > 250
    assert np.median(rel) < 1e-5 and np.quantile(rel, 0.99) < 1e-3


def test_range_and_sentinel_rules(oracle_medium, coarse):
    g, tab, lt = coarse
    hmax, hmin = float(tab[0, 0]), float(tab[0, -1])
    for H in (hmax + 1.0, hmin - 1.0, -10.0):   # .cc:1430-1441
        ok, o, fl = oracle.table_lookup(oracle_medium, lt, H * 100, 100.0 * 100, DEPTH_CM, ICE_CM)
        assert not ok and o[0] == 0 and o[1] == 0 and o[4] == 0 and o[5] == 0
        assert fl & oracle.LOOKUP_UNPINNED  # interpolated slots never initialised
    # D beyond every THD of both rows: both sentinels -> false (.cc:1422-1425)
    ok, o, fl = oracle.table_lookup(oracle_medium, lt, 5000 * 100, 1e9, DEPTH_CM, ICE_CM)
    assert not ok and not (fl & oracle.LOOKUP_FALLBACK)


def test_fallback_quirk(oracle_medium, coarse):
    """One-sided sentinel -> the minimizer runs with cm*100 arguments and the optical /
    geometric output slots swapped (.cc:1418-1420)."""
    g, tab, lt = coarse
    H, D = parity.lookup_queries(tab, 4000, seed=99)
    out, ok, fl = oracle.table_lookup_batch(oracle_medium, lt, H, D, DEPTH_CM, ICE_CM)
    fb = np.flatnonzero(fl & oracle.LOOKUP_FALLBACK)
    assert fb.size > 0
    for i in fb[:20]:
        ok2, f = oracle.hdtip(oracle_medium, H[i] * 100, D[i] * 100, DEPTH_CM * 100, ICE_CM)
        exp = np.array([f[2], f[3], f[0], f[1], f[4], f[5], f[6], f[7], f[8]])
        if not ok[i]:
            exp[[0, 1, 4, 5]] = 0
        np.testing.assert_array_equal(out[:, i], exp)


def test_batch_matches_scalar(oracle_medium, coarse):
    g, tab, lt = coarse
    H, D = parity.lookup_queries(tab, 300, seed=5)
    out, ok, fl = oracle.table_lookup_batch(oracle_medium, lt, H, D, DEPTH_CM, ICE_CM)
    for i in range(0, H.size, 7):
        ok1, o1, fl1 = oracle.table_lookup(oracle_medium, lt, H[i], D[i], DEPTH_CM, ICE_CM)
        assert ok1 == bool(ok[i]) and fl1 == fl[i]
        np.testing.assert_array_equal(o1, out[:, i])


def test_hdtip_batch_matches_scalar(oracle_medium):
    """or_hdtip_batch (the RunMultiRayCode_loop harness's checker) is or_hdtip per row."""
    rng = np.random.default_rng(21)
    n = 64
    H = rng.uniform(3100, 99000, n) * 100
    D = rng.uniform(10, 40000, n) * 100
    out, ok, st = oracle.hdtip_batch(oracle_medium, H, D, np.full(n, DEPTH_CM), ICE_CM, nthreads=4)
    assert out.shape == (9, n) and ok.dtype == bool
    for i in range(n):
        ok1, o1 = oracle.hdtip(oracle_medium, H[i], D[i], DEPTH_CM, ICE_CM)
        assert bool(ok1) == ok[i]
        np.testing.assert_array_equal(out[:, i], o1)
