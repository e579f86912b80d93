"""The root finder's guarded bisection (evaluating f only at midpoints between the sign guards)
must reproduce GSL bisection with f evaluated at every midpoint, bit for bit: same roots, same
status bits, same outputs.  AIRICE_BISECT_EXACT=1 selects the every-midpoint form on the same
device f, so the comparison isolates the sign prediction from the evaluation's rounding.  Since
round 4 the two guards around a converged secant search are placed from the secant slope instead
of being evaluated; these batches check that the placed guards decide every
midpoint as its evaluation does."""
import os

import numpy as np
import pytest

from tests import parity

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def solvers():
    from airiceraytracing_amd import AirIceSolver, VARIANT_MULTIRAY, VARIANT_PYWRAPPER
    return AirIceSolver(variant=VARIANT_MULTIRAY), AirIceSolver(variant=VARIANT_PYWRAPPER)


def _both(fn):
    old = os.environ.pop("AIRICE_BISECT_EXACT", None)
    try:
        fast = fn()
        os.environ["AIRICE_BISECT_EXACT"] = "1"
        exact = fn()
    finally:
        os.environ.pop("AIRICE_BISECT_EXACT", None)
        if old is not None:
            os.environ["AIRICE_BISECT_EXACT"] = old
    return fast, exact


def _same(a, b):
    a = np.asarray(a)
    b = np.asarray(b)
    assert a.shape == b.shape
    same = (a == b) | (np.isnan(a) & np.isnan(b))
    bad = np.argwhere(~same)
    assert bad.size == 0, f"{bad.shape[0]} differing entries, first {bad[:5].tolist()}"


def test_replay_cfg3(solvers):
    s, _ = solvers
    txh, dist, depth = parity.cfg3_queries(200000, seed=99)
    (out_f, st_f), (out_e, st_e) = _both(lambda: s.solve_host(txh, dist, depth, 3000.0))
    _same(st_f, st_e)
    _same(out_f, out_e)


def test_replay_wide_ranges(solvers):
    """Far distances (no straddle, root outside the bracket), Rx in air, tiny D, grazing Tx."""
    s, _ = solvers
    rng = np.random.default_rng(7)
    n = 100000
    txh = np.concatenate([rng.uniform(3001, 100000, n // 2), rng.uniform(3000.5, 3300, n // 2)])
    dist = np.concatenate([rng.uniform(0, 300000, n // 2), rng.uniform(0, 5, n // 2)])
    depth = np.concatenate([-rng.uniform(0, 300, n // 2), rng.uniform(-5, 500, n // 2)])
    (out_f, st_f), (out_e, st_e) = _both(lambda: s.solve_host(txh, dist, depth, 3000.0))
    _same(st_f, st_e)
    _same(out_f, out_e)


def test_replay_pywrapper_trace(solvers):
    _, sp = solvers
    depth, ice, txh, dist = parity.cfg5_queries(100000, seed=5)
    fast, exact = _both(lambda: sp.trace_ice_to_air_host(depth, ice, txh, dist))
    _same(fast, exact)


def test_replay_hdtip_cm(solvers):
    import torch
    s, _ = solvers
    rng = np.random.default_rng(11)
    n = 50000
    src = rng.uniform(300100, 1e7, n)
    dist = rng.uniform(0, 5e6, n)
    dep = -rng.uniform(0, 30000, n)
    dev = torch.device("cuda:0")

    def run():
        t = [torch.from_numpy(a).to(dev) for a in (src, dist, dep)]
        out = torch.empty((9, n), dtype=torch.float64, device=dev)
        ok = torch.empty(n, dtype=torch.uint8, device=dev)
        s.hdtip_device(t[0], t[1], t[2], 300000.0, out, ok, stream=torch.cuda.current_stream())
        torch.cuda.synchronize()
        return np.concatenate([out.cpu().numpy(), ok.cpu().numpy()[None].astype(np.float64)])

    fast, exact = _both(run)
    _same(fast, exact)


def test_replay_edge_grid(solvers):
    """Tx exactly on layer bounds / at the atmosphere top, zero and tiny distances, antennas at
    the surface, ice heights on layer bounds (per-query ice through the pythonwrapper trace)."""
    import itertools
    _, sp = solvers
    txh = [3000.5, 3217.48275, 3217.4828, 8363.53902, 23141.7538, 50000.0, 99999.99, 100000.0]
    dist = [0.0, 1e-9, 1e-3, 1.0, 1000.0, 5e4, 5e5]
    depth = [-300.0, -1e-9, 0.0, 1e-9, 300.0]
    ice = [0.0, 3000.0, 3217.48275, 8363.53902 - 1.0]
    g = np.array(list(itertools.product(txh, dist, depth, ice)))
    keep = g[:, 0] > g[:, 3] + np.maximum(g[:, 2], 0) + 0.1  # Tx above the Rx
    g = g[keep]
    fast, exact = _both(lambda: sp.trace_ice_to_air_host(g[:, 2], g[:, 3], g[:, 0], g[:, 1]))
    _same(fast, exact)


def test_replay_grazing_and_layer_bounds(solvers):
    """Where f is most curved: launch angles near 90 degrees (distances of 5-400x the height over
    the ice: the probe runs and f steepens towards the NaN edge) and transmitters within a metre
    of the atmosphere's layer bounds.  The slope-placed guards (placed only where the last two
    secant slopes agree within 2x, else evaluated) must decide every midpoint as its evaluation
    does."""
    s, _ = solvers
    rng = np.random.default_rng(21)
    n = 60000
    bounds = np.array([3217.48275, 8363.53902, 23141.7538, 50000.0])
    h1 = rng.uniform(3050, 20000, n // 2)
    d1 = (h1 - 3000) * rng.uniform(5, 400, n // 2)
    h2 = rng.choice(bounds, n // 2) + rng.uniform(-1, 1, n // 2)
    d2 = (h2 - 3000) * rng.uniform(0.01, 50, n // 2)
    txh = np.concatenate([h1, h2])
    dist = np.concatenate([d1, d2])
    depth = -rng.uniform(0, 200, n)
    (out_f, st_f), (out_e, st_e) = _both(lambda: s.solve_host(txh, dist, depth, 3000.0))
    _same(st_f, st_e)
    _same(out_f, out_e)


def test_block_ice_endpoint_matches_per_lane_form(solvers, oracle_medium):
    """roots_kernel forms the batch's ice endpoint once per block and a wave takes it only when
    every lane has that ice height; antennas above the ice shift the height and keep the per-lane
    form.  The in-ice queries must come out bit-identical whether their waves are uniform (alone)
    or mixed with shifted queries (interleaved), and the mixed batch must match the oracle."""
    import oracle
    s, _ = solvers
    rng = np.random.default_rng(33)
    n = 40000
    txh = rng.uniform(3100, 60000, n)
    dist = (txh - 3000) * rng.uniform(0.05, 5, n)
    depth = np.where(np.arange(n) % 3 == 0, rng.uniform(0, 80, n), -rng.uniform(1, 200, n))
    inice = depth < 0
    out_mix, st_mix = s.solve_host(txh, dist, depth, 3000.0)
    out_ice, st_ice = s.solve_host(txh[inice], dist[inice], depth[inice], 3000.0)
    _same(st_mix[inice], st_ice)
    _same(out_mix[:, inice], out_ice)
    sub = np.arange(0, n, 7)
    ref, rst = oracle.solve_batch(oracle_medium, txh[sub], dist[sub], depth[sub], 3000.0)
    mask = (rst & oracle.SOLVE_UNPINNED) == 0
    np.testing.assert_array_equal(st_mix[sub][mask] & 0x1F, rst[mask] & 0x1F)
    rep = parity.compare_columns(out_mix[:, sub], ref, parity.SOLVE_FLOORS, mask=mask)
    assert rep["ok"], rep
