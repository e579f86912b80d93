"""Boundary cases of the C-ABI entry points on the GPU: empty batches (n = 0 launches nothing and
returns AIRICE_OK), degenerate grids (one launch angle, one Tx row, a single ray), and a grid whose
row count is not a multiple of anything the kernel tiles by -- each compared with the oracle."""
import numpy as np
import pytest

import oracle
from tests import parity

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def solver():
    from airiceraytracing_amd import AirIceSolver
    return AirIceSolver()


@pytest.fixture(scope="module")
def solver_py():
    from airiceraytracing_amd import AirIceSolver, VARIANT_PYWRAPPER
    return AirIceSolver(variant=VARIANT_PYWRAPPER)


def test_empty_batches(solver, solver_py):
    import torch
    dev = torch.device("cuda:0")
    e = np.zeros(0)
    out, st = solver.solve_host(e, e, e, 3000.0)
    assert out.shape[-1] == 0 and st.size == 0
    rows = solver_py.trace_ice_to_air_host(e, e, e, e)
    assert rows.shape == (0, 10)
    z = torch.zeros(0, dtype=torch.float64, device=dev)
    o = torch.zeros((18, 0), dtype=torch.float64, device=dev)
    solver.rays_device(z, z, 3000.0, -200.0, True, o)
    torch.cuda.synchronize()


@pytest.mark.parametrize("depth_cm,hstep,a0,a1,astep", [
    (-20000.0, 20.0, 180.0, 180.0, 0.5),    # one launch angle (the forced last column, 180 deg)
    (-20000.0, 97000.0, 92.0, 180.0, 0.5),  # two Tx rows: 100 km and the forced 3 km stop row
    (-20000.0, 97000.0, 180.0, 180.0, 0.5),  # two rays
    (-1234.0, 37.0, 90.1, 180.0, 0.37),     # ragged: 2,622 rows x 243 angles
])
def test_degenerate_and_ragged_grids(solver, oracle_medium, depth_cm, hstep, a0, a1, astep):
    from airiceraytracing_amd import make_grid
    g = make_grid(depth_cm, 300000.0, hstep, a0, a1, astep)
    og = oracle.grid_init(depth_cm, 300000.0, hstep, a0, a1, astep)
    assert (g.height_steps, g.angle_steps) == (og.height_steps, og.angle_steps)
    table, full = solver.table_host(g, full=True)
    ot, of = oracle.table_rows(oracle_medium, og, 0, og.height_steps, full=True, nthreads=16)
    rep = parity.compare_columns(full, of, parity.RAY_FLOORS)
    assert rep["ok"], rep
    assert parity.float_ulp_diff(table, ot) <= 1


@pytest.mark.parametrize("depth_cm,ice_cm,hstep", [
    (-20000.0, 0.0, 500.0),      # sea-level ice: the Tx = 0 row is skipped (.cc:2082)
    (+5000.0, 0.0, 500.0),       # Rx in the air over sea-level ice
    (-100.0, -150000.0, 1000.0),  # ice below sea level: two rows skipped
    (-100.0, -100.0, 3.0),       # last row kept, forced to Tx = -1 m
])
def test_tables_skip_nonpositive_tx_rows(solver, oracle_medium, depth_cm, ice_cm, hstep):
    from airiceraytracing_amd import make_grid
    g = make_grid(depth_cm, ice_cm, hstep, 92.0, 180.0, 0.5)
    og = oracle.grid_init(depth_cm, ice_cm, hstep, 92.0, 180.0, 0.5)
    assert g.table_rows == og.table_rows
    r0 = max(0, g.table_rows - 40)  # the rows next to the skipped ones (and the forced last row)
    table, full = solver.table_host(g, row_begin=r0, full=True)
    ot, of = oracle.table_rows(oracle_medium, og, r0, og.height_steps, full=True, nthreads=16)
    assert table.shape == ot.shape
    rep = parity.compare_columns(full, of, parity.RAY_FLOORS)
    assert rep["ok"], rep
    assert parity.float_ulp_diff(table, ot) <= 1


@pytest.mark.parametrize("where", ["host", "device"])
def test_single_query_batches(solver, oracle_medium, where):
    """n = 1 through airice_solve_host: on the calling thread in AIRICE_SCALAR_HOST mode (no
    kernel), on the GPU's one-query kernel (scalar_solve_kernel) in AIRICE_SCALAR_DEVICE mode --
    the launch counters prove which ran -- and, on the device, bit for bit the same query inside
    a batch (n = 2: roots_kernel + solve_out_kernel)."""
    from airiceraytracing_amd import _lib
    from airiceraytracing_amd.solver import scalar_mode
    mode = _lib.SCALAR_HOST if where == "host" else _lib.SCALAR_DEVICE
    for txh, dist, depth in ((5000.0, 1000.0, -200.0), (99999.0, 49999.0, -300.0),
                             (3001.0, 0.0, -0.5), (20000.0, 5000.0, 10.0)):
        with scalar_mode(mode), _lib.launched("scalar_solve_kernel") as k1, \
                _lib.launched("roots_kernel") as kr:
            out, st = solver.solve_host(np.array([txh]), np.array([dist]), np.array([depth]),
                                        3000.0)
        assert k1.count == (1 if where == "device" else 0) and kr.count == 0
        ref, rst = oracle.solve_batch(oracle_medium, np.array([txh]), np.array([dist]),
                                      np.array([depth]), 3000.0)
        mask = (rst & oracle.SOLVE_UNPINNED) == 0
        rep = parity.compare_columns(out, ref, parity.SOLVE_FLOORS, mask=mask)
        assert rep["ok"], (txh, dist, depth, rep)
        assert st[0] == rst[0]
        with _lib.launched("roots_kernel") as kr:
            pair, pst = solver.solve_host(np.array([txh, txh]), np.array([dist, dist]),
                                          np.array([depth, depth]), 3000.0)
        assert kr.count == 1
        if where == "device":
            assert np.array_equal(out[:, 0].view(np.int64), pair[:, 0].view(np.int64))
            assert np.array_equal(out[:, 0].view(np.int64), pair[:, 1].view(np.int64))
            assert st[0] == pst[0] == pst[1]
        else:  # the host's libm and correctly rounded quotients: within about an ulp
            np.testing.assert_allclose(out[:, 0], pair[:, 0], rtol=1e-12, atol=1e-12)
