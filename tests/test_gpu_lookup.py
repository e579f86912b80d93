"""GPU parity of the batched table lookup (airice_table_lookup_launch; reference
MultiRayAirIceRefraction.cc:1305-1462) against the oracle restatement on the SAME table.

The table is built on the GPU and copied to the host, so both sides read identical floats.
The lookup itself is float->double interpolation arithmetic, so non-fallback lanes must be
bit-identical (NaN positions included); lanes finished by the minimizer fallback
(.cc:1418-1420) follow the minimizer tolerance (1e-9 relative, parity.HDTIP_FLOORS), with
rows whose bracket set-up reads uninitialised GSL state masked as in test_gpu_parity.
"""
import os

import numpy as np
import pytest

import oracle
from tests import parity

pytestmark = pytest.mark.gpu

NTHREADS = min(16, os.cpu_count() or 1)
ICE_CM = 300000.0


@pytest.fixture(scope="module")
def solver():
    from airiceraytracing_amd import AirIceSolver
    return AirIceSolver()


def _device_table(solver, depth_cm, hstep, a0, a1, astep):
    import torch
    from airiceraytracing_amd import make_grid
    g = make_grid(depth_cm, ICE_CM, hstep, a0, a1, astep)
    table = torch.empty((11, g.n_rays), dtype=torch.float32, device="cuda:0")
    solver.table_device(g, table, stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    return g, table


def _run_case(solver, oracle_medium, depth_cm, hstep, a0, a1, astep, nq, seed):
    import torch
    g, table = _device_table(solver, depth_cm, hstep, a0, a1, astep)
    host = table.cpu().numpy()
    og = oracle.grid_init(depth_cm, ICE_CM, hstep, a0, a1, astep)
    src, dist = parity.lookup_queries(host, nq, seed=seed)
    dep = np.full(src.size, depth_cm)
    n = src.size
    dev = torch.device("cuda:0")
    ts, td, tp = (torch.from_numpy(a).to(dev) for a in (src, dist, dep))
    out = torch.empty((9, n), dtype=torch.float64, device=dev)
    ok = torch.empty(n, dtype=torch.uint8, device=dev)
    fl = torch.empty(n, dtype=torch.uint8, device=dev)
    lt = solver.lookup_table(table, g)
    solver.table_lookup_device(lt, ts, td, tp, ICE_CM, out, ok, fl,
                               stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    out, ok, fl = out.cpu().numpy(), ok.cpu().numpy(), fl.cpu().numpy()
    # the packed table (airice_lookup_pack): the same floats from 128-byte pair records -> identical
    lp = solver.lookup_table(table, g)
    solver.lookup_pack(lp, stream=torch.cuda.current_stream())
    out_p = torch.empty_like(torch.from_numpy(out)).to(dev)
    ok_p = torch.empty(n, dtype=torch.uint8, device=dev)
    fl_p = torch.empty(n, dtype=torch.uint8, device=dev)
    solver.table_lookup_device(lp, ts, td, tp, ICE_CM, out_p, ok_p, fl_p,
                               stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    assert np.array_equal(out_p.cpu().numpy(), out, equal_nan=True)
    assert np.array_equal(ok_p.cpu().numpy(), ok) and np.array_equal(fl_p.cpu().numpy(), fl)
    flat = lp._packed.cpu().numpy()
    ne, asteps = host.shape[1], g.angle_steps
    from airiceraytracing_amd import _lib
    assert flat.size == _lib.lookup_pack_floats(ne, asteps)
    # pair record i (64 B): columns 2, 3, 5-10 of entries i, i+1 (THD and the launch angle come
    # from the search and the angle vector)
    cols = [2, 3, 5, 6, 7, 8, 9, 10]
    packed = flat[:ne * 16].reshape(-1, 16)
    assert np.array_equal(packed[:, :8].T, host[cols], equal_nan=True)
    assert np.array_equal(packed[:-1, 8:].T, host[cols][:, 1:], equal_nan=True)
    assert np.isnan(packed[-1, 8:]).all()
    # the angle vector: column 4 of the first row, verified against every row (word = 1)
    a0 = _lib.lookup_rows_offset(ne) + (ne // asteps) * _lib.LOOKUP_ROW_FLOATS
    assert np.array_equal(flat[a0:a0 + asteps], host[4][:asteps])
    assert flat[a0 + (asteps + 3) // 4 * 4:].view(np.int32)[0] == 1
    assert np.array_equal(host[4].reshape(-1, asteps), np.tile(host[4][:asteps], (ne // asteps, 1)))
    # row records: the row's usable-THD span inside the row and the values at its ends
    r0 = _lib.lookup_rows_offset(ne)
    rows = flat[r0:a0].reshape(ne // asteps, _lib.LOOKUP_ROW_FLOATS)
    ri = rows.view(np.int32)
    r = np.arange(rows.shape[0])
    okr = ri[:, 7] == 1
    assert okr.mean() > 0.9
    s1, e1 = ri[okr, 0], ri[okr, 1]
    assert (s1 >= r[okr] * asteps).all() and (e1 <= r[okr] * asteps + asteps - 1).all()
    assert np.array_equal(rows[okr, 2], host[0][r[okr]])
    assert np.array_equal(rows[okr, 3], host[0][s1]) and np.array_equal(rows[okr, 5], host[1][s1])
    # bisection trees: node 0 of the first height's tree is the THD at FindClosestTHD's first
    # midpoint of (s1, e1), where the span is wide enough to take a step
    tr = ri[okr, 23]
    assert ((tr & 1) != 0).mean() > 0.9
    wide = ((tr & 1) != 0) & (e1 - s1 >= 3)
    assert np.array_equal(rows[okr, 8][wide], host[1][(s1[wide] + e1[wide]) // 2])
    rout, rok, rfl = oracle.table_lookup_batch(oracle_medium, oracle.lookup_table(host, og),
                                               src, dist, dep, ICE_CM, nthreads=NTHREADS)
    assert np.array_equal(fl, rfl), np.flatnonzero(fl != rfl)[:10]
    fb = (rfl & oracle.LOOKUP_FALLBACK) != 0
    # non-fallback lanes: bit-identical
    a, b = out[:, ~fb], rout[:, ~fb]
    same = (a == b) | (np.isnan(a) & np.isnan(b))
    assert same.all(), np.argwhere(~same)[:10]
    assert np.array_equal(ok[~fb], rok[~fb])
    # fallback lanes: the minimizer with the reference's x100 arguments
    idx = np.flatnonzero(fb)
    mask = np.ones(idx.size, dtype=bool)
    for j, i in enumerate(idx):
        _, st = oracle.air2ice(oracle_medium, src[i], dist[i], ICE_CM / 100, dep[i])
        mask[j] = (st & oracle.SOLVE_UNPINNED) == 0
    if idx.size:
        assert np.array_equal(ok[idx][mask], rok[idx][mask])
        rep = parity.compare_columns(out[:, idx], rout[:, idx], parity.HDTIP_FLOORS, mask=mask)
        assert rep["ok"], rep
    print(f"[lookup {depth_cm:+.0f}cm {hstep}m/{astep}deg] n={n} ok={int(ok.sum())} "
          f"fallback={idx.size} (masked {int((~mask).sum())}) "
          f"unpinned={int(np.count_nonzero(rfl & oracle.LOOKUP_UNPINNED))}")
    return n


def test_lookup_cfg2_table(solver, oracle_medium):
    """BASELINE cfg2 table (20 m x 0.5 deg, Rx at -200 m)."""
    _run_case(solver, oracle_medium, -20000.0, 20.0, 92.0, 180.0, 0.5, 100000, 4242)


def test_lookup_reference_default_table(solver, oracle_medium):
    """Reference default grid (10 m x 0.1 deg, 8.7M entries)."""
    _run_case(solver, oracle_medium, -20000.0, 10.0, 90.1, 180.0, 0.1, 100000, 77)


def test_lookup_rx_in_air(solver, oracle_medium):
    """Antenna above the ice (InIce=false): LoopStopHeight = ice + depth (.cc:2058)."""
    _run_case(solver, oracle_medium, 5000.0, 100.0, 90.1, 180.0, 0.3, 30000, 5)


def test_lookup_on_saved_table(solver, tmp_path):
    """Table persistence (f2): a GPU-built cfg2 table saved from the host copy, loaded back and
    uploaded gives bit-identical lookups to the table it was saved from."""
    import torch
    g, table = _device_table(solver, -20000.0, 20.0, 92.0, 180.0, 0.5)
    host = table.cpu().numpy()
    solver.save_table(str(tmp_path / "cfg2.airtbl"), g, table)
    g2, loaded = solver.load_table(str(tmp_path / "cfg2.airtbl"))
    assert loaded.tobytes() == host.tobytes()
    dev = torch.device("cuda:0")
    t2 = torch.from_numpy(loaded).to(dev)
    src, dist = parity.lookup_queries(host, 20000, seed=99)
    n = src.size
    ts, td, tp = (torch.from_numpy(a).to(dev) for a in (src, dist, np.full(n, -20000.0)))
    res = []
    for tab, grid in ((table, g), (t2, g2)):
        out = torch.empty((9, n), dtype=torch.float64, device=dev)
        ok = torch.empty(n, dtype=torch.uint8, device=dev)
        fl = torch.empty(n, dtype=torch.uint8, device=dev)
        solver.table_lookup_device(solver.lookup_table(tab, grid), ts, td, tp, ICE_CM, out, ok, fl,
                                   stream=torch.cuda.current_stream())
        torch.cuda.synchronize()
        res.append((out.cpu().numpy(), ok.cpu().numpy(), fl.cpu().numpy()))
    assert np.array_equal(res[0][0], res[1][0], equal_nan=True)
    assert np.array_equal(res[0][1], res[1][1]) and np.array_equal(res[0][2], res[1][2])


def test_lookup_empty_batch(solver):
    import torch
    g, table = _device_table(solver, -20000.0, 1000.0, 92.0, 180.0, 1.0)
    e = torch.empty(0, dtype=torch.float64, device="cuda:0")
    u = torch.empty(0, dtype=torch.uint8, device="cuda:0")
    solver.table_lookup_device(solver.lookup_table(table, g), e, e, e, ICE_CM,
                               torch.empty((9, 0), dtype=torch.float64, device="cuda:0"), u, u)
    torch.cuda.synchronize()


def test_lookup_pack_angle_vector_fallback(solver, oracle_medium):
    """Pack format 2's angle vector is used only when every row's column 4 equals row 0's bit for
    bit; a table where one row differs (perturbed by one float ulp here) gets verification word 0,
    and lookup_kernel then reads column 4 itself: outputs, ok and flags bit-identical to the
    unpacked (entries = NULL) column path, and to the oracle on the same floats."""
    import torch
    from airiceraytracing_amd import _lib
    g, table = _device_table(solver, -20000.0, 100.0, 92.0, 180.0, 0.5)
    asteps = g.angle_steps
    row = g.table_rows // 2
    c4 = table[4, row * asteps:(row + 1) * asteps]
    table[4, row * asteps:(row + 1) * asteps] = torch.nextafter(c4, torch.full_like(c4, 1e9))
    torch.cuda.synchronize()
    host = table.cpu().numpy()
    assert not np.array_equal(host[4][row * asteps:(row + 1) * asteps], host[4][:asteps])
    src, dist = parity.lookup_queries(host, 20000, seed=17)
    n = src.size
    dev = torch.device("cuda:0")
    dep = np.full(n, -20000.0)
    ts, td, tp = (torch.from_numpy(a).to(dev) for a in (src, dist, dep))
    res = []
    for packed in (False, True):
        lt = solver.lookup_table(table, g)
        if packed:
            solver.lookup_pack(lt, stream=torch.cuda.current_stream())
            torch.cuda.synchronize()
            flat = lt._packed.cpu().numpy()
            ne = host.shape[1]
            a0 = _lib.lookup_rows_offset(ne) + (ne // asteps) * _lib.LOOKUP_ROW_FLOATS
            assert flat[a0 + (asteps + 3) // 4 * 4:].view(np.int32)[0] == 0  # not verified
        out = torch.empty((9, n), dtype=torch.float64, device=dev)
        ok = torch.empty(n, dtype=torch.uint8, device=dev)
        fl = torch.empty(n, dtype=torch.uint8, device=dev)
        with _lib.launched("lookup_kernel") as k:
            solver.table_lookup_device(lt, ts, td, tp, ICE_CM, out, ok, fl,
                                       stream=torch.cuda.current_stream())
            torch.cuda.synchronize()
        assert k.count == 1
        res.append((out.cpu().numpy(), ok.cpu().numpy(), fl.cpu().numpy()))
    assert np.array_equal(res[0][0].view(np.int64), res[1][0].view(np.int64))
    assert np.array_equal(res[0][1], res[1][1]) and np.array_equal(res[0][2], res[1][2])
    og = oracle.grid_init(-20000.0, ICE_CM, 100.0, 92.0, 180.0, 0.5)
    rout, rok, rfl = oracle.table_lookup_batch(oracle_medium, oracle.lookup_table(host, og),
                                               src, dist, dep, ICE_CM, nthreads=NTHREADS)
    out, ok, fl = res[1]
    assert np.array_equal(fl, rfl)
    nf = (rfl & oracle.LOOKUP_FALLBACK) == 0
    a, b = out[:, nf], rout[:, nf]
    assert ((a == b) | (np.isnan(a) & np.isnan(b))).all()
    assert np.array_equal(ok[nf], rok[nf])
