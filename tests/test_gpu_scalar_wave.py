"""One-query calls take the fused wave-parallel kernel (scalar_solve_kernel: the lanes of one wave
share each f evaluation); batches take the per-lane kernels.  The two must agree bit for bit --
roots, status bits and every output column -- for Air2IceRayTracing, the CoREAS entry and
Py_TraceIceToAir, over the cfg3/cfg5 distributions and the edge geometries of
tests/test_gpu_bisect_replay.py (Rx above the ice, Tx just above the ice, Tx above the atmosphere,
near-horizontal rays that run the probe loop)."""
import numpy as np
import pytest

from tests import parity

pytestmark = pytest.mark.gpu


def _queries():
    txh, dist, dep = parity.cfg3_queries(160)
    rng = np.random.default_rng(5)
    n = 40
    near = (rng.uniform(3000.5, 3300.0, n), rng.uniform(0.0, 5.0, n), rng.uniform(-5.0, 500.0, n))
    horiz = (rng.uniform(3001.0, 6000.0, n), rng.uniform(3e4, 5e4, n), -rng.uniform(0.0, 300.0, n))
    above = (rng.uniform(1.0e5, 1.2e5, n), rng.uniform(0.0, 5e4, n), -rng.uniform(0.0, 300.0, n))
    return [np.concatenate([a, near[i], horiz[i], above[i]])
            for i, a in enumerate((txh, dist, dep))]


def _same(a, b):
    return np.array_equal(a.view(np.int64), b.view(np.int64))


def test_one_query_solves_match_the_batch():
    import torch
    from airiceraytracing_amd import AirIceSolver
    dev = torch.device("cuda:0")
    s = AirIceSolver()
    txh, dist, dep = [torch.from_numpy(a).to(dev) for a in _queries()]
    n = txh.numel()
    out = torch.empty((17, n), dtype=torch.float64, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    s.solve_device(txh, dist, dep, 3000.0, out, st)
    one = torch.empty((17, n), dtype=torch.float64, device=dev)
    st1 = torch.empty(n, dtype=torch.uint8, device=dev)
    o1 = torch.empty((17, 1), dtype=torch.float64, device=dev)
    for i in range(n):
        s.solve_device(txh[i:i + 1], dist[i:i + 1], dep[i:i + 1], 3000.0, o1, st1[i:i + 1])
        one[:, i] = o1[:, 0]
    torch.cuda.synchronize()
    a, b = out.cpu().numpy(), one.cpu().numpy()
    bad = np.flatnonzero(~np.all(a.view(np.int64) == b.view(np.int64), axis=0))
    assert bad.size == 0, (bad[:10], a[:, bad[:3]], b[:, bad[:3]])
    assert np.array_equal(st.cpu().numpy(), st1.cpu().numpy())


def test_one_query_hdtip_and_trace_match_the_batch():
    import torch
    from airiceraytracing_amd import AirIceSolver, VARIANT_PYWRAPPER
    dev = torch.device("cuda:0")
    s = AirIceSolver()
    txh, dist, dep = _queries()
    src, dcm, pcm = [torch.from_numpy(a * 100).to(dev) for a in (txh, dist, dep)]
    n = src.numel()
    out = torch.empty((9, n), dtype=torch.float64, device=dev)
    ok = torch.empty(n, dtype=torch.uint8, device=dev)
    s.hdtip_device(src, dcm, pcm, 300000.0, out, ok)
    one = torch.empty((9, n), dtype=torch.float64, device=dev)
    ok1 = torch.empty(n, dtype=torch.uint8, device=dev)
    o1 = torch.empty((9, 1), dtype=torch.float64, device=dev)
    for i in range(n):
        s.hdtip_device(src[i:i + 1], dcm[i:i + 1], pcm[i:i + 1], 300000.0, o1, ok1[i:i + 1])
        one[:, i] = o1[:, 0]
    torch.cuda.synchronize()
    assert _same(out.cpu().numpy(), one.cpu().numpy())
    assert np.array_equal(ok.cpu().numpy(), ok1.cpu().numpy())

    sp = AirIceSolver(variant=VARIANT_PYWRAPPER)
    d5, ice5, t5, x5 = parity.cfg5_queries(200)
    d, ice, t, x = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in (d5, ice5, t5, x5)]
    m = d.numel()
    rows = torch.empty((m, 10), dtype=torch.float64, device=dev)
    sp.trace_ice_to_air_device(d, ice, t, x, rows)
    rows1 = torch.empty((m, 10), dtype=torch.float64, device=dev)
    for i in range(m):
        sp.trace_ice_to_air_device(d[i:i + 1], ice[i:i + 1], t[i:i + 1], x[i:i + 1],
                                   rows1[i:i + 1])
    torch.cuda.synchronize()
    assert _same(rows.cpu().numpy(), rows1.cpu().numpy())


def test_one_ray_matches_the_batch():
    """GetRayTracingSolutions for one ray (scalar_ray_kernel: the segments on lanes 0-4 of one
    wave) against the batch rays_kernel, bit for bit, over launch angles 90..180 deg, Tx heights
    across every layer (on a layer bound, just above the ice, above the atmosphere), Rx in the ice
    and in the air, and the NaN rays (grazing launches)."""
    import torch
    from airiceraytracing_amd import AirIceSolver
    dev = torch.device("cuda:0")
    s = AirIceSolver()
    rng = np.random.default_rng(11)
    la = np.concatenate([rng.uniform(90.0, 180.0, 150), [90.0, 90.1, 92.0, 179.99, 180.0, 135.0]])
    h = np.concatenate([rng.uniform(3000.0, 100000.0, 150),
                        [8363.53902, 23141.7538, 3000.0001, 150000.0, 3217.48275, 50000.0]])
    for ice_m, depth_m in ((3000.0, -200.0), (3000.0, 100.0), (2000.0, -5.0)):
        launch = torch.from_numpy(la).to(dev)
        txh = torch.from_numpy(h).to(dev)
        n = launch.numel()
        out = torch.empty((18, n), dtype=torch.float64, device=dev)
        s.rays_device(launch, txh, ice_m, depth_m, depth_m < 0, out)
        one = torch.empty((18, n), dtype=torch.float64, device=dev)
        o1 = torch.empty((18, 1), dtype=torch.float64, device=dev)
        for i in range(n):
            s.rays_device(launch[i:i + 1], txh[i:i + 1], ice_m, depth_m, depth_m < 0, o1)
            one[:, i] = o1[:, 0]
        torch.cuda.synchronize()
        a, b = out.cpu().numpy(), one.cpu().numpy()
        bad = np.flatnonzero(~np.all(a.view(np.int64) == b.view(np.int64), axis=0))
        assert bad.size == 0, (ice_m, depth_m, bad[:10], a[:, bad[:2]], b[:, bad[:2]])
        assert np.isnan(a[2]).any() and np.isfinite(a[2]).any()


def test_one_query_inside_a_1e6_batch():
    """BASELINE cfg3 (1e6 queries, seed 12345): queries picked across the batch -- every status
    class the batch produced among them -- solved one at a time through the C-ABI's one-query
    route in AIRICE_SCALAR_DEVICE mode (scalar_solve_kernel, counted) equal the batch's
    roots_kernel + solve_out_kernel outputs bit for bit."""
    import torch
    from airiceraytracing_amd import AirIceSolver, _lib
    from airiceraytracing_amd.solver import scalar_mode
    dev = torch.device("cuda:0")
    s = AirIceSolver()
    txh, dist, dep = parity.cfg3_queries(1_000_000)
    t, d, p = [torch.from_numpy(a).to(dev) for a in (txh, dist, dep)]
    n = t.numel()
    out = torch.empty((17, n), dtype=torch.float64, device=dev)
    st = torch.empty(n, dtype=torch.uint8, device=dev)
    with _lib.launched("roots_kernel") as kr:
        s.solve_device(t, d, p, 3000.0, out, st)
        torch.cuda.synchronize()
    assert kr.count == 1
    a, sa = out.cpu().numpy(), st.cpu().numpy()
    pick = list(np.linspace(0, n - 1, 40).astype(int))
    for bit in (1, 2, 4, 8, 16, 32):  # a few queries of each status bit present
        pick += list(np.flatnonzero(sa & bit)[:4])
    pick = sorted(set(int(i) for i in pick))
    with scalar_mode(_lib.SCALAR_DEVICE), _lib.launched("scalar_solve_kernel") as k1:
        for i in pick:
            o, so = s.solve_host(txh[i:i + 1], dist[i:i + 1], dep[i:i + 1], 3000.0)
            assert np.array_equal(o[:, 0].view(np.int64), a[:, i].view(np.int64)), (i, o[:, 0],
                                                                                     a[:, i])
            assert so[0] == sa[i], (i, so[0], sa[i])
    assert k1.count == len(pick)
    print(f"[n=1 vs 1e6 batch] {len(pick)} queries bit-identical, status classes "
          f"{sorted(set(int(sa[i]) for i in pick))}")
