"""Several antennas' tables in one launch (airice_table_launch_multi, table_multi_kernel): bit for
bit the tables of one airice_table_launch per antenna, for antennas in the ice, in the air and
with different row counts."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_multi_antenna_launch_equals_single_launches():
    import torch
    from airiceraytracing_amd import AirIceSolver, make_grid
    s = AirIceSolver()
    dev = torch.device("cuda:0")
    depths = [-20000.0, -10000.0, 5000.0, -30000.0, 0.0]  # cm: in ice, in air (stop 3050 m), at 0
    grids = [make_grid(d, 300000.0, 20.0, 92.0, 180.0, 0.5) for d in depths]
    assert len({g.table_rows for g in grids}) > 1
    single = []
    for g in grids:
        t = torch.full((11, g.n_rays), float("nan"), dtype=torch.float32, device=dev)
        s.table_device(g, t)
        single.append(t)
    multi = [torch.full((11, g.n_rays), float("nan"), dtype=torch.float32, device=dev)
             for g in grids]
    s.tables_device(grids, multi)
    torch.cuda.synchronize()
    for a, (x, y) in enumerate(zip(single, multi)):
        assert torch.equal(x.view(torch.int32), y.view(torch.int32)), a
    # a second call with the same set reuses the device constants; a changed set uploads anew
    s.tables_device(grids[::-1], multi[::-1])
    torch.cuda.synchronize()
    for x, y in zip(single, multi):
        assert torch.equal(x.view(torch.int32), y.view(torch.int32))


def test_multi_antenna_launch_padded_stride_and_empty():
    import torch
    from airiceraytracing_amd import AirIceSolver, make_grid
    s = AirIceSolver()
    dev = torch.device("cuda:0")
    g = make_grid(-20000.0, 300000.0, 500.0, 92.0, 180.0, 2.0)
    ref = torch.empty((11, g.n_rays), dtype=torch.float32, device=dev)
    s.table_device(g, ref)
    wide = torch.zeros((11, g.n_rays + 37), dtype=torch.float32, device=dev)  # ld > rays
    s.tables_device([g], [wide])
    s.tables_device([], [])
    torch.cuda.synchronize()
    assert torch.equal(wide[:, :g.n_rays].view(torch.int32), ref.view(torch.int32))
    assert np.all(wide[:, g.n_rays:].cpu().numpy() == 0)


def test_sharded_host_assembly_with_registered_slabs(tmp_path):
    """The multi-GPU host assembly (bench --workload cfg4, N > 1) in one process: each "rank"
    page-locks only its own rows of every column of a shared /dev/shm-style table and copies its
    device slab there with airice_table_to_host.  The copy must stay inside the registered rows
    (a 2-D copy over the whole pitch failed with "invalid argument" on the GPU box)."""
    import ctypes
    import torch
    from airiceraytracing_amd import AirIceSolver, _lib, make_grid
    from airiceraytracing_amd.distributed import SharedHostTable, assemble_to_host, shard_rows
    L = _lib.lib()
    s = AirIceSolver()
    dev = torch.device("cuda:0")
    g = make_grid(-20000.0, 300000.0, 20.0, 92.0, 180.0, 0.5)
    whole = torch.empty((11, g.n_rays), dtype=torch.float32, device=dev)
    s.table_device(g, whole)
    host = SharedHostTable(str(tmp_path / "table"), 11, g.n_rays, create=True)
    host.tensor.fill_(float("nan"))
    world = 3
    for rank in range(world):
        begin, count, per = shard_rows(g.table_rows, world, rank)
        slab = torch.empty((11, per * g.angle_steps + 64), dtype=torch.float32, device=dev)
        s.table_device(g, slab, None, row_begin=begin, row_count=count, ld=slab.shape[1])
        torch.cuda.synchronize()
        first, items = begin * g.angle_steps, count * g.angle_steps

        def reg(ptr, nbytes):
            _lib.check(L.airice_host_register(ctypes.c_void_p(ptr), nbytes), "register")

        def copy(sl, cnt, h, f):
            _lib.check(L.airice_table_to_host(ctypes.c_void_p(sl.data_ptr()), sl.stride(0), cnt,
                                              ctypes.c_void_p(h.data_ptr() + 4 * f), h.stride(0),
                                              None), "airice_table_to_host")

        host.register_columns(first, items, reg)
        assemble_to_host(slab, items, first, host.tensor, copy)
        torch.cuda.synchronize()
        host.unregister(lambda p: _lib.check(L.airice_host_unregister(ctypes.c_void_p(p)),
                                             "unregister"))
    ref = whole.cpu().numpy()
    got = host.tensor.numpy()
    assert np.array_equal(ref.view(np.int32), got.view(np.int32))
    host.close()


def test_row_constant_cache_follows_medium_and_grid(oracle_medium):
    """The table launch reads its row constants from a device cache keyed by the medium, the ice
    constants row_const reads and the grid heights, and its start-angle sines from one keyed by
    the angle grid and the variant's degree-to-radian factor (first launch of a key: formed in the
    kernel; second: filled, stream-ordered; later: read): alternating grids, antenna depths and the
    two variants must each give the tables an uncached build gives (checked against the oracle's
    float table), on every visit."""
    import torch
    import oracle
    from airiceraytracing_amd import AirIceSolver, make_grid
    from tests import parity
    s = AirIceSolver()
    dev = torch.device("cuda:0")
    cases = [(-20000.0, 300000.0, 100.0, 92.0, 180.0, 1.0),
             (-5000.0, 300000.0, 100.0, 92.0, 180.0, 1.0),     # other antenna depth: same rows
             (-20000.0, 310000.0, 100.0, 92.0, 180.0, 1.0),    # other ice height
             (-20000.0, 300000.0, 70.0, 92.0, 180.0, 1.0),     # other height step
             (-20000.0, 300000.0, 100.0, 90.1, 180.0, 0.7)]    # other angle grid (AIRICE_ANGLE_CACHE)
    first = {}
    for rep in range(3):
        for args in cases:
            g = make_grid(*args)
            t = torch.empty((11, g.n_rays), dtype=torch.float32, device=dev)
            s.table_device(g, t)
            torch.cuda.synchronize()
            got = t.cpu().numpy()
            if rep == 0:
                ref = oracle.table_rows(oracle_medium, oracle.grid_init(*args), 0, g.table_rows)
                assert parity.float_ulp_diff(got, ref) <= 1, args
                first[args] = got
            else:
                assert np.array_equal(got.view(np.int32), first[args].view(np.int32)), args


def test_cached_table_equals_per_lane_rays():
    """The table launch's cached row constants and start-angle sines against rays_kernel, which
    forms both per lane: the 18 doubles of every entry bit for bit, for the media of both solver
    variants, built alternately (MakeRayTracingTable is MultiRay's, so both use its pi)."""
    import torch
    from airiceraytracing_amd import AirIceSolver, VARIANT_MULTIRAY, VARIANT_PYWRAPPER, make_grid
    dev = torch.device("cuda:0")
    g = make_grid(-20000.0, 300000.0, 100.0, 92.0, 180.0, 1.0)
    n = g.n_rays
    for rep in range(2):
        for variant in (VARIANT_MULTIRAY, VARIANT_PYWRAPPER):
            s = AirIceSolver(variant=variant)
            t = torch.empty((11, n), dtype=torch.float32, device=dev)
            full = torch.empty((18, n), dtype=torch.float64, device=dev)
            s.table_device(g, t, full)
            rays = torch.empty((18, n), dtype=torch.float64, device=dev)
            s.rays_device(full[11].contiguous(), full[1].contiguous(), g.stop_height, g.depth_m,
                          bool(g.in_ice), rays)
            torch.cuda.synchronize()
            assert torch.equal(full.view(torch.int64), rays.view(torch.int64)), (rep, variant)


def _warm(s, g, t):
    """Three uncaptured builds of grid g: key recorded, caches filled, fill known complete."""
    import torch
    for _ in range(3):
        s.table_device(g, t)
        torch.cuda.synchronize()


def test_table_launch_in_a_captured_graph():
    """Table launches captured into a HIP graph (torch.cuda.graph): one whose grid is already in
    the row / angle caches (the captured launch pins the entries) and one whose grid is not
    (capture forbids allocating and filling an entry, so that launch forms its rows and sines in
    the kernel); each replay gives the uncaptured launch's table bit for bit."""
    import torch
    from airiceraytracing_amd import AirIceSolver, _lib, make_grid
    s = AirIceSolver()
    dev = torch.device("cuda:0")
    g_hot = make_grid(-20000.0, 300000.0, 100.0, 92.0, 180.0, 1.0)
    g_new = make_grid(-17000.0, 300000.0, 90.0, 91.0, 180.0, 0.9)  # not built before
    ref = {}
    t_hot = torch.empty((11, g_hot.n_rays), dtype=torch.float32, device=dev)
    _warm(s, g_hot, t_hot)
    ref["hot"] = t_hot.clone()
    t_new = torch.full((11, g_new.n_rays), float("nan"), dtype=torch.float32, device=dev)
    t_hot.fill_(float("nan"))
    graph = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        with torch.cuda.graph(graph, stream=side):
            s.table_device(g_hot, t_hot, stream=side)
            s.table_device(g_new, t_new, stream=side)
    torch.cuda.synchronize()
    st = _lib.table_cache_stats()
    assert st["rows"]["pinned"] >= 1 and st["angles"]["pinned"] >= 1, st
    graph.replay()
    torch.cuda.synchronize()
    want_new = torch.empty_like(t_new)
    s.table_device(g_new, want_new)  # uncaptured: builds the cache entries
    torch.cuda.synchronize()
    assert torch.equal(t_hot.view(torch.int32), ref["hot"].view(torch.int32))
    assert torch.equal(t_new.view(torch.int32), want_new.view(torch.int32))


def test_new_antenna_depths_share_row_constants():
    """RunMultiRayCode.C:29-52 builds one table per antenna depth.  The row constants depend only
    on the medium, the grid heights and the Tx-layer ends, not on the depth of an antenna in the
    ice, so tables of one grid for three new in-ice depths add ONE row-constant key (filled at
    the second build, stream-ordered) and one angle key; every table -- the first (rows formed in
    the kernel), the second (filled ahead of it) and the third (read from the cache) -- equals
    the per-lane rays of the same grid bit for bit."""
    import torch
    from airiceraytracing_amd import AirIceSolver, _lib, make_grid
    s = AirIceSolver()
    dev = torch.device("cuda:0")
    before = _lib.table_cache_stats()
    depths = [-23100.0, -41700.0, -8800.0]  # cm, new to this process
    for d in depths:
        g = make_grid(d, 300000.0, 130.0, 91.3, 180.0, 1.3)
        t = torch.empty((11, g.n_rays), dtype=torch.float32, device=dev)
        full = torch.empty((18, g.n_rays), dtype=torch.float64, device=dev)
        s.table_device(g, t, full)
        rays = torch.empty((18, g.n_rays), dtype=torch.float64, device=dev)
        s.rays_device(full[11].contiguous(), full[1].contiguous(), g.stop_height, g.depth_m,
                      bool(g.in_ice), rays)
        torch.cuda.synchronize()
        assert torch.equal(full.view(torch.int64), rays.view(torch.int64)), d
    after = _lib.table_cache_stats()
    assert after["rows"]["keys"] - before["rows"]["keys"] == 1, (before, after)
    assert after["rows"]["filled"] - before["rows"]["filled"] == 1, (before, after)
    assert after["angles"]["keys"] - before["angles"]["keys"] == 1, (before, after)


def test_captured_table_launch_survives_cache_eviction():
    """A captured table launch keeps the addresses of the cache entries it reads in the graph:
    those entries are pinned, so pushing more than the cache's 64 keys through it afterwards
    (evicting every unpinned entry) leaves the replay's table bit for bit the uncaptured one."""
    import torch
    from airiceraytracing_amd import AirIceSolver, _lib, make_grid
    s = AirIceSolver()
    dev = torch.device("cuda:0")
    g = make_grid(-21300.0, 300000.0, 170.0, 91.7, 180.0, 1.1)
    t = torch.empty((11, g.n_rays), dtype=torch.float32, device=dev)
    _warm(s, g, t)
    want = t.clone()
    t.fill_(float("nan"))
    graph = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        with torch.cuda.graph(graph, stream=side):
            s.table_device(g, t, stream=side)
    torch.cuda.synchronize()
    pinned = _lib.table_cache_stats()
    assert pinned["rows"]["pinned"] >= 1 and pinned["angles"]["pinned"] >= 1, pinned
    # 70 new small grids, each built twice (key, then fill): new row and angle keys every time
    for a in range(70):
        ga = make_grid(-20000.0, 300000.0 + a + 1, 5000.0, 92.0 + 1e-6 * (a + 1), 180.0, 8.0)
        ta = torch.empty((11, ga.n_rays), dtype=torch.float32, device=dev)
        s.table_device(ga, ta)
        s.table_device(ga, ta)
    torch.cuda.synchronize()
    st = _lib.table_cache_stats()
    assert st["rows"]["keys"] <= 64 + st["rows"]["pinned"], st
    assert st["rows"]["pinned"] == pinned["rows"]["pinned"], st
    graph.replay()
    torch.cuda.synchronize()
    assert torch.equal(t.view(torch.int32), want.view(torch.int32))


def test_multi_antenna_launch_in_a_captured_graph():
    """airice_table_launch_multi under graph capture: after uncaptured launches of the same antenna
    set (its device constants resident), the captured launch pins them and each replay gives the
    uncaptured tables bit for bit."""
    import torch
    from airiceraytracing_amd import AirIceSolver, make_grid
    s = AirIceSolver()
    dev = torch.device("cuda:0")
    grids = [make_grid(d, 300000.0, 150.0, 92.0, 180.0, 1.5) for d in (-20000.0, -7000.0, 5000.0)]
    tabs = [torch.empty((11, g.n_rays), dtype=torch.float32, device=dev) for g in grids]
    for _ in range(3):
        s.tables_device(grids, tabs)
        torch.cuda.synchronize()
    want = [t.clone() for t in tabs]
    for t in tabs:
        t.fill_(float("nan"))
    graph = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        with torch.cuda.graph(graph, stream=side):
            s.tables_device(grids, tabs, stream=side)
    torch.cuda.synchronize()
    for _ in range(2):
        graph.replay()
        torch.cuda.synchronize()
        for t, w in zip(tabs, want):
            assert torch.equal(t.view(torch.int32), w.view(torch.int32))
