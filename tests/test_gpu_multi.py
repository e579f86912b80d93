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
