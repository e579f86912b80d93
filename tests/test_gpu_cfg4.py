"""BASELINE cfg4 at full size on one GPU: the fine table (97,001 x 8,991 = 872,135,991 rays,
38.4 GB of float columns in HBM).  Parity through sampled rows against the oracle (<= 1 float
ulp, identical NaN pattern) and size-independent properties of the whole table: the TxH and
launch-angle columns equal the grid's (MakeRayTracingTable .cc:2080-2094), row by row."""
import numpy as np
import pytest

import oracle
from tests import parity

pytestmark = pytest.mark.gpu

CFG4 = (-20000.0, 300000.0, 1.0, 90.1, 180.0, 0.01)


def test_cfg4_full_size(oracle_medium):
    import torch
    from airiceraytracing_amd import AirIceSolver, make_grid
    s = AirIceSolver()
    g = make_grid(*CFG4)
    assert (g.height_steps, g.angle_steps) == (97001, 8991)
    n = g.n_rays
    dev = torch.device("cuda:0")
    table = torch.empty((11, n), dtype=torch.float32, device=dev)
    s.table_device(g, table, stream=torch.cuda.current_stream())
    torch.cuda.synchronize()
    og = oracle.grid_init(*CFG4)
    for r in (0, 1, 23141, 48500, 97000 - 2, 97000):
        got = table[:, r * g.angle_steps:(r + 1) * g.angle_steps].cpu().numpy()
        ref = oracle.table_rows(oracle_medium, og, r, r + 1, nthreads=16)
        assert parity.float_ulp_diff(got, ref) <= 1, r
        assert np.array_equal(np.isnan(got), np.isnan(ref)), r
    # TxH column: row heights (start - step * i, last row forced to the stop height)
    i = torch.arange(g.height_steps, dtype=torch.float64, device=dev)
    h = g.start_height - g.height_step * i
    h[-1] = g.stop_height
    col0 = table[0].view(g.height_steps, g.angle_steps)
    assert torch.equal(col0, h.float()[:, None].expand_as(col0))
    # launch-angle column: start + step * j, last column forced to the stop angle
    j = torch.arange(g.angle_steps, dtype=torch.float64, device=dev)
    th = g.start_angle + g.angle_step * j
    th[-1] = g.stop_angle
    col4 = table[4].view(g.height_steps, g.angle_steps)
    assert torch.equal(col4, th.float()[None, :].expand_as(col4))
