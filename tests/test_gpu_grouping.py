"""The minimizer's batch-wide grouping (roots_sorted_kernel) against its block-local
form (roots_kernel): a grouped batch is sorted across the whole batch by straight-line angle and
layer span and solved in that order (the default of the trace source), a block-local one inside
each 1,024-query block (the default of the other sources), but every query is still solved on its
own and written by its index, so the two schedules must give bit-identical outputs.  Both are run in fresh processes
(AIRICE_GROUP_MIN=0: never group; =1: always group) through the minimizer entries --
airice_solve_launch, airice_hdtip_launch and airice_trace_ice_to_air_launch, plus the table
lookup, whose fallback pass stays block-local in both -- and the grouped solve is also checked
against the oracle on a strided sample."""
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle
from tests import parity

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = 300000

CHILD = r"""
import sys
import numpy as np
import torch
sys.path.insert(0, sys.argv[1])
from airiceraytracing_amd import AirIceSolver, VARIANT_PYWRAPPER, make_grid
from tests import parity
n, path = int(sys.argv[2]), sys.argv[3]
dev = torch.device("cuda:0")
s = AirIceSolver()
res = {}
txh, dist, depth = parity.cfg3_queries(n)
t = [torch.from_numpy(a).to(dev) for a in (txh, dist, depth)]
out = torch.empty((17, n), dtype=torch.float64, device=dev)
st = torch.empty(n, dtype=torch.uint8, device=dev)
s.solve_device(t[0], t[1], t[2], 3000.0, out, st, stream=torch.cuda.current_stream())
torch.cuda.synchronize()
res["solve"], res["solve_st"] = out.cpu().numpy(), st.cpu().numpy()
tc = [x * 100 for x in t]
out9 = torch.empty((9, n), dtype=torch.float64, device=dev)
ok = torch.empty(n, dtype=torch.uint8, device=dev)
s.hdtip_device(tc[0], tc[1], tc[2], 300000.0, out9, ok, stream=torch.cuda.current_stream())
torch.cuda.synchronize()
res["hdtip"], res["hdtip_ok"] = out9.cpu().numpy(), ok.cpu().numpy()
g = make_grid(-20000.0, 300000.0, 20.0, 92.0, 180.0, 0.5)
table = torch.empty((11, g.n_rays), dtype=torch.float32, device=dev)
s.table_device(g, table, stream=torch.cuda.current_stream())
torch.cuda.synchronize()
src, dq = parity.lookup_queries(table.cpu().numpy(), n, seed=99)
m = src.size
ts, td = torch.from_numpy(src).to(dev), torch.from_numpy(dq).to(dev)
tp = torch.full((m,), -20000.0, dtype=torch.float64, device=dev)
outl = torch.empty((9, m), dtype=torch.float64, device=dev)
okl = torch.empty(m, dtype=torch.uint8, device=dev)
fl = torch.empty(m, dtype=torch.uint8, device=dev)
s.table_lookup_device(s.lookup_table(table, g), ts, td, tp, 300000.0, outl, okl, fl,
                      stream=torch.cuda.current_stream())
torch.cuda.synchronize()
res["lookup"], res["lookup_ok"], res["lookup_fl"] = outl.cpu().numpy(), okl.cpu().numpy(), fl.cpu().numpy()
sp = AirIceSolver(variant=VARIANT_PYWRAPPER)
d5, i5, t5, x5 = parity.cfg5_queries(n)
res["trace"] = sp.trace_ice_to_air_host(d5, i5, t5, x5)
np.savez(path, **res)
"""


def _run(group_min, path):
    env = dict(os.environ)
    env["AIRICE_GROUP_MIN"] = str(group_min)
    env.pop("AIRICE_SOLVE_STATS", None)
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT, str(N), path], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return np.load(path)


@pytest.fixture(scope="module")
def both(tmp_path_factory):
    d = tmp_path_factory.mktemp("grouping")
    return _run(0, str(d / "local.npz")), _run(1, str(d / "grouped.npz"))


@pytest.mark.parametrize("key", ["solve", "solve_st", "hdtip", "hdtip_ok", "lookup", "lookup_ok",
                                 "lookup_fl", "trace"])
def test_grouped_equals_block_local(both, key):
    a, b = both[0][key], both[1][key]
    assert a.shape == b.shape
    if a.dtype.kind == "f":
        assert np.array_equal(a.view(np.uint64), b.view(np.uint64)) or \
            np.array_equal(a, b, equal_nan=True), key
    else:
        assert np.array_equal(a, b), key


def test_grouped_lookup_ran_fallback(both):
    fl = both[1]["lookup_fl"]
    assert int(((fl & oracle.LOOKUP_FALLBACK) != 0).sum()) > 10  # 82 of 375,014 on this table


def test_grouped_solve_vs_oracle(both, oracle_medium):
    idx = np.arange(0, N, 97)
    txh, dist, depth = (a[idx] for a in parity.cfg3_queries(N))
    ref, rst = oracle.solve_batch(oracle_medium, txh, dist, depth, 3000.0)
    out = both[1]["solve"][:, idx]
    mask = (rst & oracle.SOLVE_UNPINNED) == 0
    rep = parity.compare_columns(out, ref, parity.SOLVE_FLOORS, mask=mask)
    assert rep["ok"], rep
