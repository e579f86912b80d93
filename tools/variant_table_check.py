import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from airiceraytracing_amd import _lib
_lib.LIB_PATH = os.path.abspath(sys.argv[1])
from airiceraytracing_amd import AirIceSolver, VARIANT_PYWRAPPER, VARIANT_MULTIRAY, make_grid
import oracle
from tests import parity
import gzip
txt = gzip.open("airiceraytracing_amd/data/Atmosphere.dat.gz", "rb").read()
args = (-20000.0, 300000.0, 100.0, 92.0, 180.0, 1.0)
for variant, pi in ((VARIANT_MULTIRAY, None), (VARIANT_PYWRAPPER, oracle.PI_EXACT)):
    om = oracle.parse_atmosphere(txt, pi) if pi is not None else oracle.parse_atmosphere(txt)
    s = AirIceSolver(variant=variant)
    g = make_grid(*args)
    t = torch.empty((11, g.n_rays), dtype=torch.float32, device="cuda:0")
    s.table_device(g, t); torch.cuda.synchronize()
    ref = oracle.table_rows(om, oracle.grid_init(*args), 0, g.table_rows)
    got = t.cpu().numpy()
    d = got.view(np.int32) != ref.view(np.int32)
    print(sys.argv[1], variant, "ulp", parity.float_ulp_diff(got, ref), "cols differing", d.sum(axis=1))
