"""cfg1 (SingleRayAirIceRefraction) on the CPU: the oracle restatement against the SURVEY §4 KAT,
and the library's host-side plan (layer skips, path sample counts) against the oracle's loops."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import oracle
from tests.conftest import ROOT

CLI = os.path.join(ROOT, "airiceraytracing_amd", "bin", "SingleRayAirIceRefraction")

# (depth m > 0 in ice, launch deg, TxH m, ice m): cfg1, Tx in each layer, ice above the first
# layer boundary (SkipLayersBelow = 1, where the sampler's layer-stop indexing differs from the
# trace's, .C:241), grazing and vertical launches, fractional and zero depth
CASES = [(200, 170, 20000, 3000), (50, 135, 23141.0295, 3000), (10, 100, 5000, 3000),
         (0, 179.5, 3100, 3000), (300.5, 150, 12000, 4000), (1000, 180, 9000, 2000),
         (25, 91, 8363.53902, 3000), (75, 120, 3217.48275, 0)]


def test_kat_cfg1(oracle_medium):
    """SingleRayAirIceRefraction 200 170 20000 3000 prints THD_air 2997.35 and writes
    17,206 path lines (§8 a19) ending at the total THD of GetRayTracingSolutions (3018.907...)."""
    r, x, z = oracle.single_ray(oracle_medium, 200, 170, 20000, 3000)
    assert "%g" % r.thd_air == "2997.35"
    assert abs(r.thd_air - 2997.35470293107) < 1e-9 * 2997.35
    assert r.n_air + r.n_ice == 17206 and r.n_ice == 201
    assert abs(x[-1] - 3018.90722843851) < 1e-9 * 3018.9
    assert z[0] == 20000 and z[r.n_air - 1] == 3000 and z[-1] == 2800
    # the path is continuous at layer boundaries (LastRefracted_x offsets) and monotone in x
    assert np.all(np.diff(x) >= 0)


@pytest.mark.parametrize("case", CASES)
def test_plan_matches_oracle_loops(oracle_medium, case):
    from airiceraytracing_amd import _lib
    m = _lib.load_medium()
    info = _lib.SingleRayInfo()
    assert _lib.lib().airice_single_ray_plan(ctypes.byref(m), *map(float, case),
                                             ctypes.byref(info)) == 0
    r, _, _ = oracle.single_ray(oracle_medium, *map(float, case))
    assert (info.skip_above, info.skip_below, info.n_layers) == (r.skip_above, r.skip_below,
                                                                 r.n_layers)
    assert (info.n_air, info.n_ice) == (r.n_air, r.n_ice)


def test_cli_usage_without_gpu(tmp_path):
    """Argument handling happens before any device call (.C:11-31)."""
    assert os.path.exists(CLI), "build with __graft_entry__.build()"
    out = subprocess.run([CLI], cwd=tmp_path, capture_output=True, text=True, timeout=60)
    assert out.returncode == 0
    assert out.stdout.startswith("No Extra Command Line Argument Passed Other Than Program Name")
    out = subprocess.run([CLI, "1", "2"], cwd=tmp_path, capture_output=True, text=True, timeout=60)
    assert out.stdout.startswith("More Arguments needed!")
    out = subprocess.run([CLI, "1", "2", "3", "4", "5"], cwd=tmp_path, capture_output=True,
                         text=True, timeout=60)
    assert out.stdout.startswith("More Arguments than needed!")
    assert not (tmp_path / "RayPathinAirnIce.txt").exists()
