"""cfg1 on the GPU: airice_single_ray_host (trace + path sampler kernels) against the oracle
restatement of SingleRayAirIceRefraction.C / RayTracingFunctions.cc, and the CLI drop-in's stdout
and RayPathinAirnIce.txt against the same restatement formatted as the reference's ostreams.

Tolerance: 1e-9 relative (north_star) with a 1e-6 m floor on x; heights z are exact (they are
the reference's loop variable).  The text file is compared line by line: a line may differ
only where the two doubles straddle a 6-significant-digit rounding boundary."""
import gzip
import os
import subprocess

import numpy as np
import pytest

import oracle
from tests.conftest import ATMOSPHERE_GZ, ROOT
from tests.test_single_ray_cpu import CASES, CLI

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def solver():
    from airiceraytracing_amd import AirIceSolver
    return AirIceSolver()


@pytest.mark.parametrize("case", CASES)
def test_single_ray_device(solver, oracle_medium, case):
    summary, x, z, info = solver.single_ray_host(*map(float, case))
    r, rx, rz = oracle.single_ray(oracle_medium, *map(float, case))
    ref = np.array([r.thd_air, r.L, r.inc_ice, r.thd_ice, r.recv_ice, r.t_ice])
    floors = np.array([1e-6, 1e-9, 1e-9, 1e-6, 1e-9, 1e-15])
    both_nan = np.isnan(summary) & np.isnan(ref)
    assert np.array_equal(np.isnan(summary), np.isnan(ref)), (summary, ref)
    err = np.where(both_nan, 0, np.abs(summary - ref) / np.maximum(np.abs(ref), floors))
    assert err.max() <= 1e-9, (case, summary, ref)
    assert x.size == rx.size
    assert np.array_equal(z, rz)
    assert np.array_equal(np.isnan(x), np.isnan(rx))
    ok = ~np.isnan(rx)
    rel = np.abs(x[ok] - rx[ok]) / np.maximum(np.abs(rx[ok]), 1e-6)
    assert rel.size == 0 or rel.max() <= 1e-9, (case, rel.max())


def _g(v):
    return "%g" % v


def test_cli_cfg1(tmp_path, oracle_medium):
    with open(ATMOSPHERE_GZ, "rb") as f:
        (tmp_path / "Atmosphere.dat").write_bytes(gzip.decompress(f.read()))
    out = subprocess.run([CLI, "200", "170", "20000", "3000"], cwd=tmp_path, capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    lines = out.stdout.splitlines()
    r, rx, rz = oracle.single_ray(oracle_medium, 200.0, 170.0, 20000.0, 3000.0)
    expect = [
        "Antenna Depth is set at 200 m, The Ray Launch Angle is set at 170 deg, Tx Height is set "
        "at 20000 m, Ice Layer Height is set as 3000 m",
        "Tx Height is in this layer with a height range of 23141.8 m to 8363.54 m and is at a "
        "height of 20000 m",
        "Ice Layer is in the layer with a height range of 0 m to 3217.48 m and is at a height of "
        "3000 m",
        "Total horizontal distance travelled by the ray using Multiple Layer fitting is "
        + _g(r.thd_air),
        "Now treating the atmosphere refrative index profile as a single layer and fitting it and "
        "propogating the ray",
    ]
    assert lines[:5] == expect
    assert lines[5].startswith("total time taken by the script: ")
    assert "2997.35" in lines[3]
    got = (tmp_path / "RayPathinAirnIce.txt").read_text().splitlines()
    assert len(got) == 17206 == rx.size
    differ = 0
    for k, ln in enumerate(got):
        want = "%d %s %s" % (k, _g(rx[k]), _g(rz[k]))
        if ln != want:
            differ += 1
            i, xv, zv = ln.split()
            assert int(i) == k and float(zv) == float(_g(rz[k]))
            assert abs(float(xv) - rx[k]) <= 1e-5 * max(abs(rx[k]), 1.0), (ln, want)
    assert differ <= 2, differ


def test_cli_clamps(tmp_path, oracle_medium):
    """Tx above the data (clamped to h_data.back().back()) and a launch angle <= 90 (-> 135)."""
    with open(ATMOSPHERE_GZ, "rb") as f:
        (tmp_path / "Atmosphere.dat").write_bytes(gzip.decompress(f.read()))
    out = subprocess.run([CLI, "100", "45", "50000", "3000"], cwd=tmp_path, capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    s = out.stdout
    assert ("Tx Height is set higher than maximum available height for atmospheric refractive "
            "index which is 23141") in s
    assert "Setting RayLaunchAngle at135" in s
    r, rx, rz = oracle.single_ray(oracle_medium, 100.0, 135.0, oracle_medium.h_top, 3000.0)
    assert ("is " + _g(r.thd_air) + "\n") in s
    got = (tmp_path / "RayPathinAirnIce.txt").read_text().splitlines()
    assert len(got) == rx.size
