"""The C++ drop-in (include/MultiRayAirIceRefraction.h) driven by a CoREAS-style caller
(tests/cpp/multiray_driver.cpp, the RunMultiRayCode.C:29-59 sequence) on the GPU, checked
against the oracle."""
import gzip
import json
import math
import os
import re
import subprocess

import numpy as np
import pytest

import oracle
from tests import parity
from tests.conftest import ATMOSPHERE_GZ, ROOT

DRIVER = os.path.join(ROOT, "tests", "cpp", "multiray_driver")


def test_mangled_namespace_symbols_exported():
    """CPU: the reference's Itanium-mangled entry points resolve in libairice.so."""
    from airiceraytracing_amd import _lib
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                        text=True, check=True).stdout
    syms = set(ln.split()[-1] for ln in nm.splitlines())
    for s in ("_ZN24MultiRayAirIceRefraction19MakeRayTracingTableEddi",
              "_ZN24MultiRayAirIceRefraction17Air2IceRayTracingEdddddPd",
              "_ZN24MultiRayAirIceRefraction22GetRayTracingSolutionsEddddPdRb",
              "_ZN24MultiRayAirIceRefraction14MakeAtmosphereEv",
              "_ZN24MultiRayAirIceRefraction9Getnz_airEd",
              "AllTableAllAntData", "TotalAngleSteps", "LoopStopHeight", "MaxAirTxHeight"):
        assert s in syms, s
    hd = [s for s in syms if "GetHorizontalDistanceToIntersectionPoint" in s]
    assert hd, "GetHorizontalDistanceToIntersectionPoint missing"
    # the library must not define the caller-owned globals (reference .h:23-24)
    assert "AntennaDepths" not in syms and "AntennaTableAlreadyMade" not in syms


@pytest.mark.gpu
def test_cpp_caller_against_oracle(tmp_path, oracle_medium):
    assert os.path.exists(DRIVER), "build with __graft_entry__.build()"
    with open(ATMOSPHERE_GZ, "rb") as f:
        (tmp_path / "Atmosphere.dat").write_bytes(gzip.decompress(f.read()))
    out = subprocess.run([DRIVER], cwd=tmp_path, capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    txt = re.sub(r"-?\b(nan|inf)\b", lambda mm: {"nan": "NaN", "-nan": "NaN", "inf": "Infinity",
                                                   "-inf": "-Infinity"}[mm.group(0)], out.stdout)
    r = json.loads(txt)
    m = oracle_medium
    ok, ref = oracle.hdtip(m, 5000e2, 1000e2, -200e2, 3000e2)
    assert r["hdtip_ok"] == int(ok) == 1
    rep = parity.compare_columns(np.array(r["hdtip"])[:, None], ref[:, None], parity.HDTIP_FLOORS)
    assert rep["ok"], rep
    thR = 180 - (math.atan(1000.0 / 2200.0) * (180.0 / 3.1415927))
    ref2, _ = oracle.air2ice(m, 5000.0, 1000.0, 3000.0, -200.0, thR)
    rep = parity.compare_columns(np.array(r["air2ice"])[:, None], ref2[:, None],
                                 parity.SOLVE_FLOORS)
    assert rep["ok"], rep
    ref3 = oracle.ray_solution(m, 170.0, 20000.0, 3000.0, -200.0, True)
    rep = parity.compare_columns(np.array(r["ray"])[:, None], ref3[:, None], parity.RAY_FLOORS)
    assert rep["ok"], rep
    # Fresnel (.cc:267-337) at 0.3 rad
    n1, n2 = oracle.getnz_air(m, 3000.0), oracle.getnz_ice(m, 0.0)
    sq = math.sqrt(1 - ((n1 / n2) * math.sin(0.3)) ** 2)
    num, den = n1 * math.cos(0.3) - n2 * sq, n1 * math.cos(0.3) + n2 * sq
    nump, denp = n1 * sq - n2 * math.cos(0.3), n1 * sq + n2 * math.cos(0.3)
    np.testing.assert_allclose(r["fresnel"], [num / den, 1 + num / den, -nump / denp,
                                              (1 - nump / denp) * (n1 / n2)], rtol=1e-14)
    np.testing.assert_allclose(r["nz"], [oracle.getnz_air(m, 3000.0), oracle.getnz_air(m, 50000.0),
                                         oracle.getnz_ice(m, 200.0)], rtol=0, atol=0)
    # two distinct antennas -> two tables (dedupe of the repeated -200 m antenna)
    og = oracle.grid_init(-10000.0, 300000.0, 2000.0, 92.0, 180.0, 5.0)
    assert r["tables"] == 2 and r["rows"] == og.height_steps and r["cols"] == og.angle_steps
    assert r["LoopStopHeight"] == 3000.0
    ot = oracle.table_rows(m, og, 0, og.height_steps)
    got = np.array(r["table1_row123"], dtype=np.float32)
    assert parity.float_ulp_diff(got, ot[:, 123]) <= 1

    # GetHorizontalDistanceToIntersectionPoint_Table through the reference entry: antenna 1
    # shares antenna 0's depth -> table 0; antenna 2 -> table 1 (.cc:1348-1352).  The oracle
    # runs on the very floats the library holds, so non-fallback outputs match bit for bit.
    tabs = [np.array(r[f"table{i}"], dtype=np.float32) for i in (0, 1)]
    assert parity.float_ulp_diff(tabs[1], ot) <= 1
    lts = [oracle.lookup_table(np.ascontiguousarray(t), og) for t in tabs]
    depths = [-200e2, -200e2, -100e2]
    table_of = [0, 0, 1]
    n_ok = 0
    for row in r["lookup"]:
        a, src, dist = int(row[0]), row[1], row[2]
        ok_ref, o_ref, fl = oracle.table_lookup(m, lts[table_of[a]], src, dist, depths[a], 3000e2)
        assert bool(row[3]) == ok_ref, row
        if fl & oracle.LOOKUP_FALLBACK:
            continue
        got = np.array(row[4:13])
        assert np.array_equal(got, o_ref, equal_nan=True), (row, o_ref)
        n_ok += ok_ref
    assert n_ok >= 6
    assert r["MaxAirTxHeight"] == float(tabs[1][0, 0])
    assert r["MinAirTxHeight"] == float(tabs[1][0, -1])
