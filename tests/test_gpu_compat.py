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
@pytest.mark.parametrize("scalar", ["host", "device"])
def test_cpp_caller_against_oracle(tmp_path, oracle_medium, scalar):
    """scalar: the one-query calls on the host (the default) or on the GPU (AIRICE_SCALAR)."""
    assert os.path.exists(DRIVER), "build with __graft_entry__.build()"
    with open(ATMOSPHERE_GZ, "rb") as f:
        (tmp_path / "Atmosphere.dat").write_bytes(gzip.decompress(f.read()))
    out = subprocess.run([DRIVER], cwd=tmp_path, capture_output=True, text=True, timeout=120,
                         env=dict(os.environ, AIRICE_SCALAR=scalar))
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


INNER = os.path.join(ROOT, "tests", "cpp", "multiray_inner_driver")


def _run_driver(exe, tmp_path, scalar="host"):
    """scalar: where the one-query ray and ray-layer calls run (AIRICE_SCALAR: the host by
    default, or the one-wave device kernels)."""
    assert os.path.exists(exe), "build with __graft_entry__.build()"
    with open(ATMOSPHERE_GZ, "rb") as f:
        (tmp_path / "Atmosphere.dat").write_bytes(gzip.decompress(f.read()))
    env = dict(os.environ, AIRICE_SCALAR=scalar)
    out = subprocess.run([exe], cwd=tmp_path, capture_output=True, text=True, timeout=120,
                         env=env)
    assert out.returncode == 0, out.stderr
    txt = re.sub(r"-?\b(nan|inf)\b", lambda mm: {"nan": "NaN", "-nan": "NaN", "inf": "Infinity",
                                                   "-inf": "-Infinity"}[mm.group(0)], out.stdout)
    return json.loads(txt)


def _close(got, ref, rtol=1e-9, floor=1e-12):
    got, ref = np.asarray(got, dtype=np.float64), np.asarray(ref, dtype=np.float64)
    assert got.shape == ref.shape
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    fin = ~np.isnan(ref)
    err = np.abs(got[fin] - ref[fin]) / np.maximum(np.abs(ref[fin]), floor)
    assert err.size == 0 or err.max() <= rtol, (got, ref, err.max())


@pytest.mark.gpu
@pytest.mark.parametrize("scalar", ["host", "device"])
def test_cpp_inner_api_against_oracle(tmp_path, oracle_medium, scalar):
    """Every MultiRayAirIceRefraction.h function of the reference (.h:84-204) driven by a C++
    caller (tests/cpp/multiray_inner_driver.cpp): the ray layer -- on the host (the default for
    one-query calls) and on the GPU (AIRICE_SCALAR=device) -- within 1e-9 of the oracle, the table
    walks on the host bit for bit, the exported _Table (with its antenna remap) bit-identical to
    the batched GPU lookup."""
    r = _run_driver(INNER, tmp_path, scalar)
    m = oracle_medium
    ML = m.max_layers
    # namespace data
    assert r["MaxLayers"] == ML
    assert r["ATMLAY"] == list(m.atmlay) and r["B_air"] == list(m.B_air)
    assert r["C_air"] == list(m.C_air)
    assert r["h_layers"] == ML - 1 and r["h_points"] == m.n_points
    # the ray layer vs the oracle's MultiRay restatements (op codes as AIRICE_RTF_ / AIRICE_MR_)
    A_ice, B_ice, C_ice, A_air = 1.78, -0.43, 0.0132, 1.0
    lay = lambda z: min([i for i in range(ML) if abs(z) < m.atmlay[i + 1] / 100] + [ML - 1])  # noqa
    Ba, Ca = m.B_air[lay(5000)], m.C_air[lay(5000)]
    _close(r["f_ice"], [oracle.rtf_eval(m, 5, [-150, A_ice, B_ice, -C_ice, 1.5])[0],
                        oracle.rtf_eval(m, 6, [-150, A_ice, B_ice, -C_ice, 299792458.0, 1.5, 0])[0],
                        oracle.rtf_eval(m, 9, [-150, A_ice, B_ice, -C_ice, 299792458.0, 1.5])[0]])
    _close(r["f_air"], [oracle.rtf_eval(m, 5, [5000, A_air, Ba, -Ca, 0.8])[0],
                        oracle.rtf_eval(m, 6, [5000, A_air, Ba, -Ca, 299792458.0, 0.8, 1])[0],
                        oracle.rtf_eval(m, 9, [5000, A_air, Ba, -Ca, 299792458.0, 0.8])[0]])
    _close(r["paths"], [oracle.rtf_eval(m, 1, [A_air, 3000, 9000, 0.7, 1])[0],
                        oracle.rtf_eval(m, 2, [A_air, 3000, 9000, 0.7, 1])[0],
                        oracle.rtf_eval(m, 10, [A_air, 3000, 9000, 0.7, 1])[0],
                        oracle.rtf_eval(m, 1, [A_ice, -200, 0, 1.2, 0])[0],
                        oracle.rtf_eval(m, 2, [A_ice, -200, 0, 1.2, 0])[0],
                        oracle.rtf_eval(m, 10, [A_ice, -200, 0, 1.2, 0])[0]])
    _close(r["hit_air"], oracle.rtf_eval(m, 11, [oracle.getnz_air(m, 9000), 3000, 9000, 35.0, 1]))
    _close(r["hit_ice"], oracle.rtf_eval(m, 11, [oracle.getnz_air(m, 3000), -200, 0, 35.0, 0]))
    for k, (la, txh) in enumerate(((160.0, 20000.0), (120.0, 90000.0), (95.0, 5000.0))):
        _close(r[f"air_prop{k}"], oracle.rtf_eval(m, 12, [la, txh, 3000]))
        assert r[f"air_prop{k}"][5 * ML + 1] >= 1
    _close(r["ice_prop"], oracle.rtf_eval(m, 13, [30.0, 3000, -200, 0.9]))
    _close(r["min_launch"], [oracle.rtf_eval(m, 14, [150.0 + 5 * k, 20000.0, 3000.0, -200.0,
                                                     1000.0 + 9000.0 * k])[0] for k in range(3)],
           floor=1e-6)
    # A_ice is read at every call
    m2 = oracle.load_atmosphere(ATMOSPHERE_GZ)
    m2.A_ice = 1.775
    _close(r["a_ice_1775"], [oracle.getnz_ice(m2, -100), oracle.rtf_eval(m2, 13,
                                                                          [30.0, 3000, -200, 0.9])[0]])
    # B_air is read at every call: the edited medium's solve, ray and n(z)
    m3 = oracle.load_atmosphere(ATMOSPHERE_GZ)
    m3.B_air[1] = m.B_air[1] * 1.001
    thR = 180 - (math.atan(1000.0 / 2200.0) * (180.0 / 3.1415927))
    ref_e, st_e = oracle.air2ice(m3, 5000.0, 1000.0, 3000.0, -200.0, thR)
    rep = parity.compare_columns(np.array(r["air2ice_b_air_edit"])[:, None], ref_e[:, None],
                                 parity.SOLVE_FLOORS)
    assert rep["ok"] and st_e == 0, rep
    ref_e0, _ = oracle.air2ice(m, 5000.0, 1000.0, 3000.0, -200.0, thR)
    assert abs(r["air2ice_b_air_edit"][2] - ref_e0[2]) > 1e-6  # the edit changed the ray
    rep = parity.compare_columns(np.array(r["ray_b_air_edit"])[:, None],
                                 oracle.ray_solution(m3, 170.0, 20000.0, 3000.0, -200.0,
                                                     True)[:, None], parity.RAY_FLOORS)
    assert rep["ok"], rep
    assert r["nz_b_air_edit"] == [oracle.getnz_air(m3, 5000.0), m3.B_air[1]]
    # MakeRayTracingTables (one launch for three antennas) == one MakeRayTracingTable each
    assert r["multi_tables_equal"] == [1, 1, 1]
    # table walks on table 0, bit for bit against the oracle's restatement on the same floats
    stop, step, hsteps, asteps = r["grid"]
    og = oracle.grid_init(-20000.0, 300000.0, 2000.0, 92.0, 180.0, 5.0)
    assert (stop, step, hsteps, asteps) == (og.stop_height, 2000.0, og.height_steps,
                                            og.angle_steps)
    t0 = np.ascontiguousarray(np.array(r["table0"], dtype=np.float32))
    lt = oracle.lookup_table(t0, og)
    heights = [99999.0, 51234.5, 23000.0, 3000.0, 4321.0, 8000.0]
    for k, h in enumerate(heights):
        (s1, e1, s2, e2), (c1, c2), _ = oracle.lookup_closest_txh(lt, h)
        assert r["closest_txh"][k] == [s1, e1, c1, s2, e2, c2], (h, r["closest_txh"][k])
        (rs, re_), c, _ = oracle.lookup_closest_thd(lt, 1500.0 * (k + 1), s1, e1)
        assert r["closest_thd"][k] == [rs, re_, c]
        h1, p1, h2, p2, _ = oracle.lookup_par_values(lt, h, 1500.0 * (k + 1))
        got = np.array(r["par_values"][k])
        ref = np.concatenate([[h1], p1, [h2], p2])
        assert np.array_equal(got, ref, equal_nan=True), (h, got, ref)
    assert r["MaxMinAirTxHeight"] == [float(t0[0, 0]), float(t0[0, -1])]
    # Extrapolate / FindExtrapolationLimit (.cc:997-1031) on the table floats
    def extrap(tab, par, i, x):
        x1, x2, y1, y2 = (float(tab[1][i]), float(tab[1][i + 1]), float(tab[par][i]),
                          float(tab[par][i + 1]))
        mm = (y2 - y1) / (x2 - x1)
        return mm * x + (y1 - mm * x1)

    def limit(tab, i):
        x1, x2, y1, y2 = float(tab[1][i]), float(tab[1][i + 1]), float(tab[4][i]), float(tab[4][i + 1])
        mm = (y1 - y2) / (x1 - x2)
        return (90 - (y1 - mm * x1)) / mm
    t1 = [[np.float32(a), np.float32(b)] for a, b in r["table1_col"]]
    t1p = [np.zeros(43, dtype=np.float32) for _ in range(11)]
    for c in range(11):
        t1p[c][41], t1p[c][42] = t1[c]
    ex = [extrap(t0, 2, 40, 12000.0), extrap(t1p, 7, 41, 3000.0), limit(t0, 40), limit(t1p, 41)]
    assert np.array_equal(np.array(r["extrapolate"]), np.array(ex), equal_nan=True)
    # _Table (host, remapped antenna) vs the batched GPU lookup: same bits, and a fallback row ran
    rows = r["table_scalar_vs_batch"]
    assert all(row[3] == 1 for row in rows), [row for row in rows if row[3] != 1]
    assert sum(row[2] for row in rows) >= 10
