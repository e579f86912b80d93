"""The pythonwrapper library's C++ surface (include/AirIceRayTracing.h: the AirIceRayTracing::
namespace of pythonwrapper/AirIceRayTracing.h:23-146 and the C++ TraceIceToAir of
TraceIceToAir.C:5-73) driven by a C++ caller (tests/cpp/pywrapper_driver.cpp) on the GPU, checked
against the oracle's pythonwrapper restatement (or_py_air2ice / or_py_trace_ice_to_air, pi =
4*atan(1)) within the 1e-9 parity rule."""
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

DRIVER = os.path.join(ROOT, "tests", "cpp", "pywrapper_driver")


def _queries():
    """cfg5-distributed queries (seed 777) plus the geometries the entry points branch on:
    Rx in the air above the ice (depth >= 0, .cc:937-941), short distances (CheckSolution's
    D <= 100 branch, .cc:916), D = 0, a Tx just above the ice."""
    d, ice, txh, dist = parity.cfg5_queries(40)
    extra = np.array([[10.0, 3000.0, 9000.0, 4000.0], [0.0, 3000.0, 15000.0, 12000.0],
                      [-50.0, 3000.0, 8000.0, 60.0], [-200.0, 3000.0, 20000.0, 0.0],
                      [-5.0, 3000.0, 3001.0, 30.0], [-300.0, 3000.0, 19999.0, 29999.0]])
    q = np.concatenate([np.stack([d, ice, txh, dist], axis=1), extra])
    return q


def _run(tmp_path, q, scalar="host"):
    """scalar: where the one-query calls run (AIRICE_SCALAR: the host by default, or the GPU)."""
    assert os.path.exists(DRIVER), "build with __graft_entry__.build()"
    with open(ATMOSPHERE_GZ, "rb") as f:
        (tmp_path / "Atmosphere.dat").write_bytes(gzip.decompress(f.read()))
    qf = tmp_path / "queries.txt"
    qf.write_text("".join("%.17g %.17g %.17g %.17g\n" % tuple(r) for r in q))
    out = subprocess.run([DRIVER, str(qf)], cwd=tmp_path, capture_output=True, text=True,
                         timeout=120, env=dict(os.environ, AIRICE_SCALAR=scalar))
    assert out.returncode == 0, out.stderr
    txt = re.sub(r"-?\b(nan|inf)\b", lambda mm: {"nan": "NaN", "-nan": "NaN", "inf": "Infinity",
                                                   "-inf": "-Infinity"}[mm.group(0)], out.stdout)
    return json.loads(txt)


def _check_solves(rows, q, m, mask_unpinned=True, m_trace=None):
    """rows: [ok, GetRayTracingSolution x8, Air2IceRayTracing dummy[0..14], TraceIceToAir x10];
    m_trace: the medium TraceIceToAir sees (it re-reads the file first, TraceIceToAir.C:25)."""
    m_trace = m if m_trace is None else m_trace
    rows = np.array(rows, dtype=np.float64)
    n = len(q)
    assert rows.shape == (n, 1 + 8 + 15 + 10)
    py = np.zeros((15, n))
    tr = np.zeros((10, n))
    oks, sts = np.zeros(n, dtype=bool), np.zeros(n, dtype=np.int64)
    for i, (dep, ice, txh, dist) in enumerate(q):
        thR = oracle.straight_angle_of(m, txh, dist, ice, dep)
        py[:, i], sts[i] = oracle.py_air2ice(m, txh, dist, ice, dep, thR)
        ok_i, tr[:, i] = oracle.py_trace_ice_to_air(m_trace, dep, ice, txh, dist)
        oks[i] = bool(ok_i)
    ok_sol = np.array([bool(oracle.py_trace_ice_to_air(m, dep, ice, txh, dist)[0])
                       for (dep, ice, txh, dist) in q])
    mask = (sts & oracle.SOLVE_UNPINNED) == 0 if mask_unpinned else np.ones(n, dtype=bool)
    # Air2IceRayTracing: the whole 15-slot layout
    rep = parity.compare_columns(rows[:, 9:24].T, py, parity.PYSOLVE_FLOORS, mask=mask)
    assert rep["ok"], rep
    # GetRayTracingSolution: its eight outputs are slots 5, 6, 14, 13, 10, 2, 11, 12 (.cc:902-910)
    sel = [5, 6, 14, 13, 10, 2, 11, 12]
    rep = parity.compare_columns(rows[:, 1:9].T, py[sel], parity.PYSOLVE_FLOORS[sel], mask=mask)
    assert rep["ok"], rep
    assert np.array_equal(rows[mask, 0].astype(bool), ok_sol[mask])
    # TraceIceToAir: ArrayParameters[10]
    rep = parity.compare_columns(rows[:, 24:34].T, tr, parity.TRACE_FLOORS, mask=mask)
    assert rep["ok"], rep
    return int(mask.sum()), int(oks[mask].sum())


@pytest.mark.gpu
@pytest.mark.parametrize("scalar", ["host", "device"])
def test_pywrapper_cpp_caller_against_oracle(tmp_path, oracle_medium_py, scalar):
    q = _queries()
    r = _run(tmp_path, q, scalar)
    m = oracle_medium_py
    ML = m.max_layers
    # namespace data filled by MakeAtmosphere("Atmosphere.dat")
    assert r["MaxLayers"] == ML and r["ATMLAY"] == list(m.atmlay)
    assert r["B_air"] == list(m.B_air) and r["C_air"] == list(m.C_air)
    assert r["h_layers"] == ML - 1 and r["h_points"] == m.n_points
    lay = lambda z: min([i for i in range(ML) if abs(z) < m.atmlay[i + 1] / 100] + [ML - 1])  # noqa
    np.testing.assert_array_equal(r["nz"], [oracle.getnz_air(m, 3000), oracle.getnz_air(m, 50000),
                                            oracle.getnz_ice(m, -200), m.B_air[lay(12000)],
                                            m.C_air[lay(12000)], oracle.getnz_air(m, -7000)])
    n1, n2 = oracle.getnz_air(m, 3000.0), oracle.getnz_ice(m, 0.0)
    sq = math.sqrt(1 - ((n1 / n2) * math.sin(0.3)) ** 2)
    num, den = n1 * math.cos(0.3) - n2 * sq, n1 * math.cos(0.3) + n2 * sq
    nump, denp = n1 * sq - n2 * math.cos(0.3), n1 * sq + n2 * math.cos(0.3)
    np.testing.assert_allclose(r["fresnel"], [num / den, 1 + num / den, -nump / denp,
                                              (1 - nump / denp) * (n1 / n2)], rtol=1e-14)
    # the ray layer: the MultiRay forms with the pythonwrapper's pi (AirIceRayTracing.cc:356-857)
    A_ice, B_ice, C_ice, A_air = 1.78, -0.43, 0.0132, 1.0
    Ba, Ca = m.B_air[lay(5000)], m.C_air[lay(5000)]
    close = lambda got, ref, floor=1e-12: _close(got, ref, floor)  # noqa
    close(r["f_ice"], [oracle.rtf_eval(m, 5, [-150, A_ice, B_ice, -C_ice, 1.5])[0],
                       oracle.rtf_eval(m, 6, [-150, A_ice, B_ice, -C_ice, 299792458.0, 1.5, 0])[0],
                       oracle.rtf_eval(m, 9, [-150, A_ice, B_ice, -C_ice, 299792458.0, 1.5])[0]])
    close(r["f_air"], [oracle.rtf_eval(m, 5, [5000, A_air, Ba, -Ca, 0.8])[0],
                       oracle.rtf_eval(m, 6, [5000, A_air, Ba, -Ca, 299792458.0, 0.8, 1])[0],
                       oracle.rtf_eval(m, 9, [5000, A_air, Ba, -Ca, 299792458.0, 0.8])[0]])
    close(r["paths"], [oracle.rtf_eval(m, op, [A, rx, tx, L, air])[0]
                       for (A, rx, tx, L, air) in ((A_air, 3000, 9000, 0.7, 1),
                                                   (A_ice, -200, 0, 1.2, 0))
                       for op in (1, 2, 10)])
    close(r["hit_air"], oracle.rtf_eval(m, 11, [oracle.getnz_air(m, 9000), 3000, 9000, 35.0, 1]))
    close(r["air_prop"], oracle.rtf_eval(m, 12, [160.0, 20000.0, 3000.0]))
    close(r["ice_prop"], oracle.rtf_eval(m, 13, [30.0, 3000, 200, 0.9]))
    close(r["min_launch"], [oracle.rtf_eval(m, 14, [150.0 + 5 * k, 20000.0, 3000.0, 200.0,
                                                    1000.0 + 9000.0 * k])[0] for k in range(3)],
          floor=1e-6)
    # the three solve entry points on every query
    n_pinned, n_ok = _check_solves(r["solves"], q, m)
    assert n_pinned >= len(q) - 3 and n_ok >= len(q) // 2
    # FindFunctionRoot(MinimizeforLaunchAngle, bisection / brent): the reference's own search
    # driven from the host over GPU evaluations lands on the launch angle Air2IceRayTracing returns
    rows = np.array(r["solves"])
    for i, (lo, thR, r_bis, r_brent) in enumerate(r["find_root"]):
        dep, ice, txh, dist = q[i]
        assert thR == oracle.straight_angle_of(m, txh, dist, ice, dep)
        ref, st = oracle.py_air2ice(m, txh, dist, ice, dep, thR)
        if st & oracle.SOLVE_UNPINNED or lo != thR - 16:
            continue
        assert abs(r_bis - ref[10]) <= 1e-9 * abs(ref[10]), (i, r_bis, ref[10])
        assert abs(rows[i, 9 + 10] - ref[10]) <= 1e-9 * abs(ref[10])
        fb = oracle.rtf_eval(m, 14, [r_brent, txh, ice, -dep, dist])[0]
        assert abs(fb) < 1e-3, (i, r_brent, fb)  # Brent converged on a root of the same f
    # a B_air edit after MakeAtmosphere is read by the next calls
    m_edit = oracle.parse_atmosphere(gzip.decompress(open(ATMOSPHERE_GZ, "rb").read()),
                                     oracle.PI_EXACT)
    m_edit.B_air[1] = m.B_air[1] * 1.001
    _check_solves(r["solves_b_air_edit"], q[:3], m_edit, m_trace=m)
    # constant refractive index (TraceIceToAir.C:27-29): GetB_air = 0, GetC_air = 1e-9,
    # Getnz_air = A_const, bracket [90, thR] (AirIceRayTracing.cc:173-239, 955-982).  Every such
    # solve starts on a non-finite f(90) (the GSL-UB case), so the rows are unpinned against the
    # reference; GPU and oracle model the same zero state and must agree.
    c = oracle.getnz_air(m, 3000.0)
    assert r["const_nz"] == [c, 0.0, 1e-9, c]
    m_c = oracle.parse_atmosphere(gzip.decompress(open(ATMOSPHERE_GZ, "rb").read()),
                                  oracle.PI_EXACT)
    m_c.constant_air_index, m_c.A_const, m_c.A_air = 1, c, c
    _check_solves(r["solves_const"], q[:3], m_c, mask_unpinned=False)
    # and the namespace is back to the file's after MakeAtmosphere
    assert r["restored"] == [m.B_air[1], oracle.getnz_air(m, 3000.0)]


def _close(got, ref, floor=1e-12, rtol=1e-9):
    got, ref = np.asarray(got, dtype=np.float64), np.asarray(ref, dtype=np.float64)
    assert got.shape == ref.shape
    assert np.array_equal(np.isnan(got), np.isnan(ref))
    fin = ~np.isnan(ref)
    err = np.abs(got[fin] - ref[fin]) / np.maximum(np.abs(ref[fin]), floor)
    assert err.size == 0 or err.max() <= rtol, (got, ref, err.max())
