"""pythonwrapper drop-in (airiceraytracing_amd/pythonwrapper/AirIceRayTracing.py) -- the module a
script written for the reference's pythonwrapper/AirIceRayTracing.py (:1-11) imports.

CPU: the module loads libairice.so and declares the reference's argtypes (no compute call).
GPU: a TraceIceToAir.py-style script (``from AirIceRayTracing import *``, the reference's
usage pattern, written here from scratch) run in a fresh process reproduces the SURVEY.md §4
Py_TraceIceToAir KAT; the batch form matches the oracle and the scalar symbol row for row.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

from tests.conftest import ROOT

WRAPPER_DIR = os.path.join(ROOT, "airiceraytracing_amd", "pythonwrapper")
KAT = [8050, 10000, 13.134949577955233, 11195.189413293168, 39.505164153620896,
       63.19239972035086, 9991.484652020625, 41.39177304098942, 0, 0]

SCRIPT = """
import sys
sys.path.insert(0, {wrapper!r})
from AirIceRayTracing import *
arr = (ctypes.c_double * 10)(*([1.0] * 10))
Py_TraceIceToAir(-10, 3000, 8050, 10000, arr)
for x in arr:
    print(repr(x))
"""


def test_module_surface_cpu():
    code = ("import sys, ctypes; sys.path.insert(0, %r)\n"
            "import AirIceRayTracing as m\n"
            "at = m.handle.Py_TraceIceToAir.argtypes\n"
            "assert at[:4] == [ctypes.c_double] * 4, at\n"
            "assert at[4]._type_ is ctypes.c_double and at[4]._length_ == 10\n"
            "assert callable(m.Py_TraceIceToAir) and callable(m.Py_TraceIceToAir_batch)\n"
            "print('ok')\n") % WRAPPER_DIR
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr


@pytest.mark.gpu
def test_trace_script_kat(tmp_path, atmosphere_text):
    (tmp_path / "Atmosphere.dat").write_bytes(atmosphere_text)
    (tmp_path / "trace.py").write_text(SCRIPT.format(wrapper=WRAPPER_DIR))
    r = subprocess.run([sys.executable, "trace.py"], cwd=tmp_path, capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    vals = [float(v) for v in r.stdout.split()[-10:]]
    np.testing.assert_allclose(vals, KAT, rtol=1e-9, atol=1e-12)


@pytest.mark.gpu
def test_batch_matches_oracle_and_scalar(tmp_path, monkeypatch, atmosphere_text,
                                         oracle_medium_py):
    import oracle
    from tests import parity
    sys.path.insert(0, WRAPPER_DIR)
    try:
        import AirIceRayTracing as m
    finally:
        sys.path.remove(WRAPPER_DIR)
    (tmp_path / "Atmosphere.dat").write_bytes(atmosphere_text)
    monkeypatch.chdir(tmp_path)
    depth, ice, txh, dist = parity.cfg5_queries(4096, seed=99)
    out = m.Py_TraceIceToAir_batch(depth, ice, txh, dist)
    assert out.shape == (4096, 10)
    ref = oracle.py_trace_batch(oracle_medium_py, depth, ice, txh, dist, nthreads=8)
    assert np.array_equal(out[:, 0] == -1000, ref[:, 0] == -1000)
    rep = parity.compare_columns(out.T, ref.T, parity.TRACE_FLOORS)
    assert rep["ok"], rep
    # one query per call: on the host by default (the same source, the host's sqrt and quotients:
    # within an ulp or so of the batch), and bit for bit the batch on the GPU's one-wave kernel
    from airiceraytracing_amd import _lib
    from airiceraytracing_amd.solver import scalar_mode
    for i in (0, 17, 4095):
        arr = (ctypes.c_double * 10)()
        m.Py_TraceIceToAir(depth[i], ice[i], txh[i], dist[i], arr)
        np.testing.assert_allclose(np.array(list(arr)), out[i], rtol=1e-12, atol=1e-12)
        with scalar_mode(_lib.SCALAR_DEVICE):
            m.Py_TraceIceToAir(depth[i], ice[i], txh[i], dist[i], arr)
        assert np.array_equal(np.array(list(arr)), out[i])
