"""The RayTracingFunctions:: drop-in (include/RayTracingFunctions.h, RayTracingFunctions.cc of
the reference, the cfg1 CLI's library): exported symbols (CPU), a C++ caller
(tests/cpp/rtf_driver.cpp) and every scalar op on random arguments against the oracle (GPU).
Tolerance as everywhere: 1e-9 relative with the per-quantity floors, NaN positions equal."""
import gzip
import json
import os
import re
import subprocess

import numpy as np
import pytest

import oracle
from tests.conftest import ATMOSPHERE_GZ, ROOT

DRIVER = os.path.join(ROOT, "tests", "cpp", "rtf_driver")


def _close(got, ref, floor=1e-12, rtol=1e-9):
    got = np.asarray(got, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    assert got.shape == ref.shape
    nan = np.isnan(ref)
    assert np.array_equal(np.isnan(got), nan), (got, ref)
    err = np.abs(got[~nan] - ref[~nan])
    lim = rtol * np.maximum(np.abs(ref[~nan]), floor)
    assert np.all(err <= lim), (got, ref, err / np.maximum(np.abs(ref[~nan]), floor))


def test_rtf_symbols_exported():
    from airiceraytracing_amd import _lib
    nm = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                        text=True, check=True).stdout
    syms = set(ln.split()[-1] for ln in nm.splitlines())
    for s in ("_ZN19RayTracingFunctions14MakeAtmosphereEv",
              "_ZN19RayTracingFunctions9Getnz_airEd",
              "_ZN19RayTracingFunctions19GetLayerHitPointParEddddi",
              "_ZN19RayTracingFunctions20GetAirPropagationParEddd",
              "_ZN19RayTracingFunctions20GetIcePropagationParEdddd",
              "_ZN19RayTracingFunctions22MinimizeforLaunchAngleEdPv",
              "_ZN19RayTracingFunctions5fDnfREdPv", "_ZN19RayTracingFunctions6ftimeDEdPv",
              "_ZN19RayTracingFunctions6ATMLAYE", "_ZN19RayTracingFunctions9MaxLayersE",
              "_ZN19RayTracingFunctions6h_dataE"):
        assert s in syms, s


def _medium():
    with open(ATMOSPHERE_GZ, "rb") as f:
        return oracle.parse_atmosphere(gzip.decompress(f.read()), oracle.PI_MULTIRAY)


@pytest.mark.gpu
@pytest.mark.parametrize("scalar", ["host", "device"])
def test_rtf_cpp_caller(tmp_path, scalar):
    """The C++ caller with the one-query calls on the host (default) and on the GPU."""
    assert os.path.exists(DRIVER), "build with __graft_entry__.build()"
    with open(ATMOSPHERE_GZ, "rb") as f:
        (tmp_path / "Atmosphere.dat").write_bytes(gzip.decompress(f.read()))
    out = subprocess.run([DRIVER], cwd=tmp_path, capture_output=True, text=True, timeout=120,
                         env=dict(os.environ, AIRICE_SCALAR=scalar))
    assert out.returncode == 0, out.stderr
    txt = re.sub(r"-?\bnan\b", "NaN", out.stdout)
    r = json.loads(txt)
    m = _medium()
    assert r["max_layers"] == m.max_layers
    assert r["atmlay"] == list(m.atmlay)
    assert r["b_air"] == list(m.B_air) and r["c_air"] == list(m.C_air)
    assert r["h_data_sizes"] == list(m.layer_sizes)[:m.max_layers - 1]
    assert r["h_top"] == m.h_top
    assert r["nh_flat"] == m.n_points
    _close(r["nz"], [oracle.getnz_air(m, 0.0), oracle.getnz_air(m, 5000.0),
                     oracle.getnz_air(m, 30000.0), oracle.getnz_ice(m, -100.0)])
    _close(r["hit_air"], oracle.rtf_eval(m, 0, [oracle.getnz_air(m, 20000.0), 8363.53902,
                                                20000.0, 10.0, 1]))
    _close(r["hit_ice"], oracle.rtf_eval(m, 0, [1.0003, -200.0, 0.0, 9.9979, 0]))
    air = oracle.rtf_eval(m, 3, [170.0, 20000.0, 3000.0])
    _close(r["air_prop"], air)
    # KAT: THD in air of the cfg1 ray prints as 2997.35
    assert f"{air[0] + air[4] + air[8]:g}" == "2997.35"
    _close(r["ice_prop"], oracle.rtf_eval(m, 4, [9.9979, 3000.0, 200.0, 0.17365]))
    b5000, c5000 = m.B_air[1], m.C_air[1]
    ref = [oracle.rtf_eval(m, 7, [170.0, 20000.0, 3000.0, 200.0, 3000.0])[0],
           oracle.rtf_eval(m, 5, [5000.0, 1.0, b5000, -c5000, 0.5])[0],
           oracle.rtf_eval(m, 6, [100.0, 1.78, -0.43, -0.0132, 299792458.0, 0.6, 0])[0],
           oracle.rtf_eval(m, 1, [1.0, 3000.0, 8000.0, 0.4, 1])[0],
           oracle.rtf_eval(m, 2, [1.78, 150.0, 0.0, 0.9, 0])[0]]
    _close(r["scalars"], ref, floor=1e-15)
    m2 = _medium()
    m2.C_air[1] = m.C_air[1] * 1.002
    air2 = oracle.rtf_eval(m2, 3, [170.0, 20000.0, 3000.0])
    _close(r["c_air_edit"], [air2[0] + air2[4] + air2[8], oracle.getnz_air(m2, 5000.0),
                             m2.C_air[1]])
    assert abs(r["c_air_edit"][0] - (air[0] + air[4] + air[8])) > 1e-6


def _rtf_cases(m, n=150, seed=3):
    from airiceraytracing_amd import _lib
    rng = np.random.default_rng(seed)
    cases = []
    for _ in range(n):
        txh = rng.uniform(3001, 99000)
        ice = rng.choice([3000.0, rng.uniform(0, 3500)])
        la = rng.uniform(91, 180)
        air = int(rng.integers(0, 2))
        if air:
            tx, rx = rng.uniform(0, 60000), rng.uniform(0, 60000)
            n1 = oracle.getnz_air(m, tx) * rng.uniform(0.9999, 1.0001)
        else:
            tx, rx = -rng.uniform(0, 300), -rng.uniform(0, 300)
            n1 = rng.uniform(1.0, 1.78)
        L = rng.uniform(0, 1.0)
        cases += [
            (_lib.RTF_HIT_POINT, [n1, rx, tx, rng.uniform(0, 89.9), air]),
            (_lib.RTF_AIR_PROPAGATION, [la, txh, ice]),
            (_lib.RTF_MIN_LAUNCH, [la, txh, ice, rng.uniform(0, 300), rng.uniform(0, 50000)]),
            (_lib.MR_AIR_PROPAGATION, [la, txh, ice]),
            (_lib.MR_MIN_LAUNCH, [la, txh, ice, rng.uniform(0, 300), rng.uniform(0, 50000)]),
        ]
    return cases


@pytest.mark.gpu
def test_host_matches_device(oracle_medium):
    """The one-query ray layer on the host (the default) against the same op on the GPU: the same
    expressions with the host's libm in place of ocml, so within a few ulps of each other."""
    from airiceraytracing_amd import AirIceSolver, _lib
    from airiceraytracing_amd.solver import scalar_mode
    s = AirIceSolver()
    worst = 0.0
    cases = _rtf_cases(oracle_medium, 60, seed=8)
    with _lib.launched("rtf_kernel") as k:
        for op, args in cases:
            with scalar_mode(_lib.SCALAR_HOST):
                host = s.rtf_eval(op, args)
            with scalar_mode(_lib.SCALAR_DEVICE):
                dev = s.rtf_eval(op, args)
            _close(host, dev, floor=1e-6, rtol=1e-12)
            fin = np.isfinite(dev) & (np.abs(dev) > 1e-6)
            if fin.any():
                worst = max(worst, float(np.max(np.abs(host[fin] - dev[fin]) / np.abs(dev[fin]))))
    assert k.count == len(cases)  # one rtf_kernel per device call, none for the host calls
    assert worst < 1e-12, worst


@pytest.mark.gpu
def test_air2ice_host_matches_device(oracle_medium):
    """AIRICE_RTF_AIR2ICE (the Air2IceRayTracing CLI's GSL-Brent search, Air2IceRayTracing.C:137)
    on the host and on the GPU: the same status bits, probe steps and filled layers; the roots
    within the 1e-9 contract of each other (a last-ulp difference in f can move one Brent step),
    and both within 1e-9 of the oracle.  Rx in the ice and in the air (AirRayTracing.C)."""
    from airiceraytracing_amd import AirIceSolver, _lib
    from airiceraytracing_amd.solver import scalar_mode
    s = AirIceSolver()
    rng = np.random.default_rng(44)
    same_bits = 0
    n = 0
    with _lib.launched("rtf_kernel") as k:
        for _ in range(80):
            if rng.uniform() < 0.75:
                args = [rng.uniform(3100, 99000), rng.uniform(0, 40000), rng.choice([3000.0, 0.0]),
                        rng.uniform(1, 300)]
            else:
                args = [rng.uniform(3100, 60000), rng.uniform(0, 45000), rng.uniform(0, 3000), 0.0]
            with scalar_mode(_lib.SCALAR_HOST):
                host = s.rtf_eval(_lib.RTF_AIR2ICE, args)
            with scalar_mode(_lib.SCALAR_DEVICE):
                dev = s.rtf_eval(_lib.RTF_AIR2ICE, args)
            n += 1
            ref = oracle.rtf_eval(oracle_medium, _lib.RTF_AIR2ICE, args)
            assert host[12] == dev[12] == ref[12], (args, host[12:], dev[12:], ref[12:])
            assert host[14] == dev[14] and host[15] == dev[15], (args, host[12:], dev[12:])
            same_bits += int(np.array_equal(host[:12].view(np.int64), dev[:12].view(np.int64)))
            if int(ref[12]) & (oracle.SOLVE_NONFINITE_END | oracle.SOLVE_BAD_BRACKET):
                continue  # reference UB: status only
            _close(dev[:12], ref[:12], floor=1e-6)
            _close(host[:12], ref[:12], floor=1e-6)
            _close(host[:12], dev[:12], floor=1e-6)
    assert k.count == n
    print(f"[air2ice host/device] {n} solves, {same_bits} bit-identical")


@pytest.mark.gpu
@pytest.mark.parametrize("scalar", ["host", "device"])
def test_rtf_ops_random(oracle_medium, scalar):
    from airiceraytracing_amd import AirIceSolver, _lib
    from airiceraytracing_amd.solver import scalar_mode
    s = AirIceSolver()
    mode = scalar_mode(_lib.SCALAR_HOST if scalar == "host" else _lib.SCALAR_DEVICE)
    mode.__enter__()
    m = oracle_medium
    rng = np.random.default_rng(3)
    n = 150
    cases = []
    for _ in range(n):
        txh = rng.uniform(3001, 99000)
        ice = rng.choice([3000.0, rng.uniform(0, 3500)])
        la = rng.uniform(91, 180)
        air = int(rng.integers(0, 2))
        if air:
            tx, rx = rng.uniform(0, 60000), rng.uniform(0, 60000)
            n1 = oracle.getnz_air(m, tx) * rng.uniform(0.9999, 1.0001)
        else:
            tx, rx = -rng.uniform(0, 300), -rng.uniform(0, 300)
            n1 = rng.uniform(1.0, 1.78)
        L = rng.uniform(0, 1.0)
        cases += [
            (_lib.RTF_HIT_POINT, [n1, rx, tx, rng.uniform(0, 89.9), air]),
            (_lib.RTF_OPTICAL_PATH, [1.0 if air else 1.78, rx, tx, L, air]),
            (_lib.RTF_PROPAGATION_TIME, [1.0 if air else 1.78, rx, tx, L, air]),
            (_lib.RTF_AIR_PROPAGATION, [la, txh, ice]),
            (_lib.RTF_ICE_PROPAGATION, [rng.uniform(0, 60), ice, rng.uniform(0, 300), L]),
            (_lib.RTF_FDNFR, [rng.uniform(-300, 60000), 1.0, rng.uniform(1e-4, 4e-4),
                              -rng.uniform(1e-4, 2e-4), L]),
            (_lib.RTF_FTIMED, [rng.uniform(-300, 60000), 1.0 if air else 1.78, 0.0,
                               -rng.uniform(1e-4, 0.02), 299792458.0, L, air]),
            (_lib.RTF_MIN_LAUNCH, [la, txh, ice, rng.uniform(0, 300), rng.uniform(0, 50000)]),
        ]
    try:
        for op, args in cases:
            got = s.rtf_eval(op, args)
            ref = oracle.rtf_eval(m, op, args)
            floor = 1e-15 if op in (_lib.RTF_PROPAGATION_TIME, _lib.RTF_FTIMED) else 1e-6
            _close(got, ref, floor=floor)
    finally:
        mode.__exit__()
