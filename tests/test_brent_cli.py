"""The Air2IceRayTracing CLI path (reference Air2IceRayTracing.C): GSL-Brent launch-angle search
under RayTracingFunctions::FindFunctionRoot (RayTracingFunctions.cc:256-290, max_iter 20).

GNU GSL is absent from this image and the reference ships no output for this CLI, so the Brent
restatement (oracle or_brent, GSL 2.x roots/brent.c) is **parity unpinned** against the reference
itself.  It is checked here against the algorithm's defining properties and against scipy's
independent brentq, and the whole CLI solve against the pinned MultiRay known answer of the same
geometry (Air2IceRayTracing(5000, 1000, 3000, -200) -> launch 154.70167146999108,
THD 1000.0000012374369, found there by GSL bisection).  GPU: the device restatement
(AIRICE_RTF_AIR2ICE) against the oracle, and the CLI's stdout.
"""
import math
import os
import subprocess

import numpy as np
import pytest

import oracle
from tests.conftest import ROOT

CLI = os.path.join(ROOT, "airiceraytracing_amd", "bin", "Air2IceRayTracing")


def test_brent_converges_like_brentq():
    from scipy.optimize import brentq
    for f, lo, hi in ((lambda x: x ** 3 - 2.0, 0.0, 2.0), (lambda x: math.cos(x) - x, 0.0, 1.0),
                      (lambda x: 150.0 - x, 140.0, 160.0), (lambda x: math.exp(x) - 10, 1, 5)):
        r, st, calls, it = oracle.brent(f, lo, hi, tol=1e-9)
        ref = brentq(f, lo, hi, xtol=1e-15, rtol=1e-15)
        assert st == 0 and it <= 20
        assert abs(r - ref) <= 1e-9 * abs(ref) + 1e-15, (r, ref)
        assert calls[:2] == [lo, hi]  # brent_init: f(lower) then f(upper)


def test_brent_linear_function_one_step():
    # inverse interpolation is exact on a line: the first iterate lands on the root (f == 0), the
    # next iterate reports root = lo = hi = b, and the interval test converges
    r, st, calls, it = oracle.brent(lambda x: 150.0 - x, 140.0, 160.0)
    assert r == 150.0 and st == 0 and len(calls) == 3


def test_brent_nonfinite_end_zero_state():
    # f(lower) non-finite: brent_init returns before storing the state (reference: uninitialised
    # memory); modelled as a zero state -> the first iterate returns root b = 0
    r, st, calls, it = oracle.brent(lambda x: float("nan") if x < 1 else x - 2, 0.0, 3.0)
    assert st & oracle.SOLVE_NONFINITE_END and r == 0.0 and len(calls) == 1


def test_brent_bad_bracket_and_max_iter():
    r, st, calls, it = oracle.brent(lambda x: x, 2.0, 1.0)
    assert st & oracle.SOLVE_BAD_BRACKET and r == 0.0 and calls == []
    # a same-sign bracket never passes the interval test before max_iter
    r, st, calls, it = oracle.brent(lambda x: x * x + 1.0, -1.0, 2.0, max_iter=20)
    assert it == 20 and st & oracle.SOLVE_MAXITER


def test_cli_solve_matches_pinned_multiray_answer(oracle_medium):
    r = oracle.rtf_eval(oracle_medium, oracle.RTF_AIR2ICE, (5000.0, 1000.0, 3000.0, 200.0))
    assert r[12] == 0  # status
    assert abs(r[2] - 154.70167146999108) < 1e-9 * 154.7 * 2  # both at tolerance 1e-9 relative
    assert abs(r[10] - 1000.0) < 1e-5
    # the air / ice split at the root agrees with the MultiRay KAT to the root's precision
    assert abs(r[3] - 945.29336825318615) < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("where", ["host", "device"])
def test_air2ice_matches_oracle(oracle_medium, where):
    """AIRICE_RTF_AIR2ICE (the Brent search of Air2IceRayTracing.C:137 over
    RayTracingFunctions::FindFunctionRoot, .cc:256-290) on the calling thread (AIRICE_SCALAR_HOST)
    and on the GPU (AIRICE_SCALAR_DEVICE: rtf_kernel, whose launches are counted so the device
    case cannot silently run on the host) against the oracle: <= 1e-9 relative, status bits
    and probe steps equal."""
    from airiceraytracing_amd import AirIceSolver, _lib
    from airiceraytracing_amd.solver import scalar_mode
    s = AirIceSolver()
    rng = np.random.default_rng(31)
    worst = 0.0
    n_cmp = 0
    n_calls = 0
    mode = scalar_mode(_lib.SCALAR_HOST if where == "host" else _lib.SCALAR_DEVICE)
    with mode, _lib.launched("rtf_kernel") as k:
        for _ in range(150):
            args = (rng.uniform(3100, 99000), rng.uniform(0, 40000), 3000.0, rng.uniform(1, 300))
            g = s.rtf_eval(oracle.RTF_AIR2ICE, args)
            n_calls += 1
            r = oracle.rtf_eval(oracle_medium, oracle.RTF_AIR2ICE, args)
            _check_air2ice(g, r, args)
            if int(r[12]) & (oracle.SOLVE_NONFINITE_END | oracle.SOLVE_BAD_BRACKET):
                continue
            n_cmp += 1
            fin = np.isfinite(r[:12]) & (np.abs(r[:12]) > 1e-6)
            if fin.any():
                worst = max(worst, float(np.max(np.abs(g[:12][fin] - r[:12][fin]) /
                                                np.abs(r[:12][fin]))))
    assert k.count == (n_calls if where == "device" else 0), (where, k.count, n_calls)
    assert n_cmp > 100
    print(f"[air2ice {where}] {n_cmp} solves, max rel {worst:.2e}")


def _check_air2ice(g, r, args):
    """One solve: status bits, probe steps and filled layers equal, then <= 1e-9 relative
    unless the row is reference UB."""
    assert g[12] == r[12] and g[14] == r[14] and g[15] == r[15], (args, g[12:], r[12:])
    if int(r[12]) & (oracle.SOLVE_NONFINITE_END | oracle.SOLVE_BAD_BRACKET):
        return  # reference UB (uninitialised GSL state): status only
    for i in range(12):
        if np.isnan(r[i]):
            assert np.isnan(g[i])
            continue
        rel = abs(g[i] - r[i]) / max(abs(r[i]), 1e-6)
        assert rel <= 1e-9, (args, i, g[i], r[i])


def _cli_env(where):
    return dict(os.environ, AIRICE_SCALAR=where, AIRICE_LAUNCH_REPORT="1")


def _rtf_launches(stderr):
    """rtf_kernel launches the child process reported at exit (AIRICE_LAUNCH_REPORT)."""
    for line in stderr.splitlines():
        if line.startswith("airice launches:"):
            for tok in line.split()[2:]:
                k, v = tok.split("=")
                if k == "rtf_kernel":
                    return int(v)
    raise AssertionError(f"no launch report in stderr: {stderr!r}")


@pytest.mark.gpu
@pytest.mark.parametrize("where", ["host", "device"])
def test_cli_stdout(tmp_path, atmosphere_text, oracle_medium, where):
    """The Air2IceRayTracing CLI with its solve on the host (AIRICE_SCALAR=host, the default) and
    on the GPU (AIRICE_SCALAR=device: two rtf_kernel launches, the Brent search and the ice leg,
    read from the child's launch report)."""
    assert os.path.exists(CLI), "build with __graft_entry__.build()"
    (tmp_path / "Atmosphere.dat").write_bytes(atmosphere_text)
    p = subprocess.run([CLI, "5000", "1000", "3000", "200"], cwd=tmp_path, capture_output=True,
                       text=True, timeout=120, env=_cli_env(where))
    assert p.returncode == 0, p.stderr
    assert _rtf_launches(p.stderr) == (2 if where == "device" else 0), p.stderr
    vals = {}
    for line in p.stdout.splitlines():
        parts = line.split()
        if len(parts) >= 2 and parts[0] in ("TotalHorizontalDistanceinAir", "IncidentAngleonIce",
                                            "PropagationTimeAir", "TotalHorizontalDistanceinIce",
                                            "IncidentAngleonAntenna", "LvalueIce",
                                            "PropagationTimeIce", "TotalHorizontalDistance",
                                            "TotalPropagationTime"):
            vals[parts[0]] = float(parts[1])
        if line.startswith("Launch Angle search range is:"):
            vals["start"] = float(line.split("Startangle")[1].split(",")[0])
            vals["end"] = float(line.split("Endangle")[1])
    r = oracle.rtf_eval(oracle_medium, oracle.RTF_AIR2ICE, (5000.0, 1000.0, 3000.0, 200.0))
    want = {"start": r[0], "end": r[1], "TotalHorizontalDistanceinAir": r[3],
            "IncidentAngleonIce": r[4], "PropagationTimeAir": r[6],
            "TotalHorizontalDistanceinIce": r[7], "IncidentAngleonAntenna": r[8],
            "LvalueIce": r[5], "PropagationTimeIce": r[9], "TotalHorizontalDistance": r[10],
            "TotalPropagationTime": r[11]}
    for k, v in want.items():  # std::cout default precision: 6 significant digits
        assert float(f"{v:.6g}") == vals[k], (k, vals[k], v)
    # usage paths print and exit 0 without touching the GPU
    p = subprocess.run([CLI], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0 and "No Extra Command Line Argument" in p.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("where", ["host", "device"])
@pytest.mark.parametrize("tx,rx,dist", [(5000.0, 3100.0, 1000.0), (3100.0, 5000.0, 1000.0),
                                        (60000.0, 3000.0, 45000.0)])
def test_air_ray_cli_stdout(tmp_path, atmosphere_text, oracle_medium, tx, rx, dist, where):
    """AirRayTracing (AirRayTracing.C): the same search with the Rx in the air (no ice leg); a Tx
    below the Rx is swapped and its angles reported as 180 - angle."""
    exe = os.path.join(ROOT, "airiceraytracing_amd", "bin", "AirRayTracing")
    assert os.path.exists(exe), "build with __graft_entry__.build()"
    (tmp_path / "Atmosphere.dat").write_bytes(atmosphere_text)
    p = subprocess.run([exe, repr(tx), repr(rx), repr(dist)], cwd=tmp_path, capture_output=True,
                       text=True, timeout=120, env=_cli_env(where))
    assert p.returncode == 0, p.stderr
    assert (_rtf_launches(p.stderr) > 0) == (where == "device"), p.stderr
    got = {}
    for line in p.stdout.splitlines():
        parts = line.split()
        if line.startswith("Result from the minimization"):
            got["launch"] = float(parts[-2])
        elif line.startswith("startangle"):
            got["start"], got["end"] = float(parts[1]), float(parts[3])
        elif parts and parts[0] in ("TotalHorizontalDistanceinAir", "IncidentAngleonRx",
                                    "LvalueAir", "PropagationTimeAir"):
            got[parts[0]] = float(parts[1])
    hi, lo = max(tx, rx), min(tx, rx)
    r = oracle.rtf_eval(oracle_medium, oracle.RTF_AIR2ICE, (hi, dist, lo, 0.0))
    inc = 180 - r[4] if tx < rx else r[4]
    want = {"start": r[0], "end": r[1], "launch": r[2], "TotalHorizontalDistanceinAir": r[3],
            "IncidentAngleonRx": inc, "LvalueAir": r[5], "PropagationTimeAir": r[6]}
    for k, v in want.items():
        assert float(f"{v:.6g}") == got[k], (k, got[k], v)
    assert abs(r[3] - dist) < 1e-3  # the solve lands on the requested distance
