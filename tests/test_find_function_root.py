"""FindFunctionRoot of the three reference namespaces (MultiRayAirIceRefraction.cc:340-374,
RayTracingFunctions.cc:256-290, pythonwrapper/AirIceRayTracing.cc:315-353) through their mangled
C++ exports, on the CPU: the caller's host function is searched with GSL 2.x bisection / Brent
semantics (compat_roots.cpp).  Checked against the oracle's independent restatements of the same
GSL machines (or_bisect / or_brent): same root bits and the same sequence of evaluation points,
including the reference's undefined cases as both model them (non-finite bracket ends, a
non-finite midpoint, lower > upper, non-straddling brackets).  Parity vs real GSL is unpinned
(GSL is absent from the image)."""
import ctypes
import math

import pytest

import oracle
from airiceraytracing_amd import _lib

_FN = ctypes.CFUNCTYPE(ctypes.c_double, ctypes.c_double, ctypes.c_void_p)


class GslFunction(ctypes.Structure):  # struct gsl_function_struct (gsl/gsl_math.h)
    _fields_ = [("function", _FN), ("params", ctypes.c_void_p)]


SYMS = {
    "MultiRayAirIceRefraction": ("_ZN24MultiRayAirIceRefraction16FindFunctionRootE19gsl_function_"
                                 "structddPK21gsl_root_fsolver_typed", 40),
    "RayTracingFunctions": ("_ZN19RayTracingFunctions16FindFunctionRootE19gsl_function_structddPK"
                            "21gsl_root_fsolver_typed", 20),
    "AirIceRayTracing": ("_ZN16AirIceRayTracing16FindFunctionRootE19gsl_function_structddPK21gsl_"
                         "root_fsolver_typedi", None),
}


def _solver_types(L):
    return {name: ctypes.c_void_p.in_dll(L, f"airice_root_fsolver_{name}").value
            for name in ("bisection", "brent")}


def _find_root(ns, fn, lo, hi, solver, tol, iterations=None):
    L = ctypes.CDLL(_lib.LIB_PATH)
    sym, _ = SYMS[ns]
    f = getattr(L, sym)
    D = ctypes.c_double
    calls = []

    def cb(x, _p):
        calls.append(x)
        return float(fn(x))

    cfn = _FN(cb)
    F = GslFunction(cfn, None)
    args = [GslFunction, D, D, ctypes.c_void_p, D]
    vals = [F, lo, hi, _solver_types(L)[solver], tol]
    if iterations is not None:
        args.append(ctypes.c_int)
        vals.append(iterations)
    f.argtypes = args
    f.restype = D
    return f(*vals), calls


def _midgap(x):
    return float("nan") if 0.4 < x < 0.6 else x - 0.55


CASES = [
    (lambda x: x * x - 2.0, 0.0, 2.0, 1e-9),
    (lambda x: math.cos(x) - x, 0.0, 1.0, 1e-9),
    (lambda x: 100.0 - 10.0 * x, 5.0, 20.0, 1e-9),          # decreasing, like f(theta)
    (lambda x: math.exp(x) - 3.0, -10.0, 10.0, 1e-12),
    (lambda x: x * x + 1.0, 0.0, 1.0, 1e-9),                  # ends do not straddle 0
    (lambda x: math.sqrt(x - 0.5) - 0.3 if x >= 0.5 else float("nan"), 0.0, 1.0, 1e-9),  # f(lo) NaN
    (lambda x: 1.0 / (x - 1.0) if x != 1.0 else float("inf"), 0.0, 1.0, 1e-9),  # f(hi) inf
    (_midgap, 0.0, 1.0, 1e-9),                                # non-finite midpoint
    (lambda x: x, 0.0, 1.0, 1e-9),                            # f(lo) == 0
    (lambda x: x - 1.0, 0.0, 1.0, 1e-9),                      # f(hi) == 0
    (lambda x: x - 0.3, 1.0, 0.0, 1e-9),                      # lower > upper
    (lambda x: 150.0 - x, 90.001, 175.5, 1e-9),               # a launch-angle bracket
]


@pytest.mark.parametrize("ns", list(SYMS))
@pytest.mark.parametrize("case", range(len(CASES)))
def test_bisection_matches_oracle(ns, case):
    fn, lo, hi, tol = CASES[case]
    iters = SYMS[ns][1] or 40
    r, calls = _find_root(ns, fn, lo, hi, "bisection", tol,
                          None if SYMS[ns][1] else iters)
    r_ref, _, calls_ref = oracle.bisect(fn, lo, hi, tol, iters)
    assert calls == calls_ref
    assert r == r_ref or (math.isnan(r) and math.isnan(r_ref)), (r, r_ref)


@pytest.mark.parametrize("ns", list(SYMS))
@pytest.mark.parametrize("case", range(len(CASES)))
def test_brent_matches_oracle(ns, case):
    fn, lo, hi, tol = CASES[case]
    iters = SYMS[ns][1] or 13
    r, calls = _find_root(ns, fn, lo, hi, "brent", tol, None if SYMS[ns][1] else iters)
    r_ref, _, calls_ref, _ = oracle.brent(fn, lo, hi, tol, iters)
    assert calls == calls_ref
    assert r == r_ref or (math.isnan(r) and math.isnan(r_ref)), (r, r_ref)


def test_roots_converge_and_iteration_cap():
    r, _ = _find_root("AirIceRayTracing", lambda x: x * x - 2.0, 0.0, 2.0, "bisection", 1e-9, 40)
    assert abs(r - math.sqrt(2.0)) < 1e-8
    r, _ = _find_root("RayTracingFunctions", lambda x: x * x - 2.0, 0.0, 2.0, "brent", 1e-9)
    assert abs(r - math.sqrt(2.0)) < 1e-12
    # iterations bounds the driver loop: 3 bisection steps = 2 end + 3 midpoint evaluations
    _, calls = _find_root("AirIceRayTracing", lambda x: x - 0.7, 0.0, 1.0, "bisection", 1e-9, 3)
    assert len(calls) == 5
    # a negative tolerance ends the loop after one iterate (gsl_root_test_interval: GSL_EBADTOL)
    _, calls = _find_root("AirIceRayTracing", lambda x: x - 0.7, 0.0, 1.0, "bisection", -1.0, 40)
    assert len(calls) == 3


def test_solver_types_exported_with_gsl_names():
    L = ctypes.CDLL(_lib.LIB_PATH)
    t = _solver_types(L)

    class T(ctypes.Structure):  # gsl_root_fsolver_type's public layout: name first
        _fields_ = [("name", ctypes.c_char_p), ("size", ctypes.c_size_t)]

    for name, addr in t.items():
        assert T.from_address(addr).name == name.encode()
