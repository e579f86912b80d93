"""TEST INFRASTRUCTURE ONLY: ctypes binding of the CPU oracle (oracle/airice_oracle.c).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker / CPU baseline.  The product path
(``airiceraytracing_amd``) never imports it.

The oracle restates the reference hot path (MultiRayAirIceRefraction.cc and
pythonwrapper/AirIceRayTracing.cc); see airice_oracle.h for the per-function
citations and the parity-pinning status.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "liboracle_airice.so")

PI_MULTIRAY = 3.1415927             # MultiRayAirIceRefraction.h:29, RayTracingFunctions.h:26
PI_EXACT = 4.0 * np.arctan(1.0)     # pythonwrapper/AirIceRayTracing.h:25

TABLE_COLUMNS = (1, 2, 7, 6, 11, 3, 14, 15, 16, 17, 13)  # .cc:2101-2111 -> dummy index

SOLVE_NONFINITE_END = 1
SOLVE_BAD_BRACKET = 2
SOLVE_STALE_MID = 4
SOLVE_PROBED = 8
SOLVE_MAXITER = 16
SOLVE_NO_AIR_LAYER = 32
SOLVE_UNPINNED = SOLVE_NONFINITE_END | SOLVE_BAD_BRACKET | SOLVE_NO_AIR_LAYER
LOOKUP_FALLBACK = 1  # minimizer fallback ran (.cc:1418-1420)
LOOKUP_UNPINNED = 2  # the reference reads uninitialised / out-of-range memory


class Medium(ctypes.Structure):
    _fields_ = [
        ("atmlay", ctypes.c_double * 5),
        ("abc", (ctypes.c_double * 3) * 5),
        ("C_air", ctypes.c_double * 5),
        ("B_air", ctypes.c_double * 5),
        ("N0", ctypes.c_double),
        ("max_layers", ctypes.c_int),
        ("n_points", ctypes.c_int),
        ("layer_sizes", ctypes.c_int * 8),
        ("A_air", ctypes.c_double),
        ("A_ice", ctypes.c_double),
        ("B_ice", ctypes.c_double),
        ("C_ice", ctypes.c_double),
        ("pi", ctypes.c_double),
        ("h_top", ctypes.c_double),
        ("constant_air_index", ctypes.c_int),
        ("A_const", ctypes.c_double),
    ]


class Grid(ctypes.Structure):
    _fields_ = [
        ("start_height", ctypes.c_double),
        ("stop_height", ctypes.c_double),
        ("height_step", ctypes.c_double),
        ("height_steps", ctypes.c_int),
        ("start_angle", ctypes.c_double),
        ("stop_angle", ctypes.c_double),
        ("angle_step", ctypes.c_double),
        ("angle_steps", ctypes.c_int),
        ("depth_m", ctypes.c_double),
        ("ice_m", ctypes.c_double),
        ("in_ice", ctypes.c_int),
        ("table_rows", ctypes.c_int),
    ]

    @property
    def n_rays(self) -> int:
        return int(self.table_rows) * int(self.angle_steps)


def build() -> str:
    """Compile the oracle with its Makefile (gcc is in the image and on the GPU box)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


_lib = None
_FN = ctypes.CFUNCTYPE(ctypes.c_double, ctypes.c_double, ctypes.c_void_p)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        D, I, P = ctypes.c_double, ctypes.c_int, ctypes.c_void_p
        M = ctypes.POINTER(Medium)
        L.or_parse_atmosphere.argtypes = [ctypes.c_char_p, ctypes.c_size_t, D, M]
        L.or_load_atmosphere.argtypes = [ctypes.c_char_p, D, M]
        L.or_spline_eval_at.argtypes = [P, P, I, D]
        L.or_spline_eval_at.restype = D
        L.or_getnz_air.argtypes = [M, D]
        L.or_getnz_air.restype = D
        L.or_getnz_ice.argtypes = [M, D]
        L.or_getnz_ice.restype = D
        L.or_layer_hit_point_par.argtypes = [M, D, D, D, D, I, P]
        L.or_ray_solution.argtypes = [M, D, D, D, D, I, P]
        L.or_grid_init.argtypes = [ctypes.POINTER(Grid), D, D, D, D, D, D]
        L.or_table_rows.argtypes = [M, ctypes.POINTER(Grid), I, I, P, P, ctypes.c_size_t, I]
        L.or_air2ice.argtypes = [M, D, D, D, D, D, P]
        L.or_air2ice.restype = I
        L.or_bisect.argtypes = [_FN, P, D, D, D, I, ctypes.POINTER(I)]
        L.or_bisect.restype = D
        L.or_straight_angle.argtypes = [M, D, D, D, D]
        L.or_straight_angle.restype = D
        L.or_solve_batch.argtypes = [M, P, P, P, D, ctypes.c_size_t, P, ctypes.c_size_t, P, I]
        L.or_hdtip.argtypes = [M, D, D, D, D, P]
        L.or_hdtip.restype = I
        L.or_hdtip_batch.argtypes = [M, P, P, P, D, ctypes.c_size_t, P, ctypes.c_size_t, P, P, I]
        L.or_py_air2ice.argtypes = [M, D, D, D, D, D, P]
        L.or_py_air2ice.restype = I
        L.or_py_trace_ice_to_air.argtypes = [M, D, D, D, D, P]
        L.or_py_trace_ice_to_air.restype = I
        L.or_py_trace_batch.argtypes = [M, P, P, P, P, ctypes.c_size_t, P, I]
        L.or_table_lookup.argtypes = [M, ctypes.POINTER(LookupTable), D, D, D, D, P,
                                      ctypes.POINTER(I)]
        L.or_table_lookup.restype = I
        L.or_table_lookup_batch.argtypes = [M, ctypes.POINTER(LookupTable), P, P, P, D,
                                            ctypes.c_size_t, P, ctypes.c_size_t, P, P, I]
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(ctypes.c_void_p)


def parse_atmosphere(text: bytes, pi: float = PI_MULTIRAY) -> Medium:
    m = Medium()
    rc = lib().or_parse_atmosphere(text, len(text), pi, ctypes.byref(m))
    if rc != 0:
        raise ValueError("oracle: could not parse atmosphere text")
    return m


def load_atmosphere(path: str, pi: float = PI_MULTIRAY) -> Medium:
    with open(path, "rb") as f:
        data = f.read()
    if path.endswith(".gz"):
        import gzip
        data = gzip.decompress(data)
    return parse_atmosphere(data, pi)


def getnz_air(m: Medium, z: float) -> float:
    return lib().or_getnz_air(ctypes.byref(m), z)


def getnz_ice(m: Medium, z: float) -> float:
    return lib().or_getnz_ice(ctypes.byref(m), z)


def ray_solution(m: Medium, launch_deg, txh, ice_h, depth, in_ice=True) -> np.ndarray:
    out = np.zeros(18)
    lib().or_ray_solution(ctypes.byref(m), launch_deg, txh, ice_h, depth, int(in_ice), _ptr(out))
    return out


def grid_init(depth_cm, ice_cm, height_step=10.0, start_angle=90.1, stop_angle=180.0,
              angle_step=0.1) -> Grid:
    g = Grid()
    lib().or_grid_init(ctypes.byref(g), depth_cm, ice_cm, height_step, start_angle, stop_angle,
                       angle_step)
    return g


def table_rows(m: Medium, g: Grid, row0: int, row1: int, full: bool = False, nthreads: int = 0):
    """Rays of rows [row0, row1) clipped to the table's rows (g.table_rows: the reference skips
    Tx heights <= 0, .cc:2082), so the arrays are as long as the reference's table slice."""
    row1 = max(row0, min(row1, int(g.table_rows)))
    n = (row1 - row0) * g.angle_steps
    table = np.zeros((11, n), dtype=np.float32)
    fullarr = np.zeros((18, n), dtype=np.float64) if full else None
    lib().or_table_rows(ctypes.byref(m), ctypes.byref(g), row0, row1, _ptr(table), _ptr(fullarr),
                        n, nthreads)
    return (table, fullarr) if full else table


def air2ice(m: Medium, txh, dist, ice_h, depth, straight_angle=None):
    if straight_angle is None:
        straight_angle = straight_angle_of(m, txh, dist, ice_h, depth)
    out = np.zeros(17)
    st = lib().or_air2ice(ctypes.byref(m), txh, dist, ice_h, depth, straight_angle, _ptr(out))
    return out, st


def bisect(fn, lo: float, hi: float, tol: float = 1e-9, max_iter: int = 40):
    """GSL-bisection emulation (FindFunctionRoot, .cc:340-374) on a Python callable.
    Returns (root, status bits, number of f evaluations)."""
    calls = []

    def cb(x, _ctx):
        calls.append(x)
        return float(fn(x))

    cfn = _FN(cb)
    st = ctypes.c_int(0)
    r = lib().or_bisect(cfn, None, lo, hi, tol, max_iter, ctypes.byref(st))
    return r, st.value, calls


def brent(fn, lo: float, hi: float, tol: float = 1e-9, max_iter: int = 20):
    """GSL-Brent emulation (RayTracingFunctions FindFunctionRoot, .cc:256-290) on a Python
    callable.  Returns (root, status bits, f evaluation points, iterations)."""
    calls = []

    def cb(x, _ctx):
        calls.append(x)
        return float(fn(x))

    L = lib()
    if not getattr(L, "_brent_sig", False):
        L.or_brent.argtypes = [_FN, ctypes.c_void_p, ctypes.c_double, ctypes.c_double,
                               ctypes.c_double, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                               ctypes.POINTER(ctypes.c_int)]
        L.or_brent.restype = ctypes.c_double
        L._brent_sig = True
    cfn = _FN(cb)
    st, it = ctypes.c_int(0), ctypes.c_int(0)
    r = L.or_brent(cfn, None, lo, hi, tol, max_iter, ctypes.byref(st), ctypes.byref(it))
    return r, st.value, calls, it.value


RTF_AIR2ICE = 8  # AIRICE_RTF_AIR2ICE


def straight_angle_of(m: Medium, txh, dist, ice_h, depth) -> float:
    return lib().or_straight_angle(ctypes.byref(m), txh, dist, ice_h, depth)


def solve_batch(m: Medium, txh, dist, depth, ice_h, nthreads: int = 0):
    txh = np.ascontiguousarray(txh, dtype=np.float64)
    dist = np.ascontiguousarray(dist, dtype=np.float64)
    depth = np.ascontiguousarray(depth, dtype=np.float64)
    n = txh.size
    out = np.zeros((17, n))
    st = np.zeros(n, dtype=np.uint8)
    lib().or_solve_batch(ctypes.byref(m), _ptr(txh), _ptr(dist), _ptr(depth), ice_h, n,
                         _ptr(out), n, _ptr(st), nthreads)
    return out, st


def hdtip(m: Medium, src_cm, dist_cm, depth_cm, ice_cm):
    out = np.zeros(9)
    ok = lib().or_hdtip(ctypes.byref(m), src_cm, dist_cm, depth_cm, ice_cm, _ptr(out))
    return bool(ok), out


def hdtip_batch(m: Medium, src_cm, dist_cm, depth_cm, ice_cm, nthreads: int = 0):
    """or_hdtip over arrays (cm): (out (9, n), ok bool (n,), status of the solve (n,))."""
    src = np.ascontiguousarray(src_cm, dtype=np.float64)
    dst = np.ascontiguousarray(dist_cm, dtype=np.float64)
    dep = np.ascontiguousarray(np.broadcast_to(depth_cm, src.shape), dtype=np.float64)
    n = src.size
    out = np.zeros((9, n))
    ok = np.zeros(n, dtype=np.uint8)
    st = np.zeros(n, dtype=np.uint8)
    lib().or_hdtip_batch(ctypes.byref(m), _ptr(src), _ptr(dst), _ptr(dep), ice_cm, n, _ptr(out),
                         n, _ptr(ok), _ptr(st), nthreads)
    return out, ok.astype(bool), st


def py_air2ice(m: Medium, txh, dist, ice_h, depth, straight_angle):
    out = np.zeros(15)
    st = lib().or_py_air2ice(ctypes.byref(m), txh, dist, ice_h, depth, straight_angle, _ptr(out))
    return out, st


def py_trace_ice_to_air(m: Medium, depth, ice_h, txh, dist):
    out = np.zeros(10)
    ok = lib().or_py_trace_ice_to_air(ctypes.byref(m), depth, ice_h, txh, dist, _ptr(out))
    return bool(ok), out


def py_trace_batch(m: Medium, depth, ice, txh, dist, nthreads: int = 0):
    arrs = [np.ascontiguousarray(a, dtype=np.float64) for a in (depth, ice, txh, dist)]
    n = arrs[0].size
    out = np.zeros((n, 10))
    lib().or_py_trace_batch(ctypes.byref(m), *[_ptr(a) for a in arrs], n, _ptr(out), nthreads)
    return out


class LookupTable(ctypes.Structure):
    """or_lookup_table: one antenna's AllTableAllAntData[ant] + the grid globals (.cc:1035)."""
    _fields_ = [("col", ctypes.c_void_p * 11), ("n", ctypes.c_long),
                ("LoopStopHeight", ctypes.c_double), ("HeightStepSize", ctypes.c_double),
                ("TotalHeightSteps", ctypes.c_int), ("TotalAngleSteps", ctypes.c_int)]


def lookup_table(table: np.ndarray, g: Grid) -> LookupTable:
    """table: (11, n) float32 (C-contiguous, kept alive by the caller); g: the grid of the
    last table made (its stop height / step / row and angle counts)."""
    assert table.dtype == np.float32 and table.flags.c_contiguous and table.shape[0] == 11
    t = LookupTable()
    for c in range(11):
        t.col[c] = table[c].ctypes.data
    t.n = table.shape[1]
    t.LoopStopHeight = g.stop_height
    t.HeightStepSize = g.height_step
    t.TotalHeightSteps = g.height_steps
    t.TotalAngleSteps = g.angle_steps
    return t


def table_lookup(m: Medium, t: LookupTable, src_cm, dist_cm, depth_cm, ice_cm):
    """GetHorizontalDistanceToIntersectionPoint_Table (.cc:1305-1462) for one query:
    (ok, outs[9], flags)."""
    out = np.zeros(9)
    fl = ctypes.c_int(0)
    ok = lib().or_table_lookup(ctypes.byref(m), ctypes.byref(t), src_cm, dist_cm, depth_cm,
                               ice_cm, _ptr(out), ctypes.byref(fl))
    return bool(ok), out, fl.value


def table_lookup_batch(m: Medium, t: LookupTable, src_cm, dist_cm, depth_cm, ice_cm,
                       nthreads: int = 0):
    """Vector form of ``table_lookup``: (out (9, n), ok (n,) uint8, flags (n,) uint8)."""
    arrs = [np.ascontiguousarray(np.broadcast_to(a, np.shape(src_cm)), dtype=np.float64).ravel()
            for a in (src_cm, dist_cm, depth_cm)]
    n = arrs[0].size
    out = np.zeros((9, n))
    ok = np.zeros(n, dtype=np.uint8)
    fl = np.zeros(n, dtype=np.uint8)
    lib().or_table_lookup_batch(ctypes.byref(m), ctypes.byref(t), *[_ptr(a) for a in arrs],
                                ice_cm, n, _ptr(out), n, _ptr(ok), _ptr(fl), nthreads)
    return out, ok, fl


class SingleRay(ctypes.Structure):
    """or_single_ray (SingleRayAirIceRefraction.C:33-299)."""
    _fields_ = [("skip_above", ctypes.c_int), ("skip_below", ctypes.c_int),
                ("n_layers", ctypes.c_int), ("thd_air", ctypes.c_double), ("L", ctypes.c_double),
                ("inc_ice", ctypes.c_double), ("thd_ice", ctypes.c_double),
                ("recv_ice", ctypes.c_double), ("t_ice", ctypes.c_double),
                ("n_air", ctypes.c_long), ("n_ice", ctypes.c_long)]


def single_ray(m: Medium, depth, launch_deg, txh, ice):
    """cfg1 forward trace + RayPathinAirnIce.txt samples (after the CLI's clamps; depth > 0
    in ice).  Returns (SingleRay, x, z)."""
    L = lib()
    if not getattr(L, "_single_ray_sig", False):
        L.or_single_ray_trace.argtypes = [ctypes.POINTER(Medium), ctypes.c_double, ctypes.c_double,
                                          ctypes.c_double, ctypes.c_double,
                                          ctypes.POINTER(SingleRay), ctypes.c_void_p,
                                          ctypes.c_void_p, ctypes.c_long]
        L._single_ray_sig = True
    r = SingleRay()
    L.or_single_ray_trace(ctypes.byref(m), depth, launch_deg, txh, ice, ctypes.byref(r), None,
                          None, 0)
    n = r.n_air + r.n_ice
    x = np.zeros(n)
    z = np.zeros(n)
    L.or_single_ray_trace(ctypes.byref(m), depth, launch_deg, txh, ice, ctypes.byref(r), _ptr(x),
                          _ptr(z), n)
    return r, x, z


def rtf_eval(m: Medium, op: int, args) -> np.ndarray:
    """RayTracingFunctions:: scalar function `op` (AIRICE_RTF_*) in the reference's layout."""
    L = lib()
    if not getattr(L, "_rtf_sig", False):
        L.or_rtf_eval.argtypes = [ctypes.POINTER(Medium), ctypes.c_int, ctypes.c_void_p,
                                  ctypes.c_void_p]
        L.or_rtf_eval.restype = ctypes.c_int
        L._rtf_sig = True
    a = np.zeros(8)
    a[:len(args)] = args
    out = np.zeros(4 * 8 + 1)
    n = L.or_rtf_eval(ctypes.byref(m), op, _ptr(a), _ptr(out))
    if n < 0:
        raise ValueError(f"unknown op {op}")
    return out[:n].copy()


def lookup_closest_txh(t: LookupTable, P: float):
    """FindClosestAirTxHeight (.cc:1033-1126): ((s1, e1, s2, e2), (c1, c2), flags)."""
    idx = (ctypes.c_long * 4)()
    c = (ctypes.c_double * 2)()
    fl = ctypes.c_int(0)
    lib().or_lookup_closest_txh(ctypes.byref(t), ctypes.c_double(P), idx, c, ctypes.byref(fl))
    return tuple(idx), tuple(c), fl.value


def lookup_closest_thd(t: LookupTable, P: float, s: int, e: int):
    """FindClosestTHD (.cc:1128-1169): ((start, end), closest, flags)."""
    idx = (ctypes.c_long * 2)()
    c = ctypes.c_double(0)
    fl = ctypes.c_int(0)
    lib().or_lookup_closest_thd(ctypes.byref(t), ctypes.c_double(P), ctypes.c_long(s),
                                ctypes.c_long(e), idx, ctypes.byref(c), ctypes.byref(fl))
    return tuple(idx), c.value, fl.value


def lookup_par_values(t: LookupTable, H: float, D: float):
    """GetParValues (.cc:1172-1302): (H1, Par1[10], H2, Par2[10], flags)."""
    out = np.zeros(22)
    fl = ctypes.c_int(0)
    lib().or_lookup_par_values(ctypes.byref(t), ctypes.c_double(H), ctypes.c_double(D), _ptr(out),
                               ctypes.byref(fl))
    return out[0], out[1:11].copy(), out[11], out[12:22].copy(), fl.value
