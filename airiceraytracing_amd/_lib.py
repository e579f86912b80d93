"""ctypes binding of libairice.so (include/airice.h).

The product path: every compute call goes through the HIP library.  There is no
CPU fallback -- if ``libairice.so`` is missing or cannot be loaded, import of the
compute entry points raises :class:`AirIceLibraryError`.
"""
from __future__ import annotations

import ctypes
import gzip
import os
import subprocess

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "libairice.so")
CSRC_DIR = os.path.join(PKG_DIR, "csrc")
DATA_DIR = os.path.join(PKG_DIR, "data")

AIRICE_OK = 0
VARIANT_MULTIRAY = 0
VARIANT_PYWRAPPER = 1

SOLVE_NONFINITE_END = 1
SOLVE_BAD_BRACKET = 2
SOLVE_STALE_MID = 4
SOLVE_PROBED = 8
SOLVE_MAXITER = 16
SOLVE_NO_AIR_LAYER = 32

TABLE_COLUMNS = 11
RAY_FIELDS = 18
SOLVE_FIELDS = 17
PYSOLVE_FIELDS = 15
HDTIP_FIELDS = 9


class AirIceLibraryError(RuntimeError):
    pass


class Medium(ctypes.Structure):
    """airice_medium (include/airice.h)."""

    _fields_ = [
        ("atmlay_cm", ctypes.c_double * 5),
        ("abc", (ctypes.c_double * 3) * 5),
        ("B_air", ctypes.c_double * 5),
        ("C_air", ctypes.c_double * 5),
        ("N0", ctypes.c_double),
        ("max_layers", ctypes.c_int32),
        ("n_points", ctypes.c_int32),
        ("A_air", ctypes.c_double),
        ("A_ice", ctypes.c_double),
        ("B_ice", ctypes.c_double),
        ("C_ice", ctypes.c_double),
        ("pi", ctypes.c_double),
        ("h_top", ctypes.c_double),
        ("constant_air_index", ctypes.c_int32),
        ("reserved_", ctypes.c_int32),
        ("A_const", ctypes.c_double),
    ]


class Grid(ctypes.Structure):
    """airice_grid (include/airice.h)."""

    _fields_ = [
        ("start_height", ctypes.c_double),
        ("stop_height", ctypes.c_double),
        ("height_step", ctypes.c_double),
        ("height_steps", ctypes.c_int32),
        ("start_angle", ctypes.c_double),
        ("stop_angle", ctypes.c_double),
        ("angle_step", ctypes.c_double),
        ("angle_steps", ctypes.c_int32),
        ("depth_m", ctypes.c_double),
        ("ice_m", ctypes.c_double),
        ("in_ice", ctypes.c_int32),
        ("table_rows", ctypes.c_int32),
    ]

    @property
    def n_rays(self) -> int:
        """Entries of the table: table_rows x angle_steps (rows with Tx <= 0 are skipped)."""
        return int(self.table_rows) * int(self.angle_steps)


class LookupTable(ctypes.Structure):
    """airice_lookup_table (include/airice.h): one antenna's HBM-resident table + the grid
    globals the reference's lookup reads (MultiRayAirIceRefraction.cc:1035-1039)."""

    _fields_ = [
        ("table", ctypes.c_void_p),
        ("ld", ctypes.c_size_t),
        ("n_entries", ctypes.c_size_t),
        ("loop_stop_height", ctypes.c_double),
        ("height_step", ctypes.c_double),
        ("total_height_steps", ctypes.c_int32),
        ("total_angle_steps", ctypes.c_int32),
        ("entries", ctypes.c_void_p),
    ]


SCALAR_HOST, SCALAR_DEVICE = 0, 1  # AIRICE_SCALAR_HOST / AIRICE_SCALAR_DEVICE

LOOKUP_ENTRY_FLOATS = 16  # AIRICE_LOOKUP_ENTRY_FLOATS (pack format 2)
LOOKUP_ROW_FLOATS = 64  # AIRICE_LOOKUP_ROW_FLOATS


def lookup_rows_offset(n):
    """AIRICE_LOOKUP_ROWS_OFFSET: first float of the row records in the packed copy."""
    return (n * LOOKUP_ENTRY_FLOATS + 31) // 32 * 32


def lookup_pack_floats(n, asteps):
    """AIRICE_LOOKUP_PACK_FLOATS: floats of the whole packed copy."""
    return lookup_rows_offset(n) + n // asteps * LOOKUP_ROW_FLOATS + (asteps + 3) // 4 * 4 + 4


class SingleRayInfo(ctypes.Structure):
    """airice_single_ray_info (include/airice.h)."""

    _fields_ = [("skip_above", ctypes.c_int32), ("skip_below", ctypes.c_int32),
                ("n_layers", ctypes.c_int32), ("pad_", ctypes.c_int32),
                ("n_air", ctypes.c_int64), ("n_ice", ctypes.c_int64)]


class TableFileInfo(ctypes.Structure):
    """airice_table_file_info (include/airice.h): the header of a table file."""

    _fields_ = [("medium", Medium), ("grid", Grid), ("n_rays", ctypes.c_uint64),
                ("checksum", ctypes.c_uint64)]


TABLE_FILE_HEADER = 512  # AIRICE_TABLE_FILE_HEADER

SINGLE_RAY_FIELDS = 6  # AIRICE_SINGLE_RAY_FIELDS
SINGLE_RAY_WORK = 32   # AIRICE_SINGLE_RAY_WORK

LOOKUP_FALLBACK = 1  # AIRICE_LOOKUP_FALLBACK
LOOKUP_UNPINNED = 2  # AIRICE_LOOKUP_UNPINNED

# Every symbol include/airice.h declares (checked by tests/test_capi.py).
# RayTracingFunctions:: scalar ops (include/airice.h AIRICE_RTF_*)
RTF_HIT_POINT, RTF_OPTICAL_PATH, RTF_PROPAGATION_TIME, RTF_AIR_PROPAGATION = 0, 1, 2, 3
RTF_ICE_PROPAGATION, RTF_FDNFR, RTF_FTIMED, RTF_MIN_LAUNCH = 4, 5, 6, 7
RTF_AIR2ICE = 8  # the Air2IceRayTracing CLI's Brent search (AIRICE_RTF_AIR2ICE_FIELDS outputs)
# MultiRayAirIceRefraction:: forms of the ray layer (AIRICE_MR_*)
MR_FPATHD, MR_GEOMETRIC_PATH, MR_HIT_POINT, MR_AIR_PROPAGATION = 9, 10, 11, 12
MR_ICE_PROPAGATION, MR_MIN_LAUNCH = 13, 14

EXPORTED_SYMBOLS = (
    "airice_last_error", "airice_version", "airice_atmosphere_load", "airice_atmosphere_parse",
    "airice_nz_air", "airice_nz_ice", "airice_grid_init", "airice_table_launch",
    "airice_table_launch_multi",
    "airice_table_host", "airice_rays_launch", "airice_rays_host", "airice_scalar_mode", "airice_solve_launch", "airice_solve_host",
    "airice_hdtip_launch", "airice_table_lookup_launch", "airice_lookup_pack", "airice_lookup_pack_floats", "airice_single_ray_plan",
    "airice_single_ray_launch", "airice_single_ray_host", "airice_trace_ice_to_air_launch",
    "airice_trace_ice_to_air_host", "airice_rtf_outputs", "airice_rtf_eval",
    "airice_rtf_eval_variant", "Py_TraceIceToAir", "airice_device_count", "airice_set_device", "airice_malloc",
    "airice_free", "airice_memcpy_h2d", "airice_memcpy_d2h", "airice_synchronize",
    "airice_kernel_timing", "airice_kernel_time", "airice_launch_count",
    "airice_table_cache_stats", "airice_table_to_host",
    "airice_host_register", "airice_host_unregister", "airice_table_checksum",
    "airice_table_save", "airice_table_file_read_info", "airice_table_load",
)


def build(force: bool = False) -> str:
    """Compile libairice.so for gfx950 with hipcc (csrc/Makefile)."""
    args = ["make", "-s", "-C", CSRC_DIR]
    if force:
        args.append("-B")
    subprocess.run(args, check=True)
    return LIB_PATH


_lib = None


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise AirIceLibraryError(
            f"{LIB_PATH} not found: build it with __graft_entry__.build() or "
            f"'make -C {CSRC_DIR}' (no CPU fallback exists)")
    # One HIP runtime per process: torch bundles its own libamdhip64 (SONAME
    # libamdhip64.so.7).  Loading torch first makes libairice.so's NEEDED entry resolve
    # to that copy; loading libairice.so first would pull /opt/rocm's copy in beside
    # torch's and torch.cuda would then see no device.
    try:
        import torch  # noqa: F401
    except ImportError:  # plain ctypes users (the Py_TraceIceToAir drop-in) need no torch
        pass
    try:
        L = ctypes.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover - depends on the box
        raise AirIceLibraryError(f"cannot load {LIB_PATH}: {e}") from e
    D, I, P, S = ctypes.c_double, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t
    M, G = ctypes.POINTER(Medium), ctypes.POINTER(Grid)
    sig = {
        "airice_last_error": ([], ctypes.c_char_p),
        "airice_version": ([], ctypes.c_char_p),
        "airice_atmosphere_load": ([ctypes.c_char_p, I, M], I),
        "airice_atmosphere_parse": ([ctypes.c_char_p, S, I, M], I),
        "airice_nz_air": ([M, D], D),
        "airice_nz_ice": ([M, D], D),
        "airice_grid_init": ([G, D, D, D, D, D, D], I),
        "airice_table_launch": ([M, G, ctypes.c_int32, ctypes.c_int32, P, P, S, P], I),
        "airice_table_host": ([M, G, ctypes.c_int32, ctypes.c_int32, P, P, S], I),
        "airice_table_launch_multi": ([M, G, ctypes.c_int32, P, P, P], I),
        "airice_rays_launch": ([M, P, P, D, D, ctypes.c_int32, S, P, S, P], I),
        "airice_rays_host": ([M, P, P, D, D, ctypes.c_int32, S, P, S], I),
        "airice_scalar_mode": ([I], I),
        "airice_solve_launch": ([M, I, D, P, P, P, P, S, P, S, P, P], I),
        "airice_solve_host": ([M, I, D, P, P, P, P, S, P, S, P], I),
        "airice_hdtip_launch": ([M, P, P, P, D, S, P, S, P, P], I),
        "airice_table_lookup_launch": ([M, ctypes.POINTER(LookupTable), P, P, P, D, S, P, S, P,
                                        P, P], I),
        "airice_lookup_pack": ([ctypes.POINTER(LookupTable), P, S, P], I),
        "airice_lookup_pack_floats": ([S, ctypes.c_int32], S),
        "airice_single_ray_plan": ([M, D, D, D, D, ctypes.POINTER(SingleRayInfo)], I),
        "airice_single_ray_launch": ([M, D, D, D, D, P, P, P, S, P], I),
        "airice_single_ray_host": ([M, D, D, D, D, P, P, P, S], I),
        "airice_rtf_outputs": ([I, I], I),
        "airice_rtf_eval": ([M, I, P, S, P, S], I),
        "airice_rtf_eval_variant": ([M, I, I, P, S, P, S], I),
        "airice_table_to_host": ([P, S, S, P, S, P], I),
        "airice_host_register": ([P, S], I),
        "airice_host_unregister": ([P], I),
        "airice_table_checksum": ([P, S, S], ctypes.c_uint64),
        "airice_table_save": ([ctypes.c_char_p, M, G, P, S, S], I),
        "airice_table_file_read_info": ([ctypes.c_char_p, ctypes.POINTER(TableFileInfo)], I),
        "airice_table_load": ([ctypes.c_char_p, M, P, S, ctypes.POINTER(TableFileInfo)], I),
        "airice_trace_ice_to_air_launch": ([M, P, P, P, P, S, P, P], I),
        "airice_trace_ice_to_air_host": ([M, P, P, P, P, S, P], I),
        "Py_TraceIceToAir": ([D, D, D, D, ctypes.POINTER(D)], None),
        "airice_device_count": ([ctypes.POINTER(I)], I),
        "airice_set_device": ([I], I),
        "airice_malloc": ([ctypes.POINTER(P), S], I),
        "airice_free": ([P], I),
        "airice_memcpy_h2d": ([P, P, S], I),
        "airice_memcpy_d2h": ([P, P, S], I),
        "airice_synchronize": ([], I),
        "airice_kernel_timing": ([I], I),
        "airice_kernel_time": ([ctypes.c_char_p, ctypes.POINTER(D), ctypes.POINTER(ctypes.c_int64),
                                I], I),
        "airice_launch_count": ([ctypes.c_char_p, ctypes.POINTER(ctypes.c_int64), I], I),
    }
    for name, (args, res) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    _lib = L
    return L


def check(rc: int, what: str) -> None:
    if rc != AIRICE_OK:
        msg = lib().airice_last_error().decode(errors="replace")
        raise AirIceLibraryError(f"{what} failed (rc={rc}): {msg}")


def ptr(a) -> ctypes.c_void_p | None:
    """Host numpy array or device tensor -> void*."""
    if a is None:
        return None
    if isinstance(a, np.ndarray):
        return a.ctypes.data_as(ctypes.c_void_p)
    if hasattr(a, "data_ptr"):
        return ctypes.c_void_p(a.data_ptr())
    if isinstance(a, int):
        return ctypes.c_void_p(a)
    raise TypeError(f"cannot take a pointer of {type(a)!r}")


def default_atmosphere_path() -> str:
    """Atmosphere.dat lookup: $AIRICE_ATMOSPHERE, ./Atmosphere.dat (the reference reads the
    working directory, MultiRayAirIceRefraction.cc:27), then the bundled GDAS file."""
    env = os.environ.get("AIRICE_ATMOSPHERE")
    if env and os.path.exists(env):
        return env
    if os.path.exists("Atmosphere.dat"):
        return os.path.abspath("Atmosphere.dat")
    return os.path.join(DATA_DIR, "Atmosphere.dat.gz")


def read_atmosphere_text(path: str | None = None) -> bytes:
    path = path or default_atmosphere_path()
    with open(path, "rb") as f:
        data = f.read()
    if path.endswith(".gz"):
        data = gzip.decompress(data)
    return data


def load_medium(path: str | None = None, variant: int = VARIANT_MULTIRAY) -> Medium:
    text = read_atmosphere_text(path)
    m = Medium()
    check(lib().airice_atmosphere_parse(text, len(text), variant, ctypes.byref(m)),
          "airice_atmosphere_parse")
    return m


def kernel_timing(on: bool) -> None:
    """Bracket launches of the timed kernels with hipEvent pairs (airice_kernel_timing)."""
    check(lib().airice_kernel_timing(1 if on else 0), "airice_kernel_timing")


def kernel_time(name: str, reset: bool = True) -> tuple[float, int]:
    """(summed ms, launches) of one timed kernel since the last reset (airice_kernel_time)."""
    ms = ctypes.c_double(0.0)
    cnt = ctypes.c_int64(0)
    check(lib().airice_kernel_time(name.encode(), ctypes.byref(ms), ctypes.byref(cnt),
                                   1 if reset else 0), "airice_kernel_time")
    return ms.value, cnt.value


def launch_count(name: str, reset: bool = False) -> int:
    """Launches of one kernel in this process since the last reset (airice_launch_count)."""
    cnt = ctypes.c_int64(0)
    check(lib().airice_launch_count(name.encode(), ctypes.byref(cnt), 1 if reset else 0),
          "airice_launch_count")
    return cnt.value


class launched:
    """``with launched("rtf_kernel") as n: ...`` -- n.count is how many launches of that kernel
    the block made (airice_launch_count; a device test asserts it is > 0)."""

    def __init__(self, name: str):
        self.name = name
        self.count = 0
        self._start = 0

    def __enter__(self):
        self._start = launch_count(self.name)
        return self

    def __exit__(self, *exc):
        self.count = launch_count(self.name) - self._start
        return False


def table_cache_stats() -> dict:
    """Entries of the table launch's per-grid caches on the current device
    (airice_table_cache_stats): keys seen, filled and pinned, for the row constants and the
    start-angle sines."""
    out = (ctypes.c_int * 6)()
    fn = lib().airice_table_cache_stats  # bound here: tools/ab_table.py loads older builds too
    fn.argtypes, fn.restype = [ctypes.POINTER(ctypes.c_int)], ctypes.c_int
    check(fn(out), "airice_table_cache_stats")
    return {"rows": {"keys": out[0], "filled": out[1], "pinned": out[2]},
            "angles": {"keys": out[3], "filled": out[4], "pinned": out[5]}}
