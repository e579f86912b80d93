"""Batched host API over libairice.so.

Two flavours of every entry point:
  * ``*_device``: inputs/outputs already resident in HBM (torch CUDA tensors or raw
    device pointers), stream-ordered, asynchronous -- the path ``bench.py`` times;
  * ``*_host``: numpy in, numpy out (the library copies, launches, synchronises).

Layouts follow the reference: the table is 11 float columns
(``AllTableAllAntData[ant][col][row]``, MultiRayAirIceRefraction.cc:2101-2111), ray and
solve outputs are the reference ``dummy[]`` slots as double columns.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import (Grid, LookupTable, Medium, VARIANT_MULTIRAY, VARIANT_PYWRAPPER, check, lib,
                   ptr)


def make_grid(antenna_depth_cm: float, ice_height_cm: float, height_step: float = 10.0,
              start_angle: float = 90.1, stop_angle: float = 180.0,
              angle_step: float = 0.1) -> Grid:
    """MakeRayTracingTable grid (MultiRayAirIceRefraction.cc:12-21, 2019-2061).  Defaults are
    the reference's globals (10 m x 0.1 deg, 90.1..180 deg, 100 km down to the ice)."""
    g = Grid()
    check(lib().airice_grid_init(ctypes.byref(g), antenna_depth_cm, ice_height_cm, height_step,
                                 start_angle, stop_angle, angle_step), "airice_grid_init")
    return g


class scalar_mode:
    """Where the one-query ray and ray-layer calls run (airice_scalar_mode), for a ``with`` block:
    _lib.SCALAR_HOST (the library's default) or _lib.SCALAR_DEVICE."""

    def __init__(self, mode: int):
        self.mode = mode
        self.prev = None

    def __enter__(self):
        self.prev = lib().airice_scalar_mode(self.mode)
        return self

    def __exit__(self, *exc):
        lib().airice_scalar_mode(self.prev)
        return False


def _stream_handle(stream):
    if stream is None:
        return None
    if isinstance(stream, int):
        return ctypes.c_void_p(stream)
    return ctypes.c_void_p(stream.cuda_stream)  # torch.cuda.Stream


class AirIceSolver:
    """One medium (parsed GDAS atmosphere + ice model) and the batched GPU entry points."""

    def __init__(self, atmosphere: str | None = None, variant: int = VARIANT_MULTIRAY):
        self.variant = variant
        self.medium: Medium = _lib.load_medium(atmosphere, variant)

    # ------------------------------------------------------------------ table
    def table_device(self, grid: Grid, table, full=None, row_begin: int = 0,
                     row_count: int | None = None, ld: int | None = None, stream=None) -> None:
        if row_count is None:
            row_count = grid.table_rows - row_begin
        n = row_count * grid.angle_steps
        ld = n if ld is None else ld
        check(lib().airice_table_launch(ctypes.byref(self.medium), ctypes.byref(grid), row_begin,
                                        row_count, ptr(table), ptr(full), ld,
                                        _stream_handle(stream)), "airice_table_launch")

    def tables_device(self, grids, tables, stream=None) -> None:
        """Several antennas' whole tables in one launch (airice_table_launch_multi): grids[a] and
        tables[a] (11 x >= grids[a].n_rays float32 device tensors, one per antenna)."""
        n = len(grids)
        garr = (Grid * n)(*grids)
        ptrs = (ctypes.c_void_p * n)(*[ptr(t).value for t in tables])
        lds = (ctypes.c_size_t * n)(*[int(t.shape[-1]) for t in tables])
        check(lib().airice_table_launch_multi(ctypes.byref(self.medium), garr, n, ptrs, lds,
                                              _stream_handle(stream)),
              "airice_table_launch_multi")

    def table_host(self, grid: Grid, row_begin: int = 0, row_count: int | None = None,
                   full: bool = False):
        if row_count is None:
            row_count = grid.table_rows - row_begin
        n = row_count * grid.angle_steps
        table = np.empty((_lib.TABLE_COLUMNS, n), dtype=np.float32)
        fullarr = np.empty((_lib.RAY_FIELDS, n), dtype=np.float64) if full else None
        check(lib().airice_table_host(ctypes.byref(self.medium), ctypes.byref(grid), row_begin,
                                      row_count, ptr(table), ptr(fullarr), n),
              "airice_table_host")
        return (table, fullarr) if full else table

    # ------------------------------------------------------------------ table files
    def save_table(self, path: str, grid: Grid, table) -> None:
        """airice_table_save: one antenna's table (11 x n float32, numpy or a torch tensor on
        any device) with this medium and ``grid`` in the header."""
        if hasattr(table, "detach"):
            table = table.detach().cpu().numpy()
        t = np.asarray(table)
        if t.dtype != np.float32 or t.ndim != 2 or t.shape[0] != _lib.TABLE_COLUMNS:
            raise ValueError(f"save_table: want an ({_lib.TABLE_COLUMNS}, n) float32 table, "
                             f"got {t.dtype} {t.shape}")
        if t.strides[1] != 4:
            t = np.ascontiguousarray(t)
        check(lib().airice_table_save(str(path).encode(), ctypes.byref(self.medium),
                                      ctypes.byref(grid), ptr(t), t.strides[0] // 4, t.shape[1]),
              "airice_table_save")

    @staticmethod
    def table_file_info(path: str) -> _lib.TableFileInfo:
        info = _lib.TableFileInfo()
        check(lib().airice_table_file_read_info(str(path).encode(), ctypes.byref(info)),
              "airice_table_file_read_info")
        return info

    def load_table(self, path: str, check_medium: bool = True):
        """airice_table_load: (grid, 11 x n float32 numpy table), checksum-verified; with
        ``check_medium`` a table traced in another medium is refused."""
        info = self.table_file_info(path)
        n = int(info.n_rays)
        table = np.empty((_lib.TABLE_COLUMNS, n), dtype=np.float32)
        check(lib().airice_table_load(str(path).encode(),
                                      ctypes.byref(self.medium) if check_medium else None,
                                      ptr(table), max(n, 1), ctypes.byref(info)),
              "airice_table_load")
        return info.grid, table

    # ------------------------------------------------------------------ rays
    def rays_device(self, launch_deg, txh, ice_h: float, depth: float, in_ice: bool, out,
                    ld: int | None = None, stream=None) -> None:
        n = int(launch_deg.numel())
        check(lib().airice_rays_launch(ctypes.byref(self.medium), ptr(launch_deg), ptr(txh),
                                       ice_h, depth, int(in_ice), n, ptr(out),
                                       n if ld is None else ld, _stream_handle(stream)),
              "airice_rays_launch")

    def rays_host(self, launch_deg, txh, ice_h: float, depth: float, in_ice: bool) -> np.ndarray:
        """airice_rays_host: GetRayTracingSolutions for host arrays on the CPU (the one-query
        drop-in's path, same source as the device kernels); (18, n) doubles."""
        a = np.ascontiguousarray(launch_deg, dtype=np.float64).ravel()
        h = np.ascontiguousarray(np.broadcast_to(txh, a.shape), dtype=np.float64).ravel()
        out = np.empty((_lib.RAY_FIELDS, a.size), dtype=np.float64)
        check(lib().airice_rays_host(ctypes.byref(self.medium), ptr(a), ptr(h), ice_h, depth,
                                     int(in_ice), a.size, ptr(out), max(a.size, 1)),
              "airice_rays_host")
        return out

    # ------------------------------------------------------------------ minimizer
    def solve_device(self, txh, dist, depth, ice_h: float, out, status=None,
                     straight_angle=None, ld: int | None = None, stream=None,
                     variant: int | None = None) -> None:
        n = int(txh.numel())
        v = self.variant if variant is None else variant
        check(lib().airice_solve_launch(ctypes.byref(self.medium), v, ice_h, ptr(txh), ptr(dist),
                                        ptr(depth), ptr(straight_angle), n, ptr(out),
                                        n if ld is None else ld, ptr(status),
                                        _stream_handle(stream)), "airice_solve_launch")

    def solve_host(self, txh, dist, depth, ice_h: float, straight_angle=None,
                   variant: int | None = None):
        v = self.variant if variant is None else variant
        txh = np.ascontiguousarray(txh, dtype=np.float64)
        dist = np.ascontiguousarray(dist, dtype=np.float64)
        depth = np.ascontiguousarray(depth, dtype=np.float64)
        thr = None if straight_angle is None else np.ascontiguousarray(straight_angle, np.float64)
        n = txh.size
        fields = _lib.PYSOLVE_FIELDS if v == VARIANT_PYWRAPPER else _lib.SOLVE_FIELDS
        out = np.empty((fields, n), dtype=np.float64)
        st = np.empty(n, dtype=np.uint8)
        check(lib().airice_solve_host(ctypes.byref(self.medium), v, ice_h, ptr(txh), ptr(dist),
                                      ptr(depth), ptr(thr), n, ptr(out), n, ptr(st)),
              "airice_solve_host")
        return out, st

    # ------------------------------------------------------------------ CoREAS entry
    def hdtip_device(self, src_cm, dist_cm, depth_cm, ice_cm: float, out, ok,
                     ld: int | None = None, stream=None) -> None:
        n = int(src_cm.numel())
        check(lib().airice_hdtip_launch(ctypes.byref(self.medium), ptr(src_cm), ptr(dist_cm),
                                        ptr(depth_cm), ice_cm, n, ptr(out),
                                        n if ld is None else ld, ptr(ok),
                                        _stream_handle(stream)), "airice_hdtip_launch")

    # ------------------------------------------------------------------ table lookup
    @staticmethod
    def lookup_table(table, grid: Grid, n_entries: int | None = None,
                     ld: int | None = None) -> LookupTable:
        """Describe an HBM-resident table (11 float columns, column stride ``ld``) for
        ``table_lookup_device``; ``grid`` supplies the globals of the last table made
        (LoopStopHeight, HeightStepSize, TotalHeightSteps, TotalAngleSteps, .cc:1035-1039)."""
        n = grid.n_rays if n_entries is None else n_entries
        t = LookupTable()
        t.table = ptr(table).value
        t.ld = n if ld is None else ld
        t.n_entries = n
        t.loop_stop_height = grid.stop_height
        t.height_step = grid.height_step
        t.total_height_steps = grid.height_steps
        t.total_angle_steps = grid.angle_steps
        return t

    @staticmethod
    def lookup_pack(lt: LookupTable, stream=None):
        """airice_lookup_pack: a packed copy of the table (pack format 2: one 64-byte pair record
        per entry, holding it and the next entry, one 256-byte record per table row and the angle
        vector; torch tensor on the table's device) that ``lt`` then reads; the tensor is kept on
        ``lt``."""
        import torch
        n, asteps = int(lt.n_entries), int(lt.total_angle_steps)
        if n < 1 or asteps < 1:  # as airice_lookup_pack: the row records divide by the row length
            raise ValueError(f"lookup_pack: n_entries ({n}) and total_angle_steps ({asteps}) "
                             "must be >= 1")
        floats = int(lib().airice_lookup_pack_floats(n, asteps))
        packed = torch.empty(floats, dtype=torch.float32,
                             device=torch.device("cuda", torch.cuda.current_device()))
        check(lib().airice_lookup_pack(ctypes.byref(lt), ptr(packed), floats,
                                       _stream_handle(stream)), "airice_lookup_pack")
        lt.entries = ptr(packed).value
        lt._packed = packed
        return packed

    def table_lookup_device(self, lt: LookupTable, src_cm, dist_cm, depth_cm, ice_cm: float,
                            out, ok, flags, ld: int | None = None, stream=None) -> None:
        """Batched GetHorizontalDistanceToIntersectionPoint_Table (.cc:1305-1462): out is the
        9 double columns of ``hdtip_device``; ok the returned bool; flags AIRICE_LOOKUP_*."""
        n = int(src_cm.numel())
        check(lib().airice_table_lookup_launch(ctypes.byref(self.medium), ctypes.byref(lt),
                                               ptr(src_cm), ptr(dist_cm), ptr(depth_cm), ice_cm,
                                               n, ptr(out), n if ld is None else ld, ptr(ok),
                                               ptr(flags), _stream_handle(stream)),
              "airice_table_lookup_launch")

    # ------------------------------------------------------------------ single ray (cfg1)
    def single_ray_host(self, antenna_depth: float, launch_deg: float, txh: float, ice: float,
                        path: bool = True):
        """SingleRayAirIceRefraction (BASELINE cfg1) on the GPU: the forward trace of one launch
        angle and, with ``path``, the RayPathinAirnIce.txt samples.  Inputs after the CLI's
        clamps; antenna depth positive in ice (SingleRayAirIceRefraction.C:166).  Returns
        (summary[6], x, z): thd_air, L, incident angle on ice, thd_ice, receive angle in ice,
        ice propagation time."""
        info = _lib.SingleRayInfo()
        check(lib().airice_single_ray_plan(ctypes.byref(self.medium), antenna_depth, launch_deg,
                                           txh, ice, ctypes.byref(info)), "airice_single_ray_plan")
        n = int(info.n_air + info.n_ice) if path else 0
        summary = np.empty(_lib.SINGLE_RAY_FIELDS)
        x = np.empty(n)
        z = np.empty(n)
        check(lib().airice_single_ray_host(ctypes.byref(self.medium), antenna_depth, launch_deg,
                                           txh, ice, ptr(summary), ptr(x) if path else None,
                                           ptr(z) if path else None, n),
              "airice_single_ray_host")
        return summary, x, z, info

    # ------------------------------------------------------------------ pythonwrapper
    def trace_ice_to_air_device(self, depth, ice, txh, dist, out10, stream=None) -> None:
        n = int(depth.numel())
        check(lib().airice_trace_ice_to_air_launch(ctypes.byref(self.medium), ptr(depth), ptr(ice),
                                                   ptr(txh), ptr(dist), n, ptr(out10),
                                                   _stream_handle(stream)),
              "airice_trace_ice_to_air_launch")

    def rtf_eval(self, op: int, args) -> np.ndarray:
        """One RayTracingFunctions:: scalar function (AIRICE_RTF_*, include/airice.h) where
        scalar_mode() says -- the host by default, else the GPU -- in the reference's output
        layout."""
        a = np.ascontiguousarray(args, dtype=np.float64)
        n = lib().airice_rtf_outputs(op, int(self.medium.max_layers))
        if n < 0:
            raise ValueError(f"unknown RayTracingFunctions op {op}")
        out = np.zeros(n, dtype=np.float64)
        check(lib().airice_rtf_eval(ctypes.byref(self.medium), op, ptr(a), a.size, ptr(out), n),
              "airice_rtf_eval")
        return out

    def trace_ice_to_air_host(self, depth, ice, txh, dist):
        arrs = [np.ascontiguousarray(np.broadcast_to(a, np.shape(depth)), dtype=np.float64).ravel()
                for a in (depth, ice, txh, dist)]
        n = arrs[0].size
        out = np.empty((n, 10), dtype=np.float64)
        check(lib().airice_trace_ice_to_air_host(ctypes.byref(self.medium), *[ptr(a) for a in arrs],
                                                 n, ptr(out)), "airice_trace_ice_to_air_host")
        return out
