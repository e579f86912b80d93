"""Drop-in for the reference's ctypes module ``pythonwrapper/AirIceRayTracing.py`` (:1-11).

Same names and argument meaning: ``handle`` is the loaded library, ``handle.Py_TraceIceToAir``
has the reference's argtypes (4 doubles + ``c_double*10``), and ``Py_TraceIceToAir(AntennaDepth,
IceLayerHeight, AirTxHeight, HorizontalDistance, ArrayParameters)`` fills the caller's 10-slot
array in the layout of ``TraceIceToAir.C:46-68`` (solution row, or ten -1000 sentinels).  A script
written for the reference (``TraceIceToAir.py``: ``from AirIceRayTracing import *``) runs unchanged
with this directory on ``sys.path``.

Differences, all additive: the library is ``libairice.so`` (HIP, gfx950) instead of the GSL build;
``Atmosphere.dat`` is read from the working directory once per process instead of on every call
(``TraceIceToAir.C:25``; ``$AIRICE_ATMOSPHERE`` names another file when the working directory has
none); nothing is printed per call (``TraceIceToAir.C:36-58`` writes to stdout); and
``Py_TraceIceToAir_batch`` solves whole numpy arrays in one GPU launch (BASELINE cfg5: 1e7 queries).
There is no CPU fallback: a missing or unloadable library raises at import.
"""
from __future__ import annotations

import ctypes
import os
import sys

_PKG_PARENT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.realpath(__file__))))
if _PKG_PARENT not in sys.path:
    sys.path.insert(0, _PKG_PARENT)

# lib() imports torch first when it is present (one HIP runtime per process) and raises
# AirIceLibraryError when libairice.so is missing
from airiceraytracing_amd._lib import lib as _lib  # noqa: E402

handle = _lib()
handle.Py_TraceIceToAir.argtypes = [ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                    ctypes.c_double, ctypes.c_double * 10]
handle.Py_TraceIceToAir.restype = None


def Py_TraceIceToAir(AntennaDepth, IceLayerHeight, AirTxHeight, HorizontalDistance,
                     ArrayParameters):
    return handle.Py_TraceIceToAir(AntennaDepth, IceLayerHeight, AirTxHeight, HorizontalDistance,
                                   ArrayParameters)


def Py_TraceIceToAir_batch(AntennaDepth, IceLayerHeight, AirTxHeight, HorizontalDistance,
                           atmosphere=None):
    """Vectorised Py_TraceIceToAir: broadcastable arrays (m) in, an (n, 10) float64 array out,
    row i equal to what ``Py_TraceIceToAir`` writes for query i."""
    import numpy as np

    from airiceraytracing_amd import AirIceSolver, VARIANT_PYWRAPPER
    if atmosphere is None:
        atmosphere = "Atmosphere.dat" if os.path.exists("Atmosphere.dat") else \
            os.environ.get("AIRICE_ATMOSPHERE")
    solver = AirIceSolver(atmosphere, variant=VARIANT_PYWRAPPER)
    arrs = np.broadcast_arrays(*[np.asarray(a, dtype=np.float64) for a in
                                 (AntennaDepth, IceLayerHeight, AirTxHeight, HorizontalDistance)])
    return solver.trace_ice_to_air_host(*[a.ravel() for a in arrs])
