"""airiceraytracing_amd -- MI355X (gfx950) air->ice ray solver.

A from-scratch HIP implementation of the uzairlatif90/AirIceRayTracing hot path
(MultiRayAirIceRefraction table generation + Air2Ice launch-angle root finding, and
the pythonwrapper ``Py_TraceIceToAir`` surface) behind a C-ABI (``include/airice.h``,
``libairice.so``).  See DESIGN.md.
"""
from ._lib import (AirIceLibraryError, Grid, LOOKUP_FALLBACK, LOOKUP_UNPINNED, LookupTable,
                   Medium, VARIANT_MULTIRAY, VARIANT_PYWRAPPER, build, default_atmosphere_path,
                   lib, load_medium)
from .solver import AirIceSolver, make_grid

__all__ = [
    "AirIceLibraryError", "AirIceSolver", "Grid", "LOOKUP_FALLBACK", "LOOKUP_UNPINNED",
    "LookupTable", "Medium", "VARIANT_MULTIRAY",
    "VARIANT_PYWRAPPER", "build", "default_atmosphere_path", "lib", "load_medium", "make_grid",
]
__version__ = "0.2.0"
