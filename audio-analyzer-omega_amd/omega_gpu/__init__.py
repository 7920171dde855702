"""omega_gpu -- MI355X engine for the OMEGA-4 analysis hot path, behind the reference's own Python
surfaces (see include/omega.h for the C ABI and the reference file:line each entry point replaces).

Everything numeric runs in libomega.so (hand-written HIP for gfx950); importing a facade without the
built library raises ImportError -- there is no CPU fallback.
"""
from ._lib import LIB_PATH, OmegaError, UnsupportedError, lib
from .engine import DEFAULT_RESOLUTIONS, METER_KEYS, NORTHSTAR_RESOLUTIONS, BandTable, Engine, Resolution

__all__ = [
    "LIB_PATH", "OmegaError", "UnsupportedError", "lib", "Engine", "Resolution", "BandTable",
    "DEFAULT_RESOLUTIONS", "NORTHSTAR_RESOLUTIONS", "METER_KEYS",
]
