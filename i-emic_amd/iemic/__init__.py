"""iemic -- MI355X-native Newton-Krylov core for the THCM ocean model (host side).

The compute path lives in the HIP library ``i-emic_amd/lib/libiemic_amd.so`` (C ABI in
``include/iemic.h``); this package holds the Ocean-shaped host interface, configuration
and input preparation.
"""
from . import config
from .config import THCMConfig, landmask, preset, synthetic_state
from ._lib import IemicError

__all__ = ["config", "THCMConfig", "landmask", "preset", "synthetic_state", "IemicError",
           "Ocean"]


def __getattr__(name):
    if name == "Ocean":
        from .ocean import Ocean
        return Ocean
    raise AttributeError(name)
