"""romis_amd -- MI355X-native ReSTIR direct-lighting sampler (host side of the drop-in boundary).

The product is libromis_amd.so (HIP kernels for gfx950 + the C ABI of include/restir_c.h).  This package
holds its ctypes binding (romis_amd.restir), the host scene model (romis_amd.scene) and the build script
(romis_amd.build).  It never imports anything from oracle/ (test infrastructure).
"""
from . import _abi  # noqa: F401

__all__ = ["_abi"]
