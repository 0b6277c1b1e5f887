"""MI355X-native drop-in for the metabodecon Python module.

Same public surface as metabodecon-python/metabodecon/__init__.py and
_metabodecon.pyi (Deconvoluter, Deconvolution, Lorentzian, Spectrum,
exceptions); the deconvolution hot path runs as hand-written HIP kernels in
libmdgpu.so (C ABI: include/mdgpu.h). There is no CPU fallback.
"""
from . import exceptions
from ._deconvolution import Deconvoluter, Deconvolution, Lorentzian, superposition_vec
from ._spectrum import Spectrum

__version__ = "0.1.0+mi355x"

__all__ = [
    "__version__",
    "Deconvoluter",
    "Deconvolution",
    "Lorentzian",
    "Spectrum",
    "exceptions",
    "superposition_vec",
]
