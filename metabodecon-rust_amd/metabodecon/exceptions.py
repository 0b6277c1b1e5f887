"""Exception hierarchy of the reference's Python module.

Mirrors metabodecon-python/src/error.rs:5-28 (create_exception! tree) and
metabodecon/exceptions.pyi, so ``except metabodecon.exceptions.NoPeaksDetected``
works unchanged against this engine.
"""


class Error(Exception):
    """Base class for all Metabodecon errors."""


class UnexpectedError(Error):
    """An unexpected error occurred."""


class ThreadPoolError(Error):
    """Thread pool construction failed."""


class SerializationError(Error):
    """Serialization or deserialization failed."""


class SpectrumError(Error):
    """Errors of the Spectrum class."""


class EmptyData(SpectrumError):
    """Input data is empty."""


class DataLengthMismatch(SpectrumError):
    """Input data lengths do not match."""


class NonUniformSpacing(SpectrumError):
    """Chemical shifts are not uniformly spaced."""


class InvalidIntensities(SpectrumError):
    """Intensities contain invalid values."""


class InvalidSignalBoundaries(SpectrumError):
    """Signal boundaries are invalid."""


class MissingMetadata(SpectrumError):
    """Metadata is missing from an NMR format file."""


class MalformedMetadata(SpectrumError):
    """Metadata in an NMR format file is malformed."""


class MissingData(SpectrumError):
    """An NMR format file contains no data."""


class MalformedData(SpectrumError):
    """Data in an NMR format file is malformed."""


class DeconvolutionError(Error):
    """Errors during the deconvolution process."""


class InvalidSmoothingSettings(DeconvolutionError):
    """Smoothing settings are invalid."""


class InvalidSelectionSettings(DeconvolutionError):
    """Peak selection settings are invalid."""


class InvalidFittingSettings(DeconvolutionError):
    """Peak fitting settings are invalid."""


class InvalidIgnoreRegion(DeconvolutionError):
    """Ignore region boundaries are invalid."""


class NoPeaksDetected(DeconvolutionError):
    """No peaks were detected in the spectrum."""


class EmptySignalRegion(DeconvolutionError):
    """Signal region contains no peaks."""


class EmptySignalFreeRegion(DeconvolutionError):
    """Signal-free region contains no peaks."""


# mdg_status -> exception (metabodecon-python/src/error.rs:45-96 mapping)
_STATUS = {
    1: (NoPeaksDetected, "no peaks detected in the spectrum"),
    2: (EmptySignalRegion, "no peaks found in the signal region of the spectrum"),
    3: (EmptySignalFreeRegion, "no peaks found in the signal-free region of the spectrum"),
    10: (InvalidSmoothingSettings, "invalid smoothing settings"),
    11: (InvalidSelectionSettings, "invalid selection settings"),
    12: (InvalidFittingSettings, "invalid fitting settings"),
    13: (InvalidIgnoreRegion, "invalid ignore region"),
}


def from_status(status: int, detail: str | None = None) -> Exception:
    cls, msg = _STATUS.get(status, (UnexpectedError, f"unexpected error: status {status}"))
    if status == 30:
        msg = "the reference implementation panics on this input (slice bounds)"
    return cls(detail or msg)
