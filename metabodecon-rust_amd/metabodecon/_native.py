"""ctypes binding of libmdgpu.so (the C ABI declared in include/mdgpu.h).

This is the only way the Python package reaches the hot path. There is no CPU
fallback: if the HIP library is missing or no MI355X is visible, the compute
entry points raise ``NativeLibraryError``/``DeviceUnavailableError`` loudly.
"""
from __future__ import annotations

import ctypes
import os
import threading
import weakref

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("MDGPU_LIB", os.path.join(_HERE, "libmdgpu.so"))

OK = 0
NO_PEAKS_DETECTED = 1
EMPTY_SIGNAL_REGION = 2
EMPTY_SIGNAL_FREE_REGION = 3
INVALID_SMOOTHING = 10
INVALID_SELECTION = 11
INVALID_FITTING = 12
INVALID_IGNORE_REGION = 13
INVALID_ARGUMENT = 20
CAPACITY = 21
REFERENCE_PANIC = 30
ERR_HIP = 100
ERR_NO_DEVICE = 101
ERR_OUT_OF_MEMORY = 102
OPTION_EXACT_MSE = 1  # mdg_settings.options (mdgpu.h MDG_OPTION_EXACT_MSE)

N_STAGES = 12
STAGE_NAMES = ["prep", "smooth", "detect", "select", "fit_init", "fit_superposition",
               "fit_update", "retain", "mse_superposition", "mse_exact", "superposition_vec",
               "synth"]

# every symbol include/mdgpu.h declares (checked by tests/test_capi_exports.py)
EXPORTS = [
    "mdg_abi_version", "mdg_build_info", "mdg_strerror", "mdg_settings_default", "mdg_settings_validate",
    "mdg_ignore_region_add", "mdg_synth_lorentzians", "mdg_synth_noise", "mdg_device_count",
    "mdg_host_alloc", "mdg_host_free",
    "mdg_ctx_create", "mdg_ctx_destroy", "mdg_ctx_set_stream", "mdg_ctx_synchronize",
    "mdg_ctx_set_profiling", "mdg_ctx_stage_times", "mdg_ctx_reset_stage_times",
    "mdg_deconvolute", "mdg_deconvolute_batch", "mdg_deconvolute_rows", "mdg_deconvolute_batch_device",
    "mdg_deconvolute_rows_i32", "mdg_decode_rows_i32_device",
    "mdg_superposition_vec", "mdg_superposition_vec_device", "mdg_synth_batch_device",
    "mdg_ctx_last_peaks", "mdg_ctx_last_smoothed", "mdg_ctx_last_range_flags",
    "mdg_ctx_set_profiling_mask",
    "mdg_optimize_settings", "mdg_ordered_sum", "mdg_check_fast_division",
    "mdg_check_division", "mdg_division_hard_case", "mdg_ctx_stage_kernel", "mdg_ctx_get_stream",
    "mdg_synth_lorentzians_hw", "mdg_synth_batch_device_hw",
    "mdg_queue_create", "mdg_queue_submit", "mdg_queue_flush", "mdg_queue_set_flush_us",
    "mdg_queue_synchronize",
    "mdg_queue_lane", "mdg_queue_stats", "mdg_queue_destroy", "mdg_queue_fail_next_launch",
    "mdg_jcampdx_decode", "mdg_ctx_set_latency_mode", "mdg_ctx_reload_switches", "mdg_ctx_set_tracing",
]


class NativeLibraryError(ImportError):
    pass


class DeviceUnavailableError(RuntimeError):
    pass


class Settings(ctypes.Structure):
    _fields_ = [
        ("smoother", ctypes.c_int32),
        ("smooth_iterations", ctypes.c_uint32),
        ("smooth_window", ctypes.c_uint32),
        ("selector", ctypes.c_int32),
        ("scoring", ctypes.c_int32),
        ("fit_iterations", ctypes.c_uint32),
        ("fitter", ctypes.c_int32),
        ("options", ctypes.c_int32),  # MDG_OPTION_* bits
        ("threshold", ctypes.c_double),
    ]

    def copy(self) -> "Settings":
        s = Settings()
        ctypes.memmove(ctypes.byref(s), ctypes.byref(self), ctypes.sizeof(Settings))
        return s


_dp = ctypes.POINTER(ctypes.c_double)
_szp = ctypes.POINTER(ctypes.c_size_t)
_i32p = ctypes.POINTER(ctypes.c_int32)
_u64p = ctypes.POINTER(ctypes.c_uint64)
_vp = ctypes.c_void_p
_sz = ctypes.c_size_t

_lib = None
_lib_lock = threading.Lock()

# the engine sources in the Makefile's order (SRC then HDR): their sha256 is compiled
# into the library (mdg_build_info) so a stale build is refused at load time
_PKG_ROOT = os.path.dirname(_HERE)
SOURCE_FILES = ["csrc/mdg_kernels.hip", "csrc/mdg_capi.hip", "csrc/mdg_jcampdx.cpp", "csrc/mdg_common.hpp",
                "csrc/mdg_kernels.hpp", "csrc/mdg_chain_asm.inc", "../include/mdgpu.h"]


def _default_hipflags(makefile: str) -> str | None:
    """The Makefile's default HIPFLAGS as make expands them (ARCH = gfx950), joined
    by single spaces as `echo` prints them."""
    import re
    try:
        text = open(makefile).read().replace("\\\n", " ")
    except OSError:
        return None
    m = re.search(r"^HIPFLAGS \?= (.*)$", text, re.M)
    if not m:
        return None
    return " ".join(m.group(1).replace("$(ARCH)", "gfx950").split())


def source_hash() -> str | None:
    """sha256 (first 16 hex digits) of the engine sources next to this package, as
    the Makefile computes it (SRC_HASH); None when the sources are not present."""
    import hashlib
    h = hashlib.sha256()
    for rel in SOURCE_FILES:
        path = os.path.join(_PKG_ROOT, rel)
        if not os.path.exists(path):
            return None
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


def flags_hash() -> str | None:
    """sha256 (16 hex digits) of the Makefile's default HIPFLAGS (FLAGS_HASH)."""
    import hashlib
    flags = _default_hipflags(os.path.join(_PKG_ROOT, "Makefile"))
    if flags is None:
        return None
    return hashlib.sha256((flags + "\n").encode()).hexdigest()[:16]


def _parse_build_info(raw: str) -> dict:
    out = {}
    head, _, comp = raw.partition(" compiler=")
    for tok in head.split():
        k, _, v = tok.partition("=")
        out[k] = v
    out["compiler"] = comp
    return out


def build_info() -> dict:
    """{"src": source hash the library was built from, "tree": hash of the sources
    here, "flags": hash of its compile flags, "default_flags": hash of the
    Makefile's defaults, "compiler": ..., "path": loaded library}."""
    b = _parse_build_info(lib().mdg_build_info().decode())
    return {"src": b.get("src"), "tree": source_hash(), "flags": b.get("flags"),
            "default_flags": flags_hash(), "compiler": b["compiler"],
            "path": os.path.realpath(LIB_PATH)}


def _share_torch_hip_runtime():
    """torch (ROCm wheel) bundles its own libamdhip64.so.7 with the same SONAME as
    /opt/rocm's. Whichever is loaded first serves every later NEEDED entry, so
    load torch's first: then libmdgpu and torch share ONE HIP runtime and device
    pointers/streams from torch are valid here (and torch keeps working)."""
    if os.environ.get("MDGPU_NO_TORCH"):
        return
    try:
        import torch  # noqa: F401  (loads libamdhip64 without initialising a device)
    except Exception:
        pass


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        with _lib_lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise NativeLibraryError(
                        f"libmdgpu.so not found at {LIB_PATH}; build it with "
                        "`make -C metabodecon-rust_amd` (hipcc, gfx950)")
                _share_torch_hip_runtime()
                L = ctypes.CDLL(LIB_PATH)
                _declare(L)
                _check_provenance(L)
                _lib = L
    return _lib


def _check_provenance(L):
    """Refuse a library built from other sources than the tree next to it (a stale
    build would silently run old kernels); MDGPU_ALLOW_STALE=1 skips the check. A
    build with other compile flags than the Makefile's defaults (make ARCH=..., an
    A/B -D override) is only reported: same sources, deliberate flags."""
    if os.environ.get("MDGPU_ALLOW_STALE"):
        return
    b = _parse_build_info(L.mdg_build_info().decode())
    tree = source_hash()
    if tree is not None and b.get("src") != tree:
        raise NativeLibraryError(
            f"{LIB_PATH} was built from sources {b.get('src')}, the tree has {tree}: rebuild it "
            "with `make -C metabodecon-rust_amd`")
    dflt = flags_hash()
    if dflt is not None and b.get("flags") != dflt:
        import warnings
        warnings.warn(f"{LIB_PATH} was built with non-default compile flags "
                      f"({b.get('flags')} != {dflt})", RuntimeWarning, stacklevel=3)


def _declare(L):
    sp = ctypes.POINTER(Settings)
    L.mdg_abi_version.restype = ctypes.c_int
    L.mdg_build_info.restype = ctypes.c_char_p
    L.mdg_strerror.argtypes = [ctypes.c_int]
    L.mdg_strerror.restype = ctypes.c_char_p
    L.mdg_settings_default.argtypes = [sp]
    L.mdg_settings_default.restype = None
    L.mdg_settings_validate.argtypes = [sp]
    L.mdg_ignore_region_add.argtypes = [_dp, _sz, _sz, ctypes.c_double, ctypes.c_double, _szp]
    L.mdg_synth_lorentzians.argtypes = [ctypes.c_uint64, _sz, ctypes.c_double, ctypes.c_double, _dp]
    L.mdg_synth_lorentzians_hw.argtypes = [ctypes.c_uint64, _sz, ctypes.c_double, ctypes.c_double,
                                           ctypes.c_double, _dp]
    L.mdg_synth_noise.argtypes = [ctypes.c_uint64, _sz, ctypes.c_double, _dp]
    L.mdg_device_count.argtypes = [ctypes.POINTER(ctypes.c_int)]
    L.mdg_host_alloc.argtypes = [ctypes.c_int, _sz, ctypes.POINTER(_vp)]
    L.mdg_host_free.argtypes = [_vp]
    L.mdg_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(_vp)]
    L.mdg_ctx_destroy.argtypes = [_vp]
    L.mdg_ctx_set_stream.argtypes = [_vp, _vp]
    L.mdg_ctx_get_stream.argtypes = [_vp, ctypes.POINTER(_vp)]
    L.mdg_ctx_synchronize.argtypes = [_vp]
    L.mdg_ctx_set_profiling.argtypes = [_vp, ctypes.c_int]
    L.mdg_ctx_set_profiling_mask.argtypes = [_vp, ctypes.c_uint32]
    L.mdg_ctx_stage_times.argtypes = [_vp, _dp, _u64p, ctypes.c_int]
    L.mdg_ctx_reset_stage_times.argtypes = [_vp]
    L.mdg_ctx_stage_kernel.argtypes = [_vp, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p)]
    L.mdg_ctx_set_latency_mode.argtypes = [_vp, ctypes.c_int]
    L.mdg_ctx_reload_switches.argtypes = [_vp]
    L.mdg_ctx_set_tracing.argtypes = [_vp, ctypes.c_int]
    L.mdg_deconvolute.argtypes = [_vp, _dp, _dp, _sz, ctypes.c_double, ctypes.c_double, sp, _dp,
                                  _sz, _dp, _sz, _szp, _dp]
    L.mdg_deconvolute_batch.argtypes = [_vp, _sz, _sz, _dp, _sz, _dp, _sz, _dp, sp, _dp, _sz,
                                        _dp, _sz, _szp, _dp, ctypes.POINTER(ctypes.c_int)]
    # the host-row entry points take plain addresses (ints) as well as ctypes pointers:
    # the per-call ctypes.cast of numpy's data_as costs ~4 us a pointer here, a dozen
    # per batched call (Deconvoluter._run_batch / _run_one)
    L.mdg_deconvolute_rows.argtypes = [_vp, _sz, _sz, _vp, _vp, _vp, sp, _vp, _sz, _vp, _sz, _vp,
                                       _vp, _vp]
    L.mdg_deconvolute_rows_i32.argtypes = [_vp, _sz, _sz, _vp, _vp, _vp, _vp, sp, _vp, _sz, _vp,
                                           _sz, _vp, _vp, _vp]
    L.mdg_decode_rows_i32_device.argtypes = [_vp, _sz, _sz, _vp, _vp, _vp, _vp]
    L.mdg_deconvolute_batch_device.argtypes = [_vp, _sz, _sz, _vp, _sz, _vp, _sz, _vp, sp, _dp,
                                               _sz, _vp, _sz, _vp, _vp, _vp]
    L.mdg_superposition_vec.argtypes = [_vp, _dp, _sz, _dp, _sz, _dp]
    L.mdg_superposition_vec_device.argtypes = [_vp, _vp, _sz, _vp, _sz, _vp]
    L.mdg_ctx_last_peaks.argtypes = [_vp, _sz, ctypes.c_int, _i32p, _i32p, _i32p, _sz, _szp]
    L.mdg_ctx_last_smoothed.argtypes = [_vp, _sz, _dp, _sz]
    L.mdg_ctx_last_range_flags.argtypes = [_vp, _sz, _i32p, ctypes.POINTER(ctypes.c_uint32), _i32p]
    L.mdg_optimize_settings.argtypes = [_vp, _dp, _dp, _sz, ctypes.c_double, ctypes.c_double, _dp,
                                        _sz, sp, _dp]
    L.mdg_ordered_sum.argtypes = [_vp, _dp, _sz, ctypes.c_double, _dp]
    L.mdg_check_fast_division.argtypes = [_vp, ctypes.c_uint64, ctypes.c_uint64, _u64p]
    L.mdg_check_division.argtypes = [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_uint64,
                                     ctypes.c_uint64, _u64p, _u64p]
    L.mdg_division_hard_case.argtypes = [ctypes.c_uint64, ctypes.c_uint64, _dp, _dp]
    L.mdg_synth_batch_device.argtypes = [_vp, _sz, _sz, ctypes.c_double, ctypes.c_double,
                                         ctypes.c_uint64, _sz, ctypes.c_double, ctypes.c_double,
                                         ctypes.c_double, _vp, _vp]
    L.mdg_queue_create.argtypes = [ctypes.c_int, _sz, _sz, ctypes.c_int, sp, _dp, _sz,
                                   ctypes.POINTER(_vp)]
    L.mdg_queue_submit.argtypes = [_vp, _vp, _vp, ctypes.c_double, ctypes.c_double, _vp, _sz, _vp,
                                   _vp, _vp]
    L.mdg_queue_flush.argtypes = [_vp]
    L.mdg_queue_set_flush_us.argtypes = [_vp, ctypes.c_int64]
    L.mdg_queue_synchronize.argtypes = [_vp]
    L.mdg_queue_lane.argtypes = [_vp, ctypes.c_int, ctypes.POINTER(_vp)]
    L.mdg_queue_stats.argtypes = [_vp, _u64p, _u64p, _szp]
    L.mdg_queue_destroy.argtypes = [_vp]
    L.mdg_queue_fail_next_launch.argtypes = [_vp, ctypes.c_int]
    L.mdg_jcampdx_decode.argtypes = [ctypes.c_char_p, _sz, ctypes.c_double, _dp, _sz, _szp]
    L.mdg_synth_batch_device_hw.argtypes = [_vp, _sz, _sz, ctypes.c_double, ctypes.c_double,
                                            ctypes.c_uint64, _sz, ctypes.c_double, ctypes.c_double,
                                            ctypes.c_double, ctypes.c_double, _vp, _vp]


def strerror(status: int) -> str:
    return lib().mdg_strerror(status).decode()


def default_settings() -> Settings:
    s = Settings()
    lib().mdg_settings_default(ctypes.byref(s))
    return s


def validate(s: Settings) -> int:
    return lib().mdg_settings_validate(ctypes.byref(s))


def ptr(a: np.ndarray, t=_dp):
    return a.ctypes.data_as(t)


_pinned_off = False  # no engine library or no device: ordinary memory from now on


def pinned_empty(shape, dtype=np.float64, device: int | None = None) -> np.ndarray | None:
    """An uninitialised C-contiguous array in page-locked host memory
    (mdg_host_alloc), released when the last view of it goes; None without the engine
    library or a device, or beyond MDGPU_PINNED_MAX, and the caller then keeps
    ordinary memory. The host-buffer calls DMA straight from and into such arrays
    (no bounce copy through the context's ring)."""
    global _pinned_off
    if _pinned_off:
        return None
    dt = np.dtype(dtype)
    count = int(np.prod(shape))
    nbytes = count * dt.itemsize
    if nbytes == 0:
        return None
    try:
        L = lib()
        if device is None:
            device = default_device()
    except (NativeLibraryError, OSError):
        _pinned_off = True
        return None
    p = _vp()
    st = L.mdg_host_alloc(device, nbytes, ctypes.byref(p))
    if st:
        if st == ERR_NO_DEVICE:
            _pinned_off = True
        return None
    buf = (ctypes.c_char * nbytes).from_address(p.value)
    weakref.finalize(buf, L.mdg_host_free, _vp(p.value))
    return np.frombuffer(buf, dtype=dt, count=count).reshape(shape)


def pinned_copy(a) -> np.ndarray:
    """A C-contiguous f64 copy of `a`, page-locked when pinned_empty can give it."""
    src = np.asarray(a, dtype=np.float64).reshape(-1)
    out = pinned_empty(src.shape)
    if out is None:
        return np.array(src, dtype=np.float64, copy=True)
    out[...] = src
    return out


class Context:
    """One device context (stream + reusable HBM workspace) of libmdgpu."""

    def __init__(self, device: int = 0):
        n = ctypes.c_int(0)
        lib().mdg_device_count(ctypes.byref(n))
        if n.value <= 0:
            raise DeviceUnavailableError(
                "no HIP device visible: the metabodecon GPU engine needs an MI355X "
                "(there is deliberately no CPU fallback)")
        h = _vp()
        st = lib().mdg_ctx_create(device, ctypes.byref(h))
        if st:
            raise DeviceUnavailableError(f"mdg_ctx_create({device}) failed: {strerror(st)}")
        self.handle = h
        self.device = device
        self.lock = threading.Lock()
        self._host: dict = {}  # host_rows / pinned_rows buffers
        _live.add(self)

    def host_rows(self, name: str, shape: tuple, dtype=np.float64) -> np.ndarray:
        """A C-contiguous host array of `shape` for this context's host-buffer calls
        (use it under self.lock), backed by a buffer kept across calls and grown
        geometrically. Fresh arrays of tens of MiB each call cost page faults, and a
        pageable copy into or out of memory HIP has not seen before is slow: a
        16-spectrum call with fresh stacked inputs and result rows spent ~8 ms there
        against ~1.2 ms of GPU time. Only the pages a call touches
        become resident."""
        dt = np.dtype(dtype)
        need = int(np.prod(shape)) * dt.itemsize
        buf = self._host.get(name)
        if buf is None or buf.nbytes < need:
            size = max(need, 2 * buf.nbytes if buf is not None else 0)
            # page-locked when possible: the results come back by DMA
            buf = pinned_empty((size,), np.uint8, self.device)
            if buf is None:
                buf = np.empty(size, dtype=np.uint8)
            self._host[name] = buf
        return buf[:need].view(dt).reshape(shape)

    def close(self):
        if getattr(self, "handle", None):
            lib().mdg_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover - interpreter shutdown order
        try:
            self.close()
        except Exception:
            pass

    def set_latency_mode(self, on: bool):
        """mdg_ctx_set_latency_mode: a one-spectrum pipeline of this context expects
        the GPU to itself (True, the engine's default) or shares it with other
        contexts running concurrently (False). Bit-identical results either way."""
        st = lib().mdg_ctx_set_latency_mode(self.handle, 1 if on else 0)
        if st:
            raise RuntimeError(strerror(st))

    def set_tracing(self, on: bool) -> bool:
        """roctx ranges around every pipeline stage of this context (rocprofv3
        --marker-trace attributes the kernels to stages); False when the roctx
        library is not available."""
        return lib().mdg_ctx_set_tracing(self.handle, 1 if on else 0) == 0

    def reload_switches(self):
        """Re-read the MDG_* engine switches from the environment (the engine reads
        them once, when the context is created)."""
        if getattr(self, "handle", None):
            lib().mdg_ctx_reload_switches(self.handle)

    def set_stream(self, stream_ptr: int | None):
        lib().mdg_ctx_set_stream(self.handle, _vp(stream_ptr or 0))

    def stream(self) -> int:
        """hipStream_t (as an int) the context enqueues on."""
        p = _vp()
        lib().mdg_ctx_get_stream(self.handle, ctypes.byref(p))
        return p.value or 0

    def synchronize(self):
        st = lib().mdg_ctx_synchronize(self.handle)
        if st:
            raise RuntimeError(strerror(st))

    def set_profiling(self, on: bool):
        lib().mdg_ctx_set_profiling(self.handle, 1 if on else 0)

    def set_profiling_stages(self, names):
        """Time only the named stages (STAGE_NAMES) with hipEvents."""
        mask = 0
        for n in names:
            mask |= 1 << STAGE_NAMES.index(n)
        lib().mdg_ctx_set_profiling_mask(self.handle, mask)

    def stage_times(self) -> dict:
        ms = np.zeros(N_STAGES)
        n = np.zeros(N_STAGES, dtype=np.uint64)
        lib().mdg_ctx_stage_times(self.handle, ptr(ms), ptr(n, _u64p), N_STAGES)
        return {STAGE_NAMES[i]: (float(ms[i]), int(n[i])) for i in range(N_STAGES)}

    def stage_kernels(self) -> dict:
        """Kernel names the last pipeline run launched, per stage (mdg_ctx_stage_kernel)."""
        out = {}
        for i, name in enumerate(STAGE_NAMES):
            p = ctypes.c_char_p()
            lib().mdg_ctx_stage_kernel(self.handle, i, ctypes.byref(p))
            if p.value:
                out[name] = p.value.decode()
        return out

    def last_range_flags(self, spectrum: int) -> tuple[int, int, int]:
        """(x_ok, slow_mask, unsafe_kept) of `spectrum` from the last batch run (test
        hook, mdg_ctx_last_range_flags): which launches took the plain division."""
        xo, uk = ctypes.c_int32(0), ctypes.c_int32(0)
        m = ctypes.c_uint32(0)
        st = lib().mdg_ctx_last_range_flags(self.handle, spectrum, ctypes.byref(xo), ctypes.byref(m),
                                            ctypes.byref(uk))
        if st:
            raise RuntimeError(strerror(st))
        return xo.value, m.value, uk.value

    def last_smoothed(self, spectrum: int, n: int) -> np.ndarray:
        """Smoothed intensities of `spectrum` from the last batch run (diagnostic)."""
        out = np.empty(n, dtype=np.float64)
        st = lib().mdg_ctx_last_smoothed(self.handle, spectrum, ptr(out), n)
        if st:
            raise RuntimeError(strerror(st))
        return out

    def last_peaks(self, spectrum: int, which: str = "selected") -> np.ndarray:
        """(count, 3) int32 (left, center, right) of the last batch run."""
        k = 0 if which == "detected" else 1
        cnt = ctypes.c_size_t(0)
        lib().mdg_ctx_last_peaks(self.handle, spectrum, k, None, None, None, 0, ctypes.byref(cnt))
        n = cnt.value
        l, c, r = (np.zeros(max(n, 1), dtype=np.int32) for _ in range(3))
        st = lib().mdg_ctx_last_peaks(self.handle, spectrum, k, ptr(l, _i32p), ptr(c, _i32p),
                                      ptr(r, _i32p), n, ctypes.byref(cnt))
        if st:
            raise RuntimeError(strerror(st))
        return np.stack([l[:n], c[:n], r[:n]], axis=1)

    def reset_stage_times(self):
        lib().mdg_ctx_reset_stage_times(self.handle)


class _LaneView(Context):
    """A queue lane's engine context (owned by the queue: never destroyed here)."""

    def __init__(self, handle, device):  # noqa: D107 (no Context.__init__: no new context)
        self.handle = handle
        self.device = device
        self.lock = threading.Lock()

    def close(self):
        self.handle = None


class SpectrumQueue:
    """mdg_queue: single-spectrum submissions on device arrays, gathered into
    batches of up to `max_batch` spectra that run one pipeline each on `lanes`
    engine contexts (include/mdgpu.h). The serving form of many concurrent
    ``Deconvoluter.par_deconvolute_spectrum`` calls."""

    def __init__(self, device: int, n: int, max_batch: int, lanes: int, settings: Settings,
                 ignore: np.ndarray | None = None):
        c = ctypes.c_int(0)
        lib().mdg_device_count(ctypes.byref(c))
        if c.value <= 0:
            raise DeviceUnavailableError("no HIP device visible: the metabodecon GPU engine "
                                         "needs an MI355X (there is deliberately no CPU fallback)")
        ign = np.zeros(0) if ignore is None else np.ascontiguousarray(ignore, dtype=np.float64)
        h = _vp()
        st = lib().mdg_queue_create(device, n, max_batch, lanes, ctypes.byref(settings),
                                    ptr(ign) if ign.size else None, ign.size // 2, ctypes.byref(h))
        if st:
            raise RuntimeError(f"mdg_queue_create failed: {strerror(st)}")
        self.handle, self.device, self.n = h, device, n
        self.max_batch, self.lanes = max_batch, lanes
        _live.add(self)

    def reload_switches(self):
        """Re-read the MDG_* engine switches on every lane context."""
        if getattr(self, "handle", None):
            for k in range(self.lanes):
                self.lane(k).reload_switches()

    def submit(self, x_ptr: int, y_ptr: int, sb, out_ptr: int, cap: int, count_ptr: int,
               mse_ptr: int, status_ptr: int) -> None:
        st = lib().mdg_queue_submit(self.handle, x_ptr, y_ptr, float(sb[0]), float(sb[1]), out_ptr,
                                    cap, count_ptr, mse_ptr, status_ptr)
        if st:
            raise RuntimeError(f"mdg_queue_submit: {strerror(st)}")

    def flush(self) -> None:
        st = lib().mdg_queue_flush(self.handle)
        if st:
            raise RuntimeError(f"mdg_queue_flush: {strerror(st)}")

    def set_flush_us(self, us: int) -> None:
        """Launch the open batch once its first submission has waited `us` µs (0: off)."""
        st = lib().mdg_queue_set_flush_us(self.handle, int(us))
        if st:
            raise RuntimeError(f"mdg_queue_set_flush_us: {strerror(st)}")

    def synchronize(self) -> None:
        st = lib().mdg_queue_synchronize(self.handle)
        if st:
            raise RuntimeError(f"mdg_queue_synchronize: {strerror(st)}")

    def fail_next_launch(self, status: int) -> None:
        """Test support: the next batch launch fails with `status` (sticky afterwards)."""
        st = lib().mdg_queue_fail_next_launch(self.handle, int(status))
        if st:
            raise RuntimeError(strerror(st))

    def lane(self, k: int) -> Context:
        h = _vp()
        st = lib().mdg_queue_lane(self.handle, k, ctypes.byref(h))
        if st:
            raise RuntimeError(strerror(st))
        return _LaneView(h, self.device)

    def stats(self) -> dict:
        b, s = ctypes.c_uint64(0), ctypes.c_uint64(0)
        o = ctypes.c_size_t(0)
        lib().mdg_queue_stats(self.handle, ctypes.byref(b), ctypes.byref(s), ctypes.byref(o))
        return {"batches": b.value, "spectra": s.value, "open": o.value}

    def close(self):
        if getattr(self, "handle", None):
            lib().mdg_queue_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


_ctx: dict[int, Context] = {}
_ctx_lock = threading.Lock()
# every live Context / SpectrumQueue, for reload_switches
_live: "weakref.WeakSet" = weakref.WeakSet()


def reload_switches() -> None:
    """Re-read the MDG_* engine switches (tests, measurements) on every live context
    and queue of this process: the engine reads the environment only when a context
    is created, never on a call's path."""
    for obj in list(_live):
        obj.reload_switches()


def device_count() -> int:
    n = ctypes.c_int(0)
    lib().mdg_device_count(ctypes.byref(n))
    return n.value


def default_device() -> int:
    """MDGPU_DEVICE if set; else LOCAL_RANK modulo the visible devices (one process
    per GPU under torchrun sees all GPUs and takes its own; a launcher that exposes
    one GPU per rank, HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES, leaves device 0);
    else 0."""
    env = os.environ.get("MDGPU_DEVICE")
    if env is not None:
        return int(env)
    env = os.environ.get("LOCAL_RANK")
    if env is not None:
        n = device_count()
        return int(env) % n if n > 0 else 0
    return 0


def context(device: int | None = None) -> Context:
    if device is None:
        device = default_device()
    with _ctx_lock:
        c = _ctx.get(device)
        if c is None:
            c = Context(device)
            _ctx[device] = c
        return c


_lanes: dict[int, list[Context]] = {}


def lane_contexts(device: int | None, n: int) -> list[Context]:
    """n engine contexts on `device` (each its own HIP stream and workspace), for
    spectra deconvoluted concurrently; created on first use and kept."""
    if device is None:
        device = default_device()
    with _ctx_lock:
        lanes = _lanes.setdefault(device, [])
        while len(lanes) < n:
            c = Context(device)
            c.set_latency_mode(False)  # lanes run concurrently: no B = 1 pipeline has the GPU to itself
            lanes.append(c)
        return lanes[:n]


def release_context(device: int | None = None) -> None:
    """Destroy the shared context of `device` (all devices when None): its idle stream
    holds a hardware queue. It is re-created by the next call that needs it."""
    with _ctx_lock:
        for d in ([device] if device is not None else list(_ctx)):
            c = _ctx.pop(d, None)
            if c is not None:
                with c.lock:
                    c.close()


def release_lanes(device: int | None = None) -> None:
    """Destroy the lane contexts of `device` (all devices when None): their idle
    streams still hold hardware queues, and with 16 of them alive a single-stream
    pipeline on the same GPU ran ~15% slower. They are re-created on
    the next concurrent call."""
    with _ctx_lock:
        for d in ([device] if device is not None else list(_lanes)):
            for c in _lanes.pop(d, []):
                with c.lock:
                    c.close()
