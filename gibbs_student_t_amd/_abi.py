"""ctypes binding of libgst.so (C ABI declared in include/gst.h).

The product path has no CPU fallback: if the shared library is missing or cannot be
loaded, ``load()`` raises ``GstNativeError``.
"""
from __future__ import annotations

import ctypes as ct
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libgst.so")

GST_MODEL_GAUSSIAN, GST_MODEL_T, GST_MODEL_MIXTURE, GST_MODEL_VVH17 = 0, 1, 2, 3
STAGE_WHITE, STAGE_HYPER, STAGE_B = 1, 2, 4
STAGE_THETA, STAGE_Z, STAGE_ALPHA, STAGE_DF = 8, 16, 32, 64
STAGE_ALL = 0x7F
STAGE_B_FORCE = 0x80
STAGE_GRAM = 0x100          # timing diagnostic: Gram + timing-model elimination only
TAPE_WHITE, TAPE_HYPER, TAPE_DELTA = 0, 80, 120
PATH_AUTO, PATH_PERSISTENT, PATH_LARGE = 0, 1, 2
DEBUG_POISON = 1
DEBUG_LARGE_GRAM = 2
DEBUG_LARGE_HYPER = 4
DEBUG_EXACT_BDRAW = 8
DEBUG_MFMA_GRAM = 16
DEBUG_EPOCHS_LDS = 32
STATUS_FLOOR = 16          # status bit 4: a b draw ran at the SVD noise floor
STATUS_FLAGS = 0xff        # bits 0-7: flags; bits 8..30: the number of floor draws (ABI 5)
STATUS_ERRORS = STATUS_FLAGS & ~STATUS_FLOOR   # every flag but the informational floor bit
STATUS_FLOOR_COUNT_SHIFT = 8


def floor_draws(status):
    """Per chain: the b draws made at the SVD noise floor since status was last zeroed."""
    import numpy as np
    return np.asarray(status) >> STATUS_FLOOR_COUNT_SHIFT
PATHS = {"auto": PATH_AUTO, "persistent": PATH_PERSISTENT, "large": PATH_LARGE}
KERNEL_KINDS = ("record", "white", "gram", "tmelim", "hyper", "btm", "tb", "toa")

ABI_VERSION = 6
EXPORTS = ("gst_version", "gst_tape_stride", "gst_last_error", "gst_ctx_create",
           "gst_ctx_destroy", "gst_model_set", "gst_model_set_batch", "gst_model_info",
           "gst_sweep", "gst_set_path", "gst_get_path", "gst_set_waves", "gst_set_debug", "gst_set_timing", "gst_kernel_times", "gst_eval_lnlike", "gst_sync",
           "gst_last_sweep_ms", "gst_debug_stamps", "gst_simulate",
           # ABI 6
           "gst_gram_counts", "gst_debug_variates")

# diagnostics that older builds (A/B timing of library variants) may lack; calling one on
# such a build raises AttributeError
OPTIONAL = ("gst_set_debug", "gst_gram_counts", "gst_debug_variates")

_P = ct.POINTER
_D = _P(ct.c_double)
_I = _P(ct.c_int)


class GstNativeError(RuntimeError):
    pass


class ModelDesc(ct.Structure):
    _fields_ = [
        ("n", ct.c_int), ("m", ct.c_int), ("nfourier", ct.c_int), ("ntm", ct.c_int),
        ("nparams", ct.c_int),
        ("T", _D), ("residuals", _D), ("toaerrs", _D), ("ffreqs", _D),
        ("tm_weight", ct.c_double),
        ("idx_efac", ct.c_int), ("idx_equad", ct.c_int), ("idx_log10_A", ct.c_int),
        ("idx_gamma", ct.c_int),
        ("efac_const", ct.c_double),
        ("pmin", _D), ("pmax", _D),
        ("hyper_idx", _I), ("n_hyper", ct.c_int), ("white_idx", _I), ("n_white", ct.c_int),
        ("model", ct.c_int), ("vary_df", ct.c_int), ("vary_alpha", ct.c_int),
        ("theta_prior_beta", ct.c_int), ("mprior", ct.c_double), ("pspin", ct.c_double),
        ("df_A", _D), ("df_B", _D),
        # ABI 3: general white noise (per-backend parameters, ECORR basis columns)
        ("nbackend", ct.c_int), ("backend", _I), ("efac_idx", _I), ("equad_idx", _I),
        ("ecorr_idx", _I), ("n_ecorr", ct.c_int), ("ecorr_backend", _I),
    ]


class State(ct.Structure):
    _fields_ = [("x", ct.c_void_p), ("b", ct.c_void_p), ("z", ct.c_void_p),
                ("alpha", ct.c_void_p), ("pout", ct.c_void_p), ("theta", ct.c_void_p),
                ("nu", ct.c_void_p), ("status", ct.c_void_p), ("dataset", ct.c_void_p)]


class Records(ct.Structure):
    _fields_ = [("x", ct.c_void_p), ("b", ct.c_void_p), ("z", ct.c_void_p),
                ("alpha", ct.c_void_p), ("pout", ct.c_void_p), ("theta", ct.c_void_p),
                ("nu", ct.c_void_p), ("nrec", ct.c_int)]


class Tape(ct.Structure):
    _fields_ = [("data", ct.c_void_p), ("stride", ct.c_int)]


class SimDesc(ct.Structure):
    """gst_sim_desc (device pointers)."""
    _fields_ = [("n", ct.c_int), ("nfourier", ct.c_int), ("ntm", ct.c_int),
                ("ndatasets", ct.c_int),
                ("F", ct.c_void_p), ("log_f", ct.c_void_p), ("log_df", ct.c_void_p),
                ("log_fyr", ct.c_double), ("U", ct.c_void_p), ("red", ct.c_void_p),
                ("toaerrs", ct.c_void_p), ("theta", ct.c_void_p), ("sigma_out", ct.c_void_p),
                ("log10_A", ct.c_void_p), ("gamma", ct.c_void_p), ("dof", ct.c_void_p),
                ("seed", ct.c_ulonglong), ("dataset0", ct.c_longlong),
                ("residuals", ct.c_void_p), ("toaerrs_out", ct.c_void_p), ("z", ct.c_void_p),
                ("residuals_clean", ct.c_void_p)]


_lib = None


def load(path: str | None = None):
    """Load libgst.so once; raise GstNativeError if it is absent or broken."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or os.environ.get("GST_LIB", LIB_PATH)
    # PyTorch owns the device buffers: its HIP runtime must be the one libgst binds to
    # (same soname libamdhip64.so.7), so import it before dlopen-ing the library.
    try:
        import torch  # noqa: F401
    except ImportError:  # pragma: no cover
        pass
    if not os.path.exists(p):
        raise GstNativeError(
            f"native library {p} not found: build it with `python __graft_entry__.py` "
            "(hipcc --offload-arch=gfx950); there is no CPU fallback")
    try:
        lib = ct.CDLL(p)
    except OSError as e:  # pragma: no cover - depends on the machine
        raise GstNativeError(f"cannot load {p}: {e}") from e
    for name in EXPORTS:
        if not hasattr(lib, name) and name not in OPTIONAL:
            raise GstNativeError(f"{p} lacks symbol {name}")
    lib.gst_version.restype = ct.c_int
    lib.gst_tape_stride.argtypes = [ct.c_int, ct.c_int]
    lib.gst_last_error.argtypes = [ct.c_char_p, ct.c_size_t]
    lib.gst_ctx_create.argtypes = [ct.c_int, _P(ct.c_void_p)]
    lib.gst_ctx_destroy.argtypes = [ct.c_void_p]
    lib.gst_model_set.argtypes = [ct.c_void_p, _P(ModelDesc)]
    lib.gst_model_set_batch.argtypes = [ct.c_void_p, _P(ModelDesc), ct.c_int]
    lib.gst_model_info.argtypes = [ct.c_void_p, _P(ct.c_int), _P(ct.c_int), _P(ct.c_int)]
    lib.gst_sweep.argtypes = [ct.c_void_p, _P(State), _P(Records), _P(Tape), ct.c_int,
                              ct.c_int, ct.c_longlong, ct.c_int, ct.c_uint, ct.c_ulonglong,
                              ct.c_longlong, ct.c_void_p]
    lib.gst_eval_lnlike.argtypes = [ct.c_void_p, _P(State), ct.c_int, ct.c_void_p,
                                    ct.c_void_p, ct.c_void_p]
    lib.gst_sync.argtypes = [ct.c_void_p, ct.c_void_p]
    lib.gst_set_path.argtypes = [ct.c_void_p, ct.c_int]
    lib.gst_get_path.argtypes = [ct.c_void_p, _P(ct.c_int)]
    lib.gst_set_waves.argtypes = [ct.c_void_p, ct.c_int]
    if hasattr(lib, "gst_set_debug"):
        lib.gst_set_debug.argtypes = [ct.c_void_p, ct.c_int]
    lib.gst_set_timing.argtypes = [ct.c_void_p, ct.c_int]
    lib.gst_kernel_times.argtypes = [ct.c_void_p, _P(ct.c_double), _P(ct.c_int), ct.c_int]
    lib.gst_last_sweep_ms.argtypes = [ct.c_void_p, _P(ct.c_double)]
    lib.gst_debug_stamps.argtypes = [ct.c_void_p, ct.c_void_p]
    lib.gst_simulate.argtypes = [_P(SimDesc), ct.c_void_p]
    if hasattr(lib, "gst_gram_counts"):
        lib.gst_gram_counts.argtypes = [ct.c_void_p, _P(ct.c_longlong), ct.c_int]
    if hasattr(lib, "gst_debug_variates"):
        lib.gst_debug_variates.argtypes = [ct.c_int, ct.c_double, ct.c_double, ct.c_longlong,
                                           ct.c_ulonglong, ct.c_uint, ct.c_void_p, ct.c_void_p]
    for name in EXPORTS:
        if name != "gst_version" and hasattr(lib, name):
            getattr(lib, name).restype = ct.c_int
    if lib.gst_version() != ABI_VERSION and not os.environ.get("GST_ALLOW_ABI_MISMATCH"):
        # (A/B timing of an older build of the classic model sets GST_ALLOW_ABI_MISMATCH:
        # ABI 3 only appended descriptor fields that such a build ignores)
        raise GstNativeError(f"{p}: ABI version {lib.gst_version()} != {ABI_VERSION}; rebuild")
    if path is None:
        _lib = lib
    return lib


def last_error(lib) -> str:
    buf = ct.create_string_buffer(1024)
    lib.gst_last_error(buf, len(buf))
    return buf.value.decode(errors="replace")


def check(lib, rc: int, what: str):
    if rc != 0:
        raise GstNativeError(f"{what} failed: {last_error(lib)}")
