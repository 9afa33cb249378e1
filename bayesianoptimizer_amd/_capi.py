"""ctypes binding of libgpx.so (include/gpx.h).

This is the only place Python touches the native library.  The library is built in-tree
(``bayesianoptimizer_amd/lib/libgpx.so``, see ``__graft_entry__.build``); if it is missing the import of
the engine fails loudly — there is no CPU fallback on the product path.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import re
import sys
from ctypes import POINTER, c_char_p, c_double, c_int32, c_int64, c_size_t, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GPX_LIB", os.path.join(_HERE, "lib", "libgpx.so"))
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "gpx.h")

GPX_MAX_DIM = 32
GPX_MAX_RHS = 8
GPX_TILE = 128
GPX_MAX_Q = 32
GPX_MAX_GRAD_CANDIDATES = 16384
GPX_COMM_ID_BYTES = 128

GPX_OK, GPX_NOT_PD, GPX_INVALID_ARG, GPX_HIP_ERROR, GPX_RCCL_ERROR, GPX_TIMEOUT = 0, 1, 2, 3, 4, 5
STATUS_NAMES = {0: "OK", 1: "NOT_PD", 2: "INVALID_ARG", 3: "HIP_ERROR", 4: "RCCL_ERROR", 5: "TIMEOUT"}
GPX_INFO_TIMEOUT = -(2 ** 31)  # device info word of a factorisation / solve whose in-launch hand-off timed out

# per-handle options (include/gpx.h GPX_OPT_*; slot 0 is GPX_OPT_RESERVED_0, the removed potrf_schedule)
OPTIONS = {"spin_limit": 1, "sweep_fused": 2, "gram_split": 3, "potrf_lazy": 4, "potrf_mode": 5, "potrf_switch": 6,
           "potrf_split": 7}
GPX_OPT_RESERVED = (0,)
GPX_OPT_COUNT = len(OPTIONS) + len(GPX_OPT_RESERVED)

KERNEL_RBF, KERNEL_MATERN52, KERNEL_SCALE_LINEAR_MATERN52 = 0, 1, 2
ACQ_EI, ACQ_LOGEI, ACQ_UCB, ACQ_VARIANCE = 0, 1, 2, 3
TIMERS = {"gram": 0, "potrf": 1, "trtri": 2, "alpha": 3, "kstar": 4, "trmm": 5, "acq": 6, "mll": 7}

# gpx_mll_grad_f64 output layout (include/gpx.h)
MLL_NLL, MLL_QUAD, MLL_LOGDET, MLL_D_NOISE, MLL_D_OUTPUTSCALE, MLL_D_MEAN = 0, 1, 2, 3, 4, 5
MLL_D_LENGTHSCALE, MLL_D_LINVAR, MLL_NOUT = 8, 40, 72


class GPXLibraryError(RuntimeError):
    """libgpx.so is missing or failed to load (the HIP path is required; there is no fallback)."""


class GPXError(RuntimeError):
    def __init__(self, status: int, message: str):
        super().__init__(f"gpx {STATUS_NAMES.get(status, status)}: {message}")
        self.status = status


class NotPositiveDefiniteError(GPXError):
    """Raised when the Cholesky of K(X,X)+noise*I fails; ``pivot`` is 0-based (reference retries with
    a larger jitter, optimization/Bayesian6.py:481-488)."""

    def __init__(self, pivot: int, message: str = ""):
        super().__init__(GPX_NOT_PD, message or f"matrix not positive definite at pivot {pivot}")
        self.pivot = pivot


class GPXTimeoutError(GPXError):
    """A persistent launch (the triangular solve) gave up on an in-launch hand-off after its
    bounded spin: the factor / alpha of that call are invalid.  Distinct from NotPositiveDefiniteError, because a larger
    jitter (the reference's retry, optimization/Bayesian6.py:481-488) does not cure it."""

    def __init__(self, message: str = ""):
        super().__init__(GPX_TIMEOUT, message or "in-launch hand-off timed out (GPX_OPT_SPIN_LIMIT)")


def info_error(value: int, what: str = ""):
    """The exception a device ``info`` word stands for (None for 0): NotPositiveDefiniteError for a failed pivot
    (value = pivot + 1 > 0), GPXTimeoutError for GPX_INFO_TIMEOUT (any negative value)."""
    value = int(value)
    prefix = f"{what}: " if what else ""
    if value > 0:
        return NotPositiveDefiniteError(value - 1, f"{prefix}not positive definite at pivot {value - 1}")
    if value < 0:
        return GPXTimeoutError(f"{prefix}in-launch hand-off timed out (info {value})")
    return None


class KernelParamsC(ctypes.Structure):
    _fields_ = [
        ("kind", c_int32),
        ("d", c_int32),
        ("lengthscale", c_double * GPX_MAX_DIM),
        ("linear_variance", c_double * GPX_MAX_DIM),
        ("outputscale", c_double),
        ("noise", c_double),
        ("jitter", c_double),
        ("const_mean", c_double),
        ("cov_fp32", c_int32),
        ("reserved", c_int32),
    ]


class AcqParamsC(ctypes.Structure):
    _fields_ = [
        ("kind", c_int32),
        ("reserved", c_int32),
        ("best_f", c_double),
        ("beta", c_double),
        ("y_mean", c_double),
        ("y_scale", c_double),
    ]


_h = c_void_p
_p = c_void_p  # device pointers
_PROTOS = {
    "gpx_version": (c_char_p, []),
    "gpx_create": (c_int32, [c_int32, POINTER(c_void_p)]),
    "gpx_destroy": (c_int32, [_h]),
    "gpx_set_stream": (c_int32, [_h, c_void_p]),
    "gpx_last_error": (c_char_p, [_h]),
    "gpx_padded_n": (c_int64, [c_int64]),
    "gpx_kernel_params_size": (c_size_t, []),
    "gpx_acq_params_size": (c_size_t, []),
    "gpx_set_option": (c_int32, [_h, c_int32, c_int64]),
    "gpx_get_option": (c_int32, [_h, c_int32, POINTER(c_int64)]),
    "gpx_gram_f64": (c_int32, [_h, POINTER(KernelParamsC), c_int64, _p, c_int64, _p, c_int64]),
    "gpx_potrf_f64": (c_int32, [_h, c_int64, _p, c_int64, _p, _p]),
    "gpx_trtri_workspace_size": (c_int32, [c_int64, POINTER(c_size_t)]),
    "gpx_trtri_f64": (c_int32, [_h, c_int64, _p, c_int64, _p, _p, c_int64, _p, c_size_t]),
    "gpx_trtri_batched_workspace_size": (c_int32, [c_int64, c_int64, POINTER(c_size_t)]),
    "gpx_trtri_batched_f64": (c_int32, [_h, c_int64, c_int64, _p, c_int64, c_int64, _p, c_int64, _p, c_int64, c_int64,
                                        _p, c_size_t]),
    "gpx_alpha_workspace_size": (c_int32, [c_int64, c_int64, POINTER(c_size_t)]),
    "gpx_alpha_f64": (c_int32, [_h, c_int64, _p, c_int64, _p, c_int64, c_int64, c_double, _p, _p, c_size_t]),
    "gpx_fit_workspace_size": (c_int32, [c_int64, c_int64, POINTER(c_size_t)]),
    "gpx_fit_f64": (c_int32, [_h, POINTER(KernelParamsC), c_int64, _p, c_int64, _p, c_int64, c_int64, _p, c_int64,
                              _p, _p, c_int64, _p, _p, _p, c_size_t]),
    "gpx_fit_f64_sync": (c_int32, [_h, POINTER(KernelParamsC), c_int64, _p, c_int64, _p, c_int64, c_int64, _p,
                                   c_int64, _p, _p, c_int64, _p, _p, _p, c_size_t, POINTER(c_int32)]),
    "gpx_fit_batched_workspace_size": (c_int32, [c_int64, c_int64, c_int64, POINTER(c_size_t)]),
    "gpx_fit_batched_f64": (c_int32, [_h, POINTER(KernelParamsC), c_int64, c_int64, _p, c_int64, c_int64, _p,
                                      c_int64, c_int64, c_int64, _p, c_int64, c_int64, _p, c_int64, _p, c_int64,
                                      c_int64, _p, c_int64, _p, _p, c_size_t]),
    "gpx_fit_batched_params_f64": (c_int32, [_h, POINTER(KernelParamsC), c_int64, c_int64, _p, c_int64, c_int64, _p,
                                             c_int64, c_int64, c_int64, _p, c_int64, c_int64, _p, c_int64, _p, c_int64,
                                             c_int64, _p, c_int64, _p, _p, c_size_t]),
    "gpx_fit_factor_batched_params_f64": (c_int32, [_h, POINTER(KernelParamsC), c_int64, c_int64, _p, c_int64, c_int64,
                                                    _p, c_int64, c_int64, c_int64, _p, c_int64, c_int64, _p, c_int64,
                                                    _p, c_int64, _p, _p, c_size_t]),
    "gpx_potrs_workspace_size": (c_int32, [c_int64, c_int64, POINTER(c_size_t)]),
    "gpx_potrs_f64": (c_int32, [_h, c_int64, _p, c_int64, _p, _p, c_int64, c_int64, c_double, _p, _p, _p, c_size_t]),
    "gpx_fit_factor_workspace_size": (c_int32, [c_int64, c_int64, POINTER(c_size_t)]),
    "gpx_fit_factor_f64": (c_int32, [_h, POINTER(KernelParamsC), c_int64, _p, c_int64, _p, c_int64, c_int64, _p,
                                     c_int64, _p, _p, _p, _p, c_size_t]),
    "gpx_fit_factor_batched_workspace_size": (c_int32, [c_int64, c_int64, c_int64, POINTER(c_size_t)]),
    "gpx_fit_factor_batched_f64": (c_int32, [_h, POINTER(KernelParamsC), c_int64, c_int64, _p, c_int64, c_int64, _p,
                                             c_int64, c_int64, c_int64, _p, c_int64, c_int64, _p, c_int64, _p, c_int64,
                                             _p, _p, c_size_t]),
    "gpx_append_workspace_size": (c_int32, [c_int64, c_int64, c_int64, POINTER(c_size_t)]),
    "gpx_append_f64": (c_int32, [_h, POINTER(KernelParamsC), c_int64, c_int64, _p, c_int64, _p, c_int64, c_int64, _p,
                                 c_int64, _p, _p, c_int64, _p, _p, _p, c_size_t]),
    "gpx_moments_grad_workspace_size": (c_int32, [c_int64, c_int64, POINTER(c_size_t)]),
    "gpx_moments_grad_f64": (c_int32, [_h, POINTER(KernelParamsC), c_int64, _p, c_int64, _p, c_int64, _p, _p, c_int64,
                                       c_int64, c_int64, _p, _p, _p, _p, _p, c_size_t]),
    "gpx_sweep_workspace_size": (c_int32, [c_int64, c_int64, c_int64, POINTER(c_size_t)]),
    "gpx_posterior_f64": (c_int32, [_h, POINTER(KernelParamsC), c_int64, _p, c_int64, _p, c_int64, _p, c_int64,
                                    _p, c_int64, c_int64, POINTER(c_double), POINTER(c_double), _p, c_int64, _p,
                                    _p, c_size_t]),
    "gpx_acquire_argmax_f64": (c_int32, [_h, POINTER(KernelParamsC), c_int64, _p, c_int64, _p, c_int64, _p, _p,
                                         c_int64, c_int64, POINTER(AcqParamsC), c_int64, _p, _p, _p, _p,
                                         c_size_t]),
    "gpx_sweep_multi_workspace_size": (c_int32, [c_int64, c_int64, POINTER(c_size_t)]),
    "gpx_acquire_argmax_multi_f64": (c_int32, [_h, POINTER(KernelParamsC), c_int64, c_int64, _p, c_int64,
                                               POINTER(c_void_p), POINTER(c_int64), POINTER(c_void_p),
                                               POINTER(c_double), POINTER(c_double), POINTER(c_double), _p, c_int64,
                                               c_int64, POINTER(AcqParamsC), c_int64, _p, _p, _p, _p, c_size_t]),
    "gpx_argmax_combine_f64": (c_int32, [_h, _p, _p, c_int64, _p, _p]),
    "gpx_comm_unique_id": (c_int32, [c_void_p]),
    "gpx_comm_init": (c_int32, [_h, c_void_p, c_int32, c_int32, POINTER(c_void_p)]),
    "gpx_comm_destroy": (c_int32, [c_void_p]),
    "gpx_allreduce_argmax_workspace_size": (c_int32, [c_void_p, POINTER(c_size_t)]),
    "gpx_allreduce_argmax": (c_int32, [_h, c_void_p, _p, _p, _p, c_size_t]),
    "gpx_mll_workspace_size": (c_int32, [c_int64, POINTER(c_size_t)]),
    "gpx_mll_grad_f64": (c_int32, [_h, POINTER(KernelParamsC), c_int64, _p, c_int64, _p, c_int64, c_int64, _p,
                                   c_int64, _p, c_int64, _p, _p, _p, c_size_t]),
    "gpx_mll_grad_batched_f64": (c_int32, [_h, POINTER(KernelParamsC), c_int64, c_int64, _p, c_int64, c_int64, _p,
                                           c_int64, c_int64, c_int64, _p, c_int64, c_int64, _p, c_int64, c_int64, _p,
                                           c_int64, _p, _p, c_size_t]),
    "gpx_svgp_prepare_workspace_size": (c_int32, [c_int64, c_int64, POINTER(c_size_t)]),
    "gpx_svgp_prepare_f64": (c_int32, [_h, POINTER(KernelParamsC), c_int64, c_int64, c_double, _p, c_int64, c_int64,
                                       _p, c_int64, _p, c_int64, c_int64, _p, _p, _p, _p, _p, c_size_t]),
    "gpx_svgp_predict_workspace_size": (c_int32, [c_int64, c_int64, POINTER(c_size_t)]),
    "gpx_svgp_predict_f64": (c_int32, [_h, POINTER(KernelParamsC), c_int64, c_int64, _p, c_int64, c_int64, _p, _p,
                                       _p, _p, c_int64, c_int64, c_double, _p, c_int64, _p, c_int64, _p, _p,
                                       c_size_t]),
    "gpx_topk_workspace_size": (c_int32, [c_int64, POINTER(c_size_t)]),
    "gpx_topk_f64": (c_int32, [_h, _p, c_int64, c_int64, _p, _p, _p, c_size_t]),
    "gpx_fps_f64": (c_int32, [_h, _p, c_int64, c_int64, c_int64, c_int64, c_int64, _p]),
    "gpx_timing_enable": (c_int32, [_h, c_int32]),
    "gpx_timing_reset": (c_int32, [_h]),
    "gpx_timing_query": (c_int32, [_h, c_int32, POINTER(c_double), POINTER(c_int64)]),
}

_lib = None


def load() -> ctypes.CDLL:
    """Load libgpx.so once; raise GPXLibraryError (never fall back) when it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise GPXLibraryError(
            f"libgpx.so not found at {LIB_PATH}; build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "or `make -C bayesianoptimizer_amd/csrc` (hipcc --offload-arch=gfx950)")
    if "GPX_LIB" in os.environ:  # A/B tooling only: say so, the product path never sets it
        print(f"gpx: loading libgpx from GPX_LIB={LIB_PATH}", file=sys.stderr)
    try:
        lib = ctypes.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover - depends on the ROCm runtime being present
        raise GPXLibraryError(f"failed to load {LIB_PATH}: {e}") from e
    for name, (res, args) in _PROTOS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    # the struct definitions above must match the ones compiled into the library (a truncated struct would make the
    # library read past the caller's object, include/gpx.h)
    for cls, fn in ((KernelParamsC, lib.gpx_kernel_params_size), (AcqParamsC, lib.gpx_acq_params_size)):
        if ctypes.sizeof(cls) != fn():
            raise GPXLibraryError(f"{cls.__name__} is {ctypes.sizeof(cls)} bytes, libgpx expects {fn()}")
    _lib = lib
    return lib


def source_sha256() -> str:
    """sha256 over the library's sources as bayesianoptimizer_amd/csrc/Makefile stamps it into gpx_version(): every
    csrc/*.cpp|*.hip|*.h sorted by name, then include/gpx.h, contents concatenated."""
    csrc = os.path.join(_HERE, "csrc")
    names = sorted(f for f in os.listdir(csrc) if f.endswith((".cpp", ".hip", ".h")))
    h = hashlib.sha256()
    for f in names + [HEADER_PATH]:
        with open(os.path.join(csrc, f) if not os.path.isabs(f) else f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def library_source_sha256(lib=None) -> str:
    """The source hash stamped into the loaded library's gpx_version() ('unstamped' for a build outside the Makefile)."""
    v = (lib or load()).gpx_version().decode()
    return v.rsplit(" src ", 1)[-1] if " src " in v else "unstamped"


def header_symbols(path: str = HEADER_PATH):
    """Names of every function declared in include/gpx.h (used by the ABI test)."""
    text = open(path).read()
    return sorted(set(re.findall(r"\b(gpx_[a-z0-9_]+)\s*\(", text)))


def check(status: int, handle=None):
    if status == GPX_OK:
        return
    msg = ""
    if handle is not None and _lib is not None:
        raw = _lib.gpx_last_error(handle)
        msg = raw.decode() if raw else ""
    if status == GPX_TIMEOUT:
        raise GPXTimeoutError(msg)
    raise GPXError(status, msg)
