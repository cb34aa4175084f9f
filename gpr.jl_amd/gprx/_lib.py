"""ctypes binding of the C ABI declared in include/gprx.h (libgprx.so, built for gfx950).

There is no CPU fallback: if the shared library is missing this module raises at import time, and
every compute entry point runs on the MI355X through the library.
"""
from __future__ import annotations

import ctypes as C
import os
import pathlib

_HERE = pathlib.Path(__file__).resolve().parent
LIB_PATH = pathlib.Path(os.environ.get("GPRX_LIB", _HERE.parent / "lib" / "libgprx.so"))

# the header's GPRX_ABI_VERSION this binding is written against (include/gprx.h); the loader refuses
# a library that reports another one (a variant build selected by GPRX_LIB skips the build-id check)
ABI_VERSION = 3

OK = 0
NOT_POSITIVE_DEFINITE = 1
INVALID_ARGUMENT = 2
DEVICE_ERROR = 3
OUT_OF_MEMORY = 4
NOT_READY = 5

WANT_GRAD = 1
WANT_PREDICT = 2

DIST_EXPANDED = 0
DIST_DIRECT = 1

MEM_HOST = 0
MEM_DEVICE = 1

OPT_LEAF_TILES = 1
OPT_SMALL_N = 2
OPT_GRAPHS = 3
OPT_NODE_WAVES = 4

STOP_NAMES = {0: "iterations", 1: "g_tol", 2: "x_tol", 3: "f_tol", 4: "linesearch", 5: "max_evals", 6: "time_limit",
              7: "nan_gradient"}
STOP_CONVERGED = 0x100


class OptOptions(C.Structure):
    """gprx_opt_options (include/gprx.h); gprx_opt_defaults fills Optim's defaults."""
    _fields_ = [("m", C.c_int), ("iterations", C.c_int), ("max_evals", C.c_int), ("ls_iterations", C.c_int),
                ("scaleinvH0", C.c_int), ("refit", C.c_int),
                ("successive_f_tol", C.c_int), ("g_abstol", C.c_double), ("time_limit", C.c_double),
                ("alphaguess", C.c_double), ("c_1", C.c_double), ("rho_hi", C.c_double), ("rho_lo", C.c_double)]


_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int)
_vp = C.c_void_p

# name -> (restype, argtypes); must list every function declared in include/gprx.h
SIGNATURES = {
    "gprx_abi_version": (C.c_int, []),
    "gprx_status_string": (C.c_char_p, [C.c_int]),
    "gprx_build_id": (C.c_char_p, []),
    "gprx_device_count": (C.c_int, []),
    "gprx_ctx_create": (C.c_int, [C.c_int, C.POINTER(_vp)]),
    "gprx_ctx_destroy": (None, [_vp]),
    "gprx_ctx_last_error": (C.c_char_p, [_vp]),
    "gprx_ctx_set_dist_mode": (C.c_int, [_vp, C.c_int]),
    "gprx_ctx_device": (C.c_int, [_vp]),
    "gprx_ctx_set_profiling": (C.c_int, [_vp, C.c_int]),
    "gprx_ctx_set_option": (C.c_int, [_vp, C.c_int, C.c_int]),
    "gprx_ctx_kernel_stats": (C.c_int, [_vp, C.c_char_p, _dp, C.POINTER(C.c_int64), _dp, _dp]),
    "gprx_ctx_reset_stats": (C.c_int, [_vp]),
    "gprx_ctx_mem_info": (C.c_int, [_vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64)]),
    "gprx_batch_bytes": (C.c_int, [C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_uint64)]),
    "gprx_batch_create": (C.c_int, [_vp, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(_vp)]),
    "gprx_batch_destroy": (None, [_vp]),
    "gprx_batch_set_train": (C.c_int, [_vp, _vp, C.c_int64, _vp, C.c_int64, C.c_int]),
    "gprx_batch_set_test": (C.c_int, [_vp, _vp, C.c_int, C.c_int64, C.c_int]),
    "gprx_batch_run": (C.c_int, [_vp, _dp, C.c_uint, _dp, _dp, _dp, _dp, _ip, _ip]),
    "gprx_batch_predict": (C.c_int, [_vp, _dp, _dp]),
    "gprx_batch_dims": (C.c_int, [_vp, _ip, _ip, _ip, _ip]),
    "gprx_batch_alpha": (C.c_int, [_vp, _dp]),
    "gprx_opt_defaults": (None, [C.POINTER(OptOptions)]),
    "gprx_batch_optimize": (C.c_int, [_vp, _dp, C.POINTER(OptOptions), _dp, _dp, _ip, _ip, _ip, _ip, _ip]),
    "gprx_batch_set_opt_trace": (C.c_int, [_vp, _dp, C.c_int, C.c_int64]),
    "gprx_gp_create": (C.c_int, [_vp, _dp, C.c_int, C.c_int, _dp, C.POINTER(_vp)]),
    "gprx_gp_destroy": (None, [_vp]),
    "gprx_gp_lml": (C.c_int, [_vp, _dp, _dp]),
    "gprx_gp_lml_grad": (C.c_int, [_vp, _dp, _dp, _dp]),
    "gprx_gp_predict": (C.c_int, [_vp, _dp, C.c_int, _dp, _dp]),
    "gprx_gp_batch": (_vp, [_vp]),
    "gprx_rollout_min": (C.c_int, [_vp, C.c_int, C.c_int, C.c_double, C.c_int, C.c_int, C.POINTER(_vp), _ip, C.c_int,
                                   _ip, _dp, _dp]),
    "gprx_vi_step": (C.c_int, [_vp, C.c_int, C.c_double, C.c_int, _dp, C.c_double, C.c_int, C.c_double, _dp, _ip, _ip]),
    "gprx_projectv": (C.c_int, [_vp, C.c_int, C.c_double, C.c_int, _dp, _dp, C.c_double, C.c_int, C.c_double, _dp, _ip,
                                _ip]),
    "gprx_rollout_max": (C.c_int, [_vp, C.c_int, C.c_double, C.c_int, C.c_double, C.c_int, C.POINTER(_vp), _ip, C.c_int,
                                   _ip, C.c_int, _ip, _dp, _dp, _dp, _ip]),
    "gprx_cstate_pack": (C.c_int, [C.c_int, _dp, _dp, _dp, _dp, _dp]),
    "gprx_select_outputs": (C.c_int, [_dp, C.c_int, C.c_int, _ip, C.c_int, _dp]),
}


def _load():
    # PyTorch-ROCm ships its own libamdhip64 / libhsa-runtime64 (SONAME libamdhip64.so.7).  Loading
    # torch first makes libgprx.so bind to that same runtime (one HSA runtime per process), so
    # device pointers can be shared with torch and torch.distributed sees the GPUs.  Without torch
    # (e.g. a Julia ccall host) the library uses /opt/rocm's runtime.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not LIB_PATH.exists():
        raise ImportError(
            f"gprx: native library {LIB_PATH} not found -- build it with "
            "`make -C gpr.jl_amd` (or __graft_entry__.build()); there is no CPU fallback"
        )
    lib = C.CDLL(str(LIB_PATH))
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    abi = lib.gprx_abi_version()
    if abi != ABI_VERSION:
        raise ImportError(f"gprx: {LIB_PATH} implements ABI version {abi}, this binding expects {ABI_VERSION}")
    want = source_build_id()
    got = lib.gprx_build_id().decode()
    if want is not None and got != want:
        raise ImportError(f"gprx: {LIB_PATH} was built from other sources (build id {got}, sources {want}): "
                          "stale library -- rebuild with `make -C gpr.jl_amd` (or __graft_entry__.build())")
    return lib


# the library's sources, in the order gpr.jl_amd/Makefile hashes them (SRC then HDR)
BUILD_SOURCES = ["csrc/gprx_kernels.hip", "csrc/gprx_lbfgs.hip", "csrc/gprx_projection.hip", "csrc/gprx_api.hip",
                 "csrc/gprx_internal.h", "../include/gprx.h"]


def source_build_id():
    """SHA-256 prefix of the sources next to the default library (None when the library comes from
    elsewhere via GPRX_LIB, or the sources are not shipped)."""
    import hashlib

    if "GPRX_LIB" in os.environ:
        return None
    root = _HERE.parent
    h = hashlib.sha256()
    for f in BUILD_SOURCES:
        p = root / f
        if not p.exists():
            return None
        h.update(p.read_bytes())
    return h.hexdigest()[:16]


lib = _load()


class GPRXError(RuntimeError):
    def __init__(self, status: int, msg: str = ""):
        s = lib.gprx_status_string(status).decode()
        super().__init__(f"gprx status {status} ({s}){': ' + msg if msg else ''}")
        self.status = status


class NotPositiveDefinite(GPRXError):
    """Mirrors LinearAlgebra.PosDefException raised by cholesky! in the reference [ext]."""


def check(status: int, ctx=None):
    if status == OK:
        return
    msg = ""
    if ctx is not None:
        m = lib.gprx_ctx_last_error(ctx)
        msg = m.decode() if m else ""
    if status == NOT_POSITIVE_DEFINITE:
        raise NotPositiveDefinite(status, msg)
    raise GPRXError(status, msg)


def dptr(a):
    return a.ctypes.data_as(_dp) if a is not None else None


def iptr(a):
    return a.ctypes.data_as(_ip) if a is not None else None
