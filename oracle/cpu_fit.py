"""ORACLE -- test infrastructure only (tests/ and bench.py's cpu_baseline leg).

ctypes binding of oracle/cpu_fit.c (libcpufit.so, `make -C oracle`): the reference algorithm in C
on the host's OpenBLAS LAPACK, the CPU baseline BASELINE.md section 2 plans.  Same statements as
gp_oracle.fit (direct distances); parity against it in tests/test_cpu_fit.py."""
from __future__ import annotations

import ctypes as C
import glob
import os
import pathlib

import numpy as np

_HERE = pathlib.Path(__file__).resolve().parent
_lib = None


def openblas_path() -> str:
    """The scipy wheel's bundled OpenBLAS (LP64, symbols scipy_*)."""
    import scipy

    base = pathlib.Path(scipy.__file__).resolve().parent.parent
    hits = sorted(glob.glob(str(base / "scipy.libs" / "libscipy_openblas*.so*")))
    if not hits:
        raise OSError("no libscipy_openblas*.so next to scipy")
    return hits[0]


def load():
    global _lib
    if _lib is not None:
        return _lib
    path = _HERE / "libcpufit.so"
    if not path.exists():
        raise OSError(f"{path} missing: build it with `make -C oracle`")
    lib = C.CDLL(str(path))
    lib.cpufit_init.argtypes = [C.c_char_p]
    lib.cpufit_blas_threads.argtypes = [C.c_int]
    lib.cpufit_get_blas_threads.restype = C.c_int
    dp = C.POINTER(C.c_double)
    lib.cpufit_fit.argtypes = [C.c_int, C.c_int, C.c_int, dp, dp, dp, dp, dp, dp, dp, dp]
    lib.cpufit_timed.argtypes = [C.c_int, C.c_int, C.c_int, C.c_int, dp, dp, dp, dp, C.c_int, C.c_int, C.c_double,
                                 C.c_int, dp]
    rc = lib.cpufit_init(openblas_path().encode())
    if rc != 0:
        raise OSError(f"cpufit_init failed ({rc})")
    _lib = lib
    return lib


def _p(a):
    return a.ctypes.data_as(C.POINTER(C.c_double)) if a is not None else None


def fit(X, y, theta, Xs=None, blas_threads: int | None = None) -> dict:
    """One fit: X (d, N), y (N,), theta (d+2,), Xs (d, M) or None -> mll, grad, mu, var.
    blas_threads: the OpenBLAS thread count for this call (restored afterwards); None keeps it."""
    lib = load()
    X = np.ascontiguousarray(X, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    th = np.ascontiguousarray(theta, dtype=np.float64)
    d, N = X.shape
    M = 0 if Xs is None else Xs.shape[1]
    Xs = None if Xs is None else np.ascontiguousarray(Xs, dtype=np.float64)
    mll = np.zeros(1)
    g = np.zeros(d + 2)
    mu = np.zeros(max(M, 1))
    var = np.zeros(max(M, 1))
    saved = lib.cpufit_get_blas_threads()
    if blas_threads is not None:
        lib.cpufit_blas_threads(int(blas_threads))
    try:
        rc = lib.cpufit_fit(d, N, M, _p(X), _p(y), _p(th), _p(Xs), _p(mll), _p(g), _p(mu), _p(var))
    finally:
        lib.cpufit_blas_threads(saved)
    if rc != 0:
        raise RuntimeError(f"cpufit_fit: {rc}")
    out = dict(mll=float(mll[0]), grad=g)
    if M:
        out["mu"] = mu[:M]
        out["var"] = var[:M]
    return out


def timed(X, Y, T, XT, threads: int, blas_threads: int, max_seconds: float, max_fits: int):
    """Fits of slots 0, 1, ... (round robin) until max_seconds: `threads` OpenMP threads of whole
    fits with BLAS single-threaded (trial-parallel), or threads = 1 with BLAS on blas_threads
    cores (single fit).  Returns (fits, seconds)."""
    lib = load()
    X = np.ascontiguousarray(X, dtype=np.float64)
    Y = np.ascontiguousarray(Y, dtype=np.float64)
    T = np.ascontiguousarray(T, dtype=np.float64)
    XT = None if XT is None else np.ascontiguousarray(XT, dtype=np.float64)
    B, d, N = X.shape
    M = 0 if XT is None else XT.shape[2]
    sec = np.zeros(1)
    os.environ.setdefault("OMP_WAIT_POLICY", "PASSIVE")
    n = lib.cpufit_timed(B, d, N, M, _p(X), _p(Y), _p(T), _p(XT), int(threads), int(blas_threads), float(max_seconds),
                         int(max_fits), _p(sec))
    return int(n), float(sec[0])
