"""Context / batch wrappers over the C ABI (include/gprx.h).

A `GPBatch` holds B GP slots of equal (d, N) in HBM -- the G per-output GPs of a trial
(examples/maximal_coordinates/CPnoise.jl:37-43) and/or several trials (examples/parallel/core.jl:28)
-- and evaluates all of them with one launch sequence per call.
"""
from __future__ import annotations

import atexit
import ctypes as C
import threading
import weakref

import numpy as np

from . import _lib as L

_ctx_lock = threading.Lock()
_default_ctx: dict[int, "Context"] = {}
# live handles, released before interpreter teardown: the HIP runtime's own static destructors run
# after Python finalisation, and a batch or context freed after them aborts the process
_live_batches: "weakref.WeakSet[GPBatch]" = weakref.WeakSet()
_live_ctxs: "weakref.WeakSet[Context]" = weakref.WeakSet()


@atexit.register
def _release_all():
    for b in list(_live_batches):
        b.close()
    for c in list(_live_ctxs):
        c.close()


class Context:
    """One device + one HIP stream (gprx_ctx).  Safe to share across threads; calls serialise."""

    def __init__(self, device: int = 0, dist_mode: int = L.DIST_DIRECT):
        h = C.c_void_p()
        L.check(L.lib.gprx_ctx_create(int(device), C.byref(h)))
        self.h = h
        self.device = int(device)
        _live_ctxs.add(self)
        self.set_dist_mode(dist_mode)

    def set_dist_mode(self, mode: int):
        L.check(L.lib.gprx_ctx_set_dist_mode(self.h, int(mode)), self.h)
        self.dist_mode = int(mode)

    def set_option(self, option: int, value: int):
        """Launch-geometry option (gprx_ctx_set_option: L.OPT_LEAF_TILES / OPT_SMALL_N / OPT_GRAPHS);
        results are identical under every setting."""
        L.check(L.lib.gprx_ctx_set_option(self.h, int(option), int(value)), self.h)

    def set_profiling(self, enable: bool):
        L.check(L.lib.gprx_ctx_set_profiling(self.h, 1 if enable else 0), self.h)

    def reset_stats(self):
        L.check(L.lib.gprx_ctx_reset_stats(self.h), self.h)

    def kernel_stats(self, name: str) -> dict:
        ms = C.c_double()
        n = C.c_int64()
        fl = C.c_double()
        by = C.c_double()
        L.check(L.lib.gprx_ctx_kernel_stats(self.h, name.encode(), C.byref(ms), C.byref(n), C.byref(fl), C.byref(by)))
        return dict(ms=ms.value, launches=n.value, flops=fl.value, bytes=by.value)

    def close(self):
        if getattr(self, "h", None):
            L.lib.gprx_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def default_context(device: int = 0) -> Context:
    with _ctx_lock:
        c = _default_ctx.get(device)
        if c is None:
            c = Context(device)
            _default_ctx[device] = c
        return c


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def host_empty(shape) -> np.ndarray:
    """An fp64 host array for per-test-point outputs, page-locked when torch's HIP runtime is
    usable (its caching pinned allocator: no allocation cost after the first calls), so that the
    library copies the predictive mean / variance straight into it by DMA; else plain numpy."""
    try:
        import torch

        if torch.cuda.is_available():
            return torch.empty(shape, dtype=torch.float64, pin_memory=True).numpy()
    except Exception:  # noqa: BLE001 -- any failure: pageable memory, the library stages the copy
        pass
    return np.empty(shape)


def opt_options(method=None, options=None, refit: bool = True) -> "L.OptOptions":
    """gprx_opt_options from gprx.optim.LBFGS / Options, validated here (ValueError) with the same
    bounds gprx_batch_optimize enforces, so a rejected call never reaches the library."""
    import math

    from .optim import LBFGS, Options

    method = method or LBFGS()
    options = options or Options()
    ls = method.linesearch
    if ls.order != 2:
        raise ValueError("device optimiser: BackTracking order 2 only (the experiments' setting)")
    if not 1 <= int(method.m) <= 64:
        raise ValueError(f"LBFGS m = {method.m}: the device optimiser keeps 1..64 history pairs")
    if int(options.iterations) < 0 or int(ls.iterations) < 0 or int(options.successive_f_tol) < 0:
        raise ValueError("iterations, linesearch iterations and successive_f_tol must be >= 0")
    if not (ls.c_1 > 0 and ls.rho_lo > 0 and ls.rho_hi > 0) or not math.isfinite(method.alphaguess) \
            or math.isnan(options.g_abstol):
        raise ValueError("c_1, rho_lo, rho_hi > 0; finite alphaguess; g_abstol not NaN")
    o = L.OptOptions()
    L.lib.gprx_opt_defaults(C.byref(o))
    o.m, o.iterations, o.ls_iterations = method.m, options.iterations, ls.iterations
    o.scaleinvH0, o.refit = int(method.scaleinvH0), int(refit)
    o.successive_f_tol = int(options.successive_f_tol)
    o.max_evals = 0 if options.max_evals is None else int(options.max_evals)  # <= 0: no limit (Optim)
    o.g_abstol, o.alphaguess = options.g_abstol, method.alphaguess
    o.time_limit = options.time_limit  # NaN: none
    o.c_1, o.rho_hi, o.rho_lo = ls.c_1, ls.rho_hi, ls.rho_lo
    return o


class GPBatch:
    """B exact SE-ARD GPs with shared (d, N); per-slot X, y, theta.

    X: (B, d, N) or (d, N) shared; y: (B, N) = targets minus prior mean.
    theta rows: [logσn, logℓ_1..d, logσf] (GaussianProcesses get_params order).
    """

    def __init__(self, B: int, d: int, N: int, M_max: int = 0, ctx: Context | None = None):
        self.ctx = ctx or default_context()
        h = C.c_void_p()
        L.check(L.lib.gprx_batch_create(self.ctx.h, int(B), int(d), int(N), int(M_max), C.byref(h)), self.ctx.h)
        self.h = h
        self.B, self.d, self.N = int(B), int(d), int(N)
        self.M = 0
        _live_batches.add(self)

    # -- inputs -----------------------------------------------------------------------------
    def set_train(self, X, Y):
        """Host numpy arrays.  X: (d, N) shared or (B, d, N); Y: (B, N)."""
        X = _f64(X)
        Y = _f64(Y)
        if X.ndim == 2:
            assert X.shape == (self.d, self.N), X.shape
            xs = 0
        else:
            assert X.shape == (self.B, self.d, self.N), X.shape
            xs = self.d * self.N
        assert Y.shape == (self.B, self.N), Y.shape
        # numpy (d, N) row-major is the transpose of the ABI's d x N column-major layout
        Xc = np.ascontiguousarray(np.swapaxes(X, -1, -2))  # (..., N, d): column t contiguous
        L.check(L.lib.gprx_batch_set_train(self.h, Xc.ctypes.data, xs, Y.ctypes.data, self.N, L.MEM_HOST), self.ctx.h)

    def set_train_device(self, X_ptr: int, x_slot_stride: int, Y_ptr: int, y_slot_stride: int):
        """Device pointers (e.g. torch tensors' data_ptr()), ABI layout: per slot N x d row-major
        (= d x N column-major) and N targets."""
        L.check(
            L.lib.gprx_batch_set_train(self.h, C.c_void_p(X_ptr), x_slot_stride, C.c_void_p(Y_ptr), y_slot_stride,
                                       L.MEM_DEVICE),
            self.ctx.h,
        )

    def set_test(self, Xs):
        """Xs: (d, M) shared or (B, d, M)."""
        Xs = _f64(Xs)
        if Xs.ndim == 2:
            M = Xs.shape[1]
            xs = 0
        else:
            assert Xs.shape[0] == self.B
            M = Xs.shape[2]
            xs = self.d * M
        assert Xs.shape[-2] == self.d
        Xc = np.ascontiguousarray(np.swapaxes(Xs, -1, -2))
        L.check(L.lib.gprx_batch_set_test(self.h, Xc.ctypes.data, int(M), xs, L.MEM_HOST), self.ctx.h)
        self.M = int(M)

    def set_test_device(self, Xs_ptr: int, M: int, xs_slot_stride: int):
        L.check(L.lib.gprx_batch_set_test(self.h, C.c_void_p(Xs_ptr), int(M), xs_slot_stride, L.MEM_DEVICE), self.ctx.h)
        self.M = int(M)

    # -- evaluation ---------------------------------------------------------------------------
    def run(self, theta, grad: bool = True, predict: bool = False, raise_on_error: bool = False,
            variance: bool = True):
        """Returns dict(mll[B], grad[B,d+2] | None, mu[B,M] | None, var[B,M] | None, status[B], info[B]).
        variance=False skips the predictive variance (its O(N^2 M) GEMM); var is then None."""
        theta = _f64(theta)
        if theta.ndim == 1:
            theta = np.broadcast_to(theta, (self.B, self.d + 2)).copy()
        assert theta.shape == (self.B, self.d + 2), theta.shape
        mll = np.empty(self.B)
        g = np.empty((self.B, self.d + 2)) if grad else None
        pred = predict and self.M > 0
        mu = host_empty((self.B, self.M)) if pred else None
        var = host_empty((self.B, self.M)) if pred and variance else None
        st = np.empty(self.B, dtype=np.int32)
        info = np.empty(self.B, dtype=np.int32)
        flags = (L.WANT_GRAD if grad else 0) | (L.WANT_PREDICT if pred else 0)
        rc = L.lib.gprx_batch_run(self.h, L.dptr(theta), flags, L.dptr(mll), L.dptr(g), L.dptr(mu), L.dptr(var),
                                  L.iptr(st), L.iptr(info))
        if rc not in (L.OK, L.NOT_POSITIVE_DEFINITE, L.INVALID_ARGUMENT) or (raise_on_error and rc != L.OK):
            L.check(rc, self.ctx.h)
        return dict(mll=mll, grad=g, mu=mu, var=var, status=st, info=info)

    def optimize(self, theta0, method=None, options=None, refit: bool = True, trace_rounds: int = 0):
        """GaussianProcesses.optimize!(gp, LBFGS(linesearch=BackTracking(order=2)), options) for
        every slot (CPnoise.jl:41), on the device (k_lbfgs: gprx/optim.py's algorithm as a per-slot
        state machine, lock-step over the batch).  method / options: gprx.optim.LBFGS / Options.
        Returns (results, rounds) like gprx.optim.optimize_batch; with refit the batch ends
        factorised at the minimisers (optimize!'s update_target!), so predict() uses them.  A
        minimiser whose refit fails raises (update_target!'s PosDefException / ArgumentError) with
        the results attached as `err.results`; the batch is then left unfactorised.
        trace_rounds > 0 records the first rounds' evaluations (gprx_batch_set_opt_trace) in
        `self.last_opt_trace`: (rounds, B, 2n+2) rows [active, theta(n), mll, dmll(n)], n = d+2."""
        from .optim import Result

        o = opt_options(method, options, refit)
        theta0 = _f64(theta0)
        if theta0.ndim == 1:
            theta0 = np.broadcast_to(theta0, (self.B, self.d + 2)).copy()
        assert theta0.shape == (self.B, self.d + 2), theta0.shape
        B, n = self.B, self.d + 2
        th = np.empty((B, n))
        fmin = np.empty(B)
        its, fc, gc = (np.empty(B, dtype=np.int32) for _ in range(3))
        stp = np.full(B, -1, dtype=np.int32)  # -1: not written (the call rejected its input)
        rounds = C.c_int(0)
        tr = None
        if trace_rounds > 0:
            tr = np.full((int(trace_rounds), B, 2 * n + 2), np.nan)
            L.check(L.lib.gprx_batch_set_opt_trace(self.h, L.dptr(tr), int(trace_rounds), tr.size), self.ctx.h)
        try:
            rc = L.lib.gprx_batch_optimize(self.h, L.dptr(theta0), C.byref(o), L.dptr(th), L.dptr(fmin), L.iptr(its),
                                           L.iptr(fc), L.iptr(gc), L.iptr(stp), C.byref(rounds))
        finally:
            if tr is not None:
                L.lib.gprx_batch_set_opt_trace(self.h, None, 0, 0)
        self.last_opt_trace = tr[:max(0, min(int(rounds.value), tr.shape[0]))] if tr is not None else None
        if rc not in (L.OK, L.NOT_POSITIVE_DEFINITE, L.INVALID_ARGUMENT) or np.any(stp < 0):
            L.check(rc if rc != L.OK else L.DEVICE_ERROR, self.ctx.h)  # no search ran: no results
        res = [Result(th[s].copy(), float(fmin[s]), int(its[s]), int(fc[s]), int(gc[s]),
                      bool(stp[s] & L.STOP_CONVERGED), L.STOP_NAMES[int(stp[s]) & 0xFF]) for s in range(B)]
        if rc != L.OK:  # the refit at a minimiser failed: the search results are still valid
            try:
                L.check(rc, self.ctx.h)
            except L.GPRXError as e:
                e.results = (res, int(rounds.value))
                raise
        return res, int(rounds.value)

    def predict(self, variance: bool = True):
        """Predictive mean (and variance) at the current test points from the last run's
        factorisation; variance=False returns (mu, None) without the variance GEMM."""
        mu = host_empty((self.B, self.M))
        var = host_empty((self.B, self.M)) if variance else None
        L.check(L.lib.gprx_batch_predict(self.h, L.dptr(mu), L.dptr(var)), self.ctx.h)
        return mu, var

    def alpha(self):
        """alpha = K^-1 (y - mean) per slot from the last factorisation (gp.alpha); NaN rows for the
        slots that failed in it."""
        out = np.empty((self.B, self.N))
        L.check(L.lib.gprx_batch_alpha(self.h, L.dptr(out)), self.ctx.h)
        return out

    def close(self):
        if getattr(self, "h", None):
            if getattr(self.ctx, "h", None):  # a closed context already synchronised its stream
                L.lib.gprx_batch_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
