"""Host-side mirror of the GaussianProcesses.jl v0.12.4 surface the reference calls
(GP / SEArd / MeanZero / MeanDynamics-style means / optimize! / predict_y / predict_f), with every
evaluation running on the MI355X through the C ABI (include/gprx.h).

Reference call pattern (examples/maximal_coordinates/CPnoise.jl:37-43):
    kernel = SEArd(log.(params[2:end]), log(params[1]))
    mean   = meandynamics ? MeanDynamics(...) : MeanZero()
    gp     = GP(xtrain_old, yi, mean, kernel)                  # logNoise defaults to -2.0
    GaussianProcesses.optimize!(gp, LBFGS(linesearch=BackTracking(order=2)), Optim.Options(time_limit=10.))
and predict_y(gp, obs)[1][1]  (examples/utils/predictdynamics.jl:13).

Prior means: a mean is any object with `mean(X) -> (N,)` and `num_params() == 0` -- the
reference's MeanDynamics has no hyper-parameters (src/mDynamics.jl:29), so μ(X) is evaluated once
per training set and y - μ(X) is what the device sees.  Means with parameters are out of scope.
"""
from __future__ import annotations

import math

import numpy as np

from . import _lib as L
from .batch import GPBatch, Context, default_context


class MeanZero:
    """GaussianProcesses.MeanZero."""

    def num_params(self) -> int:
        return 0

    def mean(self, X) -> np.ndarray:
        return np.zeros(np.asarray(X).shape[1])


class MeanFunction:
    """A θ-independent prior mean given as a callable on one input column (the role of
    GPR.MeanDynamics, src/mDynamics.jl:41-55, whose single-slot cache keyed by the input column
    is kept: consecutive calls at the same column reuse the previous value)."""

    def __init__(self, f):
        self.f = f
        self._key = None
        self._val = None

    def num_params(self) -> int:
        return 0

    def _at(self, x):
        if self._key is None or not np.array_equal(self._key, x):
            self._key = np.array(x, copy=True)
            self._val = float(self.f(x))
        return self._val

    def mean(self, X) -> np.ndarray:
        X = np.asarray(X)
        return np.array([self._at(X[:, t]) for t in range(X.shape[1])])


class SEArd:
    """SEArd(ll, lσ): squared-exponential ARD kernel, ll = log length scales, lσ = log σ_f."""

    def __init__(self, ll, lsigma):
        self.ll = np.asarray(ll, dtype=np.float64).copy()
        self.lsigma = float(lsigma)

    def num_params(self) -> int:
        return self.ll.shape[0] + 1

    def get_params(self) -> np.ndarray:
        return np.concatenate([self.ll, [self.lsigma]])

    def set_params(self, hyp):
        hyp = np.asarray(hyp, dtype=np.float64)
        self.ll = hyp[:-1].copy()
        self.lsigma = float(hyp[-1])


class GPE:
    """Exact GP with Gaussian noise (GaussianProcesses.GPE) evaluated on the device.

    Attributes mirror the reference object: x, y, mean, kernel, logNoise, mll, dmll, target,
    dtarget, alpha is kept on the device.
    """

    def __init__(self, x, y, mean, kernel: SEArd, logNoise: float = -2.0, ctx: Context | None = None):
        self.x = np.ascontiguousarray(x, dtype=np.float64)
        if self.x.ndim == 1:
            self.x = self.x[None, :]
        self.dim, self.nobs = self.x.shape
        self.y = np.ascontiguousarray(y, dtype=np.float64)
        assert self.y.shape == (self.nobs,), "y must have one entry per column of x"
        if kernel.ll.shape[0] != self.dim:
            raise ValueError("SEArd needs one length scale per input dimension")
        if mean.num_params() != 0:
            raise NotImplementedError("only parameter-free prior means (MeanZero, MeanDynamics)")
        self.mean = mean
        self.kernel = kernel
        self.logNoise = float(logNoise)
        self.ctx = ctx or default_context()
        self._mu = np.asarray(mean.mean(self.x), dtype=np.float64)  # θ-independent prior mean
        self._batch = GPBatch(1, self.dim, self.nobs, 0, ctx=self.ctx)
        self._batch.set_train(self.x, (self.y - self._mu)[None, :])
        self.mll = -math.inf
        self.dmll = np.zeros(self.dim + 2)
        self.update_mll()  # GPE construction computes the target (initialise_target!)

    # -- parameters ---------------------------------------------------------------------------
    def get_params(self) -> np.ndarray:
        return np.concatenate([[self.logNoise], self.kernel.get_params()])

    def set_params(self, hyp):
        hyp = np.asarray(hyp, dtype=np.float64)
        if hyp.shape != (self.dim + 2,):
            raise ValueError("hyperparameter vector has the wrong length")
        self.logNoise = float(hyp[0])
        self.kernel.set_params(hyp[1:])

    @property
    def target(self) -> float:
        return self.mll

    @property
    def dtarget(self) -> np.ndarray:
        return self.dmll

    # -- evaluation ---------------------------------------------------------------------------
    def _run(self, grad: bool):
        theta = self.get_params()
        if not np.all(np.isfinite(theta)):
            raise ValueError("non-finite hyperparameters")  # ArgumentError in the reference
        r = self._batch.run(theta[None, :], grad=grad)
        st = int(r["status"][0])
        if st == L.NOT_POSITIVE_DEFINITE:
            raise L.NotPositiveDefinite(st, f"pivot {int(r['info'][0])}")
        if st != L.OK:
            L.check(st, self.ctx.h)
        self.mll = float(r["mll"][0])
        if grad:
            self.dmll = r["grad"][0].copy()
        return self.mll

    def update_mll(self):
        return self._run(grad=False)

    def update_mll_and_dmll(self):
        self._run(grad=True)
        return self.mll, self.dmll

    update_target = update_mll
    update_target_and_dtarget = update_mll_and_dmll

    def predict_f(self, xs):
        """(μ_f, σ²_f) per test column, full_cov=false [ext predict_f]."""
        xs = np.asarray(xs, dtype=np.float64)
        if xs.ndim == 1:
            xs = xs[:, None]
        if xs.shape[0] != self.dim:
            raise ValueError("test inputs have the wrong dimension")
        self._batch.set_test(xs)
        mu, var = self._batch.predict()
        return mu[0].copy(), var[0].copy()

    def predict_y(self, xs):
        """predict_f + prior mean, variance + exp(2 logNoise)  [ext predict_y]."""
        xs = np.asarray(xs, dtype=np.float64)
        if xs.ndim == 1:
            xs = xs[:, None]
        mu, var = self.predict_f(xs)
        return mu + self.mean.mean(xs), var + math.exp(2.0 * self.logNoise)

    def predict_y_mean(self, xs):
        """predict_y(gp, obs)[1] without the variance: the rollout call of
        examples/utils/predictdynamics.jl:13 (uses the mean only); skips the O(N^2 M) variance."""
        xs = np.asarray(xs, dtype=np.float64)
        if xs.ndim == 1:
            xs = xs[:, None]
        if xs.shape[0] != self.dim:
            raise ValueError("test inputs have the wrong dimension")
        self._batch.set_test(xs)
        mu, _ = self._batch.predict(variance=False)
        return mu[0] + self.mean.mean(xs)


def GP(x, y, mean, kernel, logNoise: float = -2.0, ctx: Context | None = None) -> GPE:
    """GaussianProcesses.GP(x, y, mean, kernel[, logNoise])."""
    return GPE(x, y, mean, kernel, logNoise, ctx=ctx)


def predict_y(gp: GPE, xs):
    return gp.predict_y(xs)


def predict_f(gp: GPE, xs):
    return gp.predict_f(xs)
