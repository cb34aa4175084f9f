"""ORACLE -- test infrastructure only (imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg as the checker / CPU baseline; never by the product path).

CPU restatement (numpy + scipy/OpenBLAS LAPACK, fp64) of the exact-GP arithmetic that
amacati/GPR.jl delegates to GaussianProcesses.jl v0.12.4 (pinned in
/root/reference/Manifest.toml, block [[GaussianProcesses]]; its source is NOT in the reference tree,
so the statements marked [ext] restate its published algorithm).

Parity status: the reference has no tests, fixtures or golden vectors (SURVEY.md section 4,
8c), and Julia / GaussianProcesses.jl cannot run in this container.  This restatement is pinned
against an independent implementation instead -- scikit-learn 1.7.2 GaussianProcessRegressor
(ConstantKernel*RBF(ARD)+WhiteKernel) log-marginal-likelihood and its gradient -- and against
central finite differences (tests/test_oracle.py, tests/golden/make_golden.py).  With respect to
the reference's own rounding the parity is "unpinned".

Reference call sites the formulas follow:
  theta  : SEArd(log.(p[2:end]), log(p[1])) and GP(X, y, mean, kernel) with the default
           logNoise = -2  (examples/maximal_coordinates/CPnoise.jl:38-40)
  X      : reduce(hcat, CState.(sold)), d x N column-major  (CPnoise.jl:26, src/CState.jl:19-28)
  y      : [s[i] for s in X_curr] per vwindex  (CPnoise.jl:28-29), minus the prior mean
           (MeanZero, or MeanDynamics, which is theta-independent: src/mDynamics.jl:29,41-55)
  predict: predict_y(gp, obs)[1][1]  (examples/utils/predictdynamics.jl:13)
"""
from __future__ import annotations

import math

import numpy as np
import scipy.linalg as sla

LOG2PI = math.log(2.0 * math.pi)  # Julia's log2π
EPS = float(np.finfo(np.float64).eps)  # Julia's eps()

DIST_EXPANDED = 0
DIST_DIRECT = 1
# [ext] GaussianProcesses' cov_ij for StationaryARD kernels evaluates the Gram (and the predictive
# cross-covariance) through distij over WeightedSqEuclidean: s += w_d (x1_d - x2_d)^2 -- exact
# differences, the DIST_DIRECT form and the default here.  The per-dimension Distances.jl stack
# (DIST_EXPANDED rounding) is kept by KernelData for the gradient; restating the whole path in that
# rounding is the second formulation whose spread calibrates the tolerances.
DEFAULT_MODE = DIST_DIRECT


def kernel_params(theta: np.ndarray, d: int):
    """theta = [logσn, logℓ_1..d, logσf]  ->  (iℓ2, σf², σn², noise_diag).

    [ext] SEArd stores iℓ2 = exp(-2 logℓ) and σ2 = exp(2 logσ); update_cK! adds
    exp(2 logNoise) + eps() to the diagonal.
    """
    theta = np.asarray(theta, dtype=np.float64)
    assert theta.shape == (d + 2,)
    with np.errstate(over="ignore"):  # Julia exp overflows to Inf (then cholesky fails)
        il2 = np.exp(-2.0 * theta[1 : d + 1])
        sf2 = float(np.exp(2.0 * theta[d + 1]))
        sn2 = float(np.exp(2.0 * theta[0]))
    return il2, sf2, sn2, sn2 + EPS


def dist_stack(XA: np.ndarray, XB: np.ndarray, mode: int = DIST_DIRECT) -> np.ndarray:
    """Per-dimension squared distances, shape (d, NA, NB).

    [ext] GaussianProcesses' KernelData for StationaryARD kernels fills dist_stack[:,:,p] with
    Distances.jl 0.10.5 pairwise(SqEuclidean(), X1[p:p,:], X2[p:p,:]), whose _pairwise! expands
    |a-b|^2 = a^2 + b^2 - 2ab (clamped at 0)  -> mode DIST_EXPANDED.
    DIST_DIRECT is the exact-difference form (a-b)^2 of cov_ij / distij (the default).
    """
    A = np.asarray(XA, dtype=np.float64)
    B = np.asarray(XB, dtype=np.float64)
    if mode == DIST_EXPANDED:
        a = A[:, :, None]
        b = B[:, None, :]
        s = a * a + b * b  # sa2[i] + sb2[j]
        v = s - 2.0 * (a * b)  # - 2 * r[i,j]
        return np.maximum(v, 0.0)
    t = A[:, :, None] - B[:, None, :]
    return t * t


def dist_lazy(XA: np.ndarray, XB: np.ndarray, mode: int = DIST_DIRECT):
    """The same stack as dist_stack, one dimension at a time (a list-like of (NA, NB) arrays made
    on access): the large configurations (FB N=4096, d=52: a 7 GB stack) keep one slice alive."""
    A = np.asarray(XA, dtype=np.float64)
    B = np.asarray(XB, dtype=np.float64)

    class _Lazy:
        shape = (A.shape[0], A.shape[1], B.shape[1])

        def __getitem__(self, p):
            return dist_stack(A[p:p + 1], B[p:p + 1], mode)[0]

    return _Lazy()


STACK_MAX = 1 << 28  # elements; above this the stack is evaluated lazily (identical arithmetic)


def weighted_r(D: np.ndarray, il2: np.ndarray) -> np.ndarray:
    """r_ij = sum_p D[p,i,j] * iℓ2_p, accumulated in order p = 1..d from 0.0 (cov_ij loop)."""
    r = np.zeros(D.shape[1:], dtype=np.float64)
    for p in range(D.shape[0]):
        r = r + D[p] * il2[p]
    return r


def gram(X: np.ndarray, theta: np.ndarray, mode: int = DIST_DIRECT, D: np.ndarray | None = None):
    """[ext] update_cK!: K = σ2 exp(-r/2) + (exp(2 logNoise) + eps) I, plus the noise-free Kf."""
    d = X.shape[0]
    il2, sf2, sn2, noise = kernel_params(theta, d)
    if D is None:
        D = dist_stack(X, X, mode) if d * X.shape[1] ** 2 <= STACK_MAX else dist_lazy(X, X, mode)
    Kf = sf2 * np.exp(-weighted_r(D, il2) * 0.5)
    K = Kf.copy()
    idx = np.arange(K.shape[0])
    K[idx, idx] = K[idx, idx] + noise
    return K, Kf, D


class NotPosDef(Exception):
    def __init__(self, info: int):
        super().__init__(f"not positive definite at pivot {info}")
        self.info = info


def cholesky_upper(K: np.ndarray) -> np.ndarray:
    """[ext] cholesky!(Symmetric(K, :U)) -> OpenBLAS dpotrf('U'); PosDefException on failure."""
    U, info = sla.lapack.dpotrf(K, lower=0, clean=1, overwrite_a=0)
    if info > 0:
        raise NotPosDef(int(info))
    if info < 0:
        raise ValueError("dpotrf argument error")
    dg = np.diag(U)
    if not np.all(np.isfinite(dg)):  # Inf entries (exp overflow): NaN pivots make dpotrf fail
        raise NotPosDef(int(np.argmin(np.isfinite(dg))) + 1)
    return U


def lml(X, y, theta, mode: int = DIST_DIRECT, want_grad: bool = False, D=None):
    """update_mll! (+ update_dmll!) restated [ext].

    mll  = -(y'α + logdet(K) + N log2π)/2,  α = K \\ y,  logdet = 2 Σ log U_ii
    W    = αα' - K⁻¹   (get_ααinvcKI!: ldiv!(chol, I) then ger!)
    dmll = [σn² tr(W),  ½ Σ_ij W_ij ∂K_ij/∂logℓ_p (p=1..d),  ½ Σ_ij W_ij ∂K_ij/∂logσ]
           with ∂K/∂logℓ_p = Kf ∘ dist_p iℓ2_p, ∂K/∂logσ = 2 Kf  (dmll_kern! / dKij_dθ!)
    Returns (mll, grad or None, aux dict).
    """
    X = np.asarray(X, dtype=np.float64)
    y = np.asarray(y, dtype=np.float64)
    d, N = X.shape
    K, Kf, D = gram(X, theta, mode, D)
    U = cholesky_upper(K)
    alpha = sla.cho_solve((U, False), y)
    logdet = 2.0 * np.sum(np.log(np.diag(U)))
    mll = -(float(y @ alpha) + logdet + LOG2PI * N) / 2.0
    aux = dict(K=K, Kf=Kf, U=U, alpha=alpha, logdet=logdet, D=D)
    if not want_grad:
        return mll, None, aux
    il2, sf2, sn2, _ = kernel_params(theta, d)
    Kinv = sla.cho_solve((U, False), np.eye(N))
    W = np.outer(alpha, alpha) - Kinv
    WK = W * Kf
    g = np.empty(d + 2)
    g[0] = sn2 * np.trace(W)
    for p in range(d):
        g[1 + p] = 0.5 * np.sum(WK * D[p]) * il2[p]
    g[d + 1] = 0.5 * np.sum(WK) * 2.0
    aux["W"] = W
    aux["Kinv"] = Kinv
    return mll, g, aux


def predict_f(X, theta, alpha, U, Xs, mode: int = DIST_DIRECT):
    """[ext] predict_f(gp, x*; full_cov=false): per test point k* = σ2 exp(-r(X, x*)/2),
    μ = k*'α, v = U'⁻¹ k* (whiten!), σ² = max(Kpred - v'v, 0), Kpred = σ2 exp(-r(x*,x*)/2)."""
    X = np.asarray(X, dtype=np.float64)
    Xs = np.asarray(Xs, dtype=np.float64)
    d = X.shape[0]
    il2, sf2, _, _ = kernel_params(theta, d)
    Ks = sf2 * np.exp(-weighted_r(dist_stack(X, Xs, mode), il2) * 0.5)  # N x M
    mu = Ks.T @ alpha
    V = sla.solve_triangular(U, Ks, trans="T", lower=False)
    kss = sf2 * np.exp(-weighted_r(dist_stack(Xs, Xs, mode), il2).diagonal() * 0.5)
    var = np.maximum(kss - np.sum(V * V, axis=0), 0.0)
    return mu, var


def predict_y(X, theta, alpha, U, Xs, mean_s=None, mode: int = DIST_DIRECT):
    """[ext] predict_y = predict_f + prior mean, variance + exp(2 logNoise)."""
    mu, var = predict_f(X, theta, alpha, U, Xs, mode)
    if mean_s is not None:
        mu = mu + np.asarray(mean_s)
    return mu, var + math.exp(2.0 * float(theta[0]))


def fit(X, y, theta, Xs=None, mode: int = DIST_DIRECT):
    """One 'fit' (SURVEY.md section 8d): Gram+Cholesky+α+LML, ∂LML, predict at Xs.

    mll_sens (test calibration, not part of the reference's output): 4 eps ||W o K||_F, the size of
    the LML change under a random 4-ulp relative perturbation of K (dLML = ½ Σ W_ij dK_ij) -- what
    any other summation order of the Gram or of a blocked factorisation can move the LML by."""
    m, g, aux = lml(X, y, theta, mode, want_grad=True)
    out = dict(mll=m, grad=g, alpha=aux["alpha"], mll_sens=4.0 * EPS * float(np.linalg.norm(aux["W"] * aux["K"])))
    if Xs is not None:
        mu, var = predict_f(X, theta, aux["alpha"], aux["U"], Xs, mode)
        out["mu"] = mu
        out["var"] = var
    return out


# ---- CState layout (bit-exact copies) -------------------------------------------------------
def cstate_pack(xc, q_wxyz, vc, wc) -> np.ndarray:
    """CState(::Vector{State}): per body [xc(3), q.w, q.x, q.y, q.z, vc(3), ωc(3)]
    (src/CState.jl:25-28)."""
    xc = np.asarray(xc, dtype=np.float64).reshape(-1, 3)
    q = np.asarray(q_wxyz, dtype=np.float64).reshape(-1, 4)
    vc = np.asarray(vc, dtype=np.float64).reshape(-1, 3)
    wc = np.asarray(wc, dtype=np.float64).reshape(-1, 3)
    return np.concatenate([xc, q, vc, wc], axis=1).reshape(-1).copy()


def select_outputs(Xcurr: np.ndarray, idx1) -> np.ndarray:
    """ytrain = [[s[i] for s in X_curr] for i in vωindices] with 1-based indices
    (examples/maximal_coordinates/CPnoise.jl:28-29)."""
    Xcurr = np.asarray(Xcurr)
    return np.stack([Xcurr[i - 1, :] for i in idx1], axis=0)


# ---- rollout in minimal coordinates (examples/utils/predictdynamics.jl:38-102) ---------------
ROLL_ANGLE = {"P1": (True,), "P2": (True, True), "CP": (False, True), "FB": (True, True)}


def rollout_min(mech: str, gps, start, steps: int, usesin: bool = False, dt: float = 0.01,
                mode: int = DIST_DIRECT) -> np.ndarray:
    """predictdynamicsmin's loop for T start observations at once (each trajectory independent).
    gps: nc tuples (X (d, N), theta, alpha) with MeanZero, GP g predicting coordinate g's rate.
    start: (T, 2nc) = (q_old, qdot_old) per coordinate.  Returns (T, 2nc) = (q_curr, qdot_last).

      qcurr = qold + Δt*qdot_old                                 (:41, :55, :72, :87)
      for 1:steps
          obs = (q_old, qdot_old) or (sin, cos, qdot) per angle   (:43, :57, :74, :89)
          qdot_curr_g = predict_y(gp_g, obs)[1][1]               (:44, :58, :75, :90)
          q_old, qdot_old = q_curr, qdot_curr ; q_curr += qdot_curr*Δt   (:45-46, :59-61, ...)
    """
    ang = ROLL_ANGLE[mech]
    nc = len(ang)
    st = np.array(start, dtype=np.float64).reshape(-1, 2 * nc)
    qo = st[:, 0::2].copy()
    vo = st[:, 1::2].copy()
    qc = qo + dt * vo
    for _ in range(steps):
        rows = []
        for c in range(nc):
            if usesin and ang[c]:
                rows += [np.sin(qo[:, c]), np.cos(qo[:, c]), vo[:, c]]
            else:
                rows += [qo[:, c], vo[:, c]]
        obs = np.stack(rows, axis=0)  # (d, T)
        pred = np.empty_like(qo)
        for g, (X, theta, alpha) in enumerate(gps):
            il2, sf2, _, _ = kernel_params(np.asarray(theta, dtype=np.float64), X.shape[0])
            Ks = sf2 * np.exp(-weighted_r(dist_stack(np.asarray(X, dtype=np.float64), obs, mode), il2) * 0.5)
            pred[:, g] = Ks.T @ alpha
        qo, vo = qc.copy(), pred
        qc = qc + pred * dt
    out = np.empty_like(st)
    out[:, 0::2] = qc
    out[:, 1::2] = vo
    return out
