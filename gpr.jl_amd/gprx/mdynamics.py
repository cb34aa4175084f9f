"""The MeanDynamics variants of the noise.jl sweep (experiment_*_md_max / _md_min / _md_min_sin,
examples/noise.jl:83-85, 93-95, 103-105, 113-115): GPs whose prior mean is one variational-
integrator step of the mechanism (GPR's MeanDynamics, src/mDynamics.jl:13-60, physics in
gprx/vi.py).

Training: μ(X) is θ-independent (num_params = 0, mDynamics.jl:29), so it is evaluated ONCE per
training set, for all columns at once, and the device fits y - μ(X) (the reference re-solves the
physics for every column at every LBFGS evaluation: its single-slot cache misses on every column).
Prediction: predict_y(gp, obs) = μ(obs) + k*^T alpha -- in a rollout the physics runs at every
step's states (here vectorised over all trajectories of all trials), the GP means in one batched
device predict per step, the projection (maximal coordinates) on the device.

The physics step runs on the device (k_vi_step through gprx.projection.vi_step, one wave per
state); gprx.vi holds the host restatement it is tested against (tests/test_vi.py,
tests/test_vi_device.py).  Every function takes `physics` (a callable (mech, states) -> (solution,
iterations, status)) to run the same logic on another implementation, e.g. physics=vi.vi_step.

Maximal coordinates (e.g. examples/maximal_coordinates/P2noise.jl:28-33): the CState input,
getμ(vωindices) of the solution CState.  Minimal coordinates (e.g. minimal_coordinates/
P2noise.jl:40-61): the experiment's xtransform builds the CState from (q, qdot) (velocities by the
0.01 finite difference of the positions), and _getμ reads the solution's rates: P1 [11], P2
(w1, w2 - w1) of bodies 1 and 2, CP [9, 24], FB [11, 37] (1-based CState positions).
"""
from __future__ import annotations


import numpy as np

from . import data, vi
from .rollout import LENGTHS, NCOORD, final_cstate

DT = 0.01
MIN_IDX = {"P1": [11], "CP": [9, 24], "FB": [11, 37]}  # getμ(...) of the minimal-coordinate experiments


def _rotx(th):
    return np.stack([np.cos(th / 2), np.sin(th / 2), np.zeros_like(th), np.zeros_like(th)], axis=-1)


def _pos(y, z):
    return np.stack([np.zeros_like(y), y, z], axis=-1)


def xtransform(mech: str, Xmin, usesin: bool) -> np.ndarray:
    """The experiments' xtransform (minimal_coordinates/*noise.jl) for every column of Xmin (d, N):
    (N, 13 nb) CStates."""
    X = np.asarray(Xmin, dtype=np.float64)
    h = 0.01  # the literal 0.01 of the reference's finite difference
    if mech == "P1":
        (l,) = LENGTHS["P1"]
        th, w = (np.arctan2(X[0], X[1]), X[2]) if usesin else (X[0], X[1])
        x = _pos(0.5 * np.sin(th) * l, -0.5 * np.cos(th) * l)
        tn = th + w * h
        v = (_pos(0.5 * np.sin(tn) * l, -0.5 * np.cos(tn) * l) - x) / h
        z = np.zeros_like(th)
        return np.concatenate([x, _rotx(th), v, np.stack([w, z, z], 1)], axis=1)
    if mech == "P2":
        l1, l2 = LENGTHS["P2"]
        if usesin:
            t1, w1, t2, w2 = np.arctan2(X[0], X[1]), X[2], np.arctan2(X[3], X[4]), X[5]
        else:
            t1, w1, t2, w2 = X
        x1 = _pos(0.5 * np.sin(t1) * l1, -0.5 * np.cos(t1) * l1)
        x2 = _pos(np.sin(t1) * l1 + 0.5 * np.sin(t1 + t2) * l2, -np.cos(t1) * l1 - 0.5 * np.cos(t1 + t2) * l2)
        n1, n2 = t1 + w1 * h, t2 + w2 * h
        x1n = _pos(0.5 * np.sin(n1) * l1, -0.5 * np.cos(n1) * l1)
        x2n = _pos(np.sin(n1) * l1 + 0.5 * np.sin(n1 + n2) * l2, -np.cos(n1) * l1 - 0.5 * np.cos(n1 + n2) * l2)
        z = np.zeros_like(t1)
        return np.concatenate([x1, _rotx(t1), (x1n - x1) / h, np.stack([w1, z, z], 1),
                               x2, _rotx(t1 + t2), (x2n - x2) / h, np.stack([w1 + w2, z, z], 1)], axis=1)
    if mech == "CP":
        (l,) = LENGTHS["CP"]
        if usesin:
            xc, vc, th, w = X[0], X[1], np.arctan2(X[2], X[3]), X[4]
        else:
            xc, vc, th, w = X
        z = np.zeros_like(xc)
        x2 = _pos(xc + 0.5 * np.sin(th) * l, -0.5 * np.cos(th) * l)
        tn = w * h + th
        x2n = _pos(xc + vc * h + 0.5 * np.sin(tn) * l, -0.5 * np.cos(tn) * l)
        cart = np.stack([z, xc, z, z + 1, z, z, z, z, vc, z, z, z, z], axis=1)
        return np.concatenate([cart, x2, _rotx(th), (x2n - x2) / h, np.stack([w, z, z], 1)], axis=1)
    if mech == "FB":
        (l,) = LENGTHS["FB"]
        if usesin:
            t1, w1, t2, w2 = np.arctan2(X[0], X[1]), X[2], np.arctan2(X[3], X[4]), X[5]
        else:
            t1, w1, t2, w2 = X

        def poses(a, b):
            return (_pos(0.5 * np.sin(a) * l, -0.5 * np.cos(a) * l),
                    _pos(np.sin(a) * l + 0.5 * np.sin(b) * l, -np.cos(a) * l - 0.5 * np.cos(b) * l),
                    _pos(0.5 * np.sin(b) * l, -0.5 * np.cos(b) * l),
                    _pos(np.sin(b) * l + 0.5 * np.sin(a) * l, -np.cos(b) * l - 0.5 * np.cos(a) * l))

        p = poses(t1, t2)
        pn = poses(0.01 * w1 + t1, 0.01 * w2 + t2)
        z = np.zeros_like(t1)
        q1, q2 = _rotx(t1), _rotx(t2)
        wa, wb = np.stack([w1, z, z], 1), np.stack([w2, z, z], 1)
        rows = []
        for k, (q, w) in enumerate(((q1, wa), (q2, wb), (q2, wb), (q1, wa))):
            rows += [p[k], q, (pn[k] - p[k]) / h, w]
        return np.concatenate(rows, axis=1)
    raise ValueError(f"Experiment {mech} not supported!")


def vi_step(mech: str, states, ctx=None):
    """The product path's physics step: one variational-integrator step for every state on the device
    (gprx.projection.vi_step -> gprx_vi_step -> k_vi_step)."""
    from .projection import vi_step as device_step

    return device_step(mech, states, ctx=ctx)


def _physics(physics, ctx):
    return physics if physics is not None else (lambda mech, S: vi_step(mech, S, ctx))


def mean_max(mech: str, X, physics=None, ctx=None) -> np.ndarray:
    """μ(X) of the maximal-coordinate MD GPs: (G, N), output k = getμ(vωindices)[k] of the solution
    CState of each column (vi.mean_dynamics' contract)."""
    sol, _, _ = _physics(physics, ctx)(mech, np.asarray(X, dtype=np.float64).T)
    return sol[:, np.asarray(data.VW_INDICES[mech]) - 1].T.copy()


def mean_min(mech: str, Xmin, usesin: bool, physics=None, ctx=None) -> np.ndarray:
    """μ(X) of the minimal-coordinate MD GPs: (nc, N)."""
    sol, _, _ = _physics(physics, ctx)(mech, xtransform(mech, Xmin, usesin))
    if mech == "P2":  # _getμ: (w1, w2 - w1) of the solution (minimal_coordinates/P2noise.jl:58)
        return np.stack([sol[:, 10], sol[:, 23] - sol[:, 10]])
    return sol[:, np.asarray(MIN_IDX[mech]) - 1].T.copy()


def _gp_means(rb, feats) -> np.ndarray:
    """The GP means (k*^T alpha, no prior mean) of every slot of RankBatch rb at its trial's points:
    feats (n_local, d, M) -> (n_local, G, M), one batched device predict."""
    b = rb.batch
    feats = np.asarray(feats, dtype=np.float64)
    nd = getattr(rb, "n_dev", rb.n)
    if nd > rb.n:  # a chunk padded to the group's launch geometry (shard.plan_chunks): copies of the last trial
        feats = np.concatenate([feats, np.repeat(feats[-1:], nd - rb.n, axis=0)])
    Xs = np.repeat(feats, rb.G, axis=0)  # slot t*G + g: trial t's points
    b.set_test(Xs)
    mu, _ = b.predict(variance=False)
    return mu.reshape(nd, rb.G, -1)[: rb.n]


def simulate(mech: str, cstates, steps: int, physics=None, ctx=None):
    """The physics-only baseline (vi.simulate's contract, examples/baseline.jl): steps + 1 physics
    steps of every start state; (final CStates (T, 13 nb), OR of the per-step status flags (T,))."""
    step = _physics(physics, ctx)
    S = np.atleast_2d(np.asarray(cstates, dtype=np.float64))
    bad = np.zeros(S.shape[0], dtype=np.int32)
    for _ in range(steps + 1):
        S, _, st = step(mech, S)
        bad |= st
    return S, bad


def rollout_max(mech: str, rb, trials: list[int], starts, steps: int, regularizer=None, ctx=None, physics=None):
    """predictdynamics (examples/utils/predictdynamics.jl:7-22) with MeanDynamics GPs for the
    trajectories starts (n_local, M, 13 nb) of every local trial of rb: per step the GP means (one
    device predict for all trials), the physics means μ(obs) (all states at once), getvω, projectv!
    (device) and updatestate!.  Only the trials listed in `trials` are kept.  Returns (final
    CStates (len(trials), M, d), mean projection error per step (len(trials), M), status
    (len(trials), M))."""
    from .projection import NBODIES, getvw, projectv

    nb = NBODIES[mech]
    S = np.array(starts, dtype=np.float64)  # (n, M, d)
    n, M, d = S.shape
    idx = np.asarray(data.VW_INDICES[mech]) - 1
    perr = np.zeros((n, M))
    status = np.zeros((n, M), dtype=np.int32)
    bad = np.setdiff1d(np.arange(n), np.asarray(trials, dtype=int))  # not rolled out: finite dummies
    for _ in range(steps):
        mu = _gp_means(rb, np.swapaxes(S, 1, 2))  # (n, G, M)
        mu[bad] = 0.0
        S[bad] = np.asarray(starts, dtype=np.float64)[bad]
        sol, _, _ = _physics(physics, ctx)(mech, S.reshape(n * M, d))
        mu = mu + sol[:, idx].reshape(n, M, -1).transpose(0, 2, 1)
        vw_pred = getvw(mu.transpose(0, 2, 1), data.VW_INDICES[mech], nb)  # (n, M, 6 nb)
        vw, _, st = projectv(mech, S.reshape(n * M, d), vw_pred.reshape(n * M, -1), regularizer, ctx=ctx)
        status |= st.reshape(n, M)
        perr += np.linalg.norm(vw.reshape(n, M, -1) - vw_pred, axis=2)
        S = _update(S, vw.reshape(n, M, nb, 6), nb)
    S = _update(S, S.reshape(n, M, nb, 13)[..., 7:13], nb)  # the closing updatestate!
    keep = np.asarray(trials, dtype=int)
    return S[keep], (perr / max(steps, 1))[keep], status[keep]


def _update(S, vw, nb):
    """updatestate! then CState(mechanism): [x + v dt, q * wbar(w) dt/2, v', w'] per body."""
    n, M, d = S.shape
    c = S.reshape(n, M, nb, 13)
    x2 = c[..., 0:3] + c[..., 7:10] * DT
    q2 = vi.step_q(c[..., 3:7], c[..., 10:13], DT)
    return np.concatenate([x2, q2, vw[..., 0:3], vw[..., 3:6]], axis=-1).reshape(n, M, d)


def rollout_min(mech: str, rb, trials: list[int], starts, steps: int, usesin: bool, physics=None, ctx=None):
    """predictdynamicsmin (examples/utils/predictdynamics.jl:30-102) with MeanDynamics GPs for the
    start observations starts (n_local, M, 2 nc) of every local trial of rb: per step the GP means
    at the previous state (one device predict for all trials) plus μ(obs), then the coordinates
    advance by rate * dt.  Returns the final CStates (len(trials), M, 13 nb) (velocities zero, as
    the reference builds them)."""
    nc = NCOORD[mech]
    st = np.array(starts, dtype=np.float64)  # (n, M, 2nc): (q_1, qdot_1, ..., q_nc, qdot_nc)
    n, M, _ = st.shape
    q_old, qd_old = st[..., 0::2].copy(), st[..., 1::2].copy()
    q_cur = q_old + DT * qd_old
    bad = np.setdiff1d(np.arange(n), np.asarray(trials, dtype=int))
    for _ in range(steps):
        q_old[bad], qd_old[bad], q_cur[bad] = st[bad][..., 0::2], st[bad][..., 1::2], st[bad][..., 0::2]
        obs = np.empty((n, M, 2 * nc))
        obs[..., 0::2], obs[..., 1::2] = q_old, qd_old
        feats = data.min_features(mech, obs.reshape(n * M, 2 * nc), usesin)  # (d, n M)
        mu = _gp_means(rb, feats.reshape(-1, n, M).transpose(1, 0, 2))  # (n, nc, M)
        mu[bad] = 0.0
        mu = mu + mean_min(mech, feats, usesin, physics, ctx).reshape(nc, n, M).transpose(1, 0, 2)
        rates = mu.transpose(0, 2, 1)  # (n, M, nc)
        q_old, qd_old = q_cur, rates
        q_cur = q_cur + rates * DT
    keep = np.asarray(trials, dtype=int)
    return np.stack([np.stack([final_cstate(mech, q_cur[i, j]) for j in range(M)]) for i in keep])
