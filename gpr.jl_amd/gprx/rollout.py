"""Rollouts.  Minimal coordinates: predictdynamicsmin (examples/utils/predictdynamics.jl:30-102)
for many trajectories in one device launch (gprx_rollout_min, include/gprx.h).  Maximal
coordinates: predictdynamics (:7-22) with batched mean-only predictions per step and the physics
(projectv!, updatestate!) injected by the caller.

The reference calls `predict_y(gp, obs)[1][1]` once per GP per step per test trajectory
(predictdynamics.jl:44,58,75,90) -- G x steps x testsamples single-point predictions, each with
an O(N^2) variance it discards.  Here one workgroup per trajectory runs the whole step chain on
the MI355X, reading each GP's training inputs, alpha and kernel parameters from its batch slot.

Coordinates (startobservation layout, predictdynamics.jl:40,54,71,86):
    P1  (theta, omega)                       -> 1 GP  (omega)
    P2  (theta1, omega1, theta2, omega2)     -> 2 GPs (omega1, omega2), theta2 relative
    CP  (x, v, theta, omega)                 -> 2 GPs (v, omega)
    FB  (theta1, omega1, theta3, omega3)     -> 2 GPs (omega1, omega3)
GP inputs per step: that vector, or with usesin (sin q, cos q, qdot) for the angle coordinates.
Only MeanZero GPs roll out on the device (MeanDynamics needs a physics solve per step).
"""
from __future__ import annotations

import ctypes as C
import math

import numpy as np

from . import _lib as L
from .batch import Context, GPBatch

MECH = {"P1": 1, "P2": 2, "CP": 3, "FB": 4}
NCOORD = {"P1": 1, "P2": 2, "CP": 2, "FB": 2}
ANGLE = {"P1": (True,), "P2": (True, True), "CP": (False, True), "FB": (True, True)}
DT = 0.01  # mechanism.Δt of the experiments (P2noise.jl(min):14)
# link lengths of the experiment mechanisms (examples/utils/simulations.jl:11,53-54,111; FB l = 1)
LENGTHS = {"P1": (1.0,), "P2": (1.0, 1.0), "CP": (0.5,), "FB": (1.0,)}


def input_dim(mech: str, usesin: bool) -> int:
    return sum(3 if (usesin and a) else 2 for a in ANGLE[mech])


def rollout_min(mech: str, groups, start, steps: int, usesin: bool = False, dt: float = DT,
                traj_group=None, ctx: Context | None = None) -> np.ndarray:
    """Run T rollouts.  groups: list of rollout groups, each a list of nc GP references -- a
    GPE or a (GPBatch, slot) pair -- for coordinates 1..nc.  start: (T, 2nc).  traj_group: (T,)
    group index per trajectory (default: all group 0).  Returns (T, 2nc) = (q_cur, qdot_last) per
    coordinate after `steps` steps."""
    if mech not in MECH:
        raise ValueError(f"Experiment {mech} not supported!")  # predictdynamics.jl:35
    nc = NCOORD[mech]
    start = np.ascontiguousarray(start, dtype=np.float64)
    if start.ndim == 1:
        start = start[None, :]
    T = start.shape[0]
    if start.shape != (T, 2 * nc):
        raise ValueError(f"start must be (T, {2 * nc})")
    if traj_group is None:
        traj_group = np.zeros(T, dtype=np.int32)
    traj_group = np.ascontiguousarray(traj_group, dtype=np.int32)
    if traj_group.shape != (T,):
        raise ValueError("traj_group must have one entry per trajectory")
    refs = []
    for grp in groups:
        if len(grp) != nc:
            raise ValueError(f"{mech} rollouts use {nc} GP(s) per group")
        for g in grp:
            refs.append(_slot_ref(g))
    batches = (C.c_void_p * len(refs))(*[b.h.value for b, _ in refs])
    slots = np.ascontiguousarray([s for _, s in refs], dtype=np.int32)
    ctx = ctx or refs[0][0].ctx
    out = np.empty((T, 2 * nc), dtype=np.float64)
    L.check(
        L.lib.gprx_rollout_min(ctx.h, MECH[mech], 1 if usesin else 0, float(dt), int(steps), len(groups), batches,
                               L.iptr(slots), T, L.iptr(traj_group), L.dptr(start), L.dptr(out)),
        ctx.h,
    )
    return out


def _slot_ref(g):
    if isinstance(g, tuple):
        b, s = g
        if not isinstance(b, GPBatch):
            raise TypeError("a GP reference is a GPE or a (GPBatch, slot) pair")
        return b, int(s)
    from .gp import MeanZero  # GPE
    if not isinstance(g.mean, MeanZero):
        raise NotImplementedError("device rollouts need MeanZero GPs (MeanDynamics solves physics per step)")
    return g._batch, 0


def _rotx_q(th):
    return [math.cos(th / 2), math.sin(th / 2), 0.0, 0.0]  # q2vec(UnitQuaternion(RotX(θ)))


def final_cstate(mech: str, q, lengths=None) -> np.ndarray:
    """The CState predictdynamicsmin returns, built from the final coordinates q (velocities zero):
    P1 predictdynamics.jl:48-49, P2 :63-66, CP :80-81, FB :95-101."""
    ls = LENGTHS[mech] if lengths is None else tuple(lengths)
    z6 = [0.0] * 6
    if mech == "P1":
        (th,), (l,) = q, ls
        return np.array([0.0, 0.5 * l * math.sin(th), -0.5 * l * math.cos(th)] + _rotx_q(th) + z6)
    if mech == "P2":
        (t1, t2), (l1, l2) = q, ls
        x1 = [0.0, 0.5 * l1 * math.sin(t1), -0.5 * l1 * math.cos(t1)]
        x2 = [0.0, l1 * math.sin(t1) + 0.5 * l2 * math.sin(t1 + t2), -l1 * math.cos(t1) - 0.5 * l2 * math.cos(t1 + t2)]
        return np.array(x1 + _rotx_q(t1) + z6 + x2 + _rotx_q(t1 + t2) + z6)
    if mech == "CP":
        (x, th), (l,) = q, ls
        return np.array([0.0, x, 0.0, 1.0] + [0.0] * 10 + [0.5 * l * math.sin(th) + x, -0.5 * l * math.cos(th)]
                        + _rotx_q(th) + z6)
    if mech == "FB":
        (t1, t2), (l,) = q, ls
        x1 = [0.0, 0.5 * math.sin(t1) * l, -0.5 * math.cos(t1) * l]
        x2 = [0.0, math.sin(t1) * l + 0.5 * math.sin(t2) * l, -math.cos(t1) * l - 0.5 * math.cos(t2) * l]
        x3 = [0.0, 0.5 * math.sin(t2) * l, -0.5 * math.cos(t2) * l]
        x4 = [0.0, math.sin(t2) * l + 0.5 * math.sin(t1) * l, -math.cos(t2) * l - 0.5 * math.cos(t1) * l]
        q1, q2 = _rotx_q(t1), _rotx_q(t2)
        return np.array(x1 + q1 + z6 + x2 + q2 + z6 + x3 + q2 + z6 + x4 + q1 + z6)
    raise ValueError(f"Experiment {mech} not supported!")


def predictdynamicsmin(mech: str, gps, startobservation, steps: int, usesin: bool = False,
                       dt: float = DT, lengths=None) -> np.ndarray:
    """predictdynamicsmin(mechanism, etype, gps, startobservation, steps; usesin) for one start
    observation (predictdynamics.jl:30-36): returns the predicted CState after `steps` steps."""
    fin = rollout_min(mech, [list(gps)], np.asarray(startobservation, dtype=np.float64)[None, :], steps, usesin, dt)
    return final_cstate(mech, fin[0, 0::2], lengths)


def predictdynamicsmin_batch(mech: str, gps, startobservations, steps: int, usesin: bool = False,
                             dt: float = DT, lengths=None) -> np.ndarray:
    """The experiments' test loop `for i in 1:length(xtest_old) predictdynamicsmin(...)`
    (e.g. P2noise.jl(min):73-76) in one launch: (T, 13 nbodies) predicted CStates."""
    fin = rollout_min(mech, [list(gps)], startobservations, steps, usesin, dt)
    return np.stack([final_cstate(mech, f[0::2], lengths) for f in fin])


def predictdynamics(gps, startobservations, steps: int, getvw, advance, prior_mean=None):
    """predictdynamics(mechanism, gps, startobservation, steps, getvω) for T maximal-coordinate
    trajectories at once (examples/utils/predictdynamics.jl:7-22).

    Per step the G GPs predict the next-step velocities at all T current CStates in ONE mean-only
    device evaluation (no variance: the reference discards it), instead of G x T single-point
    predict_y calls.  The physics stays on the host and is injected:
      gps               a GPBatch whose G slots share the training states (one trial's outputs,
                        CPnoise.jl:37-43), or a list of GPEs
      startobservations (T, d) CStates
      getvw(mu)         mu (G,) -> (vcurr, wcurr)             (the experiment's getvω)
      advance(s, v, w)  one trajectory's state (d,), predicted v, w -> (next state (d,), projection
                        error)  -- projectv! + updatestate! in the reference (ConstrainedDynamics)
      prior_mean        optional callable (d, T) -> (G, T) prior means added to the GP means for a
                        GPBatch (a GPE adds its own mean)
    Returns (final states (T, d), mean projection error per trajectory (T,))."""
    S = np.array(startobservations, dtype=np.float64)
    if S.ndim == 1:
        S = S[None, :]
    T = S.shape[0]
    err = np.zeros(T)
    for _ in range(steps):
        obs = np.ascontiguousarray(S.T)  # (d, T)
        if isinstance(gps, GPBatch):
            gps.set_test(obs)
            mu, _ = gps.predict(variance=False)  # (G, T)
            if prior_mean is not None:
                mu = mu + np.asarray(prior_mean(obs))
        else:
            mu = np.stack([g.predict_y_mean(obs) for g in gps])
        for t in range(T):
            v, w = getvw(mu[:, t])
            S[t], e = advance(S[t], v, w)
            err[t] += e
    return S, err / max(steps, 1)
