"""Maximal-coordinate rollout physics on the MI355X (include/gprx.h gprx_projectv,
gprx_rollout_max).

`projectv` is GPR's projectv! (src/projections/implicitProjection.jl:80-107): the Newton projection
of a predicted twist (v, w per body) onto the mechanism's joint constraints, for many mechanism
states in one launch.  `predictdynamics` is examples/utils/predictdynamics.jl:7-22 for many test
trajectories in one launch: per step the G GPs' mean predictions at the current CState, getvw,
projectv! and updatestate!, all on the device.

Mechanisms are the experiments' (examples/utils/data/simulations.jl): P1 pendulum, P2 double
pendulum, CP cart-pole, FB four-bar (which the experiments project with regularizer=1e-10,
FBnoise.jl:43).  The constraint functions and the state update restate ConstrainedDynamics 0.7.4
(absent from the reference tree; oracle/projection_oracle.py documents what is restated and what
pins it).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L
from .batch import Context, GPBatch
from .rollout import MECH

NBODIES = {"P1": 1, "P2": 2, "CP": 2, "FB": 4}
REGULARIZER = {"P1": 0.0, "P2": 0.0, "CP": 0.0, "FB": 1e-10}  # the experiments' projectv! settings
DT = 0.01


def getvw(mu, vw_indices, nb: int) -> np.ndarray:
    """The experiments' getvw (e.g. P2noise.jl:46): mu_k at 1-based CState position vw_indices[k],
    zero elsewhere, returned as (..., 6 nb) = (v_1, w_1, ..., v_nb, w_nb)."""
    mu = np.asarray(mu, dtype=np.float64)
    c = np.zeros(mu.shape[:-1] + (13 * nb,))
    for k, i in enumerate(vw_indices):
        c[..., i - 1] = mu[..., k]
    c = c.reshape(mu.shape[:-1] + (nb, 13))
    return c[..., 7:13].reshape(mu.shape[:-1] + (6 * nb,))


def projectv(mech: str, cstates, vw_pred, regularizer: float | None = None, newton_iter: int = 100, eps: float = 1e-10,
             dt: float = DT, ctx: Context | None = None):
    """projectv!(vu, wu, mechanism; newtonIter, eps, regularizer) for T mechanism states.
    cstates (T, 13 nb): the mechanism's CState (setstates!); vw_pred (T, 6 nb): predicted (v, w) per
    body.  Returns (vw (T, 6 nb) projected, iterations (T,), status (T,): 1 = singular KKT matrix)."""
    if mech not in MECH:
        raise ValueError(f"Experiment {mech} not supported!")
    nb = NBODIES[mech]
    cs = np.ascontiguousarray(np.atleast_2d(cstates), dtype=np.float64)
    vw = np.ascontiguousarray(np.atleast_2d(vw_pred), dtype=np.float64)
    T = cs.shape[0]
    if cs.shape != (T, 13 * nb) or vw.shape != (T, 6 * nb):
        raise ValueError(f"cstates must be (T, {13 * nb}) and vw_pred (T, {6 * nb})")
    reg = REGULARIZER[mech] if regularizer is None else float(regularizer)
    ctx = ctx or _default_ctx()
    out = np.empty((T, 6 * nb))
    it = np.empty(T, dtype=np.int32)
    st = np.empty(T, dtype=np.int32)
    L.check(L.lib.gprx_projectv(ctx.h, MECH[mech], float(dt), T, L.dptr(cs), L.dptr(vw), reg, int(newton_iter), float(eps),
                                L.dptr(out), L.iptr(it), L.iptr(st)), ctx.h)
    return out, it, st


def vi_step(mech: str, cstates, regularizer: float | None = None, newton_iter: int = 100, eps: float = 1e-10,
            dt: float = DT, ctx: Context | None = None):
    """One variational-integrator step (ConstrainedDynamics newton! after setstates!, the MeanDynamics
    prior mean of src/mDynamics.jl:41-60) for T states on the device (k_vi_step, one wave each); the
    same contract as the host restatement gprx.vi.vi_step: cstates (T, 13 nb) -> (solution CStates
    (T, 13 nb) [x2, q2, v2, w2] per body, NaN rows for failed states; iterations (T,); status (T,):
    0 converged, 1 not converged, 2 failed)."""
    from . import vi

    if mech not in MECH:
        raise ValueError(f"Experiment {mech} not supported!")
    nb = NBODIES[mech]
    cs = np.ascontiguousarray(np.atleast_2d(cstates), dtype=np.float64)
    T = cs.shape[0]
    if cs.shape != (T, 13 * nb):
        raise ValueError(f"cstates must be (T, {13 * nb})")
    reg = vi.REGULARIZER[mech] if regularizer is None else float(regularizer)
    ctx = ctx or _default_ctx()
    out = np.empty((T, 13 * nb))
    it = np.empty(T, dtype=np.int32)
    st = np.empty(T, dtype=np.int32)
    L.check(L.lib.gprx_vi_step(ctx.h, MECH[mech], float(dt), T, L.dptr(cs), reg, int(newton_iter), float(eps),
                               L.dptr(out), L.iptr(it), L.iptr(st)), ctx.h)
    return out, it, st


def predictdynamics(mech: str, groups, start, steps: int, vw_indices, regularizer: float | None = None,
                    traj_group=None, dt: float = DT, ctx: Context | None = None):
    """predictdynamics(mechanism, gps, startobservation, steps, getvw; regularizer) for T
    trajectories.  groups: list of rollout groups, each a list of G GP references -- (GPBatch,
    slot) pairs or MeanZero GPEs -- factorised at their hyperparameters; start (T, 13 nb) CStates;
    vw_indices: the experiment's 1-based vwindices (output g's CState position).  Returns (final
    CStates (T, 13 nb), mean projection error per step (T,), status (T,))."""
    from .rollout import _slot_ref

    if mech not in MECH:
        raise ValueError(f"Experiment {mech} not supported!")
    nb = NBODIES[mech]
    S = np.ascontiguousarray(np.atleast_2d(start), dtype=np.float64)
    T = S.shape[0]
    if S.shape != (T, 13 * nb):
        raise ValueError(f"start must be (T, {13 * nb})")
    G = len(vw_indices)
    refs = []
    for grp in groups:
        if len(grp) != G:
            raise ValueError(f"each group needs {G} GPs (one per vw index)")
        refs += [_slot_ref(g) for g in grp]
    tg = np.zeros(T, dtype=np.int32) if traj_group is None else np.ascontiguousarray(traj_group, dtype=np.int32)
    batches = (C.c_void_p * len(refs))(*[b.h.value for b, _ in refs])
    slots = np.ascontiguousarray([s for _, s in refs], dtype=np.int32)
    vwi = np.ascontiguousarray(vw_indices, dtype=np.int32)
    reg = REGULARIZER[mech] if regularizer is None else float(regularizer)
    ctx = ctx or refs[0][0].ctx
    out = np.empty((T, 13 * nb))
    pe = np.empty(T)
    st = np.empty(T, dtype=np.int32)
    L.check(L.lib.gprx_rollout_max(ctx.h, MECH[mech], float(dt), int(steps), reg, len(groups), batches, L.iptr(slots), G,
                                   L.iptr(vwi), T, L.iptr(tg), L.dptr(S), L.dptr(out), L.dptr(pe), L.iptr(st)), ctx.h)
    return out, pe, st


def _default_ctx():
    """The context of this process's device, in this order:
      * GPRX_DEVICE (an explicit device index);
      * torch's current device, when this process has already initialised torch's HIP runtime (a
        caller that chose a GPU with torch.cuda.set_device(k) keeps it; nothing is initialised here);
      * GPU LOCAL_RANK (mod the visible devices, as shard.init_ranks binds a rank; 0 without a
        launcher)."""
    import os
    import sys

    from .batch import default_context

    return default_context(default_device(int(L.lib.gprx_device_count()), os.environ, sys.modules.get("torch")))


def default_device(ndev: int, env, torch=None) -> int:
    """_default_ctx's device index (ndev visible devices, env a mapping, torch the imported module
    or None)."""
    n = max(1, int(ndev))
    if str(env.get("GPRX_DEVICE", "")).strip():
        return int(env["GPRX_DEVICE"]) % n
    if torch is not None and torch.cuda.is_initialized():
        return int(torch.cuda.current_device()) % n
    return int(env.get("LOCAL_RANK", "0") or 0) % n
