"""One variational-integrator step of the experiment mechanisms: the prior mean of GPR's
MeanDynamics (src/mDynamics.jl:41-60) -- setstates!(mechanism, CState(x)), then
ConstrainedDynamics.newton!(mechanism), then getμ = CState(mechanism, usesolution=true)[vωindices]
(:57-60) -- for many states at once, on the host (the reference keeps the mean in Julia; the north
star keeps the mDynamics mean-function cache on the host too).  μ(X) does not depend on the GP
hyperparameters (num_params = 0, :29), so it is computed once per training set and the device sees
y - μ(X); in a rollout it is evaluated at every step's states.

The discrete mechanics restate ConstrainedDynamics 0.7.4 (Manifest.toml; its source is not in the
reference tree): per body, with current state (x1, q1, v1, w1), discrete pose x2 = x1 + v1 dt,
q2 = q1 * wbar(w1) dt/2 (discretizestate!), the step solves for (v2, w2) and the constraint impulses
lambda

    m ((v2 - v1)/dt + [0, 0, 9.81]) - sum_c (dg_c/dx2)^T lambda_c = 0
    (sq2 I + [w2 x]) J w2 - (sq1 I - [w1 x]) J w1 - sum_c (dg_c/dphi2)^T lambda_c = 0,
        sq = sqrt(4/dt^2 - w.w)
    g(x3, q3) = 0,  x3 = x2 + v2 dt,  q3 = q2 * wbar(w2) dt/2,  wbar(w) = (sqrt(4/dt^2 - w.w), w)

by Newton's method (newton!, eps 1e-10), where dg/dphi2 is the derivative along q2 * (1, phi)
(ConstrainedDynamics' dg/d^r pos, the k-pose force Jacobian) and the joint constraint functions are
those of the projection (Revolute = T3 + R2, Prismatic = T2 + R3, Cylindrical = T2 + R2).  Bodies
and inertias as examples/utils/data/simulations.jl builds them: m = 1, J = I m l^2 / 12 (P1, P2,
FB: l = 1; the cart-pole's pole l = 0.5; its cart a 0.2 x 0.3 x 0.1 box, diag(y^2+z^2, x^2+z^2,
x^2+y^2) m / 12), gravity -9.81 along z, dt = 0.01.  The four-bar's loop constraints are redundant
(rank 22 of 24): the impulses are regularised by 1e-10 (the experiments' projectv! setting,
FBnoise.jl:43), which leaves the velocities unique.

Parity status: UNPINNED (ConstrainedDynamics is absent).  oracle/vi_oracle.py restates the same step
independently from the discrete action (finite-difference discrete Euler-Lagrange equations, a
generic root finder), and tests/test_vi.py pins both by the constraint residual at the next pose,
the continuous-time limit of the pendulum (w' = w - dt (3 g / 2 l) sin theta), and energy
behaviour over many steps.
"""
from __future__ import annotations

import numpy as np

DT = 0.01
GRAV = 9.81  # |mechanism.g| (simulations.jl:10, :107; ConstrainedDynamics' default for P2 / FB)
EX, EY = np.array([1.0, 0.0, 0.0]), np.array([0.0, 1.0, 0.0])

# sub-joint: (kind, parent, child, pa, pb, axis); parent 0 = origin; kinds T3 / T2 (free along
# axis) / R2 (free about axis) / R3
_Z = (0.0, 0.0, 0.0)


def _revolute(a, b, axis, pa=_Z, pb=_Z):
    return [("T3", a, b, pa, pb, axis), ("R2", a, b, pa, pb, axis)]


def _prismatic(a, b, axis, pa=_Z, pb=_Z):
    return [("T2", a, b, pa, pb, axis), ("R3", a, b, pa, pb, axis)]


def _cylindrical(a, b, axis, pa=_Z, pb=_Z):
    return [("T2", a, b, pa, pb, axis), ("R2", a, b, pa, pb, axis)]


def _box_inertia(m, x, y, z):
    return np.diag([y * y + z * z, x * x + z * z, x * x + y * y]) * m / 12.0


MECHANISMS = {
    # simplependulum2D: Cylinder(r, l=1, m=1), J = I m l^2 / 12, Revolute(origin, link, ex; p2=[0,0,l/2])
    "P1": dict(nb=1, m=[1.0], J=[np.eye(3) / 12.0], joints=_revolute(0, 1, EX, pb=(0.0, 0.0, 0.5))),
    # doublependulum2D: two Box(.1, .1, 1, 1) links, J = I / 12
    "P2": dict(nb=2, m=[1.0, 1.0], J=[np.eye(3) / 12.0] * 2,
               joints=_revolute(0, 1, EX, pb=(0.0, 0.0, 0.5)) + _revolute(1, 2, EX, pa=(0.0, 0.0, -0.5),
                                                                          pb=(0.0, 0.0, 0.5))),
    # cartpole: Box(.2, .3, .1, 1) cart on a prismatic joint along y, Cylinder pole l = .5, J = I / 48
    "CP": dict(nb=2, m=[1.0, 1.0], J=[_box_inertia(1.0, 0.2, 0.3, 0.1), np.eye(3) / 48.0],
               joints=_prismatic(0, 1, EY) + _revolute(1, 2, EX, pb=(0.0, 0.0, 0.25))),
    # fourbar: four Box(.1, .1, 1, 1) links, J = I / 12
    "FB": dict(nb=4, m=[1.0] * 4, J=[np.eye(3) / 12.0] * 4,
               joints=_revolute(0, 1, EX, pb=(0.0, 0.0, 0.5))
               + _revolute(1, 2, EX, pa=(0.0, 0.0, -0.5), pb=(0.0, 0.0, 0.5))
               + _cylindrical(1, 3, EX, pa=(0.0, 0.0, 0.5), pb=(0.0, 0.0, 0.5))
               + _revolute(3, 4, EX, pa=(0.0, 0.0, -0.5), pb=(0.0, 0.0, 0.5))
               + _revolute(2, 4, EX, pa=(0.0, 0.0, -0.5), pb=(0.0, 0.0, -0.5))),
}
REGULARIZER = {"P1": 0.0, "P2": 0.0, "CP": 0.0, "FB": 1e-10}
ROWS = {"T3": 3, "T2": 2, "R2": 2, "R3": 3}


def _rows_normal(axis):
    a = np.asarray(axis, dtype=np.float64)
    a = a / np.linalg.norm(a)
    t = np.array([0.0, 0.0, 1.0]) if abs(a[2]) < 0.9 else np.array([1.0, 0.0, 0.0])
    u = np.cross(a, t)
    u /= np.linalg.norm(u)
    return np.stack([u, np.cross(a, u)])


def _cmat(kind, axis):
    return np.eye(3) if kind in ("T3", "R3") else _rows_normal(axis)


# ---- quaternions (w, x, y, z), batched over the leading axes ----------------------------------
def qmul(p, q):
    p0, pv, q0, qv = p[..., :1], p[..., 1:], q[..., :1], q[..., 1:]
    w = p0 * q0 - np.sum(pv * qv, axis=-1, keepdims=True)
    return np.concatenate([w, p0 * qv + q0 * pv + np.cross(pv, qv)], axis=-1)


def qconj(q):
    return q * np.array([1.0, -1.0, -1.0, -1.0])


def rotmat(q):
    """R(q) (..., 3, 3) of a unit quaternion."""
    w, x, y, z = q[..., 0], q[..., 1], q[..., 2], q[..., 3]
    R = np.empty(q.shape[:-1] + (3, 3))
    R[..., 0, 0] = w * w + x * x - y * y - z * z
    R[..., 0, 1] = 2 * (x * y - w * z)
    R[..., 0, 2] = 2 * (x * z + w * y)
    R[..., 1, 0] = 2 * (x * y + w * z)
    R[..., 1, 1] = w * w - x * x + y * y - z * z
    R[..., 1, 2] = 2 * (y * z - w * x)
    R[..., 2, 0] = 2 * (x * z - w * y)
    R[..., 2, 1] = 2 * (y * z + w * x)
    R[..., 2, 2] = w * w - x * x - y * y + z * z
    return R


def skew(v):
    S = np.zeros(v.shape[:-1] + (3, 3))
    S[..., 0, 1], S[..., 0, 2] = -v[..., 2], v[..., 1]
    S[..., 1, 0], S[..., 1, 2] = v[..., 2], -v[..., 0]
    S[..., 2, 0], S[..., 2, 1] = -v[..., 1], v[..., 0]
    return S


def lmat(p):
    """p * q = lmat(p) q  (..., 4, 4)."""
    M = np.zeros(p.shape[:-1] + (4, 4))
    M[..., 0, 0] = p[..., 0]
    M[..., 0, 1:] = -p[..., 1:]
    M[..., 1:, 0] = p[..., 1:]
    M[..., 1:, 1:] = p[..., 0, None, None] * np.eye(3) + skew(p[..., 1:])
    return M


def rmat(q):
    """p * q = rmat(q) p  (..., 4, 4)."""
    M = np.zeros(q.shape[:-1] + (4, 4))
    M[..., 0, 0] = q[..., 0]
    M[..., 0, 1:] = -q[..., 1:]
    M[..., 1:, 0] = q[..., 1:]
    M[..., 1:, 1:] = q[..., 0, None, None] * np.eye(3) - skew(q[..., 1:])
    return M


def wbar(w, dt=DT):
    return np.concatenate([np.sqrt(4.0 / dt ** 2 - np.sum(w * w, axis=-1, keepdims=True)), w], axis=-1)


def step_q(q, w, dt=DT):
    """q * wbar(w) * dt / 2 (getq3 / discretizestate!)."""
    return qmul(q, wbar(w, dt)) * (dt / 2.0)


# ---- constraints: values and Jacobians along (x, phi) of each body, phi: q -> q * (1, phi) ------
def _pose(x, q, b):
    T = x.shape[0]
    if b == 0:
        return np.zeros((T, 3)), np.tile([1.0, 0.0, 0.0, 0.0], (T, 1))
    return x[:, b - 1], q[:, b - 1]


def constraints(mech: dict, x, q):
    """g at poses x (T, nb, 3), q (T, nb, 4): (T, nd)."""
    out = []
    for kind, a, b, pa, pb, axis in mech["joints"]:
        xa, qa = _pose(x, q, a)
        xb, qb = _pose(x, q, b)
        C = _cmat(kind, axis)
        if kind[0] == "T":
            y = xb + np.einsum("tij,j->ti", rotmat(qb), np.asarray(pb)) - xa
            e = np.einsum("tji,tj->ti", rotmat(qa), y) - np.asarray(pa)
        else:
            e = qmul(qconj(qa), qb)[:, 1:]
        out.append(e @ C.T)
    return np.concatenate(out, axis=1)


def jac_phi(mech: dict, x, q):
    """dg / d(x_1, phi_1, ..., x_nb, phi_nb) at poses x, q: (T, nd, 6 nb)."""
    T, nb = x.shape[0], mech["nb"]
    nd = sum(ROWS[j[0]] for j in mech["joints"])
    Jg = np.zeros((T, nd, 6 * nb))
    r = 0
    for kind, a, b, pa, pb, axis in mech["joints"]:
        C = _cmat(kind, axis)
        n = C.shape[0]
        xa, qa = _pose(x, q, a)
        xb, qb = _pose(x, q, b)
        Ra, Rb = rotmat(qa), rotmat(qb)
        RaT = np.swapaxes(Ra, -1, -2)
        ob = 6 * (b - 1)
        if kind[0] == "T":
            y = xb + np.einsum("tij,j->ti", Rb, np.asarray(pb)) - xa
            u = np.einsum("tij,tj->ti", RaT, y)  # R(qa)^T y
            Jg[:, r:r + n, ob:ob + 3] += C @ RaT
            Jg[:, r:r + n, ob + 3:ob + 6] += C @ (RaT @ Rb @ (-2.0 * skew(np.asarray(pb, dtype=np.float64))))
            if a > 0:
                oa = 6 * (a - 1)
                Jg[:, r:r + n, oa:oa + 3] -= C @ RaT
                Jg[:, r:r + n, oa + 3:oa + 6] += C @ (2.0 * skew(u))
        else:
            rq = qmul(qconj(qa), qb)
            Jg[:, r:r + n, ob + 3:ob + 6] += C @ lmat(rq)[:, 1:, 1:]
            if a > 0:
                oa = 6 * (a - 1)
                Jg[:, r:r + n, oa + 3:oa + 6] -= C @ rmat(rq)[:, 1:, 1:]
        r += n
    return Jg


def _dphi_dw(q2, q3, w, dt=DT):
    """d phi3 / d w for q3(w) = q2 * wbar(w) dt/2, phi3 the variation along q3 * (1, phi): (T, 3, 3)."""
    s = np.sqrt(4.0 / dt ** 2 - np.sum(w * w, axis=-1))
    dwb = np.zeros(w.shape[:-1] + (4, 3))
    dwb[..., 0, :] = -w / s[..., None]
    dwb[..., 1:, :] = np.eye(3)
    dq3 = lmat(q2) @ dwb * (dt / 2.0)
    return (np.swapaxes(lmat(q3), -1, -2) @ dq3)[..., 1:, :]


# ---- the step -----------------------------------------------------------------------------------
def vi_step(mech_name: str, cstates, dt: float = DT, eps: float = 1e-10, newton_iter: int = 100):
    """newton!(mechanism) after setstates!(mechanism, CState(x)) for T states.  cstates (T, 13 nb)
    -> the solution CStates (T, 13 nb) = [x2, q2, v2, w2] per body (CState(mechanism,
    usesolution=true), src/CState.jl:66-71), iterations (T,), status (T,) (1: not converged; 2:
    failed, where the reference throws (DomainError / SingularException): its row is NaN)."""
    mech = MECHANISMS[mech_name]
    nb = mech["nb"]
    cs = np.atleast_2d(np.asarray(cstates, dtype=np.float64))
    T = cs.shape[0]
    c = cs.reshape(T, nb, 13)
    x1, q1, v1, w1 = c[..., 0:3], c[..., 3:7], c[..., 7:10], c[..., 10:13]
    x2 = x1 + v1 * dt
    q2 = step_q(q1, w1, dt)
    m = np.asarray(mech["m"])
    J = np.stack(mech["J"])  # (nb, 3, 3)
    n6 = 6 * nb
    Gpos = jac_phi(mech, x2, q2)  # (T, nd, n6): the k-pose force Jacobian (fixed during the solve)
    nd = Gpos.shape[1]
    Jw1 = np.einsum("bij,tbj->tbi", J, w1)
    sq1 = np.sqrt(4.0 / dt ** 2 - np.sum(w1 * w1, axis=-1))
    mom1 = sq1[..., None] * Jw1 - np.cross(w1, Jw1)  # (sq1 I - [w1 x]) J w1
    reg = REGULARIZER[mech_name]
    v2, w2 = v1.copy(), w1.copy()  # setsolution!: the solution starts at the current velocities
    lam = np.zeros((T, nd))
    it = np.zeros(T, dtype=np.int32)
    done = np.zeros(T, dtype=bool)
    failed = np.zeros(T, dtype=bool)

    def residual(a, v2a, w2a, lama):
        """residual of the states a (index array) at (v2a, w2a, lama)"""
        Jw2 = np.einsum("bij,tbj->tbi", J, w2a)
        sq2 = np.sqrt(4.0 / dt ** 2 - np.sum(w2a * w2a, axis=-1))
        dT = m[None, :, None] * ((v2a - v1[a]) / dt + np.array([0.0, 0.0, GRAV]))
        dR = sq2[..., None] * Jw2 + np.cross(w2a, Jw2) - mom1[a]
        d = np.concatenate([dT, dR], axis=-1).reshape(len(a), n6) - np.einsum("tcj,tc->tj", Gpos[a], lama)
        x3 = x2[a] + v2a * dt
        q3 = step_q(q2[a], w2a, dt)
        return np.concatenate([d, constraints(mech, x3, q3)], axis=1), Jw2, sq2, x3, q3

    a = np.arange(T)  # the states still iterating (converged ones drop out)
    for k in range(1, newton_iter + 1):
        na = len(a)
        f, Jw2, sq2, x3, q3 = residual(a, v2[a], w2[a], lam[a])
        F = np.zeros((na, n6 + nd, n6 + nd))
        for b in range(nb):
            o = 6 * b
            F[:, o:o + 3, o:o + 3] = np.eye(3) * (m[b] / dt)
            # d/dw2 [(sq2 I + [w2 x]) J w2]
            wb = w2[a, b]
            F[:, o + 3:o + 6, o + 3:o + 6] = (sq2[:, b, None, None] * J[b] + skew(wb) @ J[b] - skew(Jw2[:, b])
                                              - Jw2[:, b, :, None] * wb[:, None, :] / sq2[:, b, None, None])
        F[:, :n6, n6:] = -np.swapaxes(Gpos[a], 1, 2)
        Gphi3 = jac_phi(mech, x3, q3)
        for b in range(nb):
            o = 6 * b
            F[:, n6:, o:o + 3] = Gphi3[:, :, o:o + 3] * dt
            F[:, n6:, o + 3:o + 6] = Gphi3[:, :, o + 3:o + 6] @ _dphi_dw(q2[a, b], q3[:, b], w2[a, b], dt)
        if reg:
            F[:, n6:, n6:] -= reg * np.eye(nd)
        # a state whose system is not finite (|w| beyond 2/dt: the reference's sqrt throws a
        # DomainError) or singular (LinearAlgebra's SingularException) fails alone: its solution
        # is NaN and it leaves the iteration; the other states are solved as before
        ds = np.full((na, n6 + nd), np.nan)
        okf = np.nonzero(np.all(np.isfinite(F), axis=(1, 2)) & np.all(np.isfinite(f), axis=1))[0]
        if len(okf):
            try:
                ds[okf] = np.linalg.solve(F[okf], f[okf][..., None])[..., 0]
            except np.linalg.LinAlgError:
                for j in okf:
                    try:
                        ds[j] = np.linalg.solve(F[j], f[j])
                    except np.linalg.LinAlgError:
                        pass
        bad = ~np.all(np.isfinite(ds), axis=1)
        if bad.any():
            failed[a[bad]] = True
            v2[a[bad]] = np.nan
            w2[a[bad]] = np.nan
            a, ds = a[~bad], ds[~bad]
            na = len(a)
            if na == 0:
                break
        v2[a] -= ds[:, :n6].reshape(na, nb, 6)[..., 0:3]
        w2[a] -= ds[:, :n6].reshape(na, nb, 6)[..., 3:6]
        lam[a] -= ds[:, n6:]
        it[a] = k
        fn = np.linalg.norm(residual(a, v2[a], w2[a], lam[a])[0], axis=1)
        conv = (fn < eps) & (np.linalg.norm(ds, axis=1) < eps)
        done[a[conv]] = True
        a = a[~conv]
        if len(a) == 0:
            break
    out = np.concatenate([x2, q2, v2, w2], axis=-1).reshape(T, 13 * nb)
    out[failed] = np.nan
    return out, it, np.where(failed, 2, (~done).astype(np.int32)).astype(np.int32)


def mean_dynamics(mech_name: str, X, vw_indices, dt: float = DT):
    """MeanDynamics(mechanism, getμ(vωindices), k, cache) for every column of X (d x N CStates):
    (G, N) means, row k = output k (mDynamics.jl:41-60).  θ-independent: computed once per training
    set (the single-slot cache of the reference misses on every training column)."""
    sol, _, _ = vi_step(mech_name, np.asarray(X, dtype=np.float64).T, dt)
    idx = np.asarray(vw_indices) - 1
    return sol[:, idx].T.copy()


def simulate(mech_name: str, cstates, steps: int, dt: float = DT):
    """predictdynamics(mechanism, startobservation, steps) of the physics-only baseline
    (examples/utils/predictdynamics.jl:24-28 -> ConstrainedDynamics.simulate!(mechanism, 1:steps+1):
    newton! then updatestate!, steps + 1 times) for T start CStates: the final CStates (T, 13 nb)
    and the states whose Newton solve did not converge at some step (T,)."""
    S = np.atleast_2d(np.asarray(cstates, dtype=np.float64))
    bad = np.zeros(S.shape[0], dtype=np.int32)
    for _ in range(steps + 1):
        S, _, st = vi_step(mech_name, S, dt)  # the solution CState = CState(mechanism) after updatestate!
        bad |= st
    return S, bad
