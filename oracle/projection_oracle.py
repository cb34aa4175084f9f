"""ORACLE -- test infrastructure only (imported by tests/ and bench/scratch checkers; never by the
product path).

CPU restatement (numpy + LAPACK getrf/getrs, fp64) of the maximal-coordinate rollout physics that
the reference's predictdynamics uses (examples/utils/predictdynamics.jl:7-22):

  * projectv!  -- GPR's Newton projection of a predicted twist onto the joint constraints
                  (src/projections/implicitProjection.jl:80-107, helpers :1-78);
  * setstates! / discretizestate! / setsolution! / updatestate! / CState(mechanism) -- the state
                  handling of ConstrainedDynamics.jl 0.7.4 (Manifest.toml [[ConstrainedDynamics]],
                  git-tree 2d639b2a..., NOT in the reference tree) that the loop calls;
  * the joint constraint functions g and their velocity Jacobians dg/d(v, w) of the joints the four
                  experiment mechanisms use (examples/utils/data/simulations.jl:7-214):
                  Revolute = Translational3 + Rotational2, Prismatic = Translational2 +
                  Rotational3, Cylindrical = Translational2 + Rotational2.

Parity status: UNPINNED.  ConstrainedDynamics' source is absent and the reference has no tests or
vectors for this path.  What is restated [ext, from the package's
published variational-integrator formulation]:
  x3 = xk + v dt,  q3 = qk * wbar(w) * dt / 2,  wbar(w) = (sqrt(4/dt^2 - w.w), w)   (getx3/getq3)
  Translational: g = C R(qa3)^T (xb3 + R(qb3) pb - xa3) - C pa   (C: I3 or the 2 rows normal to
                 the axis);  Rotational: g = C Im(qa3^-1 * qb3)  (qoffset = identity)
What pins the result independently of those conventions: the projection's fixed point is the KKT
point of  min |s - s_u|^2  s.t.  g(x3(s), q3(s)) = 0  (implicitProjection.jl:60-62), which depends
only on the constraint ZERO SETS and the x3/q3 maps, not on the frame or basis a row is written
in; tests/test_projection.py checks the KKT conditions, the Jacobians against central finite
differences, and the zero sets against the mechanisms' own kinematics (gprx/data.py).

The reference's quirk updateMechanism! `offset = Nbodies` (implicitProjection.jl:36, likely meant
6 Nbodies) writes the wrong slice of s into eqc.lambdasol; nothing on this path reads lambdasol, so it
has no effect on the result and is not restated.
"""
from __future__ import annotations

import math

import numpy as np
import scipy.linalg as sla

DT = 0.01  # mechanism.dt of the experiments (e.g. P2noise.jl:14)

# ---- mechanisms (examples/utils/data/simulations.jl) ----------------------------------------
# body ids 1-based as ConstrainedDynamics' mechanism.bodies; parent 0 = origin.
# sub-joint: (kind, parent, child, pa, pb, axis); kinds: "T3", "T2" (free along axis), "R2" (free
# about axis), "R3".  One list per EqualityConstraint, rows in order.
EX, EY = (1.0, 0.0, 0.0), (0.0, 1.0, 0.0)


def _rev(a, b, axis, pa=(0.0, 0.0, 0.0), pb=(0.0, 0.0, 0.0)):
    return [("T3", a, b, pa, pb, axis), ("R2", a, b, pa, pb, axis)]


def _pri(a, b, axis, pa=(0.0, 0.0, 0.0), pb=(0.0, 0.0, 0.0)):
    return [("T2", a, b, pa, pb, axis), ("R3", a, b, pa, pb, axis)]


def _cyl(a, b, axis, pa=(0.0, 0.0, 0.0), pb=(0.0, 0.0, 0.0)):
    return [("T2", a, b, pa, pb, axis), ("R2", a, b, pa, pb, axis)]


def mechanism(name: str) -> dict:
    """nb bodies and the equality constraints of the experiment mechanism (simulations.jl)."""
    if name == "P1":  # simplependulum2D: l = 1, p2 = [0, 0, l/2] (:10-14, :44)
        return dict(nb=1, eqcs=[_rev(0, 1, EX, pb=(0.0, 0.0, 0.5))])
    if name == "P2":  # doublependulum2D: l1 = l2 = 1, vert11 = [0,0,l1/2], vert12 = -vert11 (:53-60, :85-86)
        return dict(nb=2, eqcs=[_rev(0, 1, EX, pb=(0.0, 0.0, 0.5)),
                                _rev(1, 2, EX, pa=(0.0, 0.0, -0.5), pb=(0.0, 0.0, 0.5))])
    if name == "CP":  # cartpole: prismatic along y, revolute about x, pole l = 0.5 (:107-117, :138-139)
        return dict(nb=2, eqcs=[_pri(0, 1, EY), _rev(1, 2, EX, pb=(0.0, 0.0, 0.25))])
    if name == "FB":  # fourbar: l = 1, vert11 = [0,0,l/2], vert12 = -vert11 (:161-169, :206-209)
        v11, v12 = (0.0, 0.0, 0.5), (0.0, 0.0, -0.5)
        return dict(nb=4, eqcs=[_rev(0, 1, EX, pb=v11),
                                _rev(1, 2, EX, pa=v12, pb=v11) + _cyl(1, 3, EX, pa=v11, pb=v11),
                                _rev(3, 4, EX, pa=v12, pb=v11),
                                _rev(2, 4, EX, pa=v12, pb=v12)])
    raise ValueError(f"Experiment {name} not supported!")


ROWS = {"T3": 3, "T2": 2, "R2": 2, "R3": 3}


def ndims(mech: dict) -> int:
    return sum(ROWS[s[0]] for eqc in mech["eqcs"] for s in eqc)


def normal_rows(axis) -> np.ndarray:
    """Two orthonormal rows spanning the plane normal to the axis (any basis of it gives the same
    projection: the constraint zero set is what the Newton fixed point depends on)."""
    a = np.asarray(axis, dtype=np.float64)
    a = a / np.linalg.norm(a)
    t = np.array([0.0, 0.0, 1.0]) if abs(a[2]) < 0.9 else np.array([1.0, 0.0, 0.0])
    v1 = np.cross(a, t)
    v1 /= np.linalg.norm(v1)
    v2 = np.cross(a, v1)
    return np.stack([v1, v2])


def cmat(kind, axis) -> np.ndarray:
    return np.eye(3) if kind in ("T3", "R3") else normal_rows(axis)


# ---- quaternions (w, x, y, z), Hamilton product ----------------------------------------------
def qmul(p, q):
    p0, pv = p[0], p[1:]
    q0, qv = q[0], q[1:]
    return np.concatenate([[p0 * q0 - pv @ qv], p0 * qv + q0 * pv + np.cross(pv, qv)])


def qconj(q):
    return np.array([q[0], -q[1], -q[2], -q[3]])


def rot(q, p):
    """R(q) p = (q0^2 - |qv|^2) p + 2 qv (qv.p) + 2 q0 qv x p."""
    q0, qv = q[0], q[1:]
    p = np.asarray(p, dtype=np.float64)
    return (q0 * q0 - qv @ qv) * p + 2.0 * qv * (qv @ p) + 2.0 * q0 * np.cross(qv, p)


def skew(v):
    return np.array([[0.0, -v[2], v[1]], [v[2], 0.0, -v[0]], [-v[1], v[0], 0.0]])


def Lmat(p):
    """p * q = Lmat(p) q."""
    M = np.empty((4, 4))
    M[0, 0] = p[0]
    M[0, 1:] = -p[1:]
    M[1:, 0] = p[1:]
    M[1:, 1:] = p[0] * np.eye(3) + skew(p[1:])
    return M


def Rmat(q):
    """p * q = Rmat(q) p."""
    M = np.empty((4, 4))
    M[0, 0] = q[0]
    M[0, 1:] = -q[1:]
    M[1:, 0] = q[1:]
    M[1:, 1:] = q[0] * np.eye(3) - skew(q[1:])
    return M


def drot(q, p):
    """d (R(q) p) / dq  (3 x 4), of the polynomial formula of rot."""
    q0, qv = q[0], q[1:]
    p = np.asarray(p, dtype=np.float64)
    J = np.empty((3, 4))
    J[:, 0] = 2.0 * q0 * p + 2.0 * np.cross(qv, p)
    J[:, 1:] = -2.0 * np.outer(p, qv) + 2.0 * (qv @ p) * np.eye(3) + 2.0 * np.outer(qv, p) - 2.0 * q0 * skew(p)
    return J


CONJ = np.diag([1.0, -1.0, -1.0, -1.0])


def wbar_step(qk, w, dt=DT):
    """getq3: qk * wbar(w, dt) * dt / 2 with wbar = (sqrt(4/dt^2 - w.w), w), in the reference's
    evaluation order ((qk * wbar) * dt) / 2."""
    wb = np.concatenate([[math.sqrt(4.0 / dt ** 2 - float(w @ w))], w])
    return qmul(qk, wb) * dt / 2.0


def dq3_dw(qk, w, dt=DT):
    """d q3 / d w (4 x 3) for q3 = qk * (sqrt(4/dt^2 - w.w), w) * dt / 2."""
    s = math.sqrt(4.0 / dt ** 2 - float(w @ w))
    Wp = np.vstack([-w[None, :] / s, np.eye(3)])  # d wbar / d w
    return Lmat(qk) @ Wp * (dt / 2.0)


# ---- mechanism state --------------------------------------------------------------------------
class State:
    """Per body: current xc, qc, vc, wc; discrete xk, qk; solution vsol, wsol (ConstrainedDynamics
    State fields used on this path)."""

    def __init__(self, cstate, nb, dt=DT):
        c = np.asarray(cstate, dtype=np.float64).reshape(nb, 13)
        self.nb, self.dt = nb, dt
        self.xc, self.qc = c[:, 0:3].copy(), c[:, 3:7].copy()
        self.vc, self.wc = c[:, 7:10].copy(), c[:, 10:13].copy()
        # setstates! -> discretizestate! (xk = xc + vc dt, qk = qc * wbar(wc) dt/2) -> setsolution!
        self.xk = self.xc + self.vc * dt
        self.qk = np.stack([wbar_step(self.qc[b], self.wc[b], dt) for b in range(nb)])
        self.vsol, self.wsol = self.vc.copy(), self.wc.copy()

    def x3(self, b):
        return self.xk[b] + self.vsol[b] * self.dt

    def q3(self, b):
        return wbar_step(self.qk[b], self.wsol[b], self.dt)

    def cstate(self):
        """CState(mechanism): [xc, qc, vc, wc] per body (src/CState.jl:60-64)."""
        return np.concatenate([np.concatenate([self.xc[b], self.qc[b], self.vc[b], self.wc[b]])
                               for b in range(self.nb)])

    def update(self):
        """updatestate!: current <- discrete / solution, then the next discrete position."""
        dt = self.dt
        for b in range(self.nb):
            self.xc[b], self.qc[b] = self.xk[b].copy(), self.qk[b].copy()
            self.vc[b], self.wc[b] = self.vsol[b].copy(), self.wsol[b].copy()
            self.xk[b] = self.xk[b] + self.vsol[b] * dt
            self.qk[b] = wbar_step(self.qk[b], self.wsol[b], dt)


def _pose(st: State, b):
    if b == 0:
        return np.zeros(3), np.array([1.0, 0.0, 0.0, 0.0])
    return st.x3(b - 1), st.q3(b - 1)


def constraints(mech: dict, st: State) -> np.ndarray:
    """g(mechanism): every equality constraint's rows at x3, q3 (implicitProjection.jl:64-73)."""
    out = []
    for eqc in mech["eqcs"]:
        for kind, a, b, pa, pb, axis in eqc:
            xa, qa = _pose(st, a)
            xb, qb = _pose(st, b)
            C = cmat(kind, axis)
            if kind[0] == "T":
                e = rot(qconj(qa), xb + rot(qb, pb) - xa) - np.asarray(pa)
            else:
                e = qmul(qconj(qa), qb)[1:]
            out.append(C @ e)
    return np.concatenate(out)


def jacobian(mech: dict, st: State) -> np.ndarray:
    """G = dg / d(v_1, w_1, ..., v_nb, w_nb) at x3, q3 (ConstrainedDynamics.d g d^r vel, the blocks
    updateF! writes, implicitProjection.jl:1-18)."""
    nb, dt = st.nb, st.dt
    nd = ndims(mech)
    G = np.zeros((nd, 6 * nb))
    r = 0
    for eqc in mech["eqcs"]:
        for kind, a, b, pa, pb, axis in eqc:
            C = cmat(kind, axis)
            n = C.shape[0]
            xa, qa = _pose(st, a)
            xb, qb = _pose(st, b)
            ob = 6 * (b - 1)
            dqb = dq3_dw(st.qk[b - 1], st.wsol[b - 1], dt)
            if kind[0] == "T":
                RaT = np.array([rot(qconj(qa), e) for e in np.eye(3)]).T  # R(qa)^T
                G[r:r + n, ob:ob + 3] += C @ RaT * dt
                G[r:r + n, ob + 3:ob + 6] += C @ RaT @ drot(qb, pb) @ dqb
                if a > 0:
                    oa = 6 * (a - 1)
                    y = xb + rot(qb, pb) - xa
                    dqa = dq3_dw(st.qk[a - 1], st.wsol[a - 1], dt)
                    G[r:r + n, oa:oa + 3] += -C @ RaT * dt
                    G[r:r + n, oa + 3:oa + 6] += C @ drot(qconj(qa), y) @ CONJ @ dqa
            else:
                P = np.hstack([np.zeros((3, 1)), np.eye(3)])  # Im part
                G[r:r + n, ob + 3:ob + 6] += C @ P @ Lmat(qconj(qa)) @ dqb
                if a > 0:
                    oa = 6 * (a - 1)
                    dqa = dq3_dw(st.qk[a - 1], st.wsol[a - 1], dt)
                    G[r:r + n, oa + 3:oa + 6] += C @ P @ Rmat(qb) @ CONJ @ dqa
            r += n
    return G


def _set_solution(st: State, s):
    nb = st.nb
    for b in range(nb):
        st.vsol[b] = s[6 * b:6 * b + 3]
        st.wsol[b] = s[6 * b + 3:6 * b + 6]


def projectv(mech: dict, st: State, vu, wu, newton_iter: int = 100, eps: float = 1e-10, regularizer: float = 0.0):
    """projectv!(vu, wu, mechanism; newtonIter, eps, regularizer) (implicitProjection.jl:80-107).
    Leaves the solution in st.vsol / st.wsol (updateMechanism!) and returns (v, w, iterations)."""
    nb = st.nb
    nd = ndims(mech)
    n6 = 6 * nb
    F = np.zeros((n6 + nd, n6 + nd))
    F[np.arange(n6), np.arange(n6)] = 1.0
    s = np.zeros(n6 + nd)
    for b in range(nb):  # updateS!
        s[6 * b:6 * b + 3] = vu[b]
        s[6 * b + 3:6 * b + 6] = wu[b]
    su = s[:n6].copy()
    _set_solution(st, s)
    G = jacobian(mech, st)  # updateF!
    F[n6:, :n6] = G
    F[:n6, n6:] = G.T
    F = F + np.eye(n6 + nd) * regularizer

    def f(s, Gv):
        return np.concatenate([-su + s[:n6] + Gv.T @ s[n6:], constraints(mech, st)])

    it = 0
    for it in range(1, newton_iter + 1):
        G = jacobian(mech, st)
        F[n6:, :n6] = G
        F[:n6, n6:] = G.T
        ds = sla.lu_solve(sla.lu_factor(F, check_finite=False), f(s, F[n6:, :n6]), check_finite=False)  # F \ f(s)
        s = s - ds
        _set_solution(st, s)
        if np.linalg.norm(f(s, F[n6:, :n6])) < eps and np.linalg.norm(ds) < eps:
            break
    v = [s[6 * b:6 * b + 3].copy() for b in range(nb)]
    w = [s[6 * b + 3:6 * b + 6].copy() for b in range(nb)]
    return v, w, it


def getvw(mu, vw_indices, nb):
    """The experiments' getvw: mu_k placed at CState position vw_indices[k] (1-based; body b's v at
    13(b-1) + 8..10, w at 11..13), zero elsewhere (e.g. P2noise.jl:46, CPnoise.jl:47)."""
    c = np.zeros(13 * nb)
    for k, i in enumerate(vw_indices):
        c[i - 1] = mu[k]
    c = c.reshape(nb, 13)
    return [c[b, 7:10].copy() for b in range(nb)], [c[b, 10:13].copy() for b in range(nb)]


def predictdynamics(mech_name: str, predict, start, steps: int, vw_indices, regularizer: float = 0.0, dt: float = DT):
    """predictdynamics(mechanism, gps, startobservation, steps, getvw; regularizer)
    (examples/utils/predictdynamics.jl:7-22) for one trajectory.  predict(cstate (d,)) -> mu (G,)
    (the G GPs' predict_y means).  Returns (final CState, mean projection error per step)."""
    mech = mechanism(mech_name)
    nb = mech["nb"]
    st = State(start, nb, dt)
    obs = np.asarray(start, dtype=np.float64).copy()
    perr = 0.0
    for _ in range(steps):
        mu = predict(obs)
        vu, wu = getvw(mu, vw_indices, nb)
        v, w, _ = projectv(mech, st, vu, wu, regularizer=regularizer)
        perr += float(np.linalg.norm(np.concatenate([np.concatenate([v[b] - vu[b] for b in range(nb)]),
                                                     np.concatenate([w[b] - wu[b] for b in range(nb)])])))
        st.update()
        obs = st.cstate()
    st.update()
    return st.cstate(), perr / steps
