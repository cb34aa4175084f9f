"""ORACLE -- test infrastructure only (imported by tests/; never by the product path).

An independent restatement of the one-step variational integrator behind GPR's MeanDynamics
(src/mDynamics.jl:41-60 -> ConstrainedDynamics.newton!; ConstrainedDynamics 0.7.4 is NOT in the
reference tree).  Where the product (gprx/vi.py) writes the discrete Euler-Lagrange equations out
analytically and solves them with its own Newton iteration, this oracle starts from the discrete
action and differentiates it numerically:

    L_d(s_a, s_b) = dt (m/2) |(x_b - x_a)/dt|^2 + (2/dt) w^T J w - dt V(x_a),
        w = Im(conj(q_a) * q_b),  V(x) = m 9.81 z
    DEL at the middle pose s2:  D2 L_d(s1, s2) + D1 L_d(s2, s3) + dt G(s2)^T lambda = 0
    constraints at the next pose: g(s3) = 0

with s2 = (x1 + v1 dt, q1 * wbar(w1) dt/2) (discretizestate!) and the unknown next pose
s3 = (x2 + v2 dt, q2 * wbar(w2) dt/2); rotational variations along q -> q * (sqrt(1 - |phi|^2), phi);
D1, D2 and G by central finite differences (step 1e-6); the system solved per state by MINPACK's
Levenberg-Marquardt (scipy.optimize.root(method='lm')), which also copes with the four-bar's
redundant loop constraints.  (With q_b = q_a * wbar(w) dt/2 the rotational term is dt w^T J w / 2,
the kinetic energy; the left-point potential gives the same DEL as any other consistent choice.)

Parity status: UNPINNED (no reference outputs exist); what pins it: the physics tests in
tests/test_vi.py (pendulum continuous-time limit, constraint residual, energy behaviour).
Mechanisms, masses and inertias restated from examples/utils/data/simulations.jl.
"""
from __future__ import annotations

import numpy as np
import scipy.optimize as so

from oracle import projection_oracle as P

DT = 0.01
G0 = 9.81
H = 1e-6

# body masses and inertias (simulations.jl: Δm = ΔJ = 1; link J = I m l^2 / 12, the cart-pole's cart
# a Box(0.2, 0.3, 0.1) with the default box inertia)
BODIES = {
    "P1": ([1.0], [np.eye(3) / 12.0]),
    "P2": ([1.0, 1.0], [np.eye(3) / 12.0] * 2),
    "CP": ([1.0, 1.0], [np.diag([0.3 ** 2 + 0.1 ** 2, 0.2 ** 2 + 0.1 ** 2, 0.2 ** 2 + 0.3 ** 2]) / 12.0,
                        np.eye(3) * 0.5 ** 2 / 12.0]),
    "FB": ([1.0] * 4, [np.eye(3) / 12.0] * 4),
}


def _retract(q, phi):
    return P.qmul(q, np.concatenate([[np.sqrt(1.0 - phi @ phi)], phi]))


def _g(mech, xs, qs):
    """constraint rows at poses xs (nb, 3), qs (nb, 4)."""
    out = []
    for eqc in mech["eqcs"]:
        for kind, a, b, pa, pb, axis in eqc:
            xa, qa = (np.zeros(3), np.array([1.0, 0, 0, 0])) if a == 0 else (xs[a - 1], qs[a - 1])
            xb, qb = (np.zeros(3), np.array([1.0, 0, 0, 0])) if b == 0 else (xs[b - 1], qs[b - 1])
            C = P.cmat(kind, axis)
            if kind[0] == "T":
                e = P.rot(P.qconj(qa), xb + P.rot(qb, pb) - xa) - np.asarray(pa)
            else:
                e = P.qmul(P.qconj(qa), qb)[1:]
            out.append(C @ e)
    return np.concatenate(out)


def _ld(m, J, xa, qa, xb, qb, dt):
    v = (xb - xa) / dt
    w = P.qmul(P.qconj(qa), qb)[1:]
    return dt * 0.5 * m * (v @ v) + (2.0 / dt) * (w @ J @ w) - dt * m * G0 * xa[2]


def _var(f, x, q):
    """d f / d(x, phi) at (x, q) by central differences (6,)."""
    out = np.empty(6)
    for i in range(3):
        e = np.zeros(3)
        e[i] = H
        out[i] = (f(x + e, q) - f(x - e, q)) / (2 * H)
        out[3 + i] = (f(x, _retract(q, e)) - f(x, _retract(q, -e))) / (2 * H)
    return out


def vi_step(mech_name: str, cstate, dt: float = DT):
    """One state (13 nb,) -> the solution CState [x2, q2, v2, w2] per body."""
    mech = P.mechanism(mech_name)
    nb = mech["nb"]
    ms, Js = BODIES[mech_name]
    c = np.asarray(cstate, dtype=np.float64).reshape(nb, 13)
    x1, q1, v1, w1 = c[:, 0:3], c[:, 3:7], c[:, 7:10], c[:, 10:13]
    x2 = x1 + v1 * dt
    q2 = np.stack([P.wbar_step(q1[b], w1[b], dt) for b in range(nb)])
    nd = P.ndims(mech)
    # force Jacobian at the middle pose: dg/d(x_b, phi_b)
    G = np.zeros((nd, 6 * nb))
    for b in range(nb):
        for i in range(6):
            e = np.zeros(3)
            e[i % 3] = H
            xp, xm, qp, qm = x2.copy(), x2.copy(), q2.copy(), q2.copy()
            if i < 3:
                xp[b] += e
                xm[b] -= e
            else:
                qp[b] = _retract(q2[b], e)
                qm[b] = _retract(q2[b], -e)
            G[:, 6 * b + i] = (_g(mech, xp, qp) - _g(mech, xm, qm)) / (2 * H)
    d2 = [_var(lambda x, q, b=b: _ld(ms[b], Js[b], x1[b], q1[b], x, q, dt), x2[b], q2[b]) for b in range(nb)]

    def F(z):
        v2 = z[:3 * nb].reshape(nb, 3)
        w2 = z[3 * nb:6 * nb].reshape(nb, 3)
        lam = z[6 * nb:]
        x3 = x2 + v2 * dt
        q3 = np.stack([P.wbar_step(q2[b], w2[b], dt) for b in range(nb)])
        rows = []
        for b in range(nb):
            d1 = _var(lambda x, q, b=b: _ld(ms[b], Js[b], x, q, x3[b], q3[b], dt), x2[b], q2[b])
            rows.append(d2[b] + d1)
        del_ = np.concatenate(rows) + dt * G.T @ lam
        return np.concatenate([del_ / dt, _g(mech, x3, q3)])

    z0 = np.concatenate([v1.ravel(), w1.ravel(), np.zeros(nd)])
    sol = so.root(F, z0, method="lm", options=dict(xtol=1e-15, ftol=1e-15, maxiter=20000))
    v2 = sol.x[:3 * nb].reshape(nb, 3)
    w2 = sol.x[3 * nb:6 * nb].reshape(nb, 3)
    return np.concatenate([np.concatenate([x2[b], q2[b], v2[b], w2[b]]) for b in range(nb)]), sol
