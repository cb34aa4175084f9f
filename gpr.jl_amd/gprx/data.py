"""Synthetic maximal-coordinate datasets (the reference's `.jls` datasets are git-ignored and absent,
/root/reference/.gitignore:4), generated with the reference's own kinematics.

Per sample: draw minimal coordinates, perturb θ/ω (and the cart's x/v) with N(0, Σ=1e-3) noise
(examples/noise.jl:42), then rebuild x and v from θ/ω exactly as the noise model does
(examples/utils/data/transformations.jl:48-140, Δtsim = 1e-4 from examples/noise.jl:62), and pack
each body as a CState block [x(3), q.w, q.x, q.y, q.z, v(3), ω(3)] (src/CState.jl:25-28).
Targets are the next state (Δt = 0.01, the experiments' mechanism step) at the GP output
coordinates `VW_INDICES` (1-based, examples/maximal_coordinates/*noise.jl).

Link lengths: P1 l=1 (examples/utils/data/simulations.jl:11), P2 l1=l2=1 (:53-54),
CP pole l=0.5 (:111), FB l=1 (:165).
"""
from __future__ import annotations

import json
import math
import pathlib

import numpy as np

DT = 0.01  # mechanism Δt used by the experiments (e.g. CPnoise.jl:19)
DT_SIM = 1e-4  # Δtsim (examples/noise.jl:62)
SIGMA = 1e-3  # Σ (examples/noise.jl:42)
G = 9.81

NBODIES = {"P1": 1, "P2": 2, "CP": 2, "FB": 4}
VW_INDICES = {  # vωindices of the maximal-coordinate experiments
    "P1": [9, 10, 11],  # P1noise.jl:26
    "P2": [9, 10, 22, 23, 11, 24],  # P2noise.jl:25
    "CP": [9, 22, 23, 24],  # CPnoise.jl:28
    "FB": [9, 10, 22, 23, 35, 36, 48, 49, 11, 24, 37, 50],  # FBnoise.jl:24
}
CONFIG_ID = {"P1": 1, "P2": 2, "CP": 3, "FB": 4}

_THETA_FILE = pathlib.Path(__file__).resolve().parent / "theta_config.json"


def load_theta_config() -> dict:
    """The reference's tuned hyper-parameters (examples/config/config.json, keys
    '<ID>_<MAX|MIN><N>' -> [σ_f, ℓ_1..ℓ_d], read at examples/noise.jl:39-41), vendored as data."""
    with open(_THETA_FILE) as f:
        return json.load(f)


def theta_from_params(p, log_noise: float = -2.0) -> np.ndarray:
    """SEArd(log.(p[2:end]), log(p[1])) + GP default logNoise (CPnoise.jl:38-40)
    -> [logσn, logℓ_1..d, logσf]."""
    p = np.asarray(p, dtype=np.float64)
    return np.concatenate([[log_noise], np.log(p[1:]), [np.log(p[0])]])


def theta0(mech: str, key_n: int, coords: str = "MAX") -> np.ndarray:
    return theta_from_params(load_theta_config()[f"{mech}_{coords}{key_n}"])


def _rotx(th):
    return np.stack([np.cos(th / 2), np.sin(th / 2), np.zeros_like(th), np.zeros_like(th)], axis=-1)


def _body(x, q, v, w):
    return np.concatenate([x, q, v, w], axis=-1)  # (n, 13)


def _vec(a, b, c):
    return np.stack([a, b, c], axis=-1)


def _zeros(n):
    return np.zeros(n)


def _cstates(mech: str, m: dict) -> np.ndarray:
    """Minimal coordinates -> CState matrix (d, n), velocities by the Δtsim forward difference."""
    h = DT_SIM
    if mech == "P1":
        th, om = m["th"], m["om"]
        l = 1.0
        pos = lambda t: _vec(_zeros(t.shape[0]), l / 2 * np.sin(t), -l / 2 * np.cos(t))
        x = pos(th)
        v = (pos(th + h * om) - x) / h
        n = th.shape[0]
        blocks = [_body(x, _rotx(th), v, _vec(om, _zeros(n), _zeros(n)))]
    elif mech == "P2":
        t1, t2, o1, o2 = m["t1"], m["t2"], m["o1"], m["o2"]
        l1 = l2 = 1.0
        n = t1.shape[0]
        p1 = lambda a: _vec(_zeros(n), l1 / 2 * np.sin(a), -l1 / 2 * np.cos(a))
        p2 = lambda a, b: _vec(_zeros(n), l1 * np.sin(a) + l2 / 2 * np.sin(a + b), -l1 * np.cos(a) - l2 / 2 * np.cos(a + b))
        x1, x2 = p1(t1), p2(t1, t2)
        v1 = (p1(t1 + h * o1) - x1) / h
        v2 = (p2(t1 + h * o1, t2 + h * o2) - x2) / h
        blocks = [
            _body(x1, _rotx(t1), v1, _vec(o1, _zeros(n), _zeros(n))),
            _body(x2, _rotx(t1 + t2), v2, _vec(o1 + o2, _zeros(n), _zeros(n))),
        ]
    elif mech == "CP":
        xc, vc, th, om = m["x"], m["v"], m["th"], m["om"]
        l = 0.5
        n = th.shape[0]
        x1 = _vec(_zeros(n), xc, _zeros(n))
        v1 = _vec(_zeros(n), vc, _zeros(n))
        q1 = np.tile(np.array([1.0, 0.0, 0.0, 0.0]), (n, 1))
        pole = lambda t: _vec(_zeros(n), l / 2 * np.sin(t), -l / 2 * np.cos(t))
        x2 = x1 + pole(th)
        v2 = (x1 + v1 * h + pole(th + h * om) - x2) / h
        blocks = [
            _body(x1, q1, v1, np.zeros((n, 3))),
            _body(x2, _rotx(th), v2, _vec(om, _zeros(n), _zeros(n))),
        ]
    elif mech == "FB":
        t1, t2, o1, o2 = m["t1"], m["t2"], m["o1"], m["o2"]
        l = 1.0
        n = t1.shape[0]
        z = _zeros(n)
        P = [
            lambda a, b: _vec(z, 0.5 * np.sin(a) * l, -0.5 * np.cos(a) * l),
            lambda a, b: _vec(z, np.sin(a) * l + 0.5 * np.sin(b) * l, -np.cos(a) * l - 0.5 * np.cos(b) * l),
            lambda a, b: _vec(z, 0.5 * np.sin(b) * l, -0.5 * np.cos(b) * l),
            lambda a, b: _vec(z, np.sin(b) * l + 0.5 * np.sin(a) * l, -np.cos(b) * l - 0.5 * np.cos(a) * l),
        ]
        qs = [_rotx(t1), _rotx(t2), _rotx(t2), _rotx(t1)]
        ws = [_vec(o1, z, z), _vec(o2, z, z), _vec(o2, z, z), _vec(o1, z, z)]
        blocks = []
        for k in range(4):
            xk = P[k](t1, t2)
            vk = (P[k](t1 + h * o1, t2 + h * o2) - xk) / h
            blocks.append(_body(xk, qs[k], vk, ws[k]))
    else:
        raise ValueError(f"unknown mechanism {mech}")
    return np.concatenate(blocks, axis=-1).T.copy()  # (13*nb, n)


def _sample_minimal(mech: str, n: int, rng) -> dict:
    U = rng.uniform
    if mech == "P1":
        return dict(th=U(-math.pi, math.pi, n), om=U(-2, 2, n))
    if mech in ("P2", "FB"):
        return dict(t1=U(-math.pi, math.pi, n), t2=U(-math.pi, math.pi, n), o1=U(-2, 2, n), o2=U(-2, 2, n))
    if mech == "CP":
        return dict(x=U(-0.5, 0.5, n), v=U(-1, 1, n), th=U(-math.pi, math.pi, n), om=U(-2, 2, n))
    raise ValueError(mech)


def _step(mech: str, m: dict) -> dict:
    """One Δt step of the minimal coordinates (P1: rod pendulum θ̈ = -1.5 g/l sinθ; others:
    constant rates -- synthetic targets for the GP hot path, not a physics reference)."""
    m = {k: v.copy() for k, v in m.items()}
    if mech == "P1":
        m["om"] = m["om"] - DT * 1.5 * G * np.sin(m["th"])
        m["th"] = m["th"] + DT * m["om"]
    elif mech in ("P2", "FB"):
        m["t1"] = m["t1"] + DT * m["o1"]
        m["t2"] = m["t2"] + DT * m["o2"]
    elif mech == "CP":
        m["x"] = m["x"] + DT * m["v"]
        m["th"] = m["th"] + DT * m["om"]
    return m


def _noisy(mech: str, m: dict, rng) -> dict:
    m = {k: v + SIGMA * rng.standard_normal(v.shape[0]) for k, v in m.items()}
    return m


def make_trial(mech: str, N: int, M: int = 100, seed: int = 0, noise: bool = True) -> dict:
    """One trial's training/test data.  Returns X (d,N), Xcurr (d,N), Y (G,N), Xs (d,M),
    idx (1-based output coordinates), d.  noise=False: the simulated states as the datasets hold
    them (hyperparameter.jl applies no noise; noise.jl does, applynoise! at e.g. CPnoise.jl:23)."""
    rng = np.random.default_rng(seed)
    nz = (lambda m, r: _noisy(mech, m, r)) if noise else (lambda m, r: m)
    m_old = _sample_minimal(mech, N, rng)
    m_cur = _step(mech, m_old)
    X = _cstates(mech, nz(m_old, rng))
    Xcurr = _cstates(mech, nz(m_cur, rng))
    rng_t = np.random.default_rng(seed + 500000)
    Xs = _cstates(mech, nz(_sample_minimal(mech, M, rng_t), rng_t)) if M > 0 else None
    idx = VW_INDICES[mech]
    Y = np.stack([Xcurr[i - 1, :] for i in idx], axis=0)
    return dict(X=X, Xcurr=Xcurr, Y=Y, Xs=Xs, idx=idx, d=X.shape[0])


def trial_seed(mech: str, trial: int) -> int:
    return 1000 * CONFIG_ID[mech] + trial


# ---- minimal-coordinate experiments (examples/minimal_coordinates/*.jl) ---------------------
# coordinate order of max2mincoordinates (examples/utils/data/transformations.jl:7-34):
# per joint (q, qdot); FB uses bodies 1 and 3 (transformations.jl:25-34)
MIN_COORDS = {"P1": (("th", "om"),), "P2": (("t1", "o1"), ("t2", "o2")), "CP": (("x", "v"), ("th", "om")),
              "FB": (("t1", "o1"), ("t2", "o2"))}
MIN_ANGLE = {"P1": (True,), "P2": (True, True), "CP": (False, True), "FB": (True, True)}


def min_features(mech: str, q: np.ndarray, usesin: bool) -> np.ndarray:
    """(n, 2nc) minimal states -> (d, n) GP inputs: per coordinate (q, qdot), or (sin q, cos q,
    qdot) for angles when usesin (e.g. P2noise.jl(min):24-28, CPnoise.jl(min):25)."""
    q = np.asarray(q, dtype=np.float64)
    rows = []
    for c, ang in enumerate(MIN_ANGLE[mech]):
        if usesin and ang:
            rows += [np.sin(q[:, 2 * c]), np.cos(q[:, 2 * c]), q[:, 2 * c + 1]]
        else:
            rows += [q[:, 2 * c], q[:, 2 * c + 1]]
    return np.stack(rows, axis=0)


def make_trial_min(mech: str, N: int, M: int = 100, seed: int = 0, usesin: bool = False, noise: bool = True) -> dict:
    """One minimal-coordinate trial: X (d, N) inputs at the noisy old states, Y (nc, N) the noisy
    next-step rates (ytrain = [[s[id] for s in xtrain_curr] for id in [2,4]], P2noise.jl(min):30),
    start (M, 2nc) the noisy test states (xtest_old, :33).  noise=False as for make_trial."""
    rng = np.random.default_rng(seed)
    nz = (lambda m, r: _noisy(mech, m, r)) if noise else (lambda m, r: m)
    m_old = _sample_minimal(mech, N, rng)
    m_cur = _step(mech, m_old)
    old, cur = nz(m_old, rng), nz(m_cur, rng)
    keys = MIN_COORDS[mech]
    q_old = np.stack([old[k] for pair in keys for k in pair], axis=1)
    Y = np.stack([cur[rate] for _, rate in keys], axis=0)
    rng_t = np.random.default_rng(seed + 500000)
    tst = nz(_sample_minimal(mech, M, rng_t), rng_t)
    start = np.stack([tst[k] for pair in keys for k in pair], axis=1)
    X = min_features(mech, q_old, usesin)
    return dict(X=X, Y=Y, start=start, d=X.shape[0])


def theta0_min(mech: str, key_n: int, usesin: bool = False) -> np.ndarray:
    """θ from config '<ID>_MIN<N>' = [σ_f, ℓ per minimal coordinate]; with usesin the angle's ℓ is
    shared by its sin and cos features (P2noise.jl(min):36)."""
    p = np.asarray(load_theta_config()[f"{mech}_MIN{key_n}"], dtype=np.float64)
    ell = []
    for c, ang in enumerate(MIN_ANGLE[mech]):
        lq, lv = p[1 + 2 * c], p[2 + 2 * c]
        ell += [lq, lq, lv] if (usesin and ang) else [lq, lv]
    return theta_from_params(np.concatenate([[p[0]], ell]))


# ---- ground truth of the sweep's test rollouts ----------------------------------------------
def test_truth(mech: str, M: int, seed: int, steps: int) -> dict:
    """The noise-free test states of make_trial / make_trial_min (the same draws from the test
    generator, before the noise the experiments add to testdf: CPnoise.jl:21-24) advanced by the
    generator's own dynamics over steps + 1 mechanism steps -- the rollout's final time: the
    minimal-coordinate loop first moves q by qdot*dt, then takes `steps` predicted steps
    (predictdynamics.jl:41-46); the maximal-coordinate loop takes `steps` predicted steps and one
    closing updatestate! (:11-21).  Plays the role of testdf.sfuture (xtest_future_true, :17).
    Returns q (M, 2nc) minimal coordinates and X (d, M) CStates of the final states."""
    rng_t = np.random.default_rng(seed + 500000)
    m = _sample_minimal(mech, M, rng_t)
    for _ in range(steps + 1):
        m = _step(mech, m)
    keys = MIN_COORDS[mech]
    q = np.stack([m[k] for pair in keys for k in pair], axis=1)
    return dict(q=q, X=_cstates(mech, m))


def position_mse(truth: np.ndarray, pred: np.ndarray) -> float:
    """simulationerror(groundtruth, predictions) (examples/utils/utils.jl:36-46): squared position
    error over every body of every test sample / (3 Nbodies M); NaN -> Inf.  truth, pred: (M, d)
    CStates."""
    truth = np.asarray(truth, dtype=np.float64)
    pred = np.asarray(pred, dtype=np.float64)
    M, d = truth.shape
    nb = d // 13
    err = 0.0
    for i in range(M):
        for b in range(nb):
            o = 13 * b
            err += float(np.sum((truth[i, o:o + 3] - pred[i, o:o + 3]) ** 2))
    err /= 3 * nb * M
    return math.inf if math.isnan(err) else err
