"""Generates the committed golden fixtures (tests/golden/*.npz) from the oracle restatement
(oracle/gp_oracle.py) and cross-checks every case against scikit-learn 1.7.2's
GaussianProcessRegressor (an independent implementation) before writing.

The reference (Julia / GaussianProcesses.jl 0.12.4) cannot run in this container and ships no
tests or golden vectors, so these fixtures pin the restatement, not the
reference's own rounding.  Inputs: synthetic CStates from the reference kinematics
(gprx/data.py) and the reference's tuned hyper-parameters (examples/config/config.json).

Run:  python tests/golden/make_golden.py
"""
import pathlib
import sys

import numpy as np

HERE = pathlib.Path(__file__).resolve().parent
REPO = HERE.parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "gpr.jl_amd"))

from oracle import gp_oracle as O  # noqa: E402
from gprx import data  # noqa: E402

CASES = [  # name, mechanism, N, config key N, M, seed
    ("p1_n50", "P1", 50, 64, 8, 11),
    ("cp_n64", "CP", 64, 512, 8, 12),
    ("p2_n100", "P2", 100, 2048, 8, 13),
    ("p2_n256", "P2", 256, 256, 8, 14),
    ("fb_n64", "FB", 64, 512, 8, 15),
]


def sklearn_lml(X, y, theta):
    """LML and gradient mapped to [logσn, logℓ, logσf] via sklearn's log-parameterisation."""
    from sklearn.gaussian_process import GaussianProcessRegressor
    from sklearn.gaussian_process.kernels import RBF, ConstantKernel, WhiteKernel

    d = X.shape[0]
    il2, sf2, sn2, noise = O.kernel_params(theta, d)
    k = ConstantKernel(sf2) * RBF(np.exp(theta[1 : d + 1])) + WhiteKernel(noise)
    gpr = GaussianProcessRegressor(kernel=k, alpha=0.0, optimizer=None, normalize_y=False).fit(X.T, y)
    lml, g = gpr.log_marginal_likelihood(gpr.kernel_.theta, eval_gradient=True)
    # sklearn theta = [log σf², log ℓ_1..d, log(noise)]
    grad = np.empty(d + 2)
    grad[d + 1] = 2.0 * g[0]
    grad[1 : d + 1] = g[1 : d + 1]
    grad[0] = 2.0 * g[d + 1] * sn2 / noise  # d/dlogσn of (σn² + eps) = 2σn²
    return lml, grad


def main():
    for name, mech, N, key, M, seed in CASES:
        tr = data.make_trial(mech, N, M, seed=seed)
        X, Y, Xs = tr["X"], tr["Y"], tr["Xs"]
        theta = data.theta0(mech, key)
        out = dict(X=X, Y=Y, Xs=Xs, theta=theta, idx=np.array(tr["idx"]), Xcurr=tr["Xcurr"])
        for mode, tag in ((O.DIST_EXPANDED, "exp"), (O.DIST_DIRECT, "dir")):
            mlls, grads, mus, vars_, alphas = [], [], [], [], []
            for g in range(Y.shape[0]):
                f = O.fit(X, Y[g], theta, Xs, mode)
                mlls.append(f["mll"]), grads.append(f["grad"]), mus.append(f["mu"]), vars_.append(f["var"])
                alphas.append(f["alpha"])
                if mode == O.DIST_DIRECT and g == 0:
                    sl, sg = sklearn_lml(X, Y[g], theta)
                    rel = abs(sl - f["mll"]) / max(1.0, abs(f["mll"]))
                    grel = np.max(np.abs(sg - f["grad"])) / max(1.0, np.max(np.abs(f["grad"])))
                    print(f"{name}: sklearn |Δmll|/|mll|={rel:.2e}  |Δgrad|/|grad|={grel:.2e}")
                    assert rel < 1e-8 and grel < 1e-6, (name, rel, grel)
            out[f"mll_{tag}"] = np.array(mlls)
            out[f"grad_{tag}"] = np.array(grads)
            out[f"mu_{tag}"] = np.array(mus)
            out[f"var_{tag}"] = np.array(vars_)
            out[f"alpha_{tag}"] = np.array(alphas)
        if N <= 100:
            K, _, _ = O.gram(X, theta, O.DIST_EXPANDED)
            out["K_exp"] = K
        np.savez_compressed(HERE / f"{name}.npz", **out)
        print("wrote", name)
    # forced non-positive-definite case: duplicated columns, σn -> e^-20
    tr = data.make_trial("P1", 40, 0, seed=21)
    X = tr["X"].copy()
    X[:, 20:] = X[:, :20]
    theta = data.theta0("P1", 64)
    theta[0] = -20.0
    theta[-1] = np.log(400.0)
    try:
        O.lml(X, tr["Y"][0], theta)
        info = 0
    except O.NotPosDef as e:
        info = e.info
    print("nonpd info", info)
    assert info > 0
    np.savez_compressed(HERE / "nonpd_p1.npz", X=X, Y=tr["Y"], theta=theta, info=np.array(info))
    # CState known-answer vector: P1 at θ=0.3, ω=0.7 without noise (hand-derived layout)
    th, om, h = 0.3, 0.7, data.DT_SIM
    x = np.array([0.0, 0.5 * np.sin(th), -0.5 * np.cos(th)])
    xn = np.array([0.0, 0.5 * np.sin(th + h * om), -0.5 * np.cos(th + h * om)])
    cs = np.concatenate([x, [np.cos(th / 2), np.sin(th / 2), 0.0, 0.0], (xn - x) / h, [om, 0.0, 0.0]])
    np.savez_compressed(HERE / "cstate_kat.npz", theta=th, omega=om, cstate=cs)


if __name__ == "__main__":
    main()
