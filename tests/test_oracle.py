"""The oracle restatement (oracle/gp_oracle.py) against the committed golden fixtures, against
scikit-learn (independent implementation), central finite differences, and the reference's
failure semantics.  CPU only."""
import math

import numpy as np
import pytest

from oracle import gp_oracle as O

CASES = ["p1_n50", "cp_n64", "p2_n100", "p2_n256", "fb_n64"]


@pytest.mark.parametrize("name", CASES)
@pytest.mark.parametrize("tag,mode", [("exp", O.DIST_EXPANDED), ("dir", O.DIST_DIRECT)])
def test_oracle_reproduces_golden(golden_dir, name, tag, mode):
    z = np.load(golden_dir / f"{name}.npz")
    for g in range(z["Y"].shape[0]):
        f = O.fit(z["X"], z["Y"][g], z["theta"], z["Xs"], mode)
        assert f["mll"] == pytest.approx(z[f"mll_{tag}"][g], rel=1e-12, abs=1e-12)
        np.testing.assert_allclose(f["grad"], z[f"grad_{tag}"][g], rtol=1e-10, atol=1e-10 * np.max(np.abs(f["grad"])))
        np.testing.assert_allclose(f["mu"], z[f"mu_{tag}"][g], rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(f["var"], z[f"var_{tag}"][g], rtol=1e-9, atol=1e-14)


@pytest.mark.parametrize("name", ["p1_n50", "p2_n100"])
def test_oracle_matches_sklearn(golden_dir, name):
    sk = pytest.importorskip("sklearn")
    from sklearn.gaussian_process import GaussianProcessRegressor
    from sklearn.gaussian_process.kernels import RBF, ConstantKernel, WhiteKernel

    z = np.load(golden_dir / f"{name}.npz")
    X, y, th = z["X"], z["Y"][0], z["theta"]
    d = X.shape[0]
    il2, sf2, sn2, noise = O.kernel_params(th, d)
    k = ConstantKernel(sf2) * RBF(np.exp(th[1 : d + 1])) + WhiteKernel(noise)
    gpr = GaussianProcessRegressor(kernel=k, alpha=0.0, optimizer=None).fit(X.T, y)
    lml, g = gpr.log_marginal_likelihood(gpr.kernel_.theta, eval_gradient=True)
    m, grad, _ = O.lml(X, y, th, O.DIST_DIRECT, want_grad=True)
    assert m == pytest.approx(lml, rel=1e-9)
    assert grad[d + 1] == pytest.approx(2 * g[0], rel=1e-7, abs=1e-9)
    np.testing.assert_allclose(grad[1 : d + 1], g[1 : d + 1], rtol=1e-7, atol=1e-9 * np.max(np.abs(grad)))
    mu_sk, sd_sk = gpr.predict(z["Xs"].T, return_std=True)
    _, _, aux = O.lml(X, y, th, O.DIST_DIRECT)
    mu, var = O.predict_f(X, th, aux["alpha"], aux["U"], z["Xs"], O.DIST_DIRECT)
    np.testing.assert_allclose(mu, mu_sk, rtol=1e-9, atol=1e-10)
    # sklearn's predictive std includes the WhiteKernel noise
    np.testing.assert_allclose(var + noise, sd_sk**2, rtol=1e-7, atol=1e-12)


@pytest.mark.parametrize("name", ["p1_n50", "cp_n64"])
def test_oracle_gradient_finite_differences(golden_dir, name):
    z = np.load(golden_dir / f"{name}.npz")
    X, y, th = z["X"], z["Y"][1], z["theta"].copy()
    _, g, _ = O.lml(X, y, th, O.DIST_DIRECT, want_grad=True)
    h = 1e-5
    for q in range(th.shape[0]):
        tp, tm = th.copy(), th.copy()
        tp[q] += h
        tm[q] -= h
        fd = (O.lml(X, y, tp, O.DIST_DIRECT)[0] - O.lml(X, y, tm, O.DIST_DIRECT)[0]) / (2 * h)
        assert g[q] == pytest.approx(fd, rel=2e-5, abs=2e-6 * max(1.0, np.max(np.abs(g))))


def test_distance_modes_spread_is_small(golden_dir):
    """Calibration of the distance-formulation tolerance (DESIGN.md 'distance modes')."""
    for name in CASES:
        z = np.load(golden_dir / f"{name}.npz")
        rel = np.max(np.abs(z["mll_exp"] - z["mll_dir"]) / np.maximum(1.0, np.abs(z["mll_dir"])))
        assert rel < 1e-8, (name, rel)
        mu_rel = np.max(np.abs(z["mu_exp"] - z["mu_dir"])) / np.max(np.abs(z["Y"]))
        assert mu_rel < 1e-8, (name, mu_rel)


def test_gram_layout_and_noise(golden_dir):
    z = np.load(golden_dir / "p1_n50.npz")
    K, Kf, _ = O.gram(z["X"], z["theta"], O.DIST_EXPANDED)
    np.testing.assert_array_equal(K, z["K_exp"])
    il2, sf2, sn2, noise = O.kernel_params(z["theta"], z["X"].shape[0])
    assert noise == sn2 + np.finfo(float).eps
    np.testing.assert_array_equal(np.diag(K), np.diag(Kf) + noise)
    np.testing.assert_array_equal(np.diag(Kf), np.full(K.shape[0], sf2))  # exact zero self-distance
    np.testing.assert_array_equal(K, K.T)


def test_not_positive_definite_reports_pivot(golden_dir):
    z = np.load(golden_dir / "nonpd_p1.npz")
    with pytest.raises(O.NotPosDef) as e:
        O.lml(z["X"], z["Y"][0], z["theta"])
    assert e.value.info == int(z["info"])


def test_theta_convention():
    th = np.array([-2.0, math.log(0.5), math.log(2.0), math.log(3.0)])
    il2, sf2, sn2, noise = O.kernel_params(th, 2)
    assert il2[0] == math.exp(-2 * math.log(0.5))
    assert sf2 == math.exp(2 * math.log(3.0))
    assert sn2 == math.exp(-4.0)
