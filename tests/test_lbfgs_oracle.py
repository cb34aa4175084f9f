"""The independent optimiser restatement (oracle/lbfgs_oracle.py: Optim 1.4.1 LBFGS +
LineSearches 7.1.1 BackTracking(order=2), written in the packages' own structure) pinned by
hand-derived known answers, and the product's host restatement (gprx/optim.py) checked against it
on the GP targets of the experiments.  Parity with Optim itself is unpinned (not runnable here).
The device optimiser (k_lbfgs) is checked against this oracle in tests/test_gpu.py."""
import math

import numpy as np
import pytest

from oracle import gp_oracle as O
from oracle import lbfgs_oracle as LO


def _phi_recorder(fn):
    calls = []

    def phi(a):
        calls.append(a)
        return fn(a)

    return phi, calls


def test_backtracking_quadratic_interpolation_kat():
    # phi(a) = 1 - a + a^2: phi(0) = 1, phi'(0) = -1, phi(1) = 1 fails Armijo (1 > 1 - 1e-4);
    # the quadratic through phi(0), phi'(0), phi(1) has its minimum at -(-1 * 1)/(2 (1 - 1 + 1)) = 1/2
    phi, calls = _phi_recorder(lambda a: 1 - a + a * a)
    a, v = LO.backtracking(phi, 1.0, 1.0, -1.0)
    assert (a, v, calls) == (0.5, 0.75, [1.0, 0.5])
    # phi(a) = 1 - a + 10 a^2: the quadratic step 1/20 is clamped to rho_lo = 0.1 (phi = 1.0 still
    # fails), then -(-1 * 0.01)/(2 (1 - 1 + 0.1)) = 0.05 = rho_hi * 0.1: accepted, phi = 0.975
    phi, calls = _phi_recorder(lambda a: 1 - a + 10 * a * a)
    a, v = LO.backtracking(phi, 1.0, 1.0, -1.0)
    assert calls == [1.0, 0.1, 0.05] and a == 0.05 and v == pytest.approx(0.975, abs=1e-15)


def test_backtracking_halves_through_infinite_values():
    phi, calls = _phi_recorder(lambda a: math.inf if a > 0.2 else (a - 0.1) ** 2)
    a, v = LO.backtracking(phi, 1.0, 0.01, -0.2)
    assert calls[:4] == [1.0, 0.5, 0.25, 0.125] and a <= 0.2 and math.isfinite(v)
    phi, calls = _phi_recorder(lambda a: math.inf)  # never finite: 1 + iterfinitemax (52) trials
    LO.backtracking(phi, 1.0, math.inf, math.nan)
    assert len(calls) == 53


def test_twoloop_scaleinvH0_kat():
    # one history pair dx = (1, 0), dg = (2, 0) (rho = 1/2), gradient (1, 1), pseudo-iteration 2:
    #   alpha = rho dx.g = 0.5 ; q = g - alpha dg = (0, 1)
    #   scaleinvH0: gamma = dx.dg / dg.dg = 0.5 -> q = (0, 0.5) ; beta = rho dg.q = 0
    #   s = -(q + dx (alpha - beta)) = (-0.5, -0.5)      (without scaling: (-0.5, -1))
    m = 10
    dxh = [np.zeros(2) for _ in range(m)]
    dgh = [np.zeros(2) for _ in range(m)]
    rho = np.zeros(m)
    dxh[0], dgh[0], rho[0] = np.array([1.0, 0.0]), np.array([2.0, 0.0]), 0.5
    s = np.zeros(2)
    LO.twoloop(s, np.array([1.0, 1.0]), rho, dxh, dgh, m, 2, np.zeros(m), True)
    assert np.array_equal(s, [-0.5, -0.5])
    LO.twoloop(s, np.array([1.0, 1.0]), rho, dxh, dgh, m, 2, np.zeros(m), False)
    assert np.array_equal(s, [-0.5, -1.0])
    # pseudo-iteration 1 (first iteration or after a reset): steepest descent, no scaling
    LO.twoloop(s, np.array([1.0, 1.0]), rho, dxh, dgh, m, 1, np.zeros(m), True)
    assert np.array_equal(s, [-1.0, -1.0])


def test_converges_on_a_quadratic():
    A = np.diag([1.0, 10.0, 100.0])
    r = LO.optimize(lambda x: (0.5 * x @ A @ x, A @ x), np.array([1.0, 1.0, 1.0]))
    assert r["converged"] and r["stopped_by"] == "g_tol" and np.max(np.abs(r["minimizer"])) < 1e-8
    assert r["f_calls"] >= r["g_calls"] >= 2  # value_gradient!! counts one of each


def _gp_fg(X, y):
    def fg(h):
        try:
            m, g, _ = O.lml(X, y, h, want_grad=True)
            return -m, -g
        except O.NotPosDef:
            return math.inf, np.full(h.shape[0], np.nan)

    return fg


@pytest.mark.parametrize("name,limit", [("p1_n50", 40), ("cp_n64", 25), ("p2_n100", 30)])
def test_host_restatement_equals_the_oracle(golden_dir, name, limit):
    from gprx.optim import LBFGS, Options, lbfgs_minimize

    z = np.load(golden_dir / f"{name}.npz")
    X, Y, th = z["X"], z["Y"], z["theta"]
    rng = np.random.default_rng(9)
    for g in range(min(2, Y.shape[0])):
        th0 = th + 0.05 * rng.standard_normal(th.shape[0])
        fg = _gp_fg(X, Y[g])
        ref = LO.optimize(fg, th0, f_calls_limit=limit)
        got = lbfgs_minimize(lambda h: fg(h)[0], fg, th0, LBFGS(), Options(max_evals=limit))
        np.testing.assert_array_equal(got.minimizer, ref["minimizer"])
        assert got.minimum == ref["minimum"]
        assert (got.iterations, got.f_calls, got.g_calls, got.stopped_by, got.converged) == (
            ref["iterations"], ref["f_calls"], ref["g_calls"], ref["stopped_by"], ref["converged"])


def test_failed_start_matches_the_oracle(golden_dir):
    from gprx.optim import LBFGS, Options, lbfgs_minimize

    z = np.load(golden_dir / "nonpd_p1.npz")
    fg = _gp_fg(z["X"], z["Y"][0])
    ref = LO.optimize(fg, z["theta"], f_calls_limit=80)
    got = lbfgs_minimize(lambda h: fg(h)[0], fg, z["theta"], LBFGS(), Options(max_evals=80))
    assert ref["stopped_by"] == got.stopped_by == "nan_gradient"
    assert (got.iterations, got.f_calls, got.g_calls) == (ref["iterations"], ref["f_calls"], ref["g_calls"])
