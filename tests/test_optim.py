"""Host optimiser (Optim LBFGS + LineSearches BackTracking(order=2) restatement) -- CPU only,
driven by analytic functions and by the oracle GP target."""
import math

import numpy as np
import pytest

from gprx.optim import BackTracking, LBFGS, Options, lbfgs_minimize
from oracle import gp_oracle as O


def rosen(x):
    return float(100 * (x[1] - x[0] ** 2) ** 2 + (1 - x[0]) ** 2)


def rosen_fg(x):
    g = np.array([-400 * x[0] * (x[1] - x[0] ** 2) - 2 * (1 - x[0]), 200 * (x[1] - x[0] ** 2)])
    return rosen(x), g


def test_lbfgs_rosenbrock():
    r = lbfgs_minimize(rosen, rosen_fg, np.array([-1.2, 1.0]))
    assert r.converged and r.stopped_by == "g_tol"
    np.testing.assert_allclose(r.minimizer, [1.0, 1.0], atol=1e-6)


def test_lbfgs_quadratic_exact():
    A = np.diag([1.0, 10.0, 100.0])
    f = lambda x: 0.5 * float(x @ A @ x)
    r = lbfgs_minimize(f, lambda x: (f(x), A @ x), np.ones(3), options=Options(g_abstol=1e-10))
    assert r.converged and np.max(np.abs(r.minimizer)) < 1e-9


def test_backtracking_quadratic_interpolation_step():
    # phi(a) = (a - 0.3)^2 from phi(0) = 0.09, phi'(0) = -0.6: one quadratic step hits 0.3 exactly
    phi = lambda a: (a - 0.3) ** 2
    a, v = BackTracking()(phi, 1.0, 0.09, -0.6)
    assert a == pytest.approx(0.3) and v == pytest.approx(0.0, abs=1e-15)


def test_backtracking_anchors_every_step_at_phi0():
    # LineSearches 7.1.1: the sufficient-decrease test and the quadratic model use phi(0), not the
    # previous trial value.  phi(1) = 10 -> a = 0.1 (clamped); phi(0.1) = 0.15 -> the quadratic
    # through (0, 0), slope -1, (0.1, 0.15) has its minimum at 0.02 (anchoring at phi(1) would give
    # a negative step, clamped to 0.01)
    vals = {1.0: 10.0, 0.1: 0.15}
    seen = []

    def phi(a):
        seen.append(a)
        return vals.get(a, -0.1)

    a, v = BackTracking()(phi, 1.0, 0.0, -1.0)
    assert seen[:2] == [1.0, 0.1] and a == pytest.approx(0.02, rel=1e-12) and v == -0.1


def test_backtracking_recovers_from_infinite_values():
    phi = lambda a: math.inf if a > 0.2 else (a - 0.1) ** 2
    a, v = BackTracking()(phi, 1.0, 0.01, -0.2)
    assert a <= 0.2 and math.isfinite(v) and v < 0.01


def test_max_evals_budget_is_deterministic():
    r1 = lbfgs_minimize(rosen, rosen_fg, np.array([-1.2, 1.0]), options=Options(max_evals=15))
    r2 = lbfgs_minimize(rosen, rosen_fg, np.array([-1.2, 1.0]), options=Options(max_evals=15))
    # Optim's f_calls_limit: soft, checked after each iteration (the last line search may pass it)
    assert r1.stopped_by == "max_evals" and 15 <= r1.f_calls <= 15 + 10
    np.testing.assert_array_equal(r1.minimizer, r2.minimizer)


def test_max_evals_zero_is_no_limit():
    """Optim: f_limit_reached = f_calls_limit > 0 && ... -- a budget of 0 (Optim's default) or
    less is no limit, not a stop after the first iteration."""
    free = lbfgs_minimize(rosen, rosen_fg, np.array([-1.2, 1.0]))
    for lim in (0, -1):
        r = lbfgs_minimize(rosen, rosen_fg, np.array([-1.2, 1.0]), options=Options(max_evals=lim))
        assert r.stopped_by == free.stopped_by == "g_tol" and r.f_calls == free.f_calls
        np.testing.assert_array_equal(r.minimizer, free.minimizer)


def test_lbfgs_improves_gp_target(golden_dir):
    z = np.load(golden_dir / "p1_n50.npz")
    X, y, th0 = z["X"], z["Y"][0], z["theta"]

    def f(h):
        try:
            return -O.lml(X, y, h)[0]
        except O.NotPosDef:
            return math.inf

    def fg(h):
        try:
            m, g, _ = O.lml(X, y, h, want_grad=True)
            return -m, -g
        except O.NotPosDef:
            return math.inf, np.full(h.shape[0], np.nan)

    r = lbfgs_minimize(f, fg, th0, LBFGS(), Options(max_evals=40))
    assert r.minimum < f(th0)


class _OracleBatch:
    """Stand-in for GPBatch.run backed by the oracle (CPU): same per-slot contract."""

    def __init__(self, X, Ys):
        self.X, self.Ys = X, Ys
        self.calls = 0

    def run(self, theta, grad=True, predict=False):
        self.calls += 1
        B = theta.shape[0]
        mll = np.empty(B)
        g = np.empty_like(theta)
        st = np.zeros(B, dtype=np.int32)
        for s in range(B):
            try:
                m, gg, _ = O.lml(self.X, self.Ys[s], theta[s], want_grad=True)
                mll[s], g[s] = m, gg
            except O.NotPosDef:
                st[s] = 1
        return dict(mll=mll, grad=g, status=st)


def test_optimize_batch_matches_sequential(golden_dir):
    from gprx.optim import optimize_batch

    z = np.load(golden_dir / "p1_n50.npz")
    X, Ys, th0 = z["X"], z["Y"], z["theta"]
    B = Ys.shape[0]
    rng = np.random.default_rng(4)
    thetas = np.stack([th0 + 0.1 * rng.standard_normal(th0.shape[0]) for _ in range(B)])
    opts = Options(max_evals=25)
    fake = _OracleBatch(X, Ys)
    res, rounds = optimize_batch(fake, thetas, LBFGS(), opts)
    for s in range(B):

        def f(h, s=s):
            try:
                return -O.lml(X, Ys[s], h)[0]
            except O.NotPosDef:
                return math.inf

        def fg(h, s=s):
            try:
                m, g, _ = O.lml(X, Ys[s], h, want_grad=True)
                return -m, -g
            except O.NotPosDef:
                return math.inf, np.full(h.shape[0], np.nan)

        ref = lbfgs_minimize(f, fg, thetas[s], LBFGS(), opts)
        np.testing.assert_array_equal(res[s].minimizer, ref.minimizer)
        assert res[s].minimum == ref.minimum and res[s].stopped_by == ref.stopped_by
    # lock-step sharing: far fewer batch calls than the total number of evaluations
    assert rounds == fake.calls and rounds <= max(r.f_calls for r in res)


def test_twoloop_and_linesearch_follow_ieee_division():
    # a flat objective gives dx . dg = 0 and dg . dg = 0: Julia divides to Inf/NaN, never raises
    r = lbfgs_minimize(lambda x: 0.0, lambda x: (0.0, np.zeros_like(x)), np.ones(3))
    assert r.converged
    f = lambda x: float(abs(x[0]))  # kink: identical gradients on one side
    r = lbfgs_minimize(f, lambda x: (f(x), np.array([np.sign(x[0])])), np.array([3.0]), options=Options(max_evals=20))
    assert r.converged or r.f_calls >= 20


def test_f_tol_needs_successive_repeats():
    # f is constant to the last bit while the (fake) gradient is 1e-20: BackTracking accepts the
    # unit step (the Armijo margin c_1 * a * dphi_0 = -1e-44 vanishes next to f = 1), x moves and
    # f repeats exactly.  Optim counts that f convergence only on successive_f_tol + 1 = 2
    # successive iterations (optimize.jl's counter_f_tol).
    fg = lambda x: (1.0, np.array([1e-20]))
    args = (lambda x: 1.0, fg, np.zeros(1), LBFGS(scaleinvH0=False))
    r = lbfgs_minimize(*args, Options(g_abstol=0.0))
    assert r.converged and r.stopped_by == "f_tol" and r.iterations == 2
    r0 = lbfgs_minimize(*args, Options(g_abstol=0.0, successive_f_tol=0))
    assert r0.converged and r0.stopped_by == "f_tol" and r0.iterations == 1


def test_nan_gradient_terminates_early():
    # every evaluation fails (+Inf, gradient NaN as GaussianProcesses leaves it): one iteration of
    # 52 step halvings after the first trial (BackTracking's iterfinite 0 -> 52), the NaN step is
    # accepted against phi(0) = Inf, and Optim's "Terminated early due to NaN in gradient" ends
    # the loop; f calls = 1 (value_gradient!!) + 1 + 52 trials, g calls = 1 + update_g!
    r = lbfgs_minimize(lambda x: math.inf, lambda x: (math.inf, np.full(2, np.nan)), np.zeros(2))
    assert (r.iterations, r.f_calls, r.g_calls, r.stopped_by, r.converged) == (1, 54, 2, "nan_gradient", False)


def test_compare_optimisers_names_the_first_differing_evaluation():
    """gprx.optim.compare_optimisers (the bench's device_vs_host report): NaN minima compare by
    their bits, and with both traces the first evaluation where two runs part is named, whether
    the same theta was answered differently or a different theta was asked."""
    from gprx.optim import Result, compare_optimisers

    n, B, R = 3, 2, 4

    def res(x, f):
        return Result(np.array(x, dtype=float), f, 1, 3, 2, False, "max_evals")

    a = [res([1, 2, 3], 1.5), res([0, 0, 0], math.nan)]
    assert compare_optimisers(a, [res([1, 2, 3], 1.5), res([0, 0, 0], math.nan)])["equal"]
    tr = np.zeros((R, B, 2 * n + 2))
    tr[:, :, 0] = 1.0
    tr[:, :, 1:1 + n] = np.arange(R)[:, None, None] + 0.5
    tr[:, :, 1 + n] = -np.arange(R)[:, None]
    tb = tr.copy()
    tb[2, 1, 1 + n] += 1e-15 * 4  # slot 1's third answer differs in its last bits
    b = [res([1, 2, 3], 1.5), res([0, 0, 1e-16], math.nan)]
    rep = compare_optimisers(a, b, tr, tb)
    assert not rep["equal"] and rep["first_slot"] == 1 and rep["n_differ"] == 1
    assert rep["first_eval_diff"]["kind"] == "same theta answered differently"
    assert rep["first_eval_diff"]["index"] == 2 and rep["first_eval_diff"]["round"] == [2, 2]
    assert rep["nonfinite_minimum"] == [True, True]
    tc = tr.copy()
    tc[1, 1, 0] = 0.0  # slot 1 skips round 1 in run c: its second evaluation is round 2's theta
    rep = compare_optimisers(a, b, tr, tc)
    assert rep["first_eval_diff"]["kind"] == "different theta requested"
    assert rep["first_eval_diff"]["round"] == [1, 2]
