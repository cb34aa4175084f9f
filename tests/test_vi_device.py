"""The device variational-integrator step (k_vi_step via gprx_vi_step / gprx.projection.vi_step),
which the MeanDynamics sweep variants and the physics-only baseline run on: against the host
restatement gprx/vi.py on every experiment mechanism, against the independent action-based oracle
(oracle/vi_oracle.py), failure isolation as the host's, and the baseline simulation.  Parity with
ConstrainedDynamics itself is unpinned (absent from the reference tree; tests/test_vi.py pins the
physics).  Tolerances: converged states are solved to |f| < 1e-10 and |ds| < 1e-10, so two solvers
of the same equations agree to that order; states that do not converge in 100 iterations (the
four-bar's redundant loop constraints) only have the same status."""
import numpy as np
import pytest

from gprx import data, mdynamics, projection, vi
from oracle import vi_oracle as VO

pytestmark = pytest.mark.gpu
MECHS = ("P1", "P2", "CP", "FB")


@pytest.fixture(scope="module")
def ctx():
    import gprx

    c = gprx.Context(0)
    yield c
    c.close()


@pytest.mark.parametrize("mech", MECHS)
def test_device_step_matches_the_host_restatement(ctx, mech):
    tr = data.make_trial(mech, 200, 56, seed=17)
    S = np.concatenate([tr["X"].T, tr["Xs"].T])  # training states and noisy test starts
    h, hi, hs = vi.vi_step(mech, S)
    g, gi, gs = projection.vi_step(mech, S, ctx=ctx)
    np.testing.assert_array_equal(gs, hs)
    conv = hs == 0
    assert conv.mean() > 0.9
    np.testing.assert_allclose(g[conv], h[conv], rtol=0, atol=1e-9)
    # the same Newton path up to rounding; the four-bar's rank-deficient loop constraints make a few
    # paths diverge (the regularised iteration creeps): they still converge to the same solution
    assert np.mean(np.abs(gi[conv] - hi[conv]) <= 1) > (0.9 if mech == "FB" else 0.999)
    nb = projection.NBODIES[mech]
    pose = np.concatenate([np.r_[13 * b:13 * b + 7] for b in range(nb)])
    np.testing.assert_array_equal(g[:, pose], h[:, pose])  # the discrete pose x2, q2 (no solve)
    assert np.all(np.isfinite(g[hs != 2]))


@pytest.mark.parametrize("mech", MECHS)
def test_device_step_matches_the_action_based_oracle(ctx, mech):
    tr = data.make_trial(mech, 3, 0, seed=41)
    X = tr["X"]
    g, _, st = projection.vi_step(mech, X.T, ctx=ctx)
    for j in range(X.shape[1] if mech != "FB" else 1):
        o, ok = VO.vi_step(mech, X[:, j])
        assert ok and st[j] == 0
        np.testing.assert_allclose(g[j], o, rtol=0, atol=1e-9)


def test_failed_state_is_isolated_on_the_device(ctx):
    """|w| beyond 2/dt (ConstrainedDynamics' sqrt throws a DomainError): status 2 and a NaN row for
    that state alone; the others are bit-identical to a batch without it, as on the host."""
    tr = data.make_trial("P2", 2, 3, seed=2)
    S = tr["Xs"].T.copy()
    good, _, st_good = projection.vi_step("P2", S, ctx=ctx)
    bad = S.copy()
    bad[1, 10:13] = 1e3 / vi.DT
    out, _, st = projection.vi_step("P2", bad, ctx=ctx)
    assert st[1] == 2 and np.isnan(out[1]).all()
    np.testing.assert_array_equal(out[[0, 2]], good[[0, 2]])
    np.testing.assert_array_equal(st[[0, 2]], st_good[[0, 2]])
    h, _, hs = vi.vi_step("P2", bad)
    np.testing.assert_array_equal(st, hs)


@pytest.mark.parametrize("mech", ("P1", "FB"))
def test_device_baseline_simulation(ctx, mech):
    """predictdynamics of the physics-only baseline (steps + 1 physics steps, predictdynamics.jl:24-28)
    on the device against the host simulation."""
    tr = data.make_trial(mech, 2, 8, seed=5)
    S = tr["Xs"].T
    fin, bad = mdynamics.simulate(mech, S, 4, ctx=ctx)
    ref, rbad = vi.simulate(mech, S, 4)
    np.testing.assert_array_equal(bad, rbad)
    ok = rbad == 0
    np.testing.assert_allclose(fin[ok], ref[ok], rtol=0, atol=1e-8)
