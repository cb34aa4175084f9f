"""The variational-integrator step behind MeanDynamics (gprx/vi.py; src/mDynamics.jl:41-60 ->
ConstrainedDynamics.newton!, absent from the reference tree: parity UNPINNED) against the
independent action-based restatement in oracle/vi_oracle.py, plus what pins both physically: the
constraint residual at the next pose, the pendulum's continuous-time limit
w' = w - dt (3 g / 2 l) sin(theta) + O(dt^2), bounded energy over many steps (a variational
integrator does not drift), and the minimal-coordinate xtransform against the data generator's
kinematics."""
import numpy as np
import pytest

from gprx import data, mdynamics, vi
from oracle import vi_oracle as VO

MECHS = ("P1", "P2", "CP", "FB")


@pytest.mark.parametrize("mech", MECHS)
def test_step_matches_the_action_based_oracle(mech):
    tr = data.make_trial(mech, 3 if mech != "FB" else 1, 0, seed=41)
    X = tr["X"]
    sol, it, st = vi.vi_step(mech, X.T)
    assert np.all(st == 0) and np.all(it <= 10)
    for j in range(X.shape[1]):
        o, r = VO.vi_step(mech, X[:, j])
        assert r.success, r.message
        np.testing.assert_allclose(sol[j], o, rtol=0, atol=1e-9)


@pytest.mark.parametrize("mech", MECHS)
def test_constraints_hold_at_the_next_pose(mech):
    tr = data.make_trial(mech, 64, 0, seed=7)
    sol, _, st = vi.vi_step(mech, tr["X"].T)
    M = vi.MECHANISMS[mech]
    c = sol.reshape(sol.shape[0], M["nb"], 13)
    g = vi.constraints(M, c[..., 0:3] + c[..., 7:10] * vi.DT, vi.step_q(c[..., 3:7], c[..., 10:13]))
    assert np.max(np.abs(g[st == 0])) < 1e-12
    assert np.mean(st) < 0.05  # the four-bar's redundant loop may stall a few Newton solves


def test_pendulum_continuous_time_limit():
    rng = np.random.default_rng(0)
    th, om = rng.uniform(-3, 3, 100), rng.uniform(-2, 2, 100)
    X = data._cstates("P1", dict(th=th, om=om))
    ratios = []
    for dt in (0.01, 0.005, 0.0025):
        s, _, _ = vi.vi_step("P1", X.T, dt=dt)
        ratios.append(np.max(np.abs(s[:, 10] - (om - dt * 1.5 * vi.GRAV * np.sin(th)))) / dt ** 2)
    # the one-step error is O(dt^2) with a stable constant
    assert max(ratios) < 50 and max(ratios) / min(ratios) < 1.1


def _energy(mech, S):
    M = vi.MECHANISMS[mech]
    c = S.reshape(S.shape[0], M["nb"], 13)
    E = np.zeros(S.shape[0])
    for b in range(M["nb"]):
        v, w = c[:, b, 7:10], c[:, b, 10:13]
        E += 0.5 * M["m"][b] * np.sum(v * v, axis=1) + 0.5 * np.einsum("ti,ij,tj->t", w, M["J"][b], w)
        E += M["m"][b] * vi.GRAV * c[:, b, 2]
    return E


@pytest.mark.parametrize("mech", ("P1", "P2"))
def test_energy_stays_bounded(mech):
    """1000 steps of 10 ms: the discrete energy oscillates but does not drift."""
    tr = data.make_trial(mech, 8, 0, seed=3, noise=False)
    S = tr["X"].T
    E0 = _energy(mech, S)
    Es = []
    for _ in range(1000):
        S, _, st = vi.vi_step(mech, S)
        assert np.all(st == 0)
        Es.append(_energy(mech, S))
    Es = np.array(Es)
    scale = 1.0 + np.abs(E0)
    assert np.max(np.abs(Es - E0) / scale) < 0.1  # O(dt) oscillation (large swings)
    drift = np.abs(Es[-200:].mean(axis=0) - Es[:200].mean(axis=0)) / scale
    assert np.max(drift) < 0.03  # window means of a chaotic double pendulum move by ~1%


@pytest.mark.parametrize("mech", MECHS)
@pytest.mark.parametrize("usesin", (False, True))
def test_xtransform_matches_the_generator_kinematics(mech, usesin):
    """The experiments' xtransform (minimal_coordinates/*noise.jl) rebuilds the generator's CState
    exactly in positions, orientations and angular velocities (the linear velocities differ only
    by the finite-difference step: 0.01 there, dt_sim 1e-4 in the generator)."""
    rng = np.random.default_rng(5)
    m = data._sample_minimal(mech, 16, rng)
    q = np.stack([m[k] for pair in data.MIN_COORDS[mech] for k in pair], axis=1)
    A = mdynamics.xtransform(mech, data.min_features(mech, q, usesin), usesin)
    B = data._cstates(mech, m).T
    nb = A.shape[1] // 13
    exact = np.concatenate([np.r_[13 * b:13 * b + 7, 13 * b + 10:13 * b + 13] for b in range(nb)])
    np.testing.assert_allclose(A[:, exact], B[:, exact], rtol=0, atol=1e-15)
    vel = np.concatenate([np.r_[13 * b + 7:13 * b + 10] for b in range(nb)])
    assert np.max(np.abs(A[:, vel] - B[:, vel])) < 0.05


@pytest.mark.parametrize("mech", MECHS)
def test_mean_functions_shapes_and_reference_rates(mech):
    """getμ(vωindices) of the maximal-coordinate experiments and the minimal-coordinate _getμ
    (P2: (w1, w2 - w1)): read from the same solution CState."""
    tr = data.make_trial(mech, 5, 0, seed=9)
    mu = mdynamics.mean_max(mech, tr["X"], physics=vi.vi_step)  # the host step (no GPU here)
    sol, _, _ = vi.vi_step(mech, tr["X"].T)
    np.testing.assert_array_equal(mu, sol[:, np.asarray(data.VW_INDICES[mech]) - 1].T)
    tm = data.make_trial_min(mech, 5, 0, seed=9)
    mm = mdynamics.mean_min(mech, tm["X"], False, physics=vi.vi_step)
    assert mm.shape == (len(data.MIN_COORDS[mech]), 5)
    s2, _, _ = vi.vi_step(mech, mdynamics.xtransform(mech, tm["X"], False))
    if mech == "P2":
        np.testing.assert_array_equal(mm, np.stack([s2[:, 10], s2[:, 23] - s2[:, 10]]))
    else:
        np.testing.assert_array_equal(mm, s2[:, np.asarray(mdynamics.MIN_IDX[mech]) - 1].T)


def test_vi_baseline_simulates_steps_plus_one():
    """predictdynamics(mechanism, start, steps) = simulate!(mechanism, 1:steps+1) (predictdynamics.jl:24-28)."""
    tr = data.make_trial("P1", 2, 3, seed=1)
    S = tr["Xs"].T
    fin, bad = vi.simulate("P1", S, 4)
    ref = S
    for _ in range(5):
        ref, _, _ = vi.vi_step("P1", ref)
    np.testing.assert_array_equal(fin, ref)
    assert not bad.any()


def test_failed_state_is_isolated():
    """A state the reference cannot step (|w| beyond 2/dt: ConstrainedDynamics' sqrt throws a
    DomainError) fails alone: status 2 and a NaN row; the other states' solutions are bit-identical
    to a batch without it.  The sweep drops the trial of such a state (core.jl:41-53)."""
    tr = data.make_trial("P2", 2, 3, seed=2)
    S = tr["Xs"].T.copy()
    good, _, st_good = vi.vi_step("P2", S)
    bad = S.copy()
    bad[1, 10:13] = 1e3 / vi.DT  # body 1's angular velocity far beyond 2/dt
    out, _, st = vi.vi_step("P2", bad)
    assert st[1] == 2 and np.isnan(out[1]).all()
    np.testing.assert_array_equal(out[[0, 2]], good[[0, 2]])
    np.testing.assert_array_equal(st[[0, 2]], st_good[[0, 2]])
    fin, flags = vi.simulate("P2", bad, 2)
    assert flags[1] & 2 and np.isnan(fin[1]).all() and np.isfinite(fin[[0, 2]]).all()
