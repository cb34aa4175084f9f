"""Rollouts in minimal coordinates (predictdynamicsmin, examples/utils/predictdynamics.jl:30-102).

CPU: the oracle's loop against hand-evaluated cases and its own per-trajectory form; the host
CState builder against the data generator's kinematics.  GPU: gprx_rollout_min (one launch, all
trajectories) against the oracle rollout with the oracle's own alpha, for all four mechanisms with
and without sin/cos features, several trials per launch, and the single-trajectory GPE mirror.

Tolerance on the final states: max(1e-9 * max(1, |state|), 10x the spread between the oracle's two
distance formulations) -- the per-step prediction bound of tests/test_gpu.py carried through the
step chain (20 steps of dt = 0.01 do not amplify it measurably).
"""
import math

import numpy as np
import pytest

from oracle import gp_oracle as O

MECHS = ["P1", "P2", "CP", "FB"]
TOL = 1e-9


def _data():
    import gprx.data as D

    return D


def _oracle_gps(D, mech, trial, theta, mode):
    gps = []
    for g in range(trial["Y"].shape[0]):
        _, _, aux = O.lml(trial["X"], trial["Y"][g], theta, mode)
        gps.append((trial["X"], theta, aux["alpha"]))
    return gps


# ---------------------------------------------------------------------------------- CPU
def test_oracle_rollout_zero_steps_is_first_euler_step():
    D = _data()
    tr = D.make_trial_min("P2", 16, 5, seed=3)
    theta = D.theta0_min("P2", 16)
    gps = _oracle_gps(D, "P2", tr, theta, O.DIST_EXPANDED)
    out = O.rollout_min("P2", gps, tr["start"], 0)
    st = tr["start"]
    assert np.array_equal(out[:, 0::2], st[:, 0::2] + 0.01 * st[:, 1::2])
    assert np.array_equal(out[:, 1::2], st[:, 1::2])


def test_oracle_rollout_trajectories_independent():
    D = _data()
    tr = D.make_trial_min("CP", 24, 6, seed=4, usesin=True)
    theta = D.theta0_min("CP", 16, usesin=True)
    gps = _oracle_gps(D, "CP", tr, theta, O.DIST_EXPANDED)
    allt = O.rollout_min("CP", gps, tr["start"], 7, usesin=True)
    for t in range(tr["start"].shape[0]):
        one = O.rollout_min("CP", gps, tr["start"][t:t + 1], 7, usesin=True)
        # equal up to the order of the k*'alpha sums (BLAS blocks T=1 and T=6 differently); the
        # cartpole alphas are large and of mixed sign, so that order shows at ~1e-10
        np.testing.assert_allclose(one[0], allt[t], rtol=1e-9, atol=1e-12)


def test_oracle_rollout_one_step_by_hand():
    """P1 with one GP: one step = q_cur' = q_old + dt*v_old + dt*mu(obs(start))."""
    D = _data()
    tr = D.make_trial_min("P1", 10, 3, seed=5)
    theta = D.theta0_min("P1", 8)
    gps = _oracle_gps(D, "P1", tr, theta, O.DIST_DIRECT)
    out = O.rollout_min("P1", gps, tr["start"], 1, mode=O.DIST_DIRECT)
    X, _, alpha = gps[0]
    il2, sf2, _, _ = O.kernel_params(theta, 2)
    for t, (q, v) in enumerate(tr["start"]):
        k = np.array([sf2 * math.exp(-0.5 * ((X[0, j] - q) ** 2 * il2[0] + (X[1, j] - v) ** 2 * il2[1]))
                      for j in range(X.shape[1])])
        m = float(k @ alpha)
        assert out[t, 1] == pytest.approx(m, rel=1e-12, abs=1e-14)
        assert out[t, 0] == pytest.approx((q + 0.01 * v) + m * 0.01, rel=1e-14)


def test_min_features_layout():
    D = _data()
    q = np.array([[0.3, -1.0, 2.0, 0.5]])
    assert np.array_equal(D.min_features("P2", q, False)[:, 0], q[0])
    f = D.min_features("CP", q, True)[:, 0]
    assert np.array_equal(f, [0.3, -1.0, math.sin(2.0), math.cos(2.0), 0.5])
    f = D.min_features("FB", q, True)[:, 0]
    assert np.array_equal(f, [math.sin(0.3), math.cos(0.3), -1.0, math.sin(2.0), math.cos(2.0), 0.5])
    th = D.theta0_min("P2", 64, usesin=True)
    assert th.shape == (8,) and th[1] == th[2] and th[4] == th[5]


@pytest.mark.parametrize("mech", MECHS)
def test_final_cstate_matches_kinematics(mech):
    """The returned CState (positions + orientations, zero velocities) equals the generator's
    CState for the same minimal coordinates (same reference kinematics)."""
    import gprx.rollout as R

    D = _data()
    rng = np.random.default_rng(7)
    m = D._sample_minimal(mech, 5, rng)
    cs = D._cstates(mech, m)  # (13 nb, 5)
    keys = D.MIN_COORDS[mech]
    for t in range(5):
        q = [m[pair[0]][t] for pair in keys]
        got = R.final_cstate(mech, q)
        ref = cs[:, t].copy()
        for b in range(ref.shape[0] // 13):
            ref[13 * b + 7:13 * b + 13] = 0.0  # predictdynamicsmin zeroes the velocities
        np.testing.assert_allclose(got, ref, rtol=0, atol=2e-15)


# ---------------------------------------------------------------------------------- GPU
def _gpu_case(mech, usesin, N, T, steps, trials=1, seed=11):
    import gprx
    import gprx.rollout as R

    D = _data()
    nc = R.NCOORD[mech]
    trs = [D.make_trial_min(mech, N, T, seed=seed + k, usesin=usesin) for k in range(trials)]
    theta = D.theta0_min(mech, 256 if N >= 256 else 64, usesin=usesin)
    d = trs[0]["d"]
    b = gprx.GPBatch(trials * nc, d, N)
    X = np.stack([tr["X"] for tr in trs for _ in range(nc)])
    Y = np.concatenate([tr["Y"] for tr in trs])
    b.set_train(X, Y)
    r = b.run(np.tile(theta, (trials * nc, 1)))
    assert np.all(r["status"] == 0)
    groups = [[(b, k * nc + g) for g in range(nc)] for k in range(trials)]
    start = np.concatenate([tr["start"] for tr in trs])
    tg = np.repeat(np.arange(trials), T)
    out = R.rollout_min(mech, groups, start, steps, usesin, traj_group=tg)
    mode = b.ctx.dist_mode
    refs, alts = [], []
    for k, tr in enumerate(trs):
        refs.append(O.rollout_min(mech, _oracle_gps(D, mech, tr, theta, mode), tr["start"], steps, usesin, mode=mode))
        alts.append(O.rollout_min(mech, _oracle_gps(D, mech, tr, theta, 1 - mode), tr["start"], steps, usesin,
                                  mode=1 - mode))
    ref, alt = np.concatenate(refs), np.concatenate(alts)
    tol = np.maximum(TOL * np.maximum(1.0, np.abs(ref)), 10 * np.abs(ref - alt))
    return out, ref, tol, b


@pytest.mark.gpu
@pytest.mark.parametrize("mech", MECHS)
@pytest.mark.parametrize("usesin", [False, True])
def test_rollout_matches_oracle(mech, usesin):
    out, ref, tol, _ = _gpu_case(mech, usesin, N=256, T=40, steps=20)
    assert np.all(np.isfinite(out))
    assert np.all(np.abs(out - ref) <= tol), float(np.max(np.abs(out - ref) / tol))


@pytest.mark.gpu
def test_rollout_many_trials_one_launch():
    out, ref, tol, _ = _gpu_case("P2", True, N=300, T=25, steps=20, trials=5, seed=40)
    assert np.all(np.abs(out - ref) <= tol)


@pytest.mark.gpu
def test_rollout_first_step_equals_predict():
    """One step's rate is the GP predictive mean at the start observation (same kernel sums as
    gprx_batch_predict, up to the order of the final reduction)."""
    import gprx.rollout as R

    D = _data()
    out, _, _, b = _gpu_case("FB", False, N=200, T=30, steps=1)
    tr = D.make_trial_min("FB", 200, 30, seed=11)
    b.set_test(D.min_features("FB", tr["start"], False))
    mu, _ = b.predict(variance=False)
    for g in range(R.NCOORD["FB"]):
        np.testing.assert_allclose(out[:, 2 * g + 1], mu[g], rtol=1e-12, atol=1e-13 * np.max(np.abs(mu[g])))


@pytest.mark.gpu
def test_rollout_zero_steps_and_edges():
    import gprx
    import gprx.rollout as R

    out, _, _, b = _gpu_case("CP", False, N=64, T=8, steps=0)
    D = _data()
    st = D.make_trial_min("CP", 64, 8, seed=11)["start"]
    assert np.array_equal(out[:, 0::2], st[:, 0::2] + 0.01 * st[:, 1::2])
    assert np.array_equal(out[:, 1::2], st[:, 1::2])
    # no trajectories: nothing to do
    assert R.rollout_min("CP", [[(b, 0), (b, 1)]], np.zeros((0, 4)), 5).shape == (0, 4)
    # input dimension must match the mechanism's features (usesin: 5, batch has 4)
    with pytest.raises(gprx.GPRXError):
        R.rollout_min("CP", [[(b, 0), (b, 1)]], st, 3, usesin=True)
    # slot out of range
    with pytest.raises(gprx.GPRXError):
        R.rollout_min("CP", [[(b, 0), (b, 2)]], st, 3)
    # a batch that has not been factorised
    b2 = gprx.GPBatch(2, 4, 64)
    b2.set_train(D.make_trial_min("CP", 64, 1, seed=2)["X"], D.make_trial_min("CP", 64, 1, seed=2)["Y"])
    with pytest.raises(gprx.GPRXError):
        R.rollout_min("CP", [[(b2, 0), (b2, 1)]], st, 3)


@pytest.mark.gpu
def test_predictdynamicsmin_gpe_mirror():
    """The GPE-level mirror: GP(...) per output, then predictdynamicsmin for one start state and
    the batched test loop; CState built as predictdynamics.jl:63-66."""
    import gprx
    import gprx.rollout as R

    D = _data()
    tr = D.make_trial_min("P2", 128, 6, seed=21, usesin=True)
    theta = D.theta0_min("P2", 128, usesin=True)
    gps = []
    for g in range(2):
        k = gprx.SEArd(theta[1:-1], theta[-1])
        gps.append(gprx.GP(tr["X"], tr["Y"][g], gprx.MeanZero(), k, logNoise=theta[0]))
    allc = R.predictdynamicsmin_batch("P2", gps, tr["start"], 20, usesin=True)
    one = R.predictdynamicsmin("P2", gps, tr["start"][2], 20, usesin=True)
    np.testing.assert_array_equal(one, allc[2])
    mode = gps[0].ctx.dist_mode
    ref = O.rollout_min("P2", _oracle_gps(D, "P2", tr, theta, mode), tr["start"], 20, True, mode=mode)
    for t in range(tr["start"].shape[0]):
        np.testing.assert_allclose(allc[t], R.final_cstate("P2", ref[t, 0::2]), rtol=1e-9, atol=1e-9)
    # MeanDynamics-style means need the host physics per step
    gm = gprx.GP(tr["X"], tr["Y"][0], gprx.MeanFunction(lambda x: 0.0), gprx.SEArd(theta[1:-1], theta[-1]))
    with pytest.raises(NotImplementedError):
        R.predictdynamicsmin("P2", [gm, gps[1]], tr["start"][0], 3, usesin=True)


@pytest.mark.gpu
def test_predictdynamics_maximal_batched_matches_oracle():
    """predictdynamics.jl:7-22 with the physics injected: per step one mean-only evaluation of the
    trial's G GPs at all T CStates; an explicit-Euler 'advance' stands in for projectv! +
    updatestate!.  Against the same loop on the oracle's predictive means."""
    import gprx
    import gprx.rollout as R

    D = _data()
    tr = D.make_trial("P2", 256, 8, seed=31)
    th = D.theta0("P2", 256)
    G = tr["Y"].shape[0]
    b = gprx.GPBatch(G, 26, 256, 8)
    b.set_train(tr["X"], tr["Y"])
    assert np.all(b.run(np.tile(th, (G, 1)))["status"] == 0)
    idx = D.VW_INDICES["P2"]  # outputs = v_y, v_z, omega_x of both bodies (1-based CState entries)

    def getvw(mu):
        return mu[[0, 1, 3, 4]], mu[[2, 5]]

    def advance(s, v, w):
        s = s.copy()
        for k, i in enumerate([9, 10, 22, 23]):
            s[i - 1] = v[k]
        s[10], s[23] = w[0], w[1]
        s[1] += 0.01 * s[8]
        s[2] += 0.01 * s[9]
        s[14] += 0.01 * s[21]
        s[15] += 0.01 * s[22]
        return s, 0.0

    start = tr["Xs"].T.copy()  # (T, 26)
    got, err = R.predictdynamics(b, start, 5, getvw, advance)
    mode = b.ctx.dist_mode
    alphas = [O.lml(tr["X"], tr["Y"][g], th, mode)[2]["alpha"] for g in range(G)]
    il2, sf2, _, _ = O.kernel_params(th, 26)
    S = start.copy()
    for _ in range(5):
        Ks = sf2 * np.exp(-O.weighted_r(O.dist_stack(tr["X"], S.T, mode), il2) * 0.5)  # N x T
        mu = np.stack([Ks.T @ alphas[g] for g in range(G)])
        for t in range(S.shape[0]):
            S[t], _ = advance(S[t], *getvw(mu[:, t]))
    assert idx == [9, 10, 22, 23, 11, 24]
    np.testing.assert_allclose(got, S, rtol=1e-9, atol=1e-10)
    assert np.all(err == 0.0)
