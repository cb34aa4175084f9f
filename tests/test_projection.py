"""projectv! (src/projections/implicitProjection.jl:80-107) and the maximal-coordinate rollout
(examples/utils/predictdynamics.jl:7-22).

Parity is UNPINNED w.r.t. the reference: ConstrainedDynamics 0.7.4 (constraint functions, state
update) is absent and the reference has no vectors (oracle/projection_oracle.py).  What the CPU
tests pin the restatement to instead:
  * the joint zero sets: every mechanism's constraints vanish at the data generator's states
    (gprx/data.py, the reference's kinematics) -- the geometry of simulations.jl;
  * the Jacobians: against central finite differences of the constraint functions;
  * the fixed point: the KKT conditions of min |s - s_u|^2 s.t. g(s) = 0 (g = 0 and s_u - s in the
    row space of G), which do not depend on how the constraints are written;
  * the loop structure: updatestate! after every projection and once at the end.
GPU tests: the device kernels against the oracle on the same inputs.  Tolerances: projected twists
1e-9 relative to max|s| (a converged Newton fixed point; the two LU implementations differ at
rounding level); rollouts as tests/test_rollout.py (1e-9 relative, or 10x the spread between the
oracle's two distance formulations, carried through the 20-step chain).
"""
import math

import numpy as np
import pytest

from oracle import gp_oracle as O
from oracle import projection_oracle as PO

MECHS = ["P1", "P2", "CP", "FB"]
REG = {"P1": 0.0, "P2": 0.0, "CP": 0.0, "FB": 1e-10}


def _states(mech, n, seed):
    import gprx.data as D

    return D._cstates(mech, D._sample_minimal(mech, n, np.random.default_rng(seed)))  # (d, n) clean


def _rest(cs, nb):
    c = np.array(cs, dtype=np.float64).reshape(nb, 13)
    c[:, 7:] = 0.0  # zero velocities: x3 = x, q3 = q
    return c.reshape(-1)


# ---------------------------------------------------------------------------------- CPU
@pytest.mark.parametrize("mech", MECHS)
def test_constraints_vanish_on_the_mechanism_kinematics(mech):
    m = PO.mechanism(mech)
    X = _states(mech, 6, 1)
    for t in range(X.shape[1]):
        st = PO.State(_rest(X[:, t], m["nb"]), m["nb"])
        assert np.max(np.abs(PO.constraints(m, st))) < 1e-14


@pytest.mark.parametrize("mech", MECHS)
def test_jacobian_matches_finite_differences(mech):
    m = PO.mechanism(mech)
    nb = m["nb"]
    X = _states(mech, 3, 2)
    rng = np.random.default_rng(3)
    for t in range(X.shape[1]):
        st = PO.State(X[:, t], nb)
        s = rng.standard_normal(6 * nb) * 0.5
        PO._set_solution(st, s)
        G = PO.jacobian(m, st)
        h = 1e-6
        Gf = np.empty_like(G)
        for j in range(6 * nb):
            sp, sm = s.copy(), s.copy()
            sp[j] += h
            sm[j] -= h
            PO._set_solution(st, sp)
            gp = PO.constraints(m, st)
            PO._set_solution(st, sm)
            gm = PO.constraints(m, st)
            Gf[:, j] = (gp - gm) / (2 * h)
        PO._set_solution(st, s)
        assert np.max(np.abs(G - Gf)) < 1e-8, np.max(np.abs(G - Gf))


@pytest.mark.parametrize("mech", MECHS)
def test_projection_reaches_the_kkt_point(mech):
    m = PO.mechanism(mech)
    nb = m["nb"]
    X = _states(mech, 4, 4)
    rng = np.random.default_rng(5)
    for t in range(X.shape[1]):
        st = PO.State(X[:, t], nb)
        vu = [st.vc[b] + 0.05 * rng.standard_normal(3) for b in range(nb)]
        wu = [st.wc[b] + 0.05 * rng.standard_normal(3) for b in range(nb)]
        v, w, it = PO.projectv(m, st, vu, wu, regularizer=REG[mech])
        assert it < 20
        assert np.max(np.abs(PO.constraints(m, st))) < 1e-12
        s = np.concatenate([np.concatenate([v[b], w[b]]) for b in range(nb)])
        su = np.concatenate([np.concatenate([vu[b], wu[b]]) for b in range(nb)])
        G = PO.jacobian(m, st)
        lam = np.linalg.lstsq(G.T, su - s, rcond=None)[0]
        assert np.max(np.abs(G.T @ lam - (su - s))) < 1e-10
        # an already-consistent twist is its own projection
        v2, w2, _ = PO.projectv(m, st, v, w, regularizer=REG[mech])
        np.testing.assert_allclose(np.concatenate(v2 + w2), np.concatenate(v + w), rtol=0, atol=1e-12)


def test_rollout_loop_structure_without_gps():
    """predictdynamics with a 'GP' that predicts the current state's own velocities: each step is
    projectv! + updatestate!, and the final CState comes after steps + 1 updates."""
    m = PO.mechanism("P2")
    X = _states("P2", 1, 7)[:, 0]
    idx = [9, 10, 22, 23, 11, 24]
    final, perr = PO.predictdynamics("P2", lambda obs: obs[np.array(idx) - 1], X, 3, idx)
    st = PO.State(X, 2)
    obs = X.copy()
    for _ in range(3):
        vu, wu = PO.getvw(obs[np.array(idx) - 1], idx, 2)
        PO.projectv(m, st, vu, wu)
        st.update()
        obs = st.cstate()
    st.update()
    np.testing.assert_array_equal(final, st.cstate())
    assert perr >= 0.0


def test_getvw_matches_the_experiments():
    vu, wu = PO.getvw(np.arange(1.0, 7.0), [9, 10, 22, 23, 11, 24], 2)  # P2noise.jl:46
    assert np.array_equal(vu[0], [0, 1, 2]) and np.array_equal(vu[1], [0, 3, 4])
    assert np.array_equal(wu[0], [5, 0, 0]) and np.array_equal(wu[1], [6, 0, 0])
    import gprx.projection as GP

    vw = GP.getvw(np.arange(1.0, 7.0), [9, 10, 22, 23, 11, 24], 2)
    assert np.array_equal(vw, [0, 1, 2, 5, 0, 0, 0, 3, 4, 6, 0, 0])


# ---------------------------------------------------------------------------------- GPU
@pytest.mark.gpu
@pytest.mark.parametrize("mech", MECHS)
def test_device_projectv_matches_oracle(mech):
    import gprx.projection as GP

    m = PO.mechanism(mech)
    nb = m["nb"]
    X = _states(mech, 32, 11)
    rng = np.random.default_rng(12)
    T = X.shape[1]
    vw = np.empty((T, 6 * nb))
    ref = np.empty((T, 6 * nb))
    its = []
    for t in range(T):
        st = PO.State(X[:, t], nb)
        vu = [st.vc[b] + 0.1 * rng.standard_normal(3) for b in range(nb)]
        wu = [st.wc[b] + 0.1 * rng.standard_normal(3) for b in range(nb)]
        vw[t] = np.concatenate([np.concatenate([vu[b], wu[b]]) for b in range(nb)])
        v, w, it = PO.projectv(m, st, vu, wu, regularizer=REG[mech])
        ref[t] = np.concatenate([np.concatenate([v[b], w[b]]) for b in range(nb)])
        its.append(it)
    out, it_dev, status = GP.projectv(mech, X.T, vw)
    assert np.all(status == 0)
    np.testing.assert_allclose(out, ref, rtol=0, atol=1e-9 * np.max(np.abs(ref)))
    if mech != "FB":  # FB's loop-closure constraints are redundant: the regularised KKT matrix is
        # near-singular, the multipliers are not unique and |ds| may stall above eps on either side
        # (the twists themselves agree, above)
        assert np.max(np.abs(it_dev - np.array(its))) <= 1


@pytest.mark.gpu
@pytest.mark.parametrize("mech", MECHS)
def test_device_max_rollout_matches_oracle(mech):
    """The maximal-coordinate predictdynamics of the experiments (MeanZero GPs on CState inputs,
    theta from config.json, 20 steps) on the device against the oracle loop: the same GP means (the
    oracle's alpha), projectv! and updatestate! per step."""
    import gprx
    import gprx.data as D
    import gprx.projection as GP

    N, T, steps = 96, 12, 20
    tr = D.make_trial(mech, N, T, seed=D.trial_seed(mech, 5))
    th = D.theta0(mech, 64)
    G = tr["Y"].shape[0]
    b = gprx.GPBatch(G, tr["d"], N, 0)
    b.set_train(tr["X"], tr["Y"])
    assert np.all(b.run(np.tile(th, (G, 1)))["status"] == 0)
    idx = D.VW_INDICES[mech]
    out, pe, st = GP.predictdynamics(mech, [[(b, g) for g in range(G)]], tr["Xs"].T, steps, idx)
    assert np.all(st == 0)
    mode = b.ctx.dist_mode

    def oracle_run(md):
        alphas = [O.lml(tr["X"], tr["Y"][g], th, md)[2]["alpha"] for g in range(G)]
        il2, sf2, _, _ = O.kernel_params(th, tr["d"])

        def predict(obs):
            Ks = sf2 * np.exp(-O.weighted_r(O.dist_stack(tr["X"], obs[:, None], md), il2) * 0.5)[:, 0]
            return np.array([Ks @ a for a in alphas])

        res = [PO.predictdynamics(mech, predict, tr["Xs"][:, t], steps, idx, regularizer=REG[mech]) for t in range(T)]
        return np.stack([r[0] for r in res]), np.array([r[1] for r in res])

    ref, pref = oracle_run(mode)
    alt, _ = oracle_run(1 - mode)
    tol = np.maximum(1e-9 * np.maximum(1.0, np.abs(ref)), 10 * np.abs(ref - alt))
    assert np.all(np.isfinite(out))
    assert np.all(np.abs(out - ref) <= tol), float(np.max(np.abs(out - ref) / tol))
    np.testing.assert_allclose(pe, pref, rtol=1e-6, atol=1e-12)
    b.close()


def test_default_device_choice():
    """projection._default_ctx's device: GPRX_DEVICE, else torch's current device when
    torch's HIP runtime is already initialised (torch.cuda.set_device is honoured), else LOCAL_RANK
    modulo the visible devices; no runtime is initialised by the lookup."""
    from gprx.projection import default_device

    class FakeCuda:
        def __init__(self, init, cur):
            self.init, self.cur = init, cur

        def is_initialized(self):
            return self.init

        def current_device(self):
            return self.cur

    class FakeTorch:
        def __init__(self, init, cur):
            self.cuda = FakeCuda(init, cur)

    assert default_device(8, {}) == 0
    assert default_device(8, {"LOCAL_RANK": "5"}) == 5
    assert default_device(4, {"LOCAL_RANK": "5"}) == 1
    assert default_device(8, {"LOCAL_RANK": "5"}, FakeTorch(False, 3)) == 5
    assert default_device(8, {"LOCAL_RANK": "5"}, FakeTorch(True, 3)) == 3
    assert default_device(8, {"LOCAL_RANK": "5", "GPRX_DEVICE": "6"}, FakeTorch(True, 3)) == 6
    assert default_device(0, {"GPRX_DEVICE": "2"}) == 0
