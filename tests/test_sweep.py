"""The noise.jl sweep (BASELINE config 5) through the product sharding path on the GPU: a reduced
sweep (4 mechanisms x 3 sizes x 8 trials, the three MeanZero variants) through
gprx.sweep.run_group (one shard.RankBatch per group: B = trials x outputs, device LBFGS, device
rollouts) checked against the oracle, and gprx.sweep.run under a world-size-1 gloo group (the
gather path).  Plus the FB hyperparameter.jl-shaped optimise loop at the BASELINE size N=4096.

Oracle checks: the LML at every checked minimiser (oracle fit at the device's theta*), the k-step
rollout final states (oracle rollout with the oracle's alpha at theta*), and the error metric
recomputed on the host.  Tolerances as tests/test_gpu.py (LML) and tests/test_rollout.py
(rollouts: 10x the oracle's distance-mode spread)."""
import math
import os
import socket

import numpy as np
import pytest
import scipy.linalg as sla

pytestmark = pytest.mark.gpu

from oracle import gp_oracle as O  # noqa: E402

MECHS = ("P1", "P2", "CP", "FB")
SIZES = (8, 64, 256)
TRIALS = 8
TESTS = 16
STEPS = 20


@pytest.fixture(scope="module")
def ctx():
    import gprx

    c = gprx.Context(0)
    yield c
    c.close()


def _mll_ok(got, X, y, th, mode):
    f = O.fit(X, y, th, None, mode)
    f2 = O.fit(X, y, th, None, 1 - mode)
    tol = max(1e-9 * max(1.0, abs(f["mll"])), 10 * abs(f["mll"] - f2["mll"]), 10 * f["mll_sens"])
    return abs(got - f["mll"]) <= tol, (got, f["mll"], tol)


@pytest.mark.parametrize("mech", MECHS)
def test_reduced_sweep_against_oracle(ctx, mech):
    from gprx import data, sweep
    from gprx.rollout import NCOORD, final_cstate

    mode = ctx.dist_mode
    for N in SIZES:
        for var in ("max", "min", "min_sin"):  # the MeanDynamics ones: test_meandynamics_variants_against_oracle
            r = sweep.run_group(mech, N, var, range(TRIALS), ctx, testsamples=TESTS, simsteps=STEPS, max_evals=20,
                                keep=True)
            rb, trials = r["rb"], r["trials"]
            G = rb.G
            assert r["kstep_mse"].shape == (TRIALS,) and r["status"].shape == (TRIALS, G)
            assert np.all(r["f_calls"] >= 1)  # the initial evaluation at least (soft f_calls_limit 20)
            for t in (0, TRIALS - 1):  # the LML at the device minimisers against the oracle
                for g in range(G):
                    if r["status"][t, g] != 0:
                        continue
                    ok, info = _mll_ok(r["mll"][t, g], trials[t]["X"], np.atleast_2d(trials[t]["Y"])[g],
                                       r["theta"][t, g], mode)
                    assert ok, (mech, N, var, t, g, info)
            if var == "max":  # device predictdynamics (projectv! + updatestate!) against the oracle loop
                from oracle import projection_oracle as PO

                assert np.sum(np.isfinite(r["kstep_mse"])) >= TRIALS // 2, (mech, N, r["status"])
                idx = data.VW_INDICES[mech]
                for t in ((0,) if N == SIZES[1] else ()):  # one size: the oracle loop is slow Python
                    if not (np.all(r["status"][t] == 0) and np.isfinite(r["kstep_mse"][t])):
                        continue
                    tr = trials[t]
                    truth = data.test_truth(mech, TESTS, tr["seed"], STEPS)["X"].T

                    def kerr_max(md):
                        al = [O.fit(tr["X"], tr["Y"][g], r["theta"][t, g], None, md)["alpha"] for g in range(G)]
                        pars = [O.kernel_params(r["theta"][t, g], tr["X"].shape[0]) for g in range(G)]

                        def predict(obs):
                            D = O.dist_stack(tr["X"], obs[:, None], md)
                            return np.array([(pars[g][1] * np.exp(-O.weighted_r(D, pars[g][0]) * 0.5))[:, 0] @ al[g]
                                             for g in range(G)])

                        fin = [PO.predictdynamics(mech, predict, tr["Xs"][:, m], STEPS, idx,
                                                  regularizer=1e-10 if mech == "FB" else 0.0)[0] for m in range(TESTS)]
                        return data.position_mse(truth, np.stack(fin))

                    e_ref, e_alt = kerr_max(mode), kerr_max(1 - mode)
                    tol = max(1e-8 * max(1.0, abs(e_ref)), 10 * abs(e_ref - e_alt))
                    assert abs(r["kstep_mse"][t] - e_ref) <= tol, (mech, N, t, r["kstep_mse"][t], e_ref, tol)
                continue
            usesin = var == "min_sin"
            nc = NCOORD[mech]
            for t in (0, TRIALS - 1):
                if not np.all(r["status"][t] == 0):
                    continue
                tr = trials[t]
                # three legitimate formulations: the oracle in this distance mode (reference), in the
                # other mode, and with alpha by an LU solve instead of the Cholesky solve -- after
                # optimisation K can be ill-conditioned, and the 20-step rollout carries alpha's
                # rounding (cond(K) eps) forward; the tolerance is 10x the largest spread
                gps, gps2, gps3 = [], [], []
                for g in range(nc):
                    th = r["theta"][t, g]
                    gps.append((tr["X"], th, O.fit(tr["X"], tr["Y"][g], th, None, mode)["alpha"]))
                    gps2.append((tr["X"], th, O.fit(tr["X"], tr["Y"][g], th, None, 1 - mode)["alpha"]))
                    K = O.gram(tr["X"], th, mode)[0]
                    gps3.append((tr["X"], th, sla.solve(K, tr["Y"][g], assume_a="gen")))
                truth = data.test_truth(mech, TESTS, tr["seed"], STEPS)["X"].T

                def kerr(gl, md):
                    fin = O.rollout_min(mech, gl, tr["start"], STEPS, usesin, mode=md)
                    return data.position_mse(truth, np.stack([final_cstate(mech, row[0::2]) for row in fin]))

                err_ref, err_alt, err_lu = kerr(gps, mode), kerr(gps2, 1 - mode), kerr(gps3, mode)
                spread = max(abs(err_ref - err_alt), abs(err_ref - err_lu))
                tol = max(1e-9 * max(1.0, abs(err_ref)), 10 * spread)
                assert abs(r["kstep_mse"][t] - err_ref) <= tol, (mech, N, var, t, r["kstep_mse"][t], err_ref, tol)
            rb.close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_sweep_run_gathers_through_a_process_group(ctx):
    """gprx.sweep.run under an initialised (gloo, world 1) group: the gathered checkpoint equals
    the per-group results, in the reference's final-checkpoint shape (core.jl:79-82)."""
    import torch.distributed as dist

    from gprx import sweep

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        res = sweep.run(("P2", "CP"), (16,), ("min", "max"), n_trials=4, testsamples=TESTS, simsteps=STEPS,
                        max_evals=10, ctx=ctx)
    finally:
        dist.destroy_process_group()
    assert set(res["results"]["noisy"]) == {"P2_MIN16", "P2_MAX16", "CP_MIN16", "CP_MAX16"}
    e = res["results"]["noisy"]["P2_MIN16"]
    r = sweep.run_group("P2", 16, "min", range(4), ctx, TESTS, STEPS, 10)
    # failed trials are dropped from the lists (core.jl:41-53), nprocessed still counts them
    assert e["nprocessed"] == 4 and len(e["kstep_mse"]) == 4 - int(r["failed"].sum()) == 4 - e["dropped"]
    np.testing.assert_array_equal(e["kstep_mse"], r["kstep_mse"][~r["failed"]])
    assert len(e["projectionerror"]) == len(e["kstep_mse"])


def test_fb_hyperparameter_optimise_n4096(ctx):
    """examples/hyperparameter.jl:50-60 -> experimentFBMax (maximal_coordinates/FBparam.jl:23-33)
    at the BASELINE size: FB, N=4096, d=52, the 12 output GPs of one trial, all starting from the
    trial's ONE random draw params = [1, 10 ./ std(X)] .+ (5rand .- 0.999) .* params (gprx.search),
    MeanZero, device LBFGS + BackTracking(order=2) with a 30-evaluation budget.  The LML at the
    minimisers against the oracle; the optimiser improves every slot it does not fail on."""
    import gprx
    from gprx import data, search
    from gprx.optim import LBFGS, Options

    # the generator's noisy states: its noise-free four-bar targets are an exact function of the
    # inputs, which drives sigma_n -> 0 and cond(K) past what an LML comparison can resolve
    tr = data.make_trial("FB", 4096, 0, seed=data.trial_seed("FB", 1))
    X, Y = tr["X"], tr["Y"]
    G = Y.shape[0]
    p = search.init_params("FB_MAX", X, search.draw_rng("FB_MAX", 4096, 1))
    stdx = X.std(axis=1, ddof=1)
    stdx[stdx == 0] = 1000.0
    base = np.concatenate([[1.0], 10.0 / stdx])
    assert np.all((p >= 0.001 * base - 1e-12) & (p <= 5.001 * base + 1e-12))  # (5 rand - 0.999) jitter
    th0 = np.tile(data.theta_from_params(p), (G, 1))  # one draw shared by all 12 outputs
    b = gprx.GPBatch(G, 52, 4096, 0, ctx=ctx)
    b.set_train(X, Y)
    start = b.run(th0, grad=False)
    res, rounds = b.optimize(th0, LBFGS(), Options(max_evals=30), refit=True)
    # max_evals is Optim's soft f_calls_limit (checked after each iteration: the last line search
    # may overrun it); a round is at most one f call of each running slot
    assert rounds <= max(x.f_calls for x in res)
    thmin = np.stack([x.minimizer for x in res])
    r = b.run(thmin, grad=False)
    for s in range(G):
        assert res[s].converged or res[s].f_calls >= 30
        if start["status"][s] == 0:
            assert r["mll"][s] >= start["mll"][s]
    for s in (0, 5, 11):
        ok, info = _mll_ok(r["mll"][s], X, Y[s], thmin[s], ctx.dist_mode)
        assert ok, (s, info)
    b.close()


@pytest.mark.parametrize("mech", ("P1", "P2", "CP", "FB"))
def test_meandynamics_variants_against_oracle(ctx, mech):
    """noise.jl's experiment_*_md_max / _md_min / _md_min_sin (MeanDynamics GPs) through the product
    path (gprx.sweep.run_group -> gprx.mdynamics): mu(X) once per training set against the
    independent action-based VI oracle, the LML at the device minimisers against the oracle GP on
    y - mu(X), and the rollouts (GP mean + physics mean per step; projectv! for maximal
    coordinates) against an oracle loop (oracle GP means, oracle VI, oracle projection)."""
    from gprx import data, mdynamics, sweep
    from gprx.projection import REGULARIZER
    from gprx.rollout import final_cstate
    from oracle import projection_oracle as PO
    from oracle import vi_oracle as VO

    mode = ctx.dist_mode
    N, M, steps = 16, 4, 3
    for var in ("md_max", "md_min", "md_min_sin"):
        r = sweep.run_group(mech, N, var, range(2), ctx, testsamples=M, simsteps=steps, max_evals=10, keep=True)
        rb, trials = r["rb"], r["trials"]
        tr = trials[0]
        usesin = var == "md_min_sin"
        # the physics mean of the first training column against the oracle
        if var == "md_max":
            o, _ = VO.vi_step(mech, tr["X"][:, 0])
            mu_o = o[np.asarray(data.VW_INDICES[mech]) - 1]
        else:
            o, _ = VO.vi_step(mech, mdynamics.xtransform(mech, tr["X"][:, :1], usesin)[0])
            mu_o = (np.array([o[10], o[23] - o[10]]) if mech == "P2"
                    else o[np.asarray(mdynamics.MIN_IDX[mech]) - 1])
        np.testing.assert_allclose(tr["mu"][:, 0], mu_o, rtol=0, atol=1e-9)
        assert np.all(r["status"][0] == 0)
        G = rb.G
        th = r["theta"][0]
        for g in range(G):
            ok, info = _mll_ok(r["mll"][0, g], tr["X"], tr["Y"][g], th[g], mode)
            assert ok, (var, g, info)
        al = [O.fit(tr["X"], tr["Y"][g], th[g], None, mode)["alpha"] for g in range(G)]

        def gp_mean(feat):
            out = []
            for g in range(G):
                il2, sf2 = np.exp(-2 * th[g][1:-1]), np.exp(2 * th[g][-1])
                D = O.dist_stack(tr["X"], feat[:, None], mode)
                out.append(float((sf2 * np.exp(-0.5 * np.einsum("pij,p->ij", D, il2)))[:, 0] @ al[g]))
            return np.array(out)

        if var == "md_max":
            starts = np.stack([t["Xs"].T for t in trials])
            fin, pe, st = mdynamics.rollout_max(mech, rb, [0], starts, steps, ctx=ctx)
            assert np.all(st == 0)
            for j in range(2):
                def predict(obs):
                    s, _ = VO.vi_step(mech, obs)
                    return gp_mean(obs) + s[np.asarray(data.VW_INDICES[mech]) - 1]

                # the experiments' projectv! regulariser (1e-10 for the four-bar, FBnoise.jl:43)
                ref, perr = PO.predictdynamics(mech, predict, starts[0, j], steps, data.VW_INDICES[mech],
                                               regularizer=REGULARIZER[mech])
                np.testing.assert_allclose(fin[0, j], ref, rtol=0, atol=1e-7)
                assert abs(pe[0, j] - perr) <= 1e-7 * max(1.0, perr)
        else:
            starts = np.stack([t["start"] for t in trials])
            fin = mdynamics.rollout_min(mech, rb, [0], starts, steps, usesin)
            for j in range(2):
                q_old, qd_old = starts[0, j, 0::2].copy(), starts[0, j, 1::2].copy()
                q_cur = q_old + 0.01 * qd_old
                for _ in range(steps):
                    obs = np.empty(2 * len(q_old))
                    obs[0::2], obs[1::2] = q_old, qd_old
                    feat = data.min_features(mech, obs[None, :], usesin)[:, 0]
                    o, _ = VO.vi_step(mech, mdynamics.xtransform(mech, feat[:, None], usesin)[0])
                    mo = (np.array([o[10], o[23] - o[10]]) if mech == "P2"
                          else o[np.asarray(mdynamics.MIN_IDX[mech]) - 1])
                    rates = gp_mean(feat) + mo
                    q_old, qd_old = q_cur, rates
                    q_cur = q_cur + 0.01 * rates
                np.testing.assert_allclose(fin[0, j], final_cstate(mech, q_cur), rtol=0, atol=1e-9)
        rb.close()


@pytest.mark.parametrize("mech,N,variant,n_tr,fit", [("P2", 512, "max", 8, 6), ("CP", 128, "md_max", 12, 8),
                                                     ("P2", 128, "min", 9, 4)])
def test_chunked_group_equals_one_batch(ctx, mech, N, variant, n_tr, fit):
    """A group whose trials do not fit the device budget runs as several device batches one after
    another (shard.group_plan), with results bit-identical to one batch: the optimiser's minimisers,
    f-call counts, LML, status and the rollout errors.  `fit` trials per batch fit the forced
    budget; P2 max (6 outputs, 48 slots) and CP md_max (4 outputs, 48 slots) run two chunks padded
    to the 32-slot launch geometry, P2 min (2 outputs, 18 slots) three unpadded chunks
    (examples/hyperparameter.jl:43 runs 100 trials through one parallelrun, core.jl:27-67)."""
    from gprx import shard, sweep

    trials = sweep.local_trials(mech, N, variant, range(n_tr), 8, ctx)
    G = np.atleast_2d(trials[0]["Y"]).shape[0]
    d = trials[0]["X"].shape[0]
    M = 0 if trials[0].get("Xs") is None else trials[0]["Xs"].shape[1]
    one, two = shard.batch_bytes(1, d, N, M), shard.batch_bytes(2, d, N, M)
    budget = (2 * one - two) + fit * G * (two - one)
    plan = shard.group_plan(trials, ctx, budget)
    assert len(plan) >= 2 and all(nd <= fit for _, _, nd in plan)
    if n_tr * G >= 32:
        assert all(nd * G >= 32 for _, _, nd in plan)
    kw = dict(testsamples=8, simsteps=5, max_evals=12, trials=trials)
    single = sweep.run_group(mech, N, variant, range(n_tr), ctx, **kw)
    chunked = sweep.run_group(mech, N, variant, range(n_tr), ctx, budget=budget, **kw)
    assert chunked["batches"] == len(plan) and single["batches"] == 1
    for k in ("theta", "f_calls", "mll", "status", "kstep_mse", "projectionerror", "failed"):
        np.testing.assert_array_equal(chunked[k], single[k], err_msg=k)
    assert np.sum(single["status"] == 0) > 0
    with pytest.raises(ValueError):
        sweep.run_group(mech, N, variant, range(n_tr), ctx, budget=budget, keep=True, **kw)


def test_gpu_evaluator_chunked_equals_one_batch(ctx):
    """shard.gpu_evaluator (run_trials_sharded's product evaluator) with a budget that forces three
    device batches: mll, gradient, mean and variance bit-identical to one batch."""
    from gprx import data, shard

    n_tr, N = 10, 256
    trials = []
    for t in range(n_tr):
        tr = data.make_trial("P2", N, 12, seed=data.trial_seed("P2", 30 + t))
        trials.append(dict(X=tr["X"], Y=tr["Y"], Xs=tr["Xs"], theta=np.tile(data.theta0("P2", N), (6, 1))))
    one, two = shard.batch_bytes(1, 26, N, 12), shard.batch_bytes(2, 26, N, 12)
    budget = (2 * one - two) + 6 * 6 * (two - one)
    assert len(shard.group_plan(trials, ctx, budget)) == 2
    a = shard.gpu_evaluator(ctx=ctx)(trials)
    b = shard.gpu_evaluator(ctx=ctx, budget=budget)(trials)
    assert set(a) == set(b) and {"mll", "grad", "mu", "var", "status"} <= set(a)
    for k in a:
        assert a[k].shape[:2] == (n_tr, 6)
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
