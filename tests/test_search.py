"""The hyperparameter.jl random-restart search (gprx.search; examples/hyperparameter.jl:50-60 over
examples/parallel/core.jl:94-112).  CPU: the per-experiment random starts (the eight *param.jl
files), the trial inputs, the params_final shape and createconfig.jl's argmin.  GPU: a reduced
search through the product path (one RankBatch per group, device LBFGS, device rollouts), the LML
at the minimisers against the oracle, and the gathered checkpoint under a world-1 process group."""
import math
import os
import socket

import numpy as np
import pytest

from gprx import data, search


def test_experiment_table_matches_the_param_files():
    # (sigma_f, numerator, fill) as the experiment files write them (file:line in gprx/search.py)
    assert search.INIT["P1_MAX"] == (100.0, 10.0, 1000.0)
    assert search.INIT["P2_MAX"] == (1.1, 50.0, 1000.0)
    assert search.INIT["CP_MAX"] == (100.0, 50.0, 1000.0)
    assert search.INIT["FB_MAX"] == (1.0, 10.0, 1000.0)
    assert search.INIT["P1_MIN"] == (1.1, 10.0, 100.0)
    assert search.INIT["P2_MIN"] == (1.1, 50.0, 1000.0)
    assert search.INIT["CP_MIN"] == (100.0, 50.0, 1000.0)
    assert search.INIT["FB_MIN"] == (1.0, 10.0, 1000.0)
    assert search.SIZES == (2, 4, 8, 16, 32, 64, 128, 256, 512, 1024, 2048)
    assert set(search.EXPERIMENTS) == set(search.INIT)


def test_init_params_formula():
    """params = [SF, C ./ std(X, dims=2)] (corrected std, zero std -> FILL), then
    params .+ (5 rand .- 0.999) .* params with ONE uniform vector per trial."""
    X = np.array([[1.0, 2.0, 4.0], [3.0, 3.0, 3.0], [0.0, -1.0, 1.0]])
    u = np.random.default_rng(5).random(4)
    p = search.init_params("P1_MIN", X, np.random.default_rng(5))
    std = np.array([np.std([1.0, 2.0, 4.0], ddof=1), 100.0, 1.0])  # P1_MIN fills a zero std with 100
    base = np.concatenate([[1.1], 10.0 / std])
    np.testing.assert_array_equal(p, base + (5.0 * u - 0.999) * base)
    p2 = search.init_params("CP_MAX", X, np.random.default_rng(5))
    std2 = np.array([std[0], 1000.0, 1.0])
    base2 = np.concatenate([[100.0], 50.0 / std2])
    np.testing.assert_array_equal(p2, base2 + (5.0 * u - 0.999) * base2)


@pytest.mark.parametrize("exp", search.EXPERIMENTS)
def test_local_trials_share_one_draw(exp):
    trs = search.local_trials(exp, 8, [0, 3], 4)
    mech, coords = search.split(exp)
    for tr in trs:
        G = tr["Y"].shape[0]
        assert G == (len(data.VW_INDICES[mech]) if coords == "MAX" else len(data.MIN_COORDS[mech]))
        th = data.theta_from_params(tr["params"])
        np.testing.assert_array_equal(tr["theta"], np.tile(th, (G, 1)))
        assert tr["theta"].shape[1] == tr["X"].shape[0] + 2
        assert np.all(np.isfinite(tr["theta"]))
    assert not np.array_equal(trs[0]["params"], trs[1]["params"])
    again = search.local_trials(exp, 8, [3], 4)[0]  # deterministic per (experiment, N, trial)
    np.testing.assert_array_equal(again["params"], trs[1]["params"])


def test_search_data_are_noise_free():
    """hyperparameter.jl applies no noise: the search's inputs are the simulated states."""
    a = data.make_trial("P2", 16, 4, seed=11, noise=False)
    b = data.make_trial("P2", 16, 4, seed=11, noise=True)
    assert np.max(np.abs(a["X"] - b["X"])) < 1e-2 and not np.array_equal(a["X"], b["X"])
    q = data.make_trial_min("P2", 16, 4, seed=11, noise=False)
    # noise-free P2 rates: qdot at the next step equals qdot at the old step (constant rates)
    np.testing.assert_array_equal(q["Y"][0], q["X"][1])


def test_createconfig_picks_the_smallest_error():
    res = {"params": {"P2_MAX8": {"params": [[1.0, 2.0], [3.0, 4.0], [5.0, 6.0]], "kstep_mse": [0.5, 0.1, 0.1]},
                      "CP_MAX8": {"params": [[1.0], [2.0]], "kstep_mse": [math.inf, 7.0]},
                      "FB_MAX8": {"params": [], "kstep_mse": []}}}
    cfg = search.createconfig(res)
    assert cfg == {"P2_MAX8": [3.0, 4.0], "CP_MAX8": [2.0]}


# ---- GPU -------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def ctx():
    import gprx

    c = gprx.Context(0)
    yield c
    c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("exp", search.EXPERIMENTS)
def test_reduced_search_group_against_oracle(ctx, exp):
    """One (experiment, N) group for 4 trials: the device minimisers' LML against the oracle and the
    per-trial start params recorded."""
    from oracle import gp_oracle as O

    for N in (8, 64):
        r = search.run_search_group(exp, N, range(4), ctx, testsamples=8, simsteps=5, max_evals=15, keep=True)
        trials = r["trials"]
        assert r["params"].shape == (4, trials[0]["X"].shape[0] + 1)
        for t, tr in enumerate(trials):
            np.testing.assert_array_equal(r["params"][t], tr["params"])
        for t in (0, 3):
            if not np.all(r["status"][t] == 0):
                continue
            tr = trials[t]
            for g in range(tr["Y"].shape[0]):
                th = r["theta"][t, g]
                try:
                    f = O.fit(tr["X"], tr["Y"][g], th, None, ctx.dist_mode)
                    f2 = O.fit(tr["X"], tr["Y"][g], th, None, 1 - ctx.dist_mode)
                except O.NotPosDef:
                    # the noise-free search inputs can drive a minimiser to the edge of positive
                    # definiteness, where LAPACK's and the device's pivots fall either side of 0
                    assert math.isfinite(r["mll"][t, g])
                    continue
                tol = max(1e-9 * max(1.0, abs(f["mll"])), 10 * abs(f["mll"] - f2["mll"]), 10 * f["mll_sens"])
                assert abs(r["mll"][t, g] - f["mll"]) <= tol, (exp, N, t, g, r["mll"][t, g], f["mll"], tol)
        assert np.sum(~r["failed"]) >= 2, (exp, N, r["status"])
        r["rb"].close()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
def test_search_run_gathers_params_final(ctx):
    """gprx.search.run under an initialised (gloo, world 1) group: the params_final checkpoint
    (core.jl:107-109 shape) equals the per-group results; createconfig picks each argmin."""
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        res = search.run(("P2_MAX", "CP_MIN"), (16,), n_trials=4, testsamples=8, simsteps=5, max_evals=10, ctx=ctx)
    finally:
        dist.destroy_process_group()
    e = res["results"]["params"]["P2_MAX16"]
    r = search.run_search_group("P2_MAX", 16, range(4), ctx, 8, 5, 10)
    keep = ~r["failed"]
    assert e["nprocessed"] == 4 and len(e["params"]) == len(e["kstep_mse"]) == int(keep.sum())
    np.testing.assert_array_equal(e["kstep_mse"], r["kstep_mse"][keep])
    np.testing.assert_array_equal(np.array(e["params"]), r["params"][keep])
    best = int(np.argmin(r["kstep_mse"][keep]))
    assert res["config"]["P2_MAX16"] == list(r["params"][keep][best])
    assert set(res["results"]["params"]) == {"P2_MAX16", "CP_MIN16"}
