"""Multi-process sharding host logic on CPU: gloo process groups of world size 2 and 3, the oracle
as the injected per-rank evaluator (the product evaluator is gprx.shard.RankBatch: one GPBatch per
rank over all its trials x outputs, exercised on the GPU in tests/test_sweep.py)."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from gprx import data, shard


def test_round_robin_covers_every_unit_once():
    for world in (1, 2, 3, 8):
        got = sorted(t for r in range(world) for t in shard.shard_trials(100, r, world))
        assert got == list(range(100))
        got = sorted(k for r in range(world) for k in shard.shard_outputs(6, r, world))
        assert got == list(range(6))


def _oracle_eval(trials):
    """Batch evaluator contract: list of local trials -> dict of (n_local, G, ...) arrays."""
    from oracle import gp_oracle as O

    out = {k: [] for k in ("mll", "grad", "mu", "var")}
    for tr in trials:
        Y = np.atleast_2d(tr["Y"])
        rows = {k: [] for k in out}
        for g in range(Y.shape[0]):
            f = O.fit(tr["X"], Y[g], tr["theta"][g], tr["Xs"])
            for k in out:
                rows[k].append(f[k])
        for k in out:
            out[k].append(np.array(rows[k]))
    r = {k: np.stack(v) for k, v in out.items()}
    r["status"] = np.zeros(r["mll"].shape, dtype=np.int32)
    return r


def _trial(t):
    th0 = data.theta0("P2", 256)
    tr = data.make_trial("P2", 48, 4, seed=100 + t)
    return dict(X=tr["X"], Y=tr["Y"], theta=np.tile(th0, (6, 1)), Xs=tr["Xs"])


def _worker(rank, world, port, n_trials, q):
    import sys, pathlib

    repo = pathlib.Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(repo), str(repo / "gpr.jl_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = shard.run_trials_sharded(n_trials, _trial, _oracle_eval)
        allres = shard.run_trials_sharded(n_trials, _trial, _oracle_eval, dst=None)
        split = shard.run_trial_split(_trial(0) if rank == 0 else None, _oracle_eval)
        q.put((rank, res, split, allres))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, n_trials):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_trials, q)) for r in range(world)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(world):
        rank, res, split, allres = q.get(timeout=180)
        got[rank] = (res, split, allres)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    return got


def _check(got, world, n_trials):
    res, split, _ = got[0]
    for r in range(1, world):
        assert got[r][0] is None and got[r][1] is None  # gathered on rank 0 only
    for t in range(n_trials):
        tr = _trial(t)
        ref = _oracle_eval([tr])
        for k in ("mll", "grad", "mu", "var"):
            np.testing.assert_array_equal(res[k][t], ref[k][0])
        assert res["status"].dtype == np.int32 and np.all(res["status"] == 0)
    for r in range(world):  # dst=None: every rank holds the assembled results
        np.testing.assert_array_equal(got[r][2]["mll"], res["mll"])
    ref0 = _oracle_eval([_trial(0)])
    np.testing.assert_array_equal(split["mll"], ref0["mll"][0])
    np.testing.assert_array_equal(split["grad"], ref0["grad"][0])


def test_gloo_world2_matches_single_process():
    got = _run(2, 3)
    _check(got, 2, 3)


def test_gloo_world3_with_an_idle_rank():
    """Fewer trials than ranks: rank 2 owns nothing and still takes part in every gather."""
    got = _run(3, 2)
    _check(got, 3, 2)


def test_plan_chunks_budget_balance_and_geometry_padding():
    """Device-batch chunking (shard.plan_chunks): one batch when the group fits; otherwise balanced
    chunks under the budget, each padded to the 32-slot launch-geometry threshold when the whole
    group is above it (so chunked results equal the single batch's bit for bit)."""
    from gprx.shard import plan_chunks

    slot, fixed = 1000, 50
    assert plan_chunks(10, 6, slot, fixed, 10 * 6 * slot + fixed) == [(0, 10, 10)]
    assert plan_chunks(0, 6, slot, fixed, 1) == []
    p = plan_chunks(10, 6, slot, fixed, 6 * 6 * slot + fixed)  # 6 trials per batch fit -> 2 chunks of 5
    assert p == [(0, 5, 6), (5, 10, 6)]  # 5 trials x 6 = 30 slots < 32: padded to 6 trials (36 slots)
    p = plan_chunks(20, 6, slot, fixed, 7 * 6 * slot + fixed)  # 7 fit -> 3 chunks 7/7/6
    assert p == [(0, 7, 7), (7, 14, 7), (14, 20, 6)]
    assert all(nd * 6 >= 32 for _, _, nd in p)
    # padding never exceeds the budget: 6 trials x 6 outputs must fit, else MemoryError
    with pytest.raises(MemoryError):
        plan_chunks(10, 6, slot, fixed, 5 * 6 * slot + fixed)
    # FB-like: 100 trials x 12 outputs, 671 MB per slot, 250 GB budget -> 31 trials per batch fit
    p = plan_chunks(100, 12, 671_000_000, 10_000, 250_000_000_000)
    assert [h - l for l, h, _ in p] == [25, 25, 25, 25]
    assert all(nd == h - l for l, h, nd in p)
    assert p[0][0] == 0 and p[-1][1] == 100 and all(p[i][1] == p[i + 1][0] for i in range(len(p) - 1))
    # a group under 32 slots is never padded (it already runs the small-batch geometry)
    p = plan_chunks(5, 3, slot, fixed, 2 * 3 * slot + fixed)
    assert [nd for _, _, nd in p] == [2, 2, 1] and [h - l for l, h, _ in p] == [2, 2, 1]
