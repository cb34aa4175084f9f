"""Multi-process sharding host logic on CPU: gloo process groups of world size 2 and 3, the oracle
as the injected per-rank evaluator (the product evaluator is gprx.shard.RankBatch: one GPBatch per
rank over all its trials x outputs, exercised on the GPU in tests/test_sweep.py)."""
import os
import socket

import numpy as np
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
