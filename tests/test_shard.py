"""Multi-process sharding host logic on CPU: world_size 2 with the gloo backend, the oracle as
injected per-rank evaluator (the product evaluator is gprx.shard.gpu_evaluator)."""
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


def _oracle_eval(X, Y, theta, Xs=None):
    from oracle import gp_oracle as O

    Y = np.atleast_2d(Y)
    out = {k: [] for k in ("mll", "grad", "mu", "var")}
    for g in range(Y.shape[0]):
        f = O.fit(X, Y[g], theta[g], Xs)
        for k in out:
            out[k].append(f[k])
    r = {k: np.array(v) for k, v in out.items()}
    r["status"] = np.zeros(Y.shape[0], dtype=np.int32)
    return r


def _trials():
    th0 = data.theta0("P2", 256)
    out = []
    for t in range(3):
        tr = data.make_trial("P2", 48, 4, seed=100 + t)
        out.append(dict(X=tr["X"], Y=tr["Y"], theta=np.tile(th0, (6, 1)), Xs=tr["Xs"]))
    return out


def _worker(rank, world, port, q):
    import sys, pathlib

    repo = pathlib.Path(__file__).resolve().parents[1]
    sys.path[:0] = [str(repo), str(repo / "gpr.jl_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        trials = _trials()
        res = shard.run_trials_sharded(trials, _oracle_eval)
        split = shard.run_trial_split(trials[0] if rank == 0 else None, _oracle_eval)
        if rank == 0:
            q.put((res, split))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_gloo_world2_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res, split = q.get(timeout=120)
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    trials = _trials()
    for t, tr in enumerate(trials):
        ref = _oracle_eval(tr["X"], tr["Y"], tr["theta"], tr["Xs"])
        np.testing.assert_array_equal(res["mll"][t], ref["mll"])
        np.testing.assert_array_equal(res["mu"][t], ref["mu"])
    ref0 = _oracle_eval(trials[0]["X"], trials[0]["Y"], trials[0]["theta"], trials[0]["Xs"])
    np.testing.assert_array_equal(split["mll"], ref0["mll"])
    np.testing.assert_array_equal(split["grad"], ref0["grad"])
