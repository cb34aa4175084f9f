"""Multi-GPU sharding of the embarrassingly parallel GP work.

The reference parallelises only over experiment trials with host threads
(`Threads.@threads for jobid in ...`, examples/parallel/core.jl:28); inside a trial the G
per-output GPs share X but are independent (examples/maximal_coordinates/CPnoise.jl:37-43).
Here one process drives one GPU (torch.distributed; backend "nccl" = RCCL over xGMI on ROCm,
"gloo" for the CPU tests) and the unit of work is a (trial, output) pair:

  * trial-major round robin: whole trials go to ranks, so a trial's X is uploaded once per GPU
    and no data moves between GPUs during a fit (`shard_trials`);
  * when a single trial must be spread (G outputs over several GPUs, e.g. one P2 trial on 8
    GPUs), the owning rank broadcasts X, Y, theta once (`broadcast_trial`, ≤ 1.7 MB) and every
    rank evaluates its outputs k ≡ rank (mod world);
  * results (mll, gradient, predictive mean / variance: a few KB) are gathered to rank 0
    (`gather_results`).

There is no all-reduce on the hot path.  The per-rank evaluator is injected (`evaluate(X, Y,
theta, Xs) -> dict`), so the host logic is testable on CPU with gloo; the product evaluator is
`gpu_evaluator()` (GPBatch on the rank's MI355X).
"""
from __future__ import annotations

from typing import Callable, Sequence

import numpy as np


def shard_trials(n_trials: int, rank: int, world: int) -> list[int]:
    """Trial-major round robin (the mapping core.jl's threads get, by jobid mod ngpu)."""
    return list(range(rank, n_trials, world))


def shard_outputs(G: int, rank: int, world: int) -> list[int]:
    return list(range(rank, G, world))


def gpu_evaluator(device: int | None = None, ctx=None):
    """Evaluator running on this rank's GPU: one GPBatch per call (B = number of GPs)."""
    from .batch import GPBatch, Context

    if ctx is None:
        import torch

        ctx = Context(torch.cuda.current_device() if device is None else device)

    def evaluate(X, Y, theta, Xs=None):
        X = np.asarray(X, dtype=np.float64)
        Y = np.atleast_2d(np.asarray(Y, dtype=np.float64))
        theta = np.atleast_2d(np.asarray(theta, dtype=np.float64))
        B = Y.shape[0]
        d, N = X.shape[-2], X.shape[-1]
        M = 0 if Xs is None else np.asarray(Xs).shape[-1]
        b = GPBatch(B, d, N, M, ctx=ctx)
        try:
            b.set_train(X, Y)
            if M:
                b.set_test(Xs)
            return b.run(theta, grad=True, predict=M > 0)
        finally:
            b.close()

    return evaluate


def _dist():
    import torch.distributed as dist

    return dist


def broadcast_trial(X, Y, theta, Xs=None, src: int = 0, device=None):
    """Broadcast one trial's arrays from `src` to every rank (RCCL/gloo broadcast).  Non-src ranks
    pass None and receive the arrays; shapes travel first as a small int tensor."""
    import torch

    dist = _dist()
    rank = dist.get_rank()
    dev = device if device is not None else ("cuda" if dist.get_backend() == "nccl" else "cpu")
    meta = torch.zeros(5, dtype=torch.int64, device=dev)
    if rank == src:
        X = np.asarray(X, dtype=np.float64)
        Y = np.atleast_2d(np.asarray(Y, dtype=np.float64))
        theta = np.atleast_2d(np.asarray(theta, dtype=np.float64))
        meta[:] = torch.tensor([X.shape[0], X.shape[1], Y.shape[0], theta.shape[1],
                                0 if Xs is None else np.asarray(Xs).shape[1]])
    dist.broadcast(meta, src)
    d, N, G, P, M = (int(v) for v in meta.tolist())

    def bc(a, shape):
        t = torch.empty(shape, dtype=torch.float64, device=dev)
        if rank == src:
            t.copy_(torch.from_numpy(np.ascontiguousarray(a)))
        dist.broadcast(t, src)
        return t.cpu().numpy()

    X = bc(X, (d, N))
    Y = bc(Y, (G, N))
    theta = bc(theta, (G, P))
    Xs = bc(Xs, (d, M)) if M else None
    return X, Y, theta, Xs


def gather_results(local: dict, n_total: int, index: Sequence[int], dst: int = 0):
    """Gather per-unit results (mll, grad, mu, var, status) from all ranks into global order on
    `dst`; returns the assembled dict on dst and None elsewhere."""
    dist = _dist()
    world = dist.get_world_size()
    payload = {"index": list(index)}
    for k in ("mll", "grad", "mu", "var", "status", "info"):
        v = local.get(k)
        payload[k] = None if v is None else np.asarray(v)
    objs = [None] * world if dist.get_rank() == dst else None
    dist.gather_object(payload, objs, dst=dst)
    if dist.get_rank() != dst:
        return None
    out: dict = {}
    for p in objs:
        for k, v in p.items():
            if k == "index" or v is None:
                continue
            if k not in out:
                out[k] = np.zeros((n_total,) + v.shape[1:], dtype=v.dtype)
            out[k][p["index"]] = v
    return out


def run_trials_sharded(trials: Sequence[dict], evaluate: Callable, dst: int = 0):
    """Evaluate every (trial, output) unit, trials sharded over ranks; results gathered on dst.

    trials[i] = dict(X (d,N), Y (G,N), theta (G,d+2), Xs (d,M) or None); all with equal G.
    Returns dict of arrays shaped (n_trials, G, ...) on dst, None elsewhere.
    """
    dist = _dist()
    rank, world = dist.get_rank(), dist.get_world_size()
    mine = shard_trials(len(trials), rank, world)
    G = trials[0]["Y"].shape[0]
    local: dict = {}
    index = []
    for t in mine:
        tr = trials[t]
        r = evaluate(tr["X"], tr["Y"], tr["theta"], tr.get("Xs"))
        for k, v in r.items():
            if v is None:
                continue
            local.setdefault(k, []).append(np.asarray(v))
        index.extend(range(t * G, (t + 1) * G))
    local = {k: np.concatenate(v, axis=0) for k, v in local.items()}
    out = gather_results(local, len(trials) * G, index, dst)
    if out is None:
        return None
    return {k: v.reshape((len(trials), G) + v.shape[1:]) for k, v in out.items()}


def run_trial_split(trial: dict | None, evaluate: Callable, src: int = 0):
    """One trial whose G outputs are spread over the ranks: src broadcasts X/Y/theta/Xs, rank r
    evaluates outputs k ≡ r (mod world), results are gathered on src."""
    dist = _dist()
    rank, world = dist.get_rank(), dist.get_world_size()
    if rank == src:
        X, Y, th, Xs = broadcast_trial(trial["X"], trial["Y"], trial["theta"], trial.get("Xs"), src)
    else:
        X, Y, th, Xs = broadcast_trial(None, None, None, None, src)
    ks = shard_outputs(Y.shape[0], rank, world)
    local = evaluate(X, Y[ks], th[ks], Xs) if ks else {}
    return gather_results(local, Y.shape[0], ks, src)
