"""Multi-GPU sharding of the embarrassingly parallel GP work.

The reference parallelises only over experiment trials with host threads
(`Threads.@threads for jobid in ...`, examples/parallel/core.jl:28); inside a trial the G
per-output GPs share X but are independent (examples/maximal_coordinates/CPnoise.jl:37-43).
Here one process drives one GPU (torch.distributed; backend "nccl" = RCCL over xGMI on ROCm,
"gloo" for the CPU tests) and the unit of work is a (trial, output) pair:

  * trial-major round robin: whole trials go to ranks (`shard_trials`), and each rank evaluates
    ALL of its trials x G outputs as ONE device batch (`RankBatch`: B = local trials x G slots,
    built once, reused for every evaluation and optimiser round) -- the batching the bench
    measures, instead of one small launch sequence per trial.  A rank whose group does not fit
    the card (FB N=4096: 671 MB per slot) runs it as a few such batches one after another, sized
    from the free HBM (`group_plan`), with results bit-identical to one batch;
  * no data moves between GPUs during a fit; trial inputs are generated (or loaded) on the rank
    that owns them;
  * when a single trial must be spread (G outputs over several GPUs, e.g. one P2 trial on 8
    GPUs), the owning rank broadcasts X, Y, theta once (`broadcast_trial`, <= 1.7 MB) and every
    rank evaluates its outputs k = rank (mod world) (`run_trial_split`);
  * results (mll, gradient, theta*, predictive mean / variance, status: a few KB per trial) are
    gathered as raw fp64 tensors with one all_gather per array (`gather_rows`), over RCCL when
    the group is nccl.

There is no all-reduce on the data path.  The per-rank evaluator is injected
(`evaluate(local_trials) -> dict of (n_local, G, ...) arrays`), so the host logic is testable on
CPU with gloo and the oracle; the product evaluator is `RankBatch` (one GPBatch on the rank's
MI355X).
"""
from __future__ import annotations

from typing import Callable, Sequence

import numpy as np


def init_ranks(rehearse: bool = False) -> int:
    """One process per GPU under torch.distributed.run: bind this rank to GPU LOCAL_RANK and, for a
    world size > 1, join the RCCL (`nccl`) group.  More ranks than visible GPUs is an error unless
    `rehearse` (ranks then share devices over a gloo group: a rehearsal, never a measurement).
    Returns the world size."""
    import os

    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    if ndev < 1 or (world > ndev and not rehearse):
        raise SystemExit(f"gprx: {world} rank(s) need {world} GPUs, {ndev} visible (rehearse=True shares devices)")
    torch.cuda.set_device(local % ndev)
    if world > 1:
        backend = "gloo" if rehearse else "nccl"
        _dist().init_process_group(backend)
        assert _dist().get_backend() == backend and _dist().get_world_size() == world
    return world


def entry_script(name: str) -> str:
    """The repo-root wrapper (sweep.py, search.py) that a self-launch starts on every rank, whatever
    way this process was started (`python sweep.py`, `python -m gprx.sweep`, main() from code):
    sys.argv[0] names the package module under -m, which cannot run as a plain script."""
    import pathlib

    return str(pathlib.Path(__file__).resolve().parents[2] / f"{name}.py")


def launch_cmd(script: str, gpus: int, argv: list[str]) -> list[str]:
    """torch.distributed.run for one node, N ranks: a c10d rendezvous that binds its own free port
    on 127.0.0.1 (--standalone; no probe-then-reuse race on a port number)."""
    import sys

    return [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1", "--nnodes=1",
            f"--nproc-per-node={gpus}", script, *argv]


def launch_ranks(script: str, gpus: int, rehearse: bool, argv: list[str], tag: str = "gprx") -> int:
    """`<script> --gpus N` (N > 1) started without a launcher: start N ranks, one per GPU, as a
    torch.distributed.run child running `script` with `argv`, and return its exit code.  Call
    before this process touches a GPU (device_count() does not initialise one on this image).
    Fewer visible GPUs than N is an error (exit 2), not a silent one-rank run; `rehearse` lets
    ranks share devices.  sweep.py and search.py start their ranks through this; bench.py keeps a
    copy of it (_launch_ranks, same command line) so that its parent never imports the library."""
    import subprocess
    import sys

    import torch

    ndev = torch.cuda.device_count()
    if ndev < gpus and not rehearse:
        print(f"{tag}: --gpus {gpus} needs {gpus} visible GPUs, this host has {ndev} "
              f"(--rehearse runs the ranks on shared devices, for a rehearsal only)", file=sys.stderr)
        return 2
    cmd = launch_cmd(script, gpus, argv)
    print(f"{tag}: launching {gpus} ranks: {' '.join(cmd[1:8])} ...", file=sys.stderr, flush=True)
    return subprocess.run(cmd).returncode


def check_world(gpus: int, tag: str = "gprx") -> None:
    """Under a launcher, `--gpus N` must equal WORLD_SIZE (exit 2 otherwise)."""
    import os
    import sys

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != gpus:
        print(f"{tag}: --gpus {gpus} but WORLD_SIZE={world}: launch one rank per GPU "
              f"(--gpus N without a launcher starts them itself)", file=sys.stderr)
        raise SystemExit(2)


def shard_trials(n_trials: int, rank: int, world: int) -> list[int]:
    """Trial-major round robin (the mapping core.jl's threads get, by jobid mod ngpu)."""
    return list(range(rank, n_trials, world))


def shard_outputs(G: int, rank: int, world: int) -> list[int]:
    return list(range(rank, G, world))


def _dist():
    import torch.distributed as dist

    return dist


def _device(dev=None):
    dist = _dist()
    if dev is not None:
        return dev
    return "cuda" if dist.get_backend() == "nccl" else "cpu"


# ---- device-batch sizing: a rank's trials in batches that fit the card -----------------------
# gprx_api.hip set_geometry: the recursion's leaf size and GEMM units switch at 32 slots, so a
# batch under 32 slots rounds differently from one above.  Chunks of a group whose whole batch has
# >= 32 slots are therefore padded to 32 (copies of their last trial, results discarded): every
# chunk then runs the launch geometry the single batch would, and the results are bit-identical.
GEOMETRY_SLOTS = 32


def batch_bytes(B: int, d: int, N: int, M: int) -> int:
    """Device bytes of GPBatch(B, d, N, M) (gprx_batch_bytes: host arithmetic, no GPU)."""
    import ctypes as C

    from . import _lib as L

    out = C.c_uint64()
    rc = L.lib.gprx_batch_bytes(int(B), int(d), int(N), int(M), C.byref(out))
    if rc != L.OK:
        raise L.GPRXError(rc, f"batch sizes B={B} d={d} N={N} M={M}")
    return int(out.value)


def default_budget(ctx) -> int:
    """Device bytes a rank's batch may take: 90% of the free HBM less 1 GiB (the optimiser's
    workspace, the rollouts' buffers and torch's own allocations come on top)."""
    import ctypes as C

    from . import _lib as L

    free, total = C.c_uint64(), C.c_uint64()
    L.check(L.lib.gprx_ctx_mem_info(ctx.h, C.byref(free), C.byref(total)), ctx.h)
    return max(int(0.9 * free.value) - (1 << 30), 0)


def plan_chunks(n_trials: int, G: int, slot_bytes: int, fixed_bytes: int, budget: int,
                geometry_slots: int = GEOMETRY_SLOTS) -> list[tuple[int, int, int]]:
    """Split n_trials trials of G slots into device batches of at most `budget` bytes
    (slot_bytes per slot + fixed_bytes per batch).  Returns [(lo, hi, dev_trials)]: trials
    [lo, hi) in one batch of dev_trials >= hi - lo trials (padding up to the 32-slot geometry
    threshold when the whole group has >= 32 slots, so that chunked and single-batch results are
    bit-identical).  Chunks are balanced (sizes differ by at most one trial).  A budget that cannot
    hold one padded chunk raises MemoryError (the allocation would fail with GPRX_OUT_OF_MEMORY)."""
    if n_trials <= 0:
        return []
    per_trial = slot_bytes * G
    if fixed_bytes + n_trials * per_trial <= budget:
        return [(0, n_trials, n_trials)]
    pad = -(-geometry_slots // G) if n_trials * G >= geometry_slots else 1  # trials per chunk at least
    fit = (budget - fixed_bytes) // per_trial if budget > fixed_bytes else 0
    if fit < max(pad, 1):
        raise MemoryError(f"gprx: a device batch of {max(pad, 1)} trial(s) x {G} outputs needs "
                          f"{fixed_bytes + max(pad, 1) * per_trial} bytes, budget {budget}")
    nch = -(-n_trials // fit)
    base, extra = divmod(n_trials, nch)
    out, lo = [], 0
    for c in range(nch):
        hi = lo + base + (1 if c < extra else 0)
        out.append((lo, hi, max(hi - lo, pad)))
        lo = hi
    return out


def group_plan(trials: Sequence[dict], ctx=None, budget: int | None = None) -> list[tuple[int, int, int]]:
    """plan_chunks for a rank's trials (budget None: default_budget(ctx))."""
    if not trials:
        return []
    d, N = np.asarray(trials[0]["X"]).shape
    G = np.atleast_2d(trials[0]["Y"]).shape[0]
    xs0 = trials[0].get("Xs")
    M = 0 if xs0 is None else np.asarray(xs0).shape[1]
    one, two = batch_bytes(1, d, N, M), batch_bytes(2, d, N, M)
    if budget is None:
        budget = default_budget(ctx)
    return plan_chunks(len(trials), G, two - one, 2 * one - two, budget)


# ---- the product evaluator: one device batch per rank ----------------------------------------
class RankBatch:
    """A rank's trials x G outputs as one GPBatch (B = n_local * G slots, slot t*G + g = local
    trial t, output g), built once and reused.  Each trial's X / Xs is the slot's own input
    (trials differ), the G outputs of a trial share it.

    trials: list of dicts X (d, N), Y (G, N) (targets minus prior mean), Xs (d, M) or None.
    dev_trials > len(trials): the device batch holds that many trials, the extra ones copies of
    the last (a chunk padded to the group's launch geometry, plan_chunks); they are evaluated and
    their results dropped.  A group larger than the card runs as several RankBatches one after
    another (group_plan; gprx.sweep.run_group, gpu_evaluator)."""

    def __init__(self, trials: Sequence[dict], ctx=None, device: int | None = None, dev_trials: int | None = None):
        from .batch import Context, GPBatch

        if ctx is None:
            import torch

            ctx = Context(torch.cuda.current_device() if device is None else device)
        self.ctx = ctx
        self.n = len(trials)
        if self.n == 0:
            self.batch = None
            return
        self.n_dev = max(self.n, dev_trials or 0)
        dev = list(trials) + [trials[-1]] * (self.n_dev - self.n)
        X0 = np.asarray(trials[0]["X"])
        self.d, self.N = X0.shape
        self.G = np.atleast_2d(trials[0]["Y"]).shape[0]
        xs0 = trials[0].get("Xs")
        self.M = 0 if xs0 is None else np.asarray(xs0).shape[1]
        B = self.n_dev * self.G
        self.batch = GPBatch(B, self.d, self.N, self.M, ctx=ctx)
        X = np.repeat(np.stack([np.asarray(t["X"], dtype=np.float64) for t in dev]), self.G, axis=0)
        Y = np.concatenate([np.atleast_2d(np.asarray(t["Y"], dtype=np.float64)) for t in dev], axis=0)
        self.batch.set_train(X, Y)
        if self.M:
            Xs = np.repeat(np.stack([np.asarray(t["Xs"], dtype=np.float64) for t in dev]), self.G, axis=0)
            self.batch.set_test(Xs)

    def _shape(self, a):
        """Device rows (n_dev * G, ...) -> (n_local, G, ...), padding rows dropped."""
        if a is None:
            return None
        a = np.asarray(a)
        return a.reshape((self.n_dev, self.G) + a.shape[1:])[: self.n]

    def _rows(self, theta):
        """(n_local, G, d+2) -> (n_dev * G, d+2), the padding trials repeating the last trial's rows."""
        th = np.asarray(theta, dtype=np.float64).reshape(self.n, self.G, -1)
        if self.n_dev > self.n:
            th = np.concatenate([th, np.repeat(th[-1:], self.n_dev - self.n, axis=0)])
        return th.reshape(self.n_dev * self.G, -1)

    def evaluate(self, theta, grad: bool = True, predict: bool | None = None, variance: bool = True) -> dict:
        """theta (n_local, G, d+2) -> dict of (n_local, G, ...) arrays (mll, grad, mu, var, status,
        info)."""
        if self.batch is None:
            return {}
        pred = self.M > 0 if predict is None else predict
        r = self.batch.run(self._rows(theta), grad=grad, predict=pred, variance=variance)
        return {k: self._shape(v) for k, v in r.items() if v is not None}

    def optimize(self, theta0, method=None, options=None) -> dict:
        """optimize! for every GP of every local trial in one device call (k_lbfgs, lock-step),
        then one evaluation at the minimisers (update_target!, with prediction when the trials
        have test points).  A slot whose refit fails is reported in `status` (the reference's
        experiment throws and the trial is dropped, core.jl:41-46), the others stay valid."""
        if self.batch is None:
            return {}
        th0 = self._rows(theta0)
        res, rounds = self.batch.optimize(th0, method, options, refit=False)
        thmin = np.stack([r.minimizer for r in res])
        ok = np.all(np.isfinite(thmin), axis=1)
        # a non-finite minimiser (NaN-gradient stop) is evaluated at its start and marked failed
        r = self.batch.run(np.where(ok[:, None], thmin, th0), grad=False, predict=self.M > 0, variance=False)
        status = np.where(ok, r["status"], 2).astype(np.int32)
        out = {"theta": thmin, "minimum": np.array([x.minimum for x in res]), "mll": r["mll"], "status": status,
               "f_calls": np.array([x.f_calls for x in res], dtype=np.int32),
               "iterations": np.array([x.iterations for x in res], dtype=np.int32)}
        if r.get("mu") is not None:
            out["mu"] = r["mu"]
        out = {k: self._shape(v) for k, v in out.items()}
        out["rounds"] = rounds
        return out

    def slot(self, t: int, g: int) -> int:
        return t * self.G + g

    def close(self):
        if self.batch is not None:
            self.batch.close()
            self.batch = None


def gpu_evaluator(device: int | None = None, ctx=None, budget: int | None = None):
    """Evaluator for run_trials_sharded on this rank's GPU: the local trials as RankBatches that
    fit the card (group_plan; one batch when they fit), theta taken from each trial dict.  Callers
    that evaluate the same trials repeatedly (an optimiser, a sweep) keep a RankBatch themselves
    and call its evaluate / optimize."""

    def evaluate(trials):
        c = ctx
        if c is None:
            import torch

            from .batch import Context

            c = Context(torch.cuda.current_device() if device is None else device)
        parts = []
        for lo, hi, nd in group_plan(trials, c, budget):
            rb = RankBatch(trials[lo:hi], ctx=c, dev_trials=nd)
            try:
                parts.append(rb.evaluate(np.stack([np.atleast_2d(t["theta"]) for t in trials[lo:hi]])))
            finally:
                rb.close()
        return {k: np.concatenate([p[k] for p in parts]) for k in parts[0]} if parts else {}

    return evaluate


# ---- collectives: raw fp64 tensors ----------------------------------------------------------
def gather_rows(local: np.ndarray, counts: Sequence[int], device=None) -> list[np.ndarray]:
    """All-gather of per-rank row blocks (rank r holds counts[r] rows of equal trailing shape):
    one fixed-size fp64 tensor per rank (padded to max(counts) rows), one all_gather.  Returns the
    list of every rank's rows (on every rank)."""
    import torch

    dist = _dist()
    dev = _device(device)
    world = dist.get_world_size()
    local = np.asarray(local, dtype=np.float64)
    tail = local.shape[1:]
    width = int(np.prod(tail)) if tail else 1
    nmax = max(max(counts), 1)
    buf = torch.zeros((nmax, width), dtype=torch.float64, device=dev)
    if local.shape[0]:
        buf[: local.shape[0]] = torch.from_numpy(np.ascontiguousarray(local.reshape(local.shape[0], width))).to(dev)
    outs = [torch.empty_like(buf) for _ in range(world)]
    dist.all_gather(outs, buf)
    return [o[: counts[r]].cpu().numpy().reshape((counts[r],) + tail) for r, o in enumerate(outs)]


def gather_results(local: dict, n_total: int, index_of_rank: Callable[[int], Sequence[int]], dst: int | None = 0,
                   keys: Sequence[str] = ("mll", "grad", "mu", "var", "status", "info", "theta", "minimum")):
    """Gather per-unit result arrays (first axis = local units, in the order index_of_rank(rank)
    lists them) from every rank into global order.  Every key must be present on every rank with
    the same trailing shape (a rank with no units sends zero rows).  Integer arrays travel as fp64
    (exact).  Returns the assembled dict on dst (on every rank when dst is None), else None."""
    dist = _dist()
    rank, world = dist.get_rank(), dist.get_world_size()
    idx = [list(index_of_rank(r)) for r in range(world)]
    counts = [len(i) for i in idx]
    out: dict = {}
    for k in keys:
        if k not in local:
            continue
        v = np.asarray(local[k])
        parts = gather_rows(v.astype(np.float64), counts)
        full = np.zeros((n_total,) + v.shape[1:], dtype=np.float64)
        for r in range(world):
            if counts[r]:
                full[idx[r]] = parts[r]
        out[k] = full.astype(v.dtype) if np.issubdtype(v.dtype, np.integer) else full
    if dst is not None and rank != dst:
        return None
    return out


def broadcast_trial(X, Y, theta, Xs=None, src: int = 0, device=None):
    """Broadcast one trial's arrays from `src` to every rank (RCCL/gloo broadcast).  Non-src ranks
    pass None and receive the arrays; shapes travel first as a small int tensor."""
    import torch

    dist = _dist()
    rank = dist.get_rank()
    dev = _device(device)
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


def run_trials_sharded(n_trials: int, get_trial: Callable[[int], dict], evaluate: Callable, dst: int | None = 0):
    """Evaluate every (trial, output) unit, trials sharded over ranks; results gathered on dst.

    get_trial(t) -> dict(X (d,N), Y (G,N), theta (G,d+2), Xs (d,M) or None) is called only for the
    rank's own trials (inputs are made or loaded where they are evaluated); evaluate(local_trials)
    -> dict of (n_local, G, ...) arrays (RankBatch / gpu_evaluator on the GPU).  Returns dict of
    arrays shaped (n_trials, G, ...) on dst (every rank when dst is None), None elsewhere."""
    dist = _dist()
    rank, world = dist.get_rank(), dist.get_world_size()
    mine = shard_trials(n_trials, rank, world)
    trials = [get_trial(t) for t in mine]
    local = evaluate(trials) if trials else {}
    local = {k: v for k, v in local.items() if np.ndim(v) >= 2}  # per-unit arrays only
    # ranks without trials (n_trials < world) still take part in every gather: G and the result
    # layout come from rank 0, which always holds trial 0
    G, keys = _agree_keys((np.atleast_2d(trials[0]["Y"]).shape[0], describe(local)) if rank == 0 else None)
    if not trials:
        local = _empty_like_remote(keys, G)
    flat = {k: np.asarray(v).reshape((-1,) + np.asarray(v).shape[2:]) for k, v in local.items()}
    out = gather_results(flat, n_trials * G, lambda r: [t * G + g for t in shard_trials(n_trials, r, world)
                                                         for g in range(G)], dst, keys=[k for k, _, _ in keys])
    if out is None:
        return None
    return {k: v.reshape((n_trials, G) + v.shape[1:]) for k, v in out.items()}


def _agree_keys(meta):
    """Every rank learns rank 0's result layout (object broadcast of a few bytes of metadata; the
    data itself travels as tensors)."""
    dist = _dist()
    obj = [meta]
    dist.broadcast_object_list(obj, src=0)
    return obj[0]


def _empty_like_remote(keys, G):
    return {k: np.zeros((0, G) + tuple(shape), dtype=dt) for k, shape, dt in keys}


def describe(local: dict):
    """(key, trailing shape after (n_local, G), dtype str) per result array."""
    return [(k, tuple(np.asarray(v).shape[2:]), str(np.asarray(v).dtype)) for k, v in sorted(local.items())]


def run_trial_split(trial: dict | None, evaluate: Callable, src: int = 0):
    """One trial whose G outputs are spread over the ranks: src broadcasts X/Y/theta/Xs, rank r
    evaluates outputs k = r (mod world), results are gathered on src.  evaluate([trial]) as for
    run_trials_sharded."""
    dist = _dist()
    rank, world = dist.get_rank(), dist.get_world_size()
    if rank == src:
        X, Y, th, Xs = broadcast_trial(trial["X"], trial["Y"], trial["theta"], trial.get("Xs"), src)
    else:
        X, Y, th, Xs = broadcast_trial(None, None, None, None, src)
    G = Y.shape[0]
    ks = shard_outputs(G, rank, world)
    local = evaluate([dict(X=X, Y=Y[ks], theta=th[ks], Xs=Xs)]) if ks else {}
    local = {k: v for k, v in local.items() if np.ndim(v) >= 2}
    keys = _agree_keys(describe(local) if rank == 0 else None)
    flat = {k: np.asarray(v)[0] for k, v in local.items()} if ks else {k: np.zeros((0,) + tuple(s), dtype=dt)
                                                                        for k, s, dt in keys}
    return gather_results(flat, G, lambda r: shard_outputs(G, r, world), src, keys=[k for k, _, _ in keys])
