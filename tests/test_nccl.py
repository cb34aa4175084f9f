"""The RCCL path of the sharding module on the MI355X: a world-size-1 `nccl` process group (RCCL
over the device, the backend bench.py and the sweep use with one rank per GPU), with
gather_rows / broadcast_trial on device tensors and run_trials_sharded / run_trial_split driving
the product evaluator (shard.gpu_evaluator: one RankBatch on the rank's GPU), checked bit for bit
against the same evaluations made without a process group.  The reference's unit is the trial
loop of examples/parallel/core.jl:27-67 (Threads.@threads over job ids)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from gprx import data, shard

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _trial(t):
    th0 = data.theta0("P2", 256)
    tr = data.make_trial("P2", 48, 4, seed=300 + t)
    rng = np.random.default_rng(t)
    return dict(X=tr["X"], Y=tr["Y"], theta=th0 + 0.05 * rng.standard_normal((6, th0.shape[0])), Xs=tr["Xs"])


@pytest.mark.gpu
def test_nccl_world1_collectives_and_rank_batch():
    import torch
    import torch.distributed as dist

    import gprx

    torch.cuda.set_device(0)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    ctx = gprx.Context(0)
    try:
        assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
        # raw fp64 rows through RCCL all_gather on device tensors; integers travel exactly
        a = np.random.default_rng(0).standard_normal((3, 5, 2))
        (got,) = shard.gather_rows(a, [3])
        np.testing.assert_array_equal(got, a)
        big = np.array([[2**52 + 1], [-7], [0]], dtype=np.int64)
        (gi,) = shard.gather_rows(big.astype(np.float64), [3])
        np.testing.assert_array_equal(gi.astype(np.int64), big)
        # broadcast of one trial's arrays (device tensors)
        tr = _trial(0)
        X, Y, th, Xs = shard.broadcast_trial(tr["X"], tr["Y"], tr["theta"], tr["Xs"])
        for u, v in ((X, tr["X"]), (Y, tr["Y"]), (th, tr["theta"]), (Xs, tr["Xs"])):
            np.testing.assert_array_equal(u, v)
        # trials sharded over the (one) rank, evaluated as one RankBatch, gathered over RCCL
        n = 3
        res = shard.run_trials_sharded(n, _trial, shard.gpu_evaluator(ctx=ctx))
        rb = shard.RankBatch([_trial(t) for t in range(n)], ctx=ctx)
        ref = rb.evaluate(np.stack([_trial(t)["theta"] for t in range(n)]))
        rb.close()
        for k in ("mll", "grad", "mu", "var", "status", "info"):
            np.testing.assert_array_equal(res[k], ref[k])
        assert res["status"].dtype == np.int32 and np.all(res["status"] == 0)
        # one trial's outputs split over the ranks (broadcast + gather)
        split = shard.run_trial_split(_trial(1), shard.gpu_evaluator(ctx=ctx))
        rb1 = shard.RankBatch([_trial(1)], ctx=ctx)
        ref1 = rb1.evaluate(_trial(1)["theta"][None])
        rb1.close()
        for k in ("mll", "grad", "mu", "var", "status"):
            np.testing.assert_array_equal(split[k], ref1[k][0])
    finally:
        ctx.close()
        dist.destroy_process_group()


def test_bench_refuses_more_ranks_than_gpus():
    """`bench.py --gpus N` with fewer visible GPUs than N exits non-zero with a message instead of
    silently timing one rank (it launches the ranks itself when there are enough GPUs)."""
    import torch

    if torch.cuda.device_count() >= 2:
        pytest.skip("enough GPUs here: the launch would succeed")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--no-cpu", "--no-opt"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 2, (p.returncode, p.stderr[-2000:])
    assert "needs 2 visible GPUs" in p.stderr
    assert p.stdout.strip() == ""  # no JSON line
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2"], capture_output=True,
                       text=True, timeout=300, env=dict(env, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"))
    assert p.returncode == 2 and "WORLD_SIZE=1" in p.stderr


@pytest.mark.parametrize("script", ["sweep.py", "search.py"])
def test_drivers_refuse_more_ranks_than_gpus(script):
    """sweep.py and search.py start their ranks as bench.py does (shard.launch_ranks): `--gpus N`
    with fewer visible GPUs than N exits 2 with a message, and a --gpus that disagrees with the
    launcher's WORLD_SIZE exits 2 before any work."""
    import torch

    if torch.cuda.device_count() >= 2:
        pytest.skip("enough GPUs here: the launch would succeed")
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(REPO, script), "--gpus", "2", "--trials", "1"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 2, (p.returncode, p.stderr[-2000:])
    assert "needs 2 visible GPUs" in p.stderr
    p = subprocess.run([sys.executable, os.path.join(REPO, script), "--gpus", "2", "--trials", "1"], capture_output=True,
                       text=True, timeout=300, env=dict(env, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"))
    assert p.returncode == 2 and "WORLD_SIZE=1" in p.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("entry", ["module", "script"])
def test_sweep_self_launch_two_ranks_equals_one_rank(tmp_path, entry):
    """The launch path itself, not only its refusals: `python -m gprx.sweep --gpus 2 --rehearse`
    (and `python sweep.py ...`) starts two ranks through shard.launch_ranks (the repo-root wrapper
    on every rank, a c10d rendezvous on a free 127.0.0.1 port), the ranks share the one card over a
    gloo control plane, and the gathered checkpoint equals the one-rank run's."""
    args = ["--mechs", "P2", "--sizes", "8", "--variants", "min,max", "--trials", "4", "--testsamples", "3",
            "--simsteps", "3", "--max-evals", "6"]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    one, two = tmp_path / "one.json", tmp_path / "two.json"
    p = subprocess.run([sys.executable, os.path.join(REPO, "sweep.py"), *args, "--out", str(one)], capture_output=True,
                       text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    if entry == "module":
        cmd, cwd = [sys.executable, "-m", "gprx.sweep"], os.path.join(REPO, "gpr.jl_amd")
    else:
        cmd, cwd = [sys.executable, os.path.join(REPO, "sweep.py")], REPO
    p = subprocess.run([*cmd, *args, "--gpus", "2", "--rehearse", "--out", str(two)], capture_output=True, text=True,
                       timeout=300, env=env, cwd=cwd)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-4000:]
    import json

    a, b = json.loads(one.read_text()), json.loads(two.read_text())
    assert b["world"] == 2 and a["world"] == 1
    assert a["results"] == b["results"]
