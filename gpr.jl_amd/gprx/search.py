"""The hyperparameter.jl random-restart search on MI355X: 8 experiments x N in {2..2048} x trials,
trial-sharded over the ranks of a torch.distributed group (examples/hyperparameter.jl:50-60 over
examples/parallel/core.jl:94-112, `parallelsearch`).

Per (experiment, N) the reference runs `parallelsearch(experiment, expand_config(config, ID, N,
datasets))`: `Threads.@threads for jobid in 1:nruns` (core.jl:28), each job one trial of e.g.
experimentP2Max (examples/maximal_coordinates/P2param.jl:10-44):

    stdx = std(xtrain_old, dims=2); stdx[stdx .== 0] .= FILL
    params = [SF, (C ./ stdx)...]                                      one draw per trial,
    params = params .+ (5rand(length(params)) .- 0.999) .* params      shared by all its outputs
    per output: GP(X, y, MeanZero(), SEArd(log.(params[2:end]), log(params[1])))
                optimize!(gp, LBFGS(linesearch=BackTracking(order=2)), Options(time_limit=10.))
    predictdynamics / predictdynamicsmin for the test samples, `simsteps` steps
    return predictedstates, xtest_future, params

and `resultcallback!` (core.jl:101-105) records kstep_mse = simulationerror(...) (Inf when the
prediction is `nothing`) and the trial's raw start params; an experiment that throws is dropped
(core.jl:41-53).  createconfig.jl then keeps the params of the smallest error per ID.

The initial params per experiment (SF, C, FILL), as the eight experiment files write them:
    P1_MAX [100, 10/std] fill 1000  (maximal_coordinates/P1param.jl:23-26)
    P2_MAX [1.1, 50/std] fill 1000  (maximal_coordinates/P2param.jl:24-27)
    CP_MAX [100, 50/std] fill 1000  (maximal_coordinates/CPparam.jl:28-31)
    FB_MAX [1,   10/std] fill 1000  (maximal_coordinates/FBparam.jl:23-26)
    P1_MIN [1.1, 10/std] fill 100   (minimal_coordinates/P1param.jl:22-25)
    P2_MIN [1.1, 50/std] fill 1000  (minimal_coordinates/P2param.jl:22-25)
    CP_MIN [100, 50/std] fill 1000  (minimal_coordinates/CPparam.jl:24-27)
    FB_MIN [1,   10/std] fill 1000  (minimal_coordinates/FBparam.jl:23-26)
std is Julia's corrected (n - 1) standard deviation over the training inputs X (d x N).

Here one rank holds every GP of its trials as ONE device batch (shard.RankBatch via
sweep.run_group: device LBFGS for all of them at once, a fixed evaluation budget per GP in place of
the machine-dependent 10 s cap, then every test rollout in one launch), and the per-trial
(kstep_mse, params) pairs are gathered as raw tensors into the shape of the reference's
params_final checkpoint: {"params": {ID<N>: {nprocessed, params[], kstep_mse[]}}}.  The search
trains on the simulated states without noise (hyperparameter.jl applies none) and its minimal-
coordinate experiments use plain (q, qdot) inputs (predictdynamicsmin without usesin).  Data are
the synthetic generator's (gprx.data; the .jls datasets are absent); the draws are seeded per
(experiment, N, trial) where the reference leaves its RNG unseeded.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import time

import numpy as np

from . import data, shard

EXPERIMENTS = ("P1_MAX", "P2_MAX", "CP_MAX", "FB_MAX", "P1_MIN", "P2_MIN", "CP_MIN", "FB_MIN")  # hyperparameter.jl:51-59
SIZES = (2, 4, 8, 16, 32, 64, 128, 256, 512, 1024, 2048)  # hyperparameter.jl:50
# (sigma_f, length-scale numerator, fill for a zero std) per experiment (see the module docstring)
INIT = {"P1_MAX": (100.0, 10.0, 1000.0), "P2_MAX": (1.1, 50.0, 1000.0), "CP_MAX": (100.0, 50.0, 1000.0),
        "FB_MAX": (1.0, 10.0, 1000.0), "P1_MIN": (1.1, 10.0, 100.0), "P2_MIN": (1.1, 50.0, 1000.0),
        "CP_MIN": (100.0, 50.0, 1000.0), "FB_MIN": (1.0, 10.0, 1000.0)}
_EXP_ID = {e: i for i, e in enumerate(EXPERIMENTS)}


def split(exp: str) -> tuple[str, str]:
    mech, coords = exp.split("_")
    return mech, coords


def draw_rng(exp: str, N: int, trial: int):
    """The generator of a trial's random start (the reference's `rand` is unseeded)."""
    return np.random.default_rng([7, _EXP_ID[exp], N, trial])


def init_params(exp: str, X: np.ndarray, rng) -> np.ndarray:
    """The trial's random start in raw form [sigma_f, ell_1..ell_d] (e.g. P2param.jl:24-27):
    params = [SF, C ./ std(X, dims=2)] with std == 0 -> FILL, then params .+ (5 rand - 0.999) .* params."""
    sf, c, fill = INIT[exp]
    X = np.asarray(X, dtype=np.float64)
    stdx = X.std(axis=1, ddof=1)  # Julia std: corrected
    stdx[stdx == 0] = fill
    p = np.concatenate([[sf], c / stdx])
    return p + (5.0 * rng.random(p.shape[0]) - 0.999) * p


def local_trials(exp: str, N: int, trial_ids, testsamples: int) -> list[dict]:
    """The rank's trials of one (experiment, N): noise-free inputs, one random start per trial
    shared by its outputs (theta = SEArd(log.(p[2:end]), log(p[1])), logNoise -2)."""
    mech, coords = split(exp)
    out = []
    for t in trial_ids:
        seed = data.trial_seed(mech, t)
        if coords == "MAX":
            tr = data.make_trial(mech, N, testsamples, seed=seed, noise=False)
            d = dict(X=tr["X"], Y=tr["Y"], Xs=tr["Xs"])
        else:
            tr = data.make_trial_min(mech, N, testsamples, seed=seed, usesin=False, noise=False)
            d = dict(X=tr["X"], Y=tr["Y"], Xs=None, start=tr["start"])
        p = init_params(exp, d["X"], draw_rng(exp, N, t))
        d.update(theta=np.tile(data.theta_from_params(p), (d["Y"].shape[0], 1)), params=p, trial=t, seed=seed)
        out.append(d)
    return out


def run_search_group(exp: str, N: int, trial_ids, ctx, testsamples: int = 100, simsteps: int = 20,
                     max_evals: int | None = 30, time_limit: float = float("nan"), keep: bool = False) -> dict:
    """One (experiment, N) of parallelsearch for this rank's trials (sweep.run_group on the
    search's inputs).  Adds the per-trial raw start params (n_local, d+1)."""
    from .sweep import run_group

    mech, coords = split(exp)
    trials = local_trials(exp, N, trial_ids, testsamples)
    if not trials:
        return {}
    r = run_group(mech, N, "max" if coords == "MAX" else "min", [t["trial"] for t in trials], ctx, testsamples,
                  simsteps, max_evals, time_limit, keep=keep, trials=trials)
    r["params"] = np.stack([t["params"] for t in trials])
    return r


def createconfig(results: dict) -> dict:
    """examples/utils/createconfig.jl:8-16: per ID the params of the smallest kstep_mse (entries
    whose error is `nothing` skipped; Julia's argmin: first minimum, NaN counts as largest here
    because simulationerror maps NaN to Inf)."""
    cfg = {}
    for key, e in results.get("params", {}).items():
        errs = [(v, i) for i, v in enumerate(e["kstep_mse"]) if v is not None]
        if not errs:
            continue
        best = min(errs, key=lambda vi: (math.isnan(vi[0]), vi[0], vi[1]))[1]
        cfg[key] = list(e["params"][best])
    return cfg


def _dist():
    import torch.distributed as dist

    return dist if dist.is_available() and dist.is_initialized() else None


def run(experiments=EXPERIMENTS, sizes=SIZES, n_trials: int = 100, testsamples: int = 100, simsteps: int = 20,
        max_evals: int | None = 30, time_limit: float = float("nan"), ctx=None, log=None) -> dict:
    """hyperparameter.jl's loop (N outer, experiments inner).  Every rank runs its trials of every
    group; rank 0 returns the gathered params_final checkpoint (other ranks None).  Without an
    initialised process group: one rank."""
    from .batch import Context

    dist = _dist()
    rank, world = (dist.get_rank(), dist.get_world_size()) if dist else (0, 1)
    if ctx is None:
        import torch

        ctx = Context(torch.cuda.current_device())
    mine = shard.shard_trials(n_trials, rank, world)
    results: dict = {"params": {}}
    timing: dict = {}
    for N in sizes:
        for exp in experiments:
            mech, coords = split(exp)
            d = 13 * data.NBODIES[mech] if coords == "MAX" else 2 * len(data.MIN_COORDS[mech])
            r = run_search_group(exp, N, mine, ctx, testsamples, simsteps, max_evals, time_limit)
            n = len(mine)
            nb = int(r.get("batches", 1 if r else 0))
            local = {"kstep_mse": r.get("kstep_mse", np.zeros(0)),
                     "failed": r.get("failed", np.zeros(0, dtype=bool)).astype(np.float64),
                     "params": r.get("params", np.zeros((0, d + 1))),
                     "t": np.full(n, r.get("t_opt", 0.0) + r.get("t_eval", 0.0))}
            width = {"params": d + 1}
            local = {k: np.asarray(v, dtype=np.float64).reshape(n, width.get(k, 1)) for k, v in local.items()}
            if dist:
                g = shard.gather_results(local, n_trials, lambda q: shard.shard_trials(n_trials, q, world), 0,
                                         keys=("kstep_mse", "failed", "params", "t"))
            else:
                g = local
            key = f"{exp}{N}"
            if rank == 0:
                keep = g["failed"][:, 0] == 0  # a trial whose experiment throws is dropped (core.jl:41-53)
                results["params"][key] = {"nprocessed": n_trials,
                                          "params": [[float(x) for x in row] for row in g["params"][keep]],
                                          "kstep_mse": [float(v) for v in g["kstep_mse"][keep, 0]],
                                          "dropped": int((~keep).sum())}
                timing[key] = {"seconds_max_rank": float(np.max(g["t"][:, 0])) if n_trials else 0.0,
                               "device_batches_rank0": nb,
                               "gp_fits": n_trials * (len(data.VW_INDICES[mech]) if coords == "MAX"
                                                      else len(data.MIN_COORDS[mech]))}
                if log:
                    e = results["params"][key]
                    fin = [v for v in e["kstep_mse"] if math.isfinite(v)]
                    log(f"{key}: {len(e['kstep_mse'])}/{n_trials} kept, best kstep_mse "
                        f"{min(fin) if fin else math.inf:.4g}, {timing[key]['seconds_max_rank']:.3f} s")
    if rank != 0:
        return None
    return {"results": results, "config": createconfig(results), "timing": timing, "world": world,
            "n_trials": n_trials, "max_evals": max_evals, "time_limit": time_limit, "testsamples": testsamples,
            "simsteps": simsteps}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--experiments", default=",".join(EXPERIMENTS))
    ap.add_argument("--sizes", default=",".join(map(str, SIZES)))
    ap.add_argument("--trials", type=int, default=100)
    ap.add_argument("--testsamples", type=int, default=100)
    ap.add_argument("--simsteps", type=int, default=20)
    ap.add_argument("--max-evals", type=int, default=30, help="evaluation budget per GP (<= 0: none)")
    ap.add_argument("--time-limit", type=float, default=float("nan"), help="seconds per group call (NaN: none)")
    ap.add_argument("--out", default="gpurun_out/params_final_checkpoint.json")
    ap.add_argument("--rehearse", action="store_true", help="allow ranks to share GPUs (gloo control plane)")
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks, one per GPU; without a launcher N > 1 starts them itself (as bench.py does)")
    a = ap.parse_args(argv)
    if a.gpus is not None:
        if "WORLD_SIZE" not in os.environ and a.gpus > 1:  # parent: no GPU call has been made
            import sys

            raise SystemExit(shard.launch_ranks(shard.entry_script("search"), a.gpus, a.rehearse,
                                                sys.argv[1:] if argv is None else list(argv), "search"))
        shard.check_world(a.gpus, "search")
    world = shard.init_ranks(a.rehearse)
    t0 = time.perf_counter()
    res = run([e for e in a.experiments.split(",") if e], [int(s) for s in a.sizes.split(",") if s], a.trials,
              a.testsamples, a.simsteps, a.max_evals if a.max_evals > 0 else None, a.time_limit,
              log=lambda s: print(s, flush=True))
    wall = time.perf_counter() - t0
    if res is not None:
        res["wall_seconds"] = wall
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f)
        fits = sum(v["gp_fits"] for v in res["timing"].values())
        print(json.dumps({"search_wall_s": round(wall, 3), "groups": len(res["timing"]), "gp_optimisations": fits,
                          "world": res["world"], "out": a.out}), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
