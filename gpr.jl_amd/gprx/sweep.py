"""The noise.jl sweep on MI355X: {P1, P2, CP, FB} x dataset sizes x trials, trial-sharded over the
ranks of a torch.distributed group (examples/noise.jl:78-116 over examples/parallel/core.jl:27-89).

The reference runs, per (experiment, N), `parallelsim(experiment, expand_config(ID, N, ...))`:
`Threads.@threads for jobid in 1:nruns` (core.jl:28), each job one trial:

    GP(X, y_k, MeanZero(), SEArd(theta0)) ; optimize!(gp, LBFGS(BackTracking(order=2)),
    Options(time_limit=10.)) for every output k     (e.g. P2noise.jl:37-43, P2noise.jl(min):68-71)
    predictdynamics / predictdynamicsmin for the 100 test samples, 20 steps   (:45-51 / :73-76)
    kstep_mse = simulationerror(xtest_future_true, predictions)               (core.jl:75-76)

Here one rank holds its trials' G outputs as ONE device batch (shard.RankBatch: B = local
trials x G), optimises every GP at once with the device LBFGS (k_lbfgs; a fixed evaluation budget
per GP replaces the machine-dependent 10 s cap, or a wall-clock limit for the whole call), and
rolls out every test trajectory of every local trial in one launch (gprx_rollout_min).  Results
are gathered as raw tensors (shard.gather_results) and written in the shape of the reference's
final checkpoint (core.jl:79-82): {etype: {ID<N>: {nprocessed, kstep_mse[], projectionerror[]}}}.

Variants (all of noise.jl:72-85):
    max      maximal coordinates, CState inputs (experiment_*_mz_max): optimise + 20-step device
             predictdynamics (GP means, projectv!, updatestate!: gprx.projection), error =
             simulationerror of the final CStates, projectionerror = the mean projection error
    min      minimal coordinates (experiment_*_mz_min): optimise + 20-step device rollout, error =
             simulationerror of the final CStates (position MSE)
    min_sin  as min with (sin, cos) angle features (experiment_*_mz_min_sin)
    vi       the physics-only baseline (noise.jl:72-75, examples/baseline.jl): the noisy test starts
             simulated by the variational integrator alone (gprx.mdynamics.simulate: the device
             step k_vi_step), no GP
    md_*     the same three with MeanDynamics GPs (experiment_*_md_*): the prior mean is one
             variational-integrator step (device k_vi_step via gprx.mdynamics; host restatement
             gprx.vi), computed once per training
             set for the fit (y - mu(X) on the device) and at every rollout step's states; the
             GP means of a rollout step come from one batched device predict, the projection
             from the device
Data are the synthetic generator's (gprx.data; the .jls datasets are absent), seeded per
(mechanism, trial) as 1000 * config_id + trial (data.trial_seed).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import time

import numpy as np

from . import data, shard
from . import mdynamics
from .rollout import NCOORD, final_cstate, rollout_min

MECHS = ("P1", "P2", "CP", "FB")
SIZES = (2, 4, 8, 16, 32, 64, 128, 256, 512)  # noise.jl:64
VARIANTS = ("vi", "max", "min", "min_sin", "md_max", "md_min", "md_min_sin")  # noise.jl:72-85 order
# parallelsim idmod (noise.jl:80-85): etype = "noisy" * idmod
ETYPE = {"max": "noisy", "min": "noisy", "min_sin": "noisysin", "md_max": "noisyMD", "md_min": "noisyMD",
         "md_min_sin": "noisyMDsin"}
# What each entry's numbers are checked against.  The vi baseline and the md_* variants depend on a
# host restatement of ConstrainedDynamics 0.7.4's variational-integrator step (gprx.vi), which is not
# in the reference tree: its only cross-check is the repo's own action-based oracle/vi_oracle.py
# (same modelling assumptions), so those entries are not reference-equivalent numbers.
PARITY = {"max": "gp: oracle-pinned; physics: projectv! restated (unpinned vs ConstrainedDynamics)",
          "min": "gp: oracle-pinned", "min_sin": "gp: oracle-pinned",
          "vi": "unpinned: gprx.vi restates ConstrainedDynamics 0.7.4 newton! (absent from the reference tree)",
          "md_max": "unpinned: MeanDynamics mean from gprx.vi (ConstrainedDynamics absent)",
          "md_min": "unpinned: MeanDynamics mean from gprx.vi (ConstrainedDynamics absent)",
          "md_min_sin": "unpinned: MeanDynamics mean from gprx.vi (ConstrainedDynamics absent)"}


def _dist():
    import torch.distributed as dist

    return dist if dist.is_available() and dist.is_initialized() else None


def local_trials(mech: str, N: int, variant: str, trial_ids, testsamples: int, ctx=None) -> list[dict]:
    """The trials' GP inputs, built on the rank that owns them (MeanDynamics means on ctx's device)."""
    out = []
    md = variant.startswith("md_")
    base = variant[3:] if md else variant
    for t in trial_ids:
        seed = data.trial_seed(mech, t)
        if base == "max":
            tr = data.make_trial(mech, N, testsamples, seed=seed)
            th = data.theta0(mech, N, "MAX")
            d = dict(X=tr["X"], Y=tr["Y"], Xs=tr["Xs"], theta=np.tile(th, (tr["Y"].shape[0], 1)), trial=t, seed=seed)
            if md:  # MeanDynamics prior mean, once per training set (gprx.mdynamics)
                d["mu"] = mdynamics.mean_max(mech, tr["X"], ctx=ctx)
        else:
            usesin = base == "min_sin"
            tr = data.make_trial_min(mech, N, testsamples, seed=seed, usesin=usesin)
            th = data.theta0_min(mech, N, usesin)
            d = dict(X=tr["X"], Y=tr["Y"], Xs=None, start=tr["start"], theta=np.tile(th, (tr["Y"].shape[0], 1)),
                     trial=t, seed=seed)
            if md:  # the rollout predicts at the test starts' features with the batch's test capacity
                d["mu"] = mdynamics.mean_min(mech, tr["X"], usesin, ctx=ctx)
                d["Xs"] = data.min_features(mech, tr["start"], usesin)
        if md:
            # a training column whose physics step fails (vi_step status 2, NaN) throws in the
            # reference's GP construction: the trial is dropped; its GPs fit a finite dummy target
            d["vi_failed"] = not np.all(np.isfinite(d["mu"]))
            if d["vi_failed"]:
                d["mu"] = np.nan_to_num(d["mu"], nan=0.0, posinf=0.0, neginf=0.0)
            d["Y_raw"] = d["Y"]
            d["Y"] = d["Y"] - d["mu"]  # the device fits y - μ(X) (mDynamics.jl: θ-independent mean)
        out.append(d)
    return out


def run_group(mech: str, N: int, variant: str, trial_ids, ctx, testsamples: int = 100, simsteps: int = 20,
              max_evals: int | None = 30, time_limit: float = float("nan"), keep: bool = False,
              trials: list | None = None, budget: int | None = None) -> dict:
    """One (mechanism, N, variant) group for this rank's trials: device optimise of every GP,
    then the variant's evaluation.  Returns per-trial arrays (n_local, ...) and timings.
    trials: prebuilt local_trials-shaped inputs (the hyper-parameter search's), else noise.jl's.
    The trials run as one device batch when they fit `budget` bytes (None: the free HBM,
    shard.default_budget), else as several batches one after another (shard.group_plan), with
    bit-identical results; keep=True (the batch returned for inspection) needs one batch."""
    if trials is None:
        trials = local_trials(mech, N, variant, trial_ids, testsamples, ctx)
    n = len(trials)
    if n == 0:
        return {}
    plan = shard.group_plan(trials, ctx, budget)
    if keep and len(plan) > 1:
        raise ValueError(f"run_group(keep=True): the group needs {len(plan)} device batches")
    parts = []
    for lo, hi, nd in plan:
        rb = shard.RankBatch(trials[lo:hi], ctx=ctx, dev_trials=nd)
        part = _run_chunk(mech, variant, trials[lo:hi], rb, ctx, testsamples, simsteps, max_evals, time_limit)
        if keep:
            part.update(rb=rb, trials=trials)
        else:
            rb.close()
        parts.append(part)
    if len(parts) == 1:
        return parts[0]
    out = {k: np.concatenate([p[k] for p in parts]) for k in ("kstep_mse", "projectionerror", "failed", "mll", "theta",
                                                              "status", "f_calls")}
    out.update(rounds=sum(p["rounds"] for p in parts), t_opt=sum(p["t_opt"] for p in parts),
               t_eval=sum(p["t_eval"] for p in parts), slots=sum(p["slots"] for p in parts), batches=len(parts))
    return out


def _run_chunk(mech, variant, trials, rb, ctx, testsamples, simsteps, max_evals, time_limit) -> dict:
    """run_group's work for the trials of one device batch rb."""
    from .optim import LBFGS, Options

    n = len(trials)
    t0 = time.perf_counter()
    th0 = np.stack([t["theta"] for t in trials])
    opt = rb.optimize(th0, LBFGS(), Options(max_evals=max_evals, time_limit=time_limit))
    t_opt = time.perf_counter() - t0
    G = rb.G
    ok_gp = opt["status"] == 0  # (n, G)
    ok_gp &= np.array([[not t.get("vi_failed", False)] for t in trials])  # MeanDynamics mean failed: dropped
    err = np.full(n, math.inf)
    perr = np.zeros(n)
    # a trial whose experiment would throw in the reference (a failed refit: PosDefException /
    # ArgumentError from update_target!; a singular projection: SingularException) is dropped by
    # parallelrun (core.jl:41-53: result = nothing, resultcallback! throws, nothing is pushed)
    failed = np.ones(n, dtype=bool)
    t1 = time.perf_counter()
    if variant == "max":
        # predictdynamics for every test CState of every good trial in one launch
        from .projection import predictdynamics

        good = [i for i in range(n) if np.all(ok_gp[i])]
        if good:
            groups = [[(rb.batch, rb.slot(i, g)) for g in range(G)] for i in good]
            start = np.concatenate([trials[i]["Xs"].T for i in good])
            tg = np.repeat(np.arange(len(good), dtype=np.int32), testsamples)
            fin, pe, st = predictdynamics(mech, groups, start, simsteps, data.VW_INDICES[mech], traj_group=tg, ctx=ctx)
            for k, i in enumerate(good):
                sl = slice(k * testsamples, (k + 1) * testsamples)
                if np.any(st[sl] != 0):  # a singular projection throws in the reference: trial dropped
                    continue
                truth = data.test_truth(mech, testsamples, trials[i]["seed"], simsteps)["X"].T
                err[i] = data.position_mse(truth, fin[sl])
                perr[i] = float(np.mean(pe[sl]))  # projectionerror / length(xtest_old) (P2noise.jl:51)
                failed[i] = False
    elif variant == "md_max":
        # predictdynamics with MeanDynamics GPs: GP means on the device + the physics mean per step
        good = [i for i in range(n) if np.all(ok_gp[i])]
        if good:
            starts = np.stack([trials[i]["Xs"].T for i in range(n)])  # (n, M, d)
            fin, pe, st = mdynamics.rollout_max(mech, rb, good, starts, simsteps, ctx=ctx)
            for k, i in enumerate(good):
                if np.any(st[k] != 0) or np.isnan(fin[k]).any():  # singular projection / failed physics mean
                    continue
                truth = data.test_truth(mech, testsamples, trials[i]["seed"], simsteps)["X"].T
                err[i] = data.position_mse(truth, fin[k])
                perr[i] = float(np.mean(pe[k]))
                failed[i] = False
    elif variant in ("md_min", "md_min_sin"):
        good = [i for i in range(n) if np.all(ok_gp[i])]
        if good:
            starts = np.stack([trials[i]["start"] for i in range(n)])  # (n, M, 2 nc)
            fin = mdynamics.rollout_min(mech, rb, good, starts, simsteps, usesin=variant == "md_min_sin", ctx=ctx)
            for k, i in enumerate(good):
                if np.isnan(fin[k]).any():  # a failed physics mean (vi_step status 2) throws in the reference
                    continue
                truth = data.test_truth(mech, testsamples, trials[i]["seed"], simsteps)["X"].T
                err[i] = data.position_mse(truth, fin[k])
                failed[i] = False
    else:
        usesin = variant == "min_sin"
        nc = NCOORD[mech]
        good = [i for i in range(n) if np.all(ok_gp[i])]
        if good:
            groups = [[(rb.batch, rb.slot(i, g)) for g in range(nc)] for i in good]
            start = np.concatenate([trials[i]["start"] for i in good])
            tg = np.repeat(np.arange(len(good), dtype=np.int32), testsamples)
            fin = rollout_min(mech, groups, start, simsteps, usesin=usesin, traj_group=tg, ctx=ctx)
            for k, i in enumerate(good):
                f = fin[k * testsamples:(k + 1) * testsamples]
                pred = np.stack([final_cstate(mech, row[0::2]) for row in f])
                truth = data.test_truth(mech, testsamples, trials[i]["seed"], simsteps)["X"].T
                err[i] = data.position_mse(truth, pred)
                failed[i] = False
    t_eval = time.perf_counter() - t1
    return dict(kstep_mse=err, projectionerror=perr, failed=failed, mll=opt["mll"], theta=opt["theta"],
                status=opt["status"], f_calls=opt["f_calls"], rounds=opt["rounds"], t_opt=t_opt, t_eval=t_eval,
                slots=n * G, batches=1)


def run_vi_baseline(mech: str, trial_ids, testsamples: int = 100, simsteps: int = 20, ctx=None) -> dict:
    """The pure variational-integrator baseline (noise.jl:72-75, examples/baseline.jl:3-16
    experimentVarInt): every noisy test start simulated for simsteps + 1 physics steps
    (gprx.mdynamics.simulate, the device step), error = simulationerror against the noise-free
    truth.  No GP."""

    n = len(trial_ids)
    err = np.full(n, math.inf)
    failed = np.zeros(n, dtype=bool)
    if n == 0:
        return dict(kstep_mse=err, failed=failed)
    seeds = [data.trial_seed(mech, t) for t in trial_ids]
    # every test start of every local trial in one vectorised simulation (the states are
    # independent: each one's Newton iterates are those of a per-trial call)
    start = np.concatenate([data.make_trial(mech, 2, testsamples, seed=sd)["Xs"].T for sd in seeds])
    fin, st = mdynamics.simulate(mech, start, simsteps, ctx=ctx)
    for k, sd in enumerate(seeds):
        sl = slice(k * testsamples, (k + 1) * testsamples)
        # a test start whose physics step fails (vi_step status 2: the reference's DomainError /
        # SingularException) throws the whole experiment: the trial is dropped (core.jl:41-53)
        if np.any(st[sl] & 2):
            failed[k] = True
            continue
        err[k] = data.position_mse(data.test_truth(mech, testsamples, sd, simsteps)["X"].T, fin[sl])
    return dict(kstep_mse=err, failed=failed)


def run(mechs=MECHS, sizes=SIZES, variants=VARIANTS, n_trials: int = 100, testsamples: int = 100, simsteps: int = 20,
        max_evals: int | None = 30, time_limit: float = float("nan"), ctx=None, log=None) -> dict:
    """The sweep.  Every rank runs its trials of every group; rank 0 returns the gathered
    checkpoint dict (other ranks None).  Without an initialised process group: one rank."""
    from .batch import Context

    dist = _dist()
    rank, world = (dist.get_rank(), dist.get_world_size()) if dist else (0, 1)
    if ctx is None:
        import torch

        ctx = Context(torch.cuda.current_device())
    mine = shard.shard_trials(n_trials, rank, world)
    results: dict = {}
    timing: dict = {}
    for mech in mechs:
        if "vi" in variants:  # the pure variational-integrator baseline (noise.jl:72-75, idmod "VI")
            t0 = time.perf_counter()
            r = run_vi_baseline(mech, mine, testsamples, simsteps, ctx)
            loc = {"kstep_mse": r["kstep_mse"].reshape(-1, 1), "failed": r["failed"].astype(np.float64).reshape(-1, 1),
                   "t": np.full((len(mine), 1), time.perf_counter() - t0)}
            g = shard.gather_results(loc, n_trials, lambda q: shard.shard_trials(n_trials, q, world), 0,
                                     keys=("kstep_mse", "failed", "t")) if dist else loc
            if rank == 0:
                keep = g["failed"][:, 0] == 0  # failed trials left out of the lists (core.jl:41-53)
                results.setdefault("noisyVI", {})[f"{mech}_MIN2"] = {
                    "nprocessed": n_trials, "kstep_mse": [float(v) for v in g["kstep_mse"][keep, 0]],
                    "projectionerror": [0.0] * int(keep.sum()), "variant": "vi", "dropped": int((~keep).sum()),
                    "parity": PARITY["vi"]}
                timing[f"{mech}_MIN2/vi"] = {"seconds_max_rank": float(np.max(g["t"][:, 0])) if n_trials else 0.0,
                                             "gp_fits": 0}
                if log:
                    log(f"{mech}_MIN2 vi: {timing[f'{mech}_MIN2/vi']['seconds_max_rank']:.3f} s")
        for N in sizes:
            for var in variants:
                if var == "vi":
                    continue
                r = run_group(mech, N, var, mine, ctx, testsamples, simsteps, max_evals, time_limit)
                local = {"kstep_mse": r.get("kstep_mse", np.zeros(0)), "perr": r.get("projectionerror", np.zeros(0)),
                         "failed": r.get("failed", np.zeros(0, dtype=bool)).astype(np.float64),
                         "ok": np.all(r["status"] == 0, axis=1).astype(np.float64) if r else np.zeros(0),
                         "t": np.full(len(mine), r.get("t_opt", 0.0) + r.get("t_eval", 0.0))}
                if dist:
                    g = shard.gather_results({k: v.reshape(-1, 1) for k, v in local.items()}, n_trials,
                                             lambda q: shard.shard_trials(n_trials, q, world), 0,
                                             keys=("kstep_mse", "perr", "failed", "ok", "t"))
                else:
                    g = {k: v.reshape(-1, 1) for k, v in local.items()}
                key = f"{mech}_{'MAX' if var.endswith('max') else 'MIN'}{N}"
                if rank == 0:
                    # failed trials are left out of both lists (core.jl:41-53), nprocessed counts them;
                    # a non-finite error of a trial that ran (a diverged rollout) is kept as the
                    # reference keeps it (written as JSON Infinity / NaN)
                    keep = g["failed"][:, 0] == 0
                    et = ETYPE[var]
                    results.setdefault(et, {})[key] = {"nprocessed": n_trials,
                                                       "kstep_mse": [float(v) for v in g["kstep_mse"][keep, 0]],
                                                       "projectionerror": [float(v) for v in g["perr"][keep, 0]],
                                                       "variant": var, "ok": int(g["ok"][:, 0].sum()),
                                                       "dropped": int((~keep).sum()), "parity": PARITY[var]}
                    timing[f"{key}/{var}"] = {"seconds_max_rank": float(np.max(g["t"][:, 0])) if n_trials else 0.0,
                                              "gp_fits": n_trials * (len(data.VW_INDICES[mech]) if var.endswith("max")
                                                                     else NCOORD[mech])}
                    if log:
                        log(f"{key} {var}: ok {results[et][key]['ok']}/{n_trials}, "
                            f"{timing[f'{key}/{var}']['seconds_max_rank']:.3f} s")
    if rank != 0:
        return None
    return {"results": results, "timing": timing, "world": world, "n_trials": n_trials, "max_evals": max_evals,
            "time_limit": time_limit, "testsamples": testsamples, "simsteps": simsteps}


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--mechs", default=",".join(MECHS))
    ap.add_argument("--sizes", default=",".join(map(str, SIZES)))
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--trials", type=int, default=100)
    ap.add_argument("--testsamples", type=int, default=100)
    ap.add_argument("--simsteps", type=int, default=20)
    ap.add_argument("--max-evals", type=int, default=30, help="evaluation budget per GP (<= 0: none, as Optim's f_calls_limit)")
    ap.add_argument("--time-limit", type=float, default=float("nan"), help="seconds per group call (NaN: none)")
    ap.add_argument("--out", default="gpurun_out/sweep_final_checkpoint.json")
    ap.add_argument("--rehearse", action="store_true", help="allow ranks to share GPUs (gloo control plane)")
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks, one per GPU; without a launcher N > 1 starts them itself (as bench.py does)")
    a = ap.parse_args(argv)
    if a.gpus is not None:
        if "WORLD_SIZE" not in os.environ and a.gpus > 1:  # parent: no GPU call has been made
            import sys

            raise SystemExit(shard.launch_ranks(shard.entry_script("sweep"), a.gpus, a.rehearse,
                                                sys.argv[1:] if argv is None else list(argv), "sweep"))
        shard.check_world(a.gpus, "sweep")
    world = shard.init_ranks(a.rehearse)
    t0 = time.perf_counter()
    res = run([m for m in a.mechs.split(",") if m], [int(s) for s in a.sizes.split(",") if s],
              [v for v in a.variants.split(",") if v], a.trials, a.testsamples, a.simsteps,
              a.max_evals if a.max_evals > 0 else None, a.time_limit,
              log=lambda s: print(s, flush=True))
    wall = time.perf_counter() - t0
    if res is not None:
        res["wall_seconds"] = wall
        os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f)
        fits = sum(v["gp_fits"] for v in res["timing"].values())
        print(json.dumps({"sweep_wall_s": round(wall, 3), "groups": len(res["timing"]), "gp_optimisations": fits,
                          "world": res["world"], "out": a.out}), flush=True)
    if world > 1:
        import torch.distributed as dist

        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
