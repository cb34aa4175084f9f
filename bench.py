#!/usr/bin/env python3
"""GP fits/sec on MI355X (BASELINE.json metric), fp64, N=2048, d=26 CState (P2 double pendulum).

One "fit"  = Gram build + Cholesky + alpha + log marginal likelihood,
one full gradient of the LML (one optimiser evaluation), and the predictive mean + variance at
M=100 test CStates -- for one per-output GP at its own hyper-parameters.
One "step" = one batch of fits: T trials x 6 output GPs (vwindices of P2noise.jl:25) per GPU,
each GP with its own theta (config.json P2_MAX2048 jittered, as during optimisation), inputs
resident in HBM before the timed region.

Launch: python bench.py [--gpus N --steps K --warmup W]; for N>1 under torch.distributed.run
(one rank per GPU).  Trials are sharded over ranks (weak scaling, no data-path collective).
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import os
import pathlib
import sys
import time

import numpy as np

REPO = pathlib.Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "gpr.jl_amd"))

MECH, N, M, KEY = "P2", 2048, 100, 2048
G = 6
PEAK_FP64_TFLOPS = 78.6  # MI355X fp64 matrix peak (MI355X_MICROARCH.md); sustained under DVFS with random
# operands: 61-67 TF/s measured (scratch/mfma_sustain.hip)
PEAK_HBM_GBS = 8000.0


def fit_flops(N: int, d: int, Mt: int) -> float:
    """Algorithmic flops of one fit, SURVEY.md section 8d."""
    return (3 * N * N * d + N**3 / 3 + 2 * N * N + 2 * N**3 / 3 + 2 * N * N * d + 4 * N * N
            + N * N * Mt + 3 * N * Mt * d + 2 * N * Mt)


def make_workload(trials_per_gpu: int, rank: int, world: int, seed_base: int = 0):
    from gprx import data

    th0 = data.theta0(MECH, KEY)
    Xs, Ys, Ts, XTs = [], [], [], []
    for k in range(trials_per_gpu):
        trial = rank + world * k  # trial-major round robin over ranks
        tr = data.make_trial(MECH, N, M, seed=data.trial_seed(MECH, trial) + seed_base)
        rng = np.random.default_rng(10_000 + trial)
        for g in range(G):
            Xs.append(tr["X"])
            XTs.append(tr["Xs"])
            Ys.append(tr["Y"][g])
            Ts.append(th0 + 0.05 * rng.standard_normal(th0.shape[0]))
    return np.stack(Xs), np.stack(Ys), np.stack(Ts), np.stack(XTs)


# library stat name -> kernel symbol (prefix) in rocprofv3 output; k_gemm serves several stats
SYMBOL = {"gram": "k_gram", "leaf": "k_leaf", "diag": "k_diag", "alpha": "k_alpha", "lauum_grad": "k_lauum_grad",
          "finalize": "k_finalize", "pred_cross": "k_pred_cross", "pred_final": "k_pred_final"}


def pmc_traffic(stat: str, global_batch: int):
    """HBM bytes per launch of `stat`'s kernel from the committed PMC summary (profiles/collect.sh),
    if it was collected on this same workload; else None."""
    f = REPO / "profiles" / "pmc_latest.json"
    sym = SYMBOL.get(stat)
    if sym is None or not f.exists():
        return None
    try:
        s = json.loads(f.read_text())
        if (s.get("bench_under_rocprof") or {}).get("config", {}).get("global_batch") != global_batch:
            return None
        for k, e in s["kernels"].items():
            if k.startswith(sym) and "traffic_bytes_per_launch" in e:
                return {"bytes_per_launch": e["traffic_bytes_per_launch"], "source": f"profiles/{s['round']}_summary.json",
                        "kernel_symbol": k}
    except Exception:
        return None
    return None


def cpu_baseline(X, Y, T, XT, gpu=None, max_seconds: float = 15.0, max_fits: int = 32):
    """Oracle (CPU restatement, numpy + OpenBLAS LAPACK) on a bounded sample of the same workload.
    With `gpu` (the last timed step's results) the same sample also gives the metric's accuracy
    part: max |mu_gpu - mu_cpu| of the predictive means (BASELINE.json 'pred-mean max-err')."""
    sys.path.insert(0, str(REPO))
    from oracle import gp_oracle as O

    try:
        from threadpoolctl import threadpool_info

        threads = max([i.get("num_threads", 1) for i in threadpool_info() if i.get("internal_api") == "openblas"] or [1])
    except Exception:
        threads = int(os.environ.get("OMP_NUM_THREADS", "1"))
    t0 = time.perf_counter()
    n = 0
    err = dict(mu_abs=0.0, mu_rel=0.0, mll_rel=0.0, grad_rel=0.0)
    for s in range(min(max_fits, X.shape[0])):
        f = O.fit(X[s], Y[s], T[s], XT[s])
        n += 1
        if gpu is not None:
            e_mu = float(np.max(np.abs(gpu["mu"][s] - f["mu"])))
            err["mu_abs"] = max(err["mu_abs"], e_mu)
            err["mu_rel"] = max(err["mu_rel"], e_mu / float(np.max(np.abs(Y[s]))))
            err["mll_rel"] = max(err["mll_rel"], abs(gpu["mll"][s] - f["mll"]) / max(1.0, abs(f["mll"])))
            err["grad_rel"] = max(err["grad_rel"], float(np.max(np.abs(gpu["grad"][s] - f["grad"])))
                                  / max(1.0, float(np.max(np.abs(f["grad"])))))
        if time.perf_counter() - t0 > max_seconds:
            break
    dt = time.perf_counter() - t0
    base = dict(value=n / dt, unit="fits/s", cores=int(threads), kind="port",
                sample=f"{n} P2 fits (N=2048, d=26, M=100) via oracle/gp_oracle.py: reference algorithm "
                       f"(distij direct distances, OpenBLAS dpotrf, K^-1 by cho_solve(I), per-param grad "
                       f"sums), {dt:.1f}s, OpenBLAS threads={threads}")
    acc = None
    if gpu is not None:
        acc = dict(err, slots=n, tolerance_mu_rel=1e-9, tolerance_mll_rel=1e-9, tolerance_grad_rel=1e-7,
                   note="GPU vs CPU restatement on the same inputs; mu_rel = max|dmu| / max|y|")
    return base, acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--trials", type=int, default=int(os.environ.get("GPRX_BENCH_TRIALS", "32")),
                    help="P2 trials per GPU per step (x6 output GPs)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-prof", action="store_true")
    ap.add_argument("--no-opt", action="store_true")
    ap.add_argument("--opt-evals", type=int, default=30)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    dist = None
    ndev = torch.cuda.device_count()
    dev = local % max(1, ndev)  # rehearsal with more ranks than GPUs shares a device
    torch.cuda.set_device(dev)
    backend = "nccl"
    if world > 1:
        import torch.distributed as dist

        # the collectives here are control plane only (barrier, max of the timings); RCCL when every
        # rank has its own GPU, gloo for a shared-device rehearsal
        backend = "nccl" if ndev >= world else "gloo"
        dist.init_process_group(backend)

    import gprx

    ctx = gprx.Context(dev)
    X, Y, T, XT = make_workload(args.trials, rank, world)
    B, d = X.shape[0], X.shape[1]
    batch = gprx.GPBatch(B, d, N, M, ctx=ctx)
    batch.set_train(X, Y)
    batch.set_test(XT)

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    for _ in range(args.warmup):
        r = batch.run(T, grad=True, predict=True)
    ok = bool(np.all(r["status"] == 0)) if args.warmup else True

    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        r = batch.run(T, grad=True, predict=True)
    barrier()
    dt = time.perf_counter() - t0
    ok = ok and bool(np.all(r["status"] == 0))
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{dev}" if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    fits = B * args.steps * world
    value = fits / dt

    # roofline: per-kernel HIP-event timing on the library stream, same workload, separate pass
    roof = None
    kern = {}
    if not args.no_prof:
        ctx.set_profiling(True)
        ctx.reset_stats()
        nprof = max(1, min(args.steps, 3))
        for _ in range(nprof):
            batch.run(T, grad=True, predict=True)
        ctx.set_profiling(False)
        names = ["gram", "leaf", "diag", "potrf_trsm", "potrf_syrk", "trtri_tt", "syrk_tt", "trtri_linv21", "alpha", "lauum_grad",
                 "finalize", "pred_cross", "pred_var", "pred_mu", "pred_final"]
        for nme in names:
            kern[nme] = ctx.kernel_stats(nme)
        dom = max(kern, key=lambda k: kern[k]["ms"])
        s = kern[dom]
        avg_ms = s["ms"] / max(1, s["launches"])
        per_launch_flops = s["flops"] / max(1, s["launches"])
        achieved = per_launch_flops / (avg_ms * 1e-3) / 1e12
        tr = pmc_traffic(dom, B * world)
        roof = {"bound": "mfma", "kernel": dom, "achieved": round(achieved, 3), "peak": PEAK_FP64_TFLOPS,
                "unit": "TFLOP/s", "frac": round(achieved / PEAK_FP64_TFLOPS, 4),
                "traffic": round(tr["bytes_per_launch"]) if tr else None,
                "traffic_unit": "bytes/launch (PMC 2*FETCH_SIZE+WRITE_SIZE)", "traffic_source": tr,
                "algorithmic_bytes_per_launch": round(s["bytes"] / max(1, s["launches"])),
                "algorithmic_flops_per_launch": per_launch_flops,
                "avg_launch_ms": round(avg_ms, 4), "launches_per_step": s["launches"] // nprof}
    step_flops = B * fit_flops(N, d, M)
    # secondary figure: optimise-fits/sec with a fixed evaluation budget --
    # every slot runs Optim-style LBFGS + BackTracking(order=2) from its theta, all slots sharing
    # one device evaluation per round.  Device optimiser (k_lbfgs, GPBatch.optimize, with
    # optimize!'s closing refit) is the figure; the host lock-step restatement
    # (gprx.optim.optimize_batch) is timed beside it and must give bit-identical minimisers.
    opt = None
    if not args.no_opt:
        from gprx.optim import LBFGS, Options, optimize_batch

        def timed(fn):
            barrier()
            t0 = time.perf_counter()
            out = fn()
            barrier()
            t = time.perf_counter() - t0
            if dist is not None:
                tt = torch.tensor([t], dtype=torch.float64, device=f"cuda:{dev}" if backend == "nccl" else "cpu")
                dist.all_reduce(tt, op=dist.ReduceOp.MAX)
                t = float(tt.item())
            return out, t

        o = Options(max_evals=args.opt_evals)
        (hres, hrounds), t_host = timed(lambda: optimize_batch(batch, T, LBFGS(), o))
        (res, rounds), t_opt = timed(lambda: batch.optimize(T, LBFGS(), o, refit=True))
        same = all(np.array_equal(a.minimizer, b.minimizer) and a.minimum == b.minimum for a, b in zip(res, hres))
        opt = {"value": round(B * world / t_opt, 3), "unit": "optimised GP fits/s", "max_evals_per_gp": args.opt_evals,
               "optimiser": "device k_lbfgs (+ refit)", "device_rounds": rounds, "seconds": round(t_opt, 3),
               "host_lockstep": {"value": round(B * world / t_host, 3), "seconds": round(t_host, 3),
                                 "device_rounds": hrounds},
               "device_equals_host": bool(same),
               "stopped_by": {k: sum(1 for r in res if r.stopped_by == k) for k in sorted({r.stopped_by for r in res})}}
    cpu = acc = None
    if rank == 0 and not args.no_cpu:
        if world == 1:  # the CPU baseline is an N=1 figure
            cpu, acc = cpu_baseline(X, Y, T, XT, gpu=r)
        else:  # N > 1: the metric's accuracy part only, on two of rank 0's slots
            _, acc = cpu_baseline(X, Y, T, XT, gpu=r, max_fits=2)

    if rank == 0:
        out = {
            "metric": "GP fits/sec (fp64, N=2048, d=26 CState)",
            "value": round(value, 3),
            "unit": "fits/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (P2 CState generator, reference kinematics; theta from config.json P2_MAX2048)",
            "config": {"workload": f"P2 double pendulum: {args.trials} trials x {G} output GPs per GPU, N={N}, "
                                   f"d={d}, M={M} test points; fit = Gram+Cholesky+alpha+LML, full dLML, predict mean+var",
                       "global_batch": fits // args.steps, "N": N, "d": d, "M": M, "parallelism": f"trial-shard x{world}"},
            "fit_ok": ok,
            "whole_step_tflops": round(step_flops / (dt / args.steps) / 1e12 * 1.0, 3),
            "whole_step_frac_of_fp64_peak": round(step_flops / (dt / args.steps) / 1e12 / PEAK_FP64_TFLOPS, 4),
            "roofline": roof,
            "kernels_ms_per_step": {k: round(v["ms"] / max(1, (min(args.steps, 3))), 3) for k, v in kern.items()} if kern else None,
            "cpu_baseline": cpu,
            "pred_mean_max_err": acc,
            "optimise": opt,
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
