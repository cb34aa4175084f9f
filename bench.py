#!/usr/bin/env python3
"""GP fits/sec on MI355X (BASELINE.json metric), fp64, N=2048, d=26 CState (P2 double pendulum).

One "fit"  = Gram build + Cholesky + alpha + log marginal likelihood,
one full gradient of the LML (one optimiser evaluation), and the predictive mean + variance at
M=100 test CStates -- for one per-output GP at its own hyper-parameters.
One "step" = one batch of fits: T trials x 6 output GPs (vwindices of P2noise.jl:25) per GPU,
each GP with its own theta (config.json P2_MAX2048 jittered, as during optimisation), inputs
resident in HBM before the timed region.

Launch: python bench.py [--gpus N --steps K --warmup W].  For N>1 the ranks run one per GPU over
RCCL: under torch.distributed.run (the driver's form), or started by this script itself as a
torch.distributed.run child when WORLD_SIZE is unset; fewer visible GPUs than N is an error
(--rehearse lets ranks share devices with a gloo control plane, for rehearsals only), and every
rank checks world size == N and the backend.  Trials are sharded over ranks by the product sharding module
(gprx.shard: trial-major round robin, one RankBatch = one device batch of all the rank's trials x
outputs per GPU; weak scaling, no data-path collective).  Rank 0 prints ONE JSON line.
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


def make_trial(t: int) -> dict:
    """Trial t of the workload: P2 training/test CStates (seed data.trial_seed + t) and each output
    GP's own theta (config.json P2_MAX2048 jittered, as during optimisation)."""
    from gprx import data

    th0 = data.theta0(MECH, KEY)
    tr = data.make_trial(MECH, N, M, seed=data.trial_seed(MECH, t))
    rng = np.random.default_rng(10_000 + t)
    theta = np.stack([th0 + 0.05 * rng.standard_normal(th0.shape[0]) for _ in range(G)])
    return dict(X=tr["X"], Y=tr["Y"], Xs=tr["Xs"], theta=theta)


def make_workload(trials_per_gpu: int, rank: int, world: int):
    """This rank's trials (gprx.shard.shard_trials over trials_per_gpu * world trials: rank,
    rank + world, ...), flattened to per-slot arrays (slot = local trial x G + output)."""
    from gprx import shard

    trs = [make_trial(t) for t in shard.shard_trials(trials_per_gpu * world, rank, world)]
    X = np.stack([t["X"] for t in trs for _ in range(G)])
    Y = np.concatenate([t["Y"] for t in trs])
    T = np.concatenate([t["theta"] for t in trs])
    XT = np.stack([t["Xs"] for t in trs for _ in range(G)])
    return trs, X, Y, T, XT


# library stat name -> kernel symbol (prefix) in rocprofv3 output; k_gemm serves several stats
SYMBOL = {"gram": "k_gram", "leaf": "k_leaf", "node8": "k_node8", "diag": "k_diag", "alpha": "k_alpha", "lauum_grad": "k_lauum_grad",
          "finalize": "k_finalize", "pred_cross": "k_pred_cross", "pred_final": "k_pred_final", "pred_var": "k_gemm_pv"}


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
            if k.split()[-1].startswith(sym) and "traffic_bytes_per_launch" in e:  # "void k_gram<1>"
                return {"bytes_per_launch": e["traffic_bytes_per_launch"], "source": f"profiles/{s['round']}_summary.json",
                        "kernel_symbol": k}
    except Exception:
        return None
    return None


def pmc_field(stat: str, global_batch: int, fields):
    """Selected per-kernel fields of the committed PMC summary (same workload only), or None."""
    f = REPO / "profiles" / "pmc_latest.json"
    sym = SYMBOL.get(stat)
    if sym is None or not f.exists():
        return None
    try:
        s = json.loads(f.read_text())
        if (s.get("bench_under_rocprof") or {}).get("config", {}).get("global_batch") != global_batch:
            return None
        for k, e in s["kernels"].items():
            if k.split()[-1].startswith(sym):
                return {q: e.get(q) for q in fields} | {"source": f"profiles/{s['round']}_summary.json"}
    except Exception:
        return None
    return None


def roofline_parts(kern: dict, nprof: int, global_batch: int) -> dict:
    """The north star's two roofline figures beside the dominant kernel's: the Gram build against
    HBM (algorithmic bytes 8 (Npad^2/2 + Npad d) per slot: the lower tiles of K written, X read)
    and the whole factorisation (leaf, the fused 8-tile node halves, TRSM + SYRK/TT + LINV21:
    Cholesky and L^-1, N^3/3 + N^3/3
    flops per slot) against the fp64 MFMA peak; the prediction-variance GEMM too.  Achieved =
    algorithmic work / HIP-event time on the library stream, per launch."""
    def part(names, bound):
        ms = sum(kern[k]["ms"] for k in names)
        n = sum(kern[k]["launches"] for k in names)
        fl = sum(kern[k]["flops"] for k in names)
        by = sum(kern[k]["bytes"] for k in names)
        if ms <= 0:
            return None
        if bound == "hbm":
            ach = by / (ms * 1e-3) / 1e9
            d = {"bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                 "frac": round(ach / PEAK_HBM_GBS, 4), "algorithmic_bytes_per_step": by / nprof}
        else:
            ach = fl / (ms * 1e-3) / 1e12
            d = {"bound": "mfma", "achieved": round(ach, 3), "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s",
                 "frac": round(ach / PEAK_FP64_TFLOPS, 4), "algorithmic_flops_per_step": fl / nprof}
        d.update(kernels=list(names), ms_per_step=round(ms / nprof, 4), launches_per_step=n // nprof)
        if len(names) == 1:
            tr = pmc_traffic(names[0], global_batch)
            d["traffic"] = round(tr["bytes_per_launch"]) if tr else None
            d["traffic_source"] = tr
        return d

    gram = part(["gram"], "hbm")
    if gram is not None:
        # the Gram is priced against HBM (the north star's figure) but HBM does not bind it: its
        # PMC traffic is ~1.03x the algorithmic bytes and its VALU issue floor (SQ_INSTS_VALU x 4
        # cycles / 1024 SIMDs at the PMC clock) is ~0.9 of its time: VALU(+LDS)-bound
        gram["binding_limit"] = "valu"
        gram["valu_floor"] = pmc_field("gram", global_batch, ("valu_floor_ms", "valu_floor_frac", "clock_ghz_est"))
    return {"gram": gram,
            "factorisation": part(["leaf", "node8", "diag", "potrf_trsm", "syrk_tt", "trtri_linv21"], "mfma"),
            "lauum_grad": part(["lauum_grad"], "mfma"),
            "pred_var": part(["pred_var"], "mfma")}


def _cgroup_cpus():
    """The CPU quota of this process's cgroup: (raw text, CPUs as a float or None when unlimited /
    unreadable).  cgroup v2 cpu.max ("quota period" or "max period"), else v1 cfs_quota_us /
    cfs_period_us."""
    cands = ["/sys/fs/cgroup/cpu.max"]
    try:  # the process's own cgroup path (v2: "0::/path")
        for line in pathlib.Path("/proc/self/cgroup").read_text().splitlines():
            parts = line.split(":", 2)
            if len(parts) == 3 and parts[0] == "0" and parts[2] not in ("", "/"):
                cands.insert(0, f"/sys/fs/cgroup{parts[2]}/cpu.max")
    except OSError:
        pass
    for p in cands:
        try:
            raw = pathlib.Path(p).read_text().strip()
        except OSError:
            continue
        q, per = (raw.split() + ["100000"])[:2]
        return f"{p}: {raw}", (None if q == "max" else int(q) / int(per))
    for d in ("/sys/fs/cgroup/cpu", "/sys/fs/cgroup/cpu,cpuacct"):
        try:
            q = int(pathlib.Path(d, "cpu.cfs_quota_us").read_text())
            per = int(pathlib.Path(d, "cpu.cfs_period_us").read_text())
        except (OSError, ValueError):
            continue
        return f"{d}/cpu.cfs_quota_us: {q} / {per}", (None if q < 0 else q / per)
    return "no cgroup cpu controller readable", None


def _host_cores():
    """The CPUs the box grants this process and how the baseline's thread count follows from them:
    affinity (sched_getaffinity), the cgroup quota and OMP_NUM_THREADS are all read and reported.
    cores = the affinity capped by the cgroup quota when one is set (the CPUs the kernel will
    actually schedule us on); without a quota, the launcher's stated share (OMP_NUM_THREADS) caps
    it; else the whole affinity set.  Returns (cores, facts dict)."""
    nproc = len(os.sched_getaffinity(0))
    raw, quota = _cgroup_cpus()
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if quota is not None:
        cores, rule = max(1, min(nproc, int(quota))), "min(affinity, cgroup quota)"
    elif share > 0:
        cores, rule = min(share, nproc), "no cgroup quota: min(affinity, OMP_NUM_THREADS)"
    else:
        cores, rule = nproc, "no cgroup quota, no OMP_NUM_THREADS: affinity"
    return cores, dict(affinity=nproc, cgroup=raw, cgroup_quota_cpus=quota, omp_num_threads=share or None, rule=rule)


def _oracle_fit_worker(args):
    """One process of the trial-parallel CPU mode: BLAS single-threaded, fits slots until the
    deadline (the reference's Threads.@threads over trials, one fit per thread, core.jl:28)."""
    slots, X, Y, T, XT, deadline = args
    from threadpoolctl import threadpool_limits

    sys.path.insert(0, str(REPO))
    from oracle import gp_oracle as O

    n = 0
    with threadpool_limits(1):
        for s in slots:
            if time.time() > deadline:
                break
            O.fit(X[s], Y[s], T[s], XT[s])
            n += 1
    return n


def cpu_baseline(X, Y, T, XT, gpu=None, max_seconds: float = 15.0, max_fits: int = 32, modes=("single", "parallel")):
    """The CPU restatement of the reference algorithm timed on a bounded sample of the same
    workload, in the two SURVEY.md section 8d modes:
      single   one fit at a time, BLAS on every used core;
      parallel trial-parallel: whole fits on every used core at once, BLAS single-threaded (the
               reference's Threads.@threads over trials, core.jl:28).
    Timed implementation: oracle/cpu_fit.c (C on the host's OpenBLAS, OpenMP threads for the
    trial-parallel mode), or the numpy oracle when libcpufit.so is absent.
    With `gpu` (the last timed step's results) a few slots are also checked against the numpy oracle
    (oracle/gp_oracle.py): the metric's accuracy part, max |mu_gpu - mu_cpu| of the predictive
    means (BASELINE.json 'pred-mean max-err').  Returns (baseline dict, accuracy dict)."""
    sys.path.insert(0, str(REPO))
    from oracle import gp_oracle as O
    from threadpoolctl import threadpool_limits

    cores, facts = _host_cores()
    nproc = facts["affinity"]
    out = {}
    impl = "numpy"
    try:
        from oracle import cpu_fit as CF

        CF.load()
        impl = "c"
    except OSError:
        CF = None
    if impl == "c":
        if "single" in modes:
            n, dt = CF.timed(X, Y, T, XT, threads=1, blas_threads=cores, max_seconds=max_seconds, max_fits=1 << 20)
            out["single"] = dict(value=n / dt, fits=n, seconds=round(dt, 2), blas_threads=cores)
        if "parallel" in modes:
            n, dt = CF.timed(X, Y, T, XT, threads=cores, blas_threads=1, max_seconds=max_seconds, max_fits=1 << 20)
            out["parallel"] = dict(value=n / dt, fits=n, seconds=round(dt, 2), threads=cores, blas_threads_each=1)
    else:
        if "single" in modes:
            t0 = time.perf_counter()
            n = 0
            with threadpool_limits(cores):
                for s in range(min(max_fits, X.shape[0])):
                    O.fit(X[s], Y[s], T[s], XT[s])
                    n += 1
                    if time.perf_counter() - t0 > max_seconds:
                        break
            dt = time.perf_counter() - t0
            out["single"] = dict(value=n / dt, fits=n, seconds=round(dt, 2), blas_threads=cores)
        if "parallel" in modes:
            import multiprocessing as mp

            P = cores
            deadline = time.time() + max_seconds
            # every process gets its own slots (round robin), enough for the deadline
            per = max(2, max_fits // P + 2)
            jobs = [([(k + P * i) % X.shape[0] for i in range(per)], X, Y, T, XT, deadline) for k in range(P)]
            t0 = time.perf_counter()
            with mp.get_context("fork").Pool(P) as pool:
                counts = pool.map(_oracle_fit_worker, jobs)
            dt = time.perf_counter() - t0
            out["parallel"] = dict(value=sum(counts) / dt, fits=int(sum(counts)), seconds=round(dt, 2), processes=P,
                                   blas_threads_each=1)
    err = dict(mu_abs=0.0, mu_rel=0.0, mll_rel=0.0, grad_rel=0.0)
    n_err = 0
    if gpu is not None:  # accuracy on a few slots against the numpy oracle
        with threadpool_limits(cores):
            for s in range(min(4, X.shape[0])):
                f = O.fit(X[s], Y[s], T[s], XT[s])
                e_mu = float(np.max(np.abs(gpu["mu"][s] - f["mu"])))
                err["mu_abs"] = max(err["mu_abs"], e_mu)
                err["mu_rel"] = max(err["mu_rel"], e_mu / float(np.max(np.abs(Y[s]))))
                err["mll_rel"] = max(err["mll_rel"], abs(gpu["mll"][s] - f["mll"]) / max(1.0, abs(f["mll"])))
                err["grad_rel"] = max(err["grad_rel"], float(np.max(np.abs(gpu["grad"][s] - f["grad"])))
                                      / max(1.0, float(np.max(np.abs(f["grad"])))))
                n_err += 1
    best = max(out, key=lambda k: out[k]["value"])
    how = ("oracle/cpu_fit.c: C on the host's OpenBLAS (dpotrf/dpotrs/dtrsm), OpenMP threads for the trial-parallel "
           "mode" if impl == "c" else "oracle/gp_oracle.py: numpy + the host's OpenBLAS")
    base = dict(value=out[best]["value"], unit="fits/s", cores=cores, kind="port", nproc=nproc, host_cpus=facts,
                mode=best, modes=out, impl=impl,
                sample=f"P2 fits (N=2048, d=26, M=100) of the bench workload via {how} (reference algorithm: "
                       f"KernelData distance stack, direct distances, dpotrf, K^-1 by dpotrs on I, per-parameter "
                       f"gradient sums), each mode bounded to ~{max_seconds:.0f} s; value = the faster mode ({best}); "
                       f"{cores} of nproc={nproc} host CPUs used ({facts['rule']}; {facts['cgroup']})")
    acc = None
    if gpu is not None and n_err:
        acc = dict(err, slots=n_err, tolerance_mu_rel=1e-9, tolerance_mll_rel=1e-10, tolerance_grad_rel=1e-7,
                   note="GPU vs CPU restatement (oracle/gp_oracle.py) on the same inputs; mu_rel = max|dmu| / max|y|")
    return base, acc


def _progress(rank: int, msg: str):
    """One progress line on stderr (rank 0): the JSON result stays the only stdout line."""
    if rank == 0:
        print(f"bench: {msg}", file=sys.stderr, flush=True)


def _launch_ranks(args) -> int:
    """`bench.py --gpus N` (N > 1) started without a launcher: start N ranks, one per GPU, as a
    torch.distributed.run child (the driver's own command line), and return its exit code.  Runs
    before this process touches a GPU (device_count() does not initialise one on this image).  Too
    few visible GPUs is an error, not a silent one-rank run; --rehearse lets ranks share devices."""
    import torch

    ndev = torch.cuda.device_count()
    if ndev < args.gpus and not args.rehearse:
        print(f"bench: --gpus {args.gpus} needs {args.gpus} visible GPUs, this host has {ndev} "
              f"(--rehearse runs the ranks on shared devices, for a rehearsal only)", file=sys.stderr)
        return 2
    # the command line of gprx.shard.launch_cmd (c10d rendezvous on a free port of 127.0.0.1),
    # written out here so that this parent never imports the library
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr", "127.0.0.1", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", str(pathlib.Path(__file__).resolve()), *sys.argv[1:]]
    _progress(0, f"launching {args.gpus} ranks: {' '.join(cmd[1:8])} ...")
    import subprocess

    return subprocess.run(cmd).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    # 40 trials = 240 slots: the fused leaf (one workgroup per slot) then covers 240 of the 256 CUs;
    # measured 5578 fits/s against 5489 at 32 trials and 5551 at 42 (scratch/bsweep.sh, one box)
    ap.add_argument("--trials", type=int, default=int(os.environ.get("GPRX_BENCH_TRIALS", "40")),
                    help="P2 trials per GPU per step (x6 output GPs)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-prof", action="store_true")
    ap.add_argument("--no-opt", action="store_true")
    ap.add_argument("--opt-evals", type=int, default=30)
    ap.add_argument("--rehearse", action="store_true",
                    help="allow more ranks than visible GPUs (ranks share devices, gloo control plane): a "
                         "rehearsal of the distributed path, never a measurement")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(_launch_ranks(args))  # parent: no GPU call has been made
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"bench: --gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU "
              f"(python bench.py --gpus N starts them itself)", file=sys.stderr)
        sys.exit(2)
    import torch

    dist = None
    ndev = torch.cuda.device_count()
    if ndev < 1 or (world > ndev and not args.rehearse):
        print(f"bench: {world} rank(s) need {world} GPUs, {ndev} visible", file=sys.stderr)
        sys.exit(2)
    dev = local % ndev  # only a --rehearse run puts two ranks on one device
    torch.cuda.set_device(dev)
    backend = None
    if world > 1:
        import torch.distributed as dist

        # the collectives here are control plane only (barrier, max of the timings, the per-rank
        # rates): RCCL over xGMI, one rank per GPU; gloo only for a shared-device --rehearse run
        backend = "gloo" if args.rehearse else "nccl"
        dist.init_process_group(backend)
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)
        assert dist.get_backend() == backend, dist.get_backend()

    import gprx

    from gprx import shard

    ctx = gprx.Context(dev)
    trs, X, Y, T, XT = make_workload(args.trials, rank, world)
    B, d = X.shape[0], X.shape[1]
    rb = shard.RankBatch(trs, ctx=ctx)  # one device batch: this rank's trials x G outputs
    batch = rb.batch

    def barrier():
        if dist is not None:
            dist.barrier()
        torch.cuda.synchronize()

    TH = T.reshape(rb.n, G, -1)  # per (local trial, output)
    _progress(rank, f"{B} slots per rank, {world} rank(s); warm-up")
    for _ in range(args.warmup):
        r = rb.evaluate(TH)
    ok = bool(np.all(r["status"] == 0)) if args.warmup else True

    barrier()
    _progress(rank, f"timing {args.steps} steps")
    t0 = time.perf_counter()
    for _ in range(args.steps):
        r = rb.evaluate(TH)
    barrier()
    dt = time.perf_counter() - t0
    ok = ok and bool(np.all(r["status"] == 0))
    r = {k: np.asarray(v).reshape((B,) + np.asarray(v).shape[2:]) for k, v in r.items()}  # per slot
    per_rank = [B * args.steps / dt]
    if dist is not None:
        cdev = f"cuda:{dev}" if backend == "nccl" else "cpu"
        t = torch.tensor([dt, B * args.steps / dt, float(ok)], dtype=torch.float64, device=cdev)
        allt = [torch.empty_like(t) for _ in range(world)]
        dist.all_gather(allt, t)
        allt = torch.stack(allt).cpu().numpy()
        dt = float(allt[:, 0].max())  # the slowest rank's time
        per_rank = [float(v) for v in allt[:, 1]]
        ok = bool(np.all(allt[:, 2] == 1.0))
    fits = B * args.steps * world
    value = fits / dt

    # roofline: per-kernel HIP-event timing on the library stream, same workload, separate pass
    roof = parts = None
    kern = {}
    if not args.no_prof:
        _progress(rank, "per-kernel timing pass")
        ctx.set_profiling(True)
        ctx.reset_stats()
        nprof = max(1, min(args.steps, 3))
        for _ in range(nprof):
            rb.evaluate(TH)
        ctx.set_profiling(False)
        names = ["gram", "leaf", "node8", "diag", "potrf_trsm", "syrk_tt", "trtri_linv21", "alpha", "lauum_grad",
                 "finalize", "pred_cross", "pred_var", "pred_final"]
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
        parts = roofline_parts(kern, nprof, B * world)
    step_flops = B * fit_flops(N, d, M)
    # secondary figure: optimise-fits/sec with a fixed evaluation budget --
    # every slot runs Optim-style LBFGS + BackTracking(order=2) from its theta, all slots sharing
    # one device evaluation per round.  Device optimiser (k_lbfgs, GPBatch.optimize, with
    # optimize!'s closing refit) is the figure; the host lock-step restatement
    # (gprx.optim.optimize_batch) is timed beside it and must give bit-identical minimisers.
    opt = None
    if not args.no_opt:
        from gprx.optim import LBFGS, Options, compare_optimisers, optimize_batch

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

        _progress(rank, "optimiser leg")
        o = Options(max_evals=args.opt_evals)
        # both legs record their evaluations (theta asked, answer given, per round): a mismatch is
        # then reported down to the first evaluation where the legs part (compare_optimisers)
        htrace = []
        ntr = 4 * args.opt_evals + 8  # rounds to record: more than the budget can use
        (hres, hrounds), t_host = timed(lambda: optimize_batch(batch, T, LBFGS(), o, trace=htrace))
        (res, rounds), t_opt = timed(lambda: batch.optimize(T, LBFGS(), o, refit=True, trace_rounds=ntr))
        cmp = compare_optimisers(res, hres, batch.last_opt_trace, np.stack(htrace) if htrace else None)
        same = cmp["equal"]
        opt = {"value": round(B * world / t_opt, 3), "unit": "optimised GP fits/s", "max_evals_per_gp": args.opt_evals,
               "optimiser": "device k_lbfgs (+ refit)", "device_rounds": rounds, "seconds": round(t_opt, 3),
               "host_lockstep": {"value": round(B * world / t_host, 3), "seconds": round(t_host, 3),
                                 "device_rounds": hrounds},
               "device_equals_host": bool(same),
               "device_vs_host": cmp,
               "stopped_by": {k: sum(1 for r in res if r.stopped_by == k) for k in sorted({r.stopped_by for r in res})}}
    cpu = acc = None
    if rank == 0 and not args.no_cpu:
        _progress(rank, "CPU baseline leg")
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
            "ranks": world,
            "backend": backend or "single process",
            "per_rank_fits_per_s": [round(v, 3) for v in per_rank],
            "fit_ok": ok,
            "whole_step_tflops": round(step_flops / (dt / args.steps) / 1e12 * 1.0, 3),
            "whole_step_frac_of_fp64_peak": round(step_flops / (dt / args.steps) / 1e12 / PEAK_FP64_TFLOPS, 4),
            "roofline": roof,
            "roofline_parts": parts,
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
