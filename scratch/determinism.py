"""Reproducibility probe for the bench workload (P2 N=2048, B=240): are evaluations bit-identical
run to run, and do the device and host optimisers agree bit for bit?

1. Alternating evaluations: theta_a, theta_b, theta_a, ... (grad, no predict: the optimiser's
   evaluation; then grad + predict: the bench's).  Every theta_a result must equal the first one
   bit for bit, whatever ran in between.
2. The bench's optimiser legs (max_evals 30) several times, host and device, each pair compared
   with gprx.optim.compare_optimisers (first differing evaluation).

Run on the GPU box: python scratch/determinism.py [--reps R] [--opt-reps K]
"""
from __future__ import annotations

import argparse
import json
import pathlib
import sys
import time

import numpy as np

REPO = pathlib.Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))
sys.path.insert(0, str(REPO / "gpr.jl_amd"))


def bits(r):
    return {k: np.ascontiguousarray(v).view(np.uint64).copy() for k, v in r.items()
            if v is not None and np.asarray(v).dtype == np.float64}


def diff(a, b):
    out = {}
    for k in a:
        bad = np.nonzero(np.any((a[k] != b[k]).reshape(a[k].shape[0], -1), axis=1))[0]
        if bad.size:
            fa = a[k].view(np.float64)
            fb = b[k].view(np.float64)
            out[k] = dict(slots=bad[:12].tolist(), n=int(bad.size),
                          max_abs=float(np.nanmax(np.abs(fa[bad] - fb[bad]))))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=12)
    ap.add_argument("--opt-reps", type=int, default=3)
    ap.add_argument("--trials", type=int, default=40)
    args = ap.parse_args()
    import bench
    import gprx
    from gprx import shard
    from gprx.optim import LBFGS, Options, compare_optimisers, optimize_batch

    ctx = gprx.Context(0)
    trs, X, Y, T, XT = bench.make_workload(args.trials, 0, 1)
    rb = shard.RankBatch(trs, ctx=ctx)
    batch = rb.batch
    rng = np.random.default_rng(7)
    Ta = T
    Tb = T + 0.02 * rng.standard_normal(T.shape)
    rep = {}
    for mode, kw in (("grad", dict(grad=True, predict=False)), ("grad+pred", dict(grad=True, predict=True))):
        t0 = time.time()
        ref_a = bits(batch.run(Ta, **kw))
        ref_b = bits(batch.run(Tb, **kw))
        bad = []
        for i in range(args.reps):
            for nm, th, ref in (("a", Ta, ref_a), ("b", Tb, ref_b)):
                d = diff(ref, bits(batch.run(th, **kw)))
                if d:
                    bad.append(dict(rep=i, theta=nm, diff=d))
        rep[mode] = dict(evaluations=2 * args.reps + 2, mismatches=len(bad), first=bad[:4],
                         seconds=round(time.time() - t0, 2))
        print(f"determinism {mode}: {len(bad)} mismatching evaluations of {2 * args.reps}", file=sys.stderr, flush=True)
    o = Options(max_evals=30)
    legs = []
    for i in range(args.opt_reps):
        ht = []
        hres, _ = optimize_batch(batch, T, LBFGS(), o, trace=ht)
        dres, _ = batch.optimize(T, LBFGS(), o, refit=True, trace_rounds=128)
        legs.append(("host", hres, np.stack(ht)))
        legs.append(("device", dres, batch.last_opt_trace))
        print(f"optimiser rep {i} done", file=sys.stderr, flush=True)
    base = legs[0]
    rep["optimiser"] = [dict(leg=f"{nm}{i // 2}", vs="host0", **compare_optimisers(r, base[1], t, base[2]))
                        for i, (nm, r, t) in enumerate(legs[1:], start=1)]
    print(json.dumps(rep, default=str))


if __name__ == "__main__":
    main()
