"""fits/s of the bench workload (P2, N=2048, d=26, M=100, gradient + mean/var) at arbitrary slot
counts: the first B (trial, output) pairs of ceil(B/6) trials, one batch per call.
    python scratch/slots_sweep.py 240,248,256 [reps]"""
import sys
import time
import pathlib

REPO = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "gpr.jl_amd"), str(REPO)]
import numpy as np  # noqa: E402

import gprx  # noqa: E402
from gprx import data  # noqa: E402

ctx = gprx.Context(0)
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
for B in [int(s) for s in sys.argv[1].split(",")]:
    T = -(-B // 6)
    trs = [data.make_trial("P2", 2048, 100, seed=data.trial_seed("P2", t)) for t in range(T)]
    X = np.stack([tr["X"] for tr in trs for _ in range(6)])[:B]
    Y = np.concatenate([tr["Y"] for tr in trs])[:B]
    XT = np.stack([tr["Xs"] for tr in trs for _ in range(6)])[:B]
    th = np.tile(data.theta0("P2", 2048), (B, 1))
    b = gprx.GPBatch(B, X.shape[1], 2048, 100, ctx=ctx)
    b.set_train(X, Y)
    b.set_test(XT)
    for _ in range(2):
        r = b.run(th, grad=True, predict=True)
    t0 = time.perf_counter()
    for _ in range(reps):
        r = b.run(th, grad=True, predict=True)
    dt = (time.perf_counter() - t0) / reps
    print(f"B={B:4d}: {dt * 1e3:8.3f} ms/step  {B / dt:9.1f} fits/s  ok={int((r['status'] == 0).sum())}/{B}", flush=True)
    b.close()
