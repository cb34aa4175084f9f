"""CP (N=512, 26 outputs) fits/s under the launch-geometry options (leaf tiles, small-node unit,
graphs): python scratch/cp_geom.py TRIALS"""
import pathlib
import sys
import time

REPO = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "gpr.jl_amd"), str(REPO)]
import numpy as np  # noqa: E402

import gprx  # noqa: E402
from gprx import data  # noqa: E402

T = int(sys.argv[1]) if len(sys.argv) > 1 else 39
trs = [data.make_trial("CP", 512, 100, seed=data.trial_seed("CP", t)) for t in range(T)]
X = np.stack([tr["X"] for tr in trs for _ in range(26)])
Y = np.concatenate([tr["Xcurr"] for tr in trs])
XT = np.stack([tr["Xs"] for tr in trs for _ in range(26)])
B, d = X.shape[0], X.shape[1]
th = np.tile(data.theta0("CP", 512), (B, 1))
ref = None
for leaf, small, graphs in [(0, 0, 0), (2, 0, 0), (1, 0, 0), (0, 8, 0), (0, 0, 1), (0, 0, 0)]:
    ctx = gprx.Context(0)
    ctx.set_option(gprx.OPT_LEAF_TILES, leaf)
    ctx.set_option(gprx.OPT_SMALL_N, small)
    ctx.set_option(gprx.OPT_GRAPHS, graphs)
    b = gprx.GPBatch(B, d, 512, 100, ctx=ctx)
    b.set_train(X, Y)
    b.set_test(XT)
    for _ in range(2):
        r = b.run(th, grad=True, predict=True)
    n = 10
    t0 = time.perf_counter()
    for _ in range(n):
        r = b.run(th, grad=True, predict=True)
    dt = (time.perf_counter() - t0) / n
    same = ref is None or (np.array_equal(r["mll"], ref["mll"]) and np.array_equal(r["grad"], ref["grad"]))
    if ref is None:
        ref = r
    print(f"leaf={leaf} small_n={small} graphs={graphs}: {dt * 1e3:7.3f} ms/batch {B / dt:10.1f} fits/s  "
          f"ok={int((r['status'] == 0).sum())}/{B} same_as_default={same}", flush=True)
    b.close()
    ctx.close()
