"""Bit-for-bit output check between library builds: evaluates the bench workload (P2, N=2048, trials
x 6 slots, plus a B < 32 batch that takes the single-tile diagonal path) with gradient and
prediction and prints one SHA-256 over every output array.  Run once per library (GPRX_LIB selects
a variant build) and compare the lines:  python scratch/bitcmp.py [trials]"""
import hashlib
import sys

sys.path[:0] = ["/root/repo", "/root/repo/gpr.jl_amd"]
import numpy as np  # noqa: E402

import bench  # noqa: E402
import gprx  # noqa: E402
from gprx import data  # noqa: E402

trials = int(sys.argv[1]) if len(sys.argv) > 1 else 8
_, X, Y, T, XT = bench.make_workload(trials, 0, 1)
ctx = gprx.Context(0)
h = hashlib.sha256()
b = gprx.GPBatch(X.shape[0], 26, 2048, 100, ctx=ctx)
b.set_train(X, Y)
b.set_test(XT)
r = b.run(T, grad=True, predict=True)
for k in ("mll", "grad", "mu", "var", "status", "info"):
    h.update(np.ascontiguousarray(r[k]).tobytes())
b.close()
# small batch (B = 6 < 32): leaf size 1, the standalone diagonal kernel
tr = data.make_trial("P2", 700, 16, seed=3)
th = np.tile(data.theta0("P2", 512), (6, 1))  # the config holds theta per experiment size
b = gprx.GPBatch(6, tr["d"], 700, 16, ctx=ctx)
b.set_train(tr["X"], tr["Y"])
b.set_test(tr["Xs"])
r2 = b.run(th, grad=True, predict=True)
for k in ("mll", "grad", "mu", "var", "status"):
    h.update(np.ascontiguousarray(r2[k]).tobytes())
print("outputs sha256", h.hexdigest()[:32], "status", int(np.sum(r["status"])), "mll0", repr(float(r["mll"][0])))
