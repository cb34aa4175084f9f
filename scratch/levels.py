"""Per-recursion-level kernel times of the bench workload (P2, N=2048, B = trials x 6) from the
library's HIP-event profiling: python scratch/levels.py [trials] [reps]"""
import sys

sys.path.insert(0, "/root/repo/gpr.jl_amd")
sys.path.insert(0, "/root/repo")
import bench
import gprx

trials = int(sys.argv[1]) if len(sys.argv) > 1 else 32
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
_, X, Y, T, XT = bench.make_workload(trials, 0, 1)
ctx = gprx.Context(0)
import os
from gprx import _lib as L
if os.environ.get("SMALL_N"):
    ctx.set_option(L.OPT_SMALL_N, int(os.environ["SMALL_N"]))
if os.environ.get("LEAF"):
    ctx.set_option(L.OPT_LEAF_TILES, int(os.environ["LEAF"]))
b = gprx.GPBatch(X.shape[0], 26, 2048, 100, ctx=ctx)
b.set_train(X, Y)
b.set_test(XT)
for _ in range(2):
    b.run(T, grad=True, predict=True)
ctx.set_profiling(True)
ctx.reset_stats()
for _ in range(reps):
    b.run(T, grad=True, predict=True)
ctx.set_profiling(False)
names = ["gram", "leaf/n4", "leaf/n2", "node8/n8", "diag"]
for op in ("potrf_trsm", "syrk_tt", "trtri_linv21"):
    names += [f"{op}/n{n}" for n in (32, 16, 8, 4, 2)]
names += ["alpha", "lauum_grad", "finalize", "pred_cross", "pred_var", "pred_mu", "pred_final"]
tot = 0.0
for nm in names:
    try:
        s = ctx.kernel_stats(nm)
    except Exception:
        continue
    if s["launches"] == 0:
        continue
    ms = s["ms"] / reps
    tot += ms
    tf = s["flops"] / (s["ms"] * 1e-3) / 1e12 if s["ms"] > 0 else 0.0
    print(f"{nm:22s} {ms:8.3f} ms/step  {s['launches'] // reps:3d} launches  {1e3 * s['ms'] / s['launches']:8.1f} us/launch  {tf:6.1f} TF/s", flush=True)
print(f"{'sum':22s} {tot:8.3f} ms/step")
