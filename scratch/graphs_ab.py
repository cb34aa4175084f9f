"""Step time of the bench workload with direct launches vs the captured hipGraph replay
(GPRX_OPT_GRAPHS), alternating, REPS x STEPS evaluations each: python scratch/graphs_ab.py [reps] [steps]"""
import sys
import time

sys.path[:0] = ["/root/repo", "/root/repo/gpr.jl_amd"]
import bench  # noqa: E402
import gprx  # noqa: E402
from gprx import _lib as L  # noqa: E402
from gprx import shard  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
trs, X, Y, T, XT = bench.make_workload(40, 0, 1)
ctx = gprx.Context(0)
rb = shard.RankBatch(trs, ctx=ctx)
TH = T.reshape(rb.n, bench.G, -1)
res = {0: [], 1: []}
for r in range(reps):
    for g in (0, 1):
        ctx.set_option(L.OPT_GRAPHS, g)
        for _ in range(2):
            rb.evaluate(TH)
        t0 = time.perf_counter()
        for _ in range(steps):
            rb.evaluate(TH)
        res[g].append((time.perf_counter() - t0) / steps * 1e3)
for g in (0, 1):
    print(f"graphs={g} ms/step", [round(v, 3) for v in res[g]], flush=True)
