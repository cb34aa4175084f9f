"""Per-wave timeline of one GEMM launch (or, with GPRX_GSTAMPS=999, of the gradient GEMM k_lauum_grad) of the bench workload, from a -DGPRX_GSTAMPS=op*100+n
diagnostic build (scratch/varbuild.sh gts_NAME scratch/var/k_gts.hip -DGPRX_GSTAMPS=...):

    GPRX_LIB=scratch/var/libgprx_gts_NAME.so python scratch/gemm_timeline.py [trials]

Every wave stamps s_memrealtime (100 MHz, after its memory operations landed) at tile entry, core
start, core end and epilogue end, for its first two tiles.  Prints the launch span and the medians
(and 90th percentiles) of each phase in us."""
import ctypes as C
import json
import sys

import numpy as np

sys.path[:0] = ["/root/repo", "/root/repo/gpr.jl_amd"]
import bench  # noqa: E402
import gprx  # noqa: E402
from gprx import _lib as L  # noqa: E402
from gprx import shard  # noqa: E402

trials = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 40
f = L.lib.gprx_dbg_gts
f.restype = C.c_int
f.argtypes = [C.c_void_p, C.c_longlong, C.c_int]
trs, X, Y, T, XT = bench.make_workload(trials, 0, 1)
rb = shard.RankBatch(trs, ctx=gprx.Context(0))
TH = T.reshape(rb.n, bench.G, -1)
for _ in range(3):
    rb.evaluate(TH)
assert f(None, 0, 1) == 0
rb.evaluate(TH)
n = (1 << 17) * 8
buf = np.zeros(n, dtype=np.uint64)
assert f(buf.ctypes.data, n, 0) == 0
t = buf.reshape(-1, 8).astype(np.float64)
t = t[t[:, 0] > 0]
t0 = t[:, 0].min()
us = lambda a: (a / 100.0)  # noqa: E731


def stat(a):
    return [round(float(np.median(a)), 2), round(float(np.percentile(a, 90)), 2)]


if "--lau2" in sys.argv:  # unit 0 detail (GPRX_GSTAMPS=998)
    t = t[t[:, 3] > 0]
    out = {"waves": int(len(t))}
    for name, a, b in (("pre", 0, 1), ("main", 1, 2), ("sync1", 2, 4), ("alpha_sync2", 4, 5), ("G_kf", 5, 6),
                       ("sums_Q", 6, 7), ("tail_sync3", 7, 3)):
        ok = (t[:, a] > 0) & (t[:, b] > 0)
        out[name] = stat(us(t[ok, b] - t[ok, a]))
    print(json.dumps(out), flush=True)
    sys.exit(0)
if "--lauum" in sys.argv:  # entry, then per unit: main start, main end, unit end
    t = t[t[:, 3] > 0]
    out = {"waves": int(len(t))}
    out["u0_pre"] = stat(us(t[:, 1] - t[:, 0]))
    out["u0_main"] = stat(us(t[:, 2] - t[:, 1]))
    out["u0_epilogue"] = stat(us(t[:, 3] - t[:, 2]))
    two = t[t[:, 6] > 0]
    out["u1_gap"] = stat(us(two[:, 4] - two[:, 3]))
    out["u1_main"] = stat(us(two[:, 5] - two[:, 4]))
    out["u1_epilogue"] = stat(us(two[:, 6] - two[:, 5]))
    end = np.where(t[:, 6] > 0, t[:, 6], t[:, 3])
    out["job_life"] = stat(us(end - t[:, 0]))
    out["span_us"] = round(us(end.max() - t0), 1)
    print(json.dumps(out), flush=True)
    sys.exit(0)
out = {"waves": int(len(t)), "span_us": round(us(np.nanmax(np.where(t[:, 7] > 0, t[:, 7], t[:, 3])) - t0), 1)}
out["entry_us"] = stat(us(t[:, 0] - t0))
out["p0_prologue"] = stat(us(t[:, 1] - t[:, 0]))
out["p0_core"] = stat(us(t[:, 2] - t[:, 1]))
out["p0_epilogue"] = stat(us(t[:, 3] - t[:, 2]))
two = t[t[:, 4] > 0]
if len(two):
    out["two_tile_waves"] = int(len(two))
    out["p1_gap"] = stat(us(two[:, 4] - two[:, 3]))
    out["p1_prologue"] = stat(us(two[:, 5] - two[:, 4]))
    out["p1_core"] = stat(us(two[:, 6] - two[:, 5]))
    out["p1_epilogue"] = stat(us(two[:, 7] - two[:, 6]))
end = np.where(t[:, 7] > 0, t[:, 7], t[:, 3])
out["wave_life"] = stat(us(end - t[:, 0]))
out["end_us"] = stat(us(end - t0))
print(json.dumps(out), flush=True)
