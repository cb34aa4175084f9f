"""Per-wave timeline of k_node8's SYRK + TT phase on the bench workload, from a -DGPRX_GSTAMPS=1208
diagnostic build (scratch/varbuild.sh gts1208 ../gpr.jl_amd/csrc/gprx_kernels.hip -DGPRX_GSTAMPS=1208):
    GPRX_LIB=scratch/var/libgprx_gts1208.so python scratch/node8_gts.py [trials]
Per tile of a wave's plan list (<= 4): entry -> core start (prologue: the SYRK's C loads), core
(loads landed), epilogue (stores landed), in us (medians over the waves of the last node launch)."""
import ctypes as C
import sys

import numpy as np

sys.path[:0] = ["/root/repo", "/root/repo/gpr.jl_amd"]
import bench  # noqa: E402
import gprx  # noqa: E402
from gprx import _lib as L  # noqa: E402
from gprx import shard  # noqa: E402

trials = int(sys.argv[1]) if len(sys.argv) > 1 else 40
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
B = rb.n * bench.G
n = B * 8 * 16
buf = np.zeros(n, dtype=np.uint64)
assert f(buf.ctypes.data, n, 0) == 0
t = buf.reshape(B, 8, 4, 4).astype(np.float64) / 100.0  # us; the last node launch's stamps
ok = t[..., 0] > 0
for k in range(4):
    m = ok[:, :, k] & (t[:, :, k, 3] > 0)
    if not m.any():
        continue
    pro = (t[:, :, k, 1] - t[:, :, k, 0])[m]
    core = (t[:, :, k, 2] - t[:, :, k, 1])[m]
    epi = (t[:, :, k, 3] - t[:, :, k, 2])[m]
    print(f"tile {k}: waves {m.sum()}, prologue {np.median(pro):.2f}, core {np.median(core):.2f} (p90 {np.percentile(core, 90):.2f}), "
          f"epilogue {np.median(epi):.2f} us", flush=True)
    if k > 0:
        gap = (t[:, :, k, 0] - t[:, :, k - 1, 3])[m & ok[:, :, k - 1]]
        print(f"   gap after tile {k - 1}: {np.median(gap):.2f} us")
first = np.where(ok[..., 0], t[..., 0, 0], np.inf).min(axis=1)
last = np.max(np.where(t[..., 3] > 0, t[..., 3], 0), axis=(1, 2))
wend = np.max(np.where(t[..., 3] > 0, t[..., 3], 0), axis=2)  # per wave
wstart = np.where(ok[..., 0], t[..., 0, 0], np.inf)
print(f"phase span per slot: median {np.median(last - first):.1f} us; per-wave busy median {np.median(wend - wstart):.1f}, "
      f"spread of wave ends within a slot (max-min) median {np.median(wend.max(1) - wend.min(1)):.1f} us", flush=True)
