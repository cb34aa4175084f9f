"""Timeline of the fused leaf (k_leaf) on the bench workload, from the diagnostic build's stamps
(scratch/varbuild.sh stamps gpr.jl_amd/csrc/gprx_kernels.hip -DGPRX_STAMPS):

    GPRX_LIB=scratch/var/libgprx_stamps.so python scratch/leaf_timeline.py [trials]

Wave 0 of every leaf workgroup stamps s_memrealtime (100 MHz) at: 0 start; 1+3k after diagonal
tile k; 2+3k after step k's TRSM tasks; 3+3k after its SYRK tasks; 12+s after the inverse's
sub-diagonal s; 16 end.  Prints the median over slots of each phase's duration per leaf (us)."""
import ctypes as C
import json
import sys

import numpy as np

sys.path[:0] = ["/root/repo", "/root/repo/gpr.jl_amd"]
import bench  # noqa: E402
import gprx  # noqa: E402
from gprx import _lib as L  # noqa: E402
from gprx import shard  # noqa: E402

trials = int(sys.argv[1]) if len(sys.argv) > 1 else 40
f = L.lib.gprx_dbg_stamps
f.restype = C.c_int
f.argtypes = [C.c_int, C.c_void_p, C.c_longlong, C.c_int]
trs, X, Y, T, XT = bench.make_workload(trials, 0, 1)
rb = shard.RankBatch(trs, ctx=gprx.Context(0))
TH = T.reshape(rb.n, bench.G, -1)
for _ in range(3):
    rb.evaluate(TH)
assert f(2, None, 0, 1) == 0
rb.evaluate(TH)
n = 8 * 256 * 32
buf = np.zeros(n, dtype=np.uint64)
assert f(2, buf.ctypes.data, n, 0) == 0
ts = buf.reshape(8, 256, 32).astype(np.float64)[:, : rb.n * bench.G]
names = ["start"]
for k in range(4):
    names += [f"diag{k}", f"trsm{k}", f"syrk{k}"]
names += ["inv_s1", "inv_s2", "inv_s3", "end"]
out = {}
for leaf in range(8):
    t = ts[leaf]
    if not (t[:, 0] > 0).all():
        continue
    row = {}
    for ev in range(1, 17):
        d = (t[:, ev] - t[:, ev - 1]) / 100.0
        row[names[ev]] = round(float(np.median(d)), 2)
    row["total"] = round(float(np.median((t[:, 16] - t[:, 0]) / 100.0)), 2)
    row["spread_start_us"] = round(float((t[:, 0].max() - t[:, 0].min()) / 100.0), 2)
    out[f"leaf{leaf}"] = row
print(json.dumps(out, indent=1), flush=True)
