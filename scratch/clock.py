"""In-kernel clock of the lauum and top-level SYRK/TT main loops on the bench workload
(MI355X_MICROARCH.md 'DVFS give-back' item 6): run with the diagnostic library
(scratch/varbuild.sh stamps gpr.jl_amd/csrc/gprx_kernels.hip -DGPRX_STAMPS):

    GPRX_LIB=scratch/var/libgprx_stamps.so python scratch/clock.py [trials] [seconds]

Evaluates the workload back to back for >= `seconds`, clears the stamps, evaluates once more and
reports per region the median over waves of clock = d(s_memtime) / d(s_memrealtime) x 100 MHz and
the main-loop cycles per MFMA (the 64 x 64 core issues K / 4 x 16 MFMAs per wave)."""
import ctypes as C
import json
import sys
import time

import numpy as np

sys.path[:0] = ["/root/repo", "/root/repo/gpr.jl_amd"]
import bench  # noqa: E402
import gprx  # noqa: E402
from gprx import _lib as L  # noqa: E402

trials = int(sys.argv[1]) if len(sys.argv) > 1 else 40
secs = float(sys.argv[2]) if len(sys.argv) > 2 else 3.0
f = L.lib.gprx_dbg_stamps
f.restype = C.c_int
f.argtypes = [C.c_int, C.c_void_p, C.c_longlong, C.c_int]
trs, X, Y, T, XT = bench.make_workload(trials, 0, 1)
ctx = gprx.Context(0)
from gprx import shard  # noqa: E402

rb = shard.RankBatch(trs, ctx=ctx)
TH = T.reshape(rb.n, bench.G, -1)
t0 = time.perf_counter()
n = 0
while time.perf_counter() - t0 < secs:
    rb.evaluate(TH)
    n += 1
NW = 1 << 18
out = {"evals_before": n, "seconds_before": round(time.perf_counter() - t0, 2)}
for reg in (0, 1):
    assert f(reg, None, 0, 1) == 0
rb.evaluate(TH)
for reg, name in ((0, "lauum_main_loop"), (1, "top_syrk_tt_main_loop")):
    buf = np.zeros((NW, 4), dtype=np.uint64)
    assert f(reg, buf.ctypes.data, NW * 4, 0) == 0
    buf = buf[buf[:, 1] > 0].astype(np.float64)
    dt = buf[:, 1] - buf[:, 0]
    dr = buf[:, 3] - buf[:, 2]
    ok = dr > 0
    clk = dt[ok] / dr[ok] * 100e6 / 1e9
    out[name] = {"waves": int(ok.sum()), "clock_ghz_median": round(float(np.median(clk)), 4),
                 "clock_ghz_p10_p90": [round(float(np.percentile(clk, 10)), 4), round(float(np.percentile(clk, 90)), 4)],
                 "wave_us_median": round(float(np.median(dr[ok])) / 100.0, 2)}
print(json.dumps(out), flush=True)
