"""Timeline of the overlapped leaf (k_leaf8) on the bench workload, from a diagnostic build's
stamps (scratch/devbuild.sh l8stamps -DGPRX_STAMPS -DGPRX_NODE8=0 -DGPRX_LAUUM_FWD -DGPRX_SLOTWG_N=0):

    GPRX_LIB=scratch/var/libgprx_l8stamps.so python scratch/leaf8_timeline.py [trials]

Events (s_memrealtime, 100 MHz; median over slots, us from the leaf's start): 0 start; diagonal
wave: 1+2k / 2+2k start / end of tile k; task wave 0: 9+4k step k begins (tile k's inverse is
ready), 10+4k after the chain tasks (tile k+1 handed over), 11+4k after the other TRSM tasks and
inverse row k, 12+4k after the other SYRK tasks; 25 end.  Plus the diagonal routine's phases
(diag_ts) per tile."""
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
nd = 8 * 256 * 4 * 16
nw = 8 * 256 * 8 * 32
buf = np.zeros(n + nd + nw, dtype=np.uint64)
assert f(2, buf.ctypes.data, n + nd + nw, 0) == 0
ws = buf[n + nd:].reshape(8, 256, 8, 32).astype(np.float64)[:, : rb.n * bench.G]
ts = buf[:n].reshape(8, 256, 32).astype(np.float64)[:, : rb.n * bench.G]
ds = buf[n:n + nd].reshape(8, 256, 4, 16).astype(np.float64)[:, : rb.n * bench.G]
names = {0: "start", 25: "end"}
for k in range(4):
    names[1 + 2 * k], names[2 + 2 * k] = f"d{k}_start", f"d{k}_end"
    names[9 + 4 * k], names[10 + 4 * k], names[11 + 4 * k], names[12 + 4 * k] = (
        f"s{k}_begin", f"s{k}_chain_done", f"s{k}_trsm_inv_done", f"s{k}_syrk_done")
out = {}
for leaf in range(8):
    t = ts[leaf]
    if not (t[:, 0] > 0).all():
        continue
    row = {names[e]: round(float(np.median((t[:, e] - t[:, 0]) / 100.0)), 2) for e in sorted(names) if (t[:, e] > 0).all()}
    # the launch's spread: slots' start and end against the earliest start of the launch (us)
    t0 = t[:, 0].min()
    row["abs_start_p50_max"] = [round(float(np.percentile((t[:, 0] - t0) / 100.0, q)), 2) for q in (50, 100)]
    row["abs_end_p10_p50_p90_max"] = [round(float(np.percentile((t[:, 25] - t0) / 100.0, q)), 2) for q in (10, 50, 90, 100)]
    out[f"leaf{leaf}"] = row
    # the diagonal routine's phases per tile (durations, us): zero, then per P factor / TRSM / SYRK,
    # inverse off-diagonal blocks, logdet
    d = ds[leaf]
    if (d[:, :, 9] > 0).all() and not (d[:, :, 15] > 0).any():  # k_leaf9's diag_w1: 0, factor/panel per P, inverse
        dur = np.median(np.diff(d[:, :, :10], axis=2) / 100.0, axis=0)
        lab = [f"{x}{P}" for P in range(4) for x in ("fac", "panel")] + ["inv"]
        out[f"leaf{leaf}_diag"] = {f"tile{k}": dict(zip(lab, [round(float(v), 2) for v in dur[k]])) for k in range(4)}
    elif (d[:, :, 15] > 0).all():
        dur = np.median(np.diff(d, axis=2) / 100.0, axis=0)  # (4 tiles, 15)
        lab = ["zero"] + [f"{x}{P}" for P in range(4) for x in ("fac", "trsm", "syrk")] + ["inv", "logdet"]
        out[f"leaf{leaf}_diag"] = {f"tile{k}": dict(zip(lab, [round(float(v), 2) for v in dur[k]])) for k in range(4)}
    # phase B per wave (k_leaf9 W_TS): step k: 8k start, 8k+1.. after each item, 8k+7 end (us from leaf start)
    w = ws[leaf]
    if (w[:, 1:, 7] > 0).any():
        ph = {}
        for k in range(3):
            for wv in range(1, 8):
                t = w[:, wv, 8 * k: 8 * k + 8]
                if not (t[:, 0] > 0).all():
                    continue
                rel = (t - ts[leaf][:, :1]) / 100.0
                ph[f"s{k}_w{wv}"] = [round(float(np.median(rel[:, i])), 1) if (t[:, i] > 0).all() else None for i in range(8)]
        out[f"leaf{leaf}_phaseB"] = ph
        # round 5: step 0 per wave: 24 phase A start, 25 after the chain, 26 A items done, 27 after
        # the A barrier, 28 first B item's C loaded, 29 its products done (stamps build waits)
        a0 = {}
        for wv in range(1, 8):
            t = w[:, wv, 24:30]
            rel = (t - ts[leaf][:, :1]) / 100.0
            a0[f"w{wv}"] = [round(float(np.median(rel[:, i])), 1) if (t[:, i] > 0).all() else None for i in range(6)]
        out[f"leaf{leaf}_A0"] = a0
print(json.dumps(out, indent=1), flush=True)
