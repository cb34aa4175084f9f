"""Phase timeline of the whole-8-tile-node kernels (k_node8: 8 waves, k_node8h: 4 waves) on one
batch, from a stamps build (scratch/varbuild.sh nstamps ../gpr.jl_amd/csrc/gprx_kernels.hip -DGPRX_STAMPS):
    GPRX_LIB=scratch/var/libgprx_nstamps.so python scratch/node_timeline.py MECH N KEY G TRIALS
Per form: median phase durations per slot (us) and, per CU, how many slots overlap in time."""
import collections
import ctypes as C
import pathlib
import sys

REPO = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "gpr.jl_amd"), str(REPO)]
import numpy as np  # noqa: E402

import gprx  # noqa: E402
from gprx import _lib as L, data  # noqa: E402

mech, N, key, G, trials = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
f = L.lib.gprx_dbg_stamps
f.restype = C.c_int
f.argtypes = [C.c_int, C.c_void_p, C.c_longlong, C.c_int]
trs = [data.make_trial(mech, N, 100, seed=data.trial_seed(mech, t)) for t in range(trials)]
Ysel = (lambda tr: tr["Xcurr"]) if G == 26 else (lambda tr: tr["Y"])
X = np.stack([tr["X"] for tr in trs for _ in range(G)])
Y = np.concatenate([Ysel(tr) for tr in trs])
B, d = X.shape[0], X.shape[1]
th = np.tile(data.theta0(mech, key), (B, 1))
ctx = gprx.Context(0)
b = gprx.GPBatch(B, d, N, 0, ctx=ctx)
b.set_train(X, Y)
for w in (8, 4):
    ctx.set_option(L.OPT_NODE_WAVES, w)
    for _ in range(2):
        b.run(th, grad=False)
    assert f(0, None, 0, 1) == 0
    b.run(th, grad=False)
    buf = np.zeros(524288 + 32768 * 8, dtype=np.uint64)
    assert f(0, buf.ctypes.data, buf.size, 0) == 0
    st = buf[524288:524288 + B * 8].reshape(B, 8)
    t = st[:, :6].astype(np.float64) / 100.0  # us
    dur = np.diff(t, axis=1)
    names = ["leaf_top", "trsm", "syrk_tt", "leaf_bot", "linv21"]
    med = {n: round(float(np.median(dur[:, i])), 1) for i, n in enumerate(names)}
    tot = t[:, 5] - t[:, 0]
    hw, xcc = st[:, 6], st[:, 7]
    cu = [(int(xcc[s]) & 15, int(hw[s] >> 13) & 7, int(hw[s] >> 12) & 1, int(hw[s] >> 8) & 15) for s in range(B)]
    by = collections.defaultdict(list)
    for s in range(B):
        by[cu[s]].append((t[s, 0], t[s, 5], s))
    ov = collections.Counter()
    for k, v in by.items():
        for i, (a0, a1, _) in enumerate(v):
            ov[sum(1 for (b0, b1, _) in v if b0 < a1 and a0 < b1) - 1] += 1
    span = (t[:, 5].max() - t[:, 0].min())
    print(f"waves={w} B={B}: per-slot median {med}, node {np.median(tot):.1f} us (p10 {np.percentile(tot, 10):.1f}, "
          f"p90 {np.percentile(tot, 90):.1f}); launch span {span:.1f} us; CUs {len(by)}; slots overlapping k others: "
          f"{dict(sorted(ov.items()))}", flush=True)
ctx.set_option(L.OPT_NODE_WAVES, 0)
