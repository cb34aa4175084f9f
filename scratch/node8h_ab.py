"""k_node8 (8 waves, one slot per CU) against k_node8h (4 waves, two slots per CU): per-level times
of a batch under each form, same process, alternating.
    python scratch/node8h_ab.py MECH N KEY G TRIALS [reps]"""
import pathlib
import sys

REPO = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "gpr.jl_amd"), str(REPO)]
import numpy as np  # noqa: E402

import gprx  # noqa: E402
from gprx import _lib as L, data  # noqa: E402

mech, N, key, G, trials = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 5
trs = [data.make_trial(mech, N, 100, seed=data.trial_seed(mech, t)) for t in range(trials)]
Ysel = (lambda tr: tr["Xcurr"]) if G == 26 else (lambda tr: tr["Y"])
X = np.stack([tr["X"] for tr in trs for _ in range(G)])
Y = np.concatenate([Ysel(tr) for tr in trs])
XT = np.stack([tr["Xs"] for tr in trs for _ in range(G)])
B, d = X.shape[0], X.shape[1]
th = np.tile(data.theta0(mech, key), (B, 1))
ctx = gprx.Context(0)
b = gprx.GPBatch(B, d, N, 100, ctx=ctx)
b.set_train(X, Y)
b.set_test(XT)
res = {}
for rnd in range(2):
    for w in (8, 4):
        ctx.set_option(L.OPT_NODE_WAVES, w)
        r = b.run(th, grad=True, predict=True)
        r = b.run(th, grad=True, predict=True)
        ctx.set_profiling(True)
        ctx.reset_stats()
        for _ in range(reps):
            b.run(th, grad=True, predict=True)
        ctx.set_profiling(False)
        tot = 0.0
        parts = []
        for nm in ("gram", "node8/n8", "node8h/n8", "potrf_trsm/n16", "syrk_tt/n16", "trtri_linv21/n16", "alpha",
                   "lauum_grad", "pred_cross", "pred_var"):
            s = ctx.kernel_stats(nm)
            if s["launches"]:
                ms = s["ms"] / reps
                tot += ms
                parts.append(f"{nm} {ms:.3f}")
        res.setdefault(w, []).append(r)
        print(f"{mech} N={N} B={B} waves={w} round {rnd}: {' '.join(parts)} | sum {tot:.3f} ms = {B / tot * 1e3:.0f} fits/s",
              flush=True)
ctx.set_option(L.OPT_NODE_WAVES, 0)
same = all(np.array_equal(res[4][0][k], res[8][0][k]) for k in ("mll", "grad", "mu", "var"))
print("bit-identical:", same, flush=True)
