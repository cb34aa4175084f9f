"""Per-level kernel times (library HIP-event profiling) of one BASELINE configuration:
    python scratch/levels_cfg.py MECH N KEY G TRIALS [reps]"""
import pathlib
import sys

REPO = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "gpr.jl_amd"), str(REPO)]
import numpy as np  # noqa: E402

import gprx  # noqa: E402
from gprx import data  # noqa: E402

mech, N, key, G, trials = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
reps = int(sys.argv[6]) if len(sys.argv) > 6 else 3
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
for _ in range(2):
    b.run(th, grad=True, predict=True)
ctx.set_profiling(True)
ctx.reset_stats()
for _ in range(reps):
    b.run(th, grad=True, predict=True)
ctx.set_profiling(False)
names = ["gram", "leaf/n4", "leaf/n2", "node8/n8", "diag"]
for op in ("potrf_trsm", "syrk_tt", "trtri_linv21"):
    names += [f"{op}/n{n}" for n in (64, 32, 16, 8, 4, 2)]
names += ["alpha", "lauum_grad", "finalize", "pred_cross", "pred_var", "pred_final"]
tot = 0.0
print(f"{mech} N={N} d={d} B={B}")
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
    print(f"{nm:22s} {ms:8.3f} ms/batch {s['launches'] // reps:3d} launches {1e3 * s['ms'] / s['launches']:9.1f} us/launch {tf:6.1f} TF/s",
          flush=True)
print(f"{'sum':22s} {tot:8.3f} ms/batch")
