"""Where a batch call's wall time goes beyond the kernels (CP B=1014 or P1): python scratch/host_overhead.py MECH N KEY G TRIALS"""
import ctypes as C
import pathlib
import sys
import time

REPO = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "gpr.jl_amd"), str(REPO)]
import numpy as np  # noqa: E402

import gprx  # noqa: E402
from gprx import _lib as L, data  # noqa: E402

mech, N, key, G, trials = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5])
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


def wall(fn, n=20):
    for _ in range(3):
        fn()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    return (time.perf_counter() - t0) / n * 1e3


M = XT.shape[2]
mll, g = np.empty(B), np.empty((B, d + 2))
mu, var = np.empty((B, M)), np.empty((B, M))
from gprx.batch import host_empty  # noqa: E402
pmu, pvar = host_empty((B, M)), host_empty((B, M))
st, info = np.empty(B, dtype=np.int32), np.empty(B, dtype=np.int32)
thc = np.ascontiguousarray(th)


def raw(pred=True, var_on=True, pinned=False):
    flags = L.WANT_GRAD | (L.WANT_PREDICT if pred else 0)
    m_, v_ = (pmu, pvar) if pinned else (mu, var)
    L.lib.gprx_batch_run(b.h, L.dptr(thc), flags, L.dptr(mll), L.dptr(g), L.dptr(m_) if pred else None,
                         L.dptr(v_) if (pred and var_on) else None, L.iptr(st), L.iptr(info))


print(f"{mech} N={N} B={B} M={M}")
print(f"GPBatch.run grad+pred      {wall(lambda: b.run(th, grad=True, predict=True)):.3f} ms")
print(f"raw C call grad+pred       {wall(lambda: raw(True)):.3f} ms")
print(f"raw C call grad+pred (mean){wall(lambda: raw(True, False)):.3f} ms")
print(f"raw C call grad+pred pinned{wall(lambda: raw(True, True, True)):.3f} ms")
raw(True, True, False)
m0, v0 = mu.copy(), var.copy()
raw(True, True, True)
print("pinned outputs equal:", np.array_equal(m0, pmu) and np.array_equal(v0, pvar))
print(f"raw C call grad only       {wall(lambda: raw(False)):.3f} ms")
ctx.set_profiling(True)
ctx.reset_stats()
n = 10
for _ in range(n):
    raw(True)
ctx.set_profiling(False)
tot = 0.0
for nm in ("gram", "node8/n8", "leaf/n4", "alpha", "lauum_grad", "finalize", "pred_cross", "pred_var", "pred_final"):
    s = ctx.kernel_stats(nm)
    tot += s["ms"] / n
print(f"kernel sum (events)        {tot:.3f} ms")
