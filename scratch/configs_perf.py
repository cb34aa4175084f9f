"""fits/s of the four BASELINE configurations (fit = Gram+Cholesky+alpha+LML, full gradient,
mean+variance at M=100), one batch per call."""
import sys, time
sys.path.insert(0, '/root/repo/gpr.jl_amd'); sys.path.insert(0, '/root/repo')
import numpy as np, gprx
from gprx import data
ctx = gprx.Context(0)
cases = [(m, n, k, g, t) for m, n, k, g, t in [("P1", 50, 64, 3, 256), ("CP", 512, 512, 26, 8), ("CP", 512, 512, 26, 16), ("P2", 2048, 2048, 6, 32), ("FB", 4096, 512, 12, 4), ("FB", 4096, 512, 12, 8)]]
for mech, N, key, G, trials in cases:
    trs = [data.make_trial(mech, N, 100, seed=data.trial_seed(mech, t)) for t in range(trials)]
    Ysel = (lambda tr: tr["Xcurr"]) if G == 26 else (lambda tr: tr["Y"])
    X = np.stack([tr["X"] for tr in trs for _ in range(G)])
    Y = np.concatenate([Ysel(tr) for tr in trs])
    XT = np.stack([tr["Xs"] for tr in trs for _ in range(G)])
    B = X.shape[0]; d = X.shape[1]
    th = np.tile(data.theta0(mech, key), (B, 1))
    b = gprx.GPBatch(B, d, N, 100, ctx=ctx); b.set_train(X, Y); b.set_test(XT)
    r = b.run(th, grad=True, predict=True)
    n = 5 if N <= 2048 else 3
    t0 = time.perf_counter()
    for _ in range(n): r = b.run(th, grad=True, predict=True)
    dt = (time.perf_counter() - t0) / n
    print(f"{mech} N={N} d={d} B={B} ({trials} trials x {G} GPs): {dt*1e3:.2f} ms/batch  {B/dt:.1f} fits/s  ok={int((r['status']==0).sum())}/{B}", flush=True)
    b.close()
