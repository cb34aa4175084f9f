"""Optimised GP fits/s per configuration: device optimiser (k_lbfgs, GPBatch.optimize, with the
closing refit) against the host lock-step restatement (gprx.optim.optimize_batch), same batch,
same 30-evaluation budget per GP; both must give bit-identical minimisers."""
import sys, time
sys.path.insert(0, '/root/repo/gpr.jl_amd'); sys.path.insert(0, '/root/repo')
import numpy as np, gprx
from gprx import data
from gprx.optim import LBFGS, Options, optimize_batch
ctx = gprx.Context(0)
cases = [("P1", 50, 64, 3, 256), ("CP", 512, 512, 4, 32), ("CP", 512, 512, 26, 8), ("P2", 2048, 2048, 6, 32)]
o = Options(max_evals=30)
for mech, N, key, G, trials in cases:
    trs = [data.make_trial(mech, N, 0, seed=data.trial_seed(mech, t)) for t in range(trials)]
    Ysel = (lambda tr: tr["Xcurr"]) if G == 26 else (lambda tr: tr["Y"])
    X = np.stack([tr["X"] for tr in trs for _ in range(G)])
    Y = np.concatenate([Ysel(tr) for tr in trs])
    B, d = X.shape[0], X.shape[1]
    rng = np.random.default_rng(3)
    th = np.tile(data.theta0(mech, key), (B, 1)) + 0.05 * rng.standard_normal((B, d + 2))
    b = gprx.GPBatch(B, d, N, 0, ctx=ctx); b.set_train(X, Y)
    b.optimize(th, LBFGS(), Options(max_evals=4))  # warm-up (graph capture)
    t0 = time.perf_counter(); hres, hr = optimize_batch(b, th, LBFGS(), o); th_ = time.perf_counter() - t0
    t0 = time.perf_counter(); dres, dr = b.optimize(th, LBFGS(), o); td = time.perf_counter() - t0
    same = all(np.array_equal(a.minimizer, c.minimizer) and a.minimum == c.minimum for a, c in zip(dres, hres))
    print(f"{mech} N={N} d={d} B={B}: device {td*1e3:.1f} ms ({dr} rounds + refit, {B/td:.0f} opt-fits/s) | "
          f"host {th_*1e3:.1f} ms ({hr} rounds, {B/th_:.0f} opt-fits/s) | speedup {th_/td:.2f}x | identical={same}", flush=True)
    b.close()
