import sys
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/gpr.jl_amd')
import numpy as np, gprx
from gprx import data
from oracle import gp_oracle as O
ctx = gprx.Context(0)
for N in [33, 63, 64, 65, 127, 130, 200]:
    B, M = 3, 7
    trs = [data.make_trial("CP", N, M, seed=200 + s) for s in range(B)]
    X = np.stack([t["X"] for t in trs]); Y = np.stack([t["Y"][s % 4] for s, t in enumerate(trs)])
    Xs = np.stack([t["Xs"] for t in trs])
    rng = np.random.default_rng(N)
    th = np.stack([data.theta0("CP", 512) + 0.1 * rng.standard_normal(28) for _ in range(B)])
    for mode in (0, 1):
        ctx.set_dist_mode(mode)
        b = gprx.GPBatch(B, 26, N, M, ctx=ctx); b.set_train(X, Y); b.set_test(Xs)
        r = b.run(th, grad=True, predict=True); b.close()
        for s in range(B):
            f = O.fit(X[s], Y[s], th[s], Xs[s], mode); f2 = O.fit(X[s], Y[s], th[s], Xs[s], 1 - mode)
            print(f"N={N:4d} mode={mode} s={s}: dmll={abs(r['mll'][s]-f['mll']):.2e} modes={abs(f['mll']-f2['mll']):.2e} "
                  f"sens={f['mll_sens']:.2e} |mll|={abs(f['mll']):.2e} dmu={np.max(np.abs(r['mu'][s]-f['mu'])):.2e}", flush=True)
