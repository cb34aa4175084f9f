# quick GPU parity check against the oracle (scratch, first bring-up)
import sys, time, pathlib
sys.path.insert(0, '/root/repo/gpr.jl_amd'); sys.path.insert(0, '/root/repo')
import numpy as np
import gprx
from gprx import data
from oracle import gp_oracle as O

def check(mech, N, M, B=2, mode=0, key=None, seed=1):
    tr = data.make_trial(mech, N, M, seed=seed)
    d = tr['d']; X = tr['X']; Y = tr['Y'][:B] if tr['Y'].shape[0] >= B else np.repeat(tr['Y'][:1], B, 0)
    th0 = data.theta0(mech, key)
    rng = np.random.default_rng(seed)
    thetas = np.stack([th0 + 0.05 * rng.standard_normal(d + 2) for _ in range(B)])
    ctx = gprx.default_context(); ctx.set_dist_mode(mode)
    b = gprx.GPBatch(B, d, N, M)
    b.set_train(X, Y); b.set_test(tr['Xs'])
    t0 = time.time(); r = b.run(thetas, grad=True, predict=True); t1 = time.time()
    worst = {}
    for s in range(B):
        o = O.fit(X, Y[s], thetas[s], tr['Xs'], mode)
        e_m = abs(r['mll'][s] - o['mll']) / max(1, abs(o['mll']))
        e_g = np.max(np.abs(r['grad'][s] - o['grad'])) / max(1, np.max(np.abs(o['grad'])))
        e_mu = np.max(np.abs(r['mu'][s] - o['mu'])) / max(1e-300, np.max(np.abs(Y[s])))
        e_v = np.max(np.abs(r['var'][s] - o['var'])) / max(1e-300, np.exp(2*thetas[s][-1]))
        for k, v in dict(mll=e_m, grad=e_g, mu=e_mu, var=e_v).items(): worst[k] = max(worst.get(k, 0), v)
    print(f"{mech} N={N} M={M} B={B} mode={mode}: status={r['status'].tolist()} t={t1-t0:.3f}s rel-err {worst}", flush=True)

check('P1', 50, 8, B=3, key=64)
check('P1', 50, 8, B=3, key=64, mode=1)
check('CP', 130, 20, B=4, key=128)
check('CP', 512, 100, B=4, key=512)
check('P2', 256, 100, B=6, key=256)
check('FB', 200, 30, B=8, key=256)
check('P2', 2048, 100, B=2, key=2048)
