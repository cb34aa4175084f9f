"""CP (N=512, d=26, all 26 outputs) per-kernel times per batch for leaf / small_n choices."""
import os, sys, time
sys.path[:0] = ['/root/repo', '/root/repo/gpr.jl_amd']
import numpy as np, gprx
from gprx import data
trials = int(os.environ.get('CP_TRIALS', 16))
trs = [data.make_trial('CP', 512, 100, seed=data.trial_seed('CP', t)) for t in range(trials)]
X = np.stack([tr['X'] for tr in trs for _ in range(26)]); Y = np.concatenate([tr['Xcurr'] for tr in trs])
XT = np.stack([tr['Xs'] for tr in trs for _ in range(26)])
B = X.shape[0]
th = np.tile(data.theta0('CP', 512), (B, 1))
names = ('gram', 'leaf', 'diag', 'potrf_trsm', 'syrk_tt', 'trtri_linv21', 'alpha', 'lauum_grad', 'finalize', 'pred_cross', 'pred_var', 'pred_mu', 'pred_final')
for arg in sys.argv[1:] or ['0,0']:
    leaf, small = (int(v) for v in arg.split(','))
    ctx = gprx.Context(0); ctx.set_option(gprx.OPT_LEAF_TILES, leaf); ctx.set_option(gprx.OPT_SMALL_N, small)
    b = gprx.GPBatch(B, 26, 512, 100, ctx=ctx); b.set_train(X, Y); b.set_test(XT)
    b.run(th, grad=True, predict=True)
    t0 = time.perf_counter()
    for _ in range(5): r = b.run(th, grad=True, predict=True)
    dt = (time.perf_counter() - t0) / 5
    ctx.set_profiling(True); ctx.reset_stats()
    for _ in range(3): b.run(th, grad=True, predict=True)
    ks = {k: round(ctx.kernel_stats(k)['ms'] / 3, 3) for k in names}
    print(f'leaf {leaf} small_n {small}: {dt*1e3:.2f} ms/batch {B/dt:.0f} fits/s', {k: v for k, v in ks.items() if v}, flush=True)
    b.close(); ctx.close()
