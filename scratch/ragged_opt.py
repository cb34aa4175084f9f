"""Ragged device optimisation: B=192 P2 N=512 GPs from jittered starts, Optim defaults (g_tol 1e-8,
f_calls_limit 80): rounds, time, and the per-round active-slot profile (GPRX_LIB selects the build)."""
import sys, time
sys.path[:0] = ['/root/repo', '/root/repo/gpr.jl_amd']
import numpy as np, gprx
from gprx import data
import gprx.optim as OP
B, N = 192, 512
trs = [data.make_trial('P2', N, 0, seed=data.trial_seed('P2', t)) for t in range(B // 6)]
X = np.stack([trs[s // 6]['X'] for s in range(B)]); Y = np.stack([trs[s // 6]['Y'][s % 6] for s in range(B)])
rng = np.random.default_rng(3)
th0 = data.theta0('P2', N)
T = np.stack([th0 + 0.3 * rng.standard_normal(th0.shape[0]) for _ in range(B)])
b = gprx.GPBatch(B, 26, N, 0); b.set_train(X, Y)
b.optimize(T[:, :], OP.LBFGS(), OP.Options(max_evals=4))  # warm-up (graph capture)
t0 = time.time()
res, rounds = b.optimize(T, OP.LBFGS(), OP.Options(max_evals=80))
dt = time.time() - t0
fc = np.array([r.f_calls for r in res])
print('rounds', rounds, 'seconds', round(dt, 3), 'f_calls min/median/max', fc.min(), int(np.median(fc)), fc.max(),
      'stops', {s: sum(r.stopped_by == s for r in res) for s in set(r.stopped_by for r in res)}, flush=True)
