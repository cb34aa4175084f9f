"""Device vs oracle on overflowing hyperparameters (exp(2 log sf) = Inf, exp(-2 log ell) = Inf)."""
import sys
sys.path[:0] = ['/root/repo', '/root/repo/gpr.jl_amd']
import numpy as np, gprx
from oracle import gp_oracle as O
z = np.load('/root/repo/tests/golden/p1_n50.npz')
X, Y, th = z['X'], z['Y'], z['theta']
cases = {'sf_inf': (-1, 400.0), 'ell0_zero': (1, -400.0), 'noise_inf': (0, 400.0), 'sf_tiny': (-1, -400.0)}
b = gprx.GPBatch(1, X.shape[0], X.shape[1], 0)
b.set_train(X, Y[:1])
for name, (i, v) in cases.items():
    t = th.copy(); t[i] = v
    r = b.run(t[None], grad=True)
    try:
        m, g, _ = O.lml(X, Y[0], t, want_grad=True)
        ref = ('ok', m)
    except O.NotPosDef as e:
        ref = ('notpd', e.info)
    print(name, 'device status', int(r['status'][0]), 'info', int(r['info'][0]), 'mll', float(r['mll'][0]), '| oracle', ref, flush=True)
