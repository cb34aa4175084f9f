"""Relative LML error of the device path vs the oracle on the well-conditioned configs (sets the
1e-10 bound of tests/test_gpu.py)."""
import sys
sys.path[:0] = ['/root/repo', '/root/repo/gpr.jl_amd']
import numpy as np, gprx
from gprx import data
from oracle import gp_oracle as O
ctx = gprx.Context(0)
for mode in (0, 1):
    ctx.set_dist_mode(mode)
    tag = 'exp' if mode == 0 else 'dir'
    for name in ['p1_n50', 'p2_n100', 'p2_n256', 'fb_n64', 'cp_n64']:
        z = np.load(f'/root/repo/tests/golden/{name}.npz')
        G = z['Y'].shape[0]
        b = gprx.GPBatch(G, z['X'].shape[0], z['X'].shape[1], 0, ctx=ctx); b.set_train(z['X'], z['Y'])
        r = b.run(np.tile(z['theta'], (G, 1)))
        ref = z[f'mll_{tag}']
        print(name, tag, 'max rel', float(np.max(np.abs(r['mll'] - ref) / np.maximum(1, np.abs(ref)))), flush=True)
        b.close()
ctx.set_dist_mode(1)
for mech, N, key in [('P2', 2048, 2048), ('FB', 4096, 512), ('P1', 512, 512)]:
    tr = data.make_trial(mech, N, 0, seed=data.trial_seed(mech, 0))
    th = data.theta0(mech, key)
    G = tr['Y'].shape[0]
    Y = tr['Y'] - 0.05 * tr['X'][8] if mech == 'FB' else tr['Y']
    b = gprx.GPBatch(G, tr['d'], N, 0, ctx=ctx); b.set_train(tr['X'], Y)
    r = b.run(np.tile(th, (G, 1)))
    for s in (0, G - 1):
        f = O.fit(tr['X'], Y[s], th, None, 1)
        print(mech, N, s, 'rel', abs(r['mll'][s] - f['mll']) / max(1, abs(f['mll'])), 'sens rel', f['mll_sens'] / max(1, abs(f['mll'])), flush=True)
    b.close()
