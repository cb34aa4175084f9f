"""The reference's only published number (benchmark/b_inference.jl:48-51):
predictdynamics for the fourbar, N=100 training points, 12 MeanZero GPs, 20 steps, 1 test sample:
75 ms (zero mean).  Here: the same call shape on the device (k_rollout_max: GP means + projectv! +
updatestate! per step), T = 1 and T = 100 test samples, wall time per call including the launch."""
import sys, time
sys.path[:0] = ['/root/repo', '/root/repo/gpr.jl_amd']
import numpy as np, gprx
import gprx.data as D
import gprx.projection as GP
mech, N = 'FB', 100
tr = D.make_trial(mech, N, 100, seed=D.trial_seed(mech, 7))
th = D.theta0(mech, 128)
G = tr['Y'].shape[0]
b = gprx.GPBatch(G, tr['d'], N, 0); b.set_train(tr['X'], tr['Y'])
assert np.all(b.run(np.tile(th, (G, 1)))['status'] == 0)
idx = D.VW_INDICES[mech]
for T in (1, 100):
    S = tr['Xs'].T[:T]
    GP.predictdynamics(mech, [[(b, g) for g in range(G)]], S, 20, idx)
    ts = []
    for _ in range(10):
        t0 = time.perf_counter()
        out, pe, st = GP.predictdynamics(mech, [[(b, g) for g in range(G)]], S, 20, idx)
        ts.append(time.perf_counter() - t0)
    print(f'{mech} N={N} G={G} steps=20 test samples={T}: median {np.median(ts)*1e3:.2f} ms per call '
          f'(min {min(ts)*1e3:.2f}), status ok {int((st == 0).sum())}/{T}', flush=True)
