"""k_rollout_max / k_project timing for FB (the sweep's slowest groups): T trajectories of `steps`
steps, and T single projections."""
import sys, time, hashlib
sys.path[:0] = ['/root/repo', '/root/repo/gpr.jl_amd']
import numpy as np, gprx
import gprx.data as D
import gprx.projection as GP
from oracle import projection_oracle as PO
for mech in sys.argv[1:] or ['FB']:
    N, T = 64, 10000
    tr = D.make_trial(mech, N, 100, seed=D.trial_seed(mech, 5))
    th = D.theta0(mech, 64)
    G = tr['Y'].shape[0]
    b = gprx.GPBatch(G, tr['d'], N, 0); b.set_train(tr['X'], tr['Y'])
    b.run(np.tile(th, (G, 1)))
    idx = D.VW_INDICES[mech]
    S = np.tile(tr['Xs'].T, (T // tr['Xs'].shape[1], 1))
    for steps in (1, 20):
        GP.predictdynamics(mech, [[(b, g) for g in range(G)]], S[:100], steps, idx)
        t0 = time.perf_counter()
        out, pe, st = GP.predictdynamics(mech, [[(b, g) for g in range(G)]], S, steps, idx)
        dt = time.perf_counter() - t0
        print(mech, 'rollout_max T', T, 'steps', steps, f'{dt*1e3:.1f} ms', 'ok', int((st == 0).sum()),
              'digest', hashlib.md5(out.tobytes()).hexdigest()[:8], hashlib.md5(pe.tobytes()).hexdigest()[:8], flush=True)
    nb = GP.NBODIES[mech]
    X = D._cstates(mech, D._sample_minimal(mech, T, np.random.default_rng(1))).T
    rng = np.random.default_rng(2)
    vw = np.concatenate([X[:, 13 * b_ + 7:13 * b_ + 13] for b_ in range(nb)], axis=1) + 0.05 * rng.standard_normal((T, 6 * nb))
    GP.projectv(mech, X[:100], vw[:100])
    t0 = time.perf_counter()
    out, it, st = GP.projectv(mech, X, vw)
    dt = time.perf_counter() - t0
    print(mech, 'projectv T', T, f'{dt*1e3:.1f} ms', 'mean iters', float(it.mean()), 'ok', int((st == 0).sum()),
          'digest', hashlib.md5(out.tobytes()).hexdigest()[:8], hashlib.md5(it.tobytes()).hexdigest()[:8], flush=True)
    b.close()
