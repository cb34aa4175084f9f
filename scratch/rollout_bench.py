"""Timing of gprx_rollout_min: P2 minimal coordinates (usesin), N=2048, 20 steps, 100 test
trajectories per trial; 1 trial and 32 trials per launch.  Also the per-step predict loop
(one mean-only predict per step for all trajectories) for comparison."""
import sys, time
sys.path.insert(0, 'gpr.jl_amd'); sys.path.insert(0, '.')
import numpy as np
import gprx, gprx.data as D, gprx.rollout as R

mech, N, T, steps = "P2", 2048, 100, 20
for trials in (1, 32):
    trs = [D.make_trial_min(mech, N, T, seed=k, usesin=True) for k in range(trials)]
    th = D.theta0_min(mech, 2048, usesin=True)
    b = gprx.GPBatch(2 * trials, 6, N, T)
    b.set_train(np.stack([tr["X"] for tr in trs for _ in range(2)]), np.concatenate([tr["Y"] for tr in trs]))
    r = b.run(np.tile(th, (2 * trials, 1)))
    assert np.all(r["status"] == 0)
    groups = [[(b, 2 * k), (b, 2 * k + 1)] for k in range(trials)]
    start = np.concatenate([tr["start"] for tr in trs])
    tg = np.repeat(np.arange(trials), T)
    R.rollout_min(mech, groups, start, steps, True, traj_group=tg)
    b.ctx.set_profiling(True); b.ctx.reset_stats()
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        out = R.rollout_min(mech, groups, start, steps, True, traj_group=tg)
    wall = (time.perf_counter() - t0) / reps * 1e3
    st = b.ctx.kernel_stats("rollout")
    b.ctx.set_profiling(False)
    print(f"trials={trials:3d} T={T*trials:5d} steps={steps}: rollout call {wall:.3f} ms wall, kernel {st['ms']/max(st['launches'],1):.3f} ms "
          f"({T*trials*steps/ (wall/1e3):.3e} trajectory-steps/s)")
    # per-step host loop over mean-only predicts (trial 0 only when trials == 1)
    if trials == 1:
        qo = start[:, 0::2].copy(); vo = start[:, 1::2].copy(); qc = qo + 0.01 * vo
        t0 = time.perf_counter()
        for _ in range(steps):
            q = np.empty((T, 4)); q[:, 0::2] = qo; q[:, 1::2] = vo
            b.set_test(D.min_features(mech, q, True))
            mu, _ = b.predict(variance=False)
            pred = np.stack([mu[0], mu[1]], axis=1)
            qo, vo = qc.copy(), pred; qc = qc + pred * 0.01
        loop = (time.perf_counter() - t0) * 1e3
        print(f"  per-step predict loop: {loop:.3f} ms; max |diff| vs rollout {np.max(np.abs(qc - out[:, 0::2])):.2e}")
