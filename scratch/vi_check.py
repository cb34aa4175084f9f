"""Device variational-integrator step (k_vi_step) against the host restatement gprx.vi.vi_step on
every experiment mechanism: training-like states (data generator) and noisy test starts, plus the
run time of each side.  python scratch/vi_check.py"""
import sys
import time

sys.path[:0] = ["/root/repo", "/root/repo/gpr.jl_amd"]
import numpy as np  # noqa: E402

from gprx import data, projection, vi  # noqa: E402

for mech in ("P1", "P2", "CP", "FB"):
    tr = data.make_trial(mech, 256, 64, seed=11)
    S = np.concatenate([tr["X"].T, tr["Xs"].T])
    t0 = time.perf_counter()
    h, hi, hs = vi.vi_step(mech, S)
    t1 = time.perf_counter()
    g, gi, gs = projection.vi_step(mech, S)
    t2 = time.perf_counter()
    ok = (hs != 2) & (gs != 2)
    err = np.max(np.abs(h[ok] - g[ok])) if ok.any() else 0.0
    print(f"{mech}: T={len(S)} max|dev-host|={err:.3e} status host {np.bincount(hs, minlength=3)} dev {np.bincount(gs, minlength=3)} "
          f"iters host {hi.mean():.1f} dev {gi.mean():.1f}  host {1e3 * (t1 - t0):.1f} ms  dev {1e3 * (t2 - t1):.1f} ms", flush=True)
