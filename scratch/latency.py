# single-GP evaluation latency (the drop-in shim's call pattern: one GP per gprx_gp_lml_grad)
import sys, time, os
sys.path.insert(0, '/root/repo/gpr.jl_amd'); sys.path.insert(0, '/root/repo')
import numpy as np, gprx
from gprx import data
for mech, N, key in [("CP", 512, 512), ("P2", 2048, 2048)]:
    tr = data.make_trial(mech, N, 100, seed=3)
    th = data.theta0(mech, key)
    b = gprx.GPBatch(1, tr['d'], N, 100)
    b.set_train(tr['X'], tr['Y'][:1]); b.set_test(tr['Xs'])
    for _ in range(3): b.run(th[None], grad=True, predict=False)
    n = 20; t0 = time.perf_counter()
    for _ in range(n): b.run(th[None], grad=True, predict=False)
    dt = (time.perf_counter() - t0) / n
    print(f"{mech} N={N}: lml+grad latency {dt*1e3:.3f} ms  (GPRX_GRAPHS={os.environ.get('GPRX_GRAPHS','1')})", flush=True)
    b.close()
