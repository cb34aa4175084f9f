# evaluation latency at small batch: one GP per call (the drop-in shim's gprx_gp_lml_grad pattern)
# and one trial's six P2 outputs (CPnoise.jl:37-43 loop as one batch)
import sys, time, os
sys.path.insert(0, '/root/repo/gpr.jl_amd'); sys.path.insert(0, '/root/repo')
import numpy as np, gprx
from gprx import data
ctx = gprx.Context(0)
names = ["gram","leaf","diag","potrf_trsm","syrk_tt","trtri_linv21","alpha","lauum_grad","finalize"]
for mech, N, key, B in [("CP", 512, 512, 1), ("P2", 2048, 2048, 1), ("P2", 2048, 2048, 6)]:
    tr = data.make_trial(mech, N, 100, seed=3)
    th = data.theta0(mech, key)
    b = gprx.GPBatch(B, tr['d'], N, 100, ctx=ctx)
    b.set_train(tr['X'], tr['Y'][:B]); b.set_test(tr['Xs'])
    T = np.tile(th, (B, 1))
    for _ in range(3): b.run(T, grad=True, predict=False)
    n = 20; t0 = time.perf_counter()
    for _ in range(n): b.run(T, grad=True, predict=False)
    dt = (time.perf_counter() - t0) / n
    ctx.set_profiling(True); ctx.reset_stats(); b.run(T, grad=True, predict=False); ctx.set_profiling(False)
    ks = {k: ctx.kernel_stats(k) for k in names}
    br = "  ".join(f"{k}={v['ms']:.2f}" for k, v in ks.items() if v['launches'])
    print(f"{mech} N={N} B={B}: lml+grad {dt*1e3:.3f} ms/call  [{br}]", flush=True)
    b.close()
