import sys, time
sys.path.insert(0, '/root/repo/gpr.jl_amd'); sys.path.insert(0, '/root/repo')
import numpy as np, gprx, bench
for mode in (0, 1, 0, 1):
    ctx = gprx.Context(0, dist_mode=mode)
    X, Y, T, XT = bench.make_workload(32, 0, 1)
    B = X.shape[0]
    b = gprx.GPBatch(B, 26, 2048, 100, ctx=ctx)
    b.set_train(X, Y); b.set_test(XT)
    b.run(T, grad=True, predict=True)
    t0 = time.perf_counter()
    for _ in range(5): r = b.run(T, grad=True, predict=True)
    dt = (time.perf_counter() - t0) / 5
    ctx.set_profiling(True); ctx.reset_stats(); b.run(T, grad=True, predict=True); ctx.set_profiling(False)
    g = ctx.kernel_stats("gram"); pc = ctx.kernel_stats("pred_cross")
    print(f"mode={mode}: {dt*1e3:.2f} ms/step {B/dt:.1f} fits/s gram {g['ms']:.3f} ms pred_cross {pc['ms']:.3f} ms ok={bool((r['status']==0).all())}", flush=True)
    b.close(); ctx.close()
