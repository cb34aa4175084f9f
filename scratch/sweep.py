import sys, time, pathlib, json
sys.path.insert(0, '/root/repo/gpr.jl_amd'); sys.path.insert(0, '/root/repo')
import numpy as np
import gprx
import bench
ctx = gprx.Context(0)
for trials in [int(a) for a in sys.argv[1:]] or [1, 4, 8, 16]:
    X, Y, T, XT = bench.make_workload(trials, 0, 1)
    B = X.shape[0]
    b = gprx.GPBatch(B, 26, 2048, 100, ctx=ctx)
    b.set_train(X, Y); b.set_test(XT)
    b.run(T, grad=True, predict=True)
    t0 = time.perf_counter(); n = 3
    for _ in range(n): r = b.run(T, grad=True, predict=True)
    dt = (time.perf_counter() - t0) / n
    ctx.set_profiling(True); ctx.reset_stats()
    b.run(T, grad=True, predict=True)
    ctx.set_profiling(False)
    ks = {k: ctx.kernel_stats(k) for k in ["gram","leaf","diag","potrf_trsm","potrf_syrk","trtri_tt","syrk_tt","trtri_linv21","alpha","lauum_grad","finalize","pred_cross","pred_var","pred_mu","pred_final"]}
    tot = sum(v['ms'] for v in ks.values())
    print(f"trials={trials} B={B}: {dt*1e3:.2f} ms/step  {B/dt:.1f} fits/s  {B*bench.fit_flops(2048,26,100)/dt/1e12:.2f} TF  status_ok={bool((r['status']==0).all())}  prof_sum={tot:.2f}ms", flush=True)
    for k, v in ks.items():
        print(f"   {k:13s} {v['ms']:8.3f} ms  n={v['launches']:3d}  {v['flops']/max(v['ms'],1e-9)/1e9:8.2f} TF(algo)  {v['bytes']/max(v['ms'],1e-9)/1e6:8.1f} GB/s", flush=True)
    for op in ["potrf_trsm","potrf_syrk","trtri_tt","syrk_tt","trtri_linv21","leaf"]:
        for n in [64, 32, 16, 8, 4, 2]:
            v = ctx.kernel_stats(f"{op}/n{n}")
            if v['launches']:
                print(f"      {op+'/n'+str(n):18s} {v['ms']:8.3f} ms  n={v['launches']:3d}  {v['flops']/max(v['ms'],1e-9)/1e9:8.2f} TF", flush=True)
    b.close()
