"""fits/s of the four BASELINE configurations (fit = Gram+Cholesky+alpha+LML, full gradient,
mean+variance at M=100), one batch per call, and the algorithmic TF/s of each (bench.fit_flops).
    python scratch/configs_perf.py [out.json] [--cp T1,T2,...]   (--cp: only CP at those trial counts)"""
import json
import pathlib
import sys
import time

REPO = pathlib.Path(__file__).resolve().parents[1]
sys.path[:0] = [str(REPO / "gpr.jl_amd"), str(REPO)]
import numpy as np  # noqa: E402

import bench  # noqa: E402
import gprx  # noqa: E402
from gprx import data  # noqa: E402

ctx = gprx.Context(0)
cases = [("P1", 50, 64, 3, 256), ("CP", 512, 512, 26, 8), ("CP", 512, 512, 26, 19), ("CP", 512, 512, 26, 39),
         ("CP", 512, 512, 26, 59), ("P2", 2048, 2048, 6, 40), ("FB", 4096, 512, 12, 4), ("FB", 4096, 512, 12, 8)]
if "--cp" in sys.argv:
    i = sys.argv.index("--cp")
    cases = [("CP", 512, 512, 26, int(t)) for t in sys.argv[i + 1].split(",")]
    del sys.argv[i:i + 2]
rows = []
for mech, N, key, G, trials in cases:
    trs = [data.make_trial(mech, N, 100, seed=data.trial_seed(mech, t)) for t in range(trials)]
    Ysel = (lambda tr: tr["Xcurr"]) if G == 26 else (lambda tr: tr["Y"])
    X = np.stack([tr["X"] for tr in trs for _ in range(G)])
    Y = np.concatenate([Ysel(tr) for tr in trs])
    XT = np.stack([tr["Xs"] for tr in trs for _ in range(G)])
    B = X.shape[0]
    d = X.shape[1]
    th = np.tile(data.theta0(mech, key), (B, 1))
    b = gprx.GPBatch(B, d, N, 100, ctx=ctx)
    b.set_train(X, Y)
    b.set_test(XT)
    r = b.run(th, grad=True, predict=True)
    n = 5 if N <= 2048 else 3
    t0 = time.perf_counter()
    for _ in range(n):
        r = b.run(th, grad=True, predict=True)
    dt = (time.perf_counter() - t0) / n
    tf = B * bench.fit_flops(N, d, 100) / dt / 1e12
    row = dict(config=mech, N=N, d=d, trials=trials, gps_per_trial=G, batch=B, ms_per_batch=round(dt * 1e3, 3),
               fits_per_s=round(B / dt, 1), tflops_algorithmic=round(tf, 2), ok=int((r["status"] == 0).sum()))
    rows.append(row)
    print(f"{mech:3s} N={N:5d} d={d:2d} B={B:4d} ({trials:3d} trials x {G:2d} GPs): {dt * 1e3:8.2f} ms/batch "
          f"{B / dt:11.1f} fits/s  {tf:6.2f} TF/s  ok={row['ok']}/{B}", flush=True)
    b.close()
if len(sys.argv) > 1:
    pathlib.Path(sys.argv[1]).write_text(json.dumps(rows, indent=1))
