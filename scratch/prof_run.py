import sys, time
sys.path.insert(0, '/root/repo/gpr.jl_amd'); sys.path.insert(0, '/root/repo')
import numpy as np, gprx, bench
trials = int(sys.argv[1]) if len(sys.argv) > 1 else 8
X, Y, T, XT = bench.make_workload(trials, 0, 1)
b = gprx.GPBatch(X.shape[0], 26, 2048, 100)
b.set_train(X, Y); b.set_test(XT)
for _ in range(3): r = b.run(T, grad=True, predict=True)
print("ok", bool((r['status'] == 0).all()))
