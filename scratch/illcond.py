import sys, numpy as np
sys.path.insert(0,'/root/repo'); sys.path.insert(0,'/root/repo/gpr.jl_amd')
from oracle import gp_oracle as O
from gprx import data
for N in [1, 2, 5, 33, 63, 64, 65, 127, 130, 200, 320]:
    B, M = 3, 7
    trs = [data.make_trial("CP", N, M, seed=200 + s) for s in range(B)]
    rng = np.random.default_rng(N)
    th = np.stack([data.theta0("CP", 512) + 0.1 * rng.standard_normal(28) for _ in range(B)])
    out = []
    for s in range(B):
        X = trs[s]["X"]; y = trs[s]["Y"][s % 4]
        m0 = O.fit(X, y, th[s], trs[s]["Xs"], 0)["mll"]; m1 = O.fit(X, y, th[s], trs[s]["Xs"], 1)["mll"]
        K, Kf, D = O.gram(X, th[s], 0)
        out.append(f"s{s}: mll={m0:.4g} modespread={abs(m0-m1)/max(1,abs(m0)):.1e} cond={np.linalg.cond(K):.1e}")
    print(N, " | ".join(out))
