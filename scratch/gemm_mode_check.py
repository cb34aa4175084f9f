# numpy experiment: LML/grad/mu with a GEMM-form (centred) distance vs the oracle's expanded mode
import sys, numpy as np, glob
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/gpr.jl_amd')
from oracle import gp_oracle as O
def gemm_D_r(X, il2):
    Xc = X - X.mean(axis=1, keepdims=True)
    n = (il2[:, None] * Xc * Xc).sum(0)
    g = (Xc * il2[:, None]).T @ Xc
    r = n[:, None] + n[None, :] - 2 * g
    np.fill_diagonal(r, 0.0)
    return np.maximum(r, 0.0)
for f in sorted(glob.glob('/root/repo/tests/golden/*_n*.npz')):
    z = np.load(f)
    X, Y, th = z['X'], z['Y'], z['theta']
    d = X.shape[0]
    il2, sf2, sn2, noise = O.kernel_params(th, d)
    worst = {}
    for g in range(Y.shape[0]):
        res = {}
        for mode in (0, 1, 'gemm'):
            if mode == 'gemm':
                r = gemm_D_r(X, il2)
            else:
                r = O.weighted_r(O.dist_stack(X, X, mode), il2)
            K = sf2 * np.exp(-0.5 * r); K[np.diag_indices_from(K)] += noise
            U = np.linalg.cholesky(K)
            a = np.linalg.solve(K, Y[g])
            mll = -(Y[g] @ a + 2 * np.log(np.diag(U)).sum() + len(a) * O.LOG2PI) / 2
            res[mode] = mll
        for m in (1, 'gemm'):
            worst[m] = max(worst.get(m, 0), abs(res[m] - res[0]) / max(1, abs(res[0])))
    print(f.split('/')[-1], {k: f"{v:.2e}" for k, v in worst.items()})
z = np.load('/root/repo/tests/golden/cp_n64.npz'); X, th = z['X'], z['theta']
il2, sf2, sn2, noise = O.kernel_params(th, X.shape[0])
print("il2", np.array2string(il2, precision=2)); print("sf2", sf2, "sn2", sn2)
Xc = X - X.mean(1, keepdims=True); n = (il2[:, None] * Xc * Xc).sum(0); print("n range", n.min(), n.max())
r = O.weighted_r(O.dist_stack(X, X, 0), il2); print("r offdiag min", np.min(r + np.eye(len(r))*1e9), "median", np.median(r))
print("cond K", np.linalg.cond(sf2*np.exp(-0.5*r) + noise*np.eye(len(r))))
