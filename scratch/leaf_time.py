"""Per-kernel times of one P2 B=192 N=2048 evaluation (LML + gradient) for leaf sizes 1/2/4 through
the library's own profiling timers (GPRX_LIB selects the build)."""
import sys
sys.path[:0] = ['/root/repo', '/root/repo/gpr.jl_amd']
import numpy as np, gprx
from gprx import data
B = 192
trs = [data.make_trial('P2', 2048, 0, seed=data.trial_seed('P2', t)) for t in range(B // 6)]
X = np.stack([trs[s // 6]['X'] for s in range(B)]); Y = np.stack([trs[s // 6]['Y'][s % 6] for s in range(B)])
th = np.tile(data.theta0('P2', 2048), (B, 1))
for arg in sys.argv[1:] or ['4']:
    leaf, small = (int(v) for v in (arg.split(',') + ['0'])[:2])
    ctx = gprx.Context(0)
    ctx.set_option(gprx.OPT_LEAF_TILES, leaf)
    ctx.set_option(gprx.OPT_SMALL_N, small)
    b = gprx.GPBatch(B, 26, 2048, 0, ctx=ctx); b.set_train(X, Y)
    b.run(th)
    ctx.set_profiling(True); ctx.reset_stats()
    for _ in range(3): r = b.run(th)
    out = {k: round(ctx.kernel_stats(k)['ms'] / 3, 3) for k in ('leaf', 'diag', 'potrf_trsm', 'syrk_tt', 'trtri_linv21', 'lauum_grad')}
    print('leaf', leaf, 'small_n', small, out, 'status', set(r['status'].tolist()), flush=True)
    b.close(); ctx.close()
