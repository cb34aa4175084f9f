"""The C CPU baseline (oracle/cpu_fit.c) against the numpy oracle it restates: same statements,
LAPACK calls and distance order; the sums differ only in numpy's pairwise summation order.  Bounds:
the larger of a rounding-level fixed bound (1e-11 relative LML, 1e-9 gradient, 1e-12 mean and
variance) and 10x the spread between the oracle's two distance formulations -- on the
ill-conditioned cartpole inputs rounding-order changes move the results by that much (as in
tests/test_gpu.py)."""
import numpy as np
import pytest

from oracle import gp_oracle as O

cf = pytest.importorskip("oracle.cpu_fit")


@pytest.fixture(scope="module")
def lib():
    try:
        return cf.load()
    except OSError as e:  # pragma: no cover - the library is built by build() / make -C oracle
        pytest.skip(str(e))


@pytest.mark.parametrize("mech,N,key", [("P2", 64, 64), ("CP", 130, 512), ("P1", 50, 64), ("FB", 96, 128)])
def test_c_fit_matches_numpy_oracle(lib, mech, N, key):
    from gprx import data

    tr = data.make_trial(mech, N, 9, seed=data.trial_seed(mech, 3))
    th = data.theta0(mech, key)
    for g in range(min(2, tr["Y"].shape[0])):
        ref = O.fit(tr["X"], tr["Y"][g], th, tr["Xs"], O.DIST_DIRECT)
        alt = O.fit(tr["X"], tr["Y"][g], th, tr["Xs"], O.DIST_EXPANDED)
        got = cf.fit(tr["X"], tr["Y"][g], th, tr["Xs"])

        def spread(k):
            return float(np.max(np.abs(np.asarray(ref[k]) - np.asarray(alt[k]))))

        assert abs(got["mll"] - ref["mll"]) <= max(1e-11 * max(1.0, abs(ref["mll"])), 10 * ref["mll_sens"])
        assert np.max(np.abs(got["grad"] - ref["grad"])) <= max(1e-9 * max(1.0, np.max(np.abs(ref["grad"]))),
                                                                 10 * spread("grad"))
        assert np.max(np.abs(got["mu"] - ref["mu"])) <= max(1e-12 * np.max(np.abs(tr["Y"][g])), 10 * spread("mu"))
        assert np.max(np.abs(got["var"] - ref["var"])) <= max(1e-12 * np.exp(2 * th[-1]), 10 * spread("var"))


def test_c_fit_not_positive_definite(lib, golden_dir):
    z = np.load(golden_dir / "nonpd_p1.npz")
    with pytest.raises(RuntimeError):
        cf.fit(z["X"], z["Y"][0], z["theta"])


def test_c_timed_modes_count_fits(lib):
    from gprx import data

    tr = data.make_trial("P2", 64, 9, seed=1)
    B = 4
    X = np.stack([tr["X"]] * B)
    Y = np.stack([tr["Y"][s % 6] for s in range(B)])
    T = np.tile(data.theta0("P2", 64), (B, 1))
    XT = np.stack([tr["Xs"]] * B)
    n1, s1 = cf.timed(X, Y, T, XT, threads=1, blas_threads=1, max_seconds=5.0, max_fits=6)
    n2, s2 = cf.timed(X, Y, T, XT, threads=2, blas_threads=1, max_seconds=5.0, max_fits=6)
    assert n1 == 6 and n2 == 6 and s1 > 0 and s2 > 0
