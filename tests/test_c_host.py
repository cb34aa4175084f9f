"""The C ABI from a plain C host (gpr.jl_amd/examples/gprx_c_host.c, built by the Makefile with gcc
against include/gprx.h only): the FFI boundary a Julia ccall shim uses, exercised without Python in
the compute process.  GPU: its single-GP results and batch LMLs against the oracle."""
import math
import pathlib
import subprocess

import numpy as np
import pytest

from oracle import gp_oracle as O

HOST = pathlib.Path(__file__).resolve().parents[1] / "gpr.jl_amd" / "lib" / "gprx_c_host"


def test_c_host_built_and_checks_arguments():
    assert HOST.exists(), "build with make -C gpr.jl_amd (or __graft_entry__.build())"
    r = subprocess.run([str(HOST)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "usage" in r.stderr


@pytest.mark.gpu
def test_c_host_matches_oracle(tmp_path):
    from gprx import data, dataset

    tr = data.make_trial("P2", 300, 12, seed=17)
    th = data.theta0("P2", 256)
    dataset.write_cstates(tmp_path / "t.cst", tr["X"], tr["Y"])
    th.astype("<f8").tofile(tmp_path / "theta.f64")
    np.ascontiguousarray(tr["Xs"].T).astype("<f8").tofile(tmp_path / "xs.f64")  # d x M column-major
    r = subprocess.run([str(HOST), str(tmp_path / "t.cst"), str(tmp_path / "theta.f64"), str(tmp_path / "xs.f64"), "12"],
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    out = {ln.split()[0]: np.array([float(v) for v in ln.split()[1:]]) for ln in r.stdout.splitlines() if ln.strip()}
    f = O.fit(tr["X"], tr["Y"][0], th, tr["Xs"])
    assert abs(out["mll"][0] - f["mll"]) <= max(1e-9 * abs(f["mll"]), 10 * f["mll_sens"])
    assert np.max(np.abs(out["grad"] - f["grad"])) <= 1e-7 * np.max(np.abs(f["grad"]))
    assert np.max(np.abs(out["mu"] - f["mu"])) <= 1e-9 * np.max(np.abs(tr["Y"][0]))
    assert np.max(np.abs(out["var"] - f["var"])) <= 1e-9 * math.exp(2 * th[-1])
    for g in range(6):
        m, _, _ = O.lml(tr["X"], tr["Y"][g], th)
        assert abs(out["batch_mll"][g] - m) <= 1e-9 * max(1.0, abs(m))
    # the device optimiser from C equals the same call through the Python mirror, bit for bit
    import gprx
    from gprx.optim import LBFGS, Options

    b = gprx.GPBatch(6, tr["d"], 300, 0, ctx=gprx.Context(0))
    b.set_train(tr["X"], tr["Y"])
    res, _ = b.optimize(np.tile(th, (6, 1)), LBFGS(), Options(max_evals=15))
    np.testing.assert_array_equal(out["opt_min"], [r.minimum for r in res])
    np.testing.assert_array_equal(out["opt_evals"], [r.f_calls for r in res])
    np.testing.assert_array_equal(out["opt_theta0"], res[0].minimizer)
    assert np.all(out["opt_min"] < -out["batch_mll"])
