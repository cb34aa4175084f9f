"""Raw fp64 CState dataset files (gprx/dataset.py): exact round trips, the
documented byte layout, rejection of malformed files, and a GPU fit fed from a file equal to the
in-memory one bit for bit."""
import struct

import numpy as np
import pytest


def _ds():
    import gprx.dataset as DS

    return DS


def test_round_trip_bit_exact(tmp_path):
    from gprx import data

    DS = _ds()
    tr = data.make_trial("P2", 37, 0, seed=3)
    p = tmp_path / "p2.cst"
    DS.write_cstates(p, tr["X"], tr["Y"])
    for mm in (True, False):
        z = DS.read_cstates(p, mmap=mm)
        assert (z["d"], z["N"], z["G"]) == (26, 37, 6)
        assert np.array_equal(z["X"], tr["X"]) and np.array_equal(z["Y"], tr["Y"])
    DS.write_cstates(p, tr["X"])
    z = DS.read_cstates(p)
    assert z["G"] == 0 and z["Y"] is None and np.array_equal(z["X"], tr["X"])


def test_layout_is_column_major_cstates(tmp_path):
    DS = _ds()
    X = np.arange(26 * 3, dtype=np.float64).reshape(3, 26).T  # column t = [26t, 26t+1, ...]
    p = tmp_path / "x.cst"
    DS.write_cstates(p, X, np.array([[7.0, 8.0, 9.0]]))
    raw = p.read_bytes()
    assert raw[:8] == b"GPRXCST1" and struct.unpack("<IIQQ", raw[8:32]) == (26, 1, 3, 0)
    vals = np.frombuffer(raw[32:], dtype="<f8")
    assert np.array_equal(vals[:78], np.arange(78.0)) and np.array_equal(vals[78:], [7.0, 8.0, 9.0])


def test_malformed_files_rejected(tmp_path):
    DS = _ds()
    p = tmp_path / "bad.cst"
    p.write_bytes(b"GPRX")
    with pytest.raises(ValueError):
        DS.read_cstates(p)
    DS.write_cstates(p, np.ones((13, 4)), np.ones((2, 4)))
    raw = p.read_bytes()
    p.write_bytes(raw[:-8])  # truncated
    with pytest.raises(ValueError):
        DS.read_cstates(p)
    p.write_bytes(b"NOTMAGIC" + raw[8:])
    with pytest.raises(ValueError):
        DS.read_cstates(p)
    with pytest.raises(ValueError):
        DS.write_cstates(p, np.ones((13, 4)), np.ones((2, 5)))


@pytest.mark.gpu
def test_file_fed_fit_equals_in_memory(tmp_path):
    import gprx
    from gprx import data

    DS = _ds()
    tr = data.make_trial("CP", 200, 9, seed=8)
    th = np.tile(data.theta0("CP", 256), (4, 1))
    p = tmp_path / "cp.cst"
    DS.write_cstates(p, tr["X"], tr["Y"])
    z = DS.read_cstates(p)
    out = []
    for X, Y in ((tr["X"], tr["Y"]), (z["X"], z["Y"])):
        b = gprx.GPBatch(4, 26, 200, 9)
        b.set_train(X, Y)
        b.set_test(tr["Xs"])
        out.append(b.run(th, grad=True, predict=True))
        b.close()
    for k in ("mll", "grad", "mu", "var"):
        np.testing.assert_array_equal(out[0][k], out[1][k])
