"""CState layout / output selection (bit-exact) and the synthetic generator.  CPU only."""
import json
import math

import numpy as np
import pytest

from gprx import data
from oracle import gp_oracle as O


def test_cstate_known_answer(golden_dir):
    z = np.load(golden_dir / "cstate_kat.npz")
    cs = data._cstates("P1", {"th": np.array([float(z["theta"])]), "om": np.array([float(z["omega"])])})
    np.testing.assert_array_equal(cs[:, 0], z["cstate"])


@pytest.mark.parametrize("mech,nb", [("P1", 1), ("P2", 2), ("CP", 2), ("FB", 4)])
def test_generator_shapes_and_indices(mech, nb):
    tr = data.make_trial(mech, 37, 5, seed=3)
    assert tr["X"].shape == (13 * nb, 37) and tr["Xs"].shape == (13 * nb, 5)
    assert tr["Y"].shape == (len(data.VW_INDICES[mech]), 37)
    np.testing.assert_array_equal(tr["Y"], O.select_outputs(tr["Xcurr"], data.VW_INDICES[mech]))
    q = tr["X"].reshape(nb, 13, -1)[:, 3:7, :]
    np.testing.assert_allclose(np.sum(q * q, axis=1), 1.0, rtol=0, atol=1e-14)  # unit quaternions
    # output coordinates are the velocity / angular-velocity slots 13(b-1)+{8..13}
    for i in data.VW_INDICES[mech]:
        assert (i - 1) % 13 >= 7


def test_generator_deterministic():
    a = data.make_trial("P2", 64, 8, seed=5)
    b = data.make_trial("P2", 64, 8, seed=5)
    for k in ("X", "Y", "Xs"):
        np.testing.assert_array_equal(a[k], b[k])


def test_theta_config_matches_reference_format():
    cfg = data.load_theta_config()
    assert len(cfg) == 84
    for key, nb in (("P1_MAX64", 1), ("P2_MAX2048", 2), ("CP_MAX512", 2), ("FB_MAX512", 4)):
        assert len(cfg[key]) == 13 * nb + 1
    th = data.theta0("P2", 2048)
    p = cfg["P2_MAX2048"]
    assert th[0] == -2.0 and th[-1] == math.log(p[0]) and th[1] == math.log(p[1])


def test_cstate_pack_oracle_layout():
    xc = np.arange(6.0).reshape(2, 3)
    q = np.arange(10.0, 18.0).reshape(2, 4)
    vc = np.arange(20.0, 26.0).reshape(2, 3)
    wc = np.arange(30.0, 36.0).reshape(2, 3)
    cs = O.cstate_pack(xc, q, vc, wc)
    np.testing.assert_array_equal(cs[:13], [0, 1, 2, 10, 11, 12, 13, 20, 21, 22, 30, 31, 32])
    np.testing.assert_array_equal(cs[13:], [3, 4, 5, 14, 15, 16, 17, 23, 24, 25, 33, 34, 35])
