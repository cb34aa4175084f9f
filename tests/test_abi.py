"""The C-ABI library loads and exports every entry point include/gprx.h declares; host-only
helpers (CState packing, output selection) are bit-exact copies.  No GPU compute here."""
import ctypes as C
import pathlib
import re

import numpy as np
import pytest

from gprx import _lib as L
from oracle import gp_oracle as O

REPO = pathlib.Path(__file__).resolve().parents[1]
HEADER = REPO / "include" / "gprx.h"


def declared_functions():
    txt = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\**\s*(gprx_[a-z_0-9]+)\s*\(", txt, flags=re.M)))


def test_header_lists_the_abi():
    names = declared_functions()
    assert "gprx_batch_run" in names and "gprx_gp_lml_grad" in names and len(names) >= 20


def test_library_exports_every_declared_symbol():
    lib = C.CDLL(str(L.LIB_PATH))
    for name in declared_functions():
        assert hasattr(lib, name), name
    assert set(declared_functions()) == set(L.SIGNATURES), "ctypes table out of sync with gprx.h"


def test_abi_version_and_status_strings():
    assert L.lib.gprx_abi_version() == 3
    # the bindings' constants follow the header
    hdr = (REPO / "include" / "gprx.h").read_text()
    assert f"#define GPRX_ABI_VERSION {L.ABI_VERSION}\n" in hdr
    jl = (REPO / "gpr.jl_amd" / "julia" / "GPRx.jl").read_text()
    assert f"const ABI = Cint({L.ABI_VERSION})" in jl
    assert L.lib.gprx_status_string(1) == b"not positive definite"


def test_library_is_built_from_the_shipped_sources(tmp_path):
    """gprx_build_id() = the hash gpr.jl_amd/Makefile takes of the sources; the loader refuses a
    library whose id differs from the sources next to it (a stale prebuilt libgprx.so)."""
    assert L.lib.gprx_build_id().decode() == L.source_build_id()
    assert len(L.source_build_id()) == 16
    # a changed source gives another id
    import hashlib

    root = L._HERE.parent
    h = hashlib.sha256()
    for i, f in enumerate(L.BUILD_SOURCES):
        b = (root / f).read_bytes()
        h.update(b + (b" " if i == 0 else b""))
    assert h.hexdigest()[:16] != L.source_build_id()


def test_device_count_without_gpu():
    import torch

    if torch.cuda.device_count() > 0:
        assert L.lib.gprx_device_count() == torch.cuda.device_count()
    else:
        assert L.lib.gprx_device_count() == 0


def test_cstate_pack_bit_exact():
    rng = np.random.default_rng(0)
    nb = 4
    xc, q, vc, wc = (rng.standard_normal((nb, k)) for k in (3, 4, 3, 3))
    out = np.empty(13 * nb)
    rc = L.lib.gprx_cstate_pack(nb, L.dptr(np.ascontiguousarray(xc)), L.dptr(np.ascontiguousarray(q)),
                                L.dptr(np.ascontiguousarray(vc)), L.dptr(np.ascontiguousarray(wc)), L.dptr(out))
    assert rc == 0
    np.testing.assert_array_equal(out, O.cstate_pack(xc, q, vc, wc))


def test_select_outputs_bit_exact_and_validates():
    rng = np.random.default_rng(1)
    d, N = 52, 33
    Xc = rng.standard_normal((d, N))
    idx = np.array([9, 10, 22, 23, 35, 36, 48, 49, 11, 24, 37, 50], dtype=np.int32)  # FBnoise.jl:24
    Y = np.empty((idx.shape[0], N))
    Xabi = np.ascontiguousarray(Xc.T)  # ABI: d x N column-major
    assert L.lib.gprx_select_outputs(L.dptr(Xabi), d, N, L.iptr(idx), idx.shape[0], L.dptr(Y)) == 0
    np.testing.assert_array_equal(Y, O.select_outputs(Xc, idx))
    bad = np.array([0], dtype=np.int32)  # 1-based: 0 is invalid
    assert L.lib.gprx_select_outputs(L.dptr(Xabi), d, N, L.iptr(bad), 1, L.dptr(Y)) == L.INVALID_ARGUMENT


def test_ctx_create_fails_cleanly_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    h = C.c_void_p()
    rc = L.lib.gprx_ctx_create(0, C.byref(h))
    assert rc in (L.DEVICE_ERROR, L.INVALID_ARGUMENT) and not h.value


def test_null_handles_are_invalid_arguments():
    """Every entry point rejects null handles with GPRX_INVALID_ARGUMENT (no GPU needed)."""
    assert L.lib.gprx_rollout_min(None, 2, 0, 0.01, 5, 1, None, None, 1, None, None, None) == L.INVALID_ARGUMENT
    assert L.lib.gprx_batch_run(None, None, 0, None, None, None, None, None, None) == L.INVALID_ARGUMENT
    assert L.lib.gprx_batch_predict(None, None, None) == L.INVALID_ARGUMENT
    assert L.lib.gprx_gp_lml_grad(None, None, None, None) == L.INVALID_ARGUMENT
    assert L.lib.gprx_gp_predict(None, None, 1, None, None) == L.INVALID_ARGUMENT
    assert L.lib.gprx_gp_batch(None) is None


def test_optimizer_defaults_and_null_handle():
    """gprx_opt_defaults fills Optim 1.4.1 / LineSearches 7.1.1 defaults (LBFGS m = 10,
    InitialStatic alpha 1, scaleinvH0; BackTracking c_1 1e-4, rho 0.1..0.5, 1000 iterations;
    Options g_abstol 1e-8, iterations 1000, successive_f_tol 1, no time limit); the Python
    mirror's dataclasses agree; a null batch is an invalid argument (no GPU needed)."""
    import ctypes as C
    import math

    from gprx.optim import LBFGS, Options

    o = L.OptOptions()
    L.lib.gprx_opt_defaults(C.byref(o))
    m, ls, op = LBFGS(), LBFGS().linesearch, Options()
    assert (o.m, o.iterations, o.max_evals, o.ls_iterations, o.scaleinvH0, o.refit, o.successive_f_tol) == (
        m.m, op.iterations, -1, ls.iterations, 1, 1, op.successive_f_tol)
    assert (o.g_abstol, o.alphaguess, o.c_1, o.rho_hi, o.rho_lo) == (op.g_abstol, m.alphaguess, ls.c_1, ls.rho_hi,
                                                                    ls.rho_lo)
    assert math.isnan(o.time_limit) and math.isnan(op.time_limit)
    th = (C.c_double * 4)()
    assert L.lib.gprx_batch_optimize(None, th, C.byref(o), None, None, None, None, None, None, None) == L.INVALID_ARGUMENT


def test_optimizer_options_are_validated_on_the_host():
    """gprx.batch.opt_options rejects what gprx_batch_optimize would (ValueError before any call)
    and maps Options(max_evals=None) to Optim's f_calls_limit = 0 (no limit)."""
    import math

    from gprx.batch import opt_options
    from gprx.optim import LBFGS, BackTracking, Options

    o = opt_options()
    assert o.m == 10 and o.max_evals == 0 and o.refit == 1 and math.isnan(o.time_limit)
    assert opt_options(options=Options(max_evals=30), refit=False).max_evals == 30
    for kw in (dict(method=LBFGS(m=65)), dict(method=LBFGS(m=0)), dict(options=Options(iterations=-1)),
               dict(options=Options(successive_f_tol=-1)), dict(method=LBFGS(alphaguess=math.nan)),
               dict(method=LBFGS(linesearch=BackTracking(order=3))), dict(options=Options(g_abstol=math.nan))):
        with pytest.raises(ValueError):
            opt_options(**kw)


def _bytes(B, d, N, M):
    out = C.c_uint64()
    rc = L.lib.gprx_batch_bytes(B, d, N, M, C.byref(out))
    return rc, int(out.value)


def test_batch_bytes_and_the_addressing_guard():
    """gprx_batch_bytes (host arithmetic, no GPU): five Npad x Npad fp64 matrices per slot dominate,
    linear in B; sizes past the kernels' 32-bit buffer offsets (Npad * max(Npad, Mpad) * 8 >= 2^31
    - 16) are refused, as gprx_batch_create refuses them (a K walk past 2 GiB would read
    zeros silently)."""
    rc, b1 = _bytes(1, 26, 2048, 100)
    assert rc == 0
    rc, b2 = _bytes(2, 26, 2048, 100)
    assert rc == 0
    per = b2 - b1
    assert 5 * 2048 * 2048 * 8 < per < 5.2 * 2048 * 2048 * 8
    assert _bytes(240, 26, 2048, 100)[1] == b1 + 239 * per
    # FB N=4096: 671 MB per slot
    fb = _bytes(2, 52, 4096, 100)[1] - _bytes(1, 52, 4096, 100)[1]
    assert 6.7e8 < fb < 6.9e8
    # the limit: N = 16320 (Npad^2 * 8 = 2.13e9) is addressable, 16321 (Npad = 16384: 2^31) is not
    assert _bytes(1, 13, 16320, 0)[0] == 0
    assert _bytes(1, 13, 16321, 0)[0] == L.INVALID_ARGUMENT
    # test points: N = 2048 allows Mpad * 2048 * 8 < 2^31 - 16, i.e. M <= 131008
    assert _bytes(1, 13, 2048, 131008)[0] == 0
    assert _bytes(1, 13, 2048, 131009)[0] == L.INVALID_ARGUMENT
    for bad in ((0, 1, 1, 0), (1, 0, 1, 0), (1, 65, 1, 0), (1, 1, 0, 0), (1, 1, 1, -1)):
        assert _bytes(*bad)[0] == L.INVALID_ARGUMENT
    assert L.lib.gprx_batch_bytes(1, 1, 1, 0, None) == L.INVALID_ARGUMENT


def test_opt_trace_capacity_is_checked_without_a_batch():
    """gprx_batch_set_opt_trace(NULL, ...) is an argument error (the capacity check itself needs a
    batch: tests/test_gpu.py::test_opt_trace_capacity_checked)."""
    buf = np.zeros(8)
    assert L.lib.gprx_batch_set_opt_trace(None, L.dptr(buf), 1, 8) == L.INVALID_ARGUMENT
