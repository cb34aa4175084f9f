"""Machine-code checks of the gfx950 build (CPU only): the store-data and DPP hazards that the
compiler's hazard recognizer leaves to us (tests/isa_hazards.py)."""
import pathlib

import pytest

import isa_hazards as H

LIB = pathlib.Path(__file__).resolve().parents[1] / "gpr.jl_amd" / "lib"
OBJS = sorted(LIB.glob("gprx_*.o"))


@pytest.mark.skipif(not OBJS or not (H.LLVM / "llvm-objdump").exists(), reason="library objects / ROCm LLVM tools absent")
@pytest.mark.parametrize("obj", OBJS, ids=lambda p: p.name)
def test_no_store_data_or_dpp_hazards(obj):
    """Every >64-bit VMEM store keeps its data VGPRs for 2 wait states (k_gram's MUBUF stores,
    whose register soffset made the compiler skip them, wrote corrupted K values on the card under
    memory back-pressure), and every DPP source (k_leaf9's v_fmac_f64_dpp inline assembly) was
    written by a VALU at least 2 wait states before."""
    bad = H.check(H.parse(H.disassemble(obj)))
    assert not bad, "\n".join(bad[:20])


def test_checker_flags_the_hazards():
    """The checker itself, on hand-written sequences in llvm-objdump's format."""
    f = "0000000000001000 <k>:\n"
    store = "\tbuffer_store_dwordx4 v[20:23], v36, s[36:39], s8 offen offset:16 // 0\n"
    over = "\tv_fma_f64 v[22:23], -v[16:17], s[28:29], v[4:5] // 0\n"
    other = "\tv_mov_b32_e32 v0, v1 // 0\n"
    assert H.check(H.parse(f + store + over))
    assert H.check(H.parse(f + store + other + over))
    assert not H.check(H.parse(f + store + other + other + over))
    assert not H.check(H.parse(f + store + "\ts_nop 1 // 0\n" + over))
    x2 = "\tglobal_store_dwordx2 v[4:5], v[0:1], off // 0\n\tv_mov_b32_e32 v0, v1 // 0\n"
    assert not H.check(H.parse(f + x2))  # 64-bit data: no hazard
    dpp = "\tv_fmac_f64_dpp v[32:33], v[30:31], v[96:97] row_newbcast:1 row_mask:0xf bank_mask:0xf // 0\n"
    w = "\tv_mul_f64 v[30:31], v[2:3], v[4:5] // 0\n"
    assert H.check(H.parse(f + w + dpp))
    assert H.check(H.parse(f + w + other + dpp))
    assert not H.check(H.parse(f + w + other + other + dpp))
