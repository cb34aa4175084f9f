"""Machine-code checks of the gfx950 build (CPU only): the store-data and DPP hazards that the
compiler's hazard recognizer leaves to us (tests/isa_hazards.py)."""
import pathlib

import pytest

import isa_hazards as H

LIB = pathlib.Path(__file__).resolve().parents[1] / "gpr.jl_amd" / "lib"
OBJS = sorted(LIB.glob("gprx_*.o"))


def test_objects_present_with_the_library():
    """A built library ships its objects next to it (the hazard checks below must not skip
    silently on a tree that has the library)."""
    if (LIB / "libgprx.so").exists():
        assert {o.name for o in OBJS} >= {"gprx_kernels.o", "gprx_api.o", "gprx_lbfgs.o", "gprx_projection.o"}


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


def _at(off, text, target=None):
    """One instruction line of function k (base 0x1000) at byte offset `off`."""
    t = f" <k+{target:#x}>" if target is not None else ""
    return f"\t{text} // {0x1000 + off:012X}: 00000000{t}\n"


def test_checker_follows_branches_and_back_edges():
    """Hazards that straddle a block boundary: a store whose block ends in a branch to a VALU write
    of its data, and a DPP read at a loop head whose source the loop's last instruction writes
    before the back-edge.  The same sequences with the write two instructions away pass."""
    f = "0000000000001000 <k>:\n"
    store = "buffer_store_dwordx4 v[20:23], v36, s[36:39], 0 offen"
    over = "v_fma_f64 v[22:23], -v[16:17], s[28:29], v[4:5]"
    mov = "v_mov_b32_e32 v0, v1"
    # store; s_branch to +0x20; (dead filler); +0x20: the overwrite -> 1 wait state on the taken path
    seq = f + _at(0, store) + _at(8, "s_branch 5", 0x20) + _at(12, mov) + _at(16, mov) + _at(0x20, over) + _at(0x28, "s_endpgm")
    assert H.check(H.parse(seq))
    seq_ok = f + _at(0, store) + _at(8, "s_branch 5", 0x20) + _at(12, mov) + _at(16, mov) + _at(0x20, mov) + \
        _at(0x24, over) + _at(0x2c, "s_endpgm")
    assert not H.check(H.parse(seq_ok))
    # conditional branch: the fall-through path is hazard-free, the taken one is not
    seq_c = f + _at(0, store) + _at(8, "s_cbranch_scc1 5", 0x20) + _at(12, mov) + _at(16, mov) + _at(20, over) + \
        _at(0x20, over) + _at(0x28, "s_endpgm")
    assert H.check(H.parse(seq_c))
    # loop: +0: the DPP read of v[30:31]; ...; +0x18: write of v[30:31]; +0x20: s_cbranch back to +0
    dpp = "v_fmac_f64_dpp v[32:33], v[30:31], v[96:97] row_newbcast:1 row_mask:0xf bank_mask:0xf"
    w = "v_mul_f64 v[30:31], v[2:3], v[4:5]"
    loop = f + _at(0, dpp) + _at(8, mov) + _at(12, mov) + _at(0x18, w) + _at(0x20, "s_cbranch_scc1 65527", 0) + \
        _at(0x24, "s_endpgm")
    assert H.check(H.parse(loop))
    loop_ok = f + _at(0, dpp) + _at(8, mov) + _at(12, mov) + _at(0x18, w) + _at(0x20, "s_nop 0") + \
        _at(0x24, "s_cbranch_scc1 65526", 0) + _at(0x28, "s_endpgm")
    assert not H.check(H.parse(loop_ok))


@pytest.mark.skipif(not OBJS or not (H.LLVM / "llvm-objdump").exists(), reason="library objects / ROCm LLVM tools absent")
def test_checker_sees_the_branches_of_the_library():
    """The control-flow graph of the real objects has the branch edges (every printed target
    resolves to an instruction; otherwise parse/_cfg raise)."""
    insts = H.parse(H.disassemble(next(o for o in OBJS if o.name == "gprx_kernels.o")))
    succ, _ = H._cfg(insts)
    branches = sum(1 for i in insts if i[4] is not None)
    assert branches > 1000
    assert sum(len(s) for s in succ) > len(insts) - 100  # fall-through edges plus the branch edges
