"""Static checks on the gfx950 machine code of libgprx's objects (test infrastructure).

Two hazards the compiler's hazard recognizer does not cover for this code:

* VMEM store data: a VALU write to a VGPR that a preceding store with more than 64 bits of data
  still has to read needs 2 wait states on gfx950.  The recognizer exempts MUBUF stores with a
  register soffset; on the card, under memory back-pressure, such a store in k_gram read the next
  exp's intermediate instead of its K value ("Store-data hazard").  Checked for every
  store, whatever its encoding.
* DPP source: a VALU write followed by a DPP read of the same VGPR needs 2 wait states; inline
  assembly (k_node8's v_fmac_f64_dpp) is not covered by the recognizer.

Wait states: every instruction issued in between counts 1, `s_nop N` counts N + 1.

The windows follow the control-flow graph of each function, built from the instruction addresses
and the branch targets llvm-objdump prints: forward from a store through every successor (the
fall-through unless the instruction is `s_branch` / `s_endpgm`, and the branch target), backward
from a DPP read through every predecessor (the layout predecessor unless it ends its block
unconditionally, and every branch to the address).  So a hazard that straddles a block boundary,
a loop back-edge or a jump is seen.  A path that leaves the function (its entry, an `s_endpgm`)
ends the window: nothing runs before a kernel's entry or after its end.
"""
from __future__ import annotations

import pathlib
import re
import subprocess
import tempfile

LLVM = pathlib.Path("/opt/rocm/lib/llvm/bin")
WAIT = 2

_reg = re.compile(r"\bv(?:\[(\d+):(\d+)\]|(\d+)\b)")
_addr = re.compile(r"//\s*([0-9A-Fa-f]+):")
_target = re.compile(r"<([^>+]+)(?:\+0x([0-9a-fA-F]+))?>\s*$")
_NOFALL = ("s_branch", "s_endpgm", "s_setpc_b64")


def disassemble(obj: pathlib.Path, arch: str = "gfx950") -> str:
    """Device code of one HIP object (its .hip_fatbin bundle), as llvm-objdump text."""
    secs = subprocess.run([str(LLVM / "llvm-readelf"), "-S", str(obj)], check=True, capture_output=True, text=True).stdout
    if ".hip_fatbin" not in secs:
        return ""  # host code only
    with tempfile.TemporaryDirectory() as td:
        fat, code = pathlib.Path(td, "fat.bin"), pathlib.Path(td, "code.o")
        subprocess.run([str(LLVM / "llvm-objcopy"), f"--dump-section=.hip_fatbin={fat}", str(obj),
                        str(pathlib.Path(td, "junk.o"))], check=True, capture_output=True)
        subprocess.run([str(LLVM / "clang-offload-bundler"), "--type=o", f"--targets=hipv4-amdgcn-amd-amdhsa--{arch}",
                        f"--input={fat}", f"--output={code}", "--unbundle"], check=True, capture_output=True)
        return subprocess.run([str(LLVM / "llvm-objdump"), "-d", f"--mcpu={arch}", str(code)], check=True,
                              capture_output=True, text=True).stdout


def _regs(op: str) -> set[int]:
    out = set()
    for a, b, c in _reg.findall(op):
        if c:
            out.add(int(c))
        else:
            out.update(range(int(a), int(b) + 1))
    return out


class Inst(tuple):
    """(function, mnemonic, operands, address or None, branch target (function, offset) or None)."""
    __slots__ = ()

    def __new__(cls, fn, mn, ops, addr=None, target=None):
        return super().__new__(cls, (fn, mn, ops, addr, target))


def parse(text: str) -> list[Inst]:
    """Instructions in program order.  A function header is recorded as a ('<label>', ...) entry
    (the function's entry: no predecessor inside the object)."""
    fn = "?"
    fn_base = 0
    out = []
    for line in text.splitlines():
        m = re.match(r"^([0-9a-f]+) <(.+)>:", line)
        if m:
            fn, fn_base = m.group(2), int(m.group(1), 16)
            out.append(Inst(fn, "<label>", []))
            continue
        raw = line
        a = _addr.search(raw)
        tg = _target.search(raw)
        line = line.split("//")[0].strip()
        if not line or line.endswith(":"):
            continue
        parts = line.split(None, 1)
        ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
        target = None
        if tg and parts[0].startswith(("s_branch", "s_cbranch")):
            target = (tg.group(1), int(tg.group(2) or "0", 16))
        addr = int(a.group(1), 16) - fn_base if a else None
        out.append(Inst(fn, parts[0], ops, addr, target))
    return out


def _valu_def(mn: str, ops: list[str]) -> set[int]:
    if not mn.startswith("v_") or mn.startswith(("v_readlane", "v_readfirstlane", "v_cmp")) or not ops:
        return set()
    return _regs(ops[0])


def _store_data(mn: str, ops: list[str]) -> set[int]:
    if not re.match(r"(buffer|global|flat|scratch)_store_(dwordx[34]|b96|b128)", mn):
        return set()
    if mn.startswith("buffer_"):
        return _regs(ops[0])
    return _regs(ops[1]) if len(ops) > 1 else set()


def _wait(mn: str, ops: list[str]) -> int:
    if mn == "s_nop":
        return int(ops[0], 0) + 1 if ops else 1
    return 1


def _cfg(insts):
    """Successor and predecessor index lists per instruction (within its function)."""
    n = len(insts)
    at = {(i[0], i[3]): k for k, i in enumerate(insts) if i[3] is not None}
    succ = [[] for _ in range(n)]
    pred = [[] for _ in range(n)]
    for k, (fn, mn, ops, addr, target) in enumerate(insts):
        if mn == "<label>":
            continue
        if not mn.startswith(_NOFALL) and k + 1 < n and insts[k + 1][1] != "<label>" and insts[k + 1][0] == fn:
            succ[k].append(k + 1)
        if target is not None:
            t = at.get((target[0], target[1])) if target[0] == fn else None
            if t is None:
                raise ValueError(f"{fn}: {mn} {', '.join(ops)}: branch target +{target[1]:#x} is not an instruction")
            succ[k].append(t)
    for k, ss in enumerate(succ):
        for s in ss:
            pred[s].append(k)
    return succ, pred


def _walk(insts, start, edges, hit):
    """Every path from `start` (exclusive) along `edges` until WAIT wait states have passed;
    returns the first instruction index on such a path for which hit(index) holds within fewer
    than WAIT wait states, with the wait states counted before it, or None."""
    stack = [(s, 0) for s in edges[start]]
    seen = set()
    while stack:
        j, ws = stack.pop()
        if (j, ws) in seen:
            continue
        seen.add((j, ws))
        fn, mn, ops = insts[j][:3]
        if hit(j):
            return j, ws
        ws2 = ws + _wait(mn, ops)
        if ws2 < WAIT:
            stack.extend((s, ws2) for s in edges[j])
    return None


def check(insts) -> list[str]:
    bad = []
    succ, pred = _cfg(insts)
    for i, (fn, mn, ops, _a, _t) in enumerate(insts):
        data = _store_data(mn, ops)
        if data:  # a later VALU write of the data within WAIT wait states, on any path
            r = _walk(insts, i, succ, lambda j: bool(_valu_def(insts[j][1], insts[j][2]) & data))
            if r:
                j, ws = r
                bad.append(f"{fn}: {mn} {', '.join(ops)} -> {insts[j][1]} {', '.join(insts[j][2])} after {ws} wait states")
        if "_dpp" in mn and len(ops) > 1:  # src0 written by a VALU within WAIT wait states before, on any path
            src = _regs(ops[1])
            r = _walk(insts, i, pred, lambda j: bool(_valu_def(insts[j][1], insts[j][2]) & src))
            if r:
                j, ws = r
                bad.append(f"{fn}: {insts[j][1]} {', '.join(insts[j][2])} -> {mn} {', '.join(ops)} after {ws} wait states")
    return bad
