"""Static checks on the gfx950 machine code of libgprx's objects (test infrastructure).

Two hazards the compiler's hazard recognizer does not cover for this code:

* VMEM store data: a VALU write to a VGPR that a preceding store with more than 64 bits of data
  still has to read needs 2 wait states on gfx950.  The recognizer exempts MUBUF stores with a
  register soffset; on the card, under memory back-pressure, such a store in k_gram read the next
  exp's intermediate instead of its K value ("Store-data hazard").  Checked for every
  store, whatever its encoding.
* DPP source: a VALU write followed by a DPP read of the same VGPR needs 2 wait states; inline
  assembly (k_leaf9's v_fmac_f64_dpp) is not covered by the recognizer.

Wait states: every instruction issued in between counts 1, `s_nop N` counts N + 1.
"""
from __future__ import annotations

import pathlib
import re
import subprocess
import tempfile

LLVM = pathlib.Path("/opt/rocm/lib/llvm/bin")
WAIT = 2

_reg = re.compile(r"\bv(?:\[(\d+):(\d+)\]|(\d+)\b)")


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


def parse(text: str):
    """[(function, mnemonic, operand list)] in program order; a label starts a new basic block
    (recorded as a ('<label>', ...) entry so that windows do not run across branches)."""
    fn = "?"
    out = []
    for line in text.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:", line)
        if m:
            fn = m.group(1)
            out.append((fn, "<label>", []))
            continue
        line = line.split("//")[0].strip()
        if not line or line.endswith(":"):
            if line:
                out.append((fn, "<label>", []))
            continue
        parts = line.split(None, 1)
        ops = [o.strip() for o in parts[1].split(",")] if len(parts) > 1 else []
        out.append((fn, parts[0], ops))
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
    if mn.startswith("scratch_"):
        return _regs(ops[1]) if len(ops) > 1 else set()
    return _regs(ops[1]) if len(ops) > 1 else set()


def _wait(mn: str, ops: list[str]) -> int:
    if mn == "s_nop":
        return int(ops[0], 0) + 1 if ops else 1
    return 1


def check(insts) -> list[str]:
    bad = []
    n = len(insts)
    for i, (fn, mn, ops) in enumerate(insts):
        data = _store_data(mn, ops)
        if data:  # later VALU writes of the data within WAIT wait states
            ws = 0
            for j in range(i + 1, n):
                fj, mj, oj = insts[j]
                if mj == "<label>" or fj != fn:
                    break
                if _valu_def(mj, oj) & data and ws < WAIT:
                    bad.append(f"{fn}: {mn} {', '.join(ops)} -> {mj} {', '.join(oj)} after {ws} wait states")
                    break
                ws += _wait(mj, oj)
                if ws >= WAIT:
                    break
        if "_dpp" in mn and len(ops) > 1:  # src0 written by a VALU within WAIT wait states before
            src = _regs(ops[1])
            ws = 0
            for j in range(i - 1, -1, -1):
                fj, mj, oj = insts[j]
                if mj == "<label>" or fj != fn:
                    break
                if _valu_def(mj, oj) & src and ws < WAIT:
                    bad.append(f"{fn}: {mj} {', '.join(oj)} -> {mn} {', '.join(ops)} after {ws} wait states")
                    break
                ws += _wait(mj, oj)
                if ws >= WAIT:
                    break
    return bad
