"""Where do a kernel's register spills sit?  Splits each kernel of the library's gfx950 assembly
(`make -C gpr.jl_amd asm`) into basic blocks and reports, for every block with >= 16 MFMAs (the
K loops and peeled trips of the GEMM cores), its MFMA / load count and the spill traffic inside it:
v_writelane / v_readlane (SGPR spills live in VGPR lanes), scratch loads / stores (VGPR spills)
and AGPR copies.  python scratch/isa_loops.py [kernel-substring ...]"""
import re
import sys
from collections import Counter

S = open("/root/repo/gpr.jl_amd/lib/asm/gprx_kernels-hip-amdgcn-amd-amdhsa-gfx950.s").read()
want = sys.argv[1:] or ["k_gemm"]
for m in re.finditer(r"^(_Z\S+):\s*;\s*@", S, re.M):
    name = m.group(1)
    if not any(w in name for w in want):
        continue
    end = S.index(".Lfunc_end", m.end())
    body = S[m.end():end].split("\n")
    blocks, cur, label = [], [], "entry"
    for line in body:
        lm = re.match(r"^(\.LBB\S+):", line)
        if lm:
            blocks.append((label, cur))
            label, cur = lm.group(1), []
            continue
        t = line.strip()
        if t and not t.startswith((";", ".")):
            cur.append(t.split()[0])
            if t.startswith(("s_cbranch", "s_branch", "s_setpc", "s_endpgm")):  # a block ends at its branch
                blocks.append((label, cur))
                label, cur = label + "+", []
    blocks.append((label, cur))
    tot = Counter(i for _, b in blocks for i in b)
    print(f"{name}: {sum(len(b) for _, b in blocks)} instructions; whole kernel: "
          f"v_writelane {tot['v_writelane_b32']}, v_readlane {tot['v_readlane_b32']}, "
          f"scratch_load {sum(v for k, v in tot.items() if k.startswith('scratch_load'))}, "
          f"scratch_store {sum(v for k, v in tot.items() if k.startswith('scratch_store'))}")
    for label, b in blocks:
        c = Counter(b)
        nm = c["v_mfma_f64_16x16x4_f64"]
        if nm < 16:
            continue
        sl = sum(v for k, v in c.items() if k.startswith("scratch_load"))
        ss = sum(v for k, v in c.items() if k.startswith("scratch_store"))
        print(f"  {label:14s} mfma {nm:3d} global_load {sum(v for k, v in c.items() if k.startswith('global_load')):3d} "
              f"waitcnt {c['s_waitcnt']:3d} | v_writelane {c['v_writelane_b32']} v_readlane {c['v_readlane_b32']} "
              f"scratch_load {sl} scratch_store {ss} accvgpr {c['v_accvgpr_read_b32'] + c['v_accvgpr_write_b32']}")
