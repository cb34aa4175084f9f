#!/bin/bash
# VGPR / scratch report of named kernels in a dev build: scratch/regs.sh [hipcc flags] -- kernel...
cd "$(dirname "$0")"
flags=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do flags+=("$1"); shift; done; shift
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off -w -Idev "${flags[@]}" -c dev/gprx_kernels.hip -o /tmp/regs_k.o -save-temps=obj -o /tmp/regs/k.o 2>&1 | grep -v warning | head -5
python3 - "$@" <<'PY'
import re,sys
s=open('/tmp/regs/gprx_kernels-hip-amdgcn-amd-amdhsa-gfx950.s').read()
for k in sys.argv[1:]:
    for m in re.finditer(r'^(_ZN4gprx\d+'+k+r'\S*):', s, re.M):
        seg=s[m.start():s.find('.end_amdhsa_kernel',m.start())+4000]
        g=lambda key: (re.search(r';\s*'+key+r':\s*(\d+)',seg) or [None,None])[1]
        print(m.group(1)[:40], 'vgpr', g('NumVgprs'), 'agpr', g('NumAgprs'), 'scratch', g('ScratchSize'), 'occ', g('Occupancy'))
PY
