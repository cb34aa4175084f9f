import re, sys, subprocess
cur = None; rows = {}
for line in open(sys.argv[1] if len(sys.argv) > 1 else '/root/repo/gpr.jl_amd/lib/asm/resource.txt'):
    m = re.search(r'Function Name: (\S+)', line)
    if m:
        cur = subprocess.run(['c++filt', m.group(1)], capture_output=True, text=True).stdout.strip().split('(')[0].replace('gprx::', ''); rows[cur] = {}; continue
    for k in ['VGPRs', 'AGPRs', 'VGPRs Spill', 'Occupancy \[waves/SIMD\]', 'LDS Size \[bytes/block\]']:
        m = re.search(r'\s' + k + r': (\d+)', line)
        if m and cur: rows[cur][k.split(' ')[0] + ('_spill' if 'Spill' in k else '')] = int(m.group(1))
for k, v in rows.items(): print(f"{k:28s} {v}")
