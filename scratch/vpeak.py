"""Per-window max VGPR/AGPR index of one kernel in a device .s file (find register peaks)."""
import re, sys
s = open(sys.argv[1]).read().split('\n')
key = sys.argv[2]
start = [i for i, l in enumerate(s) if l.startswith(key + ':')][0]
end = [i for i in range(start, len(s)) if s[i].strip().startswith('.Lfunc_end')][0]
body = s[start:end]
win = int(sys.argv[3]) if len(sys.argv) > 3 else 150
print(len(body), 'lines')
for i in range(0, len(body), win):
    seg = body[i:i + win]
    mx = ag = 0
    for l in seg:
        if l.strip().startswith(';'):
            continue
        for m in re.finditer(r'\bv\[(\d+):(\d+)\]|\bv(\d+)\b', l):
            mx = max(mx, int(m.group(2) or m.group(3)))
        for m in re.finditer(r'\ba\[(\d+):(\d+)\]|\ba(\d+)\b', l):
            ag = max(ag, int(m.group(2) or m.group(3)))
    lab = next((x.strip() for x in seg if x.startswith('.LBB')), '')
    print(f"{i:6d} v{mx:4d} a{ag:4d} {lab[:30]:30s} {seg[0].strip()[:50]}")
