import csv, sys, collections
rows = collections.defaultdict(dict)
for r in csv.DictReader(open(sys.argv[1])):
    k = r["Dispatch_Id"]
    rows[k]["name"] = r["Kernel_Name"].split("(")[0].replace("gprx::", "")
    rows[k]["grid"] = int(r["Grid_Size"])
    rows[k]["dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    rows[k][r["Counter_Name"]] = float(r["Counter_Value"])
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for k, r in rows.items():
    key = (r["name"], r["grid"])
    a = agg[key]; a["n"] += 1
    for c, v in r.items():
        if isinstance(v, float): a[c] += v
cs = sys.argv[2].split(",")
for key, a in sorted(agg.items(), key=lambda kv: -kv[1]["dur"]):
    if a["dur"] < 1e-4: continue
    s = f"{key[0]:18s} grid={key[1]:8d} n={int(a['n']):3d} avg={a['dur']/a['n']*1e3:7.3f}ms"
    wc = a.get("SQ_WAVE_CYCLES", 0) or 1
    for c in cs:
        if c in a: s += f" {c.replace('SQ_','')}={a[c]/wc if c.startswith('SQ_WAIT') or c.startswith('SQ_ACTIVE') else a[c]/a['n']:.3g}"
    if "SQ_VALU_MFMA_BUSY_CYCLES" in a and "GRBM_GUI_ACTIVE" in a:
        s += f" mfma_busy/gui={a['SQ_VALU_MFMA_BUSY_CYCLES']/(a['GRBM_GUI_ACTIVE']/8*1024):.3f}"
    if "SQ_BUSY_CYCLES" in a and "GRBM_GUI_ACTIVE" in a:
        s += f" clk={a['GRBM_GUI_ACTIVE']/8/a['dur']/1e9:.2f}"
    print(s)
