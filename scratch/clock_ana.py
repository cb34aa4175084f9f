import csv, sys, collections
rows = collections.defaultdict(dict)
for r in csv.DictReader(open(sys.argv[1])):
    k = (r["Dispatch_Id"])
    rows[k]["name"] = r["Kernel_Name"].split("(")[0].replace("gprx::", "")
    rows[k]["grid"] = int(r["Grid_Size"])
    rows[k]["dur"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    rows[k][r["Counter_Name"]] = float(r["Counter_Value"])
    rows[k]["vgpr"] = (r["VGPR_Count"], r["Accum_VGPR_Count"], r["SGPR_Count"], r["LDS_Block_Size"])
agg = collections.defaultdict(lambda: collections.defaultdict(float))
for k, r in rows.items():
    if "GRBM_GUI_ACTIVE" not in r: continue
    key = (r["name"], r["grid"])
    a = agg[key]; a["n"] += 1; a["dur"] += r["dur"]; a["grbm"] += r["GRBM_GUI_ACTIVE"]; a["mfma"] += r.get("SQ_INSTS_VALU_MFMA_F64", 0)
    a["vgpr"] = r["vgpr"]
for key, a in sorted(agg.items(), key=lambda kv: -kv[1]["dur"]):
    if a["dur"] < 1e-4: continue
    clk = a["grbm"] / 8 / a["dur"] / 1e9
    tf = a["mfma"] * 2048 / a["dur"] / 1e12
    print(f"{key[0]:22s} grid={key[1]:8d} n={int(a['n']):3d} avg={a['dur']/a['n']*1e3:8.3f}ms clk={clk:5.2f}GHz mfmaTF={tf:6.2f} regs={a['vgpr']}")
