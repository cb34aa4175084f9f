"""Summarise a profiles/collect.sh run: per-kernel durations (rocprofv3 --stats) and PMC-derived
HBM traffic per launch.  traffic = 2 * FETCH_SIZE + WRITE_SIZE (KB -> bytes): on gfx950
FETCH_SIZE tallies 128-B requests at 64 B (MI355X_MICROARCH.md, HBM section); WRITE_SIZE is exact.
usage: python3 profiles/summarize.py <collect-out-dir> <round>
"""
import csv
import glob
import json
import pathlib
import shutil
import sys
from collections import defaultdict

out, rnd = pathlib.Path(sys.argv[1]), sys.argv[2]
here = pathlib.Path(__file__).resolve().parent


def short(name):
    return name.split("(")[0].replace("gprx::", "")


kern = {}
stats = glob.glob(str(out / "trace" / "*kernel_stats.csv"))
if stats:
    shutil.copy(stats[0], here / f"{rnd}_kernel_stats.csv")
    with open(stats[0]) as f:
        for row in csv.DictReader(f):
            kern[short(row["Name"])] = dict(calls=int(row["Calls"]), avg_ms=float(row["AverageNs"]) / 1e6,
                                            total_ms=float(row["TotalDurationNs"]) / 1e6, pct=float(row["Percentage"]))

pmc = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> per-dispatch values
for f in glob.glob(str(out / "pmc_*" / "*counter_collection.csv")):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            pmc[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))

for k, cs in pmc.items():
    e = kern.setdefault(k, {})
    avg = {c: sum(v) / len(v) for c, v in cs.items() if v}
    if "FETCH_SIZE" in avg:
        e["fetch_kb_per_launch"] = avg["FETCH_SIZE"]
    if "WRITE_SIZE" in avg:
        e["write_kb_per_launch"] = avg["WRITE_SIZE"]
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        e["traffic_bytes_per_launch"] = (2 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024
    if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
        e["l2_hit"] = avg["TCC_HIT_sum"] / max(1.0, avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
    if "SQ_INSTS_VALU_MFMA_F64" in avg:
        e["mfma_f64_insts_per_launch"] = avg["SQ_INSTS_VALU_MFMA_F64"]
    if "SQ_INSTS_VALU" in avg:
        # VALU issue floor: every wave64 fp64 VALU instruction occupies its SIMD-32 for >= 4
        # cycles (78.6 TF/s fp64 vector = 16 FMA lanes/clk/SIMD); 1024 SIMDs; clock = GRBM_GUI_ACTIVE
        # (summed over the 8 XCDs) / 8 / duration.  valu_floor_frac = floor / duration: near 1
        # means VALU-issue-bound (transcendentals cost more, so this is a lower bound)
        e["valu_insts_per_launch"] = avg["SQ_INSTS_VALU"]
        if "SQ_ACTIVE_INST_VALU" in avg:
            e["active_inst_valu_per_launch"] = avg["SQ_ACTIVE_INST_VALU"]
        if "GRBM_GUI_ACTIVE" in avg and e.get("avg_ms"):
            dur = e["avg_ms"] * 1e-3
            clk = avg["GRBM_GUI_ACTIVE"] / 8.0 / dur
            e["clock_ghz_est"] = clk / 1e9
            e["valu_floor_ms"] = avg["SQ_INSTS_VALU"] * 4.0 / 1024.0 / clk * 1e3
            e["valu_floor_frac"] = e["valu_floor_ms"] / e["avg_ms"]

bench = None
try:
    bench = json.loads((out / "bench_under_rocprof.json").read_text().strip().splitlines()[-1])
except Exception:
    pass
summary = {"round": rnd, "bench_under_rocprof": bench, "kernels": kern,
           "note": "traffic = (2*FETCH_SIZE + WRITE_SIZE)*1024 per launch, gfx950 FETCH correction"}
(here / f"{rnd}_summary.json").write_text(json.dumps(summary, indent=1))
(here / "pmc_latest.json").write_text(json.dumps(summary, indent=1))
for k, e in sorted(kern.items(), key=lambda kv: -kv[1].get("total_ms", 0)):
    print(f"{k:28s} calls={e.get('calls', 0):5d} avg={e.get('avg_ms', 0):9.4f} ms  "
          f"traffic={e.get('traffic_bytes_per_launch', 0) / 1e6:10.2f} MB/launch  l2hit={e.get('l2_hit', 0):.3f}")
