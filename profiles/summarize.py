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
