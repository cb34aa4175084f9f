#!/bin/bash
# k_lauum_grad FETCH_SIZE / WRITE_SIZE and duration per variant library (one PMC pass each):
# usage (GPU box): scratch/lauum_traffic.sh NAME...   (scratch/var/libgprx_NAME.so)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/lt
for v in "$@"; do
  for c in FETCH_SIZE WRITE_SIZE; do
    GPRX_LIB=scratch/var/libgprx_$v.so timeout -s KILL 120 rocprofv3 --pmc $c --kernel-trace --output-format csv \
      -d gpurun_out/lt/${v}_$c -o p -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-prof --no-opt > /dev/null 2>&1 || exit 1
  done
  python3 - "$v" <<'PY'
import csv, glob, sys
v = sys.argv[1]
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    rows = [r for f in glob.glob(f"gpurun_out/lt/{v}_{c}/**/*counter_collection.csv", recursive=True) for r in csv.DictReader(open(f))]
    vals = [float(r["Counter_Value"]) for r in rows if "k_lauum_grad" in r.get("Kernel_Name", "") and r.get("Counter_Name") == c]
    n = len(set((r.get("Dispatch_Id")) for r in rows if "k_lauum_grad" in r.get("Kernel_Name", "")))
    print(v, c, "sum/launch KB", sum(vals) / max(n, 1), "launches", n)
PY
done
