#!/bin/bash
# per-level times of the bench workload (scratch/levels.py) and a trials sweep of the bench line
mkdir -p gpurun_out
timeout -k 10 200 python scratch/levels.py 40 3 > gpurun_out/r05_levels.txt 2>&1 || exit 1
for t in ${TRIALS:-40 41 42}; do
  timeout -k 10 200 python bench.py --steps 10 --trials $t --no-cpu --no-opt > gpurun_out/tr_$t.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/tr_$t.json').read().strip().splitlines()[-1]); print($t, d['value'], d['ms_per_step'])"
done
