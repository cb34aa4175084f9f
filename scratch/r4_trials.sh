#!/bin/bash
# fits/s at several trial counts (6 slots per trial), REPS passes, same box
# usage: REPS=2 scratch/r4_trials.sh 40 42 ...
set -e
mkdir -p gpurun_out
for i in $(seq 1 ${REPS:-1}); do
  for t in "$@"; do
    timeout -k 10 200 python bench.py --steps 10 --trials $t --no-cpu --no-opt --no-prof > gpurun_out/tr_${t}_$i.json 2>/dev/null
    python -c "import json; d=json.loads(open('gpurun_out/tr_${t}_$i.json').read().strip().splitlines()[-1]); print('trials', $t, 'pass', $i, 'fits/s', round(d['value'],1), 'ms', d['ms_per_step'])" | tee -a gpurun_out/trials.txt
  done
done
