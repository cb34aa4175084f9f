#!/bin/bash
# fits/s of the bench workload at several trial counts per GPU (B = 6 x trials), one GPU call
set -e
for t in "$@"; do
  timeout -k 10 200 python bench.py --trials $t --steps 5 --no-cpu --no-opt > gpurun_out/bs_$t.log 2>&1
  python -c "
import json
for l in open('gpurun_out/bs_$t.log'):
    if l.startswith('{'): d=json.loads(l); print('trials $t B', d['config']['global_batch'], 'ms', d['ms_per_step'], 'fits/s', d['value'], 'leaf', d['kernels_ms_per_step']['leaf'], flush=True)"
done
