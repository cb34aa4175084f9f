#!/bin/bash
# A/B/C...: the in-tree library and each GPRX_LIB given as an argument, alternating, twice;
# prints ms_per_step and the per-kernel ms of the bench (no CPU / optimiser legs)
set -e
for i in $(seq 1 ${REPS:-2}); do
  for v in in-tree "$@"; do
    if [ $v = in-tree ]; then unset GPRX_LIB; else export GPRX_LIB=$v; fi
    tag=$(basename $v .so)$i
    timeout -k 10 200 python bench.py --steps ${STEPS:-5} --no-cpu --no-opt > gpurun_out/abm_$tag.log 2>&1
    python -c "
import json
for l in open('gpurun_out/abm_$tag.log'):
    if l.startswith('{'): d=json.loads(l); k=d['kernels_ms_per_step']; print('$tag', d['ms_per_step'], ' '.join(f'{a} {b}' for a,b in k.items() if b > 0.05), flush=True)"
  done
done
