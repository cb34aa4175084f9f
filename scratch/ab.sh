#!/bin/bash
# A/B of the in-tree library against scratch/abl/libgprx_abl.so in one GPU session:
# bench (no CPU / optimiser legs) alternating A B A B; prints ms_per_step and lauum ms
set -e
for i in 1 2; do
  for v in A B; do
    if [ $v = B ]; then export GPRX_LIB=scratch/abl/libgprx_abl.so; else unset GPRX_LIB; fi
    timeout -k 10 200 python bench.py --steps 5 --no-cpu --no-opt > gpurun_out/ab_$v$i.log 2>&1
    python -c "
import json,sys
for l in open('gpurun_out/ab_$v$i.log'):
    if l.startswith('{'): d=json.loads(l); k=d['kernels_ms_per_step']; print('$v$i', d['ms_per_step'], 'lauum', k['lauum_grad'], 'leaf', k['leaf'], 'trsm', k['potrf_trsm'], 'syrk', k['syrk_tt'], 'linv', k['trtri_linv21'], 'alpha', k['alpha'], 'pv', k['pred_var'], 'gram', k['gram'], flush=True)"
  done
done
