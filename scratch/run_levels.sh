#!/bin/bash
# per-level kernel times at the default geometry and with small_n / leaf variants (one GPU call)
set -e
timeout -k 10 180 python scratch/levels.py 32 3 > gpurun_out/levels_default.txt 2>&1
for v in "SMALL_N=4" "SMALL_N=16" "LEAF=2"; do
  env $v timeout -k 10 180 python scratch/levels.py 32 3 > gpurun_out/levels_$v.txt 2>&1
done
