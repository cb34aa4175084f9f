#!/bin/bash
# balanced node8 SYRK+TT plan (in-tree) against HEAD (prev); tests of the paths that use the plan
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu.py -k "n8_plan or four_wave or fused_node or production or factorisation_paths or small" > gpurun_out/r6_plan_tests.txt 2>&1
tail -n 1 gpurun_out/r6_plan_tests.txt
for i in 1 2; do
  timeout -k 10 300 python scratch/levels.py 40 3 > gpurun_out/r6_plan_new_p2$i.txt 2>&1
  GPRX_LIB=scratch/var/libgprx_prev.so timeout -k 10 300 python scratch/levels.py 40 3 > gpurun_out/r6_plan_old_p2$i.txt 2>&1
  timeout -k 10 300 python scratch/levels_cfg.py CP 512 512 26 39 5 > gpurun_out/r6_plan_new_cp$i.txt 2>&1
  GPRX_LIB=scratch/var/libgprx_prev.so timeout -k 10 300 python scratch/levels_cfg.py CP 512 512 26 39 5 > gpurun_out/r6_plan_old_cp$i.txt 2>&1
done
echo "ab ok"
GPRX_LIB=scratch/var/libgprx_l8stamps.so timeout -k 10 200 python scratch/leaf8_timeline.py 40 > gpurun_out/r6_leaf_tl.txt 2>&1
echo "diag ok"
