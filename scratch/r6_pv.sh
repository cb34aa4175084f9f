#!/bin/bash
# prediction-variance 4 x 1 balanced units (in-tree) against the 2 x 2 units (pv22); node8 and GEMM diagnostics
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu.py -k "golden or full_size or pred or production or ragged" > gpurun_out/r6_pv_tests.txt 2>&1
tail -n 1 gpurun_out/r6_pv_tests.txt
for i in 1 2; do
  timeout -k 10 300 python scratch/levels.py 40 3 > gpurun_out/r6_pv_new_p2$i.txt 2>&1
  GPRX_LIB=scratch/var/libgprx_pv22.so timeout -k 10 300 python scratch/levels.py 40 3 > gpurun_out/r6_pv_old_p2$i.txt 2>&1
done
timeout -k 10 300 python scratch/levels_cfg.py CP 512 512 26 39 5 > gpurun_out/r6_pv_new_cp.txt 2>&1
GPRX_LIB=scratch/var/libgprx_pv22.so timeout -k 10 300 python scratch/levels_cfg.py CP 512 512 26 39 5 > gpurun_out/r6_pv_old_cp.txt 2>&1
echo "ab ok"
GPRX_LIB=scratch/var/libgprx_l8stamps.so timeout -k 10 200 python scratch/leaf8_timeline.py 40 > gpurun_out/r6_leaf_tl.json 2>&1
GPRX_LIB=scratch/var/libgprx_gts1208.so timeout -k 10 200 python scratch/node8_gts.py 40 > gpurun_out/r6_node8_gts.txt 2>&1
echo "diag ok"
