#!/bin/bash
# leaf items kept off the diagonal wave's SIMD-mate (GPRX_L9_HW=6) against the in-tree build
set -e
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 300 python scratch/levels_cfg.py CP 512 512 26 39 5 > gpurun_out/r6_hw_base_cp$i.txt 2>&1
  GPRX_LIB=scratch/var/libgprx_hw6.so timeout -k 10 300 python scratch/levels_cfg.py CP 512 512 26 39 5 > gpurun_out/r6_hw_6_cp$i.txt 2>&1
  timeout -k 10 300 python scratch/levels.py 40 3 > gpurun_out/r6_hw_base_p2$i.txt 2>&1
  GPRX_LIB=scratch/var/libgprx_hw6.so timeout -k 10 300 python scratch/levels.py 40 3 > gpurun_out/r6_hw_6_p2$i.txt 2>&1
done
echo ok
