#!/bin/bash
set -e
mkdir -p gpurun_out
GPRX_LIB=scratch/var/libgprx_l8stamps.so timeout -k 10 200 python scratch/leaf8_timeline.py 40 > gpurun_out/r6_leaf_tl.json 2>&1
echo "leaf tl ok"
GPRX_LIB=scratch/var/libgprx_gts1208.so timeout -k 10 200 python scratch/node8_gts.py 40 > gpurun_out/r6_node8_gts.txt 2>&1
echo "gts ok"
