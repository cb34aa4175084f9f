#!/bin/bash
set -e
mkdir -p gpurun_out
GPRX_LIB=scratch/var/libgprx_nstamps.so timeout -k 10 200 python scratch/node_timeline.py CP 512 512 26 39 > gpurun_out/r6_node_tl_cp39.txt 2>&1
GPRX_LIB=scratch/var/libgprx_nstamps.so timeout -k 10 200 python scratch/node_timeline.py CP 512 512 26 9 > gpurun_out/r6_node_tl_cp9.txt 2>&1
echo "tl ok"
GPRX_LIB=scratch/var/libgprx_norot.so timeout -k 10 300 python scratch/node8h_ab.py CP 512 512 26 39 3 > gpurun_out/r6_n8h_cp39_norot.txt 2>&1
timeout -k 10 300 python scratch/node8h_ab.py CP 512 512 26 39 3 > gpurun_out/r6_n8h_cp39_rot.txt 2>&1
echo "ab ok"
