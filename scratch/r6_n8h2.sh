#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 60 scratch/hwid_probe 1024 20000 > gpurun_out/r6_hwid.txt 2>&1
echo "probe ok"
timeout -k 10 300 python scratch/node8h_ab.py CP 512 512 26 39 5 > gpurun_out/r6_n8h_cp39_rot.txt 2>&1
GPRX_LIB=scratch/var/libgprx_norot.so timeout -k 10 300 python scratch/node8h_ab.py CP 512 512 26 39 5 > gpurun_out/r6_n8h_cp39_norot.txt 2>&1
echo "ab ok"
