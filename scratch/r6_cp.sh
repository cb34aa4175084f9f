#!/bin/bash
set -e
mkdir -p gpurun_out
CP_TRIALS=39 timeout -k 10 200 python scratch/cp_time.py > gpurun_out/r6_cp_time.txt 2>&1
timeout -k 10 200 python scratch/host_overhead.py CP 512 512 26 39 > gpurun_out/r6_cp_host.txt 2>&1
echo ok
