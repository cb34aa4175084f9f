#!/bin/bash
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu.py -k "four_wave or fused_node or n8_plan" > gpurun_out/r6_n8h_tests.txt 2>&1
echo "tests ok"
timeout -k 10 300 python scratch/node8h_ab.py CP 512 512 26 39 5 > gpurun_out/r6_n8h_cp39.txt 2>&1
echo "cp39 ok"
timeout -k 10 300 python scratch/node8h_ab.py CP 512 512 26 20 5 > gpurun_out/r6_n8h_cp20.txt 2>&1
timeout -k 10 300 python scratch/node8h_ab.py P2 2048 2048 6 40 3 > gpurun_out/r6_n8h_p2.txt 2>&1
echo "ab ok"
