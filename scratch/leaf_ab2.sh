#!/bin/bash
# one GPU call: leaf-focused GPU tests on the in-tree build, A/B bench against base, the new leaf timeline
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/lb_gputests.txt 2>&1
echo "tests ok"
REPS=2 bash scratch/ab_multi.sh scratch/var/libgprx_base.so > gpurun_out/lb_ab.txt 2>&1
echo "ab ok"
GPRX_LIB=scratch/var/libgprx_stamps.so timeout -k 10 300 python scratch/leaf_timeline.py 40 > gpurun_out/lb_tl_new.txt 2>&1
echo "timeline ok"
