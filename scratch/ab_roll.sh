#!/bin/bash
# A/B of the projection kernels: tests of the in-tree build, then rollmax timing A (in-tree) / B (abl)
set -e
timeout -k 10 300 python -u -m pytest tests/test_projection.py tests/test_rollout.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/proj_tests.log 2>&1
timeout -k 10 200 python -u scratch/rollmax_time.py FB P2 > gpurun_out/rollmax_A.log 2>&1
GPRX_LIB=scratch/abl/libgprx_abl.so timeout -k 10 200 python -u scratch/rollmax_time.py FB P2 > gpurun_out/rollmax_B.log 2>&1
