#!/bin/bash
# factorisation/prediction GPU tests, bit-compare and timing against scratch/var/libgprx_prev.so
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu.py -k "production or golden or fused_node or factorisation_paths or full_size or fb_full or cp_all or bench_shape or graph or pred or small" > gpurun_out/gab_tests.txt 2>&1
tail -n 2 gpurun_out/gab_tests.txt
REPS=${REPS:-3} bash scratch/ab_bits.sh scratch/var/libgprx_prev.so
