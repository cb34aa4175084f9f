#!/bin/bash
# factorisation-path GPU tests, bit-compare + timing against scratch/var/libgprx_prev.so, levels
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu.py -k "production or golden or fused_node or factorisation_paths or full_size or fb_full or cp_all or bench_shape or graph" > gpurun_out/la_tests.txt 2>&1
tail -n 2 gpurun_out/la_tests.txt
REPS=2 bash scratch/ab_bits.sh scratch/var/libgprx_prev.so
timeout -k 10 200 python scratch/levels.py 40 3 > gpurun_out/la_levels.txt 2>&1
cat gpurun_out/la_levels.txt | grep -v amdgpu.ids
GPRX_LIB=scratch/var/libgprx_stamps.so timeout -k 10 300 python scratch/leaf8_timeline.py 40 > gpurun_out/la_tl.json 2>&1
echo timeline ok
