#!/bin/bash
# round-3 evidence on the in-tree build (one GPU call): GPU tests, smoke, the default bench line,
# rocprofv3 trace + PMC passes (profiles/collect.sh r03), per-level times, in-kernel clock, leaf timeline
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/ev_gputests.txt 2>&1
echo "tests ok"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/ev_smoke.txt 2>&1
echo "smoke ok"
timeout -k 10 400 python bench.py > gpurun_out/ev_bench.json 2> gpurun_out/ev_bench.err
echo "bench ok"
timeout -k 10 900 bash profiles/collect.sh r03 > gpurun_out/ev_collect.txt 2>&1
echo "collect ok"
timeout -k 10 300 python scratch/levels.py 40 3 > gpurun_out/ev_levels.txt 2>&1
echo "levels ok"
GPRX_LIB=scratch/var/libgprx_stamps.so timeout -k 10 300 python scratch/clock.py 40 3 > gpurun_out/ev_clock.txt 2>&1
GPRX_LIB=scratch/var/libgprx_stamps.so timeout -k 10 300 python scratch/leaf_timeline.py 40 > gpurun_out/ev_leaf_tl.txt 2>&1
echo "stamps ok"
