#!/bin/bash
# round-4 closing evidence on the in-tree build: GPU tests, smoke, PMC/trace profile, default bench
# line (after the profile, so it carries this build's PMC traffic)
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fin_gputests.txt 2>&1
echo "tests ok"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.txt 2>&1
echo "smoke ok"
timeout -k 10 900 bash profiles/collect.sh r04 > gpurun_out/fin_collect.txt 2>&1
echo "collect ok"
timeout -k 10 400 python bench.py > gpurun_out/fin_bench1.json 2> gpurun_out/fin_bench1.err
echo "bench ok"
timeout -k 10 300 python scratch/levels2.py 40 3 > gpurun_out/fin_levels.txt 2>&1
echo "levels ok"
