#!/bin/bash
# round-3 closing evidence on the in-tree build: GPU tests, smoke, PMC/trace profile, default bench
# line (after the profile, so it carries this build's PMC traffic), refused 2-GPU run, 2-rank rehearsal
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/fin_gputests.txt 2>&1
echo "tests ok"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/fin_smoke.txt 2>&1
echo "smoke ok"
timeout -k 10 900 bash profiles/collect.sh r03 > gpurun_out/fin_collect.txt 2>&1
echo "collect ok"
timeout -k 10 400 python bench.py > gpurun_out/fin_bench1.json 2> gpurun_out/fin_bench1.err
echo "bench ok"
rc=0; timeout -k 10 120 python bench.py --gpus 2 --no-cpu --no-opt > gpurun_out/fin_bench2_refused.txt 2>&1 || rc=$?
echo "bench --gpus 2 on one GPU: rc=$rc (expected 2)"
timeout -k 10 600 python bench.py --gpus 2 --rehearse --steps 3 --warmup 1 --no-cpu --no-opt > gpurun_out/fin_bench2.json 2> gpurun_out/fin_bench2.err
echo "2-rank rehearsal ok"
timeout -k 10 300 python scratch/levels.py 40 3 > gpurun_out/fin_levels.txt 2>&1
echo "levels ok"
