#!/bin/bash
# round-6 evidence, part A: GPU suite, smoke, the default bench line, per-level times
set -e
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r6_gputests.txt 2>&1
echo "tests ok: $(tail -n 1 gpurun_out/r6_gputests.txt)"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_smoke.txt 2>&1
echo "smoke ok"
timeout -k 10 400 python bench.py > gpurun_out/r6_bench1.json 2> gpurun_out/r6_bench1.err
echo "bench ok"
timeout -k 10 300 python scratch/levels.py 40 3 > gpurun_out/r6_levels.txt 2>&1
echo "levels ok"
rc=0; timeout -k 10 120 python bench.py --gpus 2 --no-cpu --no-opt > gpurun_out/r6_bench2_refused.txt 2>&1 || rc=$?
echo "bench --gpus 2 on one GPU: rc=$rc (expected 2)"
timeout -k 10 600 python bench.py --gpus 2 --rehearse --steps 3 --warmup 1 --no-cpu --no-opt > gpurun_out/r6_bench2.json 2> gpurun_out/r6_bench2.err
echo "2-rank rehearsal ok"
