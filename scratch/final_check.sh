#!/bin/bash
# one GPU call: A/B of the in-tree build against the given variants (scratch/ab_multi.sh), then the
# round-end rehearsal: GPU tests, smoke, and the 2-rank distributed bench path (two ranks sharing
# the card; gloo control plane)
set -e
if [ $# -gt 0 ]; then bash scratch/ab_multi.sh "$@" > gpurun_out/final_ab.txt 2>&1; echo "ab ok"; fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final_gputests.txt 2>&1
echo "tests ok"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.txt 2>&1
echo "smoke ok"
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 2 --steps 3 --warmup 1 --no-cpu --no-opt > gpurun_out/final_bench2.json 2> gpurun_out/final_bench2.err
echo "2-rank bench ok"
