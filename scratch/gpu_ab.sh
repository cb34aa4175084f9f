#!/bin/bash
# GPU tests on the in-tree build, then the A/B of the given library variants (scratch/ab_multi.sh)
set -e
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests.txt 2>&1
echo "tests ok"
bash scratch/ab_multi.sh "$@" > gpurun_out/ab.txt 2>&1
