#!/bin/bash
# one GPU call: a subset (or all) of the GPU tests on the in-tree build, then scratch/ab_multi.sh
# against the given variant libraries.  usage: scratch/run_ab_tests.sh "PYTEST_K_EXPR|all" [variant.so...]
set -e
mkdir -p gpurun_out
k=$1; shift
sel=(); if [ "$k" != all ]; then sel=(-k "$k"); fi
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread "${sel[@]}" > gpurun_out/abt_tests.txt 2>&1
echo "tests ok: $(tail -1 gpurun_out/abt_tests.txt)"
bash scratch/ab_multi.sh "$@"
