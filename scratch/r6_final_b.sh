#!/bin/bash
# round-6 evidence, part B: rocprofv3 kernel stats + PMC passes of the bench, configs table
set -e
mkdir -p gpurun_out
bash profiles/collect.sh ${R:-r06} > gpurun_out/r6_collect.txt 2>&1
echo "collect ok"
timeout -k 10 400 python scratch/configs_perf.py gpurun_out/r6_configs_perf.json > gpurun_out/r6_configs_perf.txt 2>&1
echo "configs ok"
