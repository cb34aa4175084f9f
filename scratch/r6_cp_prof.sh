#!/bin/bash
# rocprofv3 kernel statistics of the CP configuration (N=512, 39 trials x 26 outputs = 1014 slots)
set -e
mkdir -p gpurun_out/prof_cp
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_cp -o run -- python3 scratch/levels_cfg.py CP 512 512 26 39 5 > gpurun_out/r6_cp_prof.txt 2>&1
echo ok
