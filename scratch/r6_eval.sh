#!/bin/bash
# round 6: FB N=4096 search group through the chunked device batches, per-level times of the bench
# workload and of CP at 39 trials x 26 outputs
set -e
mkdir -p gpurun_out
timeout -k 10 600 python -u search.py --experiments FB_MAX --sizes 4096 --trials ${FBT:-40} --testsamples 100 --simsteps 20 \
  --max-evals 30 --out gpurun_out/r6_fb4096_search.json > gpurun_out/r6_fb4096_search.txt 2>&1
echo "fb search ok"
timeout -k 10 300 python scratch/levels.py 40 3 > gpurun_out/r6_levels.txt 2>&1
echo "levels ok"
timeout -k 10 300 python scratch/levels_cfg.py CP 512 512 26 39 3 > gpurun_out/r6_levels_cp.txt 2>&1
echo "cp levels ok"
