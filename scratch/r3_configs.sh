#!/bin/bash
# all-configuration fits/s on the current build, then the full noise.jl sweep and hyperparameter.jl
# search on one GPU, wall-timed
set -e
mkdir -p gpurun_out
timeout -k 10 300 python scratch/configs_perf.py > gpurun_out/cfg_perf.txt 2>&1
echo "configs ok"
s=$(date +%s.%N); timeout -k 10 900 python -u sweep.py --out gpurun_out/sweep_final_checkpoint.json > gpurun_out/cfg_sweep.txt 2>&1; e=$(date +%s.%N)
echo "sweep wall $(echo "$e - $s" | bc) s" | tee -a gpurun_out/cfg_sweep.txt
s=$(date +%s.%N); timeout -k 10 900 python -u search.py --out gpurun_out/params_final_checkpoint.json > gpurun_out/cfg_search.txt 2>&1; e=$(date +%s.%N)
echo "search wall $(echo "$e - $s" | bc) s" | tee -a gpurun_out/cfg_search.txt
