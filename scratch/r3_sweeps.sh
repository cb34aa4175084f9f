#!/bin/bash
# the noise.jl sweep (P1, P2, CP: every variant; FB: VI baseline and the MeanZero variants) and the
# hyperparameter.jl search on one GPU, wall-timed
set -e
mkdir -p gpurun_out
s=$(date +%s.%N); timeout -k 10 560 python -u sweep.py --mechs P1,P2,CP --out gpurun_out/sweep_p1p2cp.json > gpurun_out/sw_a.txt 2>&1; e=$(date +%s.%N)
echo "sweep P1,P2,CP all variants wall $(echo "$e - $s" | bc) s" | tee -a gpurun_out/sw_a.txt
s=$(date +%s.%N); timeout -k 10 300 python -u sweep.py --mechs FB --variants vi,max,min,min_sin --out gpurun_out/sweep_fb.json > gpurun_out/sw_b.txt 2>&1; e=$(date +%s.%N)
echo "sweep FB vi+MeanZero wall $(echo "$e - $s" | bc) s" | tee -a gpurun_out/sw_b.txt
s=$(date +%s.%N); timeout -k 10 400 python -u search.py --out gpurun_out/params_final_checkpoint.json > gpurun_out/sw_search.txt 2>&1; e=$(date +%s.%N)
echo "search wall $(echo "$e - $s" | bc) s" | tee -a gpurun_out/sw_search.txt
