#!/bin/bash
# the whole noise.jl sweep on one GPU with the device VI step (MeanDynamics means and the VI
# baseline on k_vi_step): P1, P2, CP, then FB, every variant, wall-timed
set -e
mkdir -p gpurun_out
s=$(date +%s.%N); timeout -k 10 ${T1:-400} python -u sweep.py --mechs P1,P2,CP --out gpurun_out/sweep_p1p2cp_r4.json > gpurun_out/sw4_a.txt 2>&1; e=$(date +%s.%N)
echo "sweep P1,P2,CP all variants wall $(python3 -c "print(round($e - $s, 1))") s" | tee -a gpurun_out/sw4_a.txt
s=$(date +%s.%N); timeout -k 10 ${T2:-500} python -u sweep.py --mechs FB --out gpurun_out/sweep_fb_r4.json > gpurun_out/sw4_b.txt 2>&1; e=$(date +%s.%N)
echo "sweep FB all variants wall $(python3 -c "print(round($e - $s, 1))") s" | tee -a gpurun_out/sw4_b.txt
