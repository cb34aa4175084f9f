#!/bin/bash
# lauum: Kf row blocks loaded right after the main loop (in-tree: 3 of 4) against 0 (kf0) and 2 (kf2)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu.py -k "golden or full_size or production or ragged or extremes" > gpurun_out/r6_kf_tests.txt 2>&1
tail -n 1 gpurun_out/r6_kf_tests.txt
for i in 1 2 3; do
  for v in in-tree kf0 kf2; do
    if [ $v = in-tree ]; then unset GPRX_LIB; else export GPRX_LIB=scratch/var/libgprx_$v.so; fi
    timeout -k 10 300 python scratch/levels.py 40 3 > gpurun_out/r6_kf_${v}_$i.txt 2>&1
    echo "$v $i $(grep lauum gpurun_out/r6_kf_${v}_$i.txt | awk '{print $2}') $(grep sum gpurun_out/r6_kf_${v}_$i.txt | awk '{print $2}')"
  done
done
unset GPRX_LIB
timeout -k 10 300 python scratch/levels_cfg.py CP 512 512 26 39 5 > gpurun_out/r6_kf_cp_new.txt 2>&1
GPRX_LIB=scratch/var/libgprx_kf0.so timeout -k 10 300 python scratch/levels_cfg.py CP 512 512 26 39 5 > gpurun_out/r6_kf_cp_old.txt 2>&1
echo "cp new $(grep lauum gpurun_out/r6_kf_cp_new.txt | awk '{print $2}') old $(grep lauum gpurun_out/r6_kf_cp_old.txt | awk '{print $2}')"
