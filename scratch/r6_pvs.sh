#!/bin/bash
# prediction variance: test-tile roles swapped on alternate workgroups (in-tree: bit-8 parity, pvs2: hash) against none (pvs0)
set -e
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu.py -k "pred or mean or var or production or full_size or cp or pinned" > gpurun_out/r6_pvs_tests.txt 2>&1
tail -n 1 gpurun_out/r6_pvs_tests.txt
for v in in-tree pvs0 pvs2; do
  if [ $v = in-tree ]; then unset GPRX_LIB; else export GPRX_LIB=scratch/var/libgprx_$v.so; fi
  echo "$v bits $(timeout -k 10 200 python scratch/bitcmp.py 8 2>/dev/null | tail -n 1)"
done
for i in 1 2 3; do
  for v in in-tree pvs0 pvs2; do
    if [ $v = in-tree ]; then unset GPRX_LIB; else export GPRX_LIB=scratch/var/libgprx_$v.so; fi
    timeout -k 10 300 python scratch/levels.py 40 3 > gpurun_out/r6_pvs_${v}_p2$i.txt 2>&1
    timeout -k 10 300 python scratch/levels_cfg.py CP 512 512 26 39 5 > gpurun_out/r6_pvs_${v}_cp$i.txt 2>&1
    echo "$v $i p2 pred_var $(grep pred_var gpurun_out/r6_pvs_${v}_p2$i.txt | awk '{print $2}') sum $(grep '^sum' gpurun_out/r6_pvs_${v}_p2$i.txt | awk '{print $2}') cp pred_var $(grep pred_var gpurun_out/r6_pvs_${v}_cp$i.txt | awk '{print $2}')"
  done
done
