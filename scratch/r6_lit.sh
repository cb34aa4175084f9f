#!/bin/bash
# leaf X items: transposed 16-B Linv stores (in-tree) against one row per lane (lit0)
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu.py -k "node8 or n8_plan or four_wave or fused_node or production or factorisation_paths or small or full_size" > gpurun_out/r6_lit_tests.txt 2>&1
tail -n 1 gpurun_out/r6_lit_tests.txt
for v in in-tree lit0; do
  if [ $v = in-tree ]; then unset GPRX_LIB; else export GPRX_LIB=scratch/var/libgprx_$v.so; fi
  echo "$v bits $(timeout -k 10 200 python scratch/bitcmp.py 8 2>/dev/null | tail -n 1)"
done
for i in 1 2 3; do
  for v in in-tree lit0; do
    if [ $v = in-tree ]; then unset GPRX_LIB; else export GPRX_LIB=scratch/var/libgprx_$v.so; fi
    timeout -k 10 300 python scratch/levels.py 40 3 > gpurun_out/r6_lit_${v}_p2$i.txt 2>&1
    timeout -k 10 300 python scratch/levels_cfg.py CP 512 512 26 39 5 > gpurun_out/r6_lit_${v}_cp$i.txt 2>&1
    echo "$v $i p2 node8 $(grep node8 gpurun_out/r6_lit_${v}_p2$i.txt | awk '{print $2}') cp node8 $(grep node8 gpurun_out/r6_lit_${v}_cp$i.txt | awk '{print $2}')"
  done
done
