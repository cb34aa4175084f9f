#!/bin/bash
# round 4 A/B: bit-for-bit outputs and per-level times, in-tree library against scratch/var variants
# usage: scratch/r4_ab.sh VARIANT...   (names of scratch/var/libgprx_NAME.so)
set -e
mkdir -p gpurun_out
for v in in-tree "$@"; do
  if [ $v = in-tree ]; then unset GPRX_LIB; else export GPRX_LIB=scratch/var/libgprx_$v.so; fi
  echo "== $v" >> gpurun_out/ab_bit.txt
  timeout -k 10 120 python scratch/bitcmp.py 8 >> gpurun_out/ab_bit.txt 2>&1
done
for i in $(seq 1 ${REPS:-2}); do
  for v in in-tree "$@"; do
    if [ $v = in-tree ]; then unset GPRX_LIB; else export GPRX_LIB=scratch/var/libgprx_$v.so; fi
    timeout -k 10 150 python scratch/levels.py 40 3 > gpurun_out/ab_levels_${v}_$i.txt 2>&1
    echo "$v $i $(grep -E '^(leaf|lauum|sum)' gpurun_out/ab_levels_${v}_$i.txt | tr -s ' ' | tr '\n' ' ')"
  done
done
