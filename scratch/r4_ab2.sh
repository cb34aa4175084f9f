#!/bin/bash
# A/B of variant libraries (scratch/var/libgprx_NAME.so) against the in-tree one: bit-for-bit output
# hash (scratch/bitcmp.py), per-level times (scratch/levels2.py) and the bench's step, REPS passes
# usage: REPS=2 scratch/r4_ab2.sh NAME...
set -e
mkdir -p gpurun_out
for v in in-tree "$@"; do
  if [ $v = in-tree ]; then unset GPRX_LIB; else export GPRX_LIB=scratch/var/libgprx_$v.so; fi
  echo "== $v $(timeout -k 10 120 python scratch/bitcmp.py 8 2>&1 | grep sha256)" >> gpurun_out/ab2_bit.txt
done
for i in $(seq 1 ${REPS:-1}); do
  for v in in-tree "$@"; do
    if [ $v = in-tree ]; then unset GPRX_LIB; else export GPRX_LIB=scratch/var/libgprx_$v.so; fi
    timeout -k 10 150 python scratch/levels2.py 40 3 > gpurun_out/ab2_levels_${v}_$i.txt 2>&1
    timeout -k 10 200 python bench.py --steps 10 --no-cpu --no-opt --no-prof > gpurun_out/ab2_bench_${v}_$i.json 2>/dev/null
    ms=$(python -c "import json; print(json.loads(open('gpurun_out/ab2_bench_${v}_$i.json').read().strip().splitlines()[-1])['ms_per_step'])")
    echo "$v $i step_ms $ms $(grep -E '^(leaf|node8a|potrf_trsm/n8|syrk_tt/n8|trtri_linv21/n8|lauum|sum)' gpurun_out/ab2_levels_${v}_$i.txt | awk '{printf "%s %s ", $1, $2}')"
  done
done
