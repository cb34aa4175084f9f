#!/bin/bash
# bit-compare (scratch/bitcmp.py) and time (bench.py, no CPU / optimiser legs) the in-tree library
# against variant libraries: bash scratch/ab_bits.sh LIB...
set -e
mkdir -p gpurun_out
for v in in-tree "$@"; do
  if [ $v = in-tree ]; then unset GPRX_LIB; else export GPRX_LIB=$v; fi
  echo "$v $(timeout -k 10 200 python scratch/bitcmp.py 8 2>/dev/null | tail -1)"
done
REPS=${REPS:-2} bash scratch/ab_multi.sh "$@"
