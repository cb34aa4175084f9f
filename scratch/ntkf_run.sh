#!/bin/bash
# A/B: in-tree vs nontemporal Kf loads in the gradient epilogue (time), then FETCH_SIZE of both
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
REPS=3 bash scratch/ab_multi.sh scratch/var/libgprx_ntkf.so > gpurun_out/nt_ab.txt 2>&1
echo "ab ok"
for v in base ntkf; do
  if [ $v = ntkf ]; then export GPRX_LIB=scratch/var/libgprx_ntkf.so; else unset GPRX_LIB; fi
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/nt_pmc_$v -o p -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu --no-prof --no-opt > /dev/null 2>&1
  echo "pmc $v ok"
done
