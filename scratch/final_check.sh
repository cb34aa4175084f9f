#!/bin/bash
# one GPU call: A/B of the in-tree build against the given variants (scratch/ab_multi.sh), then the
# round-end rehearsal: GPU tests, smoke, the default bench line, bench --gpus 2 refusing a 1-GPU
# box, and the 2-rank distributed bench path rehearsed on the one card (--rehearse: gloo control plane)
set -e
mkdir -p gpurun_out
{ cat /proc/self/cgroup; for f in /sys/fs/cgroup/cpu.max /sys/fs/cgroup/cpu/cpu.cfs_quota_us; do echo "$f: $(cat $f 2>&1)"; done;
  echo "nproc $(nproc) OMP_NUM_THREADS=$OMP_NUM_THREADS"; } > gpurun_out/final_host.txt 2>&1 || true
if [ $# -gt 0 ]; then bash scratch/ab_multi.sh "$@" > gpurun_out/final_ab.txt 2>&1; echo "ab ok"; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/final_gputests.txt 2>&1
echo "tests ok"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.txt 2>&1
echo "smoke ok"
timeout -k 10 400 python bench.py > gpurun_out/final_bench1.json 2> gpurun_out/final_bench1.err
echo "bench ok"
rc=0; timeout -k 10 120 python bench.py --gpus 2 --no-cpu --no-opt > gpurun_out/final_bench2_refused.txt 2>&1 || rc=$?
echo "bench --gpus 2 on one GPU: rc=$rc (expected 2)"
timeout -k 10 600 python bench.py --gpus 2 --rehearse --steps 3 --warmup 1 --no-cpu --no-opt > gpurun_out/final_bench2.json 2> gpurun_out/final_bench2.err
echo "2-rank rehearsal ok"
if [ -n "$LEVELS" ]; then timeout -k 10 300 python scratch/levels.py 40 3 > gpurun_out/final_levels.txt 2>&1; echo "levels ok"; fi
if [ -n "$CLOCK" ]; then GPRX_LIB=scratch/var/libgprx_stamps.so timeout -k 10 300 python scratch/clock.py 40 3 > gpurun_out/final_clock.txt 2>&1; echo "clock ok"; fi
