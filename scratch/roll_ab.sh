set -e
for nt in 256 512 1024 256; do echo "NT=$nt"; GPRX_ROLL_NT=$nt timeout -k 10 120 python scratch/rollout_bench.py 2>&1 | grep -v amdgpu.ids; done
