set -e
timeout -k 10 300 python scratch/gpu_check.py 2>&1 | grep -v amdgpu.ids
for L in 1 2 4; do echo "LEAF=$L"; GPRX_LEAF=$L timeout -k 10 100 python scratch/latency.py 2>&1 | grep -v amdgpu.ids; done
