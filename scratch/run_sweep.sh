set -e
timeout -k 10 300 python scratch/gpu_check.py 2>&1 | grep -v amdgpu.ids
for G in 0 1; do GPRX_GRAPHS=$G timeout -k 10 100 python scratch/latency.py 2>&1 | grep -v amdgpu.ids; done
for G in 0 1; do echo "GRAPHS=$G"; GPRX_GRAPHS=$G timeout -k 10 200 python scratch/sweep.py 8 32 | grep -E "trials"; done
