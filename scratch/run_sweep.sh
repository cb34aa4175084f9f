set -e
timeout -k 10 300 python scratch/gpu_check.py 2>&1 | grep -v amdgpu.ids
for F in 0 1; do echo "FUSE_TT=$F"; GPRX_FUSE_TT=$F timeout -k 10 200 python scratch/sweep.py 8 32 | grep -v amdgpu.ids; done
