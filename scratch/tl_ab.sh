set -e
mkdir -p gpurun_out
GPRX_LIB=scratch/var/libgprx_stamps.so timeout -k 10 300 python scratch/leaf8_timeline.py 40 > gpurun_out/tl_new.json 2>&1
GPRX_LIB=scratch/var/libgprx_stamps0.so timeout -k 10 300 python scratch/leaf8_timeline.py 40 > gpurun_out/tl_old.json 2>&1
echo ok
