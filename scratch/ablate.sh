set -e
timeout -k 10 200 python scratch/gpu_check.py
timeout -k 10 200 python scratch/sweep.py 8 16
GPRX_STREAMS=2 timeout -k 10 200 python scratch/sweep.py 8 16 | grep trials
