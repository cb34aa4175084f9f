set -e
for v in 0 1 2; do echo "LAUUMV=$v"; GPRX_LAUUMV=$v GPRX_LEAF=2 timeout -k 10 200 python scratch/sweep.py 8 32 | grep -E "trials|lauum"; done
timeout -k 10 300 python scratch/gpu_check.py
