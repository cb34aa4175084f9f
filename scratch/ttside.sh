set -e
for v in 0 32 16 8 0 32 16; do echo "TT_SIDE=$v"; GPRX_TT_SIDE=$v timeout -k 10 120 python scratch/sweep.py 32 2>&1 | grep -E "^trials"; done
