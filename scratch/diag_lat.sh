set -e
for v in 1 2 0; do echo "DIAGV=$v"; GPRX_LEAF=1 GPRX_DIAGV=$v timeout -k 10 120 python scratch/sweep.py 32 2>&1 | grep -E "^trials|   diag "; done
