set -e
for ab in 0 8 16 32 56; do echo "ABLATE=$ab"; GPRX_ABLATE=$ab timeout -k 10 120 python scratch/sweep.py 32 2>&1 | grep -E "leaf/n4|potrf_trsm/n8|syrk_tt/n8"; done
