set -e
for ab in 0 1 2 64 128 192; do echo "ABLATE=$ab"; GPRX_ABLATE=$ab timeout -k 10 120 python scratch/sweep.py 32 2>&1 | grep -E "lauum_grad"; done
