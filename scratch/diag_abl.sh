set -e
for ab in 0 256 512 1024 2048 3840; do echo "ABLATE=$ab"; GPRX_ABLATE=$ab timeout -k 10 120 python scratch/sweep.py 32 2>&1 | grep -E "leaf/n4"; done
