set -e
for a in 0 4 8; do echo "ABLATE=$a"; GPRX_ABLATE=$a timeout -k 10 200 python scratch/sweep.py 8 | grep -E "trials|potrf|trtri"; done
