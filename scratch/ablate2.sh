set -e
for cfg in "1 0" "2 0" "4 0" "4 4" "4 8"; do set -- $cfg; echo "LEAF=$1 ABLATE=$2"; GPRX_LEAF=$1 GPRX_ABLATE=$2 timeout -k 10 200 python scratch/sweep.py 8 | grep -E "trials|leaf|diag|potrf|trtri"; done
