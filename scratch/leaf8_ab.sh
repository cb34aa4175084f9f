set -e
echo "default (leaf 4, 4 waves)"; timeout -k 10 120 python scratch/sweep.py 32 2>&1 | grep -E "^trials|leaf/n|/n8|/n16"
echo "LEAF=8 LEAFW=4"; GPRX_LEAF=8 GPRX_LEAFW=4 timeout -k 10 120 python scratch/sweep.py 32 2>&1 | grep -E "^trials|leaf/n|/n8|/n16"
echo "LEAF=8 LEAFW=8"; GPRX_LEAF=8 GPRX_LEAFW=8 timeout -k 10 120 python scratch/sweep.py 32 2>&1 | grep -E "^trials|leaf/n|/n8|/n16"
echo "LEAF=4 LEAFW=8"; GPRX_LEAF=4 GPRX_LEAFW=8 timeout -k 10 120 python scratch/sweep.py 32 2>&1 | grep -E "^trials|leaf/n|/n8|/n16"
