set -e
run() { echo "== $*"; env "$@" timeout -k 10 100 python scratch/sweep.py 32 2>&1 | grep -E "^trials|/n16"; }
run GPRX_X=0
run GPRX_SN_LINV=16
run GPRX_SN_TRSM=16
run GPRX_SN_SYRK=16
run GPRX_X=0
run GPRX_SN_LINV=16
