set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pyt.log 2>&1 || { tail -30 gpurun_out/pyt.log; exit 1; }
tail -2 gpurun_out/pyt.log
for v in ${LAUUMVS:-1 2}; do GPRX_LAUUMV=$v timeout -k 10 200 python scratch/sweep.py 32 > gpurun_out/sweep_l$v.txt 2>&1; echo "lauumv=$v"; grep -E "trials|lauum|syrk_tt  " gpurun_out/sweep_l$v.txt; done
