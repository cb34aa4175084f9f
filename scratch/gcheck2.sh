set -e
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pyt.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/pyt.log | head -20; tail -5 gpurun_out/pyt.log; exit 1; }
tail -2 gpurun_out/pyt.log
timeout -k 10 200 python scratch/sweep.py 32 > gpurun_out/st.txt 2>&1; grep -E 'trials|leaf' gpurun_out/st.txt
GPRX_LEAF=1 GPRX_DIAGV=2 timeout -k 10 200 python scratch/sweep.py 32 > gpurun_out/st2.txt 2>&1; grep -E 'trials|diag ' gpurun_out/st2.txt
