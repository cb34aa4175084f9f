set -e
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pyt.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/pyt.log | head -20; tail -5 gpurun_out/pyt.log; exit 1; }
tail -1 gpurun_out/pyt.log
for cfg in "GPRX_SIDE=1" "GPRX_SIDE=0" "GPRX_SIDE=1" "GPRX_SIDE=0"; do
  env $cfg timeout -k 10 200 python scratch/sweep.py 32 > gpurun_out/st.txt 2>&1; echo "$cfg $(grep -E 'trials' gpurun_out/st.txt)"
done
GPRX_GRAPHS=1 timeout -k 10 200 python scratch/sweep.py 32 > gpurun_out/st.txt 2>&1; echo "graphs $(grep -E 'trials' gpurun_out/st.txt)"
