set -e
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "golden or ragged" > gpurun_out/pyt.log 2>&1 || { tail -30 gpurun_out/pyt.log; exit 1; }
for cfg in "GPRX_LEAFV=0" "GPRX_LEAFV=1" "GPRX_LEAFV=2"; do
  env $cfg timeout -k 10 200 python scratch/sweep.py 32 > gpurun_out/st.txt 2>&1; echo "$cfg $(grep -E 'trials' gpurun_out/st.txt) $(grep -E 'leaf/n4' gpurun_out/st.txt)"
done
GPRX_LEAFV=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "golden or ragged or full" > gpurun_out/pyt1.log 2>&1 || { tail -30 gpurun_out/pyt1.log; exit 1; }
tail -1 gpurun_out/pyt1.log
