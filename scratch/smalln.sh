set -e
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pyt.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/pyt.log | head -20; tail -5 gpurun_out/pyt.log; exit 1; }
tail -1 gpurun_out/pyt.log
for cfg in "GPRX_SMALL_N=16" "GPRX_SMALL_N=8" "GPRX_SMALL_N=32"; do
  env $cfg timeout -k 10 200 python scratch/sweep.py 32 > gpurun_out/st_$cfg.txt 2>&1; echo "$cfg $(grep -E 'trials' gpurun_out/st_$cfg.txt)"
done
