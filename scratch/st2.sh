set -e
for cfg in "GPRX_STREAMS=1" "GPRX_STREAMS=2" "GPRX_STREAMS=2 GPRX_STAGGER=0" "GPRX_STREAMS=1" "GPRX_STREAMS=2"; do
  env $cfg timeout -k 10 200 python scratch/sweep.py 32 > gpurun_out/st.txt 2>&1; echo "$cfg $(grep -E 'trials' gpurun_out/st.txt | cut -c1-70)"
done
