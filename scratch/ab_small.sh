set -e
for cfg in "GPRX_SMALL_N=16" "GPRX_SMALL_N=8" "GPRX_SMALL_N=4" "GPRX_SMALL_N=16"; do
  env $cfg timeout -k 10 200 python scratch/sweep.py 32 > gpurun_out/st.txt 2>&1; echo "$cfg $(grep -E 'trials' gpurun_out/st.txt)"; grep -E "/n16|/n8" gpurun_out/st.txt
done
