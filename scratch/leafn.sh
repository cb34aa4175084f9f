set -e
for cfg in "GPRX_LEAF=4" "GPRX_LEAF=8" "GPRX_LEAF=2" "GPRX_LEAF=4"; do
  env $cfg timeout -k 10 200 python scratch/sweep.py 32 > gpurun_out/st.txt 2>&1; echo "$cfg $(grep -E 'trials' gpurun_out/st.txt)"; grep -E "leaf/|/n8|/n4 " gpurun_out/st.txt
done
