set -e
for cfg in "GPRX_LEAF=1 GPRX_DIAGV=1" "GPRX_LEAF=1 GPRX_DIAGV=0"; do
  env $cfg timeout -k 10 200 python scratch/sweep.py 32 > gpurun_out/st.txt 2>&1; echo "$cfg"; grep -E "trials|diag  |/n2 |/n4 " gpurun_out/st.txt
done
