set -e
for cfg in "GPRX_GEMMV_SMALL=2" "GPRX_GEMMV_SMALL=1 GPRX_SMALL_N=16" "GPRX_GEMMV_SMALL=0 GPRX_SMALL_N=16" "GPRX_GEMMV=1" "GPRX_GEMMV=0"; do
  env $cfg timeout -k 10 200 python scratch/sweep.py 32 > gpurun_out/st.txt 2>&1; echo "$cfg $(grep -E 'trials' gpurun_out/st.txt)"; grep -E "/n32|/n16|/n8" gpurun_out/st.txt
done
