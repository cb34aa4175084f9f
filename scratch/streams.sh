set -e
for cfg in "GPRX_STREAMS=1" "GPRX_STREAMS=2" "GPRX_STREAMS=4" "GPRX_LEAF=2" "GPRX_LEAF=8" "GPRX_STREAMS=2 GPRX_LEAF=2"; do
  env $cfg timeout -k 10 200 python scratch/sweep.py 32 > gpurun_out/st.txt 2>&1; echo "$cfg"; grep -E "trials|leaf/|potrf_trsm/n8|lauum_grad " gpurun_out/st.txt
done
