set -e
for cfg in "GPRX_SMALL_N=8" "GPRX_SMALL_N=64" "GPRX_SMALL_N=64 GPRX_DIAGV=2" "GPRX_SMALL_N=64 GPRX_LEAF=4" "GPRX_SMALL_N=64 GPRX_LEAF=2" "GPRX_SMALL_N=16 GPRX_DIAGV=2"; do
  env $cfg timeout -k 10 200 python scratch/latency.py > gpurun_out/lat.txt 2>&1; echo "== $cfg"; grep -E "P2|CP" gpurun_out/lat.txt | cut -c1-60
done
