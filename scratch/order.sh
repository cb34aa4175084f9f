set -e
for o in 0 1 2; do GPRX_LAUUM_ORDER=$o timeout -k 10 200 python scratch/sweep.py 32 > gpurun_out/o_$o.txt 2>&1; echo "order=$o"; grep -E "trials|lauum_grad " gpurun_out/o_$o.txt; done
