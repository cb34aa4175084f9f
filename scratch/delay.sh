set -e
for dl in 0 10 30 60 0; do GPRX_DELAY=$dl timeout -k 10 200 python scratch/sweep.py 32 > gpurun_out/dl_$dl.txt 2>&1; echo "delay=$dl $(grep -E 'lauum_grad ' gpurun_out/dl_$dl.txt)"; done
