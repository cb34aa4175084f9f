set -e
for a in 0 2 1 0; do GPRX_ABLATE=$a timeout -k 10 200 python scratch/sweep.py 32 > gpurun_out/abl_$a.txt 2>&1; echo "ablate=$a $(grep -E 'lauum_grad ' gpurun_out/abl_$a.txt)"; done
