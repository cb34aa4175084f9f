set -e
for a in 0 256 512 1024 2048 3840; do GPRX_LEAF=1 GPRX_DIAGV=2 GPRX_ABLATE=$a timeout -k 10 200 python scratch/sweep.py 32 > gpurun_out/abl_$a.txt 2>&1; echo "ablate=$a $(grep -E 'diag  ' gpurun_out/abl_$a.txt)"; done
