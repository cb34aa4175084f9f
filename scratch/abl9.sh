set -e
for a in 0 8 16 32 56; do GPRX_ABLATE=$a timeout -k 10 200 python scratch/sweep.py 32 > gpurun_out/abl_$a.txt 2>&1; echo "ablate=$a $(grep -E 'leaf/n4' gpurun_out/abl_$a.txt)"; done
