set -e
for a in 0 8192 0 8192; do GPRX_ABLATE=$a timeout -k 10 200 python scratch/sweep.py 32 > gpurun_out/st.txt 2>&1; echo "ablate=$a $(grep -E 'trials' gpurun_out/st.txt | cut -c1-60) $(grep -E 'trtri_linv21/n8' gpurun_out/st.txt)"; done
