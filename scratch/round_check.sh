set -e
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pyt.log 2>&1
echo "pytest ok"
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
echo "bench ok"
for L in 2 4; do GPRX_LEAF=$L timeout -k 10 200 python scratch/sweep.py 8 32 | grep -E "trials|leaf|/n4|/n8"; done
