set -e
timeout -k 10 200 python -u -m pytest tests/test_gpu.py -q -x --timeout 120 --timeout-method thread -k "split_k or gpe_mirror or ragged" 2>&1 | tail -3
for v in 1 2 4 8; do echo "SPLITK=$v"; GPRX_SPLITK=$v timeout -k 10 100 python scratch/latency.py 2>&1 | grep ms/call; done
