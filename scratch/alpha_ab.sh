set -e
for v in 1 2 1 2; do echo "ALPHA_V=$v"; GPRX_ALPHA_V=$v timeout -k 10 120 python scratch/sweep.py 32 2>&1 | grep -E "^trials|  alpha"; done
GPRX_ALPHA_V=2 timeout -k 10 300 python -u -m pytest tests/test_gpu.py -q -x --timeout 120 --timeout-method thread -k "golden or full_size or production" 2>&1 | tail -2
