set -e
timeout -k 10 300 python -u -m pytest tests/test_gpu.py -q -x --timeout 120 --timeout-method thread -k "golden or factorisation or ragged or nonpd or production" 2>&1 | tail -2
AB_GREP="leaf/n4" bash scratch/ab_lib.sh
for L in gpr.jl_amd/lib/libgprx_A.so gpr.jl_amd/lib/libgprx.so; do echo "== $L"; GPRX_LIB=$L timeout -k 10 100 python scratch/latency.py 2>&1 | grep ms/call; done
