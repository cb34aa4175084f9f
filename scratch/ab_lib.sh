# A/B two builds of the library in one call: A = gpr.jl_amd/lib/libgprx_A.so, B = libgprx.so
set -e
for v in A B A B; do
  if [ $v = A ]; then L=gpr.jl_amd/lib/libgprx_A.so; else L=gpr.jl_amd/lib/libgprx.so; fi
  echo "== $v"; GPRX_LIB=$L timeout -k 10 120 python scratch/sweep.py 32 2>&1 | grep -E "^trials|${AB_GREP:-/n32}"
done
