#!/bin/bash
# GEMM tile timelines (diagnostic builds) of the bench workload, one launch each
set -e
mkdir -p gpurun_out
for v in trsm32 trsm16 trsm8 syrk32 linv8; do
  GPRX_LIB=scratch/var/libgprx_gts_$v.so timeout -k 10 200 python scratch/gemm_timeline.py 40 > gpurun_out/gts_$v.txt 2>&1
  echo "$v $(tail -1 gpurun_out/gts_$v.txt)"
done
# builds (scratch/): for v in "trsm32 32" "trsm16 16" "trsm8 8" "syrk32 132" "linv8 308"; do set -- $v;
#   bash varbuild.sh gts_$1 ../gpr.jl_amd/csrc/gprx_kernels.hip -DGPRX_GSTAMPS=$2; done
#   bash varbuild.sh gts_lauum ../gpr.jl_amd/csrc/gprx_kernels.hip -DGPRX_GSTAMPS=999   (gemm_timeline.py --lauum)
#   bash varbuild.sh gts_lau2 ../gpr.jl_amd/csrc/gprx_kernels.hip -DGPRX_GSTAMPS=998    (gemm_timeline.py --lau2)
