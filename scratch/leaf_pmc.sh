#!/bin/bash
# PMC counters of the fused leaf on the bench workload (one pass per counter group)
set -e
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 60 rocprofv3 -L > gpurun_out/lp_avail.txt 2>&1 || true
grep -o "SQ_[A-Z0-9_]*\|TA_[A-Z0-9_]*\|TD_[A-Z0-9_]*\|TCP_[A-Z0-9_]*" gpurun_out/lp_avail.txt | sort -u > gpurun_out/lp_names.txt || true
echo "names $(wc -l < gpurun_out/lp_names.txt)"
pass() {
  tag=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv -d gpurun_out/lp_$tag -o p -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu --no-prof --no-opt > /dev/null 2>&1
  echo "pass $tag ok"
}
pass a SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES
pass b SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE
