set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for c in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU_MFMA_F64 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  tag=$(echo $c | cut -d' ' -f1)
  timeout -k 10 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc_$tag -o p -- python3 scratch/prof_run.py 8 > /dev/null 2>&1 || { echo "pmc $c failed"; exit 1; }
  echo "done $c"
done
