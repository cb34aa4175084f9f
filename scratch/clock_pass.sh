set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU_MFMA_F64 SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/clk -o p -- python3 scratch/prof_run.py 32 > /dev/null 2>&1
echo done
head -3 gpurun_out/clk/*counter_collection.csv
