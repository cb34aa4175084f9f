set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for f in 0 1; do
GPRX_LAUUM_FOLD=$f timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/pf$f -o p -- python3 scratch/prof_run.py 32 > /dev/null 2>&1
echo "fold=$f"; python3 scratch/sq_ana.py gpurun_out/pf$f/p_counter_collection.csv TCC_HIT_sum,TCC_MISS_sum | grep -E "lauum|k_gemm "
done
