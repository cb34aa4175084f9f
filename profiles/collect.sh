#!/bin/bash
# Round profile: rocprofv3 kernel trace + stats of the default bench, then PMC passes (one counter
# group per pass, --kernel-trace only, as MI355X_MICROARCH.md prescribes), summarised into
# profiles/<round>_summary.json (+ pmc_latest.json, read by bench.py for roofline.traffic).
# usage (GPU box):  bash profiles/collect.sh r01 [bench args...]
set -e
R=${1:-r01}; shift || true
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp && cd "$ROOT"
OUT=gpurun_out/prof_$R
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu --no-opt "$@" > $OUT/bench_under_rocprof.json
echo "trace done"
for c in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "SQ_INSTS_VALU_MFMA_F64 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE"; do
  tag=$(echo $c | cut -d' ' -f1)_$(echo $c | wc -w)
  timeout -s KILL 400 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/pmc_$tag -o p -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu --no-prof --no-opt "$@" > /dev/null
  echo "pmc $c done"
done
python3 profiles/summarize.py $OUT $R
# the summaries land in the box's profiles/; copy them back with the run's other outputs
cp profiles/${R}_summary.json profiles/pmc_latest.json $OUT/
