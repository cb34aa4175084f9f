#!/bin/bash
# Reproducibility under a concurrent GPU process, one library variant after another:
#   bash scratch/conc_ab.sh SECONDS NAME[=LIB] ...   (LIB empty: the in-tree library)
S=scratch/concurrency.py
secs=$1; shift
mkdir -p gpurun_out
for v in "$@"; do
  name=${v%%=*}; lib=${v#*=}; [ "$lib" = "$v" ] && lib=""
  timeout -k 10 300 python -u $S load-torch --seconds $((secs + 20)) > gpurun_out/cab_load_$name.json 2>&1 &
  lp=$!
  sleep 8
  if [ -n "$lib" ]; then export GPRX_LIB=$lib; else unset GPRX_LIB; fi
  timeout -k 10 300 python -u $S probe --seconds $secs > gpurun_out/cab_$name.json 2> gpurun_out/cab_$name.err
  rc=$?
  unset GPRX_LIB
  wait $lp
  python3 -c "import json; d=json.load(open('gpurun_out/cab_$name.json')); print('$name', d['evaluations'], d['mismatches'], [list(r.get('status',{}).values()) for r in d['first'][:4]])" || echo "$name rc=$rc"
done
