#!/bin/bash
# 8-rank pipelined root mismatch: stream-priority knobs (checks, not faults: a failing run does
# not stop the next; a timeout / abort / crash ends it)
export TMPDIR=/tmp
OUT=gpurun_out/r03ab; mkdir -p $OUT
run() {  # name, env
  for i in 1 2 3 4 5 6 7 8; do
    env $2 timeout -k 10 300 python -u -m pytest tests/test_gpu_shard_native.py -k "pipeline_world8" -x -q --timeout 280 --timeout-method thread > $OUT/$1_$i.log 2>&1
    rc=$?
    echo "$1 run $i rc=$rc $(grep -o "bad_root_polys': \[([0-9]*" $OUT/$1_$i.log | sort | uniq -c | tr '\n' ' ')"
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo stopping; exit $rc; fi
  done
}
run oneprio "LCPC_PRIORITY_STREAMS=0"
run sharedsp "LCPC_SHARD_PRIO=0"
echo ok
