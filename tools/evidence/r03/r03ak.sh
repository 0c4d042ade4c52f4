#!/bin/bash
# the mixed-priority race (LCPC_SHARD_PRIO=2) with and without the immediate flush after every
# event record (checks: a failing run does not stop the next; a timeout / abort / crash ends it)
export TMPDIR=/tmp
OUT=gpurun_out/r03ak; mkdir -p $OUT
run() {  # name, env
  fails=0
  for i in 1 2 3 4 5 6 7 8 9 10; do
    env $2 timeout -k 10 300 python -u -m pytest tests/test_gpu_shard_native.py -k "pipeline_world8" -x -q --timeout 280 --timeout-method thread > $OUT/$1_$i.log 2>&1
    rc=$?
    if [ $rc -eq 1 ]; then fails=$((fails+1)); fi
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "$1 run $i rc=$rc stopping"; exit $rc; fi
  done
  echo "$1: failures $fails of 10"
}
run mixed_flush "LCPC_SHARD_PRIO=2"
run mixed_noflush "LCPC_SHARD_PRIO=2 LCPC_SHARD_FLUSH=0"
echo ok
