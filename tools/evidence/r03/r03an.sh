#!/bin/bash
# the mixed-priority race vs hardware-queue pressure: mode 2 (mixed) with one hardware queue per
# priority per process, and mode 2 as is (checks: a failing run does not stop the next)
export TMPDIR=/tmp
OUT=gpurun_out/r03an2; mkdir -p $OUT
run() {  # name, env
  fails=0
  for i in $(seq 1 18); do
    env $2 timeout -k 10 300 python -u -m pytest tests/test_gpu_shard_native.py -k "pipeline_world8" -x -q --timeout 280 --timeout-method thread > $OUT/$1_$i.log 2>&1
    rc=$?
    if [ $rc -eq 1 ]; then fails=$((fails+1)); fi
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "$1 run $i rc=$rc stopping"; exit $rc; fi
  done
  echo "$1: failures $fails of 18"
}
run mixed_q1 "LCPC_SHARD_PRIO=2 GPU_MAX_HW_QUEUES=1"
run mixed_q4 "LCPC_SHARD_PRIO=2"
echo ok
