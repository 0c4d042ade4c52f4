#!/bin/bash
# 8-rank pipelined root mismatch: is it the reuse of the commit scratch blocks? (checks, not
# faults: a failing run does not stop the next; a timeout / abort / crash ends it)
export TMPDIR=/tmp
OUT=gpurun_out/r03aa; mkdir -p $OUT
for i in 1 2 3 4 5 6 7 8 9 10 11 12; do
  env LCPC_SHARD_KEEP_SCRATCH=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_shard_native.py -k "pipeline_world8" -x -q --timeout 280 --timeout-method thread > $OUT/keep_$i.log 2>&1
  rc=$?
  echo "keep run $i rc=$rc $(grep -o "bad_root_polys': \[([0-9]*" $OUT/keep_$i.log | sort | uniq -c | tr '\n' ' ')"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo stopping; exit $rc; fi
done
echo ok
