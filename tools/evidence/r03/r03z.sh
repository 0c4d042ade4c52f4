#!/bin/bash
# the 8-rank pipelined root mismatch: dump every rank's subtree roots at each commit and, on a
# mismatch, the single commitment's (checks, not faults: a failing run does not stop the next)
export TMPDIR=/tmp
OUT=gpurun_out/r03z; mkdir -p $OUT
export LCPC_SHARD_ROOT_CHECK=1
fails=0
for i in 1 2 3 4 5 6 7 8 9 10; do
  timeout -k 10 300 python -u -m pytest tests/test_gpu_shard_native.py -k "pipeline_world8" -x -q -s --timeout 280 --timeout-method thread > $OUT/run$i.log 2>&1
  rc=$?
  echo "run $i rc=$rc"
  if [ $rc -eq 1 ]; then fails=$((fails+1)); fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo stopping; exit $rc; fi
  if [ $fails -ge 2 ]; then break; fi
done
echo ok
