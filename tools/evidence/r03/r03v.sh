#!/bin/bash
# reproduce the 8-rank pipelined root mismatch seen once under pytest (checks, not a fault: a
# failing run does not stop the next; a timeout / abort / crash ends the script)
export TMPDIR=/tmp
OUT=gpurun_out/r03v3; mkdir -p $OUT
export LCPC_SHARD_ROOT_CHECK=1
for i in 1 2 3 4 5 6 7 8 9 10; do
  timeout -k 10 300 python -u -m pytest tests/test_gpu_shard_native.py -k "pipeline_world8" -x -q --timeout 280 --timeout-method thread > $OUT/run$i.log 2>&1
  rc=$?
  echo "run $i rc=$rc"; grep -E "AssertionError|passed|failed|staged root" $OUT/run$i.log | head -12 | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo stopping; exit $rc; fi
done
echo ok
