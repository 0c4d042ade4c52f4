#!/bin/bash
# the sharded driver's prove streams at the encode stream's priority: the 8-rank pipelined test
# twelve times (checks: a failing run does not stop the next; a timeout / abort / crash ends the
# script), then the GPU suite and the K = 20 line (its sharded_n1 figure)
export TMPDIR=/tmp
OUT=gpurun_out/r03ac; mkdir -p $OUT
fails=0
for i in $(seq 1 12); do
  timeout -k 10 300 python -u -m pytest tests/test_gpu_shard_native.py -k "pipeline_world8" -x -q --timeout 280 --timeout-method thread > $OUT/w8_$i.log 2>&1
  rc=$?
  echo "world8 run $i rc=$rc $(grep -o "bad_root_polys': \[([0-9]*" $OUT/w8_$i.log | sort | uniq -c | tr '\n' ' ')"
  if [ $rc -eq 1 ]; then fails=$((fails+1)); fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo stopping; exit $rc; fi
done
echo "world8 failures: $fails of 12"
set -e
timeout -k 10 700 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu_fast.log 2>&1
tail -1 $OUT/pytest_gpu_fast.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --cpu-baseline off > $OUT/k20.json 2> $OUT/b.err
echo ok
