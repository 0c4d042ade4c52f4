#!/bin/bash
# prove-stream modes: 3 = every driver stream high priority, 0 = prove work on the encode stream.
# The 8-rank pipelined test 8 times each (checks: a failing run does not stop the next; a
# timeout / abort / crash ends it), then the sharded N = 1 K = 20 rate of each mode twice
export TMPDIR=/tmp
OUT=gpurun_out/r03af; mkdir -p $OUT
for m in 3 0; do
  fails=0
  for i in 1 2 3 4 5 6 7 8; do
    LCPC_SHARD_PRIO=$m timeout -k 10 300 python -u -m pytest tests/test_gpu_shard_native.py -k "pipeline_world8" -x -q --timeout 280 --timeout-method thread > $OUT/m${m}_$i.log 2>&1
    rc=$?
    if [ $rc -eq 1 ]; then fails=$((fails+1)); fi
    if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "mode $m run $i rc=$rc stopping"; exit $rc; fi
  done
  echo "mode $m: world8 failures $fails of 8"
done
set -e
B="timeout -k 10 300 python bench.py --mode sharded --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0"
for rep in 1 2; do
  for m in 3 0 2; do
    LCPC_SHARD_PRIO=$m $B > $OUT/rate_m${m}_$rep.json 2>> $OUT/b.err
    python -c "import json;d=json.loads(open('$OUT/rate_m${m}_$rep.json').read().strip().splitlines()[-1]);print('mode $m rep $rep', round(d['value']/1e9,3), round(d['ms_per_step'],3))"
  done
done
echo ok
