#!/bin/bash
# the sharded engine at N = 1, K = 20 under the three prove-stream modes (same box, interleaved)
set -e
export TMPDIR=/tmp
OUT=gpurun_out/r03ae; mkdir -p $OUT
B="timeout -k 10 300 python bench.py --mode sharded --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0"
for rep in 1 2; do
  for m in 1 0 2; do
    LCPC_SHARD_PRIO=$m $B > $OUT/prio${m}_$rep.json 2>> $OUT/b.err
    python -c "import json;d=json.loads(open('$OUT/prio${m}_$rep.json').read().strip().splitlines()[-1]);print('prio $m rep $rep', round(d['value']/1e9,3), round(d['ms_per_step'],3))"
  done
done
echo ok
