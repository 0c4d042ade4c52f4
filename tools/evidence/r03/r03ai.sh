#!/bin/bash
# the sharded engine at N = 1, K = 20: encodes queued ahead 3 / 6 / 10, and lag 3 / 5 (A/B)
set -e
export TMPDIR=/tmp
OUT=gpurun_out/r03ai; mkdir -p $OUT
B="timeout -k 10 300 python bench.py --mode sharded --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0"
for rep in 1 2; do
  for a in 3 6 10; do
    LCPC_SHARD_AHEAD=$a $B > $OUT/a${a}_$rep.json 2>> $OUT/b.err
    python -c "import json;d=json.loads(open('$OUT/a${a}_$rep.json').read().strip().splitlines()[-1]);print('ahead $a rep $rep', round(d['value']/1e9,3), round(d['ms_per_step'],3))"
  done
  LCPC_SHARD_AHEAD=6 $B --lag 5 > $OUT/a6_lag5_$rep.json 2>> $OUT/b.err || true
  python -c "import json;d=json.loads(open('$OUT/a6_lag5_$rep.json').read().strip().splitlines()[-1]);print('ahead 6 lag 5 rep $rep', round(d['value']/1e9,3), round(d['ms_per_step'],3))" || true
done
echo ok
