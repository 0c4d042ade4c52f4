#!/bin/bash
# the bench line's sharded_n1 (in the same process after the replicas run) and the standalone
# sharded N = 1 rate under prove-stream modes 0 / 1 / 3, interleaved on one box
set -e
export TMPDIR=/tmp
OUT=gpurun_out/r03ah; mkdir -p $OUT
for rep in 1 2; do
  for m in 3 0 1; do
    LCPC_SHARD_PRIO=$m timeout -k 10 400 python bench.py --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 > $OUT/line_m${m}_$rep.json 2>> $OUT/b.err
    LCPC_SHARD_PRIO=$m timeout -k 10 300 python bench.py --mode sharded --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 > $OUT/sh_m${m}_$rep.json 2>> $OUT/b.err
    python -c "import json;d=json.loads(open('$OUT/line_m${m}_$rep.json').read().strip().splitlines()[-1]);e=json.loads(open('$OUT/sh_m${m}_$rep.json').read().strip().splitlines()[-1]);print('mode $m rep $rep line', round(d['value']/1e9,3), 'sharded_n1', round(d['sharded_n1']['value']/1e9,3), 'standalone', round(e['value']/1e9,3))"
  done
done
echo ok
