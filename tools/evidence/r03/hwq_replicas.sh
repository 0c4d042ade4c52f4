#!/bin/bash
# cfg3 replicas at the driver's K = 20: hardware queues per process (HIP's default 4 against 8),
# alternating so box drift shows.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${1:-hwq}; mkdir -p $OUT
C="--steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 --no-prof --sharded-n1 0"
for rep in 1 2 3; do
  for q in 4 8; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py $C > $OUT/q${q}_$rep.json 2> $OUT/q${q}_$rep.err
    python3 -c "import json; d=json.loads(open('$OUT/q${q}_$rep.json').read().strip().splitlines()[-1]); print('hwq=$q rep $rep', round(d['value']/1e9,2), round(d['ms_per_step'],3))"
  done
done
