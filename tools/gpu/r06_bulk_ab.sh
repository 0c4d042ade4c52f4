#!/bin/bash
# the row-sharded driver's encode streams (LCPC_SHARD_BULK_STREAMS 2 / 3 / 4) on one GPU,
# interleaved, at K = 160 (the weak N = 8 line's commitment count) and K = 20
set -o pipefail
O=gpurun_out/${1:-r06t}
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2; do
  for b in 2 3 4; do
    for k in 160 20; do
      LCPC_SHARD_BULK_STREAMS=$b timeout -k 10 300 python bench.py --mode sharded --steps $k --warmup 5 --cpu-baseline off --verify-reps 0 --sharded-n1 0 --no-prof > $O/b${b}_k${k}_r${rep}.json 2> $O/b${b}_k${k}_r${rep}.err || { tail -20 $O/b${b}_k${k}_r${rep}.err; exit 1; }
    done
  done
done
echo done
