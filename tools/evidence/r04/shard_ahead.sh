#!/bin/bash
# round 4: the one-rank sharded K = 20 line over the encode look-ahead (LCPC_SHARD_AHEAD) with two
# encode streams, interleaved twice
set -o pipefail
O=gpurun_out/r04t
mkdir -p $O
for r in a b; do
  for a in 3 4 6; do
    LCPC_SHARD_AHEAD=$a timeout -k 10 300 python -u bench.py --mode sharded --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 > $O/ahead${a}_$r.json 2> $O/ahead${a}_$r.err || exit 1
  done
done
