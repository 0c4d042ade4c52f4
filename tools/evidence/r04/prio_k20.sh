#!/bin/bash
# round 4: cfg3 K = 20 under the three stream-priority policies (LCPC_PRIORITY_STREAMS 1 / 2 / 0),
# interleaved twice, with the replicas timeline of each
set -o pipefail
O=gpurun_out/r04l
mkdir -p $O
for r in a b; do
  for m in 1 2 0; do
    LCPC_PRIORITY_STREAMS=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --sharded-n1 0 --cpu-baseline off --verify-reps 0 > $O/k20_p${m}_$r.json 2> $O/k20_p${m}_$r.err || exit 1
  done
done
