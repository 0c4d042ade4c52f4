#!/bin/bash
# Round 5: the host phases of every proof in a K = 20 run (LCPC_PROF_TIMELINE, host scopes only),
# aligned with the per-step timeline: where the last proof's 4.7 ms goes against its 3.9 ms alone
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05l
mkdir -p $O
for r in a b; do
  rm -f $O/phases_$r.csv
  LCPC_PROF_TIMELINE=$O/phases_$r.csv LCPC_PROF_HOST_ONLY=1 timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 \
    --prof-timed --timeline $O/tl_$r.json --cpu-baseline off --sharded-n1 0 --verify-reps 0 > $O/k20_$r.json 2> $O/k20_$r.err \
    || { tail -20 $O/k20_$r.err; exit 1; }
done
echo done
