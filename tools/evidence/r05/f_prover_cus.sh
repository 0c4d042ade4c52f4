#!/bin/bash
# Round 5: K = 20 with lcpc_prove's streams on k CUs (LCPC_PROVER_CUS; 0 = all), interleaved.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05f
mkdir -p $O
Q="--gpus 1 --steps 20 --warmup 5 --cpu-baseline off --sharded-n1 0 --verify-reps 0"
run() {
  local tag=$1; shift
  timeout -k 10 180 env "$@" > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$tag.json')); print('$tag', round(d['value']/1e9,3), round(d['ms_per_step'],4))"
}
for r in a b; do
  for k in 0 32 64 16; do
    run k20_cus${k}_$r LCPC_PROVER_CUS=$k python3 bench.py $Q --timeline $O/tl_cus${k}_$r.json
  done
done
echo done
