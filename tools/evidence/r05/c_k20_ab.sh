#!/bin/bash
# Round 5: K = 20 admission / priority A/B (interleaved, quick lines: no cpu baseline, no sharded
# N = 1 child, no verify), one line with every host phase timed inside the timed region.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05c
mkdir -p $O
Q="--gpus 1 --steps 20 --warmup 5 --cpu-baseline off --sharded-n1 0 --verify-reps 0"
run() {  # tag, env / args...
  local tag=$1; shift
  timeout -k 10 180 env "$@" > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$O/$tag.json')); print('$tag', round(d['value']/1e9,3), round(d['ms_per_step'],4))"
}
for r in a b; do
  run k20_cs4_$r python3 bench.py $Q --timeline $O/tl_cs4_$r.json
  run k20_cs2_$r python3 bench.py $Q --commit-slots 2 --timeline $O/tl_cs2_$r.json
  run k20_cs3_$r python3 bench.py $Q --commit-slots 3
  run k20_cs6_$r python3 bench.py $Q --commit-slots 6
  run k20_p1_$r LCPC_PRIORITY_STREAMS=1 python3 bench.py $Q --timeline $O/tl_p1_$r.json
  run k20_w20_$r python3 bench.py $Q --workers 20
done
run k20_proftimed python3 bench.py $Q --prof-timed --timeline $O/tl_proftimed.json
echo done
