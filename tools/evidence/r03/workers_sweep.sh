#!/bin/bash
# Host worker threads (steps in flight) at the driver's K = 20 and at K = 64: cfg4 (Brakedown,
# host-transcript bound) and cfg3 (Ligero, the BASELINE metric), alternating so box drift shows.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${1:-workers}; mkdir -p $OUT
T="timeout -k 10"
C="--cpu-baseline off --verify-reps 0 --no-prof --sharded-n1 0"
run() {  # tag, args...
  local tag=$1; shift
  $T 200 python bench.py $C "$@" > $OUT/$tag.json 2> $OUT/$tag.err
  python3 -c "import json; d=json.loads(open('$OUT/$tag.json').read().strip().splitlines()[-1]); print('$tag', round(d['value']/1e9,2), round(d['ms_per_step'],3))"
}
for rep in 1 2; do
  for w in 16 20 24; do run sdig_k20_w${w}_$rep --code sdig --steps 20 --warmup 5 --workers $w; done
  for w in 16 20 24; do run sdig_k64_w${w}_$rep --code sdig --steps 64 --warmup 5 --workers $w; done
  for w in 16 20; do run lig_k20_w${w}_$rep --steps 20 --warmup 5 --workers $w; done
done
