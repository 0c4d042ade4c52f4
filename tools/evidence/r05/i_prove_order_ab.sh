#!/bin/bash
# Round 5: K = 20 with the proofs interleaved (default) against commits-first scheduling
# (--prove-order), alternating on one box, 16 and 20 workers; a timeline of each order.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05i
mkdir -p $O
common="--gpus 1 --steps 20 --warmup 5 --cpu-baseline off --sharded-n1 0 --verify-reps 0"
for rep in 1 2 3; do
  for order in interleaved commits-first; do
    for w in 16 20; do
      timeout -k 10 200 python bench.py $common --prove-order $order --workers $w > $O/k20_${order}_w${w}_$rep.json 2> $O/k20_${order}_w${w}_$rep.err || { tail -20 $O/k20_${order}_w${w}_$rep.err; exit 1; }
      python3 -c "import json;d=json.loads(open('$O/k20_${order}_w${w}_$rep.json').read().strip().splitlines()[-1]);print('$order w$w rep$rep', round(d['value']/1e9,3), round(d['ms_per_step'],4))"
    done
  done
done
for order in interleaved commits-first; do
  timeout -k 10 200 python bench.py $common --prove-order $order --timeline $O/timeline_${order}.json > $O/k20_${order}_tl.json 2> $O/k20_${order}_tl.err || { tail -20 $O/k20_${order}_tl.err; exit 1; }
done
echo done
