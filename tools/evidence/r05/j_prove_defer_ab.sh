#!/bin/bash
# Round 5: K = 20 with up to M finished commitments' proofs deferred while commitments run
# (--prove-defer M, FIFO), M = 0 (default) / 4 / 6 / 8, 16 and 20 workers, alternating on one box.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05j
mkdir -p $O
common="--gpus 1 --steps 20 --warmup 5 --cpu-baseline off --sharded-n1 0 --verify-reps 0"
for rep in 1 2; do
  for m in 0 4 6 8; do
    for w in 16 20; do
      timeout -k 10 200 python bench.py $common --prove-defer $m --workers $w > $O/k20_m${m}_w${w}_$rep.json 2> $O/k20_m${m}_w${w}_$rep.err || { tail -20 $O/k20_m${m}_w${w}_$rep.err; exit 1; }
      python3 -c "import json;d=json.loads(open('$O/k20_m${m}_w${w}_$rep.json').read().strip().splitlines()[-1]);print('m$m w$w rep$rep', round(d['value']/1e9,3), round(d['ms_per_step'],4), d.get('steps_agree'))"
    done
  done
done
for m in 0 6; do
  timeout -k 10 200 python bench.py $common --prove-defer $m --workers 20 --timeline $O/timeline_m$m.json > $O/k20_m${m}_tl.json 2> $O/k20_m${m}_tl.err || { tail -20 $O/k20_m${m}_tl.err; exit 1; }
done
echo done
