#!/bin/bash
# the default line with sharded_n1 from a fresh child process, twice
set -e
export TMPDIR=/tmp
OUT=gpurun_out/r03al; mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 500 python bench.py --steps 20 --warmup 5 --cpu-baseline off > $OUT/k20_$i.json 2>> $OUT/b.err
  python -c "import json;d=json.loads(open('$OUT/k20_$i.json').read().strip().splitlines()[-1]);print('k20', round(d['value']/1e9,3), 'sharded_n1', d['sharded_n1'])"
done
echo ok
