#!/bin/bash
# cfg2 (R-S encode alone) at round 2's step count, twice, and at the default
set -e
export TMPDIR=/tmp
OUT=gpurun_out/r03ao; mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 300 python bench.py --code encode --steps 512 --warmup 32 --cpu-baseline off > $OUT/enc512_$i.json 2>> $OUT/b.err
  python -c "import json;d=json.loads(open('$OUT/enc512_$i.json').read().strip().splitlines()[-1]);print('512', round(d['value']/1e9,3), round(d['ms_per_step']*1e3,1), 'us', d['host_cpu'] if 'host_cpu' in d else '')" | cut -c1-300
done
timeout -k 10 300 python bench.py --code encode --cpu-baseline off > $OUT/enc_def.json 2>> $OUT/b.err
python -c "import json;d=json.loads(open('$OUT/enc_def.json').read().strip().splitlines()[-1]);print('default', d['steps'], round(d['value']/1e9,3), round(d['ms_per_step']*1e3,1), 'us')"
echo ok
