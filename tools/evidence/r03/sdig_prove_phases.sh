#!/bin/bash
# cfg4 replicas: where a proof's host time goes (transcript vs waits on the GPU) at K = 20 and 64,
# from the library's host scopes (bench.py --prof-timed; averages per call in the line's "kernels").
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${1:-sdig_phases}; mkdir -p $OUT
T="timeout -k 10"
for k in 20 64; do
  $T 200 python bench.py --code sdig --steps $k --warmup 5 --cpu-baseline off --verify-reps 0 --sharded-n1 0 --prof-timed > $OUT/k$k.json 2> $OUT/k$k.err
  python3 -c "
import json; d=json.loads(open('$OUT/k$k.json').read().strip().splitlines()[-1])
print('K=$k', round(d['value']/1e9,2), round(d['ms_per_step'],3), 'cores_busy', d.get('host_cpu',{}).get('cores_busy'))
for n,v in sorted(d['kernels'].items()):
    if n.startswith('host_'): print('  ', n, v)
"
done
