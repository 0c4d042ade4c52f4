#!/bin/bash
# cfg4 (Brakedown) at the driver's K = 20: per-step gate / commit / prove timelines at the default
# admission (2 commit slots, 16 workers) and at two alternatives, to see where the host-transcript
# bound run loses time against 20 x 26 ms of Keccak over a 16-CPU quota.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${1:-sdig_k20}; mkdir -p $OUT
T="timeout -k 10"
B="python bench.py --code sdig --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 --no-prof"
$T 200 $B --timeline $OUT/tl_default.json > $OUT/default.json 2> $OUT/default.err
$T 200 $B --commit-slots 4 --timeline $OUT/tl_slots4.json > $OUT/slots4.json 2> $OUT/slots4.err
$T 200 $B --workers 20 --timeline $OUT/tl_workers20.json > $OUT/workers20.json 2> $OUT/workers20.err
$T 200 $B --workers 10 --timeline $OUT/tl_workers10.json > $OUT/workers10.json 2> $OUT/workers10.err
for f in default slots4 workers20 workers10; do
  python3 -c "import json,sys; d=json.loads(open('$OUT/$f.json').read().strip().splitlines()[-1]); print('$f', round(d['value']/1e9,2), round(d['ms_per_step'],2), d.get('host_cpu',{}).get('cores_busy'))"
done
