#!/bin/bash
# the row-major leaf kernel's per-chunk body as a device function (no behaviour change): GPU suite
set -e
export TMPDIR=/tmp
OUT=gpurun_out/r03aq; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu_fast.log 2>&1
tail -1 $OUT/pytest_gpu_fast.log
timeout -k 10 800 python -u -m pytest tests -m "gpu and slow" -x -q --timeout 600 --timeout-method thread > $OUT/pytest_gpu_slow.log 2>&1
tail -1 $OUT/pytest_gpu_slow.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --cpu-baseline off > $OUT/k20.json 2> $OUT/b.err
python -c "import json;d=json.loads(open('$OUT/k20.json').read().strip().splitlines()[-1]);print('k20', round(d['value']/1e9,3), 'leaf', round(d['roofline_leaf']['avg_ms'],4), 'sharded_n1', round(d['sharded_n1'].get('value',0)/1e9,3))"
echo ok
