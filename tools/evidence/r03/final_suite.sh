#!/bin/bash
# The driver's round-end GPU steps on the final tree: pytest -m gpu (one process), smoke(), and
# the default bench line at the driver's K = 20 / W = 5.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${1:-final_suite}; mkdir -p $OUT
T="timeout -k 10"
$T 800 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
tail -1 $OUT/pytest_gpu.log
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
$T 400 python bench.py --steps 20 --warmup 5 > $OUT/bench_k20.json 2> $OUT/bench_k20.err
python3 -c "import json; d=json.loads(open('$OUT/bench_k20.json').read().strip().splitlines()[-1]); print(round(d['value']/1e9,2), round(d['ms_per_step'],3), (d.get('sharded_n1') or {}).get('value'))"
