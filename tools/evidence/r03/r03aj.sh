#!/bin/bash
# two-chunk column-major leaves hashed whole by one wave: parity (leaf, SDIG, PoS, verify paths)
# and the cfg4 line's leaf roofline
set -e
export TMPDIR=/tmp
OUT=gpurun_out/r03aj; mkdir -p $OUT
timeout -k 10 700 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu_fast.log 2>&1
tail -1 $OUT/pytest_gpu_fast.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py -x -q --timeout 280 --timeout-method thread -k cfg4 > $OUT/pytest_cfg4.log 2>&1
tail -1 $OUT/pytest_cfg4.log
timeout -k 10 400 python bench.py --code sdig --steps 20 --warmup 5 --cpu-baseline off > $OUT/sdig.json 2> $OUT/b.err
python -c "import json;d=json.loads(open('$OUT/sdig.json').read().strip().splitlines()[-1]);print('sdig', round(d['value']/1e9,3), d['roofline_leaf']['frac'], d['roofline_leaf']['avg_ms'])"
echo ok
