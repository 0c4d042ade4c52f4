#!/bin/bash
# two-pass leaf merge + LDS-staged pack7: GPU suite (fast), PoS and cfg3 lines
set -e
export TMPDIR=/tmp
OUT=gpurun_out/r03p; mkdir -p $OUT
T="timeout -k 10"
$T 700 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu_fast.log 2>&1
tail -1 $OUT/pytest_gpu_fast.log
B="python bench.py --code pos --steps 16 --warmup 4 --cpu-baseline off"
$T 300 $B --pipeline 1 > $OUT/pos_p1.json 2>> $OUT/b.err
$T 300 $B --pipeline 2 > $OUT/pos_p2.json 2>> $OUT/b.err
$T 400 python bench.py --steps 20 --warmup 5 --cpu-baseline off > $OUT/k20.json 2>> $OUT/b.err
$T 400 python bench.py --code sdig --steps 20 --warmup 5 --cpu-baseline off > $OUT/sdig.json 2>> $OUT/b.err
echo ok
