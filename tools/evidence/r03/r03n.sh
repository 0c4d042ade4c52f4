#!/bin/bash
# pass A with the [t][c] inter-pass twiddle table: GPU suite (fast), nttbench, PoS and cfg3 lines
set -e
export TMPDIR=/tmp
OUT=gpurun_out/r03n; mkdir -p $OUT
T="timeout -k 10"
$T 700 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu_fast.log 2>&1
tail -1 $OUT/pytest_gpu_fast.log
$T 120 ./tools/microbench/nttbench 5 > $OUT/nttbench5.txt 2>&1
$T 120 ./tools/microbench/nttbench 1 > $OUT/nttbench1.txt 2>&1
B="python bench.py --code pos --steps 16 --warmup 4 --cpu-baseline off"
$T 300 $B --pipeline 1 > $OUT/pos_p1.json 2>> $OUT/b.err
$T 300 $B --pipeline 2 > $OUT/pos_p2.json 2>> $OUT/b.err
$T 400 python bench.py --steps 20 --warmup 5 --cpu-baseline off > $OUT/k20.json 2>> $OUT/b.err
echo ok
