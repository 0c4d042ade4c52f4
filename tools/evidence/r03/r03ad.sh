#!/bin/bash
# after the priority fix: the full-size set (incl. cfg3 over 8 RCCL ranks on one GPU), smoke and
# the default K = 20 line twice
set -e
export TMPDIR=/tmp
OUT=gpurun_out/r03ad; mkdir -p $OUT
T="timeout -k 10"
$T 800 python -u -m pytest tests -m "gpu and slow" -x -v --timeout 600 --timeout-method thread > $OUT/pytest_gpu_slow.log 2>&1
tail -1 $OUT/pytest_gpu_slow.log
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
$T 400 python bench.py --steps 20 --warmup 5 > $OUT/k20_a.json 2> $OUT/b.err
$T 400 python bench.py --steps 20 --warmup 5 --cpu-baseline off > $OUT/k20_b.json 2>> $OUT/b.err
echo ok
