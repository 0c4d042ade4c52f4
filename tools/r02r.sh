#!/bin/bash
# sharded-driver teardown fix: its GPU tests, the one-rank sharded line (prof-timed phases and
# plain, lags 3/4/auto), then the whole fast GPU suite and the driver's default line
set -e
OUT=gpurun_out/r02r; mkdir -p $OUT
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_shard_native.py -k "not full_size" > $OUT/pytest_shard.log 2>&1
$T 200 python bench.py --mode sharded --steps 128 --warmup 8 --lag 4 --prof-timed --cpu-baseline off --verify-reps 0 > $OUT/bench_sharded_proftimed.json 2> $OUT/bench.err
for lag in 0 3 4; do
  $T 200 python bench.py --mode sharded --steps 256 --warmup 8 --lag $lag --cpu-baseline off --verify-reps 0 > $OUT/bench_sharded_k256_lag$lag.json 2>> $OUT/bench.err
done
$T 200 python bench.py --mode sharded --steps 20 --warmup 5 --lag 4 --cpu-baseline off --verify-reps 0 > $OUT/bench_sharded_k20.json 2>> $OUT/bench.err
$T 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu_fast.log 2>&1
$T 200 python bench.py --steps 20 --warmup 5 > $OUT/bench_default.json 2>> $OUT/bench.err
echo ok
