#!/bin/bash
# round-2 GPU measurement script: bench contract tests, the driver's default bench command, and
# engine / depth variants of the cfg3 line.  Every GPU step has its own time limit; the chain
# stops at the first failure.
set -e
OUT=${OUT:-gpurun_out/r02}
mkdir -p $OUT
T="timeout -k 10"
$T 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_bench_contract.py > $OUT/pytest_bench_contract.log 2>&1
$T 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_default_k20.json 2> $OUT/bench_default_k20.err
$T 300 python bench.py --gpus 1 --steps 256 --warmup 16 --cpu-baseline off > $OUT/bench_sharded_k256.json 2> $OUT/bench_sharded_k256.err
$T 300 python bench.py --gpus 1 --steps 20 --warmup 5 --mode replicas --cpu-baseline off > $OUT/bench_replicas_k20.json 2> $OUT/bench_replicas_k20.err
$T 300 python bench.py --gpus 1 --steps 256 --warmup 16 --mode replicas --cpu-baseline off > $OUT/bench_replicas_k256.json 2> $OUT/bench_replicas_k256.err
for lag in 1 3; do
  $T 300 python bench.py --gpus 1 --steps 64 --warmup 8 --lag $lag --cpu-baseline off --verify-reps 0 > $OUT/bench_sharded_lag$lag.json 2> $OUT/bench_sharded_lag$lag.err
done
