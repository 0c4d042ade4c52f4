set -e
OUT=gpurun_out/r02c; mkdir -p $OUT
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_shard_native.py -k "not full_size" > $OUT/pytest_shard_native.log 2>&1
for lag in 2 3 4 6; do
  $T 200 python bench.py --gpus 1 --steps 256 --warmup 16 --lag $lag --cpu-baseline off --verify-reps 0 > $OUT/bench_lag$lag.json 2> $OUT/bench_lag$lag.err
done
$T 200 python bench.py --gpus 1 --steps 20 --warmup 5 --lag 4 --cpu-baseline off --verify-reps 0 > $OUT/bench_lag4_k20.json 2> $OUT/bench_lag4_k20.err
echo ok
