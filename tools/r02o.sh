set -e
OUT=gpurun_out/r02o; mkdir -p $OUT
T="timeout -k 10"
$T 500 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_sdig.py tests/test_gpu_collapse.py tests/test_gpu_shard_native.py > $OUT/pytest.log 2>&1
$T 200 python bench.py --mode sharded --steps 128 --warmup 8 --lag 4 --prof-timed --cpu-baseline off --verify-reps 0 > $OUT/bench_sharded_proftimed.json 2>> $OUT/bench.err
echo ok
