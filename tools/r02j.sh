set -e
OUT=gpurun_out/r02j; mkdir -p $OUT
T="timeout -k 10"
$T 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_shard_native.py tests/test_gpu_bench_contract.py > $OUT/pytest.log 2>&1
$T 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_default.json 2>> $OUT/bench.err
$T 200 python bench.py --gpus 1 --steps 256 --warmup 16 --cpu-baseline off --verify-reps 0 > $OUT/bench_k256.json 2>> $OUT/bench.err
$T 200 python bench.py --gpus 1 --mode sharded --steps 128 --warmup 8 --prof-timed --cpu-baseline off --verify-reps 0 > $OUT/bench_sharded_proftimed.json 2>> $OUT/bench.err
$T 200 python bench.py --gpus 1 --mode sharded --steps 256 --warmup 8 --lag 4 --cpu-baseline off --verify-reps 0 > $OUT/bench_sharded_k256.json 2>> $OUT/bench.err
echo ok
