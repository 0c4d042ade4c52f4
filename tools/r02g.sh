set -e
OUT=gpurun_out/r02g; mkdir -p $OUT
T="timeout -k 10"
for lag in 3 4 6; do
  $T 200 python bench.py --gpus 1 --steps 256 --warmup 8 --lag $lag --prof-timed --cpu-baseline off --verify-reps 0 > $OUT/bench_lag${lag}_k256.json 2>> $OUT/bench.err
  $T 200 python bench.py --gpus 1 --steps 20 --warmup 5 --lag $lag --cpu-baseline off --verify-reps 0 > $OUT/bench_lag${lag}_k20.json 2>> $OUT/bench.err
done
$T 200 python bench.py --gpus 1 --steps 20 --warmup 5 --mode replicas --cpu-baseline off --verify-reps 0 > $OUT/bench_replicas_k20.json 2>> $OUT/bench.err
$T 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_sdig.py > $OUT/pytest_sdig.log 2>&1
$T 200 python bench.py --gpus 1 --code sdig --steps 32 --warmup 8 --cpu-baseline off --verify-reps 1 > $OUT/bench_sdig.json 2>> $OUT/bench.err
LCPC_SDIG_VALU=1 $T 200 python bench.py --gpus 1 --code sdig --steps 32 --warmup 8 --cpu-baseline off --verify-reps 1 > $OUT/bench_sdig_valu.json 2>> $OUT/bench.err
echo ok
