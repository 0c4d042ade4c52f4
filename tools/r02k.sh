set -e
OUT=gpurun_out/r02k; mkdir -p $OUT
T="timeout -k 10"
$T 200 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 > $OUT/bench_default.json 2>> $OUT/bench.err
LCPC_SDIG_ROWS=16 $T 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_gpu_sdig.py > $OUT/pytest_sdig_rows16.log 2>&1
for r in 0 40 24 16; do
  LCPC_SDIG_ROWS=$r $T 200 python bench.py --gpus 1 --code sdig --steps 32 --warmup 8 --cpu-baseline off --verify-reps 0 > $OUT/bench_sdig_rows$r.json 2>> $OUT/bench.err
  LCPC_SDIG_VALU=1 LCPC_SDIG_ROWS=$r $T 200 python bench.py --gpus 1 --code sdig --steps 32 --warmup 8 --cpu-baseline off --verify-reps 0 > $OUT/bench_sdig_valu_rows$r.json 2>> $OUT/bench.err
done
echo ok
