set -e
OUT=gpurun_out/r02i; mkdir -p $OUT
T="timeout -k 10"
$T 300 python tools/encode_rows_bench.py --rows 512 --threads 16 > $OUT/encode_rows.json 2> $OUT/encode_rows.err
for cs in 4 6; do
  $T 200 python bench.py --gpus 1 --steps 20 --warmup 5 --commit-slots $cs --cpu-baseline off --verify-reps 0 --no-prof > $OUT/bench_cs${cs}_k20.json 2>> $OUT/bench.err
  $T 200 python bench.py --gpus 1 --steps 256 --warmup 16 --commit-slots $cs --cpu-baseline off --verify-reps 0 --no-prof > $OUT/bench_cs${cs}_k256.json 2>> $OUT/bench.err
done
for cs in 1 3 4; do
  $T 200 python bench.py --gpus 1 --code sdig --steps 32 --warmup 8 --commit-slots $cs --cpu-baseline off --verify-reps 0 --no-prof > $OUT/bench_sdig_cs${cs}.json 2>> $OUT/bench.err
done
$T 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_bench_contract.py > $OUT/pytest_contract.log 2>&1
echo ok
