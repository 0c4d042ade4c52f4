set -e
OUT=gpurun_out/r02h; mkdir -p $OUT
T="timeout -k 10"
for cs in 0 1 2 3; do
  $T 200 python bench.py --gpus 1 --steps 20 --warmup 5 --commit-slots $cs --cpu-baseline off --verify-reps 0 --no-prof > $OUT/bench_cs${cs}_k20.json 2>> $OUT/bench.err
  $T 200 python bench.py --gpus 1 --steps 256 --warmup 16 --commit-slots $cs --cpu-baseline off --verify-reps 0 --no-prof > $OUT/bench_cs${cs}_k256.json 2>> $OUT/bench.err
done
for cs in 0 2; do
  $T 200 python bench.py --gpus 1 --code sdig --steps 32 --warmup 8 --commit-slots $cs --cpu-baseline off --verify-reps 0 --no-prof > $OUT/bench_sdig_cs${cs}.json 2>> $OUT/bench.err
done
$T 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_sdig -o run --output-format csv -- python3 bench.py --code sdig --steps 4 --warmup 2 --pipeline 1 --cpu-baseline off --verify-reps 0 > $OUT/bench_sdig_prof.json 2> $OUT/prof_sdig.err
echo ok
