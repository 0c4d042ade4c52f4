set -e
OUT=gpurun_out/r02l; mkdir -p $OUT
T="timeout -k 10"
for w in 5 20 5 40; do
  $T 200 python bench.py --gpus 1 --steps 20 --warmup $w --cpu-baseline off --verify-reps 0 --no-prof >> $OUT/bench_w.jsonl 2>> $OUT/bench.err
done
$T 200 python bench.py --gpus 1 --steps 20 --warmup 5 --pipeline 8 --cpu-baseline off --verify-reps 0 --no-prof >> $OUT/bench_p8.jsonl 2>> $OUT/bench.err
$T 200 python bench.py --gpus 1 --steps 20 --warmup 5 --pipeline 10 --cpu-baseline off --verify-reps 0 --no-prof >> $OUT/bench_p8.jsonl 2>> $OUT/bench.err
echo ok
