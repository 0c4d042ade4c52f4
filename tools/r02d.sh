set -e
OUT=gpurun_out/r02d; mkdir -p $OUT
T="timeout -k 10"
$T 200 python bench.py --gpus 1 --steps 128 --warmup 8 --prof-timed --cpu-baseline off --verify-reps 0 > $OUT/bench_proftimed.json 2> $OUT/bench_proftimed.err
$T 100 tools/microbench/transcript_bench > $OUT/transcript_bench.txt
LCPC_KECCAK=scalar $T 100 tools/microbench/transcript_bench > $OUT/transcript_bench_scalar.txt
echo ok
