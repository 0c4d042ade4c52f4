set -e
OUT=gpurun_out/r02n; mkdir -p $OUT
T="timeout -k 10"
$T 60 tools/microbench/transcript_bench > $OUT/tb_auto.txt
LCPC_KECCAK=scalar $T 60 tools/microbench/transcript_bench > $OUT/tb_scalar.txt
$T 200 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 --timeline $OUT/tl_k20.json > $OUT/bench_k20.json 2>> $OUT/bench.err
$T 200 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 --no-prof --timeline $OUT/tl_k20_noprof.json > $OUT/bench_k20_noprof.json 2>> $OUT/bench.err
echo ok
