set -e
OUT=gpurun_out/r02m; mkdir -p $OUT
T="timeout -k 10"
$T 60 tools/microbench/transcript_bench > $OUT/tb_auto.txt
LCPC_KECCAK=scalar $T 60 tools/microbench/transcript_bench > $OUT/tb_scalar.txt
LCPC_KECCAK=avx512 $T 60 tools/microbench/transcript_bench > $OUT/tb_avx512.txt
$T 200 python bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off --verify-reps 2 > $OUT/bench_k20.json 2>> $OUT/bench.err
$T 200 python bench.py --gpus 1 --steps 256 --warmup 16 --cpu-baseline off --verify-reps 0 > $OUT/bench_k256.json 2>> $OUT/bench.err
$T 200 python bench.py --gpus 1 --code sdig --steps 32 --warmup 8 --cpu-baseline off --verify-reps 2 > $OUT/bench_sdig.json 2>> $OUT/bench.err
$T 300 python -u -m pytest -x -q --timeout 280 --timeout-method thread tests/test_abi.py tests/test_golden.py tests/test_gpu_parity.py > $OUT/pytest.log 2>&1
echo ok
