#!/bin/bash
# RCCL multi-rank path on the one GPU: the pytest cases, and the sharded bench lines (2 / 4 ranks)
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03k}; mkdir -p $OUT
T="timeout -k 10"
$T 500 python -u -m pytest tests/test_gpu_shard_native.py -m gpu -k "rccl_one_gpu" -x -v --timeout 300 --timeout-method thread > $OUT/pytest_rccl.log 2>&1
tail -8 $OUT/pytest_rccl.log
export LCPC_BENCH_BACKEND=gloo LCPC_BENCH_SHARE_GPU=1 LCPC_BENCH_RCCL_SAME_GPU=1
$T 300 python bench.py --gpus 2 --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 > $OUT/sharded_2ranks_rccl_k20.json 2> $OUT/b.err
$T 300 python bench.py --gpus 2 --steps 64 --warmup 5 --cpu-baseline off --verify-reps 0 > $OUT/sharded_2ranks_rccl_k64.json 2>> $OUT/b.err
$T 300 python bench.py --gpus 4 --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 > $OUT/sharded_4ranks_rccl_k20.json 2>> $OUT/b.err
$T 300 python bench.py --gpus 2 --code pos --mode sharded --steps 8 --warmup 2 > $OUT/pos_2ranks_rccl.json 2>> $OUT/b.err
echo ok
