#!/bin/bash
# bench.py's N = 8 sharded path end to end with the 8 ranks sharing GPU 0 over RCCL (plumbing:
# one GPU does eight ranks' work, so the rate is not a scaling figure)
set -e
export TMPDIR=/tmp
OUT=gpurun_out/r03s; mkdir -p $OUT
export LCPC_BENCH_BACKEND=gloo LCPC_BENCH_SHARE_GPU=1 LCPC_BENCH_RCCL_SAME_GPU=1
timeout -k 10 400 python bench.py --gpus 8 --steps 20 --warmup 5 --cpu-baseline off > $OUT/bench_sharded_8ranks_rccl_k20_one_gpu.json 2> $OUT/b.err
tail -c 1500 $OUT/bench_sharded_8ranks_rccl_k20_one_gpu.json
echo ok
