#!/bin/bash
# round 3: sharded PoS request tests + sharded-engine profiling (N=1, K=20) + cfg5 sharded lines.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03c}; mkdir -p $OUT
T="timeout -k 10"
$T 200 python bench.py --mode sharded --steps 20 --warmup 5 --prof-timed --cpu-baseline off --verify-reps 0 > $OUT/sharded_n1_k20_prof.json 2> $OUT/sharded.err
$T 200 python bench.py --mode sharded --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 > $OUT/sharded_n1_k20.json 2>> $OUT/sharded.err
$T 200 python bench.py --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 > $OUT/replicas_k20.json 2>> $OUT/sharded.err
$T 300 python bench.py --code pos --mode sharded --steps 10 --warmup 2 > $OUT/pos_sharded_n1.json 2> $OUT/pos.err
LCPC_BENCH_BACKEND=gloo LCPC_BENCH_SHARE_GPU=1 $T 300 python bench.py --gpus 2 --code pos --mode sharded --steps 6 --warmup 2 > $OUT/pos_sharded_2ranks_shared.json 2>> $OUT/pos.err
echo ok
