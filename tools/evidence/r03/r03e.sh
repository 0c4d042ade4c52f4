#!/bin/bash
# sharded N=1 K=20 after moving the commit's post stages to the prove (priority) stream: lag 2 / 3,
# replicas beside it, a kernel trace of the sharded run, and the shard parity tests.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03f}; mkdir -p $OUT
T="timeout -k 10"
$T 500 python -u -m pytest tests/test_gpu_shard_native.py tests/test_gpu_pos_shard.py tests/test_gpu_shard.py -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread > $OUT/pytest_shard.log 2>&1
for i in 1 2; do
  $T 200 python bench.py --mode sharded --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 > $OUT/sharded_k20_lag2_$i.json 2>> $OUT/b.err
  $T 200 python bench.py --mode sharded --steps 20 --warmup 5 --lag 3 --cpu-baseline off --verify-reps 0 > $OUT/sharded_k20_lag3_$i.json 2>> $OUT/b.err
  $T 200 python bench.py --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 > $OUT/replicas_k20_$i.json 2>> $OUT/b.err
done
$T 200 python bench.py --mode sharded --steps 20 --warmup 5 --prof-timed --cpu-baseline off --verify-reps 0 > $OUT/sharded_k20_prof.json 2>> $OUT/b.err
$T 300 rocprofv3 --kernel-trace -d $OUT/prof_sharded -o run --output-format csv -- \
  python3 bench.py --mode sharded --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 --no-prof > $OUT/sharded_under_prof.json 2> $OUT/prof.err
echo ok
