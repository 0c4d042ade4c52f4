#!/bin/bash
# FIFO commits: GPU suite, K=20 A/B (LCPC_COMMIT_FIFO=1 default / 0), K=256, cfg4 / cfg5 lines
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03i}; mkdir -p $OUT
T="timeout -k 10"
$T 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu_fast.log 2>&1
B="python bench.py --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 --sharded-n1 0"
for i in 1 2 3; do
  $T 200 $B --timeline $OUT/tl_fifo_$i.json > $OUT/k20_fifo_$i.json 2>> $OUT/b.err
  LCPC_COMMIT_FIFO=0 $T 200 $B > $OUT/k20_nofifo_$i.json 2>> $OUT/b.err
done
for cs in 2 8; do $T 200 $B --commit-slots $cs > $OUT/k20_fifo_cs$cs.json 2>> $OUT/b.err; done
$T 200 $B --steps 256 > $OUT/k256_fifo.json 2>> $OUT/b.err
$T 300 python bench.py --code sdig --steps 32 --warmup 8 --cpu-baseline off --verify-reps 0 > $OUT/sdig_fifo.json 2>> $OUT/b.err
LCPC_COMMIT_FIFO=0 $T 300 python bench.py --code sdig --steps 32 --warmup 8 --cpu-baseline off --verify-reps 0 > $OUT/sdig_nofifo.json 2>> $OUT/b.err
$T 300 python bench.py --code pos --steps 16 --warmup 4 --cpu-baseline off > $OUT/pos_fifo.json 2>> $OUT/b.err
LCPC_COMMIT_FIFO=0 $T 300 python bench.py --code pos --steps 16 --warmup 4 --cpu-baseline off > $OUT/pos_nofifo.json 2>> $OUT/b.err
echo ok
