#!/bin/bash
# round 3: GPU suite after the leaf-kernel remap and the sharded driver's prove streams / reserve;
# sharded N=1 K=20 A/B (prove stream priority on / off), replicas K=20, Brakedown levels + leaves.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03d}; mkdir -p $OUT
T="timeout -k 10"
$T 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu_fast.log 2>&1
$T 400 python -u -m pytest tests -m "gpu and slow" -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu_slow.log 2>&1
for i in 1 2; do
  $T 200 python bench.py --mode sharded --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 > $OUT/sharded_k20_prio_$i.json 2>> $OUT/b.err
  LCPC_SHARD_PRIO=0 $T 200 python bench.py --mode sharded --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 > $OUT/sharded_k20_noprio_$i.json 2>> $OUT/b.err
done
$T 200 python bench.py --mode sharded --steps 20 --warmup 5 --prof-timed --cpu-baseline off --verify-reps 0 > $OUT/sharded_k20_prof.json 2>> $OUT/b.err
$T 200 python bench.py --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 > $OUT/replicas_k20.json 2>> $OUT/b.err
$T 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_sdig -o run --output-format csv -- \
  python3 bench.py --code sdig --steps 6 --warmup 2 --pipeline 1 --cpu-baseline off --verify-reps 0 > $OUT/sdig_serial.json 2> $OUT/sdig_serial.err
python tools/sdig_levels.py $(find $OUT/prof_sdig -name "*kernel_trace.csv" | head -1) > $OUT/sdig_levels.txt
echo ok
