#!/bin/bash
# round-2 measurement pass: the driver's default bench command, engine / depth variants, the
# rocprofv3 kernel-trace summary of the default command and the two HBM PMC passes.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -e
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/r02b}
mkdir -p $OUT
T="timeout -k 10"
$T 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_default_k20.json 2> $OUT/bench_default_k20.err
$T 300 python bench.py --gpus 1 --steps 256 --warmup 16 --cpu-baseline off > $OUT/bench_sharded_k256.json 2> $OUT/bench_sharded_k256.err
$T 300 python bench.py --gpus 1 --steps 256 --warmup 16 --mode replicas --cpu-baseline off > $OUT/bench_replicas_k256.json 2> $OUT/bench_replicas_k256.err
$T 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off > $OUT/bench_under_prof.json 2> $OUT/prof.err
$T 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/pmc_fetch -o run --output-format csv -- \
  python3 bench.py --steps 2 --warmup 1 --pipeline 1 --cpu-baseline off --no-prof --verify-reps 0 > /dev/null 2> $OUT/pmc_fetch.err
$T 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/pmc_write -o run --output-format csv -- \
  python3 bench.py --steps 2 --warmup 1 --pipeline 1 --cpu-baseline off --no-prof --verify-reps 0 > /dev/null 2> $OUT/pmc_write.err
echo done
