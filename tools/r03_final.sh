#!/bin/bash
# round-3 evidence on the final tree: GPU suite (fast + full-size), smoke(), the driver's default
# line (K=20, W=5) and its rocprofv3 kernel-trace summary, the HBM PMC passes of the encode.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03fin}; mkdir -p $OUT
T="timeout -k 10"
$T 700 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu_fast.log 2>&1
tail -1 $OUT/pytest_gpu_fast.log
$T 400 python -u -m pytest tests -m "gpu and slow" -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu_slow.log 2>&1
tail -1 $OUT/pytest_gpu_slow.log
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
$T 400 python bench.py --steps 20 --warmup 5 > $OUT/bench_k20.json 2> $OUT/bench_k20.err
$T 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
  python3 bench.py --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 --sharded-n1 0 > $OUT/bench_under_prof.json 2> $OUT/prof.err
for c in FETCH_SIZE WRITE_SIZE; do
  n=$(echo "$c" | cut -d_ -f1 | tr 'A-Z' 'a-z')
  $T 120 rocprofv3 --pmc "$c" -d "$OUT/pmc_$n" -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --pipeline 1 --cpu-baseline off --no-prof --verify-reps 0 --sharded-n1 0 > /dev/null 2> "$OUT/pmc_$n.err"
done
$T 300 python bench.py --code pos --pipeline 2 --steps 16 --warmup 4 > $OUT/bench_pos.json 2> $OUT/bench_pos.err
$T 300 python bench.py --code sdig --steps 20 --warmup 5 > $OUT/bench_sdig.json 2> $OUT/bench_sdig.err
echo ok
