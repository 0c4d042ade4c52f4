#!/bin/bash
# canonical Brakedown codewords: GPU suite (fast + slow), cfg4 per-level / leaf trace, cfg4 line
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03l}; mkdir -p $OUT
T="timeout -k 10"
$T 700 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu_fast.log 2>&1
tail -1 $OUT/pytest_gpu_fast.log
$T 400 python -u -m pytest tests -m "gpu and slow" -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu_slow.log 2>&1
tail -1 $OUT/pytest_gpu_slow.log
$T 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_sdig -o run --output-format csv -- \
  python3 bench.py --code sdig --steps 6 --warmup 2 --pipeline 1 --cpu-baseline off --verify-reps 0 > $OUT/sdig_serial.json 2> $OUT/sdig_serial.err
python tools/sdig_levels.py $(find $OUT/prof_sdig -name "*kernel_trace.csv" | head -1) > $OUT/sdig_levels.txt
$T 300 python bench.py --code sdig --steps 32 --warmup 8 > $OUT/bench_sdig.json 2> $OUT/bench_sdig.err
echo ok
