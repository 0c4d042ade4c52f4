#!/bin/bash
# round-2 evidence pass: fast GPU parity suite, the default (driver) bench line with its
# rocprofv3 kernel-trace summary and HBM PMC passes, the same for cfg4 (sdig), and the per-row
# encode drop-in bench.  Every GPU step has its own time limit; the chain stops at the first failure.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/r02ev; mkdir -p $OUT
T="timeout -k 10"
$T 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu_fast.log 2>&1
bash tools/prof_workload.sh r02ev/ligero 20 --warmup 5
bash tools/prof_workload.sh r02ev/sdig 32 --code sdig --warmup 8
$T 300 python tools/encode_rows_bench.py --rows 512 --threads 16 > $OUT/encode_rows.json 2> $OUT/encode_rows.err
echo ok
