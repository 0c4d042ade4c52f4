#!/bin/bash
# round 3: GPU suite, the driver's default line x3 (with sharded_n1), cfg5 / cfg4 evidence with
# rocprofv3 kernel traces and the HBM PMC passes.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r03g}; mkdir -p $OUT
T="timeout -k 10"
$T 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu_fast.log 2>&1
for i in 1 2 3; do
  $T 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_k20_$i.json 2>> $OUT/b.err
done
bash tools/prof_workload.sh r03g/pos 16 --code pos --warmup 4
bash tools/prof_workload.sh r03g/sdig 16 --code sdig --warmup 4
echo ok
