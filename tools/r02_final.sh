#!/bin/bash
# round-2 evidence: GPU parity (fast + full-size), smoke(), the driver's default bench line with
# its rocprofv3 kernel-trace summary and HBM PMC passes, cfg4 / cfg5 / cfg2 lines with their
# summaries, the two-rank (shared-GPU, gloo) sharded line, the transcript and per-row encode
# microbenches.  Each GPU step has its own limit; the chain stops at the first failure.
set -e
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r02fin}; mkdir -p $OUT
T="timeout -k 10"
$T 600 python -u -m pytest tests -m "gpu and not slow" -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu_fast.log 2>&1
$T 560 python -u -m pytest tests -m "gpu and slow" -x -v --timeout 900 --timeout-method thread > $OUT/pytest_gpu_slow.log 2>&1
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
bash tools/prof_workload.sh ${1:-r02fin}/ligero 20 --warmup 5
bash tools/prof_workload.sh ${1:-r02fin}/sdig 32 --code sdig --warmup 8
$T 300 python bench.py --code pos --steps 64 --warmup 4 > $OUT/bench_pos.json 2> $OUT/bench_pos.err
$T 300 python bench.py --code encode --steps 512 --warmup 32 > $OUT/bench_encode.json 2> $OUT/bench_encode.err
$T 200 python bench.py --steps 256 --warmup 16 --cpu-baseline off --verify-reps 0 > $OUT/bench_ligero_k256.json 2>> $OUT/bench.err
$T 200 python bench.py --mode sharded --steps 256 --warmup 8 --lag 4 --cpu-baseline off --verify-reps 0 > $OUT/bench_sharded_k256.json 2>> $OUT/bench.err
LCPC_BENCH_BACKEND=gloo LCPC_BENCH_SHARE_GPU=1 $T 300 python bench.py --gpus 2 --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 > $OUT/bench_2ranks_shared_gpu.json 2>> $OUT/bench.err
$T 60 tools/microbench/transcript_bench > $OUT/transcript_bench.txt
$T 300 python tools/encode_rows_bench.py --rows 512 --threads 16 > $OUT/encode_rows.json 2> $OUT/encode_rows.err
echo ok
