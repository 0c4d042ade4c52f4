#!/bin/bash
# Round 5, first box: the GPU suite on the stream-ordered pool / one-priority / pruned tree, the
# driver's K = 20 line with a per-step timeline, the same line under a rocprofv3 kernel trace (GPU
# busy intervals), and the cfg2 / sdig-encode lines with their all-cores oracle baselines.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --timeline $O/timeline_k20.json > $O/bench_k20.json 2> $O/bench_k20.err || { tail -20 $O/bench_k20.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/kt -o run --output-format csv -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 --cpu-baseline off --verify-reps 0 --sharded-n1 0 --timeline $O/timeline_k20_prof.json > $O/bench_k20_prof.json 2> $O/bench_k20_prof.err || { tail -20 $O/bench_k20_prof.err; exit 1; }
timeout -k 10 300 python bench.py --code encode --steps 512 --warmup 16 > $O/bench_encode.json 2> $O/bench_encode.err || { tail -20 $O/bench_encode.err; exit 1; }
timeout -k 10 300 python bench.py --code sdig-encode --steps 64 --warmup 8 > $O/bench_sdig_encode.json 2> $O/bench_sdig_encode.err || { tail -20 $O/bench_sdig_encode.err; exit 1; }
echo done
