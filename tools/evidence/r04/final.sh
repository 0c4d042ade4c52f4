#!/bin/bash
# round 4, final tree: the driver's order (pytest -m gpu in one process, smoke, the K = 20 line),
# then the K = 20 command under rocprofv3 (kernel trace + stats) with its two PMC traffic passes
set -o pipefail
O=gpurun_out/${R04_OUT:-r04k}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_k20.json 2> $O/bench_k20.err && \
bash tools/prof_workload.sh ${R04_OUT:-r04k}/prof_k20 20 --warmup 5 --sharded-n1 0 > $O/prof_k20.log 2>&1
